#!/bin/bash
# Probe build of the library with the sequential hole-fill's clock stamps
# (-DOFD_SQ_PROF), loaded through OFD_FW_LIB; prints the phase split of the
# deepest image.  Build here, run on the GPU box:
#   tools/seq_probe.sh build      (CPU container)
#   tools/seq_probe.sh run [B]    (GPU box)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/opticalflowfromdepth_amd/_build/libofd_fw_sqprof.so"
if [ "$1" = build ]; then
  mkdir -p "$(dirname "$OUT")"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DOFD_SQ_PROF \
    -I "$R/include" -o "$OUT" "$R"/opticalflowfromdepth_amd/csrc/ofd_fw.hip \
    "$R"/opticalflowfromdepth_amd/csrc/ofd_inpaint.hip "$R"/opticalflowfromdepth_amd/csrc/ofd_inpaint_seq.hip \
    "$R"/opticalflowfromdepth_amd/csrc/ofd_deflate.hip
else
  OFD_FW_LIB="$OUT" python3 -u "$R/tools/seq_time.py" "${2:-16}"
fi
