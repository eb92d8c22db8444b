#!/bin/bash
# tools/profile_fused.sh -- kernel table and HBM traffic of the fused first-stage
# warps (tools/fused_time.py: warp_disparity f32/f64 depth, warp_ego f64/f32
# depth, plain FW; 64 x 768x1024, 11 calls each).  Run on the GPU box from the
# repo root; writes gpurun_out/prof_fused_<tag>/.
set -euo pipefail
TAG=${1:-r02}
R=$(pwd)
OUT=$R/gpurun_out/prof_fused_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/tools/fused_time.py" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$R/tools/fused_time.py" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$R/tools/fused_time.py" > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_kernels.py" "$OUT/trace" "$OUT/fetch" "$OUT/write" > "$OUT/summary.txt"
