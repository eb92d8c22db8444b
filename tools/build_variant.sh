#!/bin/bash
# Probe build of the library with extra -D flags, for tools/ab_lib.sh:
#   tools/build_variant.sh ord3 -DOFD_TILE_ORDER=3
# -> opticalflowfromdepth_amd/_build/libofd_fw_ord3.so
set -e
name=$1; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall -I include "$@" \
  -o opticalflowfromdepth_amd/_build/libofd_fw_$name.so opticalflowfromdepth_amd/csrc/ofd_fw.hip \
  opticalflowfromdepth_amd/csrc/ofd_inpaint.hip opticalflowfromdepth_amd/csrc/ofd_inpaint_seq.hip \
  opticalflowfromdepth_amd/csrc/ofd_deflate.hip
