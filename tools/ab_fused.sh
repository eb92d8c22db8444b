#!/bin/bash
# A/B of library builds on the fused warps (tools/fused_time.py), interleaved, 3 rounds.
# usage: bash tools/ab_fused.sh base old ...   ("base" = in-tree build; X = _build/libofd_fw_X.so)
set -e
for round in 1 2 3; do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/opticalflowfromdepth_amd/_build/libofd_fw_$v.so"
    echo "== $v"
    OFD_FW_LIB=$lib timeout -k 10 120 python3 tools/fused_time.py 2>&1 | grep "ms per call"
  done
done
