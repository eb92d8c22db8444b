#!/bin/bash
# Persistent SPLAT grid: workgroups per CU from the occupancy API vs forced (OFD_SPLAT_WG_PER_CU).
set -euo pipefail
mkdir -p gpurun_out
for v in "" 3 4 "" 4 3; do
  echo "== OFD_SPLAT_WG_PER_CU=${v:-api}" >> gpurun_out/occ.txt
  OFD_SPLAT_WG_PER_CU=$v timeout -k 10 120 python3 tools/fused_time.py >> gpurun_out/occ.txt 2>&1
done
