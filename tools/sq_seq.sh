#!/bin/bash
# SQ counters of the sequential hole-fill's kernels (tools/seq_time.py), two passes of 8.
set -euo pipefail
R=$(pwd)
OUT=$R/gpurun_out/sq_seq
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS -d "$OUT/p1" -o run --output-format csv -- python3 "$R/tools/seq_time.py" 64 > "$OUT/p1.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/p2" -o run --output-format csv -- python3 "$R/tools/seq_time.py" 64 > "$OUT/p2.log" 2>&1
for p in p1 p2; do
  python3 "$R/tools/pmc_kernels.py" --counters "$OUT/$p/run_counter_collection.csv" "sq_colour3_kernel" "sq_colour3df_kernel" "sq_fmm_kernel" "sq_record3_kernel" > "$OUT/$p.txt"
done
rm -rf "$OUT/p1" "$OUT/p2"
