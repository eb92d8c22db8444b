#!/bin/bash
# HBM traffic of the hole-fill kernels (tools/seq_time.py 64: the layered then
# the sequential fill of the bench's 64 warped 768x1024 images): a kernel
# trace, then separate FETCH_SIZE and WRITE_SIZE passes (never combined with
# other tracing), tabulated by tools/pmc_kernels.py.  GPU box, repo root.
set -euo pipefail
R=$(pwd)
OUT=$R/gpurun_out/seq_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/tools/seq_time.py" 64 > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$R/tools/seq_time.py" 64 > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$R/tools/seq_time.py" 64 > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_kernels.py" "$OUT/trace" "$OUT/fetch" "$OUT/write" > "$OUT/seq_pmc.txt"
cp "$OUT/trace/run_kernel_stats.csv" "$OUT/seq_kernel_stats.csv"
rm -rf "$OUT/fetch" "$OUT/write"
