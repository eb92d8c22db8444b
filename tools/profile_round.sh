#!/bin/bash
# tools/profile_round.sh -- the round's GPU profiling recipe (run on the GPU box
# via gpurun from the repo root).  Writes under gpurun_out/prof_<tag>/.
#   1. rocprofv3 --kernel-trace --stats over a short bench.py run
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE (never combined with
#      other tracing), summarised by tools/pmc_summary.py
set -euo pipefail
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-hole-fill --no-fused --no-bf16 --no-config2 > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-hole-fill --no-fused --no-bf16 --no-config2 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-hole-fill --no-fused --no-bf16 --no-config2 > "$OUT/write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT/fetch" "$OUT/write" "$OUT/trace" 64 6 768 1024 "$OUT/pmc_traffic.json"
python3 "$R/tools/trace_summary.py" "$OUT/trace/run_kernel_trace.csv" 3 > "$OUT/trace_summary.txt"
