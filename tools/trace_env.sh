#!/bin/bash
# Kernel timeline of the headline call under an environment setting:
#   tools/trace_env.sh TAG VAR=value[,VAR=value]   (GPU box, repo root)
# rocprofv3 --kernel-trace over a short bench.py run, summarised by
# tools/trace_summary.py (the last few dispatches with start / duration).
set -euo pipefail
TAG=$1; R=$(pwd); OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
envs=(); [ "${2:--}" != - ] && IFS=, read -r -a envs <<< "$2"
cd /tmp && export TMPDIR=/tmp
for kv in "${envs[@]}"; do export "$kv"; done
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-hole-fill --no-fused --no-bf16 --no-config2 > "$OUT/trace.log" 2>&1
python3 "$R/tools/trace_summary.py" "$OUT/trace/run_kernel_trace.csv" 8 > "$OUT/summary.txt"
rm -rf "$OUT/trace"
cat "$OUT/summary.txt"
