#!/bin/bash
# Headline ms/step against the warm-up length: alternating runs of bench.py
# (headline only) at --warmup W for each W given, K = 20 timed steps.
# usage: tools/warm_ab.sh 5 100 [rounds]
set -o pipefail
A=${1:-5}; B=${2:-100}; R=${3:-3}
for r in $(seq "$R"); do
  for w in "$A" "$B"; do
    line=$(timeout -k 10 180 python3 bench.py --steps 20 --warmup "$w" --no-cpu-baseline --no-hole-fill \
           --no-fused --no-bf16 --no-config2 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('warmup', sys.argv[2], d['ms_per_step'], d['roofline']['frac'])" "$line" "$w"
  done
done
