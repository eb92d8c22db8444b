#!/bin/bash
# A/B of launch variants selected by an environment variable: interleaved
# bench runs (3 rounds), one JSON summary line per run in gpurun_out/ab.log.
VAR=$1; shift
for round in 1 2 3; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hole-fill --no-fused > /tmp/ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/ab_$v.json').read().strip().splitlines()[-1]); print('$VAR=$v', d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['value'])"
  done
done
