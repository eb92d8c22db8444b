#!/bin/bash
# A/B of hole-fill variants selected by an environment variable: interleaved
# bench hole-fill phases (3 rounds), ms per 64-image batch.
VAR=$1; shift
for round in 1 2 3; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fused --no-bf16 --hole-fill-steps 5 > /tmp/ab_ip.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/ab_ip.json').read().strip().splitlines()[-1]); h=d['hole_fill']; print('$VAR=$v', h['ms_per_step'], h['value'])"
  done
done
