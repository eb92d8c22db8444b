#!/bin/bash
# A/B of library knobs set through the environment: interleaved headline
# bench runs, $ROUNDS rounds (default 3), one summary line per run.
#   tools/ab_env.sh OFD_FW_ROWPATH=1 OFD_FW_ROWPATH=0
# ("-" = no extra variable; A=1,B=2 sets both).  Extra bench flags: BENCH_ARGS.
ROUNDS=${ROUNDS:-3}
for round in $(seq "$ROUNDS"); do
  for v in "$@"; do
    envs=(); [ "$v" != - ] && IFS=, read -r -a envs <<< "$v"
    env "${envs[@]}" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hole-fill \
        --no-fused --no-bf16 ${BENCH_ARGS} > /tmp/ab_env.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/ab_env.json').read().strip().splitlines()[-1]); c=d.get('config2') or {}; print('$v', d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['value'], 'cfg2', c.get('ms_per_step'))"
  done
done
