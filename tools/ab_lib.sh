#!/bin/bash
# A/B of probe builds of the library (OFD_FW_LIB=<path>; "base" = the in-tree
# build; tools/build_variant.sh makes them): interleaved bench runs, $ROUNDS
# rounds (default 3), one summary line per run.  Extra bench flags: BENCH_ARGS
# (e.g. "--height 480 --width 640 --batch 32 --no-config2" for config 2 alone).
ROUNDS=${ROUNDS:-3}
for round in $(seq "$ROUNDS"); do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/opticalflowfromdepth_amd/_build/libofd_fw_$v.so"
    OFD_FW_LIB=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hole-fill \
        --no-fused --no-bf16 ${BENCH_ARGS} > /tmp/ab_lib.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/ab_lib.json').read().strip().splitlines()[-1]); c=d.get('config2') or {}; print('$v', d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['value'], 'cfg2', c.get('ms_per_step'), (c.get('roofline') or {}).get('event_ms_per_launch'))"
  done
done
