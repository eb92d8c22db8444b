#!/bin/bash
# A/B of probe builds of the library (OFD_FW_LIB=<path>; "base" = the in-tree
# build): interleaved bench runs, 3 rounds, one summary line per run.
for round in 1 2 3; do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/opticalflowfromdepth_amd/_build/libofd_fw_$v.so"
    OFD_FW_LIB=$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hole-fill --no-fused --no-bf16 > /tmp/ab_lib.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/ab_lib.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['value'])"
  done
done
