#!/bin/bash
# A/B of probe builds on the config-5 bf16 warp (368x560, B=64; bench.py's
# bf16_warp phase, next to the f32 warp of the same batch): interleaved,
# $ROUNDS rounds (default 3); "base" = the in-tree build, "base:VAR=VALUE" the
# in-tree build with one environment variable set.
ROUNDS=${ROUNDS:-3}
for round in $(seq "$ROUNDS"); do
  for v in "$@"; do
    lib=""; envv="OFD_AB_UNUSED=1"
    case "$v" in
      base) ;;
      base:*) envv="${v#base:}" ;;
      *) lib="$PWD/opticalflowfromdepth_amd/_build/libofd_fw_$v.so" ;;
    esac
    env "$envv" OFD_FW_LIB=$lib timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-hole-fill \
        --no-fused --no-config2 > /tmp/ab_bf16.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/ab_bf16.json').read().strip().splitlines()[-1]); b=d['bf16_warp']; print('$v', b['ms_per_step'], b['f32_ms_per_step'], round(1 - b['ms_per_step'] / b['f32_ms_per_step'], 4), b['equals_f32_path'])"
  done
done
