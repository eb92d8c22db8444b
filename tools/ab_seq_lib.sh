#!/bin/bash
# A/B of probe builds of the library on the sequential hole-fill
# (tools/seq_time.py B: layered then sequential fill of B warped 768x1024
# images; "base" = the in-tree build, else _build/libofd_fw_<name>.so from
# tools/build_variant.sh; "base:VAR=VALUE" = the in-tree build with one
# environment variable set, "base:A=1,B=2" several): interleaved, $ROUNDS
# rounds (default 3).
ROUNDS=${ROUNDS:-3}
B=${B:-64}
for round in $(seq "$ROUNDS"); do
  for v in "$@"; do
    lib=""; envv="OFD_AB_UNUSED=1"
    case "$v" in
      base) ;;
      base:*) envv="${v#base:}"; envv="${envv//,/ }" ;;
      *) lib="$PWD/opticalflowfromdepth_amd/_build/libofd_fw_$v.so" ;;
    esac
    env $envv OFD_FW_LIB=$lib timeout -k 10 120 python tools/seq_time.py "$B" > /tmp/ab_seq.txt 2>&1 || exit 1
    echo "$v $(grep "^${PHASE:-sequential}" /tmp/ab_seq.txt)"
  done
done
