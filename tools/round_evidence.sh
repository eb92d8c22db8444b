#!/bin/bash
# tools/round_evidence.sh TAG -- one gpurun call's worth of round evidence, run
# from the repo root on the GPU box: the GPU tests, smoke(), the default bench
# line, then the rocprof kernel stats + PMC traffic of the warp
# (tools/profile_round.sh) and of the sequential hole-fill (tools/seq_pmc.sh).
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-r03}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
bash tools/profile_round.sh ${TAG}
bash tools/seq_pmc.sh
tail -2 gpurun_out/${TAG}_gputests.log
tail -1 gpurun_out/${TAG}_bench.json | cut -c1-600
