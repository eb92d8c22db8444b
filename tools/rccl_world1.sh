#!/bin/bash
# The RCCL code paths at world size 1 on the one-GPU box (GPU box, repo root):
# bench.py and both on-the-fly train steps under torch.distributed.run, with
# NCCL_DEBUG=INFO so the logs show RCCL initialising its communicator.
set -euo pipefail
mkdir -p gpurun_out/rccl
export NCCL_DEBUG=INFO
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline --no-hole-fill \
    > gpurun_out/rccl/bench.json 2> gpurun_out/rccl/bench.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29612 -m opticalflowfromdepth_amd.onthefly --steps 10 --warmup 2 --arch raft \
    > gpurun_out/rccl/raft.json 2> gpurun_out/rccl/raft.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29613 -m opticalflowfromdepth_amd.onthefly --steps 10 --warmup 2 --arch gmflow \
    > gpurun_out/rccl/gmflow.json 2> gpurun_out/rccl/gmflow.err
grep -h "NCCL INFO.*nranks 1" gpurun_out/rccl/*.json | cut -c1-200 || true
grep -h '^{' gpurun_out/rccl/bench.json gpurun_out/rccl/raft.json gpurun_out/rccl/gmflow.json | cut -c1-300
