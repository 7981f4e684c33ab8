#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks share the GPU over gloo
# (RCCL refuses two ranks on one device).  The driver's 8-GPU runs use nccl.
# The headline leg goes through bench.py's own launcher (--gpus 2 without
# torchrun: it starts the ranks itself; JDS_BENCH_REHEARSE=1 allows sharing the
# one GPU); the sweep leg through torchrun as the driver launches it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --frames 16 --no-cpu-baseline \
  > gpurun_out/rehearse_main.json 2> gpurun_out/rehearse_main.err || { tail -20 gpurun_out/rehearse_main.err; exit 1; }
grep '^{' gpurun_out/rehearse_main.json | cut -c1-400
export JDS_BENCH_BACKEND=gloo JDS_BENCH_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --gpus 2 --sweep --steps 2 --warmup 1 --frames 8 \
  > gpurun_out/rehearse_sweep.json 2> gpurun_out/rehearse_sweep.err || { tail -20 gpurun_out/rehearse_sweep.err; exit 1; }
grep '^{' gpurun_out/rehearse_sweep.json | cut -c1-400
