#!/bin/bash
# 16x16 fast inverse session: its GPU tests and the existing 16x16 ones, then
# kernel times of configs[4] (16 x 4K 4:2:2 16x16) with the plan's default
# (k_inv16_fast) and with the exact inverse forced (--exact-inv).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_inv_fast16.py tests/test_gpu_fast16.py tests/test_gpu_block16.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_b16.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_b16.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16" bash tools/var_prof.sh base || exit 1
echo done
