#!/bin/bash
# 4:4:4 inverse A/B: the fast-inverse GPU tests, then kernel times of 256 x
# 512^2 4:4:4 with the plan's default inverse and with the certified fast
# inverse forced (--inv-fast).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_inv_fast.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_444.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_444.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0" bash tools/var_prof.sh base || exit 1
BENCH_ARGS="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0 --inv-fast" bash tools/var_prof.sh base || exit 1
echo done
