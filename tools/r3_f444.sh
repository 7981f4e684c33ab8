#!/bin/bash
# Wave-local 4:4:4 forward (k_fwd444w) vs k_fwd32i<4:4:4> (JDS_FWD444_TILED=1): every GPU
# test, then kernel times at 256 x 512^2 4:4:4 (cfg1 geometry), same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_f444.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_f444.log; [ $rc -eq 0 ] || exit $rc
A="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0"
BENCH_ARGS="$A" bash tools/var_prof.sh base || exit 1
JDS_FWD444_TILED=1 BENCH_ARGS="$A" bash tools/var_prof.sh base || exit 1
echo done
