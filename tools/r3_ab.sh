#!/bin/bash
# A/B session: full -m gpu suite on the in-tree build, the parity-relevant GPU
# tests on each variant library in $VARS (tools/bin/ab/libjds_<v>.so), then
# rocprofv3 kernel times of every variant (var_prof.sh) with $BENCH_ARGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ -z "${SKIP_FULL:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
for v in $VARS; do
  [ $v = base ] && continue
  JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_plan_4k.py tests/test_gpu_inv_fast.py tests/test_gpu_sweep_plan.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${TAG}_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/var_prof.sh base $VARS || exit 1
echo done
