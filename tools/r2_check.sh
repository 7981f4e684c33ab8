#!/bin/bash
# GPU session: concurrency + odd-size tests, then the default bench line (all legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_oddsize.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2>gpurun_out/bench_default.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default.err; exit $rc; }
cat gpurun_out/bench_default.json
