#!/bin/bash
# ring split v3: straight-line interleaved interior and ring chains vs the round-6 base
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "inv or parity or plan" > gpurun_out/r06_r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06_r_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 NS=0 bash tools/r6_ab.sh r06_r "default tools/bin/ab/libjds_r6base.so" || exit 1
TESTS=0 NS=0 bash tools/r6_ab.sh r06_r2 "default tools/bin/ab/libjds_r6base.so" || exit 1
echo r-done
