#!/bin/bash
# k_inv_fast<4:2:0> with the ring split (default build) vs the round-6 base: inverse tests, then A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "inv or parity or plan or fast or sweep" > gpurun_out/r06_o_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06_o_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_o "default tools/bin/ab/libjds_r6base.so" || exit 1
echo o-done
