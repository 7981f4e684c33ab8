#!/bin/bash
# k_fix_fwd with the quantiser row requested beside the block's pixels (qearly) vs at its use
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_qearly.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "fwd or fix or plan or sweep or parity or stats" > gpurun_out/r06_x_pytest.log 2>&1
rc=$?; echo "pytest(qearly) rc=$rc"; tail -2 gpurun_out/r06_x_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_x "default tools/bin/ab/libjds_qearly.so" || exit 1
TESTS=0 NS=0 bash tools/r6_ab.sh r06_x2 "default tools/bin/ab/libjds_qearly.so" || exit 1
echo x-done
