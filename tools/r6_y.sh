#!/bin/bash
# k_inv_fast with MAGIC + 128 folded into the luma row pass's DC input (timing + tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_mfold.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "inv or parity or plan" > gpurun_out/r06_y_pytest.log 2>&1
rc=$?; echo "pytest(mfold) rc=$rc"; tail -2 gpurun_out/r06_y_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_y "default tools/bin/ab/libjds_mfold.so" || exit 1
TESTS=0 NS=0 bash tools/r6_ab.sh r06_y2 "default tools/bin/ab/libjds_mfold.so" || exit 1
echo y-done
