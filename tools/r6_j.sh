#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_v3w4.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "inv or parity or plan" > gpurun_out/r06_j_pytest.log 2>&1
rc=$?; echo "pytest(v3w4) rc=$rc"; tail -2 gpurun_out/r06_j_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 NS=0 bash tools/r6_ab.sh r06_j "default tools/bin/ab/libjds_v3w4.so tools/bin/ab/libjds_v3w4np.so tools/bin/ab/libjds_v3w4np_p1.so tools/bin/ab/libjds_v3w6.so tools/bin/ab/libjds_v3w6np.so"
