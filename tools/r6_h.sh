#!/bin/bash
# k_inv_fast6 layout v2 and the flat fix-up grid: the -m gpu suite on each
# variant library, then the A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in v2w6 ff2k; do
  JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06_h_pytest_$v.log 2>&1
  rc=$?; echo "pytest($v) rc=$rc"; tail -2 gpurun_out/r06_h_pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
TESTS=0 NS=0 bash tools/r6_ab.sh r06_h "default tools/bin/ab/libjds_v2w6.so tools/bin/ab/libjds_v2w6np.so tools/bin/ab/libjds_v2w4np.so tools/bin/ab/libjds_v2w4np_p1.so tools/bin/ab/libjds_v2w6np_p1.so tools/bin/ab/libjds_ff4k.so tools/bin/ab/libjds_ff2k.so tools/bin/ab/libjds_ff1k.so"
