#!/bin/bash
# k_fix_fwd as workgroups of 2 / 4 / 8 independent fix-up waves (fewer workgroups to dispatch) vs one wave
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in fw4 fw8; do
  JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "fwd or fix or plan or sweep or parity or stats" > gpurun_out/r06_t_pytest_$v.log 2>&1
  rc=$?; echo "pytest($v) rc=$rc"; tail -2 gpurun_out/r06_t_pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
TESTS=0 bash tools/r6_ab.sh r06_t "default tools/bin/ab/libjds_fw2.so tools/bin/ab/libjds_fw4.so tools/bin/ab/libjds_fw8.so" || exit 1
echo t-done
