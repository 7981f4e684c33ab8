#!/bin/bash
# k_inv_fast6 (buffer loads/stores, row loads + int16 transpose) at 4 and 6
# waves per SIMD: tests on the 4-wave build, A/B, then the PMC record of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_v4w4.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "inv or parity or plan" > gpurun_out/r06_k_pytest.log 2>&1
rc=$?; echo "pytest(v4w4) rc=$rc"; tail -2 gpurun_out/r06_k_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 NS=0 bash tools/r6_ab.sh r06_k "default tools/bin/ab/libjds_v4w4.so tools/bin/ab/libjds_v4w6.so" || exit 1
for v in v4w4 v4w6; do
  JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so bash tools/r6_pmc.sh r06_k_pmc_$v || exit 1
done
echo k-done
