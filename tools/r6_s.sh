#!/bin/bash
# k_inv_fast over a persistent grid (512 / 1024 / 2048 workgroups) vs one tile per workgroup
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_pers512.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "inv or parity or plan" > gpurun_out/r06_s_pytest.log 2>&1
rc=$?; echo "pytest(pers512) rc=$rc"; tail -2 gpurun_out/r06_s_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_s "default tools/bin/ab/libjds_pers512.so tools/bin/ab/libjds_pers1024.so tools/bin/ab/libjds_pers2048.so tools/bin/ab/libjds_r6base.so" || exit 1
echo s-done
