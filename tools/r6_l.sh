#!/bin/bash
# load_col as one 16-B row load + DPP int16 transpose (default build) vs the
# element loads (libjds_elems) and k_inv_fast6 (v4w4 / v4w6): the inverse tests
# on the default build, A/B on both lines, PMC records of v4w4 and the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "inv or parity or plan or fast" > gpurun_out/r06_l_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06_l_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_l "default tools/bin/ab/libjds_elems.so tools/bin/ab/libjds_fregx.so tools/bin/ab/libjds_v4w4.so tools/bin/ab/libjds_v4w6.so" || exit 1
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_v4w4.so bash tools/r6_pmc.sh r06_l_pmc_v4w4 || exit 1
bash tools/r6_pmc.sh r06_l_pmc_rows || exit 1
echo l-done
