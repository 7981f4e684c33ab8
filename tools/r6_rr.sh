#!/bin/bash
# the luma band map in waves 2-3 (two pixels a lane) beside the fill in waves
# 0-1 (JDS_SB_MAPW): SSIM + sweep tests on that build, then the 384-pair batch,
# whole and luma alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_sb_mapw.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_rr_pytest.log 2>&1
rc=$?; echo "pytest(sb_mapw) rc=$rc"; tail -1 gpurun_out/r06_rr_pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_sb_mapw.so tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_sb_mapw_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_rr_probe.txt
echo rr-done
