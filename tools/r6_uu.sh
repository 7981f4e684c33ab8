#!/bin/bash
# the luma map folded into leaf sums inside k_ss_band again, on the round-6
# band (fill groups, map in waves 2-3; the leaf lanes' constants kept out of
# the loop: 124 VGPRs, no spills): tests, then A/B against JDS_SSIM_NO_LF
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py tests/test_gpu_sweep_ranks.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_uu_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06_uu_pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ss_nolf.so tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_ss_nolf_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_uu_probe.txt
echo uu-done
