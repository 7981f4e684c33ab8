#!/bin/bash
# the serial luma band in <= 32 KB of LDS (ring 40 slots, the fill lanes'
# checkpoints in registers) and chain groups of 8 / 4 steps (96 VGPRs: five
# workgroups per CU): SSIM + sweep tests on each build, then the 384-pair
# batch against the round-6 library (sb_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for lib in default tools/bin/ab/libjds_sb_cq.so tools/bin/ab/libjds_sb_cq4.so; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r06_oo_pytest.log 2>&1
  rc=$?; echo "pytest($(basename $lib)) rc=$rc"; tail -1 gpurun_out/r06_oo_pytest.log; [ $rc -eq 0 ] || exit $rc
done
unset JDS_LIB_PATH
for pass in 1 2 3; do
  for lib in tools/bin/ab/libjds_sb_base.so default tools/bin/ab/libjds_sb_cq.so tools/bin/ab/libjds_sb_cq4.so tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_sb_cq_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_oo_probe.txt
echo oo-done
