#!/bin/bash
# k_ss_rows (A ring of doubles, now shipped) with the means' axis-0 outputs from
# an LDS table (JDS_SSR_MTAB): SSIM tests on that build, then the 384-pair
# batch against the shipped kernel, whole and rows alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_hh_pytest.log 2>&1
rc=$?; echo "pytest(default) rc=$rc"; tail -2 gpurun_out/r06_hh_pytest.log; [ $rc -eq 0 ] || exit $rc
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_ssr_mtab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_hh_pytest2.log 2>&1
rc=$?; echo "pytest(mtab) rc=$rc"; tail -2 gpurun_out/r06_hh_pytest2.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ssr_mtab.so tools/bin/ab/libjds_ssim_noluma.so tools/bin/ab/libjds_ssr_mtab_noluma.so tools/bin/ab/libjds_ssim_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_hh_probe.txt
echo hh-done
