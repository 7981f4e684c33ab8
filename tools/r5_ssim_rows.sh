#!/bin/bash
# SSIM rows kernel: GPU SSIM tests, then per-item times of library variants at two batch sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/ssr_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ssr_pytest.log; [ $rc -eq 0 ] || exit $rc
for b in ${BATCHES:-96 384}; do
  for lib in ${SSIM_LIBS:-default}; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "batch $b $lib "; BATCH=$b REPS=4 timeout -k 10 300 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-160 || exit 1
  done
done
