#!/bin/bash
# Round 4: K4 v2 (batched band SSIM) parity vs legacy + oracle, then timing and kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_parity.py -k "ssim or psnr or golden" -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_ssim_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4_ssim_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ssim_probe.py > gpurun_out/r4_ssim_probe.json 2> gpurun_out/r4_ssim_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/r4_ssim_probe.json; tail -3 gpurun_out/r4_ssim_probe.err; [ $rc -eq 0 ] || exit $rc
cd /tmp
LEGACY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r4_ssim_prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/tools/ssim_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/r4_ssim_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$GRAFT_REPO_ROOT/gpurun_out/r4_ssim_prof" -name "*kernel_stats.csv" -exec cp {} "$GRAFT_REPO_ROOT/gpurun_out/r4_ssim_kernel_stats.csv" \;
cut -d, -f1-4 "$GRAFT_REPO_ROOT/gpurun_out/r4_ssim_kernel_stats.csv" | head -12
echo done
