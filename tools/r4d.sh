set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_sweep_plan.py tests/test_gpu_sweep_ranks.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4d_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4d_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_check.sh r4d probe ssimprof
