set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep_ranks.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4c_ranks.log 2>&1
rc=$?; echo "ranks rc=$rc"; tail -5 gpurun_out/r4c_ranks.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_check.sh r4c pmc4k ssimprof bench
