#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_entropy.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4m_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r4m_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ent_probe.py; rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/r4l.sh
