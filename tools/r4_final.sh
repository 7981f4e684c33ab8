#!/bin/bash
# Round-4 closing check: the whole -m gpu suite, smoke(), bench (all legs), --sweep, rocprof of the bench.
set -u
cd "${GRAFT_REPO_ROOT}"
TAG=${1:-r4f}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_check.sh ${TAG} bench sweep prof
