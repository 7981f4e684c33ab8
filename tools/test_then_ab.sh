#!/bin/bash
# GPU parity suite, then (only if green) rocprof kernel stats of the listed
# library variants (tools/var_prof.sh).  Usage: tools/test_then_ab.sh TAG variant...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/var_prof.sh "$@"
