#!/bin/bash
# One GPU session: parity tests, then (only if no fault/timeout) bench + rocprof.
# Each GPU step has its own time limit; a fault, abort, segfault or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { case "$1" in 0|1) return 0;; *) echo "stopping: rc=$1"; exit "$1";; esac; }
STAGE="${1:-all}"

if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest-gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; [ $rc -eq 0 ] || exit $rc
fi
echo done
