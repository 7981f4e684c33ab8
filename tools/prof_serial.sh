#!/bin/bash
# rocprofv3 kernel trace of the default bench (serial steps), for the timeline / gap analysis.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_s" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity --no-entropy ${BENCH_ARGS:-} \
  > "$ROOT/gpurun_out/prof_s.log" 2>&1
rc=$?; grep '^{' "$ROOT/gpurun_out/prof_s.log"; exit $rc
