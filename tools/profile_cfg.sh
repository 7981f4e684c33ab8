#!/bin/bash
# One configuration end to end on the GPU box: bench line, rocprofv3 kernel
# stats, then the two HBM-traffic PMC passes (FETCH_SIZE and WRITE_SIZE each in
# a run of its own, kernel trace only).  Usage: tools/profile_cfg.sh TAG bench-args...
# Output: gpurun_out/cfg/TAG/{bench.json,stats/,fetch/,write/}.  Every GPU step
# has its own time limit; a failure ends the script.
set -u
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT="$ROOT/gpurun_out/cfg/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "stopping after $1 rc=$2"; exit "$2"; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-entropy "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; stop bench $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity --no-entropy "$@" \
  > "$OUT/stats.log" 2>&1
rc=$?; [ $rc -eq 0 ] || stop stats $rc
[ "${NO_PMC:-0}" = 1 ] && { echo done; exit 0; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy "$@" \
  > "$OUT/fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || stop fetch $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy "$@" \
  > "$OUT/write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || stop write $rc
echo done
