#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of tools/bin/fetch_cal (known byte counts, the headline
# kernels' own load shapes), one pass per counter.  usage: r6_fetch_cal.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG="${1:-r06_fetch_cal}"
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d "$ROOT/$OUT/p$i" -o run --output-format csv \
    -- "$ROOT/tools/bin/fetch_cal" > "$ROOT/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($c) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo cal-done
