#!/bin/bash
# Bench line (no CPU legs) + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-quick}
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --no-entropy --no-host-path ${BENCH_ARGS:-} > gpurun_out/$TAG.json 2>gpurun_out/$TAG.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/$TAG.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/$TAG.json'));print(d['value'], d['ms_per_step'], d['kernels_ms'], d.get('fixups_last_step'), d.get('parity'))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-north-star --no-entropy --no-host-path --no-parity ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit $rc; }
f=$(find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={r['Percentage']}")
PY
