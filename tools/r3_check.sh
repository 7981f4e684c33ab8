#!/bin/bash
# Round-3 GPU session: every -m gpu test, smoke, the default bench (headline +
# north-star leg + CPU legs + host path), the 2-rank gloo rehearsal, and
# rocprofv3 kernel stats of the headline and of the north-star point.
# Each GPU step under its own limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3}
STEPS=${STEPS:-tests smoke bench rehearse prof}
for st in $STEPS; do case $st in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
bench)
  timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));n=d.get('north_star',{});print('bench', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d['pipeline_roofline_frac'], d['fixups_last_step'], d.get('parity')); print('north_star', n.get('value'), n.get('ms_per_step'), n.get('kernels_ms'), n.get('pipeline_roofline_frac'), n.get('parity'))" ;;
rehearse)
  bash tools/rehearse_ranks.sh > gpurun_out/rehearse_$TAG.log 2>&1; rc=$?; tail -4 gpurun_out/rehearse_$TAG.log; [ $rc -eq 0 ] || exit $rc ;;
prof)
  for pt in headline ns; do
    args="--no-cpu-baseline --no-north-star --no-entropy --no-host-path --no-parity"
    [ $pt = ns ] && args="$args --height 2160 --width 3840 --frames 16"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_${TAG}_$pt" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" $args > "$ROOT/gpurun_out/prof_${TAG}_$pt.log" 2>&1) \
      || { tail -5 "gpurun_out/prof_${TAG}_$pt.log"; exit 1; }
    f=$(find "gpurun_out/prof_${TAG}_$pt" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$pt" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2] + ': ' + '  '.join(f"{r['Name'].split('(')[0].replace('void jds::', '').replace('jds::', '')[:22]}={float(r['AverageNs'])/1e3:.1f}" for r in rows[:5]))
PY
  done ;;
esac; done
echo done
