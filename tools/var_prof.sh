#!/bin/bash
# rocprofv3 kernel stats of bench.py per library variant (tools/bin/ab/libjds_<name>.so;
# "base" = the in-tree build): the top kernels' average durations side by side.
# Usage: BENCH_ARGS="..." tools/var_prof.sh name [name ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  lib=$ROOT/tools/bin/ab/libjds_$v.so; [ "$v" = base ] && lib=$ROOT/jpeg-dsp-studio_amd/jds/libjds.so
  (cd /tmp && JDS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/vprof_$v" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-north-star --no-entropy --no-host-path --no-parity \
    ${BENCH_ARGS:-} > "$ROOT/gpurun_out/vprof_$v.log" 2>&1) || { echo "$v failed"; tail -3 "$ROOT/gpurun_out/vprof_$v.log"; exit 1; }
  f=$(find "$ROOT/gpurun_out/vprof_$v" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2] + ': ' + '  '.join(f"{r['Name'].split('(')[0].replace('void jds::', '').replace('jds::', '')[:22]}={float(r['AverageNs'])/1e3:.1f}" for r in rows[:5]))
PY
done
