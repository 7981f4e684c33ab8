#!/bin/bash
# Kernel durations (rocprofv3 stats) of bench.py $BENCH_ARGS for each library build in tools/bin/ab;
# prints kernels whose name matches $KPAT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
for L in ${LIBS:-A B}; do
  JDS_LIB_PATH=$ROOT/tools/bin/ab/libjds_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/kl$L" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-north-star ${ENT_FLAG---no-entropy} ${BENCH_ARGS:-} > "$ROOT/gpurun_out/kl$L.log" 2>&1 || exit $?
  python3 - "$ROOT/gpurun_out/kl$L/run_kernel_stats.csv" "$L" "${KPAT:-k_}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r['Name']):
        print(sys.argv[2], r['Name'].split('(')[0][:32], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
  grep -o '"parity[^}]*}' "$ROOT/gpurun_out/kl$L.log" || true
  grep -o '"value": [0-9.]*' "$ROOT/gpurun_out/kl$L.log" || true
done
