#!/bin/bash
# k_fix_fwd / forward kernel durations for each library build in tools/bin/ab (rocprofv3 kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
for L in ${LIBS:-A W5 W6 W7}; do
  JDS_LIB_PATH=$ROOT/tools/bin/ab/libjds_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fl$L" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-entropy > "$ROOT/gpurun_out/fl$L.log" 2>&1 || exit $?
  python3 - "$ROOT/gpurun_out/fl$L/run_kernel_stats.csv" "$L" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'k_fix_fwd' in n or 'k_fwd32' in n or 'k_inv2' in n:
        print(sys.argv[2], n.split('(')[0][:28], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
  grep -o '"parity[^}]*}' "$ROOT/gpurun_out/fl$L.log" || true
done
