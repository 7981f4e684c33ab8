#!/bin/bash
# Steady-state vs short-warmup bench (DVFS ramp check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for wv in "3 20" "100 100" "3 200"; do
  set -- $wv
  timeout -k 10 300 python bench.py --warmup $1 --steps $2 --no-cpu-baseline --no-north-star --no-parity --no-entropy > gpurun_out/warm_$1_$2.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/warm_$1_$2.json'));print('$1 $2', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
