#!/bin/bash
# k_fix_fwd duration vs its grid size (JDS_FIX_GRID probe override).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
for G in ${GRIDS:-2048 4096 16384 65536}; do
  JDS_FIX_GRID=$G timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/fg$G" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity --no-entropy > "$ROOT/gpurun_out/fg$G.log" 2>&1 || exit $?
  echo "G=$G"; grep -h "k_fix_fwd\|k_fwd32<" $(find "$ROOT/gpurun_out/fg$G" -name '*kernel_stats.csv') | cut -d, -f1,2,4 | sed 's/(jds::Geo.*"//'
done
