#!/bin/bash
# rocprofv3 kernel statistics of the quality sweep (configs[3], SSIM included) on the final code
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/r06_sweep_prof2 -o run --output-format csv \
  -- python3 $ROOT/bench.py --sweep --steps 3 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/r06_sweep_prof2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
