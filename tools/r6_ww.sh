#!/bin/bash
# the SSE input row requested before the colour work in k_inv_fast<MODE,1>
# (JDS_SSE_EARLY): the sweep-plan SSE tests on that build, then the sweep
# line against the shipped library, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_sse_early.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep_plan.py tests/test_gpu_inv_fast.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_ww_pytest.log 2>&1
rc=$?; echo "pytest(sse_early) rc=$rc"; tail -1 gpurun_out/r06_ww_pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2 3; do
  for lib in tools/bin/ab/libjds_sse_base.so tools/bin/ab/libjds_sse_early.so; do
    export JDS_LIB_PATH=$PWD/$lib
    timeout -k 10 400 python -u bench.py --sweep --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_ww_one.json 2>> gpurun_out/r06_ww.err \
      || { echo "rc=$? $lib"; tail -5 gpurun_out/r06_ww.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06_ww_one.json').read().strip().splitlines()[-1])
print('$pass', '$lib'.split('/')[-1], d['value'], d['ms_per_step'], d.get('parity', {}).get('mismatches'))" | tee -a gpurun_out/r06_ww.txt
  done
done
echo ww-done
