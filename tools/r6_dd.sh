#!/bin/bash
# exact integer luma SSE (luma_sse_e6) in every inverse kernel: the full -m gpu suite,
# smoke and the sweep line against the previous commit's library (fp64 two-luma SSE)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06_dd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06_dd_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_dd_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r06_dd_smoke.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for lib in default tools/bin/ab/libjds_r6cc.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 400 python -u bench.py --sweep --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_dd_one.json 2>> gpurun_out/r06_dd.err \
      || { echo "rc=$? $lib"; tail -5 gpurun_out/r06_dd.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06_dd_one.json').read().strip().splitlines()[-1])
print('$pass', '$lib'.split('/')[-1], d['value'], d['ms_per_step'], d.get('parity'), d.get('ssim',{}).get('ms_per_item'))" | tee -a gpurun_out/r06_dd.txt
  done
done
echo dd-done
