#!/bin/bash
# SSE runs (the quality sweep) through the certified fast inverse k_inv_fast<MODE,1> (libjds_ssefast)
# vs the exact k_inv2<MODE,1>: sweep / SSE tests on the variant, then the sweep line with --inv-fast on both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_ssefast.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "sweep or sse or psnr or metrics or plan or parity" > gpurun_out/r06_bb_pytest.log 2>&1
rc=$?; echo "pytest(ssefast) rc=$rc"; tail -2 gpurun_out/r06_bb_pytest.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for lib in default tools/bin/ab/libjds_ssefast.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 400 python -u bench.py --sweep --inv-fast --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r06_bb_one.json 2>> gpurun_out/r06_bb.err \
      || { echo "rc=$? $lib"; tail -5 gpurun_out/r06_bb.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06_bb_one.json').read().strip().splitlines()[-1])
print('$pass', '$lib'.split('/')[-1], d['value'], d['ms_per_step'], d.get('parity'), d.get('ssim',{}).get('ms_per_item'))" | tee -a gpurun_out/r06_bb.txt
  done
done
echo bb-done
