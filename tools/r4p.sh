#!/bin/bash
# statistics reduction beside the fix-up: GPU suite, then bench A/B (JDS_REDUCE_SIDE=0 vs default), twice
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p_gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4p_gputests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    JDS_REDUCE_SIDE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-entropy --no-cpu-baseline --no-north-star --no-host-path > gpurun_out/r4p_b$v.json 2> gpurun_out/r4p_b$v.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/r4p_b$v.json'));print('side=$v', d['value'], d['ms_per_step'], d.get('kernels_ms'), d['parity']['recon_mismatch_bytes'], d['parity']['coeff_mismatch'])"
  done
done
