#!/bin/bash
# image-stream pipelining re-measured on the round-6 kernels: the headline
# command with and without --pipeline 1 (forward of batch k+1 beside the
# inverse of batch k on a second stream), interleaved on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for pl in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --pipeline $pl \
      > gpurun_out/r06_ee_one.json 2>> gpurun_out/r06_ee.err || { echo "rc=$? pipeline=$pl"; tail -5 gpurun_out/r06_ee.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r06_ee_one.json').read().strip().splitlines()[-1])
print('$pass', 'pipeline=$pl', d['value'], d['ms_per_step'], d.get('parity', {}).get('mismatches') if isinstance(d.get('parity'), dict) else d.get('parity'))" | tee -a gpurun_out/r06_ee.txt
  done
done
echo ee-done
