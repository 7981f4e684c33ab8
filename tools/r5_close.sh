#!/bin/bash
# Round-5 closing check: the -m gpu suite, smoke(), the default bench line and the
# sweep (configs[3] with SSIM).  Every GPU step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5close}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
timeout -k 10 600 python -u bench.py --sweep --steps 10 --warmup 3 > gpurun_out/${TAG}_sweep.json 2> gpurun_out/${TAG}_sweep.err
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_sweep.err; exit $rc; }
python3 - <<PY
import json
d = json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d.get('entropy', {}).get('ms_per_step'),
      d.get('host_path', {}).get('ms_per_frame'), d['north_star'].get('value'), d['parity'])
w = json.loads(open('gpurun_out/${TAG}_sweep.json').read().strip().splitlines()[-1])
print('sweep', w['value'], w['ms_per_step'], w.get('ssim', {}).get('ms_per_item'), w.get('parity'))
PY
echo done
