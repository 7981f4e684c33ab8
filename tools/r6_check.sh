#!/bin/bash
# Round-6 check: the -m gpu suite, smoke(), the default bench line with a
# rocprofv3 kernel-stats pass of the same command, then (optional, PMC=1) the
# PMC passes and the FETCH_SIZE calibration.  Every GPU step has its own limit;
# the first failure ends it.   usage: r6_check.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6check}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/${TAG}_prof -o run --output-format csv \
  -- python3 $ROOT/bench.py --no-cpu-baseline --no-host-path --no-parity > $ROOT/gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT
if [ "${SWEEP:-0}" = 1 ]; then
  timeout -k 10 600 python -u bench.py --sweep --steps 10 --warmup 3 > gpurun_out/${TAG}_sweep.json 2> gpurun_out/${TAG}_sweep.err
  rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_sweep.err; exit $rc; }
fi
if [ "${PMC:-0}" = 1 ]; then
  timeout -k 10 60 rocprofv3 -L > gpurun_out/${TAG}_counters_list.txt 2>&1 || true
  bash tools/r6_pmc.sh ${TAG}_pmc; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  bash tools/r6_fetch_cal.sh ${TAG}_cal; rc=$?; echo "cal rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
python3 - <<PY
import json
d = json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d.get('entropy', {}).get('ms_per_step'),
      d.get('host_path', {}).get('ms_per_frame'), d['north_star'].get('value'), d['parity'])
PY
echo done
