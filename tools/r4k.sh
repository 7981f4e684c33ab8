#!/bin/bash
# entropy (single pass + LDS-assembled stuffing) and SSIM (planned staging) parity, then their probes
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_entropy.py tests/test_gpu_ssim.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r4k_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/ent_probe.py > gpurun_out/r4k_ent.json 2> gpurun_out/r4k_ent.err; rc=$?; cat gpurun_out/r4k_ent.json; [ $rc -eq 0 ] || exit $rc
LEGACY=0 timeout -k 10 200 python -u tools/ssim_probe.py > gpurun_out/r4k_ssim.json 2> gpurun_out/r4k_ssim.err; rc=$?; cut -c1-200 gpurun_out/r4k_ssim.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4k_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ent_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r4k_prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r4k_prof/run_kernel_stats.csv')):
    if 'ent' in r['Name'] or 'rocprim' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
exit $rc
