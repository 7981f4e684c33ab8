#!/bin/bash
# entropy kernel breakdown (rocprof stats of the 64 x 1080p probe)
set -u
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4l_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ent_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r4l_prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r4l_prof/run_kernel_stats.csv')):
    if 'ent' in r['Name'] or 'rocprim' in r['Name'] or 'rocclr' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
exit $rc
