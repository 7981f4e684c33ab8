#!/bin/bash
# closing evidence: 2-rank gloo rehearsal of bench.py (headline + sweep), entropy PMC of the one-pass coder
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 700 bash tools/rehearse_ranks.sh > gpurun_out/r4o_rehearse.log 2>&1
rc=$?; echo "rehearse rc=$rc"; cut -c1-300 gpurun_out/r4o_rehearse.log | tail -4; [ $rc -eq 0 ] || exit $rc
bash tools/r4_probe_pmc.sh r4o_entpmc tools/ent_probe.py > gpurun_out/r4o_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; grep "k_ent" gpurun_out/r4o_pmc.log | head; exit $rc
