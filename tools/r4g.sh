#!/bin/bash
# inverse unroll / int16-load variants (kernel stats of bench.py per library), then entropy PMC
set -u
cd "${GRAFT_REPO_ROOT}"
LIBS="A UC UY UCY I A" KPAT="k_inv_fast|k_fwd32i" bash tools/kernlib_probe.sh 2>&1 | tee gpurun_out/r4g_kl.txt
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
bash tools/r4_probe_pmc.sh r4g_entpmc tools/ent_probe.py && grep -A3 "k_ent" gpurun_out/r4g_entpmc/report.txt
