#!/bin/bash
# the entropy coder's walk parameters re-tuned on the round-6 code: ES_DENSE
# (zigzag positions coded by the unrolled walk) 24 / 40, ES_SW (LDS staging
# words per lane) 4 / 12, ES_WPE 5; ent_probe, file digest must match
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ent_d24.so tools/bin/ab/libjds_ent_d40.so tools/bin/ab/libjds_ent_sw4.so tools/bin/ab/libjds_ent_sw12.so tools/bin/ab/libjds_ent_wpe5.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; timeout -k 10 200 python -u tools/ent_probe.py 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_batch'], d['bytes'], d['sha16'])" || exit 1
  done
done | tee gpurun_out/r06_ss_ent.txt
echo ss-done
