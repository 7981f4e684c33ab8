#!/bin/bash
# the entropy walk's waves per workgroup (JDS_ES_WAVES) 6 / 8 against the
# shipped 4; ent_probe, file digest must match
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ent_w6.so tools/bin/ab/libjds_ent_w8.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; timeout -k 10 200 python -u tools/ent_probe.py 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_batch'], d['bytes'], d['sha16'])" || exit 1
  done
done | tee gpurun_out/r06_xx2_ent.txt
echo xx-done
