#!/bin/bash
# timing probe: the luma band's SSIM map computed but not stored, and the
# chunks launch for the map skipped (wrong values) -- what the map's HBM round
# trip (16 MB each way per 1080p item) costs the 384-pair batch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ss_nosmap.so tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_ss_nosmap_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_jj_probe.txt
echo jj-done
