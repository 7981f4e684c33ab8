#!/bin/bash
# big luma launches on the overlapped band schedule (chain beside the next
# chunk's fill, 46 KB: three workgroups per CU; map stored) against the serial
# leaf-folded band: the 384-pair batch, whole and luma alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ss_ov.so tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_ss_ov_norgb.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110 || exit 1
  done
done | tee gpurun_out/r06_vv_probe.txt
echo vv-done
