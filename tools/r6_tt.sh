#!/bin/bash
# per-kernel times of the luma half alone (NORGB probe build) and of the whole
# batched SSIM, 384 1080p pairs, on the current code (rocprofv3 kernel stats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$R"
for lib in default tools/bin/ab/libjds_ssim_norgb.so; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; tag=all; else export JDS_LIB_PATH=$PWD/$lib; tag=luma; fi
  BATCH=384 REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/r06_tt_$tag -o run -- python3 tools/ssim_probe.py > gpurun_out/r06_tt_$tag.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
  f=$(find gpurun_out/r06_tt_$tag -name "*kernel_stats.csv"); cp "$f" gpurun_out/r06_tt_${tag}_kernel_stats.csv
done
echo tt-done
