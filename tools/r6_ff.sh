#!/bin/bash
# the batched SSIM on the round-6 code: per-kernel stats of a 384-pair batch
# (rocprofv3), then the batch timed with both halves, the luma half alone
# (NORGB probe) and the R, G, B rows half alone (NOLUMA probe)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$R"
BATCH=384 REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r06_ff_ksk -o run -- python3 tools/ssim_probe.py > gpurun_out/r06_ff_ksk.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
f=$(find gpurun_out/r06_ff_ksk -name "*kernel_stats.csv"); cp "$f" gpurun_out/r06_ff_ssim_kernel_stats.csv
grep "jds::" "$f" | cut -d, -f1-4
for pass in 1 2; do
  for lib in default tools/bin/ab/libjds_ssim_norgb.so tools/bin/ab/libjds_ssim_noluma.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-200 || exit 1
  done
done | tee gpurun_out/r06_ff_probe.txt
echo ff-done
