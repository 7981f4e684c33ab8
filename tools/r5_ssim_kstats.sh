#!/bin/bash
# Per-kernel stats of the batched SSIM (BATCH items) for each library in SSIM_LIBS, one rocprofv3 pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in ${SSIM_LIBS:-default}; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
  tag=$(basename "$lib" .so)
  echo "== $tag"; BATCH=${BATCH:-384} REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/ksk_$tag -o run -- python3 tools/ssim_probe.py > gpurun_out/ksk_$tag.log 2>&1 || exit 1
  f=$(find gpurun_out/ksk_$tag -name "*kernel_stats.csv"); grep "jds::" $f | cut -d, -f1-4
done
