#!/bin/bash
# 4:4:4 inverse per quality: plan default (now k_inv_fast444) vs the exact
# inverse forced (--exact-inv), 256 x 512^2 frames, Q in $QS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for q in ${QS:-10 50 90}; do
  BENCH_ARGS="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0 --quality $q" bash tools/var_prof.sh base || exit 1
done
echo done
