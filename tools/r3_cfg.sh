#!/bin/bash
# Weak configurations: kernel times of 512x512 4:4:4 (plan default k_inv2 vs the
# certified fast inverse forced) and of the 4K 4:2:2 16x16 stretch, plus every
# BASELINE config's bench line (configs_bench.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/configs_bench.sh || exit 1
BENCH_ARGS="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0" bash tools/var_prof.sh base || exit 1
BENCH_ARGS="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0 --inv-fast" bash tools/var_prof.sh base || exit 1
BENCH_ARGS="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16" bash tools/var_prof.sh base || exit 1
echo done
