#!/bin/bash
# A/B session over several workloads: the full -m gpu suite on the in-tree
# build, the parity tests on every variant named in the pairs, then
# var_prof.sh per workload: "WORKLOAD:variant,variant" items in $PAIRS, where
# WORKLOAD is one of hd (64 x 1080p 4:2:0), q422 (16 x 4K 4:2:2), s444 (256 x 512^2 4:4:4),
# b16 (16 x 4K 4:2:2 16x16), q10 (16 x 4K Q10 4:2:0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
# SKIP_FULL=1: no full suite (the in-tree build unchanged); SKIP_VPARITY=1: timing-only probe
# variants (e.g. statistics removed) skip the parity tests
if [ -z "${SKIP_FULL:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
seen=" "
[ -n "${SKIP_VPARITY:-}" ] && seen=" $(echo $PAIRS | tr ' ' '\n' | sed 's/^[^:]*://' | tr ',' ' ' | tr '\n' ' ') "
for p in $PAIRS; do for v in $(echo ${p#*:} | tr , ' '); do
  case "$seen" in *" $v "*) continue ;; esac; seen="$seen$v "
  JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_plan_4k.py tests/test_gpu_inv_fast.py tests/test_gpu_sweep_plan.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${TAG}_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"; [ $rc -eq 0 ] || exit $rc
done; done
for p in $PAIRS; do
  w=${p%%:*}
  case $w in
    hd) a="" ;;
    q422) a="--height 2160 --width 3840 --frames 16 --mode 4:2:2" ;;
    s444) a="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0" ;;
    b16) a="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16" ;;
    b16f) a="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16 --inv-fast" ;;
    q10) a="--height 2160 --width 3840 --frames 16 --quality 10" ;;
  esac
  echo "== $w"; BENCH_ARGS="$a" bash tools/var_prof.sh base $(echo ${p#*:} | tr , ' ') || exit 1
done
echo done
