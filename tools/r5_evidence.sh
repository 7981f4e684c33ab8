#!/bin/bash
# Round-5 evidence runs.  usage: tools/r5_evidence.sh TAG stage...
#   tests   the -m gpu suite (one process, per-test limit)
#   micro   tools/bin/mfma_rate (MFMA / VALU issue rates and overlap, fp64 and fp32)
#   head    tools/profile_cfg.sh on the headline (64 x 1080p Q50 4:2:0 pf): bench, rocprof stats, FETCH / WRITE
#   4k      the same at the north-star point (16 x 4K Q50 4:2:0)
#   cfg1 cfg3 cfg5b8 cfg5b16   the other BASELINE configs (tools/configs_bench.sh's arguments)
# Output under gpurun_out/ (cfg/TAG_*/ per configuration).  The first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for st in "$@"; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/${TAG}_pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    micro)
      timeout -k 10 120 ./tools/bin/mfma_rate > gpurun_out/${TAG}_mfma_rate.txt 2>&1
      rc=$?; echo "micro rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    head) A="" ;;
    4k) A="--height 2160 --width 3840 --frames 16 --no-north-star --no-host-path" ;;
    cfg1) A="--height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0 --no-cpu-baseline --no-north-star --no-host-path" ;;
    cfg3) A="--height 2160 --width 3840 --frames 16 --quality 10 --no-cpu-baseline --no-north-star --no-host-path" ;;
    cfg5b8) A="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --no-cpu-baseline --no-north-star --no-host-path" ;;
    cfg5b16) A="--height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16 --no-cpu-baseline --no-north-star --no-host-path" ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
  case $st in
    tests|micro) ;;
    *)
      timeout -k 10 900 bash tools/profile_cfg.sh ${TAG}_$st $A > gpurun_out/${TAG}_$st.log 2>&1
      rc=$?; echo "$st rc=$rc"; tail -2 gpurun_out/${TAG}_$st.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
echo done
