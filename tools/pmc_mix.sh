#!/bin/bash
# Instruction-mix PMC passes (one rocprofv3 --pmc pass per group, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out/pmcmix; export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy}"
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/gpurun_out/pmcmix/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/gpurun_out/pmcmix/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done <<'GROUPS'
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32
SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_WAVES
GROUPS
cd "$ROOT" && python3 tools/pmc_report.py gpurun_out/pmcmix > gpurun_out/pmcmix/report.txt
echo pmc-done
