#!/bin/bash
# VALU-roofline PMC passes over a short bench run (one rocprofv3 --pmc pass per group,
# kernel trace only; each pass its own time limit), then tools/valu_roofline.py.
# usage: r4_pmc.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG="${1:-pmcv}"; shift || true
ARGS="${*:---steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy --no-host-path}"
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/$OUT/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32
SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU SQ_WAVES
GROUPS
cd "$ROOT" && python3 tools/pmc_report.py $OUT > $OUT/report.txt && python3 tools/valu_roofline.py $OUT
echo pmc-done
