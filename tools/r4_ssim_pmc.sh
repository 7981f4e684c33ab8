#!/bin/bash
# PMC passes over tools/ssim_probe.py (K4 kernels), one --pmc pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=gpurun_out/${1:-ssimpmc}; mkdir -p $OUT; export TMPDIR=/tmp REPS=4
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/$OUT/p$i" -o run --output-format csv \
    -- python3 "$ROOT/tools/ssim_probe.py" > "$ROOT/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32
GROUPS
cd "$ROOT" && python3 tools/pmc_report.py $OUT > $OUT/report.txt && python3 tools/valu_roofline.py $OUT; grep -A2 "k_ss" $OUT/report.txt
