#!/bin/bash
# Round-6 PMC passes of the headline kernels at a bench configuration (VERDICT r05
# item 1): instruction mix by class, the wave-cycle split (active / dependency
# wait / parked), VALU and LDS activity, LDS bank conflicts, HBM bytes; one
# rocprofv3 --pmc pass per group (kernel trace only), each under its own limit.
# Then tools/pmc_report.py + tools/valu_roofline.py on the passes.
# usage: r6_pmc.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG="${1:-r06_pmc}"; shift || true
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
  case $rc in 124|134|137|139) exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32
SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
FETCH_SIZE GRBM_GUI_ACTIVE
WRITE_SIZE
GROUPS
cd "$ROOT" && python3 tools/pmc_report.py $OUT > $OUT/report.txt && python3 tools/valu_roofline.py $OUT > $OUT/valu.txt
echo pmc-done
