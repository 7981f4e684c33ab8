#!/bin/bash
# Two PMC passes (instruction counts + active cycles) over a short bench run; per-kernel report.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=gpurun_out/${PMC_TAG:-pmcutil}; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-entropy --no-host-path}"
cd /tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/$OUT/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD
GROUPS
cd "$ROOT" && python3 tools/pmc_report.py $OUT > $OUT/report.txt; grep -A2 "k_inv_fast\|k_fwd32i" $OUT/report.txt
