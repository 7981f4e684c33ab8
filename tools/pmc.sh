#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 --pmc pass per counter group;
# kernel-trace only, never combined with sys/runtime traces).  Output: gpurun_out/pmc/<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity}"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$ROOT/gpurun_out/pmc/counters_list.txt" 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/gpurun_out/pmc/p$i" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD
FETCH_SIZE GRBM_GUI_ACTIVE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
echo pmc-done
