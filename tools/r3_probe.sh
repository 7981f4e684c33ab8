#!/bin/bash
# Round-3 probe session: MFMA vs VALU issue rates (tools/microbench/mfma_rate.hip),
# kernel times of the probe / A-B library variants in tools/bin/ab (var_prof.sh),
# and dynamic instruction counts (PMC) of the headline kernels per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r3p}
VARS=${VARS:-base s1 nostats norare nostore col16int}
if [ -x tools/bin/mfma_rate ] && [ -z "${NO_MB:-}" ]; then
  timeout -k 10 120 tools/bin/mfma_rate > gpurun_out/mfma_rate_$TAG.txt 2>&1; rc=$?; cat gpurun_out/mfma_rate_$TAG.txt
  [ $rc -eq 0 ] || exit $rc
fi
bash tools/var_prof.sh $VARS || exit 1
for v in $VARS; do
  lib=$ROOT/tools/bin/ab/libjds_$v.so; [ $v = base ] && lib=$ROOT/jpeg-dsp-studio_amd/jds/libjds.so
  (cd /tmp && JDS_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 -d "$ROOT/gpurun_out/pmcv_${TAG}_$v" -o run \
    --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-north-star --no-parity \
    --no-entropy --no-host-path > "$ROOT/gpurun_out/pmcv_${TAG}_$v.log" 2>&1); rc=$?
  case $rc in 0|1) ;; *) echo "pmc $v rc=$rc"; exit $rc;; esac
  python3 - "$ROOT/gpurun_out/pmcv_${TAG}_$v" "$v" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    if 'k_fwd32i' in k or 'k_inv_fast' in k or 'k_fix_fwd' in k:
        m = {c: sum(v) / len(v) for c, v in d.items()}
        w = max(1.0, m.get('SQ_WAVES', 1))
        print(sys.argv[2], k.replace('void jds::', '')[:26], 'waves', int(w), ' '.join(
            f"{c.replace('SQ_INSTS_', '')}={m[c] / w:.1f}" for c in sorted(m) if c != 'SQ_WAVES'))
PY
done
echo done
