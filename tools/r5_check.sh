#!/bin/bash
# Round 5 GPU check.  usage: r5_check.sh TAG [stages...]
#   tests    the whole -m gpu suite (one process, per-test time limit)
#   quick    the parity-critical GPU tests only (plan 4K/cfg2 goldens, inverse, entropy, ssim)
#   bench    bench.py default line (all legs) -> gpurun_out/TAG_bench.json
#   cfg      tools/profile_cfg.sh on the headline: bench + rocprofv3 stats + FETCH / WRITE passes
#   cfg4k    the same at the north-star point (16 x 4K Q50 4:2:0)
#   sweep    bench.py --sweep
#   ent4k    entropy probe on 16 x 4K frames
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-r5}"; shift || true
STAGES="${*:-tests bench}"
has() { case " $STAGES " in *" $1 "*) return 0;; *) return 1;; esac; }
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if has quick; then
  timeout -k 10 900 python -u -m pytest ${QUICK_TESTS:-tests/test_gpu_plan_4k.py tests/test_gpu_inv_fast.py tests/test_gpu_entropy.py \
    tests/test_gpu_ssim.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_quick.log 2>&1
  rc=$?; echo "quick rc=$rc"; tail -4 gpurun_out/${TAG}_quick.log; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json'))
r=d['roofline']; p=d.get('kernels_profile') or {}
print('value',d['value'],'ms',d['ms_per_step'],'pipe',d['pipeline_roofline_frac'],'kernel',r['kernel'],r['avg_launch_ms'],'frac',r['frac'],'traffic',r['traffic'])
print('kernels',d['kernels_ms'],'profiled',p.get('profiled_step_ms'),'sum',p.get('sum_ms'))
print('ent',d.get('entropy',{}).get('ms_per_step'),'host',d.get('host_path',{}).get('ms_per_frame'))
print('ns',d.get('north_star',{}).get('value'),d.get('north_star',{}).get('pipeline_roofline_frac'),'parity',d.get('parity'),d.get('parity_ranks',{}).get('all_exact'))
"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
fi
if has cfg; then
  timeout -k 10 900 bash tools/profile_cfg.sh ${TAG}_1080p > gpurun_out/${TAG}_cfg.log 2>&1
  rc=$?; echo "cfg rc=$rc"; tail -3 gpurun_out/${TAG}_cfg.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
if has cfg4k; then
  timeout -k 10 900 bash tools/profile_cfg.sh ${TAG}_4k_q50_420 --height 2160 --width 3840 --frames 16 --no-north-star \
    --no-host-path > gpurun_out/${TAG}_cfg4k.log 2>&1
  rc=$?; echo "cfg4k rc=$rc"; tail -3 gpurun_out/${TAG}_cfg4k.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
if has q10; then
  # configs[2] (16 x 4K Q10 4:2:0): the plan default (k_inv2 at this table) vs the certified fast inverse vs k_inv2 asked for
  for v in default --inv-fast --exact-inv; do
    a=$v; [ "$v" = default ] && a=""
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --height 2160 --width 3840 --frames 16 --quality 10 \
      --prefilter 0 --no-north-star --no-host-path --no-entropy --no-cpu-baseline $a >> gpurun_out/${TAG}_q10.jsonl \
      2>> gpurun_out/${TAG}_q10.err
    rc=$?; [ $rc -eq 0 ] || { echo "q10 $v rc=$rc"; tail -5 gpurun_out/${TAG}_q10.err; exit $rc; }
  done
  python3 -c "
import json
for l in open('gpurun_out/${TAG}_q10.jsonl'):
    d=json.loads(l); print(d['value'], d['ms_per_step'], d['pipeline_roofline_frac'], d['kernels_ms'], d['fixups_last_step'], d['parity'])
"
fi
if has sweep; then
  timeout -k 10 600 python -u bench.py --sweep --steps 10 --warmup 3 > gpurun_out/${TAG}_sweep.json 2> gpurun_out/${TAG}_sweep.err
  rc=$?; echo "sweep rc=$rc"; head -c 1500 gpurun_out/${TAG}_sweep.json; echo; [ $rc -eq 0 ] || exit $rc
fi
if has ent4k; then
  for lib in default ${ENT_LIBS:-}; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    for geo in 1080x1920x64 2160x3840x16; do
      IFS=x read -r h w f <<< "$geo"
      HEIGHT=$h WIDTH=$w FRAMES=$f REPS=50 timeout -k 10 200 python -u tools/ent_probe.py >> gpurun_out/${TAG}_ent.jsonl \
        2>> gpurun_out/${TAG}_ent.err
      rc=$?; [ $rc -eq 0 ] || { echo "ent probe rc=$rc"; tail -5 gpurun_out/${TAG}_ent.err; exit $rc; }
    done
  done
  unset JDS_LIB_PATH; cat gpurun_out/${TAG}_ent.jsonl
fi
echo done
