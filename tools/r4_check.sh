#!/bin/bash
# Round 4 check: SSIM + entropy GPU tests, SSIM probe, bench (full legs), rocprof kernel stats of the bench.
# usage: r4_check.sh TAG [tests|probe|bench|prof ...]  (default: all)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${1:-r4}"; shift || true
STAGES="${*:-tests probe bench prof}"
has() { case " $STAGES " in *" $1 "*) return 0;; *) return 1;; esac; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ssim.py tests/test_gpu_entropy.py tests/test_gpu_sweep_plan.py \
    tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if has probe; then
  timeout -k 10 300 python -u tools/ssim_probe.py > gpurun_out/${TAG}_ssim_probe.json 2> gpurun_out/${TAG}_ssim_probe.err
  rc=$?; echo "probe rc=$rc"; cat gpurun_out/${TAG}_ssim_probe.json; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'],'pipe',d['pipeline_roofline_frac'])
print('kernels',d['kernels_ms'],'ent',d.get('entropy',{}).get('ms_per_step'),'host',d.get('host_path',{}).get('ms_per_frame'))
print('ns',d.get('north_star',{}).get('value'),d.get('north_star',{}).get('pipeline_roofline_frac'),'parity',d.get('parity'),d.get('parity_ranks',{}).get('all_exact'))
"; [ $rc -eq 0 ] || exit $rc
fi
if has sweep; then
  timeout -k 10 600 python -u bench.py --sweep --steps 10 --warmup 3 > gpurun_out/${TAG}_sweep.json 2> gpurun_out/${TAG}_sweep.err
  rc=$?; echo "sweep rc=$rc"; head -c 1500 gpurun_out/${TAG}_sweep.json; echo; [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity \
    > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_kernel_stats.csv
  cut -d, -f1-4 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-140 | head -30
fi
if has pmc; then
  timeout -k 10 700 bash tools/r4_pmc.sh ${TAG}_pmc > gpurun_out/${TAG}_pmc.log 2>&1
  rc=$?; echo "pmc rc=$rc"; tail -12 gpurun_out/${TAG}_pmc.log; [ $rc -eq 0 ] || exit $rc
fi
if has rehearse; then
  timeout -k 10 700 bash tools/rehearse_ranks.sh > gpurun_out/${TAG}_rehearse.log 2>&1
  rc=$?; echo "rehearse rc=$rc"; cut -c1-300 gpurun_out/${TAG}_rehearse.log | tail -4; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/rehearse_main.json gpurun_out/${TAG}_rehearse_main.json; cp gpurun_out/rehearse_sweep.json gpurun_out/${TAG}_rehearse_sweep.json
fi
if has ab; then
  for lib in default tools/bin/ab/libjds_ent_old.so tools/bin/ab/libjds_ent_bits.so default; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python -u tools/ent_probe.py >> gpurun_out/${TAG}_ent_ab.jsonl 2>> gpurun_out/${TAG}_ent_ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "ent probe rc=$rc"; exit $rc; }
  done
  unset JDS_LIB_PATH; cat gpurun_out/${TAG}_ent_ab.jsonl
  for lib in default tools/bin/ab/libjds_ssim_bh16.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    LEGACY=0 timeout -k 10 200 python -u tools/ssim_probe.py >> gpurun_out/${TAG}_ssim_ab.jsonl 2>> gpurun_out/${TAG}_ssim_ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "ssim probe rc=$rc"; exit $rc; }
  done
  unset JDS_LIB_PATH; cut -c1-200 gpurun_out/${TAG}_ssim_ab.jsonl
fi
if has pmc4k; then
  timeout -k 10 700 bash tools/r4_pmc.sh ${TAG}_pmc4k --height 2160 --width 3840 --frames 16 --steps 3 --warmup 1 \
    --no-cpu-baseline --no-north-star --no-parity --no-entropy --no-host-path > gpurun_out/${TAG}_pmc4k.log 2>&1
  rc=$?; echo "pmc4k rc=$rc"; tail -8 gpurun_out/${TAG}_pmc4k.log; [ $rc -eq 0 ] || exit $rc
fi
if has ssimprof; then
  cd /tmp
  LEGACY=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_ssimprof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/ssim_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_ssimprof.log" 2>&1
  rc=$?; echo "ssimprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$GRAFT_REPO_ROOT"
fi
echo done
