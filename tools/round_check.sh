#!/bin/bash
# Full GPU session: all -m gpu tests, smoke, default bench (all legs), sweep bench,
# rocprofv3 kernel stats of the default bench.  Each step under its own limit;
# a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-rc}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', d['value'], d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'], d['fixups_last_step'])"
timeout -k 10 300 python bench.py --sweep --no-cpu-baseline --no-north-star > gpurun_out/sweep_$TAG.json 2> gpurun_out/sweep_$TAG.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep_$TAG.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/sweep_$TAG.json'));print('sweep', d['value'], d['ms_per_step'], d.get('parity'))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-north-star --no-entropy --no-host-path --no-parity > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit $rc; }
echo done
