#!/bin/bash
# GPU parity tests + a steady-state bench line (each under its own limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --no-entropy ${BENCH_ARGS:-} > gpurun_out/quick.json 2>gpurun_out/quick.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/quick.err; exit $rc; }
python3 -c "import json;d=json.load(open('gpurun_out/quick.json'));print(d['value'], d['ms_per_step'], d['kernels_ms'], d.get('parity'))"
