#!/bin/bash
# Bench line per library variant (tools/bin/ab/libjds_<name>.so; "base" = the
# in-tree build), no parity/CPU legs: kernels_ms and ms_per_step side by side.
# Usage: BENCH_ARGS="..." tools/var_bench.sh name [name ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in "$@"; do
  lib=$PWD/tools/bin/ab/libjds_$v.so; [ "$v" = base ] && lib=$PWD/jpeg-dsp-studio_amd/jds/libjds.so
  JDS_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-north-star --no-entropy --no-host-path --no-parity \
    ${BENCH_ARGS:-} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "$v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/var_$v.json'));print('$v', d['ms_per_step'], d['kernels_ms'], d.get('fixups_last_step'))"
done
