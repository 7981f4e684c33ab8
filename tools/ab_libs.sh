#!/bin/bash
# Same-box A/B of library variants on the headline bench line (kernel legs only).
# usage: tools/ab_libs.sh TAG "lib1 lib2 ..." [bench args...]   (lib "default" = jds/libjds.so;
# others are paths under tools/bin/ab/).  Two interleaved passes; prints value and per-kernel ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; LIBS=$2; shift 2
for pass in 1 2; do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-north-star --no-host-path --no-entropy \
      --no-cpu-baseline --no-parity "$@" > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}.err \
      || { echo "rc=$? $lib"; tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json'))
print('$pass', '$lib'.split('/')[-1], d['value'], d['ms_per_step'], d['kernels_ms'], d.get('fixups_last_step'))" | tee -a gpurun_out/${TAG}.txt
  done
done
