#!/bin/bash
# Q10 4K inverse A/B over variant libraries (timing probes; parity is not checked for probe builds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${1:-q10ab}
for lib in default tools/bin/ab/libjds_nofb.so tools/bin/ab/libjds_norare.so tools/bin/ab/libjds_norare_nofb.so; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
  for v in default --inv-fast; do
    a=$v; [ "$v" = default ] && a=""
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --height 2160 --width 3840 --frames 16 --quality 10 \
      --prefilter 0 --no-north-star --no-host-path --no-entropy --no-cpu-baseline --no-parity $a > gpurun_out/${TAG}_one.json \
      2>> gpurun_out/${TAG}.err || { echo "rc=$? $lib $v"; tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); print('$lib', '$v', d['kernels_ms'], d['fixups_last_step'])" | tee -a gpurun_out/${TAG}.txt
  done
done
