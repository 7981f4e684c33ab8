#!/bin/bash
# entropy walk: put() without the divergent branch (entbf) vs the shipped one; the digests must agree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_entbf.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python -u tools/ent_probe.py > gpurun_out/r06_w_one.json 2>> gpurun_out/r06_w.err || { echo "rc=$? $lib"; tail -5 gpurun_out/r06_w.err; exit 1; }
    echo "$pass $(basename $lib) $(tail -1 gpurun_out/r06_w_one.json)" | tee -a gpurun_out/r06_w.txt
  done
done
echo w-done
