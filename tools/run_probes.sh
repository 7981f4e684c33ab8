#!/bin/bash
# Run the prebuilt timing probes (tools/bin/probe_*) one after another, each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${PROBES:-tools/bin/probe_*}; do
  echo "== $b"
  timeout -k 10 60 "$b" > "gpurun_out/$(basename "$b").txt" 2>&1
  rc=$?; cat "gpurun_out/$(basename "$b").txt"
  [ $rc -eq 0 ] || { echo "stopping: rc=$rc"; exit $rc; }
done
