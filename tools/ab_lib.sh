#!/bin/bash
# A/B two builds of libjds.so (tools/bin/ab/libjds_A.so vs _B.so) with tools/ab_probe.py, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for v in A B; do
    echo -n "$v: "; JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$v.so timeout -k 10 200 python tools/ab_probe.py ${VARIANTS:-serial} | tail -1 || exit $?
  done
done
