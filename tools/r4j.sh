#!/bin/bash
# entropy variants (ms per 64 x 1080p batch)
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_entropy.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4j_pytest.log; [ $rc -eq 0 ] || exit $rc
for L in A P3 P5 P6 A P3 P5 P6; do
  REPS=200 JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_$L.so timeout -k 10 120 python tools/ent_probe.py 2>/dev/null || exit $?
done | tee gpurun_out/r4j_ab.jsonl
