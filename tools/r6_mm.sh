#!/bin/bash
# LLVM's max-ilp machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp) per
# translation unit: the inverse unit (bit-exactness tests, then headline and
# 4K A/B), the SSIM unit (384-pair batch) and the entropy unit (ent_probe, file digest)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_inv_maxilp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "inv or parity or plan" > gpurun_out/r06_mm_pytest.log 2>&1
rc=$?; echo "pytest(inv_maxilp) rc=$rc"; tail -2 gpurun_out/r06_mm_pytest.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 bash tools/r6_ab.sh r06_mm "default tools/bin/ab/libjds_inv_maxilp.so" || exit 1
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ssim_maxilp.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; BATCH=384 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-150 || exit 1
  done
done | tee gpurun_out/r06_mm_ssim.txt
for pass in 1 2 3; do
  for lib in default tools/bin/ab/libjds_ent_maxilp.so tools/bin/ab/libjds_ent_itilp.so; do
    if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
    echo -n "$pass $(basename $lib) "; timeout -k 10 200 python -u tools/ent_probe.py 2>/dev/null | cut -c1-200 || exit 1
  done
done | tee gpurun_out/r06_mm_ent.txt
echo mm-done
