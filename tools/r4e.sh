set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssim.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4e_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4e_pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in default tools/bin/ab/libjds_ssim_NOCHAIN.so tools/bin/ab/libjds_ssim_NOFILL.so tools/bin/ab/libjds_ssim_NOMAP.so; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
  echo -n "$lib "; LEGACY=0 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-110
done
unset JDS_LIB_PATH
bash tools/r4_check.sh r4e ssimprof
