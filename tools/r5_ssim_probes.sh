cd "${GRAFT_REPO_ROOT}"
for lib in default ${SSIM_LIBS:-tools/bin/ab/libjds_ssim_NOCHAIN.so tools/bin/ab/libjds_ssim_NOFILL.so tools/bin/ab/libjds_ssim_NOMAP.so}; do
  if [ "$lib" = default ]; then unset JDS_LIB_PATH; else export JDS_LIB_PATH=$PWD/$lib; fi
  echo -n "$lib "; BATCH=18 REPS=4 timeout -k 10 200 python -u tools/ssim_probe.py 2>/dev/null | cut -c1-120 || exit 1
done
