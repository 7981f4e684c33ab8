#!/bin/bash
# r6 A/B: the -m gpu suite on the product library (optional, TESTS=1), then
# interleaved library variants on the headline (1080p) and north-star (4K) lines.
# usage: r6_ab.sh TAG "lib1 lib2 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=$1; LIBS=$2
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
bash tools/ab_libs.sh ${TAG}_1080 "$LIBS" || exit 1
if [ "${NS:-1}" = 1 ]; then
  bash tools/ab_libs.sh ${TAG}_4k "$LIBS" --height 2160 --width 3840 --frames 16 || exit 1
fi
echo ab-done
