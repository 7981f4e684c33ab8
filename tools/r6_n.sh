#!/bin/bash
# timing probes of k_inv_fast<4:2:0>: without the chroma ring blocks, without any chroma block
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TESTS=0 NS=0 bash tools/r6_ab.sh r06_n "default tools/bin/ab/libjds_noring.so tools/bin/ab/libjds_nochroma.so" || exit 1
echo n-done
