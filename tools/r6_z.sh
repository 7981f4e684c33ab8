#!/bin/bash
# timing probe: k_fix_fwd's launch and statistics-reduction role without the fix-ups
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TESTS=0 bash tools/r6_ab.sh r06_z "default tools/bin/ab/libjds_nofix.so" || exit 1
echo z-done
