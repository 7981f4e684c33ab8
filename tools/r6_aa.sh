#!/bin/bash
# timing probes of k_fix_fwd's per-block work: without the sampling, without the transforms, without both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TESTS=0 NS=0 bash tools/r6_ab.sh r06_aa "default tools/bin/ab/libjds_nosample.so tools/bin/ab/libjds_nodct.so tools/bin/ab/libjds_noboth.so" || exit 1
echo aa-done
