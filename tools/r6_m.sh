#!/bin/bash
# PMC record of k_inv_fast6 at 6 waves per SIMD (libjds_v4w6) for the occupancy / spill evidence
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
JDS_LIB_PATH=$PWD/tools/bin/ab/libjds_v4w6.so bash tools/r6_pmc.sh r06_m_pmc_v4w6 || exit 1
echo m-done
