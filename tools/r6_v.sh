#!/bin/bash
# PMC passes over the entropy coder's kernels (bench's entropy leg, 64 x 1080p Q50)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash tools/r6_pmc.sh r06_ent_pmc --steps 2 --warmup 1 --no-cpu-baseline --no-north-star --no-parity --no-host-path || exit 1
echo v-done
