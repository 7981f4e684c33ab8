#!/bin/bash
# Round-3 closing session: every -m gpu test, smoke, the default bench with
# rocprofv3 kernel stats (headline + north-star point), the 2-rank gloo
# rehearsal, then the headline and north-star configurations with FETCH_SIZE /
# WRITE_SIZE passes (tools/profile_cfg.sh) for profiles/pmc_traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r3final}
TAG=$TAG STEPS="tests smoke bench prof rehearse" bash tools/r3_check.sh || exit $?
bash tools/profile_cfg.sh ${TAG}_hd > gpurun_out/pcfg_hd.log 2>&1 || { tail -3 gpurun_out/pcfg_hd.log; exit 1; }
tail -1 gpurun_out/pcfg_hd.log
bash tools/profile_cfg.sh ${TAG}_4k --height 2160 --width 3840 --frames 16 > gpurun_out/pcfg_4k.log 2>&1 || { tail -3 gpurun_out/pcfg_4k.log; exit 1; }
tail -1 gpurun_out/pcfg_4k.log
echo final-done
