#!/bin/bash
# Round-6 closing, part 2: every BASELINE config through bench.py, the headline
# line again (its roofline citing the r06_final counters), and the PMC passes at
# the north-star configuration (16 x 4K).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash tools/configs_bench.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r06_final2_bench.json 2> gpurun_out/r06_final2_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_final2_bench.err; exit $rc; }
bash tools/r6_pmc.sh r06_final_4k_pmc --steps 3 --warmup 1 --height 2160 --width 3840 --frames 16 --no-cpu-baseline \
  --no-north-star --no-parity --no-entropy --no-host-path || exit 1
echo final2-done
