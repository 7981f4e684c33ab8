#!/bin/bash
# Every BASELINE config through bench.py (each under its own limit); JSON lines to gpurun_out/cfg_*.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-entropy "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err
  local rc=$?
  python3 -c "import json;d=json.load(open('gpurun_out/cfg_$name.json'));print('$name', d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('parity'))" || true
  return $rc
}
run cfg1_512_444 --height 512 --width 512 --frames 256 --mode 4:4:4 --prefilter 0 --no-cpu-baseline --no-north-star && \
run cfg3_4k_q10_420 --height 2160 --width 3840 --frames 16 --quality 10 --no-cpu-baseline --no-north-star && \
run cfg5_4k_422_b8 --height 2160 --width 3840 --frames 16 --mode 4:2:2 --no-cpu-baseline --no-north-star && \
run cfg5_4k_422_b16 --height 2160 --width 3840 --frames 16 --mode 4:2:2 --block 16 --no-cpu-baseline --no-north-star
