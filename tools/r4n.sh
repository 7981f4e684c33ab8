#!/bin/bash
# 4K Q10: the certified inverse forced (how many tiles fall back), against the plan's default
set -u
cd "${GRAFT_REPO_ROOT}"
for f in "" "--inv-fast"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-entropy --height 2160 --width 3840 --frames 16 --quality 10 --no-cpu-baseline --no-north-star --no-host-path $f > gpurun_out/r4n.json 2> gpurun_out/r4n.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r4n.json'));print('$f', d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('fixups_last_step'))"
done
