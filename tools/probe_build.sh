#!/bin/bash
# Build the timing-probe variants into tools/bin (cross-compiled here, run on the GPU box).
set -e
cd "$(dirname "$0")"
for v in ${VARIANTS:-base:"" noload:-DJDS_PROBE_NOLOAD nostore:-DJDS_PROBE_NOSTORE s1:-DJDS_PROBE_STAGE1 s2:-DJDS_PROBE_STAGE2 s1nl:"-DJDS_PROBE_STAGE1 -DJDS_PROBE_NOLOAD"}; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -w -std=c++17 -O3 --offload-arch=gfx950 -I ../include -fno-slp-vectorize $EXTRA $flags probe_fwd.cpp -o bin/probe_$name &
done
wait
ls -la bin
