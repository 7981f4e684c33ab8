#!/bin/bash
# Build the round-4 A/B variant libraries (CPU side; the .so files travel with the tree).
# H: the committed entropy source (git HEAD) for a same-box comparison.
set -e
cd "$(dirname "$0")/.."
rm -f tools/bin/ab/*.so tools/bin/ab/*.o
python3 tools/build_variant.py A "" jds_entropy.hip
python3 tools/build_variant.py S0 "-DJDS_ENT_SPLIT=0" jds_entropy.hip
git show HEAD:jpeg-dsp-studio_amd/csrc/jds_entropy.hip > /tmp/ent_head.hip
O=jpeg-dsp-studio_amd/jds/_obj
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -c -fno-slp-vectorize -ffp-contract=off -w \
  -Iinclude -Ijpeg-dsp-studio_amd/csrc -o tools/bin/ab/H_jds_entropy.hip.o /tmp/ent_head.hip
objs=""
for f in $(python3 -c "import sys; sys.path.insert(0,'jpeg-dsp-studio_amd'); from jds import build as B; print(' '.join(B.SOURCES))"); do
  if [ "$f" = jds_entropy.hip ]; then objs="$objs tools/bin/ab/H_jds_entropy.hip.o"; else objs="$objs $O/$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/ab/libjds_H.so $objs
echo tools/bin/ab/libjds_H.so
