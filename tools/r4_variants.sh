#!/bin/bash
# Build the round-4 A/B variant libraries (CPU side; the .so files travel with the tree).
set -e
cd "$(dirname "$0")/.."
rm -f tools/bin/ab/*.so tools/bin/ab/*.o
python3 tools/build_variant.py A "" jds_entropy.hip
python3 tools/build_variant.py L0 "-DJDS_ENT_LEFT=0" jds_entropy.hip
python3 tools/build_variant.py S0 "-DJDS_ENT_SPLIT=0" jds_entropy.hip
