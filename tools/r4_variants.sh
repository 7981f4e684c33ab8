#!/bin/bash
# Build the round-4 A/B variant libraries (CPU side; the .so files travel with the tree).
set -e
cd "$(dirname "$0")/.."
rm -f tools/bin/ab/*.so tools/bin/ab/*.o
python3 tools/build_variant.py A "" jds_entropy.hip
python3 tools/build_variant.py P3 "-DJDS_ENT_WPE=3" jds_entropy.hip
python3 tools/build_variant.py P5 "-DJDS_ENT_WPE=5" jds_entropy.hip
python3 tools/build_variant.py P6 "-DJDS_ENT_WPE=6" jds_entropy.hip
