#!/bin/bash
# Build the round-4 A/B variant libraries (CPU side; the .so files travel with the tree).
set -e
cd "$(dirname "$0")/.."
rm -f tools/bin/ab/*.so tools/bin/ab/*.o
for v in NOCHAIN NOFILL NOMAP; do
  python3 tools/build_variant.py ssim_$v "-DJDS_SSIM_PROBE_$v" jds_ssim_band.hip
done
