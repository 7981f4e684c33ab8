#!/bin/bash
# Build the round-4 A/B variant libraries (CPU side; the .so files travel with the tree).
set -e
cd "$(dirname "$0")/.."
python3 tools/build_variant.py ent_old "-DJDS_ENT_BITS_TABLE=0 -DJDS_ENT_PACK_TABLE=0" jds_entropy.hip
python3 tools/build_variant.py ent_bits "-DJDS_ENT_BITS_TABLE=1 -DJDS_ENT_PACK_TABLE=0" jds_entropy.hip
python3 tools/build_variant.py ssim_bh16 "-DJDS_SSIM_BH=16" jds_ssim_band.hip
