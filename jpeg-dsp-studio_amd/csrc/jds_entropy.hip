// jds_entropy.hip — baseline JPEG entropy coding of the quantised coefficients
// (SURVEY.md §8(f)4).  The reference stops at a size estimate
// (utils/metrics.py:51-92, "no entropy coding") and keeps the zigzag order
// unused (utils/constants.py:18-27); this turns its all_quantized_coeffs
// (engines/pipeline.py:56,99) into a standard JFIF file per frame: one
// quantisation table (all planes use the luma table, pipeline.py:43), the
// T.81 Annex K standard Huffman tables, three non-interleaved scans (Y, Cb,
// Cr; a non-interleaved scan's raster block order is exactly the reference's
// block order).  Byte-for-byte definition: oracle/jpeg_entropy.py.
//
// Integer / byte work.  Pipeline per batch of frames (segments = 64
// consecutive blocks of one scan, one wave each; DESIGN.md §4 "Round 4: one
// pass"):
//   k_ent_walk   each lane codes its block (zigzag walk, T.81 Annex K tables,
//                left-aligned symbols appended by funnel shifts) into staging
//                words; per-lane bit counts and per-segment totals.
//   k_ent_place  each segment's bit offset within its scan (the sum of the
//                scan's earlier segment totals); each lane's words shifted into place in the packed scan
//                (shared words combined by a segmented OR across the wave,
//                the word shared with the next segment completed from that
//                segment's leading bits), the scan's pad bits, the 0xFF bytes
//                per segment.
//   k_ent_fscan  per frame: 0xFF prefixes, every segment's output offset, the
//                headers (host-built template: SOI, APP0, DQT, SOF0, DHT),
//                the three SOS markers, EOI, file length.
//   k_ent_emit3  stuffed copy to the file (0x00 after every 0xFF).
// (The rounds 1-3 multi-pass coder -- a counting walk, a block scan, a packing
// walk with LDS atomics, per-chunk stuffing -- measured 0.54 ms per 64 x 1080p
// against this one's 0.30, and a one-launch form with a decoupled look-back
// 0.386 ms; both are retired, their A/Bs are in DESIGN.md §4.)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <initializer_list>

#include "jds_internal.hpp"

namespace jds {

// ------------------------------------------------------------ tables --

// T.81 Annex K.3 (tables K.3 - K.6): BITS[1..16] and HUFFVAL
static const uint8_t K3_BITS[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t K4_BITS[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t DC_VALS[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t K5_BITS[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t K5_VALS[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
static const uint8_t K6_BITS[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t K6_VALS[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
// utils/constants.py:18-27: row-major index of the k-th zigzag coefficient
static const uint8_t ZZ[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Code tables as (length << 16 | code): [0] luma, [1] chroma.
struct EntTab {
  uint32_t dc[2][16];
  uint32_t ac[2][256];
  uint8_t zz[64];
};

// left-aligned symbols: code << (32 - len) | len (len <= 16 sits below the code)
// AC table row stride: (run, size) at run * 11 + size spreads a wave's lookups
// over the LDS banks (32: 0.271 vs 11: 0.258 ms per 64 x 1080p; a stride of 32
// put every even run on the same 11 banks)
constexpr int ES_RS = 11;
static_assert(ES_RS >= 11, "sizes 0..10");
struct EsTab {
  uint32_t ac[2][16 * ES_RS];  // (run & 15, size) -> AC symbol, size clamped to 10 (code_ac's clamp); 0 for size 0
  uint32_t dc[2][16];
  uint32_t zrl[2], eob[2];
};

__host__ __device__ __forceinline__ uint32_t es_left(uint32_t e) {  // (len << 16 | code) -> left-aligned | len
  const uint32_t len = e >> 16;
  return len ? (((e & 0xFFFFu) << (32u - len)) | len) : 0u;
}

// T.81 Annex C: code lengths and codes in order of increasing length
static void huff_codes(const uint8_t* bits, const uint8_t* vals, uint32_t* out, int nsym) {
  for (int i = 0; i < nsym; ++i) out[i] = 0;
  uint32_t code = 0;
  int k = 0;
  for (int len = 1; len <= 16; ++len) {
    for (int i = 0; i < bits[len - 1]; ++i, ++k) out[vals[k]] = ((uint32_t)len << 16) | code++;
    code <<= 1;
  }
}

void ent_build_tables(EntTab* t) {
  memset(t, 0, sizeof *t);
  huff_codes(K3_BITS, DC_VALS, t->dc[0], 16);
  huff_codes(K4_BITS, DC_VALS, t->dc[1], 16);
  huff_codes(K5_BITS, K5_VALS, t->ac[0], 256);
  huff_codes(K6_BITS, K6_VALS, t->ac[1], 256);
  memcpy(t->zz, ZZ, 64);
  // the single-pass coder's left-aligned symbols follow the table (ent_tab_size)
  EsTab* es = reinterpret_cast<EsTab*>(t + 1);
  for (int c = 0; c < 2; ++c) {
    for (int i = 0; i < 16 * ES_RS; ++i) {
      const int run = i / ES_RS, sz = i % ES_RS;
      es->ac[c][i] = sz ? es_left(t->ac[c][(run << 4) | (sz > 10 ? 10 : sz)]) : 0u;
    }
    for (int i = 0; i < 16; ++i) es->dc[c][i] = es_left(t->dc[c][i]);
    es->zrl[c] = es_left(t->ac[c][0xF0]);
    es->eob[c] = es_left(t->ac[c][0x00]);
  }
}

size_t ent_tab_size() { return sizeof(EntTab) + sizeof(EsTab); }

// JFIF header template (oracle/jpeg_entropy.py::jfif_headers): returns its length
// (ENT_HDR bytes) or -1 if the table is not baseline (integers in [1, 255]).
constexpr int ENT_HDR = 2 + 18 + 69 + 19 + 2 * (4 + 1 + 16 + 12) + 2 * (4 + 1 + 16 + 162);
constexpr int ENT_SOS = 10;

int ent_header(const double* q, int mode, int H, int W, uint8_t* o) {
  int p = 0;
  auto put = [&](std::initializer_list<int> b) {
    for (int v : b) o[p++] = (uint8_t)v;
  };
  put({0xFF, 0xD8});
  put({0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0});
  put({0xFF, 0xDB, 0x00, 0x43, 0x00});
  for (int k = 0; k < 64; ++k) {
    const double v = q[ZZ[k]];
    if (!(v >= 1.0 && v <= 255.0) || v != (double)(int)v) return -1;
    o[p++] = (uint8_t)(int)v;
  }
  const int smp = mode == M420 ? 0x22 : (mode == M422 ? 0x21 : 0x11);
  put({0xFF, 0xC0, 0x00, 0x11, 0x08, H >> 8, H & 255, W >> 8, W & 255, 3, 1, smp, 0, 2, 0x11, 0, 3, 0x11, 0});
  const uint8_t* bits[4] = {K3_BITS, K5_BITS, K4_BITS, K6_BITS};
  const uint8_t* vals[4] = {DC_VALS, K5_VALS, DC_VALS, K6_VALS};
  const int nv[4] = {12, 162, 12, 162}, id[4] = {0x00, 0x10, 0x01, 0x11};
  for (int t = 0; t < 4; ++t) {
    const int len = 3 + 16 + nv[t];
    put({0xFF, 0xC4, len >> 8, len & 255, id[t]});
    for (int i = 0; i < 16; ++i) o[p++] = bits[t][i];
    for (int i = 0; i < nv[t]; ++i) o[p++] = vals[t][i];
  }
  return p;
}

// ------------------------------------------------------------ kernels --

struct EntGeo {
  int nb;          // blocks per frame (Y + Cb + Cr)
  int first[4];    // first block of each scan within the frame, first[3] = nb
  int sfirst[4];   // single-pass coder: first 64-block segment of each scan within the frame, sfirst[3] = per frame
  int cap_w[3];    // packed-scan capacity in 32-bit words (worst case 1660 bits per block)
  long long raw_w; // packed words per frame
  long long hdr;   // header template bytes per frame
};

__device__ __forceinline__ long long raw_base(const EntGeo& e, int frame, int s) {
  return (long long)frame * e.raw_w + (s == 0 ? 0 : (s == 1 ? e.cap_w[0] : e.cap_w[0] + e.cap_w[1]));
}

// Inclusive prefix sum over the wave (every lane active): row_shr 1, 2, 4, 8
// within the 16-lane rows, then row_bcast 15 / 31 across them -- six DPP adds
// (the log-step shuffle form, six ds_bpermute round trips, measured slower).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, int lane) {
  (void)lane;
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}

__device__ __forceinline__ int wave_excl_sum(int x, int lane) {
  return (int)(wave_incl_sum((uint32_t)x, lane) - (uint32_t)x);
}

__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// lane l <- lane l + 1 across the whole wave (DPP wave_shl:1; lane 63 <- 0)
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}
// lane l <- lane l - 1 (DPP wave_shr:1; lane 0 <- 0)
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, true); }

// wave-wide totals (every lane active), read from lane 63 of the DPP scan
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return lane63(wave_incl_sum(v, (int)__lane_id())); }

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return lane63(v);
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return lane63(v);
}

// One LANE per block: its 64 coefficients sit in 32 VGPRs (packed int16
// pairs) and the zigzag walk is unrolled at compile time, so every register
// index is a constant; the per-coefficient work is a handful of integer ops
// under the lane's own "nonzero" mask.  (A wave per block, one lane per
// coefficient, spent ~400 wave instructions per block on ballots, shuffles
// and divergent branches.)
struct BlockRegs {
  uint32_t w[32];
};

__device__ __forceinline__ BlockRegs load_block(const int16_t* __restrict__ p) {
  BlockRegs r;
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 x = q[i];
    r.w[4 * i] = x.x; r.w[4 * i + 1] = x.y; r.w[4 * i + 2] = x.z; r.w[4 * i + 3] = x.w;
  }
  return r;
}

template <int IDX>
__device__ __forceinline__ int coef_at(const BlockRegs& r) {
  return (int)(int16_t)((IDX & 1) ? (r.w[IDX >> 1] >> 16) : (r.w[IDX >> 1] & 0xFFFFu));
}

constexpr uint8_t ZZC[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ------------------------------------------------ one pass (round 4) --
//
// Segments of 64 consecutive blocks of one scan, one wave each.
//  * walk (k_ent_walk): each lane packs its block MSB-first into lane-private
//    staging words (LDS, word-major across the wave's lanes so every store hits
//    its own bank; words past ES_SW go to the segment's global rows), so the
//    block's bit count comes out of the same walk that packs it.  Appending a
//    symbol is one shift and one OR on a left-aligned 32-bit pending word.
//  * offset: the segment's bit offset within its scan is the sum of the scan's
//    earlier segment totals (k_ent_place sums them itself for short scans, a
//    per-frame prefix launch gives them for long ones).
//  * placement (k_ent_place): each lane writes its words shifted into place.
//    Words it alone covers: plain stores.  A word shared by several lanes is
//    written once, by the lane holding its first bit, with the others' bits
//    gathered by a segmented OR across the wave; the word a segment shares with
//    the next is completed from the next segment's leading bits.
//  * the 0xFF bytes of every word the segment finalises are counted there,
//    and each scan's last byte is padded with 1-bits (T.81 F.1.2.3), so the
//    stuffing pass reads final words.
// A segment that is not the last of its scan holds >= 256 bits (every block
// costs >= 4), so only consecutive segments share a word.
constexpr int ES_WPE = 4;     // waves per SIMD the walk's registers are held to (3..6: no difference)
constexpr int ES_DENSE = 32;  // zigzag positions coded by the unrolled walk; the rest by the nonzero loop
// LDS staging words per lane (more go to global): 16: 0.303, 0: 0.295, 8: 0.292
// ms per 64 x 1080p (LDS -> 5 workgroups per CU)
constexpr int ES_SW = 8;
constexpr int ES_HI = 64 - ES_DENSE;     // positions of the nonzero loop
static_assert(ES_HI <= 32, "es_hi_stash's nonzero mask is one 32-bit word (ES_DENSE = 24 dropped positions 56-63)");
constexpr int ES_MAXW = 53;              // words per block at most (1660 bits + the partial word): the spill area
#ifndef JDS_ES_WAVES  // tools: A/B builds of the walk's waves per workgroup
#define JDS_ES_WAVES 4
#endif
constexpr int ES_WAVES = JDS_ES_WAVES;

// Append the L (< 32) bits of symL (left-aligned, zero below) to the pending
// word acc (n bits, left-aligned with zeros below: an append is one shift and
// one OR; right-aligned pending bits measured 0.2405 against 0.2385 ms); a
// completed word goes to the lane's LDS staging slot k (slots 64 words apart,
// so a wave's stores hit 64 banks), slots >= ES_SW to the segment's global
// area (same word-major layout: word k of lane l at (g * ES_MAXW + k) * 64 + l).
// a table symbol without its length field
__device__ __forceinline__ uint32_t es_code(uint32_t e) { return e & ~31u; }
struct EsStage {
  uint32_t* st;
  uint32_t* ov;
  int k = 0;
  // acc: the n pending bits left-aligned (the rest zero); symL clean (zero
  // below its L bits, 0 when L = 0)
  __device__ __forceinline__ void put(uint32_t symL, int L, uint32_t& acc, int& n) {
    const int t = n + L;
    const uint32_t w = acc | (symL >> n);
    if (t >= 32) {
      if (k < ES_SW) st[k * 64] = w; else ov[k * 64] = w;
      ++k;
      acc = __builtin_amdgcn_alignbit(symL, 0u, (uint32_t)n);  // the bits that did not fit (0 when n = 0)
    } else {
      acc = w;
    }
    n = t & 31;
  }
  __device__ __forceinline__ void store(uint32_t w) {
    if (k < ES_SW) st[k * 64] = w; else ov[k * 64] = w;
  }
};

// size category of |v| (clamped to 10, code_ac's clamp)
__device__ __forceinline__ int es_size(int a) {
  const int sz = a ? 32 - __clz(a) : 0;
  return sz > 10 ? 10 : sz;
}

// The AC walk, software-pipelined: e is position K's table entry, loaded
// while position K - 1 was appended; position K + 1's lookup (its run needs
// only whether K is nonzero) is issued before K's symbol is appended.
template <int K>
__device__ __forceinline__ void es_ac(const BlockRegs& r, int last, int& aor, const uint32_t* ac, uint32_t zrl,
                                      uint32_t& acc, int& n, EsStage& o, uint32_t e, int v, int sz, int& lastK) {
  if constexpr (K < ES_DENSE) {
    const int a = v < 0 ? -v : v;
    aor |= a;
    const int run = K - 1 - last;
    const int nlast = a ? K : last;
    uint32_t e1 = 0u;
    int v1 = 0, sz1 = 0;
    if constexpr (K + 1 < ES_DENSE) {
      v1 = coef_at<ZZC[K + 1]>(r);
      sz1 = es_size(v1 < 0 ? -v1 : v1);
      e1 = ac[((K - nlast) & 15) * ES_RS + sz1];
    }
    if (a && run >= 16) {  // rare: one ZRL code per 16 zeros first
      const int zl = (int)(zrl & 31u);
      for (int i = 0; i < (run >> 4); ++i) o.put(es_code(zrl), zl, acc, n);
    }
    const int L = (int)(e & 31u) + sz;
    const uint32_t mag = (uint32_t)(v + (v >> 31)) & ((1u << sz) - 1u);  // v, or v - 1 for v < 0, in sz bits
    o.put(es_code(e) | (mag << ((32 - L) & 31)), L, acc, n);
    es_ac<K + 1>(r, nlast, aor, ac, zrl, acc, n, o, e1, v1, sz1, lastK);
  } else {
    lastK = last;
  }
}

// Zigzag positions ES_DENSE .. 63 (mostly zero at every quality but the
// finest): their coefficients go to the lane's LDS column (int16, word-major
// across the wave) with a nonzero mask, and only the nonzero ones are coded,
// in order, by a per-lane loop (run lengths from the mask).
template <int K>
__device__ __forceinline__ void es_hi_stash(const BlockRegs& r, int16_t* cz, uint32_t& m) {
  if constexpr (K < 64) {
    const int v = coef_at<ZZC[K]>(r);
    cz[(K - ES_DENSE) * 64] = (int16_t)v;
    m |= (v != 0 ? 1u : 0u) << (K - ES_DENSE);
    es_hi_stash<K + 1>(r, cz, m);
  }
}

__device__ __forceinline__ void es_hi_code(const int16_t* cz, uint32_t m, int& last, int& aor, const uint32_t* ac,
                                           uint32_t zrl, uint32_t& acc, int& n, EsStage& o) {
  while (m) {
    const int b = __builtin_ctz(m);
    m &= m - 1u;
    const int K = ES_DENSE + b;
    const int v = cz[b * 64];
    const int a = v < 0 ? -v : v;
    aor |= a;
    const int sz = es_size(a);
    const int run = K - 1 - last;
    if (run >= 16) {  // one ZRL code per 16 zeros first
      const int zl = (int)(zrl & 31u);
      for (int i = 0; i < (run >> 4); ++i) o.put(es_code(zrl), zl, acc, n);
    }
    const uint32_t e = ac[(run & 15) * ES_RS + sz];
    const int L = (int)(e & 31u) + sz;
    const uint32_t mag = (uint32_t)(v + (v >> 31)) & ((1u << sz) - 1u);
    o.put(es_code(e) | (mag << ((32 - L) & 31)), L, acc, n);
    last = K;
  }
}

// One block: DC difference, AC walk, EOB, the partial word (left-aligned).
// Returns the bit count (32 per completed word + the pending bits); bd = not
// baseline-codable.
__device__ __forceinline__ uint32_t es_block(const BlockRegs& r, int diff, const EsTab& es, int cls, EsStage& o,
                                             bool& bd, int16_t* cz) {
  uint32_t acc = 0u;
  int n = 0;
  uint32_t mhi = 0u;
  if constexpr (ES_DENSE < 64) es_hi_stash<ES_DENSE>(r, cz, mhi);
  const int v1 = coef_at<ZZC[1]>(r);
  const int sz1 = es_size(v1 < 0 ? -v1 : v1);
  const uint32_t e1 = es.ac[cls][sz1];  // run 0
  const int da = diff < 0 ? -diff : diff;
  int ds = da ? 32 - __clz(da) : 0;
  bd = ds > 11;
  ds = ds > 11 ? 11 : ds;
  const uint32_t ed = es.dc[cls][ds];
  const int Ld = (int)(ed & 31u) + ds;
  const uint32_t md = (uint32_t)(diff + (diff >> 31)) & ((1u << ds) - 1u);
  o.put(es_code(ed) | (md << ((32 - Ld) & 31)), Ld, acc, n);
  int aor = 0, last = 0;
  es_ac<1>(r, 0, aor, es.ac[cls], es.zrl[cls], acc, n, o, e1, v1, sz1, last);
  if constexpr (ES_DENSE < 64) es_hi_code(cz, mhi, last, aor, es.ac[cls], es.zrl[cls], acc, n, o);
  const uint32_t eb = es.eob[cls];
  const int Le = last < 63 ? (int)(eb & 31u) : 0;  // EOB unless coefficient 63 is set
  o.put(Le ? es_code(eb) : 0u, Le, acc, n);
  bd |= aor > 1023;  // AC size > 10
  const uint32_t nb = 32u * (uint32_t)o.k + (uint32_t)n;
  o.store(acc);
  return nb;
}

struct EsSeg {
  int f, s, seg, nseg_s, nbs;
};
__device__ __forceinline__ EsSeg es_seg(const EntGeo& e, int g) {
  EsSeg q;
  q.f = g / e.sfirst[3];
  const int r = g - q.f * e.sfirst[3];
  q.s = r < e.sfirst[1] ? 0 : (r < e.sfirst[2] ? 1 : 2);
  q.seg = r - e.sfirst[q.s];
  q.nseg_s = e.sfirst[q.s + 1] - e.sfirst[q.s];
  q.nbs = e.first[q.s + 1] - e.first[q.s];
  return q;
}

// the scan's final word: 1-bits from the scan's end to its byte boundary;
// returns the number of the word's bytes that belong to the scan
__device__ __forceinline__ int es_pad(uint32_t& v, unsigned long long W1, unsigned long long widx) {
  const int used = (int)(W1 - 32ull * widx);  // 1..32
  const int pb = (8 - (used & 7)) & 7;
  if (pb) v |= ((1u << pb) - 1u) << (32 - used - pb);
  return (used + 7) >> 3;
}

// 0xFF bytes of a word as loaded from memory (byte j = bits 8j..8j+7), among its first nvb bytes
__device__ __forceinline__ int es_ff_mem(uint32_t x, int nvb) {
  const uint32_t y = ~x;
  const uint32_t hi = ~((((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) | 0x7F7F7F7Fu);  // bit 8j+7: byte j == 0xFF
  const uint32_t vm = nvb >= 4 ? 0x80808080u : (((1u << (8 * (nvb < 0 ? 0 : nvb))) - 1u) & 0x80808080u);
  return __popc(hi & vm);
}

__device__ __forceinline__ int es_ff(uint32_t v, int nbytes) {  // 0xFF bytes among the first nbytes (stream order)
  return es_ff_mem(__builtin_bswap32(v), nbytes);
}

// Placement of a segment's staged words at scan bit offset pre (lane bits at
// pre + excl): see "one pass" above.  st: the lane's LDS staging (slots <
// ES_SW), ov: its global words (slots >= ES_SW, or all slots when st is null).
// fuse (not the scan's last segment): tailx holds the next segment's bits that
// share this segment's final word, so that word is written whole here; Wn: the
// scan's end bit when the next segment ends in that word.
__device__ __forceinline__ void es_place(const EntGeo& e, const EsSeg& q, int g, int lane, bool valid, int nvalid,
                                         bool last_seg, uint32_t nb, uint32_t excl, unsigned long long pre,
                                         unsigned long long A, const uint32_t* st, const uint32_t* ov, int k,
                                         uint32_t* __restrict__ raw, unsigned long long* __restrict__ ffs,
                                         unsigned long long* __restrict__ info,
                                         unsigned long long* __restrict__ scan_bits, bool fuse, uint32_t tailx,
                                         unsigned long long Wn) {
  const unsigned long long W1 = pre + A;
  auto stw = [&](int j) -> uint32_t { return j >= k ? 0u : ((st == nullptr || j >= ES_SW) ? ov[j * 64] : st[j * 64]); };
  const unsigned long long o = pre + excl;  // the lane's first bit in the scan
  const int sh = (int)(o & 31ull);
  const unsigned long long hw = o >> 5, tw = (o + nb - 1ull) >> 5;
  const bool single = hw == tw;
  const uint32_t s0 = stw(0);
  const uint32_t hv = s0 >> sh;
  // the next lane starts inside this lane's tail word
  // (fuse: lane 63's "next lane" is the next segment, whose bits are tailx)
  const bool c = valid && ((o + nb) & 31ull) != 0ull && (lane + 1 < nvalid || fuse);
  // X = this lane's head word bits | those of the following lanes that share it
  uint32_t X = valid ? hv : 0u;
  int F = (valid && single && c) ? 1 : 0;
  if (fuse && lane == 63 && F) {
    X |= tailx;
    F = 0;
  }
  // (every block costs >= 4 bits, so at most 7 lanes in a row lie inside one
  // word and share the next lane's word: spans of 8 lanes suffice; the host
  // model fails with spans of 4)
  {  // X_l = own_l | (F_l ? X_{l+1} : 0), one lane further per DPP wave shift (lane 63 never chains)
    // (a mask, not a select: the shifts must run with every lane active, and
    // the compiler turns a select into a branch around them)
    const uint32_t own = X, fm = 0u - (uint32_t)F;
#pragma unroll
    for (int it = 0; it < 7; ++it) X = own | (wave_shl1(X) & fm);
  }
  const uint32_t X1 = wave_shl1(X);
  const uint32_t in_tail = c ? ((fuse && lane == 63) ? tailx : X1) : 0u;
  uint32_t* rs = raw + raw_base(e, q.f, q.s);
  // word indices within the scan fit 32 bits (< 2^28 words)
  const uint32_t wlast = (uint32_t)((W1 - 1ull) >> 5);
  const bool open_end = !fuse && !last_seg && (W1 & 31ull);
  const unsigned long long Wend = last_seg ? W1 : Wn;  // the scan ends in word wlast (0: it does not)
  const uint32_t padw = Wend ? wlast : 0xFFFFFFFFu;     // the word that takes the pad bits
  const uint32_t skipw = open_end ? wlast : 0xFFFFFFFFu;  // the word the next segment counts
  int ffc = 0;
  auto put_word = [&](uint32_t widx, uint32_t v) {
    int nb4 = 4;
    if (widx == padw) nb4 = es_pad(v, Wend, widx);
    rs[widx] = __builtin_bswap32(v);  // byte 0 of the stream first
    if (widx != skipw) ffc += es_ff(v, nb4);
  };
  if (valid) {
    const bool own_head = sh == 0;
    const int nout = (int)(tw - hw);
    const uint32_t hw32 = (uint32_t)hw, tw32 = (uint32_t)tw;
    if (own_head && !single) put_word(hw32, hv);
    uint32_t prev = s0;
    int j = 1;
    for (; j + 3 < nout; j += 4) {  // four staged words requested before any is used
      const uint32_t c0 = stw(j), c1 = stw(j + 1), c2 = stw(j + 2), c3 = stw(j + 3);
      put_word(hw32 + j, __builtin_amdgcn_alignbit(prev, c0, (uint32_t)sh));
      put_word(hw32 + j + 1, __builtin_amdgcn_alignbit(c0, c1, (uint32_t)sh));
      put_word(hw32 + j + 2, __builtin_amdgcn_alignbit(c1, c2, (uint32_t)sh));
      put_word(hw32 + j + 3, __builtin_amdgcn_alignbit(c2, c3, (uint32_t)sh));
      prev = c3;
    }
    for (; j < nout; ++j) {
      const uint32_t cur = stw(j);
      put_word(hw32 + j, __builtin_amdgcn_alignbit(prev, cur, (uint32_t)sh));
      prev = cur;
    }
    const uint32_t tv = single ? hv : __builtin_amdgcn_alignbit(prev, stw(nout), (uint32_t)sh);
    if (!single || own_head) put_word(tw32, tv | in_tail);
  }
  ffc = (int)wave_sum((uint32_t)ffc);
  if (lane == 0) {
    ffs[g] = (unsigned long long)ffc;
    if (last_seg) {
      info[2 * (q.f * 3 + q.s)] = 0ull;
      info[2 * (q.f * 3 + q.s) + 1] = W1;
      if (scan_bits) scan_bits[q.f * 3 + q.s] = W1;
    }
  }
}

// k_ent_walk packs each segment's blocks and stores the staged words
// (word-major per segment), the lanes' bit counts and the segment's total;
// k_ent_place places the words at the segment's offset.
__global__ void __launch_bounds__(64 * ES_WAVES) __attribute__((amdgpu_waves_per_eu(ES_WPE))) k_ent_walk(
    const EntGeo e, const int nseg, const int16_t* __restrict__ coeffs, const EsTab* __restrict__ gt,
    uint32_t* __restrict__ gst, uint32_t* __restrict__ nbits, unsigned long long* __restrict__ agg,
    uint32_t* __restrict__ badseg, unsigned long long* __restrict__ ffs) {
  __shared__ EsTab es;
  __shared__ uint32_t stage[ES_WAVES][ES_SW > 0 ? ES_SW : 1][64];
  __shared__ int16_t czs[ES_WAVES][ES_HI > 0 ? ES_HI : 1][64];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(gt);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&es);
    for (int i = threadIdx.x; i < (int)(sizeof(EsTab) / 4); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int16_t* cz = &czs[wv][0][lane];
  const int g = blockIdx.x * ES_WAVES + wv;
  if (g >= nseg) return;  // (whole wave; no barrier follows)
  const EsSeg q = es_seg(e, g);
  const int bi = q.seg * 64 + lane;
  const bool valid = bi < q.nbs;
  const long long gb = (long long)q.f * e.nb + e.first[q.s] + (valid ? bi : q.nbs - 1);
  const BlockRegs rg = load_block(coeffs + gb * 64);
  const int dc = coef_at<0>(rg);
  int pred = wave_shr1(dc);
  if (lane == 0) pred = q.seg ? (int)coeffs[(gb - 1) * 64] : 0;
  uint32_t* st = &stage[wv][0][lane];
  uint32_t* ov = gst + (size_t)g * ES_MAXW * 64 + lane;
  uint32_t nb = 0u;
  int k = 0;
  bool bd = false;
  if (valid) {
    EsStage o{st, ov};
    nb = es_block(rg, dc - pred, es, q.s ? 1 : 0, o, bd, cz);
    k = (int)((nb + 31u) >> 5);
  }
  const bool any_bad = __ballot(bd) != 0ull;
  // the LDS slots to the segment's global area (one 256-B row per slot)
  const int kmax = (int)wave_max((uint32_t)(k < ES_SW ? k : ES_SW));
  for (int j = 0; j < kmax; ++j)
    if (j < k) ov[j * 64] = st[j * 64];
  nbits[(size_t)g * 64 + lane] = nb;
  const unsigned long long a = wave_sum(nb);  // (<= 64 * 1660 bits)
  if (lane == 0) {
    agg[g] = a;
    badseg[g] = any_bad ? 1u : 0u;  // not baseline-codable: the frame is reported (k_ent_fscan)
    if (g == nseg - 1) {            // the scans' closing zeros (no memsets)
      agg[nseg] = 0ull;
      ffs[nseg] = 0ull;
    }
  }
}

// The segment's bit offset within its scan is the sum of the scan's earlier
// segment totals.  Scans of at most ES_SELF_MAX segments (1080p: 507 luma, 128
// chroma) sum them here -- every total is final when this launch starts -- and
// need no prefix launch between the walk and the placement (0.245 -> 0.244 ms
// per 64 x 1080p); longer scans (4K: 2025 luma segments) would re-sum O(n^2)
// totals across their waves, so their frames get a per-frame exclusive prefix
// (k_ent_fscan<false>, segoff) before this launch.  Measured
// (tools/ent_probe.py, profiles/r05_entropy_selfpre_ab.jsonl): 16 x 4K, every
// scan summing itself 0.2585 ms, every scan from the prefix launch 0.2517,
// this threshold 0.2547; 64 x 1080p 0.2518 / 0.2523 / 0.2528 (noise).
constexpr int ES_SELF_MAX = 512;

// incl[g] = the segment's end bit within its scan (k_ent_fscan / k_ent_emit3
// read it as desc)
__global__ void __launch_bounds__(256) k_ent_place(const EntGeo e, const int nseg, const uint32_t* __restrict__ gst,
                                                   const uint32_t* __restrict__ nbits,
                                                   const unsigned long long* __restrict__ agg,
                                                   const unsigned long long* __restrict__ segoff,
                                                   unsigned long long* __restrict__ incl, uint32_t* __restrict__ raw,
                                                   unsigned long long* __restrict__ ffs,
                                                   unsigned long long* __restrict__ info,
                                                   unsigned long long* __restrict__ scan_bits) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nseg) return;
  const EsSeg q = es_seg(e, g);
  const bool valid = q.seg * 64 + lane < q.nbs;
  const int nvalid = q.nbs - q.seg * 64 < 64 ? q.nbs - q.seg * 64 : 64;
  const bool last_seg = q.seg == q.nseg_s - 1;
  const bool fuse = !last_seg;      // this segment completes the word it shares with the next
  const int gn = fuse ? g + 1 : g;  // the next segment of the scan (its head bits)
  const uint32_t nb = nbits[(size_t)g * 64 + lane];
  const uint32_t nbn = nbits[(size_t)gn * 64 + lane];
  const uint32_t w0n = gst[(size_t)gn * ES_MAXW * 64 + lane];  // (row 0; garbage where nbn == 0)
  unsigned long long pre;
  if (q.nseg_s <= ES_SELF_MAX) {  // (uniform: the scan's length)
    // lane sums are < 2^32 (<= 8 totals of <= 64 * 1660 bits); the wave sum in
    // two DPP scans of 8 / 24 bits
    const unsigned long long* a0 = agg + (g - q.seg);
    uint32_t ps = 0u;
    for (int j0 = 0; j0 < q.seg; j0 += 512) {  // eight loads in flight per lane
      uint32_t t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + 64 * u + lane;
        t[u] = j < q.seg ? (uint32_t)a0[j] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) ps += t[u];
    }
    pre = ((unsigned long long)wave_sum(ps >> 8) << 8) + wave_sum(ps & 255u);
  } else {
    pre = segoff[g] - segoff[g - q.seg];  // (frame-relative prefixes)
  }
  const uint32_t inc = wave_incl_sum(nb, lane), incn = wave_incl_sum(nbn, lane);
  const unsigned long long A = lane63(inc);
  const unsigned long long W1 = pre + A;
  if (lane == 0) incl[g] = W1;
  uint32_t tailx = 0u;
  unsigned long long Wn = 0ull;
  if (fuse) {
    // the next segment's lanes starting inside this segment's final word: each
    // one's bits there are its first staged word's leading bits
    const uint32_t sh = (uint32_t)(W1 & 31ull), p = sh + (incn - nbn);
    tailx = (sh && nbn && p < 32u) ? w0n >> p : 0u;
    tailx = wave_or(tailx);
    const unsigned long long An = lane63(incn);
    if (q.seg + 2 == q.nseg_s && sh && ((W1 + An - 1ull) >> 5) == ((W1 - 1ull) >> 5)) Wn = W1 + An;
  }
  es_place(e, q, g, lane, valid, nvalid, last_seg, nb, inc - nb, pre, A, nullptr,
           gst + (size_t)g * ES_MAXW * 64 + lane, (int)((nb + 31u) >> 5), raw, ffs, info, scan_bits, fuse, tailx, Wn);
}

// One wave per segment: the bytes of the words it finalised, stuffed (0x00
// after every 0xFF) at their place in the file.  Per 1 KiB of input (16 B per
// lane): the lanes' stuffed lengths by a wave prefix, the stuffed bytes
// assembled in the wave's LDS buffer at the output's alignment, then written
// out as aligned dwords (bytes at the two partial ends).
constexpr int EM_CHUNK = 1024;
// Per-frame exclusive prefix of a per-segment u64 array (one 1024-thread
// workgroup per frame; frames' segment ranges are independent): out[g] is
// frame-relative, tot[f] the frame's total.  OFFS: also each segment's first
// output byte, from the frame's own prefixes, and the frame's markers.
// (Replaced a hipCUB scan -- two launches -- and a per-segment offset launch.)
template <bool OFFS>
__global__ void __launch_bounds__(1024) k_ent_fscan(const EntGeo e, const unsigned long long* __restrict__ in,
                                                    unsigned long long* __restrict__ out,
                                                    unsigned long long* __restrict__ tot,
                                                    const unsigned long long* __restrict__ desc,
                                                    const unsigned long long* __restrict__ info,
                                                    unsigned long long* __restrict__ outoff,
                                                    const uint8_t* __restrict__ hdr, uint8_t* __restrict__ file,
                                                    long long stride, unsigned long long* __restrict__ lengths,
                                                    const uint32_t* __restrict__ badseg) {
  __shared__ unsigned long long s_w[16];
  __shared__ int s_bad;
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = e.sfirst[3];
  const long long g0 = (long long)f * n;
  const int C = (n + 1023) / 1024, i0 = t * C, i1 = min(n, i0 + C);
  unsigned long long loc = 0ull;
  for (int i = i0; i < i1; ++i) loc += in[g0 + i];
  unsigned long long inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  unsigned long long base = 0ull, all = 0ull;
  for (int w = 0; w < 16; ++w) {
    base += w < wv ? s_w[w] : 0ull;
    all += s_w[w];
  }
  unsigned long long run = base + inc - loc;
  for (int i = i0; i < i1; ++i) {
    const unsigned long long v = in[g0 + i];
    out[g0 + i] = run;
    run += v;
  }
  if (t == 0) tot[f] = all;
  if constexpr (OFFS) {
    __syncthreads();  // the frame's prefixes (global, this workgroup's writes) are visible
    long long so[3];
    long long p = e.hdr + ENT_SOS;
    for (int s2 = 0; s2 < 3; ++s2) {
      so[s2] = p;
      const unsigned long long nb = (info[2 * (f * 3 + s2) + 1] + 7) >> 3;
      const unsigned long long ffe = s2 < 2 ? out[g0 + e.sfirst[s2 + 1]] : all;
      p += (long long)(nb + ffe - out[g0 + e.sfirst[s2]]) + ENT_SOS;
    }
    int b = 0;
    for (int i = t; i < n; i += 1024) {
      const long long g = g0 + i;
      const int s2 = i < e.sfirst[1] ? 0 : (i < e.sfirst[2] ? 1 : 2);
      const int seg = i - e.sfirst[s2];
      const unsigned long long W0 = seg ? desc[g - 1] : 0ull;
      outoff[g] = (unsigned long long)so[s2] + 4 * ((W0 + 31) >> 5) + (out[g] - out[g0 + e.sfirst[s2]]);
      b |= (int)badseg[g];
    }
    // the frame's markers (k_ent_emit3 writes only the scans' bytes)
    if (t == 0) s_bad = 0;
    __syncthreads();
    if (b) s_bad = 1;
    uint8_t* dst = file + (long long)f * stride;
    for (int i = t; i < e.hdr; i += 1024) dst[i] = hdr[(long long)f * e.hdr + i];
    if (t < 3) {
      uint8_t* m = dst + so[t] - ENT_SOS;
      const uint8_t sos[ENT_SOS] = {0xFF, 0xDA, 0x00, 0x08, 0x01, (uint8_t)(t + 1), (uint8_t)(t == 0 ? 0x00 : 0x11),
                                    0x00, 0x3F, 0x00};
      for (int i = 0; i < ENT_SOS; ++i) m[i] = sos[i];
    }
    __syncthreads();
    if (t == 0) {
      const long long end = p - ENT_SOS;  // end of the Cr scan
      dst[end] = 0xFF;
      dst[end + 1] = 0xD9;
      if (lengths) lengths[f] = s_bad ? 0ull : (unsigned long long)(end + 2);  // 0: not baseline-codable
    }
  }
}

__global__ void __launch_bounds__(256) k_ent_emit3(const EntGeo e, const int nseg,
                                                   const unsigned long long* __restrict__ desc,
                                                   const unsigned long long* __restrict__ info,
                                                   const uint32_t* __restrict__ raw,
                                                   const unsigned long long* __restrict__ outoff,
                                                   uint8_t* __restrict__ out, long long stride) {
  __shared__ uint32_t sbuf[4][(2 * EM_CHUNK + 8) / 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = blockIdx.x * 4 + wv;
  if (g >= nseg) return;
  const EsSeg q = es_seg(e, g);
  const unsigned long long W0 = q.seg ? desc[g - 1] : 0ull, W1 = desc[g];
  const unsigned long long nbytes = (info[2 * (q.f * 3 + q.s) + 1] + 7) >> 3;
  const unsigned long long fw = (W0 + 31) >> 5, lw = (W1 - 1) >> 5;
  if (fw > lw) return;
  const unsigned long long b0 = 4 * fw, b1 = (4 * lw + 4 < nbytes) ? 4 * lw + 4 : nbytes;
  uint8_t* dst = out + (long long)q.f * stride + (long long)outoff[g];
  const uint32_t* w = raw + raw_base(e, q.f, q.s);
  uint8_t* lb = reinterpret_cast<uint8_t*>(sbuf[wv]);
  for (unsigned long long i0 = b0; i0 < b1; i0 += EM_CHUNK) {
    // lane l takes the chunk's dwords l, l + 64, l + 128, l + 192: coalesced
    // loads, and a wave's byte stores land on consecutive LDS words (16 B per
    // lane put lanes 16 apart on one bank)
    uint32_t x[4];
    int nvk[4], lk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned long long i = i0 + 4 * (64 * k + lane);
      nvk[k] = i < b1 ? (b1 - i < 4 ? (int)(b1 - i) : 4) : 0;
      x[k] = nvk[k] ? w[i >> 2] : 0u;
      lk[k] = nvk[k] + es_ff_mem(x[k], nvk[k]);  // <= 8
    }
    // two packed scans (16-bit fields: a field's wave sum is <= 512)
    const uint32_t pa = (uint32_t)lk[0] | ((uint32_t)lk[1] << 16), pb = (uint32_t)lk[2] | ((uint32_t)lk[3] << 16);
    const uint32_t ia = wave_incl_sum(pa, lane), ib = wave_incl_sum(pb, lane);
    const uint32_t ta = lane63(ia), tb = lane63(ib);
    const uint32_t ea = ia - pa, eb = ib - pb;
    const int t0 = (int)(ta & 0xFFFFu), t1 = (int)(ta >> 16), t2 = (int)(tb & 0xFFFFu), t3 = (int)(tb >> 16);
    const int tot = t0 + t1 + t2 + t3;
    const int sh0 = (int)((uintptr_t)dst & 3u);  // LDS byte sh0 <-> dst[0]
    const int pk[4] = {sh0 + (int)(ea & 0xFFFFu), sh0 + t0 + (int)(ea >> 16), sh0 + t0 + t1 + (int)(eb & 0xFFFFu),
                       sh0 + t0 + t1 + t2 + (int)(eb >> 16)};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int p = pk[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < nvk[k]) {
          const uint8_t b = (uint8_t)(x[k] >> (8 * j));
          lb[p++] = b;
          if (b == 0xFF) lb[p++] = 0x00;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // one wave: its LDS operations execute in order
    asm volatile("" ::: "memory");
    // out: global bytes dst[0 .. tot) <- LDS bytes [sh0, sh0 + tot); dword d covers LDS [4d, 4d + 4)
    uint8_t* a0 = dst - sh0;  // 4-byte aligned
    const int nd = (sh0 + tot + 3) >> 2;
    for (int d = lane; d < nd; d += 64) {
      const int lo = 4 * d, hi = 4 * d + 4;
      if (lo >= sh0 && hi <= sh0 + tot) {
        *reinterpret_cast<uint32_t*>(a0 + lo) = sbuf[wv][d];
      } else {
        for (int c = lo; c < hi; ++c)
          if (c >= sh0 && c < sh0 + tot) a0[c] = lb[c];
      }
    }
    __builtin_amdgcn_wave_barrier();  // the buffer is reused by the next iteration
    asm volatile("" ::: "memory");
    dst += tot;
  }
}

// ------------------------------------------------------------ driver --

EntGeo ent_geo(const Geo& g) {
  EntGeo e{};
  const int ny = g.nby * g.nbx, nc = g.ncy * g.ncx;
  e.nb = ny + 2 * nc;
  e.first[0] = 0;
  e.first[1] = ny;
  e.first[2] = ny + nc;
  e.first[3] = e.nb;
  e.sfirst[0] = 0;
  for (int s = 0; s < 3; ++s) e.sfirst[s + 1] = e.sfirst[s] + (e.first[s + 1] - e.first[s] + 63) / 64;
  e.cap_w[0] = (int)(((long long)ny * 1660 + 31) / 32) + 2;
  e.cap_w[1] = e.cap_w[2] = (int)(((long long)nc * 1660 + 31) / 32) + 2;
  e.raw_w = (long long)e.cap_w[0] + 2LL * e.cap_w[1];
  e.hdr = ENT_HDR;
  return e;
}

// worst case file: header + 3 SOS + every scan at 1660 bits per block, all bytes stuffed + EOI
long long ent_capacity(const Geo& g) {
  const EntGeo e = ent_geo(g);
  return e.hdr + 3 * ENT_SOS + 2 * 4 * e.raw_w + 2;
}

// scratch sizes (bytes): [0] segment end bits (desc, from the second word),
// segment totals (agg; reused for the output offsets once placed), their
// per-frame prefix (segoff), per-lane bit counts, per-segment error flags; [1]
// staged words (word-major per segment); [2] info; [3] packed scans; [4] 0xFF
// counts per segment; [5] their prefix and the frame totals; [6] headers; [7]
// unused.
void ent_sizes(const Geo& g, int n, size_t* sz) {
  const EntGeo e = ent_geo(g);
  sz[2] = sizeof(unsigned long long) * 7 * n;  // 6 per frame (scan start / bits) + the frame's error flag
  sz[3] = sizeof(uint32_t) * e.raw_w * n;
  sz[6] = (size_t)e.hdr * n;
  const long long nseg = (long long)n * e.sfirst[3];
  sz[0] = sizeof(unsigned long long) * (nseg + 2) + sizeof(unsigned long long) * 2 * (nseg + 1) +
          sizeof(uint32_t) * 65 * nseg;
  sz[1] = sizeof(uint32_t) * ES_MAXW * 64 * nseg;
  sz[4] = sizeof(unsigned long long) * (nseg + 1);
  sz[5] = sizeof(unsigned long long) * (nseg + 1 + n);  // + the frame totals (k_ent_fscan)
  sz[7] = 0;
}

// walk, (per-frame segment prefix for long scans,) placement, per-frame
// offsets and markers, stuffing: 4 or 5 launches per batch of frames
static hipError_t launch_entropy_fused(const Geo& g, int n, const int16_t* coeffs, void* const* buf,
                                       const uint8_t* hdr_dev, const void* tab_dev, uint8_t* out, long long stride,
                                       unsigned long long* lengths, unsigned long long* scan_bits, hipStream_t s) {
  const EntGeo e = ent_geo(g);
  const long long nseg_l = (long long)n * e.sfirst[3];
  if (nseg_l >= (1ll << 31)) return hipErrorInvalidValue;
  const int nseg = (int)nseg_l;
  auto* desc = (unsigned long long*)buf[0] + 1;
  auto* agg = desc + nseg + 1;
  auto* segoff = agg + nseg + 1;
  auto* nbits = (uint32_t*)(segoff + nseg + 1);
  auto* badseg = nbits + 64 * (size_t)nseg;
  auto* outoff = agg;  // (the segment totals, consumed by the placement)
  auto* ovf = (uint32_t*)buf[1];
  auto* info = (unsigned long long*)buf[2];
  auto* raw = (uint32_t*)buf[3];
  auto* ffs = (unsigned long long*)buf[4];
  auto* ffx = (unsigned long long*)buf[5];
  const unsigned wg = (unsigned)((nseg + ES_WAVES - 1) / ES_WAVES);
  const unsigned wg4 = (unsigned)((nseg + 3) / 4);  // k_ent_place / k_ent_emit3: four segment waves per workgroup
  const EsTab* est = reinterpret_cast<const EsTab*>((const char*)tab_dev + sizeof(EntTab));
  hipLaunchKernelGGL(k_ent_walk, dim3(wg), dim3(64 * ES_WAVES), 0, s, e, nseg, coeffs, est, ovf, nbits, agg, badseg,
                     ffs);
  kmark(s, "k_ent_walk");
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  bool long_scan = false;
  for (int c = 0; c < 3; ++c) long_scan = long_scan || e.sfirst[c + 1] - e.sfirst[c] > ES_SELF_MAX;
  if (long_scan) {
    hipLaunchKernelGGL(k_ent_fscan<false>, dim3(n), dim3(1024), 0, s, e, agg, segoff, ffx, nullptr, nullptr, nullptr,
                       nullptr, nullptr, 0ll, nullptr, nullptr);
    kmark(s, "k_ent_fscan<0>");
  }
  hipLaunchKernelGGL(k_ent_place, dim3(wg4), dim3(256), 0, s, e, nseg, ovf, nbits, agg, segoff, desc, raw, ffs, info,
                     scan_bits);
  kmark(s, "k_ent_place");
  if ((err = hipGetLastError()) != hipSuccess) return err;
  // frame-relative 0xFF prefixes, each segment's output offset and the frame's
  // markers in one launch; frame totals in ffx[nseg + 1 ..]
  unsigned long long* fftot = ffx + nseg + 1;
  hipLaunchKernelGGL(k_ent_fscan<true>, dim3(n), dim3(1024), 0, s, e, ffs, ffx, fftot, desc, info, outoff, hdr_dev,
                     out, stride, lengths, badseg);
  kmark(s, "k_ent_fscan<1>");
  hipLaunchKernelGGL(k_ent_emit3, dim3(wg4), dim3(256), 0, s, e, nseg, desc, info, raw, outoff, out, stride);
  kmark(s, "k_ent_emit3");
  return hipGetLastError();
}

hipError_t launch_entropy(const Geo& g, int n, const int16_t* coeffs, void* const* buf, const uint8_t* hdr_dev,
                          const void* tab_dev, uint8_t* out, long long stride, unsigned long long* lengths,
                          unsigned long long* scan_bits, hipStream_t s) {
  return launch_entropy_fused(g, n, coeffs, buf, hdr_dev, tab_dev, out, stride, lengths, scan_bits, s);
}

}  // namespace jds
