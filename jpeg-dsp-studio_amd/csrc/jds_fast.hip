// jds_fast.hip — the throughput path: fp32 arithmetic with CERTIFIED rounding
// decisions, plus exact fp64 fix-up of the rare ambiguous cases, so results
// stay bit-identical to the reference (engines/pipeline.py:47-63).
//
// Forward (k_fwd32): colour, prefilter, area average, 8x8 DCT (even/odd FMA
// form) and quantisation run in fp32.  For every coefficient a rigorous static
// bound E_uv on |c_fp32 - c_exact| (derived on the host from the fp32
// operation sequence, fast_fwd_thresholds) decides whether
// round-half-even(c/Q) is certain: if t = c*(1/Q) is farther than E_uv/Q (+
// the multiply's own error) from a half-integer, the fp32 quotient rounds
// exactly like the reference's fp64 quotient.  Blocks with any uncertain
// coefficient (~0.5% on random 1080p at Q50, exact ties always) are appended
// to a list; k_fix_fwd recomputes them with the pocketfft-exact fp64 path of
// jds_codec.hip from global memory, overwrites their coefficients and corrects
// the statistics.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "jds_dct8.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_fwd_common.hpp"

#pragma clang fp contract(off)

// Shipped choices whose alternatives were measured and retired (DESIGN.md
// "Retired A/B switches"): first/last tile rows folded into k_fwd32i
// (fold_rows; a uniform per-tile flag that skips the masks on the other rows
// measured no better, 339.6 vs 337.1 us per 64 x 1080p); ring rows staged on
// the lanes after the tile's rows; neighbour samples by DPP instead of
// ds_bpermute; the quantiser tables loaded by a wave without staging work.

namespace jds {

// orthonormal 8-point DCT matrix entries rounded to fp32:
// W[k][i] = s(k) cos((2i+1) k pi / 16), s(0) = sqrt(1/8), s(k) = 1/2
#define JA 0x1.6a09e6p-2f   // sqrt(1/8)
#define JC1 0x1.f6297cp-2f  // cos(1 pi/16) / 2
#define JC2 0x1.d906bcp-2f
#define JC3 0x1.a9b662p-2f
#define JC5 0x1.1c73b4p-2f
#define JC6 0x1.87de2ap-3f
#define JC7 0x1.8f8b84p-4f

// rows k of W restricted to i = 0..3; even rows act on s_i = x_i + x_{7-i},
// odd rows on d_i = x_i - x_{7-i}
static constexpr float FW[8][4] = {
    {JA, JA, JA, JA},      {JC1, JC3, JC5, JC7},    {JC2, JC6, -JC6, -JC2}, {JC3, -JC7, -JC1, -JC5},
    {JA, -JA, -JA, JA},    {JC5, -JC1, JC7, JC3},   {JC6, -JC2, JC2, -JC6}, {JC7, -JC5, JC3, -JC1},
};

// fp32 forward DCT-II of one line: 8 add/sub + 8 four-term FMA chains.  The
// host-side bound (fast_fwd_thresholds) follows exactly this sequence.
__host__ __device__ __forceinline__ void fdct8_f32(float (&x)[8]) {
  const float s0 = x[0] + x[7], s1 = x[1] + x[6], s2 = x[2] + x[5], s3 = x[3] + x[4];
  const float d0 = x[0] - x[7], d1 = x[1] - x[6], d2 = x[2] - x[5], d3 = x[3] - x[4];
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    x[k] = fmaf(FW[k][3], s3, fmaf(FW[k][2], s2, fmaf(FW[k][1], s1, FW[k][0] * s0)));
    x[k + 1] = fmaf(FW[k + 1][3], d3, fmaf(FW[k + 1][2], d2, fmaf(FW[k + 1][1], d1, FW[k + 1][0] * d0)));
  }
}

__device__ __forceinline__ void unpack32(uint32_t v, float& R, float& G, float& B) {
  R = (float)(v & 255u);
  G = (float)((v >> 8) & 255u);
  B = (float)(v >> 16);
}

struct FastQ {
  float rq[64];      // fp32(1/Q)
  float thr[2][64];  // certification limits on |t - rint(t)| (0.5 - margin): [0] luma, [1] chroma
};

constexpr int BS32 = 72;  // floats per 8x8 block in LDS (column writes conflict-free)

// k_fwd32i's chroma planes (4:2:x): the 16-B slot f of plane row `row` is
// stored at slot f ^ csw(row).  The 8 lanes of a chroma block read rows SY
// apart at the same columns (rows are 256 B = one bank row apart), 4-way
// conflicting per ds_read_b128 lane group; XOR-ing the slot with the row's
// sample index mod 4 puts them on 4 different slots (MI355X_MICROARCH.md §LDS).
template <int SY>
__device__ __forceinline__ int csw(int row) { return (row / SY) & 3; }

// The prefiltered planes hold pair sums (8 float4 slots per 128-B row): the
// 8 lanes of a chroma block read rows SY apart at the same slots, which rows
// two apart put on the same banks; XOR-ing the slot with the row's sample
// index mod 8 spreads them over 8 slots.
template <int SY>
__device__ __forceinline__ int psw(int row) { return (row / SY) & 7; }

__device__ __forceinline__ uint32_t byte_at(const uint32_t (&w)[6], int b) { return (w[b >> 2] >> (8 * (b & 3))) & 255u; }

// Per-lane statistics of the quantised coefficients.  Integer counters keep
// the work on the VALU (lane booleans would live in SGPR masks and cost scalar
// instructions per coefficient): nonzero count, magnitude bits from the binary
// exponent of the rounded quotient (frexp: 0 -> 0, |q| -> bit length), the
// histogram's common bins 22..29 (q in [-12, 19], zeros included and removed
// after the wave sum) as eight 4-bit counters, and the certification flags.
struct LaneStats {
  unsigned nz = 0u, mb = 0u, hn = 0u, nflag = 0u;
};

// Rare bins in the quality-sweep quantiser (k_quant_mq, REPL): RH_COPIES
// replicated histograms per table (lane & 3 picks one), slot 50 = q 100 (folded
// into bin 49), and lanes with nothing to count in a slot add to a private
// dummy word, so the 8 atomics of a lane need no per-coefficient branches.
constexpr int RH_COPIES = 4, RH_STRIDE = 53;
constexpr int RH_WORDS = RH_COPIES * RH_STRIDE + 64;

__device__ __forceinline__ unsigned rare_bin_total(const unsigned* s_rh, int b) {
  unsigned t = 0u;
#pragma unroll
  for (int c = 0; c < RH_COPIES; ++c) t += s_rh[c * RH_STRIDE + b] + (b == 49 ? s_rh[c * RH_STRIDE + 50] : 0u);
  return t;
}

// Round 8 coefficients c*(1/Q) to int16, certify each rounding (t farther than
// thr + |t| 2^-22 from a half-integer decides like the fp64 reference) and
// count statistics.  Rare histogram bins (|q| > 12) go to LDS atomics: into
// s_st's histogram with per-coefficient branches (REPL false: rare values are
// sparse at the headline qualities), or branch-free into replicated
// histograms at s_rh (REPL true).
template <bool REPL = false>
__device__ __forceinline__ void quant8(const float (&v)[8], const float (&rq)[8], const float (&thr)[8], bool valid,
                                       int (&q)[8], LaneStats& ls, unsigned* s_st) {
  unsigned nrare = 0u;
  // |t| <= 1024 (|c| <= 8 * 128, Q >= 1): QMAGIC rounds exactly.
  // Written for gfx950's issue costs (tools/microbench/op_rates.hip): fp32
  // add / sub / mul / fma and integer add / and / or / lshr issue in ~2.5
  // cycles per wave, compares, selects, conversions, rndne and frexp in ~4.3,
  // so the rounding is the magic add, the certificate a sign bit and the rare
  // test an OR.
  unsigned ok = 0xffffffffu, orr = 0u;
  unsigned top;  // 2^31 in a VGPR, opaque (the shift below must not fold back into 1 << x)
  asm("v_mov_b32 %0, 0x80000000" : "=v"(top));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float t = v[k] * rq[k];
    const float f = t + QMAGIC;
    const float r = f - QMAGIC;  // rintf(t)
    const uint32_t fb = __float_as_uint(f);
    // uncertain when |t - r| >= thr - |t| 2^-22 (|t - r| exact by Sterbenz;
    // thr[k] holds 0.5 - E/Q - slack, rounded down): e = |t - r| - g is < 0
    // exactly when the rounding is certain (the rounded difference keeps the
    // exact one's sign, and g > 0, so e is never -0)
    const float e = fabsf(t - r) - fmaf(fabsf(t), -0x1p-22f, thr[k]);
    ok &= __float_as_uint(e);
    q[k] = (int)(fb - QMAGIC_BITS);
    const int x = __builtin_amdgcn_frexp_expf(r);  // bit length of |q| (0 for q = 0; <= 11)
    ls.nz += (unsigned)(x + 15) >> 4;
    ls.mb += (unsigned)x;
    const unsigned o = fb - (QMAGIC_BITS - 12u);  // q + 12
    // bins 22..29: += 1 << (o & 28) as 2^31 >> ((o & 28) ^ 31) (one bitop3 and a
    // right shift instead of a left shift); a rare q lands in some nibble and is
    // taken back below
    ls.hn += top >> ((o & 28u) ^ 31u);
    orr |= o;  // any o >= 32 (q outside [-12, 19]) sets a bit >= 5
  }
  ls.nflag += (~ok) >> 31;
  nrare = REPL ? orr : (orr >= 32u ? 1u : 0u);
  if constexpr (REPL) {
    if (nrare >= 32u) {
      const int lane = threadIdx.x & 63;
      unsigned* copy = s_st + (lane & (RH_COPIES - 1)) * RH_STRIDE;
      unsigned* dummy = s_st + RH_COPIES * RH_STRIDE + lane;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const unsigned o = (unsigned)(q[k] + 12);
        const bool rare = o >= 32u;
        ls.hn -= rare ? 1u << (o & 28u) : 0u;
        const unsigned h = (unsigned)(q[k] + 100);
        atomicAdd(rare && valid && h <= 200u ? copy + (h >> 2) : dummy, 1u);
      }
    }
  } else if (nrare != 0u) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const unsigned o = (unsigned)(q[k] + 12);
      if (o >= 32u) {
        ls.hn -= 1u << (o & 28u);
        if (valid && (unsigned)(q[k] + 100) <= 200u) atomicAdd(&s_st[2 + (q[k] == 100 ? 49 : (q[k] + 100) >> 2)], 1u);
      }
    }
  }
}

__device__ __forceinline__ uint4 pack_q(const int (&q)[8]) {
  return make_uint4((uint32_t)(uint16_t)q[0] | ((uint32_t)(uint16_t)q[1] << 16),
                    (uint32_t)(uint16_t)q[2] | ((uint32_t)(uint16_t)q[3] << 16),
                    (uint32_t)(uint16_t)q[4] | ((uint32_t)(uint16_t)q[5] << 16),
                    (uint32_t)(uint16_t)q[6] | ((uint32_t)(uint16_t)q[7] << 16));
}

// Flagged blocks (any uncertain coefficient among the block's 8 lanes) are
// queued for the exact fp64 fix-up; lane 8b of a wave speaks for block b.
// Two forms, both per item (one shared device-scope counter serialises
// across the chip's XCDs):
// * flag_block_list (single-quality front ends): one atomic per wave reserves
//   the wave's slots in the item's list (`cap` entries).  The wave waits for
//   the atomic's return, which the large interior launch hides.
// * flag_block_bits (k_quant_mq, up to 8 tables per row): the block's bit in
//   the item's bitmap (`wpi` words) by an atomic OR that returns nothing the
//   wave waits for -- a third of the quantiser's waves flag something at Q95
//   and it has little other work to hide a round trip behind;
//   k_fwd_reduce_fix turns the bitmaps into lists.
__device__ __forceinline__ void flag_block_list(const LaneStats& ls, bool valid, int line, int item, int plane,
                                                int bidx, uint2* fixlist, unsigned* fixcount, long long cap) {
  const unsigned long long fm = __ballot(valid && ls.nflag != 0u);
  if (!fm) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const bool mine = valid && line == 0 && ((fm >> (lane & ~7)) & 0xffull);
  const unsigned long long lm = __ballot(mine);
  unsigned base = 0u;
  if (lane == __ffsll((long long)lm) - 1) base = atomicAdd(fixcount + item, (unsigned)__popcll(lm));
  base = __shfl(base, __ffsll((long long)lm) - 1, 64);
  if (mine) {
    const unsigned slot = base + (unsigned)__popcll(lm & ((1ull << lane) - 1ull));
    // a list holds at most every block of its item; the bound keeps a counter
    // left stale by an aborted run from writing past the item's list
    if (slot < (unsigned long long)cap)
      fixlist[(size_t)item * cap + slot] = make_uint2((unsigned)item, ((unsigned)plane << 24) | (unsigned)bidx);
  }
}

__device__ __forceinline__ void flag_block_bits(const LaneStats& ls, bool valid, int line, int item, long long gblk,
                                                uint32_t* fixbits, int wpi) {
  const unsigned long long fm = __ballot(valid && ls.nflag != 0u);
  if (!fm) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  if (valid && line == 0 && ((fm >> (lane & ~7)) & 0xffull))
    atomicOr(fixbits + (size_t)item * wpi + (gblk >> 5), 1u << (gblk & 31));
}

// The workgroup's statistics into this tile's slot of the per-tile partials.
// No workgroup-level step at all: after the 16-lane row sums of the packed
// counters (8-bit fields: a 16-lane row sums to <= 16 * 8 = 128 per bin; the
// row's valid-lane count rides in bits 8..15 of the nonzero | magnitude-bits
// word), lanes 15 / 31 / 47 / 63 store their row's three words straight into
// the tile's slot (PSLOT words: [wave][row][4]); quant8's rare bins go to the
// frame's rare row (global atomics; rare values are sparse) behind the tiles'
// slots, and k_fwd_reduce_rows decodes the records, adds the rare row and
// re-zeroes it.  (Measured against a workgroup-barrier form, a last-wave
// ticket form, LDS-atomic and per-wave record forms in round 3: this one saves
// the row broadcasts, the ticket and the last wave's decode; profiles/r03_*.)
constexpr int NW_MAX = 8;  // waves per forward workgroup (TF <= 512)
__device__ __forceinline__ void stats_flush(LaneStats ls, bool valid, uint32_t* __restrict__ slot) {
  if (!valid) ls = LaneStats();
  const unsigned h = ls.hn;
  unsigned v[3] = {h & 0x0f0f0f0fu, (h >> 4) & 0x0f0f0f0fu, ls.nz | ((valid ? 1u : 0u) << 8) | (ls.mb << 16)};
  row_sums3(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if ((lane & 15) == 15)
    *reinterpret_cast<uint4*>(slot + 4 * (4 * w + (lane >> 4))) = make_uint4(v[0], v[1], v[2], 0u);
}

// words per tile slot of the per-tile partials (8 waves x 4 rows x 4 words)
constexpr int PSLOT = 128;
// the frame's rare-bin row (64 words: [2 + bin]) behind every tile slot
__device__ __forceinline__ unsigned* rare_row(uint32_t* part, const Geo& g, int nframes, int frame) {
  return part + (size_t)nframes * g.tiles_y * g.tiles_x * PSLOT + (size_t)frame * 64;
}

// ---- general tiles ------------------------------------------------------------
//
// One workgroup per TH x TW tile, one thread per (block, line).  The RGB window
// (+1 px ring, BORDER_REFLECT_101 outside the image) is staged as packed u32;
// with the prefilter the chroma planes of the window are converted and
// row-filtered in LDS; each thread forms its block column (np.pad reflect index
// maps for padding blocks), runs the column (axis-0) DCT, exchanges through LDS
// and runs the row DCT.  Used for the border ring of tiles (or all tiles when
// the interior kernel does not apply).
template <int MODE, bool PF, bool MQ = false>
__global__ void __launch_bounds__(Cfg<MODE>::TF)
k_fwd32(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
        const FastQ* __restrict__ fq, const float* __restrict__ gk32, uint32_t* __restrict__ part,
        uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount, const int border, const int4 rect,
        float* __restrict__ dct32,
        jds_frame_stats* __restrict__ stz, const int nzq) {
  using C = Cfg<MODE>;
  constexpr int WR = C::TH + 2, WC = C::TW + 2, WN = WR * WC;
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int BLK_F = C::NB * BS32;
  constexpr int GPL_F = CPLANE ? 2 * WN : 0;
  constexpr int U_F = GPL_F > BLK_F ? GPL_F : BLK_F;
  static_assert((WN * 4) % 16 == 0, "plane alignment");

  __shared__ uint32_t s_rgb[WN];
  __shared__ __attribute__((aligned(16))) float s_u[U_F];
  __shared__ __attribute__((aligned(16))) float s_rq[64];
  __shared__ __attribute__((aligned(16))) float s_thr[2][64];

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  int ty, tx;
  // this launch owns the frame statistics' reset (replaces a memset): tile 0
  // of every frame clears its items' records before k_fwd_reduce_fix adds to them
  if (stz != nullptr && blockIdx.x == 0) {
    uint64_t* z = reinterpret_cast<uint64_t*>(stz + (size_t)frame * nzq);
    for (int i = tid; i < nzq * (int)(sizeof(jds_frame_stats) / 8); i += blockDim.x) z[i] = 0ull;
    if (MQ && tid < nzq) fixcount[gridDim.y * nzq + frame * nzq + tid] = 0u;  // and the items' list lengths
  }
  if (border) {  // tiles outside the interior rectangle rect = (ty_lo, ty_hi, tx_lo, tx_hi) only
    int e = blockIdx.x;
    const int top = rect.x * g.tiles_x, bottom = (g.tiles_y - 1 - rect.y) * g.tiles_x;
    const int rows = rect.y - rect.x + 1, left = rect.z * rows;
    if (e < top) {
      ty = e / g.tiles_x;
      tx = e - ty * g.tiles_x;
    } else if ((e -= top) < bottom) {
      ty = rect.y + 1 + e / g.tiles_x;
      tx = e - (ty - rect.y - 1) * g.tiles_x;
    } else if ((e -= bottom) < left) {
      ty = rect.x + e / rect.z;
      tx = e - (ty - rect.x) * rect.z;
    } else {
      e -= left;
      const int nr = g.tiles_x - 1 - rect.w;
      ty = rect.x + e / nr;
      tx = rect.w + 1 + e - (ty - rect.x) * nr;
    }
  } else {
    ty = blockIdx.x / g.tiles_x;
    tx = blockIdx.x - ty * g.tiles_x;
  }
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  if (!MQ && tid < 64) {
    s_rq[tid] = fq[frame].rq[tid];
    s_thr[0][tid] = fq[frame].thr[0][tid];
    s_thr[1][tid] = fq[frame].thr[1][tid];
  }

  const int blk = tid >> 3, line = tid & 7;
  int plane, by_t, bx_t;
  if (blk < C::NYB) {
    plane = 0;
    by_t = blk / C::YBC;
    bx_t = blk % C::YBC;
  } else {
    const int bi = (blk - C::NYB) % C::NCB;
    plane = 1 + (blk - C::NYB) / C::NCB;
    by_t = bi / C::CBC;
    bx_t = bi % C::CBC;
  }
  const int gy = plane == 0 ? m0y * C::SY + by_t : m0y + by_t;
  const int gx = plane == 0 ? m0x * C::SX + bx_t : m0x + bx_t;
  const int nby = plane ? g.ncy : g.nby, nbx = plane ? g.ncx : g.nbx;
  const bool valid = gy >= 0 && gx >= 0 && gy < nby && gx < nbx;
  const int bidx = gy * nbx + gx;
  const float k0 = gk32[0], k1 = gk32[1], k2 = gk32[2];
  float v[8];

  // 1. stage the RGB window
  // (every load in flight before the first LDS store: one memory latency)
  const bool inside = y0 - 1 >= 0 && x0 - 1 >= 0 && y0 + C::TH + 1 <= g.H && x0 + C::TW + 1 <= g.W;
  constexpr int NL = (WN + C::TF - 1) / C::TF;
  {
    uint32_t px[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tid + l * C::TF;
      px[l] = 0u;
      if (i < WN) {
        const int r = i / WC, c = i - r * WC;
        const int yy = inside ? y0 - 1 + r : reflect101(y0 - 1 + r, g.H);
        const int xx = inside ? x0 - 1 + c : reflect101(x0 - 1 + c, g.W);
        const uint8_t* p = img + ((size_t)yy * g.W + xx) * 3;
        px[l] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
      }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tid + l * C::TF;
      if (i < WN) s_rgb[i] = px[l];
    }
  }
  __syncthreads();

  // 2. fp32 chroma planes + Gaussian row pass
  if constexpr (CPLANE) {
    float* s_cb = s_u;
    float* s_cr = s_u + WN;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int i = tid + l * C::TF;
      if (i < WN) {
        float R, G, B;
        unpack32(s_rgb[i], R, G, B);
        s_cb[i] = cb32(R, G, B);
        s_cr[i] = cr32(R, G, B);
      }
    }
    __syncthreads();
    // k_fwd32i's combined taps: the Gaussian row pass and the area's pair sum
    // in one chain, H_j over window columns 2j .. 2j+3 (pixels 2j-1 .. 2j+2 of
    // the tile), into rows of TW / 2 at the start of the planes' space
    constexpr int NRP = WR * (C::TW / 2);
    constexpr int PER = (NRP + C::TF - 1) / C::TF;
    const float h1 = gk32[3], h2 = gk32[4];
    float tb[PER], tr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C::TF;
      if (i < NRP) {
        const int r = i / (C::TW / 2), c = 2 * (i - r * (C::TW / 2));
        const float* b = s_cb + r * WC + c;
        const float* q = s_cr + r * WC + c;
        tb[j] = fmaf(k2, b[3], fmaf(h2, b[2], fmaf(h1, b[1], k0 * b[0])));
        tr[j] = fmaf(k2, q[3], fmaf(h2, q[2], fmaf(h1, q[1], k0 * q[0])));
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C::TF;
      if (i < NRP) {
        s_cb[i] = tb[j];
        s_cr[i] = tr[j];
      }
    }
    __syncthreads();
  }

  // 3. one block column per thread, DCT along axis 0
  if (valid) {
    if (plane == 0 || MODE == M444) {
      const int sx = reflect_pad(gx * 8 + line, g.W) - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sy = reflect_pad(gy * 8 + i, g.H) - y0 + 1;
        float R, G, B;
        unpack32(s_rgb[sy * WC + sx], R, G, B);
        v[i] = (plane == 0 ? luma32(R, G, B) : (plane == 1 ? cb32(R, G, B) : cr32(R, G, B))) - 128.0f;
      }
    } else if constexpr (CPLANE) {
      // pair sums of the sample's column on window rows (pixel row + 1)
      // 2r .. 2r+3 (4:2:0: combined taps, *0.25) or r .. r+2 (4:2:2: the
      // Gaussian's column form, *0.5), np.pad samples by reflected index
      constexpr int HW = C::TW / 2;
      const float* s_pl = s_u + (plane == 1 ? 0 : WN) + (reflect_pad(gx * 8 + line, g.wc) - x0 / C::SX);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int wr0 = C::SY * reflect_pad(gy * 8 + i, g.hc) - y0 + 1;  // window row of the first pixel row
        const float* col = s_pl + wr0 * HW;
        if constexpr (C::SY == 2)
          v[i] = fmaf(k2, col[2 * HW], fmaf(gk32[4], col[HW], fmaf(gk32[3], col[0], k0 * col[-HW]))) * 0.25f - 128.0f;
        else
          v[i] = fmaf(k0, col[HW] + col[-HW], k1 * col[0]) * 0.5f - 128.0f;
      }
    } else {
      const float* s_pl = s_u + (plane == 1 ? 0 : WN);
      const int sc = reflect_pad(gx * 8 + line, g.wc);
      const int wc0 = C::SX * sc - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sr = reflect_pad(gy * 8 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;
        float s[C::SY][2];
#pragma unroll
        for (int a = 0; a < C::SY; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int w = (wr0 + a) * WC + wc0 + b;
            {  // unfiltered chroma
              float R, G, B;
              unpack32(s_rgb[w], R, G, B);
              s[a][b] = plane == 1 ? cb32(R, G, B) : cr32(R, G, B);
            }
          }
        }
        if constexpr (C::SY == 2)
          v[i] = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
        else
          v[i] = (s[0][0] + s[0][1]) * 0.5f - 128.0f;
      }
    }
    fdct8_f32(v);
  }
  if constexpr (CPLANE) __syncthreads();  // the block buffer aliases the chroma planes
  float* s_blk = s_u + blk * BS32;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_blk[i * 8 + line] = v[i];
  }
  __syncthreads();

  // 4. DCT along axis 1, certified quantisation, statistics, store
  const int u = line;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = valid ? s_blk[u * 8 + k] : 0.0f;
  fdct8_f32(v);
  if constexpr (MQ) {  // shared front end: fp32 coefficients for k_quant_mq
    if (valid) {
      float4* d = reinterpret_cast<float4*>(dct32 + (long long)frame * g.cpf +
                                            (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                                            (long long)bidx * 64 + u * 8);
      d[0] = make_float4(v[0], v[1], v[2], v[3]);
      d[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
    return;
  }
  const float4* rq4 = reinterpret_cast<const float4*>(s_rq + u * 8);
  const float4* th4 = reinterpret_cast<const float4*>(s_thr[plane ? 1 : 0] + u * 8);
  const float4 ra = rq4[0], rb = rq4[1], ta = th4[0], tb = th4[1];
  const float rq[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
  const float thr[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
  int q[8];
  LaneStats ls;
  quant8(v, rq, thr, valid, q, ls, rare_row(part, g, gridDim.y, frame));
  if (valid)
    *reinterpret_cast<uint4*>(coeffs + (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                              (long long)bidx * 64 + u * 8) = pack_q(q);
  flag_block_list(ls, valid, line, frame, plane, bidx, fixlist, fixcount, g.cpf / 64);
  stats_flush(ls, valid, part + ((size_t)frame * g.tiles_y * g.tiles_x + ty * g.tiles_x + tx) * PSLOT);
}

// ---- interior tiles ------------------------------------------------------------
//
// Tiles whose RGB window (+1 px ring) lies inside the image with no padding
// (every tile but the border ring when the frame allows it).  Rows first:
//   1. one thread per 8-pixel row segment (= one block row) loads 24 B with
//      three 8-byte loads (+8 B holding the ring pixel at the segment ends),
//      converts colour in registers, runs the luma row DCT (axis 1) right there,
//      and applies the prefilter's row pass to chroma with its neighbours from
//      adjacent lanes (4:4:4: the chroma row DCTs too);
//   2. luma threads (one per block column) run the column DCT (axis 0),
//      quantise and store, while chroma threads (one per block row) form their
//      samples (vertical filter + area average), run the chroma row DCT and
//      then, as the block's column threads, the column DCT, quantise and store
//      (the 8 threads of a block are lanes of one wave: no barrier between).
// Quantised columns turn into 16-byte rows through an int16 transpose in the
// block's own (already consumed) LDS region: the 8 lanes of a block belong to
// one wave, whose LDS operations execute in order, so no barrier is needed.
// The certified bounds cover both pass orders (fast_fwd_thresholds).
template <int MODE, bool PF, bool MQ = false>
__global__ void __launch_bounds__(Cfg<MODE>::TF)
k_fwd32i(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
         const FastQ* __restrict__ fq, const float* __restrict__ gk32, uint32_t* __restrict__ part,
         uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount, const int4 rect,
         float* __restrict__ dct32,
         jds_frame_stats* __restrict__ stz, const int nzq) {
  using C = Cfg<MODE>;
  constexpr int TH = C::TH, TW = C::TW, WR = TH + 2, SEG = TW / 8;
  static_assert(16 % SEG == 0, "staging segment groups tile the 16-lane DPP rows");
  constexpr bool SUB = MODE != M444;
  constexpr bool CPLANE = SUB && PF;
  constexpr int CR = SUB ? (CPLANE ? WR : TH) : TH;  // chroma plane rows
  constexpr int NCD = SUB ? 2 * C::NCB : 1;          // chroma row-DCT blocks (SUB)
  // luma row stride: unpadded (8 or 16 floats of padding, which put the 8
  // rows of a block's in-place int16 transpose on different banks, measured
  // level: the forward is VALU-issue bound)
  constexpr int YS = TW;
  __shared__ __attribute__((aligned(16))) float s_y[TH * YS];       // luma after the row DCT
  // chroma planes (4:4:4: after the row DCT; prefiltered 4:2:x: the horizontal
  // pair sums, TW / 2 per row)
  constexpr int CW = CPLANE ? TW / 2 : TW;
  __shared__ __attribute__((aligned(16))) float s_c[2 * CR * CW];
  __shared__ __attribute__((aligned(16))) float s_cd[NCD * BS32];   // chroma blocks after the row DCT
  __shared__ __attribute__((aligned(16))) float s_rqT[64];          // 1/Q transposed: [v][k]
  __shared__ __attribute__((aligned(16))) float s_thT[2][64];

  const int tid = threadIdx.x, frame = blockIdx.y;
  const int ncol = rect.w - rect.z + 1;
  // this launch owns the frame statistics' reset (replaces a memset): tile 0
  // of every frame clears its items' records before k_fwd_reduce_fix adds to them
  if (stz != nullptr && blockIdx.x == 0) {
    uint64_t* z = reinterpret_cast<uint64_t*>(stz + (size_t)frame * nzq);
    for (int i = tid; i < nzq * (int)(sizeof(jds_frame_stats) / 8); i += blockDim.x) z[i] = 0ull;
    if (MQ && tid < nzq) fixcount[gridDim.y * nzq + frame * nzq + tid] = 0u;  // and the items' list lengths
  }
  const int ty = rect.x + (int)blockIdx.x / ncol, tx = rect.z + (int)blockIdx.x % ncol;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  // the quantiser tables by the last wave, which has no staging work: the
  // staging waves do not wait for these loads before their own
  static_assert((TH + 2) * (TW / 8) <= Cfg<MODE>::TF - 64, "the last wave is idle in the staging pass");
  if (!MQ && tid >= Cfg<MODE>::TF - 64) {
    const int l = tid - (Cfg<MODE>::TF - 64);
    const int t = (l & 7) * 8 + (l >> 3);  // [v][k] <- [k][v]
    s_rqT[l] = fq[frame].rq[t];
    s_thT[0][l] = fq[frame].thr[0][t];
    s_thT[1][l] = fq[frame].thr[1][t];
  }
  const float k0 = gk32[0], k1 = gk32[1], k2 = gk32[2];
  float* s_cb = s_c;
  float* s_cr = s_c + CR * CW;

  // ---- 1. row segments --------------------------------------------------------
  if (tid < WR * SEG) {
    // the tile's rows 1..TH on the first TH * SEG lanes (whole waves), the
    // prefilter's ring rows 0 and TH + 1 (chroma only) after them: the wave
    // holding the ring rows skips the luma row DCT as a whole
    const int r = tid < TH * SEG ? 1 + tid / SEG : (tid < (TH + 1) * SEG ? 0 : TH + 1), c = tid % SEG;
    if (CPLANE || (r >= 1 && r <= TH)) {  // uniform per row (lane groups of SEG)
      // the tile lies inside the image; only the 1-px ring may leave it:
      // BORDER_REFLECT_101 maps row -1 to 1 and row H to H-2 (columns below)
      int yrow = y0 - 1 + r;
      yrow = yrow < 0 ? -yrow : (yrow >= g.H ? 2 * g.H - 2 - yrow : yrow);
      const uint8_t* p = img + ((size_t)yrow * g.W + x0 + 8 * c) * 3;
      const uint2* p2 = reinterpret_cast<const uint2*>(p);
      const bool left_edge = x0 == 0, right_edge = x0 + TW == g.W;
      const uint2 a = p2[0], b = p2[1], d = p2[2];
      const uint2 ring = CPLANE ? p2[c == 0 ? (left_edge ? 0 : -1) : (right_edge ? 0 : 3)] : make_uint2(0u, 0u);
      const uint32_t w[6] = {a.x, a.y, b.x, b.y, d.x, d.y};
      float yy[8], cb[8], cr[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float R = (float)byte_at(w, 3 * k), G = (float)byte_at(w, 3 * k + 1), B = (float)byte_at(w, 3 * k + 2);
        yy[k] = luma32m(R, G, B);
        cb[k] = cb32(R, G, B);
        cr[k] = cr32(R, G, B);
      }
      const int o = (r - 1) * TW + 8 * c;
      if (r >= 1 && r <= TH) {
        fdct8_f32(yy);
        float4* dy = reinterpret_cast<float4*>(s_y + (r - 1) * YS + 8 * c);
        dy[0] = make_float4(yy[0], yy[1], yy[2], yy[3]);
        dy[1] = make_float4(yy[4], yy[5], yy[6], yy[7]);
      }
      if constexpr (!SUB) {
        if (r >= 1 && r <= TH) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            cb[k] -= 128.0f;
            cr[k] -= 128.0f;
          }
          fdct8_f32(cb);
          fdct8_f32(cr);
          float4* db = reinterpret_cast<float4*>(s_cb + o);
          float4* dr = reinterpret_cast<float4*>(s_cr + o);
          db[0] = make_float4(cb[0], cb[1], cb[2], cb[3]);
          db[1] = make_float4(cb[4], cb[5], cb[6], cb[7]);
          dr[0] = make_float4(cr[0], cr[1], cr[2], cr[3]);
          dr[1] = make_float4(cr[4], cr[5], cr[6], cr[7]);
        }
      } else if constexpr (CPLANE) {
        // neighbours' edge samples by DPP row shifts (a 16-lane row holds two
        // segment groups; the lanes whose source lies outside their group,
        // c == 0 and c == SEG - 1, take the ring values below)
        float lb = dpp_f32<0x111>(cb[7]), lr = dpp_f32<0x111>(cr[7]);  // row_shr:1
        float rb = dpp_f32<0x101>(cb[0]), rr = dpp_f32<0x101>(cr[0]);  // row_shl:1
        if (c == 0) {  // bytes 5..7 of the 8 before the segment; pixel 1 at the image edge
          const float R = (float)((ring.y >> 8) & 255u), G = (float)((ring.y >> 16) & 255u), B = (float)(ring.y >> 24);
          lb = left_edge ? cb[1] : cb32(R, G, B);
          lr = left_edge ? cr[1] : cr32(R, G, B);
        }
        if (c == SEG - 1) {  // bytes 0..2 of the 8 after the segment; pixel W-2 at the image edge
          const float R = (float)(ring.x & 255u), G = (float)((ring.x >> 8) & 255u), B = (float)((ring.x >> 16) & 255u);
          rb = right_edge ? cb[6] : cb32(R, G, B);
          rr = right_edge ? cr[6] : cr32(R, G, B);
        }
        // Gaussian row pass and the area's horizontal pair sum in one chain:
        // H_j = (k0, k0+k1, k1+k2, k2) . x_{2j-1 .. 2j+2} (fwd_input_error)
        const float h0 = k0, h1 = gk32[3], h2 = gk32[4], h3 = k2;
        float ob[4], orr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float bl = j == 0 ? lb : cb[2 * j - 1], br = j == 3 ? rb : cb[2 * j + 2];
          const float ql = j == 0 ? lr : cr[2 * j - 1], qr = j == 3 ? rr : cr[2 * j + 2];
          ob[j] = fmaf(h3, br, fmaf(h2, cb[2 * j + 1], fmaf(h1, cb[2 * j], h0 * bl)));
          orr[j] = fmaf(h3, qr, fmaf(h2, cr[2 * j + 1], fmaf(h1, cr[2 * j], h0 * ql)));
        }
        const int hs = psw<C::SY>(r);
        float4* db = reinterpret_cast<float4*>(s_cb + r * CW);
        float4* dr = reinterpret_cast<float4*>(s_cr + r * CW);
        db[c ^ hs] = make_float4(ob[0], ob[1], ob[2], ob[3]);
        dr[c ^ hs] = make_float4(orr[0], orr[1], orr[2], orr[3]);
      } else {
        if (r >= 1 && r <= TH) {
          const int hs = csw<C::SY>(r - 1);
          float4* db = reinterpret_cast<float4*>(s_cb + (r - 1) * TW);
          float4* dr = reinterpret_cast<float4*>(s_cr + (r - 1) * TW);
          db[(2 * c) ^ hs] = make_float4(cb[0], cb[1], cb[2], cb[3]);
          db[(2 * c + 1) ^ hs] = make_float4(cb[4], cb[5], cb[6], cb[7]);
          dr[(2 * c) ^ hs] = make_float4(cr[0], cr[1], cr[2], cr[3]);
          dr[(2 * c + 1) ^ hs] = make_float4(cr[4], cr[5], cr[6], cr[7]);
        }
      }
    }
  }
  __syncthreads();

  // ---- 2./3. column passes ------------------------------------------------------
  const int blk = tid >> 3, line = tid & 7;
  int plane, by_t, bx_t;
  if (blk < C::NYB) {
    plane = 0;
    by_t = blk / C::YBC;
    bx_t = blk % C::YBC;
  } else {
    const int bi = (blk - C::NYB) % C::NCB;
    plane = 1 + (blk - C::NYB) / C::NCB;
    by_t = bi / C::CBC;
    bx_t = bi % C::CBC;
  }
  const int gy = plane == 0 ? m0y * C::SY + by_t : m0y + by_t;
  const int gx = plane == 0 ? m0x * C::SX + bx_t : m0x + bx_t;
  // the first and last tile rows may hold whole MCU rows outside the padded
  // planes (rect admits them when fold_rows_ok holds): those blocks do not exist
  const bool valid = (unsigned)gy < (unsigned)(plane ? g.ncy : g.nby);
  const int bidx = gy * (plane ? g.ncx : g.nbx) + gx;
  int16_t* dst = coeffs + (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                 (long long)bidx * 64;
  LaneStats ls;
  // column `line` of a row-transformed block at `src` (row stride `rs` floats):
  // axis-0 DCT, quantise, int16 transpose in place, 16-byte row store
  float* dctb = MQ ? dct32 + (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                         (long long)bidx * 64
                   : nullptr;
  auto column = [&](float* src, int rs, int pl) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = src[i * rs + line];
    fdct8_f32(v);
    if constexpr (MQ) {  // shared front end: coefficient (k, line) for k_quant_mq
      if (valid) {
#pragma unroll
        for (int k = 0; k < 8; ++k) dctb[k * 8 + line] = v[k];
      }
      return;
    }
    const float4* rq4 = reinterpret_cast<const float4*>(s_rqT + line * 8);
    const float4* th4 = reinterpret_cast<const float4*>(s_thT[pl ? 1 : 0] + line * 8);
    const float4 ra = rq4[0], rb = rq4[1], ta = th4[0], tb = th4[1];
    const float rq[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    const float thr[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    int q[8];
    quant8(v, rq, thr, valid, q, ls, rare_row(part, g, gridDim.y, frame));
    // int16 transpose in place (row k at byte offset k * rs * 4).  Rotating
    // full-width rows across the wave's 8 blocks (so a block's 8 lanes read 8
    // bank groups instead of one) measured 6 us slower: the address math
    // costs more than the conflicts.
    int16_t* tq = reinterpret_cast<int16_t*>(src);
#pragma unroll
    for (int k = 0; k < 8; ++k) tq[k * rs * 2 + line] = (int16_t)q[k];
    __builtin_amdgcn_wave_barrier();  // other lanes' rows: the LDS keeps the wave's order
    const uint4 row = *reinterpret_cast<const uint4*>(tq + line * rs * 2);
    if (valid) *reinterpret_cast<uint4*>(dst + line * 8) = row;
  };

  if constexpr (SUB) {
    if (plane == 0) {
      column(s_y + by_t * 8 * YS + bx_t * 8, YS, 0);
    } else {
      // chroma sample row `line` of the block: vertical filter + area average of
      // the row-filtered (or raw) planes, then the row DCT
      const float* P = plane == 1 ? s_cb : s_cr;
      const int i = line;
      // sample row of the plane; np.pad rows (>= hc, last tile row only) reflect
      // onto rows of the same tile (fold_rows_ok)
      int gs = gy * 8 + i;
      gs = (gs < g.hc || !valid) ? gs : 2 * (g.hc - 1) - gs;
      const int pr = C::SY * (gs - m0y * 8);  // first pixel row of the sample row (tile-relative)
      const int xc = 2 * bx_t * 8;            // first pixel column of the block
      float v[8];
      if constexpr (CPLANE) {
        // the 8 samples' pair sums on the window rows of the sample row (pixel
        // row + 1): 4:2:0 the combined taps down 4 rows, *0.25; 4:2:2 the
        // Gaussian's column form over 3 rows, *0.5 (both exact scalings)
        float R[C::SY + 2][8];
        const int f0 = 2 * bx_t;  // float4 slot of the block's first pair sum
#pragma unroll
        for (int j = 0; j < C::SY + 2; ++j) {
          const int hs = psw<C::SY>(pr + j);
          const float4* s4 = reinterpret_cast<const float4*>(P + (pr + j) * CW);
          const float4 x = s4[f0 ^ hs], y = s4[(f0 + 1) ^ hs];
          R[j][0] = x.x; R[j][1] = x.y; R[j][2] = x.z; R[j][3] = x.w;
          R[j][4] = y.x; R[j][5] = y.y; R[j][6] = y.z; R[j][7] = y.w;
        }
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          if constexpr (C::SY == 2)
            v[jj] = fmaf(k2, R[3][jj], fmaf(gk32[4], R[2][jj], fmaf(gk32[3], R[1][jj], k0 * R[0][jj]))) * 0.25f - 128.0f;
          else
            v[jj] = fmaf(k0, R[2][jj] + R[0][jj], k1 * R[1][jj]) * 0.5f - 128.0f;
        }
      } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // 4 samples (8 pixel columns) at a time
        float rows[C::SY + 2][8];
#pragma unroll
        for (int j = 0; j < (CPLANE ? C::SY + 2 : C::SY); ++j) {
          const int hs = csw<C::SY>(pr + j), f = (xc + 8 * h) >> 2;
          const float4* s4 = reinterpret_cast<const float4*>(P + (pr + j) * TW);
          const float4 x = s4[f ^ hs], y = s4[(f + 1) ^ hs];
          rows[j][0] = x.x; rows[j][1] = x.y; rows[j][2] = x.z; rows[j][3] = x.w;
          rows[j][4] = y.x; rows[j][5] = y.y; rows[j][6] = y.z; rows[j][7] = y.w;
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float s[C::SY][2];
#pragma unroll
          for (int aa = 0; aa < C::SY; ++aa) {
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
              const int x = 2 * jj + bb;
              if constexpr (CPLANE)  // window row = pixel row + 1
                s[aa][bb] = fmaf(k0, rows[aa + 2][x] + rows[aa][x], k1 * rows[aa + 1][x]);
              else
                s[aa][bb] = rows[aa][x];
            }
          }
          if constexpr (C::SY == 2)
            v[4 * h + jj] = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
          else
            v[4 * h + jj] = (s[0][0] + s[0][1]) * 0.5f - 128.0f;
        }
      }
      }
      fdct8_f32(v);
      float4* d4 = reinterpret_cast<float4*>(s_cd + (blk - C::NYB) * BS32 + i * 8);
      d4[0] = make_float4(v[0], v[1], v[2], v[3]);
      d4[1] = make_float4(v[4], v[5], v[6], v[7]);
      // the block's 8 row tasks are lanes of this wave: its columns follow
      // without a workgroup barrier (LDS operations of a wave execute in order)
      column(s_cd + (blk - C::NYB) * BS32, 8, plane);
    }
  } else {
    float* P = plane == 0 ? s_y : (plane == 1 ? s_cb : s_cr);
    column(P + by_t * 8 * TW + bx_t * 8, TW, plane);
  }
  if constexpr (!MQ) {
    flag_block_list(ls, valid, line, frame, plane, bidx, fixlist, fixcount, g.cpf / 64);
    stats_flush(ls, valid, part + ((size_t)frame * g.tiles_y * g.tiles_x + ty * g.tiles_x + tx) * PSLOT);
  }
}

// ---- 4:4:4, wave-local -----------------------------------------------------------
//
// k_fwd444w: k_fwd32i's certified arithmetic for 4:4:4 plans (no subsampling,
// no prefilter: a block reads only its own 8 x 8 pixels) without the tile
// staging.  A wave owns 8 blocks in raster order, each lane one 8-pixel row of
// its block: 24-byte RGB load (np.pad reflect rows / columns at the padded
// edge, engines/block_processor.py), fp32 colour (luma32m, cb32 - 128,
// cr32 - 128: fwd_input_error's chains), then per plane the row DCT in
// registers, the block's column pass through its own LDS slot (the 8 lanes of a
// block are one wave's, whose LDS operations execute in order: no workgroup
// barrier), certified quantisation, the in-place int16 transpose and 16-byte
// row stores.  Both pass orders are covered by fast_fwd_thresholds.  A lane
// quantises 24 coefficients, so its common-bin counts are kept in 16-bit
// fields (quant8's nibbles are folded after each plane) and each 16-lane row
// stores one 8-word record into the workgroup's slot, decoded per frame by
// k_fwd_reduce_rows<16, 1>.  Measured (256 x 512^2, same box): 190 us against
// the tiled k_fwd32i<4:4:4>'s 274; 92 VGPRs, 5 waves per SIMD -- forcing 6
// spills 10 registers and takes 255 us.
constexpr int F444_WAVES = 4;

__global__ void __launch_bounds__(64 * F444_WAVES) __attribute__((amdgpu_waves_per_eu(5)))
k_fwd444w(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs, const FastQ* __restrict__ fq,
          uint32_t* __restrict__ part, uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount,
          jds_frame_stats* __restrict__ stz) {
  __shared__ __attribute__((aligned(16))) float s_blk[8 * F444_WAVES * BS32];
  __shared__ __attribute__((aligned(16))) float s_rqT[64];
  __shared__ __attribute__((aligned(16))) float s_thT[2][64];
  const int tid = threadIdx.x, lv = tid & 7, lb = tid >> 3;
  const int frame = blockIdx.y;
  if (blockIdx.x == 0) {  // this launch owns the frame statistics' reset (k_fwd_reduce adds after it)
    uint64_t* z = reinterpret_cast<uint64_t*>(stz + frame);
    for (int i = tid; i < (int)(sizeof(jds_frame_stats) / 8); i += blockDim.x) z[i] = 0ull;
  }
  if (tid < 64) {
    const int t = (tid & 7) * 8 + (tid >> 3);  // [v][k] <- [k][v]
    s_rqT[tid] = fq[frame].rq[t];
    s_thT[0][tid] = fq[frame].thr[0][t];
    s_thT[1][tid] = fq[frame].thr[1][t];
  }
  __syncthreads();

  const int nblk = g.nby * g.nbx;
  const int blk = blockIdx.x * (8 * F444_WAVES) + lb;
  const bool valid = blk < nblk;
  const int bq = valid ? blk : 0;
  const int by = bq / g.nbx, bx = bq - by * g.nbx;
  const int y = by * 8 + lv, x0 = bx * 8;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  uint32_t w[6];
  {
    const int yr = reflect_pad(y, g.H);
    const uint8_t* row = img + (size_t)yr * g.W * 3;
    if (x0 + 8 <= g.W && (g.W & 7) == 0) {  // 8-byte aligned rows: three 8-byte loads
      const uint2* p2 = reinterpret_cast<const uint2*>(row + (size_t)x0 * 3);
      const uint2 a = p2[0], b = p2[1], c = p2[2];
      w[0] = a.x; w[1] = a.y; w[2] = b.x; w[3] = b.y; w[4] = c.x; w[5] = c.y;
    } else {
#pragma unroll
      for (int i = 0; i < 6; ++i) w[i] = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint8_t* px = row + (size_t)reflect_pad(x0 + k, g.W) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) w[(3 * k + c) >> 2] |= (uint32_t)px[c] << (8 * ((3 * k + c) & 3));
      }
    }
  }

  LaneStats ls;
  unsigned acc[4] = {0u, 0u, 0u, 0u};  // common bins 22..29 in 16-bit fields: (22, 23), (24, 25), ...
  float* slot = s_blk + lb * BS32;
  int16_t* tq = reinterpret_cast<int16_t*>(slot);
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    // the plane's samples from the packed bytes, per plane (fewer live registers
    // than all three planes at once)
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float R = (float)byte_at(w, 3 * k), G = (float)byte_at(w, 3 * k + 1), B = (float)byte_at(w, 3 * k + 2);
      v[k] = p == 0 ? luma32m(R, G, B) : (p == 1 ? cb32(R, G, B) - 128.0f : cr32(R, G, B) - 128.0f);
    }
    fdct8_f32(v);  // axis 1 of row lv
    float4* d4 = reinterpret_cast<float4*>(slot + lv * 8);
    d4[0] = make_float4(v[0], v[1], v[2], v[3]);
    d4[1] = make_float4(v[4], v[5], v[6], v[7]);
    __builtin_amdgcn_wave_barrier();
    float c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = slot[i * 8 + lv];  // column lv
    fdct8_f32(c);                                           // axis 0
    const float4* rq4 = reinterpret_cast<const float4*>(s_rqT + lv * 8);
    const float4* th4 = reinterpret_cast<const float4*>(s_thT[p ? 1 : 0] + lv * 8);
    const float4 ra = rq4[0], rb = rq4[1], ta = th4[0], tb = th4[1];
    const float rq[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    const float thr[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    int q[8];
    ls.hn = 0u;
    ls.nflag = 0u;
    // (rare bins to the frame's rare row behind the workgroups' slots)
    quant8(c, rq, thr, valid, q, ls, part + (size_t)gridDim.y * gridDim.x * PSLOT + (size_t)frame * 64);
    __builtin_amdgcn_wave_barrier();  // every lane's column read precedes the int16 rows
#pragma unroll
    for (int k = 0; k < 8; ++k) tq[k * 16 + lv] = (int16_t)q[k];
    __builtin_amdgcn_wave_barrier();
    const uint4 rowq = *reinterpret_cast<const uint4*>(tq + lv * 16);
    if (valid)
      *reinterpret_cast<uint4*>(coeffs + (long long)frame * g.cpf + (p == 0 ? 0 : (p == 1 ? g.off_cb : g.off_cr)) +
                                (long long)bq * 64 + lv * 8) = rowq;
    flag_block_list(ls, valid, lv, frame, p, bq, fixlist, fixcount, g.cpf / 64);
    const unsigned h = ls.hn;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += ((h >> (8 * j)) & 15u) | (((h >> (8 * j + 4)) & 15u) << 16);
    __builtin_amdgcn_wave_barrier();  // the rows are read before the next plane writes the slot
  }

  // ---- statistics: row sums, one record per 16-lane row
  unsigned r5[4] = {acc[0], acc[1], acc[2], acc[3]};
  unsigned nzmb = ls.nz | (ls.mb << 16);  // <= 24 and <= 24 * 16 per lane
  if (!valid) {
    r5[0] = r5[1] = r5[2] = r5[3] = 0u;
    nzmb = 0u;
  }
  row_sums4(r5);
  nzmb += (unsigned)__builtin_amdgcn_update_dpp(0, (int)nzmb, 0x111, 0xf, 0xf, true);  // row_shr 1, 2, 4, 8
  nzmb += (unsigned)__builtin_amdgcn_update_dpp(0, (int)nzmb, 0x112, 0xf, 0xf, true);
  nzmb += (unsigned)__builtin_amdgcn_update_dpp(0, (int)nzmb, 0x114, 0xf, 0xf, true);
  nzmb += (unsigned)__builtin_amdgcn_update_dpp(0, (int)nzmb, 0x118, 0xf, 0xf, true);
  // each 16-lane row's sums (and its valid lanes) straight into the
  // workgroup's slot, decoded by k_fwd_reduce_rows<16, 1>
  const int wv = tid >> 6, lane = tid & 63;
  const unsigned long long vb = __ballot(valid);  // (the whole wave's: a ballot inside the branch sees 4 lanes)
  if ((lane & 15) == 15) {
    const unsigned rv = (unsigned)__popcll(vb & (0xffffull << (lane & 48)));
    uint32_t* rec = part + ((size_t)frame * gridDim.x + blockIdx.x) * PSLOT + 8 * (4 * wv + (lane >> 4));
    *reinterpret_cast<uint4*>(rec) = make_uint4(r5[0], r5[1], r5[2], r5[3]);
    *reinterpret_cast<uint2*>(rec + 4) = make_uint2(nzmb, rv);
  }
}

// The forward statistics' reduction: the row records of 64 tiles of frame blockIdx.y per
// workgroup (nrec = 4 x waves per tile), decoded into the 8 common bins, the
// nonzero count, the magnitude bits and the zeros (8 coefficients per valid
// lane, all in bin 25 by the nibble counters: taken back), summed per thread,
// then per wave (DPP-based __reduce_add_sync) and per workgroup (LDS), and
// added to the frame stats; workgroup 0 of the frame also adds and re-zeroes
// the frame's rare-bin row for the next run.
constexpr int RROWS_TILES = 64;  // tiles per k_fwd_reduce_rows workgroup
// FMT 0: k_fwd32i's 4-word records (8-bit fields); FMT 1: k_fwd444w's 8-word
// records (16-bit fields, 24 coefficients per valid lane).  ptiles = slots per
// frame.  One workgroup of NT threads reduces tiles [RT * slice, RT * slice +
// RT) of frame f (k_fwd_reduce_rows: NT = 256, RT = 64; k_fix_fwd's reduction
// workgroups: NT = 64, RT = 16).
template <int NREC, int FMT, int NT, int RT>
__device__ __forceinline__ void reduce_rows_wg(jds_frame_stats* __restrict__ st, uint32_t* __restrict__ part,
                                               const int ptiles, const int nframes, const int f, const int slice,
                                               unsigned (*s_acc)[11]) {
  constexpr int RW = FMT ? 8 : 4;  // words per record
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int t0 = slice * RT, t1 = min(ptiles, t0 + RT);
  unsigned acc[11] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // bins 22..29, nz, mb, zeros
  const int nr = (t1 - t0) * NREC;
  // a fixed trip count with compile-time record arithmetic: every load issued before the first use
  static_assert((RT * NREC) % NT == 0, "whole record passes");
  static_assert(RW * NREC <= PSLOT, "records fit the slot");
  uint4 xs[RT * NREC / NT], ys[FMT ? RT * NREC / NT : 1];
#pragma unroll
  for (int it = 0; it < RT * NREC / NT; ++it) {
    const int i = t + NT * it;
    const int tile = t0 + i / NREC, r = i % NREC;
    const uint32_t* rec = part + ((size_t)f * ptiles + tile) * PSLOT + RW * r;
    xs[it] = i < nr ? *reinterpret_cast<const uint4*>(rec) : make_uint4(0u, 0u, 0u, 0u);
    if constexpr (FMT) ys[it] = i < nr ? *reinterpret_cast<const uint4*>(rec + 4) : make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (int it = 0; it < RT * NREC / NT; ++it) {
    const uint4 x = xs[it];
    if constexpr (FMT == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += (x.x >> (8 * j)) & 255u;
        acc[2 * j + 1] += (x.y >> (8 * j)) & 255u;
      }
      const unsigned nz = x.z & 255u, nv = (x.z >> 8) & 255u;
      acc[8] += nz;
      acc[9] += x.z >> 16;
      acc[10] += 8u * nv - nz;
    } else {
      // word j: bins 2j (low 16 bits) and 2j + 1 (high); then nz | mb << 16, valid lanes
      const uint4 y = ys[it];
      const unsigned wd[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += wd[j] & 0xffffu;
        acc[2 * j + 1] += wd[j] >> 16;
      }
      const unsigned nz = y.x & 0xffffu;
      acc[8] += nz;
      acc[9] += y.x >> 16;
      acc[10] += 24u * y.y - nz;
    }
  }
#pragma unroll
  for (int k = 0; k < 11; ++k) {
    const unsigned v = __reduce_add_sync(~0ull, acc[k]);
    if (lane == 0) s_acc[w][k] = v;
  }
  __syncthreads();
  auto wsum = [&](int k) {
    unsigned long long v = 0ull;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += s_acc[q][k];
    return v;
  };
  jds_frame_stats* sf = st + f;
  if (t < 11) {
    const unsigned long long v = wsum(t);
    if (t < 8) {
      // bin 22 + t; zeros fall in bin 25 (k_finalize adds them back)
      const unsigned long long z = t == 3 ? wsum(10) : 0ull;
      if (v - z) atomicAdd((unsigned long long*)&sf->hist[22 + t], v - z);
    } else if (t == 8) {
      if (v) atomicAdd((unsigned long long*)&sf->nonzero, v);
    } else if (t == 9) {
      const unsigned long long nz = wsum(8);
      if (v + nz) atomicAdd((unsigned long long*)&sf->magnitude_bits, v + nz);  // bit length + 1 per nonzero
    }
  }
  // slice 0 also adds the frame's rare-bin row and re-zeroes it for the next run
  const int b = NT > 64 ? t - 64 : t - 14;
  if (slice == 0 && b >= 0 && b < 50) {
    unsigned* rr = part + (size_t)nframes * ptiles * PSLOT + (size_t)f * 64;  // the frame's rare row
    const unsigned v = rr[2 + b];
    if (v) {
      atomicAdd((unsigned long long*)&sf->hist[b], (unsigned long long)v);
      rr[2 + b] = 0u;
    }
  }
}

template <int NREC, int FMT = 0>
__global__ void __launch_bounds__(256)
k_fwd_reduce_rows(const Geo g, jds_frame_stats* __restrict__ st, uint32_t* __restrict__ part, const int ptiles) {
  __shared__ unsigned s_acc[4][11];
  (void)g;
  reduce_rows_wg<NREC, FMT, 256, RROWS_TILES>(st, part, ptiles, (int)gridDim.y, (int)blockIdx.y, (int)blockIdx.x,
                                              s_acc);
}

// words of the statistics partials a single-quality 8x8 plan needs (tile slots
// of row records, plus the frames' rare-bin rows); the buffer starts zeroed
size_t fast_part_words(const Geo& g, int n) {
  return ((size_t)PSLOT * g.tiles_y * g.tiles_x + 64) * (size_t)n;
}

// workgroups per frame of k_fwd444w (its statistics partials per frame)
int fwd444w_groups(const Geo& g) { return (g.nby * g.nbx + 8 * F444_WAVES - 1) / (8 * F444_WAVES); }

// End of the certified forward's producer launches: the statistics partials
// into the frame stats (reduce_partials), then (sweep plans) bitmap -> list:
// each wave takes 64 bitmap words of the workgroup's share of item f's
// bitmap, prefix-sums their set bits, reserves its slots with one atomic on
// the item's counter (zeroed by the front-end launch), writes the block
// indices in order and clears the words for the next run.  Only this small
// launch waits for an atomic's return; the producers' atomic ORs do not.
__global__ void __launch_bounds__(512)
k_fwd_reduce_fix(const Geo g, jds_frame_stats* st, const uint32_t* __restrict__ part, int ptiles,
                 uint32_t* __restrict__ fixbits, uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount) {
  reduce_partials(st, part, ptiles);
  // sweep plans only (single-quality plans reduce in k_fix_fwd): list lengths
  // accumulate at fixcount[n + item]
  unsigned* const fixlen = fixcount + gridDim.y;
  const int item = blockIdx.y, wpi = fix_wpi(g), lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = (wpi + gridDim.x - 1) / gridDim.x, w_end = min(wpi, (blockIdx.x + 1) * per);
  const long long nyb = (long long)g.nby * g.nbx, ncb = (long long)g.ncy * g.ncx, cap = g.cpf / 64;
  uint32_t* bits = fixbits + (size_t)item * wpi;
  uint2* list = fixlist + (size_t)item * cap;
  for (int w0 = blockIdx.x * per + wave * 64; w0 < w_end; w0 += 8 * 64) {
    const int w = w0 + lane;
    uint32_t word = 0u;
    if (w < w_end) {
      word = bits[w];
      if (word) bits[w] = 0u;
    }
    if (!__ballot(word != 0u)) continue;  // wave-uniform
    const unsigned c = (unsigned)__popc(word);
    unsigned incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    unsigned base = 0u;
    if (lane == 63) base = atomicAdd(fixlen + item, incl);  // zeroed by the front-end launch
    base = __shfl(base, 63, 64) + incl - c;
    while (word) {
      const long long b = (long long)w * 32 + (__ffs(word) - 1);
      word &= word - 1u;
      const int plane = b < nyb ? 0 : (b < nyb + ncb ? 1 : 2);
      const int bidx = (int)(b - (plane == 0 ? 0 : (plane == 1 ? nyb : nyb + ncb)));
      list[base++] = make_uint2((unsigned)item, ((unsigned)plane << 24) | (unsigned)bidx);
    }
  }
}

// One listed block per 64-thread workgroup iteration (grid-strides over the
// fix list): every thread forms one sample exactly, then 8 threads run the
// column and row transforms, requantize and correct the statistics.
// Two grid shapes (a block's exact chain is latency-bound, so the lever is how
// many chains run at once):
// * per item (n_flat = 0; single-quality plans, similar list lengths): grid
//   (x, items), item blockIdx.y's list strided over blockIdx.x;
// * flat (n_flat = items; sweep plans, where the Q95 item's list is ~10x the
//   Q5 item's): one grid over the concatenated lists, so a long list gets as
//   many workgroups as it has entries.  Each workgroup prefix-sums the n list
//   lengths in LDS (dynamic, 4 (n + 1) bytes) and maps its entry index to
//   (item, slot) by binary search.
// NRED > 0 (single-quality plans): the last nred workgroups of each item's row
// are the statistics reduction instead (k_fwd_reduce_rows' work, 16 tiles of
// NRED row records each, 64 threads): both roles only add into the frame
// statistics, and the latency-bound reduction runs beside the latency-bound
// fix-up instead of after it, one launch fewer.
constexpr int FIX_RED_TILES = 16;
template <int MODE, bool PF, int NRED = 0, int RFMT = 0>
#ifndef JDS_FIX_WPE  // tools: A/B builds of the fix-up's register budget
#define JDS_FIX_WPE 5
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(JDS_FIX_WPE)))
k_fix_fwd(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
          const FrameQ* __restrict__ fq, const double* __restrict__ gk, jds_frame_stats* __restrict__ st,
          const uint2* __restrict__ fixlist, const unsigned* __restrict__ fixcount, const int nq, const int n_flat,
          unsigned* __restrict__ rearm, uint32_t* __restrict__ part = nullptr, const int ptiles = 0,
          const int nred = 0) {
  const int gfix = (int)gridDim.x - nred;  // the fix-up role's workgroups per item
  if constexpr (NRED > 0) {
    if ((int)blockIdx.x >= gfix) {  // (uniform) the reduction role
      __shared__ unsigned s_acc[1][11];
      reduce_rows_wg<NRED, RFMT, 64, FIX_RED_TILES>(st, part, ptiles, (int)gridDim.y, (int)blockIdx.y,
                                                  (int)blockIdx.x - gfix, s_acc);
      return;
    }
  }
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int SY = Cfg<MODE>::SY;
  constexpr int WRR = 8 * SY + 2, WCC = 18;  // prefilter source window of one chroma block
  __shared__ double s_b[64];
  __shared__ double s_w[CPLANE ? WRR * WCC : 1];         // fp64 chroma of the window
  __shared__ double s_rf[CPLANE ? WRR * (WCC - 2) : 1];  // after the row pass
  extern __shared__ unsigned s_off[];                    // flat grids: list starts, [n_flat + 1]
  const int t = threadIdx.x;
  const unsigned cap = (unsigned)(g.cpf / 64);  // list capacity per item
  unsigned count;
  const uint2* __restrict__ list;
  uint2 next;
  if (n_flat) {
#pragma unroll 8
    for (int i = t; i < n_flat; i += 64) s_off[i + 1] = fixcount[i];
    if (t == 0) s_off[0] = 0u;
    __syncthreads();
    unsigned run = 0u;
    for (int c0 = 0; c0 < n_flat; c0 += 64) {  // inclusive scan, 64 lengths at a time
      const int i = c0 + t;
      unsigned x = i < n_flat ? s_off[i + 1] : 0u;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o, 64);
        if (t >= o) x += y;
      }
      if (i < n_flat) s_off[i + 1] = run + x;
      run += __shfl(x, 63, 64);
    }
    __syncthreads();
    count = s_off[n_flat];
    list = fixlist;
    next = make_uint2(0u, 0u);
  } else {
    // length fixcount[item] (single-quality plans: the live counter the front
    // end appended to; sweeps: k_fwd_reduce_fix's list length); the first
    // entry is read beside it (in bounds, maybe stale when blockIdx.x >= count,
    // then unused): one memory latency instead of two
    count = min(fixcount[blockIdx.y], cap);
    list = fixlist + (size_t)blockIdx.y * cap;
    next = blockIdx.x < cap ? list[blockIdx.x] : make_uint2(0u, 0u);
    // single-quality plans: the other counter bank, which the next run appends
    // to, is re-armed here
    if (rearm != nullptr && blockIdx.x == 0 && t == 0) rearm[blockIdx.y] = 0u;
  }
  const double k[3] = {gk[0], gk[1], gk[2]};
  for (unsigned e = blockIdx.x; e < count; e += (unsigned)gfix) {
    uint2 ent;
    if (n_flat) {  // entry e of the concatenated lists: item = last start <= e
      int lo = 0, hi = n_flat - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= e) lo = mid; else hi = mid - 1;
      }
      ent = list[(size_t)lo * cap + (e - s_off[lo])];
    } else {
      ent = next;
      if (e + gfix < count) next = list[e + gfix];
    }
    const int frame = (int)ent.x;
    const int plane = (int)(ent.y >> 24);
    const int bidx = (int)(ent.y & 0xffffffu);
    const int nbx = plane ? g.ncx : g.nbx;
    const int gy = bidx / nbx, gx = bidx - gy * nbx;
    const uint8_t* img = rgb + (size_t)(frame / nq) * g.H * g.W * 3;  // item -> its frame
    const int i = t >> 3, j = t & 7;
    // lanes 0-7 (row u = t of the block): the stored row, fetched now so its
    // latency hides under the sampling below
    const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                          (long long)bidx * 64 + (t & 7) * 8;
    uint4* dst = reinterpret_cast<uint4*>(coeffs + off);
    uint4 old = make_uint4(0u, 0u, 0u, 0u);
    if (t < 8) old = *dst;
    // prefiltered chroma of a block without np.pad samples: stage the source
    // window once (colour, then the row pass, in LDS), same fp64 operations as
    // sample64; window rows/columns outside the image are cv2's
    // BORDER_REFLECT_101 pixels, so edge blocks stage too (sample64 per sample
    // chains ~4 dependent load rounds per thread: such blocks set the tail)
    const int wy0 = SY * 8 * gy - 1, wx0 = 16 * gx - 1;
    const bool staged = CPLANE && plane != 0 && gy * 8 + 8 <= g.hc && gx * 8 + 8 <= g.wc;
    if (staged) {  // uniform per workgroup
      // every window load in flight before the first use (one memory latency)
      constexpr int NWL = (WRR * WCC + 63) / 64;
      uint32_t px[NWL];
#pragma unroll
      for (int l = 0; l < NWL; ++l) {
        const int q = t + 64 * l;
        px[l] = 0u;
        if (q < WRR * WCC) {
          const int r = q / WCC, c = q - r * WCC;
          const uint8_t* p = img + ((size_t)reflect101(wy0 + r, g.H) * g.W + reflect101(wx0 + c, g.W)) * 3;
          px[l] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
        }
      }
#pragma unroll
      for (int l = 0; l < NWL; ++l) {
        const int q = t + 64 * l;
        if (q < WRR * WCC) {
          double R, G, B;
          unpack(px[l], R, G, B);
          s_w[q] = plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B);
        }
      }
      __syncthreads();
      for (int q = t; q < WRR * (WCC - 2); q += 64) {
        const int r = q / (WCC - 2), c = q - r * (WCC - 2) + 1;
        const double* w = s_w + r * WCC + c;
        double a = k[0] * w[-1];
        a = a + k[1] * w[0];
        s_rf[q] = a + k[2] * w[1];
      }
      __syncthreads();
      double sm[SY][2];
#pragma unroll
      for (int a = 0; a < SY; ++a) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const double* f = s_rf + (SY * i + a + 1) * (WCC - 2) + 2 * j + b;  // window row of pixel row
          const double d = k[1] * f[0] + 0.0;
          sm[a][b] = d + k[0] * (f[WCC - 2] + f[-(WCC - 2)]);
        }
      }
      double v;
      if constexpr (SY == 2)
        v = (((sm[0][0] + sm[0][1]) + sm[1][0]) + sm[1][1]) * 0.25;
      else
        v = (sm[0][0] + sm[0][1]) * 0.5;
      s_b[t] = v - 128.0;
    } else {
      s_b[t] = sample64<MODE, PF>(img, g, plane, gy * 8 + i, gx * 8 + j, k) - 128.0;
    }
    __syncthreads();
    double v[8];
    if (t < 8) {  // axis 0, column t
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = s_b[r * 8 + t];
      dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
      for (int r = 0; r < 8; ++r) s_b[r * 8 + t] = v[r];
    }
    __syncthreads();
    if (t < 8) {  // axis 1, row u = t; requantize and correct the stats
      const int u = t;
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = s_b[u * 8 + c];
      dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
      const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
      uint32_t nw[4] = {0u, 0u, 0u, 0u};
      long long dnz = 0, dmb = 0;
      jds_frame_stats* fs = st + frame;
      double qd[8], rq[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        qd[c] = fq[frame].q16[u * 8 + c];
        rq[c] = recip64(qd[c]);
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        // rint(v / Q) without an fp64 division (rint_quot: the division only
        // when the product lies within |t| 2^-49 of a half-integer)
        const int qn = rint_quot(v[c], qd[c], rq[c]);
        const int qo = (int16_t)((ow[c >> 1] >> ((c & 1) * 16)) & 0xffffu);
        nw[c >> 1] |= (uint32_t)(uint16_t)qn << ((c & 1) * 16);
        if (qn != qo) {
          const int mo = qo < 0 ? -qo : qo, mn = qn < 0 ? -qn : qn;
          if (mo) {
            --dnz;
            dmb -= 33 - __clz(mo);
            if (qo >= -100 && qo <= 100)
              atomicAdd((unsigned long long*)&fs->hist[qo == 100 ? 49 : (qo + 100) >> 2], ~0ull);
          }
          if (mn) {
            ++dnz;
            dmb += 33 - __clz(mn);
            if (qn >= -100 && qn <= 100)
              atomicAdd((unsigned long long*)&fs->hist[qn == 100 ? 49 : (qn + 100) >> 2], 1ull);
          }
        }
      }
      *dst = make_uint4(nw[0], nw[1], nw[2], nw[3]);
      if (dnz) atomicAdd((unsigned long long*)&fs->nonzero, (unsigned long long)dnz);
      if (dmb) atomicAdd((unsigned long long*)&fs->magnitude_bits, (unsigned long long)dmb);
    }
    __syncthreads();
  }
}


// ---- shared front end: one quality sweep item per table ------------------------
//
// A sweep plan (jds_plan_create_q) holds nq tables per frame.  The front-end
// kernels (MQ = true) write each frame's fp32 coefficients once; here one thread
// per block row certifies-and-quantises them for every table of the frame
// (item = frame * nq + q), stores the int16 rows, lists uncertain blocks for
// k_fix_fwd and keeps per-item statistics.  The colour / prefilter /
// subsample / DCT work is then done once per frame instead of once per item
// ("the Q-independent front end ... is reused across Qs").
constexpr int MAXQ = 8;

int quant_mq_tiles(const Geo& g) {  // workgroups per frame (<= 31 rows per lane: byte-wide histogram counters)
  const long long rows = g.cpf / 8;
  long long t = (rows + 256LL * 31 - 1) / (256LL * 31);
  return (int)(t < 256 ? 256 : t);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_quant_mq(const Geo g, const int nq, const float* __restrict__ dct32, int16_t* __restrict__ coeffs,
           const FastQ* __restrict__ fq, uint32_t* __restrict__ part, uint32_t* __restrict__ fixbits) {
  __shared__ __attribute__((aligned(16))) float s_rq[MAXQ][64];
  __shared__ __attribute__((aligned(16))) float s_th[MAXQ][2][64];
  __shared__ unsigned s_st[MAXQ][NSTAT];
  __shared__ unsigned s_rh[MAXQ][RH_WORDS];  // replicated rare-bin histograms (quant8<true>)
  const int tid = threadIdx.x, f = blockIdx.y, ptiles = gridDim.x;
  for (int i = tid; i < nq * 64; i += 256) {
    const int q = i >> 6, k = i & 63;
    const FastQ& t = fq[f * nq + q];
    s_rq[q][k] = t.rq[k];
    s_th[q][0][k] = t.thr[0][k];
    s_th[q][1][k] = t.thr[1][k];
  }
  for (int i = tid; i < MAXQ * NSTAT; i += 256) (&s_st[0][0])[i] = 0u;
  for (int i = tid; i < MAXQ * RH_WORDS; i += 256) (&s_rh[0][0])[i] = 0u;
  __syncthreads();
  const long long rows = g.cpf / 8, nyb = (long long)g.nby * g.nbx, ncb = (long long)g.ncy * g.ncx;
  unsigned nz[MAXQ], mb[MAXQ], be[MAXQ], bo[MAXQ], nrows = 0u;
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) nz[q] = mb[q] = be[q] = bo[q] = 0u;
  const long long step = (long long)ptiles * 256;
  // the next row's coefficients are requested before this row is quantised
  const float4* __restrict__ src = reinterpret_cast<const float4*>(dct32 + (long long)f * g.cpf);
  float4 nx = make_float4(0.f, 0.f, 0.f, 0.f), ny = nx;
  {
    const long long rw = (long long)blockIdx.x * 256 + tid;
    if (rw < rows) { nx = src[rw * 2]; ny = src[rw * 2 + 1]; }
  }
  // uniform trip count per wave (flag_block ballots over the 8 rows of a block)
  for (long long r0 = (long long)blockIdx.x * 256; r0 < rows; r0 += step) {
    const long long rw = r0 + tid;
    const bool valid = rw < rows;
    const long long b = valid ? rw >> 3 : 0;
    const int u = (int)(rw & 7);
    const int plane = b < nyb ? 0 : (b < nyb + ncb ? 1 : 2);
    const int bidx = (int)(b - (plane == 0 ? 0 : (plane == 1 ? nyb : nyb + ncb)));
    const float v[8] = {nx.x, nx.y, nx.z, nx.w, ny.x, ny.y, ny.z, ny.w};  // stale past the end (every use is masked by valid)
    nrows += valid ? 1u : 0u;
    if (rw + step < rows) { nx = src[(rw + step) * 2]; ny = src[(rw + step) * 2 + 1]; }
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      if (q < nq) {
        const float4* rq4 = reinterpret_cast<const float4*>(&s_rq[q][u * 8]);
        const float4* th4 = reinterpret_cast<const float4*>(&s_th[q][plane ? 1 : 0][u * 8]);
        const float4 ra = rq4[0], rb = rq4[1], ta = th4[0], tb = th4[1];
        const float rq[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        const float thr[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
        int qv[8];
        LaneStats ls;
        quant8<true>(v, rq, thr, valid, qv, ls, s_rh[q]);
        const int item = f * nq + q;
        if (valid) *reinterpret_cast<uint4*>(coeffs + (long long)item * g.cpf + rw * 8) = pack_q(qv);
        flag_block_bits(ls, valid, u, item, b, fixbits, fix_wpi(g));
        if (valid) {
          nz[q] += ls.nz;
          mb[q] += ls.mb;
          be[q] += ls.hn & 0x0f0f0f0fu;         // bins 22, 24, 26, 28 (bytes)
          bo[q] += (ls.hn >> 4) & 0x0f0f0f0fu;  // bins 23, 25, 27, 29
        }
      }
    }
  }
  // per item: wave sums (16-bit fields), workgroup sums in LDS, one partial slot
  const unsigned wrows = __reduce_add_sync(~0ull, nrows);
#pragma unroll
  for (int q = 0; q < MAXQ; ++q) {
    if (q < nq) {
      const unsigned w0 = __reduce_add_sync(~0ull, be[q] & 0x00ff00ffu), w1 = __reduce_add_sync(~0ull, (be[q] >> 8) & 0x00ff00ffu);
      const unsigned w2 = __reduce_add_sync(~0ull, bo[q] & 0x00ff00ffu), w3 = __reduce_add_sync(~0ull, (bo[q] >> 8) & 0x00ff00ffu);
      const unsigned wmb = __reduce_add_sync(~0ull, mb[q]), wnz = __reduce_add_sync(~0ull, nz[q]);
      if ((tid & 63) == 0) {
        atomicAdd(&s_st[q][0], wnz);
        atomicAdd(&s_st[q][1], wmb + wnz);
        const unsigned zeros = 8u * wrows - wnz;
        const unsigned c[8] = {w0 & 0xffffu, w2 & 0xffffu, w1 & 0xffffu, (w3 & 0xffffu) - zeros,
                               w0 >> 16,     w2 >> 16,     w1 >> 16,     w3 >> 16};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c[j]) atomicAdd(&s_st[q][2 + 22 + j], c[j]);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < nq * NSTAT; i += 256) {
    const int q = i / NSTAT, j = i - q * NSTAT;
    part[((size_t)(f * nq + q) * ptiles + blockIdx.x) * NSTAT + j] =
        s_st[q][j] + (j >= 2 ? rare_bin_total(s_rh[q], j - 2) : 0u);
  }
}

// ------------------------------------------------------------ launchers --

hipError_t launch_fwd_finish(const Geo& g, int n, jds_frame_stats* st, const uint32_t* part, int ptiles,
                             hipStream_t s);
// The first and last tile rows hold whole MCU rows outside the padded planes
// (tiles are bottom-aligned: ty_off MCU rows above the image; a partial last
// MCU row below it, e.g. 1080p 4:2:0).  k_fwd32i takes them too -- one launch
// instead of a border launch of a few thousand workgroups; measured per 64 x
// 1080p: k_fwd32i 327.7 + k_fwd32 26.7 -> 337.1 us; per 16 x 4K 4:2:0: 331.8 +
// 14.6 -> 339.1 us -- when
//  * H % 8 == 0: a luma block lies wholly in the image or does not exist;
//  * np.pad's reflected chroma rows of the last block row (hc .. 8 ncy - 1 ->
//    2 (hc - 1) - row) come from sample rows whose pixel rows (and the
//    prefilter's ring) lie in the same tile window;
//  * the window rows BORDER_REFLECT_101 maps (-yrow, 2H - 2 - yrow) stay in
//    the image.
// Blocks outside the planes are masked (k_fwd32i `valid`).
template <int MODE>
static void fold_rows(const Geo& g, int4& rect) {
  using C = Cfg<MODE>;
  if (g.H % 8 != 0 || g.H < C::TH + 2) return;
  if (rect.x == 1) {
    const int y0 = -g.ty_off * C::MH;  // tile row 0
    if (1 - y0 <= g.H - 1) rect.x = 0;
  }
  if (rect.y == g.tiles_y - 2) {
    const int y0 = ((g.tiles_y - 1) * C::MY - g.ty_off) * C::MH;
    bool ok = y0 >= 1 && y0 + C::TH <= 2 * g.H - 2;
    const int hp = g.ncy * 8;  // padded chroma rows
    if (MODE != M444 && hp > g.hc) {
      const int rmin = 2 * (g.hc - 1) - (hp - 1);
      ok = ok && rmin >= 0 && C::SY * rmin >= y0;
    }
    if (ok) rect.y = g.tiles_y - 1;
  }
}

// k_fix_fwd workgroups in all (x items, grid-stride over each item's list):
// typical lists (0.4 % of 3M blocks at Q50) need one block per workgroup
constexpr int FIX_GRID = 16384;

template <int MODE, bool PF>
static hipError_t fast_fwd_t(const Geo& g, int n, int nq, const uint8_t* rgb, int16_t* coeffs, const FrameQ* fq,
                             const FastQ* fq32, const double* gk, const float* gk32, jds_frame_stats* st,
                             uint32_t* part, uint32_t* fixbits, uint2* fixlist, unsigned* fixcount, float* dct32, hipStream_t s,
                             bool finish, int par) {
  using C = Cfg<MODE>;
  const bool mq = nq > 1;  // sweep plan: front end once per frame into dct32, then k_quant_mq
  const int nf = n / nq;   // frames (n = items)
  // single quality: the front end appends to live counter bank `par` (of two)
  unsigned* const fc = mq ? fixcount : fixcount + par * n;
  // Tiles lying wholly inside the image (no padding blocks, no phantom MCUs;
  // only the 1-px ring may reflect) form a rectangle of tile indices and take
  // k_fwd32i; the rest run in k_fwd32 before it on the same stream (a side
  // stream for them measured no gain: the fork / join costs what the overlap
  // returns).  4:4:4 single-quality plans: the wave-local kernel (k_fwd444w)
  // for every block.
  if (MODE == M444 && !mq) {
    const int ng = fwd444w_groups(g);
    hipLaunchKernelGGL(k_fwd444w, dim3(ng, n), dim3(64 * F444_WAVES), 0, s, g, rgb, coeffs, fq32, part, fixlist, fc, st);
    kmark(s, "k_fwd444w");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int gx = FIX_GRID / n > 1 ? FIX_GRID / n : 1;
    static_assert(F444_WAVES * 4 == 16, "16 row records per k_fwd444w workgroup");
    // the fix-up and the statistics reduction in one launch (k_fix_fwd's NRED role)
    const int nred = (ng + FIX_RED_TILES - 1) / FIX_RED_TILES;
    hipLaunchKernelGGL((k_fix_fwd<MODE, PF, 16, 1>), dim3(gx + nred, n), dim3(64), 0, s, g, rgb, coeffs, fq, gk, st,
                       fixlist, fixcount + par * n, nq, 0, fixcount + (par ^ 1) * n, part, ng, nred);
    kmark(s, "k_fix_fwd<%d,%d>", MODE, (int)PF);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return finish ? launch_fwd_finish(g, n, st, nullptr, 0, s) : hipSuccess;
  }
  int4 rect;
  rect.x = (g.ty_off * C::MH > 0) ? 1 : 0;                           // first tile row with y0 >= 0
  rect.y = (g.H / C::MH + g.ty_off) / C::MY - 1;                     // last tile row with y0 + TH <= H
  rect.z = (g.tx_off * C::MW > 0) ? 1 : 0;
  rect.w = (g.W / C::MW + g.tx_off) / C::MX - 1;
  const bool split = (g.W % 8) == 0 && g.H >= 2 && g.W >= 2 && rect.y >= rect.x && rect.w >= rect.z;
  if (split) fold_rows<MODE>(g, rect);
  hipError_t e;
  if (split) {
    const int nin = (rect.y - rect.x + 1) * (rect.w - rect.z + 1), nout = g.tiles_y * g.tiles_x - nin;
    if (nout > 0) {
      if (mq)
        hipLaunchKernelGGL((k_fwd32<MODE, PF, true>), dim3(nout, nf), dim3(C::TF), 0, s, g, rgb, coeffs, fq32, gk32,
                           part, fixlist, fixcount, 1, rect, dct32, nullptr, nq);
      else
        hipLaunchKernelGGL((k_fwd32<MODE, PF>), dim3(nout, n), dim3(C::TF), 0, s, g, rgb, coeffs, fq32, gk32, part,
                           fixlist, fc, 1, rect, nullptr, nullptr, 1);
      kmark(s, "k_fwd32<%d,%d%s>", MODE, (int)PF, mq ? ",mq" : "");
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (mq)
      hipLaunchKernelGGL((k_fwd32i<MODE, PF, true>), dim3(nin, nf), dim3(C::TF), 0, s, g, rgb, coeffs, fq32, gk32,
                         part, fixlist, fixcount, rect, dct32, st, nq);
    else
      hipLaunchKernelGGL((k_fwd32i<MODE, PF>), dim3(nin, n), dim3(C::TF), 0, s, g, rgb, coeffs, fq32, gk32, part,
                         fixlist, fc, rect, nullptr, st, 1);
    kmark(s, "k_fwd32i<%d,%d%s>", MODE, (int)PF, mq ? ",mq" : "");
    if ((e = hipGetLastError()) != hipSuccess) return e;
  } else {
    if (mq)
      hipLaunchKernelGGL((k_fwd32<MODE, PF, true>), dim3(g.tiles_y * g.tiles_x, nf), dim3(C::TF), 0, s, g, rgb,
                         coeffs, fq32, gk32, part, fixlist, fixcount, 0, rect, dct32, st, nq);
    else
      hipLaunchKernelGGL((k_fwd32<MODE, PF>), dim3(g.tiles_y * g.tiles_x, n), dim3(C::TF), 0, s, g, rgb, coeffs,
                         fq32, gk32, part, fixlist, fc, 0, rect, nullptr, st, 1);
    kmark(s, "k_fwd32<%d,%d%s>", MODE, (int)PF, mq ? ",mq" : "");
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  int ptiles = g.tiles_y * g.tiles_x;
  if (mq) {
    ptiles = quant_mq_tiles(g);
    hipLaunchKernelGGL(k_quant_mq, dim3(ptiles, nf), dim3(256), 0, s, g, nq, dct32, coeffs, fq32, part, fixbits);
    kmark(s, "k_quant_mq");
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  const int gx = FIX_GRID / n > 1 ? FIX_GRID / n : 1;
  if (!mq) {
    // single quality: one launch fixes the listed blocks and reduces the
    // statistics partials into the frame stats (reset by the front-end launch
    // above) in workgroups of their own (k_fix_fwd's NRED role); it reads the
    // live counter bank `par` the front end appended to and re-arms the other
    // bank.  Per 64 x 1080p: 31.4-32.1 us against 28.1 + 11.5 us as two
    // launches (same box, interleaved).  (Earlier forms: the reduction done by
    // the fix-up workgroups themselves, 49.4 vs 29.1 + 5.4 us; on a side
    // stream beside the fix-up, 0.627 vs 0.617 ms per step: the fork / join
    // costs more than the overlap returns.)
    static_assert(C::TF <= 64 * NW_MAX, "row records fit the tile slot");
    const int nred = (ptiles + FIX_RED_TILES - 1) / FIX_RED_TILES;
    hipLaunchKernelGGL((k_fix_fwd<MODE, PF, 4 * (C::TF / 64)>), dim3(gx + nred, n), dim3(64), 0, s, g, rgb, coeffs,
                       fq, gk, st, fixlist, fixcount + par * n, nq, 0, fixcount + (par ^ 1) * n, part, ptiles, nred);
    kmark(s, "k_fix_fwd<%d,%d>", MODE, (int)PF);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return finish ? launch_fwd_finish(g, n, st, nullptr, 0, s) : hipSuccess;
  }
  // sweeps: partials -> frame statistics, bitmaps -> lists with their lengths
  // at fixcount[n + item] (zeroed by the front-end launch)
  hipLaunchKernelGGL(k_fwd_reduce_fix, dim3((ptiles + 63) / 64, n), dim3(512), 0, s, g, st, part, ptiles,
                     fixbits, fixlist, fixcount);
  kmark(s, "k_fwd_reduce_fix");
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (n < 8192) {  // one flat grid over every item's list (list starts in <= 32 KB of LDS)
    hipLaunchKernelGGL((k_fix_fwd<MODE, PF>), dim3(FIX_GRID), dim3(64), sizeof(unsigned) * (n + 1), s, g, rgb,
                       coeffs, fq, gk, st, fixlist, fixcount + n, nq, n, nullptr);
    kmark(s, "k_fix_fwd<%d,%d>", MODE, (int)PF);
  } else {
    hipLaunchKernelGGL((k_fix_fwd<MODE, PF>), dim3(gx, n), dim3(64), 0, s, g, rgb, coeffs, fq, gk, st, fixlist,
                       fixcount + n, nq, 0, nullptr);
    kmark(s, "k_fix_fwd<%d,%d>", MODE, (int)PF);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return finish ? launch_fwd_finish(g, n, st, nullptr, 0, s) : hipSuccess;
}

hipError_t launch_fast_fwd(int mode, bool pf, const Geo& g, int n, int nq, const uint8_t* rgb, int16_t* coeffs,
                           const FrameQ* fq, const void* fq32, const double* gk, const float* gk32,
                           jds_frame_stats* st, uint32_t* part, uint32_t* fixbits, uint2* fixlist, unsigned* fixcount, float* dct32,
                           hipStream_t s, bool finish, int par) {
  const FastQ* f = (const FastQ*)fq32;
  switch (mode) {
    case M420:
      return pf ? fast_fwd_t<M420, true>(g, n, nq, rgb, coeffs, fq, f, gk, gk32, st, part, fixbits, fixlist, fixcount, dct32, s, finish, par)
                : fast_fwd_t<M420, false>(g, n, nq, rgb, coeffs, fq, f, gk, gk32, st, part, fixbits, fixlist, fixcount, dct32, s, finish, par);
    case M422:
      return pf ? fast_fwd_t<M422, true>(g, n, nq, rgb, coeffs, fq, f, gk, gk32, st, part, fixbits, fixlist, fixcount, dct32, s, finish, par)
                : fast_fwd_t<M422, false>(g, n, nq, rgb, coeffs, fq, f, gk, gk32, st, part, fixbits, fixlist, fixcount, dct32, s, finish, par);
    default:
      return fast_fwd_t<M444, false>(g, n, nq, rgb, coeffs, fq, f, gk, gk32, st, part, fixbits, fixlist, fixcount, dct32, s, finish, par);
  }
}

// ---------------------------------------------------- host: the bounds --
//
// Rigorous bound on |c_fp32 - c_exact| per coefficient for k_fwd32.  Unit
// roundoff u = 2^-24; each fp32 op rounds once: |fl(a op b) - (a op b)| <= u|result|.
// Input samples: |x| <= X = 128, |x_fp32 - x_exact| <= e_in (colour / prefilter /
// area stage bound below).  One fdct8_f32 pass over inputs (bound X, error e):
//   s_i, d_i:  |.| <= 2X,   error <= 2e + 2uX
//   output k:  |.| <= 2X b_k, error <= b_k (2e + 2uX) + 2uX (b_k + P_k)
// with b_k = sum_i |W_ki| (4 terms) and P_k = sum of the 4 partial sums of
// |W_k0..3| (the magnitudes the FMA chain can reach), the b_k term covering the
// fp32 representation error of W (<= u|W|).  Axis 0 then axis 1.

void pass_bound(double X, double e, const double* Xin, const double* ein, double* Xout, double* eout,
                       const double W[8][4]) {
  const double u = 0x1p-24;
  for (int k = 0; k < 8; ++k) {
    double b = 0, P = 0, pre = 0;
    for (int i = 0; i < 4; ++i) {
      b += fabs(W[k][i]);
      pre += fabs(W[k][i]);
      P += pre;
    }
    const double x = Xin ? Xin[0] : X, er = ein ? ein[0] : e;
    Xout[k] = 2 * x * b;
    eout[k] = b * (2 * er + 2 * u * x) + 2 * u * x * (b + P);
  }
}

// fp32 taps for the kernels: the Gaussian's k0, k1, k2 (k_fwd32, k_fix_fwd's
// sampling is fp64) and the combined taps of Gaussian + 2-sample area sum
// (k_fwd32i: x_{2j-1..2j+2} weighted k0, k0+k1, k1+k2, k2).
void combined_taps32(const double* gk, float* out5) {
  out5[0] = (float)gk[0];
  out5[1] = (float)gk[1];
  out5[2] = (float)gk[2];
  out5[3] = (float)(gk[0] + gk[1]);
  out5[4] = (float)(gk[1] + gk[2]);
}

// Error of one combined-tap chain fmaf(h3, x3, fmaf(h2, x2, fmaf(h1, x1, h0 * x0)))
// over inputs |x| <= X with error e each: the taps' own fp32 representation
// error against the real sums, the inputs' errors and one rounding per step.
static double combined_chain_error(const double* gk, double X, double e) {
  const double u = 0x1p-24;
  float h[5];
  combined_taps32(gk, h);
  const double hf[4] = {h[0], h[3], h[4], h[2]};
  const double hx[4] = {gk[0], gk[0] + gk[1], gk[1] + gk[2], gk[2]};
  double sh = 0, dh = 0, pre = 0, P = 0;
  for (int i = 0; i < 4; ++i) {
    sh += fabs(hf[i]);
    dh += fabs(hf[i] - hx[i]);
    pre += fabs(hf[i]);
    P += pre;  // |partial result| after step i <= X * (sum of |h| so far)
  }
  return sh * e + dh * X + u * X * P + 1e-12;
}

double fwd_input_error(int plane, int mode, bool pf, const double* gk, int chains) {
  const double u = 0x1p-24;
  // luma32: fmaf(kb, B, fmaf(kg, G, kr*R)); constants in fp32; then -128
  const double dkl = fabs((double)0.299f - 0.299) + fabs((double)0.587f - 0.587) + fabs((double)0.114f - 0.114);
  if (plane == 0) return 255 * dkl + u * 255 * (0.299 + 0.886 + 1.0) + u * 128 + 1e-12;
  // cb32 / cr32: fmaf(k1, ., fmaf(k2, ., fmaf(0.5f, ., 128))); 0.5x+128 exact
  const double dkb = fabs((double)-0.168736f + 0.168736) + fabs((double)-0.331264f + 0.331264);
  const double dkr = fabs((double)-0.081312f + 0.081312) + fabs((double)-0.418688f + 0.418688);
  const double ec = 255 * (dkb > dkr ? dkb : dkr) + 2 * u * 256 + 1e-12;  // before -128
  double e = ec;
  double e_comb = 0.0;  // k_fwd32i's combined-tap chain (prefiltered chroma)
  if (mode != M444 && pf) {
    const double k0 = gk[0], k1 = gk[1], k2 = gk[2];
    const double k0f = (float)k0, k1f = (float)k1, k2f = (float)k2;
    const double dk = fabs(k0f - k0) + fabs(k1f - k1) + fabs(k2f - k2);
    // k_fwd32 (per pixel): row fmaf(k2, S1, fmaf(k1, S0, k0*S_1)); |S| <= 256, taps sum to 1
    const double er = (k0f + k1f + k2f) * e + dk * 256 + u * 256 * (k0 + (k0 + k1) + 1.0) + 1e-12;
    // column: fmaf(k0, T+1 + T-1, k1*T0)
    e = (k1f + 2 * k0f) * er + dk * 512 + u * (512 + k1 * 256 + 256) + 1e-12;
    // k_fwd32i, k_fwd32 and k_fwd16f: horizontal pair sums H =
    // combined chain over 4 chroma samples
    // (|H| <= 512), then 4:2:0: the combined chain down 4 rows of H (|.| <= 1024)
    // and *0.25 (exact); 4:2:2: the column form over H (magnitudes doubled) and
    // *0.5 (exact)
    const double eh = combined_chain_error(gk, 256, ec);
    if (mode == M420)
      e_comb = combined_chain_error(gk, 512, eh) / 4;
    else
      e_comb = ((k1f + 2 * k0f) * eh + dk * 1024 + u * (1024 + k1 * 512 + 512) + 1e-12) / 2;
  }
  if (mode == M420) e = e + u * (512 + 768 + 1024) / 4;  // ((a+b)+c)+d, *0.25 exact
  if (mode == M422) e = e + u * 512 / 2;                  // (a+b), *0.5 exact
  // the bound covers the chains named (every certified forward kernel now
  // uses the combined taps: callers pass 2)
  if (mode != M444 && pf) e = (chains & 1) ? ((chains & 2) && e_comb > e ? e_comb : e) : e_comb;
  return e + u * 128;                                     // -128
}

// E[p][k][l] (p: 0 luma, 1 chroma): the rigorous bound on |c_fp32 - c_exact|
// of coefficient (k, l) for either pass order, before the quotient.
void fast_fwd_bounds(int mode, bool pf, const double* gk, double* E) {
  static const double W[8][4] = {
      {FW[0][0], FW[0][1], FW[0][2], FW[0][3]}, {FW[1][0], FW[1][1], FW[1][2], FW[1][3]},
      {FW[2][0], FW[2][1], FW[2][2], FW[2][3]}, {FW[3][0], FW[3][1], FW[3][2], FW[3][3]},
      {FW[4][0], FW[4][1], FW[4][2], FW[4][3]}, {FW[5][0], FW[5][1], FW[5][2], FW[5][3]},
      {FW[6][0], FW[6][1], FW[6][2], FW[6][3]}, {FW[7][0], FW[7][1], FW[7][2], FW[7][3]},
  };
  for (int p = 0; p < 2; ++p) {
    const double e_in = fwd_input_error(p, mode, pf, gk, 2);  // k_fwd32i and k_fwd32: combined taps
    double X1[8], e1[8];
    pass_bound(128.0, e_in, nullptr, nullptr, X1, e1, W);
    double E2[8][8];  // [first-pass frequency][second-pass frequency]
    for (int k = 0; k < 8; ++k) {
      double X2[8], e2[8];
      pass_bound(0, 0, &X1[k], &e1[k], X2, e2, W);
      for (int l = 0; l < 8; ++l) E2[k][l] = e2[l];
    }
    for (int k = 0; k < 8; ++k) {
      for (int l = 0; l < 8; ++l) {
        // coefficient (k, l): axis 0 first (k_fwd32) or axis 1 first (k_fwd32i);
        // second-order slack and the fp64 reference's own error
        const double e2l = E2[k][l] > E2[l][k] ? E2[k][l] : E2[l][k];
        E[p * 64 + k * 8 + l] = e2l * (1 + 1e-5) + 1e-9;
      }
    }
  }
}

void fast_fwd_thresholds(const double* Q, int mode, bool pf, const double* gk, float* rq, float* thr) {
  double Eb[128];
  fast_fwd_bounds(mode, pf, gk, Eb);
  for (int i = 0; i < 64; ++i) rq[i] = (float)(1.0 / Q[i]);
  for (int p = 0; p < 2; ++p) {
    for (int i = 0; i < 64; ++i) {
      // quotient scaling, stored as the certification limit on |t - rint(t)|:
      // 0.5 - t - 2^-23 (covers the fp32 rounding of the in-kernel fma), rounded down
      const double t = Eb[p * 64 + i] / Q[i] * (1 + 1e-5) + 1e-7;
      const double lim = 0.5 - t * (1 + 0x1p-20) - 0x1p-23;
      float f = (float)lim;
      if ((double)f > lim) f = nextafterf(f, 0.0f);
      thr[p * 64 + i] = f;
    }
  }
}

// ---------------------------------------------- host: the fp32 chain (tests) --
//
// The forward kernels' fp32 arithmetic restated on the host, expression for
// expression (k_fwd32i / k_fwd32: luma32m, cb32 / cr32, the prefilter's row
// then column FMA chains with BORDER_REFLECT_101, the area average, fdct8_f32
// along both axes in either order), so the CPU test suite can check the bound
// above against the exact reference on adversarial inputs.  Test-only.
static int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

int fwd32_host_plane(int mode, bool pf, const double* gk, const uint8_t* rgb, int H, int W, int plane,
                     int flags, float* out) {
  // flags bit 0: rows first (k_fwd32i's order); bit 1: the combined-tap chroma chain (k_fwd32i)
  const bool rows_first = (flags & 1) != 0, comb = (flags & 2) != 0;
  const int sy = mode == M420 ? 2 : 1, sx = mode == M444 ? 1 : 2;
  const int ph = plane == 0 ? H : H / sy, pw = plane == 0 ? W : W / sx;
  if (ph % 8 || pw % 8) return -1;
  const float k0 = (float)gk[0], k1 = (float)gk[1], k2 = (float)gk[2];
  auto px = [&](int y, int x, int c) { return (float)rgb[((size_t)y * W + x) * 3 + c]; };
  auto chroma = [&](int y, int x) {  // full-resolution chroma sample (not shifted)
    const float R = px(y, x, 0), G = px(y, x, 1), B = px(y, x, 2);
    return plane == 1 ? cb32(R, G, B) : cr32(R, G, B);
  };
  auto rowf = [&](int y, int x) {  // prefilter row pass at (y, x)
    const float bl = chroma(y, refl101(x - 1, W)), c = chroma(y, x), br = chroma(y, refl101(x + 1, W));
    return fmaf(k2, br, fmaf(k1, c, k0 * bl));
  };
  float h[5];
  combined_taps32(gk, h);
  auto pairf = [&](int y, int j) {  // k_fwd32i: combined taps over chroma columns 2j-1 .. 2j+2 of row y
    const float x0 = chroma(y, refl101(2 * j - 1, W)), x1 = chroma(y, 2 * j), x2 = chroma(y, 2 * j + 1),
                x3 = chroma(y, refl101(2 * j + 2, W));
    return fmaf(h[2], x3, fmaf(h[4], x2, fmaf(h[3], x1, h[0] * x0)));
  };
  auto sample = [&](int y, int x) -> float {  // plane sample (y, x), level-shifted
    if (plane == 0) return luma32m(px(y, x, 0), px(y, x, 1), px(y, x, 2));
    if (mode == M444) return chroma(y, x) - 128.0f;
    if (pf && comb) {  // k_fwd32i
      if (sy == 2) {
        const float r0 = pairf(refl101(2 * y - 1, H), x), r1 = pairf(2 * y, x), r2 = pairf(2 * y + 1, x),
                    r3 = pairf(refl101(2 * y + 2, H), x);
        return fmaf(h[2], r3, fmaf(h[4], r2, fmaf(h[3], r1, h[0] * r0))) * 0.25f - 128.0f;
      }
      return fmaf(k0, pairf(refl101(y + 1, H), x) + pairf(refl101(y - 1, H), x), k1 * pairf(y, x)) * 0.5f - 128.0f;
    }
    float s[2][2];
    for (int a = 0; a < sy; ++a)
      for (int b = 0; b < 2; ++b) {
        const int yy = sy * y + a, xx = 2 * x + b;
        if (pf)
          s[a][b] = fmaf(k0, rowf(refl101(yy + 1, H), xx) + rowf(refl101(yy - 1, H), xx), k1 * rowf(yy, xx));
        else
          s[a][b] = chroma(yy, xx);
      }
    if (sy == 2) return (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
    return (s[0][0] + s[0][1]) * 0.5f - 128.0f;
  };
  const int nbx = pw / 8;
  for (int by = 0; by < ph / 8; ++by)
    for (int bx = 0; bx < nbx; ++bx) {
      float b[8][8];
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) b[i][j] = sample(by * 8 + i, bx * 8 + j);
      for (int pass = 0; pass < 2; ++pass) {
        const bool rows = (pass == 0) == rows_first;  // axis 1 (along a row) or axis 0
        for (int i = 0; i < 8; ++i) {
          float v[8];
          for (int j = 0; j < 8; ++j) v[j] = rows ? b[i][j] : b[j][i];
          fdct8_f32(v);
          for (int j = 0; j < 8; ++j) (rows ? b[i][j] : b[j][i]) = v[j];
        }
      }
      float* o = out + ((size_t)by * nbx + bx) * 64;
      for (int i = 0; i < 64; ++i) o[i] = b[i / 8][i % 8];
    }
  return 0;
}

size_t fast_q_size() { return sizeof(FastQ); }

}  // namespace jds
