// jds_fast16.hip — the certified fp32 forward for 16x16 blocks (BASELINE
// configs[4] stretch): the 8x8 path's scheme (jds_fast.hip) with 16-point
// transforms.  Colour, prefilter, area average and the 16x16 DCT run in fp32;
// a host-derived rigorous bound E_uv on |c_fp32 - c_exact| per coefficient
// (fast_fwd16_thresholds: fwd_input_error for the samples, then two passes of
// 8-term FMA chains) decides whether round-half-even(c / Q16) is certain.
// Blocks with an uncertain coefficient are listed; k_fix_fwd16 recomputes them
// with the exact fp64 chain of k_fwd16 (jds_b16.hip: every sample exactly from
// global memory, pocketfft's 16-point DCT-II) and corrects the statistics by
// delta.  Results are bit-identical to k_fwd16 and to the oracle with the
// kron(Q8, ones(2,2)) table (engines/pipeline.py:47-63 with block_size 16).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "jds_dct16.hpp"
#include "jds_device.hpp"
#include "jds_fwd_common.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

// orthonormal 16-point DCT-II rows restricted to i = 0..7, rounded to fp32:
// W16[k][i] = s(k) cos((2i+1) k pi / 32), s(0) = 1/4, s(k) = sqrt(2/16); even
// rows act on s_i = x_i + x_{15-i}, odd rows on d_i = x_i - x_{15-i}
static constexpr float W16[16][8] = {
    {0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f},
    {0x1.684b9c0000000p-2f, 0x1.5a730c0000000p-2f, 0x1.3f4a240000000p-2f, 0x1.17dc140000000p-2f, 0x1.cb598c0000000p-3f, 0x1.5553e40000000p-3f, 0x1.a4608a0000000p-4f, 0x1.1be3520000000p-5f},
    {0x1.63150c0000000p-2f, 0x1.2d062e0000000p-2f, 0x1.92469c0000000p-3f, 0x1.1a855e0000000p-4f, -0x1.1a855e0000000p-4f, -0x1.92469c0000000p-3f, -0x1.2d062e0000000p-2f, -0x1.63150c0000000p-2f},
    {0x1.5a730c0000000p-2f, 0x1.cb598c0000000p-3f, 0x1.1be3520000000p-5f, -0x1.5553e40000000p-3f, -0x1.3f4a240000000p-2f, -0x1.684b9c0000000p-2f, -0x1.17dc140000000p-2f, -0x1.a4608a0000000p-4f},
    {0x1.4e7aea0000000p-2f, 0x1.1517a80000000p-3f, -0x1.1517a80000000p-3f, -0x1.4e7aea0000000p-2f, -0x1.4e7aea0000000p-2f, -0x1.1517a80000000p-3f, 0x1.1517a80000000p-3f, 0x1.4e7aea0000000p-2f},
    {0x1.3f4a240000000p-2f, 0x1.1be3520000000p-5f, -0x1.17dc140000000p-2f, -0x1.5a730c0000000p-2f, -0x1.a4608a0000000p-4f, 0x1.cb598c0000000p-3f, 0x1.684b9c0000000p-2f, 0x1.5553e40000000p-3f},
    {0x1.2d062e0000000p-2f, -0x1.1a855e0000000p-4f, -0x1.63150c0000000p-2f, -0x1.92469c0000000p-3f, 0x1.92469c0000000p-3f, 0x1.63150c0000000p-2f, 0x1.1a855e0000000p-4f, -0x1.2d062e0000000p-2f},
    {0x1.17dc140000000p-2f, -0x1.5553e40000000p-3f, -0x1.5a730c0000000p-2f, 0x1.1be3520000000p-5f, 0x1.684b9c0000000p-2f, 0x1.a4608a0000000p-4f, -0x1.3f4a240000000p-2f, -0x1.cb598c0000000p-3f},
    {0x1.0000000000000p-2f, -0x1.0000000000000p-2f, -0x1.0000000000000p-2f, 0x1.0000000000000p-2f, 0x1.0000000000000p-2f, -0x1.0000000000000p-2f, -0x1.0000000000000p-2f, 0x1.0000000000000p-2f},
    {0x1.cb598c0000000p-3f, -0x1.3f4a240000000p-2f, -0x1.a4608a0000000p-4f, 0x1.684b9c0000000p-2f, -0x1.1be3520000000p-5f, -0x1.5a730c0000000p-2f, 0x1.5553e40000000p-3f, 0x1.17dc140000000p-2f},
    {0x1.92469c0000000p-3f, -0x1.63150c0000000p-2f, 0x1.1a855e0000000p-4f, 0x1.2d062e0000000p-2f, -0x1.2d062e0000000p-2f, -0x1.1a855e0000000p-4f, 0x1.63150c0000000p-2f, -0x1.92469c0000000p-3f},
    {0x1.5553e40000000p-3f, -0x1.684b9c0000000p-2f, 0x1.cb598c0000000p-3f, 0x1.a4608a0000000p-4f, -0x1.5a730c0000000p-2f, 0x1.17dc140000000p-2f, 0x1.1be3520000000p-5f, -0x1.3f4a240000000p-2f},
    {0x1.1517a80000000p-3f, -0x1.4e7aea0000000p-2f, 0x1.4e7aea0000000p-2f, -0x1.1517a80000000p-3f, -0x1.1517a80000000p-3f, 0x1.4e7aea0000000p-2f, -0x1.4e7aea0000000p-2f, 0x1.1517a80000000p-3f},
    {0x1.a4608a0000000p-4f, -0x1.17dc140000000p-2f, 0x1.684b9c0000000p-2f, -0x1.3f4a240000000p-2f, 0x1.5553e40000000p-3f, 0x1.1be3520000000p-5f, -0x1.cb598c0000000p-3f, 0x1.5a730c0000000p-2f},
    {0x1.1a855e0000000p-4f, -0x1.92469c0000000p-3f, 0x1.2d062e0000000p-2f, -0x1.63150c0000000p-2f, 0x1.63150c0000000p-2f, -0x1.2d062e0000000p-2f, 0x1.92469c0000000p-3f, -0x1.1a855e0000000p-4f},
    {0x1.1be3520000000p-5f, -0x1.a4608a0000000p-4f, 0x1.5553e40000000p-3f, -0x1.cb598c0000000p-3f, 0x1.17dc140000000p-2f, -0x1.3f4a240000000p-2f, 0x1.5a730c0000000p-2f, -0x1.684b9c0000000p-2f},
};

// Per pass: s_i = x_i + x_{15-i}, d_i = x_i - x_{15-i} (i < 8); the fp32 even
// rows are exactly symmetric (W16[2m][7-i] = (-1)^m W16[2m][i]), so the even
// outputs are 4-term chains over e_i = s_i + s_{7-i} (m even) or
// o_i = s_i - s_{7-i} (m odd), i < 4; the odd outputs 8-term chains over d.
// 24 add/sub + 8 x 4 + 8 x 8 multiply-adds (pass_bound16 follows this).
__host__ __device__ __forceinline__ void fdct16_f32(float (&x)[16]) {
  float sv[8], dv[8], ev[4], ov[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sv[i] = x[i] + x[15 - i];
    dv[i] = x[i] - x[15 - i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ev[i] = sv[i] + sv[7 - i];
    ov[i] = sv[i] - sv[7 - i];
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const float* v = (m & 1) ? ov : ev;
    const float* w = W16[2 * m];
    float a = w[0] * v[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) a = fmaf(w[i], v[i], a);
    x[2 * m] = a;
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const float* w = W16[2 * m + 1];
    float a = w[0] * dv[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) a = fmaf(w[i], dv[i], a);
    x[2 * m + 1] = a;
  }
}

struct FastQ16 {
  float rq[256];      // fp32(1 / Q16)
  float thr[2][256];  // certification limits on |t - rint(t)|: [0] luma, [1] chroma
};

template <int MODE>
struct Cfg16F {
  static constexpr int SY = (MODE == M420) ? 2 : 1;
  static constexpr int SX = (MODE == M444) ? 1 : 2;
  static constexpr int MH = 16 * SY, MW = 16 * SX;
  static constexpr int TH = 2 * MH, TW = 64;  // jds_b16.hip's Cfg16 tiles (Geo tiles_y / tiles_x)
  static constexpr int MY = TH / MH, MX = TW / MW;
  static constexpr int YBR = TH / 16, YBC = TW / 16;
  static constexpr int CBR = MY, CBC = MX;
  static constexpr int NYB = YBR * YBC, NCB = CBR * CBC;
  static constexpr int NB = NYB + 2 * NCB;
  static constexpr int TF = NB * 16;  // one thread per block column
};

constexpr int BS16F = 272;  // floats per 16x16 block in LDS (256 + 16 pad: column writes spread over banks)

// The workgroup's statistics into its tile's slot of the per-tile partials
// (k_fwd_reduce sums them per frame): each lane's 8 common-bin counts (two
// nibble words, <= 16 per bin together) and nonzero count into three words of
// 10-bit fields, the magnitude bits into a fourth; DPP row sums (<= 256 per
// field over a 16-lane row, decoded per row), one LDS record per row, and the
// workgroup's last wave (ticket in s_st[NSTAT]; the LDS performs a wave's
// operations in order, so every row record and rare-bin atomic precedes the
// last ticket) decodes them and adds the rare bins.  Zeros are not binned here:
// k_fwd_finish / k_finalize add bin 25's zeros from the nonzero count.
constexpr int NW16 = 6;  // waves per k_fwd16f workgroup (TF <= 384)

// The wave-record form: the bin bytes widen into four words
// of 16-bit fields (a wave counts <= 64 x 16 = 1024 per bin) plus nonzero |
// magnitude bits << 16 (<= 1024, <= 64 x 240), summed over the whole wave by
// DPP (row shifts, then two row broadcasts) into lane 63, one record per
// wave; the last wave decodes one record per wave instead of four.
__device__ __forceinline__ void stats_flush16_wave(unsigned h0, unsigned h1, unsigned nz, unsigned mb, bool valid,
                                                   unsigned* s_st, uint32_t* __restrict__ slot) {
  __shared__ __attribute__((aligned(16))) unsigned s_wr[NW16][8];  // [wave][word]: 5 sums, valid lanes
  const unsigned e = (h0 & 0x0f0f0f0fu) + (h1 & 0x0f0f0f0fu);                 // bins 0, 2, 4, 6 (bytes)
  const unsigned o = ((h0 >> 4) & 0x0f0f0f0fu) + ((h1 >> 4) & 0x0f0f0f0fu);   // bins 1, 3, 5, 7
  // (0 | 4), (2 | 6), (1 | 5), (3 | 7), nz | mb
  unsigned u[5] = {e & 0x00ff00ffu, (e >> 8) & 0x00ff00ffu, o & 0x00ff00ffu, (o >> 8) & 0x00ff00ffu, nz | (mb << 16)};
  row_sums(u);
#pragma unroll
  for (int k = 0; k < 5; ++k) u[k] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)u[k], 0x142, 0xa, 0xf, false);
#pragma unroll
  for (int k = 0; k < 5; ++k) u[k] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)u[k], 0x143, 0xc, 0xf, false);
  const unsigned nvalid = (unsigned)__popcll(__ballot(valid));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = (int)(blockDim.x >> 6);
  if (lane == 63) {
    *reinterpret_cast<uint4*>(&s_wr[w][0]) = make_uint4(u[0], u[1], u[2], u[3]);
    *reinterpret_cast<uint2*>(&s_wr[w][4]) = make_uint2(u[4], nvalid);
  }
  __asm__ volatile("" ::: "memory");  // a compiler barrier (a fence would wait on the coefficient stores)
  unsigned ticket = 0u;
  if (lane == 0) ticket = atomicAdd(&s_st[NSTAT], 1u);
  ticket = (unsigned)__builtin_amdgcn_readfirstlane((int)ticket);
  if (ticket != (unsigned)(nw - 1)) return;
  __asm__ volatile("" ::: "memory");
  if (lane < NSTAT) {
    // lane 0: nz; lane 1: mb + nz; lanes 24..31: bin 22 + b from word
    // 2 (b & 1) + ((b >> 1) & 1), field b >> 2; bin 25 less the zeros
    const int b = lane - 2 - 22;
    const bool bin = (unsigned)b < 8u;
    const int k = bin ? ((b & 1) << 1) | ((b >> 1) & 1) : 4;
    const unsigned sh = bin ? 16u * (unsigned)(b >> 2) : 0u;
    const unsigned m1 = (lane < 2 || bin) ? 0xffffu : 0u, m2 = lane == 1 ? 0xffffu : 0u;
    unsigned tot = 0u, zeros = 0u;
    for (int i = 0; i < nw; ++i) {
      const unsigned x = s_wr[i][k];
      tot += ((x >> sh) & m1) + ((x >> 16) & m2);
      zeros += 16u * s_wr[i][5] - (s_wr[i][4] & 0xffffu);
    }
    if (b == 3) tot -= zeros;  // the zeros counted in bin 25
    slot[lane] = s_st[lane] + tot;
  }
}

__device__ __forceinline__ void stats_flush16(unsigned h0, unsigned h1, unsigned nz, unsigned mb, bool valid,
                                              unsigned* s_st, uint32_t* __restrict__ slot) {
  stats_flush16_wave(h0, h1, nz, mb, valid, s_st, slot);
  return;
  __shared__ __attribute__((aligned(16))) unsigned s_row[NW16][4][4];  // [wave][row][word]
  __shared__ unsigned s_nvalid[NW16];
  const unsigned e = (h0 & 0x0f0f0f0fu) + (h1 & 0x0f0f0f0fu);                 // bins 0, 2, 4, 6 (bytes)
  const unsigned o = ((h0 >> 4) & 0x0f0f0f0fu) + ((h1 >> 4) & 0x0f0f0f0fu);   // bins 1, 3, 5, 7
  unsigned v[4] = {(e & 255u) | (o & 255u) << 10 | ((e >> 8) & 255u) << 20,
                   ((o >> 8) & 255u) | ((e >> 16) & 255u) << 10 | ((o >> 16) & 255u) << 20,
                   (e >> 24) | (o >> 24) << 10 | nz << 20, mb};
  row_sums4(v);
  const unsigned nvalid = (unsigned)__popcll(__ballot(valid));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = (int)(blockDim.x >> 6);
  if ((lane & 15) == 15) {
    *reinterpret_cast<uint4*>(&s_row[w][lane >> 4][0]) = make_uint4(v[0], v[1], v[2], v[3]);
    if (lane == 63) s_nvalid[w] = nvalid;
  }
  __asm__ volatile("" ::: "memory");  // a compiler barrier (a fence would wait on the coefficient stores)
  unsigned ticket = 0u;
  if (lane == 0) ticket = atomicAdd(&s_st[NSTAT], 1u);
  ticket = (unsigned)__builtin_amdgcn_readfirstlane((int)ticket);
  if (ticket != (unsigned)(nw - 1)) return;
  __asm__ volatile("" ::: "memory");
  const int t = lane;
  if (t < NSTAT) {
    unsigned tot = s_st[t];  // rare bins
    unsigned nzt = 0u, nvt = 0u;
    for (int i = 0; i < nw; ++i) {
      nvt += s_nvalid[i];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint4 x = *reinterpret_cast<const uint4*>(&s_row[i][r][0]);
        const unsigned wv[3] = {x.x, x.y, x.z};
        const unsigned nzr = (x.z >> 20) & 1023u;
        nzt += nzr;
        if (t == 0) {
          tot += nzr;
        } else if (t == 1) {
          tot += x.w + nzr;  // magnitude bits = bit length + 1 per nonzero
        } else if (t >= 2 + 22 && t < 2 + 30) {
          const int b = t - 2 - 22;  // common bin 22 + b: word b / 3, field b % 3
          tot += (wv[b / 3] >> (10 * (b % 3))) & 1023u;
        }
      }
    }
    if (t == 2 + 25) tot -= 16u * nvt - nzt;  // the zeros counted in bin 25
    slot[t] = tot;
  }
}

// ---------------------------------------------------------------- forward --
//
// k_fwd16's decomposition in fp32: RGB window (+1 px ring) staged as packed
// u32, the chroma planes converted and row-filtered in LDS, one thread per
// block column: samples, column DCT (axis 0), LDS exchange, row DCT,
// certified quantisation, 2 x 16-B stores, statistics.
template <int MODE, bool PF>
__global__ void __launch_bounds__(Cfg16F<MODE>::TF)
k_fwd16f(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
         const FastQ16* __restrict__ fq16, const float* __restrict__ gk32, uint32_t* __restrict__ part,
         uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount, unsigned* __restrict__ fixnext,
         const unsigned cap, const int fix_all) {
  using C = Cfg16F<MODE>;
  constexpr int WR = C::TH + 2, WC = C::TW + 2, WN = WR * WC;
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int PLANE_D = CPLANE ? 2 * WN : 0;
  constexpr int BLK_D = C::NB * BS16F;
  constexpr int U_D = PLANE_D > BLK_D ? PLANE_D : BLK_D;
  constexpr int HW = C::TW / 2;  // pair sums per window row (fast staging path)

  __shared__ __attribute__((aligned(16))) uint32_t s_rgb[WN];  // 16-B aligned: the tables' float4s alias it
  __shared__ __attribute__((aligned(16))) float s_u[U_D];
  __shared__ unsigned s_st[NSTAT + 1];  // rare histogram bins (+ stats_flush16's ticket)
  // the frame's tables, rows of 20 floats (a row's four 16-B reads by the 16
  // row lanes hit distinct bank groups; lanes of other blocks broadcast):
  // rq, thr luma, thr chroma.  With the prefilter planes (the LDS-heavy
  // modes) they go into s_rgb once the sampling is done; otherwise their own.
  // 4:2:0 with the prefilter reads them from global memory instead: holding
  // them in registers across its sampling cost a wave per SIMD (94 -> 100
  // VGPRs); staging them saves ~6 us elsewhere.
  constexpr bool QLDS = !(MODE == M420 && CPLANE);
  constexpr int QR = 20, TABF = 3 * 16 * QR;
  static_assert(WN >= TABF, "tables fit the RGB window");
  __shared__ __attribute__((aligned(16))) float s_tab_own[(CPLANE || !QLDS) ? 4 : TABF];
  float* const s_tab = CPLANE ? reinterpret_cast<float*>(s_rgb) : s_tab_own;

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  const FastQ16& fq = fq16[frame];

  auto rgbf = [](uint32_t v, float& R, float& G, float& B) {
    R = (float)(v & 255u);
    G = (float)((v >> 8) & 255u);
    B = (float)((v >> 16) & 255u);
  };
  // chroma planes: each window row holds its even columns, then its odd ones
  // (the sample loop reads columns 2m+1 and 2m+2 of lane m: unit stride)
  static_assert(WC % 2 == 0, "even window width");
  auto cidx = [](int r, int c) { return r * WC + (c & 1) * (WC / 2) + (c >> 1); };
  if (tid <= NSTAT) s_st[tid] = 0u;
  float4 tabv = make_float4(0.f, 0.f, 0.f, 0.f);  // 3 tables x 16 rows x 4 float4: one per thread < 192
  const int tab_t = tid >> 6, tab_r = (tid >> 2) & 15, tab_q = tid & 3;
  if (QLDS && tid < 192) {
    const float* src = tab_t == 0 ? fq.rq : fq.thr[tab_t - 1];
    tabv = reinterpret_cast<const float4*>(src + tab_r * 16)[tab_q];
    if constexpr (!CPLANE) *reinterpret_cast<float4*>(&s_tab[tab_t * 16 * QR + tab_r * QR + 4 * tab_q]) = tabv;
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *fixnext = 0u;  // the next run's list
  const float k0 = gk32[0], k1 = gk32[1], k2 = gk32[2];

  // Tiles whose columns lie inside the image (no np.pad samples; only the
  // 1-px ring may reflect), rows 16-B aligned: one thread per 16-pixel row
  // segment loads 48 B, packs the pixels for the luma / 4:4:4 / unfiltered
  // samples and -- prefiltered chroma -- converts colour and runs the row
  // pass in registers (neighbours from the adjacent lanes), writing the
  // filtered planes directly.  Same fp32 operations as the general path.
  constexpr int SEGS = C::TW / 16;
  static_assert(WR * SEGS <= C::TF, "one thread per row segment");
  const bool fast_stage = (g.W % 16) == 0 && x0 >= 0 && x0 + C::TW <= g.W && y0 >= 0 && y0 + C::TH <= g.H;
  if (fast_stage) {  // uniform per workgroup
    const int r = tid / SEGS, c = tid - r * SEGS;
    if (r < WR) {
      const int yy = reflect101(y0 - 1 + r, g.H);
      const uint8_t* row = img + (size_t)yy * g.W * 3;
      const uint4* p4 = reinterpret_cast<const uint4*>(row + (size_t)(x0 + 16 * c) * 3);
      const bool luma_row = r >= 1 && r <= C::TH;
      const bool need = CPLANE || luma_row;  // uniform per 4-lane row group
      uint32_t w[12] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      uint4 ring = make_uint4(0u, 0u, 0u, 0u);
      if (need) {
        const uint4 a0 = p4[0], a1 = p4[1], a2 = p4[2];
        w[0] = a0.x; w[1] = a0.y; w[2] = a0.z; w[3] = a0.w;
        w[4] = a1.x; w[5] = a1.y; w[6] = a1.z; w[7] = a1.w;
        w[8] = a2.x; w[9] = a2.y; w[10] = a2.z; w[11] = a2.w;
        if (CPLANE && c == 0 && x0 > 0) ring = p4[-1];                      // bytes 13..15: pixel x0 - 1
        if (CPLANE && c == SEGS - 1 && x0 + C::TW < g.W) ring = p4[3];   // bytes 0..2: pixel x0 + TW
      }
      uint32_t px[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int b = 3 * j;
        const uint32_t lo = w[b >> 2], hi = (b >> 2) + 1 < 12 ? w[(b >> 2) + 1] : 0u;
        px[j] = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(b & 3)) & 0xffffffu;
      }
      if (luma_row) {  // luma (and 4:4:4 / unfiltered chroma) samples: rows 1..TH, columns 1..TW
#pragma unroll
        for (int j = 0; j < 16; ++j) s_rgb[r * WC + 1 + 16 * c + j] = px[j];
      }
      if constexpr (CPLANE) {
        float cb[16], cr[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          float R, G, B;
          rgbf(px[j], R, G, B);
          cb[j] = cb32(R, G, B);
          cr[j] = cr32(R, G, B);
        }
        float lb = __shfl_up(cb[15], 1, SEGS), lr = __shfl_up(cr[15], 1, SEGS);
        float rb = __shfl_down(cb[0], 1, SEGS), rr = __shfl_down(cr[0], 1, SEGS);
        if (c == 0) {  // pixel x0 - 1; pixel 1 at the image edge (BORDER_REFLECT_101)
          const float R = (float)((ring.w >> 8) & 255u), G = (float)((ring.w >> 16) & 255u), B = (float)(ring.w >> 24);
          lb = x0 == 0 ? cb[1] : cb32(R, G, B);
          lr = x0 == 0 ? cr[1] : cr32(R, G, B);
        }
        if (c == SEGS - 1) {  // pixel x0 + TW; pixel W - 2 at the image edge
          const float R = (float)(ring.x & 255u), G = (float)((ring.x >> 8) & 255u), B = (float)((ring.x >> 16) & 255u);
          const bool edge = x0 + C::TW == g.W;
          rb = edge ? cb[14] : cb32(R, G, B);
          rr = edge ? cr[14] : cr32(R, G, B);
        }
        // the Gaussian row pass and the area's horizontal pair sum as one chain
        // (k_fwd32i's combined taps, fwd_input_error): TW / 2 pair sums per row
        float* s_cb = s_u;
        float* s_cr = s_u + WR * HW;
        const float h1 = gk32[3], h2 = gk32[4];
        float ob[8], orr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float bl = j == 0 ? lb : cb[2 * j - 1], br = j == 7 ? rb : cb[2 * j + 2];
          const float ql = j == 0 ? lr : cr[2 * j - 1], qr = j == 7 ? rr : cr[2 * j + 2];
          ob[j] = fmaf(k2, br, fmaf(h2, cb[2 * j + 1], fmaf(h1, cb[2 * j], k0 * bl)));
          orr[j] = fmaf(k2, qr, fmaf(h2, cr[2 * j + 1], fmaf(h1, cr[2 * j], k0 * ql)));
        }
        float4* db = reinterpret_cast<float4*>(s_cb + r * HW + 8 * c);
        float4* dr = reinterpret_cast<float4*>(s_cr + r * HW + 8 * c);
        db[0] = make_float4(ob[0], ob[1], ob[2], ob[3]);
        db[1] = make_float4(ob[4], ob[5], ob[6], ob[7]);
        dr[0] = make_float4(orr[0], orr[1], orr[2], orr[3]);
        dr[1] = make_float4(orr[4], orr[5], orr[6], orr[7]);
      }
    }
    __syncthreads();
  } else {
    {  // every window load in flight before the first LDS store
      constexpr int NL = (WN + C::TF - 1) / C::TF;
      uint32_t px[NL];
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int i = tid + l * C::TF;
        px[l] = 0u;
        if (i < WN) {
          const int r = i / WC, c = i - r * WC;
          const int yy = reflect101(y0 - 1 + r, g.H), xx = reflect101(x0 - 1 + c, g.W);
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
    if constexpr (CPLANE) {  // full-resolution chroma, then the prefilter's row pass in place
      float* s_cb = s_u;
      float* s_cr = s_u + WN;
#pragma unroll
      for (int l = 0; l < (WN + C::TF - 1) / C::TF; ++l) {
        const int i = tid + l * C::TF;
        if (i < WN) {
          float R, G, B;
          rgbf(s_rgb[i], R, G, B);
          const int r = i / WC, c = i - r * WC;
          s_cb[cidx(r, c)] = cb32(R, G, B);
          s_cr[cidx(r, c)] = cr32(R, G, B);
        }
      }
      __syncthreads();
      // the combined-tap pair sums of the fast path (window columns 2j .. 2j+3),
      // same layout: rows of HW at the start of each plane's space
      constexpr int NRP = WR * HW;
      constexpr int PER = (NRP + C::TF - 1) / C::TF;
      const float h1 = gk32[3], h2 = gk32[4];
      float tb[PER], tr[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int i = tid + j * C::TF;
        if (i < NRP) {
          const int r = i / HW, c = 2 * (i - r * HW);
          const int i0 = cidx(r, c), i1 = cidx(r, c + 1), i2 = cidx(r, c + 2), i3 = cidx(r, c + 3);
          tb[j] = fmaf(k2, s_cb[i3], fmaf(h2, s_cb[i2], fmaf(h1, s_cb[i1], k0 * s_cb[i0])));
          tr[j] = fmaf(k2, s_cr[i3], fmaf(h2, s_cr[i2], fmaf(h1, s_cr[i1], k0 * s_cr[i0])));
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int i = tid + j * C::TF;
        if (i < NRP) {
          s_u[i] = tb[j];
          s_u[WR * HW + i] = tr[j];
        }
      }
      __syncthreads();
    }
  }

  const int blk = tid >> 4, line = tid & 15;
  int plane, gy, gx;
  if (blk < C::NYB) {
    plane = 0;
    gy = m0y * C::SY + blk / C::YBC;
    gx = m0x * C::SX + blk % C::YBC;
  } else {
    const int bi = (blk - C::NYB) % C::NCB;
    plane = 1 + (blk - C::NYB) / C::NCB;
    gy = m0y + bi / C::CBC;
    gx = m0x + bi % C::CBC;
  }
  const int nby = plane ? g.ncy : g.nby, nbx = plane ? g.ncx : g.nbx;
  const bool valid = gy >= 0 && gx >= 0 && gy < nby && gx < nbx;
  const int bidx = gy * nbx + gx;

  float v[16];
  // the samples of column `line`; tiles on the fast staging path hold no
  // np.pad samples, so their rows are linear in i (immediate LDS offsets)
  auto sample_col = [&](auto interior_tag) {
    constexpr bool INT = decltype(interior_tag)::value;
    if (plane == 0 || MODE == M444) {
      const int sx = (INT ? gx * 16 + line : reflect_pad(gx * 16 + line, g.W)) - x0 + 1;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int sy = (INT ? gy * 16 + i : reflect_pad(gy * 16 + i, g.H)) - y0 + 1;
        float R, G, B;
        rgbf(s_rgb[sy * WC + sx], R, G, B);
        v[i] = plane == 0 ? luma32m(R, G, B) : (plane == 1 ? cb32(R, G, B) : cr32(R, G, B)) - 128.0f;
      }
    } else if (CPLANE) {
      // pair sums of window rows 2r-1 .. 2r+2 (4:2:0: the combined taps, *0.25)
      // or r-1 .. r+1 (4:2:2: the Gaussian's column form, *0.5) of sample row r
      // (np.pad samples by reflected index off the fast staging path)
      const int sc = INT ? gx * 16 + line : reflect_pad(gx * 16 + line, g.wc);
      const float* s_pl = s_u + (plane == 1 ? 0 : WR * HW) + (sc - x0 / C::SX);
      const float h1 = gk32[3], h2 = gk32[4];
#pragma unroll 4
      for (int i = 0; i < 16; ++i) {
        const int sr = INT ? gy * 16 + i : reflect_pad(gy * 16 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;  // window row of the sample's first pixel row
        const float* col = s_pl + wr0 * HW;
        if constexpr (C::SY == 2)
          v[i] = fmaf(k2, col[2 * HW], fmaf(h2, col[HW], fmaf(h1, col[0], k0 * col[-HW]))) * 0.25f - 128.0f;
        else
          v[i] = fmaf(k0, col[HW] + col[-HW], k1 * col[0]) * 0.5f - 128.0f;
      }
    } else {
      // INTER_AREA mean of the unfiltered full-resolution chroma
      const int sc = INT ? gx * 16 + line : reflect_pad(gx * 16 + line, g.wc);
      const int wc0 = C::SX * sc - x0 + 1;
#pragma unroll 4  // full unrolling (window rows reused across samples) costs 20-50 VGPRs: occupancy 5 -> 3-4
      for (int i = 0; i < 16; ++i) {
        const int sr = INT ? gy * 16 + i : reflect_pad(gy * 16 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;
        float s[C::SY][2];
#pragma unroll
        for (int a = 0; a < C::SY; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {  // unfiltered chroma
            float R, G, B;
            rgbf(s_rgb[(wr0 + a) * WC + wc0 + b], R, G, B);
            s[a][b] = plane == 1 ? cb32(R, G, B) : cr32(R, G, B);
          }
        }
        if constexpr (C::SY == 2)
          v[i] = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
        else
          v[i] = (s[0][0] + s[0][1]) * 0.5f - 128.0f;
      }
    }
  };
  if (valid) {
    if (fast_stage)  // uniform per workgroup
      sample_col(std::integral_constant<bool, true>());
    else
      sample_col(std::integral_constant<bool, false>());
    fdct16_f32(v);  // axis 0 (columns) first
  }
  if constexpr (CPLANE) {
    __syncthreads();  // the block buffer aliases the chroma planes; s_rgb is free
    if (QLDS && tid < 192) *reinterpret_cast<float4*>(&s_tab[tab_t * 16 * QR + tab_r * QR + 4 * tab_q]) = tabv;
  }
  float* s_blk = s_u + blk * BS16F;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_blk[i * 17 + line] = v[i];
  }
  __syncthreads();

  // statistics per lane (one block row of 16 coefficients): nibble counters of
  // the common bins 22..29 (|q| small), two words so no nibble exceeds 8
  unsigned h[2] = {0u, 0u}, nz = 0u, mb = 0u, flag = (unsigned)fix_all;
  if (valid) {
    const int u = line;
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = s_blk[u * 17 + k];
    fdct16_f32(v);
    float rqv[16], thv[16];
    if constexpr (QLDS) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const float4 a = *reinterpret_cast<const float4*>(&s_tab[u * QR + 4 * qd]);
        const float4 b = *reinterpret_cast<const float4*>(&s_tab[(plane ? 2 : 1) * 16 * QR + u * QR + 4 * qd]);
        rqv[4 * qd] = a.x; rqv[4 * qd + 1] = a.y; rqv[4 * qd + 2] = a.z; rqv[4 * qd + 3] = a.w;
        thv[4 * qd] = b.x; thv[4 * qd + 1] = b.y; thv[4 * qd + 2] = b.z; thv[4 * qd + 3] = b.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        rqv[k] = fq.rq[u * 16 + k];
        thv[k] = fq.thr[plane ? 1 : 0][u * 16 + k];
      }
    }
    int q[16];
    // quant8's form (jds_fast.hip): |t| <= 2048 (|c| <= 16 * 128, Q >= 1), so
    // QMAGIC rounds exactly; the certificate is the sign bit of
    // |t - r| - (thr - |t| 2^-22) (< 0 exactly when certain), the rare test an OR
    unsigned ok = 0xffffffffu, orr = 0u, top;
    asm("v_mov_b32 %0, 0x80000000" : "=v"(top));  // opaque 2^31 (keeps the right shift below)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float t = v[k] * rqv[k];
      const float f = t + QMAGIC;
      const float r = f - QMAGIC;  // rintf(t)
      const uint32_t fb = __float_as_uint(f);
      // |t - r| is exact (Sterbenz); thr holds 0.5 - E/Q - slack, rounded down
      ok &= __float_as_uint(fabsf(t - r) - fmaf(fabsf(t), -0x1p-22f, thv[k]));
      q[k] = (int)(fb - QMAGIC_BITS);
      const int x = __builtin_amdgcn_frexp_expf(r);  // bit length of |q| (0 for q = 0; <= 12)
      nz += (unsigned)(x + 15) >> 4;
      mb += (unsigned)x;
      const unsigned o = fb - (QMAGIC_BITS - 12u);  // q + 12: bin 22 + o / 4 for q in [-12, 19]
      h[k >> 3] += top >> ((o & 28u) ^ 31u);       // 1 << (o & 28)
      orr |= o;
    }
    flag |= (~ok) >> 31;
    if (orr >= 32u) {  // rare values: taken back out of the nibbles, LDS atomics on the bin
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const unsigned o = (unsigned)(q[k] + 12);
        if (o >= 32u) {
          h[k >> 3] -= 1u << (o & 28u);
          if ((unsigned)(q[k] + 100) <= 200u) atomicAdd(&s_st[2 + (q[k] == 100 ? 49 : (q[k] + 100) >> 2)], 1u);
        }
      }
    }
    const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                          (long long)bidx * 256 + u * 16;
    uint4 pk[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int* qq = q + 8 * hh;
      pk[hh].x = (uint32_t)(uint16_t)qq[0] | ((uint32_t)(uint16_t)qq[1] << 16);
      pk[hh].y = (uint32_t)(uint16_t)qq[2] | ((uint32_t)(uint16_t)qq[3] << 16);
      pk[hh].z = (uint32_t)(uint16_t)qq[4] | ((uint32_t)(uint16_t)qq[5] << 16);
      pk[hh].w = (uint32_t)(uint16_t)qq[6] | ((uint32_t)(uint16_t)qq[7] << 16);
    }
    uint4* dst = reinterpret_cast<uint4*>(coeffs + off);
    dst[0] = pk[0];
    dst[1] = pk[1];
  }
  // a block with any uncertain coefficient goes to the exact fix-up: its 16
  // lanes are one quarter of a wave; the block's lane 0 appends it
  const unsigned long long fm = __ballot(valid && flag);
  if (fm) {  // wave-uniform
    const int lane = tid & 63;
    const bool mine = valid && line == 0 && ((fm >> (lane & ~15)) & 0xffffull);
    const unsigned long long lm = __ballot(mine);
    unsigned base = 0u;
    if (lane == __ffsll((long long)lm) - 1) base = atomicAdd(fixcount, (unsigned)__popcll(lm));
    base = __shfl(base, __ffsll((long long)lm) - 1, 64);
    if (mine) {
      const unsigned slot = base + (unsigned)__popcll(lm & ((1ull << lane) - 1ull));
      if (slot < cap) fixlist[slot] = make_uint2((unsigned)frame, ((unsigned)plane << 24) | (unsigned)bidx);
    }
  }
  stats_flush16(h[0], h[1], nz, mb, valid, s_st, part + ((size_t)frame * g.tiles_y * g.tiles_x + blockIdx.x) * NSTAT);
}

// ---------------------------------------------------------------- fix-up --
//
// Each 64-lane workgroup takes four listed blocks at a time, 16 lanes (one
// column each) per block; a fixed grid strides over the list (the forward
// launch completed before).  A lane forms its column's 16 samples exactly in
// registers (fix_column: the fp64 operations of sample64 / k_fwd16), runs
// pocketfft's 16-point DCT-II on them (axis 0, jds_dct16.hpp: 32x the
// reference's values), the block is transposed through LDS, the row lanes run
// the axis-1 transform, the quotient by 32 Q16 rounds half-even (k_fwd16's
// quantiser), and the statistics change by the difference to the stored row.

__device__ __forceinline__ double chroma_px(uint32_t R, uint32_t G, uint32_t B, int plane) {
  return plane == 1 ? chroma_b((double)R, (double)G, (double)B) : chroma_r((double)R, (double)G, (double)B);
}

// Four pixels x0 - 1 .. x0 + 2 of one image row: 12 bytes from byte offset a,
// read as the 4-aligned 16-byte span around them (inside the row: the caller
// keeps x0 + 3 < W).  Raw dwords first (issued one row ahead), chroma after.
struct Raw4 {
  uint32_t w0, w1, w2, w3, sh;
};
__device__ __forceinline__ Raw4 load_row4(const uint8_t* p, long long) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
  return Raw4{w[0], w[1], w[2], w[3], (uint32_t)((uintptr_t)p & 3)};
}
__device__ __forceinline__ void decode_row4(const Raw4& w, int plane, double (&c)[4]) {
  const uint32_t d0 = __builtin_amdgcn_alignbyte(w.w1, w.w0, w.sh), d1 = __builtin_amdgcn_alignbyte(w.w2, w.w1, w.sh),
                 d2 = __builtin_amdgcn_alignbyte(w.w3, w.w2, w.sh);
  c[0] = chroma_px(d0 & 255u, (d0 >> 8) & 255u, (d0 >> 16) & 255u, plane);
  c[1] = chroma_px(d0 >> 24, d1 & 255u, (d1 >> 8) & 255u, plane);
  c[2] = chroma_px((d1 >> 16) & 255u, d1 >> 24, d2 & 255u, plane);
  c[3] = chroma_px((d2 >> 8) & 255u, (d2 >> 16) & 255u, d2 >> 24, plane);
}
// the same four pixels at reflected columns xs[] of image row y (edge blocks)
struct Px4 {
  uint8_t b[12];
};
__device__ __forceinline__ Px4 load_px4(const uint8_t* img, const Geo& g, int y, const int (&xs)[4]) {
  Px4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint8_t* p = img + ((size_t)y * g.W + xs[j]) * 3;
    o.b[3 * j] = p[0];
    o.b[3 * j + 1] = p[1];
    o.b[3 * j + 2] = p[2];
  }
  return o;
}
__device__ __forceinline__ void decode_px4(const Px4& w, int plane, double (&c)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) c[j] = chroma_px(w.b[3 * j], w.b[3 * j + 1], w.b[3 * j + 2], plane);
}

// v[i] = sample(gy*16 + i, gx*16 + line) - 128 of the padded plane, exactly
// (col: the lane's column of the block's LDS tile, scratch for the interior
// prefiltered walk).
template <int MODE, bool PF>
__device__ __forceinline__ void fix_column(const uint8_t* __restrict__ img, const Geo& g, int plane, int gy, int gx,
                                           int line, const double (&k)[3], double (&v)[16], double* col) {
  constexpr int SY = Cfg16F<MODE>::SY;
  if (plane == 0 || MODE == M444) {
    const int x = reflect_pad(gx * 16 + line, g.W);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int y = reflect_pad(gy * 16 + i, g.H);
      const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
      const double R = p[0], G = p[1], B = p[2];
      v[i] = (plane == 0 ? luma(R, G, B) : (plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B))) - 128.0;
    }
    return;
  }
  const int sc = gx * 16 + line, x0 = 2 * sc;
  if constexpr (PF) {
    // the prefilter's rows walked down the column: window row r = full-
    // resolution row SY*16*gy - 1 + r (r < NR); sample i reads rows SY*i ..
    // SY*i + SY + 1.  Rows are walked in order with P rows' loads in flight,
    // the last SY + 2 row passes in a shift register; a sample is formed once
    // its last row is in and parked in the block's LDS column (runtime index).
    // Blocks inside the image read 4-aligned dword spans; blocks on the image
    // edge read bytes with BORDER_REFLECT_101 (cv2's filter border) -- every
    // block but those holding np.pad rows/columns, whose sample rows are not
    // monotone (sample64 per sample).
    const bool padded = gy * 16 + 16 > g.hc || gx * 16 + 16 > g.wc;  // uniform per 16-lane group
    if (!padded) {
      constexpr int NR = 16 * SY + 2, RING = SY + 2;
      auto walk = [&](auto load, auto decode, auto& raw, auto P_) {
        constexpr int P = decltype(P_)::value;
#pragma unroll
        for (int j = 0; j < P; ++j) raw[j] = load(j);
        double ra[RING], rb[RING];
#pragma unroll 1
        for (int r0 = 0; r0 < NR; r0 += P) {
#pragma unroll
          for (int j = 0; j < P; ++j) {
            const int r = r0 + j;
            if (r < NR) {  // uniform
#pragma unroll
              for (int q = 0; q + 1 < RING; ++q) {
                ra[q] = ra[q + 1];
                rb[q] = rb[q + 1];
              }
              double c[4];
              decode(raw[j], c);
              if (r + P < NR) raw[j] = load(r + P);
              double t = k[0] * c[0];  // cv2 RowFilter<double> at x0 and x0 + 1
              t = t + k[1] * c[1];
              ra[RING - 1] = t + k[2] * c[2];
              t = k[0] * c[1];
              t = t + k[1] * c[2];
              rb[RING - 1] = t + k[2] * c[3];
              // P is even, so r's parity is j's: the SY = 2 emission test folds
              if (r >= SY + 1 && (SY == 1 || (j & 1) == 1)) {
                const int i = (r - SY - 1) / SY;
                double sm[SY][2];
#pragma unroll
                for (int q = 0; q < SY; ++q) {  // ring[q + 1] = full-resolution row SY*(gy*16+i) + q
                  const double da = k[1] * ra[q + 1] + 0.0;  // SymmColumnFilter<double>
                  sm[q][0] = da + k[0] * (ra[q + 2] + ra[q]);
                  const double db = k[1] * rb[q + 1] + 0.0;
                  sm[q][1] = db + k[0] * (rb[q + 2] + rb[q]);
                }
                double m;
                if constexpr (SY == 2)
                  m = (((sm[0][0] + sm[0][1]) + sm[1][0]) + sm[1][1]) * 0.25;
                else
                  m = (sm[0][0] + sm[0][1]) * 0.5;
                col[i * 17] = m - 128.0;
              }
            }
          }
        }
      };
      const int yw0 = SY * 16 * gy - 1;
      const bool interior = gy > 0 && gx > 0 && yw0 + NR <= g.H && 32 * gx + 34 < g.W;  // uniform per group
      if (interior) {
        const long long stride = (long long)g.W * 3;
        const uint8_t* rowp = img + ((long long)yw0 * g.W + x0 - 1) * 3;
        Raw4 raw[8];
        walk([&](int r) { return load_row4(rowp + r * stride, 0); },
             [&](const Raw4& w, double (&c)[4]) { decode_row4(w, plane, c); }, raw,
             std::integral_constant<int, 8>());
      } else {
        const int xs[4] = {reflect101(x0 - 1, g.W), x0, x0 + 1, reflect101(x0 + 2, g.W)};
        Px4 raw[4];
        walk([&](int r) { return load_px4(img, g, reflect101(yw0 + r, g.H), xs); },
             [&](const Px4& w, double (&c)[4]) { decode_px4(w, plane, c); }, raw,
             std::integral_constant<int, 4>());
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = col[i * 17];
      return;
    }
#pragma unroll 2
    for (int i = 0; i < 16; ++i) v[i] = sample64<MODE, PF>(img, g, plane, gy * 16 + i, sc, k) - 128.0;
    return;
  } else {  // INTER_AREA mean without the prefilter
    const int xr = reflect_pad(sc, g.wc);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int sr = reflect_pad(gy * 16 + i, g.hc);
      double s[SY][2];
#pragma unroll
      for (int a = 0; a < SY; ++a) {
        const uint8_t* p = img + ((size_t)(SY * sr + a) * g.W + 2 * xr) * 3;
        s[a][0] = chroma_px(p[0], p[1], p[2], plane);
        s[a][1] = chroma_px(p[3], p[4], p[5], plane);
      }
      double m;
      if constexpr (SY == 2)
        m = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25;
      else
        m = (s[0][0] + s[0][1]) * 0.5;
      v[i] = m - 128.0;
    }
  }
}

// Workgroups past the first gfix (gridDim.x - n * per) are the statistics
// reduction instead (k_fwd_reduce's work, one launch fewer): workgroup r sums
// tiles [64 s, 64 s + 64) of frame r / per (s = r % per) of k_fwd16f's per-tile
// partials, lane j < 52 statistic j, one u64 atomic per statistic; both roles
// only add into the frame statistics.
constexpr int FIX16_RED_TILES = 64;
template <int MODE, bool PF>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
k_fix_fwd16(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
            const FrameQ* __restrict__ fq, const double* __restrict__ gk, jds_frame_stats* __restrict__ st,
            const uint2* __restrict__ fixlist, const unsigned* __restrict__ fixcount, unsigned* __restrict__ fixlen,
            const unsigned cap, const uint32_t* __restrict__ part, const int ptiles, const int nframes) {
  const int per = (ptiles + FIX16_RED_TILES - 1) / FIX16_RED_TILES;
  const int gfix = (int)gridDim.x - nframes * per;
  if ((int)blockIdx.x >= gfix) {  // (uniform) the reduction role
    const int r = (int)blockIdx.x - gfix, f = r / per, t0 = (r - f * per) * FIX16_RED_TILES;
    const int j = threadIdx.x, nt = min(FIX16_RED_TILES, ptiles - t0);
    if (j < 52) {
      const uint32_t* src = part + ((size_t)f * ptiles + t0) * 52 + j;
      unsigned long long a = 0ull;
#pragma unroll 16
      for (int i = 0; i < nt; ++i) a += src[(size_t)i * 52];
      jds_frame_stats* sf = st + f;
      unsigned long long* dst = j == 0 ? (unsigned long long*)&sf->nonzero
                                : j == 1 ? (unsigned long long*)&sf->magnitude_bits
                                         : (unsigned long long*)&sf->hist[j - 2];
      if (a) atomicAdd(dst, a);
    }
    return;
  }
  __shared__ double s_b[4 * 272];  // four blocks, rows of 17 (jds_b16.hip's BS16 layout)
  const int lane = threadIdx.x, grp = lane >> 4, line = lane & 15;
  const unsigned c = *fixcount;
  const unsigned count = c < cap ? c : cap;
  const double k[3] = {gk[0], gk[1], gk[2]};
  double* const sb = s_b + grp * 272;
  for (unsigned e0 = blockIdx.x * 4u; e0 < count; e0 += (unsigned)gfix * 4u) {
    const unsigned e = e0 + (unsigned)grp;
    const bool act = e < count;  // uniform per 16-lane group
    int frame = 0, plane = 0, bidx = 0, gy = 0, gx = 0;
    uint4 o0 = make_uint4(0u, 0u, 0u, 0u), o1 = o0;
    uint4* dst = nullptr;
    double v[16];
    if (act) {
      const uint2 ent = fixlist[e];
      frame = (int)ent.x;
      plane = (int)(ent.y >> 24);
      bidx = (int)(ent.y & 0xffffffu);
      const int nbx = plane ? g.ncx : g.nbx;
      gy = bidx / nbx;
      gx = bidx - gy * nbx;
      // row `line` of the stored block, fetched first (its latency hides under the sampling)
      const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                            (long long)bidx * 256 + line * 16;
      dst = reinterpret_cast<uint4*>(coeffs + off);
      o0 = dst[0];
      o1 = dst[1];
      fix_column<MODE, PF>(rgb + (size_t)frame * g.H * g.W * 3, g, plane, gy, gx, line, k, v, sb + line);
      dct2_line16(v);  // axis 0, column `line`
#pragma unroll
      for (int r = 0; r < 16; ++r) sb[r * 17 + line] = v[r];
    }
    __builtin_amdgcn_wave_barrier();  // the exchange is wave-local; the LDS keeps a wave's order
    if (act) {  // axis 1, row u = line; requantize and correct the statistics
      const int u = line;
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) v[cc] = sb[u * 17 + cc];
      dct2_line16(v);
      const uint32_t ow[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
      uint32_t nw[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
      long long dnz = 0, dmb = 0;
      jds_frame_stats* fs = st + frame;
      const double* q8 = fq[frame].q + (u >> 1) * 8;
      double rq[8];  // 1 / (32 Q8[u/2][j]): each serves two coefficients
#pragma unroll
      for (int j = 0; j < 8; ++j) rq[j] = recip64(32.0 * q8[j]);
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        // quantizer.py:22-24: the true quotient of the reference's coefficient
        // (v / 32, exact) by Q16 = Q8[u/2][cc/2] (rint_quot: the division only
        // near a half-integer)
        const int qn = rint_quot(v[cc], 32.0 * q8[cc >> 1], rq[cc >> 1]);
        const int qo = (int16_t)((ow[cc >> 1] >> ((cc & 1) * 16)) & 0xffffu);
        nw[cc >> 1] |= (uint32_t)(uint16_t)qn << ((cc & 1) * 16);
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
      dst[0] = make_uint4(nw[0], nw[1], nw[2], nw[3]);
      dst[1] = make_uint4(nw[4], nw[5], nw[6], nw[7]);
      if (dnz) atomicAdd((unsigned long long*)&fs->nonzero, (unsigned long long)dnz);
      if (dmb) atomicAdd((unsigned long long*)&fs->magnitude_bits, (unsigned long long)dmb);
    }
    __builtin_amdgcn_wave_barrier();  // the next iteration's column writes after these row reads
  }
  // the run's list length for jds_plan_fix_counts (the counter itself is
  // zeroed by the run after next's forward; no ticket: 4096 workgroups
  // serialising on one device-scope atomic took ~150 us)
  if (blockIdx.x == 0 && lane == 0) *fixlen = c;
}

// ------------------------------------------------------------ launchers --

constexpr int FIX16_GRID = 8192;  // k_fix_fwd16 workgroups (x 4 blocks in flight; 4096: 87 -> 73 us at configs[4] 16x16)

template <int MODE, bool PF>
static hipError_t fast16_t(const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs, const FrameQ* fq,
                           const void* fq16, const double* gk, const float* gk32, jds_frame_stats* st,
                           uint32_t* part, uint2* fixlist, unsigned* counters, int fix_all, int parity,
                           hipStream_t s) {
  using C = Cfg16F<MODE>;
  const unsigned cap = (unsigned)((g.cpf / 256) * n);
  const int tiles = g.tiles_y * g.tiles_x;
  hipLaunchKernelGGL((k_fwd16f<MODE, PF>), dim3(tiles, n), dim3(C::TF), 0, s, g, rgb, coeffs, (const FastQ16*)fq16,
                     gk32, part, fixlist, counters + parity, counters + (parity ^ 1), cap, fix_all);
  kmark(s, "k_fwd16f<%d,%d>", MODE, (int)PF);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the fix-up and the per-tile partials' reduction (order-free: u64 atomics) in one launch
  const int nred = n * ((tiles + FIX16_RED_TILES - 1) / FIX16_RED_TILES);
  hipLaunchKernelGGL((k_fix_fwd16<MODE, PF>), dim3(FIX16_GRID + nred), dim3(64), 0, s, g, rgb, coeffs, fq, gk, st,
                     fixlist, counters + parity, counters + 2, cap, part, tiles, n);
  kmark(s, "k_fix_fwd16<%d,%d>", MODE, (int)PF);
  return hipGetLastError();
}

// counters: [0..1] list lengths (this run appends to [parity]), [2] the run's length
hipError_t launch_fast_fwd16(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs,
                             const FrameQ* fq, const void* fq16, const double* gk, const float* gk32,
                             jds_frame_stats* st, uint32_t* part, uint2* fixlist, unsigned* counters, int fix_all,
                             int parity, hipStream_t s) {
  switch (mode) {
    case M420:
      return pf ? fast16_t<M420, true>(g, n, rgb, coeffs, fq, fq16, gk, gk32, st, part, fixlist, counters, fix_all, parity, s)
                : fast16_t<M420, false>(g, n, rgb, coeffs, fq, fq16, gk, gk32, st, part, fixlist, counters, fix_all, parity, s);
    case M422:
      return pf ? fast16_t<M422, true>(g, n, rgb, coeffs, fq, fq16, gk, gk32, st, part, fixlist, counters, fix_all, parity, s)
                : fast16_t<M422, false>(g, n, rgb, coeffs, fq, fq16, gk, gk32, st, part, fixlist, counters, fix_all, parity, s);
    default:
      return fast16_t<M444, false>(g, n, rgb, coeffs, fq, fq16, gk, gk32, st, part, fixlist, counters, fix_all, parity, s);
  }
}

// ---------------------------------------------------- host: the bounds --
//
// fast_fwd_bounds with 16-point passes (fdct16_f32's sequence).  A chain
// over n inputs of magnitude <= M and error <= eps, with weights W (fp32),
// has error <= b eps + u M (b + P): b = sum |W| (the inputs' error, and the
// fp32 representation error of W: <= u |W| M per term), P = the sum of the
// chain's partial sums of |W| (each step rounds a partial sum <= M * prefix).
// Inputs |x| <= X, error e: s_i, d_i have |.| <= 2X, error 2e + 2uX;
// e_i, o_i |.| <= 4X, error 4e + 8uX.
static void chain_bound(const float* w, int n, double M, double eps, double* Mout, double* eout) {
  const double u = 0x1p-24;
  double b = 0, P = 0, pre = 0;
  for (int i = 0; i < n; ++i) {
    b += fabs((double)w[i]);
    pre += fabs((double)w[i]);
    P += pre;
  }
  *Mout = M * b;
  *eout = b * eps + u * M * (b + P);
}
static void pass_bound16(double X, double e, double* Xout, double* eout) {
  const double u = 0x1p-24;
  for (int k = 0; k < 16; ++k) {
    if (k & 1)
      chain_bound(W16[k], 8, 2 * X, 2 * e + 2 * u * X, &Xout[k], &eout[k]);
    else
      chain_bound(W16[k], 4, 4 * X, 4 * e + 8 * u * X, &Xout[k], &eout[k]);
  }
}

void fast_fwd16_bounds(int mode, bool pf, const double* gk, double* E /*2 x 256*/) {
  for (int p = 0; p < 2; ++p) {
    const double e_in = fwd_input_error(p, mode, pf, gk, 2);  // both staging paths: combined taps
    double X1[16], e1[16];
    pass_bound16(128.0, e_in, X1, e1);
    double E2[16][16];
    for (int k = 0; k < 16; ++k) {
      double X2[16], e2[16];
      pass_bound16(X1[k], e1[k], X2, e2);
      for (int l = 0; l < 16; ++l) E2[k][l] = e2[l];
    }
    for (int k = 0; k < 16; ++k)
      for (int l = 0; l < 16; ++l) {
        const double e2l = E2[k][l] > E2[l][k] ? E2[k][l] : E2[l][k];  // either pass order
        E[p * 256 + k * 16 + l] = e2l * (1 + 1e-5) + 1e-9;            // + the fp64 reference's own error
      }
  }
}

// Q8: the frame's 8x8 table; the 16x16 table is Q16[u][v] = Q8[u/2][v/2].
void fast_fwd16_thresholds(const double* Q8, int mode, bool pf, const double* gk, void* out) {
  FastQ16* f = (FastQ16*)out;
  double E[512];
  fast_fwd16_bounds(mode, pf, gk, E);
  for (int i = 0; i < 256; ++i) f->rq[i] = (float)(1.0 / Q8[((i >> 4) >> 1) * 8 + ((i & 15) >> 1)]);
  for (int p = 0; p < 2; ++p)
    for (int i = 0; i < 256; ++i) {
      const double Q = Q8[((i >> 4) >> 1) * 8 + ((i & 15) >> 1)];
      const double tq = E[p * 256 + i] / Q * (1 + 1e-5) + 1e-7;
      const double lim = 0.5 - tq * (1 + 0x1p-20) - 0x1p-23;
      float v = (float)lim;
      if ((double)v > lim) v = nextafterf(v, 0.0f);
      f->thr[p][i] = v;
    }
}

size_t fast_q16_size() { return sizeof(FastQ16); }

// Test-only: the fp32 chain of k_fwd16f for every 16x16 block of one plane of
// an H x W RGB image (plane size a multiple of 16), in either pass order
// (rows_first 0 = the kernel's columns first), before quantisation.
void combined_taps32(const double* gk, float* out5);
int fwd16_host_plane(int mode, bool pf, const double* gk, const uint8_t* rgb, int H, int W, int plane,
                     int flags, float* out) {
  const bool rows_first = (flags & 1) != 0, comb = (flags & 2) != 0;  // comb: k_fwd16f's fast staging
  const int sy = mode == M420 ? 2 : 1, sx = mode == M444 ? 1 : 2;
  const int ph = plane == 0 ? H : H / sy, pw = plane == 0 ? W : W / sx;
  if (ph % 16 || pw % 16) return -1;
  const float k0 = (float)gk[0], k1 = (float)gk[1], k2 = (float)gk[2];
  auto refl = [](int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
  };
  auto px = [&](int y, int x, int c) { return (float)rgb[((size_t)y * W + x) * 3 + c]; };
  auto chroma = [&](int y, int x) {
    const float R = px(y, x, 0), G = px(y, x, 1), B = px(y, x, 2);
    return plane == 1 ? cb32(R, G, B) : cr32(R, G, B);
  };
  auto rowf = [&](int y, int x) {
    return fmaf(k2, chroma(y, refl(x + 1, W)), fmaf(k1, chroma(y, x), k0 * chroma(y, refl(x - 1, W))));
  };
  float h[5];
  combined_taps32(gk, h);
  auto pairf = [&](int y, int j) {  // combined taps over chroma columns 2j-1 .. 2j+2 of row y
    return fmaf(h[2], chroma(y, refl(2 * j + 2, W)),
                fmaf(h[4], chroma(y, 2 * j + 1), fmaf(h[3], chroma(y, 2 * j), h[0] * chroma(y, refl(2 * j - 1, W)))));
  };
  auto sample = [&](int y, int x) -> float {
    if (plane == 0) return luma32m(px(y, x, 0), px(y, x, 1), px(y, x, 2));
    if (mode == M444) return chroma(y, x) - 128.0f;
    if (pf && comb) {
      if (sy == 2)
        return fmaf(h[2], pairf(refl(2 * y + 2, H), x),
                    fmaf(h[4], pairf(2 * y + 1, x), fmaf(h[3], pairf(2 * y, x), h[0] * pairf(refl(2 * y - 1, H), x)))) *
                   0.25f - 128.0f;
      return fmaf(k0, pairf(refl(y + 1, H), x) + pairf(refl(y - 1, H), x), k1 * pairf(y, x)) * 0.5f - 128.0f;
    }
    float s[2][2];
    for (int a = 0; a < sy; ++a)
      for (int b = 0; b < 2; ++b) {
        const int yy = sy * y + a, xx = 2 * x + b;
        s[a][b] = pf ? fmaf(k0, rowf(refl(yy + 1, H), xx) + rowf(refl(yy - 1, H), xx), k1 * rowf(yy, xx))
                     : chroma(yy, xx);
      }
    if (sy == 2) return (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
    return (s[0][0] + s[0][1]) * 0.5f - 128.0f;
  };
  const int nbx = pw / 16;
  for (int by = 0; by < ph / 16; ++by)
    for (int bx = 0; bx < nbx; ++bx) {
      float b[16][16];
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) b[i][j] = sample(by * 16 + i, bx * 16 + j);
      for (int pass = 0; pass < 2; ++pass) {
        const bool rows = (pass == 0) == rows_first;
        for (int i = 0; i < 16; ++i) {
          float v[16];
          for (int j = 0; j < 16; ++j) v[j] = rows ? b[i][j] : b[j][i];
          fdct16_f32(v);
          for (int j = 0; j < 16; ++j) (rows ? b[i][j] : b[j][i]) = v[j];
        }
      }
      float* o = out + ((size_t)by * nbx + bx) * 256;
      for (int i = 0; i < 256; ++i) o[i] = b[i / 16][i % 16];
    }
  return 0;
}

}  // namespace jds
