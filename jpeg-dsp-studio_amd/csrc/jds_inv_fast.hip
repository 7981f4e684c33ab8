// jds_inv_fast.hip — the certified fast inverse: int16 coefficients -> RGB
// bytes, bit-identical to the reference (engines/pipeline.py:68-95) without
// replaying its operation order.
//
// The reference's bytes are trunc(clip(v_ref, 0, 255)) of fp64 values v_ref
// (dequantize, pocketfft idctn, +128, clip, cv2 INTER_LINEAR upsample,
// ycbcr_to_rgb: quantizer.py:27-29, dct_engine.py:23-27, color_space.py:17-24
// and :63-65).  The exact kernel (jds_inv.hip, k_inv2) replays every one of
// those roundings.  This kernel computes the same real numbers in fp64 with a
// cheaper order:
//   * AAN IDCT (5 multiplies per 8-point line) with the AAN scales and the 1/8
//     normalisation folded into the dequantisation (one product per
//     coefficient: q * Qs[u][v]), no +128: both planes clip to [-128, 127];
//   * the bilinear upsample unnormalised: a vertical sum a + 3b of the lane's
//     6 chroma columns, then a horizontal far + 3 near per pixel (one fma
//     each: 14 per lane, row and plane at 4:2:0), the result 16x (4:2:0) or 4x
//     (4:2:2) the blend, the scale folded into the colour constants;
//   * the colour terms added onto Y + 1.5 * 2^20 + 128 (one fma per term), so
//     each output lands on a grid of spacing 2^-32 whose words give both the
//     byte and the certificate (byte_cert_y).
// Every output value v_fast then differs from v_ref by at most
// E = K_LIN * Dmax + K_CONST + 2^-31, where Dmax bounds |q * Q| over the
// coefficients the tile reads and 2^-31 covers the <= 3 roundings on the grid
// (tools/inv_bound.py derives K_LIN / K_CONST rigorously for both operation
// orders as they stand in this file, every fused multiply-add counted as two
// roundings; tests/test_inv_bound_cpu.py pins the constants below to it and
// runs this file's chain on the host, jds_selftest_inv_fast, against the
// oracle on adversarial inputs).
// If no integer lies within E of v_fast, trunc(clip(v_fast)) ==
// trunc(clip(v_ref)): the byte is certified.  Each lane tracks the smallest
// distance to an integer over its samples and the largest |q|; a workgroup
// whose tile has any uncertain sample recomputes the whole tile at once with
// the exact replayed-order code (jds_inv_exact.hpp, the body of k_inv2), in the
// same LDS.  On the bench's random frames E ~ 1e-8 and a tile needs that with
// probability ~1e-3; exact ties (flat gray or saturated regions whose
// reference value is an integer up to pocketfft noise) always do, so those
// tiles cost fast + exact.  (Recomputing only the affected blocks was
// measured slower: the per-round bookkeeping cost the common path more than
// it saved.)
//
// Work decomposition and LDS layout are k_inv2's (jds_inv_common.hpp): one
// workgroup per tile, chroma window (with the ring the upsample reaches into)
// in LDS, Y in registers, one lane per 8-pixel row, 24-byte stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_inv_common.hpp"
#include "jds_inv_exact.hpp"
#include "jds_inv16_exact.hpp"

// every fusion the compiler forms is covered by the bound (two roundings per
// fused pair); reassociation stays off
#pragma clang fp contract(fast)

namespace jds {

// tools/inv_bound.py (the v25 chain as it stands in this file: unnormalised
// upsample): e_fast + e_ref <= K_LIN * Dmax + K_CONST off the magic grid, x2
// safety included (tests/test_inv_bound_cpu.py asserts kernel >= model)
constexpr double K_LIN = 8.762155e-13 * 1.01;
constexpr double K_CONST = 1.024801e-12 * 1.01;
// the same for 16x16 blocks (fidct16 vs dct3_line16, tools/inv_bound.py --b16)
constexpr double K_LIN16 = 3.345910e-12 * 1.01;
constexpr double K_CONST16 = 1.024801e-12 * 1.01;

// AAN scale factors a_k = sqrt(2) cos(k pi / 16), a_0 = 1 (correctly rounded;
// tools/inv_bound.py reads them from this list and prices their representation
// errors)
#define JDS_AAN_LIST                                                                                 \
  1.0, 0x1.63150b15e8536p+0, 0x1.4e7ae9144f0fcp+0, 0x1.2d062ef88e319p+0, 1.0, 0x1.92469c0dcf32dp-1, \
      0x1.1517a7bdb3895p-1, 0x1.1a855dec071b5p-2
__constant__ double c_aan[8] = {JDS_AAN_LIST};
static const double h_aan[8] = {JDS_AAN_LIST};  // the host restatement's copy
constexpr double F_SQ2 = 0x1.6a09e667f3bcdp+0;   // sqrt(2)
constexpr double F_A2C2 = 0x1.d906bcf328d46p+0;  // 2 cos(pi/8)
constexpr double F_K10 = 0x1.1517a7bdb3895p+0;   // 2 (cos(pi/8) - cos(3pi/8))
constexpr double F_K12 = 0x1.4e7ae9144f0fcp+1;   // 2 (cos(pi/8) + cos(3pi/8))

// 16-point lines (fidct16, the 16x16 stretch path): odd-part pre-scales
// cos(j pi / 16), j = 1..7, and post-scales sqrt(2) / (8 cos((2n+1) pi / 32)),
// n = 0..7 (correctly rounded; tools/inv_bound.py --b16 reads both lists)
#define JDS_F16_PRE_LIST                                                                                     \
  0x1.f6297cff75cb0p-1, 0x1.d906bcf328d46p-1, 0x1.a9b66290ea1a3p-1, 0x1.6a09e667f3bcdp-1, 0x1.1c73b39ae68c8p-1, \
      0x1.87de2a6aea963p-2, 0x1.8f8b83c69a60bp-3
#define JDS_F16_POST_LIST                                                                                    \
  0x1.6bca591d6776cp-3, 0x1.7a54542b3c092p-3, 0x1.9a82e694c86a2p-3, 0x1.d45957fdd6b90p-3, 0x1.1d57ab02f5b32p-2, \
      0x1.80019f8d550e5p-2, 0x1.37cbd5ba8838cp-1, 0x1.cdb4095cb49fcp+0
constexpr double F16_PRE[8] = {1.0, JDS_F16_PRE_LIST};  // [0]: W_0 = Z_0 unscaled
constexpr double F16_POST[8] = {JDS_F16_POST_LIST};

// The chain's multiply-adds go through a policy so that the host restatement
// (jds_selftest_inv_fast, tests/test_inv_bound_cpu.py) runs the same source:
// on the device MadDev writes a * b + c and the compiler fuses what it likes
// under this unit's fp contract(fast) (the bound covers either way); the host
// runs it unfused (MadSep: x86-64 has no FMA at the default target) and fully
// fused (MadFma: std::fma at every site).
struct MadDev {
  __host__ __device__ static double mad(double a, double b, double c) { return a * b + c; }
};
struct MadFma {
  static double mad(double a, double b, double c) { return std::fma(a, b, c); }
};

// One 8-point AAN IDCT line on scaled inputs (inputs pre-multiplied by
// a_u / sqrt(8) per axis; outputs are the orthonormal IDCT).  The operation
// sequence is the one tools/inv_bound.py::aan_line models.
template <class M = MadDev>
__host__ __device__ __forceinline__ void aan8(double (&v)[8]) {
  const double t10 = v[0] + v[4], t11 = v[0] - v[4];
  const double t13 = v[2] + v[6];
  const double t12 = M::mad(v[2] - v[6], F_SQ2, -t13);
  const double e0 = t10 + t13, e3 = t10 - t13, e1 = t11 + t12, e2 = t11 - t12;
  const double z13 = v[5] + v[3], z10 = v[5] - v[3], z11 = v[1] + v[7], z12 = v[1] - v[7];
  const double o7 = z11 + z13;
  const double o11 = (z11 - z13) * F_SQ2;
  const double z5 = (z10 + z12) * F_A2C2;
  const double o10 = M::mad(-z12, F_K10, z5);
  const double o12 = M::mad(-z10, F_K12, z5);
  const double o6 = o12 - o7, o5 = o11 - o6, o4 = o10 - o5;
  v[0] = e0 + o7;
  v[7] = e0 - o7;
  v[1] = e1 + o6;
  v[6] = e1 - o6;
  v[2] = e2 + o5;
  v[5] = e2 - o5;
  v[3] = e3 + o4;
  v[4] = e3 - o4;
}

// cv2 INTER_LINEAR's blends at an exact 2x scale, unnormalised: the vertical
// a * 1/4 + b * 3/4 (a the "quarter" row) as a + 3b, the horizontal (far 1/4,
// near 3/4) as far + 3 near -- one fma each; every blended axis scales the
// chroma by 4, which the colour constants take back (USC<SH> = 2^-SH, exact)
template <class M = MadDev>
__host__ __device__ __forceinline__ double fvsum(double a, double b) { return M::mad(b, 3.0, a); }
template <class M = MadDev>
__host__ __device__ __forceinline__ double fhsum(double far, double near) { return M::mad(near, 3.0, far); }
template <int SH>
constexpr double USC = SH == 0 ? 1.0 : (SH == 2 ? 0.25 : 0.0625);
// SH of a subsampling: 2 per blended axis
template <int SY, int SX>
constexpr int USH = (SY == 2 ? 2 : 0) + (SX == 2 ? 2 : 0);

// The colour terms onto Y + MAGIC + 128 (byte_cert_y's grid): out = B, Gt, R,
// G; the chroma operand at scale 2^SH (fvsum / fhsum)
template <class M = MadDev, int SH = 0>
__host__ __device__ __forceinline__ double col_b(double yv, double cb) { return M::mad(cb, 1.772 * USC<SH>, yv); }
template <class M = MadDev, int SH = 0>
__host__ __device__ __forceinline__ double col_gt(double yv, double cb) { return M::mad(cb, -0.344136 * USC<SH>, yv); }
template <class M = MadDev, int SH = 0>
__host__ __device__ __forceinline__ double col_r(double yv, double cr) { return M::mad(cr, 1.402 * USC<SH>, yv); }
template <class M = MadDev, int SH = 0>
__host__ __device__ __forceinline__ double col_g(double gt, double cr) { return M::mad(cr, -0.714136 * USC<SH>, gt); }

// Axis-0 pass of column v of one block: dequantise with the folded table,
// AAN, into the transpose buffer (no +128: fast_row clips to [-128, 127] and
// the luma's +128 rides on the magic constant, see byte_cert_y).
// qhi / qlo track the largest and smallest q the lane read (integer max3 /
// min3 chains: cheaper than an fp64 max of |q| per coefficient).
// The folded table is held transposed in LDS (column v's eight
// entries contiguous, rows padded to QS_STRIDE doubles so the 8 columns' 16-B
// slots fall on disjoint banks): four ds_read_b128 per column instead of four
// ds_read2_b64 (8 LDS cycles each at 32-bank granularity, MI355X_MICROARCH.md).
constexpr int QS_STRIDE = 10;
constexpr int QS_WORDS = 1 ? 8 * QS_STRIDE : 64;
__device__ __forceinline__ int qs_index(int r, int v) { return 1 ? v * QS_STRIDE + r : r * 8 + v; }
__device__ __forceinline__ void fast_col(const Col16& in, const double* __restrict__ qs, int v,
                                         double* __restrict__ dst, int& qhi, int& qlo) {
  double c[8];
  double t[8];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double2 d = *reinterpret_cast<const double2*>(qs + v * QS_STRIDE + 2 * p);
    t[2 * p] = d.x;
    t[2 * p + 1] = d.y;
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const double qd = (double)in.q[r];
    qhi = max(qhi, (int)in.q[r]);
    qlo = min(qlo, (int)in.q[r]);
    c[r] = qd * t[r];
  }
  aan8(c);
#pragma unroll
  for (int r = 0; r < 8; ++r) dst[tslot(r, v)] = c[r];
}

// Axis-1 pass of row u, clip to [LO, LO + 255] (dct_engine.py:27).  Both planes
// run without the reference's +128 and clip to [-128, 127] (clip(x + 128, 0,
// 255) - 128 = clip(x, -128, 127)): the chroma window holds the shifted samples
// directly and the luma's +128 rides on the magic constant; fewer roundings and
// smaller magnitudes than the +128-folded form tools/inv_bound.py models.
template <int LO = 0, bool CLIP = true>
__device__ __forceinline__ void fast_row(const double* __restrict__ src, int u, double (&c)[8]) {
  const int sw = u & 3;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double2 d = *reinterpret_cast<const double2*>(src + u * 8 + 2 * (p ^ sw));
    c[2 * p] = d.x;
    c[2 * p + 1] = d.y;
  }
  aan8(c);
  if constexpr (CLIP) {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = fmin(fmax(c[k], (double)LO), (double)(LO + 255));
  }
}

// One plane's upsampled (chroma - 128) at the lane's 8 pixels, times 2^USH
// (cv2 INTER_LINEAR at an exact 2x scale: pixel 2m weights (1/4, 3/4) on
// chroma columns (m-1, m), pixel 2m+1 (3/4, 1/4) on (m, m+1); rows likewise
// with clamped indices; fvsum / fhsum).  cv2 copies the edge column at the two
// image-edge pixels; here the window holds that column replicated into the
// ring (see the window writes), so the same blend gives the same real value:
// no per-pixel selects.
template <int MODE>
__device__ __forceinline__ void chroma8_fast(const double* __restrict__ cw, int x0, int cwx0, int wq, int wt,
                                             double (&C)[8]) {
  using I = Inv<MODE>;
  if constexpr (I::SX == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) C[k] = cw[wq * I::CWS + x0 + k - cwx0];
  } else {
    const int c0 = x0 / 2 - 1 - cwx0;
    double vb[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if constexpr (I::SY == 2)
        vb[j] = fvsum(cw[wq * I::CWS + c0 + j], cw[wt * I::CWS + c0 + j]);
      else
        vb[j] = cw[wq * I::CWS + c0 + j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      C[2 * i] = fhsum(vb[i], vb[i + 1]);          // (1/4, 3/4) on (m-1, m)
      C[2 * i + 1] = fhsum(vb[i + 2], vb[i + 1]);  // (3/4, 1/4) on (m, m+1)
    }
  }
}

// Byte and certificate of one output value v from y = v + 1.5 * 2^20
// has a fixed exponent for |v| < 2^19, so its high word is 0x41380000 +
// floor(v') and its low word is frac(v') * 2^32, where v' = y - 1.5 * 2^20 is v
// rounded to a multiple of 2^-32 (|v' - v| <= 2^-33, added to the bound).
// med3 of the high word against [0x41380000, 0x413800FF] leaves
// clamp(floor(v'), 0, 255) in its low byte (the reference's clip +
// astype(uint8), pipeline.py:95); the smallest and largest low words seen
// tell how close any value came to an integer.  The colour terms add onto
// Y + MAGIC (one add per pixel instead of one per channel): each of the <= 3
// roundings on the way (Y + MAGIC, then one or two fmas) lands on the same
// 2^-32 grid, |error| <= 2^-33 each, so the certificate adds 2^-31
// (tools/inv_bound.py prices everything off the grid: the products C * k fused
// or rounded, and the constants' representation errors).
constexpr double MAGIC = 0x1.8p+20;
constexpr uint32_t MAGIC_HI = 0x41380000u;

__device__ __forceinline__ uint32_t byte_cert_y(double y, uint32_t& lo_min, uint32_t& lo_max) {
  const uint32_t lo = (uint32_t)__double2loint(y), hi = (uint32_t)__double2hiint(y);
  lo_min = lo_min < lo ? lo_min : lo;
  lo_max = lo_max > lo ? lo_max : lo;
  const uint32_t c = hi < MAGIC_HI ? MAGIC_HI : hi;
  return c > MAGIC_HI + 255u ? MAGIC_HI + 255u : c;  // v_med3_u32; the byte is bits 0-7
}

// The same without the clamp: the high word itself, whose low 16 bits are
// floor(v') as an int16 (|v'| < 2^15), for pack4s.
__device__ __forceinline__ uint32_t cert_hi(double y, uint32_t& lo_min, uint32_t& lo_max) {
  const uint32_t lo = (uint32_t)__double2loint(y), hi = (uint32_t)__double2hiint(y);
  lo_min = lo_min < lo ? lo_min : lo;
  lo_max = lo_max > lo ? lo_max : lo;
  return hi;
}
// Four bytes clamp(int16 low half, 0, 255) of cert_hi words a, b, c, d into one
// word: the int16 pairs by two byte permutes, v_sat_pk_u8_i16 clamps and packs
// each pair, one shift-or joins them (5 operations instead of 4 med3 + 3).
__device__ __forceinline__ uint32_t sat_pk_u8_i16(uint32_t x) {
  uint32_t r;
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t pack4s(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t ab = sat_pk_u8_i16(__builtin_amdgcn_perm(b, a, 0x05040100u));  // a.lo16 | b.lo16 << 16
  const uint32_t cd = sat_pk_u8_i16(__builtin_amdgcn_perm(d, c, 0x05040100u));
  return ab | (cd << 16);
}

// Four bytes (bits 0-7 of a, b, c, d) into one word: two byte permutes and an or.
__device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t ab = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);  // a.b0 | b.b0 << 8
  const uint32_t cd = __builtin_amdgcn_perm(d, c, 0x04000c0cu);  // c.b0 << 16 | d.b0 << 24
  return ab | cd;
}

// The tile certificate's reduction: per 16-lane row by four
// DPP row shifts (lanes without a source keep the identity), then the row
// totals into three LDS words by LDS min / max atomics (no return): thread 0
// reads three words instead of looping over every wave's record, and the
// waves skip six cross-lane permutes per value.
template <int SH>
__device__ __forceinline__ void cert_row_step(uint32_t& mn, uint32_t& mx, uint32_t& qm) {
  const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)mn, 0x110 + SH, 0xf, 0xf, false);
  const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mx, 0x110 + SH, 0xf, 0xf, false);
  const uint32_t c = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)qm, 0x110 + SH, 0xf, 0xf, false);
  mn = mn < a ? mn : a;
  mx = mx > b ? mx : b;
  qm = qm > c ? qm : c;
}
__device__ __forceinline__ void cert_to_lds(uint32_t mn, uint32_t mx, uint32_t qm, uint32_t* s_cert) {
  cert_row_step<1>(mn, mx, qm);
  cert_row_step<2>(mn, mx, qm);
  cert_row_step<4>(mn, mx, qm);
  cert_row_step<8>(mn, mx, qm);  // lane 15 of each row: the row's min / max
  if ((threadIdx.x & 15) == 15) {
    atomicMin(&s_cert[0], mn);
    atomicMax(&s_cert[1], mx);
    atomicMax(&s_cert[2], qm);
  }
}

// The fast pass over one tile (sets sh.redo when the tile must be recomputed).
// (Round 5 tried an exact-value variant for coarse tables: values exact in
// both orders -- luma clipped beyond E or from an all-zero block, every chroma
// tap from an all-zero block -- taken out of the certificate.  It left 62 of
// 16320 tiles uncertain at 16 x 4K Q10 instead of 12449, but its bookkeeping
// made the kernel slower than k_inv2 there: 425 vs 358 us; DESIGN.md.)
template <int MODE, int XTRA>
__device__ __forceinline__ bool inv_fast_tile(InvShared<MODE, XTRA>& sh, const Geo& g, const int tiles_x,
                                              const int frame, const int tile, const int16_t* __restrict__ coeffs,
                                              const FrameQ* __restrict__ fq, const uint8_t* __restrict__ rgb_in,
                                              uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
                                              double* __restrict__ sse_y_part, unsigned* __restrict__ fixcount,
                                              unsigned* __restrict__ next_count, unsigned* __restrict__ cnt_now,
                                              const int in_div, const int fix_all) {
  using I = Inv<MODE>;
  constexpr int USH_ = USH<I::SY, I::SX>;  // chroma8_fast's scale
  double* s_mid = sh.mid;
  double (*s_cw)[I::CWR * I::CWS] = sh.cw;
  __shared__ __attribute__((aligned(16))) double s_qs[QS_WORDS];  // Q[u][v] * a_u * a_v / 8 at qs_index(u, v)
  __shared__ double s_qmax;
  __shared__ double s_red[I::NT / 64], s_dq[I::NT / 64];
  __shared__ uint32_t s_lmin[I::NT / 64], s_lmax[I::NT / 64];
  __shared__ uint32_t s_cert[3];  // min / max fraction word, max |q|
  __shared__ double s_dummy[64];  // the window stores' sink for ring columns outside it
  __shared__ unsigned long long s_sse;
  const int tid = threadIdx.x, lv = tid & 7, lb = tid >> 3;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  // the tile's first coefficient loads are issued before the table set-up and
  // its barrier, so their latency overlaps it
  int qhi = 0, qlo = 0;  // max / min q this lane read (max |q| = max(qhi, -qlo))

  // ---- 1. chroma window: (clip(IDCT) - 128) of the blocks the tile reaches --
  const int cby0 = Y0 / (8 * I::SY) - I::RY, cbx0 = X0 / (8 * I::SX) - I::RX;
  const int cwy0 = Y0 / I::SY - I::RY, cwx0 = X0 / I::SX - I::RX;
  auto luma_blk = [&](int r, int& by, int& bx) {
    const int blk = r * I::RB + lb;
    const int bi = blk / I::YBC, bj = blk - bi * I::YBC;
    by = Y0 / 8 + bi;
    bx = X0 / 8 + bj;
    return by < g.nby && bx < g.nbx;
  };
  auto table_setup = [&]() {
    if (tid < 64) {
      const double q = fq[frame].q[tid];
      s_qs[qs_index(tid >> 3, tid & 7)] = q * c_aan[tid >> 3] * c_aan[tid & 7] * 0.125;
      // max Q from the host's FrameQ::qmax (a scalar load at the end): no
      // cross-lane reduction before the barrier
      if (tid == 0) {
        s_cert[0] = 0xffffffffu;
        s_cert[1] = 0u;
        s_cert[2] = 0u;
      }
    }
    if (XTRA && tid == 0) s_sse = 0ull;
    __syncthreads();
  };
  Col16 lq;
  {
    int by, bx;
    const bool ok = luma_blk(0, by, bx);
    lq = load_col(cf, ((long long)by * g.nbx + bx) * 64, lv, ok);
  }
  // one chroma block task: column pass, and for the rows the tile needs the row
  // pass, clip and window stores (plane p, block row i of the window)
  auto chroma_task = [&](const int p, const int i, const int by, const int bx, const Col16& cur) {
    const bool need = !I::RY || (i == 0 ? lv == 7 : (i == I::CBR - 1 ? lv == 0 : true));
    fast_col(cur, s_qs, lv, s_mid + lb * MS, qhi, qlo);
    if (need) {
      double c[8];
      fast_row<-128>(s_mid + lb * MS, lv, c);
      double* w = &s_cw[p][(by * 8 + lv - cwy0) * I::CWS];
      const int wc0 = bx * 8 - cwx0;
      // the ring blocks' columns outside the window go to a per-lane dummy
      // slot: a select per store instead of a branch per store
#pragma unroll
      for (int k = 0; k < 8; ++k)
        *((unsigned)(wc0 + k) < (unsigned)I::CWC ? w + wc0 + k : s_dummy + (tid & 63)) = c[k];
      if constexpr (I::SX == 2) {
        // cv2's clamped taps at the image's left / right edge pixels read the
        // edge column alone: replicate it into the ring (and past the
        // plane's right end, where pixels beyond the image read too)
        if (bx == 0 && wc0 >= 1) w[wc0 - 1] = c[0];
        const int ke = g.wc - 1 - bx * 8;
        if ((unsigned)ke < 8u) {
          const double e = (ke == 0 ? c[0] : ke == 1 ? c[1] : ke == 2 ? c[2] : ke == 3 ? c[3]
                            : ke == 4 ? c[4] : ke == 5 ? c[5] : ke == 6 ? c[6] : c[7]);
          for (int col = wc0 + ke + 1; col < I::CWC; ++col) w[col] = e;
        }
      }
    }
  };
  // 4:2:2: the two planes' 2 x NCB block tasks dealt over
  // the workgroup's RB lane groups (one pass each, a second pass for the first
  // 2 NCB - RB groups) instead of NCB groups taking Cb then Cr while the other
  // waves wait at the barrier: the busiest SIMD runs 3 passes instead of 4
  constexpr bool MIXP = 1 && MODE == M422 && 2 * I::NCB > I::RB && 2 * I::NCB <= 2 * I::RB;
  if constexpr (MIXP) {
    constexpr int NTASK = 2 * I::NCB;
    auto tinfo = [&](int tt, int& pp, int& ii, int& by, int& bx, bool& ok) -> long long {
      pp = tt >= I::NCB ? 1 : 0;
      const int b = tt - pp * I::NCB;
      ii = b / I::CBC;
      const int jj = b - ii * I::CBC;
      by = cby0 + ii;
      bx = cbx0 + jj;
      ok = tt < NTASK && by >= 0 && bx >= 0 && by < g.ncy && bx < g.ncx;
      return ((long long)by * g.ncx + bx) * 64;
    };
    int pp, ii, by, bx;
    bool ok;
    long long off = tinfo(lb, pp, ii, by, bx, ok);
    Col16 cq = load_col(cf + (pp ? g.off_cr : g.off_cb), off, lv, ok);
    table_setup();
    if (tid == 0) s_qmax = fq[frame].qmax;  // (used by this thread after the next barrier)
#pragma unroll 1
    for (int tt = lb; tt < NTASK; tt += I::RB) {  // (uniform per wave: RB lane groups, 8 per wave)
      const Col16 cur = cq;
      const int pc = pp, ic = ii, byc = by, bxc = bx;
      const bool okc = ok;
      if (tt + I::RB < NTASK) {
        off = tinfo(tt + I::RB, pp, ii, by, bx, ok);
        cq = load_col(cf + (pp ? g.off_cr : g.off_cb), off, lv, ok);
      }
      if (okc) chroma_task(pc, ic, byc, bxc, cur);
    }
  } else {
    const bool ctask = tid < I::NCB * 8;
    const int ci = lb / I::CBC, cj = lb - ci * I::CBC;
    const int cby = cby0 + ci, cbx = cbx0 + cj;
    const bool cvalid = ctask && cby >= 0 && cbx >= 0 && cby < g.ncy && cbx < g.ncx;
    const long long cboff = ((long long)cby * g.ncx + cbx) * 64;
    Col16 cq = load_col(cf + g.off_cb, cboff, lv, cvalid);
    table_setup();
    if (tid == 0) s_qmax = fq[frame].qmax;  // (used by this thread after the next barrier)
    if (ctask) {
#pragma unroll 1
      for (int p = 0; p < 2; ++p) {
        const Col16 cur = cq;
        if (p == 0) cq = load_col(cf + g.off_cr, cboff, lv, cvalid);
        if (cvalid) chroma_task(p, ci, cby, cbx, cur);
      }
    }
  }
  __syncthreads();

  // ---- 2. luma rounds: IDCT, upsample, colour, certify, store ----------------
  // the certificate: smallest / largest fraction word of the lane's outputs
  uint32_t lo_min = 0xffffffffu, lo_max = 0u;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = XTRA ? rgb_in + (size_t)(frame / in_div) * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
#pragma unroll 1
  for (int r = 0; r < I::NYB / I::RB; ++r) {
    int by, bx;
    const bool bvalid = luma_blk(r, by, bx);
    // the luma SSE in the exact kernel's order: per-round sums, added per round
    unsigned long long r_sse = 0ull;
    double r_ssy = 0.0;
    const Col16 cur = lq;
    if (r + 1 < I::NYB / I::RB) {
      int by1, bx1;
      const bool ok1 = luma_blk(r + 1, by1, bx1);
      lq = load_col(cf, ((long long)by1 * g.nbx + bx1) * 64, lv, ok1);
    }
    if (bvalid) fast_col(cur, s_qs, lv, s_mid + lb * MS, qhi, qlo);
    const int y = by * 8 + lv, x0 = bx * 8;
    if (bvalid && y < g.H && x0 < g.W) {
      double Yv[8];
      fast_row<-128>(s_mid + lb * MS, lv, Yv);  // Y - 128
      int wq, wt = 0;
      if constexpr (I::SY == 2) {
        // output row 2m: rows (m-1, m) weighted (1/4, 3/4); row 2m+1: (m+1, m)
        const int m = y >> 1;
        const int rq = (y & 1) ? m + 1 : m - 1;
        wq = clampi(clampi(rq, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
        wt = clampi(clampi(m, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
      } else {
        wq = y - cwy0;
      }
      const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
      uint8_t* o = out_f + ((size_t)y * g.W + x0) * 3;
      const bool wide = nx == 8 && ((((uintptr_t)o) & 7u) == 0);
      // SSE runs: the input row requested before the colour work, so its latency
      // hides under it (sweep step 3.758 -> 3.731 ms, tools/r6_ww.sh)
      uint32_t in[6] = {0u, 0u, 0u, 0u, 0u, 0u};
      if constexpr (XTRA > 0) {
        const uint8_t* src = in_f + ((size_t)y * g.W + x0) * 3;
        if (wide) {
          const uint2* s2 = reinterpret_cast<const uint2*>(src);
          const uint2 a = s2[0], b2 = s2[1], c = s2[2];
          in[0] = a.x; in[1] = a.y; in[2] = b2.x; in[3] = b2.y; in[4] = c.x; in[5] = c.y;
        } else {
#pragma unroll
          for (int k = 0; k < 24; ++k)
            if (k < 3 * nx) in[k >> 2] |= (uint32_t)src[k] << (8 * (k & 3));
        }
      }
      uint32_t pk[6];
      // the row's smallest / largest fraction word
      uint32_t r_min = 0xffffffffu, r_max = 0u;
      {
        // channel high words (byte: clamp(low 16 bits)) in output order R0 G0 B0 R1 ...
        uint32_t cb[24];
        double C[8], Gt[8];
        chroma8_fast<MODE>(s_cw[0], x0, cwx0, wq, wt, C);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          Yv[k] = Yv[k] + (MAGIC + 128.0);  // Y on byte_cert_y's grid, shared by the three channels
          const double B = col_b<MadDev, USH_>(Yv[k], C[k]);
          Gt[k] = col_gt<MadDev, USH_>(Yv[k], C[k]);
          cb[3 * k + 2] = cert_hi(B, r_min, r_max);
        }
        chroma8_fast<MODE>(s_cw[1], x0, cwx0, wq, wt, C);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double R = col_r<MadDev, USH_>(Yv[k], C[k]);
          const double G = col_g<MadDev, USH_>(Gt[k], C[k]);
          cb[3 * k] = cert_hi(R, r_min, r_max);
          cb[3 * k + 1] = cert_hi(G, r_min, r_max);
        }
#pragma unroll
        for (int w = 0; w < 6; ++w) pk[w] = pack4s(cb[4 * w], cb[4 * w + 1], cb[4 * w + 2], cb[4 * w + 3]);
      }
      lo_min = lo_min < r_min ? lo_min : r_min;
      lo_max = lo_max > r_max ? lo_max : r_max;
      if (wide) {
        uint2* o2 = reinterpret_cast<uint2*>(o);
        o2[0] = make_uint2(pk[0], pk[1]);
        o2[1] = make_uint2(pk[2], pk[3]);
        o2[2] = make_uint2(pk[4], pk[5]);
      } else {
#pragma unroll
        for (int b = 0; b < 24; ++b)
          if (b < 3 * nx) o[b] = (uint8_t)(pk[b >> 2] >> (8 * (b & 3)));
      }
      if constexpr (XTRA > 0) {
        // reference PSNR inputs (utils/metrics.py:11-20): exact integer SSE and
        // the luma SSE as one exact integer per pixel (luma_sse_e6)
        auto byte_of = [](const uint32_t (&w)[6], int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 255u); };
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < nx) {
            const int b = 3 * k;
            const int o0 = byte_of(in, b), o1 = byte_of(in, b + 1), o2 = byte_of(in, b + 2);
            const int ur = byte_of(pk, b), ug = byte_of(pk, b + 1), ub = byte_of(pk, b + 2);
            const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
            r_sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
            r_ssy = r_ssy + luma_sse_e6(d0, d1, d2);
          }
        }
      }
    }
    if constexpr (XTRA > 0) {
      sse += r_sse;
      ssy = ssy + r_ssy;
    }
  }

  // ---- 3. certification: the tile's closest approach to an integer vs its bound
  int qm = max(qhi, -qlo);  // max |q| this lane read
  cert_to_lds(lo_min, lo_max, (uint32_t)qm, s_cert);
  if constexpr (XTRA > 0) {
    unsigned long long s = sse;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) atomicAdd(&s_sse, s);
    double d = ssy;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = d + __shfl_xor(d, o, 64);  // (no products: nothing to fuse)
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t mn = s_cert[0], mx = s_cert[1];
    const double q = (double)s_cert[2];
    // |v_fast - v_ref| <= E, plus <= 3 roundings on the magic grid (2^-33 each:
    // byte_cert); T in units of 2^-32
    const double E = K_LIN * (q * s_qmax) + K_CONST + 0x1p-31;
    const double T = ceil(E * 0x1p+32) + 1.0;
    const bool uncertain = (double)mn <= T || (double)mx >= 0x1p+32 - 1.0 - T;
    sh.redo = uncertain || fix_all;
    if (sh.redo) {
      atomicAdd(fixcount, 1u);  // tiles recomputed (jds_plan_fix_counts)
      atomicAdd(cnt_now + frame, 1u);
    } else if constexpr (XTRA > 0) {
      double a = 0.0;
      for (int i = 0; i < I::NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * gridDim.x + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, s_sse);
    }
    if (frame == 0 && tile == 0) *next_count = 0u;  // the next run counts from zero
  }
  __syncthreads();  // sh.redo is visible to the caller's uniform branch
  return sh.redo != 0;
}

// XTRA: 0 = RGB only; 1 = + exact integer SSE and luma SSE partials (sweeps),
// committed by the fast pass only for certified tiles (the exact tile code
// commits the others).
template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv<MODE>::NT) __attribute__((amdgpu_waves_per_eu(Inv<MODE>::WPE)))
k_inv_fast(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
           const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
           double* __restrict__ sse_y_part, unsigned* __restrict__ fixcount, unsigned* __restrict__ next_count,
           unsigned* __restrict__ item_cnt, const int rot, const int probe, const int in_div, const int fix_all,
           const int fin) {
  // the transpose buffer and chroma window are the exact fallback's own
  __shared__ __attribute__((aligned(16))) InvShared<MODE, XTRA> sh;
#ifdef JDS_PROBE_LDS_PAD  // tools: extra LDS per workgroup (occupancy probe)
  __shared__ unsigned s_pad[JDS_PROBE_LDS_PAD];
  if (threadIdx.x == 0) s_pad[blockIdx.x % JDS_PROBE_LDS_PAD] = 0u;
#endif
  const int tid = threadIdx.x;
  const int frame = blockIdx.y, tile = blockIdx.x;
  // k_finalize's work for runs without SSE terms (fin >= 0; fin = 1 adds the
  // zero bin the forward deferred): one launch fewer per run
  if (fin >= 0 && tile == 0 && tid == 0) finalize_frame(g, st + frame, fin);
  // per-item adaptivity (InvFix): the previous run's recomputed tiles of this item
  const unsigned n_items = gridDim.y, ntile = gridDim.x;
  unsigned* cnt_prev = item_cnt + ((rot + 2) % 3) * n_items;
  unsigned* cnt_now = item_cnt + rot * n_items;
  const unsigned prev = cnt_prev[frame];
  if (tile == 0 && tid == 0) item_cnt[((rot + 1) % 3) * n_items + frame] = 0u;  // the next run's
  const bool item_exact = !probe && !fix_all && prev * 8u > ntile;
  bool redo = false;
  if (item_exact) {
    // (uniform) this item runs the exact tile code directly and keeps its count
    if (tile == 0 && tid == 0) {
      cnt_now[frame] = prev;
      atomicAdd(fixcount, ntile);
      if (frame == 0) *next_count = 0u;
    }
  } else {
    sh.redo = 0;
    redo = inv_fast_tile<MODE, XTRA>(sh, g, tiles_x, frame, tile, coeffs, fq, rgb_in, rgb_out, st, sse_y_part,
                                         fixcount, next_count, cnt_now, in_div, fix_all);
  }
  // one call site of the exact tile code: items in exact mode, uncertain tiles
#ifndef JDS_PROBE_NOFALLBACK  // tools/stage_budget.py: the fast path's code alone
  if (item_exact || redo)  // (uniform)
    inv2_tile<MODE, XTRA>(sh, g, tiles_x, ntile, frame, tile, coeffs, fq, rgb_in, rgb_out, st, sse_y_part, nullptr,
                          nullptr, in_div);
#endif
}

#ifdef JDS_INV6  // the transpose-free variant, built for A/B only (tools/build_variant.py -DJDS_INV6; tests/test_variants_cpu.py compiles it)
// ------------------------------------- 4:2:0 without a transpose buffer --
//
// k_inv_fast6 (round 6): k_inv_fast<4:2:0, 0>'s tile (64 x 128 px, 512
// threads), operations and certificate, without the 37 KB transpose buffer
// that held k_inv_fast to two workgroups (four waves) per SIMD-quad: 45 KB of
// LDS, so three workgroups fit a CU when the registers allow it (<= 80).
//  * chroma: each block's column pass writes its outputs into the chroma
//    window at the block's own place (W6: the window widened to whole ring
//    blocks) and its row pass reads the row back, transforms, clips and
//    overwrites it -- the window is the transpose medium (the 8 lanes of a
//    block are one wave's, whose LDS operations keep their order: no barrier);
//  * luma: the column-to-row transpose in registers (xpose8), lanes b + 8 k of
//    a wave holding block b's column / row k.
// Every value goes through k_inv_fast's operations in k_inv_fast's order
// (aan8 on the folded table, the clips, the unnormalised upsample, the colour
// terms on the magic grid), so tools/inv_bound.py's bound and the certificate
// carry over unchanged; only the data movement differs.  An uncertain tile
// (and every tile of an item in exact mode) is appended to a list that
// k_inv6_fix recomputes right after with inv2_tile (the reference's order).
// a volatile 2-double LDS access: emitted as exactly one ds_read_b128 /
// ds_write_b128 (plain ones get narrowed to the used halves and re-paired as
// 8-cycle ds_read2_b64; MI355X_MICROARCH.md §LDS)
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) volatile dv2 lds_dv2;

__device__ __forceinline__ void chroma8_fast_w6(const double* __restrict__ cw, int c0, int wq, int wt,
                                                double (&C)[8]) {
  double vb[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) vb[j] = fvsum(cw[wq * W6::CWS + c0 + j], cw[wt * W6::CWS + c0 + j]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    C[2 * i] = fhsum(vb[i], vb[i + 1]);          // (1/4, 3/4) on (m-1, m)
    C[2 * i + 1] = fhsum(vb[i + 2], vb[i + 1]);  // (3/4, 1/4) on (m, m+1)
  }
}

// the folded table's column k (fast_col's four ds_read_b128) times the
// column's coefficients; qhi / qlo track the coefficient range when `track`
// (the column's LDS offset is laundered per call: otherwise the compiler keeps
// the loop-invariant table column live across the luma rounds, 16 VGPRs)
__device__ __forceinline__ void deq_col(const Col16p& in, const double* __restrict__ qs, int k, bool track,
                                        double (&c)[8], int& qhi, int& qlo) {
  double t[8];
  int off = k * QS_STRIDE;
  asm volatile("" : "+v"(off));
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double2 d = *reinterpret_cast<const double2*>(qs + off + 2 * p);
    t[2 * p] = d.x;
    t[2 * p + 1] = d.y;
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int q = in.q(r);
    qhi = track ? max(qhi, q) : qhi;
    qlo = track ? min(qlo, q) : qlo;
    c[r] = (double)q * t[r];
  }
}

#ifndef JDS_K6_WPE
#define JDS_K6_WPE 6
#endif
__global__ void __launch_bounds__(W6::NT) __attribute__((amdgpu_waves_per_eu(JDS_K6_WPE)))
k_inv_fast6(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
            uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st, unsigned* __restrict__ fixcount,
            unsigned* __restrict__ next_count, unsigned* __restrict__ item_cnt, uint2* __restrict__ fixlist,
            const int rot, const int probe, const int fix_all, const int fin) {
  __shared__ __attribute__((aligned(16))) double s_cw[2][W6::CWR * W6::CWS];
  __shared__ __attribute__((aligned(16))) double s_qs[QS_WORDS];  // Q[u][v] * a_u * a_v / 8 at qs_index(u, v)
  __shared__ uint32_t s_cert[3];                                   // min / max fraction word, max |q|
  __shared__ double s_qmax;
  const int tid = threadIdx.x;
  const int frame = blockIdx.y, tile = blockIdx.x;
  if (fin >= 0 && tile == 0 && tid == 0) finalize_frame(g, st + frame, fin);
  // per-item adaptivity (InvFix), as k_inv_fast
  const unsigned n_items = gridDim.y, ntile = gridDim.x;
  unsigned* cnt_prev = item_cnt + ((rot + 2) % 3) * n_items;
  unsigned* cnt_now = item_cnt + rot * n_items;
  const unsigned prev = cnt_prev[frame];
  if (tid == 0) {
    if (tile == 0) item_cnt[((rot + 1) % 3) * n_items + frame] = 0u;  // the next run's
    if (frame == 0 && tile == 0) *next_count = 0u;                     // the next run counts from zero
  }
#ifndef JDS_K6_PROBE
#define JDS_K6_PROBE 0  // tools: timing probes (wrong values): 1 no luma transpose, 2 no chroma row pass, 4 no chroma column writes
#endif
  const bool item_exact = !JDS_K6_PROBE && !probe && !fix_all && prev * 8u > ntile;
  if (item_exact) {  // (uniform) every tile of the item to the exact kernel; the item keeps its count
    if (tid == 0) {
      if (tile == 0) cnt_now[frame] = prev;
      fixlist[atomicAdd(fixcount, 1u)] = make_uint2((unsigned)frame, (unsigned)tile);
    }
    return;
  }

  // lane (block slot lb, in-block index k): the 8 lanes of a block are b, b + 8, .. of one wave
  const int k = (tid >> 3) & 7, lb = ((tid >> 6) << 3) | (tid & 7);
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * W6::TH, X0 = tx * W6::TW;
  // the frame's coefficients and output through buffer resources (uniform
  // bases in SGPRs, 32-bit lane offsets: fewer VGPRs than 64-bit addresses)
  const __amdgpu_buffer_rsrc_t cf = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(coeffs + (size_t)frame * g.cpf), 0, (int)(g.cpf * 2), 0x00020000);
  const int cwy0 = Y0 / 2 - 1;
  auto luma_blk = [&](int r, int& by, int& bx) {
    const int blk = r * W6::RB + lb;
    by = Y0 / 8 + (blk >> 4);
    bx = X0 / 8 + (blk & 15);
    return by < g.nby && bx < g.nbx;
  };
  auto luma_off = [&](int r, bool& ok) {
    const int blk = r * W6::RB + lb;
    const int by = Y0 / 8 + (blk >> 4), bx = X0 / 8 + (blk & 15);
    ok = by < g.nby && bx < g.nbx;
    return ((long long)by * g.nbx + bx) * 64;
  };
  int qhi = 0, qlo = 0;  // max / min q this lane read
  // the first coefficient rows (luma round 0, this lane group's Cb block) before the table set-up
  uint4 lq;
  {
    bool ok;
    const long long off = luma_off(0, ok);
    lq = load_rowq_b(cf, off, k, ok);
  }
  const int ci = lb / W6::CBC, cj = lb - ci * W6::CBC;
  const int cby = Y0 / 16 - 1 + ci, cbx = X0 / 16 - 1 + cj;
  const bool cvalid = lb < W6::NCB && cby >= 0 && cbx >= 0 && cby < g.ncy && cbx < g.ncx;
  const long long cboff = ((long long)cby * g.ncx + cbx) * 64;
  uint4 cq = load_rowq_b(cf, g.off_cb + cboff, k, cvalid);
  if (tid < 64) {
    const double q = fq[frame].q[tid];
    s_qs[qs_index(tid >> 3, tid & 7)] = q * c_aan[tid >> 3] * c_aan[tid & 7] * 0.125;
    if (tid == 0) {
      s_cert[0] = 0xffffffffu;
      s_cert[1] = 0u;
      s_cert[2] = 0u;
      s_qmax = fq[frame].qmax;
    }
  }
  __syncthreads();

  // ---- 1. chroma window: column pass into the block's place, row pass in place
  const int r0 = 8 * ci - 7, c0 = 8 * cj;  // the block's first window row / column
#pragma unroll 1
  for (int p = 0; p < 2; ++p) {
    const Col16p cur = xpose_q16(cq);  // (uniform: the whole wave)
    if (p == 0) cq = load_rowq_b(cf, g.off_cr + cboff, k, cvalid);
    if (cvalid) {
      double* w = s_cw[p];
      double c[8];
      deq_col(cur, s_qs, k, true, c, qhi, qlo);
      aan8(c);
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (!(JDS_K6_PROBE & 4) && (unsigned)(r0 + r) < (unsigned)W6::CWR) w[(r0 + r) * W6::CWS + c0 + k] = c[r];
      __builtin_amdgcn_wave_barrier();  // the block's other lanes' columns (a wave's LDS operations keep their order)
      const int wr = r0 + k;
      if (!(JDS_K6_PROBE & 2) && (unsigned)wr < (unsigned)W6::CWR) {  // the rows the window holds (a ring block: one)
        double* row = w + wr * W6::CWS + c0;  // (16-B aligned: four b128 each way)
        lds_dv2* row2 = (lds_dv2*)row;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const dv2 d = row2[j];
          c[2 * j] = d.x;
          c[2 * j + 1] = d.y;
        }
        aan8(c);
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = fmin(fmax(c[j], -128.0), 127.0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dv2 d;
          d.x = c[2 * j];
          d.y = c[2 * j + 1];
          row2[j] = d;
        }
        // cv2's clamped taps at the image's left / right edge pixels read the
        // edge column alone: replicated into the ring (and past the plane's end)
        if (cbx == 0) row[-1] = c[0];
        const int ke = g.wc - 1 - cbx * 8;
        if ((unsigned)ke < 8u) {
          const double e = (ke == 0 ? c[0] : ke == 1 ? c[1] : ke == 2 ? c[2] : ke == 3 ? c[3]
                            : ke == 4 ? c[4] : ke == 5 ? c[5] : ke == 6 ? c[6] : c[7]);
          for (int col = c0 + ke + 1; col < W6::CWC; ++col) w[wr * W6::CWS + col] = e;
        }
      }
    }
  }
  __syncthreads();

  // ---- 2. luma rounds: IDCT (transpose in registers), upsample, colour, certify, store
  uint32_t lo_min = 0xffffffffu, lo_max = 0u;
  const __amdgpu_buffer_rsrc_t out_f = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(rgb_out + (size_t)frame * g.H * g.W * 3), 0, g.H * g.W * 3, 0x00020000);
#pragma unroll 1
  for (int r = 0; r < W6::NYB / W6::RB; ++r) {
    int by, bx;
    const bool bvalid = luma_blk(r, by, bx);
#ifdef JDS_K6_NOPREFETCH
    if (r > 0) {
      bool ok;
      const long long off = luma_off(r, ok);
      lq = load_rowq_b(cf, off, k, ok);
    }
    const Col16p cur = xpose_q16(lq);
#else
    const Col16p cur = xpose_q16(lq);
    if (r + 1 < W6::NYB / W6::RB) {
      bool ok1;
      const long long off1 = luma_off(r + 1, ok1);
      lq = load_rowq_b(cf, off1, k, ok1);
    }
#endif
    // every lane transforms (xpose8 needs the whole wave); blocks outside the
    // grid neither count towards Dmax nor store
    double Yv[8];
    deq_col(cur, s_qs, k, bvalid, Yv, qhi, qlo);
    aan8(Yv);
    if (!(JDS_K6_PROBE & 1)) xpose8(Yv);
    aan8(Yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) Yv[j] = fmin(fmax(Yv[j], -128.0), 127.0);  // Y - 128
    const int y = by * 8 + k, x0 = bx * 8;
    if (bvalid && y < g.H && x0 < g.W) {
      // output row 2m: chroma rows (m-1, m) weighted (1/4, 3/4); row 2m+1: (m+1, m)
      const int m = y >> 1;
      const int rq = (y & 1) ? m + 1 : m - 1;
      const int wq = clampi(clampi(rq, 0, g.hc - 1) - cwy0, 0, W6::CWR - 1);
      const int wt = clampi(clampi(m, 0, g.hc - 1) - cwy0, 0, W6::CWR - 1);
      const int cc0 = (x0 - X0) / 2 + 7;  // window column of chroma column x0/2 - 1
      const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
      const int o = (y * g.W + x0) * 3;  // byte offset in the frame (8-B aligned when nx == 8)
      uint32_t pk[6];
      uint32_t r_min = 0xffffffffu, r_max = 0u;
      // four pixels at a time, both planes per pixel (register economy: the
      // vertical sums of the 4 chroma columns a half reads, 12 channel words
      // before packing); chroma8_fast's operations, column by column
      // (the six samples from cc0 = 4 bj + 7 as halves of the aligned pairs from cc0 - 1)
      // (volatile: exactly these b128 accesses -- the compiler otherwise narrows
      // them to the used halves and re-pairs those as 8-cycle ds_read2_b64)
      const lds_dv2* q0 = (const lds_dv2*)(s_cw[0] + wq * W6::CWS + cc0 - 1);
      const lds_dv2* t0 = (const lds_dv2*)(s_cw[0] + wt * W6::CWS + cc0 - 1);
      const lds_dv2* q1 = (const lds_dv2*)(s_cw[1] + wq * W6::CWS + cc0 - 1);
      const lds_dv2* t1 = (const lds_dv2*)(s_cw[1] + wt * W6::CWS + cc0 - 1);
      double vB[6], vR[6];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // pairs 0..2 (samples cc0 - 1 .. cc0 + 4) for the first half, pair 3 (cc0 + 5, + 6) for the second
#pragma unroll
        for (int pr = (h ? 3 : 0); pr < (h ? 4 : 3); ++pr) {
          const dv2 a = q0[pr], b = t0[pr], c = q1[pr], d = t1[pr];  // (volatile LDS reads)
          if (pr > 0) {
            vB[2 * pr - 1] = fvsum(a.x, b.x);
            vR[2 * pr - 1] = fvsum(c.x, d.x);
          }
          if (pr < 3) {
            vB[2 * pr] = fvsum(a.y, b.y);
            vR[2 * pr] = fvsum(c.y, d.y);
          }
        }
        uint32_t ch[12];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int px = 4 * h + e, i = px >> 1;
          const double Cb = (px & 1) ? fhsum(vB[i + 2], vB[i + 1]) : fhsum(vB[i], vB[i + 1]);
          const double Cr = (px & 1) ? fhsum(vR[i + 2], vR[i + 1]) : fhsum(vR[i], vR[i + 1]);
          const double Y = Yv[px] + (MAGIC + 128.0);  // Y on byte_cert_y's grid, shared by the three channels
          const double B = col_b<MadDev, 4>(Y, Cb);
          const double Gt = col_gt<MadDev, 4>(Y, Cb);
          const double R = col_r<MadDev, 4>(Y, Cr);
          const double G = col_g<MadDev, 4>(Gt, Cr);
          ch[3 * e] = cert_hi(R, r_min, r_max);
          ch[3 * e + 1] = cert_hi(G, r_min, r_max);
          ch[3 * e + 2] = cert_hi(B, r_min, r_max);
        }
#pragma unroll
        for (int w = 0; w < 3; ++w) pk[3 * h + w] = pack4s(ch[4 * w], ch[4 * w + 1], ch[4 * w + 2], ch[4 * w + 3]);
      }
      lo_min = lo_min < r_min ? lo_min : r_min;
      lo_max = lo_max > r_max ? lo_max : r_max;
      if (nx == 8) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          u2 v;
          v.x = pk[2 * w];
          v.y = pk[2 * w + 1];
          __builtin_amdgcn_raw_buffer_store_b64(v, out_f, o + 8 * w, 0, 0);
        }
      } else {
#pragma unroll
        for (int bb = 0; bb < 24; ++bb)
          if (bb < 3 * nx) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(pk[bb >> 2] >> (8 * (bb & 3))), out_f, o + bb, 0, 0);
      }
    }
  }

  // ---- 3. certification (k_inv_fast's); an uncertain tile goes to the exact kernel's list
  cert_to_lds(lo_min, lo_max, (uint32_t)max(qhi, -qlo), s_cert);
  __syncthreads();
  if (tid == 0) {
    const uint32_t mn = s_cert[0], mx = s_cert[1];
    const double q = (double)s_cert[2];
    const double E = K_LIN * (q * s_qmax) + K_CONST + 0x1p-31;
    const double T = ceil(E * 0x1p+32) + 1.0;
    const bool uncertain = (double)mn <= T || (double)mx >= 0x1p+32 - 1.0 - T;
    if (uncertain || fix_all) {
      fixlist[atomicAdd(fixcount, 1u)] = make_uint2((unsigned)frame, (unsigned)tile);  // (jds_plan_fix_counts)
      atomicAdd(cnt_now + frame, 1u);
    }
  }
}

// The exact recomputation of the tiles k_inv_fast6 listed (inv2_tile: the
// reference's operation order, k_inv2's layout), right after it on the same
// stream: a few hundred workgroups walk the list (typically a handful of tiles
// per 64 x 1080p run; every tile of an item in exact mode, all of them under
// JDS_RUN_INV_FIXALL).  Separate from k_inv_fast6 so that the fallback's
// registers and LDS do not hold the fast kernel's occupancy down.
__global__ void __launch_bounds__(Inv<M420>::NT) __attribute__((amdgpu_waves_per_eu(Inv<M420>::WPE)))
k_inv6_fix(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
           uint8_t* __restrict__ rgb_out, const unsigned* __restrict__ fixcount, const uint2* __restrict__ fixlist) {
  __shared__ __attribute__((aligned(16))) InvShared<M420, 0> sh;
  const unsigned n = *fixcount;
  for (unsigned i = blockIdx.x; i < n; i += gridDim.x) {  // (uniform)
    const uint2 e = fixlist[i];
    inv2_tile<M420, 0>(sh, g, tiles_x, 0, (int)e.x, (int)e.y, coeffs, fq, nullptr, rgb_out, nullptr, nullptr,
                       nullptr, nullptr, 1);
    __syncthreads();  // the next tile reuses the shared arrays
  }
}
#endif  // JDS_INV6

// ------------------------------------------------- 4:4:4, wave-local --
//
// k_inv_fast444: without chroma subsampling every output sample reads only the
// co-located block of each plane, so the inverse needs no chroma window, no
// ring and no workgroup barrier: a wave owns 8 blocks (raster order over the
// block grid), a block's 8 lanes run the column pass (lane = column), the
// wave-local transpose and the row pass (lane = row) for Y, Cb and Cr in turn,
// and each lane converts, certifies and stores its 8-pixel row.  The
// certificate is k_inv_fast's (E = K_LIN * Dmax + K_CONST + 2^-31), with Dmax
// over the block's own three planes; a wave with any uncertain value redoes
// its 8 blocks in the exact replayed order (idct_col / idct_row /
// colour8_exact, jds_inv_exact.hpp) and overwrites their rows.  (k_inv_fast's
// tiled 4:4:4 form measured slower than k_inv2: 383 vs 332 us per 256 x 512^2,
// its per-tile fixed costs spread over 2048 pixels.)
constexpr int I444_WAVES = 4;

__global__ void __launch_bounds__(64 * I444_WAVES)
k_inv_fast444(const Geo g, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
              uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st, unsigned* __restrict__ fixcount,
              unsigned* __restrict__ next_count, unsigned* __restrict__ item_cnt, const int rot, const int fix_all,
              const int fin) {
  __shared__ __attribute__((aligned(16))) double s_mid[8 * I444_WAVES * MS];
  __shared__ __attribute__((aligned(16))) double s_qs[QS_WORDS];
  __shared__ int s_qi[64];
  __shared__ double s_qmax;
  const int tid = threadIdx.x, lv = tid & 7, lb = tid >> 3;
  const int frame = blockIdx.y;
  if (fin >= 0 && blockIdx.x == 0 && tid == 0) finalize_frame(g, st + frame, fin);
  const unsigned n_items = gridDim.y;
  unsigned* cnt_now = item_cnt + rot * n_items;
  if (blockIdx.x == 0 && tid == 0) {
    item_cnt[((rot + 1) % 3) * n_items + frame] = 0u;  // the next run's
    if (frame == 0) *next_count = 0u;                  // the next run counts from zero
  }
  const long long nblk = (long long)g.nby * g.nbx;
  const long long blk = (long long)blockIdx.x * (8 * I444_WAVES) + lb;
  const bool bvalid = blk < nblk;
  const long long bq = bvalid ? blk : 0;
  const int by = (int)(bq / g.nbx), bx = (int)(bq - (long long)by * g.nbx);
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  double* slot = s_mid + lb * MS;
  // the coefficient loads are issued before the table set-up and its barrier
  const Col16 qy = load_col(cf, bq * 64, lv, bvalid);
  const Col16 qb = load_col(cf + g.off_cb, bq * 64, lv, bvalid);
  const Col16 qr = load_col(cf + g.off_cr, bq * 64, lv, bvalid);
  if (tid < 64) {
    const double q = fq[frame].q[tid];
    s_qs[qs_index(tid >> 3, tid & 7)] = q * c_aan[tid >> 3] * c_aan[tid & 7] * 0.125;
    s_qi[tid] = (int)q;
  }
  __syncthreads();
  const double qmax = fq[frame].qmax;
  const int y = by * 8 + lv, x0 = bx * 8;
  const bool row_ok = bvalid && y < g.H;
  const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
  uint8_t* o = rgb_out + (size_t)frame * g.H * g.W * 3 + ((size_t)y * g.W + x0) * 3;
  const bool wide = nx == 8 && ((((uintptr_t)o) & 7u) == 0);
  auto store = [&](const uint32_t (&pk)[6]) {
    if (!row_ok) return;
    if (wide) {
      uint2* o2 = reinterpret_cast<uint2*>(o);
      o2[0] = make_uint2(pk[0], pk[1]);
      o2[1] = make_uint2(pk[2], pk[3]);
      o2[2] = make_uint2(pk[4], pk[5]);
    } else {
#pragma unroll
      for (int b = 0; b < 24; ++b)
        if (b < 3 * nx) o[b] = (uint8_t)(pk[b >> 2] >> (8 * (b & 3)));
    }
  };

  // ---- the certified fast pass ---------------------------------------------
  int qhi = 0, qlo = 0;
  uint32_t lo_min = 0xffffffffu, lo_max = 0u;
  {
    // chroma planes first, luma last, then the colour terms pixel by pixel
    // (bytes packed as they come: fewer live registers than plane by plane)
    double Cb[8], Cr[8], Yv[8];
    fast_col(qb, s_qs, lv, slot, qhi, qlo);
    __builtin_amdgcn_wave_barrier();
    fast_row<-128>(slot, lv, Cb);  // Cb - 128
    __builtin_amdgcn_wave_barrier();
    fast_col(qr, s_qs, lv, slot, qhi, qlo);
    __builtin_amdgcn_wave_barrier();
    fast_row<-128>(slot, lv, Cr);  // Cr - 128
    __builtin_amdgcn_wave_barrier();
    fast_col(qy, s_qs, lv, slot, qhi, qlo);
    __builtin_amdgcn_wave_barrier();
    fast_row<-128>(slot, lv, Yv);  // Y - 128
    uint32_t cb[24];  // channel high words (byte: clamp(low 16 bits)), output order R0 G0 B0 R1 ...
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double y = Yv[k] + (MAGIC + 128.0);
      cb[3 * k] = cert_hi(col_r(y, Cr[k]), lo_min, lo_max);
      cb[3 * k + 1] = cert_hi(col_g(col_gt(y, Cb[k]), Cr[k]), lo_min, lo_max);
      cb[3 * k + 2] = cert_hi(col_b(y, Cb[k]), lo_min, lo_max);
    }
    uint32_t pk[6];
#pragma unroll
    for (int w = 0; w < 6; ++w) pk[w] = pack4s(cb[4 * w], cb[4 * w + 1], cb[4 * w + 2], cb[4 * w + 3]);
    store(pk);
  }
  // the block's Dmax over its three planes (its 8 lanes), then this lane's margin
  int qm = max(qhi, -qlo);
  // over the block's 8 lanes by DPP: quad_perm xor 1, xor 2, then row_half_mirror
  // (lane i of 8 with lane 7 - i, in the other quad)
  qm = max(qm, __builtin_amdgcn_update_dpp(0, qm, 0xb1, 0xf, 0xf, true));
  qm = max(qm, __builtin_amdgcn_update_dpp(0, qm, 0x4e, 0xf, 0xf, true));
  qm = max(qm, __builtin_amdgcn_update_dpp(0, qm, 0x141, 0xf, 0xf, true));
  const double E = K_LIN * ((double)qm * qmax) + K_CONST + 0x1p-31;
  const double T = ceil(E * 0x1p+32) + 1.0;
  const bool unc = row_ok && ((double)lo_min <= T || (double)lo_max >= 0x1p+32 - 1.0 - T);
#ifndef JDS_PROBE_NOFALLBACK
  if (__ballot(unc || fix_all) == 0ull) return;  // (uniform) the wave's rows are certified

  // ---- exact fallback: the wave's 8 blocks in the reference's order ---------
  if ((tid & 63) == 0) {
    atomicAdd(fixcount, 1u);  // waves recomputed (jds_plan_fix_counts)
    atomicAdd(cnt_now + frame, 1u);
  }
  __builtin_amdgcn_wave_barrier();
  {
    // (the coefficients reloaded: keeping them live through the fast pass costs
    // the common case registers; the empty asm hides the pointer's identity so
    // the compiler cannot forward the first loads' values)
    const int16_t* cf2 = cf;
    asm volatile("" : "+v"(cf2));
    double Yv[8], C[8], Gt[8];
    uint32_t pk[6];
    idct_col(load_col(cf2, bq * 64, lv, bvalid), s_qi, lv, slot);
    __builtin_amdgcn_wave_barrier();
    idct_row(slot, lv, Yv);
    __builtin_amdgcn_wave_barrier();
    idct_col(load_col(cf2 + g.off_cb, bq * 64, lv, bvalid), s_qi, lv, slot);
    __builtin_amdgcn_wave_barrier();
    idct_row(slot, lv, C);
    __builtin_amdgcn_wave_barrier();
    colour8_exact_cb(Yv, C, Gt, pk);
    idct_col(load_col(cf2 + g.off_cr, bq * 64, lv, bvalid), s_qi, lv, slot);
    __builtin_amdgcn_wave_barrier();
    idct_row(slot, lv, C);
    colour8_exact_cr(Yv, Gt, C, pk);
    store(pk);
  }
#else
  (void)unc;
  (void)cnt_now;
  (void)fixcount;
#endif
}

// ------------------------------------------------ 16 x 16 blocks (4:2:x) --
//
// fidct16: the orthonormal 16-point IDCT on scaled inputs.  Even outputs of
// the split x_n = E_n + O_n, x_{15-n} = E_n - O_n (n < 8): E is the 8-point
// IDCT of the even coefficients / sqrt(2), i.e. aan8 on inputs pre-scaled by
// a_m / 4 (folded into the dequantisation table with the other axis's
// scale); O_n = sqrt(2)/4 sum_m Z_m cos((2n+1)(2m+1) pi / 32) of the odd
// coefficients Z_m comes from Lee's identity 2 cos(t) cos((2m+1) t) =
// cos(2(m+1) t) + cos(2m t): 2 cos(t_n) sum_m Z_m cos((2m+1) t_n) is the
// unnormalised 8-point DCT-III of W_0 = Z_0, W_j = Z_{j-1} + Z_j, i.e. aan8 on
// W_j cos(j pi / 16) (W_0 unscaled), then scaled by
// p_n = sqrt(2) / (8 cos((2n+1) pi / 32)).  92 operations per line against
// dct3_line16's 144 (tools/inv_bound.py fast16_line models this sequence and
// checks the linear forms against the orthonormal IDCT).
template <class M = MadDev>
__host__ __device__ __forceinline__ void fidct16(double (&c)[16]) {
  double e[8], w[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) e[m] = c[2 * m];
  aan8<M>(e);
  w[0] = c[1];
#pragma unroll
  for (int j = 1; j < 8; ++j) w[j] = (c[2 * j - 1] + c[2 * j + 1]) * F16_PRE[j];
  aan8<M>(w);
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    c[n] = M::mad(w[n], F16_POST[n], e[n]);
    c[15 - n] = M::mad(w[n], -F16_POST[n], e[n]);
  }
}

// fidct16's per-axis input scale of coefficient index k: a_{k/2} / 4 (even),
// 1 (odd); the table entry is (Q16 * s_u) * s_v
__host__ __device__ __forceinline__ double s16_of(const double* aan, int k) {
  return (k & 1) ? 1.0 : aan[k >> 1] * 0.25;
}

// Dequantise and 2-D fidct16 (axis 0, then axis 1) of one 16x16 block held by
// its 16 lanes (line = 0..15) through the block's LDS slot (k_inv16s's
// exchange, rows of RS16); returns row `line` clipped to [-128, 127] (no +128:
// luma adds it on the magic grid, chroma stays shifted).  The dequantised
// input is ((q * Q16) * s_u) * s_v: q * Q16 an exact integer (|q Q| < 2^23,
// v_mul_i32_i24), then the two per-axis scales (s_u the lane's own, s_v a
// constant per unrolled k): no table in LDS, which keeps the kernel at three
// workgroups per CU.  qi: the frame's 8x8 table as integers; qhi / qlo track the
// coefficients the lane read.
__device__ __forceinline__ void fidct16_block(const Row16& rw, const int* __restrict__ qi, double* __restrict__ sb,
                                              int line, double (&r)[16], int& qhi, int& qlo) {
  {
    const uint32_t w[8] = {rw.a.x, rw.a.y, rw.a.z, rw.a.w, rw.b.x, rw.b.y, rw.b.z, rw.b.w};
    const double su = s16_of(c_aan, line);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int qv = (int)(int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
      qhi = max(qhi, qv);
      qlo = min(qlo, qv);
      sb[line * RS16 + k] = ((double)__mul24(qv, qi[(line >> 1) * 8 + (k >> 1)]) * su) * s16_of(c_aan, k);
    }
  }
  __builtin_amdgcn_wave_barrier();
  double c[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = sb[i * RS16 + line];
  fidct16(c);
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[i * RS16 + line] = c[i];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 16; ++k) c[k] = sb[line * RS16 + k];
  fidct16(c);
#pragma unroll
  for (int k = 0; k < 16; ++k) r[k] = fmin(fmax(c[k], -128.0), 127.0);
}

// byte_cert_y for a value that may lie outside the image (ok false: the byte
// is not stored and the value stays out of the certificate)
__device__ __forceinline__ uint32_t byte_cert_m(double y, bool ok, uint32_t& lo_min, uint32_t& lo_max) {
  const uint32_t lo = ok ? (uint32_t)__double2loint(y) : 0x80000000u, hi = (uint32_t)__double2hiint(y);
  lo_min = lo_min < lo ? lo_min : lo;
  lo_max = lo_max > lo ? lo_max : lo;
  const uint32_t c = hi < MAGIC_HI ? MAGIC_HI : hi;
  return c > MAGIC_HI + 255u ? MAGIC_HI + 255u : c;
}

// k_inv16_fast<MODE>: the certified fast inverse for 16x16 blocks at 4:2:x
// (plan runs without SSE terms; BASELINE configs[4]).  k_inv16s's tile, window
// and exchange layout (jds_inv16_exact.hpp: one chroma window at a time in
// LDS, Cb then Cr), with k_inv_fast's arithmetic: the folded dequantisation
// table, fidct16 lines, both planes clipped to [-128, 127], the unnormalised
// upsample (fvsum / fhsum), the colour terms on the magic grid and
// byte_cert_y's certificate, E = K_LIN16 * Dmax + K_CONST16 + 2^-31
// (tools/inv_bound.py --b16; tests/test_inv_bound_cpu.py runs this chain on
// the host against the oracle).  A tile with an uncertain value is recomputed
// by k_inv16s's exact body (inv16s_tile) in the same LDS.
template <int MODE>
__global__ void __launch_bounds__(Inv16<MODE>::NT)
k_inv16_fast(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
             uint8_t* __restrict__ rgb_out, unsigned* __restrict__ fixcount, unsigned* __restrict__ next_count,
             unsigned* __restrict__ item_cnt, const int rot, const int fix_all, jds_frame_stats* __restrict__ st,
             const int fin) {
  using I = Inv16<MODE>;
  static_assert(I::NT == 256, "one table entry per thread");
  __shared__ __attribute__((aligned(16))) double s_b[I::NG * BS16];
  __shared__ double s_cw[I::CWR * I::CWC];
  __shared__ int s_qi[64];  // (the exact fallback reads the 8x8 table from fq: 3 workgroups per CU at 4:2:2)
  __shared__ double s_qmax;
  __shared__ double s_dq[I::NT / 64];
  __shared__ uint32_t s_lmin[I::NT / 64], s_lmax[I::NT / 64];
  __shared__ uint32_t s_cert[3];  // min / max fraction word, max |q|
  __shared__ int s_redo;
  const int tid = threadIdx.x, grp = tid >> 4, line = tid & 15;
  const int frame = blockIdx.y, tile = blockIdx.x;
  // k_finalize's per-frame work (fin >= 0: the run's forward phase completed
  // before this launch; fin = 1 also adds the histogram's zero bin)
  if (fin >= 0 && tile == 0 && tid == 0) finalize_frame(g, st + frame, fin);
  const unsigned n_items = gridDim.y;
  unsigned* cnt_now = item_cnt + rot * n_items;
  if (tile == 0 && tid == 0) {
    item_cnt[((rot + 1) % 3) * n_items + frame] = 0u;  // the next run's
    if (frame == 0) *next_count = 0u;                  // the next run counts from zero
  }
  if (tid < 64) {
    double m = fq[frame].q[tid];
    s_qi[tid] = (int)m;
    m = fq[frame].qmax;
    if (tid == 0) {
      s_qmax = m;
      s_cert[0] = 0xffffffffu;
      s_cert[1] = 0u;
      s_cert[2] = 0u;
    }
  }
  __syncthreads();

  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  const int cwy0 = Y0 / I::SY - I::RY, cwx0 = X0 / 2 - 1;
  const int cby0 = (Y0 / I::SY) / 16 - I::RY, cbx0 = (X0 / 2) / 16 - 1;
  double* const sb = s_b + grp * BS16;
  constexpr int NCR = (I::NCB + I::NG - 1) / I::NG;  // chroma rounds per plane
  Row16 crow[2][NCR];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int k = 0; k < NCR; ++k) {
      const int bi = k * I::NG + grp;
      const int by = cby0 + bi / I::CBC, bx = cbx0 + bi % I::CBC;
      if (bi < I::NCB && by >= 0 && bx >= 0 && by < g.ncy && bx < g.ncx)
        crow[p][k] = load_row16(cf + (p ? g.off_cr : g.off_cb) + ((long long)by * g.ncx + bx) * 256, line);
    }
  }
  const int by = Y0 / 16 + grp / I::YBC, bx = X0 / 16 + grp % I::YBC;
  Row16 lrow;
  if (by < g.nby && bx < g.nbx) lrow = load_row16(cf + ((long long)by * g.nbx + bx) * 256, line);

  int qhi = 0, qlo = 0;
  auto build = [&](int p) {  // plane p's window: (C - 128) of the blocks the tile reaches (+ ring)
#pragma unroll
    for (int k = 0; k < NCR; ++k) {
      const int bi = k * I::NG + grp;
      if (bi < I::NCB) {
        const int cy = cby0 + bi / I::CBC, cx = cbx0 + bi % I::CBC;
        if (cy >= 0 && cx >= 0 && cy < g.ncy && cx < g.ncx) {  // uniform per 16-lane group
          double r[16];
          fidct16_block(crow[p][k], s_qi, sb, line, r, qhi, qlo);
          const int wr = cy * 16 + line - cwy0;
          if ((unsigned)wr < (unsigned)I::CWR) {
            double* w = &s_cw[wr * I::CWC];
            const int wc0 = cx * 16 - cwx0;
#pragma unroll
            for (int j = 0; j < 16; ++j)
              if ((unsigned)(wc0 + j) < (unsigned)I::CWC) w[wc0 + j] = r[j];
          }
        }
      }
    }
  };
  // one plane's upsampled (C - 128) at pixels x0 .. x0 + 7 of row (wq, wt),
  // times 2^USH_ (chroma8_fast's sums; cv2's clamped taps at the image's edge
  // pixels take the edge sample, as in k_inv16s: its vertical sum times 4)
  constexpr int USH_ = USH<I::SY, 2>;
  auto upsample = [&](int x0, int wq, int wt, double (&C)[8]) {
    const int c0 = x0 / 2 - 1 - cwx0;
    double vb[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if constexpr (I::SY == 2)
        vb[j] = fvsum(s_cw[wq * I::CWC + c0 + j], s_cw[wt * I::CWC + c0 + j]);
      else
        vb[j] = s_cw[wq * I::CWC + c0 + j];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      C[2 * i] = fhsum(vb[i], vb[i + 1]);
      C[2 * i + 1] = fhsum(vb[i + 2], vb[i + 1]);
    }
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int kl = side == 0 ? (x0 == 0 ? 0 : -1) : (g.W - 1 - x0 < 8 ? g.W - 1 - x0 : -1);
      if (kl >= 0) {
        const int e = (side == 0 ? 0 : g.wc - 1) - cwx0;
        double v = s_cw[wq * I::CWC + e];
        if constexpr (I::SY == 2) v = fvsum(v, s_cw[wt * I::CWC + e]);
        v *= 4.0;  // (exact)
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = k == kl ? v : C[k];
      }
    }
  };

  // ---- 1. Cb window; luma row, B bytes and the G partial on the grid -------
  build(0);
  __syncthreads();
  const int y = by * 16 + line;
  const bool act = by < g.nby && bx < g.nbx;  // uniform per 16-lane group
  const bool rowok = act && y < g.H;
  uint32_t lo_min = 0xffffffffu, lo_max = 0u;
  double Yv[16], Gt[16];
  uint32_t bpk[4] = {0u, 0u, 0u, 0u};  // B bytes of the row, packed
  int wq = 0, wt = 0;
  if (act) fidct16_block(lrow, s_qi, sb, line, Yv, qhi, qlo);
  if (rowok) {
    if constexpr (I::SY == 2) {  // cv2 INTER_LINEAR rows (k_inv16s): wq weight 1/4, wt weight 3/4
      float fy = (float)((y + 0.5) * g.up_sy - 0.5);
      const int sy = (int)floorf(fy);
      fy -= (float)sy;
      const int r0 = clampi(clampi(sy, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
      const int r1 = clampi(clampi(sy + 1, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
      const bool q0 = fy == 0.75f;
      wq = q0 ? r0 : r1;
      wt = q0 ? r1 : r0;
    } else {
      wq = y - cwy0;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int x0 = bx * 16 + 8 * h;
      if (x0 < g.W) {
        double C[8];
        upsample(x0, wq, wt, C);
        uint32_t cb[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double yv = Yv[8 * h + k] + (MAGIC + 128.0);
          Yv[8 * h + k] = yv;
          cb[k] = byte_cert_m(col_b<MadDev, USH_>(yv, C[k]), x0 + k < g.W, lo_min, lo_max);
          Gt[8 * h + k] = col_gt<MadDev, USH_>(yv, C[k]);
        }
        bpk[2 * h] = pack4(cb[0], cb[1], cb[2], cb[3]);
        bpk[2 * h + 1] = pack4(cb[4], cb[5], cb[6], cb[7]);
      }
    }
  }
  __syncthreads();  // every Cb read done
  // ---- 2. Cr window; R, G bytes and the stores --------------------------------
  build(1);
  __syncthreads();
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
  if (rowok) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int x0 = bx * 16 + 8 * h;
      if (x0 < g.W) {
        double C[8];
        upsample(x0, wq, wt, C);
        const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
        uint32_t ch[24];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool ok = k < nx;
          ch[3 * k] = byte_cert_m(col_r<MadDev, USH_>(Yv[8 * h + k], C[k]), ok, lo_min, lo_max);
          ch[3 * k + 1] = byte_cert_m(col_g<MadDev, USH_>(Gt[8 * h + k], C[k]), ok, lo_min, lo_max);
          ch[3 * k + 2] = (bpk[2 * h + (k >> 2)] >> (8 * (k & 3))) & 255u;
        }
        uint32_t pk[6];
#pragma unroll
        for (int w = 0; w < 6; ++w) pk[w] = pack4(ch[4 * w], ch[4 * w + 1], ch[4 * w + 2], ch[4 * w + 3]);
        uint8_t* o = out_f + ((size_t)y * g.W + x0) * 3;
        if (nx == 8 && ((((uintptr_t)o) & 7u) == 0)) {
          uint2* o2 = reinterpret_cast<uint2*>(o);
          o2[0] = make_uint2(pk[0], pk[1]);
          o2[1] = make_uint2(pk[2], pk[3]);
          o2[2] = make_uint2(pk[4], pk[5]);
        } else {
#pragma unroll
          for (int b = 0; b < 24; ++b)
            if (b < 3 * nx) o[b] = (uint8_t)(pk[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
  }

  // ---- 3. certification: the tile's closest approach to an integer vs its bound
  int qm = max(qhi, -qlo);
  cert_to_lds(lo_min, lo_max, (uint32_t)qm, s_cert);
  __syncthreads();
  if (tid == 0) {
    const uint32_t mn = s_cert[0], mx = s_cert[1];
    const double q = (double)s_cert[2];
    const double E = K_LIN16 * (q * s_qmax) + K_CONST16 + 0x1p-31;
    const double T = ceil(E * 0x1p+32) + 1.0;
    const bool uncertain = (double)mn <= T || (double)mx >= 0x1p+32 - 1.0 - T;
    s_redo = uncertain || fix_all;
    if (s_redo) {
      atomicAdd(fixcount, 1u);  // tiles recomputed (jds_plan_fix_counts)
      atomicAdd(cnt_now + frame, 1u);
    }
  }
  __syncthreads();
#ifndef JDS_PROBE_NOFALLBACK
  if (s_redo)  // (uniform) the exact tile body overwrites the tile
    inv16s_tile<MODE, 0>(s_b, s_cw, fq[frame].q, nullptr, nullptr, g, tiles_x, (int)gridDim.x, frame, tile, coeffs,
                         nullptr, rgb_out, nullptr, nullptr, nullptr, nullptr);
#endif
}

hipError_t launch_inv16_fast(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                             uint8_t* rgb_out, const InvFix& fx, hipStream_t s, jds_frame_stats* st, int fin) {
  auto go = [&](auto kern, int TH, int TW) {
    const int tx = (g.W + TW - 1) / TW, ty = (g.H + TH - 1) / TH;
    hipLaunchKernelGGL(kern, dim3(ty * tx, n), dim3(256), 0, s, g, tx, coeffs, fq, rgb_out, fx.count + fx.parity,
                       fx.count + (fx.parity ^ 1), fx.item, fx.rot, fx.fix_all, st, fin);
    kmark(s, "k_inv16_fast<%d>", mode);
    return hipGetLastError();
  };
  if (mode == M420) return go(k_inv16_fast<M420>, Inv16<M420>::TH, Inv16<M420>::TW);
  if (mode == M422) return go(k_inv16_fast<M422>, Inv16<M422>::TH, Inv16<M422>::TW);
  return hipErrorInvalidValue;  // 4:4:4 keeps k_chroma16 + k_inv16
}

// ------------------------------------------------------------ launchers --

// k_inv6_fix's workgroups (grid-stride over the list): typically a handful of
// tiles per run; an item in exact mode lists all of its tiles
constexpr int INV6_FIX_GRID = 256;

template <int MODE>
static hipError_t inv_fast_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq, const uint8_t* rgb_in,
                             uint8_t* rgb_out, jds_frame_stats* st, double* part, const InvFix& fx, hipStream_t s,
                             int in_div, int fin) {
  const int ty = (g.H + Inv<MODE>::TH - 1) / Inv<MODE>::TH, tx = (g.W + Inv<MODE>::TW - 1) / Inv<MODE>::TW;
  const dim3 grid(ty * tx, n), blk(Inv<MODE>::NT);
  // count[parity] was zeroed by the previous run; this run zeroes the other
  unsigned* cnt = fx.count + fx.parity;
  unsigned* nxt = fx.count + (fx.parity ^ 1);
#ifdef JDS_INV6  // (A/B: tools/build_variant.py -DJDS_INV6 routes 4:2:0 to the transpose-free kernel)
  if (MODE == M420 && fx.list) {
    // the transpose-free kernel, then the exact recomputation of the tiles it listed
    hipLaunchKernelGGL(k_inv_fast6, grid, dim3(W6::NT), 0, s, g, tx, coeffs, fq, rgb_out, st, cnt, nxt, fx.item,
                       fx.list, fx.rot, fx.probe, fx.fix_all, fin);
    kmark(s, "k_inv_fast6");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int nfix = std::min(ty * tx * n, INV6_FIX_GRID);
    hipLaunchKernelGGL(k_inv6_fix, dim3(nfix), dim3(Inv<M420>::NT), 0, s, g, tx, coeffs, fq, rgb_out, cnt, fx.list);
    kmark(s, "k_inv6_fix");
    return hipGetLastError();
  }
#endif
  if (rgb_in != nullptr) {
    // SSE runs (sweeps): the exact integer SSE and the luma SSE partials, per
    // certified tile by the fast pass, per uncertain tile by the exact tile code
    hipLaunchKernelGGL((k_inv_fast<MODE, 1>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part, cnt,
                       nxt, fx.item, fx.rot, fx.probe, in_div, fx.fix_all, -1);
    kmark(s, "k_inv_fast<%d,1>", MODE);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((k_inv_fast<MODE, 0>), grid, blk, 0, s, g, tx, coeffs, fq, nullptr, rgb_out, st, part, cnt, nxt,
                     fx.item, fx.rot, fx.probe, in_div, fx.fix_all, fin);
  kmark(s, "k_inv_fast<%d,0>", MODE);
  return hipGetLastError();
}

hipError_t launch_inv_fast(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                           const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                           const InvFix& fx, hipStream_t s, int in_div, int fin) {
  switch (mode) {
    case M420: return inv_fast_t<M420>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx, s, in_div, fin);
    case M422: return inv_fast_t<M422>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx, s, in_div, fin);
    default: {
      // 4:4:4: the wave-local kernel (SSE runs take the exact kernel, launch_codec)
      (void)rgb_in;
      (void)part;
      (void)in_div;
      const long long nblk = (long long)g.nby * g.nbx;
      const dim3 grid((unsigned)((nblk + 8 * I444_WAVES - 1) / (8 * I444_WAVES)), n), blk(64 * I444_WAVES);
      hipLaunchKernelGGL(k_inv_fast444, grid, blk, 0, s, g, coeffs, fq, rgb_out, st, fx.count + fx.parity,
                         fx.count + (fx.parity ^ 1), fx.item, fx.rot, fx.fix_all, fin);
      kmark(s, "k_inv_fast444");
      return hipGetLastError();
    }
  }
}

// ------------------------------------------- host: the chain (tests only) --
//
// k_inv_fast's (BS = 8) and k_inv16_fast's (BS = 16) arithmetic evaluated on
// the host for a whole image, with the kernels' own helpers (aan8 / fidct16,
// fvsum, fhsum, col_*): dequantisation with the folded table, the IDCT
// along axis 0 then axis 1, clip to [-128, 127], the unnormalised vertical
// then horizontal chroma sums with cv2's clamped taps (the
// kernels' replicated window ring or edge selects give the same operands), the
// colour terms on the magic grid and byte_cert_y's byte.  fuse = 0: every
// multiply-add rounded twice (MadDev on x86-64); 1: every one fused (MadFma).
// values[] = v' = y - MAGIC (exact), the value the certificate judges.
// Q: the 8x8 table (16x16: Q16[u][v] = Q[u/2][v/2]).
template <class M, int BS>
static void inv_fast_host_t(int mode, const int16_t* cf, const double* Q, int H, int W, double* vout,
                            uint8_t* bout) {
  const int sy = mode == M420 ? 2 : 1, sx = mode == M444 ? 1 : 2;
  // dequantised input of coefficient (u, v): 8x8, q * qs with the folded table;
  // 16x16, ((q * Q16) * s_u) * s_v (fidct16_block's order)
  double qs[64];
  for (int i = 0; i < 64; ++i) qs[i] = Q[i] * h_aan[i >> 3] * h_aan[i & 7] * 0.125;
  auto deq = [&](int q, int u, int v) {
    if constexpr (BS == 8) return (double)q * qs[u * 8 + v];
    return ((double)(q * (int)Q[(u >> 1) * 8 + (v >> 1)]) * s16_of(h_aan, u)) * s16_of(h_aan, v);
  };
  auto line = [](double(&c)[BS]) {
    if constexpr (BS == 8)
      aan8<M>(c);
    else
      fidct16<M>(c);
  };
  std::vector<double> pl[3];
  int ph[3], pw[3], st[3];
  size_t off = 0;
  for (int p = 0; p < 3; ++p) {
    ph[p] = p ? H / sy : H;
    pw[p] = p ? W / sx : W;
    const int nby = (ph[p] + BS - 1) / BS, nbx = (pw[p] + BS - 1) / BS;
    st[p] = nbx * BS;
    pl[p].assign((size_t)nby * BS * st[p], 0.0);
    for (int by = 0; by < nby; ++by)
      for (int bx = 0; bx < nbx; ++bx) {
        const int16_t* b = cf + off + ((size_t)by * nbx + bx) * BS * BS;
        double mid[BS][BS];
        for (int v = 0; v < BS; ++v) {  // axis 0
          double c[BS];
          for (int r = 0; r < BS; ++r) c[r] = deq(b[r * BS + v], r, v);
          line(c);
          for (int r = 0; r < BS; ++r) mid[r][v] = c[r];
        }
        for (int u = 0; u < BS; ++u) {  // axis 1, clip
          double c[BS];
          for (int k = 0; k < BS; ++k) c[k] = mid[u][k];
          line(c);
          for (int k = 0; k < BS; ++k)
            pl[p][(size_t)(by * BS + u) * st[p] + bx * BS + k] = fmin(fmax(c[k], -128.0), 127.0);
        }
      }
    off += (size_t)nby * nbx * BS * BS;
  }
  auto S = [&](int p, int r, int c) {  // clamped taps (cv2) = the kernel's ring / clampi rows
    r = r < 0 ? 0 : (r > ph[p] - 1 ? ph[p] - 1 : r);
    c = c < 0 ? 0 : (c > pw[p] - 1 ? pw[p] - 1 : c);
    return pl[p][(size_t)r * st[p] + c];
  };
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      double C[3];
      for (int p = 1; p < 3; ++p) {
        if (sx == 1) {
          C[p] = S(p, y, x);
          continue;
        }
        auto vb = [&](int col) {
          if (sy == 2) {
            const int m = y >> 1, rq = (y & 1) ? m + 1 : m - 1;
            return fvsum<M>(S(p, rq, col), S(p, m, col));
          }
          return S(p, y, col);
        };
        const int m = x >> 1;
        C[p] = (x & 1) == 0 ? fhsum<M>(vb(m - 1), vb(m)) : fhsum<M>(vb(m + 1), vb(m));
      }
      const double Yv = S(0, y, x) + (MAGIC + 128.0);
      double B, Gt, R, G;
      if (sx == 1) {
        B = col_b<M>(Yv, C[1]), Gt = col_gt<M>(Yv, C[1]);
        R = col_r<M>(Yv, C[2]), G = col_g<M>(Gt, C[2]);
      } else if (sy == 1) {
        B = col_b<M, 2>(Yv, C[1]), Gt = col_gt<M, 2>(Yv, C[1]);
        R = col_r<M, 2>(Yv, C[2]), G = col_g<M, 2>(Gt, C[2]);
      } else {
        B = col_b<M, 4>(Yv, C[1]), Gt = col_gt<M, 4>(Yv, C[1]);
        R = col_r<M, 4>(Yv, C[2]), G = col_g<M, 4>(Gt, C[2]);
      }
      const double o[3] = {R, G, B};
      for (int ch = 0; ch < 3; ++ch) {
        uint64_t bits;
        memcpy(&bits, &o[ch], 8);
        const uint32_t hi = (uint32_t)(bits >> 32);
        const uint32_t c = hi < MAGIC_HI ? MAGIC_HI : (hi > MAGIC_HI + 255u ? MAGIC_HI + 255u : hi);
        const size_t i = ((size_t)y * W + x) * 3 + ch;
        vout[i] = o[ch] - MAGIC;
        bout[i] = (uint8_t)(c & 255u);
      }
    }
}

int inv_fast_host(int mode, const int16_t* cf, const double* Q, int H, int W, int fuse, int block, double* vout,
                  uint8_t* bout) {
  const int sy = mode == M420 ? 2 : 1, sx = mode == M444 ? 1 : 2;
  if (H % sy || W % sx || (block != 8 && block != 16)) return -1;  // the tiled kernels' even geometries
  if (block == 16) {
    if (fuse)
      inv_fast_host_t<MadFma, 16>(mode, cf, Q, H, W, vout, bout);
    else
      inv_fast_host_t<MadDev, 16>(mode, cf, Q, H, W, vout, bout);
  } else if (fuse) {
    inv_fast_host_t<MadFma, 8>(mode, cf, Q, H, W, vout, bout);
  } else {
    inv_fast_host_t<MadDev, 8>(mode, cf, Q, H, W, vout, bout);
  }
  return 0;
}

}  // namespace jds
