// jds_fwd_common.hpp — pieces shared by the certified forward kernels
// (jds_fast.hip: 8x8 blocks, jds_fast16.hip: 16x16 blocks): the fp32 colour
// conversions whose rounding the host bound covers (fwd_input_error), the
// exact fp64 sample of a padded plane read straight from global memory (the
// fix-up kernels' input), and the host bound helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "jds_device.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int NSTAT = 52;  // per-tile statistics: nonzero, magnitude bits, hist[50]

// fp32 colour conversions (any rounding order is fine: bounded on the host)
__host__ __device__ __forceinline__ float luma32(float R, float G, float B) {
  return fmaf(0.114f, B, fmaf(0.587f, G, 0.299f * R));
}
// luma - 128 with the level shift folded into the chain: three roundings of
// magnitude <= 128 instead of luma32's, inside fwd_input_error's luma bound
__host__ __device__ __forceinline__ float luma32m(float R, float G, float B) {
  return fmaf(0.114f, B, fmaf(0.587f, G, fmaf(0.299f, R, -128.0f)));
}
__host__ __device__ __forceinline__ float cb32(float R, float G, float B) {
  return fmaf(-0.168736f, R, fmaf(-0.331264f, G, fmaf(0.5f, B, 128.0f)));
}
__host__ __device__ __forceinline__ float cr32(float R, float G, float B) {
  return fmaf(-0.081312f, B, fmaf(-0.418688f, G, fmaf(0.5f, R, 128.0f)));
}

// ---- exact fp64 recomputation of one block column from global memory ----

__device__ __forceinline__ double px_chroma64(const uint8_t* img, const Geo& g, int y, int x, int plane) {
  const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
  const double R = p[0], G = p[1], B = p[2];
  return plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B);
}

// cv2 RowFilter<double> at (y, x), BORDER_REFLECT_101
__device__ inline double row_pass64(const uint8_t* img, const Geo& g, int y, int x, int plane, const double* k) {
  double t = k[0] * px_chroma64(img, g, y, reflect101(x - 1, g.W), plane);
  t = t + k[1] * px_chroma64(img, g, y, x, plane);
  return t + k[2] * px_chroma64(img, g, y, reflect101(x + 1, g.W), plane);
}

template <int MODE, bool PF>
__device__ inline double sample64(const uint8_t* img, const Geo& g, int plane, int pr, int pc, const double* k) {
  if (plane == 0 || MODE == M444) {
    const int y = reflect_pad(pr, g.H), x = reflect_pad(pc, g.W);
    const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
    const double R = p[0], G = p[1], B = p[2];
    return plane == 0 ? luma(R, G, B) : (plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B));
  }
  constexpr int SY = Cfg<MODE>::SY;
  const int sr = reflect_pad(pr, g.hc), sc = reflect_pad(pc, g.wc);
  double s[SY][2];
#pragma unroll 1
  for (int a = 0; a < SY; ++a) {
#pragma unroll 1
    for (int b = 0; b < 2; ++b) {
      const int y = SY * sr + a, x = 2 * sc + b;
      if constexpr (PF) {
        const double d = k[1] * row_pass64(img, g, y, x, plane, k) + 0.0;
        s[a][b] = d + k[0] * (row_pass64(img, g, reflect101(y + 1, g.H), x, plane, k) +
                              row_pass64(img, g, reflect101(y - 1, g.H), x, plane, k));
      } else {
        s[a][b] = px_chroma64(img, g, y, x, plane);
      }
    }
  }
  if constexpr (SY == 2)
    return (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25;
  else
    return (s[0][0] + s[0][1]) * 0.5;
}

// Sums of four words over each 16-lane row of a wave: inclusive sums by four
// DPP row shifts, the four words interleaved so that no DPP read waits on the
// write before it.
// Round-half-even to an integer by the magic constant 1.5 * 2^23: for
// |t| < 2^22 the sum f = t + M lies in [2^23, 2^24), where the float spacing is
// 1, so the addition rounds t to the nearest integer, ties to even (rintf's
// result); r = f - M is exact, and f's encoding is 0x4B400000 + r (its low 16
// bits are r as int16).  The certified quantisers (quant8, k_fwd16f) use it
// in place of rndne + cvt: gfx950 issues fp32 add / sub in ~2.5 cycles per
// wave, conversions in ~4.3 (tools/microbench/op_rates.hip).
constexpr float QMAGIC = 0x1.8p+23f;
constexpr uint32_t QMAGIC_BITS = 0x4B400000u;

// A float from another lane of the same 16-lane row by a DPP move (lanes
// whose source lies outside the row read 0).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, true));
}

template <int SH, int N>
__device__ __forceinline__ void row_shr_add(unsigned (&v)[N]) {
  unsigned t[N];
#pragma unroll
  for (int k = 0; k < N; ++k) t[k] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v[k], 0x110 + SH, 0xf, 0xf, true);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += t[k];
}
template <int N>
__device__ __forceinline__ void row_sums(unsigned (&v)[N]) {
  row_shr_add<1>(v);
  row_shr_add<2>(v);
  row_shr_add<4>(v);
  row_shr_add<8>(v);  // lane 15 of each 16-lane row now holds the row's sums
}
__device__ __forceinline__ void row_sums3(unsigned (&v)[3]) { row_sums(v); }
__device__ __forceinline__ void row_sums4(unsigned (&v)[4]) { row_sums(v); }

// ---- host: bound helpers (jds_fast.hip) ----
// One pass of an FMA-chain transform over inputs (bound X, error e): output k's
// magnitude and error bound, rows W[k][0..3] of an 8-point even/odd split.
void pass_bound(double X, double e, const double* Xin, const double* ein, double* Xout, double* eout,
                const double W[8][4]);
// |x_fp32 - x_exact| bound of the level-shifted samples entering the DCT.
// chains (prefiltered chroma): bit 0 the per-pixel Gaussian then area chain,
// bit 1 the combined taps; the bound covers every chain named
double fwd_input_error(int plane, int mode, bool pf, const double* gk, int chains = 3);

}  // namespace jds
