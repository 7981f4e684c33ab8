// jds_device.hpp — device helpers shared by the codec kernels (exact fp64
// restatements of the reference's per-sample arithmetic and index maps).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jds {


// np.pad(mode='reflect') source index for i >= 0 (engines/block_processor.py:13)
__device__ __forceinline__ int reflect_pad(int i, int n) {
  if (i < n) return i;
  if (n == 1) return 0;
  const int p = 2 * (n - 1);
  i %= p;
  return i >= n ? p - i : i;
}

// cv2 BORDER_REFLECT_101 for any i (GaussianBlur default border)
__device__ __forceinline__ int reflect101(int i, int n) {
  if ((unsigned)i < (unsigned)n) return i;  // inside: no modulo
  if (n == 1) return 0;
  const int p = 2 * (n - 1);
  i = i < 0 ? -i : i;
  i %= p;
  return i >= n ? p - i : i;
}

// engines/color_space.py:8-14 — each product rounded, sums left to right
__device__ __forceinline__ double luma(double R, double G, double B) {
  return 0.299 * R + 0.587 * G + 0.114 * B;
}
// The luma SSE term of one pixel pair, 1e6 (Y(a) - Y(b))^2 with Y = .299 R +
// .587 G + .114 B in exact decimal arithmetic, from the byte differences
// d = a - b: D = 299 d0 + 587 d1 + 114 d2 is an integer (|D| <= 255,000), D^2 <
// 2^36 is exact in a double, and so is any sum of up to 2^17 of them, in any
// order.  Every inverse kernel sums these per tile (exact, order-free) and
// k_finalize divides the frame total by 1e6 once (round 6: two fp64 lumas per
// pixel, ~19 fp64 operations, became 3 integer and 2 fp64 ones; the total is
// the exact sum correctly rounded, not NumPy's pairwise fp64 one: jds.h).
__device__ __forceinline__ double luma_sse_e6(int d0, int d1, int d2) {
  const double x = (double)(299 * d0 + 587 * d1 + 114 * d2);
  return x * x;
}
__device__ __forceinline__ double chroma_b(double R, double G, double B) {
  return -0.168736 * R - 0.331264 * G + 0.5 * B + 128.0;
}
__device__ __forceinline__ double chroma_r(double R, double G, double B) {
  return 0.5 * R - 0.418688 * G - 0.081312 * B + 128.0;
}

__device__ __forceinline__ void unpack(uint32_t v, double& R, double& G, double& B) {
  R = (double)(v & 255u);
  G = (double)((v >> 8) & 255u);
  B = (double)(v >> 16);
}

// 1/d for d > 0 to within 2^-60 relative: v_rcp_f64 and two Newton steps
__device__ __forceinline__ double recip64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}

// rint(x / d) of the IEEE quotient (np.round(c / Q): round half to even of
// the correctly rounded fp64 quotient) with r = recip64(d): t = x * r is within
// |t| 2^-52 of x / d, and fl(x / d) within |x / d| 2^-53, so when t lies
// farther than |t| 2^-49 from its nearest half-integer both round to rint(t);
// otherwise (rare) the division decides.
__device__ __forceinline__ int rint_quot(double x, double d, double r) {
  const double t = x * r, q = __builtin_rint(t);
  const double m = fabs(fabs(t - q) - 0.5);  // distance to the nearest half-integer
  if (__builtin_expect(m > fabs(t) * 0x1p-49, 1)) return (int)q;
  return (int)__builtin_rint(x / d);
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T clampi(T v, T lo, T hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace jds
