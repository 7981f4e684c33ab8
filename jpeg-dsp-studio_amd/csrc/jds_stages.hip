// jds_stages.hip — the per-stage functions of the engines.* API
// (engines/__init__.py:10-27) as standalone HIP kernels on fp64 arrays:
//   rgb_to_ycbcr / ycbcr_to_rgb        engines/color_space.py:8-24
//   subsample_chroma (blur + area)     engines/color_space.py:27-53
//   upsample_chroma (linear / nearest) engines/color_space.py:56-66
//   dct2 / idct2 / encode / decode     engines/dct_engine.py:7-27 (8x8 blocks)
//   quantize / dequantize              engines/quantizer.py:22-29
// Same arithmetic (and operation order) as the fused codec kernels, so a
// caller chaining these stages gets the bytes the fused path produces.
// Host entry points take host arrays and stage them through the context.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct8.hpp"
#include "jds_dct16.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

__global__ void k_stage_rgb2ycc(const double* __restrict__ in, double* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double R = in[3 * i], G = in[3 * i + 1], B = in[3 * i + 2];
  out[3 * i] = 0.299 * R + 0.587 * G + 0.114 * B;
  out[3 * i + 1] = -0.168736 * R - 0.331264 * G + 0.5 * B + 128.0;
  out[3 * i + 2] = 0.5 * R - 0.418688 * G - 0.081312 * B + 128.0;
}

__global__ void k_stage_ycc2rgb(const double* __restrict__ in, double* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double Y = in[3 * i], Cb = in[3 * i + 1], Cr = in[3 * i + 2];
  const double R = Y + 1.402 * (Cr - 128.0);
  const double G = Y - 0.344136 * (Cb - 128.0) - 0.714136 * (Cr - 128.0);
  const double B = Y + 1.772 * (Cb - 128.0);
  out[3 * i] = fmin(fmax(R, 0.0), 255.0);
  out[3 * i + 1] = fmin(fmax(G, 0.0), 255.0);
  out[3 * i + 2] = fmin(fmax(B, 0.0), 255.0);
}

__device__ __forceinline__ int r101(int i, int n) {
  if (n == 1) return 0;
  const int p = 2 * (n - 1);
  i = i < 0 ? -i : i;
  i %= p;
  return i >= n ? p - i : i;
}

// cv2 RowFilter<double> with BORDER_REFLECT_101: t = k0*S[x-1]; t += k1*S[x]; t += k2*S[x+1]
__global__ void k_stage_blur_rows(const double* __restrict__ in, double* __restrict__ out, int H, int W,
                                  double k0, double k1, double k2) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)H * W) return;
  const int y = (int)(i / W), x = (int)(i - (long long)y * W);
  const double* r = in + (size_t)y * W;
  double t = k0 * r[r101(x - 1, W)];
  t = t + k1 * r[x];
  out[i] = t + k2 * r[r101(x + 1, W)];
}

// cv2 SymmColumnFilter<double>: d = k1*T[y] + 0; d += k0*(T[y+1] + T[y-1])
__global__ void k_stage_blur_cols(const double* __restrict__ in, double* __restrict__ out, int H, int W,
                                  double k0, double k1) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)H * W) return;
  const int y = (int)(i / W), x = (int)(i - (long long)y * W);
  const double d = k1 * in[i] + 0.0;
  out[i] = d + k0 * (in[(size_t)r101(y + 1, H) * W + x] + in[(size_t)r101(y - 1, H) * W + x]);
}

// cv2 INTER_AREA integer-factor fast path: ((s00 + s01) + s10) + s11) * 0.25 | (s0 + s1) * 0.5
__global__ void k_stage_area(const double* __restrict__ in, double* __restrict__ out, int H, int W, int sy) {
  const int oh = H / sy, ow = W / 2;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)oh * ow) return;
  const int y = (int)(i / ow), x = (int)(i - (long long)y * ow);
  const double* r0 = in + (size_t)(y * sy) * W + 2 * x;
  if (sy == 2) {
    const double* r1 = r0 + W;
    out[i] = (((r0[0] + r0[1]) + r1[0]) + r1[1]) * 0.25;
  } else {
    out[i] = (r0[0] + r0[1]) * 0.5;
  }
}

// cv2.resize INTER_LINEAR (resizeGeneric, 64F) or INTER_NEAREST
__global__ void k_stage_resize(const double* __restrict__ in, int h, int w, double* __restrict__ out, int H,
                               int W, double scale_y, double scale_x, int nearest) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)H * W) return;
  const int dy = (int)(i / W), dx = (int)(i - (long long)dy * W);
  if (nearest) {
    int sy = (int)floor(dy * scale_y), sx = (int)floor(dx * scale_x);
    sy = sy < h - 1 ? sy : h - 1;
    sx = sx < w - 1 ? sx : w - 1;
    out[i] = in[(size_t)sy * w + sx];
    return;
  }
  float fy = (float)((dy + 0.5) * scale_y - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const double b0 = (double)(1.f - fy), b1 = (double)fy;
  const int r0 = sy < 0 ? 0 : (sy > h - 1 ? h - 1 : sy);
  const int r1 = sy + 1 < 0 ? 0 : (sy + 1 > h - 1 ? h - 1 : sy + 1);
  float fx = (float)((dx + 0.5) * scale_x - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { sx = 0; fx = 0.f; }
  const bool copy = sx + 1 >= w;
  if (sx >= w - 1) { sx = w - 1; fx = 0.f; }
  const double a0 = (double)(1.f - fx), a1 = (double)fx;
  const double* s0 = in + (size_t)r0 * w + sx;
  const double* s1 = in + (size_t)r1 * w + sx;
  double h0, h1;
  if (copy) {
    h0 = s0[0] * 1.0;
    h1 = s1[0] * 1.0;
  } else {
    h0 = s0[0] * a0 + s0[1] * a1;
    h1 = s1[0] * a0 + s1[1] * a1;
  }
  out[i] = h0 * b0 + h1 * b1;
}

// 8x8 block transforms; op: 0 dct2, 1 idct2, 2 encode_block, 3 decode_block
__global__ void k_stage_block(const double* __restrict__ in, double* __restrict__ out, long long n, int op) {
  __shared__ double s[8][65];
  const int lb = threadIdx.x >> 3, line = threadIdx.x & 7;
  const long long b = (long long)blockIdx.x * 8 + lb;
  const bool ok = b < n;
  double c[8];
  if (ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = in[b * 64 + i * 8 + line];  // column `line`
    if (op == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = c[i] - 128.0;
    }
    if (op == 0 || op == 2)
      dct2_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
    else
      dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
    for (int i = 0; i < 8; ++i) s[lb][i * 8 + line] = c[i];
  }
  __syncthreads();
  if (!ok) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = s[lb][line * 8 + k];  // row `line`
  if (op == 0 || op == 2)
    dct2_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
  else
    dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    double v = c[k] * 0.0625;  // pocketfft fct = 1/16 (exact)
    if (op == 3) {
      v = v + 128.0;
      v = fmin(fmax(v, 0.0), 255.0);
    }
    out[b * 64 + line * 8 + k] = v;
  }
}

// quantize: int16(rint(c / Q)); dequantize: double(q) * Q (Q broadcast with period 64 or 256)
// 16x16 blocks (dctn / idctn on a 16x16 block, dct_engine.py:7-27): 16 lanes
// per block, column pass then row pass; fct = 1/32 on the first axis (exact).
__global__ void __launch_bounds__(256) k_stage_block16(const double* __restrict__ in, double* __restrict__ out,
                                                       long long n, int op) {
  __shared__ double s[16][16 * 16 + 1];
  const int lb = threadIdx.x >> 4, line = threadIdx.x & 15;
  const long long b = (long long)blockIdx.x * 16 + lb;
  const bool ok = b < n;
  double c[16];
  if (ok) {
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = in[b * 256 + i * 16 + line];  // column `line`
    if (op == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) c[i] = c[i] - 128.0;
    }
    if (op == 0 || op == 2)
      dct2_line16(c);
    else
      dct3_line16(c);
#pragma unroll
    for (int i = 0; i < 16; ++i) s[lb][i * 16 + line] = c[i];
  }
  __syncthreads();
  if (!ok) return;
#pragma unroll
  for (int k = 0; k < 16; ++k) c[k] = s[lb][line * 16 + k];  // row `line`
  if (op == 0 || op == 2)
    dct2_line16(c);
  else
    dct3_line16(c);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    double v = c[k] * 0.03125;
    if (op == 3) v = fmin(fmax(v + 128.0, 0.0), 255.0);
    out[b * 256 + line * 16 + k] = v;
  }
}

__global__ void k_stage_quant(const void* __restrict__ in, const double* __restrict__ q, void* __restrict__ out,
                              long long n, int dequant, int period) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double qq = q[i & (period - 1)];
  if (dequant)
    ((double*)out)[i] = (double)((const int16_t*)in)[i] * qq;
  else
    ((int16_t*)out)[i] = (int16_t)(int)__builtin_rint(((const double*)in)[i] / qq);
}

static inline unsigned nblk(long long n, int t) { return (unsigned)((n + t - 1) / t); }

hipError_t stage_rgb_ycc(const double* in, double* out, long long n, int inverse, hipStream_t s) {
  if (inverse)
    hipLaunchKernelGGL(k_stage_ycc2rgb, dim3(nblk(n, 256)), dim3(256), 0, s, in, out, n);
  else
    hipLaunchKernelGGL(k_stage_rgb2ycc, dim3(nblk(n, 256)), dim3(256), 0, s, in, out, n);
  return hipGetLastError();
}

hipError_t stage_subsample(const double* in, double* tmp, double* tmp2, double* out, int H, int W, int sy,
                           int prefilter, const double* k, hipStream_t s) {
  const long long n = (long long)H * W;
  const double* src = in;
  if (prefilter) {
    hipLaunchKernelGGL(k_stage_blur_rows, dim3(nblk(n, 256)), dim3(256), 0, s, in, tmp, H, W, k[0], k[1], k[2]);
    hipLaunchKernelGGL(k_stage_blur_cols, dim3(nblk(n, 256)), dim3(256), 0, s, tmp, tmp2, H, W, k[0], k[1]);
    src = tmp2;
  }
  if (!out) return hipGetLastError();  // blur only (the fractional-area caller resizes tmp2)
  hipLaunchKernelGGL(k_stage_area, dim3(nblk((long long)(H / sy) * (W / 2), 256)), dim3(256), 0, s, src, out, H, W,
                     sy);
  return hipGetLastError();
}

hipError_t stage_resize(const double* in, int h, int w, double* out, int H, int W, int nearest, hipStream_t s) {
  const double sy = 1.0 / ((double)H / h), sx = 1.0 / ((double)W / w);
  hipLaunchKernelGGL(k_stage_resize, dim3(nblk((long long)H * W, 256)), dim3(256), 0, s, in, h, w, out, H, W, sy, sx,
                     nearest);
  return hipGetLastError();
}

hipError_t stage_block(const double* in, double* out, long long n, int bs, int op, hipStream_t s) {
  if (bs == 16)
    hipLaunchKernelGGL(k_stage_block16, dim3(nblk(n, 16)), dim3(256), 0, s, in, out, n, op);
  else
    hipLaunchKernelGGL(k_stage_block, dim3(nblk(n, 8)), dim3(64), 0, s, in, out, n, op);
  return hipGetLastError();
}

hipError_t stage_quant(const void* in, const double* q, void* out, long long n, int dequant, int period,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_stage_quant, dim3(nblk(n, 256)), dim3(256), 0, s, in, q, out, n, dequant, period);
  return hipGetLastError();
}

}  // namespace jds
