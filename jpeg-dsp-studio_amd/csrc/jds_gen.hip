// jds_gen.hip — the general-geometry path: frames whose chroma subsampling is
// not an exact 2x (odd H with 4:2:0, odd W with 4:2:2 / 4:2:0).  There the
// reference's cv2.resize(..., INTER_AREA) (engines/color_space.py:42-49) takes
// OpenCV's fractional-area path (computeResizeAreaTab + resizeArea_: each
// chroma sample is a weighted sum over 2-4 source rows and columns with float
// weights), and the INTER_LINEAR upsample back to H x W
// (engines/color_space.py:63-65) has non-2x weights.  Everything stays fp64 in
// the reference's operation order (FP contraction off), so coefficients and
// bytes are bit-identical, as on the tiled path.
//
// Stages (per frame / item; planes in HBM scratch, not a throughput path):
//   k_gen_sub   RGB -> prefiltered (cv2 GaussianBlur) full-resolution chroma,
//               evaluated on the fly -> fractional INTER_AREA -> fp64 Cb/Cr
//               planes hc x wc                       (color_space.py:27-53)
//   k_gen_fwd   every 8x8 block: luma from RGB, chroma from the planes, np.pad
//               reflect, level shift, pocketfft DCT-II, round-half-even of c/Q,
//               statistics, selected block          (pipeline.py:47-63,99-151)
//   k_gen_idct  every block: dequantize, pocketfft DCT-III, +128, clip, merge +
//               crop into fp64 planes (Y: H x W, Cb/Cr: hc x wc) (pipeline.py:68-82)
//   k_gen_px    per pixel: cv2 INTER_LINEAR chroma, YCbCr -> RGB, clip,
//               truncate; SSE, IntermediateData error maps (pipeline.py:88-121)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "jds_dct8.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int GEN_NT = 256;  // threads per workgroup (32 blocks of 8 lanes in the block kernels)

// Full-resolution chroma sample (plane 1 = Cb, 2 = Cr) at an in-image pixel.
__device__ __forceinline__ double gen_chroma(const uint8_t* img, const Geo& g, int y, int x, int plane) {
  const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
  const double R = p[0], G = p[1], B = p[2];
  return plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B);
}

// cv2 RowFilter<double>: t = k0*S[x-1]; t += k1*S[x]; t += k2*S[x+1] (BORDER_REFLECT_101)
__device__ double gen_row(const uint8_t* img, const Geo& g, int y, int x, int plane, const double* k) {
  double t = k[0] * gen_chroma(img, g, y, reflect101(x - 1, g.W), plane);
  t = t + k[1] * gen_chroma(img, g, y, x, plane);
  return t + k[2] * gen_chroma(img, g, y, reflect101(x + 1, g.W), plane);
}

// The (optionally GaussianBlur-ed) chroma plane the area resize reads, at pixel (y, x).
// SymmColumnFilter<double>: d = k1*T[y] + 0; d += k0*(T[y+1] + T[y-1]).
template <bool PF>
__device__ double gen_src(const uint8_t* img, const Geo& g, int y, int x, int plane, const double* k) {
  if constexpr (PF) {
    const double d = k[1] * gen_row(img, g, y, x, plane, k) + 0.0;
    return d + k[0] * (gen_row(img, g, reflect101(y + 1, g.H), x, plane, k) +
                       gen_row(img, g, reflect101(y - 1, g.H), x, plane, k));
  } else {
    return gen_chroma(img, g, y, x, plane);
  }
}

// resizeArea_<double, double> for one destination sample: per source row of the
// y table, buf = 0; buf += S[si]*alpha over the x table; sum = 0 + beta*buf for
// the first row, sum += beta*buf for the others (table order throughout).
// With an integer scale on both axes (fy, fx > 0) cv2 takes resizeAreaFast
// instead: the fy x fx window from (cy*fy, cx*fx) in row-major order, summed from
// 0 in groups of four (sum += ((s0 + s1) + s2) + s3), the rest one by one, times
// the float 1.f/area.
template <typename Src>
__device__ __forceinline__ double area_sample(const AreaTap& ty, const AreaTap& tx, int cy, int cx, int fy, int fx,
                                              Src src) {
  if (fy > 0) {
    const int area = fy * fx;
    double sum = 0.0;
    int k = 0;
#pragma unroll 1
    for (; k <= area - 4; k += 4) {
      double g4 = src(cy * fy + k / fx, cx * fx + k % fx) + src(cy * fy + (k + 1) / fx, cx * fx + (k + 1) % fx);
      g4 = g4 + src(cy * fy + (k + 2) / fx, cx * fx + (k + 2) % fx);
      g4 = g4 + src(cy * fy + (k + 3) / fx, cx * fx + (k + 3) % fx);
      sum = sum + g4;
    }
#pragma unroll 1
    for (; k < area; ++k) sum = sum + src(cy * fy + k / fx, cx * fx + k % fx);
    return sum * (double)(1.f / (float)area);
  }
  double sum = 0.0;
#pragma unroll 1
  for (int j = 0; j < ty.n; ++j) {
    double buf = 0.0;
#pragma unroll 1
    for (int i = 0; i < tx.n; ++i) buf = buf + src(ty.si[j], tx.si[i]) * tx.a[i];
    sum = sum + ty.a[j] * buf;
  }
  return sum;
}

// sub: [frame][Cb | Cr][hc][wc] fp64
template <bool PF>
__global__ void __launch_bounds__(GEN_NT)
k_gen_sub(const Geo g, const uint8_t* __restrict__ rgb, const AreaTap* __restrict__ ytab,
          const AreaTap* __restrict__ xtab, const double* __restrict__ gk, double* __restrict__ sub) {
  const long long i = (long long)blockIdx.x * GEN_NT + threadIdx.x;
  const long long npl = (long long)g.hc * g.wc;
  if (i >= npl) return;
  const int frame = blockIdx.y;
  const int cy = (int)(i / g.wc), cx = (int)(i - (long long)cy * g.wc);
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  const double k[3] = {gk[0], gk[1], gk[2]};
  const AreaTap ty = ytab[cy], tx = xtab[cx];
  double* out = sub + (size_t)frame * 2 * npl;
#pragma unroll 1
  for (int p = 1; p <= 2; ++p)
    out[(p - 1) * npl + i] =
        area_sample(ty, tx, cy, cx, g.afy, g.afx, [&](int y, int x) { return gen_src<PF>(img, g, y, x, p, k); });
}

// Block b of a frame's coefficient array -> (plane, gy, gx); false past the end.
__device__ __forceinline__ bool gen_block(const Geo& g, long long b, int& plane, int& gy, int& gx) {
  const long long nyb = (long long)g.nby * g.nbx, ncb = (long long)g.ncy * g.ncx;
  if (b >= nyb + 2 * ncb) return false;
  long long r = b;
  plane = 0;
  if (r >= nyb) {
    r -= nyb;
    plane = 1 + (int)(r / ncb);
    r -= (plane - 1) * ncb;
  }
  const int nbx = plane ? g.ncx : g.nbx;
  gy = (int)(r / nbx);
  gx = (int)(r - (long long)gy * nbx);
  return true;
}

// One workgroup = 32 blocks x 8 lanes; lane `line` forms column `line` of its
// block, DCT along axis 0, transposes through LDS, then owns row u = line:
// DCT along axis 1, quantise, statistics, one 16-byte store.
__global__ void __launch_bounds__(GEN_NT)
k_gen_fwd(const Geo g, const uint8_t* __restrict__ rgb, const double* __restrict__ sub,
          int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq, jds_frame_stats* __restrict__ st,
          jds_selected_block* __restrict__ sel, int sel_blk, int in_div) {
  __shared__ double s_blk[GEN_NT / 8][65];
  __shared__ unsigned s_hist[50];
  __shared__ unsigned s_acc[2];
  const int tid = threadIdx.x, lb = tid >> 3, line = tid & 7;
  const int item = blockIdx.y, frame = item / in_div;
  if (tid < 50) s_hist[tid] = 0u;
  if (tid < 2) s_acc[tid] = 0u;
  const long long b = (long long)blockIdx.x * (GEN_NT / 8) + lb;
  int plane = 0, gy = 0, gx = 0;
  const bool valid = gen_block(g, b, plane, gy, gx);
  const bool is_sel = sel != nullptr && valid && plane == 0 && item == 0 && b == sel_blk;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
  const long long npl = (long long)g.hc * g.wc;
  double v[8];
  if (valid) {
    if (plane == 0) {
      const int x = reflect_pad(gx * 8 + line, g.W);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint8_t* p = img + ((size_t)reflect_pad(gy * 8 + i, g.H) * g.W + x) * 3;
        v[i] = luma((double)p[0], (double)p[1], (double)p[2]);
      }
    } else {
      const double* pl = sub + (size_t)frame * 2 * npl + (plane - 1) * npl;
      const int x = reflect_pad(gx * 8 + line, g.wc);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = pl[(size_t)reflect_pad(gy * 8 + i, g.hc) * g.wc + x];
    }
    if (is_sel) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sel->original[i * 8 + line] = v[i];
        sel->shifted[i * 8 + line] = v[i] - 128.0;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = v[i] - 128.0;  // dct_engine.py:19
    dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
    for (int i = 0; i < 8; ++i) s_blk[lb][i * 8 + line] = v[i];
  }
  __syncthreads();
  unsigned nz = 0u, mb = 0u;
  if (valid) {
    const int u = line;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s_blk[lb][u * 8 + k];
    dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    int q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      q[k] = (int)__builtin_rint(v[k] / fq[item].q16[u * 8 + k]);  // quantizer.py:22-24
      const int m = q[k] < 0 ? -q[k] : q[k];
      if (m) {
        ++nz;
        mb += 33 - __clz(m);  // ceil(log2(m+1)) + 1 (utils/metrics.py:78)
        if (q[k] >= -100 && q[k] <= 100) atomicAdd(&s_hist[q[k] == 100 ? 49 : (q[k] + 100) >> 2], 1u);
      }
    }
    if (is_sel) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sel->dct[u * 8 + k] = v[k] * 0.0625;
        sel->quantized[u * 8 + k] = (int16_t)q[k];
      }
    }
    uint4 pk;
    pk.x = (uint32_t)(uint16_t)q[0] | ((uint32_t)(uint16_t)q[1] << 16);
    pk.y = (uint32_t)(uint16_t)q[2] | ((uint32_t)(uint16_t)q[3] << 16);
    pk.z = (uint32_t)(uint16_t)q[4] | ((uint32_t)(uint16_t)q[5] << 16);
    pk.w = (uint32_t)(uint16_t)q[6] | ((uint32_t)(uint16_t)q[7] << 16);
    *reinterpret_cast<uint4*>(coeffs + (size_t)item * g.cpf + b * 64 + u * 8) = pk;
  }
  nz = (unsigned)wave_sum((int)nz);
  mb = (unsigned)wave_sum((int)mb);
  if ((tid & 63) == 0) {
    atomicAdd(&s_acc[0], nz);
    atomicAdd(&s_acc[1], mb);
  }
  __syncthreads();
  jds_frame_stats* fs = st + item;
  if (tid == 0) {
    if (s_acc[0]) atomicAdd((unsigned long long*)&fs->nonzero, (unsigned long long)s_acc[0]);
    if (s_acc[1]) atomicAdd((unsigned long long*)&fs->magnitude_bits, (unsigned long long)s_acc[1]);
  }
  if (tid < 50 && s_hist[tid]) atomicAdd((unsigned long long*)&fs->hist[tid], (unsigned long long)s_hist[tid]);
}

// rec: [item][Y H x W | Cb hc x wc | Cr hc x wc] fp64, merged and cropped
// (block_processor.py:34-48, pipeline.py:80-82)
__global__ void __launch_bounds__(GEN_NT)
k_gen_idct(const Geo g, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq, double* __restrict__ rec,
           jds_selected_block* __restrict__ sel, int sel_blk) {
  __shared__ double s_blk[GEN_NT / 8][65];
  const int tid = threadIdx.x, lb = tid >> 3, line = tid & 7;
  const int item = blockIdx.y;
  const long long b = (long long)blockIdx.x * (GEN_NT / 8) + lb;
  int plane = 0, gy = 0, gx = 0;
  const bool valid = gen_block(g, b, plane, gy, gx);
  const int16_t* cf = coeffs + (size_t)item * g.cpf + b * 64;
  double c[8];
  if (valid) {
#pragma unroll
    for (int r = 0; r < 8; ++r) c[r] = (double)cf[r * 8 + line] * fq[item].q[r * 8 + line];  // quantizer.py:27-29
    dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);  // axis 0 (dct_engine.py:12-14)
#pragma unroll
    for (int r = 0; r < 8; ++r) s_blk[lb][r * 8 + line] = c[r];
  }
  __syncthreads();
  if (!valid) return;
  const int u = line;
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = s_blk[lb][u * 8 + k];
  dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double s = c[k] * 0.0625 + 128.0;  // fct 1/16 (exact), +128 (dct_engine.py:25-26)
    c[k] = fmin(fmax(s, 0.0), 255.0);
  }
  if (sel != nullptr && item == 0 && plane == 0 && b == sel_blk) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sel->reconstructed[u * 8 + k] = c[k];
  }
  const int ph = plane ? g.hc : g.H, pw = plane ? g.wc : g.W;
  const int y = gy * 8 + u;
  if (y >= ph) return;
  double* dst = rec + (size_t)item * ((size_t)g.H * g.W + 2 * (size_t)g.hc * g.wc) +
                (plane == 0 ? 0 : (size_t)g.H * g.W + (size_t)(plane - 1) * g.hc * g.wc) + (size_t)y * pw;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (gx * 8 + k < pw) dst[gx * 8 + k] = c[k];
}

// cv2 INTER_LINEAR (resizeGeneric, 64F) of a cropped hc x wc plane at pixel (y, x):
// HResizeLinear with clamped taps (copy past xmax), VResizeLinear with clipped rows.
__device__ __forceinline__ double gen_upsample(const double* __restrict__ pl, const Geo& g, int r0, int r1, double b0,
                                               double b1, int sx, bool copy, double a0, double a1) {
  const double* s0 = pl + (size_t)r0 * g.wc + sx;
  const double* s1 = pl + (size_t)r1 * g.wc + sx;
  double h0, h1;
  if (copy) {
    h0 = s0[0] * 1.0;
    h1 = s1[0] * 1.0;
  } else {
    h0 = s0[0] * a0 + s0[1] * a1;
    h1 = s1[0] * a0 + s1[1] * a1;
  }
  return h0 * b0 + h1 * b1;
}

// One thread per pixel.  XTRA: 0 = RGB only, 1 = + SSE (exact integer) and a
// deterministic luma-SSE partial per workgroup, 2 = + IntermediateData error maps.
template <int XTRA>
__global__ void __launch_bounds__(GEN_NT)
k_gen_px(const Geo g, const double* __restrict__ rec, const uint8_t* __restrict__ rgb_in,
         uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st, double* __restrict__ sse_y_part,
         double* __restrict__ err_y, double* __restrict__ err_rgb, int in_div) {
  __shared__ double s_red[GEN_NT / 64];
  __shared__ unsigned long long s_sse;
  const int tid = threadIdx.x, item = blockIdx.y;
  if (XTRA && tid == 0) s_sse = 0ull;
  if (XTRA) __syncthreads();
  const long long i = (long long)blockIdx.x * GEN_NT + tid;
  const long long npx = (long long)g.H * g.W;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  if (i < npx) {
    const int y = (int)(i / g.W), x = (int)(i - (long long)y * g.W);
    const double* base = rec + (size_t)item * ((size_t)npx + 2 * (size_t)g.hc * g.wc);
    const double Y = base[i];
    // color_space.py:63-65: cv2.resize(c, (W, H), INTER_LINEAR); scale = 1 / (dst / src)
    float fy = (float)((y + 0.5) * g.up_sy - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const double b0 = (double)(1.f - fy), b1 = (double)fy;
    const int r0 = clampi(sy, 0, g.hc - 1), r1 = clampi(sy + 1, 0, g.hc - 1);
    float fx = (float)((x + 0.5) * g.up_sx - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { sx = 0; fx = 0.f; }
    const bool copy = sx + 1 >= g.wc;
    if (sx >= g.wc - 1) { sx = g.wc - 1; fx = 0.f; }
    const double a0 = (double)(1.f - fx), a1 = (double)fx;
    const double Cb = gen_upsample(base + npx, g, r0, r1, b0, b1, sx, copy, a0, a1);
    const double Cr = gen_upsample(base + npx + (long long)g.hc * g.wc, g, r0, r1, b0, b1, sx, copy, a0, a1);
    // engines/color_space.py:17-24, then clip and astype(uint8) (pipeline.py:93-95)
    double R = Y + 1.402 * (Cr - 128.0);
    double G = Y - 0.344136 * (Cb - 128.0) - 0.714136 * (Cr - 128.0);
    double B = Y + 1.772 * (Cb - 128.0);
    R = fmin(fmax(R, 0.0), 255.0);
    G = fmin(fmax(G, 0.0), 255.0);
    B = fmin(fmax(B, 0.0), 255.0);
    const int ur = (int)R, ug = (int)G, ub = (int)B;
    uint8_t* o = rgb_out + ((size_t)item * npx + i) * 3;
    o[0] = (uint8_t)ur;
    o[1] = (uint8_t)ug;
    o[2] = (uint8_t)ub;
    if constexpr (XTRA > 0) {
      const uint8_t* p = rgb_in + ((size_t)(item / in_div) * npx + i) * 3;
      const int o0 = p[0], o1 = p[1], o2 = p[2];
      const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
      sse = (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
      const double R0 = (double)o0, G0 = (double)o1, B0 = (double)o2;
      const double yo = luma(R0, G0, B0);
      ssy = luma_sse_e6(d0, d1, d2);
      if constexpr (XTRA > 1) {
        err_y[i] = fabs(yo - Y);                                             // pipeline.py:119-120
        err_rgb[i] = ((fabs(R0 - R) + fabs(G0 - G)) + fabs(B0 - B)) / 3.0;  // pipeline.py:121
      }
    }
  }
  if constexpr (XTRA > 0) {
    unsigned long long s = sse;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) atomicAdd(&s_sse, s);
    double d = ssy;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = d + __shfl_xor(d, o, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
    __syncthreads();
    if (tid == 0) {
      double a = 0.0;
      for (int w = 0; w < GEN_NT / 64; ++w) a = a + s_red[w];
      sse_y_part[(size_t)item * gridDim.x + blockIdx.x] = a;
      atomicAdd((unsigned long long*)&st[item].sse_rgb, s_sse);
    }
  }
}

// Per-stage API (jds_stage_subsample) on an fp64 plane that is already
// blurred (or raw): fractional INTER_AREA into h_out x w_out.
__global__ void __launch_bounds__(GEN_NT)
k_stage_area_gen(const double* __restrict__ in, int W, const AreaTap* __restrict__ ytab,
                 const AreaTap* __restrict__ xtab, double* __restrict__ out, int oh, int ow, int fy, int fx) {
  const long long i = (long long)blockIdx.x * GEN_NT + threadIdx.x;
  if (i >= (long long)oh * ow) return;
  const int cy = (int)(i / ow), cx = (int)(i - (long long)cy * ow);
  out[i] = area_sample(ytab[cy], xtab[cx], cy, cx, fy, fx, [&](int y, int x) { return in[(size_t)y * W + x]; });
}

// ------------------------------------------------------------ host side --

// OpenCV computeResizeAreaTab for one axis (src -> dst samples), grouped per
// destination index.  Returns the largest tap count, or -1 if one exceeds 4.
int area_tab_build(int src, int dst, AreaTap* tab) {
  const double scale = 1.0 / ((double)dst / (double)src);  // cv::hal::resize: 1 / inv_scale
  int most = 0;
  for (int dx = 0; dx < dst; ++dx) {
    AreaTap& t = tab[dx];
    t.n = 0;
    t.pad = 0;
    auto push = [&](int si, float a) {
      if (t.n < 4) {
        t.si[t.n] = si;
        t.a[t.n] = (double)a;
      }
      ++t.n;
    };
    const double fsx1 = dx * scale;
    const double fsx2 = fsx1 + scale;
    const double cell = std::min(scale, src - fsx1);
    int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
    sx2 = std::min(sx2, src - 1);
    sx1 = std::min(sx1, sx2);
    if (sx1 - fsx1 > 1e-3) push(sx1 - 1, (float)((sx1 - fsx1) / cell));
    for (int sx = sx1; sx < sx2; ++sx) push(sx, (float)(1.0 / cell));
    if (fsx2 - sx2 > 1e-3) push(sx2, (float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell));
    if (t.n > 4) return -1;
    most = std::max(most, t.n);
  }
  return most;
}

hipError_t stage_area_gen(const double* in, int H, int W, const AreaTap* ytab, const AreaTap* xtab, double* out,
                          int oh, int ow, hipStream_t s) {
  const long long n = (long long)oh * ow;
  int fy, fx;
  area_fast_scales(H, oh, W, ow, &fy, &fx);
  hipLaunchKernelGGL(k_stage_area_gen, dim3((unsigned)((n + GEN_NT - 1) / GEN_NT)), dim3(GEN_NT), 0, s, in, W, ytab,
                     xtab, out, oh, ow, fy, fx);
  return hipGetLastError();
}

size_t gen_sub_doubles(const Geo& g) { return 2 * (size_t)g.hc * g.wc; }
size_t gen_rec_doubles(const Geo& g) { return (size_t)g.H * g.W + 2 * (size_t)g.hc * g.wc; }
int gen_px_tiles(const Geo& g) { return (int)(((long long)g.H * g.W + GEN_NT - 1) / GEN_NT); }

hipError_t launch_fwd_finish(const Geo& g, int n, jds_frame_stats* st, const uint32_t* part, int ptiles,
                             hipStream_t s);

// phases: bit 0 forward (sub, fwd, finish), bit 1 inverse (idct, px, finalize).
// tabs = [ytab (hc) | xtab (wc)]; sub = n / in_div frames of gen_sub_doubles;
// rec = n items of gen_rec_doubles; part = n x gen_px_tiles doubles.
hipError_t launch_gen(bool pf, const Geo& g, int n, int in_div, const uint8_t* rgb, uint8_t* rgb_out,
                      int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st, double* part,
                      bool want_sse, double* err_y, double* err_rgb, jds_selected_block* sel, int sel_blk,
                      const AreaTap* tabs, double* sub, double* rec, hipStream_t s, hipEvent_t* ev, int phases) {
  hipError_t e;
  const long long nblk = g.cpf / 64;
  const unsigned bgrid = (unsigned)((nblk + GEN_NT / 8 - 1) / (GEN_NT / 8));
  if (phases & 1) {
    if (ev && (e = hipEventRecord(ev[0], s)) != hipSuccess) return e;
    const int nf = n / in_div;
    const dim3 sgrid((unsigned)(((long long)g.hc * g.wc + GEN_NT - 1) / GEN_NT), nf);
    if (pf)
      hipLaunchKernelGGL(k_gen_sub<true>, sgrid, dim3(GEN_NT), 0, s, g, rgb, tabs, tabs + g.hc, gk, sub);
    else
      hipLaunchKernelGGL(k_gen_sub<false>, sgrid, dim3(GEN_NT), 0, s, g, rgb, tabs, tabs + g.hc, gk, sub);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_gen_fwd, dim3(bgrid, n), dim3(GEN_NT), 0, s, g, rgb, sub, coeffs, fq, st, sel, sel_blk,
                       in_div);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_fwd_finish(g, n, st, nullptr, 0, s)) != hipSuccess) return e;
    if (ev && (e = hipEventRecord(ev[1], s)) != hipSuccess) return e;
  }
  if (phases & 2) {
    hipLaunchKernelGGL(k_gen_idct, dim3(bgrid, n), dim3(GEN_NT), 0, s, g, coeffs, fq, rec, sel, sel_blk);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int tiles = gen_px_tiles(g);
    const dim3 pgrid(tiles, n);
    if (err_y)
      hipLaunchKernelGGL(k_gen_px<2>, pgrid, dim3(GEN_NT), 0, s, g, rec, rgb, rgb_out, st, part, err_y, err_rgb,
                         in_div);
    else if (want_sse)
      hipLaunchKernelGGL(k_gen_px<1>, pgrid, dim3(GEN_NT), 0, s, g, rec, rgb, rgb_out, st, part, nullptr, nullptr,
                         in_div);
    else
      hipLaunchKernelGGL(k_gen_px<0>, pgrid, dim3(GEN_NT), 0, s, g, rec, nullptr, rgb_out, st, part, nullptr,
                         nullptr, in_div);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ev && (e = hipEventRecord(ev[2], s)) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace jds
