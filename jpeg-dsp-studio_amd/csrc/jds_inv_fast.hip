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
//   * AAN IDCT (5 multiplies per 8-point line) with the AAN scales, the 1/8
//     normalisation and the +128 folded into the dequantisation (one fma per
//     coefficient: q * Qs[u][v], DC + 128);
//   * chroma shifted by -128 once per window sample, so the colour transform is
//     one fma per channel term (R = Y + 1.402 Cr', ...);
//   * the bilinear upsample as a vertical blend of the lane's 6 chroma columns
//     followed by shared 3/4 products (3 operations per pixel and plane).
// Every output value v_fast then differs from v_ref by at most
// E = K_LIN * Dmax + K_CONST, where Dmax bounds |q * Q| over the coefficients the
// tile reads (tools/inv_bound.py derives K_LIN / K_CONST rigorously for both
// operation orders, with every fused multiply-add counted as two roundings).
// If no integer lies within E of v_fast, trunc(clip(v_fast)) ==
// trunc(clip(v_ref)): the byte is certified.  Each lane tracks the smallest
// distance |v - rint(v)| over its samples and the largest |q|; a workgroup
// whose tile has any uncertain sample lists (frame, tile) and the exact kernel
// recomputes that whole tile afterwards (k_inv2_list).  On the bench's random
// frames E ~ 1e-8 and a tile is listed with probability ~1e-3; exact ties
// (flat or saturated regions whose reference value is an integer up to
// pocketfft noise) are always listed, so those tiles cost fast + exact.
//
// Work decomposition and LDS layout are k_inv2's (jds_inv_common.hpp): one
// workgroup per tile, chroma window (with the ring the upsample reaches into)
// in LDS, Y in registers, one lane per 8-pixel row, 24-byte stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_inv_common.hpp"

// every fusion the compiler forms is covered by the bound (two roundings per
// fused pair); reassociation stays off
#pragma clang fp contract(fast)

namespace jds {

// tools/inv_bound.py: e_fast + e_ref <= K_LIN * Dmax + K_CONST (x2 safety included)
constexpr double K_LIN = 1.126219e-12 * 1.01;
constexpr double K_CONST = 2.810569e-12 * 1.01;

// AAN scale factors a_k = sqrt(2) cos(k pi / 16), a_0 = 1 (correctly rounded)
__constant__ double c_aan[8] = {1.0,
                                0x1.63150b15e8536p+0,
                                0x1.4e7ae9144f0fcp+0,
                                0x1.2d062ef88e319p+0,
                                1.0,
                                0x1.92469c0dcf32dp-1,
                                0x1.1517a7bdb3895p-1,
                                0x1.1a855dec071b5p-2};
constexpr double F_SQ2 = 0x1.6a09e667f3bcdp+0;   // sqrt(2)
constexpr double F_A2C2 = 0x1.d906bcf328d46p+0;  // 2 cos(pi/8)
constexpr double F_K10 = 0x1.1517a7bdb3895p+0;   // 2 (cos(pi/8) - cos(3pi/8))
constexpr double F_K12 = 0x1.4e7ae9144f0fcp+1;   // 2 (cos(pi/8) + cos(3pi/8))

// One 8-point AAN IDCT line on scaled inputs (inputs pre-multiplied by
// a_u / sqrt(8) per axis; outputs are the orthonormal IDCT).  The operation
// sequence is the one tools/inv_bound.py::aan_line models.
__device__ __forceinline__ void aan8(double (&v)[8]) {
  const double t10 = v[0] + v[4], t11 = v[0] - v[4];
  const double t13 = v[2] + v[6];
  const double t12 = (v[2] - v[6]) * F_SQ2 - t13;
  const double e0 = t10 + t13, e3 = t10 - t13, e1 = t11 + t12, e2 = t11 - t12;
  const double z13 = v[5] + v[3], z10 = v[5] - v[3], z11 = v[1] + v[7], z12 = v[1] - v[7];
  const double o7 = z11 + z13;
  const double o11 = (z11 - z13) * F_SQ2;
  const double z5 = (z10 + z12) * F_A2C2;
  const double o10 = z5 - z12 * F_K10;
  const double o12 = z5 - z10 * F_K12;
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

// Axis-0 pass of column v of one block: dequantise with the folded table
// (DC + dc_add: 128 on column 0, 0 elsewhere), AAN, into the transpose buffer.
// dq tracks max |q| of the column.
__device__ __forceinline__ void fast_col(const Col16& in, const double* __restrict__ qs, int v, double dc_add,
                                         double* __restrict__ dst, double& dq) {
  double c[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const double qd = (double)in.q[r];
    dq = fmax(dq, fabs(qd));
    c[r] = qd * qs[r * 8 + v];
  }
  c[0] = c[0] + dc_add;
  aan8(c);
#pragma unroll
  for (int r = 0; r < 8; ++r) dst[tslot(r, v)] = c[r];
}

// Axis-1 pass of row u, clip to [0, 255] (dct_engine.py:27).
__device__ __forceinline__ void fast_row(const double* __restrict__ src, int u, double (&c)[8]) {
  const int sw = u & 3;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const double2 d = *reinterpret_cast<const double2*>(src + u * 8 + 2 * (p ^ sw));
    c[2 * p] = d.x;
    c[2 * p + 1] = d.y;
  }
  aan8(c);
#pragma unroll
  for (int k = 0; k < 8; ++k) c[k] = fmin(fmax(c[k], 0.0), 255.0);
}

// One plane's upsampled (chroma - 128) at the lane's 8 pixels (cv2
// INTER_LINEAR at an exact 2x scale: pixel 2m weights (1/4, 3/4) on chroma
// columns (m-1, m), pixel 2m+1 (3/4, 1/4) on (m, m+1); rows likewise with
// clamped indices; the two image-edge pixels copy the edge column).
template <int MODE>
__device__ __forceinline__ void chroma8_fast(const double* __restrict__ cw, const Geo& g, int x0, int cwx0, int wq,
                                             int wt, double (&C)[8]) {
  using I = Inv<MODE>;
  if constexpr (I::SX == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) C[k] = cw[wq * I::CWC + x0 + k - cwx0];
  } else {
    const int c0 = x0 / 2 - 1 - cwx0;
    double vb[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if constexpr (I::SY == 2)
        vb[j] = cw[wq * I::CWC + c0 + j] * 0.25 + cw[wt * I::CWC + c0 + j] * 0.75;
      else
        vb[j] = cw[wq * I::CWC + c0 + j];
    }
    double t[6];
#pragma unroll
    for (int j = 1; j < 5; ++j) t[j] = vb[j] * 0.75;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      C[2 * i] = vb[i] * 0.25 + t[i + 1];
      C[2 * i + 1] = vb[i + 2] * 0.25 + t[i + 1];
    }
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int kl = side == 0 ? (x0 == 0 ? 0 : -1) : (g.W - 1 - x0 < 8 ? g.W - 1 - x0 : -1);
      if (kl >= 0) {
        const int e = (side == 0 ? 0 : g.wc - 1) - cwx0;
        double v = cw[wq * I::CWC + e];
        if constexpr (I::SY == 2) v = v * 0.25 + cw[wt * I::CWC + e] * 0.75;
        // (pixels past the image's right edge take 0: their window columns may
        // be outside the written ring, and they are certified like the rest)
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = k == kl ? v : (side == 1 && k > kl ? 0.0 : C[k]);
      }
    }
  }
}

__device__ __forceinline__ uint32_t byte_cert(double v, double& dmin) {
  dmin = fmin(dmin, fabs(v - rint(v)));
  return (uint32_t)clampi((int)v, 0, 255);
}

// XTRA: 0 = RGB only; 1 = + exact integer SSE and luma SSE partials (sweeps),
// committed only for certified tiles (listed tiles are redone by k_inv2_list).
template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv<MODE>::NT) __attribute__((amdgpu_waves_per_eu(Inv<MODE>::WPE)))
k_inv_fast(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
           const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
           double* __restrict__ sse_y_part, uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount,
           const int in_div, const int fix_all) {
  using I = Inv<MODE>;
  __shared__ __attribute__((aligned(16))) double s_mid[I::MB * MS];
  __shared__ __attribute__((aligned(16))) double s_cw[2][I::CWR * I::CWC];
  __shared__ double s_qs[64];  // Q[u][v] * a_u * a_v / 8
  __shared__ double s_qmax;
  __shared__ double s_red[I::NT / 64], s_dmin[I::NT / 64], s_dq[I::NT / 64];
  __shared__ unsigned long long s_sse;

  const int tid = threadIdx.x, lv = tid & 7, lb = tid >> 3;
  const int frame = blockIdx.y, tile = blockIdx.x;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  if (tid < 64) {
    const double q = fq[frame].q[tid];
    s_qs[tid] = q * c_aan[tid >> 3] * c_aan[tid & 7] * 0.125;
    double m = q;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if (tid == 0) s_qmax = m;
  }
  if (XTRA && tid == 0) s_sse = 0ull;
  __syncthreads();

  double dq = 0.0;     // max |q| this lane read
  double dmin = 1.0;   // min distance of an output value to an integer
  const double dc_add = lv == 0 ? 128.0 : 0.0;

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
  Col16 lq;
  {
    int by, bx;
    const bool ok = luma_blk(0, by, bx);
    lq = load_col(cf, ((long long)by * g.nbx + bx) * 64, lv, ok);
  }
  if (tid < I::NCB * 8) {
    const int i = lb / I::CBC, j = lb - i * I::CBC;
    const int by = cby0 + i, bx = cbx0 + j;
    const bool bvalid = by >= 0 && bx >= 0 && by < g.ncy && bx < g.ncx;
    const bool need = !I::RY || (i == 0 ? lv == 7 : (i == I::CBR - 1 ? lv == 0 : true));
    const long long boff = ((long long)by * g.ncx + bx) * 64;
    Col16 cq = load_col(cf + g.off_cb, boff, lv, bvalid);
#pragma unroll 1
    for (int p = 0; p < 2; ++p) {
      const Col16 cur = cq;
      if (p == 0) cq = load_col(cf + g.off_cr, boff, lv, bvalid);
      if (bvalid) {
        fast_col(cur, s_qs, lv, dc_add, s_mid + lb * MS, dq);
        if (need) {
          double c[8];
          fast_row(s_mid + lb * MS, lv, c);
          double* w = &s_cw[p][(by * 8 + lv - cwy0) * I::CWC];
          const int wc0 = bx * 8 - cwx0;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if ((unsigned)(wc0 + k) < (unsigned)I::CWC) w[wc0 + k] = c[k] - 128.0;
        }
      }
    }
  }
  __syncthreads();

  // ---- 2. luma rounds: IDCT, upsample, colour, certify, store ----------------
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = XTRA ? rgb_in + (size_t)(frame / in_div) * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
#pragma unroll 1
  for (int r = 0; r < I::NYB / I::RB; ++r) {
    int by, bx;
    const bool bvalid = luma_blk(r, by, bx);
    const Col16 cur = lq;
    if (r + 1 < I::NYB / I::RB) {
      int by1, bx1;
      const bool ok1 = luma_blk(r + 1, by1, bx1);
      lq = load_col(cf, ((long long)by1 * g.nbx + bx1) * 64, lv, ok1);
    }
    if (bvalid) fast_col(cur, s_qs, lv, dc_add, s_mid + lb * MS, dq);
    const int y = by * 8 + lv, x0 = bx * 8;
    if (bvalid && y < g.H && x0 < g.W) {
      double Yv[8];
      fast_row(s_mid + lb * MS, lv, Yv);
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
      uint32_t pk[6] = {0u, 0u, 0u, 0u, 0u, 0u};
      {
        double C[8], Gt[8];
        chroma8_fast<MODE>(s_cw[0], g, x0, cwx0, wq, wt, C);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double B = Yv[k] + C[k] * 1.772;
          Gt[k] = Yv[k] + C[k] * -0.344136;
          const int b = 3 * k + 2;
          const uint32_t ub = byte_cert(B, dmin);
          pk[b >> 2] |= ub << (8 * (b & 3));
        }
        chroma8_fast<MODE>(s_cw[1], g, x0, cwx0, wq, wt, C);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double R = Yv[k] + C[k] * 1.402;
          const double G = Gt[k] + C[k] * -0.714136;
          const int b = 3 * k;
          const uint32_t ur = byte_cert(R, dmin), ug = byte_cert(G, dmin);
          pk[b >> 2] |= ur << (8 * (b & 3));
          pk[(b + 1) >> 2] |= ug << (8 * ((b + 1) & 3));
        }
      }
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
        // reference PSNR inputs (utils/metrics.py:11-20): exact integer SSE,
        // fp64 luma of both uint8 images (jds_inv.hip k_inv2's XTRA = 1 terms)
        uint32_t in[6] = {0u, 0u, 0u, 0u, 0u, 0u};
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
        auto byte_of = [](const uint32_t (&w)[6], int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 255u); };
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < nx) {
            const int b = 3 * k;
            const int o0 = byte_of(in, b), o1 = byte_of(in, b + 1), o2 = byte_of(in, b + 2);
            const int ur = byte_of(pk, b), ug = byte_of(pk, b + 1), ub = byte_of(pk, b + 2);
            const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
            sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
            {
#pragma clang fp contract(off)
              const double yo = luma((double)o0, (double)o1, (double)o2);
              const double yr = luma((double)ur, (double)ug, (double)ub);
              const double dy = yo - yr;
              ssy = ssy + dy * dy;
            }
          }
        }
      }
    }
  }

  // ---- 3. certification: the tile's smallest distance vs its bound -----------
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    dmin = fmin(dmin, __shfl_xor(dmin, o, 64));
    dq = fmax(dq, __shfl_xor(dq, o, 64));
  }
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
  if ((tid & 63) == 0) {
    s_dmin[tid >> 6] = dmin;
    s_dq[tid >> 6] = dq;
  }
  __syncthreads();
  if (tid == 0) {
    double m = 1.0, q = 0.0;
    for (int i = 0; i < I::NT / 64; ++i) {
      m = fmin(m, s_dmin[i]);
      q = fmax(q, s_dq[i]);
    }
    const double E = K_LIN * (q * s_qmax) + K_CONST;
    if (m <= E || fix_all) {
      const unsigned slot = atomicAdd(fixcount, 1u);
      fixlist[slot] = make_uint2((unsigned)frame, (unsigned)tile);
    } else if constexpr (XTRA > 0) {
      double a = 0.0;
      for (int i = 0; i < I::NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * gridDim.x + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, s_sse);
    }
  }
}

// ------------------------------------------------------------ launchers --

hipError_t launch_inv2_list(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                            const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                            const uint2* list, const unsigned* count, hipStream_t s, int in_div);

template <int MODE>
static hipError_t inv_fast_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq, const uint8_t* rgb_in,
                             uint8_t* rgb_out, jds_frame_stats* st, double* part, const InvFix& fx, hipStream_t s,
                             int in_div) {
  const int ty = (g.H + Inv<MODE>::TH - 1) / Inv<MODE>::TH, tx = (g.W + Inv<MODE>::TW - 1) / Inv<MODE>::TW;
  const dim3 grid(ty * tx, n), blk(Inv<MODE>::NT);
  hipError_t e = hipMemsetAsync(fx.count, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  if (rgb_in)
    hipLaunchKernelGGL((k_inv_fast<MODE, 1>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part,
                       fx.list, fx.count, in_div, fx.fix_all);
  else
    hipLaunchKernelGGL((k_inv_fast<MODE, 0>), grid, blk, 0, s, g, tx, coeffs, fq, nullptr, rgb_out, st, part,
                       fx.list, fx.count, in_div, fx.fix_all);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return launch_inv2_list(MODE, g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx.list, fx.count, s, in_div);
}

hipError_t launch_inv_fast(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                           const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                           const InvFix& fx, hipStream_t s, int in_div) {
  switch (mode) {
    case M420: return inv_fast_t<M420>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx, s, in_div);
    case M422: return inv_fast_t<M422>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx, s, in_div);
    default: return inv_fast_t<M444>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, fx, s, in_div);
  }
}

}  // namespace jds
