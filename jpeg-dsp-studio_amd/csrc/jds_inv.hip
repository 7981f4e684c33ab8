// jds_inv.hip — the inverse half of the codec path on gfx950:
// int16 coefficients -> dequantize -> 2-D IDCT -> clip -> chroma upsample ->
// YCbCr->RGB -> clip -> truncate -> uint8 RGB.  Reference:
// engines/pipeline.py:77-95 (dequantize, idct_2d, merge_blocks, upsample_chroma,
// ycbcr_to_rgb, clip/astype) with quantizer.py:27-29, dct_engine.py:17-27,
// color_space.py:17-24 and :63-65.  Every operation is fp64 in the
// reference's order (pocketfft DCT-III butterflies, cv2 INTER_LINEAR taps,
// NumPy colour expressions), FP contraction off: bytes are bit-identical.
//
// Work decomposition (one workgroup per TH x TW pixel tile, tiles laid from the
// top-left corner):
//   1. chroma, both planes: the tile's chroma blocks plus the ring the
//      bilinear upsample reaches into.  Column (axis-0) passes run one thread
//      per block column, straight from the int16 coefficients in HBM/L2 into
//      an fp64 transpose buffer; row (axis-1) passes run on the same 8 threads
//      (lanes of one wave: no barrier) for the block rows the window needs (a
//      top/bottom ring block contributes one row), into an fp64 LDS window.
//      One workgroup barrier completes the window.
//   2. luma, NT/8 blocks per round: the same column pass, then each thread
//      owns one 8-pixel block row: row IDCT -> Y in registers, chroma taps from
//      the LDS window, colour, clip, truncate, one 24-byte store.  Again
//      wave-local: no barriers.
// Y never goes through LDS.  The upsample shares products between
// neighbouring pixels (same IEEE operations, same results).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct8.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_inv_common.hpp"

#pragma clang fp contract(off)

namespace jds {

// Dequantize (quantizer.py:27-29) and IDCT column v of a block (axis 0 first,
// dct_engine.py:12-14) into dst[r*8 + v].  `qi` holds the integer table Q:
// q*Q is formed exactly in 24-bit integer arithmetic and converted once.  The
// transform then runs on 16x the reference's operands (pocketfft's first-axis
// fct = 1/16 not applied): scaling by 2^4 commutes exactly with every rounding
// (no subnormals or overflow arise), so the row pass's outputs are exactly
// 16x the reference's and idct_row folds the 1/16 into its +128 (one fma).
__device__ __forceinline__ void idct_col(const int16_t* __restrict__ blk, const int* __restrict__ qi, int v,
                                         double* __restrict__ dst) {
  double c[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) c[r] = (double)__mul24((int)blk[r * 8 + v], qi[r * 8 + v]);
  dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
  for (int r = 0; r < 8; ++r) dst[tslot(r, v)] = c[r];
}

__device__ __forceinline__ void idct_col(const Col16& in, const int* __restrict__ qi, int v,
                                         double* __restrict__ dst) {
  double c[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) c[r] = (double)__mul24((int)in.q[r], qi[r * 8 + v]);
  dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
  for (int r = 0; r < 8; ++r) dst[tslot(r, v)] = c[r];
}

// Row u of a column-transformed block: axis-1 IDCT, fct 1/16 and +128 in one
// fma (x/16 is exact, so fl(x/16 + 128) == fl(fl(x/16) + 128)), clip
// (dct_engine.py:23-27).
__device__ __forceinline__ void idct_row(const double* __restrict__ src, int u, double (&c)[8]) {
  const int sw = u & 3;
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // pair p of row u (tslot), one 16-B read
    const double2 d = *reinterpret_cast<const double2*>(src + u * 8 + 2 * (p ^ sw));
    c[2 * p] = d.x;
    c[2 * p + 1] = d.y;
  }
  dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double s = fma(c[k], 0.0625, 128.0);
    c[k] = fmin(fmax(s, 0.0), 255.0);
  }
}

// One plane's upsampled chroma at 8 consecutive pixels of one output row (cv2
// INTER_LINEAR, color_space.py:63-65; or the co-sited sample without
// subsampling): horizontal taps on chroma rows wr0 (and wr1), then the
// vertical blend.  Horizontal subsampling implies an even width (the C-ABI
// rejects odd ones), so the scale is exactly 1/2: pixel 2m reads
// (s[m-1], s[m]) with weights (1/4, 3/4) and pixel 2m+1 reads (s[m], s[m+1])
// with (3/4, 1/4), so each product serves two pixels.
// cv2's vertical blend r0*b0 + r1*b1 for an exact 2x upsample has weights
// {1/4, 3/4} in one order or the other: with wq the window row weighted 1/4 and
// wt the row weighted 3/4 it is fl(fl(h[wq]/4) + fl(h[wt]*3/4)), and the
// quarter product is exact, so one fma reproduces the reference's two
// roundings.  Picking the rows per thread (not the weights per pixel) keeps
// the blend free of selects.
__device__ __forceinline__ double vblend(double hq, double ht) { return fma(hq, 0.25, ht * 0.75); }

template <int MODE>
__device__ __forceinline__ void chroma8(const double* __restrict__ cw, const Geo& g, int x0, int cwx0, int wq,
                                        int wt, double (&C)[8]) {
  using I = Inv<MODE>;
  if constexpr (I::SX == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) C[k] = cw[wq * I::CWC + x0 + k - cwx0];
  } else {
    const int c0 = x0 / 2 - 1 - cwx0;
    double h0[8];
#pragma unroll
    for (int rr = 0; rr < (I::SY == 2 ? 2 : 1); ++rr) {
      const double* s = &cw[(rr ? wt : wq) * I::CWC + c0];
      // s*0.25 is exact, so fl(s0*0.25 + fl(s1*0.75)) == fma(s0, 0.25, fl(s1*0.75))
      double q75[6];
#pragma unroll
      for (int j = 1; j < 5; ++j) q75[j] = s[j] * 0.75;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double e = fma(s[i], 0.25, q75[i + 1]), o = fma(s[i + 2], 0.25, q75[i + 1]);
        if (rr == 0) {
          h0[2 * i] = e;
          h0[2 * i + 1] = o;
        } else {
          C[2 * i] = vblend(h0[2 * i], e);
          C[2 * i + 1] = vblend(h0[2 * i + 1], o);
        }
      }
    }
    if constexpr (I::SY == 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) C[k] = h0[k];
    }
    // cv2's clamped taps at the two edge pixels: x = 0 has sx = -1 -> (s[0], 1.0,
    // s[1], 0.0) and x = W-1 has sx = wc-1 -> copy; both equal s[edge] exactly
    // (samples are finite and >= 0)
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int kl = side == 0 ? (x0 == 0 ? 0 : -1) : (g.W - 1 - x0 < 8 ? g.W - 1 - x0 : -1);
      if (kl >= 0) {
        const int e = (side == 0 ? 0 : g.wc - 1) - cwx0;
        const double v0 = cw[wq * I::CWC + e];
        double v = v0;
        if constexpr (I::SY == 2) v = vblend(v0, cw[wt * I::CWC + e]);
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = k == kl ? v : C[k];  // selects, not branches
      }
    }
  }
}

// XTRA: 0 = RGB only, 1 = + exact integer SSE and luma SSE partials,
//       2 = + IntermediateData error maps (pipeline.py:117-122)
// (XTRA = 2 is the single-frame host path: it trades occupancy for registers
// rather than spill to scratch)
// One tile (frame, tile) of the exact inverse; `ntiles` = tiles per frame (the
// luma-SSE partials are per tile).  The caller's shared arrays are reused
// tile after tile by the list form.
template <int MODE, int XTRA>
struct InvShared {
  double mid[Inv<MODE>::MB * MS];
  double cw[2][Inv<MODE>::CWR * Inv<MODE>::CWC];
  int q[64];  // integer quantiser table Q
  double red[Inv<MODE>::NT / 64];
  unsigned long long sse;
};

template <int MODE, int XTRA>
__device__ __forceinline__ void inv2_tile(InvShared<MODE, XTRA>& sh, const Geo& g, const int tiles_x, const int ntiles,
                                          const int frame, const int tile, const int16_t* __restrict__ coeffs,
                                          const FrameQ* __restrict__ fq, const uint8_t* __restrict__ rgb_in,
                                          uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
                                          double* __restrict__ sse_y_part, double* __restrict__ err_y,
                                          double* __restrict__ err_rgb, const int in_div) {
  using I = Inv<MODE>;
  double* s_mid = sh.mid;
  double (*s_cw)[I::CWR * I::CWC] = sh.cw;
  int* s_q = sh.q;
  double* s_red = sh.red;
  unsigned long long& s_sse = sh.sse;

  const int tid = threadIdx.x, lv = tid & 7, lb = tid >> 3;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  if (tid < 64) s_q[tid] = (int)fq[frame].q[tid];  // Q is an integer in [1, 255]
  if (XTRA && tid == 0) s_sse = 0ull;
  __syncthreads();

  // ---- 1. chroma window ----------------------------------------------------
  const int cby0 = Y0 / (8 * I::SY) - I::RY, cbx0 = X0 / (8 * I::SX) - I::RX;
  const int cwy0 = Y0 / I::SY - I::RY, cwx0 = X0 / I::SX - I::RX;
  // Each block's column pass and row pass run on the same 8 lanes (one wave),
  // whose LDS operations execute in order: no workgroup barrier until the
  // window is complete.  A top (bottom) ring block contributes only its last
  // (first) row.
  // luma round 0's coefficients are requested before any chroma math
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
#ifndef JDS_PROBE_NOCHROMA  // tools/probe: skip the chroma window
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
      if (p == 0) cq = load_col(cf + g.off_cr, boff, lv, bvalid);  // next plane in flight
      if (bvalid) {
        idct_col(cur, s_q, lv, s_mid + lb * MS);
        if (need) {
          double c[8];
          idct_row(s_mid + lb * MS, lv, c);
          double* w = &s_cw[p][(by * 8 + lv - cwy0) * I::CWC];
          const int wc0 = bx * 8 - cwx0;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if ((unsigned)(wc0 + k) < (unsigned)I::CWC) w[wc0 + k] = c[k];
        }
      }
    }
  }
  __syncthreads();
#endif
  // ---- 2. luma rounds: IDCT, upsample, colour, store --------------------------
  const bool want_in = XTRA > 0;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = want_in ? rgb_in + (size_t)(frame / in_div) * g.H * g.W * 3 : nullptr;  // sweep: item -> frame
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
#pragma unroll 1
  for (int r = 0; r < I::NYB / I::RB; ++r) {
    int by, bx;
    const bool bvalid = luma_blk(r, by, bx);
    const Col16 cur = lq;
    if (r + 1 < I::NYB / I::RB) {  // next round's coefficients in flight
      int by1, bx1;
      const bool ok1 = luma_blk(r + 1, by1, bx1);
      lq = load_col(cf, ((long long)by1 * g.nbx + bx1) * 64, lv, ok1);
    }
    if (bvalid) idct_col(cur, s_q, lv, s_mid + lb * MS);
    // (the block's row pass reads what its own wave wrote: no barrier)
    const int y = by * 8 + lv, x0 = bx * 8;
    if (bvalid && y < g.H && x0 < g.W) {
      double Yv[8];
      idct_row(s_mid + lb * MS, lv, Yv);
      // chroma rows (cv2 INTER_LINEAR: rows clamped, weights kept): wq carries
      // weight 1/4, wt weight 3/4 (4:2:0); without vertical subsampling wq = y
      int wq, wt = 0;
      if constexpr (I::SY == 2) {
        float fy = (float)((y + 0.5) * g.up_sy - 0.5);
        const int sy = (int)floorf(fy);
        fy -= (float)sy;  // 0.75 (b0 = 1/4: row sy is the quarter row) or 0.25
        const int r0 = clampi(clampi(sy, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
        const int r1 = clampi(clampi(sy + 1, 0, g.hc - 1) - cwy0, 0, I::CWR - 1);
        const bool q0 = fy == 0.75f;
        wq = q0 ? r0 : r1;
        wt = q0 ? r1 : r0;
      } else {
        wq = y - cwy0;
      }
      const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
      uint8_t* o = out_f + ((size_t)y * g.W + x0) * 3;
      const bool wide = nx == 8 && ((((uintptr_t)o) & 7u) == 0);
      // XTRA: the 8 input pixels (24 bytes, packed like the output) for the SSE
      // and the error maps, loaded before the colour math so that per-pixel
      // error terms are formed as the channels are (bounded register pressure)
      uint32_t in[6] = {0u, 0u, 0u, 0u, 0u, 0u};
      if constexpr (XTRA > 0) {
        const uint8_t* src = in_f + ((size_t)y * g.W + x0) * 3;
        if (wide) {
          const uint2* s2 = reinterpret_cast<const uint2*>(src);
          const uint2 a = s2[0], b = s2[1], c = s2[2];
          in[0] = a.x; in[1] = a.y; in[2] = b.x; in[3] = b.y; in[4] = c.x; in[5] = c.y;
        } else {
#pragma unroll
          for (int k = 0; k < 24; ++k)
            if (k < 3 * nx) in[k >> 2] |= (uint32_t)src[k] << (8 * (k & 3));
        }
      }
      auto byte_of = [](const uint32_t (&w)[6], int b) { return (int)((w[b >> 2] >> (8 * (b & 3))) & 255u); };
      // color_space.py:17-24 in NumPy's order, one chroma plane at a time to
      // bound register pressure: B and G's Cb term first, then R and G.
      uint32_t pk[6] = {0u, 0u, 0u, 0u, 0u, 0u};
      double eB[8];  // XTRA > 1: |B0 - clip(B)| (pipeline.py:121's last term)
      {
        double C[8], Gt[8];
        // floor(clip(v, 0, 255)) == clamp(trunc(v), 0, 255) for |v| < 2^31:
        // one conversion and integer min/max instead of two fp64 ops
#ifndef JDS_PROBE_NOUPS
        chroma8<MODE>(s_cw[0], g, x0, cwx0, wq, wt, C);
#else
        for (int k = 0; k < 8; ++k) C[k] = Yv[k] * 0.5;
#endif
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double B = Yv[k] + 1.772 * (C[k] - 128.0);
          Gt[k] = Yv[k] - 0.344136 * (C[k] - 128.0);
          if constexpr (XTRA > 1) eB[k] = fabs((double)byte_of(in, 3 * k + 2) - fmin(fmax(B, 0.0), 255.0));
          const int b = 3 * k + 2;
          pk[b >> 2] |= (uint32_t)clampi((int)B, 0, 255) << (8 * (b & 3));
        }
#ifndef JDS_PROBE_NOUPS
        chroma8<MODE>(s_cw[1], g, x0, cwx0, wq, wt, C);
#else
        for (int k = 0; k < 8; ++k) C[k] = Yv[k] * 0.25;
#endif
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double R = Yv[k] + 1.402 * (C[k] - 128.0);
          const double G = Gt[k] - 0.714136 * (C[k] - 128.0);
          const int b = 3 * k;
          pk[b >> 2] |= (uint32_t)clampi((int)R, 0, 255) << (8 * (b & 3));
          pk[(b + 1) >> 2] |= (uint32_t)clampi((int)G, 0, 255) << (8 * ((b + 1) & 3));
          if constexpr (XTRA > 1) {
            if (k < nx) {
              const double R0 = byte_of(in, b), G0 = byte_of(in, b + 1), B0 = byte_of(in, b + 2);
              const size_t pix = (size_t)y * g.W + x0 + k;
              err_y[pix] = fabs(luma(R0, G0, B0) - Yv[k]);  // pipeline.py:120
              err_rgb[pix] = ((fabs(R0 - fmin(fmax(R, 0.0), 255.0)) + fabs(G0 - fmin(fmax(G, 0.0), 255.0))) + eB[k]) /
                             3.0;  // pipeline.py:121
            }
          }
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
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < nx) {
            const int b = 3 * k;
            const int o0 = byte_of(in, b), o1 = byte_of(in, b + 1), o2 = byte_of(in, b + 2);
            const int ur = byte_of(pk, b), ug = byte_of(pk, b + 1), ub = byte_of(pk, b + 2);
            const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
            sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
            const double yo = luma((double)o0, (double)o1, (double)o2);
            const double yr = luma((double)ur, (double)ug, (double)ub);
            const double dy = yo - yr;
            ssy = ssy + dy * dy;
          }
        }
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
      for (int i = 0; i < I::NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * ntiles + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, s_sse);
    }
  }
}

template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv<MODE>::NT) __attribute__((amdgpu_waves_per_eu(XTRA > 1 ? 2 : Inv<MODE>::WPE)))
k_inv2(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
       const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
       double* __restrict__ sse_y_part, double* __restrict__ err_y, double* __restrict__ err_rgb, const int in_div) {
  __shared__ __attribute__((aligned(16))) InvShared<MODE, XTRA> sh;
  inv2_tile<MODE, XTRA>(sh, g, tiles_x, gridDim.x, blockIdx.y, blockIdx.x, coeffs, fq, rgb_in, rgb_out, st,
                        sse_y_part, err_y, err_rgb, in_div);
}

// The exact inverse over the tiles the certified fast inverse listed
// (jds_inv_fast.hip): a fixed grid walks the list; every workgroup re-reads the
// count, which the fast launch completed before this one started.
template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv<MODE>::NT) __attribute__((amdgpu_waves_per_eu(Inv<MODE>::WPE)))
k_inv2_list(const Geo g, const int tiles_x, const int ntiles, const int16_t* __restrict__ coeffs,
            const FrameQ* __restrict__ fq, const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out,
            jds_frame_stats* __restrict__ st, double* __restrict__ sse_y_part, const uint2* __restrict__ list,
            const unsigned* __restrict__ count, const int in_div) {
  __shared__ __attribute__((aligned(16))) InvShared<MODE, XTRA> sh;
  const unsigned n = *count;
  for (unsigned e = blockIdx.x; e < n; e += gridDim.x) {
    const uint2 ft = list[e];
    inv2_tile<MODE, XTRA>(sh, g, tiles_x, ntiles, (int)ft.x, (int)ft.y, coeffs, fq, rgb_in, rgb_out, st, sse_y_part,
                          nullptr, nullptr, in_div);
    __syncthreads();  // the next tile reloads the table and rewrites the window
  }
}

// IntermediateData.selected_block_reconstructed (pipeline.py:132-138): the
// clipped luma IDCT of one block (frame 0).
__global__ void __launch_bounds__(64) k_sel_recon(const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
                                                  jds_selected_block* sel, int sel_blk) {
  __shared__ __attribute__((aligned(16))) double s[MS];
  const int t = threadIdx.x;
  if (t < 8) {
    int qs[64];
#pragma unroll
    for (int r = 0; r < 8; ++r) qs[r * 8 + t] = (int)fq[0].q[r * 8 + t];
    idct_col(coeffs + (long long)sel_blk * 64, qs, t, s);
  }
  __syncthreads();
  if (t < 8) {
    double c[8];
    idct_row(s, t, c);
#pragma unroll
    for (int k = 0; k < 8; ++k) sel->reconstructed[t * 8 + k] = c[k];
  }
}

// ------------------------------------------------------------ launchers --

template <int MODE>
static int inv_tiles_t(int H, int W, int* tx) {
  const int ty = (H + Inv<MODE>::TH - 1) / Inv<MODE>::TH;
  *tx = (W + Inv<MODE>::TW - 1) / Inv<MODE>::TW;
  return ty * *tx;
}

int inv_tiles(int mode, int H, int W) {
  int tx;
  return mode == M420 ? inv_tiles_t<M420>(H, W, &tx)
                      : (mode == M422 ? inv_tiles_t<M422>(H, W, &tx) : inv_tiles_t<M444>(H, W, &tx));
}

template <int MODE>
static hipError_t inv2_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq, const uint8_t* rgb_in,
                         uint8_t* rgb_out, jds_frame_stats* st, double* part, double* err_y, double* err_rgb,
                         hipStream_t s, int in_div) {
  int tx;
  const int tiles = inv_tiles_t<MODE>(g.H, g.W, &tx);
  const dim3 grid(tiles, n), blk(Inv<MODE>::NT);
  if (err_y)
    hipLaunchKernelGGL((k_inv2<MODE, 2>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part, err_y,
                       err_rgb, in_div);
  else if (rgb_in)
    hipLaunchKernelGGL((k_inv2<MODE, 1>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part, nullptr,
                       nullptr, in_div);
  else
    hipLaunchKernelGGL((k_inv2<MODE, 0>), grid, blk, 0, s, g, tx, coeffs, fq, nullptr, rgb_out, st, part, nullptr,
                       nullptr, in_div);
  return hipGetLastError();
}

hipError_t launch_inv2(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                       const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part, double* err_y,
                       double* err_rgb, hipStream_t s, int in_div) {
  switch (mode) {
    case M420: return inv2_t<M420>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div);
    case M422: return inv2_t<M422>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div);
    default: return inv2_t<M444>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div);
  }
}

template <int MODE>
static hipError_t inv2_list_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq, const uint8_t* rgb_in,
                              uint8_t* rgb_out, jds_frame_stats* st, double* part, const uint2* list,
                              const unsigned* count, hipStream_t s, int in_div) {
  int tx;
  const int tiles = inv_tiles_t<MODE>(g.H, g.W, &tx);
  // a fixed grid (2 workgroups per CU) walks however many tiles were listed
  const long long total = (long long)tiles * n;
  const dim3 grid((unsigned)(total < 512 ? total : 512)), blk(Inv<MODE>::NT);
  if (rgb_in)
    hipLaunchKernelGGL((k_inv2_list<MODE, 1>), grid, blk, 0, s, g, tx, tiles, coeffs, fq, rgb_in, rgb_out, st, part,
                       list, count, in_div);
  else
    hipLaunchKernelGGL((k_inv2_list<MODE, 0>), grid, blk, 0, s, g, tx, tiles, coeffs, fq, nullptr, rgb_out, st,
                       part, list, count, in_div);
  return hipGetLastError();
}

hipError_t launch_inv2_list(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                            const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                            const uint2* list, const unsigned* count, hipStream_t s, int in_div) {
  switch (mode) {
    case M420: return inv2_list_t<M420>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, list, count, s, in_div);
    case M422: return inv2_list_t<M422>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, list, count, s, in_div);
    default: return inv2_list_t<M444>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, list, count, s, in_div);
  }
}

hipError_t launch_sel_recon(const int16_t* coeffs, const FrameQ* fq, jds_selected_block* sel, int sel_blk,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_sel_recon, dim3(1), dim3(64), 0, s, coeffs, fq, sel, sel_blk);
  return hipGetLastError();
}

}  // namespace jds
