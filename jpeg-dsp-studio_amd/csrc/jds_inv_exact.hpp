// jds_inv_exact.hpp — the exact (replayed-order) inverse of one tile, shared by
// k_inv2 (jds_inv.hip) and by the certified fast inverse's fallback
// (jds_inv_fast.hip): every operation is fp64 in the reference's order
// (engines/pipeline.py:68-95; pocketfft DCT-III butterflies, cv2 INTER_LINEAR
// taps, NumPy colour expressions) with FP contraction off.
#pragma once
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
    for (int k = 0; k < 8; ++k) C[k] = cw[wq * I::CWS + x0 + k - cwx0];
  } else {
    const int c0 = x0 / 2 - 1 - cwx0;
    double h0[8];
#pragma unroll
    for (int rr = 0; rr < (I::SY == 2 ? 2 : 1); ++rr) {
      const double* s = &cw[(rr ? wt : wq) * I::CWS + c0];
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
        const double v0 = cw[wq * I::CWS + e];
        double v = v0;
        if constexpr (I::SY == 2) v = vblend(v0, cw[wt * I::CWS + e]);
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = k == kl ? v : C[k];  // selects, not branches
      }
    }
  }
}

// 4:4:4 colour of 8 pixels from the clipped fp64 planes in NumPy's order
// (color_space.py:17-24: each expression left to right, contraction off),
// clip + astype(uint8) (pipeline.py:95) into packed output bytes: the exact
// path of k_inv_fast444's per-wave fallback (k_inv2's colour with no
// upsample), in two halves so that Cb's registers are free before Cr's pass:
// _cb writes B and G's first term Gt = Y - 0.344136 (Cb - 128), _cr adds R and
// G = Gt - 0.714136 (Cr - 128).
__device__ __forceinline__ void colour8_exact_cb(const double (&Yv)[8], const double (&Cb)[8], double (&Gt)[8],
                                                 uint32_t (&pk)[6]) {
#pragma unroll
  for (int w = 0; w < 6; ++w) pk[w] = 0u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double B = Yv[k] + 1.772 * (Cb[k] - 128.0);
    Gt[k] = Yv[k] - 0.344136 * (Cb[k] - 128.0);
    const int b = 3 * k + 2;
    pk[b >> 2] |= (uint32_t)clampi((int)B, 0, 255) << (8 * (b & 3));
  }
}
__device__ __forceinline__ void colour8_exact_cr(const double (&Yv)[8], const double (&Gt)[8], const double (&Cr)[8],
                                                 uint32_t (&pk)[6]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double R = Yv[k] + 1.402 * (Cr[k] - 128.0);
    const double G = Gt[k] - 0.714136 * (Cr[k] - 128.0);
    const int b = 3 * k;
    pk[b >> 2] |= (uint32_t)clampi((int)R, 0, 255) << (8 * (b & 3));
    pk[(b + 1) >> 2] |= (uint32_t)clampi((int)G, 0, 255) << (8 * ((b + 1) & 3));
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
  double cw[2][Inv<MODE>::CWR * Inv<MODE>::CWS];
  int q[64];  // integer quantiser table Q
  double red[Inv<MODE>::NT / 64];
  unsigned long long sse;
  int redo;  // the certified fast pass could not certify the tile (jds_inv_fast.hip)
};

// REDO (the certified fast inverse's fallback, jds_inv_fast.hip): the whole
// chroma window, then only the luma blocks whose lanes have bit r of
// `redo_mask` set in round r; the SSE terms of those rounds go to
// rsse[r] / rssy[r] and the caller reduces.  The luma SSE accumulates per round
// (ssy = ssy + round sum), so a mix of fast and redone rounds sums identically.
template <int MODE, int XTRA, bool REDO = false>
__device__ __forceinline__ void inv2_tile(InvShared<MODE, XTRA>& sh, const Geo& g, const int tiles_x, const int ntiles,
                                          const int frame, const int tile, const int16_t* __restrict__ coeffs,
                                          const FrameQ* __restrict__ fq, const uint8_t* __restrict__ rgb_in,
                                          uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
                                          double* __restrict__ sse_y_part, double* __restrict__ err_y,
                                          double* __restrict__ err_rgb, const int in_div,
                                          const unsigned redo_mask = ~0u, unsigned long long* rsse = nullptr,
                                          double* rssy = nullptr) {
  using I = Inv<MODE>;
  static_assert(I::NYB / I::RB <= 2, "at most two luma rounds per lane");
  double* s_mid = sh.mid;
  double (*s_cw)[I::CWR * I::CWS] = sh.cw;
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
          double* w = &s_cw[p][(by * 8 + lv - cwy0) * I::CWS];
          const int wc0 = bx * 8 - cwx0;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if ((unsigned)(wc0 + k) < (unsigned)I::CWC) w[wc0 + k] = c[k];
        }
      }
    }
  }
  __syncthreads();
  // ---- 2. luma rounds: IDCT, upsample, colour, store --------------------------
  const bool want_in = XTRA > 0;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = want_in ? rgb_in + (size_t)(frame / in_div) * g.H * g.W * 3 : nullptr;  // sweep: item -> frame
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
#pragma unroll 1
  for (int r = 0; r < I::NYB / I::RB; ++r) {
    int by, bx;
    const bool bvalid = luma_blk(r, by, bx) && (!REDO || ((redo_mask >> r) & 1u));
    unsigned long long r_sse = 0ull;
    double r_ssy = 0.0;
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
        chroma8<MODE>(s_cw[0], g, x0, cwx0, wq, wt, C);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double B = Yv[k] + 1.772 * (C[k] - 128.0);
          Gt[k] = Yv[k] - 0.344136 * (C[k] - 128.0);
          if constexpr (XTRA > 1) eB[k] = fabs((double)byte_of(in, 3 * k + 2) - fmin(fmax(B, 0.0), 255.0));
          const int b = 3 * k + 2;
          pk[b >> 2] |= (uint32_t)clampi((int)B, 0, 255) << (8 * (b & 3));
        }
        chroma8<MODE>(s_cw[1], g, x0, cwx0, wq, wt, C);
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
            r_sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
            r_ssy = r_ssy + luma_sse_e6(d0, d1, d2);
          }
        }
      }
    }
    if constexpr (XTRA > 0) {
      if constexpr (REDO) {
        rsse[r] = r_sse;
        rssy[r] = r_ssy;
      } else {
        sse += r_sse;
        ssy = ssy + r_ssy;
      }
    }
  }

  if constexpr (XTRA > 0 && !REDO) {
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

}  // namespace jds
