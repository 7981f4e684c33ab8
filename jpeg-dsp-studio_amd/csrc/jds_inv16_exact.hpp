// jds_inv16_exact.hpp — the exact 16x16 inverse's shared pieces (block path of
// BASELINE configs[4]): tile geometry, the 16-point IDCT of a block held by 16
// lanes, and k_inv16s's tile body, every operation fp64 in the reference's
// order (engines/pipeline.py:68-95 with block_size 16; pocketfft's 16-point
// DCT-III from jds_dct16.hpp, cv2 INTER_LINEAR taps, NumPy colour expressions)
// with FP contraction off.  Used by jds_b16.hip (k_inv16s, k_inv16f, k_inv16,
// k_chroma16) and, as the fallback of the certified fast 16x16 inverse, by
// jds_inv_fast.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct16.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

// doubles per 16x16 block in LDS: rows of 17 (a lane's row of 16 lands on 16
// distinct bank pairs; two blocks sit 32 banks apart, so 32 lanes of b64
// accesses -- rows or columns -- are conflict-free)
constexpr int BS16 = 272;
constexpr int RS16 = 17;  // row stride

template <int MODE>
struct Cfg16 {
  static constexpr int SY = (MODE == M420) ? 2 : 1;
  static constexpr int SX = (MODE == M444) ? 1 : 2;
  static constexpr int MH = 16 * SY, MW = 16 * SX;  // MCU in pixels
  // two MCU rows / >= two MCU columns per tile: the block row/column carrying
  // np.pad reflect padding (<= 15 samples) always shares its tile with the
  // block row/column it reflects into (tiles are bottom-right aligned, Geo)
  static constexpr int TH = 2 * MH, TW = 64;
  static constexpr int MY = TH / MH, MX = TW / MW;
  static constexpr int YBR = TH / 16, YBC = TW / 16;
  static constexpr int CBR = MY, CBC = MX;
  static constexpr int NYB = YBR * YBC, NCB = CBR * CBC;
  static constexpr int NB = NYB + 2 * NCB;
  static constexpr int TF = NB * 16;  // forward: one thread per block column
  static constexpr int TI = 256;      // inverse threads
};

// 32*Q16[u][v] = 32*Q8[u/2][v/2]: pocketfft's first-axis fct = 1/32 folded in (exact)
__device__ __forceinline__ double q16_of(const double* q8, int u, int v) { return q8[(u >> 1) * 8 + (v >> 1)]; }

// Dequantise + 2-D IDCT (axis 0 first) of one 16x16 block held in LDS by the
// 16 lanes (line = 0..15) that own it; the same lanes do both passes, so the
// exchange is wave-local (a block's 16 lanes are in one wave).  Returns the
// clipped spatial row `line` in r[16] (dct_engine.py:23-27).
// A lane's coefficient row of a 16x16 block (16 int16, two 16-byte loads).
struct Row16 {
  uint4 a, b;
};
__device__ __forceinline__ Row16 load_row16(const int16_t* __restrict__ src, int line) {
  const uint4* p = reinterpret_cast<const uint4*>(src + line * 16);
  return Row16{p[0], p[1]};
}

__device__ __forceinline__ void idct16_rows(const Row16& rw, const double* __restrict__ q8,
                                            double* __restrict__ s_b, int line, double* r) {
  {
    const uint4 a = rw.a, b = rw.b;
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int16_t qv = (int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
      s_b[line * RS16 + k] = (double)qv * q16_of(q8, line, k);  // quantizer.py:27-29
    }
  }
  __builtin_amdgcn_wave_barrier();  // no LDS access moves across (the exchange is wave-local)
  double c[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) c[i] = s_b[i * RS16 + line];
  dct3_line16(c);
#pragma unroll
  for (int i = 0; i < 16; ++i) s_b[i * RS16 + line] = c[i];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 16; ++k) c[k] = s_b[line * RS16 + k];
  dct3_line16(c);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double s = c[k] * 0.03125 + 128.0;  // fct 1/32 (exact), then +128
    r[k] = fmin(fmax(s, 0.0), 255.0);
  }
}

__device__ __forceinline__ void idct16_block(const int16_t* __restrict__ src, const double* __restrict__ q8,
                                             double* __restrict__ s_b, int line, double* r) {
  idct16_rows(load_row16(src, line), q8, s_b, line, r);
}

template <int MODE>
struct Inv16 {
  static constexpr int SY = Cfg16<MODE>::SY;
  static_assert(Cfg16<MODE>::SX == 2, "chroma subsampled horizontally");
  static constexpr int TH = (MODE == M420) ? 64 : 32, TW = (MODE == M420) ? 64 : 128;
  static constexpr int NT = 256, NG = NT / 16;  // 16-lane groups = blocks in flight
  static constexpr int RY = SY == 2 ? 1 : 0;
  static constexpr int CWR = TH / SY + 2 * RY, CWC = TW / 2 + 2;  // chroma window (samples)
  static constexpr int YBC = TW / 16, NYB = (TH / 16) * YBC;      // luma blocks per tile
  static constexpr int CBR = (MODE == M420) ? TH / 32 + 2 : TH / 16, CBC = TW / 32 + 2;
  static constexpr int NCB = CBR * CBC;                            // chroma blocks per plane
  static_assert(NYB == NG, "one luma round");
};


// ------------------------------------------- fused inverse, one window (4:2:x) --
//
// k_inv16s<MODE, XTRA>: k_inv16f with the two chroma windows built one after
// the other in the same LDS: Cb window -> luma IDCT, B bytes and the G partial
// Y - 0.344136 (Cb - 128) per pixel (registers) -> Cr window -> R, G bytes and
// the stores.  The reference evaluates G = Y - a (Cb - 128) - b (Cr - 128)
// left to right, so the partial is the same double; every other operation is
// k_inv16f's.  One fp64 window instead of two: 3 workgroups per CU at 4:2:2
// instead of 2 (k_inv16f: 69 KB of LDS).
// k_inv16s's tile body (the exact 16x16 inverse of tile `tile` of `frame`):
// the shared arrays are the caller's (s_b: I::NG * BS16 doubles, s_cw:
// I::CWR * I::CWC, s_q: the frame's 8x8 table, loaded and synchronised by the
// caller; s_red / s_sse only with XTRA > 0, s_sse zeroed by the caller), so
// the certified fast kernel (jds_inv_fast.hip, k_inv16_fast) runs it as its
// fallback in its own LDS.  `ntiles` = tiles per frame (sse_y partials).
template <int MODE, int XTRA>
__device__ __forceinline__ void inv16s_tile(double* __restrict__ s_b, double* __restrict__ s_cw,
                                            const double* __restrict__ s_q, double* __restrict__ s_red,
                                            unsigned long long* __restrict__ s_sse, const Geo& g, const int tiles_x,
                                            const int ntiles, const int frame, const int tile,
                                            const int16_t* __restrict__ coeffs, const uint8_t* __restrict__ rgb_in,
                                            uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
                                            double* __restrict__ sse_y_part, double* __restrict__ err_y,
                                            double* __restrict__ err_rgb) {
  using I = Inv16<MODE>;
  const int tid = threadIdx.x, grp = tid >> 4, line = tid & 15;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;

  const int cwy0 = Y0 / I::SY - I::RY, cwx0 = X0 / 2 - 1;
  const int cby0 = (Y0 / I::SY) / 16 - I::RY, cbx0 = (X0 / 2) / 16 - 1;
  double* const sb = s_b + grp * BS16;
  // every coefficient row of the lane (both planes' chroma blocks and its luma
  // block) requested before the first transform: one memory latency
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

  auto build = [&](int p) {  // plane p's window: IDCT16 of the blocks the tile reaches (+ ring)
#pragma unroll
    for (int k = 0; k < NCR; ++k) {
      const int bi = k * I::NG + grp;
      if (bi < I::NCB) {
        const int cy = cby0 + bi / I::CBC, cx = cbx0 + bi % I::CBC;
        if (cy >= 0 && cx >= 0 && cy < g.ncy && cx < g.ncx) {  // uniform per 16-lane group
          double r[16];
          idct16_rows(crow[p][k], s_q, sb, line, r);
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
  // one plane's upsampled chroma at pixels x0 .. x0 + 7 of row (wq, wt): k_inv16f's taps
  auto upsample = [&](int x0, int wq, int wt, double (&C)[8]) {
    const int c0 = x0 / 2 - 1 - cwx0;
    double h0[8];
#pragma unroll
    for (int rr = 0; rr < I::SY; ++rr) {
      const double* sp = &s_cw[(rr ? wt : wq) * I::CWC + c0];
      double q75[5];
#pragma unroll
      for (int j = 1; j < 5; ++j) q75[j] = sp[j] * 0.75;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double e = fma(sp[i], 0.25, q75[i + 1]), o = fma(sp[i + 2], 0.25, q75[i + 1]);
        if (rr == 0) {
          h0[2 * i] = e;
          h0[2 * i + 1] = o;
        } else {
          C[2 * i] = fma(h0[2 * i], 0.25, e * 0.75);
          C[2 * i + 1] = fma(h0[2 * i + 1], 0.25, o * 0.75);
        }
      }
    }
    if constexpr (I::SY == 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) C[k] = h0[k];
    }
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int kl = side == 0 ? (x0 == 0 ? 0 : -1) : (g.W - 1 - x0 < 8 ? g.W - 1 - x0 : -1);
      if (kl >= 0) {
        const int e = (side == 0 ? 0 : g.wc - 1) - cwx0;
        double v = s_cw[wq * I::CWC + e];
        if constexpr (I::SY == 2) v = fma(v, 0.25, s_cw[wt * I::CWC + e] * 0.75);
#pragma unroll
        for (int k = 0; k < 8; ++k) C[k] = k == kl ? v : C[k];
      }
    }
  };

  // ---- 1. Cb window ----
  build(0);
  __syncthreads();
  // ---- 2. luma row, Cb terms ----
  const int y = by * 16 + line;
  const bool act = by < g.nby && bx < g.nbx;  // uniform per 16-lane group
  const bool rowok = act && y < g.H;
  double Yv[16], Gt[16], Bv[XTRA > 1 ? 16 : 1];
  uint32_t bbyte[16];
  int wq = 0, wt = 0;
  if (act) idct16_rows(lrow, s_q, sb, line, Yv);
  if (rowok) {
    if constexpr (I::SY == 2) {  // cv2 INTER_LINEAR rows: wq weight 1/4, wt weight 3/4 (k_inv2)
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
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // color_space.py:17-24: the Cb terms of G and B
          const double Yk = Yv[8 * h + k];
          Gt[8 * h + k] = Yk - 0.344136 * (C[k] - 128.0);
          const double B = Yk + 1.772 * (C[k] - 128.0);
          bbyte[8 * h + k] = (uint32_t)clampi((int)B, 0, 255);
          if constexpr (XTRA > 1) Bv[8 * h + k] = B;
        }
      }
    }
  }
  __syncthreads();  // every Cb read done
  // ---- 3. Cr window ----
  build(1);
  __syncthreads();
  // ---- 4. Cr terms, store ----
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = XTRA ? rgb_in + (size_t)frame * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
  if (rowok) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int x0 = bx * 16 + 8 * h;
      if (x0 >= g.W) break;
      double C[8];
      upsample(x0, wq, wt, C);
      const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
      uint8_t* o = out_f + ((size_t)y * g.W + x0) * 3;
      uint32_t pk[6] = {0u, 0u, 0u, 0u, 0u, 0u};
      double R[8], G[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // color_space.py:17-24, pipeline.py:93-95
        const double Yk = Yv[8 * h + k];
        R[k] = Yk + 1.402 * (C[k] - 128.0);
        G[k] = Gt[8 * h + k] - 0.714136 * (C[k] - 128.0);
        const int b = 3 * k;
        pk[b >> 2] |= (uint32_t)clampi((int)R[k], 0, 255) << (8 * (b & 3));
        pk[(b + 1) >> 2] |= (uint32_t)clampi((int)G[k], 0, 255) << (8 * ((b + 1) & 3));
        pk[(b + 2) >> 2] |= bbyte[8 * h + k] << (8 * ((b + 2) & 3));
      }
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
      if constexpr (XTRA > 0) {
        const uint8_t* src = in_f + ((size_t)y * g.W + x0) * 3;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < nx) {
            const int o0 = src[3 * k], o1 = src[3 * k + 1], o2 = src[3 * k + 2];
            const int b = 3 * k;
            const int ur = (pk[b >> 2] >> (8 * (b & 3))) & 255, ug = (pk[(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 255,
                      ub = (pk[(b + 2) >> 2] >> (8 * ((b + 2) & 3))) & 255;
            const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
            sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
            const double R0 = (double)o0, G0 = (double)o1, B0 = (double)o2;
            const double yo = luma(R0, G0, B0);
            ssy = ssy + luma_sse_e6(d0, d1, d2);
            if constexpr (XTRA > 1) {
              const size_t pix = (size_t)y * g.W + x0 + k;
              err_y[pix] = fabs(yo - Yv[8 * h + k]);  // pipeline.py:120
              err_rgb[pix] = ((fabs(R0 - fmin(fmax(R[k], 0.0), 255.0)) + fabs(G0 - fmin(fmax(G[k], 0.0), 255.0))) +
                              fabs(B0 - fmin(fmax(Bv[8 * h + k], 0.0), 255.0))) / 3.0;  // pipeline.py:121
            }
          }
        }
      }
    }
  }
  if constexpr (XTRA > 0) {
    unsigned long long sv = sse;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o, 64);
    if ((tid & 63) == 0) atomicAdd(s_sse, sv);
    double d = ssy;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = d + __shfl_xor(d, o, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
    __syncthreads();
    if (tid == 0) {
      double a = 0.0;
      for (int i = 0; i < I::NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * ntiles + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, *s_sse);
    }
  }
}


}  // namespace jds
