// jds_b16.hip — the 16x16 block path (BASELINE configs[4] stretch): the same
// pipeline as the 8x8 path (engines/pipeline.py:17-167) with block_size = 16,
// which the reference's validator accepts (models/compression_params.py:19-20)
// but its quantizer cannot run (engines/quantizer.py:24 broadcasts a 16x16
// block against the 8x8 table).  Build decision, documented in include/jds.h
// and DESIGN.md: the 16x16 table is np.kron(Q8, ones((2, 2))), i.e.
// Q16[u][v] = Q8[u/2][v/2] (same frequency band, same per-pixel noise).
//
// All arithmetic is fp64 in the reference's operation order (pocketfft's
// 16-point transforms restated in jds_dct16.hpp), so coefficients and bytes
// are bit-identical to the oracle (oracle/cpu_ref.py with block_size=16).
//
//   k_fwd16<MODE,PF> : one workgroup per TH x TW tile; RGB (+1 px ring) staged
//                      in LDS, chroma prefilter row pass in LDS, one thread
//                      per (block, column): column DCT, LDS exchange, row DCT,
//                      quantise, 2 x 16-B stores; exact statistics.
//   k_chroma16<MODE> : dequantise + 16x16 IDCT of every chroma block into
//                      cropped fp64 chroma planes (scratch in HBM; the 1-sample
//                      reach of the bilinear upsample then needs no ring
//                      blocks per tile).
//   k_inv16<MODE>    : one workgroup per tile: luma IDCT into LDS, bilinear
//                      chroma from the planes, colour, clip, truncate, 24-B
//                      stores; SSE / error maps like k_inv.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct16.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_inv16_exact.hpp"

#pragma clang fp contract(off)

namespace jds {

// ---------------------------------------------------------------- forward --

template <int MODE, bool PF>
__global__ void __launch_bounds__(Cfg16<MODE>::TF)
k_fwd16(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
        const double* __restrict__ gk, jds_frame_stats* __restrict__ st) {
  using C = Cfg16<MODE>;
  constexpr int WR = C::TH + 2, WC = C::TW + 2, WN = WR * WC;
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int PLANE_D = CPLANE ? 2 * WN : 0;
  constexpr int BLK_D = C::NB * BS16;
  constexpr int U_D = PLANE_D > BLK_D ? PLANE_D : BLK_D;

  __shared__ uint32_t s_rgb[WN];
  __shared__ __attribute__((aligned(16))) double s_u[U_D];
  __shared__ double s_q32[64];
  __shared__ double s_rq32[64];  // fl(1 / (32 Q))
  __shared__ unsigned s_hist[50];
  __shared__ int s_acc[2];

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;

  {  // every window load in flight before the first LDS store (one memory latency)
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
  if (tid < 64) {
    s_q32[tid] = 32.0 * fq[frame].q[tid];  // exact
    s_rq32[tid] = 1.0 / s_q32[tid];
  }
  if (tid < 50) s_hist[tid] = 0u;
  if (tid < 2) s_acc[tid] = 0;
  __syncthreads();

  if constexpr (CPLANE) {  // full-resolution chroma + Gaussian row pass (cv2 RowFilter<double>)
    double* s_cb = s_u;
    double* s_cr = s_u + WN;
#pragma unroll
    for (int l = 0; l < (WN + C::TF - 1) / C::TF; ++l) {
      const int i = tid + l * C::TF;
      if (i < WN) {
        double R, G, B;
        unpack(s_rgb[i], R, G, B);
        s_cb[i] = chroma_b(R, G, B);
        s_cr[i] = chroma_r(R, G, B);
      }
    }
    __syncthreads();
    constexpr int NRP = WR * (WC - 2);
    constexpr int PER = (NRP + C::TF - 1) / C::TF;
    const double k0 = gk[0], k1 = gk[1], k2 = gk[2];
    double tb[PER], tr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C::TF;
      if (i < NRP) {
        const int r = i / (WC - 2), c = i - r * (WC - 2) + 1;
        const double* b = s_cb + r * WC + c;
        const double* q = s_cr + r * WC + c;
        double t = k0 * b[-1];
        t = t + k1 * b[0];
        tb[j] = t + k2 * b[1];
        t = k0 * q[-1];
        t = t + k1 * q[0];
        tr[j] = t + k2 * q[1];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C::TF;
      if (i < NRP) {
        const int r = i / (WC - 2), c = i - r * (WC - 2) + 1;
        s_cb[r * WC + c] = tb[j];
        s_cr[r * WC + c] = tr[j];
      }
    }
    __syncthreads();
  }

  // one thread per (block, column)
  const int blk = tid >> 4, line = tid & 15;
  int plane, gy, gx;
  if (blk < C::NYB) {
    plane = 0;
    gy = m0y * C::SY + blk / C::YBC;  // an MCU holds SY x SX luma blocks
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

  double v[16];
  if (valid) {
    if (plane == 0 || MODE == M444) {
      const int sx = reflect_pad(gx * 16 + line, g.W) - x0 + 1;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int sy = reflect_pad(gy * 16 + i, g.H) - y0 + 1;
        double R, G, B;
        unpack(s_rgb[sy * WC + sx], R, G, B);
        v[i] = plane == 0 ? luma(R, G, B) : (plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B));
      }
    } else {
      // INTER_AREA mean of (blurred) full-resolution chroma (color_space.py:38-49)
      const double* s_pl = s_u + (plane == 1 ? 0 : WN);
      const double k0 = gk[0], k1 = gk[1];
      const int sc = reflect_pad(gx * 16 + line, g.wc);
      const int wc0 = C::SX * sc - x0 + 1;
#pragma unroll 2  // full unrolling kept every sample's operands live: 195 VGPRs, 2 waves/SIMD
      for (int i = 0; i < 16; ++i) {
        const int sr = reflect_pad(gy * 16 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;
        double s[C::SY][2];
#pragma unroll
        for (int a = 0; a < C::SY; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int w = (wr0 + a) * WC + wc0 + b;
            if constexpr (CPLANE) {
              const double d = k1 * s_pl[w] + 0.0;  // SymmColumnFilter<double>
              s[a][b] = d + k0 * (s_pl[w + WC] + s_pl[w - WC]);
            } else {
              double R, G, B;
              unpack(s_rgb[w], R, G, B);
              s[a][b] = plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B);
            }
          }
        }
        if constexpr (C::SY == 2)
          v[i] = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25;
        else
          v[i] = (s[0][0] + s[0][1]) * 0.5;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = v[i] - 128.0;  // dct_engine.py:19
    dct2_line16(v);                                    // axis 0 (columns) first
  }
  if constexpr (CPLANE) __syncthreads();  // the block buffer aliases the chroma planes
  double* s_blk = s_u + blk * BS16;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_blk[i * RS16 + line] = v[i];
  }
  __syncthreads();

  int nz = 0, mb = 0;
  if (valid) {
    const int u = line;
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = s_blk[u * RS16 + k];
    dct2_line16(v);
    // quantizer.py:22-24: rint of the true IEEE quotient.  t = fl(v * fl(1/Q))
    // lies within 3 * 2^-53 |v/Q| of fl(v/Q), so unless t is within |t| 2^-50
    // of a half-integer both round to the same integer; the rare others (and
    // exact ties) take the division.  |t - rint(t)| is exact (Sterbenz).
    double qd[16];
    unsigned need = 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double t = v[k] * q16_of(s_rq32, u, k);
      qd[k] = __builtin_rint(t);
      need |= (fabs(fabs(t - qd[k]) - 0.5) <= fabs(t) * 0x1p-50 ? 1u : 0u) << k;
    }
    if (__ballot(need != 0u)) {  // wave-uniform: almost never taken
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if ((need >> k) & 1u) qd[k] = __builtin_rint(v[k] / q16_of(s_q32, u, k));
    }
    int q[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      q[k] = (int)qd[k];
      const int m = q[k] < 0 ? -q[k] : q[k];
      if (m) {
        ++nz;
        mb += 33 - __clz(m);
        if (q[k] >= -100 && q[k] <= 100) atomicAdd(&s_hist[q[k] == 100 ? 49 : (q[k] + 100) >> 2], 1u);
      }
    }
    const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                          (long long)bidx * 256 + u * 16;
    uint4 pk[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int* qq = q + 8 * h;
      pk[h].x = (uint32_t)(uint16_t)qq[0] | ((uint32_t)(uint16_t)qq[1] << 16);
      pk[h].y = (uint32_t)(uint16_t)qq[2] | ((uint32_t)(uint16_t)qq[3] << 16);
      pk[h].z = (uint32_t)(uint16_t)qq[4] | ((uint32_t)(uint16_t)qq[5] << 16);
      pk[h].w = (uint32_t)(uint16_t)qq[6] | ((uint32_t)(uint16_t)qq[7] << 16);
    }
    uint4* dst = reinterpret_cast<uint4*>(coeffs + off);
    dst[0] = pk[0];
    dst[1] = pk[1];
  }
  nz = wave_sum(nz);
  mb = wave_sum(mb);
  if ((tid & 63) == 0) {
    atomicAdd(&s_acc[0], nz);
    atomicAdd(&s_acc[1], mb);
  }
  __syncthreads();
  jds_frame_stats* fs = st + frame;
  if (tid == 0) {
    atomicAdd((unsigned long long*)&fs->nonzero, (unsigned long long)s_acc[0]);
    atomicAdd((unsigned long long*)&fs->magnitude_bits, (unsigned long long)s_acc[1]);
  }
  if (tid < 50 && s_hist[tid]) atomicAdd((unsigned long long*)&fs->hist[tid], (unsigned long long)s_hist[tid]);
}

// ---------------------------------------------------------------- inverse --

// Every chroma block -> cropped fp64 planes cb/cr (hc x wc each, per frame).
template <int MODE>
__global__ void __launch_bounds__(256)
k_chroma16(const Geo g, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
           double* __restrict__ planes) {
  __shared__ double s_b[16 * BS16];
  __shared__ double s_q[64];
  const int tid = threadIdx.x, frame = blockIdx.y;
  if (tid < 64) s_q[tid] = fq[frame].q[tid];
  __syncthreads();
  const int per_plane = g.ncy * g.ncx;
  const int b = blockIdx.x * 16 + (tid >> 4), line = tid & 15;
  if (b >= 2 * per_plane) return;  // whole 16-lane groups leave together
  const int p = b >= per_plane, bi = b - p * per_plane;
  const int by = bi / g.ncx, bx = bi - by * g.ncx;
  const int16_t* src = coeffs + (size_t)frame * g.cpf + (p ? g.off_cr : g.off_cb) + (long long)bi * 256;
  double r[16];
  idct16_block(src, s_q, s_b + (tid >> 4) * BS16, line, r);
  const int y = by * 16 + line;
  if (y >= g.hc) return;  // crop (pipeline.py:77-82)
  double* dst = planes + ((size_t)frame * 2 + p) * g.hc * g.wc + (size_t)y * g.wc + bx * 16;
  const int n = g.wc - bx * 16 < 16 ? g.wc - bx * 16 : 16;
#pragma unroll
  for (int k = 0; k < 16; ++k)
    if (k < n) dst[k] = r[k];
}

template <int MODE>
__global__ void __launch_bounds__(Cfg16<MODE>::TI)
k_inv16(const Geo g, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
        const double* __restrict__ planes, const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out,
        jds_frame_stats* __restrict__ st, double* __restrict__ sse_y_part, double* __restrict__ err_y,
        double* __restrict__ err_rgb) {
  using C = Cfg16<MODE>;
  constexpr int NT = C::TI;
  constexpr int NGRP = NT / 16;  // blocks in flight per round
  __shared__ double s_b[NGRP * BS16];
  __shared__ double s_y[C::TH * C::TW];
  __shared__ double s_q[64];
  __shared__ double s_red[NT / 64];
  __shared__ unsigned long long s_sse;

  const int tid = threadIdx.x, frame = blockIdx.y, tile = blockIdx.x;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  if (tid < 64) s_q[tid] = fq[frame].q[tid];
  if (tid == 0) s_sse = 0ull;
  __syncthreads();

  // luma blocks of the tile -> s_y (rows of phantom / out-of-grid blocks untouched, never read)
  for (int b0 = 0; b0 < C::NYB; b0 += NGRP) {
    const int blk = b0 + (tid >> 4), line = tid & 15;
    if (blk < C::NYB) {
      const int br = blk / C::YBC, bc = blk - br * C::YBC;
      const int by = m0y * C::SY + br, bx = m0x * C::SX + bc;
      if (by >= 0 && bx >= 0 && by < g.nby && bx < g.nbx) {
        double r[16];
        idct16_block(cf + ((long long)by * g.nbx + bx) * 256, s_q, s_b + (tid >> 4) * BS16, line, r);
        double* d = s_y + (br * 16 + line) * C::TW + bc * 16;
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = r[k];
      }
    }
  }
  __syncthreads();

  const bool want_in = rgb_in != nullptr;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = want_in ? rgb_in + (size_t)frame * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
  const double* pcb = planes + (size_t)frame * 2 * g.hc * g.wc;
  const double* pcr = pcb + (size_t)g.hc * g.wc;
  for (int t = tid; t < C::TH * (C::TW / 8); t += NT) {
    const int r = t / (C::TW / 8), sg = t - r * (C::TW / 8);
    const int y = y0 + r;
    if (y < 0 || y >= g.H) continue;
    int r0 = y, r1 = y;
    double b0 = 1.0, b1 = 0.0;
    if constexpr (MODE != M444) {  // cv2 INTER_LINEAR vertical taps (color_space.py:63-65)
      float fy = (float)((y + 0.5) * g.up_sy - 0.5);
      const int sy = (int)floorf(fy);
      fy -= (float)sy;
      b0 = (double)(1.f - fy);
      b1 = (double)fy;
      r0 = clampi(sy, 0, g.hc - 1);
      r1 = clampi(sy + 1, 0, g.hc - 1);
    }
    uint8_t px[24];
    double ey[8], er[8];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int lx = sg * 8 + k, x = x0 + lx;
      if (x < 0 || x >= g.W) { ey[k] = er[k] = 0.0; px[3 * k] = px[3 * k + 1] = px[3 * k + 2] = 0; continue; }
      ++cnt;
      const double Y = s_y[r * C::TW + lx];
      double Cb, Cr;
      if constexpr (MODE == M444) {
        Cb = pcb[(size_t)y * g.wc + x];
        Cr = pcr[(size_t)y * g.wc + x];
      } else {
        float fx = (float)((x + 0.5) * g.up_sx - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) { sx = 0; fx = 0.f; }
        const bool copy = sx + 1 >= g.wc;
        if (sx >= g.wc - 1) { sx = g.wc - 1; fx = 0.f; }
        const double a0 = (double)(1.f - fx), a1 = (double)fx;
        double hv[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const double* pl = p ? pcr : pcb;
          const double* s0 = pl + (size_t)r0 * g.wc + sx;
          const double* s1 = pl + (size_t)r1 * g.wc + sx;
          if (copy) {
            hv[p][0] = s0[0] * 1.0;
            hv[p][1] = s1[0] * 1.0;
          } else {
            hv[p][0] = s0[0] * a0 + s0[1] * a1;
            hv[p][1] = s1[0] * a0 + s1[1] * a1;
          }
        }
        Cb = hv[0][0] * b0 + hv[0][1] * b1;
        Cr = hv[1][0] * b0 + hv[1][1] * b1;
      }
      // engines/color_space.py:17-24, pipeline.py:93-95
      double R = Y + 1.402 * (Cr - 128.0);
      double G = Y - 0.344136 * (Cb - 128.0) - 0.714136 * (Cr - 128.0);
      double B = Y + 1.772 * (Cb - 128.0);
      R = fmin(fmax(R, 0.0), 255.0);
      G = fmin(fmax(G, 0.0), 255.0);
      B = fmin(fmax(B, 0.0), 255.0);
      const uint8_t ur = (uint8_t)(int)R, ug = (uint8_t)(int)G, ub = (uint8_t)(int)B;
      px[3 * k] = ur; px[3 * k + 1] = ug; px[3 * k + 2] = ub;
      if (want_in) {
        const uint8_t* o = in_f + ((size_t)y * g.W + x) * 3;
        const int o0 = o[0], o1 = o[1], o2 = o[2];
        const int d0 = o0 - ur, d1 = o1 - ug, d2 = o2 - ub;
        sse += (unsigned long long)(d0 * d0 + d1 * d1 + d2 * d2);
        const double R0 = (double)o0, G0 = (double)o1, B0 = (double)o2;
        const double yo = luma(R0, G0, B0);
        ssy = ssy + luma_sse_e6(d0, d1, d2);
        ey[k] = fabs(yo - Y);                                          // pipeline.py:120
        er[k] = ((fabs(R0 - R) + fabs(G0 - G)) + fabs(B0 - B)) / 3.0;  // pipeline.py:121
      }
    }
    const int x = x0 + sg * 8;
    if (cnt == 8 && (((size_t)y * g.W + x) * 3 & 7) == 0) {
      uint64_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        w0 |= (uint64_t)px[k] << (8 * k);
        w1 |= (uint64_t)px[8 + k] << (8 * k);
        w2 |= (uint64_t)px[16 + k] << (8 * k);
      }
      uint64_t* o64 = reinterpret_cast<uint64_t*>(out_f + ((size_t)y * g.W + x) * 3);
      o64[0] = w0; o64[1] = w1; o64[2] = w2;
    } else {
      for (int k = 0; k < 8; ++k) {
        const int xx = x + k;
        if (xx < 0 || xx >= g.W) continue;
        uint8_t* q = out_f + ((size_t)y * g.W + xx) * 3;
        q[0] = px[3 * k]; q[1] = px[3 * k + 1]; q[2] = px[3 * k + 2];
      }
    }
    if (err_y != nullptr) {
      for (int k = 0; k < 8; ++k) {
        const int xx = x + k;
        if (xx < 0 || xx >= g.W) continue;
        err_y[(size_t)y * g.W + xx] = ey[k];
        err_rgb[(size_t)y * g.W + xx] = er[k];
      }
    }
  }
  if (want_in) {
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
      for (int i = 0; i < NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * gridDim.x + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, s_sse);
    }
  }
}


// ------------------------------------------------- fused inverse (4:2:x) --
//
// k_inv16f<MODE, XTRA>: the whole inverse of one TH x TW tile in one launch,
// the 8x8 path's k_inv2 design for 16x16 blocks.  Chroma blocks covering the
// tile's chroma window (+ the 1-sample ring the bilinear taps reach) are
// dequantised and 16-point IDCT'd by 16-lane groups into an fp64 LDS window
// (the row passes' crop is implicit: the taps clamp to hc-1 / wc-1); then each
// lane IDCTs one row of a luma block, upsamples the chroma of its 16 pixels
// from the window, converts, clips, truncates and stores 48 bytes.  It replaces
// k_chroma16 + k_inv16, whose fp64 chroma planes went through HBM (16 B per
// pixel written and read again at 4:2:2).  Same operations, same order: bytes
// are identical (tests/test_gpu_block16.py).
template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv16<MODE>::NT)
k_inv16f(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
         const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
         double* __restrict__ sse_y_part, double* __restrict__ err_y, double* __restrict__ err_rgb) {
  using I = Inv16<MODE>;
  __shared__ __attribute__((aligned(16))) double s_b[I::NG * BS16];
  __shared__ double s_cw[2][I::CWR * I::CWC];
  __shared__ double s_q[64];
  __shared__ double s_red[I::NT / 64];
  __shared__ unsigned long long s_sse;

  const int tid = threadIdx.x, grp = tid >> 4, line = tid & 15;
  const int frame = blockIdx.y, tile = blockIdx.x;
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int Y0 = ty * I::TH, X0 = tx * I::TW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  if (tid < 64) s_q[tid] = fq[frame].q[tid];
  if (XTRA && tid == 0) s_sse = 0ull;
  __syncthreads();

  // ---- 1. chroma window ----------------------------------------------------
  const int cwy0 = Y0 / I::SY - I::RY, cwx0 = X0 / 2 - 1;
  const int cby0 = (Y0 / I::SY) / 16 - I::RY, cbx0 = (X0 / 2) / 16 - 1;
  double* const sb = s_b + grp * BS16;
  // every coefficient row this lane will transform (its chroma blocks and its
  // luma block) is requested before the first transform: one memory latency
  constexpr int NCR = (2 * I::NCB + I::NG - 1) / I::NG;  // chroma rounds
  Row16 crow[NCR];
#pragma unroll
  for (int k = 0; k < NCR; ++k) {
    const int blk = k * I::NG + grp;
    const int p = blk >= I::NCB, bi = blk - p * I::NCB;
    const int by = cby0 + bi / I::CBC, bx = cbx0 + bi % I::CBC;
    if (blk < 2 * I::NCB && by >= 0 && bx >= 0 && by < g.ncy && bx < g.ncx)
      crow[k] = load_row16(cf + (p ? g.off_cr : g.off_cb) + ((long long)by * g.ncx + bx) * 256, line);
  }
  const int lby = Y0 / 16 + grp / I::YBC, lbx = X0 / 16 + grp % I::YBC;
  Row16 lrow;
  if (lby < g.nby && lbx < g.nbx) lrow = load_row16(cf + ((long long)lby * g.nbx + lbx) * 256, line);
#pragma unroll
  for (int k = 0; k < NCR; ++k) {
    const int blk = k * I::NG + grp;
    if (blk < 2 * I::NCB) {
      const int p = blk >= I::NCB, bi = blk - p * I::NCB;
      const int by = cby0 + bi / I::CBC, bx = cbx0 + bi % I::CBC;
      if (by >= 0 && bx >= 0 && by < g.ncy && bx < g.ncx) {  // uniform per 16-lane group
        double r[16];
        idct16_rows(crow[k], s_q, sb, line, r);
        const int wr = by * 16 + line - cwy0;
        if ((unsigned)wr < (unsigned)I::CWR) {
          double* w = &s_cw[p][wr * I::CWC];
          const int wc0 = bx * 16 - cwx0;
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if ((unsigned)(wc0 + k) < (unsigned)I::CWC) w[wc0 + k] = r[k];
        }
      }
    }
  }
  __syncthreads();

  // ---- 2. luma row, upsample, colour, store ------------------------------------
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = XTRA ? rgb_in + (size_t)frame * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
  const int by = lby, bx = lbx;
  const int y = by * 16 + line;
  if (by < g.nby && bx < g.nbx) {  // uniform per 16-lane group
    double Yv[16];
    idct16_rows(lrow, s_q, sb, line, Yv);
    if (y < g.H) {
      int wq, wt = 0;
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
        if (x0 >= g.W) break;
        // horizontal taps (pixel 2m: (s[m-1], s[m]) x (1/4, 3/4); 2m+1: (s[m], s[m+1]) x (3/4, 1/4)),
        // vertical blend, edge pixels copied (cv2's clamped taps) -- chroma8 in jds_inv.hip
        double C[2][8];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const double* cw = s_cw[p];
          const int c0 = x0 / 2 - 1 - cwx0;
          double h0[8];
#pragma unroll
          for (int rr = 0; rr < I::SY; ++rr) {
            const double* sp = &cw[(rr ? wt : wq) * I::CWC + c0];
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
                C[p][2 * i] = fma(h0[2 * i], 0.25, e * 0.75);
                C[p][2 * i + 1] = fma(h0[2 * i + 1], 0.25, o * 0.75);
              }
            }
          }
          if constexpr (I::SY == 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) C[p][k] = h0[k];
          }
#pragma unroll
          for (int side = 0; side < 2; ++side) {
            const int kl = side == 0 ? (x0 == 0 ? 0 : -1) : (g.W - 1 - x0 < 8 ? g.W - 1 - x0 : -1);
            if (kl >= 0) {
              const int e = (side == 0 ? 0 : g.wc - 1) - cwx0;
              double v = cw[wq * I::CWC + e];
              if constexpr (I::SY == 2) v = fma(v, 0.25, cw[wt * I::CWC + e] * 0.75);
#pragma unroll
              for (int k = 0; k < 8; ++k) C[p][k] = k == kl ? v : C[p][k];
            }
          }
        }
        const int nx = g.W - x0 < 8 ? g.W - x0 : 8;
        uint8_t* o = out_f + ((size_t)y * g.W + x0) * 3;
        uint32_t pk[6] = {0u, 0u, 0u, 0u, 0u, 0u};
        double R[8], G[8], B[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // color_space.py:17-24, pipeline.py:93-95
          const double Yk = Yv[8 * h + k];
          R[k] = Yk + 1.402 * (C[1][k] - 128.0);
          G[k] = Yk - 0.344136 * (C[0][k] - 128.0) - 0.714136 * (C[1][k] - 128.0);
          B[k] = Yk + 1.772 * (C[0][k] - 128.0);
          const int b = 3 * k;
          pk[b >> 2] |= (uint32_t)clampi((int)R[k], 0, 255) << (8 * (b & 3));
          pk[(b + 1) >> 2] |= (uint32_t)clampi((int)G[k], 0, 255) << (8 * ((b + 1) & 3));
          pk[(b + 2) >> 2] |= (uint32_t)clampi((int)B[k], 0, 255) << (8 * ((b + 2) & 3));
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
                                fabs(B0 - fmin(fmax(B[k], 0.0), 255.0))) / 3.0;  // pipeline.py:121
              }
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
    if ((tid & 63) == 0) atomicAdd(&s_sse, sv);
    double d = ssy;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = d + __shfl_xor(d, o, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
    __syncthreads();
    if (tid == 0) {
      double a = 0.0;
      for (int i = 0; i < I::NT / 64; ++i) a = a + s_red[i];
      sse_y_part[(size_t)frame * gridDim.x + tile] = a;
      atomicAdd((unsigned long long*)&st[frame].sse_rgb, s_sse);
    }
  }
}

// k_inv16s: the exact fused inverse with one chroma window at a time
// (jds_inv16_exact.hpp, inv16s_tile, has the description and the body).
template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv16<MODE>::NT)
k_inv16s(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
         const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
         double* __restrict__ sse_y_part, double* __restrict__ err_y, double* __restrict__ err_rgb) {
  using I = Inv16<MODE>;
  __shared__ __attribute__((aligned(16))) double s_b[I::NG * BS16];
  __shared__ double s_cw[I::CWR * I::CWC];
  __shared__ double s_q[64];
  __shared__ double s_red[I::NT / 64];
  __shared__ unsigned long long s_sse;
  const int tid = threadIdx.x;
  if (tid < 64) s_q[tid] = fq[blockIdx.y].q[tid];
  if (XTRA && tid == 0) s_sse = 0ull;
  __syncthreads();
  inv16s_tile<MODE, XTRA>(s_b, s_cw, s_q, s_red, &s_sse, g, tiles_x, gridDim.x, blockIdx.y, blockIdx.x, coeffs,
                          rgb_in, rgb_out, st, sse_y_part, err_y, err_rgb);
}

// ------------------------------------------------------------ launchers --

hipError_t launch_fwd_finish(const Geo& g, int n, jds_frame_stats* st, const uint32_t* part, int ptiles,
                             hipStream_t s);
hipError_t launch_finalize(const Geo& g, int n, jds_frame_stats* st, const double* part, int tiles, bool with_sse,
                           hipStream_t s);
hipError_t launch_fast_fwd16(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs,
                             const FrameQ* fq, const void* fq16, const double* gk, const float* gk32,
                             jds_frame_stats* st, uint32_t* part, uint2* fixlist, unsigned* counters, int fix_all,
                             int parity, hipStream_t s);

// tiles of the fused 16x16 inverse (sse_y partials per tile); 0 for 4:4:4
int inv16_tiles(int mode, int H, int W) {
  switch (mode) {
    case M420: return ((H + Inv16<M420>::TH - 1) / Inv16<M420>::TH) * ((W + Inv16<M420>::TW - 1) / Inv16<M420>::TW);
    case M422: return ((H + Inv16<M422>::TH - 1) / Inv16<M422>::TH) * ((W + Inv16<M422>::TW - 1) / Inv16<M422>::TW);
    default: return 0;
  }
}

int tile_dims16(int mode, int* MY, int* MX) {
  switch (mode) {
    case M420: *MY = Cfg16<M420>::MY; *MX = Cfg16<M420>::MX; return Cfg16<M420>::TF;
    case M422: *MY = Cfg16<M422>::MY; *MX = Cfg16<M422>::MX; return Cfg16<M422>::TF;
    default: *MY = Cfg16<M444>::MY; *MX = Cfg16<M444>::MX; return Cfg16<M444>::TF;
  }
}

hipError_t launch_inv16_fast(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                             uint8_t* rgb_out, const InvFix& fx, hipStream_t s, jds_frame_stats* st, int fin);

template <int MODE>
static hipError_t launch16_t(bool pf, const Geo& g, int n, const uint8_t* rgb, uint8_t* rgb_out, int16_t* coeffs,
                             const FrameQ* fq, const double* gk, jds_frame_stats* st, double* part, double* planes,
                             bool want_sse, double* err_y, double* err_rgb, hipStream_t s, hipEvent_t* ev,
                             int phases, const Fwd16Fast* ff, const InvFix* fx) {
  using C = Cfg16<MODE>;
  const dim3 grid(g.tiles_y * g.tiles_x, n);
  hipError_t e = hipSuccess;
  // the certified fast inverse (RGB only) finalizes the frame statistics
  // itself: no k_fwd_finish / k_finalize launches around it
  const bool fast_inv = (phases & 2) && MODE != M444 && fx && !(want_sse || err_y);
  if (phases & 1) {
    if (ev && (e = hipEventRecord(ev[0], s)) != hipSuccess) return e;
    if (ff)  // certified fp32 forward + exact fix-up of the listed blocks (jds_fast16.hip)
      e = launch_fast_fwd16(MODE, pf, g, n, rgb, coeffs, fq, ff->fq16, gk, ff->gk32, st, ff->part, ff->fixlist, ff->counters,
                            ff->fix_all, ff->parity, s);
    else if (MODE != M444 && pf)
      hipLaunchKernelGGL((k_fwd16<MODE, (MODE != M444)>), grid, dim3(C::TF), 0, s, g, rgb, coeffs, fq, gk, st);
    else
      hipLaunchKernelGGL((k_fwd16<MODE, false>), grid, dim3(C::TF), 0, s, g, rgb, coeffs, fq, gk, st);
    if (!ff) kmark(s, "k_fwd16<%d,%d>", MODE, (int)(MODE != M444 && pf));
    if (e != hipSuccess || (e = hipGetLastError()) != hipSuccess) return e;
    if (!fast_inv && (e = launch_fwd_finish(g, n, st, nullptr, 0, s)) != hipSuccess) return e;
    if (ev && (e = hipEventRecord(ev[1], s)) != hipSuccess) return e;
  }
  if (phases & 2) {
    const uint8_t* rin = (want_sse || err_y) ? rgb : nullptr;
    int tiles = g.tiles_y * g.tiles_x;
    if constexpr (MODE != M444) {  // fused: chroma window in LDS (k_inv16f)
      using I = Inv16<MODE>;
      const int tx = (g.W + I::TW - 1) / I::TW;
      tiles = ((g.H + I::TH - 1) / I::TH) * tx;
      const dim3 gi(tiles, n), bi(I::NT);
      if (fast_inv) {  // RGB only: the certified fast inverse (jds_inv_fast.hip), zero bin if this run's forward deferred it
        return launch_inv16_fast(MODE, g, n, coeffs, fq, rgb_out, *fx, s, st, (phases & 1) ? 1 : 0);
      } else {
#define K_INV16 k_inv16s
      if (err_y)
        hipLaunchKernelGGL((K_INV16<MODE, 2>), gi, bi, 0, s, g, tx, coeffs, fq, rin, rgb_out, st, part, err_y,
                           err_rgb);
      else if (rin)
        hipLaunchKernelGGL((K_INV16<MODE, 1>), gi, bi, 0, s, g, tx, coeffs, fq, rin, rgb_out, st, part, nullptr,
                           nullptr);
      else
        hipLaunchKernelGGL((K_INV16<MODE, 0>), gi, bi, 0, s, g, tx, coeffs, fq, nullptr, rgb_out, st, part, nullptr,
                           nullptr);
      kmark(s, "k_inv16s<%d,%d>", MODE, err_y ? 2 : rin ? 1 : 0);
#undef K_INV16
      if ((e = hipGetLastError()) != hipSuccess) return e;
      }
    } else {
      const int cblocks = 2 * g.ncy * g.ncx;
      hipLaunchKernelGGL((k_chroma16<MODE>), dim3((cblocks + 15) / 16, n), dim3(256), 0, s, g, coeffs, fq, planes);
      kmark(s, "k_chroma16<%d>", MODE);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      hipLaunchKernelGGL((k_inv16<MODE>), grid, dim3(C::TI), 0, s, g, coeffs, fq, planes, rin, rgb_out, st, part,
                         err_y, err_rgb);
      kmark(s, "k_inv16<%d>", MODE);
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (ev && (e = hipEventRecord(ev[2], s)) != hipSuccess) return e;
    e = launch_finalize(g, n, st, part, tiles, rin != nullptr, s);
  }
  return e;
}

// phases: bit 0 forward, bit 1 inverse (chroma planes + tiles + finalize);
// ff: the certified fp32 forward's buffers, nullptr = the exact fp64 forward;
// fx: the certified fast inverse's counters (4:2:x runs without SSE terms),
// nullptr = the exact inverse
hipError_t launch_codec16(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, uint8_t* rgb_out,
                          int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st, double* part,
                          double* planes, bool want_sse, double* err_y, double* err_rgb, hipStream_t s,
                          hipEvent_t* ev, int phases, const Fwd16Fast* ff, const InvFix* fx) {
  switch (mode) {
    case M420:
      return launch16_t<M420>(pf, g, n, rgb, rgb_out, coeffs, fq, gk, st, part, planes, want_sse, err_y, err_rgb,
                              s, ev, phases, ff, fx);
    case M422:
      return launch16_t<M422>(pf, g, n, rgb, rgb_out, coeffs, fq, gk, st, part, planes, want_sse, err_y, err_rgb,
                              s, ev, phases, ff, fx);
    default:
      return launch16_t<M444>(false, g, n, rgb, rgb_out, coeffs, fq, gk, st, part, planes, want_sse, err_y,
                              err_rgb, s, ev, phases, ff, fx);
  }
}

}  // namespace jds
