// jds_codec.hip — fused forward / inverse kernels of the block-DCT codec path
// for gfx950 (MI355X).  Reference: engines/pipeline.py:17-167 and the stages it
// calls (engines/color_space.py, block_processor.py, dct_engine.py,
// quantizer.py).  All arithmetic is fp64 in the reference's (NumPy / pocketfft /
// OpenCV) operation order with FP contraction off, so int16 coefficients AND
// reconstructed bytes are bit-identical to the reference.
//
// Data layout in HBM (per frame, frames contiguous):
//   rgb / rgb_out : H x W x 3 uint8, C order (NumPy image layout)
//   coeffs        : int16, [Y blocks | Cb blocks | Cr blocks], each plane's
//                   padded blocks in raster order, each block row-major
//                   (= IntermediateData.all_quantized_coeffs, pipeline.py:56,99)
//
// Work decomposition: one workgroup per TH x TW pixel tile (a few MCUs).
//   k_fwd: one thread per (block, line).  The tile's RGB (+1 px ring) is staged
//          in LDS as packed u32; chroma is colour-converted and, with the
//          prefilter, row-filtered into fp64 LDS planes; each thread then forms
//          its block column (area-averaged chroma / luma) in registers, runs the
//          column DCT, exchanges through LDS, runs the row DCT, quantizes and
//          writes its 8 coefficients as one 16-byte store.
//   k_inv: chroma blocks of the tile plus the 1-block ring the bilinear
//          upsample reads are inverse-transformed into an fp64 LDS window,
//          then luma blocks into an fp64 LDS tile; every thread finally
//          produces 8 RGB pixels (upsample, colour, clip, truncate).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct8.hpp"
#include "jds_internal.hpp"
#include "jds_device.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int BLK_STRIDE = 68;  // doubles per 8x8 block in LDS (64 + 4 pad)

// ---------------------------------------------------------------- forward --

template <int MODE, bool PF>
__global__ void __launch_bounds__(Cfg<MODE>::TF)
k_fwd(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
      const FrameQ* __restrict__ fq, const double* __restrict__ gk,
      jds_frame_stats* __restrict__ st, jds_selected_block* __restrict__ sel,
      int sel_frame, int sel_blk, int in_div) {
  using C = Cfg<MODE>;
  constexpr int WR = C::TH + 2, WC = C::TW + 2, WN = WR * WC;  // RGB window with 1-px ring
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int PLANE_D = CPLANE ? 2 * WN : 0;
  constexpr int BLK_D = C::NB * BLK_STRIDE;
  constexpr int U_D = PLANE_D > BLK_D ? PLANE_D : BLK_D;

  __shared__ uint32_t s_rgb[WN];
  __shared__ __attribute__((aligned(16))) double s_u[U_D];  // chroma planes, then block buffer
  __shared__ double s_q16[64];
  __shared__ unsigned s_hist[50];
  __shared__ int s_acc[2];

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;  // tile origin (may be < 0: phantom MCUs)
  const uint8_t* img = rgb + (size_t)(frame / in_div) * g.H * g.W * 3;  // sweep plans: item -> frame

  // 1. stage RGB (+ring, BORDER_REFLECT_101 outside the image) as packed u32
  // (every load in flight before the first LDS store: one memory latency)
  constexpr int NL = (WN + C::TF - 1) / C::TF;
  {
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
  if (tid < 64) s_q16[tid] = fq[frame].q16[tid];
  if (tid < 50) s_hist[tid] = 0u;
  if (tid < 2) s_acc[tid] = 0;
  __syncthreads();

  // 2. full-resolution chroma planes + Gaussian row pass (cv2 RowFilter<double>)
  if constexpr (CPLANE) {
    double* s_cb = s_u;
    double* s_cr = s_u + WN;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
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

  // 3. each thread forms one column of one block and transforms it
  const int blk = tid >> 3, line = tid & 7;
  int plane, gy, gx;
  if (blk < C::NYB) {
    plane = 0;
    gy = m0y * C::SY + blk / C::YBC;
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
  const bool is_sel = sel != nullptr && plane == 0 && frame == sel_frame && bidx == sel_blk && valid;

  double v[8];
  if (valid) {
    if (plane == 0 || MODE == M444) {
      const int sx = reflect_pad(gx * 8 + line, g.W) - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sy = reflect_pad(gy * 8 + i, g.H) - y0 + 1;
        double R, G, B;
        unpack(s_rgb[sy * WC + sx], R, G, B);
        v[i] = plane == 0 ? luma(R, G, B) : (plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B));
      }
    } else {
      // chroma sample = INTER_AREA mean of (blurred) full-res chroma (color_space.py:38-49)
      const double* s_pl = s_u + (plane == 1 ? 0 : WN);
      const double k0 = gk[0], k1 = gk[1];
      const int sc = reflect_pad(gx * 8 + line, g.wc);
      const int wc0 = C::SX * sc - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sr = reflect_pad(gy * 8 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;
        double s[C::SY][2];
#pragma unroll
        for (int a = 0; a < C::SY; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int w = (wr0 + a) * WC + wc0 + b;
            if constexpr (CPLANE) {
              // SymmColumnFilter<double>: k1*T[y] + 0, then += k0*(T[y+1] + T[y-1])
              const double d = k1 * s_pl[w] + 0.0;
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
    if (is_sel) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sel->original[i * 8 + line] = v[i];
        sel->shifted[i * 8 + line] = v[i] - 128.0;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = v[i] - 128.0;  // encode_block level shift (dct_engine.py:19)
    // axis 0 (columns) first, as pocketfft's general_nd does
    dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  }
  if constexpr (CPLANE) __syncthreads();  // block buffer aliases the chroma planes
  double* s_blk = s_u + blk * BLK_STRIDE;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_blk[i * 8 + line] = v[i];
  }
  __syncthreads();

  // 4. row transform, quantize, store (quantizer.py:22-24: round-half-even of c/Q)
  int nz = 0, mb = 0;
  if (valid) {
    const int u = line;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s_blk[u * 8 + k];
    dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    int q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      q[k] = (int)__builtin_rint(v[k] / s_q16[u * 8 + k]);
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
    const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                          (long long)bidx * 64 + u * 8;
    uint4 pk;
    pk.x = (uint32_t)(uint16_t)q[0] | ((uint32_t)(uint16_t)q[1] << 16);
    pk.y = (uint32_t)(uint16_t)q[2] | ((uint32_t)(uint16_t)q[3] << 16);
    pk.z = (uint32_t)(uint16_t)q[4] | ((uint32_t)(uint16_t)q[5] << 16);
    pk.w = (uint32_t)(uint16_t)q[6] | ((uint32_t)(uint16_t)q[7] << 16);
    *reinterpret_cast<uint4*>(coeffs + off) = pk;
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

// Dequantize + 2-D IDCT of up to NBLK blocks listed by (plane, gy, gx); the
// clipped spatial rows are handed to `emit(blk, u, vals[8])`.
template <int NBLK, int NT, typename Locate, typename Emit>
__device__ __forceinline__ void idct_round(const int16_t* __restrict__ cf, const double* __restrict__ s_q,
                                           double* __restrict__ s_buf, Locate locate, Emit emit) {
  const int tid = threadIdx.x;
  // a. load one coefficient row (16 B) per task, dequantize (quantizer.py:27-29)
  for (int t = tid; t < NBLK * 8; t += NT) {
    const int blk = t >> 3, u = t & 7;
    long long off;
    if (locate(blk, off)) {
      const uint4 pk = *reinterpret_cast<const uint4*>(cf + off + u * 8);
      const uint32_t w[4] = {pk.x, pk.y, pk.z, pk.w};
      double* d = s_buf + blk * BLK_STRIDE + u * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int16_t qv = (int16_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
        d[k] = (double)qv * s_q[u * 8 + k];
      }
    }
  }
  __syncthreads();
  // b. axis 0 (columns), type-3, ortho (dct_engine.py:12-14)
  for (int t = tid; t < NBLK * 8; t += NT) {
    const int blk = t >> 3, vcol = t & 7;
    long long off;
    if (locate(blk, off)) {
      double* d = s_buf + blk * BLK_STRIDE + vcol;
      double c[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) c[i] = d[i * 8];
      dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i * 8] = c[i];
    }
  }
  __syncthreads();
  // c. axis 1 (rows), level shift +128, clip (dct_engine.py:23-27)
  for (int t = tid; t < NBLK * 8; t += NT) {
    const int blk = t >> 3, u = t & 7;
    long long off;
    if (locate(blk, off)) {
      const double* d = s_buf + blk * BLK_STRIDE + u * 8;
      double c[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = d[k];
      dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double s = c[k] * 0.0625 + 128.0;  // fct 1/16 (exact) then +128
        c[k] = fmin(fmax(s, 0.0), 255.0);
      }
      emit(blk, u, c);
    }
  }
  __syncthreads();
}

template <int MODE>
__global__ void __launch_bounds__(Cfg<MODE>::TI)
k_inv(const Geo g, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
      const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out,
      jds_frame_stats* __restrict__ st, double* __restrict__ sse_y_part,
      double* __restrict__ err_y, double* __restrict__ err_rgb,
      jds_selected_block* __restrict__ sel, int sel_frame, int sel_blk, int in_div) {
  using C = Cfg<MODE>;
  constexpr int NT = C::TI;
  constexpr int NCHB = 2 * C::NRB;  // chroma blocks incl. ring, both planes
  constexpr int BUF_B = (NCHB > C::NYB ? NCHB : C::NYB);
  __shared__ __attribute__((aligned(16))) double s_buf[BUF_B * BLK_STRIDE];
  __shared__ double s_cw[2][C::CWR * C::CWC];  // reconstructed chroma window (Cb, Cr)
  __shared__ double s_y[C::TH * C::TW];       // reconstructed luma tile
  __shared__ double s_q[64];
  __shared__ double s_red[NT / 64];
  __shared__ unsigned long long s_sse;

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  const int tile = blockIdx.x;
  const int ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const int16_t* cf = coeffs + (size_t)frame * g.cpf;
  if (tid < 64) s_q[tid] = fq[frame].q[tid];
  if (tid == 0) s_sse = 0ull;
  __syncthreads();

  // chroma window origin (in chroma samples)
  const int cwy0 = 8 * m0y - C::RY, cwx0 = 8 * m0x - C::RX;

  // round 1: chroma blocks of the tile + ring
  idct_round<NCHB, NT>(
      cf, s_q, s_buf,
      [&](int blk, long long& off) {
        const int p = blk / C::NRB, bi = blk - p * C::NRB;
        const int by = m0y - C::RY + bi / C::RBC, bx = m0x - C::RX + bi % C::RBC;
        if (by < 0 || bx < 0 || by >= g.ncy || bx >= g.ncx) return false;
        off = (p == 0 ? g.off_cb : g.off_cr) + ((long long)by * g.ncx + bx) * 64;
        return true;
      },
      [&](int blk, int u, const double* c) {
        const int p = blk / C::NRB, bi = blk - p * C::NRB;
        const int by = m0y - C::RY + bi / C::RBC, bx = m0x - C::RX + bi % C::RBC;
        const int wr = by * 8 + u - cwy0;
        if (wr < 0 || wr >= C::CWR) return;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int wc = bx * 8 + k - cwx0;
          if (wc >= 0 && wc < C::CWC) s_cw[p][wr * C::CWC + wc] = c[k];
        }
      });

  // round 2: luma blocks of the tile
  idct_round<C::NYB, NT>(
      cf, s_q, s_buf,
      [&](int blk, long long& off) {
        const int by = m0y * C::SY + blk / C::YBC, bx = m0x * C::SX + blk % C::YBC;
        if (by < 0 || bx < 0 || by >= g.nby || bx >= g.nbx) return false;
        off = ((long long)by * g.nbx + bx) * 64;
        return true;
      },
      [&](int blk, int u, const double* c) {
        const int br = blk / C::YBC, bc = blk - br * C::YBC;
        double* d = s_y + (br * 8 + u) * C::TW + bc * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = c[k];
        if (sel != nullptr && frame == sel_frame) {
          const int by = m0y * C::SY + br, bx = m0x * C::SX + bc;
          if (by * g.nbx + bx == sel_blk) {
#pragma unroll
            for (int k = 0; k < 8; ++k) sel->reconstructed[u * 8 + k] = c[k];
          }
        }
      });

  // 3. upsample (cv2 INTER_LINEAR, color_space.py:63-65), YCbCr->RGB, clip,
  //    truncate (pipeline.py:93-95); optional metrics / IntermediateData maps
  const bool want_in = rgb_in != nullptr;
  unsigned long long sse = 0ull;
  double ssy = 0.0;
  const uint8_t* in_f = want_in ? rgb_in + (size_t)(frame / in_div) * g.H * g.W * 3 : nullptr;
  uint8_t* out_f = rgb_out + (size_t)frame * g.H * g.W * 3;
  for (int t = tid; t < C::TH * (C::TW / 8); t += NT) {
    const int r = t / (C::TW / 8), sg = t - r * (C::TW / 8);
    const int y = y0 + r;
    if (y < 0 || y >= g.H) continue;
    // vertical taps (computed once per row)
    int wr0 = 0, wr1 = 0;
    double b0 = 1.0, b1 = 0.0;
    if constexpr (MODE != M444) {
      float fy = (float)((y + 0.5) * g.up_sy - 0.5);
      const int sy = (int)floorf(fy);
      fy -= (float)sy;
      b0 = (double)(1.f - fy);
      b1 = (double)fy;
      wr0 = clampi(clampi(sy, 0, g.hc - 1) - cwy0, 0, C::CWR - 1);
      wr1 = clampi(clampi(sy + 1, 0, g.hc - 1) - cwy0, 0, C::CWR - 1);
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
        Cb = s_cw[0][r * C::CWC + lx];
        Cr = s_cw[1][r * C::CWC + lx];
      } else {
        float fx = (float)((x + 0.5) * g.up_sx - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) { sx = 0; fx = 0.f; }
        const bool copy = sx + 1 >= g.wc;
        if (sx >= g.wc - 1) { sx = g.wc - 1; fx = 0.f; }
        const double a0 = (double)(1.f - fx), a1 = (double)fx;
        const int wc0 = sx - cwx0;
        double hv[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const double* s0 = &s_cw[p][wr0 * C::CWC + wc0];
          const double* s1 = &s_cw[p][wr1 * C::CWC + wc0];
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
      // engines/color_space.py:17-24
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
        ey[k] = fabs(yo - Y);                                                   // pipeline.py:120
        er[k] = ((fabs(R0 - R) + fabs(G0 - G)) + fabs(B0 - B)) / 3.0;           // pipeline.py:121
      }
    }
    const int x = x0 + sg * 8;
    uint8_t* o = out_f + ((size_t)y * g.W + (x < 0 ? 0 : x)) * 3;
    if (cnt == 8) {
      // 24 contiguous bytes; 8-byte aligned when W*3*y + 3*x is (x % 8 == 0)
      uint64_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        w0 |= (uint64_t)px[k] << (8 * k);
        w1 |= (uint64_t)px[8 + k] << (8 * k);
        w2 |= (uint64_t)px[16 + k] << (8 * k);
      }
      if ((((uintptr_t)o) & 7u) == 0) {
        uint64_t* o64 = reinterpret_cast<uint64_t*>(o);
        o64[0] = w0; o64[1] = w1; o64[2] = w2;
      } else {
#pragma unroll
        for (int k = 0; k < 24; ++k) o[k] = px[k];
      }
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
    // exact integer SSE: one atomic per wave, then one per workgroup
    unsigned long long s = sse;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) atomicAdd(&s_sse, s);
    // luma SSE: fixed-order tree so the per-tile partial is deterministic
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

// Dequantized selected block (host path only): IntermediateData.selected_block_dequantized.
__global__ void k_sel_dequant(const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
                              jds_selected_block* sel, int sel_blk) {
  const int i = threadIdx.x;
  if (i < 64) sel->dequantized[i] = (double)coeffs[(long long)sel_blk * 64 + i] * fq[0].q[i];
}

// Sum of the forward kernels' per-tile statistics partials into the frame
// stats (reduce_partials, jds_internal.hpp).
__global__ void __launch_bounds__(512) k_fwd_reduce(jds_frame_stats* st, const uint32_t* __restrict__ part, int ptiles) {
  reduce_partials(st, part, ptiles);
}

// End of the forward phase: per-frame constants and the histogram's zero bin.
__global__ void k_fwd_finish(const Geo g, jds_frame_stats* st) {
  if (threadIdx.x != 0) return;
  finalize_frame(g, st + blockIdx.x, 1);
}

hipError_t launch_fwd_reduce(int n, jds_frame_stats* st, const uint32_t* part, int ptiles, hipStream_t s) {
  hipLaunchKernelGGL(k_fwd_reduce, dim3((ptiles + 63) / 64, n), dim3(512), 0, s, st, part, ptiles);
  kmark(s, "k_fwd_reduce");
  return hipGetLastError();
}

hipError_t launch_fwd_finish(const Geo& g, int n, jds_frame_stats* st, const uint32_t* part, int ptiles,
                             hipStream_t s) {
  if (part) {
    hipError_t e = launch_fwd_reduce(n, st, part, ptiles, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_fwd_finish, dim3(n), dim3(64), 0, s, g, st);
  kmark(s, "k_fwd_finish");
  return hipGetLastError();
}

// Per-frame constants and the deterministic luma-SSE sum (inverse phase).
// zero_bin: the forward phase of the same run deferred k_fwd_finish's zero
// bin to here (one launch fewer per forward+inverse run; constants are set here).
__global__ void k_finalize(const Geo g, jds_frame_stats* st, const double* __restrict__ sse_y_part,
                           int tiles, int with_sse, int zero_bin) {
  const int f = blockIdx.x;
  if (threadIdx.x != 0) return;
  jds_frame_stats* s = st + f;
  finalize_frame(g, s, zero_bin);
  if (with_sse) {
    // the tiles' exact integer partials (luma_sse_e6) summed exactly in 64 bits,
    // then converted to double and scaled by 1e-6 (round-to-nearest at each step)
    unsigned long long e = 0ull;
    for (int t = 0; t < tiles; ++t) e += (unsigned long long)sse_y_part[(size_t)f * tiles + t];
    s->sse_y = (double)e / 1e6;
  }
}

hipError_t launch_finalize(const Geo& g, int n, jds_frame_stats* st, const double* part, int tiles, bool with_sse,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(n), dim3(64), 0, s, g, st, part, tiles, (int)with_sse, 0);
  kmark(s, "k_finalize");
  return hipGetLastError();
}

// ------------------------------------------------------------ launchers --

template <int MODE, bool PF>
static hipError_t launch_fwd_t(const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs, const FrameQ* fq,
                               const double* gk, jds_frame_stats* st, jds_selected_block* sel, int sel_blk,
                               hipStream_t s, int in_div) {
  dim3 grid(g.tiles_y * g.tiles_x, n);
  hipLaunchKernelGGL((k_fwd<MODE, PF>), grid, dim3(Cfg<MODE>::TF), 0, s, g, rgb, coeffs, fq, gk, st, sel,
                     sel ? 0 : -1, sel_blk, in_div);
  kmark(s, "k_fwd<%d,%d>", MODE, (int)PF);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_inv_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                               const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                               double* err_y, double* err_rgb, jds_selected_block* sel, int sel_blk,
                               hipStream_t s, int in_div) {
  dim3 grid(g.tiles_y * g.tiles_x, n);
  hipLaunchKernelGGL((k_inv<MODE>), grid, dim3(Cfg<MODE>::TI), 0, s, g, coeffs, fq, rgb_in, rgb_out, st, part,
                     err_y, err_rgb, sel, sel ? 0 : -1, sel_blk, in_div);
  kmark(s, "k_inv<%d>", MODE);
  return hipGetLastError();
}

int inv_tiles(int mode, int H, int W);
hipError_t launch_inv_fast(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                           const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part,
                           const InvFix& fx, hipStream_t s, int in_div, int fin);
hipError_t launch_inv2(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                       const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part, double* err_y,
                       double* err_rgb, hipStream_t s, int in_div, int fin);
hipError_t launch_sel_recon(const int16_t* coeffs, const FrameQ* fq, jds_selected_block* sel, int sel_blk,
                            hipStream_t s);

// phases: bit 0 = forward (k_fwd), bit 1 = inverse (k_inv2 + finalize),
//         bit 2 = use the original one-block-ring k_inv for the inverse,
//         bit 3 = finalize also adds the zero bin (the fast forward deferred it)
hipError_t launch_gen(bool pf, const Geo& g, int n, int in_div, const uint8_t* rgb, uint8_t* rgb_out,
                      int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st, double* part,
                      bool want_sse, double* err_y, double* err_rgb, jds_selected_block* sel, int sel_blk,
                      const AreaTap* tabs, double* sub, double* rec, hipStream_t s, hipEvent_t* ev, int phases);
int gen_px_tiles(const Geo& g);

// g.gen (fractional chroma resampling): the general-geometry kernels of
// jds_gen.hip with the same tail (selected block, finalize); `gb` holds their
// area tables and plane scratch.
hipError_t launch_codec(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, uint8_t* rgb_out,
                        int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st,
                        double* part, bool want_sse, double* err_y, double* err_rgb, jds_selected_block* sel,
                        int sel_blk, hipStream_t s, hipEvent_t* ev, int phases, int in_div, const GenBufs* gb,
                        const InvFix* fx) {
  hipError_t e = hipSuccess;
  const uint8_t* rin = (want_sse || err_y) ? rgb : nullptr;
  if (g.gen) {
    if (!gb) return hipErrorInvalidValue;
    e = launch_gen(pf, g, n, in_div, rgb, rgb_out, coeffs, fq, gk, st, part, rin != nullptr, err_y, err_rgb, sel,
                   sel_blk, gb->tabs, gb->sub, gb->rec, s, ev, phases & 3);
    if (e != hipSuccess || !(phases & 2)) return e;
    if (sel) {
      hipLaunchKernelGGL(k_sel_dequant, dim3(1), dim3(64), 0, s, coeffs, fq, sel, sel_blk);
      kmark(s, "k_sel_dequant");
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_finalize, dim3(n), dim3(64), 0, s, g, st, part, gen_px_tiles(g), (int)(rin != nullptr), 0);
    kmark(s, "k_finalize");
    return hipGetLastError();
  }
  if (phases & 1) {
    if (ev && (e = hipEventRecord(ev[0], s)) != hipSuccess) return e;
    switch (mode) {
      case M420:
        e = pf ? launch_fwd_t<M420, true>(g, n, rgb, coeffs, fq, gk, st, sel, sel_blk, s, in_div)
               : launch_fwd_t<M420, false>(g, n, rgb, coeffs, fq, gk, st, sel, sel_blk, s, in_div);
        break;
      case M422:
        e = pf ? launch_fwd_t<M422, true>(g, n, rgb, coeffs, fq, gk, st, sel, sel_blk, s, in_div)
               : launch_fwd_t<M422, false>(g, n, rgb, coeffs, fq, gk, st, sel, sel_blk, s, in_div);
        break;
      default:
        e = launch_fwd_t<M444, false>(g, n, rgb, coeffs, fq, gk, st, sel, sel_blk, s, in_div);
        break;
    }
    if (e == hipSuccess) e = launch_fwd_finish(g, n, st, nullptr, 0, s);
    if (e != hipSuccess || (ev && (e = hipEventRecord(ev[1], s)) != hipSuccess)) return e;
  }
  if (phases & 2) {
    int tiles = g.tiles_y * g.tiles_x;
    bool fused_fin = false;
    if (!(phases & 4)) {  // jds_inv.hip (default); bit 2 selects the original k_inv
      // certified fast inverse (jds_inv_fast.hip) unless the caller wants the
      // exact kernels or the IntermediateData maps; 4:2:x SSE runs (sweeps)
      // take k_inv_fast<MODE, 1> (round 6: 4.15 against 4.21-4.23 ms per
      // 384-item sweep step with k_inv2<MODE, 1>, sse_y bit for bit), 4:4:4
      // SSE runs the exact kernel
      if (fx && !err_y && (!rin || mode != M444)) {
        // no SSE terms: the fast kernel does k_finalize's per-frame work itself
        fused_fin = !sel && !rin;
        e = launch_inv_fast(mode, g, n, coeffs, fq, rin, rgb_out, st, part, *fx, s, in_div,
                            fused_fin ? ((phases & 8) ? 1 : 0) : -1);
      } else {
        // without SSE terms, maps or a selected block k_inv2 finalizes too
        fused_fin = !err_y && !rin && !sel;
        e = launch_inv2(mode, g, n, coeffs, fq, rin, rgb_out, st, part, err_y, err_rgb, s, in_div,
                        fused_fin ? ((phases & 8) ? 1 : 0) : -1);
      }
      tiles = inv_tiles(mode, g.H, g.W);
    } else switch (mode) {
      case M420:
        e = launch_inv_t<M420>(g, n, coeffs, fq, rin, rgb_out, st, part, err_y, err_rgb, sel, sel_blk, s, in_div);
        break;
      case M422:
        e = launch_inv_t<M422>(g, n, coeffs, fq, rin, rgb_out, st, part, err_y, err_rgb, sel, sel_blk, s, in_div);
        break;
      default:
        e = launch_inv_t<M444>(g, n, coeffs, fq, rin, rgb_out, st, part, err_y, err_rgb, sel, sel_blk, s, in_div);
        break;
    }
    if (e != hipSuccess || (ev && (e = hipEventRecord(ev[2], s)) != hipSuccess)) return e;
    if (sel) {
      hipLaunchKernelGGL(k_sel_dequant, dim3(1), dim3(64), 0, s, coeffs, fq, sel, sel_blk);
      kmark(s, "k_sel_dequant");
      if ((e = hipGetLastError()) != hipSuccess) return e;
      if (!(phases & 4) && (e = launch_sel_recon(coeffs, fq, sel, sel_blk, s)) != hipSuccess) return e;
    }
    if (!fused_fin) {
      hipLaunchKernelGGL(k_finalize, dim3(n), dim3(64), 0, s, g, st, part, tiles,
                         (int)(rin != nullptr), (phases & 8) ? 1 : 0);
      kmark(s, "k_finalize");
      e = hipGetLastError();
    }
  }
  return e;
}

}  // namespace jds
