// jds_fast.hip — the throughput path: fp32 arithmetic with CERTIFIED rounding
// decisions, plus exact fp64 fix-up of the rare ambiguous cases, so results
// stay bit-identical to the reference (engines/pipeline.py:47-63).
//
// Forward (k_fwd32): colour, prefilter, area average, 8x8 DCT (even/odd FMA
// form) and quantisation run in fp32.  For every coefficient a rigorous static
// bound E_uv on |c_fp32 - c_exact| (derived on the host from the fp32
// operation sequence, fast_fwd_thresholds) decides whether
// round-half-even(c/Q) is certain: if t = c*(1/Q) is farther than E_uv/Q (+
// the multiply's own error) from a half-integer, the fp32 quotient rounds
// exactly like the reference's fp64 quotient.  Blocks with any uncertain
// coefficient (~0.5% on random 1080p at Q50, exact ties always) are appended
// to a list; k_fix_fwd recomputes them with the pocketfft-exact fp64 path of
// jds_codec.hip from global memory, overwrites their coefficients and corrects
// the statistics.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "jds_dct8.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

// orthonormal 8-point DCT matrix entries rounded to fp32:
// W[k][i] = s(k) cos((2i+1) k pi / 16), s(0) = sqrt(1/8), s(k) = 1/2
#define JA 0x1.6a09e6p-2f   // sqrt(1/8)
#define JC1 0x1.f6297cp-2f  // cos(1 pi/16) / 2
#define JC2 0x1.d906bcp-2f
#define JC3 0x1.a9b662p-2f
#define JC5 0x1.1c73b4p-2f
#define JC6 0x1.87de2ap-3f
#define JC7 0x1.8f8b84p-4f

// rows k of W restricted to i = 0..3; even rows act on s_i = x_i + x_{7-i},
// odd rows on d_i = x_i - x_{7-i}
static constexpr float FW[8][4] = {
    {JA, JA, JA, JA},      {JC1, JC3, JC5, JC7},    {JC2, JC6, -JC6, -JC2}, {JC3, -JC7, -JC1, -JC5},
    {JA, -JA, -JA, JA},    {JC5, -JC1, JC7, JC3},   {JC6, -JC2, JC2, -JC6}, {JC7, -JC5, JC3, -JC1},
};

// fp32 forward DCT-II of one line: 8 add/sub + 8 four-term FMA chains.  The
// host-side bound (fast_fwd_thresholds) follows exactly this sequence.
__device__ __forceinline__ void fdct8_f32(float (&x)[8]) {
  const float s0 = x[0] + x[7], s1 = x[1] + x[6], s2 = x[2] + x[5], s3 = x[3] + x[4];
  const float d0 = x[0] - x[7], d1 = x[1] - x[6], d2 = x[2] - x[5], d3 = x[3] - x[4];
#pragma unroll
  for (int k = 0; k < 8; k += 2) {
    x[k] = fmaf(FW[k][3], s3, fmaf(FW[k][2], s2, fmaf(FW[k][1], s1, FW[k][0] * s0)));
    x[k + 1] = fmaf(FW[k + 1][3], d3, fmaf(FW[k + 1][2], d2, fmaf(FW[k + 1][1], d1, FW[k + 1][0] * d0)));
  }
}

// fp32 colour conversions (any rounding order is fine: bounded on the host)
__device__ __forceinline__ float luma32(float R, float G, float B) {
  return fmaf(0.114f, B, fmaf(0.587f, G, 0.299f * R));
}
__device__ __forceinline__ float cb32(float R, float G, float B) {
  return fmaf(-0.168736f, R, fmaf(-0.331264f, G, fmaf(0.5f, B, 128.0f)));
}
__device__ __forceinline__ float cr32(float R, float G, float B) {
  return fmaf(-0.081312f, B, fmaf(-0.418688f, G, fmaf(0.5f, R, 128.0f)));
}

__device__ __forceinline__ void unpack32(uint32_t v, float& R, float& G, float& B) {
  R = (float)(v & 255u);
  G = (float)((v >> 8) & 255u);
  B = (float)(v >> 16);
}

struct FastQ {
  float rq[64];      // fp32(1/Q)
  float thr[2][64];  // certification margins in quotient units: [0] luma, [1] chroma
};

constexpr int BS32 = 68;  // floats per 8x8 block in LDS

template <int MODE, bool PF>
__global__ void __launch_bounds__(Cfg<MODE>::TF)
k_fwd32(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
        const FastQ* __restrict__ fq, const float* __restrict__ gk32, jds_frame_stats* __restrict__ st,
        uint2* __restrict__ fixlist, unsigned* __restrict__ fixcount) {
  using C = Cfg<MODE>;
  constexpr int WR = C::TH + 2, WC = C::TW + 2, WN = WR * WC;
  constexpr bool CPLANE = (MODE != M444) && PF;
  constexpr int PLANE_F = CPLANE ? 2 * WN : 0;
  constexpr int BLK_F = C::NB * BS32;
  constexpr int U_F = PLANE_F > BLK_F ? PLANE_F : BLK_F;

  __shared__ uint32_t s_rgb[WN];
  __shared__ __attribute__((aligned(16))) float s_u[U_F];
  __shared__ float s_rq[64], s_thr[2][64];
  __shared__ unsigned s_hist[50];
  __shared__ int s_acc[2];

  const int tid = threadIdx.x;
  const int frame = blockIdx.y;
  const int ty = blockIdx.x / g.tiles_x, tx = blockIdx.x - ty * g.tiles_x;
  const int m0y = ty * C::MY - g.ty_off, m0x = tx * C::MX - g.tx_off;
  const int y0 = m0y * C::MH, x0 = m0x * C::MW;
  const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;

  // 1. stage the RGB window (+1 px ring, BORDER_REFLECT_101 outside the image)
  const bool interior = y0 - 1 >= 0 && x0 - 1 >= 0 && y0 + C::TH + 1 <= g.H && x0 + C::TW + 1 <= g.W;
  if (interior) {
    for (int i = tid; i < WN; i += C::TF) {
      const int r = i / WC, c = i - r * WC;
      const uint8_t* p = img + ((size_t)(y0 - 1 + r) * g.W + (x0 - 1 + c)) * 3;
      s_rgb[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
    }
  } else {
    for (int i = tid; i < WN; i += C::TF) {
      const int r = i / WC, c = i - r * WC;
      const int yy = reflect101(y0 - 1 + r, g.H), xx = reflect101(x0 - 1 + c, g.W);
      const uint8_t* p = img + ((size_t)yy * g.W + xx) * 3;
      s_rgb[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
    }
  }
  if (tid < 64) {
    s_rq[tid] = fq[frame].rq[tid];
    s_thr[0][tid] = fq[frame].thr[0][tid];
    s_thr[1][tid] = fq[frame].thr[1][tid];
  }
  if (tid < 50) s_hist[tid] = 0u;
  if (tid < 2) s_acc[tid] = 0;
  __syncthreads();

  // 2. fp32 chroma planes + Gaussian row pass
  if constexpr (CPLANE) {
    float* s_cb = s_u;
    float* s_cr = s_u + WN;
    for (int i = tid; i < WN; i += C::TF) {
      float R, G, B;
      unpack32(s_rgb[i], R, G, B);
      s_cb[i] = cb32(R, G, B);
      s_cr[i] = cr32(R, G, B);
    }
    __syncthreads();
    constexpr int NRP = WR * (WC - 2);
    constexpr int PER = (NRP + C::TF - 1) / C::TF;
    const float k0 = gk32[0], k1 = gk32[1], k2 = gk32[2];
    float tb[PER], tr[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + j * C::TF;
      if (i < NRP) {
        const int r = i / (WC - 2), c = i - r * (WC - 2) + 1;
        const float* b = s_cb + r * WC + c;
        const float* q = s_cr + r * WC + c;
        tb[j] = fmaf(k2, b[1], fmaf(k1, b[0], k0 * b[-1]));
        tr[j] = fmaf(k2, q[1], fmaf(k1, q[0], k0 * q[-1]));
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

  // 3. one block column per thread, DCT along axis 0
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

  float v[8];
  if (valid) {
    if (plane == 0 || MODE == M444) {
      const int sx = reflect_pad(gx * 8 + line, g.W) - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sy = reflect_pad(gy * 8 + i, g.H) - y0 + 1;
        float R, G, B;
        unpack32(s_rgb[sy * WC + sx], R, G, B);
        v[i] = (plane == 0 ? luma32(R, G, B) : (plane == 1 ? cb32(R, G, B) : cr32(R, G, B))) - 128.0f;
      }
    } else {
      const float* s_pl = s_u + (plane == 1 ? 0 : WN);
      const float k0 = gk32[0], k1 = gk32[1];
      const int sc = reflect_pad(gx * 8 + line, g.wc);
      const int wc0 = C::SX * sc - x0 + 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int sr = reflect_pad(gy * 8 + i, g.hc);
        const int wr0 = C::SY * sr - y0 + 1;
        float s[C::SY][2];
#pragma unroll
        for (int a = 0; a < C::SY; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int w = (wr0 + a) * WC + wc0 + b;
            if constexpr (CPLANE) {
              s[a][b] = fmaf(k0, s_pl[w + WC] + s_pl[w - WC], k1 * s_pl[w]);
            } else {
              float R, G, B;
              unpack32(s_rgb[w], R, G, B);
              s[a][b] = plane == 1 ? cb32(R, G, B) : cr32(R, G, B);
            }
          }
        }
        if constexpr (C::SY == 2)
          v[i] = (((s[0][0] + s[0][1]) + s[1][0]) + s[1][1]) * 0.25f - 128.0f;
        else
          v[i] = (s[0][0] + s[0][1]) * 0.5f - 128.0f;
      }
    }
    fdct8_f32(v);
  }
  if constexpr (CPLANE) __syncthreads();  // block buffer aliases the chroma planes
  float* s_blk = s_u + blk * BS32;
  if (valid) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_blk[i * 8 + line] = v[i];
  }
  __syncthreads();

  // 4. DCT along axis 1, certified quantisation, store
  int nz = 0, mb = 0;
  bool flag = false;
  if (valid) {
    const int u = line;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s_blk[u * 8 + k];
    fdct8_f32(v);
    const float* thr = s_thr[plane ? 1 : 0] + u * 8;
    int q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float t = v[k] * s_rq[u * 8 + k];
      const float r = rintf(t);
      const float margin = fmaf(fabsf(t), 0x1p-22f, thr[k]);
      flag |= (0.5f - fabsf(t - r)) <= margin;
      q[k] = (int)r;
      const int m = q[k] < 0 ? -q[k] : q[k];
      if (m) {
        ++nz;
        mb += 33 - __clz(m);
        if (q[k] >= -100 && q[k] <= 100) atomicAdd(&s_hist[q[k] == 100 ? 49 : (q[k] + 100) >> 2], 1u);
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
  const unsigned long long fm = __ballot(flag);
  if (valid && line == 0 && ((fm >> ((tid & 63) & ~7)) & 0xffull)) {
    const unsigned slot = atomicAdd(fixcount, 1u);
    fixlist[slot] = make_uint2((unsigned)frame, ((unsigned)plane << 24) | (unsigned)bidx);
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

// ---- exact fp64 recomputation of one block column from global memory ----

__device__ __forceinline__ double px_chroma64(const uint8_t* img, const Geo& g, int y, int x, int plane) {
  const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
  const double R = p[0], G = p[1], B = p[2];
  return plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B);
}

// cv2 RowFilter<double> at (y, x), BORDER_REFLECT_101
__device__ double row_pass64(const uint8_t* img, const Geo& g, int y, int x, int plane, const double* k) {
  double t = k[0] * px_chroma64(img, g, y, reflect101(x - 1, g.W), plane);
  t = t + k[1] * px_chroma64(img, g, y, x, plane);
  return t + k[2] * px_chroma64(img, g, y, reflect101(x + 1, g.W), plane);
}

template <int MODE, bool PF>
__device__ double sample64(const uint8_t* img, const Geo& g, int plane, int pr, int pc, const double* k) {
  if (plane == 0 || MODE == M444) {
    const int y = reflect_pad(pr, g.H), x = reflect_pad(pc, g.W);
    const uint8_t* p = img + ((size_t)y * g.W + x) * 3;
    const double R = p[0], G = p[1], B = p[2];
    return plane == 0 ? luma(R, G, B) : (plane == 1 ? chroma_b(R, G, B) : chroma_r(R, G, B));
  }
  constexpr int SY = Cfg<MODE>::SY;
  const int sr = reflect_pad(pr, g.hc), sc = reflect_pad(pc, g.wc);
  double s[SY][2];
  for (int a = 0; a < SY; ++a) {
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

// 64 threads = 8 listed blocks x 8 lines; grid-strides over the fix list
template <int MODE, bool PF>
__global__ void __launch_bounds__(64)
k_fix_fwd(const Geo g, const uint8_t* __restrict__ rgb, int16_t* __restrict__ coeffs,
          const FrameQ* __restrict__ fq, const double* __restrict__ gk, jds_frame_stats* __restrict__ st,
          const uint2* __restrict__ fixlist, const unsigned* __restrict__ fixcount) {
  __shared__ double s_blk[8][BS32];
  const int tid = threadIdx.x, lb = tid >> 3, line = tid & 7;
  const unsigned count = *fixcount;
  const double k[3] = {gk[0], gk[1], gk[2]};
  for (unsigned base = blockIdx.x * 8u; base < count; base += gridDim.x * 8u) {
    const unsigned e = base + lb;
    const bool ok = e < count;
    int frame = 0, plane = 0, bidx = 0, gy = 0, gx = 0;
    double v[8];
    if (ok) {
      const uint2 ent = fixlist[e];
      frame = (int)ent.x;
      plane = (int)(ent.y >> 24);
      bidx = (int)(ent.y & 0xffffffu);
      const int nbx = plane ? g.ncx : g.nbx;
      gy = bidx / nbx;
      gx = bidx - gy * nbx;
      const uint8_t* img = rgb + (size_t)frame * g.H * g.W * 3;
#pragma unroll 1
      for (int i = 0; i < 8; ++i) v[i] = sample64<MODE, PF>(img, g, plane, gy * 8 + i, gx * 8 + line, k) - 128.0;
      dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s_blk[lb][i * 8 + line] = v[i];
    }
    __syncthreads();
    if (ok) {
      const int u = line;
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = s_blk[lb][u * 8 + c];
      dct2_line(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
      const long long off = (long long)frame * g.cpf + (plane == 0 ? 0 : (plane == 1 ? g.off_cb : g.off_cr)) +
                            (long long)bidx * 64 + u * 8;
      uint4* dst = reinterpret_cast<uint4*>(coeffs + off);
      const uint4 old = *dst;
      const uint32_t ow[4] = {old.x, old.y, old.z, old.w};
      uint32_t nw[4] = {0u, 0u, 0u, 0u};
      long long dnz = 0, dmb = 0;
      jds_frame_stats* fs = st + frame;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int qn = (int)__builtin_rint(v[c] / fq[frame].q16[u * 8 + c]);
        const int qo = (int16_t)((ow[c >> 1] >> ((c & 1) * 16)) & 0xffffu);
        nw[c >> 1] |= (uint32_t)(uint16_t)qn << ((c & 1) * 16);
        if (qn != qo) {
          const int mo = qo < 0 ? -qo : qo, mn = qn < 0 ? -qn : qn;
          if (mo) {
            --dnz;
            dmb -= 33 - __clz(mo);
            if (qo >= -100 && qo <= 100)
              atomicAdd((unsigned long long*)&fs->hist[qo == 100 ? 49 : (qo + 100) >> 2], ~0ull);
          }
          if (mn) {
            ++dnz;
            dmb += 33 - __clz(mn);
            if (qn >= -100 && qn <= 100)
              atomicAdd((unsigned long long*)&fs->hist[qn == 100 ? 49 : (qn + 100) >> 2], 1ull);
          }
        }
      }
      *dst = make_uint4(nw[0], nw[1], nw[2], nw[3]);
      if (dnz) atomicAdd((unsigned long long*)&fs->nonzero, (unsigned long long)dnz);
      if (dmb) atomicAdd((unsigned long long*)&fs->magnitude_bits, (unsigned long long)dmb);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ launchers --

template <int MODE, bool PF>
static hipError_t fast_fwd_t(const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs, const FrameQ* fq,
                             const FastQ* fq32, const double* gk, const float* gk32, jds_frame_stats* st,
                             uint2* fixlist, unsigned* fixcount, hipStream_t s) {
  hipLaunchKernelGGL((k_fwd32<MODE, PF>), dim3(g.tiles_y * g.tiles_x, n), dim3(Cfg<MODE>::TF), 0, s, g, rgb, coeffs,
                     fq32, gk32, st, fixlist, fixcount);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_fix_fwd<MODE, PF>), dim3(1024), dim3(64), 0, s, g, rgb, coeffs, fq, gk, st, fixlist,
                     fixcount);
  return hipGetLastError();
}

hipError_t launch_fast_fwd(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, int16_t* coeffs,
                           const FrameQ* fq, const void* fq32, const double* gk, const float* gk32,
                           jds_frame_stats* st, uint2* fixlist, unsigned* fixcount, hipStream_t s) {
  const FastQ* f = (const FastQ*)fq32;
  switch (mode) {
    case M420:
      return pf ? fast_fwd_t<M420, true>(g, n, rgb, coeffs, fq, f, gk, gk32, st, fixlist, fixcount, s)
                : fast_fwd_t<M420, false>(g, n, rgb, coeffs, fq, f, gk, gk32, st, fixlist, fixcount, s);
    case M422:
      return pf ? fast_fwd_t<M422, true>(g, n, rgb, coeffs, fq, f, gk, gk32, st, fixlist, fixcount, s)
                : fast_fwd_t<M422, false>(g, n, rgb, coeffs, fq, f, gk, gk32, st, fixlist, fixcount, s);
    default:
      return fast_fwd_t<M444, false>(g, n, rgb, coeffs, fq, f, gk, gk32, st, fixlist, fixcount, s);
  }
}

// ---------------------------------------------------- host: the bounds --
//
// Rigorous bound on |c_fp32 - c_exact| per coefficient for k_fwd32.  Unit
// roundoff u = 2^-24; each fp32 op rounds once: |fl(a op b) - (a op b)| <= u|result|.
// Input samples: |x| <= X = 128, |x_fp32 - x_exact| <= e_in (colour / prefilter /
// area stage bound below).  One fdct8_f32 pass over inputs (bound X, error e):
//   s_i, d_i:  |.| <= 2X,   error <= 2e + 2uX
//   output k:  |.| <= 2X b_k, error <= b_k (2e + 2uX) + 2uX (b_k + P_k)
// with b_k = sum_i |W_ki| (4 terms) and P_k = sum of the 4 partial sums of
// |W_k0..3| (the magnitudes the FMA chain can reach), the b_k term covering the
// fp32 representation error of W (<= u|W|).  Axis 0 then axis 1.

static void pass_bound(double X, double e, const double* Xin, const double* ein, double* Xout, double* eout,
                       const double W[8][4]) {
  const double u = 0x1p-24;
  for (int k = 0; k < 8; ++k) {
    double b = 0, P = 0, pre = 0;
    for (int i = 0; i < 4; ++i) {
      b += fabs(W[k][i]);
      pre += fabs(W[k][i]);
      P += pre;
    }
    const double x = Xin ? Xin[0] : X, er = ein ? ein[0] : e;
    Xout[k] = 2 * x * b;
    eout[k] = b * (2 * er + 2 * u * x) + 2 * u * x * (b + P);
  }
}

static double fwd_input_error(int plane, int mode, bool pf, const double* gk) {
  const double u = 0x1p-24;
  // luma32: fmaf(kb, B, fmaf(kg, G, kr*R)); constants in fp32; then -128
  const double dkl = fabs((double)0.299f - 0.299) + fabs((double)0.587f - 0.587) + fabs((double)0.114f - 0.114);
  if (plane == 0) return 255 * dkl + u * 255 * (0.299 + 0.886 + 1.0) + u * 128 + 1e-12;
  // cb32 / cr32: fmaf(k1, ., fmaf(k2, ., fmaf(0.5f, ., 128))); 0.5x+128 exact
  const double dkb = fabs((double)-0.168736f + 0.168736) + fabs((double)-0.331264f + 0.331264);
  const double dkr = fabs((double)-0.081312f + 0.081312) + fabs((double)-0.418688f + 0.418688);
  const double ec = 255 * (dkb > dkr ? dkb : dkr) + 2 * u * 256 + 1e-12;  // before -128
  double e = ec;
  if (mode != M444 && pf) {
    const double k0 = gk[0], k1 = gk[1], k2 = gk[2];
    const double k0f = (float)k0, k1f = (float)k1, k2f = (float)k2;
    const double dk = fabs(k0f - k0) + fabs(k1f - k1) + fabs(k2f - k2);
    // row: fmaf(k2, S1, fmaf(k1, S0, k0*S_1)); |S| <= 256, taps sum to 1
    const double er = (k0f + k1f + k2f) * e + dk * 256 + u * 256 * (k0 + (k0 + k1) + 1.0) + 1e-12;
    // column: fmaf(k0, T+1 + T-1, k1*T0)
    e = (k1f + 2 * k0f) * er + dk * 512 + u * (512 + k1 * 256 + 256) + 1e-12;
  }
  if (mode == M420) e = e + u * (512 + 768 + 1024) / 4;  // ((a+b)+c)+d, *0.25 exact
  if (mode == M422) e = e + u * 512 / 2;                  // (a+b), *0.5 exact
  return e + u * 128;                                     // -128
}

void fast_fwd_thresholds(const double* Q, int mode, bool pf, const double* gk, float* rq, float* thr) {
  static const double W[8][4] = {
      {FW[0][0], FW[0][1], FW[0][2], FW[0][3]}, {FW[1][0], FW[1][1], FW[1][2], FW[1][3]},
      {FW[2][0], FW[2][1], FW[2][2], FW[2][3]}, {FW[3][0], FW[3][1], FW[3][2], FW[3][3]},
      {FW[4][0], FW[4][1], FW[4][2], FW[4][3]}, {FW[5][0], FW[5][1], FW[5][2], FW[5][3]},
      {FW[6][0], FW[6][1], FW[6][2], FW[6][3]}, {FW[7][0], FW[7][1], FW[7][2], FW[7][3]},
  };
  for (int i = 0; i < 64; ++i) rq[i] = (float)(1.0 / Q[i]);
  for (int p = 0; p < 2; ++p) {
    const double e_in = fwd_input_error(p, mode, pf, gk);
    double X1[8], e1[8];
    pass_bound(128.0, e_in, nullptr, nullptr, X1, e1, W);
    for (int k = 0; k < 8; ++k) {
      double X2[8], e2[8];
      pass_bound(0, 0, &X1[k], &e1[k], X2, e2, W);
      for (int l = 0; l < 8; ++l) {
        // second-order slack, the fp64 reference's own error, quotient scaling
        const double E = e2[l] * (1 + 1e-5) + 1e-9;
        const double t = E / Q[k * 8 + l] * (1 + 1e-5) + 1e-7;
        thr[p * 64 + k * 8 + l] = (float)t * (1.0f + 0x1p-20f);
      }
    }
  }
}

size_t fast_q_size() { return sizeof(FastQ); }

}  // namespace jds
