// jds_ssim_band.hip — K4 v2: PSNR / SSIM of batches of uint8 RGB image pairs,
// bit-identical to utils/metrics.py:9-28 (skimage.metrics.structural_similarity
// over scipy.ndimage.uniform_filter + NumPy means), laid out for the chip.
//
// The arithmetic contract is the one jds_ssim.hip's first kernels restate
// (kept there as the legacy path the tests compare against):
//   * uniform_filter(size 7, mode 'reflect') = uniform_filter1d along axis 0,
//     then along axis 1; per line a running sum s += (new - old) from
//     s = sum of the reflected first window (left to right from 0.0), every
//     output s / 7;
//   * the SSIM map of skimage (sample covariance 49/48, C1, C2), its mean over
//     the 3-px-cropped map, and the luma MSE, as NumPy's mean computes them:
//     8192-element buffers of the C-order stream, each summed by pairwise_sum,
//     buffer sums accumulated left to right, / n.
//
// What is serial and what is not.  Only the fp64 running sums are order-
// dependent chains; everything else is parallel.  For the R, G, B channels
// every axis-0 running sum is an exact integer (values <= 255^2 * 7 << 2^53),
// so the axis-0 output at row i is RN(S_i / 7) with S_i the exact 7-row
// window sum, computed in any order.  The luma channel's axis-0 sums are real
// fp64 chains (Y = .299R + .587G + .114B is not an integer).  Every axis-1
// running sum is a chain.  So:
//   k_ss_yplanes  Y of both images as fp64 planes (NumPy order, no FMA);
//   k_ss_ychk     the luma axis-0 chains, one lane per (column, quantity), run
//                 down the whole column keeping only the chain state at each
//                 band's first row (checkpoints; no per-row output);
//   k_ss_band     one workgroup per (band of BH output rows, channel, item):
//                 sweeps the band's columns in chunks of CW; per chunk
//                   fill   the axis-0 outputs of the chunk's new columns into
//                          an LDS ring (RGB: exact window sums; Y: the chain
//                          resumed from its checkpoint), lanes = (column, q);
//                   chain  the axis-1 running sums, one lane per (row, q),
//                          reading the ring (conflict-free, odd pitch);
//                   map    the SSIM map of the chunk, one lane per pixel,
//                          written to HBM for the NumPy-order mean;
//                 the next chunk's fill runs beside this chunk's map;
//   k_ss_chunks   the pairwise sums of every full 8192-element buffer: the
//                 buffer is staged through LDS by coalesced 16-B loads, each
//                 lane sums two of a leaf's eight accumulators, and the
//                 pairwise tree (a perfect binary tree over 64 leaves of 128
//                 for a full buffer) is a shuffle butterfly -- fp64 addition
//                 is commutative, only the association is fixed; the last,
//                 partial buffer follows NumPy's recursion (np_chunk_sum);
//   k_ss_final    buffer sums left to right, / n.
// Divisions by 7 use a quotient refined once by FMA (div7): correctly rounded
// for every finite operand (pinned by tests against the
// IEEE division of the legacy kernels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int SB_NP_BUF = 8192;  // NumPy ufunc buffer (elements)
constexpr int SB_CW = 32;        // output columns per chunk
constexpr int SB_RING = 64;      // ring slots per row (power of two >= CW + 7)
static_assert(SB_RING == 2 * SB_CW, "chain_chunk's ring phase is 0 or CW");
constexpr int SB_RP = 65;        // ring row pitch in doubles (odd: lane = row reads hit distinct banks)
constexpr int SB_SP = SB_CW + 1; // chain output tile pitch
constexpr int SB_THREADS = 256;
constexpr int SB_MAX_ITEMS = 32; // image pairs per launch (kernel-argument array)

struct SsimPair {
  const uint8_t* a;
  const uint8_t* b;
};

struct SsimBatch {
  SsimPair pairs[SB_MAX_ITEMS];  // by value: nothing to stage or keep alive on the host
  int H, W;
  int NB;                 // bands of BH output rows: ceil((H - 6) / BH)
  long long ns;           // cropped map size (H - 6) * (W - 6)
  long long ns_pitch;     // map stride per (item, channel): ns rounded up to 64 (16-B aligned buffers)
  long long n_pitch;      // luma plane stride: H * W rounded up to 64
  int nch_s, nch_y;       // 8192-element buffers of the map / of the luma MSE stream
  double c1, c2, cov_norm;
  double* yplanes;        // [item][2][n_pitch]: Y of a, Y of b (H x W each)
  double* ck;             // [item][5][NB][W] luma axis-0 chain states at band starts
  double* smap;           // [item][4][ns_pitch]
  double* chunks;         // [item][5][nch]   nch = max(nch_s, nch_y)
  double* out;            // [item][out_stride]: ssim R, G, B, Y, mse_Y
  int out_stride;
  unsigned long long* sse;  // [item]: sum of (a - b)^2 over the H*W*3 bytes (zeroed by the caller)
};

// x / 7 correctly rounded: q0 = RN(x * RN(1/7)) is within an ulp of x/7, the
// remainder x - 7 q0 is exact (FMA), and one FMA step lands on RN(x / 7):
// x / 7 is never a midpoint (7 is odd) and never within 2^-53 ulp of one.
__device__ __forceinline__ double div7(double x) {
  constexpr double r7 = 1.0 / 7.0;
  const double q0 = x * r7;
  const double r = __builtin_fma(-q0, 7.0, x);
  return __builtin_fma(r, r7, q0);
}

__device__ __forceinline__ double luma_u8(const uint8_t* img, size_t px) {
  const double R = img[px * 3], G = img[px * 3 + 1], B = img[px * 3 + 2];
  return 0.299 * R + 0.587 * G + 0.114 * B;  // utils/metrics.py:17-18, NumPy order
}

// the five filtered quantities: 0 x, 1 y, 2 x*x, 3 y*y, 4 x*y.  Branch-free
// per lane: term = f * g with f = x or y, g = 1, f or y (x * 1.0 == x exactly).
template <typename T>
__device__ __forceinline__ T qterm(int q, T x, T y) {
  const T f = (q == 1 || q == 3) ? y : x;
  const T g = q < 2 ? (T)1 : (q == 4 ? y : f);
  return f * g;
}

// ---------------------------------------------------------------- planes --

// also the RGB squared-error sum of the pair (utils/metrics.py:11, exact
// u64).  Grid-stride over at most SB_PLANE_BLOCKS workgroups per item: one
// atomic per workgroup (same-address atomics serialise at the memory side).
constexpr int SB_PLANE_BLOCKS = 512;

__global__ void __launch_bounds__(256) k_ss_yplanes(SsimBatch B) {
  __shared__ unsigned long long s_sse[4];
  const long long n = (long long)B.H * B.W;
  const SsimPair pr = B.pairs[blockIdx.y];
  double* o = B.yplanes + (size_t)blockIdx.y * 2 * B.n_pitch;
  unsigned long long e = 0;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long long)gridDim.x * 256) {
    int a[3], b[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      a[k] = pr.a[p * 3 + k];
      b[k] = pr.b[p * 3 + k];
      e += (unsigned)((a[k] - b[k]) * (a[k] - b[k]));
    }
    o[p] = 0.299 * (double)a[0] + 0.587 * (double)a[1] + 0.114 * (double)a[2];
    o[B.n_pitch + p] = 0.299 * (double)b[0] + 0.587 * (double)b[1] + 0.114 * (double)b[2];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off, 64);
  if ((threadIdx.x & 63) == 0) s_sse[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0 && B.sse) {
    const unsigned long long tot = s_sse[0] + s_sse[1] + s_sse[2] + s_sse[3];
    if (tot) atomicAdd(&B.sse[blockIdx.y], tot);
  }
}

// ----------------------------------------------------------- luma chains --

// Lane (column j, quantity Q): the axis-0 running sum of column j from row 0
// (scipy's reflected first window, then s += T(i+3) - T(i-4)), storing s at
// each band's first row 3 + BH*b.  Terms of the last 8 rows live in a
// register ring indexed by row & 7; the rows of the next block of 16 steps
// are loaded one block ahead.
template <int Q, int BH>
__device__ __forceinline__ void ychk_lane(const double* __restrict__ X, const double* __restrict__ Y, int H, int W,
                                          int j, int NB, double* __restrict__ ck) {
  constexpr bool NX = Q != 1 && Q != 3, NY = Q != 0 && Q != 2;
  constexpr int U = 16;  // steps per block; BH divides U, so a block's checkpoints sit at fixed steps
  static_assert(U % BH == 0, "band height must divide the block");
  auto term = [](double x, double y) { return qterm<double>(Q, x, y); };
  // loads are never predicated (rows clamped to the image: a clamped row is
  // only loaded past the last step, never used), so a block's loads stay in
  // flight across the previous block's steps
  auto ldx = [&](int r) { return NX ? X[(size_t)min(r, H - 1) * W + j] : 0.0; };
  auto ldy = [&](int r) { return NY ? Y[(size_t)min(r, H - 1) * W + j] : 0.0; };
  double ring[8];
#pragma unroll
  for (int r = 0; r < 7; ++r) ring[r] = term(ldx(r), ldy(r));  // H >= 7
  double s = 0.0;
  s = s + ring[2];
  s = s + ring[1];
  s = s + ring[0];
  s = s + ring[0];
  s = s + ring[1];
  s = s + ring[2];
  s = s + ring[3];
  s = s + (ring[4] - ring[2]);  // i = 1: old row reflect(-3) = 2
  s = s + (ring[5] - ring[1]);  // i = 2
  s = s + (ring[6] - ring[0]);  // i = 3
  ck[j] = s;                    // band 0 starts at row 3
  const int ilast = 3 + BH * (NB - 1);
  // step i (>= 4): new row i + 3 into slot (i + 3) & 7, old row i - 4 from slot (i - 4) & 7
  double nx[U], ny[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    nx[u] = ldx(7 + u);
    ny[u] = ldy(7 + u);
  }
  int i = 4;
  for (; i + U - 1 <= ilast; i += U) {
    double px[U], py[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the next block, in flight while this one runs
      px[u] = ldx(i + U + 3 + u);
      py[u] = ldy(i + U + 3 + u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double tn = term(nx[u], ny[u]);
      const double to = ring[u & 7];  // (i + u - 4) & 7 with i = 4 mod 16
      ring[(u + 7) & 7] = tn;         // (i + u + 3) & 7
      s = s + (tn - to);
      if ((u + 1) % BH == 0) ck[(size_t)((i + u - 3) / BH) * W + j] = s;  // i + u = 3 mod BH
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      nx[u] = px[u];
      ny[u] = py[u];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {  // the last, partial block
    const int ii = i + u;
    if (ii <= ilast) {
      const double tn = term(nx[u], ny[u]);
      const double to = ring[u & 7];
      ring[(u + 7) & 7] = tn;
      s = s + (tn - to);
      if ((u + 1) % BH == 0) ck[(size_t)((ii - 3) / BH) * W + j] = s;
    }
  }
}

template <int BH>
__global__ void __launch_bounds__(64) k_ss_ychk(SsimBatch B) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= B.W) return;
  const int item = blockIdx.z;
  const double* X = B.yplanes + (size_t)item * 2 * B.n_pitch;
  const double* Y = X + B.n_pitch;
  double* ck = B.ck + ((size_t)item * 5 + blockIdx.y) * (size_t)B.NB * B.W;
  switch (blockIdx.y) {
    case 0: ychk_lane<0, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 1: ychk_lane<1, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 2: ychk_lane<2, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 3: ychk_lane<3, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    default: ychk_lane<4, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
  }
}

// ------------------------------------------------------------ band sweep --

template <int BH>
struct BandLds {
  double ring[5][BH][SB_RP];  // axis-0 outputs, column c at slot c & (SB_RING - 1)
  double st[5][BH][SB_SP];    // axis-1 running sums of the current chunk
};

// Raw inputs of one fill lane: the bytes of rows i0 - 3 .. i0 + nr + 2 (RGB)
// or the luma planes' values and the chain's checkpoint (Y), loaded before the
// lane's map work so the loads are in flight meanwhile (nothing consumes them
// before fill_store).
template <int BH>
struct FillRegs {
  int bx[BH + 6], by[BH + 6];
  double tx[BH + 6], ty[BH + 6];
  double s0;
};

template <int BH>
__device__ __forceinline__ void fill_load(const SsimBatch& B, int c, const uint8_t* a, const uint8_t* b,
                                          const double* X, const double* Y, const double* ck, int band, int i0,
                                          int q, int col, FillRegs<BH>& R) {
  const int W = B.W;
  // in a partial last band the rows past H - 1 are clamped (loaded, never
  // used): unpredicated loads stay in flight together
  if (c < 3) {
#pragma unroll
    for (int r = 0; r < BH + 6; ++r) {
      const size_t px = ((size_t)min(i0 - 3 + r, B.H - 1) * W + col) * 3 + c;
      R.bx[r] = a[px];
      R.by[r] = b[px];
    }
  } else {
    // the chain resumes at i0 from its checkpoint (old rows from i0 - 3, new rows from i0 + 4)
    R.s0 = ck[((size_t)q * B.NB + band) * W + col];
#pragma unroll
    for (int r = 0; r < BH + 6; ++r) {
      const size_t p = (size_t)min(i0 - 3 + r, B.H - 1) * W + col;
      R.tx[r] = X[p];
      R.ty[r] = Y[p];
    }
  }
}

template <int BH>
__device__ __forceinline__ void fill_store(int c, int nr, int q, int col, const FillRegs<BH>& R, BandLds<BH>& L) {
  const int slot = col & (SB_RING - 1);
  if (c < 3) {
    int t[BH + 6];
#pragma unroll
    for (int r = 0; r < BH + 6; ++r) t[r] = qterm<int>(q, R.bx[r], R.by[r]);
    int S = 0;
#pragma unroll
    for (int r = 0; r < 7; ++r) S += t[r];  // exact
    L.ring[q][0][slot] = div7((double)S);
#pragma unroll
    for (int rr = 1; rr < BH; ++rr) {
      if (rr < nr) {
        S += t[rr + 6] - t[rr - 1];
        L.ring[q][rr][slot] = div7((double)S);
      }
    }
  } else {
    double s = R.s0;
    L.ring[q][0][slot] = div7(s);
#pragma unroll
    for (int rr = 1; rr < BH; ++rr) {
      if (rr < nr) {
        // row i = i0 + rr: new row i + 3 (index rr + 6), old row i - 4 (rr - 1)
        const double tn = qterm<double>(q, R.tx[rr + 6], R.ty[rr + 6]);
        const double to = qterm<double>(q, R.tx[rr - 1], R.ty[rr - 1]);
        s = s + (tn - to);
        L.ring[q][rr][slot] = div7(s);
      }
    }
  }
}

// One chunk of a chain lane's axis-1 running sum, steps j = jc + jj: every ring
// read first (static LDS offsets: jc is a multiple of CW, so the ring phase
// BASE = jc & (RING - 1) is 0 or CW), then the dependent adds.  FIRST: j = 0
// starts scipy's reflected window; NJ: steps in this chunk (all CW but the last).
template <int BASE, bool FIRST>
__device__ __forceinline__ void chain_chunk(const double* __restrict__ R, double* __restrict__ o, double& s, int nj) {
  constexpr int M = SB_RING - 1;
  double nv[SB_CW], ov[SB_CW];
#pragma unroll
  for (int jj = 0; jj < SB_CW; ++jj) {
    nv[jj] = R[(BASE + jj + 3) & M];
    ov[jj] = R[(BASE + jj - 4) & M];
  }
  int jj0 = 0;
  if constexpr (FIRST) {
    // scipy's first window: reflect(-3 .. 3) = 2, 1, 0, 0, 1, 2, 3; then j = 1..3
    // take their old column from reflect(j - 4) = 2, 1, 0
    const double r0 = R[0], r1 = R[1], r2 = R[2], r3 = R[3];
    s = s + r2;
    s = s + r1;
    s = s + r0;
    s = s + r0;
    s = s + r1;
    s = s + r2;
    s = s + r3;
    o[0] = s;
    s = s + (nv[1] - r2);
    o[1] = s;
    s = s + (nv[2] - r1);
    o[2] = s;
    s = s + (nv[3] - r0);
    o[3] = s;
    jj0 = 4;
  }
  if (nj == SB_CW) {
#pragma unroll
    for (int jj = FIRST ? 4 : 0; jj < SB_CW; ++jj) {
      s = s + (nv[jj] - ov[jj]);
      o[jj] = s;
    }
  } else {
#pragma unroll
    for (int jj = FIRST ? 4 : 0; jj < SB_CW; ++jj) {
      if (jj < nj) {
        s = s + (nv[jj] - ov[jj]);
        o[jj] = s;
      }
    }
  }
  (void)jj0;
}

template <int BH>
__global__ void __launch_bounds__(SB_THREADS) k_ss_band(SsimBatch B) {
  __shared__ BandLds<BH> L;
  const int band = blockIdx.x, c = blockIdx.y, item = blockIdx.z;
  const int H = B.H, W = B.W;
  const int i0 = 3 + BH * band;
  const int nr = min(BH, H - 3 - i0);
  const int t = threadIdx.x;
  const SsimPair pr = B.pairs[item];
  const double* X = B.yplanes + (size_t)item * 2 * B.n_pitch;
  const double* Y = X + B.n_pitch;
  const double* ck = B.ck + (size_t)item * 5 * B.NB * W;
  double* smap = B.smap + ((size_t)item * 4 + c) * B.ns_pitch;
  const int jend = W - 3;  // axis-1 steps j = 0 .. W - 4 (outputs 3 .. W - 4)
  const int nchunks = (jend + SB_CW - 1) / SB_CW;
  const int cw = W - 6;

  // fill lanes: (q, column) over [lo, hi); chunk 0 fills [0, CW + 3), chunk k
  // > 0 the new columns [k CW + 3, (k + 1) CW + 3), clipped to W
  auto fill_cols = [&](int k, int& lo, int& hi) {
    lo = k == 0 ? 0 : k * SB_CW + 3;
    hi = min((k + 1) * SB_CW + 3, W);
  };
  {
    int lo, hi;
    fill_cols(0, lo, hi);
    const int nc = hi - lo;
    if (t < 5 * nc) {
      FillRegs<BH> R;
      const int q = t / nc, col = lo + t % nc;
      fill_load<BH>(B, c, pr.a, pr.b, X, Y, ck, band, i0, q, col, R);
      fill_store<BH>(c, nr, q, col, R, L);
    }
  }
  __syncthreads();

  // chain lanes: (q, row)
  const int cq = t / BH, crow = t % BH;
  const bool chain_lane = t < 5 * BH && crow < nr;
  double s = 0.0;
  for (int k = 0; k < nchunks; ++k) {
    const int jc = k * SB_CW;
    if (chain_lane) {
      const double* R = L.ring[cq][crow];
      double* o = L.st[cq][crow];
      const int nj = min(SB_CW, jend - jc);
      if (k == 0)
        chain_chunk<0, true>(R, o, s, nj);
      else if (jc & SB_CW)
        chain_chunk<SB_CW, false>(R, o, s, nj);
      else
        chain_chunk<0, false>(R, o, s, nj);
    }
    __syncthreads();

    // next chunk's fill (loads first) beside this chunk's map
    int lo = 0, hi = 0;
    if (k + 1 < nchunks) fill_cols(k + 1, lo, hi);
    const int nc = hi - lo;
    const bool fl = t < 5 * nc;
    FillRegs<BH> R;
    int fq = 0, fcol = 0;
    if (fl) {
      fq = t / nc;
      fcol = lo + t % nc;
      fill_load<BH>(B, c, pr.a, pr.b, X, Y, ck, band, i0, fq, fcol, R);
    }
    for (int p = t; p < BH * SB_CW; p += SB_THREADS) {
      const int row = p / SB_CW, jj = p % SB_CW, j = jc + jj;
      if (row < nr && j >= 3 && j < jend) {
        const double ux = div7(L.st[0][row][jj]), uy = div7(L.st[1][row][jj]);
        const double uxx = div7(L.st[2][row][jj]), uyy = div7(L.st[3][row][jj]);
        const double uxy = div7(L.st[4][row][jj]);
        // skimage structural_similarity (sample covariance)
        const double vx = B.cov_norm * (uxx - ux * ux);
        const double vy = B.cov_norm * (uyy - uy * uy);
        const double vxy = B.cov_norm * (uxy - ux * uy);
        const double a1 = 2 * ux * uy + B.c1, a2 = 2 * vxy + B.c2;
        const double b1 = ux * ux + uy * uy + B.c1, b2 = vx + vy + B.c2;
        const double d = b1 * b2;
        smap[(size_t)(i0 + row - 3) * cw + (j - 3)] = (a1 * a2) / d;
      }
    }
    if (fl) fill_store<BH>(c, nr, fq, fcol, R, L);
    __syncthreads();
  }
}

// ---------------------------------------------------------- NumPy means --

// general NumPy pairwise_sum of one buffer (any m <= 8192): the in-order
// leaves of the recursion, their 8-accumulator sums, then the recursion's
// combine order (the last, partial buffer only)
struct SbLeaf {
  int off, n;
};

__device__ int sb_leaves(int n, SbLeaf* out) {
  int so[24], sn[24], sp = 1, cnt = 0;
  so[0] = 0;
  sn[0] = n;
  while (sp > 0) {
    --sp;
    const int off = so[sp], m = sn[sp];
    if (m <= 128) {
      out[cnt++] = {off, m};
    } else {
      int m2 = m / 2;
      m2 -= m2 % 8;
      so[sp] = off + m2;
      sn[sp] = m - m2;
      ++sp;
      so[sp] = off;
      sn[sp] = m2;
      ++sp;
    }
  }
  return cnt;
}

__device__ double sb_leaf_sum(const double* v, int off, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r = r + v[off + i];
    return r;
  }
  double r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = v[off + k];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = r[k] + v[off + i + k];
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + v[off + i];
  return res;
}

__device__ double sb_combine(int n, const double* ls) {
  int fn[24], fph[24];
  double fl[24];
  int sp = 1, li = 0;
  double res = 0.0;
  bool ret = false;
  fn[0] = n;
  fph[0] = 0;
  while (sp > 0) {
    const int t = sp - 1;
    if (ret) {
      ret = false;
      if (fph[t] == 1) {
        fl[t] = res;
        fph[t] = 2;
        int m2 = fn[t] / 2;
        m2 -= m2 % 8;
        fn[sp] = fn[t] - m2;
        fph[sp] = 0;
        ++sp;
      } else {
        res = fl[t] + res;
        --sp;
        ret = true;
      }
      continue;
    }
    if (fn[t] <= 128) {
      res = ls[li++];
      --sp;
      ret = true;
      continue;
    }
    int m2 = fn[t] / 2;
    m2 -= m2 % 8;
    fph[t] = 1;
    fn[sp] = m2;
    fph[sp] = 0;
    ++sp;
  }
  return res;
}

// LDS image of one buffer: element e at e + 8 * (e >> 7) (8-double pad per
// leaf: the per-leaf 16-B reads of a wave land on distinct banks)
__device__ __forceinline__ int sb_pad(int e) { return e + 8 * (e >> 7); }

// grid (nch, 5, items): y < 4 = the SSIM map of channel y, y = 4 the luma
// squared-difference stream (Y(a) - Y(b))^2 over H*W (utils/metrics.py:20 ->
// skimage mean_squared_error)
__global__ void __launch_bounds__(SB_THREADS) k_ss_chunks(SsimBatch B) {
  __shared__ double v[SB_NP_BUF + 8 * (SB_NP_BUF / 128)];
  __shared__ double wsum[4];
  __shared__ SbLeaf leaf[SB_NP_BUF / 64 + 2];
  __shared__ double lsum[SB_NP_BUF / 64 + 2];
  __shared__ int nleaf;
  const int ch = blockIdx.y, item = blockIdx.z, t = threadIdx.x;
  const long long n = ch < 4 ? B.ns : (long long)B.H * B.W;
  const long long c0 = (long long)blockIdx.x * SB_NP_BUF;
  if (c0 >= n) return;
  const int m = (int)min((long long)SB_NP_BUF, n - c0);
  const int nch = max(B.nch_s, B.nch_y);
  double* out = B.chunks + ((size_t)item * 5 + ch) * nch + blockIdx.x;
  // stage the buffer (element e of the buffer at LDS sb_pad(e))
  if (ch < 4) {
    const double* src = B.smap + ((size_t)item * 4 + ch) * B.ns_pitch + c0;
    if (m == SB_NP_BUF) {
#pragma unroll
      for (int k = 0; k < SB_NP_BUF / (2 * SB_THREADS); ++k) {
        const int e = 2 * t + 2 * SB_THREADS * k;
        const double2 w = *reinterpret_cast<const double2*>(src + e);  // 16-B aligned (ns_pitch, c0, e even)
        v[sb_pad(e)] = w.x;
        v[sb_pad(e + 1)] = w.y;
      }
    } else {
      for (int e = t; e < m; e += SB_THREADS) v[sb_pad(e)] = src[e];
    }
  } else {
    // (image0 - image1) ** 2 of the luma planes k_ss_yplanes wrote
    const double* ya = B.yplanes + (size_t)item * 2 * B.n_pitch + c0;
    const double* yb = ya + B.n_pitch;
    if (m == SB_NP_BUF) {
#pragma unroll
      for (int k = 0; k < SB_NP_BUF / (2 * SB_THREADS); ++k) {
        const int e = 2 * t + 2 * SB_THREADS * k;
        const double2 wa = *reinterpret_cast<const double2*>(ya + e);  // 16-B aligned (n_pitch, c0, e even)
        const double2 wb = *reinterpret_cast<const double2*>(yb + e);
        const double d0 = wa.x - wb.x, d1 = wa.y - wb.y;
        v[sb_pad(e)] = d0 * d0;
        v[sb_pad(e + 1)] = d1 * d1;
      }
    } else {
      for (int e = t; e < m; e += SB_THREADS) {
        const double d = ya[e] - yb[e];
        v[sb_pad(e)] = d * d;
      }
    }
  }
  __syncthreads();
  if (m == SB_NP_BUF) {
    // leaf L = t >> 2 (elements 128 L ..), accumulators k = 2 (t & 3), +1
    const int Lf = t >> 2, kp = t & 3;
    const int base = sb_pad(128 * Lf) + 2 * kp;
    double r0 = v[base], r1 = v[base + 1];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      r0 = r0 + v[base + 8 * i];
      r1 = r1 + v[base + 8 * i + 1];
    }
    double p = r0 + r1;            // (r0 + r1), (r2 + r3), (r4 + r5), (r6 + r7)
    p = p + __shfl_xor(p, 1, 64);  // ((r0 + r1) + (r2 + r3)), ((r4 + r5) + (r6 + r7))
    p = p + __shfl_xor(p, 2, 64);  // the leaf
    p = p + __shfl_xor(p, 4, 64);  // leaves 2m + (2m + 1), ...
    p = p + __shfl_xor(p, 8, 64);
    p = p + __shfl_xor(p, 16, 64);
    p = p + __shfl_xor(p, 32, 64);  // leaves 16 w .. 16 w + 15
    if ((t & 63) == 0) wsum[t >> 6] = p;
    __syncthreads();
    if (t == 0) *out = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
  } else {
    if (t == 0) nleaf = sb_leaves(m, leaf);
    __syncthreads();
    // the leaf sums read the unpadded order: copy-free via sb_pad in the getter
    for (int l = t; l < nleaf; l += SB_THREADS) {
      const SbLeaf lr = leaf[l];
      double acc;
      if (lr.n < 8) {
        acc = 0.0;
        for (int i = 0; i < lr.n; ++i) acc = acc + v[sb_pad(lr.off + i)];
      } else {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = v[sb_pad(lr.off + k)];
        int i = 8;
        for (; i < lr.n - (lr.n % 8); i += 8)
          for (int k = 0; k < 8; ++k) r[k] = r[k] + v[sb_pad(lr.off + i + k)];
        acc = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < lr.n; ++i) acc = acc + v[sb_pad(lr.off + i)];
      }
      lsum[l] = acc;
    }
    __syncthreads();
    if (t == 0) *out = sb_combine(m, lsum);
  }
}

// buffer sums left to right from 0.0, then / n: one workgroup per (item,
// quantity); the sums are loaded 256 at a time into LDS (in parallel), one
// lane adds them in order
__global__ void __launch_bounds__(256) k_ss_final(SsimBatch B) {
  __shared__ double part[256];
  const int ch = blockIdx.x, item = blockIdx.y;
  const long long n = ch < 4 ? B.ns : (long long)B.H * B.W;
  const int nb = (int)((n + SB_NP_BUF - 1) / SB_NP_BUF);
  const int nch = max(B.nch_s, B.nch_y);
  const double* cs = B.chunks + ((size_t)item * 5 + ch) * nch;
  double acc = 0.0;
  for (int k0 = 0; k0 < nb; k0 += 256) {
    if (k0 + (int)threadIdx.x < nb) part[threadIdx.x] = cs[k0 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
      const int m = min(256, nb - k0);
      for (int k = 0; k < m; ++k) acc = acc + part[k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) B.out[(size_t)item * B.out_stride + ch] = acc / (double)n;
}

// ------------------------------------------------------------------ host --

#ifndef JDS_SSIM_BH
#define JDS_SSIM_BH 8
#endif
constexpr int SB_BH = JDS_SSIM_BH;  // band height (rows per workgroup; 8 or 16)

int ssim_bands(int H) { return (H - 6 + SB_BH - 1) / SB_BH; }

// scratch doubles per item for H x W (H, W >= 7)
static long long ns_pitch_of(int H, int W) { return (((long long)(H - 6) * (W - 6)) + 63) & ~63LL; }
static long long n_pitch_of(int H, int W) { return ((long long)H * W + 63) & ~63LL; }

int ssim_batch_max_items() { return SB_MAX_ITEMS; }

// scratch doubles per item for H x W (H, W >= 7)
size_t ssim_batch_scratch_doubles(int H, int W) {
  const size_t n = (size_t)H * W;
  const size_t nch = (n + SB_NP_BUF - 1) / SB_NP_BUF;  // n > ns
  return 2 * (size_t)n_pitch_of(H, W) + 5 * (size_t)ssim_bands(H) * W + 4 * (size_t)ns_pitch_of(H, W) + 5 * nch;
}

// SSIM R, G, B, Y and the luma MSE of `items` (<= SB_MAX_ITEMS) pairs (device
// image pointers a[i], b[i]) into out[item * out_stride + 0..4], and the RGB
// squared-error sums into sse[item] (nullable; the caller zeroes it); scratch:
// items * ssim_batch_scratch_doubles(H, W).
hipError_t launch_psnr_ssim_batch(const uint8_t* const* a, const uint8_t* const* b, int items, int H, int W,
                                  double c1, double c2, double* scratch, double* out, int out_stride,
                                  unsigned long long* sse, hipStream_t s) {
  if (items < 1 || items > SB_MAX_ITEMS || H < 7 || W < 7) return hipErrorInvalidValue;
  SsimBatch B{};
  for (int i = 0; i < items; ++i) B.pairs[i] = {a[i], b[i]};
  B.H = H;
  B.W = W;
  B.NB = ssim_bands(H);
  B.ns = (long long)(H - 6) * (W - 6);
  B.ns_pitch = ns_pitch_of(H, W);
  B.n_pitch = n_pitch_of(H, W);
  const long long n = (long long)H * W;
  B.nch_s = (int)((B.ns + SB_NP_BUF - 1) / SB_NP_BUF);
  B.nch_y = (int)((n + SB_NP_BUF - 1) / SB_NP_BUF);
  const int nch = std::max(B.nch_s, B.nch_y);
  B.c1 = c1;
  B.c2 = c2;
  B.cov_norm = 49.0 / 48.0;
  B.yplanes = scratch;
  B.ck = B.yplanes + (size_t)items * 2 * B.n_pitch;
  B.smap = B.ck + (size_t)items * 5 * B.NB * W;
  B.chunks = B.smap + (size_t)items * 4 * B.ns_pitch;
  B.out = out;
  B.out_stride = out_stride;
  B.sse = sse;
  hipLaunchKernelGGL(k_ss_yplanes, dim3((unsigned)std::min<long long>((n + 255) / 256, SB_PLANE_BLOCKS), items),
                     dim3(256), 0, s, B);
  hipLaunchKernelGGL(k_ss_ychk<SB_BH>, dim3((W + 63) / 64, 5, items), dim3(64), 0, s, B);
  hipLaunchKernelGGL(k_ss_band<SB_BH>, dim3(B.NB, 4, items), dim3(SB_THREADS), 0, s, B);
  hipLaunchKernelGGL(k_ss_chunks, dim3(nch, 5, items), dim3(SB_THREADS), 0, s, B);
  hipLaunchKernelGGL(k_ss_final, dim3(5, items), dim3(256), 0, s, B);
  return hipGetLastError();
}

}  // namespace jds
