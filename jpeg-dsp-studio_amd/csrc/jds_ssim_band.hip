// jds_ssim_band.hip — K4 v2: PSNR / SSIM of batches of uint8 RGB image pairs,
// bit-identical to utils/metrics.py:9-28 (skimage.metrics.structural_similarity
// over scipy.ndimage.uniform_filter + NumPy means), laid out for the chip.
//
// The arithmetic contract (oracle/cpu_ref.py psnr_ssim_raw restates it; the
// tests compare all six values bit for bit):
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
//   k_ss_ychk     the luma axis-0 chains, one lane per column (all five), run
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
//                 partial buffer follows NumPy's recursion;
//   k_ss_final    buffer sums left to right, / n.
// Divisions by 7 use a quotient refined once by FMA (div7): correctly rounded
// for every finite operand (pinned by the tests against
// the oracle's IEEE division).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <algorithm>
#include <type_traits>

#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int SB_NP_BUF = 8192;  // NumPy ufunc buffer (elements)
constexpr int SB_CW = 32;        // output columns per chunk
// ring slots per row (k_ss_band's two schedules): a chunk's chain reads
// columns jc - 4 .. jc + CW + 2; the serial schedule fills the next chunk
// (CW columns from jc + CW + 3) after it: >= CW + 7, 48 (bases jc mod 48: 0,
// 32, 16); the overlapped one (OV) fills it in the same barrier interval: >= 2
// CW + 7, 80 (bases 0, 32, 64, 16, 48).  Row pitch RING + 1 doubles (odd:
// lane = row reads hit distinct banks).
template <bool OV>
constexpr int sb_ring() { return OV ? 80 : 48; }
static_assert(sb_ring<false>() >= SB_CW + 7 && (3 * SB_CW) % sb_ring<false>() == 0, "chain_chunk's ring phases");
static_assert(sb_ring<true>() >= 2 * SB_CW + 7 && (5 * SB_CW) % sb_ring<true>() == 0, "chain_chunk's ring phases");
constexpr int SB_SP = SB_CW + 1; // chain output tile pitch
constexpr int SB_THREADS = 256;
constexpr int SB_MAX_ITEMS = 4096;  // image pairs per launch (scratch bounds it first)
#ifdef JDS_SSIM_NO_LF  // tools: A/B builds only -- big luma launches store the map (k_ss_chunks sums it)
constexpr bool SB_LEAF_FOLD = false;
#else
constexpr bool SB_LEAF_FOLD = true;  // big luma launches fold the map into leaf sums in k_ss_band
#endif

struct SsimPair {
  const uint8_t* a;
  const uint8_t* b;
};

// NumPy's pairwise_sum recursion over the last, partial 8192-element buffer
// of a stream (m < 8192 elements), built on the host (pw_tree): its leaves in
// order (<= 65, each <= 128 elements) and its internal nodes sorted by height
// (children: index < nl a leaf, else nl + internal index), so the device sums
// the leaves in parallel and combines one height per barrier interval.
constexpr int PW_MAXN = 72;
struct PwTree {
  uint16_t off[PW_MAXN], n[PW_MAXN];
  uint8_t l[PW_MAXN], r[PW_MAXN];
  uint8_t hs[10];  // internal nodes of height h + 1: [hs[h], hs[h + 1])
  uint8_t nl, ni, nh;
};

struct SsimBatch {
  const SsimPair* pairs;  // [items] (device)
  int smap_ch;            // maps per item in smap: 4 (R, G, B, Y) or 1 (Y only: k_ss_rows takes R, G, B)
  int H, W;
  int NB;                 // bands of BH output rows: ceil((H - 6) / BH)
  long long ns;           // cropped map size (H - 6) * (W - 6)
  long long ns_pitch;     // map stride per (item, channel): ns rounded up to 64 (16-B aligned buffers)
  long long n_pitch;      // luma plane stride: H * W rounded up to 64
  long long ck_pitch;     // checkpoint stride per item: 5 * NB * W rounded up to 64
  int nch_s, nch_y;       // 8192-element buffers of the map / of the luma MSE stream
  double c1, c2, cov_norm;
  double* yplanes;        // [item][2][n_pitch]: Y of a, Y of b (H x W each)
  double* ck;             // [item][5][NB][W] luma axis-0 chain states at band starts
  double* smap;           // [item][4][ns_pitch]
  double* chunks;         // [item][5][nch]   nch = max(nch_s, nch_y)
  double* out;            // [item][out_stride]: ssim R, G, B, Y, mse_Y
  int out_stride;
  unsigned long long* sse;  // [item]: sum of (a - b)^2 over the H*W*3 bytes (zeroed by the caller)
  PwTree tree_s, tree_y;    // the partial buffers of the map stream and of the luma MSE stream
  // leaf-folded luma map (k_ss_band<.., LF>, big launches without the R, G, B
  // bands): per item at lf + item * lf_pitch, the sums of the leaves inside one
  // map row [nfull * 64], the row-crossing leaves' elements at lf_raws (128 per
  // slot) and the partial buffer's at lf_rawp (k_ss_rows' layout; k_ss_rgbsum
  // finishes them)
  double* lf;
  long long lf_pitch, lf_raws, lf_rawp, efull;
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

// map2: skimage's 2 * ux * uy + C1 and 2 * vxy + C2 as fma(2, ux * uy, C1) and
// fma(2, vxy, C2): doubling is exact (2 ux uy = 2 (ux uy) bit for bit), so
// the fma's one rounding is the sum's.
//
// n / d correctly rounded for the SSIM map's operands (d = b1 b2 >= C1 C2 ~ 380,
// both far from overflow and underflow): the compiler's fp64 division without
// its range scaling (v_div_scale: a factor of 1 here) and special-case fixup
// (v_div_fixup: finite, nonzero operands) -- reciprocal, two Newton steps, the
// quotient and its one fma correction, the same operations and roundings.
__device__ __forceinline__ double div_map(double n, double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  const double q = n * y;
  const double r = __builtin_fma(-d, q, n);
  return __builtin_fma(r, y, q);
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

// Lane = column j, all five quantities: the axis-0 running sums of column j
// from row 0 (scipy's reflected first window, then s_q += T_q(i+3) - T_q(i-4),
// T_q recomputed from the row's x and y -- the same product, the same value),
// storing s_q at each band's first row 3 + BH*b.  The lane forms the luma of
// both images from the bytes (k_ss_yplanes' expression; no planes: the band
// kernel and the luma MSE form it from the bytes too) and sums its column's
// RGB squared error.  x and y of the last 8 rows live in a register ring
// indexed by row & 7; the next block of U rows' bytes are loaded one block
// ahead, a dword per lane per image: the wave's 64 pixels of a row are 192
// contiguous bytes, and each lane takes its pixel's three bytes from the two
// dwords holding them by ds_bpermute (two loads per row instead of six byte
// loads: the byte loads kept the address units busy).
template <int BH>
__global__ void __launch_bounds__(64) k_ss_ychk(SsimBatch B) {
  constexpr int U = 8;  // steps per block; BH divides U, so a block's checkpoints sit at fixed steps
  static_assert(U % BH == 0, "band height must divide the block");
  const int H = B.H, W = B.W, NB = B.NB, item = blockIdx.y;
  const int j0 = blockIdx.x * 64 + threadIdx.x;
  const bool ok = j0 < W;
  const int j = ok ? j0 : W - 1;  // (lanes past W load column W - 1, store and count nothing)
  const SsimPair pr = B.pairs[item];
  double* ck = B.ck + (size_t)item * B.ck_pitch + j;  // [q][band][column]
  const size_t qs = (size_t)NB * W;
  unsigned long long sse = 0;
  // lane l's dword of a row: bytes [a0 + 4 l, + 4) of the wave's segment
  // (a0: the segment's first byte rounded down to a dword).  Loads are never
  // predicated: rows clamped to the image (a clamped row is only loaded past
  // the last step and never counted), addresses past the image's last whole
  // dword clamped to it, the partial last dword patched from bytes (last row
  // only).
  typedef const uint32_t __attribute__((address_space(1)))* gdw;
  const int lane = threadIdx.x;
  const uint32_t nbytes = (uint32_t)H * (uint32_t)W * 3u;  // < 2^32 (launch_psnr_ssim_batch)
  const uint32_t alast = (nbytes & ~3u) - 4u;
  const uint32_t jw0 = blockIdx.x * 64u;
  struct Px {
    uint32_t a, b;
  };
  auto seg = [&](int r) { return ((uint32_t)min(r, H - 1) * (uint32_t)W + jw0) * 3u; };
  auto ldp = [&](int r, Px& p) {
    const uint32_t a = (seg(r) & ~3u) + 4u * (uint32_t)lane;
    const uint32_t ac = a < alast ? a : alast;
    p.a = *(gdw)(pr.a + ac);
    p.b = *(gdw)(pr.b + ac);
    if (r >= H - 1 && a > alast && a < nbytes) {  // (rare: the image's last dword)
      uint32_t xa = 0u, xb = 0u;
      for (uint32_t k = 0; a + k < nbytes && k < 4; ++k) {
        xa |= (uint32_t)pr.a[a + k] << (8 * k);
        xb |= (uint32_t)pr.b[a + k] << (8 * k);
      }
      p.a = xa;
      p.b = xb;
    }
  };
  auto cvt = [&](int r, const Px& p, double& x, double& y) {
    const uint32_t o = (seg(r) & 3u) + 3u * (uint32_t)lane, d4 = (o >> 2) * 4u, sh = o & 3u;
    const uint32_t wa = __builtin_amdgcn_alignbyte((uint32_t)__builtin_amdgcn_ds_bpermute((int)d4 + 4, (int)p.a),
                                                   (uint32_t)__builtin_amdgcn_ds_bpermute((int)d4, (int)p.a), sh);
    const uint32_t wb = __builtin_amdgcn_alignbyte((uint32_t)__builtin_amdgcn_ds_bpermute((int)d4 + 4, (int)p.b),
                                                   (uint32_t)__builtin_amdgcn_ds_bpermute((int)d4, (int)p.b), sh);
    int ca[3], cb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ca[k] = (int)((wa >> (8 * k)) & 255u);
      cb[k] = (int)((wb >> (8 * k)) & 255u);
    }
    x = 0.299 * (double)ca[0] + 0.587 * (double)ca[1] + 0.114 * (double)ca[2];  // utils/metrics.py:17-18
    y = 0.299 * (double)cb[0] + 0.587 * (double)cb[1] + 0.114 * (double)cb[2];
    if (r < H) {
      if (ok) {
#pragma unroll
        for (int k = 0; k < 3; ++k) sse += (unsigned)((ca[k] - cb[k]) * (ca[k] - cb[k]));
      }
    }
  };
  double rx[8], ry[8];
  {
    Px p0[7];
#pragma unroll
    for (int r = 0; r < 7; ++r) ldp(r, p0[r]);  // H >= 7
#pragma unroll
    for (int r = 0; r < 7; ++r) cvt(r, p0[r], rx[r], ry[r]);
  }
  double s[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    auto T = [&](int r) { return qterm<double>(q, rx[r], ry[r]); };
    double v = 0.0;
    v = v + T(2);
    v = v + T(1);
    v = v + T(0);
    v = v + T(0);
    v = v + T(1);
    v = v + T(2);
    v = v + T(3);
    v = v + (T(4) - T(2));  // i = 1: old row reflect(-3) = 2
    v = v + (T(5) - T(1));  // i = 2
    v = v + (T(6) - T(0));  // i = 3
    s[q] = v;
    if (ok) ck[q * qs] = v;  // band 0 starts at row 3
  }
  const int ilast = 3 + BH * (NB - 1);
  // step i (>= 4): new row i + 3 into slot (i + 3) & 7, old row i - 4 from slot (i - 4) & 7
  double nx[U], ny[U];
  auto row_step = [&](int ii, int u) {  // ii = 4 mod 8
#pragma unroll
    for (int q = 0; q < 5; ++q)
      s[q] = s[q] + (qterm<double>(q, nx[u], ny[u]) - qterm<double>(q, rx[u & 7], ry[u & 7]));
    rx[(u + 7) & 7] = nx[u];
    ry[(u + 7) & 7] = ny[u];
    if ((u + 1) % BH == 0 && ok) {  // ii = 3 mod BH
#pragma unroll
      for (int q = 0; q < 5; ++q) ck[q * qs + (size_t)((ii - 3) / BH) * W] = s[q];
    }
  };
  Px pb[U];  // the bytes of the current block's rows i + 3 .. i + U + 2
#pragma unroll
  for (int u = 0; u < U; ++u) ldp(7 + u, pb[u]);
  int i = 4;
  for (; i + U - 1 <= ilast; i += U) {
    Px pn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ldp(i + U + 3 + u, pn[u]);  // the next block, in flight while this one runs
#pragma unroll
    for (int u = 0; u < U; ++u) cvt(i + 3 + u, pb[u], nx[u], ny[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) row_step(i + u, u);
#pragma unroll
    for (int u = 0; u < U; ++u) pb[u] = pn[u];
  }
  // the last, partial block; then the rows below the last step's window
#pragma unroll
  for (int u = 0; u < U; ++u) cvt(i + 3 + u, pb[u], nx[u], ny[u]);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i + u <= ilast) row_step(i + u, u);
  for (int r = i + U + 3; r < H; ++r) {
    Px p;
    double x, y;
    ldp(r, p);
    cvt(r, p, x, y);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sse += __shfl_xor(sse, off, 64);
  if (threadIdx.x == 0 && B.sse && sse) atomicAdd(&B.sse[item], sse);
}

// Small batches (k_ss_ychkq): lane = (column j, quantity Q), five times the
// lanes of k_ss_ychk for the latency of one item's 1,080-step columns.
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
__global__ void __launch_bounds__(64) k_ss_ychkq(SsimBatch B) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= B.W) return;
  const int item = blockIdx.z;
  const double* X = B.yplanes + (size_t)item * 2 * B.n_pitch;
  const double* Y = X + B.n_pitch;
  double* ck = B.ck + (size_t)item * B.ck_pitch + (size_t)blockIdx.y * B.NB * B.W;
  switch (blockIdx.y) {
    case 0: ychk_lane<0, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 1: ychk_lane<1, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 2: ychk_lane<2, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    case 3: ychk_lane<3, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
    default: ychk_lane<4, BH>(X, Y, B.H, B.W, j, B.NB, ck); break;
  }
}

// ------------------------------------------------------------ band sweep --

constexpr int SB_SC = SB_CW + 4;  // staged columns per chunk (chunk 0 fills CW + 3)

// LU: the luma channel's workgroups (fp64 inputs and chain checkpoints) and
// the RGB channels' (bytes) are separate kernel instances, so the RGB ones --
// three in four -- carry 34 KB of LDS instead of 51 and four fit a CU
template <int BH, bool LU, bool OV>
struct BandLds {
  double ring[5][BH][sb_ring<OV>() + 1];  // axis-0 outputs, column c at slot c mod sb_ring<OV>()
  double st[5][BH][SB_SP];    // axis-1 running sums of the current chunk
  // inputs of the fill of one chunk, double-buffered (staged two chunks ahead):
  // per staged column, rows i0 - 3 .. i0 + BH + 2 of both images.  RGB: four
  // rows per word, consecutive columns in consecutive words (the fill's and
  // the staging's accesses of a wave hit distinct banks); luma: a column's
  // 2 (BH + 6) values at an odd stride in doubles (likewise)
  struct InB {
    uint32_t b4[2][4][SB_SC];  // RGB: byte r & 3 of word [image][r >> 2][column]
  };
  struct InY {
    double y[SB_SC][2 * (BH + 6) + 1];  // luma: [column][image * (BH + 6) + r]
  };
  typename std::conditional<LU, InY, InB>::type in[1];  // (one buffer: committed in the chain phase)
  double ck[1][5][LU ? SB_SC : 1];  // luma: the axis-0 chains' states at row i0
};

// fill columns of chunk k: chunk 0 fills [0, CW + 3), chunk k > 0 the new
// columns [k CW + 3, (k + 1) CW + 3), clipped to W
__device__ __forceinline__ void fill_cols(int k, int W, int& lo, int& hi) {
  lo = k == 0 ? 0 : k * SB_CW + 3;
  hi = min((k + 1) * SB_CW + 3, W);
}

// Staging of one chunk's fill inputs: every thread loads up to SE elements
// (coalesced: consecutive threads take consecutive columns of a row) into
// registers; stage_commit writes them into the chunk's LDS buffer once the
// loads have landed, a barrier interval later in program order.  The
// per-thread element geometry does not change along the band: StagePlan holds
// it (the row's first pixel, and column | image << 8 | committed << 9 | LDS
// byte offset << 12), so a chunk costs a min, two adds and the load per element.
template <int BH>
struct StageCfg {
  static constexpr int NR = BH + 6, SE = (2 * NR * SB_SC + SB_THREADS - 1) / SB_THREADS;
};
template <int BH>
struct StagePlan {
  uint32_t row[StageCfg<BH>::SE];
  uint32_t ccv[StageCfg<BH>::SE];
};
// YP: the luma from k_ss_yplanes' planes (small batches, which run it for
// k_ss_ychkq) instead of the bytes
template <int BH, bool LU, bool YP = false>
struct StageRegs {
  uint32_t b[LU ? 1 : StageCfg<BH>::SE];
  uint32_t y[LU && !YP ? StageCfg<BH>::SE : 1][3];  // luma: the pixel's three bytes (converted when committed)
  double yp[LU && YP ? StageCfg<BH>::SE : 1];
  double ck;
};

template <int BH>
__device__ __forceinline__ StagePlan<BH> stage_plan(int c, int H, int W, int i0) {
  constexpr int NR = StageCfg<BH>::NR, SE = StageCfg<BH>::SE;
  static_assert(2 * NR * SB_SC <= SE * SB_THREADS, "staging slots");
  StagePlan<BH> P;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < SE; ++i) {
    const int e = t + i * SB_THREADS;
    const bool ok = e < 2 * NR * SB_SC;
    const int cc = e % SB_SC, r = ok ? (e / SB_SC) % NR : 0, im = ok ? e / (SB_SC * NR) : 0;
    // rows past H - 1 (partial last band) load a valid clamped element that is never used
    P.row[i] = (uint32_t)min(i0 - 3 + r, H - 1) * (uint32_t)W;
    const uint32_t off = c < 3 ? (uint32_t)(((im * 4 + (r >> 2)) * SB_SC + cc) * 4 + (r & 3))
                               : (uint32_t)((cc * (2 * NR + 1) + im * NR + r) * 8);
    P.ccv[i] = (uint32_t)cc | ((uint32_t)im << 8) | ((ok ? 1u : 0u) << 9) | (off << 12);
  }
  return P;
}

template <int BH, bool LU, bool YP>
__device__ __forceinline__ void stage_issue(const SsimBatch& B, int c, const uint8_t* a, const uint8_t* b,
                                            const double* Xp, const double* ck, int band, int k,
                                            int nchunks, const StagePlan<BH>& P, StageRegs<BH, LU, YP>& R) {
  constexpr int SE = StageCfg<BH>::SE;
  if (k >= nchunks) return;
  int lo, hi;
  fill_cols(k, B.W, lo, hi);
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < SE; ++i) {
    // columns past hi load a valid clamped element that is never used: no predicated loads
    const uint32_t cc = P.ccv[i] & 255u, col = min((uint32_t)lo + cc, (uint32_t)hi - 1u);
    const uint32_t px = P.row[i] + col;
    const bool im = (P.ccv[i] >> 8) & 1u;
#ifdef JDS_SSIM_PROBE_NOSTAGE  // tools: timing probe without the staging loads (wrong values)
    if constexpr (LU)
      R.y[i][0] = R.y[i][1] = R.y[i][2] = px & 255u;
    else
      R.b[i] = px & 255u;
    (void)im;
#else
    if constexpr (LU && YP) {
      R.yp[i] = Xp[(im ? B.n_pitch : 0) + px];
    } else if constexpr (LU) {
      const uint8_t* img = im ? b : a;
#pragma unroll
      for (int k3 = 0; k3 < 3; ++k3) R.y[i][k3] = img[px * 3u + (uint32_t)k3];
    } else {
      R.b[i] = (im ? b : a)[px * 3u + (uint32_t)c];
    }
#endif
  }
  if (LU && t < 5 * SB_SC) {
    const int q = t / SB_SC, col = min(lo + t % SB_SC, hi - 1);
    R.ck = ck[((size_t)q * B.NB + band) * B.W + col];
  }
}

template <int BH, bool LU, bool YP, class LDS>
__device__ __forceinline__ void stage_commit(int c, int k, int nchunks, const StagePlan<BH>& P,
                                             const StageRegs<BH, LU, YP>& R, LDS& L) {
  constexpr int SE = StageCfg<BH>::SE;
  if (k >= nchunks) return;
  const int t = threadIdx.x, buf = 0;
  uint8_t* base = reinterpret_cast<uint8_t*>(&L.in[buf]);
#pragma unroll
  for (int i = 0; i < SE; ++i) {
    if ((P.ccv[i] >> 9) & 1u) {
      uint8_t* d = base + (P.ccv[i] >> 12);
      if constexpr (LU)
        *reinterpret_cast<double*>(d) =  // utils/metrics.py:17-18, k_ss_yplanes' expression
            YP ? R.yp[i] : 0.299 * (double)R.y[i][0] + 0.587 * (double)R.y[i][1] + 0.114 * (double)R.y[i][2];
      else
        *d = (uint8_t)R.b[i];
    }
  }
  if constexpr (LU)
    if (t < 5 * SB_SC) L.ck[buf][t / SB_SC][t % SB_SC] = R.ck;
  (void)c;
}

// the fill of chunk k from its staged inputs: lanes (q, column), the axis-0
// outputs of the band's rows into the ring (RGB: exact window sums; luma: the
// chain resumed from its checkpoint)
template <int BH, bool LU, int RING, class LDS>
__device__ __forceinline__ void fill_chunk(int c, int nr, int k, int W, LDS& L, int t) {
  constexpr int NR = BH + 6;
  int lo, hi;
  fill_cols(k, W, lo, hi);
  const int nc = hi - lo;
  // luma: lanes (quantity group, column) -- x, x^2 | y, y^2 | x y -- so each
  // staged row is read once per group instead of once per quantity (the
  // fill's LDS reads -60 %: luma half 40.3 -> 38.5-39.3 us per 1080p item in a
  // 384-pair batch)
  if constexpr (LU) {
    if (t < 0 || t >= 3 * nc) return;
    const int g = t / nc, cc = t % nc, buf = 0;
    const int slot = (lo + cc) % RING;
    const double* tx = &L.in[buf].y[cc][0];
    const double* ty = &L.in[buf].y[cc][NR];
    if (g < 2) {  // q = g (the mean) and q = g + 2 (the square), from one image's rows
      const double* tv = g == 0 ? tx : ty;
      double s1 = L.ck[buf][g][cc], s2 = L.ck[buf][g + 2][cc];
      L.ring[g][0][slot] = div7(s1);
      L.ring[g + 2][0][slot] = div7(s2);
#pragma unroll
      for (int rr = 1; rr < BH; ++rr) {
        if (rr < nr) {
          const double vn = tv[rr + 6], vo = tv[rr - 1];
          s1 = s1 + (vn - vo);
          s2 = s2 + (vn * vn - vo * vo);
          L.ring[g][rr][slot] = div7(s1);
          L.ring[g + 2][rr][slot] = div7(s2);
        }
      }
    } else {
      double s = L.ck[buf][4][cc];
      L.ring[4][0][slot] = div7(s);
#pragma unroll
      for (int rr = 1; rr < BH; ++rr) {
        if (rr < nr) {
          s = s + (tx[rr + 6] * ty[rr + 6] - tx[rr - 1] * ty[rr - 1]);
          L.ring[4][rr][slot] = div7(s);
        }
      }
    }
  } else {  // R, G, B: lanes (quantity, column), exact integer window sums
    if (t < 0 || t >= 5 * nc) return;
    const int q = t / nc, cc = t % nc, buf = 0;
    const int slot = (lo + cc) % RING;
    (void)c;
    uint32_t xw[4], yw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xw[j] = L.in[buf].b4[0][j][cc];
      yw[j] = L.in[buf].b4[1][j][cc];
    }
    int tt[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r)
      tt[r] = qterm<int>(q, (int)((xw[r >> 2] >> (8 * (r & 3))) & 255u), (int)((yw[r >> 2] >> (8 * (r & 3))) & 255u));
    int S = 0;
#pragma unroll
    for (int r = 0; r < 7; ++r) S += tt[r];  // exact
    L.ring[q][0][slot] = div7((double)S);
#pragma unroll
    for (int rr = 1; rr < BH; ++rr) {
      if (rr < nr) {
        S += tt[rr + 6] - tt[rr - 1];
        L.ring[q][rr][slot] = div7((double)S);
      }
    }
  }
}

// One chunk of a chain lane's axis-1 running sum, steps j = jc + jj, in two
// halves of CW / 2 steps: each half's ring reads first (static LDS offsets: jc
// is a multiple of CW, so the ring phase BASE = jc mod RING is 0, 32 or 16),
// then its dependent adds (half the values in flight: fewer VGPRs for the
// workgroups a CU holds).  FIRST: j = 0 starts scipy's reflected window; NJ:
// steps in this chunk (all CW but the last).
template <int RING>
constexpr int rmod(int x) { return ((x % RING) + RING) % RING; }
template <int BASE, bool FIRST, int RING>
__device__ __forceinline__ void chain_chunk(const double* __restrict__ R, double* __restrict__ o, double& s, int nj) {
  constexpr int HC = SB_CW / 2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    double nv[HC], ov[HC];
#pragma unroll
    for (int i = 0; i < HC; ++i) {
      nv[i] = R[rmod<RING>(BASE + h * HC + i + 3)];
      ov[i] = R[rmod<RING>(BASE + h * HC + i - 4)];
    }
    int i0 = 0;
    if (FIRST && h == 0) {
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
      i0 = 4;
    }
    if (nj == SB_CW) {
#pragma unroll
      for (int i = 0; i < HC; ++i) {
        if (i >= i0) {
          s = s + (nv[i] - ov[i]);
          o[h * HC + i] = s;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < HC; ++i) {
        if (i >= i0 && h * HC + i < nj) {
          s = s + (nv[i] - ov[i]);
          o[h * HC + i] = s;
        }
      }
    }
  }
}

// OV: the overlapped schedule (chain beside the next chunk's fill; a larger
// ring, 46 KB for luma): shorter per-chunk latency, for small launches whose
// few workgroups are latency-bound; big launches keep the serial one (36 KB,
// four workgroups per CU).
// LF (luma, serial schedule): the map is not stored; it goes into an LDS tile,
// and in the next chain phase wave 1 (idle there) folds it into NumPy's leaf
// sums, one lane per (row, accumulator) -- k_ss_rows' scheme: whole leaves
// inside a map row summed here, the elements of row-crossing leaves and of the
// partial buffer written raw for k_ss_rgbsum.
template <int BH, bool LU, bool YP = false, bool OV = false, bool LF = false>
__global__ void __launch_bounds__(SB_THREADS) __attribute__((amdgpu_waves_per_eu(LU && !OV ? 4 : (LU ? 3 : 5)))) k_ss_band(SsimBatch B) {
  static_assert(!LF || (LU && !YP && !OV && BH * 8 == 64), "leaf folding: the serial luma band, one wave of (row, accumulator) lanes");
  constexpr int RING = sb_ring<OV>();
  __shared__ BandLds<BH, LU, OV> L;
  __shared__ double MT[LF ? BH : 1][LF ? SB_CW : 1];  // LF: the chunk's map values
  __shared__ double FIN[LF ? BH : 1][8];              // LF: each row's leaf accumulators, final
  const int band = blockIdx.x, c = LU ? 3 : blockIdx.y, item = blockIdx.z;
  const int H = B.H, W = B.W;
  const int i0 = 3 + BH * band;
  const int nr = min(BH, H - 3 - i0);
  const int t = threadIdx.x;
  const SsimPair pr = B.pairs[item];
  const double* ck = B.ck + (size_t)item * B.ck_pitch;
  const double* Xp = YP ? B.yplanes + (size_t)item * 2 * B.n_pitch : nullptr;
  double* smap = B.smap + ((size_t)item * B.smap_ch + (B.smap_ch == 4 ? c : 0)) * B.ns_pitch;
  const int jend = W - 3;  // axis-1 steps j = 0 .. W - 4 (outputs 3 .. W - 4)
  const int nchunks = (jend + SB_CW - 1) / SB_CW;
  const int cw = W - 6;

  if constexpr (OV) {
    // Per chunk k, two barrier intervals: (A) wave 0 runs chunk k's chains
    // while waves 1-3 fill chunk k + 1 (the ring holds both column ranges);
    // (B) every lane maps chunk k, then chunk k + 2's inputs go into the one LDS
    // input buffer (chunk k + 1's fill has read it) and chunk k + 4's loads are
    // issued (two register sets: each load has two chunk periods)
    static_assert(5 * BH <= 64 && 5 * (SB_CW + 3) <= SB_THREADS - 64, "chain lanes in wave 0, fill lanes in waves 1-3");
    const int ft = t - 64;  // fill lane
    const StagePlan<BH> P = stage_plan<BH>(c, H, W, i0);
    StageRegs<BH, LU, YP> RA, RB;
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 0, nchunks, P, RA);
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 1, nchunks, P, RB);
    stage_commit<BH, LU, YP>(c, 0, nchunks, P, RA, L);
    __syncthreads();
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 2, nchunks, P, RA);
    fill_chunk<BH, LU, RING>(c, nr, 0, W, L, ft);
    __syncthreads();
    stage_commit<BH, LU, YP>(c, 1, nchunks, P, RB, L);
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 3, nchunks, P, RB);
    __syncthreads();

    // chain lanes: (q, row)
    const int cq = t / BH, crow = t % BH;
    const bool chain_lane = t < 5 * BH && crow < nr;
    double s = 0.0;
    // one chunk: cur holds chunk k + 2's loaded inputs (committed after the
    // map), then receives chunk k + 4's
    auto step = [&](int k, StageRegs<BH, LU, YP>& cur) {
      const int jc = k * SB_CW;
  #ifndef JDS_SSIM_PROBE_NOCHAIN  // tools: timing probes only (wrong values)
      if (chain_lane) {
  #else
      if (false) {
  #endif
        const double* Rg = L.ring[cq][crow];
        double* o = L.st[cq][crow];
        const int nj = min(SB_CW, jend - jc);
        const int base = jc % RING;
        if (k == 0)
          chain_chunk<0, true, RING>(Rg, o, s, nj);
        else if (base == 32)
          chain_chunk<32, false, RING>(Rg, o, s, nj);
        else if (base == 64)
          chain_chunk<64, false, RING>(Rg, o, s, nj);
        else if (base == 16)
          chain_chunk<16, false, RING>(Rg, o, s, nj);
        else if (base == 48)
          chain_chunk<48, false, RING>(Rg, o, s, nj);
        else
          chain_chunk<0, false, RING>(Rg, o, s, nj);
      }
  #ifndef JDS_SSIM_PROBE_NOFILL
      if (k + 1 < nchunks) fill_chunk<BH, LU, RING>(c, nr, k + 1, W, L, ft);
  #endif
      __syncthreads();
      // chunk k's map, chunk k + 2's inputs, chunk k + 4's loads
  #ifdef JDS_SSIM_PROBE_NOMAP
      if (false)
  #endif
      for (int p = t; p < BH * SB_CW; p += SB_THREADS) {
        const int row = p / SB_CW, jj = p % SB_CW, j = jc + jj;
        if (row < nr && j >= 3 && j < jend) {
          const double ux = div7(L.st[0][row][jj]), uy = div7(L.st[1][row][jj]);
          const double uxx = div7(L.st[2][row][jj]), uyy = div7(L.st[3][row][jj]);
          const double uxy = div7(L.st[4][row][jj]);
          // skimage structural_similarity (sample covariance)
          const double vx = B.cov_norm * (uxx - ux * ux);
          const double vy = B.cov_norm * (uyy - uy * uy);
          const double pxy = ux * uy;
          const double vxy = B.cov_norm * (uxy - pxy);
          const double a1 = __builtin_fma(2.0, pxy, B.c1), a2 = __builtin_fma(2.0, vxy, B.c2);  // (map2: exact doubling)
          const double b1 = ux * ux + uy * uy + B.c1, b2 = vx + vy + B.c2;
          const double d = b1 * b2;
          smap[(size_t)(i0 + row - 3) * cw + (j - 3)] = div_map(a1 * a2, d);
        }
      }
      stage_commit<BH, LU, YP>(c, k + 2, nchunks, P, cur, L);
      stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, k + 4, nchunks, P, cur);
      __syncthreads();
    };
    for (int k = 0; k < nchunks; k += 2) {
      step(k, RA);
      if (k + 1 < nchunks) step(k + 1, RB);
    }
  } else {
    // chunk k's fill inputs are loaded three chunks ahead (two register sets)
    // and stored into the one LDS input buffer in the chain phase before its
    // fill: each load has a barrier interval and a half before its value is
    // needed
    const StagePlan<BH> P = stage_plan<BH>(c, H, W, i0);
    StageRegs<BH, LU, YP> RA, RB;
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 0, nchunks, P, RA);
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 1, nchunks, P, RB);
    stage_commit<BH, LU, YP>(c, 0, nchunks, P, RA, L);
    __syncthreads();
    stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, 2, nchunks, P, RA);
    fill_chunk<BH, LU, RING>(c, nr, 0, W, L, t);
    __syncthreads();

    // chain lanes: (q, row)
    const int cq = t / BH, crow = t % BH;
    const bool chain_lane = t < 5 * BH && crow < nr;
    double s = 0.0;
    // LF leaf lanes (wave 1): map row i0 + lrow - 3, accumulator lkq; its
    // stream elements [rs, rs + cw), whole leaves in [hs, te) (recomputed per
    // chunk: only the accumulator stays live across the loop)
    const bool leaf_wave = LF && t >= 64 && t < 128;
    double acc = 0.0;
    auto leaf_pass = [&](int k) {
      // (the lane's constants are re-derived here from an opaque copy of its
      // index: hoisted out of the chunk loop they held registers all along)
      int tl = t;
      asm volatile("" : "+v"(tl));
      const int lrow = ((tl - 64) >> 3) & 7, lkq = tl & 7;
      const bool lrowok = lrow < nr;
      const long long r = i0 + lrow - 3;
      const long long rs = r * cw;
      const long long hs = (rs + 127) & ~127LL, te = min((rs + cw) & ~127LL, B.efull);
      double* const lfb = B.lf + (size_t)item * B.lf_pitch;
      const int jc = k * SB_CW;
      const long long eb = rs + (jc - 3);  // element of column jc
      const int jj0 = (int)((lkq - eb) & 7LL);
#pragma unroll
      for (int i = 0; i < SB_CW / 8; ++i) {
        const int jj = jj0 + 8 * i, j = jc + jj;
        if (lrowok && j >= 3 && j < jend) {
          const long long e = eb + jj;
          const double m = MT[lrow][jj];
          if (e >= hs && e < te) {  // NumPy's leaf: accumulator e mod 8, in element order
            const int p = (int)(e & 127LL);
            acc = p < 8 ? m : acc + m;
            if (p >= 120) FIN[lrow][lkq] = acc;
          } else if (e >= B.efull) {
            lfb[B.lf_rawp + (e - B.efull)] = m;
          } else {  // a row-crossing leaf (slot: the row it ends in; narrow maps a slot per leaf)
            const long long slot = cw >= 128 ? (e < hs ? r : r + 1) : (e >> 7);
            lfb[B.lf_raws + slot * 128 + (e & 127LL)] = m;
          }
        }
      }
      // a leaf of this row ends in this chunk: its eight accumulators summed in
      // NumPy's order, ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))
      const long long elo = eb + max(0, 3 - jc), ehi = eb + min(SB_CW, jend - jc);
      const long long e127 = elo | 127LL;
      const bool done = lrowok && e127 < ehi && e127 >= hs && e127 < te;
      double x = FIN[lrow][lkq];
      x = x + __shfl_xor(x, 1, 64);
      x = x + __shfl_xor(x, 2, 64);
      x = x + __shfl_xor(x, 4, 64);
      if (done && lkq == 0) lfb[e127 >> 7] = x;
    };
    // one chunk: cur holds chunk k + 1's loaded inputs (committed beside the
    // chain), then receives chunk k + 3's
    auto step = [&](int k, StageRegs<BH, LU, YP>& cur) {
      const int jc = k * SB_CW;
  #ifndef JDS_SSIM_PROBE_NOCHAIN  // tools: timing probes only (wrong values)
      if (chain_lane) {
  #else
      if (false) {
  #endif
        const double* Rg = L.ring[cq][crow];
        double* o = L.st[cq][crow];
        const int nj = min(SB_CW, jend - jc);
        const int base = jc % RING;
        if (k == 0)
          chain_chunk<0, true, RING>(Rg, o, s, nj);
        else if (base == 32)
          chain_chunk<32, false, RING>(Rg, o, s, nj);
        else if (base == 16)
          chain_chunk<16, false, RING>(Rg, o, s, nj);
        else
          chain_chunk<0, false, RING>(Rg, o, s, nj);
      }
      if constexpr (LF)
        if (leaf_wave && k > 0) leaf_pass(k - 1);  // chunk k - 1's map (the tile is rewritten after the barrier)
      stage_commit<BH, LU, YP>(c, k + 1, nchunks, P, cur, L);  // chunk k's fill has read the buffer
      __syncthreads();
      // chunk k + 1's fill, chunk k's map, chunk k + 3's loads
  #ifndef JDS_SSIM_PROBE_NOFILL
      if (k + 1 < nchunks) fill_chunk<BH, LU, RING>(c, nr, k + 1, W, L, t);
  #endif
  #ifdef JDS_SSIM_PROBE_NOMAP
      if (false)
  #endif
      // the map in waves 2-3, two pixels a lane, beside the fill in waves 0-1
      // (its 3 * 36 lanes): one map per lane in every wave after the fill made
      // waves 0-1 the interval's long pole -- luma half 38.7 -> 36.5 us per
      // 1080p item in a 384-pair batch
      static_assert(5 * BH <= 64 && 3 * SB_SC <= 128 && BH * SB_CW == 2 * 128, "fill in waves 0-1, map in waves 2-3");
      for (int p = t - 128; t >= 128 && p < BH * SB_CW; p += 128) {
        const int row = p / SB_CW, jj = p % SB_CW, j = jc + jj;
        if (row < nr && j >= 3 && j < jend) {
          const double ux = div7(L.st[0][row][jj]), uy = div7(L.st[1][row][jj]);
          const double uxx = div7(L.st[2][row][jj]), uyy = div7(L.st[3][row][jj]);
          const double uxy = div7(L.st[4][row][jj]);
          // skimage structural_similarity (sample covariance)
          const double vx = B.cov_norm * (uxx - ux * ux);
          const double vy = B.cov_norm * (uyy - uy * uy);
          const double pxy = ux * uy;
          const double vxy = B.cov_norm * (uxy - pxy);
          const double a1 = __builtin_fma(2.0, pxy, B.c1), a2 = __builtin_fma(2.0, vxy, B.c2);  // (map2: exact doubling)
          const double b1 = ux * ux + uy * uy + B.c1, b2 = vx + vy + B.c2;
          const double d = b1 * b2;
          if constexpr (LF)
            MT[row][jj] = div_map(a1 * a2, d);
          else
            smap[(size_t)(i0 + row - 3) * cw + (j - 3)] = div_map(a1 * a2, d);
        }
      }
      stage_issue<BH, LU, YP>(B, c, pr.a, pr.b, Xp, ck, band, k + 3, nchunks, P, cur);
      __syncthreads();
    };
    for (int k = 0; k < nchunks; k += 2) {
      step(k, RB);
      if (k + 1 < nchunks) step(k + 1, RA);
    }
    if constexpr (LF)
      if (leaf_wave) leaf_pass(nchunks - 1);
  }
}

// --------------------------------------------------- RGB rows (k_ss_rows) --
//
// The R, G, B channels' SSIM maps, one lane per map row: every axis-0 window
// sum is an exact integer (order-free), so a lane forms its row's axis-0
// outputs A_q(j) = RN(S_q(j) / 7) column by column from the 7 input rows
// around it, carries scipy's axis-1 running sums s_q(j) = s_q(j - 1) +
// (A_q(j + 3) - A_q(j - 4)) itself (the last 7 columns' A_q in a register
// ring, slot column mod 7 -- static in a loop unrolled by 7) and evaluates the
// map at once.  No exchange between lanes, one
// barrier per 14-column chunk (the staging of both images' 70 input rows
// through LDS).  A workgroup is 64 map rows x 3 channels (a wave per
// channel); one launch covers every item of the batch (device pair array), so
// the grid holds ~50 waves per 1080p item instead of the band kernel's
// latency-bound chain phases.
//
// The NumPy mean is folded in: the map stream (C order over the cropped map)
// is summed in 8192-element buffers by pairwise_sum, whose leaves are the
// 128-element aligned runs; a lane sums the leaves that lie inside its row
// (eight accumulators by element index mod 8, NumPy's leaf order) and writes
// one double per leaf; the elements of leaves that cross a row boundary, and
// the last partial buffer, are written raw (k_ss_rgbsum sums them).
constexpr int SR_ROWS = 64;                                    // map rows per workgroup (a lane each)
constexpr int SR_IN = SR_ROWS + 6;                             // input rows staged
constexpr int SR_CW = 14;                                      // columns per staged chunk (2 x 7: static ring slots)
constexpr int SR_RG = (SR_IN + 3) / 4;                         // staged row groups (four rows' bytes per word)
constexpr int SR_PG = (SR_CW + 3) / 4;                         // 4-pixel groups per chunk row
constexpr int SR_THREADS = 192;                                // three channels
static_assert(2 * SR_RG * SR_PG <= SR_THREADS, "one staging item (image, row group, pixel group) per thread");

struct RgbBatch {
  const SsimPair* pairs;  // [items] (device)
  int H, W, cw;           // cw = W - 6
  int nfull, mpart;       // full 8192-element buffers of a map stream; elements of the last, partial one
  long long ns, efull;    // ns = (H - 6) * cw; efull = 8192 * nfull
  double c1, c2, cov_norm;
  double* lsum;           // [item][nchan][lsum_pitch]: sums of the leaves inside one map row
  double* raws;           // [item][nchan][raws_pitch]: elements of row-crossing leaves, 128 per slot
  double* rawp;           // [item][nchan][rawp_pitch]: the partial buffer's elements
  double* chunks;         // [item][nchan][chunks_pitch]: buffer sums
  double* out;            // [item][out_stride]: ssim R, G, B (nchan 3) or Y (nchan 1, ch_out 3)
  int out_stride;
  long long lsum_pitch, raws_pitch, rawp_pitch, chunks_pitch;
  int nchan, ch_out;      // maps per item: 3 (k_ss_rows) or 1 (k_ss_band's leaf-folded luma); first out slot
  PwTree tree;            // the partial buffer's pairwise tree
};

// slot of a row-crossing leaf starting at element e0: rows of >= 128 elements
// are crossed by one leaf per row boundary (slot = the row it ends in); narrow
// maps take a slot per leaf
__host__ __device__ __forceinline__ long long rs_slot(long long e0, int cw) { return cw >= 128 ? (e0 + 127) / cw : e0 >> 7; }

// the map value of one pixel from its five axis-1 running sums (skimage
// structural_similarity with the sample covariance; k_ss_band's order)
__device__ __forceinline__ double ssim_px(const double (&s)[5], double c1, double c2, double cov_norm) {
  const double ux = div7(s[0]), uy = div7(s[1]);
  const double uxx = div7(s[2]), uyy = div7(s[3]);
  const double uxy = div7(s[4]);
  const double vx = cov_norm * (uxx - ux * ux);
  const double vy = cov_norm * (uyy - uy * uy);
  const double pxy = ux * uy;
  const double vxy = cov_norm * (uxy - pxy);
  const double a1 = __builtin_fma(2.0, pxy, c1), a2 = __builtin_fma(2.0, vxy, c2);  // (map2: exact doubling)
  const double b1 = ux * ux + uy * uy + c1, b2 = vx + vy + c2;
  const double d = b1 * b2;
  return div_map(a1 * a2, d);
}

__global__ void __launch_bounds__(SR_THREADS) __attribute__((amdgpu_waves_per_eu(3))) k_ss_rows(RgbBatch B) {
  // [buffer][image][channel][column][row group]: a word holds one channel's
  // bytes of one column for four consecutive input rows (the staging
  // transposes), so a lane's 7-row window of a column is two words shifted by
  // its row mod 4, summed by dot4 (v_dot4_u32_u8)
  __shared__ uint32_t L[2][2][3][SR_CW][SR_RG];
  __shared__ double LF[8][SR_THREADS];  // the current leaf's eight accumulators, per lane
  // the means' axis-0 outputs RN(n / 7), n <= 7 * 255, as a table (14 KB; four
  // workgroups per CU still fit): 34.4 against 33.2 us per 1080p item alone
  __shared__ double AT[7 * 255 + 1];
  for (int i = threadIdx.x; i <= 7 * 255; i += SR_THREADS) AT[i] = div7((double)i);
  const int rb = blockIdx.x, item = blockIdx.y, t = threadIdx.x;
  const int ch = t >> 6, lane = t & 63;
  const int H = B.H, W = B.W, cw = B.cw;
  const int R0 = rb * SR_ROWS;  // map row R0 + lane reads input rows R0 + lane .. + 6
  const int r = R0 + lane;
  const bool rowok = r < H - 6;
  const SsimPair pr = B.pairs[item];
  const uint32_t nbytes = (uint32_t)H * (uint32_t)W * 3u;  // < 2^32 (launch_ssim_rgb)
  const size_t ic = (size_t)item * 3 + ch;
  double* lsum = B.lsum + ic * B.lsum_pitch;
  double* raws = B.raws + ic * B.raws_pitch;
  double* rawp = B.rawp + ic * B.rawp_pitch;
  const int nchunks = (W + SR_CW - 1) / SR_CW;

  // staging item of thread t (t < 2 SR_RG SR_PG): image si, row group sg
  // (input rows R0 + 4 sg .. + 3), pixel group sp (chunk pixels 4 sp .. + 3).
  // Per row: the 12 bytes of its four pixels from four unconditional global
  // dword loads (addresses past the image's last whole dword clamped to it:
  // those bytes belong to columns >= W or rows never used; the image's last,
  // partial dword patched from bytes, rarely), aligned by the row's byte
  // offset mod 4 when committed
  typedef const uint32_t __attribute__((address_space(1)))* gdw;
  const bool stager = t < 2 * SR_RG * SR_PG;
  const int sg = t % SR_RG, sp = (t / SR_RG) % SR_PG, si = t / (SR_RG * SR_PG);
  const uint8_t* simg = si ? pr.b : pr.a;
  const uint32_t alast = (nbytes & ~3u) - 4u;  // the last whole dword (H W 3 >= 147)
  uint32_t rowoff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rowoff[q] = (uint32_t)min(R0 + 4 * sg + q, H - 1) * (uint32_t)W * 3u + 12u * (uint32_t)sp;
  uint32_t v[4][4];
  auto issue = [&](int k) {
    if (!stager) return;
    unsigned partial = 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t o = rowoff[q] + 42u * (uint32_t)k, a0 = o & ~3u;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t a = a0 + 4u * d;
        v[q][d] = *(gdw)(simg + (a < alast ? a : alast));
        if (a > alast && a < nbytes) partial |= 1u << (4 * q + d);
      }
    }
    if (partial) {  // (rare: the image's last dword)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (partial & (1u << (4 * q + d))) {
            const uint32_t a = ((rowoff[q] + 42u * (uint32_t)k) & ~3u) + 4u * d;
            uint32_t x = 0u;
            for (uint32_t b = 0; b < 4; ++b)
              if (a + b < nbytes) x |= (uint32_t)simg[a + b] << (8 * b);
            v[q][d] = x;
          }
        }
      }
    }
  };
  // transpose: word (channel c, pixel i) = byte 3 i + c of the four rows
  auto commit = [&](int k) {
    if (!stager) return;
    uint32_t w[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t sh = (rowoff[q] + 42u * (uint32_t)k) & 3u;
#pragma unroll
      for (int d = 0; d < 3; ++d) w[q][d] = __builtin_amdgcn_alignbyte(v[q][d + 1], v[q][d], sh);
    }
    uint32_t(*dst)[3][SR_CW][SR_RG] = L[k & 1];
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) {
      const int d = kk >> 2, b = kk & 3, i = kk / 3, c = kk % 3;
      const uint32_t lo = __builtin_amdgcn_perm(w[1][d], w[0][d], 0x0c0c0000u | ((4u + b) << 8) | (uint32_t)b);
      const uint32_t hi = __builtin_amdgcn_perm(w[3][d], w[2][d], 0x00000c0cu | ((4u + b) << 24) | ((uint32_t)b << 16));
      if (4 * sp + i < SR_CW) dst[si][c][4 * sp + i][sg] = lo | hi;
    }
  };

  // this map row's stream elements [rs, re); whole leaves in [hs, te).  Column
  // jn emits element rs + jn - 6: the in-leaf columns are [jh, jt) (32-bit
  // lane constants, so the common path does no 64-bit index work)
  const long long rs = (long long)r * cw, re = rs + cw;
  const long long hs = (rs + 127) & ~127LL, te = re & ~127LL;
  const int jh = (int)(hs - rs) + 6;
  const int jt = (int)max(min(min(te, B.efull) - rs, (long long)cw), (long long)(jh - 6)) + 6;
  const long long hleaf = hs >> 7;

  issue(0);
  commit(0);
  __syncthreads();
  // the window sums of the last 7 columns, slot column mod 7: x | y << 16, xx,
  // yy, xy
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  // the axis-0 outputs A_q of the last 7 columns, slot column mod 7 (a ring of
  // their integer window sums, A(j - 4) recomputed, held 128 VGPRs at 4 waves
  // per SIMD: 37.8 against 34.5 us per 1080p item alone)
  double ra[5][7];
  auto a_of = [](int v) { return div7((double)v); };
  auto nv_q = [](const int (&n)[4], int q) { return q == 0 ? (n[0] & 0xffff) : q == 1 ? (n[0] >> 16) : n[q - 1]; };
  auto a_q = [&](int q, int u) { return ra[q][u]; };
  auto a_nq = [&](const int (&n)[4], int q) { return q < 2 ? AT[nv_q(n, q)] : a_of(nv_q(n, q)); };
  // the window sums of column jj of the staged chunk (buffer kb): input rows
  // lane .. lane + 3 and lane + 4 .. lane + 6 as two words, summed by dot4
  const int g0 = lane >> 2;
  const uint32_t gsh = (uint32_t)lane & 3u;
  auto wsum = [&](int kb, int jj, int (&n)[4]) {
    const uint32_t* ta = &L[kb][0][ch][jj][g0];
    const uint32_t* tb = &L[kb][1][ch][jj][g0];
    const uint32_t xl = __builtin_amdgcn_alignbyte(ta[1], ta[0], gsh);
    const uint32_t xh = __builtin_amdgcn_alignbyte(ta[2], ta[1], gsh) & 0x00ffffffu;
    const uint32_t yl = __builtin_amdgcn_alignbyte(tb[1], tb[0], gsh);
    const uint32_t yh = __builtin_amdgcn_alignbyte(tb[2], tb[1], gsh) & 0x00ffffffu;
    constexpr uint32_t ones = 0x01010101u;
    const uint32_t sx = __builtin_amdgcn_udot4(xh, ones, __builtin_amdgcn_udot4(xl, ones, 0u, false), false);
    const uint32_t sy = __builtin_amdgcn_udot4(yh, ones, __builtin_amdgcn_udot4(yl, ones, 0u, false), false);
    n[0] = (int)(sx | (sy << 16));
    n[1] = (int)__builtin_amdgcn_udot4(xh, xh, __builtin_amdgcn_udot4(xl, xl, 0u, false), false);
    n[2] = (int)__builtin_amdgcn_udot4(yh, yh, __builtin_amdgcn_udot4(yl, yl, 0u, false), false);
    n[3] = (int)__builtin_amdgcn_udot4(xh, yh, __builtin_amdgcn_udot4(xl, yl, 0u, false), false);
  };
  // the map value of column jn - 3 (stream element rs + jn - 6) into its leaf,
  // or raw (leaves that cross a row boundary: slot r for the head of this row,
  // r + 1 for its tail; narrow maps a slot per leaf)
  auto emit = [&](int jn) {
    if (!rowok) return;
    const double m = ssim_px(s, B.c1, B.c2, B.cov_norm);
    if (jn >= jh && jn < jt) {
      // NumPy's leaf: accumulator e mod 8 starts at the leaf's first 8
      // elements and adds every 8th after them; the sum once the leaf is full
      const int d = jn - jh, p = d & 127, kq = p & 7;
      const double a = p < 8 ? m : LF[kq][t] + m;
      LF[kq][t] = a;
      if (p == 127) {
        double rk[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) rk[kk] = kk == 7 ? a : LF[kk][t];
        lsum[hleaf + (d >> 7)] = ((rk[0] + rk[1]) + (rk[2] + rk[3])) + ((rk[4] + rk[5]) + (rk[6] + rk[7]));
      }
    } else {
      const long long e = rs + (jn - 6);
      if (e >= B.efull) {
        rawp[e - B.efull] = m;
      } else {  // e < hs or e >= te: a row-crossing leaf
        const long long slot = cw >= 128 ? (e < hs ? r : r + 1) : (e >> 7);
        raws[slot * 128 + (e & 127)] = m;
      }
    }
  };

  // column jn enters (ring slot u = jn mod 7), column jn - 7 (the same slot) leaves
  auto step = [&](int kb, int jj, int jn, int u) {
    int n[4];
    wsum(kb, jj, n);
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const double an = a_nq(n, q);
      s[q] = s[q] + (an - ra[q][u]);
      ra[q][u] = an;
    }
    emit(jn);
  };

  // chunk 0, columns 0 .. 6: scipy's first window (W >= 7): reflect(-3 .. 3) =
  // 2, 1, 0, 0, 1, 2, 3, then outputs 1 .. 3 take their old column from
  // reflect(-3 .. -1) = 2, 1, 0
  if (1 < nchunks) issue(1);
#pragma unroll
  for (int u = 0; u < 7; ++u) {
    int n[4];
    wsum(0, u, n);
#pragma unroll
    for (int q = 0; q < 5; ++q) ra[q][u] = a_nq(n, q);
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    double x = 0.0;
    x = x + a_q(q, 2);
    x = x + a_q(q, 1);
    x = x + a_q(q, 0);
    x = x + a_q(q, 0);
    x = x + a_q(q, 1);
    x = x + a_q(q, 2);
    x = x + a_q(q, 3);
    x = x + (a_q(q, 4) - a_q(q, 2));
    x = x + (a_q(q, 5) - a_q(q, 1));
    x = x + (a_q(q, 6) - a_q(q, 0));
    s[q] = x;
    __builtin_amdgcn_sched_barrier(0);  // one quantity's window at a time (registers)
  }
  emit(6);
  for (int k = 0; k < nchunks; ++k) {
    if (k > 0 && k + 1 < nchunks) issue(k + 1);
#pragma unroll 1
    for (int g7 = k == 0 ? 7 : 0; g7 < SR_CW; g7 += 7) {
#pragma unroll
      for (int j7 = 0; j7 < 7; ++j7) {
        const int jj = g7 + j7, jn = k * SR_CW + jj;  // (jn mod 7 = j7: SR_CW and g7 are multiples of 7)
        if (jn < W) step(k & 1, jj, jn, j7);
      }
    }
    if (k + 1 < nchunks) commit(k + 1);
    __syncthreads();
  }
}

// The R, G, B maps' (or the leaf-folded luma map's) buffer sums: grid (nfull +
// 1, nchan, items), 64 lanes.  A full
// buffer's 64 leaves: a lane's leaf from lsum, or, if it crosses a row
// boundary, summed here from its raw elements (NumPy's leaf order); then the
// perfect binary tree by a shuffle butterfly.  The partial buffer: the host's
// pairwise tree (pw_tree) over its raw elements.
__global__ void __launch_bounds__(64) k_ss_rgbsum(RgbBatch B) {
  __shared__ double lsh[2 * PW_MAXN];
  const int b = blockIdx.x, ch = blockIdx.y, item = blockIdx.z, t = threadIdx.x;
  const size_t ic = (size_t)item * B.nchan + ch;
  double* out = B.chunks + ic * B.chunks_pitch + b;
  auto leaf = [](const double* v, int n) {  // pairwise_sum of n <= 128 elements
    if (n < 8) {
      double a = 0.0;
      for (int i = 0; i < n; ++i) a = a + v[i];
      return a;
    }
    double r8[8];
    for (int k = 0; k < 8; ++k) r8[k] = v[k];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r8[k] = r8[k] + v[i + k];
    double a = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
    for (; i < n; ++i) a = a + v[i];
    return a;
  };
  if (b < B.nfull) {
    const long long Lf = (long long)b * 64 + t, e0 = Lf * 128;
    double p;
    if (e0 / B.cw != (e0 + 127) / B.cw)
      p = leaf(B.raws + ic * B.raws_pitch + rs_slot(e0, B.cw) * 128, 128);
    else
      p = B.lsum[ic * B.lsum_pitch + Lf];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) p = p + __shfl_xor(p, o, 64);
    if (t == 0) *out = p;
  } else if (B.mpart > 0) {
    const PwTree& T = B.tree;
    const double* v = B.rawp + ic * B.rawp_pitch;
    for (int l = t; l < T.nl; l += 64) lsh[l] = leaf(v + T.off[l], T.n[l]);
    __syncthreads();
    for (int h = 0; h < T.nh; ++h) {
      for (int i = T.hs[h] + t; i < T.hs[h + 1]; i += 64) lsh[T.nl + i] = lsh[T.l[i]] + lsh[T.r[i]];
      __syncthreads();
    }
    if (t == 0) *out = lsh[T.ni ? T.nl + T.ni - 1 : 0];
  }
}

// buffer sums left to right from 0.0, / ns: grid (nchan, items)
__global__ void __launch_bounds__(64) k_ss_rgbfinal(RgbBatch B) {
  const int ch = blockIdx.x, item = blockIdx.y;
  if (threadIdx.x != 0) return;
  const int nb = B.nfull + (B.mpart > 0 ? 1 : 0);
  const double* cs = B.chunks + ((size_t)item * B.nchan + ch) * B.chunks_pitch;
  double acc = 0.0;
  for (int k = 0; k < nb; ++k) acc = acc + cs[k];
  B.out[(size_t)item * B.out_stride + B.ch_out + ch] = acc / (double)B.ns;
}

// ---------------------------------------------------------- NumPy means --

// LDS image of one buffer: element e at e + 8 * (e >> 7) (8-double pad per
// leaf: the per-leaf 16-B reads of a wave land on distinct banks)
__device__ __forceinline__ int sb_pad(int e) { return e + 8 * (e >> 7); }

// grid (nch, channels, items) from channel ch0: ch < 4 = the SSIM map of channel ch, ch = 4 the luma
// squared-difference stream (Y(a) - Y(b))^2 over H*W (utils/metrics.py:20 ->
// skimage mean_squared_error)
__global__ void __launch_bounds__(SB_THREADS) k_ss_chunks(SsimBatch B, const int ch0) {
  __shared__ double v[SB_NP_BUF + 8 * (SB_NP_BUF / 128)];
  __shared__ double wsum[4];
  __shared__ double lsum[2 * PW_MAXN];
  const int ch = ch0 + (int)blockIdx.y, item = blockIdx.z, t = threadIdx.x;
  const long long n = ch < 4 ? B.ns : (long long)B.H * B.W;
  const long long c0 = (long long)blockIdx.x * SB_NP_BUF;
  if (c0 >= n) return;
  const int m = (int)min((long long)SB_NP_BUF, n - c0);
  const int nch = max(B.nch_s, B.nch_y);
  double* out = B.chunks + ((size_t)item * 5 + ch) * nch + blockIdx.x;
  // stage the buffer (element e of the buffer at LDS sb_pad(e))
  if (ch < 4) {
    const double* src = B.smap + ((size_t)item * B.smap_ch + (B.smap_ch == 4 ? ch : 0)) * B.ns_pitch + c0;
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
    // (Y(image0) - Y(image1)) ** 2, the lumas formed from the bytes as
    // k_ss_yplanes / k_ss_ychk form them (6 B per element read instead of the
    // planes' 16)
    const SsimPair pr = B.pairs[item];
    auto lum = [](unsigned r, unsigned g, unsigned b) {
      return 0.299 * (double)r + 0.587 * (double)g + 0.114 * (double)b;  // utils/metrics.py:17-18
    };
    if (m == SB_NP_BUF) {
      typedef const uint32_t __attribute__((address_space(1)))* gdw;
      const uint8_t* pa = pr.a + 3 * c0;  // 4-B aligned: c0 is a multiple of 8192
      const uint8_t* pb = pr.b + 3 * c0;
#pragma unroll
      for (int k = 0; k < SB_NP_BUF / (4 * SB_THREADS); ++k) {
        const int e = 4 * t + 4 * SB_THREADS * k;  // four pixels = three dwords
        uint32_t wa[3], wb[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          wa[q] = *(gdw)(pa + 3 * e + 4 * q);
          wb[q] = *(gdw)(pb + 3 * e + 4 * q);
        }
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          unsigned ca[3], cb[3];
#pragma unroll
          for (int k3 = 0; k3 < 3; ++k3) {
            const int byte = 3 * px + k3;
            ca[k3] = (wa[byte >> 2] >> (8 * (byte & 3))) & 255u;
            cb[k3] = (wb[byte >> 2] >> (8 * (byte & 3))) & 255u;
          }
          const double d = lum(ca[0], ca[1], ca[2]) - lum(cb[0], cb[1], cb[2]);
          v[sb_pad(e + px)] = d * d;
        }
      }
    } else {
      for (int e = t; e < m; e += SB_THREADS) {
        const size_t o = 3 * (size_t)(c0 + e);
        const double d = lum(pr.a[o], pr.a[o + 1], pr.a[o + 2]) - lum(pr.b[o], pr.b[o + 1], pr.b[o + 2]);
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
    // the partial buffer: host-built tree (pw_tree), leaves in parallel, then
    // one height of internal nodes per barrier interval
    const PwTree& T = ch < 4 ? B.tree_s : B.tree_y;
    for (int l = t; l < T.nl; l += SB_THREADS) {
      const int off = T.off[l], ln = T.n[l];
      double acc;
      if (ln < 8) {
        acc = 0.0;
        for (int i = 0; i < ln; ++i) acc = acc + v[sb_pad(off + i)];
      } else {
        double r8[8];
        for (int k = 0; k < 8; ++k) r8[k] = v[sb_pad(off + k)];
        int i = 8;
        for (; i < ln - (ln % 8); i += 8)
          for (int k = 0; k < 8; ++k) r8[k] = r8[k] + v[sb_pad(off + i + k)];
        acc = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
        for (; i < ln; ++i) acc = acc + v[sb_pad(off + i)];
      }
      lsum[l] = acc;
    }
    __syncthreads();
    for (int h = 0; h < T.nh; ++h) {
      for (int i = T.hs[h] + t; i < T.hs[h + 1]; i += SB_THREADS) lsum[T.nl + i] = lsum[T.l[i]] + lsum[T.r[i]];
      __syncthreads();
    }
    if (t == 0) *out = lsum[T.ni ? T.nl + T.ni - 1 : 0];
  }
}

// buffer sums left to right from 0.0, then / n: one workgroup per (item,
// quantity); the sums are loaded 256 at a time into LDS (in parallel), one
// lane adds them in order
__global__ void __launch_bounds__(256) k_ss_final(SsimBatch B, const int ch0) {
  __shared__ double part[256];
  const int ch = ch0 + blockIdx.x, item = blockIdx.y;  // (ch0 = 3: the luma SSIM and MSE; k_ss_rgbfinal took R, G, B)
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

// band height (rows per workgroup): the RGB staging holds 16 rows per image
// (b4[2][4][...]: four rows per word), i.e. the band plus its 6-row window
// (BH = 16 measured 0.40 against 0.34 ms per pair, and does not fit it)
constexpr int SB_BH = 8;
constexpr int SB_YCHK_COL_ITEMS = 8;  // from this many items a lane per column (k_ss_ychk) fills the CUs
static_assert(SB_BH + 6 <= 16, "k_ss_band's RGB staging holds 16 rows per image");

int ssim_bands(int H) { return (H - 6 + SB_BH - 1) / SB_BH; }

// scratch doubles per item for H x W (H, W >= 7)
// NumPy pairwise_sum (numpy/core/src/umath/loops_utils.h.src): n <= 128 is a
// leaf (8 accumulators); above, n2 = n / 2 rounded down to a multiple of 8 and
// pw(n2) + pw(n - n2).  The tree of a partial buffer of m elements.
static void pw_tree(int m, PwTree* T) {
  memset(T, 0, sizeof *T);
  if (m <= 0) return;
  struct Node {
    int l, r, h;  // children as signed ids: >= 0 leaf index, < 0 -(internal index + 1)
  };
  Node nodes[PW_MAXN];
  int nl = 0, ni = 0;
  struct Rec {
    static int build(int off, int n, PwTree* T, Node* nodes, int& nl, int& ni, int& h) {
      if (n <= 128) {
        T->off[nl] = (uint16_t)off;
        T->n[nl] = (uint16_t)n;
        h = 0;
        return nl++;
      }
      int n2 = n / 2;
      n2 -= n2 % 8;
      int ha, hb;
      const int a = build(off, n2, T, nodes, nl, ni, ha);
      const int b = build(off + n2, n - n2, T, nodes, nl, ni, hb);
      nodes[ni] = {a, b, (ha > hb ? ha : hb) + 1};
      h = nodes[ni].h;
      return -(ni++) - 1;
    }
  };
  int h;
  Rec::build(0, m, T, nodes, nl, ni, h);
  // internal nodes by height (a child's height is below its parent's)
  int order[PW_MAXN], rank[PW_MAXN], k = 0, nh = 0;
  for (int hh = 1; hh <= 16; ++hh) {
    T->hs[hh - 1] = (uint8_t)k;
    for (int i = 0; i < ni; ++i)
      if (nodes[i].h == hh) order[k++] = i;
    if (k == ni) {
      nh = hh;
      T->hs[hh] = (uint8_t)k;
      break;
    }
  }
  for (int i = 0; i < ni; ++i) rank[order[i]] = i;
  auto id = [&](int c) { return c >= 0 ? c : nl + rank[-c - 1]; };
  for (int i = 0; i < ni; ++i) {
    T->l[i] = (uint8_t)id(nodes[order[i]].l);
    T->r[i] = (uint8_t)id(nodes[order[i]].r);
  }
  T->nl = (uint8_t)nl;
  T->ni = (uint8_t)ni;
  T->nh = (uint8_t)nh;
}

static long long ns_pitch_of(int H, int W) { return (((long long)(H - 6) * (W - 6)) + 63) & ~63LL; }
static long long n_pitch_of(int H, int W) { return ((long long)H * W + 63) & ~63LL; }
// the axis-0 checkpoints' doubles per item (5 quantities x bands x W), rounded up
// to 64 so the maps after them stay 16-B aligned (k_ss_chunks' double2 loads)
static long long ck_pitch_of(int H, int W) { return (5LL * ssim_bands(H) * W + 63) & ~63LL; }

int ssim_batch_max_items() { return SB_MAX_ITEMS; }

// k_ss_rows' raw slots per (item, channel), 128 doubles each
static long long rgb_raws_pitch(int H, int W) {
  const int cw = W - 6;
  const long long ns = (long long)(H - 6) * cw;
  return (cw >= 128 ? (long long)(H - 5) : (ns + 127) / 128 + 1) * 128;
}

// the leaf-folded luma map's doubles per item (k_ss_band<.., LF>): leaf sums
// [nfull * 64], row-crossing leaves (raw slots), the partial buffer [8192];
// offsets of the last two
struct LfLayout {
  long long raws, rawp, pitch;
};
static LfLayout lf_layout(int H, int W) {
  const long long nfull = (long long)(H - 6) * (W - 6) / SB_NP_BUF;
  LfLayout l;
  l.raws = nfull * 64;
  l.rawp = l.raws + rgb_raws_pitch(H, W);
  l.pitch = (l.rawp + SB_NP_BUF + 63) & ~63LL;
  return l;
}

// whether a launch of `items` pairs keeps fp64 luma planes (small launches:
// k_ss_yplanes for the per-quantity chains; larger ones form the luma from
// the bytes wherever they need it)
bool ssim_batch_planes(int items) { return items < SB_YCHK_COL_ITEMS; }

// scratch doubles per item for H x W (H, W >= 7); rgb: with the band
// kernel's R, G, B maps; planes: ssim_batch_planes(items) of the launch
size_t ssim_batch_scratch_doubles(int H, int W, bool rgb, bool planes) {
  const size_t n = (size_t)H * W;
  const size_t nch = (n + SB_NP_BUF - 1) / SB_NP_BUF;  // n > ns
  // (launches without the R, G, B bands and without planes fold the luma map
  // into leaf sums instead of storing it)
  const size_t maps = rgb ? 4 * (size_t)ns_pitch_of(H, W)
                          : (planes || !SB_LEAF_FOLD ? (size_t)ns_pitch_of(H, W) : (size_t)lf_layout(H, W).pitch);
  return (planes ? 2 * (size_t)n_pitch_of(H, W) : 0) + (size_t)ck_pitch_of(H, W) + maps + 5 * nch;
}


// scratch doubles per item of the R, G, B path (k_ss_rows, k_ss_rgbsum)
size_t ssim_rgb_scratch_doubles(int H, int W) {
  const long long ns = (long long)(H - 6) * (W - 6);
  const long long nfull = ns / SB_NP_BUF;
  return 3 * (size_t)(nfull * 64 + rgb_raws_pitch(H, W) + SB_NP_BUF + nfull + 1);
}

// SSIM R, G, B of `items` pairs (pairs_dev: items x {a, b} device image
// pointers, in device memory) into out[item * out_stride + 0..2]; scratch:
// items * ssim_rgb_scratch_doubles(H, W).  One launch of each kernel for the
// whole batch.
hipError_t launch_ssim_rgb(const void* pairs_dev, int items, int H, int W, double c1, double c2, double* scratch,
                           double* out, int out_stride, hipStream_t s) {
  if (items < 1 || H < 7 || W < 7) return hipErrorInvalidValue;
  if ((unsigned long long)H * (unsigned long long)W * 3ull >= (1ull << 31)) return hipErrorInvalidValue;  // 32-bit staging offsets
  RgbBatch R{};
  R.pairs = (const SsimPair*)pairs_dev;
  R.H = H;
  R.W = W;
  R.cw = W - 6;
  R.ns = (long long)(H - 6) * R.cw;
  R.nfull = (int)(R.ns / SB_NP_BUF);
  R.efull = (long long)R.nfull * SB_NP_BUF;
  R.mpart = (int)(R.ns - R.efull);
  R.c1 = c1;
  R.c2 = c2;
  R.cov_norm = 49.0 / 48.0;
  R.lsum_pitch = (long long)R.nfull * 64;
  R.raws_pitch = rgb_raws_pitch(H, W);
  R.rawp_pitch = SB_NP_BUF;
  R.chunks_pitch = R.nfull + 1;
  R.nchan = 3;
  R.ch_out = 0;
  R.lsum = scratch;
  R.raws = R.lsum + (size_t)items * 3 * R.lsum_pitch;
  R.rawp = R.raws + (size_t)items * 3 * R.raws_pitch;
  R.chunks = R.rawp + (size_t)items * 3 * SB_NP_BUF;
  R.out = out;
  R.out_stride = out_stride;
  pw_tree(R.mpart, &R.tree);
  hipLaunchKernelGGL(k_ss_rows, dim3((H - 6 + SR_ROWS - 1) / SR_ROWS, items), dim3(SR_THREADS), 0, s, R);
  hipLaunchKernelGGL(k_ss_rgbsum, dim3(R.nfull + 1, 3, items), dim3(64), 0, s, R);
  hipLaunchKernelGGL(k_ss_rgbfinal, dim3(3, items), dim3(64), 0, s, R);
  return hipGetLastError();
}

// SSIM Y and the luma MSE of `items` (<= SB_MAX_ITEMS) pairs (pairs_dev:
// items x {a, b} device image pointers, in device memory) into out[item *
// out_stride + 3..4], and the RGB squared-error sums into sse[item] (nullable;
// the caller zeroes it); scratch: items * ssim_batch_scratch_doubles(H, W, rgb,
// ssim_batch_planes(items)).
// rgb: also SSIM R, G, B (out[.. 0..2]) by the band kernel on `side` (small
// batches; large ones take launch_ssim_rgb).
hipError_t launch_psnr_ssim_batch(const void* pairs_dev, int items, int H, int W, double c1, double c2,
                                  double* scratch, double* out, int out_stride, unsigned long long* sse,
                                  hipStream_t s, bool rgb, hipStream_t side, hipEvent_t fork, hipEvent_t join) {
  if (items < 1 || items > SB_MAX_ITEMS || H < 7 || W < 7) return hipErrorInvalidValue;
  if ((unsigned long long)H * (unsigned long long)W * 3ull >= (1ull << 32)) return hipErrorInvalidValue;  // 32-bit staging offsets
  SsimBatch B{};
  B.pairs = (const SsimPair*)pairs_dev;
  B.smap_ch = rgb ? 4 : 1;
  B.H = H;
  B.W = W;
  B.NB = ssim_bands(H);
  B.ns = (long long)(H - 6) * (W - 6);
  B.ns_pitch = ns_pitch_of(H, W);
  B.n_pitch = n_pitch_of(H, W);
  pw_tree((int)(B.ns % SB_NP_BUF), &B.tree_s);
  pw_tree((int)(((long long)H * W) % SB_NP_BUF), &B.tree_y);
  const long long n = (long long)H * W;
  B.nch_s = (int)((B.ns + SB_NP_BUF - 1) / SB_NP_BUF);
  B.nch_y = (int)((n + SB_NP_BUF - 1) / SB_NP_BUF);
  const int nch = std::max(B.nch_s, B.nch_y);
  B.c1 = c1;
  B.c2 = c2;
  B.cov_norm = 49.0 / 48.0;
  const bool planes = ssim_batch_planes(items);
  B.yplanes = planes ? scratch : nullptr;
  B.ck = scratch + (planes ? (size_t)items * 2 * B.n_pitch : 0);
  B.ck_pitch = ck_pitch_of(H, W);
  const bool lf = SB_LEAF_FOLD && !planes && !rgb;  // the luma map folded into leaf sums (k_ss_band<.., LF>)
  const LfLayout lo = lf_layout(H, W);
  B.smap = lf ? nullptr : B.ck + (size_t)items * B.ck_pitch;
  B.lf = lf ? B.ck + (size_t)items * B.ck_pitch : nullptr;
  B.lf_pitch = lo.pitch;
  B.lf_raws = lo.raws;
  B.lf_rawp = lo.rawp;
  B.efull = (B.ns / SB_NP_BUF) * SB_NP_BUF;
  B.chunks = lf ? B.lf + (size_t)items * lo.pitch : B.smap + (size_t)items * B.smap_ch * B.ns_pitch;
  B.out = out;
  B.out_stride = out_stride;
  B.sse = sse;
  hipError_t e;
  if (rgb) {
    // the RGB channels' bands need only the images: on the side stream from
    // the start, beside the luma planes, chains and band on s; joined before
    // the means
    if ((e = hipEventRecord(fork, s)) != hipSuccess || (e = hipStreamWaitEvent(side, fork, 0)) != hipSuccess)
      return e;
    hipLaunchKernelGGL((k_ss_band<SB_BH, false, false, true>), dim3(B.NB, 3, items), dim3(SB_THREADS), 0, side, B);
    hipLaunchKernelGGL(k_ss_chunks, dim3(B.nch_s, 3, items), dim3(SB_THREADS), 0, side, B, 0);
    if ((e = hipEventRecord(join, side)) != hipSuccess) return e;
  }
  if (!planes) {  // SSE and chains in one pass over the bytes
    hipLaunchKernelGGL(k_ss_ychk<SB_BH>, dim3((W + 63) / 64, items), dim3(64), 0, s, B);
  } else {
    hipLaunchKernelGGL(k_ss_yplanes, dim3((unsigned)std::min<long long>((n + 255) / 256, SB_PLANE_BLOCKS), items),
                       dim3(256), 0, s, B);
    hipLaunchKernelGGL(k_ss_ychkq<SB_BH>, dim3((W + 63) / 64, 5, items), dim3(64), 0, s, B);
  }
  if (lf) {
    hipLaunchKernelGGL((k_ss_band<SB_BH, true, false, false, true>), dim3(B.NB, 1, items), dim3(SB_THREADS), 0, s, B);
    hipLaunchKernelGGL(k_ss_chunks, dim3(B.nch_y, 1, items), dim3(SB_THREADS), 0, s, B, 4);  // luma MSE
    // the luma map's buffer sums from its leaf sums and raw elements
    RgbBatch R{};
    R.pairs = B.pairs;
    R.H = H;
    R.W = W;
    R.cw = W - 6;
    R.ns = B.ns;
    R.nfull = (int)(B.ns / SB_NP_BUF);
    R.efull = B.efull;
    R.mpart = (int)(B.ns - B.efull);
    R.lsum = B.lf;
    R.raws = B.lf + lo.raws;
    R.rawp = B.lf + lo.rawp;
    R.chunks = B.chunks;  // (the luma map's slots, [item][5][nch] at channel 3)
    R.lsum_pitch = R.raws_pitch = R.rawp_pitch = lo.pitch;
    R.chunks_pitch = 5LL * nch;
    R.nchan = 1;
    R.ch_out = 3;
    R.out = out;
    R.out_stride = out_stride;
    pw_tree(R.mpart, &R.tree);
    R.chunks += 3 * nch;  // channel 3's row of the item's [5][nch] block
    hipLaunchKernelGGL(k_ss_rgbsum, dim3(R.nfull + 1, 1, items), dim3(64), 0, s, R);
    hipLaunchKernelGGL(k_ss_rgbfinal, dim3(1, items), dim3(64), 0, s, R);
    hipLaunchKernelGGL(k_ss_final, dim3(1, items), dim3(256), 0, s, B, 4);  // the luma MSE
    return hipGetLastError();
  }
  if (!planes && !rgb)
    hipLaunchKernelGGL((k_ss_band<SB_BH, true>), dim3(B.NB, 1, items), dim3(SB_THREADS), 0, s, B);
  else if (!planes)
    hipLaunchKernelGGL((k_ss_band<SB_BH, true, false, true>), dim3(B.NB, 1, items), dim3(SB_THREADS), 0, s, B);
  else
    hipLaunchKernelGGL((k_ss_band<SB_BH, true, true, true>), dim3(B.NB, 1, items), dim3(SB_THREADS), 0, s, B);
  hipLaunchKernelGGL(k_ss_chunks, dim3(nch, 2, items), dim3(SB_THREADS), 0, s, B, 3);  // luma map, luma MSE
  if (rgb && (e = hipStreamWaitEvent(s, join, 0)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_ss_final, dim3(rgb ? 5 : 2, items), dim3(256), 0, s, B, rgb ? 0 : 3);
  return hipGetLastError();
}

}  // namespace jds
