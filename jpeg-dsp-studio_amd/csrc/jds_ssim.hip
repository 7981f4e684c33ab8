// jds_ssim.hip — K4: PSNR / SSIM of two uint8 RGB images on the GPU,
// reproducing utils/metrics.py:9-28 (skimage.metrics + scipy.ndimage + NumPy)
// bit for bit:
//   * scipy.ndimage.uniform_filter(size=7, mode='reflect') = uniform_filter1d
//     along axis 0 then axis 1; each line is a running sum of the raw values
//     (s += new - old) divided by 7 at every output (scipy NI_UniformFilter1D);
//   * skimage structural_similarity: sample covariance (49/48), K1=.01, K2=.03,
//     data_range=255, mean over the 3-px-cropped map;
//   * numpy mean over n elements: the C-order element stream is cut into
//     8192-element buffers, each buffer is summed by NumPy's pairwise_sum
//     (8 accumulators on leaves of <= 128), buffer sums accumulate left to
//     right from 0.0, then / n.
// The luma PSNR uses the same NumPy mean on (Y(orig) - Y(rec))^2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

constexpr int NP_BUF = 8192;   // NumPy ufunc buffer size (elements)
constexpr int PW_BLOCK = 128;  // NumPy PW_BLOCKSIZE

struct SsimConsts {
  double c1, c2, cov_norm;
};

__device__ __forceinline__ int refl_sym(int i, int n) {  // scipy 'reflect' (edge repeated)
  const int p = 2 * n;
  i %= p;
  if (i < 0) i += p;
  return i >= n ? p - 1 - i : i;
}

__device__ __forceinline__ double chan_val(const uint8_t* img, size_t px, int c) {
  if (c < 3) return (double)img[px * 3 + c];
  const double R = img[px * 3], G = img[px * 3 + 1], B = img[px * 3 + 2];
  return 0.299 * R + 0.587 * G + 0.114 * B;  // utils/metrics.py:17-18
}

// pass along axis 0 (columns): 5 running sums per column, one channel.
// out: 5 planes [q][H][W], q = x, y, xx, yy, xy
__global__ void k_uf_axis0(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int H, int W, int c,
                           double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= W) return;
  const size_t plane = (size_t)H * W;
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int k = -3; k <= 3; ++k) {
    const size_t px = (size_t)refl_sym(k, H) * W + j;
    const double x = chan_val(a, px, c), y = chan_val(b, px, c);
    s[0] = s[0] + x;
    s[1] = s[1] + y;
    s[2] = s[2] + x * x;
    s[3] = s[3] + y * y;
    s[4] = s[4] + x * y;
  }
  for (int q = 0; q < 5; ++q) out[q * plane + j] = s[q] / 7.0;
  for (int i = 1; i < H; ++i) {
    const size_t pn = (size_t)refl_sym(i + 3, H) * W + j, po = (size_t)refl_sym(i - 4, H) * W + j;
    const double xn = chan_val(a, pn, c), yn = chan_val(b, pn, c);
    const double xo = chan_val(a, po, c), yo = chan_val(b, po, c);
    s[0] = s[0] + (xn - xo);
    s[1] = s[1] + (yn - yo);
    s[2] = s[2] + (xn * xn - xo * xo);
    s[3] = s[3] + (yn * yn - yo * yo);
    s[4] = s[4] + (xn * yn - xo * yo);
    const size_t o = (size_t)i * W + j;
    for (int q = 0; q < 5; ++q) out[q * plane + o] = s[q] / 7.0;
  }
}

// pass along axis 1 (rows) over the 5 planes, then the SSIM map on the cropped region
__global__ void k_uf_axis1_ssim(const double* __restrict__ in, int H, int W, SsimConsts k,
                                double* __restrict__ smap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  const size_t plane = (size_t)H * W;
  const double* r[5];
  for (int q = 0; q < 5; ++q) r[q] = in + q * plane + (size_t)i * W;
  double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int t = -3; t <= 3; ++t) {
    const int jj = refl_sym(t, W);
    for (int q = 0; q < 5; ++q) s[q] = s[q] + r[q][jj];
  }
  const bool row_in = i >= 3 && i < H - 3;
  const int cw = W - 6;
  for (int j = 0; j < W; ++j) {
    if (j > 0) {
      const int jn = refl_sym(j + 3, W), jo = refl_sym(j - 4, W);
      for (int q = 0; q < 5; ++q) s[q] = s[q] + (r[q][jn] - r[q][jo]);
    }
    if (row_in && j >= 3 && j < W - 3) {
      const double ux = s[0] / 7.0, uy = s[1] / 7.0, uxx = s[2] / 7.0, uyy = s[3] / 7.0, uxy = s[4] / 7.0;
      // skimage structural_similarity (sample covariance)
      const double vx = k.cov_norm * (uxx - ux * ux);
      const double vy = k.cov_norm * (uyy - uy * uy);
      const double vxy = k.cov_norm * (uxy - ux * uy);
      const double a1 = 2 * ux * uy + k.c1, a2 = 2 * vxy + k.c2;
      const double b1 = ux * ux + uy * uy + k.c1, b2 = vx + vy + k.c2;
      const double d = b1 * b2;
      smap[(size_t)(i - 3) * cw + (j - 3)] = (a1 * a2) / d;
    }
  }
}

// ---- NumPy pairwise_sum over a <= 8192-element buffer, one workgroup ----

struct LeafRange {
  int off, n;
};

// in-order leaves of NumPy's pairwise recursion (leaf: n <= PW_BLOCK)
__device__ int pw_leaves(int n, LeafRange* out) {
  int so[24], sn[24], sp = 0, cnt = 0;
  so[0] = 0; sn[0] = n; sp = 1;
  while (sp > 0) {
    --sp;
    const int off = so[sp], m = sn[sp];
    if (m <= PW_BLOCK) {
      out[cnt++] = {off, m};
    } else {
      int m2 = m / 2;
      m2 -= m2 % 8;
      so[sp] = off + m2; sn[sp] = m - m2; ++sp;  // right, popped second
      so[sp] = off;      sn[sp] = m2;     ++sp;  // left, popped first
    }
  }
  return cnt;
}

template <typename Get>
__device__ double pw_leaf_sum(Get get, int off, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r = r + get(off + i);
    return r;
  }
  double r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = get(off + k);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = r[k] + get(off + i + k);
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res = res + get(off + i);
  return res;
}

// combine leaf sums following the same recursion (post-order)
__device__ double pw_combine(int n, const double* ls) {
  int fn[24], fph[24];
  double fl[24];
  int sp = 0, li = 0;
  double res = 0.0;
  bool ret = false;
  fn[0] = n; fph[0] = 0; sp = 1;
  while (sp > 0) {
    const int t = sp - 1;
    if (ret) {
      ret = false;
      if (fph[t] == 1) {
        fl[t] = res;
        fph[t] = 2;
        int m2 = fn[t] / 2;
        m2 -= m2 % 8;
        fn[sp] = fn[t] - m2; fph[sp] = 0; ++sp;
      } else {
        res = fl[t] + res;
        --sp;
        ret = true;
      }
      continue;
    }
    if (fn[t] <= PW_BLOCK) {
      res = ls[li++];
      --sp;
      ret = true;
      continue;
    }
    int m2 = fn[t] / 2;
    m2 -= m2 % 8;
    fph[t] = 1;
    fn[sp] = m2; fph[sp] = 0; ++sp;
  }
  return res;
}

template <typename Get>
__device__ void np_chunk_sum(Get get, long long n, double* chunk_out) {
  __shared__ LeafRange s_leaf[NP_BUF / 64 + 2];
  __shared__ double s_ls[NP_BUF / 64 + 2];
  __shared__ int s_cnt;
  const long long c0 = (long long)blockIdx.x * NP_BUF;
  const int m = (int)((n - c0) < NP_BUF ? (n - c0) : NP_BUF);
  if (threadIdx.x == 0) s_cnt = pw_leaves(m, s_leaf);
  __syncthreads();
  for (int l = threadIdx.x; l < s_cnt; l += blockDim.x) {
    const LeafRange lr = s_leaf[l];
    s_ls[l] = pw_leaf_sum([&](int i) { return get(c0 + i); }, lr.off, lr.n);
  }
  __syncthreads();
  if (threadIdx.x == 0) chunk_out[blockIdx.x] = pw_combine(m, s_ls);
}

__global__ void k_chunks_smap(const double* __restrict__ smap, long long n, double* __restrict__ chunk_out) {
  np_chunk_sum([&](long long i) { return smap[i]; }, n, chunk_out);
}

__global__ void k_chunks_ydiff(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, long long n,
                               double* __restrict__ chunk_out) {
  np_chunk_sum(
      [&](long long i) {
        const double d = chan_val(a, (size_t)i, 3) - chan_val(b, (size_t)i, 3);
        return d * d;  // (image0 - image1) ** 2
      },
      n, chunk_out);
}

__global__ void k_chunks_final(const double* __restrict__ chunks, int nchunks, long long n, double* out) {
  if (threadIdx.x != 0) return;
  double acc = 0.0;
  for (int k = 0; k < nchunks; ++k) acc = acc + chunks[k];
  *out = acc / (double)n;
}

__global__ void k_sse_u8(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, long long n,
                         unsigned long long* out) {
  unsigned long long acc = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int d = (int)a[i] - (int)b[i];
    acc += (unsigned long long)(d * d);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

hipError_t launch_sse_u8(const uint8_t* a, const uint8_t* b, long long n, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(k_sse_u8, dim3(1024), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

// utils/metrics.py:77-78 — magnitude_bits = np.sum(np.ceil(np.log2(|nz| + 1)) + 1)
// over the nonzero coefficients in all_quantized_coeffs order, a float32
// reduction: NumPy sums 8192-element buffers (exact here: terms are integers
// <= 12, so a buffer sum < 2^24) and accumulates the buffer sums in float32.
// One workgroup walks the blocks in order, ranking nonzeros with a block scan.
__global__ void __launch_bounds__(1024)
k_mag_f32(const int16_t* __restrict__ coeffs, long long nblocks, unsigned* __restrict__ chunk_sum,
          int max_chunks, double* __restrict__ out) {
  __shared__ unsigned s_scan[1024];
  __shared__ unsigned long long s_base;
  const int t = threadIdx.x;
  if (t == 0) s_base = 0;
  __syncthreads();
  for (long long b0 = 0; b0 < nblocks; b0 += 1024) {
    const long long b = b0 + t;
    unsigned cnt = 0;
    if (b < nblocks)
      for (int i = 0; i < 64; ++i) cnt += coeffs[b * 64 + i] != 0;
    s_scan[t] = cnt;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
      const unsigned v = t >= o ? s_scan[t - o] : 0u;
      __syncthreads();
      s_scan[t] += v;
      __syncthreads();
    }
    unsigned long long rank = s_base + s_scan[t] - cnt;
    if (b < nblocks) {
      for (int i = 0; i < 64; ++i) {
        const int q = coeffs[b * 64 + i];
        if (q) {
          const int m = q < 0 ? -q : q;
          const long long ch = (long long)(rank >> 13);
          if (ch < max_chunks) atomicAdd(&chunk_sum[ch], (unsigned)(33 - __clz(m)));
          ++rank;
        }
      }
    }
    __syncthreads();
    if (t == 1023) s_base += s_scan[1023];
    __syncthreads();
  }
  if (t == 0) {
    const long long nch = (long long)((s_base + 8191) >> 13);
    float acc = 0.0f;
    for (long long k = 0; k < nch && k < max_chunks; ++k) acc = acc + (float)chunk_sum[k];
    *out = (double)acc;
  }
}

hipError_t launch_mag_f32(const int16_t* coeffs, long long nblocks, unsigned* chunk_sum, int max_chunks,
                          double* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(chunk_sum, 0, sizeof(unsigned) * (size_t)max_chunks, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_mag_f32, dim3(1), dim3(1024), 0, s, coeffs, nblocks, chunk_sum, max_chunks, out);
  return hipGetLastError();
}

// ssim_out[0..3] = SSIM of R, G, B, Y; ssim_out[4] = MSE of Y (for PSNR-Y)
hipError_t launch_psnr_ssim(const uint8_t* a, const uint8_t* b, int H, int W, double c1, double c2,
                            double* scratch_planes /*5*H*W*/, double* scratch_smap /*(H-6)*(W-6)*/,
                            double* scratch_chunks /*>= ceil(H*W/8192)*/, double* out /*5 doubles*/,
                            hipStream_t s) {
  SsimConsts k{c1, c2, 49.0 / 48.0};
  const long long ns = (long long)(H - 6) * (W - 6);
  const int nch_s = (int)((ns + NP_BUF - 1) / NP_BUF);
  for (int c = 0; c < 4; ++c) {
    hipLaunchKernelGGL(k_uf_axis0, dim3((W + 63) / 64), dim3(64), 0, s, a, b, H, W, c, scratch_planes);
    hipLaunchKernelGGL(k_uf_axis1_ssim, dim3((H + 63) / 64), dim3(64), 0, s, scratch_planes, H, W, k,
                       scratch_smap);
    hipLaunchKernelGGL(k_chunks_smap, dim3(nch_s), dim3(128), 0, s, scratch_smap, ns, scratch_chunks);
    hipLaunchKernelGGL(k_chunks_final, dim3(1), dim3(64), 0, s, scratch_chunks, nch_s, ns, out + c);
  }
  const long long np_ = (long long)H * W;
  const int nch_y = (int)((np_ + NP_BUF - 1) / NP_BUF);
  hipLaunchKernelGGL(k_chunks_ydiff, dim3(nch_y), dim3(128), 0, s, a, b, np_, scratch_chunks);
  hipLaunchKernelGGL(k_chunks_final, dim3(1), dim3(64), 0, s, scratch_chunks, nch_y, np_, out + 4);
  return hipGetLastError();
}

}  // namespace jds
