// jds_ssim.hip — the statistics kernels beside the SSIM pipeline
// (jds_ssim_band.hip): the integer RGB squared-error sum behind PSNR-RGB
// (utils/metrics.py:11) and the float32 magnitude-bits reduction
// (utils/metrics.py:77-78).  (Rounds 1-4 also held the first SSIM kernels here,
// one scipy line per lane; the batched pipeline replaced them and the tests
// compare it with the oracle directly.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_internal.hpp"

#pragma clang fp contract(off)

namespace jds {

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
// <= 17, so a buffer sum < 2^24) and accumulates the buffer sums in float32.
// Three parallel passes: per-block nonzero counts with a workgroup scan, the
// scan of the workgroup totals, then each block adds its terms to the (at most
// two) buffers its nonzeros fall in; one lane accumulates the buffer sums.
constexpr int MAG_WG = 256;

__device__ __forceinline__ unsigned block_nz(const int16_t* blk) {
  const uint4* v = reinterpret_cast<const uint4*>(blk);
  unsigned n = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 w = v[i];
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) n += ((x[k] & 0xffffu) != 0u) + ((x[k] >> 16) != 0u);
  }
  return n;
}

__global__ void __launch_bounds__(MAG_WG) k_mag_count(const int16_t* __restrict__ coeffs, long long nblocks,
                                                      unsigned* __restrict__ local_rank, unsigned* __restrict__ wg_tot) {
  __shared__ unsigned s[MAG_WG];
  const long long b = (long long)blockIdx.x * MAG_WG + threadIdx.x;
  const unsigned n = b < nblocks ? block_nz(coeffs + b * 64) : 0u;
  s[threadIdx.x] = n;
  __syncthreads();
  for (int o = 1; o < MAG_WG; o <<= 1) {  // inclusive Hillis-Steele scan
    const unsigned v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
    __syncthreads();
    s[threadIdx.x] += v;
    __syncthreads();
  }
  if (b < nblocks) local_rank[b] = s[threadIdx.x] - n;
  if (threadIdx.x == MAG_WG - 1) wg_tot[blockIdx.x] = s[MAG_WG - 1];
}

// exclusive scan of the workgroup totals in place (one workgroup, 1024-wide steps)
__global__ void __launch_bounds__(1024) k_mag_scan(unsigned* __restrict__ wg_tot, int nwg) {
  __shared__ unsigned s[1024];
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nwg; b0 += 1024) {
    const int i = b0 + threadIdx.x;
    const unsigned n = i < nwg ? wg_tot[i] : 0u;
    s[threadIdx.x] = n;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const unsigned v = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0u;
      __syncthreads();
      s[threadIdx.x] += v;
      __syncthreads();
    }
    if (i < nwg) wg_tot[i] = (unsigned)(s_base + s[threadIdx.x] - n);
    __syncthreads();
    if (threadIdx.x == 1023) s_base += s[1023];
    __syncthreads();
  }
}

__global__ void __launch_bounds__(MAG_WG) k_mag_chunks(const int16_t* __restrict__ coeffs, long long nblocks,
                                                       const unsigned* __restrict__ local_rank,
                                                       const unsigned* __restrict__ wg_off,
                                                       unsigned* __restrict__ chunk_sum, int max_chunks) {
  const long long b = (long long)blockIdx.x * MAG_WG + threadIdx.x;
  if (b >= nblocks) return;
  unsigned long long rank = (unsigned long long)wg_off[blockIdx.x] + local_rank[b];
  const long long c0 = (long long)(rank >> 13);
  unsigned acc[2] = {0u, 0u};
  const uint4* v = reinterpret_cast<const uint4*>(coeffs + b * 64);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 w = v[i];
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = (int)(int16_t)(x[k >> 1] >> (16 * (k & 1)));
      if (q) {
        const int m = q < 0 ? -q : q;
        acc[(long long)(rank >> 13) - c0] += (unsigned)(33 - __clz(m));  // bit length + 1
        ++rank;
      }
    }
  }
  if (acc[0] && c0 < max_chunks) atomicAdd(&chunk_sum[c0], acc[0]);
  if (acc[1] && c0 + 1 < max_chunks) atomicAdd(&chunk_sum[c0 + 1], acc[1]);
}

__global__ void k_mag_final(const unsigned* __restrict__ chunk_sum, const unsigned* __restrict__ wg_off, int nwg,
                            const unsigned* __restrict__ wg_last, int max_chunks, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long total = (unsigned long long)wg_off[nwg - 1] + *wg_last;  // nonzeros
  const long long nch = (long long)((total + 8191) >> 13);
  float acc = 0.0f;
  for (long long k = 0; k < nch && k < max_chunks; ++k) acc = acc + (float)chunk_sum[k];
  *out = (double)acc;
}

// scratch: chunk_sum[max_chunks] | local_rank[nblocks] | wg_tot[nwg] | last wg total
size_t mag_scratch_bytes(long long nblocks, int max_chunks) {
  const long long nwg = (nblocks + MAG_WG - 1) / MAG_WG;
  return sizeof(unsigned) * ((size_t)max_chunks + (size_t)nblocks + (size_t)nwg + 1);
}

hipError_t launch_mag_f32(const int16_t* coeffs, long long nblocks, unsigned* scratch, int max_chunks, double* out,
                          hipStream_t s) {
  const int nwg = (int)((nblocks + MAG_WG - 1) / MAG_WG);
  unsigned* chunk_sum = scratch;
  unsigned* local_rank = chunk_sum + max_chunks;
  unsigned* wg_tot = local_rank + nblocks;
  unsigned* wg_last = wg_tot + nwg;
  hipError_t e = hipMemsetAsync(chunk_sum, 0, sizeof(unsigned) * (size_t)max_chunks, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_mag_count, dim3(nwg), dim3(MAG_WG), 0, s, coeffs, nblocks, local_rank, wg_tot);
  if ((e = hipMemcpyAsync(wg_last, wg_tot + nwg - 1, sizeof(unsigned), hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(k_mag_scan, dim3(1), dim3(1024), 0, s, wg_tot, nwg);
  hipLaunchKernelGGL(k_mag_chunks, dim3(nwg), dim3(MAG_WG), 0, s, coeffs, nblocks, local_rank, wg_tot, chunk_sum,
                     max_chunks);
  hipLaunchKernelGGL(k_mag_final, dim3(1), dim3(64), 0, s, chunk_sum, wg_tot, nwg, wg_last, max_chunks, out);
  return hipGetLastError();
}

}  // namespace jds
