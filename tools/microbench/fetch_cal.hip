// fetch_cal.hip — FETCH_SIZE calibration for the codec's own load patterns
// (MI355X_MICROARCH.md, HBM/rocprofv3: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel
// reads a buffer of known size once with one of the headline kernels' load
// shapes and writes one word per workgroup; rocprofv3 --pmc FETCH_SIZE (and, in
// its own pass, WRITE_SIZE) over this program gives counted / true bytes per
// pattern:
//   k_rgb24  : k_fwd32i's RGB row segments -- a lane reads 24 contiguous bytes
//              as three 8-B loads (uint2), lanes 24 B apart (64 x 1080p RGB,
//              398,131,200 bytes)
//   k_col16  : k_inv_fast's coefficient columns -- the 8 lanes of a block read
//              column v of its 8 x 8 int16 block, 8 two-byte loads 16 B apart
//              (64 x 1080p 4:2:0 coefficients, 399,114,240 bytes)
//   k_x4     : 16-B per lane streaming (the guide's calibrated x2 case)
// usage: fetch_cal   (one launch of each, after one warm launch)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e = (x);                                                                          \
    if (e != hipSuccess) {                                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                    \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

__global__ void __launch_bounds__(256) k_rgb24(const uint8_t* __restrict__ p, long long nseg, uint32_t* out) {
  const long long s = (long long)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  if (s < nseg) {
    const uint2* p2 = reinterpret_cast<const uint2*>(p + s * 24);
    const uint2 a = p2[0], b = p2[1], c = p2[2];
    acc = a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y;
  }
  for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(512) k_col16(const int16_t* __restrict__ c, long long nblk, uint32_t* out) {
  const long long b = (long long)blockIdx.x * 64 + (threadIdx.x >> 3);
  const int v = threadIdx.x & 7;
  int acc = 0;
  if (b < nblk) {
    const int16_t* blk = c + b * 64;
#pragma unroll
    for (int r = 0; r < 8; ++r) acc += blk[r * 8 + v];
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = (uint32_t)acc;
}

__global__ void __launch_bounds__(256) k_x4(const uint4* __restrict__ p, long long n4, uint32_t* out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  if (i < n4) {
    const uint4 a = p[i];
    acc = a.x ^ a.y ^ a.z ^ a.w;
  }
  for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

int main() {
  const long long rgb_bytes = 64LL * 1920 * 1080 * 3;      // 398,131,200
  const long long coef_bytes = 64LL * 3118080 * 2;          // 399,114,240 (1080p 4:2:0)
  uint8_t* rgb;
  int16_t* cf;
  uint32_t* out;
  CK(hipMalloc(&rgb, rgb_bytes));
  CK(hipMalloc(&cf, coef_bytes));
  CK(hipMalloc(&out, 64 << 20));
  CK(hipMemset(rgb, 7, rgb_bytes));
  CK(hipMemset(cf, 3, coef_bytes));
  const long long nseg = rgb_bytes / 24, nblk = coef_bytes / 128, n4 = rgb_bytes / 16;
  for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms; rocprofv3 reports both (read the second)
    hipLaunchKernelGGL(k_rgb24, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, 0, rgb, nseg, out);
    hipLaunchKernelGGL(k_col16, dim3((unsigned)((nblk + 63) / 64)), dim3(512), 0, 0, cf, nblk, out);
    hipLaunchKernelGGL(k_x4, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const uint4*)rgb, n4, out);
    CK(hipDeviceSynchronize());
  }
  printf("{\"rgb24_bytes\": %lld, \"col16_bytes\": %lld, \"x4_bytes\": %lld}\n", rgb_bytes, coef_bytes, rgb_bytes);
  CK(hipFree(rgb));
  CK(hipFree(cf));
  CK(hipFree(out));
  return 0;
}
