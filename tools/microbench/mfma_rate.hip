// Matrix-pipe vs VALU issue rates on gfx950, measured with the in-kernel clock
// (s_memtime) so DVFS does not distort the cycle counts: fp64 / fp32 VALU FMA,
// packed fp32 VALU FMA (v_pk_fma_f32), v_mfma_f64_16x16x4_f64,
// v_mfma_f64_4x4x4_4b_f64, v_mfma_f32_16x16x4_f32, and MFMA streams (fp64, and
// fp32 since round 5) interleaved with independent VALU FMAs of the same type
// (do the two pipes overlap?).  Prints cycles per wave-instruction per SIMD and FMAs per
// clock per SIMD.  Evidence for DESIGN.md's MFMA A/B (the 8-point transforms of
// the codec on the matrix pipe); tool, not product.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 2048;

struct Out {
  unsigned long long cyc;
  double sink;
};

__device__ __forceinline__ unsigned long long clk() { return __builtin_amdgcn_s_memtime(); }

__global__ void k_vf64(Out* o, double a, double b) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, b);
  const unsigned long long t1 = clk();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}
__global__ void k_vf32(Out* o, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  const unsigned long long t1 = clk();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}
__global__ void k_vpk32(Out* o, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
  const f2 a2 = {a, a}, b2 = {b, b};
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], a2, b2);
  const unsigned long long t1 = clk();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i][0] + x[i][1];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}
__global__ void k_m64(Out* o, double a, double b) {
  d4 c[4] = {};
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a + i, b, c[i], 0, 0, 0);
  const unsigned long long t1 = clk();
  double s = 0;
  for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][3];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}
__global__ void k_m64s(Out* o, double a, double b) {
  double c[4] = {};
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a + i, b, c[i], 0, 0, 0);
  const unsigned long long t1 = clk();
  double s = 0;
  for (int i = 0; i < 4; ++i) s += c[i];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}
__global__ void k_m32(Out* o, float a, float b) {
  f4 c[4] = {};
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a + i, b, c[i], 0, 0, 0);
  const unsigned long long t1 = clk();
  float s = 0;
  for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][3];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, (double)s};
}
// one 16x16x4 f64 MFMA beside NV independent fp64 VALU FMAs per iteration
template <int NV>
__global__ void k_mix(Out* o, double a, double b) {
  d4 c[2] = {};
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a + i, b, c[i], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV / 2; ++j) x[j % 8] = __builtin_fma(x[j % 8], a, b);
    }
  }
  const unsigned long long t1 = clk();
  double s = c[0][0] + c[1][1];
  for (int i = 0; i < 8; ++i) s += x[i];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, s};
}

// one 16x16x4 f32 MFMA beside NV independent fp32 VALU FMAs per iteration
// (PK: packed v_pk_fma_f32, two FMAs per lane and instruction)
template <int NV, bool PK>
__global__ void k_mix32(Out* o, float a, float b) {
  f4 c[2] = {};
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
  const f2 a2 = {a, a}, b2 = {b, b};
  const unsigned long long t0 = clk();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      c[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a + i, b, c[i], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV / 2; ++j) {
        if constexpr (PK)
          x[j % 8] = __builtin_elementwise_fma(x[j % 8], a2, b2);
        else
          x[j % 8][0] = __builtin_fmaf(x[j % 8][0], a, b);
      }
    }
  }
  const unsigned long long t1 = clk();
  float s = c[0][0] + c[1][1];
  for (int i = 0; i < 8; ++i) s += x[i][0] + x[i][1];
  if (threadIdx.x % 64 == 0) o[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = {t1 - t0, (double)s};
}

template <typename K, typename... A>
static double run(const char* name, K kern, int waves_per_simd, double instr_per_iter, double fma_per_instr,
                  A... args) {
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int threads = 256, blocks = p.multiProcessorCount * waves_per_simd;  // 4 waves per block: one per SIMD
  Out* o;
  hipMalloc(&o, sizeof(Out) * blocks * 4);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(kern, blocks, threads, 0, 0, o, args...);
  hipDeviceSynchronize();
  Out* h = (Out*)malloc(sizeof(Out) * blocks * 4);
  hipMemcpy(h, o, sizeof(Out) * blocks * 4, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < blocks * 4; ++i) mean += (double)h[i].cyc;
  mean /= blocks * 4;
  // every wave of the SIMD runs concurrently: per-SIMD cycles per instruction =
  // wave cycles / (instructions per wave x waves per SIMD)
  const double cpi = mean / (ITER * instr_per_iter * waves_per_simd);
  printf("%-34s waves/SIMD %d  %7.2f cycles per wave-instruction per SIMD  %7.1f FMA/clk/SIMD\n", name,
         waves_per_simd, cpi, fma_per_instr / cpi);
  free(h);
  hipFree(o);
  return cpi;
}

int main() {
  for (int w : {1, 4}) {
    run("v_fma_f64 (8 chains)", k_vf64, w, 8, 64, 1.0000001, 0.5);
    run("v_fma_f32 (8 chains)", k_vf32, w, 8, 64, 1.0000001f, 0.5f);
    run("v_pk_fma_f32 (8 chains)", k_vpk32, w, 8, 128, 1.0000001f, 0.5f);
    run("v_mfma_f64_16x16x4_f64 (4 acc)", k_m64, w, 4, 1024, 1.0000001, 0.5);
    run("v_mfma_f64_4x4x4_4b_f64 (4 acc)", k_m64s, w, 4, 256, 1.0000001, 0.5);
    run("v_mfma_f32_16x16x4_f32 (4 acc)", k_m32, w, 4, 1024, 1.0000001f, 0.5f);
  }
  // overlap: per iteration 2 MFMA f64 16x16x4 + NV fp64 VALU FMAs (cycles per iteration)
  printf("-- 2 x v_mfma_f64_16x16x4 + NV x v_fma_f64 per iteration, 2 waves/SIMD: cycles per iteration per SIMD\n");
  for (int w : {1, 2}) {
    run("mix NV=0", k_mix<0>, w, 1, 2048, 1.0000001, 0.5);
    run("mix NV=8", k_mix<8>, w, 1, 2048, 1.0000001, 0.5);
    run("mix NV=16", k_mix<16>, w, 1, 2048, 1.0000001, 0.5);
    run("mix NV=32", k_mix<32>, w, 1, 2048, 1.0000001, 0.5);
  }
  // the same for fp32: 2 x v_mfma_f32_16x16x4 + NV x v_fma_f32 (or v_pk_fma_f32) per iteration
  printf("-- 2 x v_mfma_f32_16x16x4 + NV x v_fma_f32 / v_pk_fma_f32 per iteration: cycles per iteration per SIMD\n");
  for (int w : {1, 2, 4}) {
    run("mix32 NV=0", k_mix32<0, false>, w, 1, 2048, 1.0000001f, 0.5f);
    run("mix32 NV=8", k_mix32<8, false>, w, 1, 2048, 1.0000001f, 0.5f);
    run("mix32 NV=16", k_mix32<16, false>, w, 1, 2048, 1.0000001f, 0.5f);
    run("mix32 NV=32", k_mix32<32, false>, w, 1, 2048, 1.0000001f, 0.5f);
    run("mix32 pk NV=16", k_mix32<16, true>, w, 1, 2048, 1.0000001f, 0.5f);
    run("mix32 pk NV=32", k_mix32<32, true>, w, 1, 2048, 1.0000001f, 0.5f);
  }
  return 0;
}
