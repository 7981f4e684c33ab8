// VALU issue-rate microbenchmark (gfx950): scalar fp32 FMA, packed fp32 FMA
// (v_pk_fma_f32), fp64 FMA and int32 mad, 8 independent accumulators per lane,
// enough waves to fill every SIMD.  Prints the per-instruction cost in cycles
// per wave (4 = full rate for a wave64 on a 16-lane SIMD).  Tool, not product.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

__global__ void k_f32(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pk(float* out, float a, float b) {
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = (f2){(float)threadIdx.x + i, (float)i};
  const f2 A = {a, a * 2.0f}, B = {b, b * 3.0f};
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], A, B);
  float s = 0; for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_f64(double* out, double a, double b) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, b);
  double s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_i32(int* out, int a, int b) {
  int x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < ITER; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = x[i] * a + b;
  int s = 0; for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
static float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) f();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

int main() {
  int dev; hipGetDevice(&dev);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  const int blocks = p.multiProcessorCount * 8, threads = 256;  // 8 waves per SIMD
  void* buf; hipMalloc(&buf, (size_t)blocks * threads * 8);
  const double waves_per_simd = (double)blocks * threads / 64 / (p.multiProcessorCount * 4);
  const double instr = (double)ITER * 8;
  const double clk_ghz = p.clockRate / 1e6;
  auto report = [&](const char* n, float ms) {
    const double cyc = ms * 1e-3 * clk_ghz * 1e9;  // at the reported max clock
    printf("%-10s %8.3f ms  ~%.2f cycles per wave-instruction per SIMD (clock %.2f GHz)\n", n, ms,
           cyc / (instr * waves_per_simd), clk_ghz);
  };
  report("fma_f32", timeit([&] { hipLaunchKernelGGL(k_f32, blocks, threads, 0, 0, (float*)buf, 1.0001f, 0.5f); }));
  report("pk_fma_f32", timeit([&] { hipLaunchKernelGGL(k_pk, blocks, threads, 0, 0, (float*)buf, 1.0001f, 0.5f); }));
  report("fma_f64", timeit([&] { hipLaunchKernelGGL(k_f64, blocks, threads, 0, 0, (double*)buf, 1.0001, 0.5); }));
  report("mad_i32", timeit([&] { hipLaunchKernelGGL(k_i32, blocks, threads, 0, 0, (int*)buf, 3, 1); }));
  return 0;
}
