// Per-instruction VALU issue cost on gfx950 (tool, not product).  Each kernel
// issues one instruction 8 x ITER times per lane on independent registers
// (inline asm, volatile: not moved, merged or removed), 8 waves per SIMD, so
// the time is the instruction's throughput; printed in cycles per
// wave-instruction per SIMD at the reported clock and relative to v_fma_f32.
// Used to price the integer / conversion / fp64 overheads of the certified
// kernels.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
constexpr int ITER = 2048;

#define K32(name, text)                                                                   \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    uint32_t x[8];                                                                        \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;                 \
    const uint32_t y = a + threadIdx.x, z = b ^ threadIdx.x;                              \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "+v"(x[i]) : "v"(y), "v"(z)); \
    }                                                                                     \
    uint32_t s = 0;                                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= x[i];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
  }
#define K64(name, text)                                                                   \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    double x[8];                                                                          \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = (double)(threadIdx.x + i);       \
    const double y = 1.0 + a * 1e-9, z = 0.5 + b * 1e-9;                                   \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "+v"(x[i]) : "v"(y), "v"(z)); \
    }                                                                                     \
    double s = 0;                                                                         \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s += x[i];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;                             \
  }
// 32-bit result from a 64-bit source (conversions f64 -> i32)
#define K64TO32(name, text)                                                               \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    uint32_t x[8];                                                                        \
    double y = 1.0 + a * 1e-9;                                                            \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "=v"(x[i]) : "v"(y)); \
    }                                                                                     \
    uint32_t s = 0;                                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= x[i];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + b;                                   \
  }
// 64-bit result from a 32-bit source (conversions i32 -> f64)
#define K32TO64(name, text)                                                               \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    double x[8];                                                                          \
    const uint32_t y = a + threadIdx.x;                                                   \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "=v"(x[i]) : "v"(y)); \
    }                                                                                     \
    double s = 0;                                                                         \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s += x[i];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s + b;                         \
  }
// compare into an SGPR pair
#define KCMP(name, text)                                                                  \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    uint64_t m[8];                                                                        \
    const uint32_t y = a + threadIdx.x, z = b ^ threadIdx.x;                              \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "=s"(m[i]) : "v"(y), "v"(z)); \
    }                                                                                     \
    uint64_t s = 0;                                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= m[i];                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;                             \
  }

K32(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
K32(k_add_f32, "v_add_f32 %0, %0, %1")
K32(k_mul_f32, "v_mul_f32 %0, %0, %1")
K32(k_add_u32, "v_add_u32 %0, %0, %1")
K32(k_and_b32, "v_and_b32 %0, %0, %1")
K32(k_lshl_b32, "v_lshlrev_b32 %0, %1, %0")
K32(k_add3_u32, "v_add3_u32 %0, %0, %1, %2")
K32(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1")
K32(k_bfe_u32, "v_bfe_u32 %0, %0, 8, 8")
K32(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(k_perm_b32, "v_perm_b32 %0, %0, %1, %2")
K32(k_med3_u32, "v_med3_u32 %0, %0, %1, %2")
K32(k_max_u32, "v_max_u32 %0, %0, %1")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
// masks from a compare outside the loop (the usual compiled form)
#define KMASK(name, text)                                                                 \
  __global__ void name(uint32_t* out, uint32_t a, uint32_t b) {                           \
    uint32_t x[8];                                                                        \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;                 \
    const uint32_t y = a + threadIdx.x;                                                   \
    const uint64_t m = __ballot(threadIdx.x & b);                                         \
    uint64_t c[8];                                                                        \
    for (int it = 0; it < ITER; ++it) {                                                   \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile(text : "+v"(x[i]), "=&s"(c[i]) : "v"(y), "s"(m) : "vcc"); \
    }                                                                                     \
    uint32_t s = 0;                                                                       \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s ^= x[i] ^ (uint32_t)c[i];             \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                       \
  }
KMASK(k_cnd_e64, "v_cndmask_b32_e64 %0, %0, %2, %3")
KMASK(k_addc_e64, "v_addc_co_u32_e64 %0, %1, %0, 0, %3")
KMASK(k_cmp_cnd, "v_cmp_lt_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1")
KMASK(k_cnd_vcc_set, "s_mov_b64 vcc, %3\n\tv_cndmask_b32 %0, %0, %2, vcc")
KMASK(k_cmp32_cnd32, "v_cmp_lt_u32 vcc, %0, %2\n\tv_cndmask_b32 %0, %0, %2, vcc")
KMASK(k_cmp32_only, "v_cmp_lt_u32 vcc, %0, %2")
KMASK(k_addco32, "v_add_co_u32 %0, vcc, %0, %2")
KMASK(k_addc32, "v_addc_co_u32 %0, vcc, %0, %2, vcc")
KMASK(k_cnd_e64_vcc, "v_cndmask_b32_e64 %0, %0, %2, vcc")
KMASK(k_sub_u32, "v_sub_u32 %0, %0, %2")
KMASK(k_or_b32, "v_or_b32 %0, %0, %2")
KMASK(k_xor_b32, "v_xor_b32 %0, %0, %2")
KMASK(k_sub_f32, "v_sub_f32 %0, %0, %2")
KMASK(k_fmac_f32, "v_fmac_f32 %0, %2, %2")
KMASK(k_fmamk_f32, "v_fmamk_f32 %0, %0, 0x3e991687, %2")
KMASK(k_lshrrev_b32, "v_lshrrev_b32 %0, 4, %0")
KMASK(k_min_f32, "v_min_f32 %0, %0, %2")
KMASK(k_max_i32, "v_max_i32 %0, %0, %2")
KMASK(k_cmp_f32_e64, "v_cmp_ge_f32_e64 %1, %0, %2")
K32(k_rndne_f32, "v_rndne_f32 %0, %0")
K32(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %0")
K32(k_cvt_f32_i32, "v_cvt_f32_i32 %0, %0")
K32(k_cvt_f32_ub0, "v_cvt_f32_ubyte0 %0, %0")
K32(k_frexp_f32, "v_frexp_exp_i32_f32 %0, %0")
K32(k_ffbh_u32, "v_ffbh_u32 %0, %0")
K32(k_mov_b32, "v_mov_b32 %0, %1")
K32(k_cvt_pk_u8, "v_cvt_pk_u8_f32 %0, %1, 0, %0")
K64(k_fma_f64, "v_fma_f64 %0, %0, %1, %2")
K64(k_add_f64, "v_add_f64 %0, %0, %1")
K64(k_mul_f64, "v_mul_f64 %0, %0, %1")
K64(k_max_f64, "v_max_f64 %0, %0, %1")
K64(k_ldexp_f64, "v_ldexp_f64 %0, %0, 3")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %1")
K64(k_mov_b64, "v_mov_b64 %0, %1")
K64TO32(k_cvt_i32_f64, "v_cvt_i32_f64 %0, %1")
K32TO64(k_cvt_f64_i32, "v_cvt_f64_i32 %0, %1")
KCMP(k_cmp_u32, "v_cmp_lt_u32_e64 %0, %1, %2")
K32(k_lshl_c, "v_lshlrev_b32 %0, 4, %0")
K32(k_lshr_v, "v_lshrrev_b32 %0, %1, %0")
K32(k_max_f32, "v_max_f32 %0, %0, %1")
K32(k_fmac_vv, "v_fmac_f32 %0, %1, %2")
K32(k_fmac_lit, "v_fmac_f32 %0, 0x3e991687, %1")
K32(k_fmaak, "v_fmaak_f32 %0, %0, %1, 0x43000000")
K32(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
K32(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x48")
K32(k_lshl_or, "v_lshl_or_b32 %0, %0, 8, %1")
K32(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
K32(k_or3, "v_or3_b32 %0, %0, %1, %2")
K32(k_max3_f32, "v_max3_f32 %0, %0, %1, %2")
K32(k_med3_f32, "v_med3_f32 %0, %0, %1, %2")
K32(k_ldexp_f32, "v_ldexp_f32 %0, %0, %1")
K32(k_cvt_f32_f16, "v_cvt_f32_f16 %0, %0")
K32(k_sub_f32_abs, "v_sub_f32_e64 %0, |%0|, %1")
K32(k_add_f32_e64, "v_add_f32_e64 %0, %0, %1")
K32(k_add_u32_e64, "v_add_u32_e64 %0, %0, %1")
K32(k_and_e64, "v_and_b32_e64 %0, %0, %1")
K32(k_mov_dpp, "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
K32(k_add_dpp, "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
K64(k_pk_add, "v_pk_add_f32 %0, %0, %1")
K64(k_pk_mul, "v_pk_mul_f32 %0, %0, %1")
K64(k_pk_fma, "v_pk_fma_f32 %0, %0, %1, %2")
K64(k_fma_f64_s, "v_fma_f64 %0, %0, %1, 0.5")
K64(k_add_f64_c, "v_add_f64 %0, %0, 1.0")
K32TO64(k_cvt_f64_f32, "v_cvt_f64_f32 %0, %1")
K64TO32(k_cvt_f32_f64, "v_cvt_f32_f64 %0, %1")

template <typename F>
static float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 2; ++w) f();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int blocks = p.multiProcessorCount * 8, threads = 256;  // 8 waves per SIMD
  uint32_t* buf;
  hipMalloc(&buf, (size_t)blocks * threads * 4);
  const double waves_per_simd = (double)blocks * threads / 64 / (p.multiProcessorCount * 4);
  const double instr = (double)ITER * 8;
  const double clk = p.clockRate * 1e3;  // Hz
  double ref = 0.0;
  struct E {
    const char* n;
    void (*k)(uint32_t*, uint32_t, uint32_t);
  };
  const E list[] = {
      {"v_fma_f32", k_fma_f32},         {"v_add_f32", k_add_f32},         {"v_mul_f32", k_mul_f32},
      {"v_add_u32", k_add_u32},         {"v_and_b32", k_and_b32},         {"v_lshlrev_b32", k_lshl_b32},
      {"v_add3_u32", k_add3_u32},       {"v_lshl_add_u32", k_lshl_add},   {"v_bfe_u32", k_bfe_u32},
      {"v_mad_u32_u24", k_mad_u24},     {"v_mul_lo_u32", k_mul_lo_u32},   {"v_perm_b32", k_perm_b32},
      {"v_med3_u32", k_med3_u32},       {"v_max_u32", k_max_u32},         {"v_cndmask_b32", k_cndmask},
      {"v_cndmask_b32_e64 (s mask)", k_cnd_e64}, {"v_addc_co_u32_e64", k_addc_e64},
      {"v_cmp_e64 + v_cndmask_e64 (pair)", k_cmp_cnd}, {"s_mov vcc + v_cndmask (pair)", k_cnd_vcc_set},
      {"v_cmp_e32 vcc + v_cndmask_e32", k_cmp32_cnd32}, {"v_cmp_e32 (vcc)", k_cmp32_only},
      {"v_add_co_u32_e32 (vcc out)", k_addco32}, {"v_addc_co_u32_e32 (vcc)", k_addc32},
      {"v_cndmask_b32_e64 (vcc)", k_cnd_e64_vcc}, {"v_sub_u32", k_sub_u32}, {"v_or_b32", k_or_b32},
      {"v_xor_b32", k_xor_b32}, {"v_sub_f32", k_sub_f32}, {"v_fmac_f32", k_fmac_f32},
      {"v_fmamk_f32", k_fmamk_f32}, {"v_lshrrev_b32", k_lshrrev_b32}, {"v_min_f32", k_min_f32},
      {"v_max_i32", k_max_i32}, {"v_cmp_ge_f32_e64", k_cmp_f32_e64},
      {"v_rndne_f32", k_rndne_f32},     {"v_cvt_i32_f32", k_cvt_i32_f32}, {"v_cvt_f32_i32", k_cvt_f32_i32},
      {"v_cvt_f32_ubyte0", k_cvt_f32_ub0}, {"v_frexp_exp_i32_f32", k_frexp_f32}, {"v_ffbh_u32", k_ffbh_u32},
      {"v_mov_b32", k_mov_b32},         {"v_cvt_pk_u8_f32", k_cvt_pk_u8}, {"v_fma_f64", k_fma_f64},
      {"v_add_f64", k_add_f64},         {"v_mul_f64", k_mul_f64},         {"v_max_f64", k_max_f64},
      {"v_ldexp_f64", k_ldexp_f64},     {"v_lshl_add_u64", k_lshl_add_u64}, {"v_mov_b64", k_mov_b64},
      {"v_cvt_i32_f64", k_cvt_i32_f64}, {"v_cvt_f64_i32", k_cvt_f64_i32}, {"v_cmp_lt_u32_e64", k_cmp_u32},
      {"v_lshlrev_b32 (const)", k_lshl_c},
      {"v_lshrrev_b32 (vgpr)", k_lshr_v},
      {"v_max_f32", k_max_f32},
      {"v_fmac_f32 (vgpr)", k_fmac_vv},
      {"v_fmac_f32 (literal)", k_fmac_lit},
      {"v_fmaak_f32", k_fmaak},
      {"v_mul_u32_u24", k_mul_u24},
      {"v_mul_hi_u32", k_mul_hi},
      {"v_bitop3_b32", k_bitop3},
      {"v_lshl_or_b32", k_lshl_or},
      {"v_and_or_b32", k_and_or},
      {"v_or3_b32", k_or3},
      {"v_max3_f32", k_max3_f32},
      {"v_med3_f32", k_med3_f32},
      {"v_ldexp_f32", k_ldexp_f32},
      {"v_cvt_f32_f16", k_cvt_f32_f16},
      {"v_sub_f32_e64 |abs|", k_sub_f32_abs},
      {"v_add_f32_e64", k_add_f32_e64},
      {"v_add_u32_e64", k_add_u32_e64},
      {"v_and_b32_e64", k_and_e64},
      {"v_mov_b32_dpp", k_mov_dpp},
      {"v_add_u32_dpp", k_add_dpp},
      {"v_pk_add_f32", k_pk_add},
      {"v_pk_mul_f32", k_pk_mul},
      {"v_pk_fma_f32", k_pk_fma},
      {"v_fma_f64 (inline const)", k_fma_f64_s},
      {"v_add_f64 (inline const)", k_add_f64_c},
      {"v_cvt_f64_f32", k_cvt_f64_f32},
      {"v_cvt_f32_f64", k_cvt_f32_f64},
  };
  printf("gfx950 VALU throughput, 8 waves/SIMD, 8 independent registers per lane, %d x 8 per lane\n", ITER);
  printf("cycles per wave-instruction per SIMD at the reported %.2f GHz; rel = / v_fma_f32\n", clk / 1e9);
  for (const E& e : list) {
    const float ms = timeit([&] { hipLaunchKernelGGL(e.k, blocks, threads, 0, 0, buf, 3u, 5u); });
    const double cyc = ms * 1e-3 * clk / (instr * waves_per_simd);
    if (ref == 0.0) ref = cyc;
    printf("%-22s %8.4f ms  %6.2f cycles  rel %5.2f\n", e.n, ms, cyc, cyc / ref);
  }
  hipFree(buf);
  return 0;
}
