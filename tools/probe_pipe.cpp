// tools/probe_pipe.cpp — pipelining probe (not product code): 64 1080p Q50 4:2:0
// frames per batch through the C-ABI plans; serial fwd+inv per batch versus
// forward of batch k+1 beside the inverse of batch k on a second stream.
#include "../jpeg-dsp-studio_amd/csrc/jds_codec.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_b16.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_inv.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_fast.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_stages.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_ssim.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_entropy.hip"
#include "../jpeg-dsp-studio_amd/csrc/jds_abi.hip"
#include <chrono>
#include <cstdio>
#include <vector>

int main() {
  const int n = 64, H = 1080, W = 1920, STEPS = 20;
  static const double Q50[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                 14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                 18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
  jds_params prm{};
  prm.block_size = 8; prm.quality = 50; prm.subsampling = JDS_SS_420; prm.prefilter = 1;
  for (int i = 0; i < 64; ++i) prm.qtable[i] = Q50[i];
  prm.gauss[0] = 0x1.3dba0f6bc8fa9p-2; prm.gauss[1] = 0x1.8489e12868ad6p-2; prm.gauss[2] = prm.gauss[0];
  std::vector<jds_params> ps(n, prm);
  jds_ctx* ctx; jds_ctx_create(0, &ctx);
  jds_plan* pl[2];
  for (int i = 0; i < 2; ++i)
    if (jds_plan_create(ctx, ps.data(), n, H, W, &pl[i])) { printf("plan: %s\n", jds_last_error()); return 1; }
  jds_geometry geo; jds_plan_geometry(pl[0], &geo);
  const size_t img = (size_t)n * H * W * 3;
  std::vector<uint8_t> h(img);
  uint32_t x = 12345;
  for (auto& b : h) { x = x * 1664525u + 1013904223u; b = (uint8_t)(x >> 24); }
  uint8_t *rgb[2], *out[2]; int16_t* cf[2]; jds_frame_stats* st[2];
  for (int i = 0; i < 2; ++i) {
    hipMalloc(&rgb[i], img); hipMalloc(&out[i], img);
    hipMalloc(&cf[i], (size_t)n * geo.coeffs_per_frame * 2); hipMalloc(&st[i], sizeof(jds_frame_stats) * n);
    hipMemcpy(rgb[i], h.data(), img, hipMemcpyHostToDevice);
  }
  hipStream_t sa, sb;
  hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
  hipEvent_t fdone[2], idone[2];
  for (int i = 0; i < 2; ++i) { hipEventCreateWithFlags(&fdone[i], hipEventDisableTiming); hipEventCreateWithFlags(&idone[i], hipEventDisableTiming); }
  auto serial = [&](int k) {
    jds_plan_run(pl[0], rgb[0], out[0], cf[0], st[0], JDS_RUN_FWD, sa);
    jds_plan_run(pl[0], rgb[0], out[0], cf[0], st[0], JDS_RUN_INV, sa);
  };
  auto piped = [&](int k) {  // fwd(k) on sa, inv(k) on sb after fwd(k); fwd(k) waits inv(k-2) (same buffers)
    const int b = k & 1;
    hipStreamWaitEvent(sa, idone[b], 0);
    jds_plan_run(pl[b], rgb[b], out[b], cf[b], st[b], JDS_RUN_FWD, sa);
    hipEventRecord(fdone[b], sa);
    hipStreamWaitEvent(sb, fdone[b], 0);
    jds_plan_run(pl[b], rgb[b], out[b], cf[b], st[b], JDS_RUN_INV, sb);
    hipEventRecord(idone[b], sb);
  };
  for (int mode = 0; mode < 2; ++mode) {
    for (int k = 0; k < 3; ++k) mode ? piped(k) : serial(k);
    hipDeviceSynchronize();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int k = 0; k < STEPS; ++k) mode ? piped(k) : serial(k);
    hipDeviceSynchronize();
    auto t1 = std::chrono::high_resolution_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / STEPS;
    printf("%-8s %8.1f us per batch  %8.0f Mpix/s\n", mode ? "piped" : "serial", us, (double)n * H * W / us);
  }
  return 0;
}
