// tools/probe_fwd.cpp — kernel-level timing probe (not product code).  Unity
// build of the HIP sources; JDS_PROBE_* macros strip parts of k_fwd32 to
// attribute its time.  Prints avg microseconds per launch for 64 1080p frames.
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
#include <cstdlib>
#include <vector>

using namespace jds;

int main(int argc, char** argv) {
  const int n = 64, H = 1080, W = 1920;
  static const double Q50[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                 14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                 18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
  jds_params prm{};
  prm.block_size = 8;
  prm.quality = 50;
  prm.subsampling = JDS_SS_420;
  prm.prefilter = 1;
  for (int i = 0; i < 64; ++i) prm.qtable[i] = Q50[i];
  prm.gauss[0] = 0.25; prm.gauss[1] = 0.5; prm.gauss[2] = 0.25;
  Geo g; int mode; bool pf;
  if (make_geo(&prm, H, W, &g, &mode, &pf)) { printf("geo fail\n"); return 1; }
  std::vector<uint8_t> h((size_t)n * H * W * 3);
  uint32_t x = 12345;
  for (auto& b : h) { x = x * 1664525u + 1013904223u; b = (uint8_t)(x >> 24); }
  uint8_t *rgb, *out; int16_t* cf; jds_frame_stats* st; FastQ* fq32; FrameQ* fq; float* gk32; double* gk; uint2* fl; unsigned* cnt; uint32_t* part;
  hipMalloc(&rgb, h.size()); hipMalloc(&out, h.size());
  hipMalloc(&cf, (size_t)n * g.cpf * 2); hipMalloc(&st, sizeof(jds_frame_stats) * n);
  hipMalloc(&fq32, sizeof(FastQ) * n); hipMalloc(&fq, sizeof(FrameQ) * n); hipMalloc(&gk32, 16); hipMalloc(&gk, 32);
  hipMalloc(&fl, 8 * (size_t)n * (g.cpf / 64)); hipMalloc(&cnt, 64); hipMalloc(&part, 4 * 52 * (size_t)n * g.tiles_y * g.tiles_x);
  hipMemcpy(rgb, h.data(), h.size(), hipMemcpyHostToDevice);
  FastQ hq; fast_fwd_thresholds(prm.qtable, mode, pf, prm.gauss, hq.rq, &hq.thr[0][0]);
  FrameQ hf; make_fq(&prm, &hf);
  for (int i = 0; i < n; ++i) { hipMemcpy(fq32 + i, &hq, sizeof hq, hipMemcpyHostToDevice); hipMemcpy(fq + i, &hf, sizeof hf, hipMemcpyHostToDevice); }
  const float g3[3] = {0.25f, 0.5f, 0.25f};
  hipMemcpy(gk32, g3, 12, hipMemcpyHostToDevice); hipMemcpy(gk, prm.gauss, 24, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto time_it = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    const int R = 20;
    for (int i = 0; i < R; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s %9.1f us\n", name, ms * 1000 / R);
  };
  using C = Cfg<M420>;
  int4 rect;
  rect.x = (g.ty_off * C::MH > 0) ? 1 : 0; rect.y = (g.H / C::MH + g.ty_off) / C::MY - 1;
  rect.z = (g.tx_off * C::MW > 0) ? 1 : 0; rect.w = (g.W / C::MW + g.tx_off) / C::MX - 1;
  const int nin = (rect.y - rect.x + 1) * (rect.w - rect.z + 1);
  const dim3 gi(nin, n), gb(g.tiles_y * g.tiles_x - nin, n), ga(g.tiles_y * g.tiles_x, n);
  time_it("fwd32 interior", [&] { hipMemsetAsync(cnt, 0, 64, 0); hipLaunchKernelGGL((k_fwd32i<M420, true>), gi, dim3(C::TF), 0, 0, g, rgb, cf, fq32, gk32, part, fl, cnt, rect, (float*)nullptr, st, 1); });
  time_it("fwd32 border", [&] { hipMemsetAsync(cnt, 0, 64, 0); hipLaunchKernelGGL((k_fwd32<M420, true>), gb, dim3(C::TF), 0, 0, g, rgb, cf, fq32, gk32, part, fl, cnt, 1, rect, (float*)nullptr, (jds_frame_stats*)nullptr, 1); });
  time_it("fwd32 general, all tiles", [&] { hipMemsetAsync(cnt, 0, 64, 0); hipLaunchKernelGGL((k_fwd32<M420, true>), ga, dim3(C::TF), 0, 0, g, rgb, cf, fq32, gk32, part, fl, cnt, 0, rect, (float*)nullptr, st, 1); });
  time_it("inv2", [&] { launch_inv2(M420, g, n, cf, fq, nullptr, out, st, nullptr, nullptr, nullptr, 0, 1); });
  {
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    auto both = [&](bool conc) {
      hipStream_t sa = s1, sb = conc ? s2 : s1;
      hipLaunchKernelGGL((k_fwd32i<M420, true>), gi, dim3(C::TF), 0, sa, g, rgb, cf, fq32, gk32, part, fl, cnt, rect, (float*)nullptr, st, 1);
      launch_inv2(M420, g, n, cf, fq, nullptr, out, st, nullptr, nullptr, nullptr, sb, 1);
    };
    for (int conc = 0; conc < 2; ++conc) {
      for (int i = 0; i < 3; ++i) both(conc);
      hipDeviceSynchronize();
      auto t0 = std::chrono::high_resolution_clock::now();
      for (int i = 0; i < 20; ++i) both(conc);
      hipDeviceSynchronize();
      auto t1 = std::chrono::high_resolution_clock::now();
      printf("fwd-interior + inv2 %-10s %9.1f us\n", conc ? "concurrent" : "serial",
             std::chrono::duration<double, std::micro>(t1 - t0).count() / 20);
    }
  }
  {
    unsigned hc = 0; hipMemset(cnt, 0, 64);
    hipLaunchKernelGGL((k_fwd32<M420, true>), gb, dim3(C::TF), 0, 0, g, rgb, cf, fq32, gk32, part, fl, cnt, 1, rect, (float*)nullptr, (jds_frame_stats*)nullptr, 1);
    hipLaunchKernelGGL((k_fwd32i<M420, true>), gi, dim3(C::TF), 0, 0, g, rgb, cf, fq32, gk32, part, fl, cnt, rect, (float*)nullptr, st, 1);
    hipMemcpy(&hc, cnt, 4, hipMemcpyDeviceToHost);
    printf("flagged blocks (64 frames): %u\n", hc);
    std::vector<uint2> hl(hc);
    hipMemcpy(hl.data(), fl, 8 * (size_t)hc, hipMemcpyDeviceToHost);
    unsigned byplane[3] = {0, 0, 0};
    for (auto& e : hl) byplane[(e.y >> 24) & 3]++;
    printf("  by plane: Y %u  Cb %u  Cr %u\n", byplane[0], byplane[1], byplane[2]);
    for (int p = 0; p < 2; ++p) {
      printf("  thr[%d] (x1e4):", p);
      for (int i = 0; i < 64; i += 9) printf(" %.3f", hq.thr[p][i] * 1e4);
      printf("\n");
    }
  }
  printf("done\n");
  return 0;
}
