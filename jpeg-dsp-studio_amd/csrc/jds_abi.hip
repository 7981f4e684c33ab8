// jds_abi.hip — the C-ABI (include/jds.h): contexts, plans, host-buffer path.
//
// Host side only orchestrates: geometry, quant-table upload, buffer
// management and launches.  All per-pixel / per-coefficient arithmetic runs
// in the HIP kernels of jds_codec.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>
#include <mutex>
#include <new>

#include "jds_dct16.hpp"
#include "jds_dct8.hpp"
#include "jds_internal.hpp"

#ifdef JDS_INV6
#define JDS_INV6_LIST 1  // the transpose-free variant's tile list (A/B builds: tools/build_variant.py)
#else
#define JDS_INV6_LIST 0
#endif

namespace jds {
hipError_t launch_codec(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, uint8_t* rgb_out,
                        int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st,
                        double* part, bool want_sse, double* err_y, double* err_rgb, jds_selected_block* sel,
                        int sel_blk, hipStream_t s, hipEvent_t* ev, int phases, int in_div, const GenBufs* gb,
                        const InvFix* fx = nullptr);
int inv_tiles(int mode, int H, int W);
int area_tab_build(int src, int dst, AreaTap* tab);
size_t gen_sub_doubles(const Geo& g);
size_t gen_rec_doubles(const Geo& g);
int gen_px_tiles(const Geo& g);
hipError_t stage_area_gen(const double* in, int H, int W, const AreaTap* ytab, const AreaTap* xtab, double* out,
                          int oh, int ow, hipStream_t s);
hipError_t launch_psnr_ssim_batch(const void* pairs_dev, int items, int H, int W, double c1, double c2,
                                  double* scratch, double* out, int out_stride, unsigned long long* sse,
                                  hipStream_t s, bool rgb, hipStream_t side, hipEvent_t fork, hipEvent_t join);
hipError_t launch_ssim_rgb(const void* pairs_dev, int items, int H, int W, double c1, double c2, double* scratch,
                           double* out, int out_stride, hipStream_t s);
size_t ssim_batch_scratch_doubles(int H, int W, bool rgb, bool planes);
bool ssim_batch_planes(int items);
size_t ssim_rgb_scratch_doubles(int H, int W);
int ssim_batch_max_items();
hipError_t launch_sse_u8(const uint8_t* a, const uint8_t* b, long long n, unsigned long long* out, hipStream_t s);
size_t mag_scratch_bytes(long long nblocks, int max_chunks);
hipError_t launch_mag_f32(const int16_t* coeffs, long long nblocks, unsigned* chunk_sum, int max_chunks,
                          double* out, hipStream_t s);
void combined_taps32(const double* gk, float* out5);
size_t fast_part_words(const Geo& g, int n);
hipError_t launch_fast_fwd(int mode, bool pf, const Geo& g, int n, int nq, const uint8_t* rgb, int16_t* coeffs,
                           const FrameQ* fq, const void* fq32, const double* gk, const float* gk32,
                           jds_frame_stats* st, uint32_t* part, uint32_t* fixbits, uint2* fixlist, unsigned* fixcount,
                           float* dct32,
                           hipStream_t s, bool finish, int par);
int quant_mq_tiles(const Geo& g);
int inv16_tiles(int mode, int H, int W);
constexpr int MAXQ_SHARED = 8;  // jds_fast.hip MAXQ
void fast_fwd_bounds(int mode, bool pf, const double* gk, double* E);
int fwd32_host_plane(int mode, bool pf, const double* gk, const uint8_t* rgb, int H, int W, int plane,
                     int flags, float* out);
void fast_fwd_thresholds(const double* Q, int mode, bool pf, const double* gk, float* rq, float* thr);
int inv_fast_host(int mode, const int16_t* cf, const double* Q, int H, int W, int fuse, int block, double* vout,
                  uint8_t* bout);
size_t fast_q_size();
hipError_t stage_rgb_ycc(const double* in, double* out, long long n, int inverse, hipStream_t s);
hipError_t stage_subsample(const double* in, double* tmp, double* tmp2, double* out, int H, int W, int sy,
                           int prefilter, const double* k, hipStream_t s);
hipError_t stage_resize(const double* in, int h, int w, double* out, int H, int W, int nearest, hipStream_t s);
hipError_t stage_block(const double* in, double* out, long long n, int bs, int op, hipStream_t s);
hipError_t stage_quant(const void* in, const double* q, void* out, long long n, int dequant, int period,
                       hipStream_t s);
int tile_dims16(int mode, int* MY, int* MX);
struct EntTab;
void ent_build_tables(EntTab* t);
size_t ent_tab_size();
int ent_header(const double* q, int mode, int H, int W, uint8_t* o);
long long ent_capacity(const Geo& g);
void ent_sizes(const Geo& g, int n, size_t* sz);
hipError_t launch_entropy(const Geo& g, int n, const int16_t* coeffs, void* const* buf, const uint8_t* hdr_dev,
                          const void* tab_dev, uint8_t* out, long long stride, unsigned long long* lengths,
                          unsigned long long* scan_bits, hipStream_t s);
hipError_t launch_codec16(int mode, bool pf, const Geo& g, int n, const uint8_t* rgb, uint8_t* rgb_out,
                          int16_t* coeffs, const FrameQ* fq, const double* gk, jds_frame_stats* st, double* part,
                          double* planes, bool want_sse, double* err_y, double* err_rgb, hipStream_t s,
                          hipEvent_t* ev, int phases, const Fwd16Fast* ff, const InvFix* fx);
void fast_fwd16_bounds(int mode, bool pf, const double* gk, double* E);
void fast_fwd16_thresholds(const double* Q8, int mode, bool pf, const double* gk, void* out);
size_t fast_q16_size();
int fwd16_host_plane(int mode, bool pf, const double* gk, const uint8_t* rgb, int H, int W, int plane,
                     int flags, float* out);
}

// skimage: C1 = (K1 * R) ** 2, C2 = (K2 * R) ** 2 with R = data_range = 255
static const double SSIM_C1 = (0.01 * 255) * (0.01 * 255);
static const double SSIM_C2 = (0.03 * 255) * (0.03 * 255);

using namespace jds;

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(e_ == hipErrorOutOfMemory ? JDS_ENOMEM : JDS_EHIP, "%s: %s (%s:%d)", #expr, \
                  hipGetErrorString(e_), __FILE__, __LINE__);                               \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct jds_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  // host path: the device -> host copies run on a stream of their own beside
  // the statistics kernels (SSIM, float32 magnitude bits) of the same call
  hipStream_t xfer = nullptr;
  hipEvent_t xfer_ev = nullptr;
  // SSIM: the R, G, B rows kernels run on a stream of its own beside the luma
  // planes, chains and band (jds_ssim_band.hip); ss_pairs: the batch's image
  // pointers (pinned host staging, device copy)
  hipStream_t ss_side = nullptr;
  hipEvent_t ss_fork = nullptr, ss_join = nullptr;
  void* ss_pairs_host = nullptr;
  size_t ss_pairs_cap = 0;
  // host-path scratch
  DevBuf rgb, out, coeffs, stats, part, fq, gk, erry, errrgb, sel;
  DevBuf ss_planes, ss_out, img_a, img_b;  // ss_planes: k_ss_* scratch
  DevBuf ss_rgb, ss_pairs;                 // k_ss_rows / k_ss_rgbsum scratch, device pair array
  DevBuf st[5];  // per-stage API staging
  DevBuf chunks;
  DevBuf planes;  // 16x16 path: reconstructed chroma planes
  DevBuf ent[8], ent_hdr, ent_tab, ent_cf, ent_out, ent_meta;  // entropy coder (jds_encode_jfif)
  DevBuf gen_tab, gen_sub, gen_rec;  // general-geometry path (jds_gen.hip)
  size_t ss_budget = 0;  // SSIM scratch budget per launch group (0: SSIM_SCRATCH; jds_ctx_set_ssim_scratch)
};

// batches from this size take the R, G, B rows kernel (jds_ssim_band.hip)
constexpr int SSIM_ROWS_MIN = 32;
// SSIM scratch (luma planes, chain checkpoints, maps) per launch group
constexpr size_t SSIM_SCRATCH = (size_t)16 << 30;

// SSIM of `items` image pairs (K4, jds_ssim_band.hip) on the context's stream:
// out[i * out_stride + 0..4] = SSIM R, G, B, Y, MSE of Y (device doubles);
// sse[i] (nullable, zeroed here) = the pair's integer RGB squared-error sum.
// Batches beyond the kernel's per-launch limit run as consecutive launches.
static int run_ssim_batch(jds_ctx* c, int items, const uint8_t* const* a, const uint8_t* const* b, int H, int W,
                          double* out, int out_stride, unsigned long long* sse) {
  // R, G, B: batches of SSIM_ROWS_MIN items or more take the rows kernel (one
  // lane per map row, every item in one launch: its grid fills the chip only
  // with many items); smaller ones the band kernel beside each luma group
  const bool rows = items >= SSIM_ROWS_MIN && (unsigned long long)H * W * 3ull < (1ull << 31);  // (32-bit staging)
  const int per = ssim_batch_max_items();
  // luma (and small batches' RGB) scratch: as many items per launch as the
  // budget holds (1080p: ~27 MB per item; launches under 8 pairs keep fp64
  // luma planes, ~60 MB, ~110 MB with RGB maps) -- the luma chains, like the
  // rows, are latency-bound per lane and need many items in flight.  A
  // launch's layout (planes or not) follows its own size, so the group size
  // is settled first and the scratch sized for the groups that actually run:
  // the full groups and the remainder.
  const size_t budget = c->ss_budget ? c->ss_budget : SSIM_SCRATCH;
  auto bytes_of = [&](int k) {  // scratch of one launch of k pairs
    return ssim_batch_scratch_doubles(H, W, !rows, ssim_batch_planes(k)) * sizeof(double) * (size_t)k;
  };
  int group = std::min(per, items);
  if (bytes_of(group) > budget) {
    const size_t each_np = ssim_batch_scratch_doubles(H, W, !rows, false) * sizeof(double);
    group = (int)std::max<size_t>(1, std::min<size_t>((size_t)group, budget / each_np));
    if (ssim_batch_planes(group) && bytes_of(group) > budget) {  // the planes layout: larger per item
      const size_t each_p = ssim_batch_scratch_doubles(H, W, !rows, true) * sizeof(double);
      group = (int)std::max<size_t>(1, std::min<size_t>((size_t)group, budget / each_p));
    }
  }
  size_t need = bytes_of(group);
  const int last = items % group;
  if (last) need = std::max(need, bytes_of(last));
  HIP_TRY(c->ss_planes.ensure(need));
  if (!c->ss_side) {
    HIP_TRY(hipStreamCreateWithFlags(&c->ss_side, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c->ss_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ss_join, hipEventDisableTiming));
  }
  // the pair array: pinned staging (reused only after the previous call's
  // final synchronisation) -> device, on the context's stream
  const size_t pbytes = sizeof(const void*) * 2 * (size_t)items;
  if (c->ss_pairs_cap < pbytes) {
    if (c->ss_pairs_host) HIP_TRY(hipHostFree(c->ss_pairs_host));
    c->ss_pairs_host = nullptr;
    c->ss_pairs_cap = 0;
    HIP_TRY(hipHostMalloc(&c->ss_pairs_host, pbytes, hipHostMallocDefault));
    c->ss_pairs_cap = pbytes;
  }
  const void** ph = (const void**)c->ss_pairs_host;
  for (int i = 0; i < items; ++i) {
    ph[2 * i] = a[i];
    ph[2 * i + 1] = b[i];
  }
  HIP_TRY(c->ss_pairs.ensure(pbytes));
  HIP_TRY(hipMemcpyAsync(c->ss_pairs.p, ph, pbytes, hipMemcpyHostToDevice, c->stream));
  auto pairs_at = [&](int i0) { return (const void*)((const char*)c->ss_pairs.p + sizeof(const void*) * 2 * (size_t)i0); };
  if (sse) HIP_TRY(hipMemsetAsync(sse, 0, sizeof(unsigned long long) * items, c->stream));
  if (rows) {
    // as many items per launch as ~4 GB of scratch holds (1080p: ~4 MB per item)
    const size_t each_rgb = ssim_rgb_scratch_doubles(H, W) * sizeof(double);
    const int group_rgb = (int)std::min<size_t>((size_t)items, std::max<size_t>(1, ((size_t)4 << 30) / each_rgb));
    HIP_TRY(c->ss_rgb.ensure(each_rgb * group_rgb));
    // on the side stream (after the copy and the stream's earlier work), beside
    // the luma groups on the context's stream; joined at the end
    HIP_TRY(hipEventRecord(c->ss_fork, c->stream));
    HIP_TRY(hipStreamWaitEvent(c->ss_side, c->ss_fork, 0));
    for (int i0 = 0; i0 < items; i0 += group_rgb) {
      const int k = std::min(group_rgb, items - i0);
#ifdef JDS_SSIM_PROBE_NORGB  // tools: timing probes only (wrong values)
      continue;
#endif
      HIP_TRY(launch_ssim_rgb(pairs_at(i0), k, H, W, SSIM_C1, SSIM_C2, (double*)c->ss_rgb.p,
                              out + (size_t)i0 * out_stride, out_stride, c->ss_side));
    }
    HIP_TRY(hipEventRecord(c->ss_join, c->ss_side));
  }
  for (int i0 = 0; i0 < items; i0 += group) {
    const int k = std::min(group, items - i0);
#ifdef JDS_SSIM_PROBE_NOLUMA  // tools: timing probes only (wrong values)
    if (rows) continue;
#endif
    HIP_TRY(launch_psnr_ssim_batch(pairs_at(i0), k, H, W, SSIM_C1, SSIM_C2, (double*)c->ss_planes.p,
                                   out + (size_t)i0 * out_stride, out_stride, sse ? sse + i0 : nullptr, c->stream,
                                   !rows, c->ss_side, c->ss_fork, c->ss_join));
  }
  if (rows) HIP_TRY(hipStreamWaitEvent(c->stream, c->ss_join, 0));
  return JDS_OK;
}

// one pair; returns the device pointer of 5 result doubles in dres
static int run_ssim(jds_ctx* c, const uint8_t* a, const uint8_t* b, int H, int W, double* dres) {
  return run_ssim_batch(c, 1, &a, &b, H, W, dres, 5, nullptr);
}

struct jds_plan {
  jds_ctx* ctx = nullptr;
  int n = 0, mode = 0;
  int nq = 1;      // tables per frame (sweep plan): items = frames * nq, item = frame * nq + q
  DevBuf dct32;    // sweep plans: fp32 coefficients of every frame (shared front end)
  bool pf = false;
  Geo g{};
  DevBuf fq, gk, part;
  // fast path: fp32 tables, fix-up lists and counters
  DevBuf fq32, gk32, fixbits, fixlist, counters, part32;  // per-item fix-up bitmaps and lists; per-tile statistics
  DevBuf invfix;  // certified fast inverse: run and per-item counters (InvFix, jds_inv_fast.hip)
  DevBuf invlist;  // k_inv_fast6 (4:2:0, -DJDS_INV6 builds): the tiles a run hands to the exact kernel (InvFix::list)
  unsigned inv_runs = 0;  // fast-inverse runs so far: picks the list counter (InvFix::parity)
  bool last_inv_fast = false;  // the last run's inverse was the certified fast one
  // Where the certified fast inverse pays (measured, 1 MI355X): 4:2:x plans
  // whose tables are not coarse.  Coarse tables (DC quantiser > 60: quality
  // below ~14 on the standard table) put most tiles on the exact path
  // (reconstructions land on integers), where k_inv2 beats k_inv_fast's
  // in-kernel fallback (4K 4:2:0: Q10 373 vs 396 us; Q20 376 vs 347).  At
  // 4:4:4 the wave-local k_inv_fast444 is faster at every quality (512x512 x
  // 256: 167.5 vs k_inv2's 331.8 us).
  bool inv_fast_ok = true;
  // some item's table is not coarse: mixed plans (quality sweeps) run the
  // certified inverse too, their coarse items seeded into its per-item exact
  // mode (InvFix), so every item takes the faster kernel for its table
  bool inv_fast_any = true;
  bool last_fwd16_fast = false;  // 16x16: the last forward was the certified fp32 one
  unsigned fwd16_runs = 0;       // 16x16 certified forward runs so far: picks the list counter
  unsigned fwd8_runs = 0;        // 8x8 single-quality certified forward runs: picks the counter bank
  int last_fwd8_bank = -1;       // bank of the last such run (jds_plan_fix_counts), -1: none
  InvFix inv_fix() const {
    return {(unsigned*)invfix.p, (unsigned*)invfix.p + 16, 0, (int)(inv_runs & 1u), (int)(inv_runs % 3u),
            (int)(inv_runs % 16u == 15u), (uint2*)invlist.p};
  }
  DevBuf planes;  // 16x16 path: reconstructed chroma planes (n x 2 x hc x wc f64)
  double* qt = nullptr;  // host copy of the per-frame 8x8 tables (entropy headers)
  DevBuf ent[8], ent_hdr, ent_tab;  // entropy coder scratch, allocated by the first jds_plan_entropy
  DevBuf gen_tab, gen_sub, gen_rec;  // general-geometry path (jds_gen.hip)
  GenBufs gen() const { return {(const AreaTap*)gen_tab.p, (double*)gen_sub.p, (double*)gen_rec.p}; }
  // jds_plan_profile: the launch marks of profiled runs (event pool + names)
  bool prof_on = false;
  KMarks marks;
};

namespace jds {
thread_local KMarks* t_kmarks = nullptr;

void kmark(hipStream_t s, const char* fmt, ...) {
  KMarks* m = t_kmarks;
  if (!m) return;
  if (m->n >= m->cap) {  // reported by jds_plan_profile_read (the totals would be short)
    m->dropped++;
    return;
  }
  if (hipEventRecord(m->ev[m->n], s) != hipSuccess) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(m->name[m->n], sizeof m->name[0], fmt, ap);
  va_end(ap);
  m->n++;
}
}  // namespace jds

// Marks the runs of a profiled plan on this thread (jds_plan_run's scope).
struct MarkScope {
  explicit MarkScope(jds_plan* p, hipStream_t s) {
    if (!p->prof_on) return;
    t_kmarks = &p->marks;
    kmark(s, "(between runs)");
  }
  ~MarkScope() { t_kmarks = nullptr; }
};

static void marks_release(KMarks& m) {
  for (int i = 0; i < m.cap; ++i) (void)hipEventDestroy(m.ev[i]);
  free(m.ev);
  free(m.name);
  m = KMarks{};
}

// ------------------------------------------------------------- geometry --

static int make_geo(const jds_params* p, int64_t H, int64_t W, Geo* g, int* mode_out, bool* pf_out) {
  if (!p || !g) return fail(JDS_EINVAL, "null argument");
  // 8: the reference's path.  16: the configs[4] stretch (jds_b16.hip; table
  // np.kron(Q8, ones((2,2)))).  Anything else fails the way the reference's
  // quantizer does (engines/quantizer.py:24).
  if (p->block_size != 8 && p->block_size != 16)
    return fail(JDS_ENOTSUP, "operands could not be broadcast together with shapes (%d,%d) (8,8) ",
                p->block_size, p->block_size);
  const int B = p->block_size;
  if (p->subsampling < JDS_SS_444 || p->subsampling > JDS_SS_420)
    return fail(JDS_EINVAL, "Unknown subsampling mode: %d", p->subsampling);
  if (H < 1 || W < 1 || H > 65536 || W > 65536 || H * W > (int64_t)1 << 28)
    return fail(JDS_EINVAL, "unsupported image size %lldx%lld", (long long)H, (long long)W);
  const int mode = p->subsampling;
  const int sy = mode == JDS_SS_420 ? 2 : 1, sx = mode == JDS_SS_444 ? 1 : 2;
  // cv2.resize(c, (W // 2, H // sy), INTER_AREA) (engines/color_space.py:42-49)
  // asserts a non-empty destination
  if (H / sy < 1 || W / sx < 1)
    return fail(JDS_EINVAL,
                "OpenCV(4.8.0) resize.cpp: error: (-215:Assertion failed) !dsize.empty() in function 'resize' "
                "(image %lldx%lld, %s)",
                (long long)H, (long long)W, mode == JDS_SS_420 ? "4:2:0" : "4:2:2");
  // odd H (4:2:0) or odd W (4:2:x): cv2's fractional INTER_AREA and non-2x
  // INTER_LINEAR -> the general-geometry kernels (jds_gen.hip)
  const bool gen = (sy == 2 && (H % 2)) || (sx == 2 && (W % 2));
  if (gen && B == 16)
    return fail(JDS_ENOTSUP, "16x16 blocks with an odd %s image size (%lldx%lld) are not supported",
                mode == JDS_SS_420 ? "4:2:0" : "4:2:2", (long long)H, (long long)W);
  Geo& G = *g;
  memset(&G, 0, sizeof G);
  G.H = (int)H;
  G.W = (int)W;
  G.hc = (int)(H / sy);
  G.wc = (int)(W / sx);
  G.bs = B;
  G.gen = gen ? 1 : 0;
  if (gen) area_fast_scales((int)H, (int)(H / sy), (int)W, (int)(W / sx), &G.afy, &G.afx);
  G.nby = (int)((H + B - 1) / B);
  G.nbx = (int)((W + B - 1) / B);
  G.ncy = (G.hc + B - 1) / B;
  G.ncx = (G.wc + B - 1) / B;
  int MY, MX;
  if (B == 16) (void)tile_dims16(mode, &MY, &MX);
  else switch (mode) {
    case JDS_SS_420: MY = Cfg<M420>::MY; MX = Cfg<M420>::MX; break;
    case JDS_SS_422: MY = Cfg<M422>::MY; MX = Cfg<M422>::MX; break;
    default: MY = Cfg<M444>::MY; MX = Cfg<M444>::MX; break;
  }
  G.nmy = mode == JDS_SS_444 ? G.nby : G.ncy;
  G.nmx = mode == JDS_SS_444 ? G.nbx : G.ncx;
  G.tiles_y = (G.nmy + MY - 1) / MY;
  G.tiles_x = (G.nmx + MX - 1) / MX;
  G.ty_off = G.tiles_y * MY - G.nmy;
  G.tx_off = G.tiles_x * MX - G.nmx;
  const long long yb = (long long)G.nby * G.nbx, cb = (long long)G.ncy * G.ncx;
  G.cpf = (long long)B * B * (yb + 2 * cb);
  G.off_cb = (long long)B * B * yb;
  G.off_cr = (long long)B * B * (yb + cb);
  // cv2.resize: inv_scale = dst/src, scale = 1/inv_scale
  G.up_sy = 1.0 / ((double)H / (double)G.hc);
  G.up_sx = 1.0 / ((double)W / (double)G.wc);
  if (mode_out) *mode_out = mode;
  if (pf_out) *pf_out = mode != JDS_SS_444 && p->prefilter != 0;
  return JDS_OK;
}

static void fill_geometry(const Geo& G, int mode, jds_geometry* o) {
  o->H = G.H;
  o->W = G.W;
  o->chroma_h = G.hc;
  o->chroma_w = G.wc;
  o->y_blocks_y = G.nby;
  o->y_blocks_x = G.nbx;
  o->c_blocks_y = G.ncy;
  o->c_blocks_x = G.ncx;
  o->coeffs_per_frame = G.cpf;
  o->cb_offset = G.off_cb;
  o->cr_offset = G.off_cr;
  o->tiles = G.tiles_y * G.tiles_x;
  if (G.bs == 16) {
    int my, mx;
    o->threads_fwd = tile_dims16(mode, &my, &mx);
    o->threads_inv = 256;
  } else {
    o->threads_fwd = mode == JDS_SS_420 ? Cfg<M420>::TF : mode == JDS_SS_422 ? Cfg<M422>::TF : Cfg<M444>::TF;
    o->threads_inv = Cfg<M420>::TI;
  }
  o->reserved = 0;
}

static void make_fq(const jds_params* p, FrameQ* q) {
  q->qmax = 0.0;
  q->pad_ = 0.0;
  for (int i = 0; i < 64; ++i) {
    q->q[i] = p->qtable[i];
    q->q16[i] = 16.0 * p->qtable[i];  // exact
    q->qmax = q->qmax > p->qtable[i] ? q->qmax : p->qtable[i];
  }
}

// scale_quant_matrix (engines/quantizer.py:7-19) yields integers in [1, 255]
// (floor, then clip); the kernels rely on it (integer dequantisation).
static int check_tables(const jds_params* p) {
  for (int i = 0; i < 64; ++i) {
    if (!(p->qtable[i] >= 1.0 && p->qtable[i] <= 255.0))
      return fail(JDS_EINVAL, "qtable[%d] = %g outside [1, 255]", i, p->qtable[i]);
    if (p->qtable[i] != floor(p->qtable[i]))
      return fail(JDS_EINVAL, "qtable[%d] = %g is not an integer", i, p->qtable[i]);
  }
  return JDS_OK;
}

// Area tables (y then x) and plane scratch of the general-geometry path for
// n items of n_frames frames.
static int gen_prepare(const Geo& g, int n_frames, int n, DevBuf& tab, DevBuf& sub, DevBuf& rec, hipStream_t s) {
  const size_t nt = (size_t)g.hc + g.wc;
  AreaTap* h = (AreaTap*)malloc(sizeof(AreaTap) * nt);
  if (!h) return fail(JDS_ENOMEM, "host allocation failed");
  if (area_tab_build(g.H, g.hc, h) < 0 || area_tab_build(g.W, g.wc, h + g.hc) < 0) {
    free(h);
    return fail(JDS_EINVAL, "INTER_AREA table with more than 4 taps per sample (%dx%d)", g.H, g.W);
  }
  hipError_t e = tab.ensure(sizeof(AreaTap) * nt);
  if (e == hipSuccess) e = hipMemcpyAsync(tab.p, h, sizeof(AreaTap) * nt, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // h is freed below
  free(h);
  HIP_TRY(e);
  HIP_TRY(sub.ensure(sizeof(double) * gen_sub_doubles(g) * (size_t)n_frames));
  HIP_TRY(rec.ensure(sizeof(double) * gen_rec_doubles(g) * (size_t)n));
  return JDS_OK;
}

// ------------------------------------------------------------------ ABI --

extern "C" {

int jds_abi_version(void) { return JDS_ABI_VERSION; }

const char* jds_last_error(void) { return g_err; }

int jds_device_count(int* n) {
  if (!n) return fail(JDS_EINVAL, "null argument");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return fail(JDS_EHIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *n = c;
  return JDS_OK;
}

void* jds_ctx_stream(jds_ctx* c) { return c ? (void*)c->stream : nullptr; }

int jds_ctx_set_ssim_scratch(jds_ctx* c, int64_t bytes) {
  if (!c) return fail(JDS_EINVAL, "null argument");
  c->ss_budget = bytes > 0 ? (size_t)bytes : 0;
  return JDS_OK;
}

int jds_geometry_of(const jds_params* p, int64_t H, int64_t W, jds_geometry* out) {
  Geo g;
  int mode;
  int rc = make_geo(p, H, W, &g, &mode, nullptr);
  if (rc) return rc;
  if (!out) return fail(JDS_EINVAL, "null argument");
  fill_geometry(g, mode, out);
  return JDS_OK;
}

int jds_ctx_create(int device, jds_ctx** out) {
  if (!out) return fail(JDS_EINVAL, "null argument");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(JDS_EINVAL, "device %d out of range (%d devices)", device, n);
  HIP_TRY(hipSetDevice(device));
  jds_ctx* c = new (std::nothrow) jds_ctx();
  if (!c) return fail(JDS_ENOMEM, "host allocation failed");
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(JDS_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  for (int i = 0; i < 3; ++i) {
    if ((e = hipEventCreate(&c->ev[i])) != hipSuccess) {
      jds_ctx_destroy(c);
      return fail(JDS_EHIP, "hipEventCreate: %s", hipGetErrorString(e));
    }
  }
  *out = c;
  return JDS_OK;
}

void jds_ctx_destroy(jds_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->xfer) {
    (void)hipStreamSynchronize(c->xfer);
    (void)hipStreamDestroy(c->xfer);
  }
  if (c->xfer_ev) (void)hipEventDestroy(c->xfer_ev);
  if (c->ss_side) {
    (void)hipStreamSynchronize(c->ss_side);
    (void)hipStreamDestroy(c->ss_side);
  }
  if (c->ss_fork) (void)hipEventDestroy(c->ss_fork);
  if (c->ss_join) (void)hipEventDestroy(c->ss_join);
  if (c->ss_pairs_host) (void)hipHostFree(c->ss_pairs_host);
  c->ss_rgb.release();
  c->ss_pairs.release();
  DevBuf* bufs[] = {&c->rgb,     &c->out,    &c->coeffs,    &c->stats,  &c->part,  &c->fq,   &c->gk,  &c->erry,
                    &c->errrgb,  &c->sel,    &c->ss_planes, &c->ss_out, &c->img_a, &c->img_b};
  for (DevBuf* b : bufs) b->release();
  for (DevBuf& b : c->st) b.release();
  c->chunks.release();
  c->planes.release();
  for (DevBuf& b : c->ent) b.release();
  c->ent_hdr.release();
  c->ent_tab.release();
  c->ent_cf.release();
  c->ent_out.release();
  c->ent_meta.release();
  c->gen_tab.release();
  c->gen_sub.release();
  c->gen_rec.release();
  for (hipEvent_t e : c->ev)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

int jds_plan_create(jds_ctx* ctx, const jds_params* params, int n, int64_t H, int64_t W, jds_plan** out) {
  return jds_plan_create_q(ctx, params, n, 1, H, W, out);
}

int jds_plan_create_q(jds_ctx* ctx, const jds_params* params, int n_frames, int n_q, int64_t H, int64_t W,
                      jds_plan** out) {
  if (!ctx || !params || !out || n_frames < 1 || n_q < 1 || (long long)n_frames * n_q > (1 << 24))
    return fail(JDS_EINVAL, "bad argument");
  if (n_q > 1 && params[0].block_size != 8)
    return fail(JDS_ENOTSUP, "quality sweep plans (n_q > 1) need 8x8 blocks");
  if (n_q > MAXQ_SHARED) return fail(JDS_ENOTSUP, "at most %d tables per frame in a sweep plan", MAXQ_SHARED);
  const int n = n_frames * n_q;
  Geo g;
  int mode;
  bool pf;
  int rc = make_geo(params, H, W, &g, &mode, &pf);
  if (rc) return rc;
  FrameQ* hq = (FrameQ*)malloc(sizeof(FrameQ) * (size_t)n);
  if (!hq) return fail(JDS_ENOMEM, "host allocation failed");
  for (int i = 0; i < n; ++i) {
    if (params[i].subsampling != params[0].subsampling || params[i].block_size != params[0].block_size ||
        (params[i].prefilter != 0) != (params[0].prefilter != 0) ||
        (pf && memcmp(params[i].gauss, params[0].gauss, sizeof params[0].gauss) != 0)) {
      free(hq);
      return fail(JDS_EINVAL, "all frames of a plan must share subsampling / prefilter (taps) / block size");
    }
    if ((rc = check_tables(params + i))) {
      free(hq);
      return rc;
    }
    make_fq(params + i, hq + i);
  }
  HIP_TRY(hipSetDevice(ctx->device));
  jds_plan* p = new (std::nothrow) jds_plan();
  if (!p) {
    free(hq);
    return fail(JDS_ENOMEM, "host allocation failed");
  }
  p->ctx = ctx;
  p->n = n;
  p->nq = n_q;
  p->qt = (double*)malloc(sizeof(double) * 64 * (size_t)n);
  if (!p->qt) {
    free(hq);
    delete p;
    return fail(JDS_ENOMEM, "host allocation failed");
  }
  for (int i = 0; i < n; ++i) memcpy(p->qt + 64 * i, params[i].qtable, 64 * sizeof(double));
  // coarse tables (DC quantiser > 60, quality below ~14) put most tiles of a
  // frame on the certified inverse's fallback (reconstructions land on
  // integers: clipped luma, all-zero chroma), where k_inv2 is faster (16 x 4K
  // 4:2:0 Q10: 358 vs 410 us; an exact-value certificate variant, 425 us, did
  // not pay either -- DESIGN.md): such plans run k_inv2 unless JDS_RUN_INV_FAST
  p->inv_fast_ok = true;
  p->inv_fast_any = mode == JDS_SS_444;
  if (mode != JDS_SS_444)
    for (int i = 0; i < n; ++i) {
      p->inv_fast_ok = p->inv_fast_ok && params[i].qtable[0] <= 60.0;
      p->inv_fast_any = p->inv_fast_any || params[i].qtable[0] <= 60.0;
    }
  p->mode = mode;
  p->pf = pf;
  p->g = g;
  hipError_t e;
  if ((e = p->fq.ensure(sizeof(FrameQ) * n)) != hipSuccess || (e = p->gk.ensure(3 * sizeof(double))) != hipSuccess ||
      (e = p->part.ensure(sizeof(double) * (size_t)n *
                          (size_t)std::max(std::max(g.tiles_y * g.tiles_x, g.gen ? gen_px_tiles(g) : 0),
                                           g.bs == 16 ? inv16_tiles(mode, (int)H, (int)W) : 0))) !=
          hipSuccess ||
      (e = hipMemcpy(p->fq.p, hq, sizeof(FrameQ) * n, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(p->gk.p, params[0].gauss, 3 * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess) {
    free(hq);
    p->fq.release();
    p->gk.release();
    p->part.release();
    delete p;
    return fail(e == hipErrorOutOfMemory ? JDS_ENOMEM : JDS_EHIP, "plan upload: %s", hipGetErrorString(e));
  }
  free(hq);
  if (g.gen) {
    // general geometry: exact fp64 kernels over HBM planes (jds_gen.hip)
    if ((rc = gen_prepare(g, n_frames, n, p->gen_tab, p->gen_sub, p->gen_rec, ctx->stream))) {
      jds_plan_destroy(p);
      return rc;
    }
  } else if (g.bs == 16) {
    // 16x16 stretch path (jds_b16.hip, jds_fast16.hip): chroma planes scratch
    // (4:4:4 inverse), the certified forward's fp32 tables, fix-up list, counters
    const size_t fqs = fast_q16_size();
    char* h16 = (char*)malloc(fqs * (size_t)n);
    if (!h16) {
      jds_plan_destroy(p);
      return fail(JDS_ENOMEM, "host allocation failed");
    }
    for (int i = 0; i < n; ++i) fast_fwd16_thresholds(params[i].qtable, mode, pf, params[i].gauss, h16 + fqs * i);
    float gk32[5];  // taps + the combined taps of k_fwd16f's fast staging
    combined_taps32(params[0].gauss, gk32);
    const size_t nblk = (size_t)n * (size_t)(g.cpf / 256);
    if ((e = p->planes.ensure(mode == JDS_SS_444 ? sizeof(double) * 2 * (size_t)n * g.hc * g.wc : 8)) !=
            hipSuccess ||
        (e = p->fq32.ensure(fqs * n)) != hipSuccess || (e = p->gk32.ensure(sizeof gk32)) != hipSuccess ||
        (e = p->fixlist.ensure(8 * nblk)) != hipSuccess || (e = p->counters.ensure(64)) != hipSuccess ||
        (e = p->invfix.ensure(64 + 12 * (size_t)n)) != hipSuccess ||
        (e = hipMemset(p->invfix.p, 0, 64 + 12 * (size_t)n)) != hipSuccess ||
        (e = p->part32.ensure(sizeof(uint32_t) * 52 * (size_t)n * g.tiles_y * g.tiles_x)) != hipSuccess ||
        (e = hipMemcpy(p->fq32.p, h16, fqs * n, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->gk32.p, gk32, sizeof gk32, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(p->counters.p, 0, 64)) != hipSuccess) {
      free(h16);
      jds_plan_destroy(p);
      return fail(e == hipErrorOutOfMemory ? JDS_ENOMEM : JDS_EHIP, "plan upload: %s", hipGetErrorString(e));
    }
    free(h16);
  } else {
    const size_t fqs = fast_q_size();
    char* h32 = (char*)malloc(fqs * (size_t)n);
    if (!h32) {
      jds_plan_destroy(p);
      return fail(JDS_ENOMEM, "host allocation failed");
    }
    for (int i = 0; i < n; ++i) {
      float* f = (float*)(h32 + fqs * i);
      fast_fwd_thresholds(params[i].qtable, mode, pf, params[i].gauss, f, f + 64);
    }
    // taps and k_fwd32i's combined taps (Gaussian then 2-sample area: k0, k0+k1, k1+k2, k2)
    const double* gs = params[0].gauss;
    float gk32[5];
    combined_taps32(gs, gk32);
    const size_t nblk = (size_t)n * (size_t)(g.cpf / 64);
    const size_t ptiles = (size_t)(n_q > 1 ? quant_mq_tiles(g) : g.tiles_y * g.tiles_x);
    if ((e = p->fq32.ensure(fqs * n)) != hipSuccess || (e = p->gk32.ensure(sizeof gk32)) != hipSuccess ||
        (e = p->fixbits.ensure(4 * (size_t)n * (size_t)fix_wpi(g))) != hipSuccess ||
        (e = p->fixlist.ensure(8 * nblk)) != hipSuccess ||
        (e = p->counters.ensure(8 * (size_t)n + 64)) != hipSuccess ||
        (e = p->part32.ensure(sizeof(uint32_t) * (n_q > 1 ? 52 * (size_t)n * ptiles
                                                          : std::max((size_t)52 * n * ptiles, fast_part_words(g, n))))) !=
            hipSuccess ||
        (e = hipMemset(p->part32.p, 0, p->part32.n)) != hipSuccess ||
        (e = p->invfix.ensure(64 + 12 * (size_t)n)) != hipSuccess ||
        (e = hipMemset(p->invfix.p, 0, 64 + 12 * (size_t)n)) != hipSuccess ||
        (JDS_INV6_LIST && mode == JDS_SS_420 && (e = p->invlist.ensure(8 * (size_t)n * inv_tiles(mode, (int)H, (int)W))) != hipSuccess) ||
        (n_q > 1 && (e = p->dct32.ensure(sizeof(float) * (size_t)n_frames * g.cpf)) != hipSuccess) ||
        (e = hipMemcpy(p->fq32.p, h32, fqs * n, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->gk32.p, gk32, sizeof gk32, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(p->counters.p, 0, 8 * (size_t)n + 64)) != hipSuccess ||
        (e = hipMemset(p->fixbits.p, 0, 4 * (size_t)n * (size_t)fix_wpi(g))) != hipSuccess) {
      // the fix-up bitmaps start clean once; k_fix_compact clears the words it consumes
      free(h32);
      jds_plan_destroy(p);
      return fail(e == hipErrorOutOfMemory ? JDS_ENOMEM : JDS_EHIP, "plan upload: %s", hipGetErrorString(e));
    }
    free(h32);
    if (p->inv_fast_any && !p->inv_fast_ok) {
      // mixed tables: the coarse items start in the certified inverse's exact
      // mode (every rotation slot of their "tiles recomputed last run" counter
      // holds all of their tiles); the probe run every 16th re-measures them
      std::vector<unsigned> seed(3 * (size_t)n, 0u);
      const unsigned nt = (unsigned)inv_tiles(mode, (int)H, (int)W);
      for (int i = 0; i < n; ++i)
        if (params[i].qtable[0] > 60.0) seed[i] = seed[n + i] = seed[2 * (size_t)n + i] = nt;
      if ((e = hipMemcpy((unsigned*)p->invfix.p + 16, seed.data(), sizeof(unsigned) * seed.size(),
                         hipMemcpyHostToDevice)) != hipSuccess) {
        jds_plan_destroy(p);
        return fail(JDS_EHIP, "plan upload: %s", hipGetErrorString(e));
      }
    }
  }
  *out = p;
  return JDS_OK;
}

int jds_plan_fix_counts(const jds_plan* p, uint32_t* counts) {
  if (!p || !counts) return fail(JDS_EINVAL, "null argument");
  // counters[bank n, bank n + n): blocks the last run's k_fix_fwd recomputed, per item;
  // invfix[0]: tiles the last run's certified inverse handed to the exact kernel
  counts[0] = counts[1] = 0u;
  if (p->g.bs == 16) {  // counters[2]: blocks the last certified 16x16 forward recomputed
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess && p->last_fwd16_fast)
      e = hipMemcpy(counts, (const uint32_t*)p->counters.p + 2, 4, hipMemcpyDeviceToHost);
    // and the tiles the last k_inv16_fast run handed to the exact tile body
    if (e == hipSuccess && p->last_inv_fast)
      e = hipMemcpy(counts + 1, (const uint32_t*)p->invfix.p + ((p->inv_runs + 1u) & 1u), 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(JDS_EHIP, "fix_counts: %s", hipGetErrorString(e));
    return JDS_OK;
  }
  if (p->g.gen || p->counters.n < 8 * (size_t)p->n) return JDS_OK;
  uint32_t* c = (uint32_t*)malloc(4 * (size_t)p->n + 4);
  if (!c) return fail(JDS_ENOMEM, "fix_counts: host allocation");
  // the last run may be in flight on any stream: wait for the device first
  hipError_t e = hipDeviceSynchronize();
  // single-quality plans: the live counter bank of the last certified run;
  // sweep plans: the list lengths k_fwd_reduce_fix built at [n, 2n)
  const int bank = p->nq > 1 ? 1 : (p->last_fwd8_bank < 0 ? 1 : p->last_fwd8_bank);
  if (e == hipSuccess)
    e = hipMemcpy(c, (const uint32_t*)p->counters.p + bank * p->n, 4 * (size_t)p->n, hipMemcpyDeviceToHost);
  // the last fast-inverse run appended to counter (inv_runs - 1) & 1
  if (e == hipSuccess && p->last_inv_fast)
    e = hipMemcpy(c + p->n, (const uint32_t*)p->invfix.p + ((p->inv_runs + 1u) & 1u), 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    free(c);
    return fail(JDS_EHIP, "fix_counts: %s", hipGetErrorString(e));
  }
  for (int i = 0; i < p->n; ++i) counts[0] += std::min(c[i], (uint32_t)(p->g.cpf / 64));  // (k_fix_fwd's clamp)
  counts[1] = p->last_inv_fast ? c[p->n] : 0u;
  free(c);
  return JDS_OK;
}

int jds_plan_geometry(const jds_plan* p, jds_geometry* out) {
  if (!p || !out) return fail(JDS_EINVAL, "null argument");
  fill_geometry(p->g, p->mode, out);
  return JDS_OK;
}

int jds_plan_run(jds_plan* p, const uint8_t* rgb, uint8_t* rgb_out, int16_t* coeffs, jds_frame_stats* stats,
                 uint32_t flags, void* stream) {
  if (!p || !rgb || !rgb_out || !coeffs || !stats) return fail(JDS_EINVAL, "null argument");
  if (((uintptr_t)rgb | (uintptr_t)rgb_out | (uintptr_t)coeffs | (uintptr_t)stats) & 15u)
    return fail(JDS_EINVAL, "rgb, rgb_out, coeffs and stats must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream (torch's default stream)
  const MarkScope marks_(p, s);         // jds_plan_profile: launch marks of this run
  int phases = (flags & JDS_RUN_FWD ? 1 : 0) | (flags & JDS_RUN_INV ? 2 : 0);
  if (!phases) phases = 3;
  const bool exact = (flags & JDS_RUN_EXACT) != 0;
  if (p->g.gen) {  // general geometry: exact kernels only (jds_gen.hip)
    if (phases & 1) HIP_TRY(hipMemsetAsync(stats, 0, sizeof(jds_frame_stats) * p->n, s));
    const GenBufs gb = p->gen();
    HIP_TRY(launch_codec(p->mode, p->pf, p->g, p->n, rgb, rgb_out, coeffs, (const FrameQ*)p->fq.p,
                         (const double*)p->gk.p, stats, (double*)p->part.p, (flags & JDS_RUN_SSE) != 0, nullptr,
                         nullptr, nullptr, 0, s, nullptr, phases, p->nq, &gb));
    return JDS_OK;
  }
  if (p->g.bs == 16) {
    // the certified fp32 forward unless JDS_RUN_EXACT (k_fix_fwd16 re-arms its counters)
    const Fwd16Fast ff{p->fq32.p, (const float*)p->gk32.p, (uint32_t*)p->part32.p, (uint2*)p->fixlist.p,
                       (unsigned*)p->counters.p,
                       (flags & JDS_RUN_FWD_FIXALL) ? 1 : 0, (int)(p->fwd16_runs & 1u)};
    if (phases & 1) HIP_TRY(hipMemsetAsync(stats, 0, sizeof(jds_frame_stats) * p->n, s));
    // the certified fast inverse (k_inv16_fast) for 4:2:x runs without SSE
    // terms unless JDS_RUN_EXACT_INV: level with the exact k_inv16s in round 3
    // (524-526 vs 520-522 us at configs[4]), 511 vs 522 us once its certificate
    // reduction went to DPP and its max Q to the host (profiles/r03_v29_ab.txt)
    InvFix fx16 = p->inv_fix();
    fx16.fix_all = (flags & JDS_RUN_INV_FIXALL) ? 1 : 0;
    const bool fast_inv16 = (phases & 2) && !exact && !(flags & JDS_RUN_EXACT_INV) &&
                            !(flags & JDS_RUN_SSE) && p->mode != JDS_SS_444 && p->invfix.p;
    HIP_TRY(launch_codec16(p->mode, p->pf, p->g, p->n, rgb, rgb_out, coeffs, (const FrameQ*)p->fq.p,
                           (const double*)p->gk.p, stats, (double*)p->part.p, (double*)p->planes.p,
                           (flags & JDS_RUN_SSE) != 0, nullptr, nullptr, s, nullptr, phases, exact ? nullptr : &ff,
                           fast_inv16 ? &fx16 : nullptr));
    if (phases & 1) {
      p->last_fwd16_fast = !exact;
      if (!exact) p->fwd16_runs++;
    }
    if (phases & 2) {
      p->last_inv_fast = fast_inv16;
      if (fast_inv16) p->inv_runs++;
    }
    return JDS_OK;
  }
  if (phases & 1) {
    // the fast forward resets the statistics in its front-end launch and
    // re-arms the fix-up counter in k_fwd_reduce (no memsets on its path)
    if (exact) HIP_TRY(hipMemsetAsync(stats, 0, sizeof(jds_frame_stats) * p->n, s));
    if (exact)
      HIP_TRY(launch_codec(p->mode, p->pf, p->g, p->n, rgb, rgb_out, coeffs, (const FrameQ*)p->fq.p,
                           (const double*)p->gk.p, stats, (double*)p->part.p, false, nullptr, nullptr, nullptr, 0,
                           s, nullptr, 1, p->nq, nullptr));
    else
      HIP_TRY(launch_fast_fwd(p->mode, p->pf, p->g, p->n, p->nq, rgb, coeffs, (const FrameQ*)p->fq.p, p->fq32.p,
                              (const double*)p->gk.p, (const float*)p->gk32.p, stats, (uint32_t*)p->part32.p,
                              (uint32_t*)p->fixbits.p, (uint2*)p->fixlist.p, (unsigned*)p->counters.p,
                              (float*)p->dct32.p, s,
                              phases == 1,  // forward + inverse: k_finalize adds the zero bin
                              (int)(p->fwd8_runs & 1u)));
    if (!exact && p->nq == 1) p->last_fwd8_bank = (int)(p->fwd8_runs++ & 1u);
  }
  InvFix fx = p->inv_fix();
  fx.fix_all = (flags & JDS_RUN_INV_FIXALL) ? 1 : 0;
  const bool exact_inv = exact || (flags & JDS_RUN_EXACT_INV) != 0 || (!p->inv_fast_any && !(flags & JDS_RUN_INV_FAST));
  if (phases & 2)
    HIP_TRY(launch_codec(p->mode, p->pf, p->g, p->n, rgb, rgb_out, coeffs, (const FrameQ*)p->fq.p,
                         (const double*)p->gk.p, stats, (double*)p->part.p, (flags & JDS_RUN_SSE) != 0, nullptr,
                         nullptr, nullptr, 0, s, nullptr, exact ? 6 : (phases == 3 ? 2 | 8 : 2), p->nq, nullptr,
                         exact_inv || !p->invfix.p ? nullptr : &fx));
  if (phases & 2) {
    p->last_inv_fast = !exact_inv && p->invfix.p;
    if (p->last_inv_fast) p->inv_runs++;
  }
  return JDS_OK;
}

int jds_plan_profile(jds_plan* p, int enable) {
  if (!p) return fail(JDS_EINVAL, "null argument");
  if (enable && !p->marks.cap) {
    HIP_TRY(hipSetDevice(p->ctx->device));
    const int cap = 8192;  // marks until the next read: ~7 per run
    KMarks m;
    m.ev = (hipEvent_t*)calloc(cap, sizeof(hipEvent_t));
    m.name = (char(*)[64])calloc(cap, sizeof *m.name);
    if (!m.ev || !m.name) {
      free(m.ev);
      free(m.name);
      return fail(JDS_ENOMEM, "host allocation failed");
    }
    for (; m.cap < cap; ++m.cap) {
      // timing-only marks: no system-scope fence (cache write-back and
      // invalidate) per mark, which otherwise lands inside the next launch's
      // interval and perturbs the profiled step (r06: +5 % over the timed one)
      hipError_t e = hipEventCreateWithFlags(&m.ev[m.cap], hipEventDisableSystemFence);
      if (e != hipSuccess) {
        marks_release(m);
        return fail(JDS_EHIP, "hipEventCreate: %s", hipGetErrorString(e));
      }
    }
    p->marks = m;
  }
  p->prof_on = enable != 0;
  p->marks.n = 0;
  p->marks.dropped = 0;
  return JDS_OK;
}

int jds_plan_profile_read(jds_plan* p, jds_kernel_time* out, int max, int* n_out, double* span_ms) {
  if (!p || !n_out || (max > 0 && !out)) return fail(JDS_EINVAL, "null argument");
  KMarks& m = p->marks;
  *n_out = 0;
  if (span_ms) *span_ms = 0.0;
  if (m.dropped) {  // the pool filled up: partial totals would under-report, so none are returned
    const long long d = m.dropped;
    if (m.n) (void)hipEventSynchronize(m.ev[m.n - 1]);
    m.n = 0;
    m.dropped = 0;
    return fail(JDS_EINVAL, "profile overflow: %lld launch marks dropped (pool of %d); read every <= %d runs",
                d, m.cap, m.cap / 8);
  }
  if (m.n < 2) {
    m.n = 0;
    return JDS_OK;
  }
  HIP_TRY(hipSetDevice(p->ctx->device));
  HIP_TRY(hipEventSynchronize(m.ev[m.n - 1]));
  int k = 0;
  for (int i = 1; i < m.n; ++i) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, m.ev[i - 1], m.ev[i]));
    int j = 0;
    while (j < k && strncmp(out[j].name, m.name[i], sizeof out[j].name) != 0) ++j;
    if (j == k) {
      if (k == max) continue;  // more distinct names than the caller's array holds
      memset(&out[k], 0, sizeof out[k]);
      snprintf(out[k].name, sizeof out[k].name, "%s", m.name[i]);
      ++k;
    }
    out[j].total_ms += ms;
    out[j].launches += 1;
  }
  if (span_ms) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, m.ev[0], m.ev[m.n - 1]));
    *span_ms = ms;
  }
  *n_out = k;
  m.n = 0;
  return JDS_OK;
}

void jds_plan_destroy(jds_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  (void)hipStreamSynchronize(p->ctx->stream);
  p->fq.release();
  p->gk.release();
  p->part.release();
  p->fq32.release();
  p->gk32.release();
  p->fixlist.release();
  p->counters.release();
  p->fixbits.release();
  p->part32.release();
  p->invfix.release();
  p->invlist.release();
  p->planes.release();
  p->dct32.release();
  p->gen_tab.release();
  p->gen_sub.release();
  p->gen_rec.release();
  for (DevBuf& b : p->ent) b.release();
  p->ent_hdr.release();
  p->ent_tab.release();
  free(p->qt);
  marks_release(p->marks);
  delete p;
}

int jds_compress_reconstruct(jds_ctx* c, const jds_params* prm, const uint8_t* rgb, int64_t H, int64_t W,
                             uint8_t* rgb_out, int16_t* coeffs, jds_frame_stats* stats, double* error_map_y,
                             double* error_map_rgb, int32_t sel_by, int32_t sel_bx, jds_selected_block* sel,
                             int32_t* sel_valid) {
  if (!c || !prm || !rgb || !rgb_out || !stats) return fail(JDS_EINVAL, "null argument");
  if ((error_map_y == nullptr) != (error_map_rgb == nullptr))
    return fail(JDS_EINVAL, "error_map_y and error_map_rgb must be requested together");
  Geo g;
  int mode;
  bool pf;
  int rc = make_geo(prm, H, W, &g, &mode, &pf);
  if (rc) return rc;
  if ((rc = check_tables(prm))) return rc;
  HIP_TRY(hipSetDevice(c->device));
  const size_t npx = (size_t)H * (size_t)W, nimg = npx * 3, ncf = (size_t)g.cpf;
  const int tiles = std::max(std::max(g.tiles_y * g.tiles_x, g.gen ? gen_px_tiles(g) : 0),
                             g.bs == 16 ? inv16_tiles(mode, (int)H, (int)W) : 0);
  HIP_TRY(c->rgb.ensure(nimg));
  HIP_TRY(c->out.ensure(nimg));
  HIP_TRY(c->coeffs.ensure(ncf * sizeof(int16_t)));
  HIP_TRY(c->stats.ensure(sizeof(jds_frame_stats)));
  HIP_TRY(c->part.ensure(sizeof(double) * tiles));
  HIP_TRY(c->fq.ensure(sizeof(FrameQ)));
  HIP_TRY(c->gk.ensure(3 * sizeof(double)));
  const bool maps = error_map_y != nullptr;
  if (maps) {
    HIP_TRY(c->erry.ensure(npx * sizeof(double)));
    HIP_TRY(c->errrgb.ensure(npx * sizeof(double)));
  }
  // selected luma block (pipeline.py:132-138): index into the padded grid
  // (8x8 only: jds_selected_block holds 8x8 arrays; the 16x16 path reports none)
  int sel_blk = -1;
  if (sel && g.bs == 16) {
    if (sel_valid) *sel_valid = 0;
  } else if (sel) {
    const long long bpr = g.nbx;
    const long long ti = (long long)sel_by * bpr + sel_bx;
    const long long nyb = (long long)g.nby * g.nbx;
    if (ti >= 0 && ti < nyb) sel_blk = (int)ti;
    if (sel_valid) *sel_valid = sel_blk >= 0;
    if (sel_blk >= 0) HIP_TRY(c->sel.ensure(sizeof(jds_selected_block)));
  }
  FrameQ hq;
  make_fq(prm, &hq);
  hipStream_t s = c->stream;
  GenBufs gb{};
  if (g.gen) {
    if ((rc = gen_prepare(g, 1, 1, c->gen_tab, c->gen_sub, c->gen_rec, s))) return rc;
    gb = {(const AreaTap*)c->gen_tab.p, (double*)c->gen_sub.p, (double*)c->gen_rec.p};
  }
  HIP_TRY(hipMemcpyAsync(c->fq.p, &hq, sizeof hq, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->gk.p, prm->gauss, 3 * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(c->rgb.p, rgb, nimg, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemsetAsync(c->stats.p, 0, sizeof(jds_frame_stats), s));
  jds_selected_block* dsel = sel_blk >= 0 ? (jds_selected_block*)c->sel.p : nullptr;
  if (g.bs == 16) {
    HIP_TRY(c->planes.ensure(sizeof(double) * 2 * (size_t)g.hc * g.wc));
    HIP_TRY(launch_codec16(mode, pf, g, 1, (const uint8_t*)c->rgb.p, (uint8_t*)c->out.p, (int16_t*)c->coeffs.p,
                           (const FrameQ*)c->fq.p, (const double*)c->gk.p, (jds_frame_stats*)c->stats.p,
                           (double*)c->part.p, (double*)c->planes.p, true, maps ? (double*)c->erry.p : nullptr,
                           maps ? (double*)c->errrgb.p : nullptr, s, c->ev, 3, nullptr, nullptr));
  } else
  HIP_TRY(launch_codec(mode, pf, g, 1, (const uint8_t*)c->rgb.p, (uint8_t*)c->out.p, (int16_t*)c->coeffs.p,
                       (const FrameQ*)c->fq.p, (const double*)c->gk.p, (jds_frame_stats*)c->stats.p,
                       (double*)c->part.p, true, maps ? (double*)c->erry.p : nullptr,
                       maps ? (double*)c->errrgb.p : nullptr, dsel, sel_blk, s, c->ev, 3, 1, &gb));
  // the outputs are final here: their copies to the caller's (pageable) arrays
  // go on the transfer stream, so the statistics kernels queued below on `s`
  // run while the host thread stages the copies
  if (!c->xfer) {
    HIP_TRY(hipStreamCreateWithFlags(&c->xfer, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c->xfer_ev, hipEventDisableTiming));
  }
  HIP_TRY(hipEventRecord(c->xfer_ev, s));
  HIP_TRY(hipStreamWaitEvent(c->xfer, c->xfer_ev, 0));
  {
    // NumPy float32 magnitude_bits (utils/metrics.py:77-78)
    const long long nblk = g.cpf / 64;
    const int max_chunks = (int)((g.cpf + 8191) / 8192) + 1;
    HIP_TRY(c->chunks.ensure(mag_scratch_bytes(nblk, max_chunks)));
    HIP_TRY(launch_mag_f32((const int16_t*)c->coeffs.p, nblk, (unsigned*)c->chunks.p, max_chunks,
                           &((jds_frame_stats*)c->stats.p)->magnitude_bits_f32, s));
  }
  if (H >= 7 && W >= 7) {
    jds_frame_stats* dst = (jds_frame_stats*)c->stats.p;
    if ((rc = run_ssim(c, (const uint8_t*)c->rgb.p, (const uint8_t*)c->out.p, (int)H, (int)W, &dst->ssim[0])))
      return rc;
  }
  hipStream_t x = c->xfer;
  // every exit from here on waits for the copies queued on x: an error return
  // must not leave copies into the caller's arrays in flight
  struct XferWait {
    hipStream_t x;
    ~XferWait() { (void)hipStreamSynchronize(x); }
  } xfer_wait{x};
  HIP_TRY(hipMemcpyAsync(rgb_out, c->out.p, nimg, hipMemcpyDeviceToHost, x));
  if (coeffs) HIP_TRY(hipMemcpyAsync(coeffs, c->coeffs.p, ncf * sizeof(int16_t), hipMemcpyDeviceToHost, x));
  if (maps) {
    HIP_TRY(hipMemcpyAsync(error_map_y, c->erry.p, npx * sizeof(double), hipMemcpyDeviceToHost, x));
    HIP_TRY(hipMemcpyAsync(error_map_rgb, c->errrgb.p, npx * sizeof(double), hipMemcpyDeviceToHost, x));
  }
  if (dsel) HIP_TRY(hipMemcpyAsync(sel, dsel, sizeof(jds_selected_block), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(stats, c->stats.p, sizeof(jds_frame_stats), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(x));
  HIP_TRY(hipStreamSynchronize(s));
  if (!(H >= 7 && W >= 7)) {
    for (int i = 0; i < 4; ++i) stats->ssim[i] = __builtin_nan("");
    stats->mse_y = __builtin_nan("");
  }
  float t0 = 0.f, t1 = 0.f;
  HIP_TRY(hipEventElapsedTime(&t0, c->ev[0], c->ev[1]));
  HIP_TRY(hipEventElapsedTime(&t1, c->ev[1], c->ev[2]));
  stats->fwd_ms = t0;
  stats->inv_ms = t1;
  return JDS_OK;
}

// jds_psnr_ssim / jds_psnr_ssim_dev: argument checks shared by both
static int psnr_ssim_args(jds_ctx* c, const uint8_t* a, const uint8_t* b, int64_t H, int64_t W, double* out) {
  if (!c || !a || !b || !out) return fail(JDS_EINVAL, "null argument");
  if (H < 7 || W < 7)
    return fail(JDS_EINVAL,
                "win_size exceeds image extent. Either ensure that your images are at least 7x7; or pass "
                "win_size explicitly in the function call, with an odd value less than or equal to the "
                "smaller side of your images. If your images are multichannel (with color channels), set "
                "channel_axis to the axis number corresponding to the channels.");
  if (H * W > (int64_t)1 << 28) return fail(JDS_EINVAL, "image too large");
  return JDS_OK;
}

// SSIM / MSE of `items` device-resident image pairs (the context's stream):
// out[6 i + 0..5] = SSIM R, G, B, Y, MSE Y, MSE RGB on the host
static int psnr_ssim_device_batch(jds_ctx* c, int items, const uint8_t* const* a, const uint8_t* const* b,
                                  int64_t H, int64_t W, double* out) {
  const size_t nb = (size_t)H * W * 3;
  const size_t bytes = (size_t)items * (5 * sizeof(double) + sizeof(unsigned long long));
  HIP_TRY(c->ss_out.ensure(bytes));
  hipStream_t s = c->stream;
  double* dres = (double*)c->ss_out.p;
  unsigned long long* dsse = (unsigned long long*)(dres + (size_t)5 * items);
  int rc = run_ssim_batch(c, items, a, b, (int)H, (int)W, dres, 5, dsse);
  if (rc) return rc;
  double* res = (double*)malloc(bytes);
  if (!res) return fail(JDS_ENOMEM, "host allocation failed");
  hipError_t e = hipMemcpyAsync(res, dres, bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    free(res);
    return fail(JDS_EHIP, "HIP error: %s", hipGetErrorString(e));
  }
  const unsigned long long* sse = (const unsigned long long*)(res + (size_t)5 * items);
  for (int i = 0; i < items; ++i) {
    for (int k = 0; k < 5; ++k) out[6 * i + k] = res[5 * i + k];
    out[6 * i + 5] = (double)sse[i] / (double)nb;  // exact: integer sum, one division (np.mean)
  }
  free(res);
  return JDS_OK;
}

static int psnr_ssim_device(jds_ctx* c, const uint8_t* a, const uint8_t* b, int64_t H, int64_t W, double* out) {
  return psnr_ssim_device_batch(c, 1, &a, &b, H, W, out);
}

int jds_psnr_ssim(jds_ctx* c, const uint8_t* a, const uint8_t* b, int64_t H, int64_t W, double* out) {
  int rc = psnr_ssim_args(c, a, b, H, W, out);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  const size_t nb = (size_t)H * W * 3;
  HIP_TRY(c->img_a.ensure(nb));
  HIP_TRY(c->img_b.ensure(nb));
  HIP_TRY(hipMemcpyAsync(c->img_a.p, a, nb, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->img_b.p, b, nb, hipMemcpyHostToDevice, c->stream));
  return psnr_ssim_device(c, (const uint8_t*)c->img_a.p, (const uint8_t*)c->img_b.p, H, W, out);
}

int jds_psnr_ssim_dev(jds_ctx* c, const uint8_t* a_dev, const uint8_t* b_dev, int64_t H, int64_t W, double* out) {
  int rc = psnr_ssim_args(c, a_dev, b_dev, H, W, out);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // the images come from other streams (plan runs, torch)
  return psnr_ssim_device(c, a_dev, b_dev, H, W, out);
}

// the context's stream waits for what `after` has queued so far (one event);
// JDS_AFTER_NONE: no wait (the caller has synchronised); NULL: the HIP null stream
static int wait_after(jds_ctx* c, void* after) {
  if (after == JDS_AFTER_NONE) return JDS_OK;
  hipEvent_t e;
  HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  hipError_t err = hipEventRecord(e, (hipStream_t)after);
  if (err == hipSuccess) err = hipStreamWaitEvent(c->stream, e, 0);
  hipError_t d = hipEventDestroy(e);  // released once the wait has completed
  if (err != hipSuccess) return fail(JDS_EHIP, "HIP error: %s", hipGetErrorString(err));
  if (d != hipSuccess) return fail(JDS_EHIP, "HIP error: %s", hipGetErrorString(d));
  return JDS_OK;
}

int jds_psnr_ssim_dev_after(jds_ctx* c, const uint8_t* a_dev, const uint8_t* b_dev, int64_t H, int64_t W,
                            double* out, void* after) {
  int rc = psnr_ssim_args(c, a_dev, b_dev, H, W, out);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  if ((rc = wait_after(c, after))) return rc;
  return psnr_ssim_device(c, a_dev, b_dev, H, W, out);
}

int jds_psnr_ssim_batch_dev(jds_ctx* c, int32_t n, const uint8_t* const* a_dev, const uint8_t* const* b_dev, int64_t H,
                            int64_t W, double* out, void* after) {
  if (!c || n < 0 || (n > 0 && (!a_dev || !b_dev || !out))) return fail(JDS_EINVAL, "null argument");
  if (n == 0) return JDS_OK;
  for (int i = 0; i < n; ++i) {
    int rc = psnr_ssim_args(c, a_dev[i], b_dev[i], H, W, out);
    if (rc) return rc;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc = wait_after(c, after);
  if (rc) return rc;
  return psnr_ssim_device_batch(c, n, a_dev, b_dev, H, W, out);
}

int jds_magnitude_bits_f32_batch_dev(jds_ctx* c, const int16_t* coeffs_dev, int32_t n_items, int64_t n_coeffs,
                                     int64_t item_stride, double* out, void* after) {
  if (!c || n_items < 0 || (n_items > 0 && (!coeffs_dev || !out)) || n_coeffs < 0 || n_coeffs % 64 ||
      item_stride < n_coeffs)
    return fail(JDS_EINVAL, "bad argument");
  if (n_coeffs > ((int64_t)1 << 31)) return fail(JDS_EINVAL, "too many coefficients");
  if (n_items == 0) return JDS_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc = wait_after(c, after);
  if (rc) return rc;
  hipStream_t s = c->stream;
  const long long nblk = n_coeffs / 64;
  const int max_chunks = (int)((n_coeffs + 8191) / 8192) + 1;
  HIP_TRY(c->chunks.ensure(mag_scratch_bytes(nblk, max_chunks)));
  HIP_TRY(c->ss_out.ensure(sizeof(double) * (size_t)n_items));
  double* d = (double*)c->ss_out.p;
  // one launch chain per item on the stream (the scratch is reused in order), one copy, one wait
  for (int i = 0; i < n_items; ++i)
    HIP_TRY(launch_mag_f32(coeffs_dev + (size_t)i * item_stride, nblk, (unsigned*)c->chunks.p, max_chunks, d + i, s));
  HIP_TRY(hipMemcpyAsync(out, d, sizeof(double) * (size_t)n_items, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return JDS_OK;
}

int jds_magnitude_bits_f32_dev(jds_ctx* c, const int16_t* coeffs_dev, int64_t n_coeffs, double* out, void* after) {
  if (!c || !coeffs_dev || !out || n_coeffs < 0 || n_coeffs % 64) return fail(JDS_EINVAL, "bad argument");
  if (n_coeffs > ((int64_t)1 << 31)) return fail(JDS_EINVAL, "too many coefficients");
  HIP_TRY(hipSetDevice(c->device));
  int rc = wait_after(c, after);
  if (rc) return rc;
  hipStream_t s = c->stream;
  const long long nblk = n_coeffs / 64;
  const int max_chunks = (int)((n_coeffs + 8191) / 8192) + 1;
  HIP_TRY(c->chunks.ensure(mag_scratch_bytes(nblk, max_chunks)));
  HIP_TRY(c->ss_out.ensure(5 * sizeof(double) + sizeof(unsigned long long)));
  double* d = (double*)c->ss_out.p;
  HIP_TRY(launch_mag_f32(coeffs_dev, nblk, (unsigned*)c->chunks.p, max_chunks, d, s));
  HIP_TRY(hipMemcpyAsync(out, d, sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return JDS_OK;
}

// ----------------------------------------------------- per-stage API --

static int stage_io(jds_ctx* c, int idx, const void* host, size_t bytes, void** dev) {
  HIP_TRY(c->st[idx].ensure(bytes));
  if (host) HIP_TRY(hipMemcpyAsync(c->st[idx].p, host, bytes, hipMemcpyHostToDevice, c->stream));
  *dev = c->st[idx].p;
  return JDS_OK;
}

static int stage_out(jds_ctx* c, void* host, const void* dev, size_t bytes) {
  HIP_TRY(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return JDS_OK;
}

static int stage_rgb(jds_ctx* c, const double* in, double* out, int64_t n, int inverse) {
  if (!c || !in || !out || n < 0) return fail(JDS_EINVAL, "bad argument");
  if (n == 0) return JDS_OK;
  HIP_TRY(hipSetDevice(c->device));
  void *di, *dout;
  int rc;
  const size_t b = (size_t)n * 3 * sizeof(double);
  if ((rc = stage_io(c, 0, in, b, &di)) || (rc = stage_io(c, 1, nullptr, b, &dout))) return rc;
  HIP_TRY(stage_rgb_ycc((const double*)di, (double*)dout, n, inverse, c->stream));
  return stage_out(c, out, dout, b);
}

int jds_stage_rgb_to_ycbcr(jds_ctx* c, const double* rgb, double* ycc, int64_t n_pixels) {
  return stage_rgb(c, rgb, ycc, n_pixels, 0);
}

int jds_stage_ycbcr_to_rgb(jds_ctx* c, const double* ycc, double* rgb, int64_t n_pixels) {
  return stage_rgb(c, ycc, rgb, n_pixels, 1);
}

int jds_stage_subsample(jds_ctx* c, const double* cb, const double* cr, int64_t H, int64_t W, int32_t mode,
                        int32_t prefilter, const double* gauss, double* cb_out, double* cr_out) {
  if (!c || !cb || !cr || !cb_out || !cr_out || !gauss || H < 1 || W < 1) return fail(JDS_EINVAL, "bad argument");
  if (mode != JDS_SS_422 && mode != JDS_SS_420) return fail(JDS_EINVAL, "Unknown subsampling mode: %d", mode);
  const int sy = mode == JDS_SS_420 ? 2 : 1;
  const int oh = (int)(H / sy), ow = (int)(W / 2);
  if (oh < 1 || ow < 1)
    return fail(JDS_EINVAL,
                "OpenCV(4.8.0) resize.cpp: error: (-215:Assertion failed) !dsize.empty() in function 'resize'");
  // odd sizes take cv2's fractional INTER_AREA path (tables as in jds_gen.hip)
  const bool gen = (W % 2) || (sy == 2 && (H % 2));
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)H * W, bi = n * sizeof(double), bo = (size_t)oh * ow * sizeof(double);
  void *din, *t1, *t2, *dout;
  int rc;
  if ((rc = stage_io(c, 1, nullptr, bi, &t1)) || (rc = stage_io(c, 2, nullptr, bi, &t2)) ||
      (rc = stage_io(c, 3, nullptr, bo, &dout)))
    return rc;
  if (gen) {
    Geo g{};
    g.H = (int)H;
    g.W = (int)W;
    g.hc = oh;
    g.wc = ow;
    if ((rc = gen_prepare(g, 0, 0, c->gen_tab, c->gen_sub, c->gen_rec, c->stream))) return rc;
  }
  const double* planes[2] = {cb, cr};
  double* outs[2] = {cb_out, cr_out};
  for (int p = 0; p < 2; ++p) {
    if ((rc = stage_io(c, 0, planes[p], bi, &din))) return rc;
    if (gen) {
      // blur (if any) as the fast path does, then the fractional area resize
      const double* src = (const double*)din;
      if (prefilter) {
        HIP_TRY(stage_subsample((const double*)din, (double*)t1, (double*)t2, nullptr, (int)H, (int)W, sy, 1, gauss,
                                c->stream));
        src = (const double*)t2;
      }
      const AreaTap* tabs = (const AreaTap*)c->gen_tab.p;
      HIP_TRY(stage_area_gen(src, (int)H, (int)W, tabs, tabs + oh, (double*)dout, oh, ow, c->stream));
    } else {
      HIP_TRY(stage_subsample((const double*)din, (double*)t1, (double*)t2, (double*)dout, (int)H, (int)W, sy,
                              prefilter, gauss, c->stream));
    }
    if ((rc = stage_out(c, outs[p], dout, bo))) return rc;
  }
  return JDS_OK;
}

int jds_stage_upsample(jds_ctx* c, const double* in, int64_t h, int64_t w, int64_t H, int64_t W, int32_t nearest,
                       double* out) {
  if (!c || !in || !out || h < 1 || w < 1 || H < 1 || W < 1) return fail(JDS_EINVAL, "bad argument");
  HIP_TRY(hipSetDevice(c->device));
  void *din, *dout;
  int rc;
  if ((rc = stage_io(c, 0, in, (size_t)h * w * sizeof(double), &din)) ||
      (rc = stage_io(c, 1, nullptr, (size_t)H * W * sizeof(double), &dout)))
    return rc;
  HIP_TRY(stage_resize((const double*)din, (int)h, (int)w, (double*)dout, (int)H, (int)W, nearest, c->stream));
  return stage_out(c, out, dout, (size_t)H * W * sizeof(double));
}

int jds_stage_block_dct_n(jds_ctx* c, const double* in, double* out, int64_t n_blocks, int32_t block_size,
                          int32_t op) {
  if (!c || !in || !out || n_blocks < 0 || op < 0 || op > 3) return fail(JDS_EINVAL, "bad argument");
  if (block_size != 8 && block_size != 16)
    return fail(JDS_ENOTSUP, "block transforms are 8x8 or 16x16 (got %d)", block_size);
  if (n_blocks == 0) return JDS_OK;
  HIP_TRY(hipSetDevice(c->device));
  const size_t b = (size_t)n_blocks * block_size * block_size * sizeof(double);
  void *din, *dout;
  int rc;
  if ((rc = stage_io(c, 0, in, b, &din)) || (rc = stage_io(c, 1, nullptr, b, &dout))) return rc;
  HIP_TRY(stage_block((const double*)din, (double*)dout, n_blocks, block_size, op, c->stream));
  return stage_out(c, out, dout, b);
}

int jds_stage_block_dct(jds_ctx* c, const double* in, double* out, int64_t n_blocks, int32_t op) {
  return jds_stage_block_dct_n(c, in, out, n_blocks, 8, op);
}

int jds_stage_quantize_n(jds_ctx* c, const void* in, const double* qtable, int32_t table_len, void* out, int64_t n,
                         int32_t dequant) {
  if (!c || !in || !qtable || !out || n < 0) return fail(JDS_EINVAL, "bad argument");
  if ((table_len != 64 && table_len != 256) || (n % table_len)) return fail(JDS_EINVAL, "bad table length");
  if (n == 0) return JDS_OK;
  HIP_TRY(hipSetDevice(c->device));
  const size_t bi = (size_t)n * (dequant ? sizeof(int16_t) : sizeof(double));
  const size_t bo = (size_t)n * (dequant ? sizeof(double) : sizeof(int16_t));
  void *din, *dq, *dout;
  int rc;
  if ((rc = stage_io(c, 0, in, bi, &din)) || (rc = stage_io(c, 4, qtable, table_len * sizeof(double), &dq)) ||
      (rc = stage_io(c, 1, nullptr, bo, &dout)))
    return rc;
  HIP_TRY(stage_quant(din, (const double*)dq, dout, n, dequant, table_len, c->stream));
  return stage_out(c, out, dout, bo);
}

int jds_stage_quantize(jds_ctx* c, const void* in, const double* qtable, void* out, int64_t n, int32_t dequant) {
  return jds_stage_quantize_n(c, in, qtable, 64, out, n, dequant);
}

// ------------------------------------------------------- entropy coding --

// Entropy-coder scratch for n frames of geometry g, plus per-frame JFIF headers
// built from the 8x8 tables qt (n x 64).
static int ent_prepare(const Geo& g, int mode, int n, const double* qt, DevBuf* ent, DevBuf& hdr, DevBuf& tab,
                       hipStream_t s) {
  if (g.bs != 8) return fail(JDS_ENOTSUP, "JPEG entropy coding needs 8x8 blocks (block_size %d)", g.bs);
  if (g.H > 65535 || g.W > 65535) return fail(JDS_ENOTSUP, "baseline JPEG is limited to 65535 x 65535");
  if (g.gen) {
    // T.81 sizes a subsampled component ceil(W/2) x ceil(H/sy); the reference's
    // planes are floor-sized (cv2.resize).  The scans are valid only when both
    // give the same block grid.
    const int sy = mode == JDS_SS_420 ? 2 : 1;
    const int jw = (g.W + 1) / 2, jh = (g.H + sy - 1) / sy;
    if ((jw + 7) / 8 != g.ncx || (jh + 7) / 8 != g.ncy)
      return fail(JDS_ENOTSUP, "%dx%d: the chroma block grid (%dx%d) differs from baseline JPEG's (%dx%d)", g.H,
                  g.W, g.ncy, g.ncx, (jh + 7) / 8, (jw + 7) / 8);
  }
  size_t sz[8];
  ent_sizes(g, n, sz);
  for (int i = 0; i < 8; ++i)
    if (i != 6) HIP_TRY(ent[i].ensure(sz[i]));
  const size_t hl = sz[6] / (size_t)n;
  uint8_t* h = (uint8_t*)malloc(sz[6]);
  if (!h) return fail(JDS_ENOMEM, "host allocation failed");
  for (int i = 0; i < n; ++i) {
    if (ent_header(qt + 64 * i, mode, g.H, g.W, h + hl * i) != (int)hl) {
      free(h);
      return fail(JDS_EINVAL, "frame %d: baseline JPEG needs integer quantisation steps in [1, 255]", i);
    }
  }
  hipError_t e = hdr.ensure(sz[6]);
  if (e == hipSuccess) e = hipMemcpyAsync(hdr.p, h, sz[6], hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // h is freed below
  free(h);
  HIP_TRY(e);
  if (!tab.p) {
    alignas(16) static thread_local char t[16384];
    if (ent_tab_size() > sizeof t) return fail(JDS_EINVAL, "entropy tables exceed the staging buffer");
    ent_build_tables((EntTab*)t);
    HIP_TRY(tab.ensure(ent_tab_size()));
    HIP_TRY(hipMemcpy(tab.p, t, ent_tab_size(), hipMemcpyHostToDevice));
  }
  return JDS_OK;
}

int jds_plan_entropy_capacity(const jds_plan* p, int64_t* bytes_per_frame) {
  if (!p || !bytes_per_frame) return fail(JDS_EINVAL, "null argument");
  if (p->g.bs != 8) return fail(JDS_ENOTSUP, "JPEG entropy coding needs 8x8 blocks (block_size %d)", p->g.bs);
  *bytes_per_frame = ent_capacity(p->g);
  return JDS_OK;
}

int jds_plan_entropy(jds_plan* p, const int16_t* coeffs, uint8_t* out, int64_t out_stride, uint64_t* lengths,
                     uint64_t* scan_bits, void* stream) {
  if (!p || !coeffs || !out || !lengths) return fail(JDS_EINVAL, "null argument");
  if (out_stride < ent_capacity(p->g))
    return fail(JDS_EINVAL, "out_stride %lld < worst-case file size %lld", (long long)out_stride,
                (long long)ent_capacity(p->g));
  HIP_TRY(hipSetDevice(p->ctx->device));
  hipStream_t s = (hipStream_t)stream;
  if (!p->ent_hdr.p) {
    int rc = ent_prepare(p->g, p->mode, p->n, p->qt, p->ent, p->ent_hdr, p->ent_tab, s);
    if (rc) return rc;
  }
  void* bufs[8];
  for (int i = 0; i < 8; ++i) bufs[i] = p->ent[i].p;
  HIP_TRY(launch_entropy(p->g, p->n, coeffs, bufs, (const uint8_t*)p->ent_hdr.p, p->ent_tab.p, out, out_stride,
                         (unsigned long long*)lengths, (unsigned long long*)scan_bits, s));
  return JDS_OK;
}

int jds_encode_jfif(jds_ctx* c, const jds_params* prm, int64_t H, int64_t W, const int16_t* coeffs, uint8_t* out,
                    int64_t out_cap, int64_t* out_len, uint64_t* scan_bits) {
  if (!c || !prm || !coeffs || !out || !out_len) return fail(JDS_EINVAL, "null argument");
  Geo g;
  int mode;
  int rc = make_geo(prm, H, W, &g, &mode, nullptr);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if ((rc = ent_prepare(g, mode, 1, prm->qtable, c->ent, c->ent_hdr, c->ent_tab, s))) return rc;
  const long long cap = ent_capacity(g);
  HIP_TRY(c->ent_cf.ensure((size_t)g.cpf * sizeof(int16_t)));
  HIP_TRY(c->ent_out.ensure((size_t)cap));
  HIP_TRY(c->ent_meta.ensure(4 * sizeof(unsigned long long)));
  HIP_TRY(hipMemcpyAsync(c->ent_cf.p, coeffs, (size_t)g.cpf * sizeof(int16_t), hipMemcpyHostToDevice, s));
  void* bufs[8];
  for (int i = 0; i < 8; ++i) bufs[i] = c->ent[i].p;
  unsigned long long* meta = (unsigned long long*)c->ent_meta.p;
  HIP_TRY(launch_entropy(g, 1, (const int16_t*)c->ent_cf.p, bufs, (const uint8_t*)c->ent_hdr.p, c->ent_tab.p,
                         (uint8_t*)c->ent_out.p, cap, meta, meta + 1, s));
  unsigned long long m[4];
  HIP_TRY(hipMemcpyAsync(m, meta, sizeof m, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (m[0] == 0)
    return fail(JDS_EINVAL, "coefficients outside baseline JPEG's range (DC difference category > 11 or "
                            "AC category > 10)");
  *out_len = (int64_t)m[0];
  if (scan_bits)
    for (int i = 0; i < 3; ++i) scan_bits[i] = m[1 + i];
  if ((long long)m[0] > out_cap) return fail(JDS_EINVAL, "output buffer too small: %llu bytes needed", m[0]);
  HIP_TRY(hipMemcpy(out, c->ent_out.p, (size_t)m[0], hipMemcpyDeviceToHost));
  return JDS_OK;
}

int jds_selftest_dct8x8(const double* in, double* out, int64_t n, int32_t inverse) {
  if (!in || !out || n < 0) return fail(JDS_EINVAL, "bad argument");
  for (int64_t b = 0; b < n; ++b) {
    double t[64];
    memcpy(t, in + 64 * b, sizeof t);
    for (int col = 0; col < 8; ++col) {  // axis 0 first
      double* c = t + col;
      if (inverse)
        dct3_line(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
      else
        dct2_line(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
    }
    for (int r = 0; r < 8; ++r) {
      double* c = t + 8 * r;
      if (inverse)
        dct3_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
      else
        dct2_line(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
    }
    for (int i = 0; i < 64; ++i) out[64 * b + i] = t[i] * 0.0625;  // pocketfft fct = 1/16
  }
  return JDS_OK;
}

int jds_selftest_fwd32(int32_t subsampling, int32_t prefilter, const double* gauss, const uint8_t* rgb, int64_t H,
                       int64_t W, int32_t plane, int32_t rows_first, float* coeffs, double* bound) {
  if (!gauss || !rgb || !coeffs || !bound || H < 1 || W < 1 || H > 4096 || W > 4096 || plane < 0 || plane > 2 ||
      subsampling < JDS_SS_444 || subsampling > JDS_SS_420)
    return fail(JDS_EINVAL, "bad argument");
  const bool pf = prefilter != 0 && subsampling != JDS_SS_444;
  double E[128];
  fast_fwd_bounds(subsampling, pf, gauss, E);
  memcpy(bound, E + (plane ? 64 : 0), 64 * sizeof(double));
  if (fwd32_host_plane(subsampling, pf, gauss, rgb, (int)H, (int)W, plane, rows_first, coeffs))
    return fail(JDS_EINVAL, "plane size must be a multiple of 8");
  return JDS_OK;
}

int jds_selftest_fwd16(int32_t subsampling, int32_t prefilter, const double* gauss, const uint8_t* rgb, int64_t H,
                       int64_t W, int32_t plane, int32_t rows_first, float* coeffs, double* bound) {
  if (!gauss || !rgb || !coeffs || !bound || H < 1 || W < 1 || H > 4096 || W > 4096 || plane < 0 || plane > 2 ||
      subsampling < JDS_SS_444 || subsampling > JDS_SS_420)
    return fail(JDS_EINVAL, "bad argument");
  const bool pf = prefilter != 0 && subsampling != JDS_SS_444;
  double E[512];
  fast_fwd16_bounds(subsampling, pf, gauss, E);
  memcpy(bound, E + (plane ? 256 : 0), 256 * sizeof(double));
  if (fwd16_host_plane(subsampling, pf, gauss, rgb, (int)H, (int)W, plane, rows_first, coeffs))
    return fail(JDS_EINVAL, "plane size must be a multiple of 16");
  return JDS_OK;
}

int jds_selftest_inv_fast(int32_t subsampling, const int16_t* coeffs, const double* qtable, int64_t H, int64_t W,
                          int32_t fuse, double* values, uint8_t* bytes) {
  if (!coeffs || !qtable || !values || !bytes || H < 1 || W < 1 || H > 4096 || W > 4096 ||
      subsampling < JDS_SS_444 || subsampling > JDS_SS_420)
    return fail(JDS_EINVAL, "bad argument");
  if (inv_fast_host(subsampling, coeffs, qtable, (int)H, (int)W, fuse, 8, values, bytes))
    return fail(JDS_EINVAL, "odd chroma geometry: the certified inverse runs even sizes only");
  return JDS_OK;
}

int jds_selftest_inv_fast16(int32_t subsampling, const int16_t* coeffs, const double* qtable, int64_t H, int64_t W,
                            int32_t fuse, double* values, uint8_t* bytes) {
  if (!coeffs || !qtable || !values || !bytes || H < 1 || W < 1 || H > 4096 || W > 4096 ||
      subsampling < JDS_SS_444 || subsampling > JDS_SS_420)
    return fail(JDS_EINVAL, "bad argument");
  if (inv_fast_host(subsampling, coeffs, qtable, (int)H, (int)W, fuse, 16, values, bytes))
    return fail(JDS_EINVAL, "odd chroma geometry: the certified inverse runs even sizes only");
  return JDS_OK;
}

int jds_selftest_area_tab(int32_t src, int32_t dst, int32_t* n, int32_t* si, double* a) {
  if (src < 1 || dst < 1 || dst > src || !n || !si || !a) return fail(JDS_EINVAL, "bad argument");
  AreaTap* t = (AreaTap*)malloc(sizeof(AreaTap) * (size_t)dst);
  if (!t) return fail(JDS_ENOMEM, "host allocation failed");
  if (area_tab_build(src, dst, t) < 0) {
    free(t);
    return fail(JDS_EINVAL, "more than 4 taps per sample");
  }
  for (int d = 0; d < dst; ++d) {
    n[d] = t[d].n;
    for (int k = 0; k < 4; ++k) {
      si[4 * d + k] = k < t[d].n ? t[d].si[k] : -1;
      a[4 * d + k] = k < t[d].n ? t[d].a[k] : 0.0;
    }
  }
  free(t);
  return JDS_OK;
}

int jds_selftest_dct16x16(const double* in, double* out, int64_t n, int32_t inverse) {
  if (!in || !out || n < 0) return fail(JDS_EINVAL, "bad argument");
  for (int64_t b = 0; b < n; ++b) {
    double t[256], c[16];
    memcpy(t, in + 256 * b, sizeof t);
    for (int col = 0; col < 16; ++col) {  // axis 0 first
      for (int i = 0; i < 16; ++i) c[i] = t[i * 16 + col];
      if (inverse) dct3_line16(c); else dct2_line16(c);
      for (int i = 0; i < 16; ++i) t[i * 16 + col] = c[i];
    }
    for (int r = 0; r < 16; ++r) {
      if (inverse) dct3_line16(t + 16 * r); else dct2_line16(t + 16 * r);
    }
    for (int i = 0; i < 256; ++i) out[256 * b + i] = t[i] * 0.03125;  // pocketfft fct = 1/32
  }
  return JDS_OK;
}

}  // extern "C"
