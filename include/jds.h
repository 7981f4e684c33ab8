/* jds.h — C-ABI of the MI355X-native JPEG-DSP-Studio block-DCT codec path.
 *
 * The reference (Xneonz0/JPEG-DSP-Studio) is pure Python and has no FFI; its
 * boundary is the Python function engines.pipeline.compress_reconstruct
 * (engines/pipeline.py:17-21) plus the per-stage functions re-exported by
 * engines/__init__.py:10-27.  This library is what sits UNDER that boundary:
 * the drop-in Python package (jpeg-dsp-studio_amd/engines) binds these entry
 * points with ctypes (jpeg-dsp-studio_amd/jds/_abi.py).
 *
 * Conventions: plain pointers and sizes, no torch/HIP types in signatures
 * (streams are passed as void*).  Every int-returning function returns
 * JDS_OK (0) or a negative code; jds_last_error() holds a thread-local message.
 * All GPU work is hand-written HIP for gfx950; there is no CPU fallback.
 */
#ifndef JDS_H
#define JDS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JDS_ABI_VERSION 3

#define JDS_OK       0
#define JDS_EINVAL  (-1)  /* bad argument                    -> ValueError   */
#define JDS_ENOTSUP (-2)  /* e.g. block_size not 8/16          -> ValueError   */
#define JDS_EHIP    (-3)  /* HIP runtime / device failure     -> RuntimeError */
#define JDS_ENOMEM  (-4)  /* device allocation failed         -> RuntimeError */

/* subsampling modes: models/compression_params.py:13 ('4:4:4','4:2:2','4:2:0') */
#define JDS_SS_444 0
#define JDS_SS_422 1
#define JDS_SS_420 2

/* jds_plan_run flags */
#define JDS_RUN_SSE 1u  /* fill sse_rgb / sse_y (PSNR); the inverse kernel re-reads the input */
#define JDS_RUN_FWD 2u  /* forward phase only (stats reset + k_fwd); with neither FWD nor INV: both */
#define JDS_RUN_INV 4u  /* inverse phase only (k_inv + finalize); needs the forward's coeffs/stats */
#define JDS_RUN_EXACT 8u /* all-fp64 kernels (default: certified fp32 + exact fp64 fix-up, same results) */
#define JDS_RUN_EXACT_INV 16u /* inverse only: the replayed-order fp64 kernel instead of the certified fast
                                 inverse + tile fix-up (same bytes; A/B and tests) */
#define JDS_RUN_INV_FIXALL 32u /* test: the certified fast inverse flags every tile, so the exact
                                  tile code recomputes the whole frame (exercises the fix-up path) */
#define JDS_RUN_INV_FAST 128u /* A/B and tests, coarse tables (DC quantiser > 60): the certified fast
                                inverse instead of the exact k_inv2 such plans run (most tiles of
                                those frames fall back) */
#define JDS_RUN_FWD_FIXALL 64u /* test, 16x16 plans: the certified fp32 forward lists every block, so
                                  k_fix_fwd16 recomputes the whole frame (exercises the fix-up path) */

/* `after` argument of the *_dev functions below: no wait, the caller has
 * synchronised the inputs.  (NULL is the HIP null stream, which is waited for.) */
#define JDS_AFTER_NONE ((void*)(intptr_t)-1)

typedef struct jds_ctx jds_ctx;    /* one per (thread, device): owns a HIP stream + scratch */
typedef struct jds_plan jds_plan;  /* fixed geometry + per-frame quant tables, device-resident */

/* Per-frame parameters.  Mirrors CompressionParams (models/compression_params.py:7-20);
 * the tables are computed on the host exactly as the reference does. */
typedef struct {
  /* 8: the reference's path.  16: the BASELINE configs[4] stretch the reference
   * stubs (models/compression_params.py:19-20 accepts it, engines/quantizer.py:24
   * then fails); its table is np.kron(qtable, ones((2, 2))), i.e.
   * Q16[u][v] = qtable[(u/2)*8 + v/2] (build decision).  Other values
   * fail with the reference's broadcast error (JDS_ENOTSUP). */
  int32_t block_size;
  int32_t quality;     /* 1..100 (informational; the table below is authoritative) */
  int32_t subsampling; /* JDS_SS_* */
  int32_t prefilter;   /* 0/1; ignored for 4:4:4 (engines/color_space.py:34-35) */
  double qtable[64];   /* scale_quant_matrix(JPEG_LUMA_Q50, quality) (engines/quantizer.py:7-19) */
  double gauss[3];     /* cv2.getGaussianKernel(3, 0.75) taps (engines/color_space.py:39-40) */
} jds_params;

/* Per-frame statistics, all exact integers; sse_y is an exact integer sum
 * converted to double and divided by 1e6.
 * estimate_bitrate_no_entropy (utils/metrics.py:51-92), histogram
 * (engines/pipeline.py:123-124) and the PSNR sums (utils/metrics.py:11,20). */
typedef struct {
  uint64_t nonzero;             /* count of q != 0 */
  uint64_t total_coeffs;        /* all_quantized_coeffs.size */
  uint64_t magnitude_bits;      /* sum over q != 0 of ceil(log2(|q|+1)) + 1 */
  uint64_t block_overhead_bits; /* 2 * ceil(H/B) * ceil(W/B) (luma grid only) */
  uint64_t hist[50];            /* np.histogram(q, bins=50, range=(-100, 100))[0] */
  uint64_t sse_rgb;             /* sum (orig - rec)^2 over H*W*3 uint8 samples (JDS_RUN_SSE) */
  double sse_y;                 /* sum (Y(orig) - Y(rec))^2, Y = .299R+.587G+.114B (JDS_RUN_SSE):
                                   sum of (299dR+587dG+114dB)^2 in 64-bit integers / 1e6 */
  uint64_t pixels;              /* H * W */
  double fwd_ms, inv_ms;        /* host path only: forward / inverse kernel time (hipEvents) */
  double ssim[4];               /* host path only: SSIM of R, G, B and of Y (utils/metrics.py:12-21) */
  double mse_y;                 /* host path only: NumPy-order mean of (Y(orig) - Y(rec))^2 */
  double magnitude_bits_f32;    /* host path only: magnitude_bits as NumPy's float32 np.sum yields it */
  uint64_t reserved[1];
} jds_frame_stats;

typedef struct {
  int64_t H, W;
  int64_t chroma_h, chroma_w;        /* after subsampling, before padding */
  int64_t y_blocks_y, y_blocks_x;    /* padded luma block grid */
  int64_t c_blocks_y, c_blocks_x;    /* padded chroma block grid (per plane) */
  int64_t coeffs_per_frame;          /* B*B * (Y blocks + 2 * chroma blocks) */
  int64_t cb_offset, cr_offset;      /* coefficient offsets of the Cb / Cr planes */
  int32_t tiles, threads_fwd, threads_inv, reserved;
} jds_geometry;

/* IntermediateData.selected_block_* (engines/pipeline.py:128-151); 8x8 path only
 * (with block_size 16, *sel_valid is always 0) */
typedef struct {
  double original[64], shifted[64], dct[64];
  int16_t quantized[64];
  double dequantized[64], reconstructed[64];
} jds_selected_block;

int jds_abi_version(void);
const char* jds_last_error(void);
int jds_device_count(int* n);

/* Geometry of one frame (host only, no device access). */
int jds_geometry_of(const jds_params* p, int64_t H, int64_t W, jds_geometry* out);

int jds_ctx_create(int device, jds_ctx** out);
void jds_ctx_destroy(jds_ctx* ctx);
void* jds_ctx_stream(jds_ctx* ctx);  /* the context's own hipStream_t */
/* SSIM scratch budget per luma launch group of jds_psnr_ssim_batch_dev (bytes;
 * <= 0: the default 16 GB).  The group size follows from it; the scratch is
 * sized for the groups that run (a single pair beyond the budget still runs). */
int jds_ctx_set_ssim_scratch(jds_ctx* ctx, int64_t bytes);

/* Device-resident batch path (bench, batch sweep).  n_frames frames of the same
 * HxW share one subsampling/prefilter setting; params[i] gives frame i's table.
 * Buffers are device pointers: rgb (n*H*W*3 u8), rgb_out (same), coeffs
 * (n * coeffs_per_frame int16, reference layout: Y blocks, Cb blocks, Cr blocks,
 * raster order, each block row-major), stats (n entries, overwritten), each
 * 16-byte aligned (JDS_EINVAL otherwise; hipMalloc / torch allocations are).
 * stream: a hipStream_t (NULL = the HIP null stream).  Asynchronous. */
int jds_plan_create(jds_ctx* ctx, const jds_params* params, int n_frames, int64_t H, int64_t W,
                    jds_plan** out);
/* Quality-sweep plan (BASELINE configs[3]; gui/worker.py:39-74 runs one
 * compress_reconstruct per quality): n_frames frames x n_q tables, params has
 * n_frames * n_q entries, item = frame * n_q + q.  jds_plan_run then takes rgb
 * with n_frames frames and writes rgb_out / coeffs / stats for the n_frames *
 * n_q items.  The quality-independent front end (colour, prefilter, subsample,
 * DCT) runs once per frame and is quantised for every table.
 * 8x8 blocks, n_q <= 8.  jds_plan_create(.., n, ..) = jds_plan_create_q(.., n, 1, ..). */
int jds_plan_create_q(jds_ctx* ctx, const jds_params* params, int n_frames, int n_q, int64_t H, int64_t W,
                      jds_plan** out);
int jds_plan_run(jds_plan* plan, const uint8_t* rgb, uint8_t* rgb_out, int16_t* coeffs,
                 jds_frame_stats* stats, uint32_t flags, void* stream);
int jds_plan_geometry(const jds_plan* plan, jds_geometry* out);
/* Entries the last run's fix-up lists received: [0] forward blocks recomputed exactly (k_fix_fwd),
   [1] inverse tiles the certified fast inverse handed to the exact kernel (k_inv2_list). */
int jds_plan_fix_counts(const jds_plan* plan, uint32_t* counts);
void jds_plan_destroy(jds_plan* plan);

/* Launch-level timing of jds_plan_run itself (bench.py's roofline; no reference
 * counterpart -- the reference's Timer covers only the colour conversions,
 * utils/metrics.py:31-48).  While profiling is on, every run of the plan marks
 * its stream before its first launch and after each kernel launch with an event;
 * jds_plan_profile_read waits for the last mark and returns, per kernel name (in
 * first-seen order), the summed time between the mark before it and its own
 * mark, and the number of launches.  "(between runs)" is the time from one run's
 * last mark to the next run's first (host gaps).  The intervals tile the span
 * from the first mark to the last, so their sum equals *span_ms.  Reading resets
 * the record; jds_plan_profile(plan, 0) stops marking.  The event pool holds
 * 8192 marks (~7 per run): a read after more marks than that fails with
 * JDS_EINVAL ("profile overflow") and returns no totals. */
typedef struct {
  char name[64];
  double total_ms;
  int64_t launches;
} jds_kernel_time;
int jds_plan_profile(jds_plan* plan, int enable);
int jds_plan_profile_read(jds_plan* plan, jds_kernel_time* out, int max, int* n_out, double* span_ms);

/* Host-buffer path: the drop-in for engines.pipeline.compress_reconstruct
 * (engines/pipeline.py:17-167).  Synchronous.  rgb: HxWx3 u8, C-contiguous.
 * Outputs (caller-allocated, all but rgb_out/stats nullable):
 *   rgb_out       HxWx3 u8   reconstructed_image            (:95)
 *   coeffs        coeffs_per_frame int16  all_quantized_coeffs (:99)
 *   error_map_y   HxW f64    |Y - Y_rec|                     (:119-120)
 *   error_map_rgb HxW f64    mean_c |rgb - rgb_rec_f|        (:121)
 *   sel           selected luma block (sel_by, sel_bx) arrays (:128-151);
 *                 *sel_valid set to 1 if the index is inside the padded grid. */
int jds_compress_reconstruct(jds_ctx* ctx, const jds_params* p, const uint8_t* rgb, int64_t H,
                             int64_t W, uint8_t* rgb_out, int16_t* coeffs, jds_frame_stats* stats,
                             double* error_map_y, double* error_map_rgb, int32_t sel_by,
                             int32_t sel_bx, jds_selected_block* sel, int32_t* sel_valid);

/* PSNR / SSIM of two HxWx3 uint8 host images on the GPU (utils/metrics.py:9-28):
 * out[0..3] = SSIM of R, G, B, Y; out[4] = MSE of Y; out[5] = MSE of RGB.
 * Bit-identical to skimage + scipy.ndimage + NumPy reductions.  H, W >= 7. */
int jds_psnr_ssim(jds_ctx* ctx, const uint8_t* a, const uint8_t* b, int64_t H, int64_t W, double* out);

/* The same on device-resident images (a_dev, b_dev: HxWx3 uint8 in device
 * memory of ctx's device, e.g. a plan's input frames and outputs), run on the
 * context's stream after a device-wide wait for earlier work; out on the host.
 * Serves the batch sweep's per-item CompressionResult metrics
 * (gui/worker.py:62-68 -> utils/metrics.py:9-28) without host copies
 * (SURVEY.md section 5 interface sketch: jds_ssim_dev). */
int jds_psnr_ssim_dev(jds_ctx* ctx, const uint8_t* a_dev, const uint8_t* b_dev, int64_t H, int64_t W, double* out);

/* jds_psnr_ssim_dev without the device-wide wait: the context's stream waits
 * only for the work queued so far on `after` (a hipStream_t, e.g. the plan
 * run's stream; NULL = the HIP null stream; JDS_AFTER_NONE = the caller has
 * already synchronised the images), so leased contexts of other threads keep
 * running.  out on the host. */
int jds_psnr_ssim_dev_after(jds_ctx* ctx, const uint8_t* a_dev, const uint8_t* b_dev, int64_t H, int64_t W,
                            double* out, void* after);

/* The same for n device-resident image pairs of one size (the batch sweep's
 * items, gui/worker.py:62-68): pair i = (a_dev[i], b_dev[i]) (host arrays of
 * device pointers); out[6 i + 0..5] as above.  The pairs run together (from
 * 32 pairs, R, G, B in one launch for all of them; the luma in groups sized by
 * a 16 GB scratch budget), so a sweep's SSIM fills the chip.  `after` as above. */
int jds_psnr_ssim_batch_dev(jds_ctx* ctx, int32_t n, const uint8_t* const* a_dev, const uint8_t* const* b_dev,
                            int64_t H, int64_t W, double* out, void* after);

/* NumPy's float32 sum of magnitude_bits over device-resident int16
 * coefficients (utils/metrics.py:77-78: np.sum(np.ceil(np.log2(|q| + 1)) + 1)
 * over the nonzero q, float32 accumulation in NumPy's 8192-element buffered
 * pairwise order; the host path's k_mag_f32 chain): what bpp and
 * compression_ratio are computed from once the exact sum passes 2^24.
 * n_coeffs: a multiple of 64 (one frame's IntermediateData layout); `after` as
 * above.  *out on the host. */
int jds_magnitude_bits_f32_dev(jds_ctx* ctx, const int16_t* coeffs_dev, int64_t n_coeffs, double* out, void* after);
/* The same for n_items coefficient arrays at coeffs_dev + i * item_stride
 * (int16 elements), one wait: out[i] on the host. */
int jds_magnitude_bits_f32_batch_dev(jds_ctx* ctx, const int16_t* coeffs_dev, int32_t n_items, int64_t n_coeffs,
                                     int64_t item_stride, double* out, void* after);

/* Per-stage functions of the engines.* API (engines/__init__.py:10-27), on host
 * fp64 arrays staged through the context's device memory.  Synchronous.
 *   rgb_to_ycbcr / ycbcr_to_rgb: n_pixels x 3 (engines/color_space.py:8-24)
 *   subsample: cb, cr HxW -> (H/2 or H) x W/2; mode JDS_SS_422 / JDS_SS_420;
 *              gauss = 3 prefilter taps (engines/color_space.py:27-53)
 *   upsample : h x w -> H x W, bilinear (nearest != 0: INTER_NEAREST) (:56-66)
 *   block_dct: n 8x8 blocks; op 0 dct2, 1 idct2, 2 encode_block, 3 decode_block
 *              (engines/dct_engine.py:7-27)
 *   quantize : n values (n % 64 == 0, 8x8-periodic table); dequant = 0:
 *              f64 -> int16 round-half-even of c/Q; 1: int16 -> f64 q*Q
 *              (engines/quantizer.py:22-29) */
int jds_stage_rgb_to_ycbcr(jds_ctx* ctx, const double* rgb, double* ycc, int64_t n_pixels);
int jds_stage_ycbcr_to_rgb(jds_ctx* ctx, const double* ycc, double* rgb, int64_t n_pixels);
int jds_stage_subsample(jds_ctx* ctx, const double* cb, const double* cr, int64_t H, int64_t W, int32_t mode,
                        int32_t prefilter, const double* gauss, double* cb_out, double* cr_out);
int jds_stage_upsample(jds_ctx* ctx, const double* in, int64_t h, int64_t w, int64_t H, int64_t W,
                       int32_t nearest, double* out);
int jds_stage_block_dct(jds_ctx* ctx, const double* in, double* out, int64_t n_blocks, int32_t op);
int jds_stage_quantize(jds_ctx* ctx, const void* in, const double* qtable, void* out, int64_t n,
                       int32_t dequant);
/* The same for 8x8 or 16x16 blocks (block_size 8 / 16; dctn / idctn of a 16x16
 * block, dct_engine.py:7-27) and for a 64- or 256-entry table broadcast over
 * n values (quantizer.py:22-29 with a 16x16 table). */
int jds_stage_block_dct_n(jds_ctx* ctx, const double* in, double* out, int64_t n_blocks, int32_t block_size,
                          int32_t op);
int jds_stage_quantize_n(jds_ctx* ctx, const void* in, const double* qtable, int32_t table_len, void* out,
                         int64_t n, int32_t dequant);

/* Baseline JPEG entropy coding (the reference only estimates
 * the size, utils/metrics.py:51-92): coefficients in the reference's layout
 * (all_quantized_coeffs, engines/pipeline.py:56,99) -> one JFIF file per frame:
 * SOI, APP0, DQT (the frame's 8x8 table, zigzag order, utils/constants.py:18-27),
 * SOF0, the T.81 Annex K Huffman tables, three non-interleaved scans (Y, Cb, Cr),
 * EOI.  Byte-for-byte definition: oracle/jpeg_entropy.py.  8x8 blocks only;
 * tables must hold integers in [1, 255].
 *   jds_plan_entropy: device buffers; coeffs as jds_plan_run writes them; frame i's
 *     file at out + i*out_stride (out_stride >= jds_plan_entropy_capacity), its
 *     length in lengths[i] (u64, device), and optionally the entropy-coded bits of
 *     its Y/Cb/Cr scans in scan_bits[3*i..] (before the byte pad).  Asynchronous.
 *     lengths[i] = 0 marks a frame whose coefficients baseline JPEG cannot code
 *     (DC difference category > 11 or AC category > 10; the codec path never
 *     produces those).
 *   jds_encode_jfif: one frame from host memory (synchronous); *out_len is set even
 *     when out_cap is too small (then JDS_EINVAL). */
int jds_plan_entropy_capacity(const jds_plan* plan, int64_t* bytes_per_frame);
int jds_plan_entropy(jds_plan* plan, const int16_t* coeffs, uint8_t* out, int64_t out_stride, uint64_t* lengths,
                     uint64_t* scan_bits, void* stream);
int jds_encode_jfif(jds_ctx* ctx, const jds_params* p, int64_t H, int64_t W, const int16_t* coeffs, uint8_t* out,
                    int64_t out_cap, int64_t* out_len, uint64_t* scan_bits);

/* Test-only: evaluate the device DCT expressions (jds_dct8.hpp) on the host so
 * the CPU test suite can pin them against SciPy without a GPU.  Not used by
 * any product path.  in/out: n blocks of 8x8 f64; inverse: 0 = dctn, 1 = idctn. */
int jds_selftest_dct8x8(const double* in, double* out, int64_t n, int32_t inverse);
/* The same for 16x16 blocks (jds_dct16.hpp). */
int jds_selftest_dct16x16(const double* in, double* out, int64_t n, int32_t inverse);

/* Test-only: the certified forward's fp32 chain (jds_fast.hip: colour, prefilter,
 * area average, fdct8_f32 along both axes) evaluated on the host for every 8x8
 * block of one plane (0 Y, 1 Cb, 2 Cr) of an H x W RGB image whose plane size is
 * a multiple of 8.  rows_first bit 0: pass order (1 = k_fwd32i's rows first,
 * 0 = k_fwd32's columns first); bit 1: prefiltered chroma through the combined
 * Gaussian + area taps (what every certified forward kernel computes; 0 = the
 * per-pixel Gaussian then area chains, an fp32 restatement kept for comparison);
 * coefficients before quantisation (n_blocks x 64 f32, raster block order);
 * bound[64] = the rigorous bound on |c_fp32 - c_exact| the kernels certify
 * with (fast_fwd_bounds).  Lets the CPU suite test the bound adversarially. */
int jds_selftest_fwd32(int32_t subsampling, int32_t prefilter, const double* gauss, const uint8_t* rgb, int64_t H,
                       int64_t W, int32_t plane, int32_t rows_first, float* coeffs, double* bound);
/* The same for the certified 16x16 forward (jds_fast16.hip: fdct16_f32, plane
 * size a multiple of 16; rows_first bit 0 as above, 0 = k_fwd16f's order; bit 1:
 * the combined taps, as k_fwd16f computes them): n_blocks x 256 f32
 * coefficients and bound[256] (fast_fwd16_bounds). */
int jds_selftest_fwd16(int32_t subsampling, int32_t prefilter, const double* gauss, const uint8_t* rgb, int64_t H,
                       int64_t W, int32_t plane, int32_t rows_first, float* coeffs, double* bound);

/* Test-only: the certified fast inverse's arithmetic (jds_inv_fast.hip,
 * k_inv_fast: folded dequantisation, AAN IDCT on both axes, clip to [-128, 127],
 * vertical then difference-form chroma blends, colour terms on the 2^-32 magic
 * grid) evaluated on the host with the kernel's own helpers, for an H x W image
 * (even H at 4:2:0, even W at 4:2:x) from coefficients in the
 * IntermediateData.all_quantized_coeffs layout and one 8x8 quant table.
 * fuse: 0 = every multiply-add rounded twice, 1 = every one fused (the device
 * compiler may pick either per site).  values: H*W*3 f64, the value v' the
 * certificate judges (RGB order); bytes: H*W*3, the kernel's byte for it.
 * Lets the CPU suite test tools/inv_bound.py's bound (K_LIN / K_CONST)
 * adversarially against the oracle's pre-truncation values. */
int jds_selftest_inv_fast(int32_t subsampling, const int16_t* coeffs, const double* qtable, int64_t H, int64_t W,
                          int32_t fuse, double* values, uint8_t* bytes);

/* Test-only: the same for 16x16 blocks (k_inv16_fast's chain: fidct16 lines,
 * coefficients in 16x16 blocks, Q16[u][v] = qtable[u/2][v/2]); pins
 * tools/inv_bound.py --b16's K_LIN16 / K_CONST16 on the CPU. */
int jds_selftest_inv_fast16(int32_t subsampling, const int16_t* coeffs, const double* qtable, int64_t H, int64_t W,
                            int32_t fuse, double* values, uint8_t* bytes);

/* Test-only: the host-built cv2 INTER_AREA table of one axis (OpenCV
 * computeResizeAreaTab, used by the odd-size path) for src -> dst samples:
 * per destination index its tap count n[d] (<= 4) and taps si[4d..], a[4d..].
 * Pinned on the CPU against oracle/cpu_ref.py:area_tab. */
int jds_selftest_area_tab(int32_t src, int32_t dst, int32_t* n, int32_t* si, double* a);

#ifdef __cplusplus
}
#endif

#endif /* JDS_H */
