// jds_inv.hip — the inverse half of the codec path on gfx950:
// int16 coefficients -> dequantize -> 2-D IDCT -> clip -> chroma upsample ->
// YCbCr->RGB -> clip -> truncate -> uint8 RGB.  Reference:
// engines/pipeline.py:77-95 (dequantize, idct_2d, merge_blocks, upsample_chroma,
// ycbcr_to_rgb, clip/astype) with quantizer.py:27-29, dct_engine.py:17-27,
// color_space.py:17-24 and :63-65.  Every operation is fp64 in the
// reference's order (pocketfft DCT-III butterflies, cv2 INTER_LINEAR taps,
// NumPy colour expressions), FP contraction off: bytes are bit-identical.
//
// Work decomposition (one workgroup per TH x TW pixel tile, tiles laid from the
// top-left corner):
//   1. chroma, both planes: the tile's chroma blocks plus the ring the
//      bilinear upsample reaches into.  Column (axis-0) passes run one thread
//      per block column, straight from the int16 coefficients in HBM/L2 into
//      an fp64 transpose buffer; row (axis-1) passes run on the same 8 threads
//      (lanes of one wave: no barrier) for the block rows the window needs (a
//      top/bottom ring block contributes one row), into an fp64 LDS window.
//      One workgroup barrier completes the window.
//   2. luma, NT/8 blocks per round: the same column pass, then each thread
//      owns one 8-pixel block row: row IDCT -> Y in registers, chroma taps from
//      the LDS window, colour, clip, truncate, one 24-byte store.  Again
//      wave-local: no barriers.
// Y never goes through LDS.  The upsample shares products between
// neighbouring pixels (same IEEE operations, same results).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_dct8.hpp"
#include "jds_device.hpp"
#include "jds_internal.hpp"
#include "jds_inv_common.hpp"
#include "jds_inv_exact.hpp"

#pragma clang fp contract(off)

namespace jds {

template <int MODE, int XTRA>
__global__ void __launch_bounds__(Inv<MODE>::NT) __attribute__((amdgpu_waves_per_eu(XTRA > 1 ? 2 : Inv<MODE>::WPE)))
k_inv2(const Geo g, const int tiles_x, const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
       const uint8_t* __restrict__ rgb_in, uint8_t* __restrict__ rgb_out, jds_frame_stats* __restrict__ st,
       double* __restrict__ sse_y_part, double* __restrict__ err_y, double* __restrict__ err_rgb, const int in_div,
       const int fin) {
  __shared__ __attribute__((aligned(16))) InvShared<MODE, XTRA> sh;
  // k_finalize's per-frame work for runs without SSE terms (fin >= 0; 1 also
  // adds the zero bin the forward deferred): one launch fewer
  if (XTRA == 0 && fin >= 0 && blockIdx.x == 0 && threadIdx.x == 0) finalize_frame(g, st + blockIdx.y, fin);
  inv2_tile<MODE, XTRA>(sh, g, tiles_x, gridDim.x, blockIdx.y, blockIdx.x, coeffs, fq, rgb_in, rgb_out, st,
                        sse_y_part, err_y, err_rgb, in_div);
}

// IntermediateData.selected_block_reconstructed (pipeline.py:132-138): the
// clipped luma IDCT of one block (frame 0).
__global__ void __launch_bounds__(64) k_sel_recon(const int16_t* __restrict__ coeffs, const FrameQ* __restrict__ fq,
                                                  jds_selected_block* sel, int sel_blk) {
  __shared__ __attribute__((aligned(16))) double s[MS];
  const int t = threadIdx.x;
  if (t < 8) {
    int qs[64];
#pragma unroll
    for (int r = 0; r < 8; ++r) qs[r * 8 + t] = (int)fq[0].q[r * 8 + t];
    idct_col(coeffs + (long long)sel_blk * 64, qs, t, s);
  }
  __syncthreads();
  if (t < 8) {
    double c[8];
    idct_row(s, t, c);
#pragma unroll
    for (int k = 0; k < 8; ++k) sel->reconstructed[t * 8 + k] = c[k];
  }
}

// ------------------------------------------------------------ launchers --

template <int MODE>
static int inv_tiles_t(int H, int W, int* tx) {
  const int ty = (H + Inv<MODE>::TH - 1) / Inv<MODE>::TH;
  *tx = (W + Inv<MODE>::TW - 1) / Inv<MODE>::TW;
  return ty * *tx;
}

int inv_tiles(int mode, int H, int W) {
  int tx;
  return mode == M420 ? inv_tiles_t<M420>(H, W, &tx)
                      : (mode == M422 ? inv_tiles_t<M422>(H, W, &tx) : inv_tiles_t<M444>(H, W, &tx));
}

template <int MODE>
static hipError_t inv2_t(const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq, const uint8_t* rgb_in,
                         uint8_t* rgb_out, jds_frame_stats* st, double* part, double* err_y, double* err_rgb,
                         hipStream_t s, int in_div, int fin) {
  int tx;
  const int tiles = inv_tiles_t<MODE>(g.H, g.W, &tx);
  const dim3 grid(tiles, n), blk(Inv<MODE>::NT);
  if (err_y)
    hipLaunchKernelGGL((k_inv2<MODE, 2>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part, err_y,
                       err_rgb, in_div, -1);
  else if (rgb_in)
    hipLaunchKernelGGL((k_inv2<MODE, 1>), grid, blk, 0, s, g, tx, coeffs, fq, rgb_in, rgb_out, st, part, nullptr,
                       nullptr, in_div, -1);
  else
    hipLaunchKernelGGL((k_inv2<MODE, 0>), grid, blk, 0, s, g, tx, coeffs, fq, nullptr, rgb_out, st, part, nullptr,
                       nullptr, in_div, fin);
  kmark(s, "k_inv2<%d,%d>", MODE, err_y ? 2 : rgb_in ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_inv2(int mode, const Geo& g, int n, const int16_t* coeffs, const FrameQ* fq,
                       const uint8_t* rgb_in, uint8_t* rgb_out, jds_frame_stats* st, double* part, double* err_y,
                       double* err_rgb, hipStream_t s, int in_div, int fin) {
  switch (mode) {
    case M420: return inv2_t<M420>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div, fin);
    case M422: return inv2_t<M422>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div, fin);
    default: return inv2_t<M444>(g, n, coeffs, fq, rgb_in, rgb_out, st, part, err_y, err_rgb, s, in_div, fin);
  }
}

hipError_t launch_sel_recon(const int16_t* coeffs, const FrameQ* fq, jds_selected_block* sel, int sel_blk,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_sel_recon, dim3(1), dim3(64), 0, s, coeffs, fq, sel, sel_blk);
  kmark(s, "k_sel_recon");
  return hipGetLastError();
}

}  // namespace jds
