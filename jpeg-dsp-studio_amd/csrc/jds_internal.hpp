// jds_internal.hpp — types shared by the HIP kernels and the host-side C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds.h"

namespace jds {

enum Mode : int { M444 = JDS_SS_444, M422 = JDS_SS_422, M420 = JDS_SS_420 };

// Frame geometry.  Tiles are laid on the MCU grid aligned to the BOTTOM-RIGHT
// corner (phantom MCUs at the top/left of the first tile row/column), so the
// block row/column that carries reflect padding always shares its tile with
// the previous block row/column it reflects into (np.pad 'reflect' reaches at
// most 7 samples back: engines/block_processor.py:10-13).
struct Geo {
  int H, W;          // image
  int hc, wc;        // chroma plane after subsampling (before padding)
  int nby, nbx;      // padded luma block grid
  int ncy, ncx;      // padded chroma block grid (per plane)
  int nmy, nmx;      // MCU grid
  int tiles_y, tiles_x, ty_off, tx_off;
  long long cpf;     // coefficients per frame
  long long off_cb, off_cr;
  double up_sy, up_sx;  // cv2.resize scale (src/dst) of the chroma upsample
  int bs;               // block size: 8, or 16 (jds_b16.hip)
  int gen;              // 1: cv2's fractional INTER_AREA applies (odd H in 4:2:0, odd W in 4:2:x):
                        // the general-geometry kernels of jds_gen.hip run instead of the tiled ones
  int afx, afy;         // gen: cv2's integer-scale INTER_AREA window (e.g. 3 x 2 for a 3-row 4:2:0
                        // frame), 0 when the fractional tables apply (area_fast_scales)
};

// One destination index of cv2's fractional INTER_AREA table on one axis
// (OpenCV computeResizeAreaTab): up to 4 source indices and their float
// weights (as doubles), in table order.  Built on the host (area_tab_build).
// cv::hal::resize's INTER_AREA dispatch for src -> dst on both axes: scale =
// 1 / (dst / src); both scales integral (|scale - cvRound(scale)| < DBL_EPSILON)
// selects resizeAreaFast.  Sets the window (fx, fy), or 0, 0 for the tables.
inline void area_fast_scales(int src_h, int dst_h, int src_w, int dst_w, int* fy, int* fx) {
  const double sy = 1.0 / ((double)dst_h / (double)src_h), sx = 1.0 / ((double)dst_w / (double)src_w);
  const double ry = __builtin_rint(sy), rx = __builtin_rint(sx);
  const double eps = 2.220446049250313e-16;
  const bool fast = __builtin_fabs(sy - ry) < eps && __builtin_fabs(sx - rx) < eps;
  *fy = fast ? (int)ry : 0;
  *fx = fast ? (int)rx : 0;
}

struct AreaTap {
  int n;
  int si[4];
  int pad;
  double a[4];
};

// Device buffers of the general-geometry path: the y then x area tables
// (hc + wc entries), fp64 subsampled chroma planes and reconstructed planes.
struct GenBufs {
  const AreaTap* tabs;
  double* sub;
  double* rec;
};

// Fix-up bitmap words per item of the certified forward path (one bit per
// 8x8 block of the item's coefficient array).
__host__ __device__ inline int fix_wpi(const Geo& g) { return (int)((g.cpf / 64 + 31) / 32); }

// Buffers of the certified 16x16 forward (jds_fast16.hip): per-frame fp32
// tables (FastQ16), the fp32 Gaussian taps, per-tile statistics partials
// (NSTAT u32 per tile), the list of blocks the exact fix-up recomputes, and
// counters: [0..1] list lengths, alternating between runs (`parity`: a run
// appends to [parity] and zeroes [parity ^ 1], which the previous run's
// fix-up has consumed), [2] the last run's list length.  Zeroed at plan
// creation.
struct Fwd16Fast {
  const void* fq16;
  const float* gk32;
  uint32_t* part;
  uint2* fixlist;
  unsigned* counters;
  int fix_all;  // test: list every block
  int parity;
};

// Counters of the certified fast inverse (jds_inv_fast.hip).
// * count[0..1]: tiles recomputed exactly in a run.  They alternate between
//   runs (`parity`): a run counts into count[parity] and zeroes
//   count[parity ^ 1] for the next; count[parity] stays readable for
//   jds_plan_fix_counts until then.
// * item[3][n]: the same per item, rotating over three runs (`rot`): a run
//   reads the previous run's counts, writes its own and zeroes the next run's.
//   An item whose previous run recomputed more than 1/8 of its tiles (e.g. very
//   low qualities: saturated, flat gray reconstructions are exact integers)
//   runs the exact tile code directly; every 16th run (`probe`) tries the fast
//   path again.
// All zeroed at plan creation.
// * list (k_inv_fast6, 4:2:0): the (frame, tile) of every tile the run hands
//   to the exact kernel, count[parity] entries (n x tiles capacity), walked by
//   k_inv6_fix right after.
struct InvFix {
  unsigned* count;
  unsigned* item;
  int fix_all;  // test: recompute every tile
  int parity;
  int rot;
  int probe;
  uint2* list;
};

// Per-frame quantiser: q16 = 16*Q (pocketfft's first-axis fct = 1/16 folded in), q = Q.
struct FrameQ {
  double q16[64];
  double q[64];
  double qmax;  // max q (the certified inverses' Dmax scale: a scalar load, no reduction)
  double pad_;
};

// Tile configuration per subsampling mode.
template <int MODE>
struct Cfg {
  static constexpr int SY = (MODE == M420) ? 2 : 1;   // chroma subsampling (rows)
  static constexpr int SX = (MODE == M444) ? 1 : 2;   // chroma subsampling (cols)
  static constexpr int MH = 8 * SY, MW = 8 * SX;      // MCU size in pixels
  static constexpr int TH = (MODE == M444) ? 16 : 32; // tile size in pixels
  static constexpr int TW = 64;
  static constexpr int MY = TH / MH, MX = TW / MW;    // MCUs per tile
  static constexpr int YBR = TH / 8, YBC = TW / 8;    // luma blocks per tile
  static constexpr int CBR = TH / MH, CBC = TW / MW;  // chroma blocks per plane per tile
  static constexpr int NYB = YBR * YBC, NCB = CBR * CBC;
  static constexpr int NB = NYB + 2 * NCB;
  static constexpr int TF = NB * 8;                   // forward threads: one per block line
  // inverse: chroma blocks including the 1-block ring the bilinear upsample reaches into
  static constexpr int RY = (SY == 2) ? 1 : 0, RX = (SX == 2) ? 1 : 0;
  static constexpr int RBR = CBR + 2 * RY, RBC = CBC + 2 * RX;
  static constexpr int NRB = RBR * RBC;               // per plane
  static constexpr int CWR = 8 * CBR + 2 * RY;        // chroma sample window kept in LDS
  static constexpr int CWC = 8 * CBC + 2 * RX;
  static constexpr int TI = 384;                      // inverse threads
};

// Launch marks (jds_plan_profile): while a profiled plan run is on this
// thread, each launch site records an event on its stream right after its
// launch, named after the kernel; jds_plan_profile_read turns consecutive marks
// into per-kernel durations.  No marks (a null pointer test) otherwise.
struct KMarks {
  hipEvent_t* ev = nullptr;
  char (*name)[64] = nullptr;
  int n = 0, cap = 0;
  long long dropped = 0;  // marks not taken since the last read (pool full)
};
extern thread_local KMarks* t_kmarks;
void kmark(hipStream_t s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Per-frame constants of the statistics and, when the forward deferred it,
// the histogram's zero bin (k_fwd_finish, k_finalize, k_inv_fast's fused tail).
__device__ inline void finalize_frame(const Geo& g, jds_frame_stats* s, int zero_bin) {
  s->total_coeffs = (uint64_t)g.cpf;
  s->block_overhead_bits = 2ull * (uint64_t)g.nby * (uint64_t)g.nbx;
  s->pixels = (uint64_t)g.H * (uint64_t)g.W;
  if (zero_bin) s->hist[25] += (uint64_t)g.cpf - s->nonzero;  // zeros fall in bin 25 ([0, 4))
}

// Workgroup (x, f) of a (ceil(ptiles / 64), n) x 512 launch: sums tiles
// [64x, 64x + 64) of frame f's per-tile statistics partials (nonzero,
// magnitude bits, hist[50] as u32 per tile) into the frame stats, 8 groups x 64
// lanes, one u64 atomic per statistic.
__device__ inline void reduce_partials(jds_frame_stats* st, const uint32_t* __restrict__ part, int ptiles) {
  __shared__ unsigned long long s_sum[8][64];
  const int f = blockIdx.y, j = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int t0 = blockIdx.x * 64 + grp * 8;
  unsigned long long a = 0ull;
  if (j < 52) {
    unsigned v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = t0 + i < ptiles ? part[((size_t)f * ptiles + t0 + i) * 52 + j] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) a += v[i];
  }
  s_sum[grp][j] = a;
  __syncthreads();
  if (threadIdx.x < 52) {
    unsigned long long b = 0ull;
#pragma unroll
    for (int i = 0; i < 8; ++i) b += s_sum[i][threadIdx.x];
    jds_frame_stats* s = st + f;
    unsigned long long* dst = threadIdx.x == 0 ? (unsigned long long*)&s->nonzero
                              : threadIdx.x == 1 ? (unsigned long long*)&s->magnitude_bits
                                                 : (unsigned long long*)&s->hist[threadIdx.x - 2];
    if (b) atomicAdd(dst, b);
  }
}

}  // namespace jds
