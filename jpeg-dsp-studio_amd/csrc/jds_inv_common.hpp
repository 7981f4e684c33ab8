// jds_inv_common.hpp — tile geometry and coefficient loads shared by the exact
// inverse (jds_inv.hip, k_inv2) and the certified fast inverse
// (jds_inv_fast.hip, k_inv_fast): both walk the same tiles, so a tile the
// fast kernel cannot certify is recomputed by the exact kernel as a whole.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jds_internal.hpp"


namespace jds {

template <int MODE>
struct Inv {
  static constexpr int SY = Cfg<MODE>::SY, SX = Cfg<MODE>::SX;
  static constexpr int TH = (MODE == M420) ? 64 : 32;
  static constexpr int TW = (MODE == M444) ? 64 : 128;
  static constexpr int NT = (MODE == M444) ? 256 : 512;
  static constexpr int RY = (SY == 2) ? 1 : 0, RX = (SX == 2) ? 1 : 0;
  static constexpr int YBC = TW / 8, NYB = (TH / 8) * YBC;
  static constexpr int RB = NT / 8;                                        // luma blocks per round
  static constexpr int CBR = TH / (8 * SY) + 2 * RY, CBC = TW / (8 * SX) + 2 * RX;  // chroma blocks incl. ring
  static constexpr int NCB = CBR * CBC;                                    // per plane
  static constexpr int CWR = TH / SY + 2 * RY, CWC = TW / SX + 2 * RX;     // chroma sample window
  // row stride of the window in LDS: 4 doubles of padding for subsampled planes
  // (66 -> 70) put the 16-lane groups' ds_read_b128 of chroma8_fast on fewer
  // shared banks (a bank model of the two luma rounds: 576 -> 192 extra LDS
  // cycles per tile)
  static constexpr int CWS = SX == 2 ? CWC + 4 : CWC;
  static constexpr int NROW = (CBR - 2 * RY) * CBC * 8 + 2 * RY * CBC;     // chroma row tasks per plane
  static constexpr int MB = NCB > RB ? NCB : RB;                           // transpose-buffer blocks
  static constexpr int WPE = (MODE == M444) ? 3 : 4;                       // 2 or 3 workgroups per CU
  static_assert(NCB * 8 <= NT && NROW <= NT && NYB % RB == 0, "one round per chroma plane");
};

constexpr int MS = 72;  // doubles per block in the transpose buffer (64 + 8: conflict-free column writes)

// Transpose-buffer slot of element (r, c) of a block: the 16-B pair c/2 of row r
// is stored at pair (c/2) ^ (r & 3).  Column passes (lane c writes row r) still
// fill each row's 64 B with two blocks per 16-lane ds_write_b64 group on
// disjoint banks; row passes (lane r reads row r as 4 x ds_read_b128) then put
// the 4 lanes of every 16-lane group that share a 64-B window (MS*8 = 576 B
// shifts blocks by 16 banks) on 4 different 16-B slots: conflict-free instead
// of 4-way (MI355X_MICROARCH.md §LDS bank rules).
__device__ __forceinline__ int tslot(int r, int c) { return r * 8 + ((((c >> 1) ^ (r & 3)) << 1) | (c & 1)); }

// The same with the column's coefficients already loaded (software
// prefetch: the loads of the next block are issued before this one's math).
// (held sign-extended: signed 16-bit loads, no per-use extension)
struct Col16 {  // int16 elements: loaded two per VGPR (k_inv2 373 -> 363 us at 4K Q10 vs int)
  int16_t q[8];
};
// Blocks outside the grid (`ok` false) read block 0 of the plane instead: the
// caller never transforms them, and unmasked loads need no per-load branches.
__device__ __forceinline__ Col16 load_col(const int16_t* __restrict__ plane, long long boff, int v, bool ok) {
  const int16_t* blk = plane + (ok ? boff : 0ll);
  Col16 c;
#pragma unroll
  for (int r = 0; r < 8; ++r) c.q[r] = blk[r * 8 + v];
  return c;
}

#ifdef JDS_INV6  // k_inv_fast6's helpers (jds_inv_fast.hip, A/B builds only)
// A column held two coefficients per VGPR (k_inv_fast6: the prefetched column
// lives across a whole luma round, 4 VGPRs instead of 8): element r in the
// low / high half of w[r / 2], loaded by d16 / d16_hi loads.
typedef short jds_short2 __attribute__((ext_vector_type(2)));
struct Col16p {
  jds_short2 w[4];
  __device__ __forceinline__ int q(int r) const { return (int)((r & 1) ? w[r >> 1].y : w[r >> 1].x); }
};
__device__ __forceinline__ Col16p load_colp(const int16_t* __restrict__ plane, long long boff, int v, bool ok) {
  const int16_t* blk = plane + (ok ? boff : 0ll);
  Col16p c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    c.w[i].x = blk[(2 * i) * 8 + v];
    c.w[i].y = blk[(2 * i + 1) * 8 + v];
  }
  return c;
}

// Row k of a block as one 16-B load (k_inv_fast6: lane b + 8 k of a wave,
// block b), and the int16 8 x 8 transpose that turns the 8 lanes' rows into
// their columns (Col16p) in registers: xpose8's three butterfly stages on
// packed coefficients -- k bit 2 / bit 1 swap dword pairs (0,2),(1,3) /
// (0,1),(2,3) by v_permlane32 / v_permlane16_swap, k bit 0 exchanges the
// 16-bit halves with lane ^ 8 (DPP row rotation by 8, one v_perm_b32 whose
// per-lane selector keeps the lane's own half): 12 instructions instead of
// eight 2-byte loads per lane, whose 16-lane address groups spanned eight
// blocks (measured: the column loads of the b + 8 k layout cost 44 us of
// k_inv_fast6 at four waves per SIMD, 127 us at six).
__device__ __forceinline__ uint4 load_rowq(const int16_t* __restrict__ plane, long long boff, int k, bool ok) {
  return *reinterpret_cast<const uint4*>(plane + (ok ? boff : 0ll) + 8 * k);
}
// the same through a buffer resource of the frame's coefficients (boff and
// the row in coefficients; the 32-bit byte offset: frames < 2 GB)
__device__ __forceinline__ uint4 load_rowq_b(__amdgpu_buffer_rsrc_t r, long long boff, int k, bool ok) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(((ok ? boff : 0ll) + 8 * k) * 2), 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ Col16p xpose_q16(uint4 v) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // k bit 2: dwords (0,2), (1,3)
    const auto a = __builtin_amdgcn_permlane32_swap(w[i], w[i + 2], false, false);
    w[i] = a[0];
    w[i + 2] = a[1];
  }
#pragma unroll
  for (int i = 0; i < 4; i += 2) {  // k bit 1: dwords (0,1), (2,3)
    const auto a = __builtin_amdgcn_permlane16_swap(w[i], w[i + 1], false, false);
    w[i] = a[0];
    w[i + 1] = a[1];
  }
  const bool odd = (threadIdx.x >> 3) & 1;  // k bit 0: the 16-bit halves with lane ^ 8
  const uint32_t sel = odd ? 0x03020706u : 0x05040100u;  // odd: partner.hi | own.hi << 16; even: own.lo | partner.lo << 16
  Col16p c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t p = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[i], 0x128, 0xf, 0xf, true);
    const uint32_t r = __builtin_amdgcn_perm(p, w[i], sel);
    c.w[i].x = (short)(r & 0xffffu);
    c.w[i].y = (short)(r >> 16);
  }
  return c;
}

// ---- the transpose-free 4:2:0 tile (k_inv_fast6, round 6) ------------------
//
// k_inv_fast's 64 x 128 tile with its chroma window widened to whole ring
// blocks, so that every chroma block's 8 x 8 samples have a place in it: a
// block's column pass writes its outputs there and its row pass reads the rows
// back and overwrites them (the window is the transpose medium), and the luma
// transposes run in registers (xpose8).  Window column 0 is chroma column
// X0/2 - 8: block j of the tile's 10 chroma block columns (ring included)
// starts at window column 8 j (16-B aligned: the row pass's ds_read_b128 /
// ds_write_b128), and the upsample's six samples at 4 bj + 7 are read as the
// aligned pairs from 4 bj + 6.  Row r of the window is chroma row Y0/2 - 1 + r
// as in k_inv_fast (the top / bottom ring blocks contribute one row each).
// Rows 82 doubles apart differ by 36 dword banks (4 mod 8): with the in-block
// index's bit 0 on lane bit 3 (xpose8) the two output rows of a 16-lane group
// read adjacent window rows on disjoint bank halves (tools/lds_bank_model.py).
struct W6 {
  static constexpr int TH = 64, TW = 128, NT = 512, SY = 2, SX = 2;
  static constexpr int RB = 64, NYB = 128, YBC = 16;   // luma blocks per round / per tile / per block row
  static constexpr int CBR = 6, CBC = 10, NCB = 60;    // chroma blocks per plane incl. the ring
  static constexpr int CWR = 34, CX = 8, CWC = 80, CWS = 82;
};

// 8 x 8 transpose of doubles across the 8 lanes of a block with no LDS.  The
// lanes of block b in a wave are b, b + 8, .., b + 56 (in-block index k =
// lane >> 3 & 7).  In: lane k holds c[i] = A[i][k] (column k); out: lane k
// holds c[j] = A[k][j] (row k).  One butterfly stage per bit of k, each
// exchanging the register halves whose index bit differs from the lane's:
// k bit 2 = lane bit 5 by v_permlane32_swap and k bit 1 = lane bit 4 by
// v_permlane16_swap (the swap of the upper lanes of one register with the
// lower lanes of the other is exactly a stage: one instruction per dword pair),
// k bit 0 = lane bit 3 by a DPP row rotation by 8 (lane ^ 8 in a 16-lane row)
// and selects.  Every lane of the wave must be active.
__device__ __forceinline__ void xswap32(double& x, double& y) {
  const auto a = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
  x = __hiloint2double((int)h[0], (int)a[0]);
  y = __hiloint2double((int)h[1], (int)a[1]);
}
__device__ __forceinline__ void xswap16(double& x, double& y) {
  const auto a = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x), (unsigned)__double2loint(y), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x), (unsigned)__double2hiint(y), false, false);
  x = __hiloint2double((int)h[0], (int)a[0]);
  y = __hiloint2double((int)h[1], (int)a[1]);
}
__device__ __forceinline__ double dpp_ror8(double v) {  // the value of lane ^ 8 (every lane has a source)
  const int l = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xf, 0xf, true);
  const int h = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xf, 0xf, true);
  return __hiloint2double(h, l);
}
__device__ __forceinline__ void xswap8(double& x, double& y, bool odd) {
  const double px = dpp_ror8(x), py = dpp_ror8(y);
  const double nx = odd ? py : x, ny = odd ? y : px;
  x = nx;
  y = ny;
}
__device__ __forceinline__ void xpose8(double (&c)[8]) {
  const bool odd = (threadIdx.x >> 3) & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) xswap32(c[i], c[i + 4]);
  xswap16(c[0], c[2]);
  xswap16(c[1], c[3]);
  xswap16(c[4], c[6]);
  xswap16(c[5], c[7]);
  xswap8(c[0], c[1], odd);
  xswap8(c[2], c[3], odd);
  xswap8(c[4], c[5], odd);
  xswap8(c[6], c[7], odd);
}
#endif  // JDS_INV6
}  // namespace jds
