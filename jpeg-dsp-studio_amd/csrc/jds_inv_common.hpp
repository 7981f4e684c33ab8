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
}  // namespace jds
