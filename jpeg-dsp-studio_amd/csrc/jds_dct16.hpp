// jds_dct16.hpp — 16-point orthonormal DCT-II / DCT-III in fp64, bit-identical
// to scipy.fft.dctn / idctn(type=2, norm='ortho') on 16x16 blocks (the
// 16x16 block path of BASELINE configs[4]; the reference's dct_engine.py:7-14
// calls dctn on whatever block it is handed).
//
// pocketfft's T_dcst23<double> for N = 16: pre-butterfly -> real backward FFT
// with factors (4, 4) (radb4 with ido = 4, then radb4 with ido = 1) ->
// post-twiddle; type 3 is the mirror (radf4 ido = 1, then radf4 ido = 4).
// Constants are the doubles pocketfft's sincos_2pibyn tables produce (several
// are 1-2 ulp off the correctly rounded cosine, e.g. DT16[11]); they and the
// operation order are derived and checked bit-for-bit against SciPy by
// tools/pocketfft_dct.py, and the compiled header is pinned against SciPy by
// tests/test_abi_cpu.py through jds_selftest_dct16x16.
//
// As in jds_dct8.hpp, the first-axis norm factor fct = 1/32 (exact power of
// two) is left to the caller, and FP contraction is off.
#pragma once
#pragma clang fp contract(off)

#ifdef __HIPCC__
#define JDS_HD __host__ __device__ __forceinline__
#else
#define JDS_HD inline
#endif

namespace jds {
namespace d16 {

// T_dcst23 twiddle[i] = sincos_2pibyn(64)[i+1].r, i = 0..14
constexpr double DT16[15] = {
    0x1.fd88da3d12526p-1, 0x1.f6297cff75cb0p-1, 0x1.e9f4156c62ddap-1, 0x1.d906bcf328d46p-1,
    0x1.c38b2f180bdb1p-1, 0x1.a9b66290ea1a3p-1, 0x1.8bc806b151741p-1, 0x1.6a09e667f3bccp-1,
    0x1.44cf325091dd6p-1, 0x1.1c73b39ae68c8p-1, 0x1.e2b5d3806f639p-2, 0x1.87de2a6aea961p-2,
    0x1.294062ed59f04p-2, 0x1.8f8b83c69a60ap-3, 0x1.917a6bc29b424p-4};
// rfftp twiddles of the ido = 4 radix-4 pass: (cos, sin)(2*pi*j/16), j = 1..3
constexpr double WR[3] = {0x1.d906bcf328d46p-1, 0x1.6a09e667f3bccp-1, 0x1.87de2a6aea963p-2};
constexpr double WI[3] = {0x1.87de2a6aea963p-2, 0x1.6a09e667f3bcdp-1, 0x1.d906bcf328d46p-1};
constexpr double SQRT2 = 0x1.6a09e667f3bcdp+0;
constexpr double HSQT2 = 0x1.6a09e667f3bcdp-1;

// radb4 (rfftp backward radix 4), IDO in {1, 4}
template <int IDO, int L1>
JDS_HD void radb4(const double* cc, double* ch) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#pragma unroll
  for (int k = 0; k < L1; ++k) {
    const double tr2 = CC(0, 0, k) + CC(IDO - 1, 3, k), tr1 = CC(0, 0, k) - CC(IDO - 1, 3, k);
    const double tr3 = 2.0 * CC(IDO - 1, 1, k), tr4 = 2.0 * CC(0, 2, k);
    CH(0, k, 0) = tr2 + tr3; CH(0, k, 2) = tr2 - tr3;
    CH(0, k, 3) = tr1 + tr4; CH(0, k, 1) = tr1 - tr4;
  }
  if constexpr (IDO == 4) {
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      const double ti1 = CC(0, 3, k) + CC(0, 1, k), ti2 = CC(0, 3, k) - CC(0, 1, k);
      const double tr2 = CC(IDO - 1, 0, k) + CC(IDO - 1, 2, k), tr1 = CC(IDO - 1, 0, k) - CC(IDO - 1, 2, k);
      CH(IDO - 1, k, 0) = tr2 + tr2;
      CH(IDO - 1, k, 1) = SQRT2 * (tr1 - ti1);
      CH(IDO - 1, k, 2) = ti2 + ti2;
      CH(IDO - 1, k, 3) = -SQRT2 * (tr1 + ti1);
    }
    // i = 2 (ic = 2): the one general butterfly of the ido = 4 pass
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      constexpr int i = 2, ic = IDO - i;
      const double tr2 = CC(i - 1, 0, k) + CC(ic - 1, 3, k), tr1 = CC(i - 1, 0, k) - CC(ic - 1, 3, k);
      const double ti1 = CC(i, 0, k) + CC(ic, 3, k), ti2 = CC(i, 0, k) - CC(ic, 3, k);
      const double tr4 = CC(i, 2, k) + CC(ic, 1, k), ti3 = CC(i, 2, k) - CC(ic, 1, k);
      const double tr3 = CC(i - 1, 2, k) + CC(ic - 1, 1, k), ti4 = CC(i - 1, 2, k) - CC(ic - 1, 1, k);
      CH(i - 1, k, 0) = tr2 + tr3;
      const double cr3 = tr2 - tr3;
      CH(i, k, 0) = ti2 + ti3;
      const double ci3 = ti2 - ti3;
      const double cr4 = tr1 + tr4, cr2 = tr1 - tr4;
      const double ci2 = ti1 + ti4, ci4 = ti1 - ti4;
      CH(i, k, 1) = WR[0] * ci2 + WI[0] * cr2; CH(i - 1, k, 1) = WR[0] * cr2 - WI[0] * ci2;
      CH(i, k, 2) = WR[1] * ci3 + WI[1] * cr3; CH(i - 1, k, 2) = WR[1] * cr3 - WI[1] * ci3;
      CH(i, k, 3) = WR[2] * ci4 + WI[2] * cr4; CH(i - 1, k, 3) = WR[2] * cr4 - WI[2] * ci4;
    }
  }
#undef CC
#undef CH
}

// radf4 (rfftp forward radix 4), IDO in {1, 4}
template <int IDO, int L1>
JDS_HD void radf4(const double* cc, double* ch) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 4 * (c))]
#pragma unroll
  for (int k = 0; k < L1; ++k) {
    const double tr1 = CC(0, k, 3) + CC(0, k, 1);
    CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
    const double tr2 = CC(0, k, 0) + CC(0, k, 2);
    CH(IDO - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
    CH(0, 0, k) = tr2 + tr1;
    CH(IDO - 1, 3, k) = tr2 - tr1;
  }
  if constexpr (IDO == 4) {
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      const double ti1 = -HSQT2 * (CC(IDO - 1, k, 1) + CC(IDO - 1, k, 3));
      const double tr1 = HSQT2 * (CC(IDO - 1, k, 1) - CC(IDO - 1, k, 3));
      CH(IDO - 1, 0, k) = CC(IDO - 1, k, 0) + tr1;
      CH(IDO - 1, 2, k) = CC(IDO - 1, k, 0) - tr1;
      CH(0, 3, k) = ti1 + CC(IDO - 1, k, 2);
      CH(0, 1, k) = ti1 - CC(IDO - 1, k, 2);
    }
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      constexpr int i = 2, ic = IDO - i;
      const double cr2 = WR[0] * CC(i - 1, k, 1) + WI[0] * CC(i, k, 1);
      const double ci2 = WR[0] * CC(i, k, 1) - WI[0] * CC(i - 1, k, 1);
      const double cr3 = WR[1] * CC(i - 1, k, 2) + WI[1] * CC(i, k, 2);
      const double ci3 = WR[1] * CC(i, k, 2) - WI[1] * CC(i - 1, k, 2);
      const double cr4 = WR[2] * CC(i - 1, k, 3) + WI[2] * CC(i, k, 3);
      const double ci4 = WR[2] * CC(i, k, 3) - WI[2] * CC(i - 1, k, 3);
      const double tr1 = cr4 + cr2, tr4 = cr4 - cr2;
      const double ti1 = ci2 + ci4, ti4 = ci2 - ci4;
      const double tr2 = CC(i - 1, k, 0) + cr3, tr3 = CC(i - 1, k, 0) - cr3;
      const double ti2 = CC(i, k, 0) + ci3, ti3 = CC(i, k, 0) - ci3;
      CH(i - 1, 0, k) = tr2 + tr1; CH(ic - 1, 3, k) = tr2 - tr1;
      CH(i, 0, k) = ti1 + ti2;     CH(ic, 3, k) = ti1 - ti2;
      CH(i - 1, 2, k) = tr3 + ti4; CH(ic - 1, 1, k) = tr3 - ti4;
      CH(i, 2, k) = tr4 + ti3;     CH(ic, 1, k) = tr4 - ti3;
    }
  }
#undef CC
#undef CH
}

}  // namespace d16

// Orthonormal DCT-II of one 16-sample line without fct (T_dcst23 type 2).
JDS_HD void dct2_line16(double* c) {
  using namespace d16;
  c[0] = c[0] * 2.0;
  c[15] = c[15] * 2.0;
#pragma unroll
  for (int k = 1; k < 15; k += 2) {  // MPINPLACE(c[k+1], c[k])
    const double t = c[k + 1];
    c[k + 1] = t - c[k];
    c[k] = c[k] + t;
  }
  double h[16], o[16];
  radb4<4, 1>(c, h);
  radb4<1, 4>(h, o);
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    const int kc = 16 - k;
    const double t1 = DT16[k - 1] * o[kc] + DT16[kc - 1] * o[k];
    const double t2 = DT16[k - 1] * o[k] - DT16[kc - 1] * o[kc];
    c[k] = 0.5 * (t1 + t2);
    c[kc] = 0.5 * (t1 - t2);
  }
  c[8] = o[8] * DT16[7];
  c[0] = o[0] * (d16::SQRT2 * 0.5);
}

// Orthonormal DCT-III of one 16-sample line without fct (T_dcst23 type 3).
JDS_HD void dct3_line16(double* c) {
  using namespace d16;
  c[0] = c[0] * d16::SQRT2;
#pragma unroll
  for (int k = 1; k < 8; ++k) {
    const int kc = 16 - k;
    const double t1 = c[k] + c[kc], t2 = c[k] - c[kc];
    c[k] = DT16[k - 1] * t2 + DT16[kc - 1] * t1;
    c[kc] = DT16[k - 1] * t1 - DT16[kc - 1] * t2;
  }
  c[8] = c[8] * (2.0 * DT16[7]);
  double g[16], o[16];
  radf4<1, 4>(c, g);
  radf4<4, 1>(g, o);
  c[0] = o[0];
  c[15] = o[15];
#pragma unroll
  for (int k = 1; k < 15; k += 2) {  // MPINPLACE(c[k], c[k+1])
    c[k] = o[k] - o[k + 1];
    c[k + 1] = o[k + 1] + o[k];
  }
}

}  // namespace jds
