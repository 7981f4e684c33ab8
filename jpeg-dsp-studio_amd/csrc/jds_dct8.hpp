// jds_dct8.hpp — 8-point orthonormal DCT-II / DCT-III in fp64, bit-identical to
// scipy.fft.dctn / idctn(type=2, norm='ortho') on 8x8 blocks.
//
// The reference calls scipy.fft (vendored pocketfft) per block
// (engines/dct_engine.py:7-14).  pocketfft's T_dcst23<double> computes the
// length-8 type-2 transform as: pre-butterfly -> real backward FFT
// (radb2 then radb4) -> post-twiddle, and type-3 as the mirror image with a
// real forward FFT (radf4 then radf2).  Its twiddles come from its own
// sincos_2pibyn tables and are NOT all correctly rounded; the constants below
// are the exact doubles pocketfft uses (found by bit-exact search against
// SciPy 1.15.3 / 1.7.1, pinned by tests/test_abi_cpu.py::
// test_device_dct_expressions_bit_exact_vs_scipy).
//
// Every expression below is one IEEE operation, evaluated in pocketfft's
// order; the translation unit is compiled with FP contraction OFF so no FMA is
// formed.  The per-axis normalisation fct = 1/16 that pocketfft applies on the
// first axis is an exact power-of-two scale and is left to the caller (it is
// folded into the quantiser divisor 16*Q and into the IDCT output scale).
#pragma once
#pragma clang fp contract(off)

#ifdef __HIPCC__
#define JDS_HD __host__ __device__ __forceinline__
#else
#define JDS_HD inline
#endif

namespace jds {

// twiddle[i] = cos(2*pi*(i+1)/32) as tabulated by pocketfft (TW6 is 1 ulp low)
constexpr double TW0 = 0x1.f6297cff75cb0p-1;
constexpr double TW1 = 0x1.d906bcf328d46p-1;
constexpr double TW2 = 0x1.a9b66290ea1a3p-1;
constexpr double TW3 = 0x1.6a09e667f3bccp-1;
constexpr double TW4 = 0x1.1c73b39ae68c8p-1;
constexpr double TW5 = 0x1.87de2a6aea963p-2;
constexpr double TW6 = 0x1.8f8b83c69a60ap-3;
// rfftp twiddle for N=8: (cos, sin)(2*pi/8); pocketfft's cos is 1 ulp low
constexpr double W8R = 0x1.6a09e667f3bccp-1;
constexpr double W8I = 0x1.6a09e667f3bcdp-1;
constexpr double SQRT2 = 0x1.6a09e667f3bcdp+0;
constexpr double HALF_SQRT2 = SQRT2 * 0.5;  // pocketfft: sqrt2*T0(0.5), exact
constexpr double TWO_TW3 = 2.0 * TW3;       // pocketfft: 2*twiddle[NS2-1], exact

// Unnormalised-by-fct orthonormal DCT-II of one line (T_dcst23::exec type 2,
// cosine=true, ortho=true).  Output = 16 * scipy value when applied along both
// axes of a block (first axis first); see header comment.
JDS_HD void dct2_line(double& c0, double& c1, double& c2, double& c3,
                      double& c4, double& c5, double& c6, double& c7) {
  c0 = c0 * 2.0;
  c7 = c7 * 2.0;
  // MPINPLACE(c[k+1], c[k]) for k = 1, 3, 5
  { double t = c2; c2 = t - c1; c1 = c1 + t; }
  { double t = c4; c4 = t - c3; c3 = c3 + t; }
  { double t = c6; c6 = t - c5; c5 = c5 + t; }
  // rfftp::exec(c, fct, r2hc=false): radb2(ido=4, l1=1)
  const double h0 = c0 + c7, h4 = c0 - c7;
  const double h3 = 2.0 * c3, h7 = -2.0 * c4;
  const double h1 = c1 + c5, tr2 = c1 - c5;
  const double ti2 = c2 + c6, h2 = c2 - c6;
  const double h6 = W8R * ti2 + W8I * tr2;
  const double h5 = W8R * tr2 - W8I * ti2;
  // radb4(ido=1, l1=2), k = 0 and k = 1
  const double a2 = h0 + h3, a1 = h0 - h3, a3 = 2.0 * h1, a4 = 2.0 * h2;
  const double b2 = h4 + h7, b1 = h4 - h7, b3 = 2.0 * h5, b4 = 2.0 * h6;
  const double o0 = a2 + a3, o4 = a2 - a3, o6 = a1 + a4, o2 = a1 - a4;
  const double o1 = b2 + b3, o5 = b2 - b3, o7 = b1 + b4, o3 = b1 - b4;
  // post-twiddle, k = 1..3 (kc = 8 - k)
  double t1, t2;
  t1 = TW0 * o7 + TW6 * o1; t2 = TW0 * o1 - TW6 * o7;
  c1 = 0.5 * (t1 + t2); c7 = 0.5 * (t1 - t2);
  t1 = TW1 * o6 + TW5 * o2; t2 = TW1 * o2 - TW5 * o6;
  c2 = 0.5 * (t1 + t2); c6 = 0.5 * (t1 - t2);
  t1 = TW2 * o5 + TW4 * o3; t2 = TW2 * o3 - TW4 * o5;
  c3 = 0.5 * (t1 + t2); c5 = 0.5 * (t1 - t2);
  c4 = o4 * TW3;
  c0 = o0 * HALF_SQRT2;
}

// Orthonormal DCT-III of one line (T_dcst23::exec type 3, cosine, ortho),
// without the fct factor.
JDS_HD void dct3_line(double& c0, double& c1, double& c2, double& c3,
                      double& c4, double& c5, double& c6, double& c7) {
  c0 = c0 * SQRT2;
  double t1, t2;
  t1 = c1 + c7; t2 = c1 - c7;
  c1 = TW0 * t2 + TW6 * t1; c7 = TW0 * t1 - TW6 * t2;
  t1 = c2 + c6; t2 = c2 - c6;
  c2 = TW1 * t2 + TW5 * t1; c6 = TW1 * t1 - TW5 * t2;
  t1 = c3 + c5; t2 = c3 - c5;
  c3 = TW2 * t2 + TW4 * t1; c5 = TW2 * t1 - TW4 * t2;
  c4 = c4 * TWO_TW3;
  // rfftp::exec(c, fct, r2hc=true): radf4(ido=1, l1=2) for k = 0, 1
  double r1 = c6 + c2; const double g2 = c6 - c2;
  double r2 = c0 + c4; const double g1 = c0 - c4;
  const double g0 = r2 + r1, g3 = r2 - r1;
  r1 = c7 + c3; const double g6 = c7 - c3;
  r2 = c1 + c5; const double g5 = c1 - c5;
  const double g4 = r2 + r1, g7 = r2 - r1;
  // radf2(ido=4, l1=1)
  const double o0 = g0 + g4, o7 = g0 - g4;
  const double o4 = -g7, o3 = g3;
  const double q2 = W8R * g5 + W8I * g6;
  const double qi = W8R * g6 - W8I * g5;
  const double o1 = g1 + q2, o5 = g1 - q2;
  const double o2 = qi + g2, o6 = qi - g2;
  // MPINPLACE(c[k], c[k+1]) for k = 1, 3, 5
  c0 = o0; c7 = o7;
  c1 = o1 - o2; c2 = o2 + o1;
  c3 = o3 - o4; c4 = o4 + o3;
  c5 = o5 - o6; c6 = o6 + o5;
}

}  // namespace jds
