// Portable transcendental kernels for the f32 path engine.
//
// Every function here is a fixed sequence of IEEE-754 operations that round identically on
// gfx950 and on an x86 host (fmaf, +, -, *, correctly rounded sqrtf and division, exact
// ldexpf, integer bit manipulation) — no hardware approximations (v_exp/v_log/v_sin_f32)
// and no contraction freedom (`fp contract(off)`, every fused op written as fmaf).  The
// CPU oracle (oracle/gbm_oracle.c, "kernel mode") restates the same sequences, so paths,
// row sums and CF targets are bit-identical between the GPU and the CPU restatement.
//
// Cost on CDNA4: the hardware transcendentals issue at quarter rate, so these full-rate
// FMA polynomials cost about the same VALU time.
//
// Coefficients: tools/fit_poly.py (near-minimax least squares on Chebyshev nodes,
// rounded to f32): |rel err| log1p 1.4e-7, exp2 7.6e-8; |abs err| sin/cos(2 pi r) 8e-8.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "smc_f64_tables.h"

#pragma clang fp contract(off)

namespace smc {
namespace math {

// ln(1 + f) / f on f in [sqrt(1/2) - 1, sqrt(2) - 1], degree 8
__device__ __forceinline__ float log1p_q(float f) {
  float q = 0.08743945509195328f;
  q = fmaf(q, f, -0.14377330243587494f);
  q = fmaf(q, f, 0.14949095249176025f);
  q = fmaf(q, f, -0.16560696065425873f);
  q = fmaf(q, f, 0.19956977665424347f);
  q = fmaf(q, f, -0.2500215470790863f);
  q = fmaf(q, f, 0.3333418369293213f);
  q = fmaf(q, f, -0.49999988079071045f);
  q = fmaf(q, f, 1.0f);
  return q;
}

// Natural log of a positive normal float.
__device__ __forceinline__ float log_pos(float u) {
  uint32_t bits = __float_as_uint(u);
  int e = static_cast<int>(bits >> 23) - 127;
  uint32_t mb = (bits & 0x007FFFFFu) | 0x3F800000u;  // m in [1, 2)
  const bool hi = mb > 0x3FB504F3u;                  // m > sqrt(2): use m / 2, e + 1
  mb -= hi ? 0x00800000u : 0u;
  e += hi ? 1 : 0;
  const float f = __uint_as_float(mb) - 1.0f;        // exact (Sterbenz)
  const float lf = f * log1p_q(f);
  return fmaf(static_cast<float>(e), 0.693147182f, lf);
}

// sin(2 pi r) / r and cos(2 pi r) as polynomials in r^2, r in [-1/8, 1/8]
__device__ __forceinline__ float sin2pi_s(float r2) {
  float s = 41.48561096191406f;
  s = fmaf(s, r2, -76.69829559326172f);
  s = fmaf(s, r2, 81.60520935058594f);
  s = fmaf(s, r2, -41.34170150756836f);
  s = fmaf(s, r2, 6.2831854820251465f);
  return s;
}

__device__ __forceinline__ float cos2pi_c(float r2) {
  float c = 59.24250793457031f;
  c = fmaf(c, r2, -85.44358825683594f);
  c = fmaf(c, r2, 64.93932342529297f);
  c = fmaf(c, r2, -19.739208221435547f);
  c = fmaf(c, r2, 1.0f);
  return c;
}

// (sin, cos)(2 pi j 2^-24) for a 24-bit integer j: exact quarter-turn reduction.
__device__ __forceinline__ void sincos2pi_u24(uint32_t j, float& s_out, float& c_out) {
  const int k = static_cast<int>((j + (1u << 21)) >> 22);          // nearest quarter turn, 0..4
  const int rem = static_cast<int>(j) - (k << 22);                 // [-2^21, 2^21)
  const float r = static_cast<float>(rem) * 0x1p-24f;              // exact, |r| <= 1/8
  const float r2 = r * r;
  const float s = r * sin2pi_s(r2);
  const float c = cos2pi_c(r2);
  // rotate by k quarter turns without branches: sin <- (s, c, -s, -c), cos <- (c, -s, -c, s)
  const bool odd = (k & 1) != 0;
  const uint32_t sflip = static_cast<uint32_t>(k & 2) << 30;
  const uint32_t cflip = static_cast<uint32_t>((k + 1) & 2) << 30;
  s_out = __uint_as_float(__float_as_uint(odd ? c : s) ^ sflip);
  c_out = __uint_as_float(__float_as_uint(odd ? s : c) ^ cflip);
}

// 2^f on f in [-1/2, 1/2], degree 6
__device__ __forceinline__ float exp2_p(float f) {
  float p = 0.00015337577497120947f;
  p = fmaf(p, f, 0.0013399859890341759f);
  p = fmaf(p, f, 0.009618519805371761f);
  p = fmaf(p, f, 0.05550329014658928f);
  p = fmaf(p, f, 0.24022646248340607f);
  p = fmaf(p, f, 0.6931471824645996f);
  p = fmaf(p, f, 1.0f);
  return p;
}

// 2^y: round-to-nearest-even integer split (v_rndne_f32), polynomial, exact ldexp.
__device__ __forceinline__ float exp2_any(float y) {
  const float n = rintf(y);
  const float f = y - n;  // exact, in [-1/2, 1/2]
  return ldexpf(exp2_p(f), static_cast<int>(n));
}

__device__ __forceinline__ float exp_any(float x) { return exp2_any(x * 1.44269502f); }

// ---- f64: twiddles cos/sin(2 pi j / N) of the N-point DFT -------------------------------
// (sin, cos)(x) for |x| <= pi/4: Taylor series to x^17 / x^18 (truncation < 1e-19)
__device__ __forceinline__ void sincos_series(double x, double& s_out, double& c_out) {
  const double u = x * x;
  double s = 2.8114572543455206e-15;                   // 1/17!
  s = fma(s, -u, 7.647163731819816e-13);               // 1/15!
  s = fma(s, -u, 1.6059043836821613e-10);              // 1/13!
  s = fma(s, -u, 2.505210838544172e-08);               // 1/11!
  s = fma(s, -u, 2.7557319223985893e-06);              // 1/9!
  s = fma(s, -u, 0.0001984126984126984);               // 1/7!
  s = fma(s, -u, 0.008333333333333333);                // 1/5!
  s = fma(s, -u, 0.16666666666666666);                 // 1/3!
  s = fma(s, -u, 1.0);
  s_out = s * x;
  double c = 1.5619206968586225e-16;                   // 1/18!
  c = fma(c, -u, 4.779477332387385e-14);               // 1/16!
  c = fma(c, -u, 1.1470745597729725e-11);              // 1/14!
  c = fma(c, -u, 2.08767569878681e-09);                // 1/12!
  c = fma(c, -u, 2.755731922398589e-07);               // 1/10!
  c = fma(c, -u, 2.48015873015873e-05);                // 1/8!
  c = fma(c, -u, 0.001388888888888889);                // 1/6!
  c = fma(c, -u, 0.041666666666666664);                // 1/4!
  c = fma(c, -u, 0.5);                                 // 1/2!
  c_out = fma(c, -u, 1.0);
}

// Exact integer reduction to the nearest quarter turn, then Taylor series in x = 2 pi r,
// |x| <= pi/4 (terms to x^17 / x^18: truncation < 1e-19).
__device__ __forceinline__ void twiddle(int64_t j, int64_t N, double& s_out, double& c_out) {
  const int64_t num = 4 * j;
  const int64_t k = (2 * num + N) / (2 * N);         // round(4 j / N)
  const int64_t rem = num - k * N;                    // |rem| <= N / 2
  const double r = static_cast<double>(rem) / static_cast<double>(4 * N);
  const double x = r * 6.283185307179586;
  double s, c;
  sincos_series(x, s, c);
  const int q = static_cast<int>(k & 3);
  const bool odd = (q & 1) != 0;
  const double sb = odd ? c : s, cb = odd ? s : c;
  s_out = (q & 2) ? -sb : sb;
  c_out = ((q + 1) & 2) ? -cb : cb;
}

// ---- f64 path engine: the Box-Muller transcendentals of 32-bit uniforms and exp ------------
// Fixed IEEE-754 sequences (fma, +, -, *, exact scaling, frexp and integer bit manipulation) over tables
// (smc_f64_tables.h: generated in 60-digit decimal arithmetic, rounded to double), restated op for op by
// oracle/gbm_oracle.c, so f64 normals are bit-identical on the CPU.  Accuracy against libm
// (tests/test_oracle.py): -2 ln u within 2 ulp, (sin, cos) within 2^-52 absolute, 2^(y/256) within 2 ulp.
// The f64 path kernel is VALU-issue-bound (PMC: VALU busy ~88-95 % of the launch, every VALU instruction,
// integer or f64, 4 cycles per wave), so the forms minimise instructions per path step.  v3 (round 4):
// -2 ln u directly (the -2 folded into the table and the polynomial as exact power-of-two scalings), its
// table indexed by the top 10 mantissa bits with no range halving (the cancellation near u = 1 is avoided
// by an exact k LN2_HI + T_HI instead), and the path exponent carried in units of ln 2 / 256 (the scale
// folded into the step constants), so e^y needs no Cody-Waite reduction, a degree-4 polynomial, a
// 256-point table and one ldexp.  v4 (round 5, 6 fewer VALU instructions per Box-Muller pair): the log's
// mantissa and exponent from v_frexp_mant / v_frexp_exp (the exponent offset folded into the table, whose
// 32-byte rows are addressed by one add, shift and mask of the mantissa's high word); the angle's table
// index from the uniform's low 10 bits and its offset from the high 22 (one shift), the offset's
// polynomial in integer units (no conversion multiply).  The kernels that run this math copy the tables
// into LDS first (f64_tables_load): a global load on the path loop would wait for the wave's outstanding
// path stores (one vmcnt counter).
struct alignas(16) F64Tables {
  double2 sc[1024];     // (sin, cos)(2 pi j / 1024)
  double log[1025][4];  // -4 INV, -2 T_HI + 66 LN2_HI, -2 T_LO + 66 LN2_LO, 0 at c = 1 + i/1024
  double ex[256];       // 2^(j / 256)
};

__device__ __forceinline__ F64Tables& f64_lds() {
  __shared__ F64Tables t;
  return t;
}

// Every thread of the workgroup, before the workgroup's first f64 path math.
__device__ inline void f64_tables_load() {
  F64Tables& t = f64_lds();
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) t.sc[k] = double2{kF64SinCosTab[k][0], kF64SinCosTab[k][1]};
  for (int k = threadIdx.x; k < 1025 * 4; k += blockDim.x) (&t.log[0][0])[k] = (&kF64LogTab[0][0])[k];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) t.ex[k] = kF64Exp2Tab[k];
  __syncthreads();
}

// X = -2 ln((a + 1/2) 2^-32), the Box-Muller radius squared: m = a + 1/2 = fr 2^e exactly (frexp: fr in
// [1/2, 1), e in 0..32, <= 33 significant bits); table point c = 1 + i/1024 nearest f = 2 fr from the top 10
// mantissa bits (round half up: i = (mh + 2^9) >> 10, i = 1024 at f -> 2; the row's byte offset 32 i is
// ((hw + 2^9) >> 5) & 0xFFE0 of fr's high word hw = 0x3FE00000 | mh); r' = -2 (f INV - 1) = fr (-4 INV) + 2
// in one fma (|r'| <= 2^-10); -2 ln(1 + r) = r' + r'^2 Q(r') with Q the r^2..r^5 terms of ln(1 + r),
// exactly rescaled (D2..D5 = 1/4, 1/12, 1/32, 1/80); then X = (e (-2 LN2_HI) + HI) + ((e (-2 LN2_LO) + LO) +
// that) with HI = -2 T_HI - 33 (-2 LN2_HI), LO the same for T_LO (k = e - 33 in -33..-1 folded into the
// row): the first sum is exact (multiples of 2^-42 below 2^6): near u = 1 (f -> 2, e = 32, c = 2) it is
// exactly 0 and X the small remainder, with no cancellation.
__device__ __forceinline__ double m2log_u32(uint32_t a) {
  const double m = static_cast<double>(a) + 0.5;  // exact
  const double fr = __builtin_amdgcn_frexp_mant(m);
  const double e = static_cast<double>(__builtin_amdgcn_frexp_exp(m));
  const uint32_t hw = static_cast<uint32_t>(static_cast<uint64_t>(__double_as_longlong(fr)) >> 32);
  const uint32_t off = ((hw + 0x200u) >> 5) & 0xFFE0u;  // 32 i
  const double* t = reinterpret_cast<const double*>(reinterpret_cast<const char*>(f64_lds().log) + off);
  const double r = fma(fr, t[0], 2.0);
  double q = 0.0125;
  q = fma(q, r, 0.03125);
  q = fma(q, r, 0.08333333333333333);
  q = fma(q, r, 0.25);
  const double p = fma(q, r * r, r);
  return fma(e, kF64M2Ln2Hi, t[1]) + (fma(e, kF64M2Ln2Lo, t[2]) + p);
}

// sqrt(x) for the Box-Muller radius x = -2 ln u in [2.3e-10, 46.1] (u never 0 or 1): the correctly
// rounded f64 sqrt sequence (rsq seed, one Goldschmidt and two Newton-Raphson corrections) without the
// denormal / huge-argument scaling and the zero case this range never needs, so the result is the IEEE
// sqrt the oracle takes.
__device__ __forceinline__ double sqrt_radius(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
}

// (sin, cos) of the angle 2 pi (j / 1024 + y 2^-32) of the 32-bit uniform b (v4): j = b mod 1024 (the table
// angle), y = b >> 10 as a signed 22-bit integer in [-2^21, 2^21) (the offset, |x| = |K y| <= pi/1024,
// K = 2 pi 2^-32): every b maps to one of the 2^32 grid angles and each grid angle to one b, so the angle is
// uniform as b is.  sin x = y (S1 + u (S3 + u S5)), cos x = 1 + u (C2 + u C4) with u = y^2 (exact) and the
// K^k folded into the coefficients, then the rotation by the table's (sin, cos)(2 pi j / 1024).
__device__ __forceinline__ void sincos2pi_u32(uint32_t b, double& s_out, double& c_out) {
  const double y = static_cast<double>(static_cast<int32_t>(b) >> 10);
  const double u = y * y;
  const double sp = fma(u, kF64SinS5, kF64SinS3);
  const double sx = fma(u, sp, kF64SinS1) * y;
  const double cp = fma(u, kF64CosC4, kF64CosC2);
  const double cx = fma(cp, u, 1.0);
  const double2 sc = f64_lds().sc[b & 1023u];
  s_out = fma(sc.x, cx, sc.y * sx);
  c_out = fma(sc.y, cx, -(sc.x * sx));
}

// Path exponents in units of ln 2 / 256 (kExpUnit: the log-Euler step constants carry the scale):
// e^y = 2^(ys / 256), ys = y 256 / ln 2.  t = ys + 1.5 2^52 rounds ys to the integer n = 256 m + j held
// in t's low word (|n| < 2^31), n = t - 1.5 2^52, rr = ys - n exactly (|rr| <= 1/2, Sterbenz);
// 2^(rr/256) - 1 to degree 4 in rr (E1..E4 = (ln 2 / 256)^k / k!); 2^(ys/256) = 2^m T (1 + em1), T =
// 2^(j/256) from the table.
constexpr double kExpUnit = 369.3299304675746;  // 256 / ln 2
struct Exp2sSplit {
  double T, em1;
  int m;
};
__device__ __forceinline__ Exp2sSplit exp2s_split(double ys) {
  const double t = ys + 6755399441055744.0;
  const int ni = static_cast<int>(static_cast<uint32_t>(__double_as_longlong(t)));
  const double rr = ys - (t - 6755399441055744.0);
  double q = kF64ExpE4;
  q = fma(q, rr, kF64ExpE3);
  q = fma(q, rr, kF64ExpE2);
  q = fma(q, rr, kF64ExpE1);
  return Exp2sSplit{f64_lds().ex[ni & 255], q * rr, ni >> 8};
}

// 2^(ys/256) (tests): T (1 + em1) scaled by 2^m.
__device__ __forceinline__ double exp2s_f64(double ys) {
  const Exp2sSplit e = exp2s_split(ys);
  return __builtin_amdgcn_ldexp(fma(e.T, e.em1, e.T), e.m);
}

// x 2^(ys/256) as the f64 log-Euler step: (x T) (1 + em1) scaled by 2^m (v_ldexp_f64: exact for the
// normal values of the path recursion).
__device__ __forceinline__ double mul_exp2s_f64(double x, double ys) {
  const Exp2sSplit e = exp2s_split(ys);
  const double xt = x * e.T;
  return __builtin_amdgcn_ldexp(fma(xt, e.em1, xt), e.m);
}

}  // namespace math
}  // namespace smc
