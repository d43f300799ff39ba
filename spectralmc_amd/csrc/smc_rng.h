// Device RNG of the GBM engine: one independent N(0,1) stream per (contract ordinal, path).
//
// The reference draws a fresh (T, P) normal matrix per contract from CuPy's XORWOW
// generator (reference src/spectralmc/async_normals.py:212-216) and reads it from HBM in
// the path kernel (gbm.py:248).  Here the normals never touch memory: each lane derives
// the stream of its group of 4 paths in registers.
//
//   paths are grouped g = p / 4 (a lane's 4 paths); one stream per (contract ordinal, group):
//   seed state  = Philox4x32-10( counter = (g_lo, g_hi, ordinal_lo, ordinal_hi),
//                                key     = (mc_seed_lo, mc_seed_hi) )      [Salmon et al. 2011]
//   u32 stream  = MWC64X seeded with Philox words (0, 1)                  [Thomas 2011]
//                 (x, c) <- A x + c (mod 2^64 split into (x, c)), output x ^ c, A = 4294883355
//   normals     = Box-Muller on consecutive u32 pairs (a, b):
//                   u1 = 2 - 1.m(a >> 9) in (0, 1],  angle = (b >> 9) 2^-23 revolutions       (f32)
//                   u1 = (a + 1/2) * 2^-32,                 u2 = b * 2^-32      (f64: smc_math.h)
//                   z0 = sqrt(-2 ln u1) cos(2 pi u2),  z1 = sqrt(-2 ln u1) sin(2 pi u2)
//                 f32: ln / sin / cos are the portable kernels of smc_math.h, so the normals
//                 are bit-identical to the CPU restatement.
//   draw order: for each step pair (t, t+1), t even: for j = 0..3 (path 4g + j): one Box-Muller
//   pair (a, b) -> normals t and t+1 of that path.  The last step of an odd T (round 4): two pairs,
//   pair k -> normal T-1 of paths 2k (z0) and 2k + 1 (z1), so no normal is drawn and discarded (at
//   T = 1, the reference's lock-step shape, that halves the transcendentals).  Draws of paths >= P
//   (ragged last group) are made and discarded, so the stream position never depends on P.
//
// Philox runs once per group (its round keys are wave-uniform, so the key schedule lives in
// SGPRs) and is amortised over 4 paths x T steps; each further u32 is one v_mad_u64_u32 plus an
// xor (and a register move): measured on gfx950 the round-2 xoshiro128+ step (three v_bitop3, an
// add, a xor, a shift and a rotate) cost ~2x as many VALU cycles per output
// (tools/micro/valurate.hip).  oracle/gbm_oracle.c restates the same stream on the CPU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "smc_math.h"

namespace smc {

__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int round = 0; round < 10; ++round) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
    const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ c3 ^ k1;
    c1 = static_cast<uint32_t>(p1);
    c3 = static_cast<uint32_t>(p0);
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

struct PathStream {
  // MWC64X (Thomas 2011): multiply-with-carry, base 2^32, multiplier kMwcA; state (x, c) with
  // c < kMwcA; output x ^ c, then (x, c) <- kMwcA x + c as one v_mad_u64_u32.
  static constexpr uint32_t kMwcA = 4294883355u;
  uint32_t x, c;

  // seed: words 0, 1 of Philox4x32-10(counter = (group, ordinal), key = mc_seed); the absorbing
  // states (0, 0) and (2^32 - 1, kMwcA - 1) are moved off
  __device__ __forceinline__ PathStream(uint64_t mc_seed, uint64_t ordinal, uint64_t group) {
    uint32_t s0 = static_cast<uint32_t>(group), s1 = static_cast<uint32_t>(group >> 32);
    uint32_t s2 = static_cast<uint32_t>(ordinal), s3 = static_cast<uint32_t>(ordinal >> 32);
    philox4x32_10(s0, s1, s2, s3, static_cast<uint32_t>(mc_seed), static_cast<uint32_t>(mc_seed >> 32));
    x = s0;
    c = s1 >= kMwcA ? s1 - kMwcA : s1;
    x |= static_cast<uint32_t>((x | c) == 0u);
    x ^= static_cast<uint32_t>(x == 0xFFFFFFFFu && c == kMwcA - 1u);
  }

  // Stream span (round 4): at T <= 2 a 4-path group draws only 4 T u32 values, so one Philox-seeded
  // stream serves kSpanGroups consecutive groups (16 paths) and the Philox-10 seed is paid once per 16
  // paths instead of once per 4: group g takes the (g mod 4)-th run of 4 T draws of stream g / 4.
  // T >= 3: one stream per group.  This constructor positions the stream at group g's first draw (a
  // kernel that walks a whole span, wave_kernel, seeds stream g / 4 once and draws the groups in order).
  static constexpr int kSpanGroups = 4;
  __device__ __forceinline__ PathStream(uint64_t mc_seed, uint64_t ordinal, uint64_t group, int T)
      : PathStream(mc_seed, ordinal, T <= 2 ? group / kSpanGroups : group) {
    if (T <= 2) {
      const int skip = 4 * T * static_cast<int>(group % kSpanGroups);
      for (int k = 0; k < skip; ++k) (void)next();
    }
  }

  __device__ __forceinline__ uint32_t next() {
    const uint32_t r = x ^ c;
    const uint64_t t = static_cast<uint64_t>(kMwcA) * x + c;
    x = static_cast<uint32_t>(t);
    c = static_cast<uint32_t>(t >> 32);
    return r;
  }

  // Scale of the f32 normal_pair<HW> output: HW returns z / sqrt(2 ln 2) (the constant is
  // folded into the caller's volatility coefficient), portable returns z itself.
  template <bool HW>
  static constexpr double kNormalScale = HW ? 1.1774100225154747 : 1.0;  // sqrt(2 ln 2)

  // Two N(0,1) draws, single precision, from 23-bit uniforms built by mantissa insertion:
  //   u1 = 2 - 1.m(a >> 9) in (0, 1]  (exact),  angle = 1.m(b >> 9) revolutions (period 1).
  // HW = false: portable IEEE-only arithmetic (smc_math.h), bit-identical to the CPU oracle:
  //   z = sqrt(-2 ln u1) (cos, sin)(2 pi angle).
  // HW = true (SMC_MATH_HW): v_log / v_sqrt / v_cos / v_sin_f32 (~1 ulp, not reproducible on
  //   a CPU), returning sqrt(-log2 u1) (cos, sin) = z / kNormalScale<true>:
  //   2 alignbit + 1 sub + 4 transcendentals + 2 mul per pair.
  template <bool HW>
  __device__ __forceinline__ void normal_pair(float& z0, float& z1) {
    const uint32_t a = next(), b = next();
    const float u1 = 2.0f - __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, a, 9));
    if constexpr (HW) {
      const float r = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u1));
      const float w = __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, b, 9));  // [1, 2) rev
      z0 = r * __builtin_amdgcn_cosf(w);
      z1 = r * __builtin_amdgcn_sinf(w);
    } else {
      const float r = __builtin_sqrtf(-2.0f * math::log_pos(u1));
      float sn, cs;
      math::sincos2pi_u24((b >> 9) << 1, sn, cs);
      z0 = r * cs;
      z1 = r * sn;
    }
  }

  // HW log-Euler fast path: exponents y = a + b z of the next two steps for the lane's 4 paths
  // (ylo: step t, yhi: step t+1), same draws as normal_pair<true>, with b folded into the
  // Box-Muller radius (one fma per normal) and path pairs packed into v_pk_* ops.
  __device__ __forceinline__ void hw_log_increments4(float b, float a, float (&ylo)[4], float (&yhi)[4]) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    float r[4], c[4], sn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t ua = next(), ub = next();
      const float u1 = 2.0f - __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, ua, 9));
      r[j] = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u1));
      const float w = __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, ub, 9));
      c[j] = __builtin_amdgcn_cosf(w);
      sn[j] = __builtin_amdgcn_sinf(w);
    }
    const f2 bb = {b, b}, aa = {a, a};
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const f2 br = f2{r[j], r[j + 1]} * bb;
      const f2 lo = __builtin_elementwise_fma(br, f2{c[j], c[j + 1]}, aa);
      const f2 hi = __builtin_elementwise_fma(br, f2{sn[j], sn[j + 1]}, aa);
      ylo[j] = lo.x;
      ylo[j + 1] = lo.y;
      yhi[j] = hi.x;
      yhi[j + 1] = hi.y;
    }
  }

  // HW log-Euler, last step of an odd T: the exponents y = a + b z of the lane's 4 paths from two
  // Box-Muller pairs (paths 0, 1: pair 0's z0, z1; paths 2, 3: pair 1's), the arithmetic of
  // hw_log_increments4.
  __device__ __forceinline__ void hw_log_tail4(float b, float a, float (&y)[4]) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t ua = next(), ub = next();
      const float u1 = 2.0f - __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, ua, 9));
      const float br = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u1)) * b;
      const float w = __uint_as_float(__builtin_amdgcn_alignbit(0x7Fu, ub, 9));
      const f2 v = __builtin_elementwise_fma(f2{br, br}, f2{__builtin_amdgcn_cosf(w), __builtin_amdgcn_sinf(w)},
                                             f2{a, a});
      y[2 * k] = v.x;
      y[2 * k + 1] = v.y;
    }
  }

  // Two N(0,1) draws, double precision: u1 = (a + 1/2) 2^-32 in (0, 1), angle = b 2^-32 revolutions;
  // -2 ln u1 and (sin, cos) of the angle from the 32-bit integers (smc_math.h m2log_u32 / sincos2pi_u32,
  // restated by the CPU oracle: bit-identical normals), sqrt correctly rounded (sqrt_radius).
  template <bool HW>
  __device__ __forceinline__ void normal_pair(double& z0, double& z1) {
    const uint32_t a = next(), b = next();
    const double r = math::sqrt_radius(math::m2log_u32(a));
    double s, c;
    math::sincos2pi_u32(b, s, c);
    z0 = r * c;
    z1 = r * s;
  }

  // f64 log-Euler: exponents y = a + (b r) (cos, sin) of the next two steps for the lane's 4 paths (ylo:
  // step t, yhi: step t + 1; a, b in units of ln 2 / 256: smc_math.h mul_exp2s_f64), the draws of
  // normal_pair<HW>(double&, double&) with b folded into the Box-Muller radius (one multiply per pair
  // instead of two)
  __device__ __forceinline__ void f64_log_increments4(double b, double a, double (&ylo)[4], double (&yhi)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t ua = next(), ub = next();
      const double br = math::sqrt_radius(math::m2log_u32(ua)) * b;
      double s, c;
      math::sincos2pi_u32(ub, s, c);
      ylo[j] = fma(br, c, a);
      yhi[j] = fma(br, s, a);
    }
  }

  // ... the last step of an odd T: paths 2k, 2k + 1 from pair k
  __device__ __forceinline__ void f64_log_tail4(double b, double a, double (&y)[4]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t ua = next(), ub = next();
      const double br = math::sqrt_radius(math::m2log_u32(ua)) * b;
      double s, c;
      math::sincos2pi_u32(ub, s, c);
      y[2 * k] = fma(br, c, a);
      y[2 * k + 1] = fma(br, s, a);
    }
  }

  // The last step of an odd T: normals of the lane's 4 paths from two pairs (paths 2k, 2k + 1 take
  // pair k's z0, z1).
  template <bool HW, typename Real>
  __device__ __forceinline__ void normal_tail(Real (&z)[4]) {
    normal_pair<HW>(z[0], z[1]);
    normal_pair<HW>(z[2], z[3]);
  }
};

}  // namespace smc
