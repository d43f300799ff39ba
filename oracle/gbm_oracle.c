/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this code, and only as the checker / CPU
 * baseline; the product (spectralmc_amd/) never links or calls it.
 *
 * CPU restatement of the reference GBM engine's per-contract arithmetic, fed with the
 * same normal stream the HIP engine draws (stream definition: spectralmc_amd/csrc/smc_rng.h,
 * restated independently here):
 *
 *   normals   reference src/spectralmc/async_normals.py:212-216 draws a (T, P) N(0,1) matrix
 *             per contract from CuPy XORWOW (absent here: normal-level parity with CuPy is
 *             unpinned).  Here: Philox4x32-10 (Salmon et al., SC'11; KAT-pinned in tests)
 *             seeds MWC64X (Thomas 2011) per (contract ordinal, group of 4 paths);
 *             per step pair, the group's 4 paths draw one Box-Muller pair each, in path order.
 *             f32: ln / sin / cos from the portable IEEE-only kernels below (bit-identical
 *             to the device's); f64: the 32-bit-uniform log / sincos below (bit-identical too).
 *
 * Two modes:
 *   REFERENCE  (oracle_gbm_paths): reference src/spectralmc/gbm.py:241-257 — the Numba
 *             kernel's arguments are Python floats, so the recursion runs in f64 and only the
 *             stores round to the sim dtype.
 *             LOG_EULER:    X *= exp((r - d - v^2/2) dt + v dW),  dW = Z sqrt(dt)
 *             SIMPLE_EULER: X += (r - d) X dt + v X dW;  X = |X|
 *             Row sums: f64 sums of the stored values (gbm.py:437 cp.mean, up to order).
 *   KERNEL     (oracle_kernel_*): the same GBM recursion in f32 with the portable exp2, the
 *             HIP engine's reduction orders (per-lane chunk sums, wave butterfly, waves 0..7)
 *             and its CF arithmetic — an exact restatement of what the f32 HIP kernels compute,
 *             so GPU results can be checked bit-for-bit.
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp, no GPU needed)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* Philox4x32-10: Random123 (Salmon, Moraes, Dror, Shaw 2011), section 4 constants. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int round = 0; round < 10; ++round) {
    if (round > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t prod0 = (uint64_t)0xD2511F53u * c0;
    uint64_t prod1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(prod0 >> 32), lo0 = (uint32_t)prod0;
    uint32_t hi1 = (uint32_t)(prod1 >> 32), lo1 = (uint32_t)prod1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* MWC64X (D. B. Thomas, "The MWC64X random number generator", 2011): multiply-with-carry with
 * multiplier A = 4294883355 and base 2^32, state (x, c), output x ^ c, then (x, c) <- A x + c.
 * Period ~2^63; one 32x32->64 multiply-add per output on the device. */
#define MWC_A 4294883355u
typedef struct {
  uint32_t x, c;
} mwc64x;

static inline uint32_t mwc_next(mwc64x* g) {
  const uint32_t r = g->x ^ g->c;
  const uint64_t t = (uint64_t)MWC_A * g->x + g->c;
  g->x = (uint32_t)t;
  g->c = (uint32_t)(t >> 32);
  return r;
}

/* ---- portable f32 math: op-for-op restatement of spectralmc_amd/csrc/smc_math.h ------
 * (coefficients from tools/fit_poly.py; compile with -ffp-contract=off) */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static float log1p_q(float f) {
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

static float log_pos(float u) {
  const uint32_t bits = f2u(u);
  int e = (int)(bits >> 23) - 127;
  uint32_t mb = (bits & 0x007FFFFFu) | 0x3F800000u;
  const int hi = mb > 0x3FB504F3u;
  if (hi) { mb -= 0x00800000u; e += 1; }
  const float f = u2f(mb) - 1.0f;
  const float lf = f * log1p_q(f);
  return fmaf((float)e, 0.693147182f, lf);
}

static void sincos2pi_u24(uint32_t j, float* s_out, float* c_out) {
  const int k = (int)((j + (1u << 21)) >> 22);
  const int rem = (int)j - (k << 22);
  const float r = (float)rem * 0x1p-24f;
  const float r2 = r * r;
  float sp = 41.48561096191406f;
  sp = fmaf(sp, r2, -76.69829559326172f);
  sp = fmaf(sp, r2, 81.60520935058594f);
  sp = fmaf(sp, r2, -41.34170150756836f);
  sp = fmaf(sp, r2, 6.2831854820251465f);
  const float s = r * sp;
  float c = 59.24250793457031f;
  c = fmaf(c, r2, -85.44358825683594f);
  c = fmaf(c, r2, 64.93932342529297f);
  c = fmaf(c, r2, -19.739208221435547f);
  c = fmaf(c, r2, 1.0f);
  const int odd = k & 1;
  const uint32_t sflip = (uint32_t)(k & 2) << 30;
  const uint32_t cflip = (uint32_t)((k + 1) & 2) << 30;
  *s_out = u2f(f2u(odd ? c : s) ^ sflip);
  *c_out = u2f(f2u(odd ? s : c) ^ cflip);
}

static float exp2_any(float y) {
  const float n = rintf(y);
  const float f = y - n;
  float p = 0.00015337577497120947f;
  p = fmaf(p, f, 0.0013399859890341759f);
  p = fmaf(p, f, 0.009618519805371761f);
  p = fmaf(p, f, 0.05550329014658928f);
  p = fmaf(p, f, 0.24022646248340607f);
  p = fmaf(p, f, 0.6931471824645996f);
  p = fmaf(p, f, 1.0f);
  return ldexpf(p, (int)n);
}

static float exp_any(float x) { return exp2_any(x * 1.44269502f); }

static void twiddle(int64_t j, int64_t N, double* s_out, double* c_out) {
  const int64_t num = 4 * j;
  const int64_t k = (2 * num + N) / (2 * N);
  const int64_t rem = num - k * N;
  const double r = (double)rem / (double)(4 * N);
  const double x = r * 6.283185307179586;
  const double u = x * x;
  double s = 2.8114572543455206e-15;
  s = fma(s, -u, 7.647163731819816e-13);
  s = fma(s, -u, 1.6059043836821613e-10);
  s = fma(s, -u, 2.505210838544172e-08);
  s = fma(s, -u, 2.7557319223985893e-06);
  s = fma(s, -u, 0.0001984126984126984);
  s = fma(s, -u, 0.008333333333333333);
  s = fma(s, -u, 0.16666666666666666);
  s = fma(s, -u, 1.0);
  s = s * x;
  double c = 1.5619206968586225e-16;
  c = fma(c, -u, 4.779477332387385e-14);
  c = fma(c, -u, 1.1470745597729725e-11);
  c = fma(c, -u, 2.08767569878681e-09);
  c = fma(c, -u, 2.755731922398589e-07);
  c = fma(c, -u, 2.48015873015873e-05);
  c = fma(c, -u, 0.001388888888888889);
  c = fma(c, -u, 0.041666666666666664);
  c = fma(c, -u, 0.5);
  c = fma(c, -u, 1.0);
  const int q = (int)(k & 3);
  const double sb = (q & 1) ? c : s, cb = (q & 1) ? s : c;
  *s_out = (q & 2) ? -sb : sb;
  *c_out = ((q + 1) & 2) ? -cb : cb;
}

/* ---- f64 normals: op-for-op restatement of smc_math.h m2log_u32 / sincos2pi_u32 --------- */
#include "f64_tables.h"
static inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* -2 ln((a + 1/2) 2^-32) as smc_math.h m2log_u32 (round 5, v4): m = a + 1/2 = fr 2^e exactly (frexp, fr in
 * [1/2, 1)); table point c = 1 + i/1024 nearest f = 2 fr, i = (mh + 2^9) >> 10 from fr's top 20 mantissa bits
 * mh (the device addresses row i as ((hw + 2^9) >> 5) & 0xFFE0 bytes, hw = fr's high word: the same i);
 * r' = fr (-4 INV) + 2 in one fma; r' + r'^2 Q(r') (Q: D5 = 1/80, D4 = 1/32, D3 = 1/12, D2 = 1/4, Horner);
 * then (e (-2 LN2_HI) + HI) + ((e (-2 LN2_LO) + LO) + that), HI / LO the row's -2 T + 33 (2 LN2) parts. */
static double m2log_u32(uint32_t a) {
  const double m = (double)a + 0.5;
  int ei;
  const double fr = frexp(m, &ei);
  const double e = (double)ei;
  const uint32_t hw = (uint32_t)(d2u(fr) >> 32);
  const uint32_t idx = ((hw & 0xFFFFFu) + 0x200u) >> 10;
  const double* t = kF64LogTab[idx];
  const double r = fma(fr, t[0], 2.0);
  double q = 0.0125;
  q = fma(q, r, 0.03125);
  q = fma(q, r, 0.08333333333333333);
  q = fma(q, r, 0.25);
  const double p = fma(q, r * r, r);
  return fma(e, kF64M2Ln2Hi, t[1]) + (fma(e, kF64M2Ln2Lo, t[2]) + p);
}

/* (sin, cos) of the angle 2 pi (j / 1024 + y 2^-32) as smc_math.h sincos2pi_u32 (round 5, v4): j = b mod
 * 1024, y = (int32) b >> 10 (arithmetic shift) in [-2^21, 2^21); sin x = y (S1 + u (S3 + u S5)), cos x =
 * 1 + u (C2 + u C4), u = y^2 (exact), the K^k (K = 2 pi 2^-32) in the coefficients; then the rotation by
 * the table's (sin, cos)(2 pi j / 1024). */
static void sincos2pi_u32(uint32_t b, double* s_out, double* c_out) {
  const double y = (double)((int32_t)b >> 10);
  const double u = y * y;
  const double sp = fma(u, kF64SinS5, kF64SinS3);
  const double sx = fma(u, sp, kF64SinS1) * y;
  const double cp = fma(u, kF64CosC4, kF64CosC2);
  const double cx = fma(cp, u, 1.0);
  const double S = kF64SinCosTab[b & 1023u][0], C = kF64SinCosTab[b & 1023u][1];
  *s_out = fma(S, cx, C * sx);
  *c_out = fma(C, cx, -(S * sx));
}

/* 2^(ys/256) as smc_math.h exp2s_split / exp2s_f64 (the f64 device path exponent in units of ln 2 / 256):
 * t = ys + 1.5 2^52 rounds ys to n = 256 m + j (t's low word), rr = ys - n exactly, 2^(rr/256) - 1 to
 * degree 4 (E1..E4), 2^m T (1 + em1) with T = 2^(j/256) from the table.  The oracle's reference mode
 * keeps libm exp. */
static void exp2s_split(double ys, double* T, double* em1, int* m) {
  const double t = ys + 6755399441055744.0;
  const int ni = (int)(uint32_t)d2u(t);
  const double rr = ys - (t - 6755399441055744.0);
  double q = kF64ExpE4;
  q = fma(q, rr, kF64ExpE3);
  q = fma(q, rr, kF64ExpE2);
  q = fma(q, rr, kF64ExpE1);
  *T = kF64Exp2Tab[ni & 255];
  *em1 = q * rr;
  *m = ni >> 8;
}

double oracle_exp2s_f64(double ys) {
  double T, em1;
  int m;
  exp2s_split(ys, &T, &em1, &m);
  return ldexp(fma(T, em1, T), m);
}

/* x 2^(ys/256) as smc_math.h mul_exp2s_f64, the f64 device log-Euler step */
double oracle_mul_exp2s_f64(double x, double ys) {
  double T, em1;
  int m;
  exp2s_split(ys, &T, &em1, &m);
  const double xt = x * T;
  return ldexp(fma(xt, em1, xt), m);
}
double oracle_m2log_u32(uint32_t a) { return m2log_u32(a); }
void oracle_sincos2pi_u32(uint32_t b, double* s, double* c) { sincos2pi_u32(b, s, c); }

float oracle_log_pos(float u) { return log_pos(u); }
float oracle_exp2(float y) { return exp2_any(y); }
void oracle_sincos2pi_u24(uint32_t j, float* s, float* c) { sincos2pi_u24(j, s, c); }

#define GROUP 4  /* paths per stream */

/* Stream seed: words 0 and 1 of Philox4x32-10(counter = (group, ordinal), key = seed) give x and
 * c (reduced below A); the two absorbing states (0, 0) and (2^32 - 1, A - 1) are moved off. */
static void path_stream(uint64_t seed, uint64_t ordinal, uint64_t group, mwc64x* g) {
  const uint32_t ctr[4] = {(uint32_t)group, (uint32_t)(group >> 32), (uint32_t)ordinal, (uint32_t)(ordinal >> 32)};
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t out[4];
  oracle_philox4x32_10(ctr, key, out);
  g->x = out[0];
  g->c = out[1] >= MWC_A ? out[1] - MWC_A : out[1];
  if ((g->x | g->c) == 0u) g->x = 1u;
  if (g->x == 0xFFFFFFFFu && g->c == MWC_A - 1u) g->x = 0xFFFFFFFEu;
}

/* The first n u32 outputs of the stream of (seed, ordinal, group): tests pin it to a Python
 * restatement of the published MWC64X recurrence on the KAT-pinned Philox seed. */
void oracle_stream_u32(uint64_t seed, uint64_t ordinal, uint64_t group, int64_t n, uint32_t* out) {
  mwc64x g;
  path_stream(seed, ordinal, group, &g);
  for (int64_t i = 0; i < n; ++i) out[i] = mwc_next(&g);
}

/* One Box-Muller pair.  f32: 23-bit uniforms and the portable kernels (bit-identical to the
 * device); f64: 32-bit uniforms and the m2log_u32 / sincos2pi_u32 sequences above (bit-identical). */
static void normal_pair(mwc64x* g, int is_f64, double* z0, double* z1) {
  const uint32_t a = mwc_next(g), b = mwc_next(g);
  if (is_f64) {
    /* u1 = (a + 1/2) 2^-32, the angle of b (sincos2pi_u32): smc_math.h m2log_u32 / sincos2pi_u32 */
    const double r = sqrt(m2log_u32(a));
    double sn, cs;
    sincos2pi_u32(b, &sn, &cs);
    *z0 = r * cs;
    *z1 = r * sn;
  } else {
    /* u1 = 2 - (1.m) with m = a >> 9: (0, 1] on the 2^-23 grid, exact; angle (b >> 9) 2^-23 rev */
    const float u1 = 2.0f - u2f(0x3F800000u | (a >> 9));
    const float r = sqrtf(-2.0f * log_pos(u1));
    float sn, cs;
    sincos2pi_u24((b >> 9) << 1, &sn, &cs);
    *z0 = (double)(r * cs);
    *z1 = (double)(r * sn);
  }
}

/* Normals of one group of 4 paths: z[t][j] for t < rows (f64 holder of dtype values).  Step pairs
 * (t, t + 1): one Box-Muller pair per path j; the last row of an odd count: two pairs, pair k -> paths
 * 2k (z0) and 2k + 1 (z1) (smc_rng.h draw order, round 4). */
/* Stream span (smc_rng.h, round 4): at T <= 2 a 4-path group draws only 4 T u32 values, so one
 * Philox-seeded stream serves 4 consecutive groups (16 paths): group g takes the (g mod 4)-th run of
 * 4 T draws of stream g / 4.  T >= 3: one stream per group. */
static void group_stream(uint64_t seed, uint64_t ordinal, uint64_t group, int32_t rows, mwc64x* g) {
  if (rows <= 2) {
    path_stream(seed, ordinal, group / 4, g);
    for (int k = 0; k < 4 * rows * (int)(group % 4); ++k) (void)mwc_next(g);
  } else {
    path_stream(seed, ordinal, group, g);
  }
}

static void group_normals(uint64_t seed, uint64_t ordinal, uint64_t group, int32_t rows, int is_f64, double* z) {
  mwc64x g;
  group_stream(seed, ordinal, group, rows, &g);
  for (int t = 0; t < rows; t += 2) {
    if (t + 1 < rows) {
      for (int j = 0; j < GROUP; ++j) {
        double z0, z1;
        normal_pair(&g, is_f64, &z0, &z1);
        z[(int64_t)t * GROUP + j] = z0;
        z[(int64_t)(t + 1) * GROUP + j] = z1;
      }
    } else {
      for (int j = 0; j < GROUP; j += 2)
        normal_pair(&g, is_f64, &z[(int64_t)t * GROUP + j], &z[(int64_t)t * GROUP + j + 1]);
    }
  }
}

/* normals[t][p] of contract ordinal `ordinal` (dtype 0: f32 out, 1: f64 out). */
void oracle_normals(uint64_t seed, int64_t ordinal, int32_t rows, int64_t cols, int32_t dtype, void* out) {
  const int64_t groups = (cols + GROUP - 1) / GROUP;
#pragma omp parallel
  {
    double* z = (double*)malloc(sizeof(double) * (size_t)(rows + 1) * GROUP);
#pragma omp for schedule(static)
    for (int64_t gi = 0; gi < groups; ++gi) {
      group_normals(seed, (uint64_t)ordinal, (uint64_t)gi, rows, dtype == 1, z);
      for (int t = 0; t < rows; ++t)
        for (int j = 0; j < GROUP; ++j) {
          const int64_t p = gi * GROUP + j;
          if (p >= cols) continue;
          if (dtype == 1)
            ((double*)out)[(int64_t)t * cols + p] = z[(int64_t)t * GROUP + j];
          else
            ((float*)out)[(int64_t)t * cols + p] = (float)z[(int64_t)t * GROUP + j];
        }
    }
    free(z);
  }
}

/*
 * Simulate B contracts.  contracts: [B][6] (X0, K, T, r, d, v).  Outputs (each optional):
 *   paths    [B][T][P] stored values (dtype), un-normalised
 *   terminal [B][P]    the last row
 *   rowsum   [B][T]    f64 sum over paths of each stored row
 * scheme 0 = LOG_EULER, 1 = SIMPLE_EULER.  nthreads <= 0: OpenMP default.
 */
void oracle_gbm_paths(const double* contracts, int64_t B, int32_t T, int64_t P, uint64_t seed, int64_t ordinal0,
                      int32_t scheme, int32_t dtype, void* paths, void* terminal, double* rowsum, int32_t nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  const int is_f64 = dtype == 1;
  for (int64_t b = 0; b < B; ++b) {
    const double* c = contracts + 6 * b;
    const double X0 = c[0], Tm = c[2], r = c[3], d = c[4], v = c[5];
    const double dt = Tm / (double)T;
    const double sqrt_dt = sqrt(dt);
    const double drift_log = r - d - 0.5 * v * v;
    const double drift_eul = r - d;
    const uint64_t ordinal = (uint64_t)(ordinal0 + b);
    double* rs = rowsum ? rowsum + b * T : NULL;
    if (rs) memset(rs, 0, sizeof(double) * (size_t)T);
    const int64_t groups = (P + GROUP - 1) / GROUP;
#pragma omp parallel
    {
      double* local = (double*)calloc((size_t)T, sizeof(double));
      double* z = (double*)malloc(sizeof(double) * (size_t)(T + 1) * GROUP);
#pragma omp for schedule(static)
      for (int64_t gi = 0; gi < groups; ++gi) {
       group_normals(seed, ordinal, (uint64_t)gi, T, is_f64, z);
       for (int j = 0; j < GROUP; ++j) {
        const int64_t p = gi * GROUP + j;
        if (p >= P) break;
        double X = X0;
        for (int t = 0; t < T; ++t) {
          const double dW = z[(int64_t)t * GROUP + j] * sqrt_dt;
          if (scheme == 0) {
            X *= exp(drift_log * dt + v * dW);
          } else {
            X += drift_eul * X * dt + v * X * dW;
            X = fabs(X);
          }
          const double stored = is_f64 ? X : (double)(float)X;
          const int64_t at = (b * T + t) * P + p;
          if (paths) {
            if (is_f64)
              ((double*)paths)[at] = stored;
            else
              ((float*)paths)[at] = (float)stored;
          }
          if (terminal && t == T - 1) {
            if (is_f64)
              ((double*)terminal)[b * P + p] = stored;
            else
              ((float*)terminal)[b * P + p] = (float)stored;
          }
          local[t] += stored;
        }
       }
      }
      free(z);
      if (rs) {
#pragma omp critical
        for (int t = 0; t < T; ++t) rs[t] += local[t];
      }
      free(local);
    }
  }
}

int32_t oracle_num_threads(void) {
#ifdef _OPENMP
  return (int32_t)omp_get_max_threads();
#else
  return 1;
#endif
}

/* ======================================================================================
 * KERNEL mode: exact restatement of the f32 HIP engine (spectralmc_amd/csrc/gbm.hip).
 * ====================================================================================== */
#define K_THREADS 512
#define K_PPL 4
#define K_CHUNK (K_THREADS * K_PPL)
#define K_WAVES (K_THREADS / 64)

/* paths: [B][T][P] (optional), terminal [B][P] (optional), rowsum [B][T] (required).
 * slice_paths: 0 = one workgroup per contract; else the contract's paths are cut into slices of
 * that many paths (gbm.hip kSliceChunks * kChunk = 8192 when smc_train_targets gets a workspace),
 * each reduced like a whole contract, and the slice sums are added in slice order from 0.0. */
void oracle_kernel_paths(const double* contracts, int64_t B, int32_t T, int64_t P, uint64_t seed, int64_t ordinal0,
                         int32_t scheme, int64_t slice_paths, int32_t wg, float* paths, float* terminal,
                         double* rowsum) {
  /* scheme | 0x400 (SMC_MATH_REF, gbm.hip rows_ref_kernel): the reference kernel's typing -- the f64
   * engine's step (Stepper<double>: a, b in f64, units of ln 2 / 256 for log-Euler, mul_exp2s_f64) of the
   * portable f32 normals, the state kept in f64 and stored rounded to f32 */
  const int step64 = (scheme & 0x400) != 0;
  scheme &= 0xff;
  /* wg: lanes of the engine workgroup (512: contract/paths/queue kernels; 1024: resident_kernel) —
   * sets the chunk (4 wg paths) and the wave count of the row-sum order */
  const int lanes = wg > 0 ? wg : K_THREADS;
  const int64_t chunk_paths = (int64_t)K_PPL * lanes;
  const int waves = lanes / 64;
  const double kLog2e = 1.4426950408889634;
  float* X = (float*)malloc(sizeof(float) * (size_t)T * (size_t)P);
  double* lane_acc = (double*)malloc(sizeof(double) * (size_t)lanes * (size_t)T);
  for (int64_t b = 0; b < B; ++b) {
    const double* c = contracts + 6 * b;
    const double dt = c[2] / (double)T;
    const double sq = sqrt(dt);
    float ca, cb;
    if (scheme == 0) {
      const double drift = c[3] - c[4] - 0.5 * c[5] * c[5];
      ca = (float)(drift * dt * kLog2e);
      cb = (float)(c[5] * sq * kLog2e);
    } else {
      ca = (float)((c[3] - c[4]) * dt);
      cb = (float)(c[5] * sq);
    }
    double ca64, cb64;
    if (scheme == 0) {
      const double drift = c[3] - c[4] - 0.5 * c[5] * c[5];
      ca64 = drift * dt * 369.3299304675746; /* smc_math.h kExpUnit = 256 / ln 2 */
      cb64 = c[5] * sq * 369.3299304675746;
    } else {
      ca64 = (c[3] - c[4]) * dt;
      cb64 = c[5] * sq;
    }
    const float x0 = (float)c[0];
    const uint64_t ordinal = (uint64_t)(ordinal0 + b);
    const int64_t groups = (P + GROUP - 1) / GROUP;
#pragma omp parallel
    {
      double* z = (double*)malloc(sizeof(double) * (size_t)(T + 1) * GROUP);
#pragma omp for schedule(static)
      for (int64_t gi = 0; gi < groups; ++gi) {
        group_normals(seed, ordinal, (uint64_t)gi, T, 0, z);
        for (int j = 0; j < GROUP; ++j) {
          const int64_t p = gi * GROUP + j;
          if (p >= P) break;
          float x = x0;
          double x64 = c[0];
          for (int t = 0; t < T; ++t) {
            const float zt = (float)z[(int64_t)t * GROUP + j];
            if (step64) {
              const double y = fma(cb64, (double)zt, ca64);
              x64 = scheme == 0 ? oracle_mul_exp2s_f64(x64, y) : fabs(fma(x64, y, x64));
              x = (float)x64;
            } else if (scheme == 0) {
              x = x * exp2_any(fmaf(cb, zt, ca));
            } else {
              x = fabsf(fmaf(x, fmaf(cb, zt, ca), x));
            }
            X[(int64_t)t * P + p] = x;
          }
        }
      }
      free(z);
    }
    if (paths) memcpy(paths + b * (int64_t)T * P, X, sizeof(float) * (size_t)T * (size_t)P);
    if (terminal) memcpy(terminal + b * P, X + (int64_t)(T - 1) * P, sizeof(float) * (size_t)P);
    const int64_t span = slice_paths > 0 && slice_paths < P ? slice_paths : P;
    const int sliced = span < P;
    for (int t = 0; t < T; ++t) rowsum[b * T + t] = 0.0;
    for (int64_t p_begin = 0; p_begin < P; p_begin += span) {
      const int64_t p_end = p_begin + span < P ? p_begin + span : P;
      /* per lane: sequential over the slice's chunks of f32 4-path partial sums, in f64 */
      memset(lane_acc, 0, sizeof(double) * (size_t)lanes * (size_t)T);
      for (int64_t chunk = p_begin; chunk < p_end; chunk += chunk_paths)
        for (int lane = 0; lane < lanes; ++lane) {
          const int64_t p0 = chunk + (int64_t)K_PPL * lane;
          for (int t = 0; t < T; ++t) {
            float part = 0.0f;
            for (int j = 0; j < K_PPL; ++j) part += (p0 + j < p_end) ? X[(int64_t)t * P + p0 + j] : 0.0f;
            lane_acc[(size_t)lane * T + t] += (double)part;
          }
        }
      for (int t = 0; t < T; ++t) {
        double tot = 0.0;
        for (int w = 0; w < waves; ++w) {
          double v[64], nv[64];
          for (int l = 0; l < 64; ++l) v[l] = lane_acc[(size_t)(64 * w + l) * T + t];
          for (int off = 32; off >= 1; off >>= 1) {
            for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
            memcpy(v, nv, sizeof(v));
          }
          tot += v[0];
        }
        if (sliced) rowsum[b * T + t] += tot; /* last arriver: slices 0..W-1 in order from 0.0 */
        else rowsum[b * T + t] = tot;
      }
    }
  }
  free(lane_acc);
  free(X);
}

/* gbm.hip use_fft / fft_row: power-of-two N in 2..2048 takes the radix-2 DIT FFT (bit-reversed
 * load, stage len = 2..N, butterfly t = x[i1] (cs - i sn)[(j mod h) N/len] with 4 products and 2
 * sums, x[i1] = x[i0] - t, x[i0] = x[i0] + t); other N the direct DFT chains. */
static int use_fft(int N) { return N >= 2 && (N & (N - 1)) == 0 && N <= 2048; }

static void fft_real(const double* avg, const double* cs, const double* sn, int N, double* xr, double* xi) {
  int logN = 0;
  while ((1 << logN) < N) ++logN;
  for (int n = 0; n < N; ++n) {
    unsigned r = 0;
    for (int bit = 0; bit < logN; ++bit) r |= (unsigned)((n >> bit) & 1) << (logN - 1 - bit);
    xr[r] = avg[n];
    xi[r] = 0.0;
  }
  for (int s = 1; s <= logN; ++s) {
    const int h = 1 << (s - 1), shift = logN - s;
    for (int j = 0; j < N / 2; ++j) {
      const int pos = j & (h - 1);
      const int i0 = ((j >> (s - 1)) << s) + pos, i1 = i0 + h;
      const double wr = cs[pos << shift], wi = -sn[pos << shift];
      const double ar = xr[i1], ai = xi[i1];
      const double tr = ar * wr - ai * wi;
      const double ti = ar * wi + ai * wr;
      const double br = xr[i0], bi = xi[i0];
      xr[i1] = br - tr;
      xi[i1] = bi - ti;
      xr[i0] = br + tr;
      xi[i0] = bi + ti;
    }
  }
}

/* targets: [B][N] interleaved complex64 (re, im) */
/* slices: workgroups per contract of the sliced resident_kernel (gbm.hip, smc_train_step with
 * P > 65,536): slice s holds batch rows [s M/slices, (s+1) M/slices); its items sum only those rows,
 * its column sums add the G groups in order from 0.0, and the M-mean adds the slices' column sums
 * in slice order from 0.0.  slices = 1 is the whole-contract order (0.0 + x == x). */
void oracle_kernel_cf(const double* contracts, int64_t B, int32_t N, int32_t M, int32_t normalize, int32_t wg,
                      int32_t slices, const float* terminal, const double* terminal_sum, float* targets) {
  const int lanes = wg > 0 ? wg : K_THREADS;  /* G = lanes / column quads (resident_kernel: 4096 / N) */
  const int W = slices > 1 ? slices : 1;
  const int Ms = M / W;
  const int64_t P = (int64_t)N * M;
  /* gbm.hip cf_targets_contract: with N % 4 == 0 a thread owns 4 adjacent columns (16-B loads),
   * so the m-groups per column are counted over N/4 column quads */
  const int cols = (N % 4 == 0 && P < ((int64_t)1 << 29)) ? N / 4 : N;
  const int G = cols <= lanes ? lanes / cols : 1;
  const int items = N * G;
  double* part = (double*)malloc(sizeof(double) * (size_t)items);
  double* avg = (double*)malloc(sizeof(double) * (size_t)N);
  double* cs = (double*)malloc(sizeof(double) * (size_t)N);
  double* sn = (double*)malloc(sizeof(double) * (size_t)N);
  double* xr = (double*)malloc(sizeof(double) * (size_t)N);
  double* xi = (double*)malloc(sizeof(double) * (size_t)N);
  for (int j = 0; j < N; ++j) twiddle(j, N, &sn[j], &cs[j]);
  for (int64_t b = 0; b < B; ++b) {
    const double* c = contracts + 6 * b;
    const float Tm = (float)c[2];
    const float F = (float)c[0] * exp_any((float)(c[3] - c[4]) * Tm);
    const float df = exp_any((float)(-c[3]) * Tm);
    const float s = normalize ? F / (float)(terminal_sum[b] / (double)P) : 1.0f;
    const float K = (float)c[1];
    const float* row = terminal + b * P;
    for (int n = 0; n < N; ++n) avg[n] = 0.0;
    for (int sl = 0; sl < W; ++sl) {
      const int m0 = sl * Ms, m1 = sl + 1 == W ? M : (sl + 1) * Ms;
      for (int item = 0; item < items; ++item) {
        const int n = item % N, g = item / N;
        double sum = 0.0;
        for (int m = m0 + g; m < m1; m += G) {
          const float xs = row[(int64_t)m * N + n] * s;
          const float diff = K - xs;
          const float pay = df * (diff > 0.0f ? diff : 0.0f);
          sum += (double)pay;
        }
        part[item] = sum;
      }
      for (int n = 0; n < N; ++n) {
        double col = 0.0;
        if (lanes == 1024 && W == 1 && N % 4 == 0 && N <= 1024 && G * N == 4096) {
          /* resident_kernel's column_sums_tree (gbm.hip, round 4): R = 1024 / N partials, partial k adds
           * groups k, k + R, k + 2R, k + 3R in order from 0.0; N < 64: the 64 / N partials of wave w
           * (k = w 64/N + j) by a butterfly over j (offsets 32/N, ..., 1: lane offsets 32, ..., N), then the
           * 16 wave sums in order; N >= 64: the R partials in k order */
          const int R = 1024 / N;
          double pk[1024];
          for (int k = 0; k < R; ++k) {
            double p = 0.0;
            for (int u = 0; u < 4; ++u) p += part[(k + u * R) * N + n];
            pk[k] = p;
          }
          if (N < 64) {
            const int per = 64 / N;
            for (int w = 0; w < 16; ++w) {
              double v[64], nv[64];
              for (int j = 0; j < per; ++j) v[j] = pk[w * per + j];
              for (int off = per / 2; off >= 1; off >>= 1) {
                for (int j = 0; j < per; ++j) nv[j] = v[j] + v[j ^ off];
                memcpy(v, nv, sizeof(double) * (size_t)per);
              }
              col += v[0];
            }
          } else {
            for (int k = 0; k < R; ++k) col += pk[k];
          }
        } else {
          for (int g = 0; g < G; ++g) col += part[g * N + n];
        }
        avg[n] += col; /* slices in order from 0.0 */
      }
    }
    for (int n = 0; n < N; ++n) avg[n] = avg[n] / (double)M;
    float* out = targets + 2 * b * N;
    if (use_fft(N)) {
      fft_real(avg, cs, sn, N, xr, xi);
      for (int k = 0; k <= N / 2; ++k) {
        out[2 * k] = (float)xr[k];
        out[2 * k + 1] = (float)xi[k];
        if (k != 0 && 2 * k != N) {
          out[2 * (N - k)] = (float)xr[k];
          out[2 * (N - k) + 1] = (float)(-xi[k]);
        }
      }
      continue;
    }
    for (int k = 0; k <= N / 2; ++k) {
      double re = 0.0, im = 0.0;
      int idx = 0;
      for (int n = 0; n < N; ++n) {
        re = fma(avg[n], cs[idx], re);
        im = fma(-avg[n], sn[idx], im);
        idx += k;
        if (idx >= N) idx -= N;
      }
      out[2 * k] = (float)re;
      out[2 * k + 1] = (float)im;
      if (k != 0 && 2 * k != N) {
        out[2 * (N - k)] = (float)re;
        out[2 * (N - k) + 1] = (float)(-im);
      }
    }
  }
  free(xr);
  free(xi);
  free(part);
  free(avg);
  free(cs);
  free(sn);
}

/* ======================================================================================
 * BASKET (extension, BASELINE.json configs[4]): exact restatement of the f32 HIP basket engine
 * (spectralmc_amd/csrc/basket.hip) in portable math.  Per-asset dynamics follow the reference
 * log-Euler recursion (gbm.py:224-257) and normalisation (gbm.py:428-440); the payoff is the
 * equal-weight basket put; targets as gbm_trainer.py:806-817 (batch mean, then N-point DFT).
 * contracts: [B][3A+4] (K, T, r, rho, X0[A], d[A], v[A]).  paths: [B][A][T][P] or NULL;
 * terminal_sum: [B][A]; targets: [B][N] interleaved complex64.
 * ====================================================================================== */
#define B_MAX_ASSETS 8

static void basket_cholesky(int A, double rho, double* L) {
  for (int i = 0; i < A; ++i)
    for (int k = 0; k <= i; ++k) {
      double s = i == k ? 1.0 : rho;
      for (int m = 0; m < k; ++m) s = s - L[i * B_MAX_ASSETS + m] * L[k * B_MAX_ASSETS + m];
      L[i * B_MAX_ASSETS + k] = i == k ? sqrt(s > 0.0 ? s : 0.0) : s / L[k * B_MAX_ASSETS + k];
    }
}

void oracle_basket_cholesky(int32_t A, double rho, double* L /* [8][8] */) { basket_cholesky(A, rho, L); }

/* wg: lanes of the engine workgroup whose reduction orders to follow (512: basket_kernel /
 * basket_cf_kernel; 1024: basket_resident_kernel); slices: workgroups per contract of
 * basket_resident_kernel (slice s holds paths [s P/W, (s+1) P/W) = batch rows [s M/W, (s+1) M/W);
 * its terminal sums and column sums are reduced like a whole contract's and the W of them are
 * added in slice order from 0.0).  wg = 512, slices = 1 is the basket_kernel order. */
void oracle_basket_kernel(const double* contracts, int64_t B, int32_t A, int32_t T, int32_t N, int32_t M,
                          uint64_t seed, int64_t ordinal0, int32_t normalize, int32_t wg, int32_t slices,
                          float* paths, double* terminal_sum, float* targets) {
  const double kLog2e = 1.4426950408889634;
  const int64_t P = (int64_t)N * M;
  const int width = 3 * A + 4;
  const int lanes = wg > 0 ? wg : K_THREADS;
  const int waves = lanes / 64;
  const int64_t chunk_paths = (int64_t)K_PPL * lanes;
  const int W = slices > 1 ? slices : 1;
  const int64_t span = P / W;
  const int Ms = M / W;
  float* X = (float*)malloc(sizeof(float) * (size_t)A * (size_t)P); /* terminal rows [A][P] */
  double* lane_acc = (double*)malloc(sizeof(double) * (size_t)lanes * (size_t)A);
  const int cols = N / 4;
  const int G = cols <= lanes ? lanes / cols : 1;
  double* part = (double*)malloc(sizeof(double) * (size_t)N * (size_t)G);
  double* avg = (double*)malloc(sizeof(double) * (size_t)N);
  double* cs = (double*)malloc(sizeof(double) * (size_t)N);
  double* sn = (double*)malloc(sizeof(double) * (size_t)N);
  double* fxr = (double*)malloc(sizeof(double) * (size_t)N);
  double* fxi = (double*)malloc(sizeof(double) * (size_t)N);
  for (int j = 0; j < N; ++j) twiddle(j, N, &sn[j], &cs[j]);
  for (int64_t b = 0; b < B; ++b) {
    const double* c = contracts + (int64_t)width * b;
    const double K = c[0], Tm = c[1], r = c[2], rho = c[3];
    double L[B_MAX_ASSETS * B_MAX_ASSETS];
    basket_cholesky(A, rho, L);
    const double dt = Tm / (double)T;
    const double sq = sqrt(dt);
    /* y_i = a_i + sum_{k<=i} (b_i L_ik) z_k, b_i L_ik rounded once from f64 */
    float ca[B_MAX_ASSETS], x0[B_MAX_ASSETS], Lb[B_MAX_ASSETS][B_MAX_ASSETS];
    for (int i = 0; i < A; ++i) {
      const double v = c[4 + 2 * A + i], d = c[4 + A + i];
      const double drift = r - d - 0.5 * v * v;
      ca[i] = (float)(drift * dt * kLog2e);
      const double bi = v * sq * kLog2e;
      x0[i] = (float)c[4 + i];
      for (int k = 0; k <= i; ++k) Lb[i][k] = (float)(bi * L[i * B_MAX_ASSETS + k]);
    }
    const uint64_t ordinal = (uint64_t)(ordinal0 + b);
    const int64_t groups = P / GROUP;
#pragma omp parallel for schedule(static)
    for (int64_t gi = 0; gi < groups; ++gi) {
      mwc64x g;
      path_stream(seed, ordinal, (uint64_t)gi, &g);
      float x[B_MAX_ASSETS][GROUP];
      for (int i = 0; i < A; ++i)
        for (int j = 0; j < GROUP; ++j) x[i][j] = x0[i];
      for (int t = 0; t < T; ++t) {
        for (int j = 0; j < GROUP; ++j) {
          float z[B_MAX_ASSETS + 1];
          for (int k = 0; k < A; k += 2) {
            double z0, z1;
            normal_pair(&g, 0, &z0, &z1);
            z[k] = (float)z0;
            z[k + 1] = (float)z1;
          }
          for (int i = 0; i < A; ++i) {
            float y = ca[i];
            for (int k = 0; k <= i; ++k) y = fmaf(Lb[i][k], z[k], y);
            x[i][j] = x[i][j] * exp2_any(y);
          }
        }
        if (paths)
          for (int i = 0; i < A; ++i)
            for (int j = 0; j < GROUP; ++j)
              paths[((b * A + i) * T + t) * P + gi * GROUP + j] = x[i][j];
      }
      for (int i = 0; i < A; ++i)
        for (int j = 0; j < GROUP; ++j) X[(int64_t)i * P + gi * GROUP + j] = x[i][j];
    }
    /* terminal sums: per slice, per lane over the slice's chunks (f32 4-path partials), wave
     * butterfly, waves in order; slices added in order */
    double tot[B_MAX_ASSETS];
    for (int i = 0; i < A; ++i) tot[i] = 0.0;
    for (int sl = 0; sl < W; ++sl) {
      memset(lane_acc, 0, sizeof(double) * (size_t)lanes * (size_t)A);
      for (int64_t chunk = sl * span; chunk < (sl + 1) * span; chunk += chunk_paths)
        for (int lane = 0; lane < lanes; ++lane)
          for (int i = 0; i < A; ++i) {
            float p = 0.0f;
            for (int j = 0; j < K_PPL; ++j) p += X[(int64_t)i * P + chunk + (int64_t)K_PPL * lane + j];
            lane_acc[(size_t)lane * A + i] += (double)p;
          }
      for (int i = 0; i < A; ++i) {
        double st = 0.0;
        for (int w = 0; w < waves; ++w) {
          double v[64], nv[64];
          for (int l = 0; l < 64; ++l) v[l] = lane_acc[(size_t)(64 * w + l) * A + i];
          for (int off = 32; off >= 1; off >>= 1) {
            for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
            memcpy(v, nv, sizeof(v));
          }
          st += v[0];
        }
        tot[i] = W > 1 ? tot[i] + st : st;
      }
    }
    for (int i = 0; i < A; ++i)
      if (terminal_sum) terminal_sum[b * A + i] = tot[i];
    /* payoff + per-column batch sums (thread item (q, g): columns 4q..4q+3, m = g, g + G, ...) */
    const float Tf = (float)Tm;
    const float df = exp_any((float)(-r) * Tf);
    const float Kf = (float)K;
    const float wA = (float)(1.0 / A);
    float sc[B_MAX_ASSETS];
    for (int i = 0; i < A; ++i) {
      const float F = (float)c[4 + i] * exp_any((float)(r - c[4 + A + i]) * Tf);
      sc[i] = normalize ? F / (float)(tot[i] / (double)P) : 1.0f;
    }
    for (int n = 0; n < N; ++n) avg[n] = 0.0;
    for (int sl = 0; sl < W; ++sl) {
      const int m0 = sl * Ms, m1 = (sl + 1) * Ms;
      for (int item = 0; item < cols * G; ++item) {
        const int q = item % cols, gg = item / cols;
        double sum[4] = {0.0, 0.0, 0.0, 0.0};
        for (int m = m0 + gg; m < m1; m += G)
          for (int e = 0; e < 4; ++e) {
            float bs = 0.0f;
            for (int i = 0; i < A; ++i) bs = bs + X[(int64_t)i * P + (int64_t)m * N + 4 * q + e] * sc[i];
            const float diff = Kf - bs * wA;
            sum[e] += (double)(df * (diff > 0.0f ? diff : 0.0f));
          }
        for (int e = 0; e < 4; ++e) part[gg * N + 4 * q + e] = sum[e];
      }
      for (int n = 0; n < N; ++n) {
        double t2 = 0.0;
        for (int gg = 0; gg < G; ++gg) t2 += part[gg * N + n];
        avg[n] = W > 1 ? avg[n] + t2 : t2; /* slices in order from 0.0 */
      }
    }
    for (int n = 0; n < N; ++n) avg[n] = avg[n] / (double)M;
    float* out = targets + 2 * b * N;
    if (lanes == 1024 && use_fft(N)) { /* basket_resident_kernel: fft_row as resident_kernel */
      fft_real(avg, cs, sn, N, fxr, fxi);
      for (int k = 0; k <= N / 2; ++k) {
        out[2 * k] = (float)fxr[k];
        out[2 * k + 1] = (float)fxi[k];
        if (k != 0 && 2 * k != N) {
          out[2 * (N - k)] = (float)fxr[k];
          out[2 * (N - k) + 1] = (float)(-fxi[k]);
        }
      }
      continue;
    }
    for (int k = 0; k <= N / 2; ++k) {
      double re = 0.0, im = 0.0;
      int idx = 0;
      for (int n = 0; n < N; ++n) {
        re = fma(avg[n], cs[idx], re);
        im = fma(-avg[n], sn[idx], im);
        idx += k;
        if (idx >= N) idx -= N;
      }
      out[2 * k] = (float)re;
      out[2 * k + 1] = (float)im;
      if (k != 0 && 2 * k != N) {
        out[2 * (N - k)] = (float)re;
        out[2 * (N - k) + 1] = (float)(-im);
      }
    }
  }
  free(fxr);
  free(fxi);
  free(part);
  free(avg);
  free(cs);
  free(sn);
  free(lane_acc);
  free(X);
}
