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
 *             seeds xoshiro128** (Blackman & Vigna) per (contract ordinal, path); Box-Muller
 *             in double precision, rounded to the sim dtype like the reference's normal array.
 *   paths     reference src/spectralmc/gbm.py:241-257: the Numba kernel's arguments are Python
 *             floats, so the recursion runs in f64 and only the stores round to the sim dtype.
 *             LOG_EULER:    X *= exp((r - d - v^2/2) dt + v dW),  dW = Z sqrt(dt)
 *             SIMPLE_EULER: X += (r - d) X dt + v X dW;  X = |X|
 *   row sums  reference gbm.py:437 (cp.mean over the P stored values): f64 sum of the stored
 *             values, divided by P by the caller.
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

typedef struct {
  uint32_t s[4];
} xoshiro128;

static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

/* xoshiro128** 1.1, reference implementation order. */
static inline uint32_t xoshiro_next(xoshiro128* g) {
  uint32_t* s = g->s;
  const uint32_t result = rotl32(s[1] * 5u, 7) * 9u;
  const uint32_t t = s[1] << 9;
  s[2] ^= s[0];
  s[3] ^= s[1];
  s[1] ^= s[2];
  s[0] ^= s[3];
  s[2] ^= t;
  s[3] = rotl32(s[3], 11);
  return result;
}

static void path_stream(uint64_t seed, uint64_t ordinal, uint64_t path, xoshiro128* g) {
  const uint32_t ctr[4] = {(uint32_t)path, (uint32_t)(path >> 32), (uint32_t)ordinal, (uint32_t)(ordinal >> 32)};
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  oracle_philox4x32_10(ctr, key, g->s);
  if ((g->s[0] | g->s[1] | g->s[2] | g->s[3]) == 0u) g->s[0] = 1u;
}

/* One Box-Muller pair; f32 streams use 24-bit uniforms, f64 streams 32-bit ones. */
static void normal_pair(xoshiro128* g, int is_f64, double* z0, double* z1) {
  const uint32_t a = xoshiro_next(g), b = xoshiro_next(g);
  double u1, u2;
  if (is_f64) {
    u1 = ((double)a + 1.0) * 0x1p-32;
    u2 = (double)b * 0x1p-32;
  } else {
    u1 = (double)((a >> 8) + 1u) * 0x1p-24;
    u2 = (double)(b >> 8) * 0x1p-24;
  }
  const double r = sqrt(-2.0 * log(u1));
  const double th = 6.283185307179586476925286766559 * u2;
  double zc = r * cos(th), zs = r * sin(th);
  if (!is_f64) {  /* the reference keeps normals in the sim dtype (async_normals.py:215) */
    zc = (double)(float)zc;
    zs = (double)(float)zs;
  }
  *z0 = zc;
  *z1 = zs;
}

/* normals[t][p] of contract ordinal `ordinal` (dtype 0: f32 out, 1: f64 out). */
void oracle_normals(uint64_t seed, int64_t ordinal, int32_t rows, int64_t cols, int32_t dtype, void* out) {
#pragma omp parallel for schedule(static)
  for (int64_t p = 0; p < cols; ++p) {
    xoshiro128 g;
    path_stream(seed, (uint64_t)ordinal, (uint64_t)p, &g);
    double z0 = 0, z1 = 0;
    for (int t = 0; t < rows; ++t) {
      if ((t & 1) == 0) normal_pair(&g, dtype == 1, &z0, &z1);
      const double z = (t & 1) ? z1 : z0;
      if (dtype == 1)
        ((double*)out)[(int64_t)t * cols + p] = z;
      else
        ((float*)out)[(int64_t)t * cols + p] = (float)z;
    }
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
#pragma omp parallel
    {
      double* local = (double*)calloc((size_t)T, sizeof(double));
#pragma omp for schedule(static)
      for (int64_t p = 0; p < P; ++p) {
        xoshiro128 g;
        path_stream(seed, ordinal, (uint64_t)p, &g);
        double X = X0, z0 = 0, z1 = 0;
        for (int t = 0; t < T; ++t) {
          if ((t & 1) == 0) normal_pair(&g, is_f64, &z0, &z1);
          const double dW = ((t & 1) ? z1 : z0) * sqrt_dt;
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
