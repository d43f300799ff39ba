// Scrambled Sobol contract generator, bit-exact with the SciPy engine the reference
// draws from (reference src/spectralmc/sobol_sampler.py:192 `Sobol(d, scramble=True,
// seed=config.seed)`, :197 `fast_forward(skip)`, :238-239 `random(n)` then
// `lower + (upper - lower) * raw`).
//
// Host side: SciPy seeds its scramble from numpy's default_rng(seed) (SeedSequence ->
// PCG64, XSL-RR output) and consumes `integers(2)` draws: first d*30 bits for the
// digital shift, then d*30*30 bits for the lower-triangular LMS matrices.  We restate
// that bit stream (numpy's published algorithms), build the Joe-Kuo direction numbers,
// apply the LMS scramble, and keep (shift, sv) per dimension.
//
// Device side: point n is x = shift ^ XOR_{c : bit c of gray(n)} sv[c] — direct index,
// no sequential dependency, so any batch / rank / graph replay can draw its own slice.

#include <cmath>
#include <cstring>
#include <new>

#include "smc_internal.h"
#include "smc_sobol.h"
#include "sobol_dirnums.h"

#pragma clang fp contract(off)  // numpy rounds (upper - lower) * raw and + lower separately

namespace {

using u128 = unsigned __int128;

// ---- numpy SeedSequence (pool of 4 x u32) --------------------------------------
constexpr uint32_t kInitA = 0x43b0d7e5u, kMultA = 0x931e8875u;
constexpr uint32_t kInitB = 0x8b51f9ddu, kMultB = 0x58f38dedu;
constexpr uint32_t kMixL = 0xca01f9ddu, kMixR = 0x4973f715u;

struct SeedPool {
  uint32_t pool[4];
  uint32_t hash_const;

  uint32_t hashmix(uint32_t value) {
    value ^= hash_const;
    hash_const *= kMultA;
    value *= hash_const;
    return value ^ (value >> 16);
  }
  static uint32_t mix(uint32_t x, uint32_t y) {
    uint32_t r = kMixL * x - kMixR * y;
    return r ^ (r >> 16);
  }

  explicit SeedPool(uint64_t seed) : hash_const(kInitA) {
    // An int seed is split into little-endian u32 words; 0 still gives one word.
    uint32_t words[2];
    int nwords = 0;
    uint64_t s = seed;
    do {
      words[nwords++] = static_cast<uint32_t>(s);
      s >>= 32;
    } while (s != 0);
    for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < nwords ? words[i] : 0u);
    for (int src = 0; src < 4; ++src)
      for (int dst = 0; dst < 4; ++dst)
        if (src != dst) pool[dst] = mix(pool[dst], hashmix(pool[src]));
  }

  // generate_state(n_words, uint32)
  void generate(uint32_t* out, int n_words) const {
    uint32_t hc = kInitB;
    for (int i = 0; i < n_words; ++i) {
      uint32_t v = pool[i % 4];
      v ^= hc;
      hc *= kMultB;
      v *= hc;
      out[i] = v ^ (v >> 16);
    }
  }
};

// ---- numpy PCG64 (128-bit LCG, XSL-RR 64-bit output, 32-bit halves low first) ----
struct Pcg64 {
  u128 state, inc;
  bool has_half = false;
  uint32_t half = 0;

  static constexpr u128 kMult =
      (static_cast<u128>(2549297995355413924ULL) << 64) | 4865540595714422341ULL;

  explicit Pcg64(uint64_t seed) {
    uint32_t w[8];
    SeedPool(seed).generate(w, 8);
    uint64_t s[4];
    for (int i = 0; i < 4; ++i) s[i] = static_cast<uint64_t>(w[2 * i]) | (static_cast<uint64_t>(w[2 * i + 1]) << 32);
    u128 initstate = (static_cast<u128>(s[0]) << 64) | s[1];
    u128 initseq = (static_cast<u128>(s[2]) << 64) | s[3];
    state = 0;
    inc = (initseq << 1) | 1u;
    step();
    state += initstate;
    step();
  }
  void step() { state = state * kMult + inc; }
  uint64_t next64() {
    step();
    uint64_t hi = static_cast<uint64_t>(state >> 64), lo = static_cast<uint64_t>(state);
    unsigned rot = static_cast<unsigned>(state >> 122);
    uint64_t x = hi ^ lo;
    return (x >> rot) | (x << ((64 - rot) & 63));
  }
  uint32_t next32() {
    if (has_half) {
      has_half = false;
      return half;
    }
    uint64_t v = next64();
    has_half = true;
    half = static_cast<uint32_t>(v >> 32);
    return static_cast<uint32_t>(v);
  }
  // Generator.integers(2, dtype=uint32): Lemire with range 1 never rejects -> top bit.
  uint32_t bit() { return next32() >> 31; }
};

// Joe-Kuo direction numbers v[d][j] (integer, scaled so bit (bits-1-j) leads column j).
void direction_numbers(int dim, uint32_t v[][SMC_SOBOL_BITS]) {
  constexpr int bits = SMC_SOBOL_BITS;
  for (int j = 0; j < bits; ++j) v[0][j] = 1;
  for (int d = 1; d < dim; ++d) {
    const uint32_t poly = smc_sobol_poly[d];
    int deg = 0;
    while ((poly >> (deg + 1)) != 0) ++deg;  // floor(log2(poly))
    for (int j = 0; j < deg; ++j) v[d][j] = smc_sobol_vinit[d][j];
    for (int j = deg; j < bits; ++j) {
      uint32_t nv = v[d][j - deg];
      uint32_t pw = 1;
      for (int k = 0; k < deg; ++k) {
        pw <<= 1;
        if ((poly >> (deg - 1 - k)) & 1u) nv ^= pw * v[d][j - k - 1];
      }
      v[d][j] = nv;
    }
  }
  for (int j = 0; j < bits; ++j)
    for (int d = 0; d < dim; ++d) v[d][j] <<= (bits - 1 - j);
}

void gray_point(const smc_sobol& h, uint64_t n, double* out) {
  const uint64_t g = n ^ (n >> 1);
  for (int d = 0; d < h.dim; ++d) {
    uint32_t x = h.shift[d];
    for (int c = 0; c < SMC_SOBOL_BITS; ++c)
      if ((g >> c) & 1u) x ^= h.sv[d * SMC_SOBOL_BITS + c];
    out[d] = static_cast<double>(x) * 0x1p-30;
  }
}

// ---- device draw ---------------------------------------------------------------
__global__ void sobol_draw_kernel(const uint32_t* __restrict__ tables, int dim,
                                  const int64_t* __restrict__ index_dev, int64_t index0,
                                  int64_t n, const double* __restrict__ lower,
                                  const double* __restrict__ upper, double* __restrict__ out,
                                  float* __restrict__ out_f32) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t idx = static_cast<uint64_t>((index_dev ? *index_dev : 0) + index0 + i);
  for (int d = 0; d < dim; ++d) {
    const double val = smc::sobol_coord(tables, dim, d, idx, lower, upper);
    out[i * dim + d] = val;
    if (out_f32) out_f32[i * dim + d] = static_cast<float>(val);
  }
}

}  // namespace

extern "C" {
#pragma GCC visibility push(default)

int32_t smc_sobol_create(int32_t dim, uint64_t seed, uint64_t skip, smc_sobol** out) {
  if (!out) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_create: out is NULL");
  *out = nullptr;
  if (dim < 1 || dim > SMC_SOBOL_MAXDIM)
    return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_create: dim must be in [1, 64]");
  if (seed >> 63) return smc::fail(SMC_ERR_SEED_OUT_OF_RANGE, "smc_sobol_create: seed >= 2^63");
  if (skip > (1ull << SMC_SOBOL_BITS))
    return smc::fail(SMC_ERR_SEQUENCE_EXHAUSTED, "smc_sobol_create: skip beyond 2^30 points");

  smc_sobol* h = new (std::nothrow) smc_sobol();
  if (!h) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_create: out of host memory");
  h->dim = dim;
  h->cursor = skip;

  static thread_local uint32_t v[SMC_SOBOL_MAXDIM][SMC_SOBOL_BITS];
  direction_numbers(dim, v);

  Pcg64 rng(seed);
  constexpr int bits = SMC_SOBOL_BITS;
  for (int d = 0; d < dim; ++d) {
    uint32_t s = 0;
    for (int j = 0; j < bits; ++j) s |= rng.bit() << j;
    h->shift[d] = s;
  }
  // ltm[d][p][k] drawn row-major; keep k < p, force the diagonal to 1.
  static thread_local uint8_t ltm[SMC_SOBOL_MAXDIM][bits][bits];
  for (int d = 0; d < dim; ++d)
    for (int p = 0; p < bits; ++p)
      for (int k = 0; k < bits; ++k) {
        const uint32_t b = rng.bit();
        ltm[d][p][k] = (k < p) ? static_cast<uint8_t>(b) : (k == p ? 1 : 0);
      }
  // sv[d][j] bit (bits-1-p) = parity( sum_k ltm[d][p][k] * bit (bits-1-k) of v[d][j] ).
  for (int d = 0; d < dim; ++d)
    for (int j = 0; j < bits; ++j) {
      const uint32_t vdj = v[d][j];
      uint32_t acc = 0;
      for (int p = 0; p < bits; ++p) {
        uint32_t par = 0;
        for (int k = 0; k <= p; ++k) par ^= ltm[d][p][k] & ((vdj >> (bits - 1 - k)) & 1u);
        acc |= par << (bits - 1 - p);
      }
      h->sv[d * bits + j] = acc;
    }

  *out = h;
  return SMC_OK;
}

void smc_sobol_destroy(smc_sobol* h) { delete h; }

int32_t smc_sobol_export_tables(const smc_sobol* h, uint32_t* tables) {
  if (!h || !tables) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_export_tables: NULL argument");
  std::memcpy(tables, h->shift, h->dim * sizeof(uint32_t));
  std::memcpy(tables + h->dim, h->sv, static_cast<size_t>(h->dim) * SMC_SOBOL_BITS * sizeof(uint32_t));
  return SMC_OK;
}

int32_t smc_sobol_state(const smc_sobol* h, uint32_t* shift, uint32_t* sv, uint64_t* cursor) {
  if (!h) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_state: NULL handle");
  if (shift) std::memcpy(shift, h->shift, h->dim * sizeof(uint32_t));
  if (sv) std::memcpy(sv, h->sv, static_cast<size_t>(h->dim) * SMC_SOBOL_BITS * sizeof(uint32_t));
  if (cursor) *cursor = h->cursor;
  return SMC_OK;
}

int32_t smc_sobol_fast_forward(smc_sobol* h, uint64_t n) {
  if (!h) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_fast_forward: NULL handle");
  if (h->cursor + n > (1ull << SMC_SOBOL_BITS))
    return smc::fail(SMC_ERR_SEQUENCE_EXHAUSTED, "smc_sobol_fast_forward: beyond 2^30 points");
  h->cursor += n;
  return SMC_OK;
}

int32_t smc_sobol_random_host(smc_sobol* h, int64_t n, double* out) {
  if (!h || (n > 0 && !out)) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_random_host: NULL argument");
  if (n < 0) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_random_host: n < 0");
  if (h->cursor + static_cast<uint64_t>(n) > (1ull << SMC_SOBOL_BITS))
    return smc::fail(SMC_ERR_SEQUENCE_EXHAUSTED, "smc_sobol_random_host: at most 2^30 points");
  for (int64_t i = 0; i < n; ++i) gray_point(*h, h->cursor + i, out + i * h->dim);
  h->cursor += n;
  return SMC_OK;
}

int32_t smc_sobol_draw(const uint32_t* tables_dev, int32_t dim, const int64_t* index_dev, int64_t index0,
                       int64_t n, const double* lower_dev, const double* upper_dev, double* out_f64,
                       float* out_f32, void* stream) {
  if (!tables_dev || !lower_dev || !upper_dev || !out_f64)
    return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_draw: NULL argument");
  if (dim < 1 || dim > SMC_SOBOL_MAXDIM)
    return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_draw: dim must be in [1, 64]");
  if (n < 0 || index0 < 0) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sobol_draw: negative size");
  if (n == 0) return SMC_OK;
  constexpr int threads = 256;
  const unsigned blocks = static_cast<unsigned>((n + threads - 1) / threads);
  smc::launch_aux(sobol_draw_kernel, dim3(blocks), dim3(threads), 0, smc::as_stream(stream),
                     tables_dev, dim, index_dev, index0, n, lower_dev, upper_dev, out_f64, out_f32);
  return smc::check_launch("sobol_draw_kernel");
}

#pragma GCC visibility pop
}  // extern "C"
