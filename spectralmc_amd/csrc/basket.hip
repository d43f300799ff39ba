// Correlated multi-asset GBM engine for gfx950 (BASELINE.json configs[4]: "multi-asset
// correlated GBM, 4 assets, Cholesky in LDS"): A assets per contract, equicorrelated
// Brownian drivers, equal-weight basket put, CF training targets.
//
// This is an extension of the reference's single-asset engine; each asset follows the
// reference dynamics (src/spectralmc/gbm.py:224-257, log-Euler) and forward normalisation
// (gbm.py:428-440); the payoff is the builder-defined basket put
//   df_T * max(K - (1/A) sum_i x_i,T * F_i / mean_p(x_i,T), 0)
// and the target is mean_m FFT_N(put.reshape(M, N)) as gbm_trainer.py:806-817.
//
// Contract row (f64, width 3A + 4): K, T, r, rho, X0[0..A), d[0..A), v[0..A).
// Correlation matrix C = (1 - rho) I + rho 11^T, factored C = L L^T once per workgroup in LDS.
//
// Layout: paths [B][A][T][pitch] f32 (STORE_ALL) or [B][A][pitch] (terminal rows only), so each
// asset's block is a single-asset [T][P] matrix.  basket_kernel: one 512-thread workgroup per
// contract; each lane owns 4 consecutive paths of a 2048-path chunk for all A assets and stores
// one dwordx4 per (asset, row).  basket_resident_kernel (the C5 kernel, below): W = P / 4096
// co-resident 1024-thread workgroups per contract keep the terminal rows on chip.
//
// Per lane, per step t, per path j = 0..3: ceil(A/2) Box-Muller pairs from the lane's
// PathStream (smc_rng.h; the same (seed, contract ordinal, group) keying as the single-asset
// engine) -> z[0..A) (an odd A discards the last pair's second normal);
// y_i = a_i + sum_{k<=i} (b_i L_ik) z_k (f32 fma chain in k order, b_i L_ik rounded once from f64);
// x_i *= 2^y_i.  oracle/gbm_oracle.c (oracle_basket_kernel) restates this bit for bit
// in portable math.

#include <cmath>

#pragma clang fp contract(off)

#include "smc_internal.h"
#include "smc_math.h"
#include "smc_rng.h"
#include "smc_device.h"

namespace smc {
namespace {

constexpr int kBThreads = 512;
constexpr int kBWaves = kBThreads / 64;
constexpr int kBPaths = 4;                      // paths per lane
constexpr int kBChunk = kBThreads * kBPaths;    // paths per workgroup pass
constexpr int kMaxAssets = 8;
constexpr double kBLog2e = 1.4426950408889634;

struct BasketArgs {
  const double* contracts;  // [B][3A + 4] of this launch
  int64_t B;
  int32_t T;
  int64_t P;
  int32_t N, M;
  uint64_t seed;
  const int64_t* ordinal_dev;
  int64_t ordinal0;
  int32_t normalize;
  int32_t store_all;
  float* paths;
  int64_t pitch;            // elements between consecutive rows
  double* terminal_sum;     // [B][A] or NULL
  float2* targets;          // [B][N]
};

__device__ __forceinline__ double bwave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// Cholesky-Banachiewicz of the equicorrelation matrix in LDS (f64, one thread; A <= 8).
__device__ void cholesky_equicorr(int A, double rho, double* L) {
  for (int i = 0; i < A; ++i)
    for (int k = 0; k <= i; ++k) {
      double s = i == k ? 1.0 : rho;
      for (int m = 0; m < k; ++m) s = s - L[i * kMaxAssets + m] * L[k * kMaxAssets + m];
      L[i * kMaxAssets + k] = i == k ? sqrt(s > 0.0 ? s : 0.0) : s / L[k * kMaxAssets + k];
    }
}

// Payoff + M-mean + DFT of contract b from its stored terminal rows and their sums tot[A] (in
// LDS): the CF phase of basket_kernel, and all of basket_cf_kernel.
template <int A>
__device__ void basket_cf(const BasketArgs& a, int64_t b, const double* tot, double* part, double* avg,
                          const double* cs, const double* sn) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int N = a.N, M = a.M;
  const int64_t P = a.P;
  const double* c = a.contracts + b * (3 * A + 4);
  const double K = c[0], Tm = c[1], r = c[2];
  const int64_t rows = a.store_all ? a.T : 1;
  const float* cbase = a.paths + b * A * rows * a.pitch;
  // payoff: per-asset forward scale, equal-weight basket, discounted put (f32, asset order)
  const float Tf = static_cast<float>(Tm);
  const float df = math::exp_any(static_cast<float>(-r) * Tf);
  const float Kf = static_cast<float>(K);
  const float wA = static_cast<float>(1.0 / A);
  float sc[A];
#pragma unroll
  for (int i = 0; i < A; ++i) {
    const float F = static_cast<float>(c[4 + i]) * math::exp_any(static_cast<float>(r - c[4 + A + i]) * Tf);
    sc[i] = a.normalize ? F / static_cast<float>(tot[i] / static_cast<double>(P)) : 1.0f;
  }
  __amdgpu_buffer_rsrc_t rs[A];
#pragma unroll
  for (int i = 0; i < A; ++i) {
    const float* trow = cbase + (i * rows + (rows - 1)) * a.pitch;
    rs[i] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(trow), static_cast<short>(0), 0x7fffffff,
                                              0x00020000);
  }
  // thread item (q, g): columns 4q..4q+3, batches m = g, g + G, ... (oracle_basket_kernel order)
  const int cols = N / 4;
  const int G = cols <= kBThreads ? kBThreads / cols : 1;
  const int items = cols * G;
  constexpr int kB = A <= 2 ? 8 : (A <= 4 ? 4 : 2);  // batches in flight per thread
  for (int item = tid; item < items; item += kBThreads) {
    const int q = item % cols, g = item / cols;
    double sum[4] = {0.0, 0.0, 0.0, 0.0};
    for (int m0 = g; m0 < M; m0 += G * kB) {
      v4f v[kB][A];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const int m = m0 + u * G < M ? m0 + u * G : M - 1;
#pragma unroll
        for (int i = 0; i < A; ++i)
          v[u][i] = __builtin_amdgcn_raw_buffer_load_b128(rs[i], (m * N + 4 * q) * 4, 0, 16 /* sc1 */);
      }
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        if (m0 + u * G < M) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float bs = 0.0f;
#pragma unroll
            for (int i = 0; i < A; ++i) bs = bs + v[u][i][e] * sc[i];
            const float diff = Kf - bs * wA;
            sum[e] += static_cast<double>(df * (diff > 0.0f ? diff : 0.0f));
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) part[g * N + 4 * q + e] = sum[e];
  }
  __syncthreads();
  for (int n = tid; n < N; n += kBThreads) {
    double t2 = 0.0;
    for (int g = 0; g < G; ++g) t2 += part[g * N + n];
    avg[n] = t2 / static_cast<double>(M);
  }
  __syncthreads();
  float2* out = a.targets + b * N;
  for (int k = tid; k <= N / 2; k += kBThreads) {
    double re = 0.0, im = 0.0;
    int idx = 0;
    for (int n = 0; n < N; ++n) {
      re = fma(avg[n], cs[idx], re);
      im = fma(-avg[n], sn[idx], im);
      idx += k;
      if (idx >= N) idx -= N;
    }
    out[k] = make_float2(static_cast<float>(re), static_cast<float>(im));
    if (k != 0 && 2 * k != N) out[N - k] = make_float2(static_cast<float>(re), static_cast<float>(-im));
  }
}

template <int A, bool HW, int MODE>  // MODE 0: simulate + CF, 1: simulate only (terminal sums out)
__global__ __launch_bounds__(kBThreads) void basket_kernel(BasketArgs a) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  const int T = a.T, N = a.N;
  const int64_t P = a.P;
  double* Ld = lds;                          // [8][8]
  double* wsum = Ld + kMaxAssets * kMaxAssets;  // [kBWaves][A]
  double* tot = wsum + kBWaves * A;          // [A]
  double* part = tot + A;                    // [max(4 kBThreads, N)]
  double* avg = part + (N > 4 * kBThreads ? N : 4 * kBThreads);  // [N]
  double* cs = avg + N;
  double* sn = cs + N;

  const double* c = a.contracts + b * (3 * A + 4);
  const double Tm = c[1], r = c[2], rho = c[3];
  if (tid == 0) cholesky_equicorr(A, rho, Ld);
  if (MODE == 0)
    for (int j = tid; j < N; j += kBThreads) math::twiddle(j, N, sn[j], cs[j]);
  __syncthreads();

  // per-asset log2-unit coefficients (Stepper of gbm.hip); HW normals come out / sqrt(2 ln 2)
  const double dt = Tm / static_cast<double>(T);
  const double sq = sqrt(dt);
  constexpr double zscale = HW ? PathStream::kNormalScale<true> : 1.0;
  // y_i = a_i + sum_{k <= i} (b_i L_ik) z_k: the volatility coefficient is folded into the factor
  float ca[A], x0[A], Lb[A][A];
#pragma unroll
  for (int i = 0; i < A; ++i) {
    const double v = c[4 + 2 * A + i], d = c[4 + A + i];
    const double drift = r - d - 0.5 * v * v;
    ca[i] = static_cast<float>(drift * dt * kBLog2e);
    const double bi = v * sq * kBLog2e * zscale;
    x0[i] = static_cast<float>(c[4 + i]);
#pragma unroll
    for (int k = 0; k < A; ++k) Lb[i][k] = k <= i ? static_cast<float>(bi * Ld[i * kMaxAssets + k]) : 0.0f;
  }

  const uint64_t ordinal = static_cast<uint64_t>((a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0 + b);
  const int64_t pitch = a.pitch;
  const int64_t rows = a.store_all ? T : 1;
  float* cbase = a.paths + b * A * rows * pitch;
  const uint32_t lane_off = static_cast<uint32_t>(kBPaths * sizeof(float)) * tid;
  double acc[A];
#pragma unroll
  for (int i = 0; i < A; ++i) acc[i] = 0.0;

  for (int64_t chunk = 0; chunk < P; chunk += kBChunk) {
    PathStream s(a.seed, ordinal, static_cast<uint64_t>(chunk / kBPaths + tid));
    float x[A][kBPaths];
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
      for (int j = 0; j < kBPaths; ++j) x[i][j] = x0[i];
    for (int t = 0; t < T; ++t) {
      // path pairs (j, j + 1): draws in path order, then the correlation and the step as packed
      // f32 ops (v_pk_fma_f32 / v_pk_mul_f32; same IEEE results as the scalar ops)
#pragma unroll
      for (int j = 0; j < kBPaths; j += 2) {
        float z0[A + 1], z1[A + 1];
#pragma unroll
        for (int k = 0; k < A; k += 2) s.template normal_pair<HW>(z0[k], z0[k + 1]);
#pragma unroll
        for (int k = 0; k < A; k += 2) s.template normal_pair<HW>(z1[k], z1[k + 1]);
#pragma unroll
        for (int i = 0; i < A; ++i) {
          f2 y = {ca[i], ca[i]};
#pragma unroll
          for (int k = 0; k <= i; ++k) y = __builtin_elementwise_fma(f2{Lb[i][k], Lb[i][k]}, f2{z0[k], z1[k]}, y);
          f2 e;
          if constexpr (HW) e = f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
          else e = f2{math::exp2_any(y.x), math::exp2_any(y.y)};
          const f2 xv = f2{x[i][j], x[i][j + 1]} * e;
          x[i][j] = xv.x;
          x[i][j + 1] = xv.y;
        }
      }
      if (a.store_all || t == T - 1) {
        const int64_t row = a.store_all ? t : 0;
#pragma unroll
        for (int i = 0; i < A; ++i) {
          const v4f v = {x[i][0], x[i][1], x[i][2], x[i][3]};
          char* rb = reinterpret_cast<char*>(cbase + (i * rows + row) * pitch + chunk);
          *reinterpret_cast<v4f*>(rb + lane_off) = v;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < A; ++i) {
      float p = 0.0f;
#pragma unroll
      for (int j = 0; j < kBPaths; ++j) p += x[i][j];
      acc[i] += static_cast<double>(p);
    }
  }

  // terminal sums: lane over chunks, wave butterfly, waves 0..7 (fixed order)
#pragma unroll
  for (int i = 0; i < A; ++i) {
    const double w = bwave_sum(acc[i]);
    if (lane == 0) wsum[wave * A + i] = w;
  }
  __syncthreads();
  if (tid < A) {
    double sum = 0.0;
    for (int w = 0; w < kBWaves; ++w) sum += wsum[w * A + tid];
    tot[tid] = sum;
    if (a.terminal_sum) a.terminal_sum[b * A + tid] = sum;
  }
  if constexpr (MODE == 1) return;  // basket_cf_kernel takes it from the stored rows and sums
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's terminal-row stores
  __syncthreads();
  basket_cf<A>(a, b, tot, part, avg, cs, sn);
}

// One workgroup per contract: the CF phase from the stored terminal rows and terminal sums
// (a separate pass after basket_kernel<MODE 1>: bit-identical to the fused kernel).
template <int A>
__global__ __launch_bounds__(kBThreads) void basket_cf_kernel(BasketArgs a) {
  extern __shared__ double lds[];
  const int N = a.N;
  const int64_t b = blockIdx.x;
  double* tot = lds;                         // [A]
  double* part = tot + kMaxAssets;           // [max(4 kBThreads, N)]
  double* avg = part + (N > 4 * kBThreads ? N : 4 * kBThreads);  // [N]
  double* cs = avg + N;
  double* sn = cs + N;
  for (int j = threadIdx.x; j < N; j += kBThreads) math::twiddle(j, N, sn[j], cs[j]);
  if (threadIdx.x < A) tot[threadIdx.x] = a.terminal_sum[b * A + threadIdx.x];
  __syncthreads();
  basket_cf<A>(a, b, tot, part, avg, cs, sn);
}


// ---- basket_resident_kernel: the terminal rows never leave the chip ------------------------------
// A C5 contract's terminal rows are A x P f32 = 2 MiB, far beyond one CU, so W = P / 4096
// co-resident workgroups run it (slice s = paths [4096 s, 4096 (s + 1)) = batch rows
// [s M/W, (s+1) M/W)), one 4096-path chunk each: lane l advances paths 4096 s + 4 l .. + 3 of all A
// assets through the 16 rows (one dwordx4 buffer store per asset and row) and keeps their terminal
// values.  The payoff needs every slice's terminal sums (the per-asset forward scales), so the
// exchange is pipelined one contract deep.  Iteration j of a workgroup:
//   0. wave 0 polls for contract j - 1's slice sums (published by every partner at the end of its
//      iteration j - 1), gathers them in one round of loads and writes the per-asset scales to LDS,
//      while waves 1..15 already simulate;
//   1. all waves simulate contract j (coefficients from an LDS table that wave 0 fills for 64
//      contracts at a time, one contract per lane: the f64 Cholesky is off the per-contract path);
//   2. the basket put of contract j - 1 from the terminal values parked in LDS (one 16-B slot per
//      lane and asset), column sums over the slice's rows (groups in order) stored to the launch's
//      column buffer [B][W][N]; contract j's terminal values replace j - 1's in the slots;
//   3. wave 0 publishes contract j's slice sums (write-through stores, one drain, an arrival add)
//      while the other waves move on.
// basket_mean_fft_kernel then adds each contract's W column sums in slice order, takes the M-mean
// and runs the FFT.  Only wave 0 ever waits on global memory.  Slice-sum slots rotate over 4
// contracts: a workgroup writes contract j's slots after its wait in iteration j saw every partner
// finish iteration j - 1, long after their reads of contract j - 4.  Reduction orders:
// oracle_basket_kernel(wg = 1024, slices = W).
constexpr int kRThreads = 1024;
constexpr int kRWaves = kRThreads / 64;
constexpr int kRChunk = kRThreads * kBPaths;  // 4096 paths: one chunk per workgroup and contract
constexpr int kRMaxSlices = 32;
constexpr int kRowBlock = 16;
constexpr int kRSlots = 4;                   // slice-sum slots (contract j mod 4)
constexpr int kRTable = 64;                  // contracts per coefficient table (one per wave-0 lane)

// Sync area of the resident basket launch (bytes): [0, 128) done counter (+0), the sticky status
// word (+SMC_SYNC_STATUS_OFFSET), the launch's failure flag (+SMC_SYNC_LAUNCH_FAIL_OFFSET) and contract
// queue (+64); per group a 128-B line of slice-sum arrivals; slice sums [groups][4][W A + 1] f64 (the
// last entry: the contract of the group's iteration j + 2, dynamic tail); column sums [chunk][W][N].
struct BasketSyncLayout {
  int64_t groups, xsum_off, xcol_off, bytes;
};
BasketSyncLayout basket_sync_layout(int A, int W, int N, int64_t groups, int64_t chunk) {
  BasketSyncLayout l{};
  l.groups = groups;
  l.xsum_off = 128 + 128 * groups;
  l.xcol_off = (l.xsum_off + groups * kRSlots * (W * A + 1) * 8 + 255) / 256 * 256;
  l.bytes = l.xcol_off + chunk * W * static_cast<int64_t>(N) * 8;
  return l;
}

constexpr int coef_stride(int A) { return 2 * A + A * A; }  // ca[A], x0[A], Lb[A][A] (f32)

size_t basket_resident_lds_bytes(int A, int N) {
  // terminal slots [A][1024] v4f, part [4096] f64, wsum [16][A] f64, scales + contract ring, two
  // coefficient tables [64][2A + A^2] f32 and two coefficient slots of dynamic contracts
  return static_cast<size_t>(A) * kRThreads * 16 +
         (4096 + kRWaves * kMaxAssets + 16) * sizeof(double) +
         (2 * kRTable + 2) * static_cast<size_t>(coef_stride(A)) * sizeof(float);
}

struct BasketResArgs {
  BasketArgs a;
  int32_t W;              // workgroups per contract
  int32_t groups;         // contract sequences (grid = groups * W)
  uint8_t* sync;          // basket_sync_layout
  int64_t xsum_off, xcol_off;
  uint32_t spin_limit;    // polls of an exchange before it gives up (status word, NaN targets)
  int32_t withhold;       // smc_test_exchange_fault: slice W-1 of group 0 skips its first arrival
};

template <int A, bool HW, bool STORE_ALL>
__global__ __launch_bounds__(kRThreads) void basket_resident_kernel(BasketResArgs ra) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  constexpr int CS = coef_stride(A);
  extern __shared__ double lds[];
  const BasketArgs& a = ra.a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.N, W = ra.W, groups = ra.groups;
  const int64_t P = a.P;
  // group (contract sequence) and slice of this workgroup: blocks b, b + 8, ... share an XCD
  int grp, slc;
  if (gridDim.x % (8 * W) == 0) {
    slc = static_cast<int>((blockIdx.x >> 3) % W);
    grp = static_cast<int>((blockIdx.x & 7) + 8 * (blockIdx.x / (8 * W)));
  } else {
    slc = static_cast<int>(blockIdx.x % W);
    grp = static_cast<int>(blockIdx.x / W);
  }
  v4f* term = reinterpret_cast<v4f*>(lds);                                   // [A][kRThreads]
  double* part = lds + static_cast<size_t>(A) * kRThreads * 2;               // [G][N] = [4096]
  double* wsum = part + 4096;                                                 // [kRWaves][A]
  float* pco = reinterpret_cast<float*>(wsum + kRWaves * kMaxAssets);         // scales[A], df, K
  int64_t* bidx = reinterpret_cast<int64_t*>(wsum + kRWaves * kMaxAssets + 12);  // [4] contract of iteration j
  float* table = reinterpret_cast<float*>(wsum + kRWaves * kMaxAssets + 16);  // [2][kRTable][CS]
  float* dco = table + 2 * kRTable * CS;                                      // [2][CS] dynamic contracts
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ra.sync + 128 + 128 * static_cast<int64_t>(grp));
  const int XS = W * A + 1;                // slice-sum slot: W x A sums + the group's contract of j + 2
  double* xsum = reinterpret_cast<double*>(ra.sync + ra.xsum_off) + static_cast<int64_t>(grp) * kRSlots * XS;
  double* xcol = reinterpret_cast<double*>(ra.sync + ra.xcol_off);           // [chunk][W][N]
  const int cols = N / 4;
  const int G = kRChunk / N;               // batch rows per slice
  const int q = tid % cols, g = tid / cols;
  const int64_t rows = STORE_ALL ? kRowBlock : 1;
  const int32_t pitch_b = static_cast<int32_t>(a.pitch * sizeof(float));  // A * rows * pitch_b < 2^31 (host check)
  const uint32_t lane_off = static_cast<uint32_t>(kBPaths * sizeof(float)) * tid;
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int width = 3 * A + 4;
  // contracts: grp + j groups for the first S iterations (every group has them), then the rest of
  // the launch from the queue, so groups on XCDs with more write bandwidth take more (per-XCD
  // finish times differed by up to 15 % with a static split).  Slice 0 takes the contract of
  // iteration j + 2 while publishing iteration j's slice sums; the partners read it with those sums
  // in iteration j + 1 (no added wait).
  constexpr int64_t kStaticQuarters = 3;  // statically assigned share of the iterations, in quarters
  const int64_t S = (a.B / groups) * kStaticQuarters / 4;
  const bool dyn = S >= 2;
  const int64_t n_static = dyn ? S * groups : a.B;
  uint32_t* queue = reinterpret_cast<uint32_t*>(ra.sync + 64);
  uint32_t* status = reinterpret_cast<uint32_t*>(ra.sync + SMC_SYNC_STATUS_OFFSET);
  uint32_t* launch_fail = reinterpret_cast<uint32_t*>(ra.sync + SMC_SYNC_LAUNCH_FAIL_OFFSET);
  auto bof = [&](int64_t jj) -> int64_t { return !dyn || jj < S ? grp + jj * groups : bidx[jj & 3]; };
  auto coefs = [&](int64_t bb, float* e) {  // simulation coefficients of contract bb (f64 Cholesky, rounded once)
    const double* c = a.contracts + bb * width;
    double L[kMaxAssets * kMaxAssets];
    cholesky_equicorr(A, c[3], L);
    const double dt = c[1] / static_cast<double>(kRowBlock);
    const double sq = sqrt(dt);
    constexpr double zscale = HW ? PathStream::kNormalScale<true> : 1.0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
      const double v = c[4 + 2 * A + i], d = c[4 + A + i];
      const double drift = c[2] - d - 0.5 * v * v;
      e[i] = static_cast<float>(drift * dt * kBLog2e);
      e[A + i] = static_cast<float>(c[4 + i]);
      const double bi = v * sq * kBLog2e * zscale;
#pragma unroll
      for (int k = 0; k < A; ++k) e[2 * A + i * A + k] = k <= i ? static_cast<float>(bi * L[i * kMaxAssets + k]) : 0.0f;
    }
  };

  // step 0 (wave 0): the payoff constants of contract jj from every slice's terminal sums
  auto gather = [&](int64_t jj) {
    const int64_t b = bof(jj);
    const double* c = a.contracts + b * width;
    const double* xs = xsum + (jj % kRSlots) * XS;
    const uint32_t want = static_cast<uint32_t>(W) * static_cast<uint32_t>(jj + 1);
    // bounded poll; once any exchange of this launch has failed (its flag set) the others stop
    // waiting at once, so a failed launch still drains in about one poll budget
    uint32_t spins = 0;
    bool ok;
    while (!(ok = get_sc1(cnt) >= want) && get_sc1(launch_fail) == 0u && ++spins < ra.spin_limit)
      __builtin_amdgcn_s_sleep(2);
    if (!ok && lane == 0) {
      __hip_atomic_fetch_or(status, SMC_SYNC_EXCHANGE_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(launch_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the W x A slice sums in one round of loads across the wave (<= 4 per lane), parked in part[]
    // (free until the payoff), then lanes 0..A-1 add their asset's W sums in slice order
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const __amdgpu_buffer_rsrc_t r = row_rsrc(xs);
    double v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = lane + 64 * k < W * A ? lane + 64 * k : 0;
      v[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, 16 /* sc1 */));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (lane + 64 * k < W * A) part[lane + 64 * k] = v[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    if (lane < A) {
      double t = 0.0;  // slices in order
      for (int s2 = 0; s2 < W; ++s2) t += part[s2 * A + lane];
      if (!ok) t = __builtin_nan("");
      if (slc == 0 && a.terminal_sum) a.terminal_sum[b * A + lane] = t;
      const float Tf = static_cast<float>(c[1]);
      const float F = static_cast<float>(c[4 + lane]) * math::exp_any(static_cast<float>(c[2] - c[4 + A + lane]) * Tf);
      pco[lane] = a.normalize ? F / static_cast<float>(t / static_cast<double>(P)) : 1.0f;
    }
    if (lane == 0) {
      // a failed exchange: NaN discount, so the targets are NaN (max(K - NaN, 0) alone would give 0)
      pco[A] = ok ? math::exp_any(static_cast<float>(-c[2]) * static_cast<float>(c[1])) : __builtin_nanf("");
      pco[A + 1] = static_cast<float>(c[0]);
      if (dyn && jj + 2 >= S) {  // the contract of iteration jj + 2 (slice 0 took it) and its coefficients
        const int64_t nb = ok ? get_sc1(reinterpret_cast<const int64_t*>(xs + W * A)) : a.B;
        bidx[(jj + 2) & 3] = nb;
        if (nb < a.B) coefs(nb, dco + ((jj + 2) & 1) * CS);
      }
    }
  };
  // step 2 (all waves, after a barrier that made pco visible): basket put of contract jj from the
  // terminal slots, column sums of the slice to the column buffer
  auto payoff = [&](int64_t jj) {
    float sc[A];
#pragma unroll
    for (int i = 0; i < A; ++i) sc[i] = pco[i];
    const float df = pco[A], Kf = pco[A + 1];
    const float wA = static_cast<float>(1.0 / A);
    v4f tv[A];
#pragma unroll
    for (int i = 0; i < A; ++i) tv[i] = term[i * kRThreads + tid];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float bs = 0.0f;
#pragma unroll
      for (int i = 0; i < A; ++i) bs = bs + tv[i][e] * sc[i];
      const float diff = Kf - bs * wA;
      part[g * N + 4 * q + e] = static_cast<double>(df * (diff > 0.0f ? diff : 0.0f));
    }
    lds_barrier();
    double* xc = xcol + (bof(jj) * W + slc) * static_cast<int64_t>(N);
    for (int n = tid; n < N; n += kRThreads) {
      double t = 0.0;
      for (int gg = 0; gg < G; ++gg) t += part[gg * N + n];
      xc[n] = t;
    }
  };

  const int64_t n_tab = dyn ? S : (a.B > grp ? (a.B - 1 - grp) / groups + 1 : 0);  // static iterations
  int64_t n_iter = 0;
  for (int64_t jj = 0;; ++jj) {
    const int64_t b = bof(jj);  // uniform (LDS ring, written before the last barrier)
    if (b >= a.B) break;
    n_iter = jj + 1;
    float* tab = table + ((jj / kRTable) & 1) * kRTable * CS;
    if (jj < n_tab && jj % kRTable == 0) {
      // wave 0 fills the coefficient table of the next 64 static contracts, one per lane
      const int64_t jl = jj + lane;
      if (wave == 0 && jl < n_tab) coefs(grp + jl * groups, tab + lane * CS);
      lds_barrier();
    }
    // 0. wave 0: contract jj - 1's scales (the other waves start simulating)
    if (jj > 0 && wave == 0) gather(jj - 1);
    const float* e = jj < n_tab ? tab + (jj % kRTable) * CS : dco + (jj & 1) * CS;
    float ca[A], x0[A], Lb[A][A];
#pragma unroll
    for (int i = 0; i < A; ++i) {
      ca[i] = e[i];
      x0[i] = e[A + i];
#pragma unroll
      for (int k = 0; k < A; ++k) Lb[i][k] = e[2 * A + i * A + k];
    }
    // 1. simulate: the lane's 4 paths of all A assets through the 16 rows
    const int64_t p0 = static_cast<int64_t>(slc) * kRChunk;
    const __amdgpu_buffer_rsrc_t crs = row_rsrc(a.paths + b * A * rows * a.pitch + p0);
    PathStream s(a.seed, static_cast<uint64_t>(ord0 + b), static_cast<uint64_t>(p0 / kBPaths + tid));
    float x[A][kBPaths];
#pragma unroll
    for (int i = 0; i < A; ++i)
#pragma unroll
      for (int j = 0; j < kBPaths; ++j) x[i][j] = x0[i];
    // a rolled row loop: unrolled, the compiler hoists all A x 16 row offsets into SGPRs and spills them
#pragma unroll 1
    for (int t = 0; t < kRowBlock; ++t) {
#pragma unroll
      for (int j = 0; j < kBPaths; j += 2) {
        float z0[A + 1], z1[A + 1];
#pragma unroll
        for (int k = 0; k < A; k += 2) s.template normal_pair<HW>(z0[k], z0[k + 1]);
#pragma unroll
        for (int k = 0; k < A; k += 2) s.template normal_pair<HW>(z1[k], z1[k + 1]);
#pragma unroll
        for (int i = 0; i < A; ++i) {
          f2 y = {ca[i], ca[i]};
#pragma unroll
          for (int k = 0; k <= i; ++k) y = __builtin_elementwise_fma(f2{Lb[i][k], Lb[i][k]}, f2{z0[k], z1[k]}, y);
          f2 ex;
          if constexpr (HW) ex = f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
          else ex = f2{math::exp2_any(y.x), math::exp2_any(y.y)};
          const f2 xv = f2{x[i][j], x[i][j + 1]} * ex;
          x[i][j] = xv.x;
          x[i][j + 1] = xv.y;
        }
      }
      if (STORE_ALL || t == kRowBlock - 1) {
        // one descriptor per contract slice; the (asset, row) offset rides in the scalar offset
#pragma unroll
        for (int i = 0; i < A; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(v4f{x[i][0], x[i][1], x[i][2], x[i][3]}, crs, lane_off,
                                                 static_cast<int>((i * rows + (STORE_ALL ? t : 0)) * pitch_b), 0);
      }
    }
    // this contract's slice sums: lane (f32 4-path partial -> f64), wave butterfly, waves in order
#pragma unroll
    for (int i = 0; i < A; ++i) {
      float p = 0.0f;
#pragma unroll
      for (int j = 0; j < kBPaths; ++j) p += x[i][j];
      const double w = bwave_sum(static_cast<double>(p));
      if (lane == 0) wsum[wave * A + i] = w;
    }
    lds_barrier();  // wsum of contract jj, scales of contract jj - 1
    // 2. contract jj - 1: payoffs and column sums (reads the terminal slots: own lane)
    if (jj > 0) payoff(jj - 1);
#pragma unroll
    for (int i = 0; i < A; ++i) term[i * kRThreads + tid] = v4f{x[i][0], x[i][1], x[i][2], x[i][3]};
    // 3. wave 0 publishes contract jj's slice sums: one drain, one arrival (the other waves go on)
    if (wave == 0) {
      if (lane < A) {
        double t = 0.0;
        for (int w2 = 0; w2 < kRWaves; ++w2) t += wsum[w2 * A + lane];
        put_sc1(xsum + (jj % kRSlots) * XS + slc * A + lane, t);
      }
      if (dyn && slc == 0 && lane == 0 && jj + 2 >= S)  // the group's contract of iteration jj + 2
        put_sc1(reinterpret_cast<int64_t*>(xsum + (jj % kRSlots) * XS + W * A), n_static + atomicAdd(queue, 1u));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0 && !(ra.withhold && grp == 0 && slc == W - 1 && jj == 0))
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lds_barrier();  // part / wsum are rewritten from here on
  }
  if (n_iter > 0) {  // the last contract
    if (wave == 0) gather(n_iter - 1);
    lds_barrier();
    payoff(n_iter - 1);
  }
  if (tid == 0) {
    // every workgroup made its last exchange before it arrives here: the last one resets the
    // group counters for the next launch
    __threadfence();
    uint32_t* done = reinterpret_cast<uint32_t*>(ra.sync);
    if (atomicAdd(done, 1u) == gridDim.x - 1) {
      for (int k = 0; k < groups; ++k) reinterpret_cast<uint32_t*>(ra.sync + 128 + 128 * static_cast<int64_t>(k))[0] = 0u;
      *queue = 0u;
      *launch_fail = 0u;
      *done = 0u;
    }
  }
}

// One workgroup per contract after basket_resident_kernel: the W slices' column sums added in
// slice order from 0.0, the M-mean and the FFT (fft_row) -> targets.
constexpr int kFThreads = 256;
__global__ __launch_bounds__(kFThreads) void basket_mean_fft_kernel(const double* __restrict__ xcol, int32_t W,
                                                                    int32_t N, int32_t M, float2* __restrict__ targets) {
  extern __shared__ double lds[];
  double* avg = lds;        // [N]
  double* cs = avg + N;     // [N]
  double* sn = cs + N;      // [N]
  double* xr = sn + N;      // [N]
  double* xi = xr + N;      // [N]
  const int64_t b = blockIdx.x;
  const double* xc = xcol + b * W * static_cast<int64_t>(N);
  for (int n = threadIdx.x; n < N; n += kFThreads) {
    math::twiddle(n, N, sn[n], cs[n]);
    double t = 0.0;
    for (int s2 = 0; s2 < W; ++s2) t += xc[static_cast<int64_t>(s2) * N + n];
    avg[n] = t / static_cast<double>(M);
  }
  __syncthreads();
  fft_row<float, kFThreads>(avg, cs, sn, N, xr, xi, targets + b * N);
}

size_t basket_lds_bytes(int A, int N) {
  const size_t part = static_cast<size_t>(N > 4 * kBThreads ? N : 4 * kBThreads);
  return (kMaxAssets * kMaxAssets + static_cast<size_t>(kBWaves) * A + A + part + 3 * static_cast<size_t>(N)) *
         sizeof(double);
}

size_t basket_cf_lds_bytes(int N) {
  const size_t part = static_cast<size_t>(N > 4 * kBThreads ? N : 4 * kBThreads);
  return (kMaxAssets + part + 3 * static_cast<size_t>(N)) * sizeof(double);
}

// Split (basket_kernel<1> then basket_cf_kernel) when the caller keeps the terminal sums: the CF
// re-read then streams at full read bandwidth instead of stalling each workgroup's store queue
// (as the single-asset paths_kernel + cf_kernel pair; kBasketSplit = false keeps the fused kernel)
constexpr bool kBasketSplit = true;

template <int A, bool HW>
const void* basket_kernel_ptr() {
  return reinterpret_cast<const void*>(basket_kernel<A, HW, kBasketSplit ? 1 : 0>);
}

// Workgroups of the kernel launched for <A, HW, N> resident on the current device (occupancy x CUs).
template <int A, bool HW>
int64_t basket_slots_k(int N) {
  int dev = 0, cus = 0, per_cu = 0;
  const size_t lds = basket_lds_bytes(A, N);
  const void* kernel = basket_kernel_ptr<A, HW>();
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return (void)hipGetLastError(), -1;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) != hipSuccess)
    return (void)hipGetLastError(), -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBThreads, lds) != hipSuccess)
    return (void)hipGetLastError(), -1;
  return static_cast<int64_t>(per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
}

template <int A, bool HW, int MODE>
int32_t launch_basket_mode(const BasketArgs& a, hipStream_t stream) {
  const size_t lds = basket_lds_bytes(A, a.N);
  auto kernel = basket_kernel<A, HW, MODE>;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "basket_kernel: cannot raise the dynamic LDS limit");
  }
  launch(kernel, dim3(static_cast<unsigned>(a.B)), dim3(kBThreads), lds, stream, a);
  return check_launch("basket_kernel");
}

template <int A, bool HW>
int32_t launch_basket_k(const BasketArgs& a, hipStream_t stream) {
  if (!kBasketSplit || !a.terminal_sum) return launch_basket_mode<A, HW, 0>(a, stream);
  if (int32_t st = launch_basket_mode<A, HW, 1>(a, stream)) return st;
  const size_t lds = basket_cf_lds_bytes(a.N);
  auto cf = basket_cf_kernel<A>;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(cf), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "basket_cf_kernel: cannot raise the dynamic LDS limit");
  }
  launch(cf, dim3(static_cast<unsigned>(a.B)), dim3(kBThreads), lds, stream, a);
  return check_launch("basket_cf_kernel");
}

// Workgroups per contract of basket_resident_kernel for this shape, or 0 when it does not take it
// (T = 16, N | 4096, 4 <= N <= 2048, P a multiple of 4096 and <= 32 x 4096, LDS within the CU's).
int basket_res_slices(int A, int T, int64_t N, int64_t M) {
  const int64_t P = N * M;
  if (T != kRowBlock || N < 4 || N > 2048 || N % 4 != 0 || kRChunk % N != 0 || P % kRChunk != 0) return 0;
  const int64_t W = P / kRChunk;
  if (W < 1 || W > kRMaxSlices || basket_resident_lds_bytes(A, static_cast<int>(N)) > 160 * 1024) return 0;
  return static_cast<int>(W);
}

// Contract sequences of the resident launch on the current device: floor(#CUs / W), -1 on failure.
int64_t basket_res_groups(int W) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return (void)hipGetLastError(), -1;
  return cus >= W ? cus / W : -1;
}

template <int A, bool HW>
int32_t launch_basket_resident_k(const BasketArgs& a, int W, int64_t groups, int64_t chunk, uint8_t* sync,
                                 hipStream_t stream) {
  const size_t lds = basket_resident_lds_bytes(A, a.N);
  auto kernel = a.store_all ? basket_resident_kernel<A, HW, true> : basket_resident_kernel<A, HW, false>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "basket_resident_kernel: cannot raise the dynamic LDS limit");
  }
  const BasketSyncLayout l = basket_sync_layout(A, W, a.N, groups, chunk);
  const BasketResArgs ra{a, W, static_cast<int32_t>(groups), sync, l.xsum_off, l.xcol_off, exchange_spin_limit(),
                        exchange_fault().withhold};
  launch(kernel, dim3(static_cast<unsigned>(groups * W)), dim3(kRThreads), lds, stream, ra);
  if (int32_t st = check_launch("basket_resident_kernel")) return st;
  const size_t flds = 5 * static_cast<size_t>(a.N) * sizeof(double);
  if (flds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(basket_mean_fft_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(flds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "basket_mean_fft_kernel: cannot raise the dynamic LDS limit");
  }
  launch(basket_mean_fft_kernel, dim3(static_cast<unsigned>(a.B)), dim3(kFThreads), flds, stream,
                     reinterpret_cast<const double*>(sync + l.xcol_off), W, a.N, a.M, a.targets);
  return check_launch("basket_mean_fft_kernel");
}

template <bool HW>
int32_t launch_basket_resident(int A, const BasketArgs& a, int W, int64_t groups, int64_t chunk, uint8_t* sync,
                               hipStream_t stream) {
  switch (A) {
    case 1: return launch_basket_resident_k<1, HW>(a, W, groups, chunk, sync, stream);
    case 2: return launch_basket_resident_k<2, HW>(a, W, groups, chunk, sync, stream);
    case 3: return launch_basket_resident_k<3, HW>(a, W, groups, chunk, sync, stream);
    case 4: return launch_basket_resident_k<4, HW>(a, W, groups, chunk, sync, stream);
    case 5: return launch_basket_resident_k<5, HW>(a, W, groups, chunk, sync, stream);
    case 6: return launch_basket_resident_k<6, HW>(a, W, groups, chunk, sync, stream);
    case 7: return launch_basket_resident_k<7, HW>(a, W, groups, chunk, sync, stream);
    case 8: return launch_basket_resident_k<8, HW>(a, W, groups, chunk, sync, stream);
    default: return fail(SMC_ERR_INVALID_ARGUMENT, "basket: n_assets must be in 1..8");
  }
}

template <bool HW>
int64_t basket_slots(int A, int N) {
  switch (A) {
    case 1: return basket_slots_k<1, HW>(N);
    case 2: return basket_slots_k<2, HW>(N);
    case 3: return basket_slots_k<3, HW>(N);
    case 4: return basket_slots_k<4, HW>(N);
    case 5: return basket_slots_k<5, HW>(N);
    case 6: return basket_slots_k<6, HW>(N);
    case 7: return basket_slots_k<7, HW>(N);
    case 8: return basket_slots_k<8, HW>(N);
    default: return -1;
  }
}

template <bool HW>
int32_t launch_basket(int A, const BasketArgs& a, hipStream_t stream) {
  switch (A) {
    case 1: return launch_basket_k<1, HW>(a, stream);
    case 2: return launch_basket_k<2, HW>(a, stream);
    case 3: return launch_basket_k<3, HW>(a, stream);
    case 4: return launch_basket_k<4, HW>(a, stream);
    case 5: return launch_basket_k<5, HW>(a, stream);
    case 6: return launch_basket_k<6, HW>(a, stream);
    case 7: return launch_basket_k<7, HW>(a, stream);
    case 8: return launch_basket_k<8, HW>(a, stream);
    default: return fail(SMC_ERR_INVALID_ARGUMENT, "basket: n_assets must be in 1..8");
  }
}

}  // namespace
}  // namespace smc

using namespace smc;

extern "C" {
#pragma GCC visibility push(default)
int32_t smc_basket_train_targets(const double* contracts_dev, int64_t n_contracts, int32_t n_assets,
                                 int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run,
                                 uint64_t mc_seed, const int64_t* ordinal_dev, int64_t ordinal0, int32_t math,
                                 int32_t normalization, int32_t store_mode, void* paths_dev, int64_t path_pitch,
                                 int64_t chunk_contracts, double* terminal_sum_dev, void* targets_dev,
                                 void* sync_dev, int64_t sync_bytes, void* stream) {
  const int64_t N = network_size, M = batches_per_mc_run, P = N * M;
  if (!contracts_dev || !paths_dev || !targets_dev)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: NULL buffer");
  if (n_assets < 1 || n_assets > kMaxAssets)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: n_assets must be in 1..8");
  if (n_contracts < 0 || n_contracts > 0x7fffffffLL || timesteps <= 0 || N <= 0 || M <= 0)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_basket_train_targets: need 0 <= B < 2^31, T > 0, N > 0, M > 0");
  if (N % 4 != 0 || N > 4096 || P % kBChunk != 0 || P >= (int64_t{1} << 29))
    return fail(SMC_ERR_INVALID_SHAPE,
                "smc_basket_train_targets: need N % 4 == 0, N <= 4096, N*M a multiple of 2048 and < 2^29");
  if (math != 0 && math != SMC_MATH_HW) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: bad math");
  if (store_mode != SMC_STORE_ALL && store_mode != SMC_STORE_TERMINAL)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: bad store_mode");
  if (path_pitch != 0 && (path_pitch < P || path_pitch % 4 != 0))
    return fail(SMC_ERR_INVALID_SHAPE, "smc_basket_train_targets: path_pitch must be 0 or a multiple of 4 >= P");
  if (chunk_contracts <= 0) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: chunk_contracts <= 0");
  if (basket_lds_bytes(n_assets, static_cast<int>(N)) > 160 * 1024)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_basket_train_targets: network_size exceeds the LDS budget");
  const int64_t width = 3 * n_assets + 4;
  // resident kernel where the shape allows and the caller passed a sync area of the right size
  const int64_t rows_all = store_mode == SMC_STORE_ALL ? timesteps : 1;
  const int64_t block_bytes = n_assets * rows_all * (path_pitch ? path_pitch : P) * 4;
  const int W = sync_dev && block_bytes < (int64_t{1} << 31) ? basket_res_slices(n_assets, timesteps, N, M) : 0;
  int64_t groups = 0;
  if (W > 0) {
    groups = basket_res_groups(W);
    if (groups <= 0) return fail(SMC_ERR_HIP, "smc_basket_train_targets: device query failed");
    // a CU-masked stream (the data-parallel step keeps its collective and network kernels on CUs of their own):
    // only as many groups as the stream's CUs hold, so every workgroup of a group is resident at once
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return (void)hipGetLastError(), fail(SMC_ERR_HIP, "smc_basket_train_targets: device query failed");
    const int64_t on_stream = stream_cus(as_stream(stream), cus) / W;
    if (on_stream <= 0) return fail(SMC_ERR_INVALID_SHAPE, "smc_basket_train_targets: fewer CUs on the stream than slices");
    if (on_stream < groups) groups = on_stream;
    if (sync_bytes < basket_sync_layout(n_assets, W, static_cast<int>(N), groups, chunk_contracts).bytes)
      return fail(SMC_ERR_INVALID_ARGUMENT, "smc_basket_train_targets: sync_bytes < smc_basket_sync_bytes(...)");
  }
  for (int64_t off = 0; off < n_contracts; off += chunk_contracts) {
    const int64_t nb = n_contracts - off < chunk_contracts ? n_contracts - off : chunk_contracts;
    BasketArgs a{contracts_dev + off * width, nb, timesteps, P, network_size, batches_per_mc_run, mc_seed,
                 ordinal_dev, ordinal0 + off, normalization != SMC_NORM_RAW, store_mode == SMC_STORE_ALL,
                 static_cast<float*>(paths_dev), path_pitch ? path_pitch : P,
                 terminal_sum_dev ? terminal_sum_dev + off * n_assets : nullptr,
                 static_cast<float2*>(targets_dev) + off * N};
    uint8_t* sync = static_cast<uint8_t*>(sync_dev);
    const int32_t st =
        W > 0 ? (math == SMC_MATH_HW
                     ? launch_basket_resident<true>(n_assets, a, W, groups, chunk_contracts, sync, as_stream(stream))
                     : launch_basket_resident<false>(n_assets, a, W, groups, chunk_contracts, sync, as_stream(stream)))
              : (math == SMC_MATH_HW ? launch_basket<true>(n_assets, a, as_stream(stream))
                                     : launch_basket<false>(n_assets, a, as_stream(stream)));
    if (st) return st;
  }
  return SMC_OK;
}

int64_t smc_basket_sync_bytes(int32_t n_assets, int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run,
                              int64_t chunk_contracts) {
  if (n_assets < 1 || n_assets > kMaxAssets || network_size <= 0 || batches_per_mc_run <= 0 || chunk_contracts <= 0)
    return -1;
  const int W = basket_res_slices(n_assets, timesteps, network_size, batches_per_mc_run);
  if (W == 0) return 0;
  const int64_t groups = basket_res_groups(W);
  if (groups <= 0) return -1;
  return basket_sync_layout(n_assets, W, network_size, groups, chunk_contracts).bytes;
}

const char* smc_basket_train_targets_kernel(int32_t n_assets, int32_t timesteps, int32_t network_size,
                                            int32_t batches_per_mc_run, int32_t with_sync, int32_t keep_sums) {
  if (with_sync && n_assets >= 1 && n_assets <= kMaxAssets && network_size > 0 && batches_per_mc_run > 0 &&
      basket_res_slices(n_assets, timesteps, network_size, batches_per_mc_run) > 0)
    return "basket_resident_kernel";
  return keep_sums && kBasketSplit ? "basket_kernel+basket_cf_kernel" : "basket_kernel";
}

int64_t smc_basket_resident_slots(int32_t n_assets, int32_t network_size, int32_t math) {
  if (n_assets < 1 || n_assets > kMaxAssets || network_size <= 0 || network_size > 4096) return -1;
  return math == SMC_MATH_HW ? basket_slots<true>(n_assets, network_size) : basket_slots<false>(n_assets, network_size);
}

#pragma GCC visibility pop
}  // extern "C"
