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
// asset's block is a single-asset [T][P] matrix.  One 512-thread workgroup per contract; each
// lane owns 4 consecutive paths of a 2048-path chunk for all A assets and stores one dwordx4
// per (asset, row).
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

namespace smc {
namespace {

constexpr int kBThreads = 512;
constexpr int kBWaves = kBThreads / 64;
constexpr int kBPaths = 4;                      // paths per lane
constexpr int kBChunk = kBThreads * kBPaths;    // paths per workgroup pass
constexpr int kMaxAssets = 8;
#ifndef SMC_BASKET_MIN_BLOCKS
#define SMC_BASKET_MIN_BLOCKS 1
#endif
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
__global__ __launch_bounds__(kBThreads, SMC_BASKET_MIN_BLOCKS) void basket_kernel(BasketArgs a) {
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
// (as the single-asset paths_kernel + cf_kernel pair; SMC_BASKET_SPLIT=0 builds keep the fused kernel)
#ifndef SMC_BASKET_SPLIT
#define SMC_BASKET_SPLIT 1
#endif

template <int A, bool HW>
const void* basket_kernel_ptr() {
  return reinterpret_cast<const void*>(basket_kernel<A, HW, SMC_BASKET_SPLIT ? 1 : 0>);
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
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(a.B)), dim3(kBThreads), lds, stream, a);
  return check_launch("basket_kernel");
}

template <int A, bool HW>
int32_t launch_basket_k(const BasketArgs& a, hipStream_t stream) {
  if (!SMC_BASKET_SPLIT || !a.terminal_sum) return launch_basket_mode<A, HW, 0>(a, stream);
  if (int32_t st = launch_basket_mode<A, HW, 1>(a, stream)) return st;
  const size_t lds = basket_cf_lds_bytes(a.N);
  auto cf = basket_cf_kernel<A>;
  if (lds > 64 * 1024 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(cf), hipFuncAttributeMaxDynamicSharedMemorySize,
                          static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "basket_cf_kernel: cannot raise the dynamic LDS limit");
  }
  hipLaunchKernelGGL(cf, dim3(static_cast<unsigned>(a.B)), dim3(kBThreads), lds, stream, a);
  return check_launch("basket_cf_kernel");
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
                                 void* stream) {
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
  for (int64_t off = 0; off < n_contracts; off += chunk_contracts) {
    const int64_t nb = n_contracts - off < chunk_contracts ? n_contracts - off : chunk_contracts;
    BasketArgs a{contracts_dev + off * width, nb, timesteps, P, network_size, batches_per_mc_run, mc_seed,
                 ordinal_dev, ordinal0 + off, normalization != SMC_NORM_RAW, store_mode == SMC_STORE_ALL,
                 static_cast<float*>(paths_dev), path_pitch ? path_pitch : P,
                 terminal_sum_dev ? terminal_sum_dev + off * n_assets : nullptr,
                 static_cast<float2*>(targets_dev) + off * N};
    const int32_t st = math == SMC_MATH_HW ? launch_basket<true>(n_assets, a, as_stream(stream))
                                           : launch_basket<false>(n_assets, a, as_stream(stream));
    if (st) return st;
  }
  return SMC_OK;
}

int64_t smc_basket_resident_slots(int32_t n_assets, int32_t network_size, int32_t math) {
  if (n_assets < 1 || n_assets > kMaxAssets || network_size <= 0 || network_size > 4096) return -1;
  return math == SMC_MATH_HW ? basket_slots<true>(n_assets, network_size) : basket_slots<false>(n_assets, network_size);
}

#pragma GCC visibility pop
}  // extern "C"
