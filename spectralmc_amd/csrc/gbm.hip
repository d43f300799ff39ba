// GBM Monte-Carlo engine for gfx950: path simulation, forward normalisation, put payoff,
// M-batch mean and the N-point DFT that yields the characteristic-function training
// targets — one workgroup per contract, one launch per (chunk of) B contracts.
//
// Reference behaviour restated (Tuee22/SpectralMC, src/spectralmc/):
//   gbm.py:224-257   SimulateBlackScholes: per path X *= exp((r-d-v^2/2)dt + v sqrt(dt) Z) (log-Euler)
//                    or X += (r-d) X dt + v X sqrt(dt) Z; X = |X| (simple Euler); row t stores X
//                    after step t+1.
//   gbm.py:428-438   times = linspace(dt, T, T) (f32); F_t = X0 e^{(r-d) t}; df_t = e^{-r t};
//                    NORMALIZE: sims[t] *= F_t / mean_p(sims[t]).
//   gbm.py:464-474   put = df_T * max(K - S_T, 0)
//   gbm_trainer.py:806-817  target = mean_m FFT_N(put.reshape(M, N))[m]  (unnormalised forward FFT)
//
// Design:
//   * 512-thread workgroup = one contract; each lane owns 4 consecutive paths per 2048-path chunk,
//     so every row store is a 16-B-per-lane dwordx4 (1 KiB per wave-instruction, coalesced).
//   * Normals are generated in registers (smc_rng.h) — no normal matrix in HBM.
//   * Row sums for the normalisation are accumulated per lane in f64 and reduced in a fixed
//     order (wave butterfly, then waves 0..7): bit-reproducible, no float atomics.
//   * The terminal row is re-read by the same workgroup after the block barrier (L2/MALL hit),
//     the payoff is summed over the M batches per column n in f64, and the real-input DFT is
//     evaluated from an LDS twiddle table (FFT linearity: FFT(mean_m x_m) == mean_m FFT(x_m)).

#include <cmath>

#pragma clang fp contract(off)

#include "smc_internal.h"
#include "smc_math.h"
#include "smc_rng.h"

namespace smc {
namespace {

#ifndef SMC_WG_THREADS
#define SMC_WG_THREADS 512
#endif
#ifndef SMC_MIN_LDS
#define SMC_MIN_LDS 0
#endif
constexpr int kThreads = SMC_WG_THREADS;
constexpr int kWaves = kThreads / 64;
constexpr int kPathsPerLane = 4;
constexpr int kChunk = kThreads * kPathsPerLane;
constexpr double kLog2e = 1.4426950408889634;
constexpr size_t kMaxLds = 160 * 1024;

struct Contract {
  double X0, K, T, r, d, v;
};

struct EngineArgs {
  const double* contracts;    // [B][6] of this launch
  int64_t B;
  int32_t T;
  int64_t P;
  int32_t N, M;
  uint64_t seed;
  const int64_t* ordinal_dev;
  int64_t ordinal0;           // ordinal of contract 0 of this launch (plus *ordinal_dev)
  int32_t scheme;
  int32_t normalize;
  int32_t store;              // SMC_STORE_TERMINAL or SMC_STORE_ALL
  int32_t simulate;           // 0: paths/rowsum already in memory (smc_cf_targets)
  int32_t all_rows;           // 1: sum every row (rowsum[B][T]); 0: terminal row only
  void* paths;
  double* rowsum;             // [B][T] or NULL
  void* targets;              // [B][N] complex or NULL
  int64_t pitch;              // elements between consecutive path rows (0: P, contiguous)
};

template <typename Real>
struct Vec4T;
template <>
struct Vec4T<float> {
  using type = float4;
};
template <>
struct Vec4T<double> {
  using type = double4;
};

template <typename Real>
struct Complex2;
template <>
struct Complex2<float> {
  using type = float2;
};
template <>
struct Complex2<double> {
  using type = double2;
};

__device__ __forceinline__ Contract load_contract(const double* c) {
  return Contract{c[0], c[1], c[2], c[3], c[4], c[5]};
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// One step of the path recursion.  f32 log-Euler works in log2 units (coefficients
// pre-scaled by log2 e) with the portable exp2 of smc_math.h; f64 uses OCML exp.
template <typename Real, bool LOG_EULER, bool HW>
struct Stepper {
  Real a, b;

  // f32 HW normals come out divided by sqrt(2 ln 2) (smc_rng.h); the factor rides on b.
  static constexpr double zscale() {
    return sizeof(Real) == 4 && HW ? PathStream::kNormalScale<true> : 1.0;
  }

  __device__ Stepper(const Contract& c, int T) {
    const double dt = c.T / static_cast<double>(T);
    const double sq = sqrt(dt);
    if (LOG_EULER) {
      const double drift = c.r - c.d - 0.5 * c.v * c.v;
      const double scale = sizeof(Real) == 4 ? kLog2e : 1.0;
      a = static_cast<Real>(drift * dt * scale);
      b = static_cast<Real>(c.v * sq * scale * zscale());
    } else {
      a = static_cast<Real>((c.r - c.d) * dt);
      b = static_cast<Real>(c.v * sq * zscale());
    }
  }

  __device__ __forceinline__ Real operator()(Real x, Real z) const {
    if constexpr (LOG_EULER) {
      if constexpr (sizeof(Real) == 4 && HW) return x * __builtin_amdgcn_exp2f(fmaf(b, z, a));
      else if constexpr (sizeof(Real) == 4) return x * math::exp2_any(fmaf(b, z, a));
      else return x * exp(fma(b, z, a));
    }
    if constexpr (sizeof(Real) == 4) return fabsf(fmaf(x, fmaf(b, z, a), x));
    else return fabs(fma(x, fma(b, z, a), x));
  }
};

constexpr int kRowBlock = 16;  // rows accumulated in registers per pass over the paths

// x[j] *= 2^y[j] for the lane's 4 paths, two v_pk_mul_f32 (f32 HW log-Euler)
template <typename Real>
__device__ __forceinline__ void advance_packed(Real (&x)[4], const Real (&y)[4]) {
  typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < 4; j += 2) {
    const f2 e = {__builtin_amdgcn_exp2f(y[j]), __builtin_amdgcn_exp2f(y[j + 1])};
    const f2 v = f2{x[j], x[j + 1]} * e;
    x[j] = v.x;
    x[j + 1] = v.y;
  }
}

// The 4 paths p0..p0+3 of one lane: steps [0, t0) are replayed without output (only when
// T > kRowBlock), rows [t0, t0 + nrows) are stored and added to acc[].  MASKED handles the
// ragged last chunk (nvalid < 4) and P % 4 != 0 with scalar stores; otherwise one dwordx4
// store per row, addressed as (wave-uniform row base) + (32-bit lane offset).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS, bool MASKED, bool FULLBLOCK>
__device__ __forceinline__ void lane_paths(const EngineArgs& a, const Stepper<Real, LOG_EULER, HW>& step, Real x0,
                                           uint64_t ordinal, int64_t chunk, int nvalid, int t0, int nrows,
                                           Real* contract_base, double (&acc)[ALLROWS ? kRowBlock : 1]) {
  using V4 = typename Vec4T<Real>::type;
  const int T = a.T;
  const int64_t P = a.P;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const bool store_all = a.store == SMC_STORE_ALL;
  const int64_t p0 = chunk + kPathsPerLane * static_cast<int64_t>(threadIdx.x);
  PathStream s(a.seed, ordinal, static_cast<uint64_t>(p0 / kPathsPerLane));  // the lane's group stream
  // f32 HW log-Euler: the RNG hands back the step exponents directly (packed path pairs)
  constexpr bool kPacked = HW && LOG_EULER && sizeof(Real) == 4;
  Real x[kPathsPerLane], zl[kPathsPerLane], zh[kPathsPerLane];
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) x[j] = x0;
  for (int t = 0; t < t0; t += 2) {  // t0 is a multiple of kRowBlock (even)
    if constexpr (kPacked) {
      s.hw_log_increments4(step.b, step.a, zl, zh);
      advance_packed(x, zl);
      advance_packed(x, zh);
    } else {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(zl[j], zh[j]);
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(step(x[j], zl[j]), zh[j]);
    }
  }
  // wave-uniform row base (SGPR pair) + 32-bit per-lane byte offset
  const uint32_t lane_off = static_cast<uint32_t>(kPathsPerLane * sizeof(Real)) * threadIdx.x;
  Real* chunk_base = contract_base + chunk;
#pragma unroll
  for (int i = 0; i < kRowBlock; ++i) {
    if (FULLBLOCK || i < nrows) {
      const int t = t0 + i;
      if constexpr (kPacked) {
        if ((i & 1) == 0) s.hw_log_increments4(step.b, step.a, zl, zh);
        advance_packed(x, (i & 1) ? zh : zl);
      } else {
        if ((i & 1) == 0) {
#pragma unroll
          for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(zl[j], zh[j]);
        }
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(x[j], (i & 1) ? zh[j] : zl[j]);
      }
      if (store_all || t == T - 1) {
        char* row = reinterpret_cast<char*>(chunk_base + (store_all ? static_cast<int64_t>(t) * pitch : 0));
        if constexpr (!MASKED) {
          V4 v4;
          v4.x = x[0];
          v4.y = x[1];
          v4.z = x[2];
          v4.w = x[3];
          *reinterpret_cast<V4*>(row + lane_off) = v4;
        } else {
          Real* r = reinterpret_cast<Real*>(row + lane_off);
#pragma unroll
          for (int j = 0; j < kPathsPerLane; ++j)
            if (j < nvalid) r[j] = x[j];
        }
      }
      if (ALLROWS || t == T - 1) {
        Real part = 0;
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) part += (!MASKED || j < nvalid) ? x[j] : Real(0);
        acc[ALLROWS ? i : 0] += static_cast<double>(part);
      }
    }
  }
}

// ---- phase 1: simulate the contract's P paths ----------------------------------------
// Fills lds_tot[0..T) (ALLROWS) or lds_tot[T-1] with the f64 sum over paths of the row(s),
// in a fixed order: per lane sequentially over its chunks, wave butterfly (xor 32..1),
// waves 0..7.  Training needs only the terminal row's sum (its normalisation scale).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__device__ void simulate_contract(const EngineArgs& a, const Contract& c, uint64_t ordinal, int64_t b,
                                  double* lds_acc, double* lds_tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T;
  const int64_t P = a.P;
  const bool store_all = a.store == SMC_STORE_ALL;
  const int64_t pitch = a.pitch ? a.pitch : P;
  Real* base = static_cast<Real*>(a.paths) + (store_all ? b * T * pitch : b * pitch);
  const bool vec_ok = (P % kPathsPerLane) == 0;
  const int64_t full_end = vec_ok ? (P / kChunk) * kChunk : 0;
  const Stepper<Real, LOG_EULER, HW> step(c, T);
  const Real x0 = static_cast<Real>(c.X0);
  constexpr int kAcc = ALLROWS ? kRowBlock : 1;

  for (int t0 = 0; t0 < T; t0 += kRowBlock) {
    const int nrows = T - t0 < kRowBlock ? T - t0 : kRowBlock;
    double acc[kAcc];
#pragma unroll
    for (int i = 0; i < kAcc; ++i) acc[i] = 0.0;
    int64_t chunk = 0;
    if (nrows == kRowBlock) {  // branch-free fast path: whole 16-row block, whole 2048-path chunks
      for (; chunk < full_end; chunk += kChunk)
        lane_paths<Real, LOG_EULER, HW, ALLROWS, false, true>(a, step, x0, ordinal, chunk, kPathsPerLane, t0, nrows,
                                                              base, acc);
    }
    for (; chunk < P; chunk += kChunk) {  // everything else: ragged rows / paths, scalar stores
      const int64_t p0 = chunk + kPathsPerLane * tid;
      const int nvalid = static_cast<int>(p0 >= P ? 0 : (P - p0 >= kPathsPerLane ? kPathsPerLane : P - p0));
      lane_paths<Real, LOG_EULER, HW, ALLROWS, true, false>(a, step, x0, ordinal, chunk, nvalid, t0, nrows, base,
                                                            acc);
    }
    if (ALLROWS || t0 + nrows == T) {  // rows of this block whose sums are wanted
#pragma unroll
      for (int i = 0; i < kAcc; ++i) {
        if (i < nrows) {
          const double w = wave_sum(acc[i]);
          if (lane == 0) lds_acc[wave * kRowBlock + i] = w;
        }
      }
      __syncthreads();
      const int first = ALLROWS ? 0 : nrows - 1;  // !ALLROWS: only the terminal row, kept in slot 0
      if (tid >= first && tid < nrows) {
        double tot = 0.0;
        for (int w = 0; w < kWaves; ++w) tot += lds_acc[w * kRowBlock + (ALLROWS ? tid : 0)];
        lds_tot[t0 + tid] = tot;
      }
      __syncthreads();
    }
  }
}

// ---- phases 2+3: normalised put payoff, mean over M batches, real-input DFT ------------
template <typename Real>
__device__ void cf_targets_contract(const EngineArgs& a, const Contract& c, int64_t b,
                                    double terminal_sum, double* lds) {
  using C2 = typename Complex2<Real>::type;
  const int tid = threadIdx.x;
  const int T = a.T, N = a.N, M = a.M;
  const int64_t P = a.P;
  const bool store_all = a.store == SMC_STORE_ALL;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const Real* row = static_cast<const Real*>(a.paths) + (store_all ? (b * T + (T - 1)) * pitch : b * pitch);

  // Reference scalar semantics: gbm.py:429-431 evaluate times/forwards/df in the sim dtype.
  Real F, df;
  const Real Tm = static_cast<Real>(c.T);
  if constexpr (sizeof(Real) == 4) {
    F = static_cast<float>(c.X0) * math::exp_any(static_cast<float>(c.r - c.d) * Tm);
    df = math::exp_any(static_cast<float>(-c.r) * Tm);
  } else {
    F = c.X0 * exp((c.r - c.d) * Tm);
    df = exp(-c.r * Tm);
  }
  const Real s = a.normalize ? F / static_cast<Real>(terminal_sum / static_cast<double>(P)) : Real(1);
  const Real K = static_cast<Real>(c.K);

  const int G = N <= kThreads ? kThreads / N : 1;
  const int items = N * G;
  double* part = lds;                                  // [max(kThreads, N)]
  double* avg = part + (N > kThreads ? N : kThreads);  // [N]
  double* cs = avg + N;                                // [N]
  double* sn = cs + N;                                 // [N]

  constexpr int kBatch = 16;  // loads in flight per thread; the sum keeps the m order
  for (int item = tid; item < items; item += kThreads) {
    const int n = item % N, g = item / N;
    double sum = 0.0;
    for (int m0 = g; m0 < M; m0 += G * kBatch) {
      Real v[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int m = m0 + u * G < M ? m0 + u * G : M - 1;  // clamped: loads stay unconditional
        v[u] = row[static_cast<int64_t>(m) * N + n];
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        if (m0 + u * G < M) {
          const Real xs = v[u] * s;  // sims *= scale (rounded to Real)
          const Real diff = K - xs;
          const Real pay = df * (diff > Real(0) ? diff : Real(0));
          sum += static_cast<double>(pay);
        }
      }
    }
    part[item] = sum;
  }
  for (int j = tid; j < N; j += kThreads) math::twiddle(j, N, sn[j], cs[j]);
  __syncthreads();
  for (int n = tid; n < N; n += kThreads) {
    double tot = 0.0;
    for (int g = 0; g < G; ++g) tot += part[g * N + n];
    avg[n] = tot / static_cast<double>(M);
  }
  __syncthreads();
  C2* out = static_cast<C2*>(a.targets) + b * N;
  for (int k = tid; k <= N / 2; k += kThreads) {
    double re = 0.0, im = 0.0;
    int idx = 0;
    for (int n = 0; n < N; ++n) {
      re = fma(avg[n], cs[idx], re);
      im = fma(-avg[n], sn[idx], im);
      idx += k;
      if (idx >= N) idx -= N;
    }
    C2 v;
    v.x = static_cast<Real>(re);
    v.y = static_cast<Real>(im);
    out[k] = v;
    if (k != 0 && 2 * k != N) {
      v.y = static_cast<Real>(-im);
      out[N - k] = v;
    }
  }
}

template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__global__ __launch_bounds__(kThreads) void contract_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  const int64_t b = blockIdx.x;
  const Contract c = load_contract(a.contracts + b * 6);
  const int T = a.T;
  double* lds_tot = lds;               // [T]
  double* lds_work = lds + T;          // simulate: [kWaves][T]; cf: part/avg/cs/sn
  double terminal_sum;
  if (a.simulate) {
    const uint64_t ordinal = static_cast<uint64_t>((a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0 + b);
    simulate_contract<Real, LOG_EULER, HW, ALLROWS>(a, c, ordinal, b, lds_work, lds_tot);
    if (ALLROWS && a.rowsum)
      for (int t = threadIdx.x; t < T; t += kThreads) a.rowsum[b * T + t] = lds_tot[t];
    terminal_sum = lds_tot[T - 1];
  } else {
    terminal_sum = a.rowsum[b * T + (T - 1)];
  }
  if (!ALLROWS && a.rowsum && threadIdx.x == 0 && a.simulate) a.rowsum[b * T + (T - 1)] = terminal_sum;
#if defined(SMC_EXPERIMENT_NO_CF)  // tools/micro decomposition builds only
  if (false) {
#else
  if (a.targets) {
#endif
    __syncthreads();  // workgroup-scope fence: phase-1 stores of the terminal row are visible
    cf_targets_contract<Real>(a, c, b, terminal_sum, lds_work);
  }
}

// In-place forward normalisation of a stored [B][T][P] matrix (gbm.py:428-438).
template <typename Real>
__global__ __launch_bounds__(256) void normalize_kernel(const double* __restrict__ contracts, int64_t B,
                                                        int32_t T, int64_t P, Real* __restrict__ paths,
                                                        const double* __restrict__ rowsum) {
  for (int64_t rowi = blockIdx.x; rowi < B * T; rowi += gridDim.x) {
    const int64_t b = rowi / T;
    const int t = static_cast<int>(rowi % T);
    const Contract c = load_contract(contracts + b * 6);
    // times = linspace(dt, T, T): computed in f64, cast to the sim dtype, last point exact.
    const double dt = c.T / static_cast<double>(T);
    const double step = T > 1 ? (c.T - dt) / static_cast<double>(T - 1) : 0.0;
    const double t64 = (t == T - 1) ? c.T : dt + static_cast<double>(t) * step;
    Real F;
    if constexpr (sizeof(Real) == 4)
      F = static_cast<float>(c.X0) * math::exp_any(static_cast<float>(c.r - c.d) * static_cast<float>(t64));
    else
      F = c.X0 * exp((c.r - c.d) * t64);
    const Real scale = F / static_cast<Real>(rowsum[rowi] / static_cast<double>(P));
    Real* row = paths + rowi * P;
    for (int64_t p = threadIdx.x; p < P; p += blockDim.x) row[p] = row[p] * scale;
  }
}

template <typename Real, bool HW>
__global__ __launch_bounds__(256) void normals_kernel(uint64_t seed, uint64_t ordinal, int32_t rows,
                                                      int64_t cols, Real* __restrict__ out) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // path group
  if (g * kPathsPerLane >= cols) return;
  PathStream s(seed, ordinal, static_cast<uint64_t>(g));
  const Real zs = sizeof(Real) == 4 ? static_cast<Real>(PathStream::kNormalScale<HW>) : Real(1);
  Real z0[kPathsPerLane], z1[kPathsPerLane];
  for (int t = 0; t < rows; ++t) {
    if ((t & 1) == 0) {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(z0[j], z1[j]);
    }
#pragma unroll
    for (int j = 0; j < kPathsPerLane; ++j) {
      const int64_t p = g * kPathsPerLane + j;
      if (p < cols) out[static_cast<int64_t>(t) * cols + p] = zs * ((t & 1) ? z1[j] : z0[j]);
    }
  }
}

// ---- host-side launch helpers ------------------------------------------------------------
size_t lds_bytes(int T, int N, bool cf) {
  size_t doubles = static_cast<size_t>(T);                       // lds_tot
  size_t work = static_cast<size_t>(kWaves) * kRowBlock;         // per-wave row partials
  if (cf) {
    const size_t cfw = static_cast<size_t>(N > kThreads ? N : kThreads) + 3 * static_cast<size_t>(N);
    if (cfw > work) work = cfw;
  }
  const size_t bytes = (doubles + work) * sizeof(double);
  return bytes < SMC_MIN_LDS ? SMC_MIN_LDS : bytes;
}

template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
int32_t launch_engine_k(const EngineArgs& a, size_t lds, hipStream_t stream) {
  auto kernel = contract_kernel<Real, LOG_EULER, HW, ALLROWS>;
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "contract_kernel: cannot raise the dynamic LDS limit");
    }
  }
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(a.B)), dim3(kThreads), lds, stream, a);
  return check_launch("contract_kernel");
}

template <typename Real>
int32_t launch_engine(const EngineArgs& a, hipStream_t stream) {
  if (a.B == 0) return SMC_OK;
  const bool cf = a.targets != nullptr;
  const size_t lds = lds_bytes(a.T, a.N, cf);
  if (lds > kMaxLds) return fail(SMC_ERR_INVALID_SHAPE, "engine: timesteps/network_size exceed the LDS budget");
  const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
  const bool hw = (a.scheme & SMC_MATH_HW) != 0 && sizeof(Real) == 4;
  const bool allrows = a.all_rows != 0;
#define SMC_LAUNCH(LE, HWM, AR) \
  if (log_euler == LE && hw == HWM && allrows == AR) return launch_engine_k<Real, LE, HWM, AR>(a, lds, stream);
  SMC_LAUNCH(true, false, false)
  SMC_LAUNCH(true, false, true)
  SMC_LAUNCH(false, false, false)
  SMC_LAUNCH(false, false, true)
  if constexpr (sizeof(Real) == 4) {
    SMC_LAUNCH(true, true, false)
    SMC_LAUNCH(true, true, true)
    SMC_LAUNCH(false, true, false)
    SMC_LAUNCH(false, true, true)
  }
#undef SMC_LAUNCH
  return fail(SMC_ERR_INVALID_ARGUMENT, "engine: unsupported scheme / math mode");
}

int32_t dispatch_engine(const EngineArgs& a, int32_t dtype, hipStream_t stream) {
  if (dtype == SMC_DTYPE_F32) return launch_engine<float>(a, stream);
  if (dtype == SMC_DTYPE_F64) return launch_engine<double>(a, stream);
  return fail(SMC_ERR_INVALID_ARGUMENT, "engine: dtype must be SMC_DTYPE_F32 or SMC_DTYPE_F64");
}

bool valid_scheme(int32_t scheme) {
  const int32_t base = scheme & 0xff, flags = scheme & ~0xff;
  return (base == SMC_SCHEME_LOG_EULER || base == SMC_SCHEME_SIMPLE_EULER) && (flags & ~SMC_MATH_HW) == 0;
}

int32_t validate_common(const double* contracts, int64_t B, int32_t T, int64_t P, int32_t dtype) {
  if (!contracts) return fail(SMC_ERR_INVALID_ARGUMENT, "engine: contracts is NULL");
  if (B < 0 || T <= 0 || P <= 0) return fail(SMC_ERR_INVALID_SHAPE, "engine: need B >= 0, T > 0, P > 0");
  if (B > 0x7fffffffLL) return fail(SMC_ERR_INVALID_SHAPE, "engine: more than 2^31-1 contracts in one call");
  if (P >= (1LL << 40)) return fail(SMC_ERR_INVALID_SHAPE, "engine: path count too large");
  if (dtype != SMC_DTYPE_F32 && dtype != SMC_DTYPE_F64)
    return fail(SMC_ERR_INVALID_ARGUMENT, "engine: bad dtype");
  return SMC_OK;
}

}  // namespace
}  // namespace smc

using namespace smc;

extern "C" {
#pragma GCC visibility push(default)

int32_t smc_gbm_simulate(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int64_t n_paths,
                         uint64_t mc_seed, const int64_t* ordinal_dev, int64_t ordinal0, int32_t scheme,
                         int32_t dtype, void* paths_dev, double* rowsum_dev, void* stream) {
  if (int32_t st = validate_common(contracts_dev, n_contracts, timesteps, n_paths, dtype)) return st;
  if (!paths_dev) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_gbm_simulate: paths_dev is NULL");
  if (!valid_scheme(scheme)) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_gbm_simulate: bad scheme");
  EngineArgs a{contracts_dev, n_contracts, timesteps, n_paths, 1, 1, mc_seed, ordinal_dev, ordinal0,
               scheme, 0, SMC_STORE_ALL, 1, 1, paths_dev, rowsum_dev, nullptr};
  return dispatch_engine(a, dtype, as_stream(stream));
}

int32_t smc_gbm_normalize(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int64_t n_paths,
                          int32_t dtype, void* paths_dev, const double* rowsum_dev, void* stream) {
  if (int32_t st = validate_common(contracts_dev, n_contracts, timesteps, n_paths, dtype)) return st;
  if (!paths_dev || !rowsum_dev) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_gbm_normalize: NULL buffer");
  const int64_t rows = n_contracts * timesteps;
  if (rows == 0) return SMC_OK;
  const unsigned blocks = static_cast<unsigned>(rows < 65536 ? rows : 65536);
  if (dtype == SMC_DTYPE_F32)
    hipLaunchKernelGGL(normalize_kernel<float>, dim3(blocks), dim3(256), 0, as_stream(stream), contracts_dev,
                       n_contracts, timesteps, n_paths, static_cast<float*>(paths_dev), rowsum_dev);
  else
    hipLaunchKernelGGL(normalize_kernel<double>, dim3(blocks), dim3(256), 0, as_stream(stream), contracts_dev,
                       n_contracts, timesteps, n_paths, static_cast<double*>(paths_dev), rowsum_dev);
  return check_launch("normalize_kernel");
}

int32_t smc_cf_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int32_t network_size,
                       int32_t batches_per_mc_run, int32_t normalization, int32_t dtype, const void* paths_dev,
                       const double* rowsum_dev, void* targets_dev, void* stream) {
  const int64_t P = static_cast<int64_t>(network_size) * batches_per_mc_run;
  if (network_size <= 0 || batches_per_mc_run <= 0)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_cf_targets: network_size and batches_per_mc_run must be > 0");
  if (int32_t st = validate_common(contracts_dev, n_contracts, timesteps, P, dtype)) return st;
  if (!paths_dev || !rowsum_dev || !targets_dev)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_cf_targets: NULL buffer");
  EngineArgs a{contracts_dev, n_contracts, timesteps, P, network_size, batches_per_mc_run, 0, nullptr, 0,
               SMC_SCHEME_LOG_EULER, normalization != SMC_NORM_RAW, SMC_STORE_ALL, 0, 0,
               const_cast<void*>(paths_dev), const_cast<double*>(rowsum_dev), targets_dev};
  return dispatch_engine(a, dtype, as_stream(stream));
}

int32_t smc_train_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int32_t network_size,
                          int32_t batches_per_mc_run, uint64_t mc_seed, const int64_t* ordinal_dev, int64_t ordinal0,
                          int32_t scheme, int32_t normalization, int32_t dtype, int32_t store_mode, void* paths_dev,
                          int64_t path_pitch, int64_t chunk_contracts, double* rowsum_dev, void* targets_dev,
                          void* stream) {
  const int64_t P = static_cast<int64_t>(network_size) * batches_per_mc_run;
  if (network_size <= 0 || batches_per_mc_run <= 0)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_train_targets: network_size and batches_per_mc_run must be > 0");
  if (int32_t st = validate_common(contracts_dev, n_contracts, timesteps, P, dtype)) return st;
  if (!paths_dev || !targets_dev) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_targets: NULL buffer");
  if (store_mode != SMC_STORE_ALL && store_mode != SMC_STORE_TERMINAL)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_targets: bad store_mode");
  if (!valid_scheme(scheme)) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_targets: bad scheme");
  if (chunk_contracts <= 0) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_targets: chunk_contracts <= 0");
  if (path_pitch != 0 && (path_pitch < P || (path_pitch != P && path_pitch % kPathsPerLane != 0)))
    return fail(SMC_ERR_INVALID_SHAPE, "smc_train_targets: path_pitch must be 0, P, or a multiple of 4 >= P");
  const size_t esz = dtype == SMC_DTYPE_F32 ? sizeof(float) : sizeof(double);
  const size_t csz = dtype == SMC_DTYPE_F32 ? 2 * sizeof(float) : 2 * sizeof(double);
  for (int64_t off = 0; off < n_contracts; off += chunk_contracts) {
    const int64_t nb = n_contracts - off < chunk_contracts ? n_contracts - off : chunk_contracts;
    EngineArgs a{contracts_dev + off * 6, nb, timesteps, P, network_size, batches_per_mc_run, mc_seed,
                 ordinal_dev, ordinal0 + off, scheme, normalization != SMC_NORM_RAW, store_mode, 1,
                 rowsum_dev ? 1 : 0, paths_dev,
                 rowsum_dev ? rowsum_dev + off * timesteps : nullptr,
                 static_cast<char*>(targets_dev) + static_cast<size_t>(off) * network_size * csz, path_pitch};
    (void)esz;
    if (int32_t st = dispatch_engine(a, dtype, as_stream(stream))) return st;
  }
  return SMC_OK;
}

int64_t smc_path_pitch(int64_t n_paths, int32_t dtype) {
  // rows at a power-of-two stride alias in the memory system (a 13 % slower store stream at
  // C2, tools/micro/pitchbench.hip): round the row up to 4 KiB, then make the stride an odd
  // multiple of 4 KiB
  if (n_paths <= 0) return 0;
  const int64_t esz = (dtype & 0xff) == SMC_DTYPE_F64 ? 8 : 4;
  const int64_t unit = 4096 / esz;
  int64_t units = (n_paths + unit - 1) / unit;
  if (units % 2 == 0) ++units;
  return units * unit;
}

int32_t smc_normals(uint64_t mc_seed, int64_t ordinal, int32_t rows, int64_t cols, int32_t dtype, void* out_dev,
                    void* stream) {
  if (!out_dev) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_normals: out_dev is NULL");
  if (rows <= 0 || cols <= 0 || ordinal < 0) return fail(SMC_ERR_INVALID_SHAPE, "smc_normals: bad shape");
  const int64_t groups = (cols + kPathsPerLane - 1) / kPathsPerLane;
  const unsigned blocks = static_cast<unsigned>((groups + 255) / 256);
  const bool hw = (dtype & SMC_MATH_HW) != 0;
  dtype &= 0xff;
  if (dtype == SMC_DTYPE_F32 && !hw)
    hipLaunchKernelGGL((normals_kernel<float, false>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<float*>(out_dev));
  else if (dtype == SMC_DTYPE_F32)
    hipLaunchKernelGGL((normals_kernel<float, true>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<float*>(out_dev));
  else if (dtype == SMC_DTYPE_F64)
    hipLaunchKernelGGL((normals_kernel<double, false>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<double*>(out_dev));
  else
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_normals: bad dtype");
  return check_launch("normals_kernel");
}

#pragma GCC visibility pop
}  // extern "C"
