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
#include <cstdlib>

#pragma clang fp contract(off)

#include "smc_internal.h"
#include "smc_sobol.h"
#include "smc_math.h"
#include "smc_rng.h"
#include "smc_device.h"

namespace smc {
namespace {

// rows_kernel occupancy: 8 waves per SIMD (<= 64 VGPRs) = 4 workgroups per CU, so C2's 4096 contracts
// are exactly 4 rounds of 1024 persistent workgroups (at 69 VGPRs: 3 per CU, 5.33 rounds)
// f64: two 8-wave workgroups per CU (4 waves per SIMD) whatever the budget between 4 and 5 waves, and the
// 4-wave budget (97 VGPRs) measured 8.27-8.28 against 8.34-8.35 ms for rows + cf at 5 (91 VGPRs)
// (profiles/r04/ab_f64_waves4.txt)
// (settled values; tools/micro/make_variant.py edits these lines for A/B builds)
constexpr int kRowsWavesF64 = 4;
constexpr int kRowsWaves = 8;
constexpr int kThreads = 512;
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
  int32_t slices;             // workgroups per contract (>= 1); > 1 needs the workspace below
  double* partials;           // [B][slices][all_rows ? T : 1] slice row sums (slices > 1)
  uint32_t* arrivals;         // [B] arrival counters, zero between launches (slices > 1)
  uint32_t* queues;           // [16] queue_kernel work counters, zero between launches (slices > 1)
  // fused training step (smc_train_step, resident_kernel only): each workgroup draws its own
  // contracts' Sobol rows, and the last workgroup to finish advances the cursor
  const uint32_t* sobol;      // table image (smc_sobol_export_tables) or NULL
  int32_t sobol_dim;          // == 6 (BlackScholes.Inputs)
  const double* lower;
  const double* upper;
  double* contracts_out;      // [B][6] f64
  float* cvnn_out;            // [B][6] f32 CVNN input or NULL
  int64_t* cursor;            // [2]: Sobol index, normal ordinal of the step's first contract
  int64_t sobol_index0;       // Sobol index offset of contract 0 of this launch (rank * B)
  int64_t advance;            // cursor[0..1] += advance after the launch
  uint32_t* done;             // workgroups finished, zero between launches
  // sliced resident_kernel (smc_train_step, P > 65,536): res_slices workgroups per contract
  // exchange their terminal sums and column sums through the sync area (res_slices <= 1: whole
  // contracts, none of these are read)
  int32_t res_slices;
  int32_t res_groups;         // capacity of the sync area in groups
  uint32_t* res_cnt;          // [groups][64]: terminal-sum arrivals at +0, column-sum arrivals at +32
  double* res_xsum;           // [groups][2][W + 1] slice terminal sums + the group's next contract
                              // (2: contract round parity)
  double* res_xcol;           // [groups][2][W][N] slice column sums of the put payoffs
  // whole-contract resident_kernel in smc_train_step: the last quarter of the contract rounds is
  // handed out from this counter (zero between launches) instead of statically, so workgroups on
  // XCDs with more write bandwidth take more contracts (NULL: all static)
  uint32_t* res_queue;
  // share of the contract rounds assigned statically, in quarters (the rest from res_queue); 0 with
  // SMC_TRAIN_DYNAMIC: every contract from the queue
  int32_t res_static_q = 3;
  // sliced resident_kernel: the sync area's sticky status word (SMC_SYNC_STATUS_OFFSET), this launch's
  // failure flag (SMC_SYNC_LAUNCH_FAIL_OFFSET, cleared by the last workgroup), the poll budget of an
  // exchange and the smc_test_exchange_fault hook (withhold: slice W-1 of group 0 skips its first
  // terminal-sum arrival)
  uint32_t* status;
  uint32_t* launch_fail;
  uint32_t spin_limit;
  int32_t withhold;
};

constexpr int kSliceChunks = 4;  // chunks (of kChunk paths) per workgroup when sliced



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


__device__ __forceinline__ Contract load_contract(const double* c) {
  return Contract{c[0], c[1], c[2], c[3], c[4], c[5]};
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// One step of the path recursion.  f32 log-Euler works in log2 units (coefficients
// pre-scaled by log2 e) with the portable exp2 of smc_math.h; f64 in units of ln 2 / 256 with
// smc_math.h mul_exp2s_f64.
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
      const double scale = sizeof(Real) == 4 ? kLog2e : math::kExpUnit;  // f64: units of ln 2 / 256
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
      else return math::mul_exp2s_f64(x, fma(b, z, a));
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
// STRAIGHT (with FULLBLOCK, T == kRowBlock): t == i, the terminal row is i == 15 and every store
// (every row with STRAIGHT_ALL, else the terminal row only) is unconditional, so the 16-row block is
// straight-line code — no per-row branches and no per-row condition masks (which otherwise spill
// SGPRs into VGPR lanes).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS, bool MASKED, bool FULLBLOCK, bool STRAIGHT = false,
          bool STRAIGHT_ALL = true>
__device__ __forceinline__ void lane_paths(const EngineArgs& a, const Stepper<Real, LOG_EULER, HW>& step, Real x0,
                                           uint64_t ordinal, int64_t chunk, int nvalid, int t0, int nrows,
                                           Real* contract_base, double (&acc)[ALLROWS ? kRowBlock : 1],
                                           Real* x_out = nullptr, int lid = -1) {
  using V4 = typename Vec4T<Real>::type;
  const int T = a.T;
  const int64_t P = a.P;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const bool store_all = STRAIGHT ? STRAIGHT_ALL : a.store == SMC_STORE_ALL;
  const int lane_id = lid < 0 ? static_cast<int>(threadIdx.x) : lid;  // the lane's 4-path slot in the chunk
  const int64_t p0 = chunk + kPathsPerLane * static_cast<int64_t>(lane_id);
  PathStream s(a.seed, ordinal, static_cast<uint64_t>(p0 / kPathsPerLane), T);  // the lane's group stream
  // f32 HW log-Euler: the RNG hands back the step exponents directly (packed path pairs); f64
  // log-Euler: the exponents too (b folded into the Box-Muller radius), x *= 2^(y/256) (mul_exp2s_f64)
  constexpr bool kPacked = HW && LOG_EULER && sizeof(Real) == 4;
  constexpr bool kY64 = LOG_EULER && sizeof(Real) == 8;
  Real x[kPathsPerLane], zl[kPathsPerLane], zh[kPathsPerLane];
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) x[j] = x0;
  for (int t = 0; t < (STRAIGHT ? 0 : t0); t += 2) {  // t0 is a multiple of kRowBlock (even)
    if constexpr (kPacked) {
      s.hw_log_increments4(step.b, step.a, zl, zh);
      advance_packed(x, zl);
      advance_packed(x, zh);
    } else if constexpr (kY64) {
      s.f64_log_increments4(step.b, step.a, zl, zh);
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) x[j] = math::mul_exp2s_f64(math::mul_exp2s_f64(x[j], zl[j]), zh[j]);
    } else {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(zl[j], zh[j]);
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(step(x[j], zl[j]), zh[j]);
    }
  }
  // wave-uniform row base (SGPR pair) + 32-bit per-lane byte offset
  const uint32_t lane_off = static_cast<uint32_t>(kPathsPerLane * sizeof(Real)) * static_cast<uint32_t>(lane_id);
  Real* chunk_base = contract_base + chunk;
  const __amdgpu_buffer_rsrc_t contract_rsrc = row_rsrc(contract_base);
#pragma unroll
  for (int i = 0; i < kRowBlock; ++i) {
    if (FULLBLOCK || i < nrows) {
      const int t = STRAIGHT ? i : t0 + i;
      // step pairs draw one Box-Muller pair per path; the last step of an odd T (only in a partial
      // block) two pairs for the 4 paths (smc_rng.h draw order)
      const bool tail = !FULLBLOCK && t + 1 == T;
      if constexpr (kPacked) {
        if ((i & 1) == 0) {
          if (tail) s.hw_log_tail4(step.b, step.a, zl);
          else s.hw_log_increments4(step.b, step.a, zl, zh);
        }
        advance_packed(x, (i & 1) ? zh : zl);
      } else if constexpr (kY64) {
        if ((i & 1) == 0) {
          if (tail) s.f64_log_tail4(step.b, step.a, zl);
          else s.f64_log_increments4(step.b, step.a, zl, zh);
        }
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) x[j] = math::mul_exp2s_f64(x[j], (i & 1) ? zh[j] : zl[j]);
      } else {
        if ((i & 1) == 0) {
          if (tail) {
            s.template normal_tail<HW>(zl);
          } else {
#pragma unroll
            for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(zl[j], zh[j]);
          }
        }
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(x[j], (i & 1) ? zh[j] : zl[j]);
      }
      const bool last = STRAIGHT ? i == kRowBlock - 1 : t == T - 1;
      if (store_all || last) {
        char* row = reinterpret_cast<char*>(chunk_base + (store_all ? static_cast<int64_t>(t) * pitch : 0));
        // the terminal row is read back by the CF phase (maybe another workgroup's): write-through
        const bool handoff = last && (STRAIGHT || a.targets != nullptr);
        if constexpr (STRAIGHT && !MASKED && sizeof(Real) == 4) {
          // one buffer descriptor on the contract base; the row offset goes in soffset (SALU adds), so
          // a row store costs no 64-bit VALU address add
          typedef float v4f __attribute__((ext_vector_type(4)));
          const v4f v4 = {x[0], x[1], x[2], x[3]};
          const uint32_t soff = static_cast<uint32_t>((chunk + (store_all ? static_cast<int64_t>(t) * pitch : 0)) *
                                                      static_cast<int64_t>(sizeof(Real)));
          if (handoff) __builtin_amdgcn_raw_buffer_store_b128(v4, contract_rsrc, lane_off, soff, 16 /* sc1 */);
          else __builtin_amdgcn_raw_buffer_store_b128(v4, contract_rsrc, lane_off, soff, 0);
        } else if constexpr (!MASKED) {
          V4 v4;
          v4.x = x[0];
          v4.y = x[1];
          v4.z = x[2];
          v4.w = x[3];
          if (handoff) store_wt(row, lane_off, v4);
          else *reinterpret_cast<V4*>(row + lane_off) = v4;
        } else {
          Real* r = reinterpret_cast<Real*>(row + lane_off);
#pragma unroll
          for (int j = 0; j < kPathsPerLane; ++j) {
            if (j < nvalid) {
              if (handoff) put_sc1(r + j, x[j]);
              else r[j] = x[j];
            }
          }
        }
      }
      if (ALLROWS || last) {
        Real part = 0;
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) part += (!MASKED || j < nvalid) ? x[j] : Real(0);
        acc[ALLROWS ? i : 0] += static_cast<double>(part);
      }
    }
  }
  if (x_out) {  // the lane's final values (the terminal row when t0 + nrows == T)
#pragma unroll
    for (int j = 0; j < kPathsPerLane; ++j) x_out[j] = x[j];
  }
}

// The lane's 4 paths p0..p0+3 through all T rows in one rolled loop over step pairs (any T >= 1):
// the stream, the draw order (one Box-Muller pair per path and step pair; an odd T's last step two
// pairs for the 4 paths) and the arithmetic are lane_paths'; x and the generator
// stay in registers from row to row (no replay of earlier rows, no per-row branches).  STORE_ALL:
// row t at row_base + t * pitch; else only the terminal row, at row_base.  The lane's 4 terminal
// values go to x_out and their sum (f32 sum for f32 paths, then f64) is added to acc.
// lane_rows_s: the same on a stream the caller positioned at the group's first draw (wave_kernel walks
// a whole stream span, smc_rng.h).
// stage (LDS, optional): the rows go there instead of to HBM, row r at stage + r * stage_stride + 4 lane_id
template <typename Real, bool LOG_EULER, bool HW, bool STORE_ALL>
__device__ __forceinline__ void lane_rows_s(PathStream& s, const Stepper<Real, LOG_EULER, HW>& step, Real x0,
                                            int64_t chunk, Real* contract_base, int T, int64_t pitch, double& acc,
                                            Real (&x_out)[kPathsPerLane], int lane_id, Real* stage = nullptr,
                                            int stage_stride = 0);

template <typename Real, bool LOG_EULER, bool HW, bool STORE_ALL>
__device__ __forceinline__ void lane_rows(const EngineArgs& a, const Stepper<Real, LOG_EULER, HW>& step, Real x0,
                                          uint64_t ordinal, int64_t chunk, Real* contract_base, int T, int64_t pitch,
                                          double& acc, Real (&x_out)[kPathsPerLane], int lid = -1) {
  const int lane_id = lid < 0 ? static_cast<int>(threadIdx.x) : lid;  // the lane's 4-path slot in the chunk
  const int64_t p0 = chunk + kPathsPerLane * static_cast<int64_t>(lane_id);
  PathStream s(a.seed, ordinal, static_cast<uint64_t>(p0 / kPathsPerLane), T);
  lane_rows_s<Real, LOG_EULER, HW, STORE_ALL>(s, step, x0, chunk, contract_base, T, pitch, acc, x_out, lane_id);
}

template <typename Real, bool LOG_EULER, bool HW, bool STORE_ALL>
__device__ __forceinline__ void lane_rows_s(PathStream& s, const Stepper<Real, LOG_EULER, HW>& step, Real x0,
                                            int64_t chunk, Real* contract_base, int T, int64_t pitch, double& acc,
                                            Real (&x_out)[kPathsPerLane], int lane_id, Real* stage,
                                            int stage_stride) {
  using V4 = typename Vec4T<Real>::type;
  constexpr bool kPacked = HW && LOG_EULER && sizeof(Real) == 4;
  constexpr bool kY64 = LOG_EULER && sizeof(Real) == 8;  // exponents drawn directly (lane_paths)
  Real x[kPathsPerLane], zl[kPathsPerLane], zh[kPathsPerLane];
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) x[j] = x0;
  const uint32_t lane_off = static_cast<uint32_t>(kPathsPerLane * sizeof(Real)) * static_cast<uint32_t>(lane_id);
  const char* row = reinterpret_cast<const char*>(contract_base + chunk);
  const int64_t rstride = STORE_ALL ? pitch * static_cast<int64_t>(sizeof(Real)) : 0;
  auto draw = [&] {
    if constexpr (kPacked) {
      s.hw_log_increments4(step.b, step.a, zl, zh);
    } else if constexpr (kY64) {
      s.f64_log_increments4(step.b, step.a, zl, zh);
    } else {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(zl[j], zh[j]);
    }
  };
  auto advance = [&](const Real (&z)[kPathsPerLane]) {
    if constexpr (kPacked) {
      advance_packed(x, z);
    } else if constexpr (kY64) {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) x[j] = math::mul_exp2s_f64(x[j], z[j]);
    } else {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(x[j], z[j]);
    }
  };
  auto store = [&] {
    V4 v;
    v.x = x[0];
    v.y = x[1];
    v.z = x[2];
    v.w = x[3];
    if (stage) {
      *reinterpret_cast<V4*>(stage + kPathsPerLane * lane_id) = v;
      stage += stage_stride;
    } else {
      store_row(row, lane_off, v);
    }
  };
#pragma unroll 1
  for (int t = 0; t + 1 < T; t += 2) {
    draw();
    advance(zl);
    if constexpr (STORE_ALL) store();
    row += rstride;
    advance(zh);
    if constexpr (STORE_ALL) store();
    row += rstride;
  }
  if (T & 1) {  // the last step of an odd T: two Box-Muller pairs for the 4 paths
    if constexpr (kPacked) s.hw_log_tail4(step.b, step.a, zl);
    else if constexpr (kY64) s.f64_log_tail4(step.b, step.a, zl);
    else s.template normal_tail<HW>(zl);
    advance(zl);
    if constexpr (STORE_ALL) store();
  }
  if constexpr (!STORE_ALL) store();
  Real part = 0;
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) {
    part += x[j];
    x_out[j] = x[j];
  }
  acc += static_cast<double>(part);
}

// ---- phase 1: simulate the contract's P paths ----------------------------------------
// Fills lds_tot[0..T) (ALLROWS) or lds_tot[T-1] with the f64 sum over paths of the row(s),
// in a fixed order: per lane sequentially over its chunks, wave butterfly (xor 32..1),
// waves 0..7.  Training needs only the terminal row's sum (its normalisation scale).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__device__ void simulate_contract(const EngineArgs& a, const Contract& c, uint64_t ordinal, int64_t b,
                                  int64_t p_begin, int64_t p_end, double* lds_acc, double* lds_tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = a.T;
  const int64_t P = a.P;
  const bool store_all = a.store == SMC_STORE_ALL;
  const int64_t pitch = a.pitch ? a.pitch : P;
  Real* base = static_cast<Real*>(a.paths) + (store_all ? b * T * pitch : b * pitch);
  const bool vec_ok = (P % kPathsPerLane) == 0;
  const int64_t full_end = vec_ok ? p_begin + ((p_end - p_begin) / kChunk) * kChunk : p_begin;
  const Stepper<Real, LOG_EULER, HW> step(c, T);
  const Real x0 = static_cast<Real>(c.X0);
  constexpr int kAcc = ALLROWS ? kRowBlock : 1;

  for (int t0 = 0; t0 < T; t0 += kRowBlock) {
    const int nrows = T - t0 < kRowBlock ? T - t0 : kRowBlock;
    double acc[kAcc];
#pragma unroll
    for (int i = 0; i < kAcc; ++i) acc[i] = 0.0;
    int64_t chunk = p_begin;
    if (nrows == kRowBlock) {  // branch-free fast path: whole 16-row block, whole 2048-path chunks
      if (T == kRowBlock && store_all) {  // the training shape: straight-line block, every row stored
        for (; chunk < full_end; chunk += kChunk)
          lane_paths<Real, LOG_EULER, HW, ALLROWS, false, true, true>(a, step, x0, ordinal, chunk, kPathsPerLane, 0,
                                                                      kRowBlock, base, acc);
      }
      for (; chunk < full_end; chunk += kChunk)
        lane_paths<Real, LOG_EULER, HW, ALLROWS, false, true>(a, step, x0, ordinal, chunk, kPathsPerLane, t0, nrows,
                                                              base, acc);
    }
    for (; chunk < p_end; chunk += kChunk) {  // everything else: ragged rows / paths, scalar stores
      const int64_t p0 = chunk + kPathsPerLane * tid;
      const int nvalid = static_cast<int>(p0 >= p_end ? 0 : (p_end - p0 >= kPathsPerLane ? kPathsPerLane : p_end - p0));
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
// Reference scalar semantics: gbm.py:429-431 evaluate times/forwards/df in the sim dtype;
// the put is df * max(K - x * scale, 0) with x * scale rounded to the sim dtype (gbm.py:437, 473).
// The contract's payoff constants that do not need the terminal sum (forward F_T, discount df_T,
// strike), taken before a contract's simulation so the f64 contract row need not stay live across it.
template <typename Real>
struct PayoffPre {
  Real F, df, K;
  __device__ explicit PayoffPre(const Contract& c) {
    const Real Tm = static_cast<Real>(c.T);
    if constexpr (sizeof(Real) == 4) {
      F = static_cast<float>(c.X0) * math::exp_any(static_cast<float>(c.r - c.d) * Tm);
      df = math::exp_any(static_cast<float>(-c.r) * Tm);
    } else {
      F = c.X0 * exp((c.r - c.d) * Tm);
      df = exp(-c.r * Tm);
    }
    K = static_cast<Real>(c.K);
  }
};

template <typename Real>
struct Payoff {
  Real s, K, df;
  Payoff() = default;
  __device__ Payoff(const EngineArgs& a, const Contract& c, double terminal_sum)
      : Payoff(a, PayoffPre<Real>(c), terminal_sum) {}
  __device__ Payoff(const EngineArgs& a, const PayoffPre<Real>& pre, double terminal_sum) {
    df = pre.df;
    s = a.normalize ? pre.F / static_cast<Real>(terminal_sum / static_cast<double>(a.P)) : Real(1);
    K = pre.K;
    // a failed exchange hands over a NaN terminal sum: keep the targets NaN (df * max(K - NaN, 0)
    // would be 0, a plausible value) so a caller that skips smc_sync_status still sees it
    if (terminal_sum != terminal_sum) df = static_cast<Real>(__builtin_nan(""));
  }
  __device__ __forceinline__ Real operator()(Real x) const {
    const Real xs = x * s;  // sims *= scale (rounded to Real)
    const Real diff = K - xs;
    return df * (diff > Real(0) ? diff : Real(0));
  }
};

// Real-input N-point DFT of avg[0..N) from the twiddle table -> targets row (bins 0..N/2 and
// their Hermitian mirror); fixed summation order.
template <typename Real>
__device__ void dft_row(const double* avg, const double* cs, const double* sn, int N,
                        typename Complex2<Real>::type* out, int tid = threadIdx.x, int nthreads = kThreads) {
  using C2 = typename Complex2<Real>::type;
  // bins k = 0..N/2-1 over the threads; when N/2 is a multiple of the workgroup the Nyquist bin
  // N/2 would take a whole extra pass for one thread, so thread 0 runs its chain inside its k = 0
  // loop instead (same fma sequence per chain: same bits).  Only for even N with kmax > 0: odd N
  // has no Nyquist bin (bin kmax is an ordinary pair with N - kmax), and N = 1 has only bin 0.
  const int kmax = N / 2;
  const bool fuse_nyq = (N % 2) == 0 && kmax > 0 && kmax % nthreads == 0;
  for (int k = tid; k < kmax || (!fuse_nyq && k == kmax); k += nthreads) {
    const bool nyq = fuse_nyq && k == 0;
    double re = 0.0, im = 0.0, rq = 0.0, iq = 0.0;
    int idx = 0, iqx = 0;
    for (int n = 0; n < N; ++n) {
      re = fma(avg[n], cs[idx], re);
      im = fma(-avg[n], sn[idx], im);
      idx += k;
      if (idx >= N) idx -= N;
      if (nyq) {
        rq = fma(avg[n], cs[iqx], rq);
        iq = fma(-avg[n], sn[iqx], iq);
        iqx += kmax;
        if (iqx >= N) iqx -= N;
      }
    }
    C2 v;
    v.x = static_cast<Real>(re);
    v.y = static_cast<Real>(im);
    out[k] = v;
    if (k != 0 && 2 * k != N) {
      v.y = static_cast<Real>(-im);
      out[N - k] = v;
    }
    if (nyq) {
      v.x = static_cast<Real>(rq);
      v.y = static_cast<Real>(iq);
      out[kmax] = v;
    }
  }
}

// Payoff sums of the f32 terminal row, N % 4 == 0: item (q, g) = column quad q (4 adjacent
// columns, one 16-B load per batch row) over batches m = g, g + G, ... in ascending order, into
// part[g][4q..4q+3].  Items are spread over `nthreads` threads from `tid`; the arithmetic of an
// item does not depend on which thread runs it.  sc1 (L1-bypassing) loads: the row may have been
// written by other workgroups (sliced contracts) or other waves of this one.
template <int kBatch>
__device__ __forceinline__ void quad_column_sums(const float* row, const Payoff<float>& pay, int N, int M,
                                                 int cols, int G, double* part, int tid, int nthreads) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), static_cast<short>(0), 0x7fffffff, 0x00020000);
  const int items = cols * G;
  for (int item = tid; item < items; item += nthreads) {
    const int q = item % cols, g = item / cols;
    double sum[4] = {0.0, 0.0, 0.0, 0.0};
    for (int m0 = g; m0 < M; m0 += G * kBatch) {
      v4f v[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int m = m0 + u * G < M ? m0 + u * G : M - 1;  // clamped: loads stay unconditional
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (m * N + 4 * q) * 4, 0, 16 /* sc1 */);
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        if (m0 + u * G < M) {
#pragma unroll
          for (int e = 0; e < 4; ++e) sum[e] += static_cast<double>(pay(v[u][e]));
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) part[g * N + 4 * q + e] = sum[e];
  }
}

// Power-of-two N (2..2048): the targets come from an in-LDS radix-2 FFT instead of the O(N^2)
// DFT (at C3, N = 1024, the DFT chains were ~20 us per contract).  oracle/gbm_oracle.c restates
// both; the CF phase's LDS work area holds the FFT's re / im arrays in place of the group sums.
__host__ __device__ inline bool use_fft(int N) { return N >= 2 && (N & (N - 1)) == 0 && N <= 2048; }
__host__ __device__ inline int cf_part_doubles(int N) {
  const int need = use_fft(N) ? 2 * N : N;
  return need > 4 * kThreads ? need : 4 * kThreads;
}


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
  const Payoff<Real> pay(a, c, terminal_sum);

  // f32 rows of N % 4 == 0 columns: each thread sums 4 adjacent columns from 16-B loads
  // (256 B in flight per lane, 128 KiB per workgroup); otherwise one column per thread.
  // Column n's batches m = g, g + G, ... are summed by one thread (group g), then the G
  // group sums in g order.
  const bool quad = sizeof(Real) == 4 && (N % 4) == 0 && (pitch % 4) == 0 && P < (int64_t{1} << 29);
  const int cols = quad ? N / 4 : N;
  const int G = cols <= kThreads ? kThreads / cols : 1;
  const int items = cols * G;
  double* part = lds;                                            // [cf_part_doubles(N)]
  double* avg = part + cf_part_doubles(N);                       // [N]
  double* cs = avg + N;                                          // [N]
  double* sn = cs + N;                                           // [N]

  constexpr int kBatch = 8;  // loads in flight per thread; the sum keeps the m order
  if constexpr (sizeof(Real) == 4) {
    if (quad) quad_column_sums<kBatch>(row, pay, N, M, cols, G, part, tid, kThreads);
  }
  for (int item = tid; item < items && !quad; item += kThreads) {
    const int n = item % N, g = item / N;
    double sum = 0.0;
    for (int m0 = g; m0 < M; m0 += G * kBatch) {
      Real v[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int m = m0 + u * G < M ? m0 + u * G : M - 1;  // clamped: loads stay unconditional
        v[u] = get_sc1(row + static_cast<int64_t>(m) * N + n);  // written by the slices' sc1 stores
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        if (m0 + u * G < M) sum += static_cast<double>(pay(v[u]));
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
  if (use_fft(N)) fft_row<Real, kThreads>(avg, cs, sn, N, part, part + N, static_cast<C2*>(a.targets) + b * N);
  else dft_row<Real>(avg, cs, sn, N, static_cast<C2*>(a.targets) + b * N);
}

// Slice k of contract b (paths [k S, (k+1) S), S = kSliceChunks * kChunk; the whole contract
// when slices == 1), then — for the workgroup that completes the contract — the CF phase.
// With slices > 1 every slice publishes its row sums (write-through) and arrives on the
// contract's counter; the last arriver sums the W slice sums in slice order 0..W-1 (a fixed
// order: bit-reproducible, oracle "sliced" mode) and runs the CF phase on the terminal row,
// which the slices wrote moments ago (write-through stores drained before arriving, L1-bypassing
// loads after: MI355X_MICROARCH.md, inter-workgroup visibility, valid forms).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__device__ void run_slice(const EngineArgs& a, int64_t b, int k, double* lds, int* lds_flag) {
  const int W = a.slices;
  const Contract c = load_contract(a.contracts + b * 6);
  const int T = a.T;
  double* lds_tot = lds;               // [T]
  double* lds_work = lds + T;          // simulate: [kWaves][T]; cf: part/avg/cs/sn
  double terminal_sum;
  if (a.simulate) {
    const uint64_t ordinal = static_cast<uint64_t>((a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0 + b);
    const int64_t span = W == 1 ? a.P : static_cast<int64_t>(kSliceChunks) * kChunk;
    const int64_t p_begin = k * span;
    const int64_t p_end = p_begin + span < a.P ? p_begin + span : a.P;
    simulate_contract<Real, LOG_EULER, HW, ALLROWS>(a, c, ordinal, b, p_begin, p_end, lds_work, lds_tot);
    if (W > 1) {
      // publish this slice's row sums, drain every wave's write-through stores, then arrive
      const int rows = ALLROWS ? T : 1;
      double* mine = a.partials + (b * W + k) * rows;
      for (int t = threadIdx.x; t < rows; t += kThreads) put_sc1(mine + t, lds_tot[ALLROWS ? t : T - 1]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint32_t before = __hip_atomic_fetch_add(a.arrivals + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_flag = before == static_cast<uint32_t>(W - 1);
        if (*lds_flag) __hip_atomic_store(a.arrivals + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!*lds_flag) return;
      const double* all = a.partials + b * W * rows;
      for (int t = threadIdx.x; t < rows; t += kThreads) {
        double tot = 0.0;
        for (int j = 0; j < W; ++j) tot += get_sc1(all + j * rows + t);
        lds_tot[ALLROWS ? t : T - 1] = tot;
      }
      __syncthreads();
    }
    if (ALLROWS && a.rowsum)
      for (int t = threadIdx.x; t < T; t += kThreads) a.rowsum[b * T + t] = lds_tot[t];
    terminal_sum = lds_tot[T - 1];
  } else {
    terminal_sum = a.rowsum[b * T + (T - 1)];
  }
  if (!ALLROWS && a.rowsum && threadIdx.x == 0 && a.simulate) a.rowsum[b * T + (T - 1)] = terminal_sum;
  if (a.targets) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's own terminal-row stores
    __syncthreads();
    cf_targets_contract<Real>(a, c, b, terminal_sum, lds_work);
  }
  __syncthreads();  // LDS is reused by the workgroup's next item
}

// One workgroup per contract (slices == 1).
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__global__ __launch_bounds__(kThreads) void contract_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  __shared__ int flag;
  if constexpr (sizeof(Real) == 8) math::f64_tables_load();
  run_slice<Real, LOG_EULER, HW, ALLROWS>(a, blockIdx.x, 0, lds, &flag);
}

// ---- split training pair: paths_kernel, then cf_kernel --------------------------------------
// The fused contract_kernel runs each round of resident workgroups into a chip-wide CF phase
// (every workgroup drains, re-reads its terminal row and evaluates the DFT at about the same
// time).  Split in two launches instead: paths_kernel simulates and stores every contract and
// leaves the terminal-row sum (f64, the normalisation's input) in that row's padding column;
// cf_kernel then streams all terminal rows back at full read bandwidth, one workgroup per
// contract.  Same arithmetic and orders as contract_kernel: bit-identical targets.
// f32 scratch only (split_ok): the first 8-B-aligned padding slot after column P of the terminal row
// (f64 scratch: the first element after column P)
template <typename Real = float>
__device__ __forceinline__ double* pad_sum(const EngineArgs& a, int64_t b) {
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  const int64_t row = a.store == SMC_STORE_ALL ? (b * a.T + (a.T - 1)) * pitch : b * pitch;
  return reinterpret_cast<double*>(static_cast<Real*>(a.paths) + row + a.P + (sizeof(Real) == 4 ? (a.P & 1) : 0));
}

// STRAIGHT (T == 16, P a multiple of 2048): only the straight-line 16-row block is compiled in
// (STORE_ALL: every row; else the terminal row), so the kernel needs ~60 VGPRs instead of ~100.
// The terminal sum keeps simulate_contract's order: lane over chunks, wave butterfly, waves 0..7.
// STRAIGHT launches are persistent: the resident workgroups run contracts b = blockIdx.x,
// + gridDim.x, ... back to back, so no workgroup drains its store queue between contracts (a
// wave retires only once its stores are acknowledged) and the chip never runs whole rounds of
// workgroups that start, ramp up and drain together.  The per-contract barrier is LDS-only.
template <bool LOG_EULER, bool HW, bool STRAIGHT, bool STORE_ALL>
__global__ __launch_bounds__(kThreads) void paths_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  if constexpr (STRAIGHT) {
    const int64_t pitch = a.pitch ? a.pitch : a.P;
    int parity = 0;
    for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x, parity ^= 1) {
      const Contract c = load_contract(a.contracts + b * 6);
      const Stepper<float, LOG_EULER, HW> step(c, kRowBlock);
      const float x0 = static_cast<float>(c.X0);
      float* base = static_cast<float*>(a.paths) + (STORE_ALL ? b * kRowBlock * pitch : b * pitch);
      double acc[1] = {0.0};
      for (int64_t chunk = 0; chunk < a.P; chunk += kChunk)
        lane_paths<float, LOG_EULER, HW, false, false, true, true, STORE_ALL>(
            a, step, x0, static_cast<uint64_t>(ord0 + b), chunk, kPathsPerLane, 0, kRowBlock, base, acc);
      // wave sums in a double-buffered LDS slot: the next contract writes the other slot
      const double w = wave_sum(acc[0]);
      double* ws = lds + parity * kWaves;
      if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = w;
      lds_barrier();
      if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int k = 0; k < kWaves; ++k) tot += ws[k];
        *pad_sum(a, b) = tot;
      }
    }
  } else {
    const int64_t b = blockIdx.x;
    const Contract c = load_contract(a.contracts + b * 6);
    const uint64_t ordinal = static_cast<uint64_t>(ord0 + b);
    simulate_contract<float, LOG_EULER, HW, false>(a, c, ordinal, b, 0, a.P, lds + a.T, lds);
    if (threadIdx.x == 0) *pad_sum(a, b) = lds[a.T - 1];
  }
}

template <typename Real>
__global__ __launch_bounds__(kThreads) void cf_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  const int64_t b = blockIdx.x;
  const Contract c = load_contract(a.contracts + b * 6);
  cf_targets_contract<Real>(a, c, b, *pad_sum<Real>(a, b), lds);
}

// rows_kernel: the split pair's path kernel for any T (f64 and the f32 shapes the resident kernel
// does not take): persistent workgroups (contracts blockIdx.x, + gridDim.x, ...), every lane's 4 paths
// of each 2048-path chunk through all T rows in registers (lane_rows: no replay, one rolled loop), the
// f64 terminal-row sum into the row padding for cf_kernel.  Terminal-sum order: lane over its chunks,
// wave butterfly, waves 0..7 (oracle kernel mode, wg = 512; paths_kernel's order).
// Contracts are assigned statically: the round-3 contract queue (every contract after the first from a
// counter, for workgroups that start late beside a network kernel) cost a store drain per contract at
// its queue barrier, and rows shapes run the step on one stream anyway (round 4, C2-f64: rows_kernel
// 7.64 ms with the queue against ~6.9 without).
// f64 rows: kRowsWavesF64 sets the register budget (round 4 A/Bs on MI355X, C2-f64: v2 math 9.01 ms
// at 6 vs 9.20-9.28 ms at 8 waves, and 9.49-9.53 ms with the CF phase fused into this kernel, which then
// re-read the terminal row while its own path math waited; v3 math 8.47-8.50 ms at 5 vs 8.65-8.67 ms at
// 6, where the 80-VGPR budget spilled outside the path loop): the larger register budget is worth more
// than the sixth wave.
template <typename Real, bool LOG_EULER, bool HW, bool STORE_ALL>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(sizeof(Real) == 8 ? kRowsWavesF64
                                                                                              : kRowsWaves)))
void rows_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  if constexpr (sizeof(Real) == 8) math::f64_tables_load();
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  const int T = a.T;
  int parity = 0;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x, parity ^= 1) {
    const Contract c = load_contract(a.contracts + b * 6);
    const Stepper<Real, LOG_EULER, HW> step(c, T);
    const Real x0 = static_cast<Real>(c.X0);
    Real* base = static_cast<Real*>(a.paths) + (STORE_ALL ? b * T * pitch : b * pitch);
    double acc = 0.0;
    for (int64_t chunk = 0; chunk < a.P; chunk += kChunk) {
      Real xt[kPathsPerLane];
      lane_rows<Real, LOG_EULER, HW, STORE_ALL>(a, step, x0, static_cast<uint64_t>(ord0 + b), chunk, base, T, pitch,
                                                acc, xt);
    }
    // wave sums in a double-buffered LDS slot: the next contract writes the other slot
    const double w = wave_sum(acc);
    double* ws = lds + parity * kWaves;
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = w;
    lds_barrier();
    if (threadIdx.x == 0) {
      double tot = 0.0;
      for (int k = 0; k < kWaves; ++k) tot += ws[k];
      *pad_sum<Real>(a, b) = tot;
    }
  }
}

// ---- reference arithmetic (SMC_MATH_REF): the reference kernel's own f32 typing --------------------
// The reference's SimulateBlackScholes (gbm.py:224-257) is a Numba kernel whose scalar arguments are
// Python floats: X, dt, sqrt_dt, the drift and the exponent are f64, only the io matrix (normals in,
// paths out) is f32 -- per step dW = z sqrt_dt (z widened), X *= exp(drift dt + v dW) (log-Euler) or
// X += drift X dt + v X dW, X = |X| (simple Euler), io = (float) X.  rows_ref_kernel computes that: the
// portable f32 normals (bit-identical to the oracle), the f64 engine's step (Stepper<double>; e^y by
// smc_math.h mul_exp2s_f64, within 2 ulp of libm), f32 stores of the rounded state, and the f32
// pipeline's terminal sum and CF phase (cf_kernel<float>).  Any P: a lane past P draws and stores
// nothing (stream positions never depend on P), a lane straddling P stores its valid paths one by one.
// Terminal-sum order of rows_kernel (oracle kernel mode with step64, wg = 512).
// HWN (SMC_MATH_REF | SMC_MATH_HW): the same draws through the hardware-transcendental Box-Muller
// (normal_pair<true>, rescaled to N(0, 1) in f32), the f64 step unchanged: the portable normals' software
// log / sincos were ~40 % of the launch (C2: 4.56 against 6.57 ms, profiles/r06/ab_refmath_hw_normals.txt)
template <bool LOG_EULER, bool STORE_ALL, bool HWN>
__device__ __forceinline__ void lane_rows_ref(const EngineArgs& a, const Stepper<double, LOG_EULER, false>& step,
                                              double x0, uint64_t ordinal, int64_t chunk, float* contract_base,
                                              int T, int64_t pitch, double& acc) {
  const int lane_id = static_cast<int>(threadIdx.x);
  const int64_t p0 = chunk + kPathsPerLane * static_cast<int64_t>(lane_id);
  const int nvalid = a.P - p0 >= kPathsPerLane ? kPathsPerLane : (a.P > p0 ? static_cast<int>(a.P - p0) : 0);
  PathStream s(a.seed, ordinal, static_cast<uint64_t>(p0 / kPathsPerLane), T);
  double x[kPathsPerLane];
  float zl[kPathsPerLane], zh[kPathsPerLane];
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) x[j] = x0;
  const uint32_t lane_off = static_cast<uint32_t>(kPathsPerLane * sizeof(float)) * static_cast<uint32_t>(lane_id);
  const char* row = reinterpret_cast<const char*>(contract_base + chunk);
  const int64_t rstride = STORE_ALL ? pitch * static_cast<int64_t>(sizeof(float)) : 0;
  auto advance = [&](const float (&z)[kPathsPerLane]) {
#pragma unroll
    for (int j = 0; j < kPathsPerLane; ++j) x[j] = step(x[j], static_cast<double>(z[j]));
  };
  auto store = [&] {
    const float4 v = {static_cast<float>(x[0]), static_cast<float>(x[1]), static_cast<float>(x[2]),
                      static_cast<float>(x[3])};
    if (nvalid == kPathsPerLane) {
      store_row(row, lane_off, v);
    } else if (nvalid > 0) {
      float* r = reinterpret_cast<float*>(const_cast<char*>(row) + lane_off);
      const float w[kPathsPerLane] = {v.x, v.y, v.z, v.w};
      for (int j = 0; j < nvalid; ++j) r[j] = w[j];
    }
  };
  constexpr float kz = static_cast<float>(PathStream::kNormalScale<HWN>);  // 1 for the portable normals
#pragma unroll 1
  for (int t = 0; t + 1 < T; t += 2) {
#pragma unroll
    for (int j = 0; j < kPathsPerLane; ++j) {
      s.template normal_pair<HWN>(zl[j], zh[j]);
      if constexpr (HWN) {
        zl[j] *= kz;
        zh[j] *= kz;
      }
    }
    advance(zl);
    if constexpr (STORE_ALL) store();
    row += rstride;
    advance(zh);
    if constexpr (STORE_ALL) store();
    row += rstride;
  }
  if (T & 1) {  // the last step of an odd T: two Box-Muller pairs for the 4 paths
    s.template normal_tail<HWN>(zl);
    if constexpr (HWN) {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) zl[j] *= kz;
    }
    advance(zl);
    if constexpr (STORE_ALL) store();
  }
  if constexpr (!STORE_ALL) store();
  float part = 0.0f;
#pragma unroll
  for (int j = 0; j < kPathsPerLane; ++j) part += j < nvalid ? static_cast<float>(x[j]) : 0.0f;
  acc += static_cast<double>(part);
}

// rows_kernel's persistent contract loop over lane_rows_ref (the f64 step's tables in LDS).  Register budget:
// 6 waves per SIMD (three 8-wave workgroups per CU with the 51 KB table image each): C2 6.59 ms against 6.65
// at 4 and 6.69 at 8 waves (profiles/r05/ab_ref_waves.txt)
constexpr int kRowsRefWaves = 6;
template <bool LOG_EULER, bool STORE_ALL, bool HWN>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kRowsRefWaves)))
void rows_ref_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  math::f64_tables_load();
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  const int T = a.T;
  int parity = 0;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x, parity ^= 1) {
    const Contract c = load_contract(a.contracts + b * 6);
    const Stepper<double, LOG_EULER, false> step(c, T);
    float* base = static_cast<float*>(a.paths) + (STORE_ALL ? b * T * pitch : b * pitch);
    double acc = 0.0;
    for (int64_t chunk = 0; chunk < a.P; chunk += kChunk)
      lane_rows_ref<LOG_EULER, STORE_ALL, HWN>(a, step, c.X0, static_cast<uint64_t>(ord0 + b), chunk, base, T, pitch, acc);
    const double w = wave_sum(acc);
    double* ws = lds + parity * kWaves;
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = w;
    lds_barrier();
    if (threadIdx.x == 0) {
      double tot = 0.0;
      for (int k = 0; k < kWaves; ++k) tot += ws[k];
      *pad_sum<float>(a, b) = tot;
    }
  }
}

// ---- resident_kernel: the terminal row never leaves the chip -----------------------------------
// For P <= 65,536 a 1024-thread workgroup (4 paths per lane, 4096-path chunks, <= 16 chunks) keeps
// the contract's whole terminal row on chip next to its stores: chunks 0..7 in LDS (128 KiB, one
// 16-B slot per lane and chunk), later chunks in registers.  Once the contract's terminal sum is
// known the workgroup evaluates the payoffs from there: lane l of chunk c holds batch
// m = g + c G (G = 4096 / N, g = 4 l / N) of column quad q = l mod N/4, so each lane's 4 column
// sums over its chunks are the items (q, g) of the CF phase, summed over m ascending; then the G
// group sums in order, the M-mean and the FFT (N divides 4096).  No re-read of the terminal row
// (1.07 GB per C2 step), no CF kernel, no store drain: every barrier is LDS-only.  Persistent: one
// workgroup per CU runs contracts blockIdx.x, + gridDim.x, ...  Reduction orders follow 1024
// lanes (oracle kernel mode, wg = 1024): lane over chunks, wave butterfly, waves 0..15 for the
// terminal sum; item sums in ascending m, groups in order.
//
// Sliced (res_slices = W > 1, smc_train_step only; C3: P = 262,144, W = 4): a group of W
// co-resident workgroups (on one XCD where the grid allows) runs each contract, slice s holding
// paths [s P/W, (s+1) P/W) on chip.  The slices publish their terminal sums, wait for all W
// (the exchange every payoff needs) and add them in slice order; each then publishes its column
// sums, and the last to arrive adds the W of them in slice order, takes the M-mean and runs the
// FFT.  Hand-offs: write-through (sc1) stores by one wave, drained, then an agent-scope add on
// the group's counter; sc1 loads after the poll matched or the add returned
// (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms, first table row).  Counters
// are monotonic within a launch (W per contract round) and reset by the last workgroup.
// Sum over g < G of part[g * N + n] in g order from 0.0, the LDS reads issued 8 at a time
__device__ __forceinline__ double group_sum(const double* part, int n, int G, int N) {
  double t = 0.0;
  for (int g0 = 0; g0 < G; g0 += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(g0 + u < G ? g0 + u : G - 1) * N + n];  // clamped: straight-line
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (g0 + u < G) t += v[u];
  }
  return t;
}

constexpr int kResThreads = 1024;
constexpr int kResWaves = kResThreads / 64;
constexpr int kResChunk = kResThreads * kPathsPerLane;  // 4096 paths
constexpr int kResMaxChunks = 16;
constexpr int kResLdsChunks = 8;                        // chunks parked in LDS
constexpr int kResRegChunks = kResMaxChunks - kResLdsChunks;
constexpr size_t kResTermBytes = static_cast<size_t>(kResLdsChunks) * kResThreads * 16;  // 128 KiB
constexpr int kResMaxSlices = 8;

constexpr int kResPreDraw = 32;  // static contracts whose Sobol rows are drawn at kernel start
constexpr int kResMaxT = 1 << 16;  // bound on T for the rolled (T != 16) row loop

size_t resident_lds_bytes(int N) {
  return kResTermBytes +
         (static_cast<size_t>(kResWaves) + 3 * static_cast<size_t>(N) + 9 + 6 * kResPreDraw) * sizeof(double);
}

// Column sums of the whole-contract CF phase (W = 1, round 4): part[G][N] (G = 4096 / N) as a tree
// instead of N threads adding G terms each: thread (k, n) = (tid / N, tid mod N) adds groups k, k + R,
// k + 2R, k + 3R (R = 1024 / N) in order from 0.0 (consecutive lanes read consecutive columns: no LDS
// bank conflicts); for N < 64 the 64 / N partials a wave holds of a column are added by a butterfly (lane
// offsets 32, 16, ..., N) and the 16 wave sums in wave order, else the R partials in k order.  Then
// avg[n] = sum / M.  The red scratch may alias part (read before the barrier inside).  Oracle:
// kernel_cf(wg=1024, slices=1).
__device__ __forceinline__ void column_sums_tree(const double* part, double* red, double* avg, int N, int M) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = kResThreads / N;
  const int n = tid % N, k = tid / N;
  double p = 0.0;
  if (tid < N * R) {  // N <= 1024 (resident_ok): R >= 1
#pragma unroll
    for (int u = 0; u < 4; ++u) p += part[(k + u * R) * N + n];
  }
  for (int off = 32; off >= N; off >>= 1) p += __shfl_xor(p, off, 64);
  lds_barrier();  // every read of part is done (red may alias it)
  if (N < 64) {
    if (lane < N) red[wave * N + n] = p;
  } else if (tid < N * R) {
    red[k * N + n] = p;
  }
  lds_barrier();
  const int terms = N < 64 ? kResWaves : R;
  for (int c = tid; c < N; c += kResThreads) {
    double t = 0.0;
    for (int w = 0; w < terms; ++w) t += red[w * N + c];
    avg[c] = t / static_cast<double>(M);
  }
}

// ONTHEFLY (RAW normalisation, whole contracts, rolled rows: the reference's lock-step shape): the scale
// is 1, so each chunk's payoffs go into the column sums as the chunk finishes (same chunk order, same
// bits) and no terminal value is parked in LDS or in the register shift register.
template <bool LOG_EULER, bool HW, bool STORE_ALL, bool T16, bool ONTHEFLY = false>
__global__ __launch_bounds__(kResThreads) void resident_kernel(EngineArgs a) {
  static_assert(!(ONTHEFLY && T16), "the on-the-fly CF phase is instantiated for the rolled row loop only");
  typedef float v4f __attribute__((ext_vector_type(4)));
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.N, M = a.M;
  const int64_t P = a.P;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const int W = a.res_slices > 1 ? a.res_slices : 1;
  // group (contract sequence) and slice of this workgroup: blocks b, b + 8, ... share an XCD
  int grp = blockIdx.x, slc = 0;
  if (W > 1) {
    if (gridDim.x % (8 * W) == 0) {
      slc = static_cast<int>((blockIdx.x >> 3) % W);
      grp = static_cast<int>((blockIdx.x & 7) + 8 * (blockIdx.x / (8 * W)));
    } else {
      slc = static_cast<int>(blockIdx.x % W);
      grp = static_cast<int>(blockIdx.x / W);
    }
  }
  const int groups = static_cast<int>(gridDim.x) / W;
  const int nch = static_cast<int>(P / (static_cast<int64_t>(W) * kResChunk));  // chunks of this slice
  const int cols = N / 4;
  const int G = kResChunk / N;            // batch rows per chunk
  const int q = tid % cols, g = tid / cols;
  v4f* term_lds = reinterpret_cast<v4f*>(lds);                      // [kResLdsChunks][kResThreads]
  double* part = lds;                     // [G][N] = [4096], aliases term_lds once it is consumed;
                                          // FFT re / im after the M-mean
  double* wsum = lds + kResTermBytes / sizeof(double);              // [kResWaves]
  double* avg = wsum + kResWaves;         // [N]
  double* cs = avg + N;                   // [N]
  double* sn = cs + N;                    // [N]
  double* row = sn + N;                   // [6] this contract's drawn Sobol row (fused step); [6]
                                          // the exchanged terminal sum, [7] the last-arriver flag,
                                          // [8] the next dynamically handed-out contract;
  double* pre = row + 9;                  // [kResPreDraw][6] Sobol rows of the first static contracts
  for (int j = tid; j < N; j += kResThreads) math::twiddle(j, N, sn[j], cs[j]);
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int64_t sob0 = a.sobol ? a.cursor[0] + a.sobol_index0 : 0;
  uint32_t round = 0;
  // contracts grp, grp + groups, ... up to n_static; then (res_queue) the rest from the counter, one
  // at a time: the per-XCD write rate differs by up to ~10 % (profiles/r02 trace), and a static
  // split ends at the slowest XCD
  // (sliced, W > 1: slice 0 takes the group's next contract during the current contract's
  // terminal-sum exchange, and the partners read it with the sums; only once every group has a
  // static contract, n_static > 0)
  // (a.res_static_q: the statically assigned share of the contract rounds, in quarters)
  const int64_t n_static0 = (a.B / groups) * a.res_static_q / 4 * groups;
  const bool dyn = a.res_queue != nullptr && (W == 1 || n_static0 > 0);
  const int64_t n_static = dyn ? n_static0 : a.B;
  auto grab = [&]() -> int64_t {
    if (tid == 0) reinterpret_cast<int64_t*>(row + 8)[0] = n_static + atomicAdd(a.res_queue, 1u);
    lds_barrier();
    return reinterpret_cast<const int64_t*>(row + 8)[0];
  };
  auto next = [&](int64_t b) -> int64_t {
    if (b + groups < n_static) return b + groups;
    if (!dyn) return a.B;
    if (W == 1) return grab();
    return reinterpret_cast<const int64_t*>(row + 8)[0];  // learned in this contract's exchange
  };
  // the Sobol rows of the first kResPreDraw static contracts are drawn here, before any path store:
  // a global load in a wave waits for that wave's outstanding stores (one vmcnt counter), so a
  // per-contract draw made wave 0 drain its store queue at every contract start
  int64_t n_pre = 0;
  if (a.sobol) {
    const int64_t mine = grp < n_static ? (n_static - 1 - grp) / groups + 1 : 0;
    n_pre = mine < kResPreDraw ? mine : kResPreDraw;
    for (int t = tid; t < n_pre * 6; t += kResThreads) {
      const int k = t / 6, d = t % 6;
      const int64_t bb = grp + static_cast<int64_t>(k) * groups;
      const double v = sobol_coord(a.sobol, a.sobol_dim, d, static_cast<uint64_t>(sob0 + bb), a.lower, a.upper);
      pre[t] = v;
      if (slc == 0) {
        a.contracts_out[bb * 6 + d] = v;
        if (a.cvnn_out) a.cvnn_out[bb * 6 + d] = static_cast<float>(v);
      }
    }
    lds_barrier();
  }
  for (int64_t b = grp < n_static ? grp : (dyn ? grab() : a.B); b < a.B; b = next(b), ++round) {
    Contract c;
    if (a.sobol && static_cast<int64_t>(round) < n_pre) {  // drawn at kernel start
      const double* r = pre + static_cast<int64_t>(round) * 6;
      c = Contract{r[0], r[1], r[2], r[3], r[4], r[5]};
    } else if (a.sobol) {  // draw the contract (sobol_sampler.py:222-246) instead of a separate kernel
      if (tid < 6) {
        const double v = sobol_coord(a.sobol, a.sobol_dim, tid, static_cast<uint64_t>(sob0 + b), a.lower, a.upper);
        row[tid] = v;
        if (slc == 0) {
          a.contracts_out[b * 6 + tid] = v;
          if (a.cvnn_out) a.cvnn_out[b * 6 + tid] = static_cast<float>(v);
        }
      }
      lds_barrier();
      c = Contract{row[0], row[1], row[2], row[3], row[4], row[5]};
    } else {
      c = load_contract(a.contracts + b * 6);
    }
    const int T = T16 ? kRowBlock : a.T;
    const Stepper<float, LOG_EULER, HW> step(c, T);
    const float x0 = static_cast<float>(c.X0);
    float* base = static_cast<float*>(a.paths) + (STORE_ALL ? b * T * pitch : b * pitch);
    const int64_t p0 = static_cast<int64_t>(slc) * nch * kResChunk;  // first path of this slice
    // chunks >= kResLdsChunks: a shift register with static indices (a rolled loop indexing a
    // register array would put it in scratch memory); chunk ch ends in slot ch - nch + kResRegChunks
    float term[kResRegChunks][kPathsPerLane];
    double acc[1] = {0.0};
    double colsum[kPathsPerLane] = {0.0, 0.0, 0.0, 0.0};
    const PayoffPre<float> pre(c);                // all the payoff needs of c after the chunk loop
    const Payoff<float> pay_raw(a, pre, 1.0);  // ONTHEFLY: RAW, the terminal sum is not needed
    for (int ch = 0; ch < nch; ++ch) {
      float xt[kPathsPerLane];
      if constexpr (T16)  // the straight-line 16-row block (the benchmark shape)
        lane_paths<float, LOG_EULER, HW, false, false, true, true, STORE_ALL>(
            a, step, x0, static_cast<uint64_t>(ord0 + b), p0 + static_cast<int64_t>(ch) * kResChunk, kPathsPerLane,
            0, kRowBlock, base, acc, xt);
      else
        lane_rows<float, LOG_EULER, HW, STORE_ALL>(a, step, x0, static_cast<uint64_t>(ord0 + b),
                                            p0 + static_cast<int64_t>(ch) * kResChunk, base, T, pitch, acc[0], xt);
      if constexpr (ONTHEFLY) {
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) colsum[j] += static_cast<double>(pay_raw(xt[j]));
      } else if (ch < kResLdsChunks) {
        term_lds[ch * kResThreads + tid] = v4f{xt[0], xt[1], xt[2], xt[3]};
      } else {
#pragma unroll
        for (int i = 0; i + 1 < kResRegChunks; ++i)
#pragma unroll
          for (int j = 0; j < kPathsPerLane; ++j) term[i][j] = term[i + 1][j];
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) term[kResRegChunks - 1][j] = xt[j];
      }
    }
    const double w = wave_sum(acc[0]);
    if (lane == 0) wsum[wave] = w;
    lds_barrier();
    // LDS reads batched ahead of the in-order sums (the CF phase is a chain of LDS round trips)
    double tot = 0.0;
    {
      double wv[kResWaves];
#pragma unroll
      for (int k = 0; k < kResWaves; ++k) wv[k] = wsum[k];
#pragma unroll
      for (int k = 0; k < kResWaves; ++k) tot += wv[k];
    }
    // this round's [W + 1] slots: the W slice sums, then the group's next contract (dynamic tail)
    const int64_t xslot = (static_cast<int64_t>(grp) * 2 + (round & 1)) * (W + 1);
    if (W > 1) {
      // terminal-sum exchange: publish, arrive, wait for the W slices, add them in slice order.
      // Slice 0 also takes the group's next contract from the queue when the next round is in the
      // dynamic tail (its atomic's latency overlaps the drain below) and publishes it in slot W.
      if (tid == 0) {
        put_sc1(a.res_xsum + xslot + slc, tot);
        if (dyn && slc == 0 && b + groups >= n_static)
          put_sc1(reinterpret_cast<int64_t*>(a.res_xsum + xslot + W), n_static + atomicAdd(a.res_queue, 1u));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t* cnt = a.res_cnt + static_cast<int64_t>(grp) * 64;
        if (!(a.withhold && grp == 0 && slc == W - 1 && round == 0))
          __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t want = static_cast<uint32_t>(W) * (round + 1);
        // bounded poll; once any exchange of this launch has failed (its flag set) the others stop
        // waiting at once, so a failed launch still drains in about one poll budget
        uint32_t spins = 0;
        bool ok;
        while (!(ok = get_sc1(cnt) >= want) && get_sc1(a.launch_fail) == 0u && ++spins < a.spin_limit)
          __builtin_amdgcn_s_sleep(2);
        if (!ok) {
          __hip_atomic_fetch_or(a.status, SMC_SYNC_EXCHANGE_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.launch_fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const double t = ordered_sum_wt(a.res_xsum + xslot, 0, W, 1);  // slices in order
        row[6] = ok ? t : __builtin_nan("");
        if (dyn && b + groups >= n_static)
          reinterpret_cast<int64_t*>(row + 8)[0] =
              ok ? get_sc1(reinterpret_cast<const int64_t*>(a.res_xsum + xslot + W)) : a.B;
      }
      lds_barrier();
      tot = row[6];
    }
    const Payoff<float> pay(a, pre, tot);
    if constexpr (!ONTHEFLY) {
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) colsum[j] = 0.0;  // (the zeros before the loop are dead here)
      v4f v[kResLdsChunks];  // every slot read (unused ones too), so the 8 reads are in flight together
#pragma unroll
      for (int ch = 0; ch < kResLdsChunks; ++ch) v[ch] = term_lds[ch * kResThreads + tid];
#pragma unroll
      for (int ch = 0; ch < kResLdsChunks; ++ch) {
        if (ch < nch) {
#pragma unroll
          for (int j = 0; j < kPathsPerLane; ++j) colsum[j] += static_cast<double>(pay(v[ch][j]));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kResRegChunks && !ONTHEFLY; ++i) {
      if (i >= kResRegChunks - (nch - kResLdsChunks)) {  // chunk kResLdsChunks + i - (...), ascending
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) colsum[j] += static_cast<double>(pay(term[i][j]));
      }
    }
    lds_barrier();  // every lane has read its LDS slots: part may overwrite them
#pragma unroll
    for (int j = 0; j < kPathsPerLane; ++j) part[g * N + 4 * q + j] = colsum[j];
    lds_barrier();
    if (W == 1) {
      column_sums_tree(part, part, avg, N, M);
    } else {
      // column-sum exchange: the slice's G group sums per column, published by wave 0; the last
      // slice to arrive adds the W column sums in slice order and runs the FFT
      for (int n = tid; n < N; n += kResThreads) {
        const double t = group_sum(part, n, G, N);
        avg[n] = t;
      }
      lds_barrier();
      double* xcol = a.res_xcol + xslot * N;
      if (wave == 0) {
        for (int n = lane; n < N; n += 64) put_sc1(xcol + static_cast<int64_t>(slc) * N + n, avg[n]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          const uint32_t before = __hip_atomic_fetch_add(a.res_cnt + static_cast<int64_t>(grp) * 64 + 32, 1u,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          reinterpret_cast<int*>(row + 7)[0] = before == static_cast<uint32_t>(W) * (round + 1) - 1;
        }
      }
      lds_barrier();
      if (!reinterpret_cast<const int*>(row + 7)[0]) continue;  // uniform: another slice runs the FFT
      for (int n = tid; n < N; n += kResThreads) avg[n] = ordered_sum_wt(xcol, n, W, N) / static_cast<double>(M);
    }
    lds_barrier();
    fft_row<float, kResThreads, true>(avg, cs, sn, N, part, part + N, static_cast<float2*>(a.targets) + b * N);
    lds_barrier();  // part (= term_lds) / avg / wsum / row are reused by the next contract
  }
  if (a.done && tid == 0) {
    // every workgroup read the cursor (and made its last exchange) before it arrives here: the last
    // one advances the cursor and resets the exchange counters
    __threadfence();
    if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
      a.cursor[0] += a.advance;
      a.cursor[1] += a.advance;
      if (a.res_queue) *a.res_queue = 0u;
      if (W > 1) {
        for (int k = 0; k < groups; ++k) {
          a.res_cnt[static_cast<int64_t>(k) * 64] = 0u;
          a.res_cnt[static_cast<int64_t>(k) * 64 + 32] = 0u;
        }
        *a.launch_fail = 0u;
      }
      *a.done = 0u;
    }
  }
}

// ---- packed_kernel: several whole contracts per workgroup (small P) ------------------------------
// For 256 <= P <= 2048 (P | 4096) a contract's paths are P/4 lanes = P/256 whole waves, so a 1024-thread
// workgroup runs K = 4096 / P contracts side by side instead of one contract on a quarter of a
// 512-thread workgroup plus a CF re-read kernel (the reference's e2e shape, P = 512:
// tests/test_e2e/test_full_stack_cvnn_pricer.py:40-51).  Persistent: workgroup w runs the contract
// groups w, w + gridDim.x, ... (contracts K g ... K g + K - 1).  Per contract, resident_kernel's orders
// with one chunk of P / 4 lanes (oracle kernel mode, wg = P / 4): lane -> f32 4-path sum -> f64, wave
// butterfly, the contract's waves in order; item (q, g) = (lane mod N/4, 4 lane / N) is batch row m = g,
// column sums over m ascending from 0.0, the M-mean, then the K FFTs side by side (fft_rows).  The
// terminal values stay in registers; every barrier is LDS-only.  With a.sobol (smc_train_step) the
// workgroup draws its contracts' Sobol rows and the last workgroup advances the cursor.
constexpr int kPackMinP = 256, kPackMaxP = 2048;

size_t packed_lds_bytes(int64_t P, int N) {
  const int64_t K = kResChunk / P;
  const int64_t part = K * P > 2 * K * N ? K * P : 2 * K * N;  // payoff sums [K][M][N]; FFT re / im [K][N] each
  return static_cast<size_t>(part + K * N + 2 * N + kResWaves + 7 * K) * sizeof(double);
}

template <bool LOG_EULER, bool HW, bool STORE_ALL, bool T16>
__global__ __launch_bounds__(kResThreads) void packed_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.N, M = a.M;
  const int64_t P = a.P;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const int lpc = static_cast<int>(P / kPathsPerLane);  // lanes per contract (a multiple of 64)
  const int K = kResThreads / lpc;                      // contracts per group
  const int wpc = lpc / 64;                             // waves per contract
  const int k = tid / lpc, l = tid - k * lpc;           // this lane's contract slot, its lane in the contract
  const int cols = N / 4;
  const int q = l % cols, g = l / cols;                 // item (q, g): columns 4q .. 4q + 3 of batch row g
  const int64_t partn = K * P > 2 * K * N ? K * P : 2 * static_cast<int64_t>(K) * N;
  double* part = lds;                                   // [K][M][N]; FFT re / im [K][N] after the M-mean
  double* avg = part + partn;                           // [K][N]
  double* cs = avg + K * N;                             // [N]
  double* sn = cs + N;                                  // [N]
  double* wsum = sn + N;                                // [kResWaves]
  double* rows = wsum + kResWaves;                      // [K][7]: the drawn Sobol row, then the terminal sum
  for (int j = tid; j < N; j += kResThreads) math::twiddle(j, N, sn[j], cs[j]);
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int64_t sob0 = a.sobol ? a.cursor[0] + a.sobol_index0 : 0;
  const int64_t ngroups = (a.B + K - 1) / K;
  for (int64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int64_t b0 = grp * K;
    const int kv = a.B - b0 < K ? static_cast<int>(a.B - b0) : K;  // contracts of this group
    if (tid < 6 * kv) {  // the group's contract rows (sobol_sampler.py:222-246, or the caller's)
      const int kk = tid / 6, d = tid - 6 * kk;
      double v;
      if (a.sobol) {
        v = sobol_coord(a.sobol, a.sobol_dim, d, static_cast<uint64_t>(sob0 + b0 + kk), a.lower, a.upper);
        a.contracts_out[(b0 + kk) * 6 + d] = v;
        if (a.cvnn_out) a.cvnn_out[(b0 + kk) * 6 + d] = static_cast<float>(v);
      } else {
        v = a.contracts[(b0 + kk) * 6 + d];
      }
      rows[kk * 7 + d] = v;
    }
    lds_barrier();
    const bool active = k < kv;
    const double* r = rows + (active ? k : 0) * 7;
    const Contract c{r[0], r[1], r[2], r[3], r[4], r[5]};
    const int T = T16 ? kRowBlock : a.T;
    float xt[kPathsPerLane] = {0.0f, 0.0f, 0.0f, 0.0f};
    double acc[1] = {0.0};
    if (active) {
      const Stepper<float, LOG_EULER, HW> step(c, T);
      const float x0 = static_cast<float>(c.X0);
      const int64_t b = b0 + k;
      float* base = static_cast<float*>(a.paths) + (STORE_ALL ? b * T * pitch : b * pitch);
      if constexpr (T16)
        lane_paths<float, LOG_EULER, HW, false, false, true, true, STORE_ALL>(
            a, step, x0, static_cast<uint64_t>(ord0 + b), 0, kPathsPerLane, 0, kRowBlock, base, acc, xt, l);
      else
        lane_rows<float, LOG_EULER, HW, STORE_ALL>(a, step, x0, static_cast<uint64_t>(ord0 + b), 0, base, T, pitch,
                                                   acc[0], xt, l);
    }
    const double w = wave_sum(acc[0]);  // a wave holds lanes of one contract only
    if (lane == 0) wsum[wave] = w;
    lds_barrier();
    if (tid < K) {  // the contract's waves in order
      double tot = 0.0;
      for (int v = 0; v < wpc; ++v) tot += wsum[tid * wpc + v];
      rows[tid * 7 + 6] = tot;
    }
    lds_barrier();
    if (active) {
      const Payoff<float> pay(a, c, r[6]);
      double* pk = part + static_cast<int64_t>(k) * P;
#pragma unroll
      for (int j = 0; j < kPathsPerLane; ++j) pk[g * N + 4 * q + j] = 0.0 + static_cast<double>(pay(xt[j]));
    }
    lds_barrier();
    for (int e = tid; e < kv * N; e += kResThreads) {  // column sums over the M batch rows in order
      const int kk = e / N, n = e - kk * N;
      avg[e] = group_sum(part + static_cast<int64_t>(kk) * P, n, M, N) / static_cast<double>(M);
    }
    lds_barrier();
    fft_rows<float, kResThreads, true>(avg, cs, sn, N, K, kv, part, part + static_cast<int64_t>(K) * N,
                                       static_cast<float2*>(a.targets) + b0 * N);
    lds_barrier();  // part / avg / rows are rewritten by the next group
  }
  if (a.done && tid == 0) {
    // every workgroup read the cursor before it arrives here: the last one advances it
    __threadfence();
    if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
      a.cursor[0] += a.advance;
      a.cursor[1] += a.advance;
      *a.done = 0u;
    }
  }
}

// ---- wave_kernel: one wave per contract (RAW normalisation, T <= 2) -------------------------------
// RAW targets need no terminal sum, so a contract's payoffs can be added up as its paths finish, and a
// whole contract fits one wave: its 64 lanes walk the contract in 1024-path chunks, each lane taking 16
// consecutive paths = one stream span (smc_rng.h: at T <= 2 one Philox-10 seed serves 4 groups of 4
// paths, drawn in group order), adding each path's payoff to its 16 column sums; after the last chunk the
// wave alone takes the M-mean and the FFT from its own LDS -- no workgroup barrier per contract.  At the
// reference's lock-step shape (T = 1, N = 16, M = 4096, RAW: tests/test_gbm_trainer.py:122-142) the
// 1024-thread resident kernel's per-contract barriers and serial CF phase cost as much as the paths
// themselves (profiles/r04/ab_lockstep_decomposition.txt), and the per-group Philox seed was the largest
// part of the paths (T = 1: 4 draws per seed).  Shapes: N a multiple of 16 dividing 1024, so a lane's 16
// paths are 16 adjacent columns of one batch row.  Orders (oracle kernel mode, wg = 256: G = 1024 / N
// batch-row groups): lane l adds its columns' rows m = 16 l / N, + G, ... ascending from 0.0 (chunk
// order), the wave adds the G partials of a column in order from 0.0, the M-mean, then the FFT of
// fft_row.  Persistent: wave w of the grid runs contracts w, w + (all waves), ...; with a.sobol
// (smc_train_step) each wave draws its contract's Sobol row and the last workgroup advances the cursor.
constexpr int kWaveThreads = 256;
constexpr int kWaveLanePaths = PathStream::kSpanGroups * kPathsPerLane;  // 16 paths per lane and chunk
constexpr int kWaveChunk = 64 * kWaveLanePaths;                           // 1024 paths per chunk
constexpr int kWaveMaxT = 2;

size_t wave_lds_bytes(int N) {
  const size_t per_wave = kWaveChunk + 3 * static_cast<size_t>(N) + 8;  // part [G][N], avg, re, im, row
  return (static_cast<size_t>(kWaveThreads / 64) * per_wave + 2 * static_cast<size_t>(N)) * sizeof(double);
}

// 4 waves per SIMD (<= 128 VGPRs): the lock-step batch of 4096 contracts is then exactly one contract
// per resident wave (256 CUs x 16 waves) instead of 1.33 rounds at 3 waves per SIMD.
template <bool LOG_EULER, bool HW, bool STORE_ALL, int TT>  // TT = T (1 or 2): no runtime step loop
__global__ __launch_bounds__(kWaveThreads) __attribute__((amdgpu_waves_per_eu(4))) void wave_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int N = a.N, M = a.M;
  constexpr int T = TT;
  const int64_t P = a.P;
  const int64_t pitch = a.pitch ? a.pitch : P;
  const int G = kWaveChunk / N;  // batch rows per chunk
  const int g = kWaveLanePaths * lane / N, n0 = kWaveLanePaths * lane % N;  // the lane's row and columns
  const int per_wave = kWaveChunk + 3 * N + 8;
  double* part = lds + wave * per_wave;  // [G][N]
  double* avg = part + kWaveChunk;       // [N]
  double* re = avg + N;                  // [N]
  double* im = re + N;                   // [N]
  double* row = im + N;                  // [6] the drawn Sobol row
  double* cs = lds + (kWaveThreads / 64) * per_wave;
  double* sn = cs + N;
  for (int j = threadIdx.x; j < N; j += kWaveThreads) math::twiddle(j, N, sn[j], cs[j]);
  __syncthreads();
  const int64_t ord0 = (a.ordinal_dev ? *a.ordinal_dev : 0) + a.ordinal0;
  const int64_t sob0 = a.sobol ? a.cursor[0] + a.sobol_index0 : 0;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (kWaveThreads / 64);
  for (int64_t b = static_cast<int64_t>(blockIdx.x) * (kWaveThreads / 64) + wave; b < a.B; b += nw) {
    Contract c;
    if (a.sobol) {  // sobol_sampler.py:222-246, one lane per dimension
      if (lane < 6) {
        const double v = sobol_coord(a.sobol, a.sobol_dim, lane, static_cast<uint64_t>(sob0 + b), a.lower, a.upper);
        row[lane] = v;
        a.contracts_out[b * 6 + lane] = v;
        if (a.cvnn_out) a.cvnn_out[b * 6 + lane] = static_cast<float>(v);
      }
      wave_lds_sync();
      c = Contract{row[0], row[1], row[2], row[3], row[4], row[5]};
    } else {
      c = load_contract(a.contracts + b * 6);
    }
    const Stepper<float, LOG_EULER, HW> step(c, T);
    const float x0 = static_cast<float>(c.X0);
    const Payoff<float> pay(a, PayoffPre<float>(c), 1.0);  // RAW: scale 1
    float* base = static_cast<float*>(a.paths) + (STORE_ALL ? b * T * pitch : b * pitch);
    double colsum[kWaveLanePaths];
#pragma unroll
    for (int k = 0; k < kWaveLanePaths; ++k) colsum[k] = 0.0;
    double acc = 0.0;  // (the terminal sum: not needed for RAW targets)
    float* stage = reinterpret_cast<float*>(part);  // [rows][1024] f32: part is free until the chunks end
    constexpr int kRows = STORE_ALL ? TT : 1;
    for (int64_t chunk = 0; chunk < P; chunk += kWaveChunk) {
      // the lane's span: stream (chunk + 16 lane) / 16, its 4 groups in order
      PathStream s(a.seed, static_cast<uint64_t>(ord0 + b),
                   static_cast<uint64_t>((chunk + kWaveLanePaths * lane) / kWaveLanePaths));
#pragma unroll
      for (int j = 0; j < PathStream::kSpanGroups; ++j) {
        float xt[kPathsPerLane];
        lane_rows_s<float, LOG_EULER, HW, STORE_ALL>(s, step, x0, chunk, base, T, pitch, acc, xt,
                                                     PathStream::kSpanGroups * lane + j,
                                                     stage, kWaveChunk);
#pragma unroll
        for (int i = 0; i < kPathsPerLane; ++i) colsum[kPathsPerLane * j + i] += static_cast<double>(pay(xt[i]));
      }
      {
        // the chunk's rows from LDS: each store instruction 64 lanes x 16 B contiguous (a lane's own 64 B
        // would make every instruction a quarter-dense 4 KiB stripe)
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
          char* rowp = reinterpret_cast<char*>(base + (STORE_ALL ? r * pitch : 0) + chunk);
#pragma unroll
          for (int k = 0; k < kWaveChunk / 256; ++k) {
            const float4 v = *reinterpret_cast<const float4*>(stage + r * kWaveChunk + 256 * k + kPathsPerLane * lane);
            store_row(rowp + 1024 * k, static_cast<uint32_t>(16 * lane), v);
          }
        }
        wave_lds_sync();  // the stage is rewritten by the next chunk
      }
    }
#pragma unroll
    for (int k = 0; k < kWaveLanePaths; ++k) part[g * N + n0 + k] = colsum[k];
    wave_lds_sync();
    for (int n = lane; n < N; n += 64) {
      double t = 0.0;
      for (int gg = 0; gg < G; ++gg) t += part[gg * N + n];
      avg[n] = t / static_cast<double>(M);
    }
    wave_lds_sync();
    fft_rows<float, 64, true, true>(avg, cs, sn, N, 1, 1, re, im, static_cast<float2*>(a.targets) + b * N);
    wave_lds_sync();  // part / avg / re / im are rewritten by the wave's next contract
  }
  __syncthreads();  // every wave of the workgroup is done with its contracts
  if (a.done && threadIdx.x == 0) {
    // every workgroup read the cursor before it arrives here: the last one advances it
    __threadfence();
    if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
      a.cursor[0] += a.advance;
      a.cursor[1] += a.advance;
      *a.done = 0u;
    }
  }
}

bool wave_ok(const EngineArgs& a, bool f32) {
  // any P (res_slices is ignored: one wave walks the whole contract, so smc_train_step takes it where the
  // sliced resident kernel would otherwise exchange between workgroups)
  return f32 && a.simulate && a.targets && !a.normalize && !a.all_rows && a.slices <= 1 &&
         a.T >= 1 && a.T <= kWaveMaxT && a.P % kWaveChunk == 0 && a.N >= kWaveLanePaths &&
         a.N % kWaveLanePaths == 0 && kWaveChunk % a.N == 0 && (a.pitch == 0 || (a.pitch % 4 == 0 && a.pitch >= a.P));
}

bool packed_ok(const EngineArgs& a, bool f32) {
  return f32 && a.simulate && a.targets && !a.all_rows && a.slices <= 1 && a.res_slices <= 1 && a.T >= 1 &&
         a.T <= kResMaxT && a.P >= kPackMinP && a.P <= kPackMaxP && kResChunk % a.P == 0 && a.N >= 4 &&
         a.N % 4 == 0 && a.P % a.N == 0 && (a.pitch == 0 || (a.pitch % 4 == 0 && a.pitch >= a.P));
}

bool resident_ok(const EngineArgs& a, bool f32) {
  const int64_t W = a.res_slices > 1 ? a.res_slices : 1;
  return f32 && a.simulate && a.targets && !a.all_rows && a.slices <= 1 && a.T >= 1 && a.T <= kResMaxT &&
         W <= kResMaxSlices && a.P % (W * kResChunk) == 0 && a.P / (W * kResChunk) <= kResMaxChunks &&
         a.N >= 4 && a.N <= 1024 && kResChunk % a.N == 0 && (a.pitch == 0 || (a.pitch % 4 == 0 && a.pitch >= a.P)) &&
         (W == 1 || (a.res_cnt && a.res_xsum && a.res_xcol && a.done));
}

// Workgroups per contract of the resident kernel in smc_train_step: the fewest (a power of two
// <= kResMaxSlices) whose slices hold <= 65,536 paths each.
int32_t resident_slices(int64_t P) {
  int32_t W = 1;
  while (W < kResMaxSlices && P > static_cast<int64_t>(W) * kResMaxChunks * kResChunk) W *= 2;
  return W;
}

// smc_train_step sync area: [0, 128) the done counter (+0), the sticky status word
// (+SMC_SYNC_STATUS_OFFSET), the launch's failure flag (+SMC_SYNC_LAUNCH_FAIL_OFFSET) and the contract
// queue (+64); then per
// group a 256-B record of two 128-B counter lines; then the slice terminal sums + next contract
// [groups][2][W + 1] and column sums [groups][2][W][N].
// groups <= 2 #CUs / W (the resident kernel fits one workgroup per CU; twice that for margin).
struct ResSyncLayout {
  int64_t groups, xsum_off, xcol_off, bytes;
};
constexpr int64_t kStepSyncBytes = 128;  // done counter (+0), status (+32), launch failure flag (+48), queue (+64)
ResSyncLayout res_sync_layout(int32_t W, int32_t N, int cus) {
  ResSyncLayout l{};
  if (W <= 1) {
    l.bytes = kStepSyncBytes;
    return l;
  }
  l.groups = (2 * static_cast<int64_t>(cus) + W - 1) / W;
  l.xsum_off = 128 + 256 * l.groups;
  l.xcol_off = (l.xsum_off + l.groups * 2 * (W + 1) * 8 + 255) / 256 * 256;
  l.bytes = l.xcol_off + l.groups * 2 * W * static_cast<int64_t>(N) * 8;
  return l;
}

bool split_ok(const EngineArgs& a, bool f32) {
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  return f32 && a.simulate && a.targets && !a.all_rows && a.slices <= 1 && pitch >= a.P + (a.P & 1) + 2;
}

// rows_kernel + cf_kernel: whole 2048-path chunks, padding for the f64 terminal sum (f32: 2 floats
// after an 8-B-aligned column P; f64: one element)
bool rows_ok(const EngineArgs& a, bool f32) {
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  return a.simulate && a.targets && !a.all_rows && a.slices <= 1 && a.T >= 1 && a.P % kChunk == 0 &&
         pitch >= a.P + (f32 ? (a.P & 1) + 2 : 1) && (a.store == SMC_STORE_ALL || a.store == SMC_STORE_TERMINAL);
}

// rows_ref_kernel + cf_kernel (SMC_MATH_REF): any P, the f32 terminal-sum padding
bool ref_ok(const EngineArgs& a) {
  const int64_t pitch = a.pitch ? a.pitch : a.P;
  return a.simulate && a.targets && !a.all_rows && a.slices <= 1 && a.T >= 1 && pitch >= a.P + (a.P & 1) + 2 &&
         (a.store == SMC_STORE_ALL || a.store == SMC_STORE_TERMINAL);
}

// Sliced contracts on persistent workgroups.  Contract b belongs to queue b mod 8; a workgroup
// takes items (slice k of a contract) from the queue of the XCD it runs on (s_getreg XCC_ID), so
// the slices of a contract run side by side on one XCD, finish within a few tens of microseconds
// of each other, and the last one's CF re-read finds the terminal row still on chip.  Placement
// is for speed only: the hand-off protocol is cross-XCD safe, and the last workgroup to leave
// runs whatever is left in any queue (an XCD without workgroups) before resetting the counters.
// queues[0..7]: next item per queue, queues[8]: workgroups done; all zero between launches.
template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
__global__ __launch_bounds__(kThreads) void queue_kernel(EngineArgs a) {
  extern __shared__ double lds[];
  __shared__ int flag;
  __shared__ int64_t next_item;
  if constexpr (sizeof(Real) == 8) math::f64_tables_load();
  const int W = a.slices;
  uint32_t* queues = a.queues;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  auto queue_items = [&](int x) -> int64_t { return x < a.B ? ((a.B - 1 - x) / 8 + 1) * W : 0; };
  auto drain_queue = [&](int x) {
    const int64_t n = queue_items(x);
    for (;;) {
      if (threadIdx.x == 0)
        next_item = __hip_atomic_fetch_add(queues + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int64_t j = next_item;
      __syncthreads();
      if (j >= n) break;
      run_slice<Real, LOG_EULER, HW, ALLROWS>(a, x + 8 * (j / W), static_cast<int>(j % W), lds, &flag);
    }
  };
  drain_queue(static_cast<int>(xcc & 7));
  if (threadIdx.x == 0)
    flag = __hip_atomic_fetch_add(queues + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (flag) {  // every other workgroup has left: finish orphaned queues, reset for the next launch
    for (int x = 0; x < 8; ++x) drain_queue(x);
    if (threadIdx.x < 9) __hip_atomic_store(queues + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  if constexpr (sizeof(Real) == 8) math::f64_tables_load();  // before any thread leaves
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // path group
  if (g * kPathsPerLane >= cols) return;
  PathStream s(seed, ordinal, static_cast<uint64_t>(g), rows);
  const Real zs = sizeof(Real) == 4 ? static_cast<Real>(PathStream::kNormalScale<HW>) : Real(1);
  Real z0[kPathsPerLane], z1[kPathsPerLane];
  for (int t = 0; t < rows; ++t) {
    if ((t & 1) == 0) {
      if (t + 1 < rows) {
#pragma unroll
        for (int j = 0; j < kPathsPerLane; ++j) s.template normal_pair<HW>(z0[j], z1[j]);
      } else {
        s.template normal_tail<HW>(z0);  // the last row of an odd count: two pairs for the 4 paths
      }
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
    const size_t cfw = static_cast<size_t>(cf_part_doubles(N)) + 3 * static_cast<size_t>(N);
    if (cfw > work) work = cfw;
  }
  const size_t bytes = (doubles + work) * sizeof(double);
  return bytes;
}

// Resident workgroups of a persistent kernel on the current device (occupancy x CUs, cached
// per (device, kernel)); grid = min(work items, that).
// CUs a stream may use: the popcount of its CU mask (hipExtStreamCreateWithCUMask), else the device's

// Persistent grid: the kernel's resident slots on the CUs `stream` may use (a CU-masked stream's
// launch is sized to its mask, so every workgroup is resident at once), at most `items`.
int32_t resident_grid(const void* kernel, int threads, size_t lds, int64_t items, unsigned* grid,
                      hipStream_t stream = nullptr) {
  struct Entry {
    int dev;
    const void* kernel;
    size_t lds;
    unsigned slots;
  };
  static Entry cache[32];
  static int used = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(SMC_ERR_HIP, "engine: hipGetDevice failed");
  unsigned slots = 0;
  for (int i = 0; i < used; ++i)
    if (cache[i].dev == dev && cache[i].kernel == kernel && cache[i].lds == lds) slots = cache[i].slots;
  if (slots == 0) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "engine: occupancy query failed");
    }
    slots = static_cast<unsigned>((per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1));
    if (used < 32) cache[used++] = Entry{dev, kernel, lds, slots};
  }
  if (stream) {  // per CU = slots / all CUs; the stream's share
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
      const int n = stream_cus(stream, cus);
      if (n < cus) slots = slots / static_cast<unsigned>(cus) * static_cast<unsigned>(n);
    } else {
      (void)hipGetLastError();
    }
  }
  *grid = static_cast<unsigned>(items < slots ? items : slots);
  return SMC_OK;
}

template <typename Real, bool LOG_EULER, bool HW, bool ALLROWS>
int32_t launch_engine_k(const EngineArgs& a, size_t lds, hipStream_t stream) {
  if (a.slices > 1) {
    auto kernel = queue_kernel<Real, LOG_EULER, HW, ALLROWS>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "queue_kernel: cannot raise the dynamic LDS limit");
    }
    unsigned grid = 0;
    if (int32_t st = resident_grid(reinterpret_cast<const void*>(kernel), kThreads, lds, a.B * a.slices, &grid))
      return st;
    launch(kernel, dim3(grid), dim3(kThreads), lds, stream, a);
    return check_launch("queue_kernel");
  }
  auto kernel = contract_kernel<Real, LOG_EULER, HW, ALLROWS>;
  if (lds > 64 * 1024) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "contract_kernel: cannot raise the dynamic LDS limit");
    }
  }
  launch(kernel, dim3(static_cast<unsigned>(a.B)), dim3(kThreads), lds, stream, a);
  return check_launch("contract_kernel");
}

// Workgroups per contract: slices of kSliceChunks chunks when a workspace is given.
int32_t slices_for(int64_t P, bool sliced) {
  if (!sliced) return 1;
  const int64_t chunks = (P + kChunk - 1) / kChunk;
  return static_cast<int32_t>((chunks + kSliceChunks - 1) / kSliceChunks);
}

size_t workspace_bytes(int64_t B, int32_t T, int64_t P, bool all_rows) {
  const int64_t W = slices_for(P, true);
  if (W <= 1) return 0;
  return static_cast<size_t>(B) * W * (all_rows ? T : 1) * sizeof(double) + static_cast<size_t>(B + 16) * sizeof(uint32_t);
}

// Resident paths_kernel workgroups per CU (its ~42 VGPRs allow 4 x 512 threads)
constexpr int kPathsWgsPerCu = 4;

template <bool LOG_EULER, bool HW, bool STRAIGHT, bool STORE_ALL>
int32_t launch_split_k(const EngineArgs& a, hipStream_t stream) {
  const size_t lds1 = lds_bytes(a.T, a.N, false), lds2 = lds_bytes(a.T, a.N, true);
  auto k1 = paths_kernel<LOG_EULER, HW, STRAIGHT, STORE_ALL>;
  auto k2 = cf_kernel<float>;
  if ((lds1 > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(k1),
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                static_cast<int>(lds1)) != hipSuccess) ||
      (lds2 > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(k2),
                                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                                static_cast<int>(lds2)) != hipSuccess)) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "paths_kernel / cf_kernel: cannot raise the dynamic LDS limit");
  }
  unsigned grid1 = static_cast<unsigned>(a.B);
  if (STRAIGHT) {  // persistent: kPathsWgsPerCu resident workgroups per CU
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "paths_kernel: device query failed");
    }
    const int64_t slots = static_cast<int64_t>(kPathsWgsPerCu) * cus;
    if (slots < a.B) grid1 = static_cast<unsigned>(slots);
  }
  launch(k1, dim3(grid1), dim3(kThreads), lds1, stream, a);
  if (int32_t st = check_launch("paths_kernel")) return st;
  launch(k2, dim3(static_cast<unsigned>(a.B)), dim3(kThreads), lds2, stream, a);
  return check_launch("cf_kernel");
}

template <typename Real, bool LOG_EULER, bool HW, bool STORE_ALL>
int32_t launch_rows_k(const EngineArgs& a, hipStream_t stream) {
  const size_t lds1 = 2 * kWaves * sizeof(double), lds2 = lds_bytes(a.T, a.N, true);
  auto k1 = rows_kernel<Real, LOG_EULER, HW, STORE_ALL>;
  auto k2 = cf_kernel<Real>;
  if (lds2 > kMaxLds) return fail(SMC_ERR_INVALID_SHAPE, "engine: network_size exceeds the LDS budget");
  if (lds2 > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(k2),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               static_cast<int>(lds2)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "cf_kernel: cannot raise the dynamic LDS limit");
  }
  unsigned grid1 = 0;
  if (int32_t st = resident_grid(reinterpret_cast<const void*>(k1), kThreads, lds1, a.B, &grid1)) return st;
  launch(k1, dim3(grid1), dim3(kThreads), lds1, stream, a);
  if (int32_t st = check_launch("rows_kernel")) return st;
  launch(k2, dim3(static_cast<unsigned>(a.B)), dim3(kThreads), lds2, stream, a);
  return check_launch("cf_kernel");
}

template <bool LOG_EULER, bool STORE_ALL, bool HWN>
int32_t launch_rows_ref_k(const EngineArgs& a, hipStream_t stream) {
  const size_t lds1 = 2 * kWaves * sizeof(double), lds2 = lds_bytes(a.T, a.N, true);
  auto k1 = rows_ref_kernel<LOG_EULER, STORE_ALL, HWN>;
  auto k2 = cf_kernel<float>;
  if (lds2 > kMaxLds) return fail(SMC_ERR_INVALID_SHAPE, "engine: network_size exceeds the LDS budget");
  if (lds2 > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(k2),
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               static_cast<int>(lds2)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "cf_kernel: cannot raise the dynamic LDS limit");
  }
  unsigned grid1 = 0;
  if (int32_t st = resident_grid(reinterpret_cast<const void*>(k1), kThreads, lds1, a.B, &grid1)) return st;
  launch(k1, dim3(grid1), dim3(kThreads), lds1, stream, a);
  if (int32_t st = check_launch("rows_ref_kernel")) return st;
  launch(k2, dim3(static_cast<unsigned>(a.B)), dim3(kThreads), lds2, stream, a);
  return check_launch("cf_kernel");
}

template <bool LOG_EULER, bool HW, bool STORE_ALL>
int32_t launch_resident_k(const EngineArgs& a, hipStream_t stream) {
  const int W = a.res_slices > 1 ? a.res_slices : 1;
  auto kernel = a.T == kRowBlock                 ? resident_kernel<LOG_EULER, HW, STORE_ALL, true>
                : (!a.normalize && W == 1) ? resident_kernel<LOG_EULER, HW, STORE_ALL, false, true>
                                           : resident_kernel<LOG_EULER, HW, STORE_ALL, false>;
  const size_t lds = resident_lds_bytes(a.N);
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "resident_kernel: cannot raise the dynamic LDS limit");
  }
  unsigned grid = 0;
  if (int32_t st = resident_grid(reinterpret_cast<const void*>(kernel), kResThreads, lds, a.B * W, &grid, stream))
    return st;
  if (W > 1) {
    // whole groups of W co-resident workgroups (every slice of a group waits for the others),
    // in multiples of 8 W where possible so a group's slices share an XCD
    unsigned groups = grid / W;
    if (groups > static_cast<unsigned>(a.res_groups)) groups = static_cast<unsigned>(a.res_groups);
    if (groups >= 8) groups -= groups % 8;
    if (groups == 0) return fail(SMC_ERR_INVALID_SHAPE, "resident_kernel: fewer resident slots than slices");
    grid = groups * W;
  }
  launch(kernel, dim3(grid), dim3(kResThreads), lds, stream, a);
  return check_launch("resident_kernel");
}

template <bool LOG_EULER, bool HW, bool STORE_ALL>
int32_t launch_wave_k(const EngineArgs& a, hipStream_t stream) {
  auto kernel = a.T == 1 ? wave_kernel<LOG_EULER, HW, STORE_ALL, 1> : wave_kernel<LOG_EULER, HW, STORE_ALL, 2>;
  const size_t lds = wave_lds_bytes(a.N);
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "wave_kernel: cannot raise the dynamic LDS limit");
  }
  unsigned grid = 0;
  const int64_t wpg = kWaveThreads / 64;
  if (int32_t st = resident_grid(reinterpret_cast<const void*>(kernel), kWaveThreads, lds, (a.B + wpg - 1) / wpg, &grid,
                                 stream))
    return st;
  launch(kernel, dim3(grid), dim3(kWaveThreads), lds, stream, a);
  return check_launch("wave_kernel");
}

template <bool LOG_EULER, bool HW, bool STORE_ALL>
int32_t launch_packed_k(const EngineArgs& a, hipStream_t stream) {
  auto kernel = a.T == kRowBlock ? packed_kernel<LOG_EULER, HW, STORE_ALL, true>
                                 : packed_kernel<LOG_EULER, HW, STORE_ALL, false>;
  const size_t lds = packed_lds_bytes(a.P, a.N);
  if (lds > kMaxLds) return fail(SMC_ERR_INVALID_SHAPE, "packed_kernel: network_size exceeds the LDS budget");
  if (lds > 64 * 1024 && hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
    return fail(SMC_ERR_HIP, "packed_kernel: cannot raise the dynamic LDS limit");
  }
  const int64_t K = kResChunk / a.P;
  unsigned grid = 0;
  if (int32_t st = resident_grid(reinterpret_cast<const void*>(kernel), kResThreads, lds, (a.B + K - 1) / K, &grid,
                                 stream))
    return st;
  launch(kernel, dim3(grid), dim3(kResThreads), lds, stream, a);
  return check_launch("packed_kernel");
}


template <typename Real>
int32_t launch_engine(EngineArgs a, hipStream_t stream) {
  if (a.B == 0) return SMC_OK;
  if ((a.scheme & SMC_MATH_REF) != 0) {
    if (sizeof(Real) != 4) return fail(SMC_ERR_INVALID_ARGUMENT, "engine: SMC_MATH_REF is an f32 mode");
    if (!ref_ok(a))
      return fail(SMC_ERR_INVALID_SHAPE, "engine: SMC_MATH_REF needs targets, whole contracts per workgroup and "
                                         "a padded pitch (smc_path_pitch)");
    const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
    const bool sa = a.store == SMC_STORE_ALL;
    if ((a.scheme & SMC_MATH_HW) != 0) {  // hardware-transcendental normals
      if (log_euler)
        return sa ? launch_rows_ref_k<true, true, true>(a, stream) : launch_rows_ref_k<true, false, true>(a, stream);
      return sa ? launch_rows_ref_k<false, true, true>(a, stream) : launch_rows_ref_k<false, false, true>(a, stream);
    }
    if (log_euler)
      return sa ? launch_rows_ref_k<true, true, false>(a, stream) : launch_rows_ref_k<true, false, false>(a, stream);
    return sa ? launch_rows_ref_k<false, true, false>(a, stream) : launch_rows_ref_k<false, false, false>(a, stream);
  }
  if constexpr (sizeof(Real) == 4) {
    if (wave_ok(a, true)) {  // RAW, T <= 2: one wave per contract
      const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
      const bool hw = (a.scheme & SMC_MATH_HW) != 0;
      const bool sa = a.store == SMC_STORE_ALL;
#define SMC_WAVE(LE, HWM, SA) \
  if (log_euler == LE && hw == HWM && sa == SA) return launch_wave_k<LE, HWM, SA>(a, stream);
      SMC_WAVE(true, true, true)
      SMC_WAVE(true, true, false)
      SMC_WAVE(true, false, true)
      SMC_WAVE(true, false, false)
      SMC_WAVE(false, true, true)
      SMC_WAVE(false, true, false)
      SMC_WAVE(false, false, true)
      SMC_WAVE(false, false, false)
#undef SMC_WAVE
    }
    if (resident_ok(a, true)) {
      const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
      const bool hw = (a.scheme & SMC_MATH_HW) != 0;
      const bool sa = a.store == SMC_STORE_ALL;
#define SMC_RES(LE, HWM, SA) \
  if (log_euler == LE && hw == HWM && sa == SA) return launch_resident_k<LE, HWM, SA>(a, stream);
      SMC_RES(true, true, true)
      SMC_RES(true, true, false)
      SMC_RES(true, false, true)
      SMC_RES(true, false, false)
      SMC_RES(false, true, true)
      SMC_RES(false, true, false)
      SMC_RES(false, false, true)
      SMC_RES(false, false, false)
#undef SMC_RES
    }
    if (packed_ok(a, true)) {  // small P: several contracts per workgroup
      const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
      const bool hw = (a.scheme & SMC_MATH_HW) != 0;
      const bool sa = a.store == SMC_STORE_ALL;
#define SMC_PACK(LE, HWM, SA) \
  if (log_euler == LE && hw == HWM && sa == SA) return launch_packed_k<LE, HWM, SA>(a, stream);
      SMC_PACK(true, true, true)
      SMC_PACK(true, true, false)
      SMC_PACK(true, false, true)
      SMC_PACK(true, false, false)
      SMC_PACK(false, true, true)
      SMC_PACK(false, true, false)
      SMC_PACK(false, false, true)
      SMC_PACK(false, false, false)
#undef SMC_PACK
    }
    // the split pair: the straight-line T = 16 paths_kernel, or (ragged chunks) simulate_contract;
    // other whole-chunk shapes take rows_kernel below
    const bool straight_split = a.T == kRowBlock && a.P % kChunk == 0;
    if (split_ok(a, true) && (straight_split || !rows_ok(a, true))) {
      const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
      const bool hw = (a.scheme & SMC_MATH_HW) != 0;
      const bool straight = straight_split;
      const bool sa = a.store == SMC_STORE_ALL;
#define SMC_SPLIT(LE, HWM, ST, SA) \
  if (log_euler == LE && hw == HWM && straight == ST && (!ST || sa == SA)) return launch_split_k<LE, HWM, ST, SA>(a, stream);
      SMC_SPLIT(true, true, true, true)
      SMC_SPLIT(true, true, true, false)
      SMC_SPLIT(true, false, true, true)
      SMC_SPLIT(true, false, true, false)
      SMC_SPLIT(false, true, true, true)
      SMC_SPLIT(false, true, true, false)
      SMC_SPLIT(false, false, true, true)
      SMC_SPLIT(false, false, true, false)
      SMC_SPLIT(true, true, false, true)
      SMC_SPLIT(true, false, false, true)
      SMC_SPLIT(false, true, false, true)
      SMC_SPLIT(false, false, false, true)
#undef SMC_SPLIT
    }
  }
  if (rows_ok(a, sizeof(Real) == 4)) {
    const bool log_euler = (a.scheme & 0xff) == SMC_SCHEME_LOG_EULER;
    const bool hw = (a.scheme & SMC_MATH_HW) != 0 && sizeof(Real) == 4;
    const bool sa = a.store == SMC_STORE_ALL;
#define SMC_ROWS(LE, HWM, SA) \
  if (log_euler == LE && hw == HWM && sa == SA) return launch_rows_k<Real, LE, HWM, SA>(a, stream);
    SMC_ROWS(true, false, true)
    SMC_ROWS(true, false, false)
    SMC_ROWS(false, false, true)
    SMC_ROWS(false, false, false)
    if constexpr (sizeof(Real) == 4) {
      SMC_ROWS(true, true, true)
      SMC_ROWS(true, true, false)
      SMC_ROWS(false, true, true)
      SMC_ROWS(false, true, false)
    }
#undef SMC_ROWS
  }
  if (a.slices < 1 || !a.simulate) a.slices = 1;
  if (a.slices > 1 && (!a.partials || !a.arrivals || !a.queues))
    return fail(SMC_ERR_INVALID_ARGUMENT, "engine: sliced contracts need a workspace");
  if (static_cast<int64_t>(a.B) * a.slices > 0x7fffffffLL)
    return fail(SMC_ERR_INVALID_SHAPE, "engine: more than 2^31-1 workgroups in one launch");
  const bool cf = a.targets != nullptr;
  const size_t lds = lds_bytes(a.T, a.N, cf);
  // f64 kernels also hold the static table image of the path math (math::F64Tables)
  if (lds + (sizeof(Real) == 8 ? sizeof(math::F64Tables) : 0) > kMaxLds)
    return fail(SMC_ERR_INVALID_SHAPE, "engine: timesteps/network_size exceed the LDS budget");
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

__global__ void advance_cursor_kernel(int64_t* cursor, int64_t advance) {
  if (threadIdx.x == 0) {
    cursor[0] += advance;
    cursor[1] += advance;
  }
}

int32_t dispatch_engine(const EngineArgs& a, int32_t dtype, hipStream_t stream) {
  if (dtype == SMC_DTYPE_F32) return launch_engine<float>(a, stream);
  if (dtype == SMC_DTYPE_F64) return launch_engine<double>(a, stream);
  return fail(SMC_ERR_INVALID_ARGUMENT, "engine: dtype must be SMC_DTYPE_F32 or SMC_DTYPE_F64");
}

bool valid_scheme(int32_t scheme) {  // SMC_MATH_REF | SMC_MATH_HW: reference arithmetic on hardware normals
  const int32_t base = scheme & 0xff, flags = scheme & ~0xff;
  return (base == SMC_SCHEME_LOG_EULER || base == SMC_SCHEME_SIMPLE_EULER) && (flags & ~(SMC_MATH_HW | SMC_MATH_REF)) == 0;
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
  if (scheme & SMC_MATH_REF)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_gbm_simulate: SMC_MATH_REF is for smc_train_targets / smc_train_step");
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
    launch_aux(normalize_kernel<float>, dim3(blocks), dim3(256), 0, as_stream(stream), contracts_dev,
                       n_contracts, timesteps, n_paths, static_cast<float*>(paths_dev), rowsum_dev);
  else
    launch_aux(normalize_kernel<double>, dim3(blocks), dim3(256), 0, as_stream(stream), contracts_dev,
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

// smc_train_targets (and smc_train_step's fallback for the shapes its fused launch does not take)
static int32_t train_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int32_t network_size,
                             int32_t batches_per_mc_run, uint64_t mc_seed, const int64_t* ordinal_dev,
                             int64_t ordinal0, int32_t scheme, int32_t normalization, int32_t dtype, int32_t store_mode,
                             void* paths_dev, int64_t path_pitch, int64_t chunk_contracts, double* rowsum_dev,
                             void* targets_dev, void* workspace_dev, int64_t workspace_size, void* stream) {
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
  const size_t csz = dtype == SMC_DTYPE_F32 ? 2 * sizeof(float) : 2 * sizeof(double);
  const int64_t chunk = chunk_contracts < n_contracts ? chunk_contracts : n_contracts;
  const bool all_rows = rowsum_dev != nullptr;
  const int32_t W = slices_for(P, workspace_dev != nullptr);
  double* partials = nullptr;
  uint32_t* arrivals = nullptr;
  uint32_t* queues = nullptr;
  if (W > 1) {
    if (workspace_size < static_cast<int64_t>(workspace_bytes(chunk, timesteps, P, all_rows)))
      return fail(SMC_ERR_INVALID_SHAPE, "smc_train_targets: workspace smaller than smc_engine_workspace_bytes");
    partials = static_cast<double*>(workspace_dev);
    arrivals = reinterpret_cast<uint32_t*>(partials + chunk * W * (all_rows ? timesteps : 1));
    queues = arrivals + chunk;
  }
  for (int64_t off = 0; off < n_contracts; off += chunk_contracts) {
    const int64_t nb = n_contracts - off < chunk_contracts ? n_contracts - off : chunk_contracts;
    EngineArgs a{contracts_dev + off * 6, nb, timesteps, P, network_size, batches_per_mc_run, mc_seed,
                 ordinal_dev, ordinal0 + off, scheme, normalization != SMC_NORM_RAW, store_mode, 1,
                 all_rows ? 1 : 0, paths_dev,
                 rowsum_dev ? rowsum_dev + off * timesteps : nullptr,
                 static_cast<char*>(targets_dev) + static_cast<size_t>(off) * network_size * csz, path_pitch,
                 W, partials, arrivals, queues};
    if (int32_t st = dispatch_engine(a, dtype, as_stream(stream))) return st;
  }
  return SMC_OK;
}

int32_t smc_train_targets(const double* contracts_dev, int64_t n_contracts, int32_t timesteps, int32_t network_size,
                          int32_t batches_per_mc_run, uint64_t mc_seed, const int64_t* ordinal_dev, int64_t ordinal0,
                          int32_t scheme, int32_t normalization, int32_t dtype, int32_t store_mode, void* paths_dev,
                          int64_t path_pitch, int64_t chunk_contracts, double* rowsum_dev, void* targets_dev,
                          void* workspace_dev, int64_t workspace_size, void* stream) {
  return train_targets(contracts_dev, n_contracts, timesteps, network_size, batches_per_mc_run, mc_seed, ordinal_dev,
                       ordinal0, scheme, normalization, dtype, store_mode, paths_dev, path_pitch, chunk_contracts,
                       rowsum_dev, targets_dev, workspace_dev, workspace_size, stream);
}

int32_t smc_train_step(const uint32_t* sobol_tables_dev, int32_t dim, const double* lower_dev, const double* upper_dev,
                       int64_t* cursor_dev, int64_t index_offset, int64_t advance, double* contracts_dev,
                       float* cvnn_input_dev, int64_t n_contracts, int32_t timesteps, int32_t network_size,
                       int32_t batches_per_mc_run, uint64_t mc_seed, int32_t scheme, int32_t normalization,
                       int32_t dtype, int32_t store_mode, void* paths_dev, int64_t path_pitch, int64_t chunk_contracts,
                       void* targets_dev, void* sync_dev, int64_t sync_bytes, void* stream) {
  if (!sobol_tables_dev || !lower_dev || !upper_dev || !cursor_dev || !contracts_dev || !sync_dev)
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_step: NULL buffer");
  if (dim != 6) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_step: dim must be 6 (BlackScholes.Inputs)");
  const bool dynamic = (scheme & SMC_TRAIN_DYNAMIC) != 0;  // every contract of the resident launch from the queue
  scheme &= ~SMC_TRAIN_DYNAMIC;
  if (index_offset < 0 || advance < 0) return fail(SMC_ERR_INVALID_ARGUMENT, "smc_train_step: negative offset");
  if (network_size <= 0 || batches_per_mc_run <= 0)
    return fail(SMC_ERR_INVALID_SHAPE, "smc_train_step: network_size and batches_per_mc_run must be > 0");
  const hipStream_t s = as_stream(stream);
  const int64_t P = static_cast<int64_t>(network_size) * batches_per_mc_run;
  if (path_pitch != 0 && (path_pitch < P || (path_pitch != P && path_pitch % kPathsPerLane != 0)))
    return fail(SMC_ERR_INVALID_SHAPE, "smc_train_step: path_pitch must be 0, P, or a multiple of 4 >= P");
  const int64_t need = smc_train_step_sync_bytes(timesteps, network_size, batches_per_mc_run, dtype, path_pitch);
  if (need <= 0) return fail(SMC_ERR_HIP, "smc_train_step: device query failed");
  if (sync_bytes < need) return fail(SMC_ERR_INVALID_SHAPE, "smc_train_step: sync area smaller than smc_train_step_sync_bytes");
  EngineArgs a{};
  a.B = n_contracts;
  a.T = timesteps;
  a.P = P;
  a.N = network_size;
  a.M = batches_per_mc_run;
  a.seed = mc_seed;
  a.ordinal_dev = cursor_dev + 1;
  a.scheme = scheme;
  a.normalize = normalization != SMC_NORM_RAW;
  a.store = store_mode;
  a.simulate = 1;
  a.paths = paths_dev;
  a.targets = targets_dev;
  a.pitch = path_pitch;
  a.slices = 1;
  a.res_slices = resident_slices(P);
  char* sync = static_cast<char*>(sync_dev);
  a.done = reinterpret_cast<uint32_t*>(sync);
  a.status = reinterpret_cast<uint32_t*>(sync + SMC_SYNC_STATUS_OFFSET);
  a.launch_fail = reinterpret_cast<uint32_t*>(sync + SMC_SYNC_LAUNCH_FAIL_OFFSET);
  a.res_queue = reinterpret_cast<uint32_t*>(sync + 64);
  a.res_static_q = dynamic ? 0 : 3;
  a.spin_limit = exchange_spin_limit();
  a.withhold = exchange_fault().withhold;
  if (a.res_slices > 1) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SMC_ERR_HIP, "smc_train_step: device query failed");
    }
    const ResSyncLayout l = res_sync_layout(a.res_slices, network_size, cus);
    a.res_groups = static_cast<int32_t>(l.groups);
    a.res_cnt = reinterpret_cast<uint32_t*>(sync + 128);
    a.res_xsum = reinterpret_cast<double*>(sync + l.xsum_off);
    a.res_xcol = reinterpret_cast<double*>(sync + l.xcol_off);
  }
  const bool fused = dtype == SMC_DTYPE_F32 && n_contracts > 0 && chunk_contracts > 0 &&
                     valid_scheme(scheme) && (scheme & SMC_MATH_REF) == 0 && (store_mode == SMC_STORE_ALL || store_mode == SMC_STORE_TERMINAL) &&
                     paths_dev && targets_dev && (wave_ok(a, true) || resident_ok(a, true) || packed_ok(a, true));
  if (fused) {
    // one resident launch per chunk of contracts; each draws its own contracts, the last advances
    // the cursor (the earlier ones read it unchanged)
    a.sobol = sobol_tables_dev;
    a.sobol_dim = dim;
    a.lower = lower_dev;
    a.upper = upper_dev;
    a.cursor = cursor_dev;
    for (int64_t off = 0; off < n_contracts; off += chunk_contracts) {
      const int64_t nb = n_contracts - off < chunk_contracts ? n_contracts - off : chunk_contracts;
      EngineArgs c = a;
      c.B = nb;
      c.ordinal0 = index_offset + off;
      c.contracts = contracts_dev + off * 6;
      c.contracts_out = contracts_dev + off * 6;
      c.cvnn_out = cvnn_input_dev ? cvnn_input_dev + off * 6 : nullptr;
      c.targets = static_cast<char*>(targets_dev) + static_cast<size_t>(off) * network_size * 2 * sizeof(float);
      c.sobol_index0 = index_offset + off;
      c.advance = off + nb == n_contracts ? advance : 0;
      if (int32_t st = dispatch_engine(c, dtype, s)) return st;
    }
    return SMC_OK;
  }
  // any other shape: the Sobol draw, the targets launch(es), then the cursor advance
  if (int32_t st = smc_sobol_draw(sobol_tables_dev, dim, cursor_dev, index_offset, n_contracts, lower_dev, upper_dev,
                                  contracts_dev, cvnn_input_dev, stream))
    return st;
  if (int32_t st = train_targets(contracts_dev, n_contracts, timesteps, network_size, batches_per_mc_run, mc_seed,
                                 cursor_dev + 1, index_offset, scheme, normalization, dtype, store_mode, paths_dev,
                                 path_pitch, chunk_contracts, nullptr, targets_dev, nullptr, 0, stream))
    return st;
  launch_aux(advance_cursor_kernel, dim3(1), dim3(64), 0, s, cursor_dev, advance);
  return check_launch("advance_cursor_kernel");
}

int64_t smc_train_step_sync_bytes(int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run, int32_t dtype,
                                  int64_t path_pitch) {
  if (network_size <= 0 || batches_per_mc_run <= 0) return kStepSyncBytes;
  EngineArgs a{};
  a.T = timesteps;
  a.N = network_size;
  a.P = static_cast<int64_t>(network_size) * batches_per_mc_run;
  a.simulate = 1;
  a.targets = &a;
  a.pitch = path_pitch;
  a.slices = 1;
  a.res_slices = resident_slices(a.P);
  if (a.res_slices <= 1) return kStepSyncBytes;
  a.res_cnt = reinterpret_cast<uint32_t*>(&a);  // any non-null: the shape test only
  a.res_xsum = a.res_xcol = reinterpret_cast<double*>(&a);
  a.done = reinterpret_cast<uint32_t*>(&a);
  if (!(resident_ok(a, (dtype & 0xff) == SMC_DTYPE_F32))) return kStepSyncBytes;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0) {
    (void)hipGetLastError();
    return -1;
  }
  return res_sync_layout(a.res_slices, network_size, cus).bytes;
}

const char* smc_train_step_kernel(int32_t timesteps, int32_t network_size, int32_t batches_per_mc_run, int32_t dtype,
                                  int64_t path_pitch) {
  EngineArgs a{};
  a.T = timesteps;
  a.N = network_size;
  a.P = static_cast<int64_t>(network_size) * batches_per_mc_run;
  a.simulate = 1;
  a.targets = &a;
  a.pitch = path_pitch;
  a.slices = 1;
  a.res_slices = resident_slices(a.P);
  a.res_cnt = reinterpret_cast<uint32_t*>(&a);
  a.res_xsum = a.res_xcol = reinterpret_cast<double*>(&a);
  a.done = reinterpret_cast<uint32_t*>(&a);
  a.normalize = (dtype & SMC_QUERY_RAW) ? 0 : 1;
  a.store = SMC_STORE_ALL;
  if (dtype & SMC_MATH_REF)  // the checks launch_engine makes (f32, the padded pitch, whole contracts)
    return (dtype & 0xff) == SMC_DTYPE_F32 && ref_ok(a) ? "rows_ref_kernel+cf_kernel" : "unsupported";
  if (wave_ok(a, (dtype & 0xff) == SMC_DTYPE_F32)) return "wave_kernel";
  if (resident_ok(a, (dtype & 0xff) == SMC_DTYPE_F32))
    return a.res_slices > 1 ? "resident_kernel(sliced)" : "resident_kernel";
  return smc_train_targets_kernel(timesteps, network_size, a.P, dtype, path_pitch, 0);
}

int64_t smc_engine_workspace_bytes(int64_t chunk_contracts, int32_t timesteps, int64_t n_paths, int32_t all_rows) {
  if (chunk_contracts <= 0 || timesteps <= 0 || n_paths <= 0) return 0;
  return static_cast<int64_t>(workspace_bytes(chunk_contracts, timesteps, n_paths, all_rows != 0));
}

const char* smc_train_targets_kernel(int32_t timesteps, int32_t network_size, int64_t n_paths, int32_t dtype,
                                     int64_t path_pitch, int32_t sliced) {
  EngineArgs a{};
  a.T = timesteps;
  a.N = network_size;
  a.P = n_paths;
  a.simulate = 1;
  a.targets = &a;  // any non-null: the training call always writes targets
  a.pitch = path_pitch;
  a.slices = slices_for(n_paths, sliced != 0);
  a.store = SMC_STORE_ALL;
  const bool f32 = (dtype & 0xff) == SMC_DTYPE_F32;
  a.normalize = (dtype & SMC_QUERY_RAW) ? 0 : 1;
  if (dtype & SMC_MATH_REF)  // the checks launch_engine makes (f32, the padded pitch, no slices)
    return f32 && ref_ok(a) ? "rows_ref_kernel+cf_kernel" : "unsupported";
  if (wave_ok(a, f32)) return "wave_kernel";
  if (resident_ok(a, f32)) return "resident_kernel";
  if (packed_ok(a, f32)) return "packed_kernel";
  if (split_ok(a, f32) && a.T == kRowBlock && a.P % kChunk == 0) return "paths_kernel+cf_kernel";
  if (rows_ok(a, f32)) return "rows_kernel+cf_kernel";
  if (split_ok(a, f32)) return "paths_kernel+cf_kernel";
  return a.slices > 1 ? "queue_kernel" : "contract_kernel";
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
    launch_aux((normals_kernel<float, false>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<float*>(out_dev));
  else if (dtype == SMC_DTYPE_F32)
    launch_aux((normals_kernel<float, true>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<float*>(out_dev));
  else if (dtype == SMC_DTYPE_F64)
    launch_aux((normals_kernel<double, false>), dim3(blocks), dim3(256), 0, as_stream(stream), mc_seed,
                       static_cast<uint64_t>(ordinal), rows, cols, static_cast<double*>(out_dev));
  else
    return fail(SMC_ERR_INVALID_ARGUMENT, "smc_normals: bad dtype");
  return check_launch("normals_kernel");
}

#pragma GCC visibility pop
}  // extern "C"
