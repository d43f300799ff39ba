// Device helpers shared by the engine kernels (gbm.hip, basket.hip): buffer-descriptor row
// stores, the write-through hand-off between workgroups, LDS-only barriers and the in-LDS FFT
// of the CF targets.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace smc {
namespace {

// Stores / loads of bytes handed from one workgroup to another (possibly on another XCD):
// write-through (sc1) 16-B stores drained before the arrival add, sc1 loads after it
// (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms).
// 16-B write-through stores through a buffer descriptor on the wave-uniform row base: the
// compiler counts them in vmcnt and pads their data hazards.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* row_base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(row_base), static_cast<short>(0), 0x7fffffff,
                                           0x00020000);
}
__device__ __forceinline__ void store_wt(const void* row_base, uint32_t off, float4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, row_rsrc(row_base), off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void store_wt(const void* row_base, uint32_t off, double4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d lo = {v.x, v.y}, hi = {v.z, v.w};
  const __amdgpu_buffer_rsrc_t r = row_rsrc(row_base);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4f, lo), r, off, 0, 16);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4f, hi), r, off + 16, 0, 16);
}
// A path row's 16-B piece through a buffer descriptor, default cache policy (A/B at C2: the same
// time as the flat global_store_dwordx4 form and as sc1, tools/micro/ringbench.hip).
__device__ __forceinline__ void store_row(const void* row_base, uint32_t off, float4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f w = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(w, row_rsrc(row_base), off, 0, 0);
}
// 4 doubles (32 B) of an f64 path row: two 16-B pieces at off and off + 16.
__device__ __forceinline__ void store_row(const void* row_base, uint32_t off, double4 v) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d lo = {v.x, v.y}, hi = {v.z, v.w};
  const __amdgpu_buffer_rsrc_t r = row_rsrc(row_base);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4f, lo), r, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4f, hi), r, off + 16, 0, 0);
}
template <typename U>
__device__ __forceinline__ void put_sc1(U* p, U v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename U>
__device__ __forceinline__ U get_sc1(const U* p) {
  return __hip_atomic_load(const_cast<U*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over s < n of base[s * stride + idx] in order from 0.0, for data other workgroups published
// with put_sc1 after the caller saw their arrivals: write-through (sc1) buffer loads on the
// wave-uniform base, 8 in flight at a time (a loop of single atomic loads would pay one memory
// latency per term).  The compiler fence keeps the loads after the arrival poll.
__device__ __forceinline__ double ordered_sum_wt(const double* base, int64_t idx, int n, int64_t stride) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  const __amdgpu_buffer_rsrc_t r = row_rsrc(base);
  double t = 0.0;
  for (int s = 0; s < n; s += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)  // a clamped index keeps the batch straight-line; extra terms are dropped
      v[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                            r, static_cast<uint32_t>(((s + k < n ? s + k : s) * stride + idx) * 8),
                                            0, 16 /* sc1 */));
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (s + k < n) t += v[k];
  }
  return t;
}

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

// In-place radix-2 decimation-in-time FFT of the real sequence avg[0..N) into xr/xi (LDS), then
// bins 0..N/2 and their Hermitian mirror -> out.  Stage len = 2, 4, ..., N: butterfly j of N/2,
// i0 = (j / h) len + j mod h, i1 = i0 + h (h = len/2), w = cs[t] - i sn[t] with t = (j mod h) N/len:
// (tr, ti) = x[i1] w (4 products, 2 sums, no contraction), x[i1] = x[i0] - t, x[i0] = x[i0] + t.
__device__ __forceinline__ void lds_barrier() {  // LDS visibility only: no vmcnt drain of the stores
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One wave's LDS hand-off (no workgroup barrier): its own LDS writes complete and visible to its lanes.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// K rows at once (avg, xr, xi: [K][N]; out: [kv][N], rows k < kv written): the per-row arithmetic and
// order of one row, the (row, index) pairs spread over the NT threads (packed_kernel's contracts).
// WAVE: one wave runs it alone (NT = 64, lane index, wave-local LDS hand-offs, no s_barrier).
template <typename Real, int NT, bool LDS_ONLY = false, bool WAVE = false>
__device__ void fft_rows(const double* avg, const double* cs, const double* sn, int N, int K, int kv, double* xr,
                         double* xi, typename Complex2<Real>::type* out) {
  using C2 = typename Complex2<Real>::type;
  static_assert(!WAVE || NT == 64, "a wave-local FFT runs on the 64 lanes of one wave");
  const int tid = WAVE ? static_cast<int>(threadIdx.x & 63) : static_cast<int>(threadIdx.x);
  const int logN = 31 - __builtin_clz(static_cast<unsigned>(N));
  auto barrier = [] {
    if constexpr (WAVE) wave_lds_sync();
    else if constexpr (LDS_ONLY) lds_barrier();
    else __syncthreads();
  };
  for (int e = tid; e < K * N; e += NT) {
    const int k = e >> logN, n = e & (N - 1);
    const int r = static_cast<int>(__builtin_bitreverse32(static_cast<unsigned>(n)) >> (32 - logN));
    xr[k * N + r] = avg[e];
    xi[k * N + r] = 0.0;
  }
  barrier();
  // one radix-2 butterfly on registers, the operations of the stage loop in the same order
  auto bfly = [](double& br, double& bi, double& ar, double& ai, double wr, double wi) {
    const double tr = ar * wr - ai * wi;
    const double ti = ar * wi + ai * wr;
    ar = br - tr;
    ai = bi - ti;
    br = br + tr;
    bi = bi + ti;
  };
  // stages s and s + 1 fused per thread on the quad i0, i0 + h, i0 + 2h, i0 + 3h (h = 2^(s-1)): the
  // same butterflies with the same twiddles as two radix-2 stages, one barrier instead of two
  int s = 1;
  for (; s + 1 <= logN; s += 2) {
    const int h = 1 << (s - 1), shift = logN - s;
    for (int e = tid; e < K * (N / 4); e += NT) {
      const int qd = e & (N / 4 - 1);
      double* yr = xr + (e >> (logN - 2)) * N;
      double* yi = xi + (e >> (logN - 2)) * N;
      const int pos = qd & (h - 1);
      const int i0 = ((qd >> (s - 1)) << (s + 1)) + pos;
      double r0 = yr[i0], m0 = yi[i0], r1 = yr[i0 + h], m1 = yi[i0 + h];
      double r2 = yr[i0 + 2 * h], m2 = yi[i0 + 2 * h], r3 = yr[i0 + 3 * h], m3 = yi[i0 + 3 * h];
      const double w1r = cs[pos << shift], w1i = -sn[pos << shift];
      bfly(r0, m0, r1, m1, w1r, w1i);  // stage s: (i0, i0 + h), (i0 + 2h, i0 + 3h)
      bfly(r2, m2, r3, m3, w1r, w1i);
      const double w2r = cs[pos << (shift - 1)], w2i = -sn[pos << (shift - 1)];
      const double w3r = cs[(pos + h) << (shift - 1)], w3i = -sn[(pos + h) << (shift - 1)];
      bfly(r0, m0, r2, m2, w2r, w2i);  // stage s + 1: (i0, i0 + 2h), (i0 + h, i0 + 3h)
      bfly(r1, m1, r3, m3, w3r, w3i);
      yr[i0] = r0;
      yi[i0] = m0;
      yr[i0 + h] = r1;
      yi[i0 + h] = m1;
      yr[i0 + 2 * h] = r2;
      yi[i0 + 2 * h] = m2;
      yr[i0 + 3 * h] = r3;
      yi[i0 + 3 * h] = m3;
    }
    barrier();
  }
  if (s == logN) {  // an odd number of stages: the last one alone
    const int h = 1 << (s - 1), shift = logN - s;  // twiddle index t = (j mod h) << shift
    for (int e = tid; e < K * (N / 2); e += NT) {
      const int j = e & (N / 2 - 1);
      double* yr = xr + (e >> (logN - 1)) * N;
      double* yi = xi + (e >> (logN - 1)) * N;
      const int pos = j & (h - 1);
      const int i0 = ((j >> (s - 1)) << s) + pos, i1 = i0 + h;
      double br = yr[i0], bi = yi[i0], ar = yr[i1], ai = yi[i1];
      bfly(br, bi, ar, ai, cs[pos << shift], -sn[pos << shift]);
      yr[i1] = ar;
      yi[i1] = ai;
      yr[i0] = br;
      yi[i0] = bi;
    }
    barrier();
  }
  const int nb = N / 2 + 1;
  for (int e = tid; e < kv * nb; e += NT) {
    const int k = e / nb, kk = e - k * nb;
    const double* yr = xr + k * N;
    const double* yi = xi + k * N;
    C2* o = out + static_cast<int64_t>(k) * N;
    C2 v;
    v.x = static_cast<Real>(yr[kk]);
    v.y = static_cast<Real>(yi[kk]);
    o[kk] = v;
    if (kk != 0 && 2 * kk != N) {
      v.y = static_cast<Real>(-yi[kk]);
      o[N - kk] = v;
    }
  }
}

// One row: in-place radix-2 DIT FFT of avg[0..N) (N a power of two) -> out (fft_rows with K = 1).
template <typename Real, int NT, bool LDS_ONLY = false>
__device__ void fft_row(const double* avg, const double* cs, const double* sn, int N, double* xr, double* xi,
                        typename Complex2<Real>::type* out) {
  fft_rows<Real, NT, LDS_ONLY>(avg, cs, sn, N, 1, 1, xr, xi, out);
}

}  // namespace
// bf16 rounding (round to nearest even, torch's float -> bfloat16; NaN kept quiet) of the MFMA operands
__host__ __device__ inline float bf16_round(float x) {
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) {
    u |= 0x00400000u;  // quiet NaN
  } else {
    u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even (torch's float -> bfloat16)
  }
  u &= 0xffff0000u;
  float y;
  __builtin_memcpy(&y, &u, 4);
  return y;
}

__device__ __forceinline__ uint16_t bf16_bits(float x) { return static_cast<uint16_t>(__float_as_uint(bf16_round(x)) >> 16); }

}  // namespace smc
