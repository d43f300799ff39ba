// f32 MFMA GEMM probe for the wide-layer network step (round 3): C[M][N] = A[M][K] . B[N][K]^T with
// v_mfma_f32_16x16x4_f32, operands staged through LDS in K stages (double-buffered, next stage's
// global loads in flight during the current stage's MFMAs).  Shapes of the C2/H=256 network:
//   fwd / bwd-input: M = 512 features, N = 4096 batch, K = 512 (A = packed weights [M][K],
//                    B = activations [N][K]: both K-contiguous, "NN" staging)
//   wgrad:           M = 512, N = 528, K = 4096 batch (A = dU stored [K][M], B = Z stored [K][N]:
//                    transposed staging), split over batch segments
//   hipcc -O3 --offload-arch=gfx950 lgemm.hip -o lgemm && ./lgemm
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ f32x4 mma4(f32x4 acc, f32x4 a, f32x4 b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
}

// BM x BN tile per workgroup of NT threads; waves WM x WN, each (BM/WM) x (BN/WN) of 16x16 tiles.
// TA / TB: the operand is stored [K][M] / [K][N] in global memory (transposed staging into LDS).
template <int BM, int BN, int WM, int WN, bool TA, bool TB, int BK = 32, bool PF = false>
__global__ __launch_bounds__(64 * WM * WN) void lgemm(const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                       int ksplit) {
  constexpr int NT = 64 * WM * WN;
  constexpr int LDK = BK + 4;  // LDS row stride (floats): an odd multiple of 16 B
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 16x16 tiles per wave
  __shared__ __attribute__((aligned(16))) float sa[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float sb[2][BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kseg = K / ksplit, kbeg = blockIdx.z * kseg;
  // staging: NN operand rows of BK floats = BK/4 float4 per row; T operand: BK rows of BM floats
  constexpr int AV = BM * BK / 4 / NT, BV = BN * BK / 4 / NT;
  f32x4 ra[AV], rb[BV];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int i = v * NT + tid;
      if constexpr (!TA) {
        const int r = i / (BK / 4), q = i % (BK / 4);
        ra[v] = *reinterpret_cast<const f32x4*>(A + static_cast<int64_t>(m0 + r) * lda + k0 + 4 * q);
      } else {
        const int kk = i / (BM / 4), q = i % (BM / 4);
        ra[v] = *reinterpret_cast<const f32x4*>(A + static_cast<int64_t>(k0 + kk) * lda + m0 + 4 * q);
      }
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int i = v * NT + tid;
      if constexpr (!TB) {
        const int r = i / (BK / 4), q = i % (BK / 4);
        rb[v] = *reinterpret_cast<const f32x4*>(B + static_cast<int64_t>(n0 + r) * ldb + k0 + 4 * q);
      } else {
        const int kk = i / (BN / 4), q = i % (BN / 4);
        rb[v] = *reinterpret_cast<const f32x4*>(B + static_cast<int64_t>(k0 + kk) * ldb + n0 + 4 * q);
      }
    }
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int i = v * NT + tid;
      if constexpr (!TA) {
        const int r = i / (BK / 4), q = i % (BK / 4);
        *reinterpret_cast<f32x4*>(&sa[buf][r * LDK + 4 * q]) = ra[v];
      } else {
        const int kk = i / (BM / 4), q = i % (BM / 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) sa[buf][(4 * q + e) * LDK + kk] = ra[v][e];
      }
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      const int i = v * NT + tid;
      if constexpr (!TB) {
        const int r = i / (BK / 4), q = i % (BK / 4);
        *reinterpret_cast<f32x4*>(&sb[buf][r * LDK + 4 * q]) = rb[v];
      } else {
        const int kk = i / (BN / 4), q = i % (BN / 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) sb[buf][(4 * q + e) * LDK + kk] = rb[v][e];
      }
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nst = kseg / BK;
  fetch(kbeg);
  put(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) fetch(kbeg + (st + 1) * BK);
    if constexpr (!PF) {
#pragma unroll
      for (int kb = 0; kb < BK; kb += 16) {
        f32x4 af[TM], bf[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const f32x4*>(&sa[buf][((wm * TM + i) * 16 + c) * LDK + kb + 4 * g]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const f32x4*>(&sb[buf][((wn * TN + j) * 16 + c) * LDK + kb + 4 * g]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma4(acc[i][j], af[i], bf[j]);
      }
    } else {  // fragments of k block kb + 16 read while block kb's MFMAs issue
      f32x4 af[2][TM], bf[2][TN];
      auto ld = [&](int s, int kb) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[s][i] = *reinterpret_cast<const f32x4*>(&sa[buf][((wm * TM + i) * 16 + c) * LDK + kb + 4 * g]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[s][j] = *reinterpret_cast<const f32x4*>(&sb[buf][((wn * TN + j) * 16 + c) * LDK + kb + 4 * g]);
      };
      ld(0, 0);
#pragma unroll
      for (int kb = 0; kb < BK; kb += 16) {
        const int s = (kb / 16) & 1;
        if (kb + 16 < BK) ld(s ^ 1, kb + 16);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mma4(acc[i][j], af[s][i], bf[s][j]);
      }
    }
    if (st + 1 < nst) put(buf ^ 1);
    __syncthreads();
  }
  // C/D fragment: lane (c, g) holds rows 4g..4g+3 of column c of each 16x16 tile
  float* Cz = C + static_cast<int64_t>(blockIdx.z) * M * N;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + (wn * TN + j) * 16 + c;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cz[static_cast<int64_t>(m0 + (wm * TM + i) * 16 + 4 * g + r) * N + col] = acc[i][j][r];
    }
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, int BK = 32, bool PF = false>
float run(const char* name, const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb,
          int ksplit, const std::vector<float>& ha, const std::vector<float>& hb) {
  dim3 grid(M / BM, N / BN, ksplit);
  auto launch = [&] { lgemm<BM, BN, WM, WN, TA, TB, BK, PF><<<grid, 64 * WM * WN>>>(A, B, C, M, N, K, lda, ldb, ksplit); };
  launch();
  (void)hipDeviceSynchronize();
  // spot check against a host dot product (split-K partials summed)
  std::vector<float> hc(static_cast<size_t>(M) * N * ksplit);
  (void)hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost);
  double maxrel = 0;
  for (int t = 0; t < 64; ++t) {
    const int m = (t * 97) % M, n = (t * 389) % N;
    double ref = 0;
    for (int k = 0; k < K; ++k) {
      const double a = TA ? ha[static_cast<size_t>(k) * lda + m] : ha[static_cast<size_t>(m) * lda + k];
      const double b = TB ? hb[static_cast<size_t>(k) * ldb + n] : hb[static_cast<size_t>(n) * ldb + k];
      ref += a * b;
    }
    double got = 0;
    for (int z = 0; z < ksplit; ++z) got += hc[static_cast<size_t>(z) * M * N + static_cast<size_t>(m) * N + n];
    maxrel = fmax(maxrel, fabs(got - ref) / (fabs(ref) + 1e-3));
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 50;
  (void)hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= iters;
  const double tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12;
  std::printf("%-34s %4dx%4dx%4d split %d: %7.2f us  %6.1f TF/s (%.2f of 157.3)  maxrel %.1e\n", name, M, N, K,
              ksplit, ms * 1e3, tf, tf / 157.3, maxrel);
  std::fflush(stdout);
  return ms;
}

int main() {
  const int M = 512, N = 4096, K = 512;
  std::vector<float> ha(static_cast<size_t>(4096) * 4096), hb(static_cast<size_t>(4096) * 4096);
  for (size_t i = 0; i < ha.size(); ++i) ha[i] = static_cast<float>((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  for (size_t i = 0; i < hb.size(); ++i) hb[i] = static_cast<float>((i * 40503u + 7) % 1000) / 1000.f - 0.5f;
  float *A, *B, *C;
  CK(hipMalloc(&A, ha.size() * 4));
  CK(hipMalloc(&B, hb.size() * 4));
  CK(hipMalloc(&C, static_cast<size_t>(4096) * 4096 * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  // fwd / bwd-input: A [512][512] weights, B [4096][512] activations
  run<64, 64, 2, 2, false, false>("NN 64x64 w2x2 bk32", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<64, 64, 2, 2, false, false, 64>("NN 64x64 w2x2 bk64", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<64, 64, 2, 2, false, false, 32, true>("NN 64x64 w2x2 bk32 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<64, 64, 2, 2, false, false, 64, true>("NN 64x64 w2x2 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<128, 64, 2, 2, false, false, 64, true>("NN 128x64 w2x2 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<64, 128, 2, 2, false, false, 64, true>("NN 64x128 w2x2 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<128, 64, 4, 1, false, false, 64, true>("NN 128x64 w4x1 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<64, 64, 1, 1, false, false, 64, true>("NN 64x64 w1x1 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  run<32, 64, 1, 2, false, false, 64, true>("NN 32x64 w1x2 bk64 pf", A, B, C, M, N, K, K, K, 1, ha, hb);
  // wgrad with K-contiguous copies (Z^T, dU^T written by the producing epilogue): NN over the batch
  run<64, 64, 2, 2, false, false, 64, true>("wgrad NN 64x64 bk64 pf split8", A, B, C, 512, 512, 4096, 4096, 4096, 8, ha, hb);
  run<64, 64, 2, 2, false, false, 64, true>("wgrad NN 64x64 bk64 pf split4", A, B, C, 512, 512, 4096, 4096, 4096, 4, ha, hb);
  run<64, 64, 2, 2, true, true, 32, true>("wgrad TT 64x64 bk32 pf split8", A, B, C, 512, 512, 4096, 512, 512, 8, ha, hb);
  return 0;
}
