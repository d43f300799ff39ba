// Store-pacing probe (round 3): the C2 path bytes (4096 contracts x 16 rows x 65536 f32) written
// with no compute run 2.85 ms through hipMemset and 2.89 ms through a 256 x 256-thread linear fill,
// but 3.3 ms through the same fill with 1024-thread workgroups, and every per-contract order of
// orderbench.hip takes 3.0-3.1 ms.  Is the difference the number of stores in flight per CU?
//   fill   linear grid-stride fill; VM = max stores in flight per wave (s_waitcnt vmcnt after each)
//   chunk  resident_kernel's order (4096-path chunks, 16 row streams), 1024 threads, VM as above
//   ilv    contract-interleaved layout [T][P/K][B][K]
//   paced  chunk / ilv with a compute proxy between stores (D dependent v_fma + v_exp_f32 per lane
//          and store, in 4 chains: about the resident kernel's VALU work per row store)
//   hipcc -O3 --offload-arch=gfx950 pacebench.hip -o pacebench && ./pacebench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), 0x7fffffff, 0x00020000);
}

template <int VM>
__device__ __forceinline__ void throttle() {
  if constexpr (VM == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (VM == 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (VM == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (VM == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (VM == 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
}

// D dependent fma + exp per chain, 4 chains (the compute proxy)
template <int D>
__device__ __forceinline__ void work(v4f& v) {
#pragma unroll
  for (int i = 0; i < D; ++i) {
    v.x = __builtin_amdgcn_exp2f(fmaf(v.x, 0.999f, 1e-7f)) * 0.5f;
    v.y = __builtin_amdgcn_exp2f(fmaf(v.y, 0.999f, 1e-7f)) * 0.5f;
    v.z = __builtin_amdgcn_exp2f(fmaf(v.z, 0.999f, 1e-7f)) * 0.5f;
    v.w = __builtin_amdgcn_exp2f(fmaf(v.w, 0.999f, 1e-7f)) * 0.5f;
  }
}

template <int NT, int VM>
__global__ __launch_bounds__(NT) void fill(float* out, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * NT;
  v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x; i < n16; i += stride) {
    reinterpret_cast<v4f*>(out)[i] = v;
    throttle<VM>();
    v.x += 1.f;
  }
}

// ILV = 0: [B][T][PITCH] in 4096-path chunks (resident_kernel); ILV = 1: [T][P/K][B][K], K = 4 NT
template <int NT, int VM, int ILV, int D>
__global__ __launch_bounds__(NT) void contracts(float* out) {
  constexpr int K = 4 * NT;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(threadIdx.x)};
    for (int c = 0; c < P / K; ++c) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float* piece = ILV ? out + ((static_cast<int64_t>(t) * (P / K) + c) * B + b) * K
                           : out + (static_cast<int64_t>(b) * T + t) * PITCH + static_cast<int64_t>(c) * K;
        work<D>(v);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(piece), threadIdx.x * 16u, 0, 0);
        throttle<VM>();
      }
    }
  }
}

template <typename F>
void timeit(const char* name, F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i) launch();
  const int iters = 8;
  (void)hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= iters;
  const double bytes = static_cast<double>(B) * T * P * 4;
  std::printf("%-40s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  std::fflush(stdout);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* out;
  CK(hipMalloc(&out, static_cast<size_t>(B) * T * PITCH * 4));
  std::printf("CUs %d, %d contracts x %d rows x %lld paths (pitch %lld)\n", cus, B, T, (long long)P, (long long)PITCH);
  const int64_t n16 = static_cast<int64_t>(B) * T * P / 4;
  for (int rep = 0; rep < 2; ++rep) {
    timeit("memset", [&] { (void)hipMemsetAsync(out, 0, static_cast<size_t>(B) * T * P * 4); });
    timeit("fill 256x256", [&] { fill<256, 0><<<256, 256>>>(out, n16); });
    timeit("fill 256x1024", [&] { fill<1024, 0><<<256, 1024>>>(out, n16); });
    timeit("fill 256x1024 vm1", [&] { fill<1024, 1><<<256, 1024>>>(out, n16); });
    timeit("fill 256x1024 vm2", [&] { fill<1024, 2><<<256, 1024>>>(out, n16); });
    timeit("fill 256x1024 vm4", [&] { fill<1024, 4><<<256, 1024>>>(out, n16); });
    timeit("chunk nt1024", [&] { contracts<1024, 0, 0, 0><<<cus, 1024>>>(out); });
    timeit("chunk nt1024 vm1", [&] { contracts<1024, 1, 0, 0><<<cus, 1024>>>(out); });
    timeit("chunk nt1024 vm2", [&] { contracts<1024, 2, 0, 0><<<cus, 1024>>>(out); });
    timeit("chunk nt1024 vm4", [&] { contracts<1024, 4, 0, 0><<<cus, 1024>>>(out); });
    timeit("chunk nt1024 vm8", [&] { contracts<1024, 8, 0, 0><<<cus, 1024>>>(out); });
    timeit("ilv nt1024", [&] { contracts<1024, 0, 1, 0><<<cus, 1024>>>(out); });
    timeit("ilv nt1024 vm1", [&] { contracts<1024, 1, 1, 0><<<cus, 1024>>>(out); });
    timeit("ilv nt1024 vm2", [&] { contracts<1024, 2, 1, 0><<<cus, 1024>>>(out); });
    timeit("ilv nt1024 vm4", [&] { contracts<1024, 4, 1, 0><<<cus, 1024>>>(out); });
    timeit("ilv nt512 (K2048)", [&] { contracts<512, 0, 1, 0><<<cus, 512>>>(out); });
    timeit("ilv nt512 x2/CU (K2048)", [&] { contracts<512, 0, 1, 0><<<2 * cus, 512>>>(out); });
    timeit("paced D4 chunk nt1024", [&] { contracts<1024, 0, 0, 4><<<cus, 1024>>>(out); });
    timeit("paced D8 chunk nt1024", [&] { contracts<1024, 0, 0, 8><<<cus, 1024>>>(out); });
    timeit("paced D12 chunk nt1024", [&] { contracts<1024, 0, 0, 12><<<cus, 1024>>>(out); });
    timeit("paced D8 chunk nt1024 vm2", [&] { contracts<1024, 2, 0, 8><<<cus, 1024>>>(out); });
    timeit("paced D8 chunk nt1024 vm4", [&] { contracts<1024, 4, 0, 8><<<cus, 1024>>>(out); });
    timeit("paced D8 ilv nt1024", [&] { contracts<1024, 0, 1, 8><<<cus, 1024>>>(out); });
    timeit("paced D8 ilv nt1024 vm2", [&] { contracts<1024, 2, 1, 8><<<cus, 1024>>>(out); });
    timeit("paced D12 ilv nt1024", [&] { contracts<1024, 0, 1, 12><<<cus, 1024>>>(out); });
  }
  CK(hipFree(out));
  return 0;
}
