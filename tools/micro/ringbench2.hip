// Store probe 6: which part of resident_kernel's structure slows its store stream?  The C2 store
// order (persistent 1024-thread workgroups, 4096-path chunks, 16 rows, padded pitch) with, per
// flag bit: 1 = 150 KB of dynamic LDS (one workgroup per CU, as resident_kernel), 2 = each lane
// parks its 4 values per chunk in LDS (chunks 0..7, as the terminal row), 4 = a Philox-like
// dependent integer chain per chunk (the PathStream seed), 8 = ten LDS-only barriers per
// contract (the CF phase), 16 = the data of each row depends on the previous row (a recursion).
//   hipcc -O3 --offload-arch=gfx950 ringbench2.hip -o ringbench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
constexpr int CHUNK = 4096, NCHUNK = P / CHUNK;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int F>
__global__ __launch_bounds__(1024) void probe(float* out, float* sink) {
  extern __shared__ v4f lds[];
  float acc = 0.f;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    float* base = out + static_cast<int64_t>(b) * T * PITCH;
#pragma unroll 1
    for (int c = 0; c < NCHUNK; ++c) {
      uint32_t s0 = threadIdx.x + c, s1 = b, s2 = 7, s3 = 11;
      if constexpr (F & 4) {
#pragma unroll
        for (int r = 0; r < 10; ++r) {
          const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * s0;
          const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * s2;
          const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ s1 ^ r;
          const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ s3 ^ (r * 3);
          s1 = static_cast<uint32_t>(p1);
          s3 = static_cast<uint32_t>(p0);
          s0 = n0;
          s2 = n2;
        }
      }
      v4f v = {1.f, 2.f, 3.f, static_cast<float>(s0 & 7)};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        *reinterpret_cast<v4f*>(reinterpret_cast<char*>(base + t * PITCH + c * CHUNK) + threadIdx.x * 16u) = v;
        if constexpr (F & 16) v = v * 1.0001f + 0.5f;
        else v.x += 1.f;
      }
      if constexpr (F & 2)
        if (c < 8) lds[c * 1024 + threadIdx.x] = v;
    }
    if constexpr (F & 8) {
#pragma unroll 1
      for (int k = 0; k < 10; ++k) {
        if constexpr (F & 2) acc += lds[(k & 7) * 1024 + (threadIdx.x ^ k)].x;
        lds_barrier();
      }
    }
  }
  if (acc == 12345.f) sink[threadIdx.x] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t alloc = (size_t)B * T * PITCH * 4;
  const double bytes = (double)B * T * P * 4;
  float *out, *sink;
  CK(hipMalloc(&out, alloc));
  CK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    (void)hipEventRecord(e0);
    const int iters = 10;
    for (int i = 0; i < iters; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= iters;
    printf("%-40s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e6));
    fflush(stdout);
  };
  const size_t big = 150 * 1024;
#define RUN(F)                                                                                      \
  do {                                                                                              \
    const size_t l = (F & 1) ? big : ((F & 2) ? 8 * 1024 * 16 : 0);                                 \
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<F>),                                 \
                           hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(big)));     \
    timeit("flags " #F, [&] { probe<F><<<cus, 1024, l>>>(out, sink); });                            \
  } while (0)
  for (int rep = 0; rep < 2; ++rep) {
    RUN(0); RUN(1); RUN(3); RUN(4); RUN(8); RUN(11); RUN(16); RUN(31);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
