// Store-rate probe, round 5 (after storebench7): the C2 path store in resident_kernel's ORDER (persistent
// 1024-thread workgroups, one per CU; per contract, per 4096-path chunk, 16 row stores of 16 B per lane), with
// and without XCD affinity.  storebench7 found that a sweep runs at 6.5-6.8 TB/s when every XCD writes only the
// address units of one residue mod 8 (1 KiB or 4 KiB units) and at 5.6-6.0 when every XCD writes every residue.
//   base    resident_kernel today: workgroup g runs contracts g, g + 256, ...; a contract's 16 chunks x 16 rows
//   aff1K   the contract split over the 8 XCDs: block g (XCD x = g mod 8) of group k = g / 8 runs contracts k,
//           k + 32, ...; of every row it writes the 1 KiB units u = x (mod 8) (with the row base aligned to
//           8 KiB: pitch a multiple of 2048 floats): 32 units = 2 passes of 16 waves
//   aff4K   the same with 4 KiB units (XCD x: units u = x mod 8 of 4 KiB; a wave writes one 1 KiB quarter)
// Each variant at several row pitches (floats): 66560 (today's, 260 KiB: rows alternate 0 / 4 KiB mod 8 KiB),
// 67584 (264 KiB = 33 x 8 KiB), 69632 (272 KiB = 17 x 16 KiB), 73728 (288 KiB = 9 x 32 KiB).
//   hipcc -O3 --offload-arch=gfx950 storebench8.hip -o v/storebench8 && ./v/storebench8
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st(float* p, float x) {
  const v4f v = {x, 2.f, 3.f, 4.f};
  *reinterpret_cast<v4f*>(p) = v;
}

// one persistent 1024-thread workgroup per CU (the dynamic LDS keeps a second one off the CU)
__global__ __launch_bounds__(1024) void base(float* out, int64_t pitch) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) lds[0] = 0.f;
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    float* cb = out + b * T * pitch;
    for (int64_t ch = 0; ch < P; ch += 4096) {
#pragma unroll
      for (int t = 0; t < T; ++t) st(cb + t * pitch + ch + 4 * threadIdx.x, static_cast<float>(t));
    }
  }
}

// UNIT = 1024 (1 KiB = 256 floats) or 4096 (4 KiB) bytes; XCD x writes units u = x mod 8 of each row
template <int UNIT>
__global__ __launch_bounds__(1024) void aff(float* out, int64_t pitch) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) lds[0] = 0.f;
  const int x = blockIdx.x & 7, k = blockIdx.x >> 3, groups = gridDim.x >> 3;
  constexpr int UF = UNIT / 4;                 // floats per unit
  constexpr int64_t units = P / UF;            // units per row
  constexpr int64_t mine = units / 8;          // this XCD's units per row
  constexpr int per_pass = 1024 * 4 / UF;      // units one pass of the workgroup covers (4 floats per lane)
  const int lane_unit = (threadIdx.x * 4) / UF, within = (threadIdx.x * 4) % UF;
  for (int64_t b = k; b < B; b += groups) {
    float* cb = out + b * T * pitch;
    for (int64_t j0 = 0; j0 < mine; j0 += per_pass) {
      const int64_t u = 8 * (j0 + lane_unit) + x;
#pragma unroll
      for (int t = 0; t < T; ++t) st(cb + t * pitch + u * UF + within, static_cast<float>(t));
    }
  }
}

template <class F>
void timeit(const char* name, int64_t pitch, F launch) {
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
  std::printf("%-8s pitch %6lld  %7.3f ms  %7.1f GB/s\n", name, (long long)pitch, ms, bytes / ms / 1e6);
  std::fflush(stdout);
}

int main(int argc, char**) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int64_t max_pitch = 98304;
  float* out;
  CK(hipMalloc(&out, static_cast<size_t>(B) * T * max_pitch * 4));
  const size_t lds = 96 * 1024;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(base), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(aff<1024>), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(aff<4096>), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  std::printf("CUs %d; buffer base %% 64 KiB = %lld\n", cus, (long long)(reinterpret_cast<uintptr_t>(out) % 65536));
  const bool sweep = argc > 1;  // pitch sweep of the base order only
  for (int rep = 0; rep < 2; ++rep) {
    if (sweep) {
      for (int64_t pad = 1024; pad <= 32768; pad += (pad < 12288 ? 1024 : 4096))
        timeit("base", P + pad, [&] { base<<<cus, 1024, lds>>>(out, P + pad); });
      continue;
    }
    for (int64_t pitch : {66560LL, 67584LL, 69632LL, 73728LL}) {
      timeit("base", pitch, [&] { base<<<cus, 1024, lds>>>(out, pitch); });
      timeit("aff1K", pitch, [&] { aff<1024><<<cus, 1024, lds>>>(out, pitch); });
      timeit("aff4K", pitch, [&] { aff<4096><<<cus, 1024, lds>>>(out, pitch); });
    }
  }
  CK(hipFree(out));
  return 0;
}
