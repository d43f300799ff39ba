// Store-pattern probe 2: the path matrix [B][T][pitch] (C2, padded pitch 66,560 floats) written
// by (a) one workgroup per contract looping over its 32 chunks of 2,048 paths (the current
// contract kernel) vs (b) several workgroups per contract, each owning G consecutive chunks,
// so that the resident grid writes few contracts' rows side by side; each with plain / sc1 / nt
// dwordx4 stores.   hipcc -O3 --offload-arch=gfx950 storebench2.hip -o storebench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
constexpr int CHUNK = 2048, NCHUNK = P / CHUNK;
typedef float v4f __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if constexpr (POL == 0) *p = v;
  else if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else if constexpr (POL == 2) __builtin_nontemporal_store(v, p);
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// G chunks per workgroup; grid = B * NCHUNK / G; workgroup w -> contract w / (NCHUNK/G)
template <int G, int POL>
__global__ __launch_bounds__(512) void split(float* out) {
  constexpr int per = NCHUNK / G;
  const int64_t b = blockIdx.x / per;
  const int64_t c0 = (blockIdx.x % per) * G;
  float* base = out + b * T * PITCH;
  for (int64_t c = c0; c < c0 + G; ++c) {
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      st<POL>(reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK) + threadIdx.x, v);
      v.x += 1.f;
    }
  }
}

// (c) contract-interleaved: resident workgroup slot s of R handles contract chunks so that
// consecutive workgroups write consecutive chunks of the same row set (G = 1 grid order but
// launched as a persistent grid of R workgroups striding over B * NCHUNK items)
template <int POL>
__global__ __launch_bounds__(512) void persistent(float* out, int items) {
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int64_t b = it / NCHUNK, c = it % NCHUNK;
    float* base = out + b * T * PITCH;
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      st<POL>(reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK) + threadIdx.x, v);
      v.x += 1.f;
    }
  }
}

__global__ __launch_bounds__(256) void grid_fill(float* out, int64_t n4) {
  v4f* o = reinterpret_cast<v4f*>(out);
  v4f v = {1.f, 2.f, 3.f, 4.f};
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) o[i] = v;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const size_t alloc = (size_t)B * T * PITCH * 4;
  const double bytes = (double)B * T * P * 4;
  float* out;
  CK(hipMalloc(&out, alloc));
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
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e6));
  };
  timeit("memset(same bytes)", [&] { (void)hipMemsetAsync(out, 0, (size_t)bytes); });
  timeit("grid_fill", [&] { grid_fill<<<2048 * 8, 256>>>(out, (int64_t)(bytes / 16)); });
#define SPLIT(G, POL, NAME) timeit(NAME, [&] { split<G, POL><<<B * NCHUNK / G, 512>>>(out); })
  SPLIT(32, 0, "wg/contract plain");
  SPLIT(32, 1, "wg/contract sc1");
  SPLIT(32, 2, "wg/contract nt");
  SPLIT(32, 3, "wg/contract sc0sc1");
  SPLIT(8, 0, "4 wg/contract plain");
  SPLIT(4, 0, "8 wg/contract plain");
  SPLIT(2, 0, "16 wg/contract plain");
  SPLIT(1, 0, "32 wg/contract plain");
  SPLIT(1, 1, "32 wg/contract sc1");
  SPLIT(4, 1, "8 wg/contract sc1");
  timeit("persistent 512 plain", [&] { persistent<0><<<512, 512>>>(out, B * NCHUNK); });
  timeit("persistent 512 sc1", [&] { persistent<1><<<512, 512>>>(out, B * NCHUNK); });
  timeit("persistent 1024 plain", [&] { persistent<0><<<1024, 512>>>(out, B * NCHUNK); });
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
