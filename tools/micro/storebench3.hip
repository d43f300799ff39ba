// Store-pattern probe 3: C2's 17.2 GB path matrix written (a) time-major [B][T][pitch] as the
// contract kernel does (16 row streams per workgroup, 8 KB per row per chunk), vs (b) path-major
// [B][P][T] — each 2,048-path chunk is one contiguous 128 KB block — stored straight from
// registers (16 strided dwordx4 per lane) or through an LDS transpose (16 KB per wave, 1 KB
// contiguous per store instruction).   hipcc -O3 --offload-arch=gfx950 storebench3.hip -o storebench3
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
  else __builtin_nontemporal_store(v, p);
}

// (a) time-major, one workgroup per contract (the current layout)
template <int POL>
__global__ __launch_bounds__(512) void time_major(float* out) {
  float* base = out + blockIdx.x * (int64_t)T * PITCH;
  for (int64_t c = 0; c < NCHUNK; ++c) {
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      st<POL>(reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK) + threadIdx.x, v);
      v.x += 1.f;
    }
  }
}

// (b1) path-major from registers: lane's 4 paths x 16 steps = 256 contiguous bytes
template <int POL>
__global__ __launch_bounds__(512) void path_major_reg(float* out) {
  float* base = out + blockIdx.x * (int64_t)T * P;
  for (int64_t c = 0; c < NCHUNK; ++c) {
    v4f* lane = reinterpret_cast<v4f*>(base + c * CHUNK * T + threadIdx.x * 4 * T);
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      st<POL>(lane + k, v);
      v.x += 1.f;
    }
  }
}

// (b2) path-major through LDS: each wave stages its 16 KB and writes it as 16 x 1 KB
template <int POL>
__global__ __launch_bounds__(512) void path_major_lds(float* out) {
  __shared__ v4f stage[512 * 16];  // 128 KB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v4f* ws = stage + wave * 64 * 16;
  float* base = out + blockIdx.x * (int64_t)T * P;
  for (int64_t c = 0; c < NCHUNK; ++c) {
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      ws[lane * 16 + (k ^ (lane & 15))] = v;  // xor swizzle against bank conflicts
      v.x += 1.f;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) — wave-local staging, no barrier
    v4f* dst = reinterpret_cast<v4f*>(base + c * CHUNK * T) + wave * 64 * 16;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = k * 64 + lane;  // linear element of the wave's 16 KB
      const int l = e >> 4, kk = e & 15;
      st<POL>(dst + e, ws[l * 16 + (kk ^ (l & 15))]);
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
  timeit("time_major plain", [&] { time_major<0><<<B, 512>>>(out); });
  timeit("time_major nt", [&] { time_major<1><<<B, 512>>>(out); });
  timeit("path_major_reg plain", [&] { path_major_reg<0><<<B, 512>>>(out); });
  timeit("path_major_reg nt", [&] { path_major_reg<1><<<B, 512>>>(out); });
  timeit("path_major_lds plain", [&] { path_major_lds<0><<<B, 512>>>(out); });
  timeit("path_major_lds nt", [&] { path_major_lds<1><<<B, 512>>>(out); });
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
