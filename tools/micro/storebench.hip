// Pure-store microbenchmark of the path-matrix write pattern (no compute): 4096 contracts x
// [16][65536] f32 = 17.2 GB per launch.  Variants isolate the memory-side cost of the
// contract kernel's store order.   hipcc -O3 --offload-arch=gfx950 storebench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536;

// A: contract kernel order — WG per contract, 2048-path chunks, 16 rows per chunk, float4/lane
template <bool NT>
__global__ __launch_bounds__(512) void rows_chunked(float* out) {
  const int64_t b = blockIdx.x;
  float* base = out + b * T * P;
  for (int64_t chunk = 0; chunk < P; chunk += 2048) {
    float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      float4* dst = reinterpret_cast<float4*>(base + t * P + chunk) + threadIdx.x;
      typedef float v4f __attribute__((ext_vector_type(4)));
      if (NT) __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(dst));
      else *dst = v;
      v.x += 1.f;
    }
  }
}
// B: WG per contract, linear over its 4 MB (row-major), float4/lane
__global__ __launch_bounds__(512) void linear_wg(float* out) {
  const int64_t b = blockIdx.x;
  float4* base = reinterpret_cast<float4*>(out + b * T * P);
  float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t i = threadIdx.x; i < T * P / 4; i += 512) { base[i] = v; v.x += 1.f; }
}
// C: grid-stride linear over the whole buffer (fill-like)
__global__ __launch_bounds__(256) void grid_fill(float* out, int64_t n4) {
  float4* o = reinterpret_cast<float4*>(out);
  float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) o[i] = v;
}
// D: chunked like A but 8 rows per chunk pass (two passes of 8 rows)
__global__ __launch_bounds__(512) void rows_chunked8(float* out) {
  const int64_t b = blockIdx.x;
  float* base = out + b * T * P;
  for (int t0 = 0; t0 < T; t0 += 8)
    for (int64_t chunk = 0; chunk < P; chunk += 2048) {
      float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        reinterpret_cast<float4*>(base + (t0 + t) * P + chunk)[threadIdx.x] = v;
        v.x += 1.f;
      }
    }
}
// E: like A but the chunk order is rotated per contract (chunk start offset = b * 7 mod 32)
__global__ __launch_bounds__(512) void rows_chunked_rot(float* out) {
  const int64_t b = blockIdx.x;
  float* base = out + b * T * P;
  for (int ci = 0; ci < 32; ++ci) {
    const int64_t chunk = ((ci + b * 7) & 31) * 2048;
    float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<float4*>(base + t * P + chunk)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}
// F: 256-thread WGs, chunk 1024 paths, 16 rows
__global__ __launch_bounds__(256) void rows_chunked256(float* out) {
  const int64_t b = blockIdx.x;
  float* base = out + b * T * P;
  for (int64_t chunk = 0; chunk < P; chunk += 1024) {
    float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<float4*>(base + t * P + chunk)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const size_t bytes = (size_t)B * T * P * 4;
  float* out;
  CK(hipMalloc(&out, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    hipEventRecord(e0);
    const int iters = 10;
    for (int i = 0; i < iters; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= iters;
    printf("%-22s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e6));
  };
  timeit("memset", [&] { hipMemsetAsync(out, 0, bytes); });
  timeit("grid_fill(2048x256)", [&] { grid_fill<<<2048 * 8, 256>>>(out, bytes / 16); });
  timeit("linear_wg", [&] { linear_wg<<<B, 512>>>(out); });
  timeit("rows_chunked", [&] { rows_chunked<false><<<B, 512>>>(out); });
  timeit("rows_chunked_nt", [&] { rows_chunked<true><<<B, 512>>>(out); });
  timeit("rows_chunked8", [&] { rows_chunked8<<<B, 512>>>(out); });
  timeit("rows_chunked_rot", [&] { rows_chunked_rot<<<B, 512>>>(out); });
  timeit("rows_chunked256", [&] { rows_chunked256<<<B, 256>>>(out); });
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
