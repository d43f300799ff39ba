// Store probe 5: does the FOOTPRINT of the path scratch set the store rate?  The C2 step writes
// 17.2 GB (4096 contracts x 16 rows x 65536 f32 at the padded pitch).  Same bytes per launch in
// every variant; the contracts land in a ring of R contract slots (R = 4096: the whole batch, as
// now; smaller R: slot b mod R, the reference's reuse of one io buffer per contract, gbm.py:400-426).
// Persistent 1024-thread workgroups, one per CU, 4096-path chunks, 16 row streams (resident_kernel's
// store order), one dwordx4 per lane per row.
//   hipcc -O3 --offload-arch=gfx950 ringbench.hip -o ringbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
constexpr int CHUNK = 4096, NCHUNK = P / CHUNK;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), 0x7fffffff, 0x00020000);
}

// AUX < 0: flat global_store_dwordx4 (the path kernel's non-terminal rows); else a buffer store
// with that cache-policy field (gfx950: 1 sc0, 2 nt, 16 sc1)
template <int AUX>
__global__ __launch_bounds__(1024) void ring_store(float* out, int R) {
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    float* base = out + static_cast<int64_t>(b % R) * T * PITCH;
#pragma unroll 1
    for (int c = 0; c < NCHUNK; ++c) {
      v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if constexpr (AUX < 0)  // wave-uniform row base + 32-bit lane offset (lane_paths' form)
          *reinterpret_cast<v4f*>(reinterpret_cast<char*>(base + t * PITCH + c * CHUNK) + threadIdx.x * 16u) = v;
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base + t * PITCH + c * CHUNK), threadIdx.x * 16, 0, AUX);
        v.x += 1.f;
      }
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
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t alloc = (size_t)B * T * PITCH * 4;
  const double bytes = (double)B * T * P * 4;
  float* out;
  CK(hipMalloc(&out, alloc));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double nbytes, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    (void)hipEventRecord(e0);
    const int iters = 10;
    for (int i = 0; i < iters; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= iters;
    printf("%-40s %8.3f ms  %7.1f GB/s\n", name, ms, nbytes / (ms * 1e6));
    fflush(stdout);
  };
  char name[64];
  timeit("memset 17.2 GB", bytes, [&] { (void)hipMemsetAsync(out, 0, (size_t)bytes); });
  for (double gb : {8.0, 4.0, 2.0, 1.0}) {
    const size_t n = (size_t)(gb * (1 << 30));
    const int reps = (int)(bytes / n + 0.5);
    snprintf(name, sizeof name, "grid_fill %.0f GiB x %d", gb, reps);
    timeit(name, (double)n * reps, [&] {
      for (int r = 0; r < reps; ++r) grid_fill<<<2048 * 8, 256>>>(out, (int64_t)(n / 16));
    });
  }
  timeit("grid_fill 17.2 GB x 1", bytes, [&] { grid_fill<<<2048 * 8, 256>>>(out, (int64_t)(bytes / 16)); });
  for (int R : {4096, 2048, 1024, 512, 256}) {
    snprintf(name, sizeof name, "ring_store sc1 R=%d (%.2f GB)", R, (double)R * T * PITCH * 4 / 1e9);
    timeit(name, bytes, [&] { ring_store<16><<<cus, 1024>>>(out, R); });
  }
  for (int rep = 0; rep < 2; ++rep) {
    timeit("ring_store flat global_store R=4096", bytes, [&] { ring_store<-1><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer aux=0 R=4096", bytes, [&] { ring_store<0><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer sc0 R=4096", bytes, [&] { ring_store<1><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer nt R=4096", bytes, [&] { ring_store<2><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer sc1 R=4096", bytes, [&] { ring_store<16><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer sc0 sc1 R=4096", bytes, [&] { ring_store<17><<<cus, 1024>>>(out, 4096); });
    timeit("ring_store buffer nt sc1 R=4096", bytes, [&] { ring_store<18><<<cus, 1024>>>(out, 4096); });
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
