// Store-pattern probe 4: does the LOCALITY of the concurrent write streams set the C2 store rate?
// The contract kernel has 512 resident workgroups, each writing its own contract's 16 rows
// (4.26 MB apart), i.e. 8192 concurrent 8-KB-piece streams spread over 2 GB.  A fill whose
// concurrently running workgroups write neighbouring addresses is the comparison.  Same bytes
// (C2: 4096 x 16 x 65536 f32 at the padded pitch) in every variant but the 8 GiB fill.
//   hipcc -O3 --offload-arch=gfx950 storebench4.hip -o storebench4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
constexpr int CHUNK = 2048, NCHUNK = P / CHUNK;
typedef float v4f __attribute__((ext_vector_type(4)));

// (a) time-major, one workgroup per contract, chunks in order (the contract kernel's stream)
__global__ __launch_bounds__(512) void time_major(float* out) {
  float* base = out + blockIdx.x * (int64_t)T * PITCH;
  for (int64_t c = 0; c < NCHUNK; ++c) {
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}

// (b) chunk-major: one workgroup per (contract, S consecutive chunks), blocks in contract order,
// so the resident grid covers 512 * S chunks = 16 * S contracts at a time
template <int S>
__global__ __launch_bounds__(512) void chunk_major(float* out) {
  const int64_t b = blockIdx.x / (NCHUNK / S);
  const int64_t c0 = (blockIdx.x % (NCHUNK / S)) * S;
  float* base = out + b * (int64_t)T * PITCH;
  for (int64_t c = c0; c < c0 + S; ++c) {
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}

// (c) persistent grid of 512 workgroups sweeping (contract, chunk) items in lock-step order:
// item i = k * 512 + blockIdx.x, contract i / 32, chunk i % 32 -> at any moment the grid writes
// 16 neighbouring contracts
__global__ __launch_bounds__(512) void sweep(float* out) {
  for (int64_t i = blockIdx.x; i < (int64_t)B * NCHUNK; i += gridDim.x) {
    const int64_t b = i / NCHUNK, c = i % NCHUNK;
    float* base = out + b * (int64_t)T * PITCH;
    v4f v = {1.f, 2.f, 3.f, (float)c};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<v4f*>(base + t * PITCH + c * CHUNK)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}

// (d) torch-style fill: each 256-thread workgroup writes 16 KB contiguous, no grid stride
__global__ __launch_bounds__(256) void block_fill(float* out) {
  v4f* o = reinterpret_cast<v4f*>(out) + blockIdx.x * 1024LL;
  const v4f v = {1.f, 2.f, 3.f, 4.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k * 256 + threadIdx.x] = v;
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
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, nbytes / (ms * 1e6));
    fflush(stdout);
  };
  const double gib8 = 8.0 * (1 << 30);
  timeit("memset (same bytes)", bytes, [&] { (void)hipMemsetAsync(out, 0, (size_t)bytes); });
  timeit("block_fill 8 GiB (torch fill_)", gib8, [&] { block_fill<<<(unsigned)(gib8 / 16384), 256>>>(out); });
  timeit("block_fill (same bytes)", bytes, [&] { block_fill<<<(unsigned)(bytes / 16384), 256>>>(out); });
  timeit("grid_fill", bytes, [&] { grid_fill<<<2048 * 8, 256>>>(out, (int64_t)(bytes / 16)); });
  timeit("time_major (contract kernel)", bytes, [&] { time_major<<<B, 512>>>(out); });
  timeit("chunk_major S=1", bytes, [&] { chunk_major<1><<<B * NCHUNK, 512>>>(out); });
  timeit("chunk_major S=4", bytes, [&] { chunk_major<4><<<B * NCHUNK / 4, 512>>>(out); });
  timeit("chunk_major S=8", bytes, [&] { chunk_major<8><<<B * NCHUNK / 8, 512>>>(out); });
  timeit("sweep (512 persistent)", bytes, [&] { sweep<<<512, 512>>>(out); });
  timeit("sweep (1024 persistent)", bytes, [&] { sweep<<<1024, 512>>>(out); });
  timeit("time_major (contract kernel) again", bytes, [&] { time_major<<<B, 512>>>(out); });
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
