// Store-order probe: does the ORDER in which a persistent workgroup writes its contract's 16 rows
// set the C2 store rate?  Same bytes in every variant (4096 contracts x 16 rows x 65536 f32 at the
// padded pitch, 17.19 GB), one persistent workgroup per CU, one dwordx4 per lane per store:
//   chunkK   resident_kernel's order: the contract in chunks of K paths, all 16 rows per chunk
//            (K = 4096: 16 row streams of 16 KiB per chunk)
//   rowmaj   row-major: row 0 of the whole contract (256 KiB contiguous), then row 1, ...
//   memset   hipMemsetAsync of the same rows (one call per row block)
//   hipcc -O3 --offload-arch=gfx950 orderbench.hip -o orderbench && ./orderbench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536, PITCH = 66560;
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), 0x7fffffff, 0x00020000);
}

// chunks of K paths (K / (4 * NT) dwordx4 per lane per row), rows in order within a chunk
template <int NT, int K, int AUX>
__global__ __launch_bounds__(NT) void chunked(float* out) {
  constexpr int PER = K / (4 * NT);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    float* base = out + static_cast<int64_t>(b) * T * PITCH;
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(threadIdx.x)};
    for (int c = 0; c < P / K; ++c) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float* row = base + t * PITCH + static_cast<int64_t>(c) * K;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(row), (k * NT + threadIdx.x) * 16u, 0, AUX);
          v.x += 1.f;
        }
      }
    }
  }
}

// row-major: each row of the contract written whole before the next
template <int NT, int AUX>
__global__ __launch_bounds__(NT) void rowmaj(float* out) {
  constexpr int PER = P / (4 * NT);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    float* base = out + static_cast<int64_t>(b) * T * PITCH;
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(threadIdx.x)};
    for (int t = 0; t < T; ++t) {
      float* row = base + t * PITCH;
#pragma unroll 8
      for (int k = 0; k < PER; ++k) {
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(row), (k * NT + threadIdx.x) * 16u, 0, AUX);
        v.x += 1.f;
      }
    }
  }
}

// row pairs: rows (t, t+1) of the whole contract interleaved per lane-block (the draw order of a
// Box-Muller pair gives both steps at once)
template <int NT, int AUX>
__global__ __launch_bounds__(NT) void rowpair(float* out) {
  constexpr int PER = P / (4 * NT);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    float* base = out + static_cast<int64_t>(b) * T * PITCH;
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(threadIdx.x)};
    for (int t = 0; t < T; t += 2) {
      float* r0 = base + t * PITCH;
      float* r1 = r0 + PITCH;
#pragma unroll 8
      for (int k = 0; k < PER; ++k) {
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(r0), (k * NT + threadIdx.x) * 16u, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(r1), (k * NT + threadIdx.x) * 16u, 0, AUX);
        v.x += 1.f;
      }
    }
  }
}

// contract-interleaved layout [T][P/K][B][K]: chunk j of row t of every contract side by side, so the
// persistent workgroups (contracts b, b + grid, ...) write neighbouring K-path pieces at the same time
template <int NT, int K>
__global__ __launch_bounds__(NT) void interleaved(float* out) {
  constexpr int PER = K / (4 * NT);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(threadIdx.x)};
    for (int c = 0; c < P / K; ++c) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        float* piece = out + ((static_cast<int64_t>(t) * (P / K) + c) * B + b) * K;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(piece), (k * NT + threadIdx.x) * 16u, 0, 0);
          v.x += 1.f;
        }
      }
    }
  }
}

// chip-wide contracts: wave w of workgroup c owns contract (r * NW + w)'s path slice c (64 lanes x 4
// paths = 256 paths; 256 workgroups cover a 65,536-path contract), so the same-numbered waves of all
// workgroups write one contract row's 256 KiB window at about the same time
template <int NT>
__global__ __launch_bounds__(NT) void chipwide(float* out) {
  constexpr int NW = NT / 64;
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
  const int slices = static_cast<int>(P / 256);  // 256 paths per wave slice
  for (int64_t task = static_cast<int64_t>(blockIdx.x) * NW + w; task < static_cast<int64_t>(B) * slices;
       task += static_cast<int64_t>(gridDim.x) * NW) {
    // tasks ordered so that consecutive workgroups take neighbouring slices of one contract
    const int64_t b = (task / NW) / slices * NW + task % NW;
    const int64_t sl = (task / NW) % slices;
    float* base = out + b * T * PITCH + sl * 256;
    v4f v = {1.f + b, 2.f, 3.f, static_cast<float>(l)};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base + t * PITCH), l * 16u, 0, 0);
      v.x += 1.f;
    }
  }
}

// linear grid-stride fill over the whole padded matrix (hipMemset's __amd_rocclr_fillBufferAligned
// runs 256 x 256 threads of this shape)
template <int NT>
__global__ __launch_bounds__(NT) void fill_linear(float* out, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * NT;
  v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x; i < n16; i += stride) {
    reinterpret_cast<v4f*>(out)[i] = v;
    v.x += 1.f;
  }
}

template <typename F>
void timeit(const char* name, F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i) launch();
  const int iters = 10;
  (void)hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= iters;
  const double bytes = static_cast<double>(B) * T * P * 4;
  std::printf("%-34s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  std::fflush(stdout);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* out;
  CK(hipMalloc(&out, static_cast<size_t>(B) * T * PITCH * 4));
  std::printf("CUs %d, %d contracts x %d rows x %lld paths (pitch %lld)\n", cus, B, T, (long long)P, (long long)PITCH);
  const int64_t n16 = static_cast<int64_t>(B) * T * PITCH / 4;
  for (int rep = 0; rep < 2; ++rep) {
    timeit("memset (rows of 17.45 GB)", [&] { (void)hipMemsetAsync(out, 0, static_cast<size_t>(B) * T * PITCH * 4); });
    timeit("fill_linear 256x256 (17.45 GB)", [&] { fill_linear<256><<<256, 256>>>(out, n16); });
    timeit("fill_linear 256x1024 (17.45 GB)", [&] { fill_linear<256><<<1024, 256>>>(out, n16); });
    timeit("fill_linear 1024x256 (17.45 GB)", [&] { fill_linear<1024><<<256, 1024>>>(out, n16); });
    timeit("fill_linear 512x512 (17.45 GB)", [&] { fill_linear<512><<<512, 512>>>(out, n16); });
    timeit("interleaved K4096 nt1024", [&] { interleaved<1024, 4096><<<cus, 1024>>>(out); });
    timeit("interleaved K8192 nt1024", [&] { interleaved<1024, 8192><<<cus, 1024>>>(out); });
    timeit("interleaved K16384 nt1024", [&] { interleaved<1024, 16384><<<cus, 1024>>>(out); });
    timeit("interleaved K4096 nt512", [&] { interleaved<512, 4096><<<cus, 512>>>(out); });
    timeit("interleaved K2048 nt512", [&] { interleaved<512, 2048><<<cus, 512>>>(out); });
    timeit("chipwide nt1024 x256", [&] { chipwide<1024><<<256, 1024>>>(out); });
    timeit("chipwide nt256 x256", [&] { chipwide<256><<<256, 256>>>(out); });
    timeit("chipwide nt512 x256", [&] { chipwide<512><<<256, 512>>>(out); });
    timeit("rowmaj nt256", [&] { rowmaj<256, 0><<<cus, 256>>>(out); });
    timeit("rowmaj nt256 x2/CU", [&] { rowmaj<256, 0><<<2 * cus, 256>>>(out); });
    timeit("rowmaj nt128", [&] { rowmaj<128, 0><<<cus, 128>>>(out); });
    timeit("chunk4096 nt256", [&] { chunked<256, 4096, 0><<<cus, 256>>>(out); });
    timeit("chunk16384 nt256", [&] { chunked<256, 16384, 0><<<cus, 256>>>(out); });
    timeit("chunk4096 nt1024 (resident)", [&] { chunked<1024, 4096, 0><<<cus, 1024>>>(out); });
    timeit("chunk8192 nt1024", [&] { chunked<1024, 8192, 0><<<cus, 1024>>>(out); });
    timeit("chunk16384 nt1024", [&] { chunked<1024, 16384, 0><<<cus, 1024>>>(out); });
    timeit("chunk16384 nt512", [&] { chunked<512, 16384, 0><<<cus, 512>>>(out); });
    timeit("chunk32768 nt512", [&] { chunked<512, 32768, 0><<<cus, 512>>>(out); });
    timeit("rowmaj nt1024", [&] { rowmaj<1024, 0><<<cus, 1024>>>(out); });
    timeit("rowmaj nt512", [&] { rowmaj<512, 0><<<cus, 512>>>(out); });
    timeit("rowmaj nt512 x2/CU", [&] { rowmaj<512, 0><<<2 * cus, 512>>>(out); });
    timeit("rowpair nt512", [&] { rowpair<512, 0><<<cus, 512>>>(out); });
    timeit("rowpair nt1024", [&] { rowpair<1024, 0><<<cus, 1024>>>(out); });
    timeit("rowmaj nt512 nt-policy", [&] { rowmaj<512, 2><<<cus, 512>>>(out); });
    timeit("chunk4096 nt1024 nt-policy", [&] { chunked<1024, 4096, 2><<<cus, 1024>>>(out); });
  }
  CK(hipFree(out));
  return 0;
}
