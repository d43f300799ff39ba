// Store-rate probe: torch's fill_ writes a 17.3 GB buffer at ~6.9 TB/s (tools/probe_fill.py) while the
// C2 path launch and round 3's persistent store patterns (orderbench.hip) stay near 6.0.  Is the gap
// the write ORDER, the store instruction, or the launch geometry (persistent workgroups against a grid
// of small one-shot workgroups)?  Same bytes in every variant: 4096 contracts x 16 rows x 65536 f32 at
// the padded pitch 66048 (17.3 GB).
//   memset            hipMemsetAsync of the whole buffer
//   lin_np_global     one-shot 256-thread workgroups, each 16 KiB contiguous (4 global_store_dwordx4 per
//                     lane), block i at i * 16 KiB: a linear sweep (torch's fill_ geometry)
//   lin_np_buffer     the same with buffer_store_dwordx4
//   lin_persist       256 persistent 1024-thread workgroups sweeping the same 16 KiB pieces
//   rows_np_contract  one-shot workgroups writing row chunks (contract b, row t, 16 KiB chunk c) in
//                     contract-major order (linear but for the pitch gaps)
//   rows_np_resident  one-shot workgroups in resident_kernel's write order: 256 contracts in flight,
//                     for each 4096-path chunk all 16 rows, the 256 contracts side by side
//   hipcc -O3 --offload-arch=gfx950 storebench6.hip -o v/storebench6 && ./v/storebench6
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
constexpr int64_t P = 65536, PITCH = 66048;
constexpr int64_t PIECE = 4096;  // floats per 16 KiB piece (one row chunk of 4096 paths)
constexpr int64_t CHUNKS = P / PIECE;  // 16
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0), 0x7fffffff, 0x00020000);
}

// a 256-thread workgroup writes VEC x 4 KiB at `p`: VEC dwordx4 per lane, each store instruction 4 KiB
// contiguous
template <bool BUFFER, int VEC = 4>
__device__ __forceinline__ void piece(float* p, float x) {
  const v4f v = {x, 2.f, 3.f, static_cast<float>(threadIdx.x)};
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    if constexpr (BUFFER)
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(p), (k * 256 + threadIdx.x) * 16u, 0, 0);
    else
      *reinterpret_cast<v4f*>(p + (k * 256 + threadIdx.x) * 4) = v;
  }
}

template <bool BUFFER, int VEC = 4>
__global__ __launch_bounds__(256) void lin_np(float* out) {
  piece<BUFFER, VEC>(out + static_cast<int64_t>(blockIdx.x) * (1024 * VEC), 1.f);
}

__global__ __launch_bounds__(1024) void lin_persist(float* out, int64_t pieces) {
  const int sub = threadIdx.x >> 8;  // four 256-thread quarters
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + sub; i < pieces; i += static_cast<int64_t>(gridDim.x) * 4) {
    const v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      *reinterpret_cast<v4f*>(out + i * PIECE + (k * 256 + (threadIdx.x & 255)) * 4) = v;
  }
}

// (contract, row, chunk) of one-shot block i, contract-major
__global__ __launch_bounds__(256) void rows_np_contract(float* out) {
  const int64_t i = blockIdx.x;
  const int64_t c = i % CHUNKS, t = (i / CHUNKS) % T, b = i / (CHUNKS * T);
  piece<false>(out + (b * T + t) * PITCH + c * PIECE, 1.f);
}

// resident order: round r of 256 contracts; within it chunk c, row t, then the 256 contracts
__global__ __launch_bounds__(256) void rows_np_resident(float* out) {
  const int64_t i = blockIdx.x;
  const int64_t j = i % 256, t = (i / 256) % T, c = (i / (256 * T)) % CHUNKS, r = i / (256 * T * CHUNKS);
  const int64_t b = r * 256 + j;
  piece<false>(out + (b * T + t) * PITCH + c * PIECE, 1.f);
}

// 4 KiB pieces (one dwordx4 per lane per block): contract-major and resident order
__global__ __launch_bounds__(256) void rows_np_contract_v1(float* out) {
  const int64_t i = blockIdx.x;
  const int64_t c = i % (P / 1024), t = (i / (P / 1024)) % T, b = i / ((P / 1024) * T);
  piece<false, 1>(out + (b * T + t) * PITCH + c * 1024, 1.f);
}
// resident order at 4 KiB pieces: round r of 256 contracts, 4096-path chunk c, row t, then the 4 pieces of
// the row chunk, then the 256 contracts
__global__ __launch_bounds__(256) void rows_np_resident_v1(float* out) {
  const int64_t i = blockIdx.x;
  const int64_t j = i % 256, q = (i / 256) % 4, t = (i / 1024) % T, c = (i / (1024 * T)) % CHUNKS,
                r = i / (1024 * T * CHUNKS);
  piece<false, 1>(out + ((r * 256 + j) * T + t) * PITCH + c * PIECE + q * 1024, 1.f);
}
// resident order with the 4 pieces of a row chunk outermost inside the chunk: (r, c, q, t, j)
__global__ __launch_bounds__(256) void rows_np_resident_v1b(float* out) {
  const int64_t i = blockIdx.x;
  const int64_t j = i % 256, t = (i / 256) % T, q = (i / (256 * T)) % 4, c = (i / (1024 * T)) % CHUNKS,
                r = i / (1024 * T * CHUNKS);
  piece<false, 1>(out + ((r * 256 + j) * T + t) * PITCH + c * PIECE + q * 1024, 1.f);
}

template <class F>
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
  const double bytes = static_cast<double>(B) * T * P * 4;  // the path bytes (the pitch gaps not counted)
  std::printf("%-28s %7.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  std::fflush(stdout);
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t total = static_cast<size_t>(B) * T * PITCH * 4;
  float* out;
  CK(hipMalloc(&out, total));
  const int64_t row_pieces = static_cast<int64_t>(B) * T * CHUNKS;  // 1,048,576 pieces of the path rows
  const int64_t lin_pieces = static_cast<int64_t>(B) * T * P / PIECE;  // the same bytes, linearly
  std::printf("CUs %d, %d contracts x %d rows x %lld paths (pitch %lld), %.2f GB\n", cus, B, T, (long long)P,
              (long long)PITCH, total / 1e9);
  for (int rep = 0; rep < 2; ++rep) {
    timeit("memset (whole buffer)", [&] { (void)hipMemsetAsync(out, 0, total); });
    timeit("lin_np_global vec4", [&] { lin_np<false><<<static_cast<unsigned>(lin_pieces), 256>>>(out); });
    timeit("lin_np_global vec1", [&] { lin_np<false, 1><<<static_cast<unsigned>(4 * lin_pieces), 256>>>(out); });
    timeit("lin_np_global vec2", [&] { lin_np<false, 2><<<static_cast<unsigned>(2 * lin_pieces), 256>>>(out); });
    timeit("lin_np_buffer", [&] { lin_np<true><<<static_cast<unsigned>(lin_pieces), 256>>>(out); });
    timeit("lin_persist 256x1024", [&] { lin_persist<<<cus, 1024>>>(out, lin_pieces); });
    timeit("lin_persist 512x1024", [&] { lin_persist<<<2 * cus, 1024>>>(out, lin_pieces); });
    timeit("rows_np_contract", [&] { rows_np_contract<<<static_cast<unsigned>(row_pieces), 256>>>(out); });
    timeit("rows_np_resident", [&] { rows_np_resident<<<static_cast<unsigned>(row_pieces), 256>>>(out); });
    timeit("rows_np_contract_v1", [&] { rows_np_contract_v1<<<static_cast<unsigned>(4 * row_pieces), 256>>>(out); });
    timeit("rows_np_resident_v1", [&] { rows_np_resident_v1<<<static_cast<unsigned>(4 * row_pieces), 256>>>(out); });
    timeit("rows_np_resident_v1b", [&] { rows_np_resident_v1b<<<static_cast<unsigned>(4 * row_pieces), 256>>>(out); });
  }
  CK(hipFree(out));
  return 0;
}
