// Store-pattern probe 5: does the per-instruction density of a wave's row stores set the store rate?
// Every variant writes the same 8 GiB as 1 KiB-per-lane-group rows (persistent grid, 16 waves per CU):
//   dense16  : each store instruction covers 64 lanes x 16 B contiguous (f32 4-path lanes, C2)
//   pair32   : each lane owns 32 contiguous bytes, written as two 16-B stores (f64 4-path lanes): each
//              instruction covers every other 16-B piece of 2 KiB
//   quad64   : each lane owns 64 contiguous bytes, four 16-B stores (f32 16-path span lanes)
//   pair32p  : as pair32, but the two halves are exchanged between lane pairs first (ds_bpermute), so
//              each instruction is again 64 x 16 B contiguous
//   hipcc -O3 --offload-arch=gfx950 storebench5.hip -o storebench5
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int64_t kBytes = int64_t{8} << 30;

template <int PER_LANE_16B, bool PERMUTE>
__global__ __launch_bounds__(256) void fill(char* out, int64_t iters) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * 4;
  const int64_t span = 64 * 16 * PER_LANE_16B;  // bytes per wave iteration
  v4f v[PER_LANE_16B];
#pragma unroll
  for (int k = 0; k < PER_LANE_16B; ++k) v[k] = v4f{1.f * k, 2.f, 3.f, 4.f};
  for (int64_t it = 0; it < iters; ++it) {
    char* base = out + (it * nwaves + wave) * span;
    if constexpr (PERMUTE) {
      // lane l holds pieces (2l, 2l+1) of the 2 KiB; instruction k stores piece 64k + l: lane l needs
      // piece (64k + l), owned by lane (64k + l) / 2, slot l & 1
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int src = (64 * k + lane) >> 1;
        v4f w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src * 4, __builtin_bit_cast(int, v[0][e])));
          const float a1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src * 4, __builtin_bit_cast(int, v[1][e])));
          w[e] = (lane & 1) ? a1 : a0;
        }
        reinterpret_cast<v4f*>(base)[64 * k + lane] = w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < PER_LANE_16B; ++k) reinterpret_cast<v4f*>(base)[PER_LANE_16B * lane + k] = v[k];
    }
#pragma unroll
    for (int k = 0; k < PER_LANE_16B; ++k) v[k].w += 1.f;
  }
}

template <int P16, bool PERM>
float run(char* buf, int grid, const char* name) {
  const int64_t span = 64 * 16 * P16;
  const int64_t iters = kBytes / (span * grid * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((fill<P16, PERM>), dim3(grid), dim3(256), 0, 0, buf, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((fill<P16, PERM>), dim3(grid), dim3(256), 0, 0, buf, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double bytes = static_cast<double>(iters) * span * grid * 4;
  printf("%-8s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  return ms;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  char* buf = nullptr;
  if (hipMalloc(&buf, kBytes + (64 << 20)) != hipSuccess) return 1;
  const int grid = cus * 4;  // 16 waves per CU
  for (int rep = 0; rep < 2; ++rep) {
    run<1, false>(buf, grid, "dense16");
    run<2, false>(buf, grid, "pair32");
    run<4, false>(buf, grid, "quad64");
    run<2, true>(buf, grid, "pair32p");
  }
  hipFree(buf);
  return 0;
}
