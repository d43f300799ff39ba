// Store-rate probe, round 5: does WHICH XCD writes WHICH addresses set the HBM write rate?
// storebench6 measured one-shot 256-thread workgroups writing 4 KiB each in a linear sweep (block i at
// i * 4 KiB) at 6.8 TB/s, but 16 KiB per workgroup (block i at i * 16 KiB) at 6.0 TB/s.  One-shot blocks are
// dealt to the 8 XCDs round-robin (block i on XCD i mod 8), so in the 4 KiB sweep XCD x writes only the 4 KiB
// units u = x (mod 8), in the 16 KiB sweep every unit residue.  If the memory side interleaves the stacks /
// channels at some unit U, an XCD-to-unit affinity could be what runs faster.
// Variants (same 17.2 GB each, one-shot 256-thread workgroups, 4 dwordx4 stores per lane = 16 KiB per block):
//   aff U s   block i (XCD x = i mod 8) writes 4 units of U bytes: unit index  ((x + s) mod 8) + 8 * (4 (i / 8) + k)
//             for k = 0..3 (an XCD only ever writes units of one residue mod 8; s rotates which); U = 1 KiB..64 KiB
//             (U < 4 KiB: each store instruction covers U contiguous bytes and several per unit)
//   mix U     the same unit size, but block i writes units with residues (x + k) mod 8: every XCD every residue
//   lin16     storebench6's vec4 sweep (block i at i * 16 KiB)
//   lin4      storebench6's vec1 sweep (4 KiB blocks)
// The XCC_ID of every block is recorded and checked against i mod 8 (the assumed dispatch order).
//   hipcc -O3 --offload-arch=gfx950 storebench7.hip -o v/storebench7 && ./v/storebench7
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int64_t TOTAL = 4096LL * 16 * 65536 * 4;  // the C2 path bytes, 17.18 GB
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x;
}

// U < 4 KiB: block i writes 16 KiB as 4 * 4096 / U units of U bytes; each 4 KiB store instruction covers
// 4096 / U of them, spaced 8 units apart.  MODE 0: every unit of XCD x has residue (x + shift) mod 8 (affinity);
// MODE 1: residue (x + kk) mod 8 (every XCD writes every residue)
template <int MODE>
__global__ __launch_bounds__(256) void units(char* out, int64_t U, int shift) {
  const int64_t i = blockIdx.x;
  const int64_t x = i & 7, grp = i >> 3;
  const v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
  const int64_t per_store = 4096 / U;  // units covered by one 4 KiB store instruction
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t lane_unit = (threadIdx.x * 16) / U, within = (threadIdx.x * 16) % U;
    const int64_t kk = k * per_store + lane_unit;  // the block's kk-th unit
    const int64_t res = MODE == 0 ? (x + shift) & 7 : (x + kk) & 7;
    const int64_t unit = res + 8 * (4 * per_store * grp + kk);
    *reinterpret_cast<v4f*>(out + unit * U + within) = v;
  }
}

// U >= 4 KiB: the sweep in units of U, each unit written as U / 4 KiB pieces by consecutive "visits": block i
// writes piece q of unit (res + 8 * g): pieces per unit = U / 4096, blocks per XCD per unit group
__global__ __launch_bounds__(256) void big_units(char* out, int64_t U, int mode, int shift, unsigned* xcc_log) {
  const int64_t i = blockIdx.x;
  const int64_t x = i & 7, j = i >> 3;  // j-th block of XCD x
  if (threadIdx.x == 0 && xcc_log) xcc_log[i] = xcc_id();
  const v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
  const int64_t ppu = U / 4096;  // 4 KiB pieces per unit
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t piece = 4 * j + k;  // the XCD's piece number
    const int64_t g = piece / ppu, q = piece % ppu;
    const int64_t res = mode == 0 ? (x + shift) & 7 : (x + g) & 7;
    const int64_t unit = res + 8 * g;
    *reinterpret_cast<v4f*>(out + unit * U + q * 4096 + threadIdx.x * 16) = v;
  }
}

template <int VEC>
__global__ __launch_bounds__(256) void lin(char* out) {
  const v4f v = {1.f, 2.f, 3.f, static_cast<float>(threadIdx.x)};
#pragma unroll
  for (int k = 0; k < VEC; ++k)
    *reinterpret_cast<v4f*>(out + static_cast<int64_t>(blockIdx.x) * (4096 * VEC) + k * 4096 + threadIdx.x * 16) = v;
}

template <class F>
double timeit(const char* name, F launch) {
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
  std::printf("%-24s %7.3f ms  %7.1f GB/s\n", name, ms, TOTAL / ms / 1e6);
  std::fflush(stdout);
  return ms;
}

int main() {
  char* out;
  CK(hipMalloc(&out, TOTAL));
  const unsigned blocks = static_cast<unsigned>(TOTAL / 16384);  // 16 KiB per block
  unsigned* xlog;
  CK(hipMalloc(&xlog, blocks * sizeof(unsigned)));
  // dispatch order check
  big_units<<<blocks, 256>>>(out, 4096, 0, 0, xlog);
  CK(hipDeviceSynchronize());
  std::vector<unsigned> h(blocks);
  CK(hipMemcpy(h.data(), xlog, blocks * sizeof(unsigned), hipMemcpyDeviceToHost));
  int64_t match = 0;
  for (unsigned i = 0; i < blocks; ++i) match += (h[i] & 7) == (i & 7);
  std::printf("blocks %u, XCC_ID == i mod 8 for %.4f of them\n", blocks, double(match) / blocks);
  for (int rep = 0; rep < 2; ++rep) {
    timeit("lin4 (4 KiB blocks)", [&] { lin<1><<<4 * blocks, 256>>>(out); });
    timeit("lin16 (16 KiB blocks)", [&] { lin<4><<<blocks, 256>>>(out); });
    char name[64];
    for (int64_t U : {1024LL, 2048LL}) {
      for (int s = 0; s < 8; s += 4) {
        std::snprintf(name, sizeof name, "aff U=%lld s=%d", (long long)U, s);
        timeit(name, [&] { units<0><<<blocks, 256>>>(out, U, s); });
      }
      std::snprintf(name, sizeof name, "mix U=%lld", (long long)U);
      timeit(name, [&] { units<1><<<blocks, 256>>>(out, U, 0); });
    }
    for (int64_t U : {4096LL, 8192LL, 16384LL, 65536LL, 262144LL}) {
      for (int s = 0; s < 8; s += (U == 4096 ? 1 : 4)) {
        std::snprintf(name, sizeof name, "aff U=%lld s=%d", (long long)U, s);
        timeit(name, [&] { big_units<<<blocks, 256>>>(out, U, 0, s, nullptr); });
      }
      std::snprintf(name, sizeof name, "mix U=%lld", (long long)U);
      timeit(name, [&] { big_units<<<blocks, 256>>>(out, U, 1, 0, nullptr); });
    }
  }
  CK(hipFree(out));
  CK(hipFree(xlog));
  return 0;
}
