// VALU throughput probe: cycles per wave-instruction per SIMD for the instruction kinds the path
// kernel's inner block is made of, at the path kernel's occupancy (1024-thread workgroups, one per
// CU = 4 waves per SIMD).  Each variant runs 8 independent register chains of one instruction kind
// (or a fixed mix); the cycle count is the wave's own s_memtime span over the loop.
//   hipcc -O3 --offload-arch=gfx950 valurate.hip -o valurate && ./valurate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 2048;

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ __launch_bounds__(1024) void probe(uint32_t* sink, uint64_t* cyc) {
  uint32_t v0 = threadIdx.x, v1 = v0 * 3 + 1, v2 = v0 * 5 + 2, v3 = v0 * 7 + 3, v4 = v0 ^ 0x55, v5 = v0 + 99,
           v6 = v0 * 11, v7 = v0 * 13 + 5;
  uint64_t d0 = v0, d1 = v1, d2 = v2, d3 = v3, d4 = v4, d5 = v5, d6 = v6, d7 = v7, e2 = v2 * 17ull, e3 = v3 * 19ull;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < kIters; ++it) {
#define ONE(i)                                                                                        \
  if constexpr (K == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v##i) : "v"(v0));                  \
  if constexpr (K == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v##i) : "v"(v1), "v"(v2)); \
  if constexpr (K == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v##i) : "v"(v1), "v"(v2));     \
  if constexpr (K == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(v##i));                                \
  if constexpr (K == 4) asm volatile("v_sin_f32 %0, %0" : "+v"(v##i));                                \
  if constexpr (K == 5) asm volatile("v_sqrt_f32 %0, %0" : "+v"(v##i));                               \
  if constexpr (K == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v##i) : "v"(v1));               \
  if constexpr (K == 7) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v##i) : "v"(v1));              \
  if constexpr (K == 8) asm volatile("v_mad_u32_u16 %0, %0, %1, %2" : "+v"(v##i) : "v"(v1), "v"(v2)); \
  if constexpr (K == 9) asm volatile("v_alignbit_b32 %0, %0, %1, 9" : "+v"(v##i) : "v"(v1));          \
  if constexpr (K == 10) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(v##i) : "v"(v1), "v"(v2));   \
  if constexpr (K == 11) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(v##i));                           \
  if constexpr (K == 12) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v##i) : "v"(v1));              \
  if constexpr (K == 13) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v##i) : "v"(v1));              \
  if constexpr (K == 14) asm volatile("v_log_f32 %0, %0" : "+v"(v##i));                               \
  if constexpr (K == 15) { /* 1 exp + 3 plain */                                                       \
    asm volatile("v_exp_f32 %0, %0" : "+v"(v##i));                                                    \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(v1) : "v"(v0));                                        \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(v2) : "v"(v0));                                        \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(v3) : "v"(v0));                                        \
  }                                                                                                   \
  if constexpr (K == 16) { /* 1 exp + 1 plain */                                                       \
    asm volatile("v_exp_f32 %0, %0" : "+v"(v##i));                                                    \
    asm volatile("v_add_u32 %0, %0, %1" : "+v"(v1) : "v"(v0));                                        \
  }                                                                                                   \
  if constexpr (K == 17) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d##i) : "v"(e2), "v"(e3)); \
  if constexpr (K == 18) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d##i) : "v"(e2));           \
  if constexpr (K == 19) asm volatile("v_lshlrev_b64 %0, 9, %0" : "+v"(d##i));                    \
  if constexpr (K == 20) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(d##i) : "v"(v1), "v"(v2) : "vcc"); \
  if constexpr (K == 21) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(d##i) : "v"(e2));    \
  if constexpr (K == 22) asm volatile("v_cvt_f32_ubyte1 %0, %0" : "+v"(v##i));                        \
  if constexpr (K == 23) asm volatile("v_pk_fma_f16 %0, %0, %1, %2" : "+v"(v##i) : "v"(v1), "v"(v2)); \
  if constexpr (K == 24) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v##i) : "v"(v1));                 \
  if constexpr (K == 25) asm volatile("v_lshlrev_b32 %0, 9, %0" : "+v"(v##i));                        \
  if constexpr (K == 26) asm volatile("v_rcp_f32 %0, %0" : "+v"(v##i));                               \
  if constexpr (K == 27) asm volatile("v_exp_f16 %0, %0" : "+v"(v##i));                               \
  if constexpr (K == 28) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(v##i) : "v"(v1), "v"(v2)); \
  if constexpr (K == 29) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d##i) : "v"(e2), "v"(e3));   \
  if constexpr (K == 30) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d##i) : "v"(e2));                \
  if constexpr (K == 31) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d##i) : "v"(v1));              \
  if constexpr (K == 32) asm volatile("v_rndne_f64 %0, %0" : "+v"(d##i));                            \
  if constexpr (K == 33) asm volatile("v_rcp_f64 %0, %0" : "+v"(d##i));                              \
  if constexpr (K == 34) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d##i) : "v"(e2));
    R8(ONE) R8(ONE) R8(ONE) R8(ONE)
#undef ONE
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * 1024 + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7 ^ static_cast<uint32_t>(d0 ^ d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7);
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int K>
void run(const char* name, uint32_t* sink, uint64_t* cyc, uint64_t* host, int cus) {
  hipLaunchKernelGGL(probe<K>, dim3(cus), dim3(1024), 0, 0, sink, cyc);  // warm
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<K>, dim3(cus), dim3(1024), 0, 0, sink, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(host, cyc, sizeof(uint64_t) * cus * 16, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < cus * 16; ++i) s += host[i];
  s /= cus * 16;
  const double insts = static_cast<double>(kIters) * 32;  // instructions (or mix groups) per wave
  // 4 waves per SIMD share it: SIMD cycles per wave-instruction = span / (4 * insts)
  std::printf("%-22s %8.3f ms  span %10.0f cyc  %6.2f cyc/inst/SIMD  (clock %.2f GHz)\n", name, ms, s,
              s / (4 * insts), s / (ms * 1e6));
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* sink;
  uint64_t* cyc;
  hipMalloc(&sink, sizeof(uint32_t) * cus * 1024);
  hipMalloc(&cyc, sizeof(uint64_t) * cus * 16);
  static uint64_t host[4096];
  std::printf("CUs %d, 1024-thread workgroups (4 waves/SIMD)\n", cus);
  run<0>("v_add_u32", sink, cyc, host, cus);
  run<1>("v_bitop3_b32", sink, cyc, host, cus);
  run<24>("v_xor_b32", sink, cyc, host, cus);
  run<25>("v_lshlrev_b32", sink, cyc, host, cus);
  run<9>("v_alignbit_b32", sink, cyc, host, cus);
  run<10>("v_perm_b32", sink, cyc, host, cus);
  run<2>("v_fma_f32", sink, cyc, host, cus);
  run<17>("v_pk_fma_f32", sink, cyc, host, cus);
  run<18>("v_pk_mul_f32", sink, cyc, host, cus);
  run<23>("v_pk_fma_f16", sink, cyc, host, cus);
  run<12>("v_pk_add_u16", sink, cyc, host, cus);
  run<3>("v_exp_f32", sink, cyc, host, cus);
  run<14>("v_log_f32", sink, cyc, host, cus);
  run<4>("v_sin_f32", sink, cyc, host, cus);
  run<5>("v_sqrt_f32", sink, cyc, host, cus);
  run<26>("v_rcp_f32", sink, cyc, host, cus);
  run<27>("v_exp_f16", sink, cyc, host, cus);
  run<15>("exp+3add (per group)", sink, cyc, host, cus);
  run<16>("exp+1add (per group)", sink, cyc, host, cus);
  run<6>("v_mul_lo_u32", sink, cyc, host, cus);
  run<13>("v_mul_hi_u32", sink, cyc, host, cus);
  run<7>("v_mul_u32_u24", sink, cyc, host, cus);
  run<28>("v_mad_u32_u24", sink, cyc, host, cus);
  run<8>("v_mad_u32_u16", sink, cyc, host, cus);
  run<20>("v_mad_u64_u32", sink, cyc, host, cus);
  run<19>("v_lshlrev_b64", sink, cyc, host, cus);
  run<21>("v_lshl_add_u64", sink, cyc, host, cus);
  run<11>("v_cvt_f32_u32", sink, cyc, host, cus);
  run<29>("v_fma_f64", sink, cyc, host, cus);
  run<30>("v_mul_f64", sink, cyc, host, cus);
  run<34>("v_add_f64", sink, cyc, host, cus);
  run<31>("v_ldexp_f64", sink, cyc, host, cus);
  run<32>("v_rndne_f64", sink, cyc, host, cus);
  run<33>("v_rcp_f64", sink, cyc, host, cus);
  run<22>("v_cvt_f32_ubyte1", sink, cyc, host, cus);
  return 0;
}
