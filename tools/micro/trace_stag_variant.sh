#!/bin/bash
# Round 6 probe: trace_variant.sh plus a start stagger of (blockIdx / 8) x 5 us within each XCD.
# Builds tools/micro/v/libsmc_trace.so: resident_kernel with per-workgroup s_memrealtime stamps (kernel start, XCC id,
# end of every contract round, kernel end) in a device array read back by smc_trace_copy (tools/kprof_step.py --trace).
# No hooks in the product sources: make_variant.py applies literal edits to a scratch copy.
set -e
cd "$(dirname "$0")/../.."
python tools/micro/make_variant.py trace_stag \
  gbm.hip 'constexpr int kResThreads = 1024;' '__device__ unsigned long long g_trace[4096 * 40];
__device__ unsigned long long g_trace_key[16];
constexpr int kResThreads = 1024;' \
  gbm.hip '  static_assert(!(ONTHEFLY && T16), "the on-the-fly CF phase is instantiated for the rolled row loop only");' '  static_assert(!(ONTHEFLY && T16), "the on-the-fly CF phase is instantiated for the rolled row loop only");
  unsigned long long* tr = g_trace;
  if (threadIdx.x == 0) {
    // the launch: slot = first free / matching entry of g_trace_key for the kernarg address of this dispatch
    const unsigned long long key = reinterpret_cast<unsigned long long>(__builtin_amdgcn_kernarg_segment_ptr());
    int slot = 15;
    for (int k = 0; k < 16; ++k) {
      const unsigned long long old = atomicCAS(&g_trace_key[k], 0ull, key);
      if (old == 0ull || old == key) { slot = k; break; }
    }
    tr = g_trace + (slot * 256 + (blockIdx.x & 255)) * 40;  // 16 launches of <= 256 workgroups
    unsigned xcc_ = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));
    tr[0] = __builtin_amdgcn_s_memrealtime();
    tr[1] = xcc_;
    tr[36] = __builtin_amdgcn_s_memtime();  // shader-clock counter: the clock the workgroup ran at
  }
  {  // PROBE: workgroup start staggered within each XCD (blocks b, b + 8, ... share an XCD) by (b / 8) x 5 us
    const unsigned long long until = __builtin_amdgcn_s_memrealtime() + (blockIdx.x >> 3) * 500ull;
    while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
  }' \
  gbm.hip '    fft_row<float, kResThreads, true>(avg, cs, sn, N, part, part + N, static_cast<float2*>(a.targets) + b * N);
    lds_barrier();  // part (= term_lds) / avg / wsum / row are reused by the next contract' '    fft_row<float, kResThreads, true>(avg, cs, sn, N, part, part + N, static_cast<float2*>(a.targets) + b * N);
    lds_barrier();  // part (= term_lds) / avg / wsum / row are reused by the next contract
    if (tid == 0 && round < 34) tr[2 + round] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) tr[38] = round + 1;' \
  gbm.hip '  if (a.done && tid == 0) {
    // every workgroup read the cursor (and made its last exchange)' '  if (tid == 0) {
    tr[37] = __builtin_amdgcn_s_memtime();
    tr[39] = __builtin_amdgcn_s_memrealtime();
  }
  if (a.done && tid == 0) {
    // every workgroup read the cursor (and made its last exchange)' \
  gbm.hip '#pragma GCC visibility pop
}  // extern "C"' '__attribute__((visibility("default"))) int32_t smc_trace_copy(void* dst, int32_t clear) {
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(smc::g_trace), sizeof(smc::g_trace)) != hipSuccess) return 1;
  if (clear) {
    static unsigned long long zeros[4096 * 40];
    if (hipMemcpyToSymbol(HIP_SYMBOL(smc::g_trace), zeros, sizeof(zeros)) != hipSuccess) return 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(smc::g_trace_key), zeros, 16 * sizeof(unsigned long long)) != hipSuccess) return 1;
  }
  return 0;
}
#pragma GCC visibility pop
}  // extern "C"'
