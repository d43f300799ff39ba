// Internal helpers shared by the translation units of libspectralmc_hip.so.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/spectralmc_hip.h"

namespace smc {

// Thread-local text of the last failure (smc_last_error_string).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

inline int32_t fail(int32_t code, const char* what) {
  set_error("%s", what);
  return code;
}

// Map the launch status of the kernel just enqueued to a status code.
inline int32_t check_launch(const char* kernel) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", kernel, hipGetErrorString(e));
    return SMC_ERR_HIP;
  }
  return SMC_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel timing (smc_time_launches): while armed, the engine's launches go through hipExtLaunchKernel with
// these events: the first records `start` at its own start, every one records `stop` at its own end (after
// the call: the last one's).  Those are the kernels' execution timestamps, as a kernel trace takes them,
// without the dispatch gaps a pair of stream events around back-to-back launches also holds.
struct LaunchTiming {
  hipEvent_t start;
  hipEvent_t stop;
};
LaunchTiming& launch_timing();  // thread-local (capi.hip)
template <typename F, typename... Args>
inline void launch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t stream, Args... args) {
  LaunchTiming& t = launch_timing();
  if (t.start || t.stop) {
    hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, t.start, t.stop, 0u, args...);
    t.start = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
  }
}
// An auxiliary kernel of an engine call (Sobol draw, cursor update, normalisation, normals): never timed by
// smc_time_launches, so the armed pair spans the path / CF kernels the roofline is quoted on.
template <typename F, typename... Args>
inline void launch_aux(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t stream, Args... args) {
  hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
}

// CUs a (CU-masked) stream may use, out of `cus` (hipExtStreamCreateWithCUMask streams: the popcount of the
// mask; other streams: all).  Persistent launches size their grids to it, so every workgroup is resident.
inline int stream_cus(hipStream_t stream, int cus) {
  if (!stream) return cus;
  uint32_t mask[16] = {};
  if (hipExtStreamGetCUMask(stream, 16, mask) != hipSuccess) {
    (void)hipGetLastError();
    return cus;
  }
  int n = 0;
  for (int i = 0; i < 16 && i * 32 < cus; ++i) n += __builtin_popcount(mask[i]);
  return n > 0 && n < cus ? n : cus;
}

// Polls of an inter-workgroup exchange before it gives up (~1 s of s_sleep(2) polling); the
// exchange then sets SMC_SYNC_EXCHANGE_TIMEOUT in the sync area's status word and writes NaN
// targets for the contracts it could not finish.
constexpr uint32_t kExchangeSpinLimit = 1u << 20;

// Test hook (smc_test_exchange_fault): applied by the host to the next exchanging launches.
struct ExchangeFault {
  int32_t withhold;     // 1: slice W-1 of group 0 skips its first arrival
  uint32_t spin_limit;  // polls before an exchange gives up (0: kExchangeSpinLimit)
};
ExchangeFault exchange_fault();
inline uint32_t exchange_spin_limit() {
  const uint32_t l = exchange_fault().spin_limit;
  return l ? l : kExchangeSpinLimit;
}

}  // namespace smc

// Opaque Sobol handle (smc_sobol_*).
struct smc_sobol {
  int32_t dim;
  uint64_t cursor;        // index of the next point of the host-side stream
  uint32_t shift[64];     // digital shift, one 30-bit word per dimension
  uint32_t sv[64 * 30];   // LMS-scrambled direction numbers [dim][30]
};
