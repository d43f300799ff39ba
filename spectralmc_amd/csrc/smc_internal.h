// Internal helpers shared by the translation units of libspectralmc_hip.so.
#pragma once

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

}  // namespace smc

// Opaque Sobol handle (smc_sobol_*).
struct smc_sobol {
  int32_t dim;
  uint64_t cursor;        // index of the next point of the host-side stream
  uint32_t shift[64];     // digital shift, one 30-bit word per dimension
  uint32_t sv[64 * 30];   // LMS-scrambled direction numbers [dim][30]
};
