// C-ABI housekeeping of libspectralmc_hip.so: ABI version and per-thread error text.
#include <cstdarg>
#include <cstdio>

#include "smc_internal.h"

namespace smc {
namespace {
thread_local char g_last_error[512] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

}  // namespace smc

extern "C" {
#pragma GCC visibility push(default)

int32_t smc_abi_version(void) { return SMC_ABI_VERSION; }

const char* smc_last_error_string(void) { return smc::g_last_error; }

#pragma GCC visibility pop
}  // extern "C"
