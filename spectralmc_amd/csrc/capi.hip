// C-ABI housekeeping of libspectralmc_hip.so: ABI version, per-thread error text, launch timing, the sync-area
// status word of the exchanging launches, and the exchange-fault test hook (spectralmc_hip_testing.h).
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "../../include/spectralmc_hip_testing.h"
#include "smc_internal.h"

namespace smc {
namespace {
thread_local char g_last_error[512] = "";
std::atomic<int32_t> g_fault_withhold{0};
std::atomic<uint32_t> g_fault_spin_limit{0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

ExchangeFault exchange_fault() { return ExchangeFault{g_fault_withhold.load(), g_fault_spin_limit.load()}; }

LaunchTiming& launch_timing() {
  thread_local LaunchTiming t{nullptr, nullptr};
  return t;
}

}  // namespace smc

extern "C" {
#pragma GCC visibility push(default)

int32_t smc_abi_version(void) { return SMC_ABI_VERSION; }

const char* smc_last_error_string(void) { return smc::g_last_error; }

int32_t smc_time_launches(void* start_event, void* stop_event) {
  smc::launch_timing() = smc::LaunchTiming{static_cast<hipEvent_t>(start_event), static_cast<hipEvent_t>(stop_event)};
  return SMC_OK;
}

int32_t smc_sync_status(void* sync_dev, int32_t clear, int32_t* status_out, void* stream) {
  if (!sync_dev || !status_out) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_sync_status: NULL pointer");
  const hipStream_t s = smc::as_stream(stream);
  uint32_t word = 0;
  char* w = static_cast<char*>(sync_dev) + SMC_SYNC_STATUS_OFFSET;
  if (hipMemcpyAsync(&word, w, sizeof(word), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    const hipError_t e = hipGetLastError();
    smc::set_error("smc_sync_status: %s", hipGetErrorString(e));
    return SMC_ERR_HIP;
  }
  if (clear && word != 0u && (hipMemsetAsync(w, 0, sizeof(word), s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)) {
    const hipError_t e = hipGetLastError();
    smc::set_error("smc_sync_status: %s", hipGetErrorString(e));
    return SMC_ERR_HIP;
  }
  *status_out = static_cast<int32_t>(word);
  return SMC_OK;
}

// spectralmc_hip_testing.h: inert unless SMC_ENABLE_TEST_HOOKS=1 (read once, at the first call)
int32_t smc_test_exchange_fault(int32_t withhold, uint32_t spin_limit) {
  static const bool enabled = [] {
    const char* e = getenv("SMC_ENABLE_TEST_HOOKS");
    return e != nullptr && e[0] == '1' && e[1] == '\0';
  }();
  if (!enabled)
    return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_test_exchange_fault: test hooks disabled (SMC_ENABLE_TEST_HOOKS=1)");
  if (withhold != 0 && withhold != 1) return smc::fail(SMC_ERR_INVALID_ARGUMENT, "smc_test_exchange_fault: withhold");
  smc::g_fault_withhold.store(withhold);
  smc::g_fault_spin_limit.store(spin_limit);
  return SMC_OK;
}

#pragma GCC visibility pop
}  // extern "C"
