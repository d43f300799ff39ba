/*
 * spectralmc_hip_testing.h — test-only entry points of libspectralmc_hip.so (not part of the product
 * ABI in spectralmc_hip.h; no reference seam).
 *
 * They are inert unless the process environment holds SMC_ENABLE_TEST_HOOKS=1 when the first of them is
 * called (tests/conftest.py sets it); otherwise they change nothing and return SMC_ERR_INVALID_ARGUMENT.
 */
#ifndef SPECTRALMC_HIP_TESTING_H
#define SPECTRALMC_HIP_TESTING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Exchange fault injection (tests/test_gpu_engine.py, tests/test_gpu_basket.py): for the exchanging
 * launches enqueued after this call, withhold = 1 makes slice W-1 of group 0 skip its first arrival (its
 * partners time out), and spin_limit (> 0) replaces the ~1 s poll budget.  (0, 0) restores normal
 * operation. */
int32_t smc_test_exchange_fault(int32_t withhold, uint32_t spin_limit);

#ifdef __cplusplus
}
#endif

#endif /* SPECTRALMC_HIP_TESTING_H */
