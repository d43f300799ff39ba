// Device-side scrambled Sobol coordinate shared by sobol_draw_kernel (sobol.hip) and the fused
// training step (gbm.hip): point n, dimension d of the table image smc_sobol_export_tables
// writes (tables[0..dim) = digital shift, tables[dim + d*30 + c] = LMS-scrambled direction
// numbers), scaled as numpy does in sobol_sampler.py:239: lower + (upper - lower) * raw with
// separately rounded f64 operations.
#pragma once

#include <cstdint>

namespace smc {

__device__ __forceinline__ double sobol_coord(const uint32_t* __restrict__ tables, int dim, int d, uint64_t n,
                                              const double* __restrict__ lower, const double* __restrict__ upper) {
#pragma clang fp contract(off)  // numpy rounds the product and the sum separately, wherever this is included
  const uint64_t g = n ^ (n >> 1);
  const uint32_t* svd = tables + dim + d * SMC_SOBOL_BITS;
  uint32_t x = tables[d];
#pragma unroll
  for (int c = 0; c < SMC_SOBOL_BITS; ++c) x ^= ((g >> c) & 1u) ? svd[c] : 0u;
  const double raw = static_cast<double>(x) * 0x1p-30;
  const double span = upper[d] - lower[d];
  const double prod = span * raw;
  return lower[d] + prod;
}

}  // namespace smc
