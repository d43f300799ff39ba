// Companion of tools/probe_fill.py: the one-shot linear store kernel of storebench6.hip as a C entry
// point, so it writes into a torch-allocated buffer next to torch's own fill_ (same allocation, same
// process).  hipcc -O3 --offload-arch=gfx950 -shared -fPIC fillcmp.hip -o v/libfillcmp.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int VEC_PER_LANE>
__global__ __launch_bounds__(256) void lin(float* out, float x) {
  const v4f v = {x, x, x, x};
  float* p = out + static_cast<int64_t>(blockIdx.x) * (256 * 4 * VEC_PER_LANE);
#pragma unroll
  for (int k = 0; k < VEC_PER_LANE; ++k) *reinterpret_cast<v4f*>(p + (k * 256 + threadIdx.x) * 4) = v;
}

extern "C" int fillcmp_lin(float* out, int64_t n_floats, float x, int vec_per_lane, void* stream) {
  const int64_t per = 256 * 4 * static_cast<int64_t>(vec_per_lane);
  const unsigned grid = static_cast<unsigned>(n_floats / per);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (vec_per_lane == 1) hipLaunchKernelGGL(lin<1>, dim3(grid), dim3(256), 0, s, out, x);
  else if (vec_per_lane == 4) hipLaunchKernelGGL(lin<4>, dim3(grid), dim3(256), 0, s, out, x);
  else hipLaunchKernelGGL(lin<16>, dim3(grid), dim3(256), 0, s, out, x);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
