// Store-pattern probe 2 of the row pitch: the C2 contract kernel's write order ([B][T][pitch],
// 2048-path chunks, 16 rows per chunk, dwordx4 per lane) for row pads 0..8192 floats in 1 KiB
// steps and an extra per-contract pad.   hipcc -O3 --offload-arch=gfx950 pitchbench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536;

__global__ __launch_bounds__(512) void rows16(float* out, int64_t pitch, int64_t cpad) {
  const int64_t b = blockIdx.x;
  float* base = out + b * (T * pitch + cpad);
  for (int64_t chunk = 0; chunk < P; chunk += 2048) {
    float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      reinterpret_cast<float4*>(base + t * pitch + chunk)[threadIdx.x] = v;
      v.x += 1.f;
    }
  }
}

int main() {
  const int64_t max_pitch = P + 8192, max_cpad = 8192;
  float* out;
  if (hipMalloc(&out, (size_t)B * (T * max_pitch + max_cpad) * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = (double)B * T * P * 4;
  for (int64_t cpad : {0, 1024, 4096}) {
    for (int64_t pad = 0; pad <= 8192; pad += 256) {
      auto launch = [&] { rows16<<<B, 512>>>(out, P + pad, cpad); };
      launch();
      (void)hipEventRecord(e0);
      for (int i = 0; i < 8; ++i) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 8;
      printf("cpad %5lld pad %5lld floats (%3lld KiB units of row %lld): %.3f ms  %.0f GB/s\n", (long long)cpad,
             (long long)pad, (long long)((P + pad) / 256), (long long)(P + pad), ms, bytes / (ms * 1e6));
    }
  }
  if (hipGetLastError() != hipSuccess) { printf("kernel error\n"); return 1; }
  return 0;
}
