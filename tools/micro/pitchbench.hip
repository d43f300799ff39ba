// Store-pattern probe: the contract kernel's write order ([B][T][pitch], 2048-path chunks,
// 16 rows per chunk, float4 per lane) at several row pitches / row-block depths.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int B = 4096, T = 16;
constexpr int64_t P = 65536;

template <int ROWS>
__global__ __launch_bounds__(512) void rows_chunked(float* out, int64_t pitch) {
  const int64_t b = blockIdx.x;
  float* base = out + b * T * pitch;
  for (int t0 = 0; t0 < T; t0 += ROWS)
    for (int64_t chunk = 0; chunk < P; chunk += 2048) {
      float4 v = make_float4(1.f, 2.f, 3.f, (float)chunk);
#pragma unroll
      for (int t = 0; t < ROWS; ++t) {
        reinterpret_cast<float4*>(base + (t0 + t) * pitch + chunk)[threadIdx.x] = v;
        v.x += 1.f;
      }
    }
}

int main() {
  const int64_t max_pitch = P + 4096;
  float* out;
  if (hipMalloc(&out, (size_t)B * T * max_pitch * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = (double)B * T * P * 4;
  for (int64_t pad : {0, 64, 256, 1024, 4096}) {
    for (int rows : {16, 8, 4}) {
      auto launch = [&] {
        if (rows == 16) rows_chunked<16><<<B, 512>>>(out, P + pad);
        else if (rows == 8) rows_chunked<8><<<B, 512>>>(out, P + pad);
        else rows_chunked<4><<<B, 512>>>(out, P + pad);
      };
      launch(); launch();
      (void)hipEventRecord(e0);
      for (int i = 0; i < 10; ++i) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
      printf("pad %5lld floats  rows/pass %2d : %.3f ms  %.0f GB/s\n", (long long)pad, rows, ms, bytes / (ms * 1e6));
    }
  }
  if (hipGetLastError() != hipSuccess) { printf("kernel error\n"); return 1; }
  return 0;
}
