// Store-path microbenchmark: 3 column outputs of n u32 written with 4-byte
// vs 16-byte lanes, aligned vs offset, from registers (no loads).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void st4(uint32_t* out, uint64_t n, uint64_t cap, int ncol, uint64_t shift) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < ncol; ++c) out[c * cap + shift + i] = (uint32_t)i + c;
}
__global__ void st16(uint4* out, uint64_t n4, uint64_t cap4, int ncol) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < ncol; ++c) out[c * cap4 + i] = make_uint4(i, i + 1, i + 2, c);
}
// wave-chunked like k_dj_write: each wave owns segments of ~470 outputs at arbitrary offsets
__global__ void stseg(uint32_t* out, uint64_t units, uint64_t cap, int ncol, uint32_t per_unit) {
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const int lane = threadIdx.x & 63;
  for (uint64_t u = blockIdx.x * (uint64_t)(blockDim.x / 64) + (threadIdx.x >> 6); u < units; u += waves) {
    uint64_t base = u * per_unit;
    for (int g = 0; g < 4; ++g) {
      const uint32_t tot = per_unit / 4 + (g == 3 ? per_unit % 4 : 0);
      for (uint32_t o0 = 0; o0 < tot; o0 += 64) {
        const uint32_t o = o0 + lane;
        if (o < tot)
          for (int c = 0; c < ncol; ++c) out[c * cap + base + o] = o + c;
      }
      base += tot;
    }
  }
}

int main() {
  const uint64_t n = 25'000'000;
  uint32_t* out;
  hipMalloc(&out, 4 * 3 * (n + 1024));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto t = [&](const char* name, auto fn) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 100, 12.0 * n / (ms * 1e-4) / 1e9);
  };
  const uint64_t cap = n + 1024;
  t("st4 aligned", [&] { hipLaunchKernelGGL(st4, dim3(8192), dim3(256), 0, 0, out, n, cap, 3, 0ull); });
  t("st4 shift 7", [&] { hipLaunchKernelGGL(st4, dim3(8192), dim3(256), 0, 0, out, n, cap, 3, 7ull); });
  t("st4 grid 65535*4", [&] { hipLaunchKernelGGL(st4, dim3((n + 255) / 256), dim3(256), 0, 0, out, n, cap, 3, 0ull); });
  t("st16", [&] { hipLaunchKernelGGL(st16, dim3(8192), dim3(256), 0, 0, (uint4*)out, n / 4, cap / 4, 3); });
  t("stseg 470/unit", [&] { hipLaunchKernelGGL(stseg, dim3(13184), dim3(256), 0, 0, out, n / 470, cap, 3, 470u); });
  t("stseg 512/unit", [&] { hipLaunchKernelGGL(stseg, dim3(12207), dim3(256), 0, 0, out, n / 512, cap, 3, 512u); });
  return 0;
}
