// FETCH_SIZE calibration for the access patterns of the query kernels
// (tools/pmc_traffic.py): each kernel reads a known number of distinct bytes
// from a 2 GiB table (well past the 256 MiB Infinity Cache), so
// FETCH_SIZE / known bytes gives the counter's factor for that pattern.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/fetch_cal tools/ubench/fetch_cal.hip
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -- tools/ubench/fetch_cal
//
//   k_stream16   16 B per lane, coalesced             : N bytes
//   k_rand_line  one 4-B load per 128-B line, random  : N / 32 loads, N bytes of lines
//   k_rand_half  one 4-B load per 64-B half line      : N / 16 loads, N bytes of lines
//   k_rand_word  4-B loads at random words, 1 per 512 B: N / 128 loads (distinct lines)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void k_stream16(const uint4* __restrict__ a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// element index of access i: a bijective scramble of the unit index (odd
// multiplier modulo a power of two) times the unit stride in words
__global__ void k_rand(const uint32_t* __restrict__ a, uint64_t units, uint32_t stride_words, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < units; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t u = (i * 0x9E3779B97F4A7C15ull) & (units - 1);
    acc ^= a[u * stride_words];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t N = 2ull << 30;   // bytes
  uint32_t* a = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&a, N));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(a, 1, N));
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream16, dim3(8192), dim3(256), 0, 0, (const uint4*)a, N / 16, out);
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, N / 128, 32u, out);   // per 128-B line
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, N / 64, 16u, out);    // per 64-B half line
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, N / 512, 128u, out);  // sparse words
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("bytes %llu: stream16 reads N; rand(stride 32 w) N; rand(stride 16 w) N; rand(stride 128 w) N/4 of lines\n",
              (unsigned long long)N);
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
