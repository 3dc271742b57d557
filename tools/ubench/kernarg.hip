// Large by-value kernel arguments on MI355X: does a 6-12 KB struct arrive
// intact, and what does its launch cost against a pointer argument plus a
// copy kernel reading pinned host memory (the grid chain's k_chain_prep)?
//   hipcc --offload-arch=gfx950 -O2 kernarg.hip -o /tmp/kernarg && /tmp/kernarg
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int W>
struct Desc { unsigned w[W]; };

template <int W>
__global__ void k_arg(Desc<W> d, unsigned* out, unsigned* flag, unsigned seq) {
  __shared__ unsigned s[W];
  const unsigned* p = d.w;
  for (int i = threadIdx.x; i < W; i += blockDim.x) s[i] = p[i];
  __syncthreads();
  unsigned acc = 0;
  for (int i = threadIdx.x; i < W; i += blockDim.x) acc += s[i] * (i + 1);
  atomicAdd(&out[blockIdx.x & 7], acc);
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int W>
__global__ void k_ptr(const unsigned* d, unsigned* out, unsigned* flag, unsigned seq) {
  __shared__ unsigned s[W];
  for (int i = threadIdx.x; i < W; i += blockDim.x) s[i] = d[i];
  __syncthreads();
  unsigned acc = 0;
  for (int i = threadIdx.x; i < W; i += blockDim.x) acc += s[i] * (i + 1);
  atomicAdd(&out[blockIdx.x & 7], acc);
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_copy(const unsigned* h, unsigned* d, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = h[i];
}

template <int W>
int run() {
  Desc<W> d;
  for (int i = 0; i < W; ++i) d.w[i] = 0x9e3779b9u * (i + 1);
  unsigned want = 0;
  for (int i = 0; i < W; ++i) want += d.w[i] * (i + 1);
  unsigned *out, *flag, *hd, *dd;
  CK(hipMalloc(&out, 64));
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&hd, sizeof(d), hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipMalloc(&dd, sizeof(d)));
  std::memcpy(hd, &d, sizeof(d));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int G = 256, reps = 400;
  double t_arg = 0, t_ptr = 0;
  unsigned seq = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemsetAsync(out, 0, 64, s));
    CK(hipStreamSynchronize(s));
    ++seq;
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_arg<W>, dim3(G), dim3(256), 0, s, d, out, flag, seq);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {}
    auto t1 = std::chrono::steady_clock::now();
    if (r >= 50) t_arg += std::chrono::duration<double, std::micro>(t1 - t0).count();
    CK(hipStreamSynchronize(s));
    unsigned o[8];
    CK(hipMemcpy(o, out, 32, hipMemcpyDeviceToHost));
    unsigned tot = 0;
    for (int k = 0; k < 8; ++k) tot += o[k];
    if (tot != want * (unsigned)G) { std::printf("W=%d by-value argument corrupted (rep %d)\n", W, r); return 1; }
    CK(hipMemsetAsync(out, 0, 64, s));
    CK(hipStreamSynchronize(s));
    ++seq;
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, s, (const unsigned*)hd, dd, W);
    hipLaunchKernelGGL(k_ptr<W>, dim3(G), dim3(256), 0, s, (const unsigned*)dd, out, flag, seq);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {}
    t1 = std::chrono::steady_clock::now();
    if (r >= 50) t_ptr += std::chrono::duration<double, std::micro>(t1 - t0).count();
    CK(hipStreamSynchronize(s));
  }
  std::printf("W=%d words (%zu B): by-value launch->done %.1f us, copy kernel + pointer launch->done %.1f us\n", W,
              sizeof(d), t_arg / (reps - 50), t_ptr / (reps - 50));
  return 0;
}

int main() {
  if (run<256>() || run<1024>() || run<1536>() || run<3072>()) return 1;
  return 0;
}
