// Copy / read / write bandwidth ceilings on MI355X for the projection and
// join-expansion kernels: 16-byte lanes, grid-stride vs unrolled, plain vs
// nontemporal stores.  Prints GB/s (bytes read + written) per variant.
//   hipcc -O3 --offload-arch=gfx950 copy_bw.hip -o copy_bw && ./copy_bw
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy_gs(const v4u* __restrict__ s, v4u* __restrict__ d, uint64_t n4) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

template <int U, bool NT>
__global__ void copy_unroll(const v4u* __restrict__ s, v4u* __restrict__ d, uint64_t n4) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], &d[i + u * stride]);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n4; i += stride) d[i] = s[i];
}

// contiguous tile per block (each block copies a run of 256*U*16 bytes)
template <int U, bool NT>
__global__ void copy_tile(const v4u* __restrict__ s, v4u* __restrict__ d, uint64_t n4) {
  const uint64_t tile = (uint64_t)blockDim.x * U;
  for (uint64_t t0 = blockIdx.x * tile; t0 < n4; t0 += (uint64_t)gridDim.x * tile) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = t0 + u * blockDim.x + threadIdx.x;
      if (i < n4) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = t0 + u * blockDim.x + threadIdx.x;
      if (i < n4) {
        if (NT) __builtin_nontemporal_store(v[u], &d[i]);
        else d[i] = v[u];
      }
    }
  }
}

template <bool NT>
__global__ void write_only(v4u* __restrict__ d, uint64_t n4) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = v4u{(uint32_t)i, 1u, 2u, 3u};
    if (NT) __builtin_nontemporal_store(v, &d[i]);
    else d[i] = v;
  }
}

__global__ void read_only(const v4u* __restrict__ s, uint64_t n4, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = s[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 2048ull) << 20;   // MiB per buffer
  const uint64_t n4 = bytes / 16;
  v4u *s, *d;
  uint32_t* sink;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(s, 1, bytes));
  CK(hipMemset(d, 0, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, double traffic, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-28s %8.1f GB/s\n", name, traffic * reps / (ms * 1e-3) / 1e9);
    return 0;
  };
  for (unsigned grid : {1024u, 2048u, 4096u, 16384u}) {
    char nm[64];
    snprintf(nm, 64, "copy grid-stride g=%u", grid);
    run(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL(copy_gs, dim3(grid), dim3(256), 0, 0, s, d, n4); });
    snprintf(nm, 64, "copy unroll4 g=%u", grid);
    run(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_unroll<4, false>), dim3(grid), dim3(256), 0, 0, s, d, n4); });
    snprintf(nm, 64, "copy unroll4 NT g=%u", grid);
    run(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_unroll<4, true>), dim3(grid), dim3(256), 0, 0, s, d, n4); });
    snprintf(nm, 64, "copy tile8 g=%u", grid);
    run(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_tile<8, false>), dim3(grid), dim3(256), 0, 0, s, d, n4); });
    snprintf(nm, 64, "copy tile8 NT g=%u", grid);
    run(nm, 2.0 * bytes, [&] { hipLaunchKernelGGL((copy_tile<8, true>), dim3(grid), dim3(256), 0, 0, s, d, n4); });
    snprintf(nm, 64, "write g=%u", grid);
    run(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((write_only<false>), dim3(grid), dim3(256), 0, 0, d, n4); });
    snprintf(nm, 64, "write NT g=%u", grid);
    run(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL((write_only<true>), dim3(grid), dim3(256), 0, 0, d, n4); });
    snprintf(nm, 64, "read g=%u", grid);
    run(nm, 1.0 * bytes, [&] { hipLaunchKernelGGL(read_only, dim3(grid), dim3(256), 0, 0, s, n4, sink); });
  }
  // hipMemcpy D2D for reference
  run("hipMemcpyAsync D2D", 2.0 * bytes, [&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
  return 0;
}
