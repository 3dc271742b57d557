// Cartesian-product expansion variants (k_cartesian): output row o =
// (probe row o / nb, build row o % nb), NC column-major u32 output columns,
// the first NP from the probe side.  Prints GB/s of output written.
//   hipcc -O3 --offload-arch=gfx950 cart_bw.hip -o cart_bw && ./cart_bw [np nb]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int NC = 6, NP = 3;
struct Cols { const uint32_t* c[NC]; };

// A: one output per thread per grid stride, 4-byte stores (the round-3 kernel)
__global__ void __launch_bounds__(256) cart_a(Cols cs, uint64_t nb, uint64_t total, uint64_t sq, uint64_t sr,
                                              uint32_t* out, uint64_t cap) {
  uint64_t o = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (o >= total) return;
  uint64_t i = o / nb, j = o - i * nb;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; o < total; o += stride) {
#pragma unroll
    for (int c = 0; c < NC; ++c) out[(uint64_t)c * cap + o] = c < NP ? cs.c[c][i] : cs.c[c][j];
    i += sq;
    j += sr;
    if (j >= nb) { j -= nb; ++i; }
  }
}

// B: four consecutive outputs per thread, one 16-byte store per column
template <bool NT>
__global__ void __launch_bounds__(256) cart_b(Cols cs, uint64_t nb, uint64_t total, uint64_t sq, uint64_t sr,
                                              uint32_t* out, uint64_t cap) {
  uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;   // quad index
  const uint64_t nq = (total + 3) / 4;
  if (q >= nq) return;
  uint64_t o = 4 * q;
  uint64_t i = o / nb, j = o - i * nb;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; q < nq; q += stride) {
    uint32_t v[NC][4];
    uint64_t ii = i, jj = j;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = 4 * q + k < total;
#pragma unroll
      for (int c = 0; c < NC; ++c) v[c][k] = ok ? (c < NP ? cs.c[c][ii] : cs.c[c][jj]) : 0u;
      if (++jj == nb) { jj = 0; ++ii; }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      v4u w = v4u{v[c][0], v[c][1], v[c][2], v[c][3]};
      v4u* p = (v4u*)(out + (uint64_t)c * cap) + q;
      if (NT) __builtin_nontemporal_store(w, p);
      else *p = w;
    }
    i += sq;
    j += sr;
    while (j >= nb) { j -= nb; ++i; }
  }
}

// C: a block writes a contiguous tile of T outputs column by column
template <int T>
__global__ void __launch_bounds__(256) cart_c(Cols cs, uint64_t nb, uint64_t total, uint32_t* out, uint64_t cap) {
  for (uint64_t t0 = blockIdx.x * (uint64_t)T; t0 < total; t0 += (uint64_t)gridDim.x * T) {
    const uint64_t i0 = t0 / nb, j0 = t0 - i0 * nb;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      uint32_t* oc = out + (uint64_t)c * cap;
      for (uint32_t k = threadIdx.x; k < T; k += 256) {
        const uint64_t o = t0 + k;
        if (o >= total) break;
        uint64_t jj = j0 + k, ii = i0;
        while (jj >= nb) { jj -= nb; ++ii; }
        oc[o] = c < NP ? cs.c[c][ii] : cs.c[c][jj];
      }
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t np = argc > 1 ? strtoull(argv[1], 0, 10) : 272048;
  const uint64_t nb = argc > 2 ? strtoull(argv[2], 0, 10) : 1000;
  const uint64_t total = np * nb, cap = (total + 63) / 64 * 64;
  Cols cs;
  for (int c = 0; c < NC; ++c) {
    uint32_t* p;
    const uint64_t n = c < NP ? np : nb;
    CK(hipMalloc(&p, 4 * n));
    CK(hipMemset(p, c, 4 * n));
    cs.c[c] = p;
  }
  uint32_t* out;
  CK(hipMalloc(&out, 4 * NC * cap));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto t = [&](const char* name, auto fn) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f us  %7.1f GB/s\n", name, ms * 200, 4.0 * NC * total / (ms * 2e-4) / 1e9);
  };
  printf("np %llu nb %llu total %llu cols %d (%.2f GB)\n", (unsigned long long)np, (unsigned long long)nb,
         (unsigned long long)total, NC, 4.0 * NC * total / 1e9);
  for (unsigned g : {524280u, 65536u, 16384u, 4096u}) {
    const uint64_t S = (uint64_t)g * 256;
    const unsigned gg = (unsigned)std::min<uint64_t>(g, (total + 255) / 256);
    char nm[64];
    snprintf(nm, 64, "A 4B g=%u", gg);
    const uint64_t SA = (uint64_t)gg * 256;
    t(nm, [&] { hipLaunchKernelGGL(cart_a, dim3(gg), dim3(256), 0, 0, cs, nb, total, SA / nb, SA % nb, out, cap); });
    const unsigned gq = (unsigned)std::min<uint64_t>(g, ((total + 3) / 4 + 255) / 256);
    const uint64_t SQ = (uint64_t)gq * 256 * 4;
    snprintf(nm, 64, "B 16B g=%u", gq);
    t(nm, [&] { hipLaunchKernelGGL(cart_b<false>, dim3(gq), dim3(256), 0, 0, cs, nb, total, SQ / nb, SQ % nb, out, cap); });
    snprintf(nm, 64, "B 16B NT g=%u", gq);
    t(nm, [&] { hipLaunchKernelGGL(cart_b<true>, dim3(gq), dim3(256), 0, 0, cs, nb, total, SQ / nb, SQ % nb, out, cap); });
    (void)S;
  }
  for (unsigned g : {16384u, 4096u}) {
    char nm[64];
    snprintf(nm, 64, "C tile4096 g=%u", g);
    t(nm, [&] { hipLaunchKernelGGL(cart_c<4096>, dim3(g), dim3(256), 0, 0, cs, nb, total, out, cap); });
  }
  return 0;
}
