// Probe-kernel ablation: the structure of das k_dj_write (wave units of 4 x 64
// probe rows, bucket gathers, per-chunk owner search, 3 output columns),
// with stages switched on one at a time.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>


template <typename T>
__device__ __forceinline__ T wscan(T x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    T y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}
__device__ __forceinline__ uint32_t lget(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// mode bits: 1 keys+lc, 2 probe cols, 4 owner search, 8 bpermute values
template <int MODE, int G>
__global__ void __launch_bounds__(256) kw(const uint32_t* key, const uint32_t* pc0, const uint32_t* pc1, uint64_t np,
                                          const uint4* lc, uint32_t range, uint64_t units, const uint64_t* uoff,
                                          uint32_t* out, uint64_t cap) {
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  for (uint64_t u = blockIdx.x * 4ull + (threadIdx.x >> 6); u < units; u += waves) {
    const uint64_t r0 = u * 64 * G;
    uint4 e[G];
    uint32_t dk[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint64_t r = r0 + g * 64 + lane;
      dk[g] = (MODE & 1) && r < np ? key[r] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (MODE & 1) {
        e[g] = dk[g] < range ? lc[dk[g]] : make_uint4(0, 0, 0, 0);
      } else {
        e[g] = make_uint4(0, 2, 5, 6);          // fan-out 2
      }
    }
    uint64_t base = uoff[u];
    for (int g = 0; g < G; ++g) {
      const uint32_t c = e[g].y;
      const uint32_t inc = wscan(c);
      const uint32_t tot = __shfl(inc, 63, 64);
      const uint32_t pre = inc - c;
      const uint64_t r = r0 + g * 64 + lane;
      uint32_t p0 = 1, p1 = 2;
      if (MODE & 2) {
        p0 = r < np ? pc0[r] : 0;
        p1 = r < np ? pc1[r] : 0;
      }
      for (uint32_t o0 = 0; o0 < tot; o0 += 64) {
        const uint32_t o = o0 + lane;
        int l = lane;
        if (MODE & 4) {
          l = 0;
#pragma unroll
          for (int s = 32; s >= 1; s >>= 1) {
            const uint32_t pl = __shfl(pre, l + s, 64);
            if (l + s < 64 && pl <= o) l += s;
          }
        }
        uint32_t v0 = p0, v1 = p1, v2 = e[g].z;
        if (MODE & 8) {
          v0 = lget(p0, l);
          v1 = lget(p1, l);
          v2 = lget(e[g].z, l);
        }
        if (o < tot) {
          out[base + o] = v0;
          out[cap + base + o] = v1;
          out[2 * cap + base + o] = v2;
        }
      }
      base += tot;
    }
  }
}

int main() {
  const uint64_t np = 13'500'000, range = 50'000, nb = 100'000;
  std::mt19937_64 rng(1);
  // zipf-ish keys
  std::vector<double> cdf(range);
  double s = 0;
  for (uint64_t i = 0; i < range; ++i) cdf[i] = (s += 1.0 / std::pow(i + 1.0, 1.1));
  std::uniform_real_distribution<double> U(0, s);
  std::vector<uint32_t> key(np), pc(np);
  for (uint64_t i = 0; i < np; ++i) {
    key[i] = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin());
    pc[i] = (uint32_t)(rng() % 200000);
  }
  std::vector<uint32_t> cnt(range, 0);
  for (uint64_t i = 0; i < nb; ++i) cnt[rng() % range]++;
  std::vector<uint4> lc(range);
  uint32_t lo = 0;
  for (uint64_t d = 0; d < range; ++d) { lc[d] = make_uint4(lo, cnt[d], d, d); lo += cnt[d]; }
  auto mkoff = [&](uint64_t rows) {
    const uint64_t units = (np + rows - 1) / rows;
    std::vector<uint64_t> uoff(units + 1, 0);
    for (uint64_t u = 0; u < units; ++u) {
      uint64_t t = 0;
      for (uint64_t r = u * rows; r < std::min(np, u * rows + rows); ++r) t += cnt[key[r]];
      uoff[u + 1] = uoff[u] + t;
    }
    return uoff;
  };
  std::vector<uint64_t> uoff = mkoff(64);
  uint64_t total = uoff.back();
  uint32_t *dk, *dp0, *dp1, *dout;
  uint4* dlc;
  uint64_t* duo;
  hipMalloc(&dk, 4 * np); hipMalloc(&dp0, 4 * np); hipMalloc(&dp1, 4 * np);
  hipMalloc(&dlc, 16 * range); hipMalloc(&duo, 8 * (np / 64 + 2)); hipMalloc(&dout, 12 * total + 4096);
  hipMemcpy(dk, key.data(), 4 * np, hipMemcpyHostToDevice);
  hipMemcpy(dp0, pc.data(), 4 * np, hipMemcpyHostToDevice);
  hipMemcpy(dp1, pc.data(), 4 * np, hipMemcpyHostToDevice);
  hipMemcpy(dlc, lc.data(), 16 * range, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  printf("outputs %lu\n", (unsigned long)total);
  auto run = [&](const char* name, auto k, unsigned grid, int G) {
    auto uo = mkoff(64ull * G);
    const uint64_t units = uo.size() - 1;
    hipMemcpy(duo, uo.data(), 8 * uo.size(), hipMemcpyHostToDevice);
    if (!grid) grid = (unsigned)((units + 3) / 4);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, dk, dp0, dp1, np, dlc, (uint32_t)range, units, duo, dout, total);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r)
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, dk, dp0, dp1, np, dlc, (uint32_t)range, units, duo, dout, total);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-34s grid %6u %8.1f us\n", name, grid, ms * 100);
  };
  run("0 stores only G4", kw<0, 4>, 0, 4);
  run("1 +keys+lc G4", kw<1, 4>, 0, 4);
  run("1 +keys+lc G8", kw<1, 8>, 0, 8);
  run("1 +keys+lc G16", kw<1, 16>, 0, 16);
  run("15 full G4", kw<15, 4>, 0, 4);
  run("15 full G8", kw<15, 8>, 0, 8);
  run("15 full G16", kw<15, 16>, 0, 16);
  run("15 full G8 grid 4096", kw<15, 8>, 4096, 8);
  return 0;
}
