// Host cost of stream-ordered allocation (hipMallocAsync / hipFreeAsync) for
// the block sizes a query step uses, with the pool's release threshold raised.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamDefault);
  hipMemPool_t pool;
  hipDeviceGetDefaultMemPool(&pool, 0);
  uint64_t keep = ~0ull;
  hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  const size_t sizes[] = {4096, 1 << 20, 108u << 20, 300u << 20};
  for (size_t sz : sizes) {
    void* p;
    hipMallocAsync(&p, sz, s);
    hipFreeAsync(p, s);
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100; ++i) {
      hipMallocAsync(&p, sz, s);
      hipFreeAsync(p, s);
    }
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    printf("size %10zu: malloc+free %8.2f us/pair host, drain %8.1f us\n", sz,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 100,
           std::chrono::duration<double, std::micro>(t2 - t1).count());
  }
  // interleaved sizes (a query step's pattern)
  void* a[6];
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 100; ++i) {
    hipMallocAsync(&a[0], 108u << 20, s);
    hipMallocAsync(&a[1], 300u << 20, s);
    hipMallocAsync(&a[2], 1 << 20, s);
    hipFreeAsync(a[2], s);
    hipFreeAsync(a[0], s);
    hipMallocAsync(&a[3], 108u << 20, s);
    hipFreeAsync(a[1], s);
    hipFreeAsync(a[3], s);
  }
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(s);
  printf("mixed step pattern: %8.2f us/iter\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  // D2D copy and small D2H read latency
  void *x, *y;
  hipMalloc(&x, 1 << 20);
  hipMalloc(&y, 1 << 20);
  uint64_t h;
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 100; ++i) hipMemcpyAsync(y, x, 200000, hipMemcpyDeviceToDevice, s);
  t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(s);
  printf("D2D memcpyAsync issue: %8.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 100; ++i) {
    hipMemcpyAsync(&h, x, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
  }
  t1 = std::chrono::steady_clock::now();
  printf("8-byte D2H read + sync: %8.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  uint64_t* pin;
  hipHostMalloc((void**)&pin, 64, hipHostMallocDefault);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 100; ++i) {
    hipMemcpyAsync(pin, x, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
  }
  t1 = std::chrono::steady_clock::now();
  printf("8-byte D2H (pinned) + sync: %8.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  return 0;
}
