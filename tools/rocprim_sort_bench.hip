// Experiment: rocPRIM's device radix sort (onesweep) vs this repository's reduce-then-scan
// sort for the binning's two sorts (1M 32-bit depth keys; 7.7M 13-bit tile keys), timed with
// HIP events.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/rocprim_sort_bench.hip
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static float bench(size_t n, int end_bit, unsigned mask) {
  std::vector<unsigned> hk(n), hv(n);
  unsigned s = 12345;
  for (size_t i = 0; i < n; ++i) { s = s * 1664525u + 1013904223u; hk[i] = (s >> 3) & mask; hv[i] = (unsigned)i; }
  unsigned *k0, *k1, *v0, *v1;
  CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
  size_t tmp = 0;
  CK(rocprim::radix_sort_pairs(nullptr, tmp, k0, k1, v0, v1, n, 0, end_bit));
  void *t; CK(hipMalloc(&t, tmp));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) CK(rocprim::radix_sort_pairs(t, tmp, k0, k1, v0, v1, n, 0, end_bit));
  CK(hipDeviceSynchronize());
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_pairs(t, tmp, k0, k1, v0, v1, n, 0, end_bit));
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  // check sortedness + stability of the output
  std::vector<unsigned> ok(n), ov(n);
  CK(hipMemcpy(ok.data(), k1, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ov.data(), v1, n * 4, hipMemcpyDeviceToHost));
  bool good = true;
  for (size_t i = 1; i < n; ++i)
    if (ok[i - 1] > ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] > ov[i])) { good = false; break; }
  CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(v0)); CK(hipFree(v1)); CK(hipFree(t));
  printf("n=%zu bits=%d: %.1f us per sort (%s)\n", n, end_bit, ms / reps * 1e3, good ? "stable, sorted" : "WRONG");
  return ms / reps;
}

int main() {
  bench(100000, 32, 0xFFFFFFFFu);
  bench(300000, 32, 0xFFFFFFFFu);
  bench(1000000, 32, 0xFFFFFFFFu);
  bench(7717748, 13, 0x1FFFu);
  bench(83276610, 15, 0x7FFFu);
  return 0;
}
