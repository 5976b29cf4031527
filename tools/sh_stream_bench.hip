// Streaming experiment for the SH colour kernels (the drop-in compute_sh_forward and the fused
// preprocess's colour part read 192 B of coefficients per Gaussian at degree 3 and run at
// ~3 TB/s): the shipped block-staged form (256 threads, one 50 KB LDS slab, a block barrier
// between the loads and the evaluation) against one wave per workgroup (12.25 KB of LDS each,
// no block barrier), against a persistent wave that loads the next 64 rows while it evaluates
// these, and against a plain read of the same bytes (the streaming ceiling).  Every variant's
// colours are compared with the shipped form's bit for bit.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I gaussctrl_exp_amd/csrc \
//          tools/sh_stream_bench.hip -o tools/sh_stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sh_math.h"

using namespace gs;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int K = 16, ROW = K * 3, ROWP = ROW | 1;

// A: the shipped sh_fwd_kernel<16>
__global__ __launch_bounds__(256) void sh_block(int n, int deg, const float *__restrict__ dirs,
                                                const float *__restrict__ coeffs,
                                                float *__restrict__ colors) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const long long g0 = (long long)blockIdx.x * 256;
  const int cnt = (int)min(256LL, (long long)n - g0);
  stage_rows<ROW, ROWP, 256>(coeffs + g0 * ROW, cnt, smem);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= cnt) return;
  const long long g = g0 + t;
  float b[25];
  const int nb = sh_basis(deg, dirs[3 * g], dirs[3 * g + 1], dirs[3 * g + 2], b);
  const float *co = smem + t * ROWP;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    colors[3 * g + c] = sh_channel<K>(b, nb, [&](int k) { return co[k * 3 + c]; });
}

// B1: one wave per workgroup, its own 64 rows staged in LDS
__global__ __launch_bounds__(64) void sh_wave(int n, int deg, const float *__restrict__ dirs,
                                              const float *__restrict__ coeffs,
                                              float *__restrict__ colors) {
  __shared__ __attribute__((aligned(16))) float smem[64 * ROWP];
  const long long g0 = (long long)blockIdx.x * 64;
  const int cnt = (int)min(64LL, (long long)n - g0);
  stage_rows<ROW, ROWP, 64>(coeffs + g0 * ROW, cnt, smem);
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= cnt) return;
  const long long g = g0 + t;
  float b[25];
  const int nb = sh_basis(deg, dirs[3 * g], dirs[3 * g + 1], dirs[3 * g + 2], b);
  const float *co = smem + t * ROWP;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    colors[3 * g + c] = sh_channel<K>(b, nb, [&](int k) { return co[k * 3 + c]; });
}

// B2: persistent waves; chunk c's rows land in LDS while chunk c + grid's loads are in flight
__global__ __launch_bounds__(64) void sh_pipe(int n, int deg, const float *__restrict__ dirs,
                                              const float *__restrict__ coeffs,
                                              float *__restrict__ colors) {
  __shared__ __attribute__((aligned(16))) float smem[64 * ROWP];
  constexpr int PER = 64 * ROW / 4 / 64;  // 12 float4 per lane
  const long long nch = ((long long)n + 63) / 64;
  const int t = threadIdx.x;
  float4 v[PER];
  auto issue = [&](long long c) {
    const long long g0 = c * 64;
    if (g0 + 64 <= n) {
      const float4 *s4 = reinterpret_cast<const float4 *>(coeffs + g0 * ROW);
#pragma unroll
      for (int u = 0; u < PER; ++u) v[u] = s4[u * 64 + t];
    }
  };
  long long c = blockIdx.x;
  if (c < nch) issue(c);
  for (; c < nch; c += gridDim.x) {
    const long long g0 = c * 64;
    const int cnt = (int)min(64LL, (long long)n - g0);
    if (cnt == 64) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int k = u * 64 + t;
        smem[sh_lds_index<ROW, ROWP>(4 * k)] = v[u].x;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 1)] = v[u].y;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 2)] = v[u].z;
        smem[sh_lds_index<ROW, ROWP>(4 * k + 3)] = v[u].w;
      }
    } else {
      stage_rows<ROW, ROWP, 64>(coeffs + g0 * ROW, cnt, smem);
    }
    __syncthreads();
    if (c + gridDim.x < nch) issue(c + gridDim.x);  // the next chunk's loads, in flight below
    if (t < cnt) {
      const long long g = g0 + t;
      float b[25];
      const int nb = sh_basis(deg, dirs[3 * g], dirs[3 * g + 1], dirs[3 * g + 2], b);
      const float *co = smem + t * ROWP;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch)
        colors[3 * g + ch] = sh_channel<K>(b, nb, [&](int k) { return co[k * 3 + ch]; });
    }
    __syncthreads();
  }
}

// R: the same bytes read and written with no evaluation (a per-Gaussian sum of its row)
__global__ __launch_bounds__(256) void stream_ref(int n, const float *__restrict__ dirs,
                                                  const float *__restrict__ coeffs,
                                                  float *__restrict__ colors) {
  const long long nv = (long long)n * ROW / 4;
  const float4 *s4 = reinterpret_cast<const float4 *>(coeffs);
  float acc = 0.f;
  for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < nv;
       k += (long long)gridDim.x * 256) {
    const float4 q = s4[k];
    acc += q.x + q.y + q.z + q.w;
  }
  for (long long g = (long long)blockIdx.x * 256 + threadIdx.x; g < n;
       g += (long long)gridDim.x * 256) {
    colors[3 * g] = acc + dirs[3 * g];
    colors[3 * g + 1] = dirs[3 * g + 1];
    colors[3 * g + 2] = dirs[3 * g + 2];
  }
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1000000;
  const int reps = 30;
  std::vector<float> hc((size_t)n * ROW), hd((size_t)n * 3);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.f / 16777216.f) - 0.5f; };
  for (auto &x : hc) x = rnd();
  for (auto &x : hd) x = rnd() + 0.01f;
  float *c, *d, *oa, *ob;
  CK(hipMalloc(&c, hc.size() * 4));
  CK(hipMalloc(&d, hd.size() * 4));
  CK(hipMalloc(&oa, (size_t)n * 12));
  CK(hipMalloc(&ob, (size_t)n * 12));
  CK(hipMemcpy(c, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double bytes = (double)n * (ROW * 4 + 12 + 12);
  auto timeit = [&](const char *name, auto launch, float *out) {
    launch(out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch(out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-34s %8.2f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  const int nb256 = (n + 255) / 256, nb64 = (n + 63) / 64;
  timeit("A block-staged (shipped)", [&](float *o) {
    hipLaunchKernelGGL(sh_block, dim3(nb256), dim3(256), 256 * ROWP * 4, 0, n, 3, d, c, o);
  }, oa);
  std::vector<float> ra((size_t)n * 3), rb((size_t)n * 3);
  CK(hipMemcpy(ra.data(), oa, ra.size() * 4, hipMemcpyDeviceToHost));
  auto check = [&](const char *name) {
    CK(hipMemcpy(rb.data(), ob, rb.size() * 4, hipMemcpyDeviceToHost));
    const bool same = memcmp(ra.data(), rb.data(), ra.size() * 4) == 0;
    printf("   %s bit-identical to A: %s\n", name, same ? "yes" : "NO");
  };
  timeit("B1 one wave per workgroup", [&](float *o) {
    hipLaunchKernelGGL(sh_wave, dim3(nb64), dim3(64), 0, 0, n, 3, d, c, o);
  }, ob);
  check("B1");
  for (int per_cu : {8, 12, 13, 16}) {
    char name[64];
    snprintf(name, sizeof name, "B2 persistent, %d waves/CU", per_cu);
    CK(hipMemset(ob, 0, (size_t)n * 12));
    timeit(name, [&](float *o) {
      hipLaunchKernelGGL(sh_pipe, dim3(min(nb64, per_cu * cus)), dim3(64), 0, 0, n, 3, d, c, o);
    }, ob);
    check("B2");
  }
  timeit("R plain read of the same bytes", [&](float *o) {
    hipLaunchKernelGGL(stream_ref, dim3(cus * 8), dim3(256), 0, 0, n, d, c, o);
  }, ob);
  printf("(bytes per launch: %.1f MB)\n", bytes / 1e6);
  return 0;
}
