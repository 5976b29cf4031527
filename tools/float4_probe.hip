// float4_probe.hip -- reduces DESIGN.md's old "float4 .z/.w read wrong values" observation to a
// cause.  The suspect: a 16-byte vector load from an address that is only 4- or
// 8-byte aligned (e.g. row g of a [N,3] float array at 12 g bytes), where the compiler may
// assume the float4 type's 16-byte alignment.  Each case loads float4s at byte offsets 0, 4,
// 8, 12 (mod 16) from a buffer holding v[i] = i, from global memory and from LDS, through
// HIP's float4 and through a clang ext_vector_type(4), and reports any component that differs
// from the expected four consecutive values.
//   hipcc --offload-arch=gfx950 -O3 tools/float4_probe.hip -o tools/float4_probe && ./tools/float4_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float ev4 __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ void put(float *o, V v) {
  o[0] = v[0];
  o[1] = v[1];
  o[2] = v[2];
  o[3] = v[3];
}
__device__ __forceinline__ void put(float *o, float4 v) {
  o[0] = v.x;
  o[1] = v.y;
  o[2] = v.z;
  o[3] = v.w;
}

// out[case][lane][4]; cases: 0 global HIP float4, 1 global ext_vector, 2 LDS HIP float4,
// 3 LDS ext_vector, 4 / 5 global / LDS with the 16-byte alignment promised to the compiler
// (__builtin_assume_aligned: what a float4 pointer into a packed [N,3] array silently promises
// when the compiler can see no better), so it emits one global_load_dwordx4 / ds_read_b128.
// Lane l reads at float index 3 l + shift (a [N,3] row start when shift = 0).
// 6: one ds_read_b128 emitted directly (inline asm) at the misaligned LDS address.
constexpr int NCASE = 7;
__global__ void probe(const float *__restrict__ src, int shift, float *__restrict__ out) {
  __shared__ float lds[512];
  const int l = threadIdx.x;
  for (int i = l; i < 512; i += 64) lds[i] = src[i];
  __syncthreads();
  const int idx = 3 * l + shift;
  put(out + (0 * 64 + l) * 4, *reinterpret_cast<const float4 *>(src + idx));
  put(out + (1 * 64 + l) * 4, *reinterpret_cast<const ev4 *>(src + idx));
  put(out + (2 * 64 + l) * 4, *reinterpret_cast<const float4 *>(lds + idx));
  put(out + (3 * 64 + l) * 4, *reinterpret_cast<const ev4 *>(lds + idx));
  put(out + (4 * 64 + l) * 4,
      *reinterpret_cast<const float4 *>(__builtin_assume_aligned(src + idx, 16)));
  put(out + (5 * 64 + l) * 4,
      *reinterpret_cast<const float4 *>(__builtin_assume_aligned(lds + idx, 16)));
  typedef __attribute__((address_space(3))) float lds_float;
  const unsigned off = (unsigned)(size_t)(lds_float *)(lds + idx);
  ev4 r;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(off) : "memory");
  put(out + (6 * 64 + l) * 4, r);
}

int main() {
  float h[512];
  for (int i = 0; i < 512; ++i) h[i] = (float)i;
  float *d_src, *d_out;
  hipMalloc(&d_src, sizeof(h));
  hipMalloc(&d_out, NCASE * 64 * 4 * sizeof(float));
  hipMemcpy(d_src, h, sizeof(h), hipMemcpyHostToDevice);
  const char *names[NCASE] = {"global HIP float4", "global ext_vector(4)", "LDS HIP float4",
                              "LDS ext_vector(4)", "global dwordx4 (16B assumed)",
                              "LDS ds_read_b128 (16B assumed)", "LDS ds_read_b128 (asm)"};
  int total_bad = 0;
  for (int shift = 0; shift < 4; ++shift) {
    float o[NCASE * 64 * 4];
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_src, shift, d_out);
    hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost);
    for (int c = 0; c < NCASE; ++c) {
      int bad = 0, first = -1, comp = -1;
      for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k)
          if (o[(c * 64 + l) * 4 + k] != (float)(3 * l + shift + k)) {
            if (first < 0) { first = l; comp = k; }
            ++bad;
          }
      const int addr_mod16 = ((3 * (first < 0 ? 1 : first) + shift) * 4) % 16;
      printf("shift %d %-31s: %s", shift, names[c], bad ? "WRONG" : "ok");
      if (bad)
        printf(" (%d components; first lane %d comp %d: got %g want %g; address %% 16 = %d)",
               bad, first, comp, o[(c * 64 + first) * 4 + comp], (float)(3 * first + shift + comp),
               addr_mod16);
      printf("\n");
      total_bad += bad;
    }
  }
  hipFree(d_src);
  hipFree(d_out);
  printf("%s\n", total_bad ? "misaligned 16-B loads return wrong components" : "all loads correct");
  return 0;
}
