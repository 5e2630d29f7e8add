// Microbenchmark: cycles per v_mfma_f32_32x32x16_f16 / 16x16x32 on one SIMD,
// with independent and 3-deep dependent accumulator chains, and with VALU
// filler.  Diagnostic tool, not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(64) void k(const h8* in, float* out, long long* cyc, int iters) {
  h8 a = in[threadIdx.x], b = in[64 + threadIdx.x];
  f16v c0 = {}, c1 = {}, c2 = {}, c3 = {};
  f4v d0 = {}, d1 = {}, d2 = {}, d3 = {};
  unsigned z = threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // 4 independent 32x32x16
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c3, 0, 0, 0);
    } else if (MODE == 1) {  // 4 independent 16x16x32
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d3, 0, 0, 0);
    } else if (MODE == 2) {  // 32x32x16, result consumed by VALU each time (key-like)
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) z = min(z, (__float_as_uint(c0[r]) & ~63u) | r);
    } else if (MODE == 3) {  // 16 VALU filler per independent MFMA
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c1, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) z = z * 3u + (unsigned)r;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  f16v s = c0 + c1 + c2 + c3;
  float acc = s[0] + d0[0] + d1[0] + d2[0] + d3[0] + (float)z;
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  h8* in; float* out; long long* cyc;
  hipMalloc(&in, 128 * sizeof(h8));
  hipMemset(in, 0, 128 * sizeof(h8));
  const int blocks = 256 * 4;  // one wave per SIMD
  hipMalloc(&out, blocks * 64 * 4);
  hipMalloc(&cyc, blocks * 8);
  long long h[1024];
  const int iters = 4096;
  auto run = [&](auto kern, const char* name, int per_iter) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, in, out, cyc, iters);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, in, out, cyc, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < blocks; ++i) avg += h[i]; avg /= blocks;
    printf("%-40s cycles/MFMA %.1f  wall %.3f ms  clk %.2f GHz\n", name, avg / iters / per_iter, ms,
           avg / (ms * 1e6));
  };
  run(k<0>, "32x32x16 f16, 4 independent", 4);
  run(k<1>, "16x16x32 f16, 4 independent", 4);
  run(k<2>, "32x32x16 + 16 dependent VALU", 1);
  run(k<3>, "2x 32x32x16 + 16 VALU (indep)", 2);
  return 0;
}
