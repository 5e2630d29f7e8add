// Microbenchmark of the config-5 L1 screen loop (csrc/screen_big.hip
// screen_big_sp) on synthetic fragments, chip-wide, with ablations:
//   mode 0 full, 1 MFMA + minimal VALU (one v_min per block), 2 VALU only
//   (no MFMA: the C rows stand in for the products), 3 full but A fragments
//   held in registers (no LDS reads in the loop).
// Diagnostic tool, not part of the product.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int DQ, int NT, int MODE>
__global__ __launch_bounds__(NT) void l1(const h8* __restrict__ frag, const float* __restrict__ cinit,
                                         const h8* __restrict__ pts, int KB, long long groups,
                                         unsigned* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* scin = reinterpret_cast<float*>(smem);
  h8* sfrag = reinterpret_cast<h8*>(smem + (size_t)KB * 32 * 4);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  for (int i = threadIdx.x; i < KB * 32; i += blockDim.x) scin[i] = cinit[i];
  for (int i = threadIdx.x; i < KB * DQ * 64; i += blockDim.x) sfrag[i] = frag[i];
  __syncthreads();
  const int wave = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (NT / 64);
  unsigned acc_out = 0;
  h8 Areg[DQ];
  for (int c = 0; c < DQ; ++c) Areg[c] = sfrag[c * 64 + lane];
  for (long long g = wave; g < groups; g += nw) {
    h8 BH[2][DQ];
    for (int t = 0; t < 2; ++t)
      for (int c = 0; c < DQ; ++c) BH[t][c] = pts[(((g & 2047) * 2 + t) * DQ + c) * 64 + lane];
    unsigned RB[2] = {~0u, ~0u}, RS[2] = {~0u, ~0u};
    auto mm = [&](int b, f16v (&acc)[2]) {
      const f4* cr = reinterpret_cast<const f4*>(scin + 32 * b + 4 * h);
      f16v ci;
      for (int q = 0; q < 4; ++q) {
        const f4 v = cr[2 * q];
        for (int i = 0; i < 4; ++i) ci[4 * q + i] = v[i];
      }
      if (MODE == 2) {
        acc[0] = ci;
        acc[1] = ci + (float)b;
        return;
      }
      h8 A[DQ];
      for (int c = 0; c < DQ; ++c) A[c] = MODE == 3 ? Areg[c] : sfrag[((size_t)b * DQ + c) * 64 + lane];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[0][0], ci, 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[0], BH[1][0], ci, 0, 0, 0);
      for (int c = 1; c < DQ; ++c) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[0][c], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[c], BH[1][c], acc[1], 0, 0, 0);
      }
    };
    auto red = [&](int b, const f16v (&acc)[2]) {
      if (MODE == 1) {
        RB[0] = min(RB[0], __float_as_uint(acc[0][b & 15]));
        RB[1] = min(RB[1], __float_as_uint(acc[1][b & 15]));
        return;
      }
      const unsigned bo = ((unsigned)b << 5) | ((unsigned)h << 4);
      for (int t = 0; t < 2; ++t) {
        auto key = [&](int i) { return (__float_as_uint(acc[t][i]) & ~15u) | (unsigned)i; };
        unsigned kb = min(key(0), key(1)), ks = max(key(0), key(1));
        for (int i = 2; i < 16; i += 2) {
          const unsigned x = key(i), y = key(i + 1);
          unsigned m;
          asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m) : "v"(kb), "v"(x), "v"(y));
          asm("v_min3_u32 %0, %1, %2, %3" : "=v"(kb) : "v"(kb), "v"(x), "v"(y));
          ks = min(ks, m);
        }
        const unsigned kj = (kb & 0xFFFFFC0Fu) | bo;
        unsigned ms;
        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(ms) : "v"(max(RB[t], kj)), "v"(RS[t]), "v"(ks));
        RS[t] = ms;
        RB[t] = min(RB[t], kj);
      }
    };
    f16v accA[2], accB[2];
    mm(0, accA);
    int b = 1;
    for (; b + 1 < KB; b += 2) {
      mm(b, accB);
      red(b - 1, accA);
      mm(b + 1, accA);
      red(b, accB);
    }
    if (b < KB) {
      mm(b, accB);
      red(b - 1, accA);
      red(b, accB);
    } else {
      red(b - 1, accA);
    }
    acc_out += RB[0] ^ RS[1] ^ RB[1] ^ RS[0];
  }
  out[blockIdx.x * NT + threadIdx.x] = acc_out;
}

template <int MODE>
float run(int KB, long long groups, const h8* frag, const float* cinit, const h8* pts, unsigned* out,
          int cus) {
  const size_t lds = (size_t)KB * 32 * 4 + (size_t)KB * 4 * 64 * 16;
  hipFuncSetAttribute(reinterpret_cast<const void*>(&l1<4, 512, MODE>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  l1<4, 512, MODE><<<cus, 512, lds>>>(frag, cinit, pts, KB, groups, out);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) l1<4, 512, MODE><<<cus, 512, lds>>>(frag, cinit, pts, KB, groups, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 3;
}

int main() {
  const int KB = 32, DQ = 4;
  const long long groups = 50000000 / 64;
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  h8 *frag, *pts;
  float* cinit;
  unsigned* out;
  hipMalloc(&frag, sizeof(h8) * KB * DQ * 64);
  hipMalloc(&cinit, sizeof(float) * KB * 32);
  hipMalloc(&pts, sizeof(h8) * 2 * DQ * 64 * 4096);  // groups wrap over 2048 (L2-resident points)
  hipMalloc(&out, sizeof(unsigned) * cus * 512);
  hipMemset(frag, 0x11, sizeof(h8) * KB * DQ * 64);
  hipMemset(cinit, 0x40, sizeof(float) * KB * 32);
  hipMemset(pts, 0x22, sizeof(h8) * 2 * DQ * 64 * 4096);
  // points: groups index pts modulo 2048 groups (the loads hit L2: this times the compute)
  const double flop = 2.0 * 50e6 * 1024 * 64;
  float t[4];
  t[0] = run<0>(KB, 2048, frag, cinit, pts, out, cus);  // warm
  t[0] = run<0>(KB, groups, frag, cinit, pts, out, cus);
  t[1] = run<1>(KB, groups, frag, cinit, pts, out, cus);
  t[2] = run<2>(KB, groups, frag, cinit, pts, out, cus);
  t[3] = run<3>(KB, groups, frag, cinit, pts, out, cus);
  const char* nm[4] = {"full", "mfma+min", "valu-only", "full,A in regs"};
  for (int m = 0; m < 4; ++m)
    printf("mode %d %-16s %8.3f ms  %7.1f TF/s\n", m, nm[m], t[m], flop / (t[m] * 1e-3) / 1e12);
  return 0;
}
