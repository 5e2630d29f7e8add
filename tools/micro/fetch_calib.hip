// Calibrates the gfx950 memory-side read counters against known byte counts
// for the access shapes of the bounded screen (MI355X_MICROARCH.md: "other
// access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern"):
//   k0 stream16   16 B per lane, coalesced (the bound-word stream)
//   k1 gather64   one lane per random 64-byte-aligned row, 4 x 16 B
//                 non-temporal loads (screen32bs16's phase-2 row gather)
//   k2 gather128  one lane per random 128-byte-aligned row, 8 x 16 B
//   k3 pair64     two random rows in one 128-byte line per lane pair
//                 (lanes 2i, 2i+1 read the two halves of one line)
//   k4 write16    16 B per lane, coalesced stores
// Every region is far larger than the 256 MiB Infinity Cache.  Run under
// rocprofv3 --pmc <counters> --kernel-trace; the program prints the bytes
// each dispatch touches.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ inline unsigned long long mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void stream16(const u4* __restrict__ src, long long n16,
                                                unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (long long)gridDim.x * 256) {
    const u4 v = __builtin_nontemporal_load(src + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// rows: row r = 4 x 16 B at src + 4 r; nrows rows in the region, nreads reads
template <int PER>  // 16-byte loads per row (4: 64 B, 8: 128 B)
__global__ __launch_bounds__(256) void gather(const u4* __restrict__ src, long long nrows,
                                              long long nreads, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nreads;
       i += (long long)gridDim.x * 256) {
    const long long r = (long long)(mix((unsigned long long)i) % (unsigned long long)nrows);
    u4 v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) v[q] = __builtin_nontemporal_load(src + r * PER + q);
#pragma unroll
    for (int q = 0; q < PER; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// lanes 2i and 2i+1: the two 64-byte halves of one random 128-byte line
__global__ __launch_bounds__(256) void pair64(const u4* __restrict__ src, long long nlines,
                                              long long nreads, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nreads;
       i += (long long)gridDim.x * 256) {
    const long long r = (long long)(mix((unsigned long long)(i >> 1)) % (unsigned long long)nlines);
    const u4* p = src + r * 8 + (i & 1) * 4;
    u4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_nontemporal_load(p + q);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void write16(u4* __restrict__ dst, long long n16) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16;
       i += (long long)gridDim.x * 256)
    dst[i] = u4{(unsigned)i, 1u, 2u, 3u};
}

int main() {
  const size_t region = 6ull << 30;  // 6 GiB: far above the Infinity Cache
  u4* buf = nullptr;
  unsigned* sink = nullptr;
  CK(hipMalloc(&buf, region));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, region));
  CK(hipDeviceSynchronize());
  const long long n16 = (long long)(region / 16);
  const int grid = 256 * 16;
  const long long nread = 8ll << 20;  // 8M random rows per gather kernel
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, buf, n16 / 3, sink);
    hipLaunchKernelGGL((gather<4>), dim3(grid), dim3(256), 0, 0, buf, (long long)(region / 64),
                       nread, sink);
    hipLaunchKernelGGL((gather<8>), dim3(grid), dim3(256), 0, 0, buf, (long long)(region / 128),
                       nread, sink);
    hipLaunchKernelGGL(pair64, dim3(grid), dim3(256), 0, 0, buf, (long long)(region / 128), nread,
                       sink);
    hipLaunchKernelGGL(write16, dim3(grid), dim3(256), 0, 0, buf, n16 / 6);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
  }
  std::printf("bytes stream16 %lld gather64 %lld gather128 %lld pair64 %lld write16 %lld\n",
              (n16 / 3) * 16, nread * 64, nread * 128, nread * 64, (n16 / 6) * 16);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
