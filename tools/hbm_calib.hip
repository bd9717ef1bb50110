// hbm_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns
// of k_level (MI355X_MICROARCH.md: "other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern"). Every buffer is far larger than the 256 MiB Infinity
// Cache and every address is touched once, so the algorithmic bytes are the HBM bytes.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/hbm_calib tools/hbm_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -f csv -d OUT -o run -- tools/_build/hbm_calib   (and WRITE_SIZE)
//
// Prints the algorithmic bytes of each kernel; tools/hbm_calib.py divides the counters by them.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

// 16 B per lane, coalesced (frontier staging)
__global__ void k_read16(const uint4* a, uint64_t n, unsigned* sink) {
  unsigned acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) *sink = acc;
}

// one random 64-B line per lane as four 16-B loads (visited-table bucket probe); every line once
__global__ void k_bucket64(const ulonglong2* t, uint64_t lines, unsigned* sink) {
  unsigned long long acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
    // a permutation of the lines: odd multiplier modulo a power of two
    const uint64_t b = (i * 0x9E3779B97F4A7C15ull + 12345) & (lines - 1);
    const ulonglong2* B = t + b * 4;
    const ulonglong2 q0 = B[0], q1 = B[1], q2 = B[2], q3 = B[3];
    acc ^= q0.x ^ q0.y ^ q1.x ^ q1.y ^ q2.x ^ q2.y ^ q3.x ^ q3.y;
  }
  if (acc == 0x12345678ull) *sink = (unsigned)acc;
}

// 4 B per lane, coalesced stores (row emission: lane L writes words L, L + 64, ...)
__global__ void k_write4(unsigned* a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = (unsigned)i;
}

// 16 B per lane at scattered (but whole-line-covering) positions (next_fp / history writes)
__global__ void k_write16_scatter(uint4* a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = (i * 0x9E3779B97F4A7C15ull + 777) & (n - 1);
    a[j] = make_uint4((unsigned)i, 1u, 2u, 3u);
  }
}

// one 64-bit CAS per lane on a random slot of distinct lines (visited-table insert)
__global__ void k_cas8(unsigned long long* t, uint64_t lines) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = (i * 0x9E3779B97F4A7C15ull + 999) & (lines - 1);
    atomicCAS(t + b * 8 + (mix(i) & 7), 0ull, (unsigned long long)i | 1ull);
  }
}

int main() {
  const uint64_t big = 2ull << 30;  // 2 GiB per buffer
  void *a, *b;
  unsigned* sink;
  CK(hipMalloc(&a, big));
  CK(hipMalloc(&b, big));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, big));
  CK(hipMemset(b, 0, big));
  CK(hipDeviceSynchronize());
  const int grid = 256 * 64, block = 256;
  // flush the Infinity Cache between kernels by streaming through the other buffer
  auto flush = [&]() { hipLaunchKernelGGL(k_write4, dim3(grid), dim3(block), 0, 0, (unsigned*)b, big / 4); };
  flush();
  hipLaunchKernelGGL(k_read16, dim3(grid), dim3(block), 0, 0, (const uint4*)a, big / 16, sink);
  printf("k_read16 read %llu write 0\n", (unsigned long long)big);
  flush();
  hipLaunchKernelGGL(k_bucket64, dim3(grid), dim3(block), 0, 0, (const ulonglong2*)a, big / 64, sink);
  printf("k_bucket64 read %llu write 0\n", (unsigned long long)big);
  flush();
  hipLaunchKernelGGL(k_write4, dim3(grid), dim3(block), 0, 0, (unsigned*)a, big / 4);
  printf("k_write4 read 0 write %llu\n", (unsigned long long)big);
  flush();
  hipLaunchKernelGGL(k_write16_scatter, dim3(grid), dim3(block), 0, 0, (uint4*)a, big / 16);
  printf("k_write16_scatter read 0 write %llu\n", (unsigned long long)big);
  flush();
  CK(hipMemset(a, 0, big));
  flush();
  hipLaunchKernelGGL(k_cas8, dim3(grid), dim3(block), 0, 0, (unsigned long long*)a, big / 64);
  printf("k_cas8 read %llu write %llu (lines touched: 64 B each; 8 B changed per line)\n",
         (unsigned long long)big, (unsigned long long)big);
  printf("k_write4 (flush) write %llu per launch\n", (unsigned long long)big);
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
