// Random-access ceilings of the C3 regime (a visited table far beyond the Infinity Cache): the
// chip-wide rate of independent 8-byte loads, each to its own random 64-byte line, and of 8-byte
// agent-scope CAS to random slots (the memory-side atomic the probe uses), over a table of the C3
// bench's size. These rates -- not the 8 TB/s streaming peak -- bound k_level in that regime.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/rand_calib tools/rand_calib.hip
// run:   tools/_build/rand_calib [log2_bytes=35] [waves_per_cu=16]   (prints one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));             \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

constexpr int U = 8;  // independent accesses in flight per lane

// every lane: `iters` rounds of U independent random 8-byte loads (each in its own 64-B line)
__global__ void k_rand_load(const unsigned long long* t, unsigned long long line_mask, int iters,
                            unsigned long long* sink) {
  const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int it = 0; it < iters; it++) {
    unsigned long long v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned long long line = mix(g * 0x9E3779B97F4A7C15ull + (unsigned long long)(it * U + u)) & line_mask;
      v[u] = __hip_atomic_load(t + line * 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u];
  }
  if (acc == 0x1234567ull) sink[0] = acc;  // never true on a zeroed table; keeps the loads
}

// every lane: `iters` rounds of U independent CAS(0 -> key) on random slots (returned values used)
__global__ void k_rand_cas(unsigned long long* t, unsigned long long slot_mask, int iters, unsigned long long* sink) {
  const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long acc = 0;
  for (int it = 0; it < iters; it++) {
    unsigned long long v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned long long h = mix(g * 0xC2B2AE3D27D4EB4Full + (unsigned long long)(it * U + u));
      v[u] = atomicCAS(t + (h & slot_mask), 0ull, h | 1ull);
    }
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u];
  }
  if (acc == 0x1234567ull) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 35;
  const int wpc = argc > 2 ? atoi(argv[2]) : 16;
  const size_t bytes = (size_t)1 << lg;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  unsigned long long *t, *sink;
  CHECK(hipMalloc(&t, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(t, 0, bytes));
  const int block = 256, blocks = cus * wpc / (block / 64);
  const unsigned long long lanes = (unsigned long long)blocks * block;
  const unsigned long long line_mask = (bytes / 64) - 1, slot_mask = (bytes / 8) - 1;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto time_it = [&](auto launch) {
    launch(2);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    launch(64);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return (double)lanes * 64 * U / (ms / 1e3);
  };
  const double loads = time_it([&](int it) { hipLaunchKernelGGL(k_rand_load, dim3(blocks), dim3(block), 0, 0, t, line_mask, it, sink); });
  const double cas = time_it([&](int it) { hipLaunchKernelGGL(k_rand_cas, dim3(blocks), dim3(block), 0, 0, t, slot_mask, it, sink); });
  CHECK(hipGetLastError());
  printf("{\"table_bytes\": %zu, \"cus\": %d, \"waves_per_cu\": %d, \"in_flight_per_lane\": %d, "
         "\"random_line_loads_per_s\": %.4g, \"random_line_load_GBps_64B\": %.1f, \"random_cas_per_s\": %.4g}\n",
         bytes, cus, wpc, U, loads, loads * 64 / 1e9, cas);
  CHECK(hipFree(t));
  CHECK(hipFree(sink));
  return 0;
}
