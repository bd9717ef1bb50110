// Instruction-fetch cost of a long straight-line code path on gfx950 (measurement tool, not the
// product): one wave per workgroup runs N 8-byte VALU instructions (4 independent chains) twice
// in a row and records s_memtime around each pass. Pass 1 fetches the code from L2 / memory
// (a cold instruction cache at kernel start); pass 2 runs it from the instruction cache when it
// fits. k_level's small levels run one chunk pass of a ~100 KB code path per workgroup, so their
// per-phase latency includes this fetch.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_build/icache_probe tools/icache_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int N>
__global__ void __launch_bounds__(64) k_probe(uint64_t* out, uint32_t seed) {
  uint32_t a0 = seed, a1 = seed ^ 1, a2 = seed ^ 2, a3 = seed ^ 3;
  uint64_t t[3];
  for (int r = 0; r < 2; r++) {
    t[r] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < N / 4; i++) {
      asm volatile("v_add_u32 %0, 0x9e3779b1, %0" : "+v"(a0));
      asm volatile("v_add_u32 %0, 0x85ebca6b, %0" : "+v"(a1));
      asm volatile("v_add_u32 %0, 0xc2b2ae35, %0" : "+v"(a2));
      asm volatile("v_add_u32 %0, 0x27d4eb2f, %0" : "+v"(a3));
    }
    asm volatile("s_waitcnt 0" ::: "memory");
  }
  t[2] = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = t[1] - t[0];
    out[blockIdx.x * 4 + 1] = t[2] - t[1];
    out[blockIdx.x * 4 + 2] = a0 ^ a1 ^ a2 ^ a3;
  }
}

template <int N>
int run(int blocks, uint64_t* d, uint64_t* h) {
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_probe<N>, dim3(blocks), dim3(64), 0, 0, d, 7u + rep);
    CHK(hipDeviceSynchronize());
  }
  CHK(hipMemcpy(h, d, sizeof(uint64_t) * 4 * blocks, hipMemcpyDeviceToHost));
  double p1 = 0, p2 = 0;
  for (int b = 0; b < blocks; b++) { p1 += h[b * 4]; p2 += h[b * 4 + 1]; }
  // s_memtime: the shader clock (cycles)
  printf("{\"instructions\": %d, \"code_bytes\": %d, \"blocks\": %d, \"pass1_cycles\": %.0f, \"pass2_cycles\": %.0f, "
         "\"pass1_per_instr\": %.2f, \"pass2_per_instr\": %.2f}\n", N, N * 8, blocks, p1 / blocks, p2 / blocks,
         p1 / blocks / N, p2 / blocks / N);
  return 0;
}

int main() {
  uint64_t* d;
  static uint64_t h[4 * 4096];
  CHK(hipMalloc(&d, sizeof(uint64_t) * 4 * 4096));
  for (int blocks : {1, 256, 1024}) {
    if (run<1024>(blocks, d, h)) return 1;
    if (run<4096>(blocks, d, h)) return 1;
    if (run<8192>(blocks, d, h)) return 1;
    if (run<16384>(blocks, d, h)) return 1;
  }
  return 0;
}
