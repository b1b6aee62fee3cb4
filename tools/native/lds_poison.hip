// Diagnostic only (tools/): fill the LDS of every CU with a seed-dependent pattern, so a
// kernel launched afterwards that reads LDS it never wrote sees values that change
// from run to run (fp16 NaNs / large finite values, never zero).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) lds_poison_kernel(uint32_t seed) {
  extern __shared__ uint32_t lds[];
  const int n = 160 * 1024 / 4;
  for (int i = threadIdx.x; i < n; i += 256) {
    uint32_t h = (i + 1) * 0x9E3779B1u ^ seed * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    // seed odd: fp16 NaN pairs; seed even: finite fp16 in [256, 2048) with random sign
    lds[i] = (seed & 1) ? (0x7E007E00u | (h & 0x01FF01FFu)) : ((h & 0x80008000u) | 0x5C005C00u | (h & 0x03FF03FFu));
  }
  __syncthreads();
  // keep the stores alive
  if (lds[(threadIdx.x * 37) % n] == 0x12345678u && seed == 0xFFFFFFFFu) lds[0] = 1;
}

extern "C" int lds_poison(uint32_t seed, int blocks, void* stream) {
  static int attr_done = 0;
  if (!attr_done) {
    if (hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024) != hipSuccess)
      return -1;
    attr_done = 1;
  }
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), 160 * 1024, (hipStream_t)stream, seed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
