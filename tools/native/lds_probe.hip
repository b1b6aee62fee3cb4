// Diagnostic only (tools/): does a workgroup's static LDS keep what it wrote while other
// kernels share the CU?  Each workgroup fills its whole static LDS array with a
// signature, sleeps, and re-checks every dword; mismatches are counted (vector atomics
// on a global buffer) with the lowest / highest mismatching byte offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t sig(uint32_t b, uint32_t i, uint32_t tag) {
  uint32_t h = (b * 0x9E3779B1u) ^ (i * 0x85EBCA77u) ^ tag;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  return h ^ (h >> 15);
}

template <int S>
__global__ void __launch_bounds__(256) lds_probe_kernel(uint32_t* err, uint32_t tag, int spins) {
  __shared__ uint32_t buf[S / 4];
  for (int i = threadIdx.x; i < S / 4; i += 256) buf[i] = sig(blockIdx.x, i, tag);
  __syncthreads();
  for (int s = 0; s < spins; ++s) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  for (int i = threadIdx.x; i < S / 4; i += 256) {
    if (buf[i] != sig(blockIdx.x, i, tag)) {
      atomicAdd(&err[0], 1u);
      atomicMin(&err[1], (uint32_t)(i * 4));
      atomicMax(&err[2], (uint32_t)(i * 4));
    }
  }
}

extern "C" int lds_probe(int size_sel, uint32_t* err, uint32_t tag, int spins, int blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  switch (size_sel) {
    case 0: hipLaunchKernelGGL(lds_probe_kernel<21008>, dim3(blocks), dim3(256), 0, s, err, tag, spins); break;
    case 1: hipLaunchKernelGGL(lds_probe_kernel<21504>, dim3(blocks), dim3(256), 0, s, err, tag, spins); break;
    case 2: hipLaunchKernelGGL(lds_probe_kernel<42016>, dim3(blocks), dim3(256), 0, s, err, tag, spins); break;
    case 3: hipLaunchKernelGGL(lds_probe_kernel<8192>, dim3(blocks), dim3(256), 0, s, err, tag, spins); break;
    case 4: hipLaunchKernelGGL(lds_probe_kernel<65536>, dim3(blocks), dim3(256), 0, s, err, tag, spins); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
