// GDN parameter preparation and LayerNorm (gfx950).
#include "lic_common.h"

namespace lic {

// beta' = max(beta, bb)^2 - ped ; gamma' = max(gamma, gb)^2 - ped, packed as a
// 1x1 conv weight [copad][1][cpad] (zero padded).  model/gdn.py:69-84,
// ops/parametrizers.py:48-51.
template <typename T>
__global__ void gdn_prepare_kernel(const float* __restrict__ beta, const float* __restrict__ gamma, int c,
                                   float bb, float gb, float ped, T* __restrict__ w, int cpad, int copad,
                                   float* __restrict__ beta_out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)copad * cpad;
  if (idx < total) {
    const int o = (int)(idx / cpad), i = (int)(idx % cpad);
    float v = 0.f;
    if (o < c && i < c) {
      const float g = fmaxf(gamma[(int64_t)o * c + i], gb);
      v = __fsub_rn(__fmul_rn(g, g), ped);
    }
    w[idx] = from_f<T>(v);
  }
  if (idx < c) {
    const float b = fmaxf(beta[idx], bb);
    beta_out[idx] = __fsub_rn(__fmul_rn(b, b), ped);
  }
}

// One wave per pixel; two-pass mean / biased variance in fp32.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(const T* __restrict__ x, int npix, int c, int ldx,
                                                        const float* __restrict__ wt, const float* __restrict__ bs,
                                                        float eps, T* __restrict__ y, int ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= npix) return;
  const T* xp = x + p * ldx;
  float s = 0.f;
  for (int k = lane; k < c; k += 64) s += to_f(xp[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)c;
  float v = 0.f;
  for (int k = lane; k < c; k += 64) {
    const float d = to_f(xp[k]) - mean;
    v += d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const float rstd = 1.0f / sqrtf(v / (float)c + eps);
  T* yp = y + p * ldy;
  for (int k = lane; k < c; k += 64) yp[k] = from_f<T>((to_f(xp[k]) - mean) * rstd * wt[k] + bs[k]);
}

}  // namespace lic

extern "C" int lic_gdn_prepare(int32_t dtype, const float* beta, const float* gamma, int32_t c, float beta_bound,
                               float gamma_bound, float pedestal, void* wgt_out, int32_t cpad, int32_t copad,
                               float* beta_out, lic_stream_t stream) {
  using namespace lic;
  if (cpad < c || copad < c) return fail("gdn_prepare: padding smaller than C");
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = (int64_t)copad * cpad;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(gdn_prepare_kernel<float>, dim3(blocks), dim3(256), 0, s, beta, gamma, c, beta_bound,
                       gamma_bound, pedestal, (float*)wgt_out, cpad, copad, beta_out);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(gdn_prepare_kernel<half_t>, dim3(blocks), dim3(256), 0, s, beta, gamma, c, beta_bound,
                       gamma_bound, pedestal, (half_t*)wgt_out, cpad, copad, beta_out);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(gdn_prepare_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, beta, gamma, c, beta_bound,
                       gamma_bound, pedestal, (bf16_t*)wgt_out, cpad, copad, beta_out);
  else
    return fail("gdn_prepare: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_layernorm_fwd(int32_t dtype, const void* x, int32_t npix, int32_t c, int32_t ldx,
                                 const float* weight, const float* bias, float eps, void* y, int32_t ldy,
                                 lic_stream_t stream) {
  using namespace lic;
  if (npix <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const unsigned blocks = (unsigned)((npix + 3) / 4);
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(layernorm_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, npix, c, ldx, weight,
                       bias, eps, (float*)y, ldy);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(layernorm_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, npix, c, ldx,
                       weight, bias, eps, (half_t*)y, ldy);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(layernorm_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)x, npix, c, ldx,
                       weight, bias, eps, (bf16_t*)y, ldy);
  else
    return fail("layernorm: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}
