// On-device rate estimate, quantisation and distortion metrics (gfx950).
// No host round trip: partial sums are written per block in fp64 and reduced by
// a single-block finalize kernel in a fixed order (deterministic).
#include "lic_common.h"

namespace lic {

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k];
  return t;  // valid in thread 0
}

// compressai GaussianConditional (eval / 'dequantize'):
//   outputs = round(y - mu) + mu ; values = |outputs - mu| ; s = max(scale, 0.11)
//   L = 0.5 erfc(-(2^-.5) (.5 - v)/s) - 0.5 erfc(-(2^-.5) (-.5 - v)/s), max(L, 1e-9)
template <typename T>
__global__ __launch_bounds__(256) void gauss_rate_kernel(const lic_rate_args a) {
  __shared__ double red[4];
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)a.npix * a.c;
  double acc = 0.0;
  if (idx < total) {
    const int64_t p = idx / a.c;
    const int k = (int)(idx - p * a.c);
    const float y = to_f(((const T*)a.y)[p * a.ldy + k]);
    const float mu = to_f(((const T*)a.mu)[p * a.ldmu + k]);
    const float sc = to_f(((const T*)a.scale)[p * a.ldsc + k]);
    const float q = rintf(__fsub_rn(y, mu));
    const float yq = __fadd_rn(q, mu);
    if (a.symbols) a.symbols[p * a.ldsym + k] = (int32_t)q;
    if (a.yq) ((T*)a.yq)[p * a.ldyq + k] = from_f<T>(yq);
    if (a.yq2) ((T*)a.yq2)[p * a.ldyq2 + k] = from_f<T>(yq);
    const float v = fabsf(__fsub_rn(yq, mu));
    const float s = fmaxf(sc, a.scale_bound);
    const float cst = -0.70710678118654752440f;
    const float upper = 0.5f * erfcf(cst * __fdiv_rn(__fsub_rn(0.5f, v), s));
    const float lower = 0.5f * erfcf(cst * __fdiv_rn(__fsub_rn(-0.5f, v), s));
    float L = __fsub_rn(upper, lower);
    L = fmaxf(L, a.likelihood_bound);
    if (a.likelihood) a.likelihood[p * a.ldlik + k] = L;
    acc = (double)logf(L);
  }
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) a.partials[blockIdx.x] = t;
}

template <typename T>
__global__ void quantize_median_kernel(const T* __restrict__ z, int npix, int c, int ldz, const float* __restrict__ m,
                                       T* __restrict__ out, int ldo) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int k = (int)(idx - p * c);
  const float zz = to_f(z[p * ldz + k]);
  const float med = m ? m[k] : 0.f;
  out[p * ldo + k] = from_f<T>(__fadd_rn(rintf(__fsub_rn(zz, med)), med));
}

__global__ __launch_bounds__(256) void bpp_finalize_kernel(const double* __restrict__ parts, int n, double num_pixels,
                                                           float* bpp, double* sum_out) {
  __shared__ double red[4];
  double v = 0.0;
  for (int k = threadIdx.x; k < n; k += 256) v += parts[k];
  const double t = block_sum_f64(v, red);
  if (threadIdx.x == 0) {
    if (sum_out) sum_out[0] = t;
    bpp[0] = (float)(t / (-0.69314718055994530942 * num_pixels));
  }
}

// xt = clamp(tanh(sum_c w[b][o][c] xtil[c]), -1, 1); NCHW fp32 x_rec; per-image
// squared error of the 8-bit reconstructions (net_ga.py:1137-1141).
template <typename T>
__global__ __launch_bounds__(256) void syntax_recon_kernel(const T* __restrict__ xtil, int h, int w, int cin, int ldx, int ldw,
                                                           const T* __restrict__ wgen, const float* __restrict__ x,
                                                           float* __restrict__ xrec, double* __restrict__ parts,
                                                           int parts_per_img) {
  __shared__ double red[4];
  __shared__ float ws[3 * 64];
  const int b = blockIdx.y;
  for (int k = threadIdx.x; k < 3 * cin; k += 256) ws[k] = to_f(wgen[(int64_t)b * ldw + k]);
  __syncthreads();
  const int64_t hw = (int64_t)h * w;
  double acc = 0.0;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < hw; p += (int64_t)parts_per_img * 256) {
    const T* xp = xtil + ((int64_t)b * hw + p) * ldx;
    float o[3] = {0.f, 0.f, 0.f};
    for (int c = 0; c < cin; ++c) {
      const float v = to_f(xp[c]);
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] += ws[k * cin + c] * v;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float t = tanhf(o[k]);
      t = fminf(fmaxf(t, -1.f), 1.f);
      const int64_t off = ((int64_t)b * 3 + k) * hw + p;
      xrec[off] = t;
      const float gt = rintf(__fmul_rn(__fadd_rn(x[off], 1.f), 127.5f));
      float xh = __fmul_rn(__fadd_rn(t, 1.f), 127.5f);
      xh = rintf(fminf(fmaxf(xh, 0.f), 255.f));
      const float d = __fsub_rn(xh, gt);
      acc += (double)(d * d);
    }
  }
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) parts[(int64_t)b * parts_per_img + blockIdx.x] = t;
}

__global__ void psnr_finalize_kernel(const double* __restrict__ parts, int n, int ppi, double count, float* v_mse,
                                     float* v_psnr) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double ps = 0.0;
  for (int b = 0; b < n; ++b) {
    double s = 0.0;
    for (int k = 0; k < ppi; ++k) s += parts[(int64_t)b * ppi + k];
    const float mse = (float)(s / count);
    v_mse[b] = mse;
    ps += (double)(20.0f * log10f(255.0f / sqrtf(mse)));
  }
  v_psnr[0] = (float)(ps / n);
}

}  // namespace lic

extern "C" int lic_gauss_rate_fwd(const lic_rate_args* a, lic_stream_t stream) {
  using namespace lic;
  if (!a || !a->y || !a->mu || !a->scale || !a->partials) return fail("rate: null tensor");
  const int64_t total = (int64_t)a->npix * a->c;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > a->max_parts) return fail("rate: partials buffer too small");
  if (blocks == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->dtype == LIC_F32)
    hipLaunchKernelGGL(gauss_rate_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, *a);
  else if (a->dtype == LIC_F16)
    hipLaunchKernelGGL(gauss_rate_kernel<half_t>, dim3((unsigned)blocks), dim3(256), 0, s, *a);
  else if (a->dtype == LIC_BF16)
    hipLaunchKernelGGL(gauss_rate_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, *a);
  else
    return fail("rate: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_quantize_median(int32_t dtype, const void* z, int32_t npix, int32_t c, int32_t ldz,
                                   const float* medians, void* out, int32_t ldo, lic_stream_t stream) {
  using namespace lic;
  const int64_t total = (int64_t)npix * c;
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(quantize_median_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)z, npix, c, ldz,
                       medians, (float*)out, ldo);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(quantize_median_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)z, npix, c, ldz,
                       medians, (half_t*)out, ldo);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(quantize_median_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)z, npix, c, ldz,
                       medians, (bf16_t*)out, ldo);
  else
    return fail("quantize: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_bpp_finalize(const double* partials, int32_t nparts, double num_pixels, float* bpp_out,
                                double* sum_out, lic_stream_t stream) {
  using namespace lic;
  hipLaunchKernelGGL(bpp_finalize_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, partials, nparts, num_pixels,
                     bpp_out, sum_out);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_syntax_recon_fwd(int32_t dtype, const void* xtil, int32_t n, int32_t h, int32_t w, int32_t cin,
                                    int32_t ldx, const void* wgen, int32_t ldw, const float* x, float* x_rec,
                                    double* sqerr_partials, int32_t parts_per_img, lic_stream_t stream) {
  using namespace lic;
  if (cin > 64) return fail("recon: cin > 64");
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(parts_per_img, n);
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(syntax_recon_kernel<float>, grid, dim3(256), 0, s, (const float*)xtil, h, w, cin, ldx, ldw,
                       (const float*)wgen, x, x_rec, sqerr_partials, parts_per_img);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(syntax_recon_kernel<half_t>, grid, dim3(256), 0, s, (const half_t*)xtil, h, w, cin, ldx, ldw,
                       (const half_t*)wgen, x, x_rec, sqerr_partials, parts_per_img);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(syntax_recon_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)xtil, h, w, cin, ldx, ldw,
                       (const bf16_t*)wgen, x, x_rec, sqerr_partials, parts_per_img);
  else
    return fail("recon: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_psnr_finalize(const double* sqerr_partials, int32_t n, int32_t parts_per_img, double count,
                                 float* v_mse, float* v_psnr, lic_stream_t stream) {
  using namespace lic;
  hipLaunchKernelGGL(psnr_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, sqerr_partials, n,
                     parts_per_img, count, v_mse, v_psnr);
  LIC_CHECK_LAUNCH();
  return 0;
}
