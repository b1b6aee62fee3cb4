// Fused ResidualBottleneck(3) of the analysis transform (net_ga.py:89-103, N = 3):
//   out = x + conv1x1_{1->3}( GELU( conv3x3_{1->1}( GELU( conv1x1_{3->1}(x) ) ) ) )
// One thread per pixel computes the 1-channel intermediate on its 3x3
// neighbourhood (zero padded like the reference's conv3x3), so the whole block is
// one HBM pass.  The output view is written over its full pixel stride `ldy`:
// channels 3..ldy-1 are set to zero, which lets the following 3->192 convolutions
// treat the image as an 8-channel (f16) / 4-channel (f32) zero-padded tensor and
// run on MFMA.  Also used for the 256x256 NCHW -> NHWC input conversion padding.
#include "lic_common.h"

namespace lic {

// p: w1[3], b1, w2[9], b2, w3[3], b3[3]  (20 floats)
template <typename T>
__global__ __launch_bounds__(256) void rb3_kernel(const T* __restrict__ x, int n, int h, int w, int ldx,
                                                  const float* __restrict__ p, T* __restrict__ y, int ldy) {
  __shared__ float sp[20];
  if (threadIdx.x < 20) sp[threadIdx.x] = p[threadIdx.x];
  __syncthreads();
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * h * w;
  if (idx >= total) return;
  const int xx = (int)(idx % w);
  const int64_t t = idx / w;
  const int yy = (int)(t % h);
  const int b = (int)(t / h);
  float acc2 = 0.f;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int iy = yy + ky - 1, ix = xx + kx - 1;
      float t1 = 0.f;
      if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
        const T* q = x + (((int64_t)b * h + iy) * w + ix) * ldx;
        const float s = sp[3] + sp[0] * to_f(q[0]) + sp[1] * to_f(q[1]) + sp[2] * to_f(q[2]);
        t1 = gelu_f(s);
      }
      acc2 += sp[4 + ky * 3 + kx] * t1;
    }
  }
  const float t2 = gelu_f(sp[13] + acc2);
  const T* q = x + idx * ldx;
  T* o = y + idx * ldy;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c] = from_f<T>(to_f(q[c]) + (sp[17 + c] + sp[14 + c] * t2));
  for (int c = 3; c < ldy; ++c) o[c] = from_f<T>(0.f);
}

}  // namespace lic

extern "C" int lic_rb3_fwd(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t ldx,
                           const float* params, void* y, int32_t ldy, lic_stream_t stream) {
  using namespace lic;
  if (ldx < 3 || ldy < 3) return fail("rb3: views need >= 3 channels");
  const int64_t total = (int64_t)n * h * w;
  if (!total) return 0;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(rb3_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, n, h, w, ldx, params,
                       (float*)y, ldy);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(rb3_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, n, h, w, ldx, params,
                       (half_t*)y, ldy);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(rb3_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)x, n, h, w, ldx, params,
                       (bf16_t*)y, ldy);
  else
    return fail("rb3: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}
