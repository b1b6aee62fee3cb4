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


// NB consecutive ResidualBottleneck(3) blocks (the a_model's first three, net_ga.py:262-264) in one
// launch.  A workgroup owns a 32 x 32 output tile; its (32 + 2 NB)^2 frame of x (3 channels, fp32 in
// LDS) is loaded once, and block k computes its 1-channel GELU(1x1) map once per frame pixel (the
// single-block kernel above recomputes it for each of the 9 taps of every pixel), then the 3x3 +
// GELU + 1x1 + residual on the frame shrunk by one pixel, in place.  Every value is rounded to T
// between blocks exactly where the one-block launches store it, and each expression is the one of
// rb3_kernel, so the chain equals NB rb3 launches (tests/test_gpu_ops2.py).  The output pixels are
// written whole (channels 3..ldy-1 zero), 16 B at a time when ldy * sizeof(T) == 16.
template <typename T, int NB>
__global__ __launch_bounds__(256) void rb3_chain_kernel(const T* __restrict__ x, int n, int h, int w, int ldx,
                                                        const float* __restrict__ p, T* __restrict__ y, int ldy) {
  constexpr int TS = 32, F = TS + 2 * NB, FF = F * F;
  __shared__ float sp[NB * 20];
  __shared__ float xs[3][FF];
  __shared__ float t1s[FF];
  const int tid = threadIdx.x;
  for (int i = tid; i < NB * 20; i += 256) sp[i] = p[i];
  const int tiles_x = (w + TS - 1) / TS, tiles_y = (h + TS - 1) / TS;
  int bid = blockIdx.x;
  const int tx0 = (bid % tiles_x) * TS;
  bid /= tiles_x;
  const int ty0 = (bid % tiles_y) * TS;
  const int b = bid / tiles_y;
  for (int q = tid; q < FF; q += 256) {
    const int iy = ty0 - NB + q / F, ix = tx0 - NB + q % F;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
      const T* src = x + (((int64_t)b * h + iy) * w + ix) * ldx;
      v0 = to_f(src[0]);
      v1 = to_f(src[1]);
      v2 = to_f(src[2]);
    }
    xs[0][q] = v0;
    xs[1][q] = v1;
    xs[2][q] = v2;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const float* P = sp + 20 * k;
    // the block's 1-channel map on frame [k, F - k)^2 (zero outside the image: conv3x3's padding)
    const int o = k, S1 = F - 2 * k;
    for (int q = tid; q < S1 * S1; q += 256) {
      const int fy = o + q / S1, fx = o + q % S1, f = fy * F + fx;
      const int iy = ty0 - NB + fy, ix = tx0 - NB + fx;
      float t1 = 0.f;
      if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
        const float s = P[3] + P[0] * xs[0][f] + P[1] * xs[1][f] + P[2] * xs[2][f];
        t1 = gelu_f(s);
      }
      t1s[f] = t1;
    }
    __syncthreads();
    const int S2 = S1 - 2;
    for (int q = tid; q < S2 * S2; q += 256) {
      const int fy = o + 1 + q / S2, fx = o + 1 + q % S2, f = fy * F + fx;
      float acc2 = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc2 += P[4 + ky * 3 + kx] * t1s[f + (ky - 1) * F + (kx - 1)];
      const float t2 = gelu_f(P[13] + acc2);
      float r[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) r[c] = to_f(from_f<T>(xs[c][f] + (P[17 + c] + P[14 + c] * t2)));
      if (k + 1 < NB) {
#pragma unroll
        for (int c = 0; c < 3; ++c) xs[c][f] = r[c];
      } else {
        const int iy = ty0 - NB + fy, ix = tx0 - NB + fx;
        if (iy < h && ix < w) {
          T* dst = y + (((int64_t)b * h + iy) * w + ix) * ldy;
          if (ldy * (int)sizeof(T) == 16 && ((uintptr_t)dst & 15) == 0) {
            T v[16 / sizeof(T)];
#pragma unroll
            for (int c = 0; c < (int)(16 / sizeof(T)); ++c) v[c] = from_f<T>(c < 3 ? r[c] : 0.f);
            *(uint4*)dst = *(const uint4*)v;
          } else {
            for (int c = 0; c < ldy; ++c) dst[c] = from_f<T>(c < 3 ? r[c] : 0.f);
          }
        }
      }
    }
    __syncthreads();
  }
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

extern "C" int lic_rb3_chain_fwd(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t ldx,
                                 const float* params, int32_t nblk, void* y, int32_t ldy, lic_stream_t stream) {
  using namespace lic;
  if (ldx < 3 || ldy < 3) return fail("rb3_chain: views need >= 3 channels");
  if (nblk < 1 || nblk > 3) return fail("rb3_chain: 1..3 blocks");
  if (x == y) return fail("rb3_chain: the output must not alias the input (other tiles read its halo)");
  const int64_t tiles = (int64_t)n * ((h + 31) / 32) * ((w + 31) / 32);
  if (!tiles) return 0;
  if (tiles >= (1LL << 31)) return fail("rb3_chain: grid too large");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)tiles);
#define RB3C_LAUNCH(T)                                                                                   \
  if (nblk == 1) hipLaunchKernelGGL((rb3_chain_kernel<T, 1>), grid, dim3(256), 0, s, (const T*)x, n, h, w, ldx, params, (T*)y, ldy); \
  else if (nblk == 2) hipLaunchKernelGGL((rb3_chain_kernel<T, 2>), grid, dim3(256), 0, s, (const T*)x, n, h, w, ldx, params, (T*)y, ldy); \
  else hipLaunchKernelGGL((rb3_chain_kernel<T, 3>), grid, dim3(256), 0, s, (const T*)x, n, h, w, ldx, params, (T*)y, ldy);
  if (dtype == LIC_F32) {
    RB3C_LAUNCH(float)
  } else if (dtype == LIC_F16) {
    RB3C_LAUNCH(half_t)
  } else if (dtype == LIC_BF16) {
    RB3C_LAUNCH(bf16_t)
  } else {
    return fail("rb3_chain: bad dtype");
  }
#undef RB3C_LAUNCH
  LIC_CHECK_LAUNCH();
  return 0;
}
