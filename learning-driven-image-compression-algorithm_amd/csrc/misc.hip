// Layout conversion and small elementwise / pooling helpers (gfx950).
#include "lic_common.h"

namespace lic {

// NCHW fp32 -> NHWC view (dtype T). One thread per output element, reads
// coalesced along w for each channel plane via a 2-D grid.
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int n, int c, int h, int w, T* __restrict__ y,
                                    int ldy, int cpad) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * cpad * h * w;
  if (idx >= total) return;
  // idx enumerates NHWC order: ((b*h + yy)*w + xx)*cpad + k; channels [c, cpad) are zero-filled
  const int k = (int)(idx % cpad);
  const int64_t pix = idx / cpad;
  const int xx = (int)(pix % w);
  const int64_t t = pix / w;
  const int yy = (int)(t % h);
  const int b = (int)(t / h);
  y[pix * ldy + k] = k < c ? from_f<T>(x[(((int64_t)b * c + k) * h + yy) * w + xx]) : from_f<T>(0.f);
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ x, int n, int h, int w, int c, int ldx, float* __restrict__ y) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * c * h * w;
  if (idx >= total) return;
  // idx enumerates NCHW order
  const int xx = (int)(idx % w);
  int64_t t = idx / w;
  const int yy = (int)(t % h);
  t /= h;
  const int k = (int)(t % c);
  const int b = (int)(t / c);
  y[idx] = to_f(x[(((int64_t)b * h + yy) * w + xx) * ldx + k]);
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, int lda, const T* __restrict__ b, int ldb, int npix, int c,
                           T* __restrict__ y, int ldy) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int k = (int)(idx - p * c);
  y[p * ldy + k] = from_f<T>(to_f(a[p * lda + k]) + to_f(b[p * ldb + k]));
}

template <typename TI, typename TO>
__global__ void copy_kernel(const TI* __restrict__ x, int ldx, int npix, int c, TO* __restrict__ y, int ldy) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int k = (int)(idx - p * c);
  y[p * ldy + k] = from_f<TO>(to_f(x[p * ldx + k]));
}

// AdaptiveAvgPool2d(1): one block per (image, 64-channel group); threads stride pixels.
template <typename T>
__global__ __launch_bounds__(256) void avgpool_kernel(const T* __restrict__ x, int hw, int c, int ldx,
                                                      T* __restrict__ y, int ldy) {
  __shared__ float red[4][64];
  const int b = blockIdx.y;
  const int k = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  float s = 0.f;
  if (k < c)
    for (int p = part; p < hw; p += 4) s += to_f(x[((int64_t)b * hw + p) * ldx + k]);
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && k < c) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    y[(int64_t)b * ldy + k] = from_f<T>(t / (float)hw);
  }
}

}  // namespace lic

using namespace lic;

#define DISPATCH_T(dtype, NAME, ...)                                   \
  do {                                                                 \
    if ((dtype) == LIC_F32) {                                          \
      typedef float T;                                                 \
      __VA_ARGS__;                                                     \
    } else if ((dtype) == LIC_F16) {                                   \
      typedef half_t T;                                                \
      __VA_ARGS__;                                                     \
    } else if ((dtype) == LIC_BF16) {                                  \
      typedef bf16_t T;                                                \
      __VA_ARGS__;                                                     \
    } else                                                             \
      return fail(std::string(NAME) + ": bad dtype");                  \
  } while (0)

static inline unsigned nblk(int64_t total) { return (unsigned)((total + 255) / 256); }

extern "C" int lic_nchw_to_nhwc(int32_t dtype, const float* x, int32_t n, int32_t c, int32_t h, int32_t w, void* y,
                                int32_t ldy, int32_t cpad, lic_stream_t stream) {
  if (cpad < c || cpad > ldy) return fail("nchw_to_nhwc: need c <= cpad <= ldy");
  const int64_t total = (int64_t)n * cpad * h * w;
  if (!total) return 0;
  DISPATCH_T(dtype, "nchw_to_nhwc",
             hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, x, n, c,
                                h, w, (T*)y, ldy, cpad));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_nhwc_to_nchw(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ldx,
                                float* y, lic_stream_t stream) {
  const int64_t total = (int64_t)n * c * h * w;
  if (!total) return 0;
  DISPATCH_T(dtype, "nhwc_to_nchw",
             hipLaunchKernelGGL(nhwc_to_nchw_kernel<T>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                (const T*)x, n, h, w, c, ldx, y));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_add(int32_t dtype, const void* a, int32_t lda, const void* b, int32_t ldb, int32_t npix, int32_t c,
                       void* y, int32_t ldy, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  DISPATCH_T(dtype, "add",
             hipLaunchKernelGGL(add_kernel<T>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, (const T*)a, lda,
                                (const T*)b, ldb, npix, c, (T*)y, ldy));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_copy(int32_t dtype_in, const void* x, int32_t ldx, int32_t npix, int32_t c, int32_t dtype_out,
                        void* y, int32_t ldy, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == LIC_F32 && dtype_out == LIC_F32)
    hipLaunchKernelGGL((copy_kernel<float, float>), dim3(nblk(total)), dim3(256), 0, s, (const float*)x, ldx, npix, c,
                       (float*)y, ldy);
  else if (dtype_in == LIC_F32 && dtype_out == LIC_F16)
    hipLaunchKernelGGL((copy_kernel<float, half_t>), dim3(nblk(total)), dim3(256), 0, s, (const float*)x, ldx, npix, c,
                       (half_t*)y, ldy);
  else if (dtype_in == LIC_F16 && dtype_out == LIC_F32)
    hipLaunchKernelGGL((copy_kernel<half_t, float>), dim3(nblk(total)), dim3(256), 0, s, (const half_t*)x, ldx, npix,
                       c, (float*)y, ldy);
  else if (dtype_in == LIC_F16 && dtype_out == LIC_F16)
    hipLaunchKernelGGL((copy_kernel<half_t, half_t>), dim3(nblk(total)), dim3(256), 0, s, (const half_t*)x, ldx, npix,
                       c, (half_t*)y, ldy);
  else if (dtype_in == LIC_F32 && dtype_out == LIC_BF16)
    hipLaunchKernelGGL((copy_kernel<float, bf16_t>), dim3(nblk(total)), dim3(256), 0, s, (const float*)x, ldx, npix, c,
                       (bf16_t*)y, ldy);
  else if (dtype_in == LIC_BF16 && dtype_out == LIC_F32)
    hipLaunchKernelGGL((copy_kernel<bf16_t, float>), dim3(nblk(total)), dim3(256), 0, s, (const bf16_t*)x, ldx, npix,
                       c, (float*)y, ldy);
  else if (dtype_in == LIC_BF16 && dtype_out == LIC_BF16)
    hipLaunchKernelGGL((copy_kernel<bf16_t, bf16_t>), dim3(nblk(total)), dim3(256), 0, s, (const bf16_t*)x, ldx, npix,
                       c, (bf16_t*)y, ldy);
  else
    return fail("copy: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_avgpool(int32_t dtype, const void* x, int32_t n, int32_t hw, int32_t c, int32_t ldx, void* y,
                           int32_t ldy, lic_stream_t stream) {
  if (!n || !c) return 0;
  dim3 grid((c + 63) / 64, n);
  DISPATCH_T(dtype, "avgpool",
             hipLaunchKernelGGL(avgpool_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)x, hw, c, ldx, (T*)y,
                                ldy));
  LIC_CHECK_LAUNCH();
  return 0;
}

namespace lic {

// Patch (im2col) map of a small-channel input for one conv's taps, fp32:
//   y[b, i, j, t*c + ch] = x[b, i*s + dy[t], j*s + dx[t], ch]   (zero outside the map),
//   channels [ntaps*c, cpad) zero.  One thread per output element.
struct PatchTaps {
  int8_t dy[32], dx[32];
};

__global__ void patches_kernel(const float* __restrict__ x, int n, int h, int w, int c, int ldx, int ho, int wo,
                               int s, int ntaps, PatchTaps tp, float* __restrict__ y, int ldy, int cpad) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)n * ho * wo * cpad;
  if (idx >= total) return;
  const int k = (int)(idx % cpad);
  const int64_t pix = idx / cpad;
  const int j = (int)(pix % wo);
  const int64_t q = pix / wo;
  const int i = (int)(q % ho);
  const int b = (int)(q / ho);
  const int t = k / c, ch = k - t * c;
  float v = 0.f;
  if (t < ntaps) {
    const int iy = i * s + tp.dy[t], ix = j * s + tp.dx[t];
    if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) v = x[(((int64_t)b * h + iy) * w + ix) * ldx + ch];
  }
  y[pix * ldy + k] = v;
}

}  // namespace lic

extern "C" int lic_patches(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ldx,
                           int32_t ho, int32_t wo, int32_t stride, int32_t ntaps, const int8_t* dy, const int8_t* dx,
                           void* y, int32_t ldy, int32_t cpad, lic_stream_t stream) {
  using namespace lic;
  if (dtype != LIC_F32) return fail("patches: fp32 only");
  if (!x || !y || !dy || !dx) return fail("patches: null pointer");
  if (n < 1 || h < 1 || w < 1 || c < 1 || ho < 1 || wo < 1 || stride < 1 || ntaps < 1 || ntaps > 32)
    return fail("patches: bad geometry");
  if (ntaps * c > cpad || ldy < cpad || ldx < c) return fail("patches: ntaps*c must fit cpad <= ldy, c <= ldx");
  PatchTaps tp{};
  for (int t = 0; t < ntaps; ++t) {
    tp.dy[t] = dy[t];
    tp.dx[t] = dx[t];
  }
  const int64_t total = (int64_t)n * ho * wo * cpad;
  hipLaunchKernelGGL(patches_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const float*)x, n, h, w, c, ldx, ho, wo, stride, ntaps, tp, (float*)y, ldy, cpad);
  LIC_CHECK_LAUNCH();
  return 0;
}
