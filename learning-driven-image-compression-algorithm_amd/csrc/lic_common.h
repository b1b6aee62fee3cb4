// Shared device/host helpers for liblic (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "../../include/lic.h"

namespace lic {

typedef _Float16 half_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// thread-local error string (lic_last_error)
void set_error(const std::string& s);
int fail(const std::string& s);

#define LIC_CHECK_LAUNCH()                                                   \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) return ::lic::fail(std::string("HIP launch: ") + hipGetErrorString(_e)); \
  } while (0)

template <typename T> struct DT;
template <> struct DT<float> { static constexpr int id = LIC_F32; };
template <> struct DT<half_t> { static constexpr int id = LIC_F16; };

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(half_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ half_t from_f<half_t>(float v) { return (half_t)v; }

// exact (erf) GELU, nn.GELU() default
__device__ __forceinline__ float gelu_f(float v) { return 0.5f * v * (1.0f + erff(v * 0.70710678118654752f)); }
__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + expf(-v)); }

__device__ __forceinline__ float apply_act(float v, int act, float slope) {
  switch (act) {
    case LIC_ACT_RELU: return v > 0.f ? v : 0.f;
    case LIC_ACT_LRELU: return v > 0.f ? v : v * slope;
    case LIC_ACT_GELU: return gelu_f(v);
    case LIC_ACT_ROUND: return rintf(v);
    default: return v;
  }
}

__device__ __forceinline__ float apply_pro(float v, int pro) {
  if (pro == LIC_PRO_SQUARE) return v * v;
  if (pro == LIC_PRO_ABS) return fabsf(v);
  return v;
}

// Shared conv epilogue (MFMA and direct kernels): acc -> output element value.
template <typename T>
__device__ __forceinline__ float conv_epilogue(const lic_conv_args& a, float acc, int nb, int64_t pix, int n) {
  float v = acc + (a.bias ? a.bias[nb] : 0.f);
  switch (a.epi) {
    case LIC_EPI_GDN_DIV: {
      float g = to_f(((const T*)a.g)[pix * a.ldg + n]);
      v = g / sqrtf(v);
      if (a.r1) v += to_f(((const T*)a.r1)[pix * a.ldr1 + n]);
      return v;
    }
    case LIC_EPI_GDN_RSQRT: {
      float g = to_f(((const T*)a.g)[pix * a.ldg + n]);
      v = g * (1.0f / sqrtf(v));
      if (a.r1) v += to_f(((const T*)a.r1)[pix * a.ldr1 + n]);
      return v;
    }
    case LIC_EPI_GDN_SQRT: {
      float g = to_f(((const T*)a.g)[pix * a.ldg + n]);
      v = g * sqrtf(v);
      if (a.r1) v += to_f(((const T*)a.r1)[pix * a.ldr1 + n]);
      return v;
    }
    case LIC_EPI_RES_ACT: {
      if (a.r1) v += to_f(((const T*)a.r1)[pix * a.ldr1 + n]);
      return apply_act(v, a.act, a.slope);
    }
    default: break;
  }
  v = apply_act(v, a.act, a.slope);
  if (a.epi == LIC_EPI_HALF_TANH) {
    float r2 = to_f(((const T*)a.r2)[pix * a.ldr2 + n]);
    return r2 + 0.5f * tanhf(v);
  }
  if (a.r1) v += to_f(((const T*)a.r1)[pix * a.ldr1 + n]);
  if (a.epi == LIC_EPI_GATE) {
    float g = to_f(((const T*)a.g)[pix * a.ldg + n]);
    float r2 = to_f(((const T*)a.r2)[pix * a.ldr2 + n]);
    v = g * sigmoid_f(v) + r2;
  }
  return v;
}

// Map output lattice index (b, i, j) and channel n to the destination pixel index
// and channel (handles PixelShuffle(2) fusion).
__device__ __forceinline__ void out_coord(const lic_conv_args& a, int b, int i, int j, int n,
                                          int64_t& pix, int& ch) {
  int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
  if (a.out_shuffle == 2) {
    oy = 2 * oy + ((n >> 1) & 1);
    ox = 2 * ox + (n & 1);
    ch = n >> 2;
  } else {
    ch = n;
  }
  pix = ((int64_t)b * a.ho + oy) * a.wo + ox;
}

}  // namespace lic
