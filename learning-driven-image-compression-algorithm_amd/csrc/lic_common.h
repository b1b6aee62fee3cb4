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

// Vector of V = 16 / sizeof(T) elements (one 16-byte access).
template <typename T> struct Vec16 { static constexpr int V = 16 / (int)sizeof(T); };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* f) {
  constexpr int V = Vec16<T>::V;
  const u32x4 raw = *(const u32x4*)p;
  const T* e = (const T*)&raw;
#pragma unroll
  for (int k = 0; k < V; ++k) f[k] = to_f(e[k]);
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* f) {
  constexpr int V = Vec16<T>::V;
  u32x4 raw;
  T* e = (T*)&raw;
#pragma unroll
  for (int k = 0; k < V; ++k) e[k] = from_f<T>(f[k]);
  *(u32x4*)p = raw;
}

// True when every activation view of the launch allows 16-byte vector accesses.
template <typename T>
__device__ __forceinline__ bool epi_vec_ok(const lic_conv_args& a) {
  constexpr int V = Vec16<T>::V;
  auto al = [](const void* p, int ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && ld % V == 0); };
  return a.out_shuffle == 0 && a.co % V == 0 && al(a.y, a.ldy) && al(a.y2, a.ldy2) && al(a.r1, a.ldr1) &&
         al(a.g, a.ldg) && al(a.r2, a.ldr2);
}

// Finish one 32x32 fp32 accumulator tile staged in LDS (row stride 33 floats):
// rows are tile pixels (destination pixel base in rowpix[], -1 = outside), columns
// output channels n0 .. n0+31.  Vector path: each lane handles 16 contiguous bytes
// of one pixel (bias, act, residual/gate/GDN/half-tanh in fp32, one 16-B store);
// scalar path for pixel-shuffle / unaligned views / channel tails.
template <typename T>
__device__ __forceinline__ void epilogue_tile(const lic_conv_args& a, const float* ct, const int* rowpix, int n0,
                                              int lane, bool vec_ok) {
  constexpr int V = Vec16<T>::V;
  constexpr int CPR = 32 / V;   // 16-B chunks per tile row
  constexpr int RPP = 64 / CPR; // rows per pass
  T* __restrict__ yg = (T*)a.y;
  T* __restrict__ y2g = (T*)a.y2;
  if (vec_ok) {
#pragma unroll
    for (int pass = 0; pass < 32 / RPP; ++pass) {
      const int row = pass * RPP + lane / CPR;
      const int cc = lane % CPR;
      const int base = rowpix[row];
      const int n = n0 + cc * V;
      if (base < 0 || n >= a.co) continue;
      const int64_t pix = base;
      float v[V], t[V];
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] = ct[row * 33 + cc * V + k] + (a.bias ? a.bias[n + k] : 0.f);
      switch (a.epi) {
        case LIC_EPI_GDN_DIV:
        case LIC_EPI_GDN_RSQRT:
        case LIC_EPI_GDN_SQRT:
          load_vec<T>((const T*)a.g + pix * a.ldg + n, t);
#pragma unroll
          for (int k = 0; k < V; ++k)
            v[k] = a.epi == LIC_EPI_GDN_DIV ? t[k] / sqrtf(v[k])
                 : (a.epi == LIC_EPI_GDN_RSQRT ? t[k] * (1.0f / sqrtf(v[k])) : t[k] * sqrtf(v[k]));
          if (a.r1) {
            load_vec<T>((const T*)a.r1 + pix * a.ldr1 + n, t);
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] += t[k];
          }
          break;
        case LIC_EPI_RES_ACT:
          if (a.r1) {
            load_vec<T>((const T*)a.r1 + pix * a.ldr1 + n, t);
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] += t[k];
          }
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = apply_act(v[k], a.act, a.slope);
          break;
        case LIC_EPI_HALF_TANH:
          load_vec<T>((const T*)a.r2 + pix * a.ldr2 + n, t);
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = t[k] + 0.5f * tanhf(apply_act(v[k], a.act, a.slope));
          break;
        default:
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = apply_act(v[k], a.act, a.slope);
          if (a.r1) {
            load_vec<T>((const T*)a.r1 + pix * a.ldr1 + n, t);
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] += t[k];
          }
          if (a.epi == LIC_EPI_GATE) {
            float r2[V];
            load_vec<T>((const T*)a.g + pix * a.ldg + n, t);
            load_vec<T>((const T*)a.r2 + pix * a.ldr2 + n, r2);
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] = t[k] * sigmoid_f(v[k]) + r2[k];
          }
          break;
      }
      store_vec<T>(yg + pix * a.ldy + n, v);
      if (y2g) store_vec<T>(y2g + pix * a.ldy2 + n, v);
    }
  } else {
    const int erow = lane >> 1, ecol = (lane & 1) * 16;
    const int base = rowpix[erow];
    if (base < 0) return;
    for (int c = 0; c < 16; ++c) {
      const int n = n0 + ecol + c;
      if (n >= a.co) break;
      int64_t pix = base;
      int ch = n;
      if (a.out_shuffle == 2) {
        pix += ((n >> 1) & 1) * a.wo + (n & 1);
        ch = n >> 2;
      }
      const float v = conv_epilogue<T>(a, ct[erow * 33 + ecol + c], n, pix, ch);
      yg[pix * a.ldy + ch] = from_f<T>(v);
      if (y2g) y2g[pix * a.ldy2 + ch] = from_f<T>(v);
    }
  }
}

template <typename T>
int conv_halo_dispatch(const lic_conv_args& a, hipStream_t s, int& status);

}  // namespace lic
