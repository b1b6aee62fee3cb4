// Split-precision fp32 convolution modes shared by the split kernels (lic_conv_args.mfma_mode).
//
// mfma_mode 2, "fp32x6" (bf16 parts, fp32 grade):
//   x = x0 + x1 + x2, x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)   (split on device)
//   w = w0 + w1 + w2 likewise                                                  (packed on the host)
//   x * w ~= x0w0 + x0w1 + x1w0 + x0w2 + x1w1 + x2w0                           (one fp32 accumulator)
// bf16 keeps fp32's exponent range and three RNE parts carry all 24 significand bits, so the
// splits are exact (no scaling, no subnormal loss); the dropped terms x1w2 + x2w1 + x2w2 are
// <= 2^-26 |x w|, below the fp32 rounding of the accumulation itself (2^-24).
//
// mfma_mode 1, "fp32x3" (fp16 parts, ~22 significand bits per product -- NOT fp32 grade):
//   x: x_hi = fp16(x),  x_lo = fp16(x - x_hi)
//   w: W1 = fp16(w) * 2^11 (exact),  W2 = fp16((w - fp16(w)) * 2^11)
//   2^11 * x * w ~= x_hi*W1 + x_hi*W2 + x_lo*W1, the accumulator scaled by 2^-11 in the epilogue.
//
// Packed split weights (lic_conv_args.wgt_split), MFMA-fragment order:
//   [copad/32][cpad/16][ntaps][NPB][64 lanes][8 x 16-bit]
// fragment (n-tile j, chunk k, tap t, part p) is the B operand of v_mfma_f32_32x32x16_{bf16,f16}
// exactly as a wave holds it: lane l carries output channel 32j + (l & 31), input channels
// 16k + 8(l >> 5) .. +7 of part p.  One wave reads it as one contiguous 1 KB (16 B per lane).
#pragma once
#include "lic_common.h"

namespace lic {

constexpr float kSplitScale = 2048.0f;  // 2^11 (mode 1)

template <int MODE> struct SplitMode;
template <> struct SplitMode<1> {   // fp16: x_hi, x_lo x W1, W2
  using T = half_t;
  static constexpr int NPA = 2, NPB = 2, NPROD = 3;
  static constexpr int PA[NPROD] = {0, 0, 1}, PB[NPROD] = {0, 1, 0};
  static constexpr float scale = 1.0f / kSplitScale;
};
template <> struct SplitMode<2> {   // bf16: x0, x1, x2 x w0, w1, w2
  using T = bf16_t;
  static constexpr int NPA = 3, NPB = 3, NPROD = 6;
  static constexpr int PA[NPROD] = {0, 0, 1, 0, 1, 2}, PB[NPROD] = {0, 1, 0, 2, 1, 0};
  static constexpr float scale = 1.0f;
};

// element offset of fragment (n-tile, chunk, tap, part) in the packed split weights
__device__ __forceinline__ int64_t split_frag_off(int ntile, int chunk, int tap, int part, int nchunks, int ntaps,
                                                  int npb) {
  return ((((int64_t)ntile * nchunks + chunk) * ntaps + tap) * npb + part) * 512;
}

// Split 4 fp32 values (after the prologue and the chunk's sign) into NPA 16-bit parts; part pl's
// 4 values as 8 bytes.  Exact residuals (the differences fit fp32).
template <int MODE>
__device__ __forceinline__ void split4(float4 v, int pro, float sg, uint2 (&out)[SplitMode<MODE>::NPA]) {
  using T = typename SplitMode<MODE>::T;
  if (pro == LIC_PRO_SQUARE) v = make_float4(v.x * v.x, v.y * v.y, v.z * v.z, v.w * v.w);
  else if (pro == LIC_PRO_ABS) v = make_float4(fabsf(v.x), fabsf(v.y), fabsf(v.z), fabsf(v.w));
  float r[4] = {sg * v.x, sg * v.y, sg * v.z, sg * v.w};
  if constexpr (MODE == 1) {   // fp16 parts: |x| > 65504 is outside fp32x3's domain (the host sends x^2
#pragma unroll                 // prologues to mode 2); such an input poisons its outputs with NaN, loudly,
    for (int e = 0; e < 4; ++e)   // instead of a silently saturated finite value
      r[e] = fabsf(r[e]) <= 65504.f ? r[e] : __builtin_nanf("");
  }
#pragma unroll
  for (int pl = 0; pl < SplitMode<MODE>::NPA; ++pl) {
    T part[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      part[e] = (T)r[e];
      r[e] -= (float)part[e];
    }
    out[pl] = *(const uint2*)part;
  }
}

}  // namespace lic
