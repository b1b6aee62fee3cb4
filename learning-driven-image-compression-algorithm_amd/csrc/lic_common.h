// Shared device/host helpers for liblic (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "../../include/lic.h"

namespace lic {

typedef _Float16 half_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// thread-local error string (lic_last_error)
void set_error(const std::string& s);
int fail(const std::string& s);

// Raise `kern`'s dynamic-LDS limit to `bytes` on the current device, once per
// (kernel, device, size); thread-safe, returns the HIP status of the first attempt
// (a failure is not cached, so the next launch tries again).
hipError_t ensure_dyn_lds(const void* kern, int bytes);

#define LIC_CHECK_LAUNCH()                                                   \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) return ::lic::fail(std::string("HIP launch: ") + hipGetErrorString(_e)); \
  } while (0)

template <typename T> struct DT;
template <> struct DT<float> { static constexpr int id = LIC_F32; };
template <> struct DT<half_t> { static constexpr int id = LIC_F16; };
template <> struct DT<bf16_t> { static constexpr int id = LIC_BF16; };

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(half_t v) { return (float)v; }
__device__ __forceinline__ float to_f(bf16_t v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ half_t from_f<half_t>(float v) { return (half_t)v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return (bf16_t)v; }   // RNE

// One 32x32x16 MFMA on 16-bit operands (8 per lane, as 16 raw bytes): fp16 or bf16 by T,
// fp32 accumulation.  v_mfma_f32_32x32x16_{f16,bf16}.
template <typename T>
__device__ __forceinline__ floatx16 mfma_k16(const u32x4& a, const u32x4& b, const floatx16& c) {
  if constexpr (DT<T>::id == LIC_BF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(*(const bf16x8*)&a, *(const bf16x8*)&b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(*(const half8*)&a, *(const half8*)&b, c, 0, 0, 0);
}

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

// One output element of the fused conv epilogue; every mode's transcendental
// appears once (keeps the unrolled epilogue code small):
//   PLAIN      act(acc+b) (+ r1)            GATE  g * sigmoid(act(acc+b) (+ r1)) + r2
//   RES_ACT    act(acc+b (+ r1))            HALF_TANH  r2 + 0.5 tanh(act(acc+b))
//   GDN_DIV / GDN_RSQRT / GDN_SQRT   g / sqrt(acc+b), g * (1/sqrt(acc+b)), g * sqrt(acc+b)  (+ r1)
__device__ __forceinline__ float epi_elem(float x, float g, float r1, float r2, int epi, int act, float slope,
                                          bool has_r1) {
  const bool gdn = epi == LIC_EPI_GDN_DIV || epi == LIC_EPI_GDN_RSQRT || epi == LIC_EPI_GDN_SQRT;
  if (epi == LIC_EPI_RES_ACT && has_r1) x += r1;
  if (gdn) {
    const float s = sqrtf(x);
    x = epi == LIC_EPI_GDN_DIV ? g / s : (epi == LIC_EPI_GDN_RSQRT ? g * (1.0f / s) : g * s);
  } else {
    x = apply_act(x, act, slope);
  }
  if (has_r1 && epi != LIC_EPI_RES_ACT && epi != LIC_EPI_HALF_TANH) x += r1;
  if (epi == LIC_EPI_GATE) x = g * sigmoid_f(x) + r2;
  else if (epi == LIC_EPI_HALF_TANH) x = r2 + 0.5f * tanhf(x);
  return x;
}

// Vector form of epi_elem over V elements: every mode / activation test is
// hoisted out of the element loops, so the executed code of a launch is one dense
// run of instructions (per-element branching spreads it over many i-cache lines).
template <int V>
__device__ __forceinline__ void act_vec(float* x, int act, float slope) {
  switch (act) {
    case LIC_ACT_RELU:
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = x[k] > 0.f ? x[k] : 0.f;
      break;
    case LIC_ACT_LRELU:
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = x[k] > 0.f ? x[k] : x[k] * slope;
      break;
    case LIC_ACT_GELU:
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = gelu_f(x[k]);
      break;
    case LIC_ACT_ROUND:
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = rintf(x[k]);
      break;
    default: break;
  }
}

template <int V, bool HAS_R1>
__device__ __forceinline__ void epi_vec(float* x, const float* g, const float* r1, const float* r2, int epi, int act,
                                        float slope) {
  if (epi == LIC_EPI_GDN_DIV || epi == LIC_EPI_GDN_RSQRT || epi == LIC_EPI_GDN_SQRT) {
    if (epi == LIC_EPI_GDN_DIV) {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = g[k] / sqrtf(x[k]);
    } else if (epi == LIC_EPI_GDN_RSQRT) {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = g[k] * (1.0f / sqrtf(x[k]));
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] = g[k] * sqrtf(x[k]);
    }
    if constexpr (HAS_R1) {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] += r1[k];
    }
    return;
  }
  if (epi == LIC_EPI_RES_ACT) {
    if constexpr (HAS_R1) {
#pragma unroll
      for (int k = 0; k < V; ++k) x[k] += r1[k];
    }
    act_vec<V>(x, act, slope);
    return;
  }
  act_vec<V>(x, act, slope);
  if (epi == LIC_EPI_HALF_TANH) {
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] = r2[k] + 0.5f * tanhf(x[k]);
    return;
  }
  if constexpr (HAS_R1) {
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] += r1[k];
  }
  if (epi == LIC_EPI_GATE) {
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] = g[k] * sigmoid_f(x[k]) + r2[k];
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
  } else if (a.out_shuffle == 3) {
    const int q = a.co >> 2, ph = n / q;
    oy = 2 * oy + (ph >> 1);
    ox = 2 * ox + (ph & 1);
    ch = n - ph * q;
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
  const bool shuf_ok = a.out_shuffle == 0 || (a.out_shuffle == 3 && (a.co >> 2) % V == 0);
  return shuf_ok && a.co % V == 0 && al(a.y, a.ldy) && al(a.y2, a.ldy2) && al(a.r1, a.ldr1) &&
         al(a.g, a.ldg) && al(a.r2, a.ldr2);
}

// Orders one wave's LDS writes before its later reads of the same words (and
// those reads before the next writes) for a wave-private LDS slot: LDS requests
// of a wave complete in order, so draining lgkmcnt is enough.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Global operands of one 32x32 output tile for the vector epilogue (g, r1, r2 per
// pass); MASK (EPI_G | EPI_R1 | EPI_R2) says at compile time which of them the
// launch reads, so every load in a variant is unconditional.  They are loaded one
// tile ahead (epi_prefetch) so that waiting for them never waits for the previous
// tile's stores (VMEM loads and stores share the in-order vmcnt counter on CDNA).
enum { EPI_G = 1, EPI_R1 = 2, EPI_R2 = 4 };

__device__ __forceinline__ int epi_mask(const lic_conv_args& a) {
  const bool gdn = a.epi == LIC_EPI_GDN_DIV || a.epi == LIC_EPI_GDN_RSQRT || a.epi == LIC_EPI_GDN_SQRT;
  return ((gdn || a.epi == LIC_EPI_GATE) ? EPI_G : 0) |
         ((a.r1 != nullptr && a.epi != LIC_EPI_HALF_TANH) ? EPI_R1 : 0) |
         ((a.epi == LIC_EPI_HALF_TANH || a.epi == LIC_EPI_GATE) ? EPI_R2 : 0);
}

template <typename T>
struct EpiOperands {
  static constexpr int V = Vec16<T>::V;
  static constexpr int NP = 32 / (64 / (32 / V));  // passes per tile
  u32x4 g[NP], r1[NP], r2[NP];
};

template <typename T, int MASK>
__device__ __forceinline__ void epi_prefetch(const lic_conv_args& a, const int* rowpix, int n0, int lane,
                                             EpiOperands<T>& o) {
  constexpr int V = Vec16<T>::V;
  constexpr int CPR = 32 / V;
  constexpr int RPP = 64 / CPR;
  constexpr int NP = EpiOperands<T>::NP;
  const int n = n0 + (lane % CPR) * V;
  const int nl = n < a.co ? n : 0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int base = rowpix[p * RPP + lane / CPR];
    const int64_t pix = base >= 0 ? base : 0;
    if constexpr ((MASK & EPI_G) != 0) o.g[p] = *(const u32x4*)((const T*)a.g + pix * a.ldg + nl);
    if constexpr ((MASK & EPI_R1) != 0) o.r1[p] = *(const u32x4*)((const T*)a.r1 + pix * a.ldr1 + nl);
    if constexpr ((MASK & EPI_R2) != 0) o.r2[p] = *(const u32x4*)((const T*)a.r2 + pix * a.ldr2 + nl);
  }
}

// Finish one 32x32 fp32 accumulator tile staged in LDS (row stride 33 floats):
// rows are tile pixels (destination pixel base in rowpix[], -1 = outside), columns
// output channels n0 .. n0+31, bias from the block's LDS copy.  Each lane handles
// 16 contiguous bytes of one pixel per pass (epi_elem in fp32, one 16-B store).
template <typename T, int MASK>
__device__ __forceinline__ void epilogue_tile(const lic_conv_args& a, const float* ct, const int* rowpix, int n0,
                                              int lane, const float* sbias, const EpiOperands<T>& o) {
  constexpr int V = Vec16<T>::V;
  constexpr int CPR = 32 / V;   // 16-B chunks per tile row
  constexpr int RPP = 64 / CPR; // rows per pass
  constexpr int NP = 32 / RPP;  // passes per tile
  T* __restrict__ yg = (T*)a.y;
  T* __restrict__ y2g = (T*)a.y2;
  const int cc = lane % CPR;
  const int n = n0 + cc * V;
  const bool nok = n < a.co;
  float bias[V];
#pragma unroll
  for (int k = 0; k < V; ++k) bias[k] = sbias[cc * V + k];
  auto unpack = [&](const u32x4& raw, float* f) {
    const T* e = (const T*)&raw;
#pragma unroll
    for (int k = 0; k < V; ++k) f[k] = to_f(e[k]);
  };
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int row = p * RPP + lane / CPR;
    const int base = rowpix[row];
    float v[V], tg[V] = {}, t1[V] = {}, t2[V] = {};
    if constexpr ((MASK & EPI_G) != 0) unpack(o.g[p], tg);
    if constexpr ((MASK & EPI_R1) != 0) unpack(o.r1[p], t1);
    if constexpr ((MASK & EPI_R2) != 0) unpack(o.r2[p], t2);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = ct[row * 33 + cc * V + k] + bias[k];
    epi_vec<V, (MASK & EPI_R1) != 0>(v, tg, t1, t2, a.epi, a.act, a.slope);
    if (base >= 0 && nok) {
      int64_t pix = base;
      int ch = n;
      if (a.out_shuffle == 3) {  // phase-major sub-pixel store (vector chunks never straddle phases)
        const int q = a.co >> 2, ph = n / q;
        pix += (ph >> 1) * a.wo + (ph & 1);
        ch = n - ph * q;
      }
      store_vec<T>(yg + pix * a.ldy + ch, v);
      if (y2g) store_vec<T>(y2g + pix * a.ldy2 + ch, v);
    }
  }
}

// Scalar finish of one staged tile (pixel-shuffle stores, unaligned views, channel
// tails): lane l handles row l>>1, channels (l&1)*16 .. +15.
template <typename T>
__device__ __forceinline__ void epilogue_tile_scalar(const lic_conv_args& a, const float* ct, const int* rowpix,
                                                     int n0, int lane) {
  T* __restrict__ yg = (T*)a.y;
  T* __restrict__ y2g = (T*)a.y2;
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
    } else if (a.out_shuffle == 3) {
      const int q = a.co >> 2, ph = n / q;
      pix += (ph >> 1) * a.wo + (ph & 1);
      ch = n - ph * q;
    }
    const float v = conv_epilogue<T>(a, ct[erow * 33 + ecol + c], n, pix, ch);
    yg[pix * a.ldy + ch] = from_f<T>(v);
    if (y2g) y2g[pix * a.ldy2 + ch] = from_f<T>(v);
  }
}

// Epilogue driver for one wave's NQ = TM x TN accumulator tiles: stage(q) writes
// tile q into the wave's private LDS slot ct.  Vector variants finish tiles in
// pairs with ping-pong operand sets (tile q+1's loads in flight while tile q is
// finished and stored); MASK < 0 is the scalar path.
// CT_STRIDE > 0: tile q is staged at ct + q * CT_STRIDE (all of a wave's tiles staged up front, so the
// accumulators are dead before the epilogue's operand loads); 0: one slot reused for every tile.
template <typename T, int NQ, int TN, int MASK, typename Stage, int CT_STRIDE = 0>
__device__ __forceinline__ void epilogue_run(const lic_conv_args& a, const float* ct0, const int* rowpix_w, int n0_w,
                                             const float* sbias_w, int lane, Stage& stage) {
  auto ctq = [&](int q) { return ct0 + q * CT_STRIDE; };
  if constexpr (MASK < 0) {
#pragma nounroll
    for (int q = 0; q < NQ; ++q) {
      stage(q);
      wave_lds_sync();
      epilogue_tile_scalar<T>(a, ctq(q), rowpix_w + (q / TN) * 32, n0_w + (q % TN) * 32, lane);
      wave_lds_sync();
    }
  } else {
    EpiOperands<T> e0, e1;
    auto tile = [&](int q, const EpiOperands<T>& eo) {
      stage(q);
      wave_lds_sync();
      epilogue_tile<T, MASK>(a, ctq(q), rowpix_w + (q / TN) * 32, n0_w + (q % TN) * 32, lane, sbias_w + (q % TN) * 32,
                             eo);
      wave_lds_sync();
    };
    auto fetch = [&](int q, EpiOperands<T>& eo) {
      q = q < NQ ? q : NQ - 1;
      epi_prefetch<T, MASK>(a, rowpix_w + (q / TN) * 32, n0_w + (q % TN) * 32, lane, eo);
    };
    fetch(0, e0);
    if constexpr (NQ <= 4) {
      // short: unrolled (a runtime loop here leaves the operand sets in scratch)
#pragma unroll
      for (int q = 0; q + 1 < NQ; q += 2) {
        fetch(q + 1, e1);
        tile(q, e0);
        fetch(q + 2, e0);
        tile(q + 1, e1);
      }
    } else {
#pragma nounroll
      for (int q = 0; q + 1 < NQ; q += 2) {
        fetch(q + 1, e1);
        tile(q, e0);
        fetch(q + 2, e0);
        tile(q + 1, e1);
      }
    }
    if constexpr (NQ % 2) tile(NQ - 1, e0);
  }
}

// Uniform dispatch to the epilogue variant of this launch.
template <typename T, int NQ, int TN, typename Stage, int CT_STRIDE = 0>
__device__ __forceinline__ void epilogue_all(const lic_conv_args& a, const float* ct, const int* rowpix_w, int n0_w,
                                             const float* sbias_w, int lane, Stage stage) {
  if (!epi_vec_ok<T>(a)) {
    epilogue_run<T, NQ, TN, -1, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage);
    return;
  }
  switch (epi_mask(a)) {
    case 0: epilogue_run<T, NQ, TN, 0, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage); break;
    case EPI_R1: epilogue_run<T, NQ, TN, EPI_R1, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage); break;
    case EPI_G: epilogue_run<T, NQ, TN, EPI_G, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage); break;
    case EPI_G | EPI_R1:
      epilogue_run<T, NQ, TN, EPI_G | EPI_R1, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage);
      break;
    case EPI_R2: epilogue_run<T, NQ, TN, EPI_R2, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage); break;
    case EPI_G | EPI_R2:
      epilogue_run<T, NQ, TN, EPI_G | EPI_R2, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage);
      break;
    default:
      epilogue_run<T, NQ, TN, EPI_G | EPI_R1 | EPI_R2, Stage, CT_STRIDE>(a, ct, rowpix_w, n0_w, sbias_w, lane, stage);
      break;
  }
}

}  // namespace lic
