// Backward kernels of the training path (train_net_unet.py:177-200,
// eval_net.py:170-179 online encoder finetune).
//
// What runs where:
//   * conv dgrad      = the forward conv kernels (lic_conv2d_fwd) over dz with the
//                       weights re-packed transposed + tap-mirrored (stride 1) or as
//                       transposed-conv phases (stride 2) — no new kernel (host packing
//                       in lic_amd/autograd.py).
//   * conv wgrad      = wgrad_kernel below: implicit GEMM dW[co][tap][ci] = sum over
//                       output pixels of dz[pix][co] * x[pix*s + tap][ci] on MFMA, K
//                       (pixels) split across work-groups, deterministic two-pass reduce.
//   * bias / beta     = channel_sum (per-channel sum over pixels, two pass).
//   * elementwise     = activation / gate / GDN chain-rule kernels, LowerBound rule.
#include "lic_common.h"

namespace lic {

// ---------------------------------------------------------------------------- wgrad
// Operand staging: a "unit" is EPC pixels x EPC channels (EPC = 16 B / element).
// A thread loads its unit as EPC 16-byte rows (one pixel each; consecutive threads
// take consecutive channel groups of the same pixel -> coalesced), transposes it in
// registers and writes EPC 16-byte LDS rows (one channel each, EPC pixels), so the
// LDS tiles are [channel][64 B of pixels] — the same swizzled layout the forward
// kernel uses for its [pixel][64 B of channels] tiles, and the same MFMA fragment
// reads (K = pixels) serve both operands.
template <typename T, int BM, int BN, int WM, int WN, int PRO>
__global__ __launch_bounds__(WM * WN * 64) void wgrad_kernel(const lic_wgrad_args a, const int K, const int chunk,
                                                              const int tiles_n, float* __restrict__ ws) {
  constexpr int NT = WM * WN * 64;
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = 4 * EPC;  // pixels per K step (64-byte LDS rows)
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "tile");
  constexpr int A_U = 4 * (BM / EPC), B_U = 4 * (BN / EPC);
  static_assert(A_U + B_U <= NT, "one load unit per thread");
  constexpr int BUF = (BM + BN) * 64;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int n0 = tm * BM, c0 = tn * BN;
  const int t = blockIdx.z;
  const int tdy = a.dy[t], tdx = a.dx[t];
  const int kbeg = blockIdx.y * chunk;
  const int kend = min(K, kbeg + chunk);
  const int mij = a.mi * a.mj;

  const bool isA = tid < A_U;
  const bool active = tid < A_U + B_U;
  const int u = isA ? tid : tid - A_U;
  const int ng = isA ? BM / EPC : BN / EPC;
  const int cg = u % ng, pg = u / ng;
  const int ch = (isA ? n0 : c0) + cg * EPC;
  const bool ch_ok = active && (isA ? ch < a.co : ch < a.ci);
  const T* __restrict__ src = isA ? (const T*)a.dz : (const T*)a.x;
  char* const region = smem + (isA ? 0 : BM * 64);
  const int row0 = cg * EPC;

  u32x4 v[EPC];
  auto gload = [&](int k0) {
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int k = k0 + pg * EPC + e;
      bool ok = ch_ok && k < kend;
      int64_t off = 0;
      if (ok) {
        const int b = k / mij;
        const int rem = k - b * mij;
        const int i = rem / a.mj;
        const int j = rem - i * a.mj;
        if (isA) {
          const int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
          off = ((int64_t)(b * a.ho + oy) * a.wo + ox) * a.ldz + ch;
        } else {
          const int iy = i * a.isy + tdy, ix = j * a.isx + tdx;
          ok = (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
          off = ok ? ((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + ch : 0;
        }
      }
      u32x4 r = *(const u32x4*)(src + off);
      if (!ok) r = u32x4{0u, 0u, 0u, 0u};
      v[e] = r;
    }
  };

  auto sstore = [&](int buf) {
    if (!active) return;
    char* base = region + buf * BUF;
    T tr[EPC][EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const T* ve = (const T*)&v[e];
#pragma unroll
      for (int c = 0; c < EPC; ++c) {
        T val = ve[c];
        if constexpr (PRO == LIC_PRO_SQUARE) {
          if (!isA) {
            const float f = to_f(val);
            val = from_f<T>(f * f);
          }
        }
        tr[c][e] = val;
      }
    }
#pragma unroll
    for (int c = 0; c < EPC; ++c) {
      const int row = row0 + c;
      *(u32x4*)(base + row * 64 + ((pg ^ ((row >> 2) & 3)) << 4)) = *(const u32x4*)tr[c];
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  const int lrow = lane & 31, lhalf = lane >> 5;
  auto compute = [&](int buf) {
    const char* base = smem + buf * BUF;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + lhalf;
      u32x4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 32 + lrow;
        fa[i] = *(const u32x4*)(base + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 32 + lrow;
        fb[j] = *(const u32x4*)(base + BM * 64 + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            half8 av = *(half8*)&fa[i];
            half8 bv = *(half8*)&fb[j];
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc[i][j], 0, 0, 0);
          } else {
            const float* af = (const float*)&fa[i];
            const float* bf = (const float*)&fb[j];
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q], bf[q], acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  const int nsteps = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nsteps > 0) {
    gload(kbeg);
    sstore(0);
    __syncthreads();
    for (int step = 0; step < nsteps; ++step) {
      const int cur = step & 1;
      if (step + 1 < nsteps) gload(kbeg + (step + 1) * BK);
      compute(cur);
      if (step + 1 < nsteps) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // partial tile -> ws[split][tap][co][ci] (fp32; lanes 0..31 write 32 consecutive ci)
  float* out = ws + ((int64_t)blockIdx.y * a.ntaps + t) * a.co * a.ci;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = c0 + wn * WTN + j * 32 + lrow;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = n0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lhalf;
        if (row < a.co && col < a.ci) out[(int64_t)row * a.ci + col] = acc[i][j][r];
      }
    }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int nsplit, int ntaps, int co, int ci, int co_out,
                                    int ci_out, float* __restrict__ dw, int64_t s_co, int64_t s_ci, int64_t s_tap,
                                    int accumulate) {
  const int64_t total = (int64_t)ntaps * co_out * ci_out;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % ci_out);
  const int64_t r = idx / ci_out;
  const int n = (int)(r % co_out);
  const int t = (int)(r / co_out);
  const int64_t stride = (int64_t)ntaps * co * ci;
  const float* p = ws + ((int64_t)t * co + n) * ci + c;
  float s = 0.f;
  for (int k = 0; k < nsplit; ++k) s += p[k * stride];
  float* o = dw + n * s_co + c * s_ci + t * s_tap;
  *o = accumulate ? *o + s : s;
}

struct WgPlan {
  int bm, bn, tiles_m, tiles_n, nsplit, chunk, K;
};

static WgPlan wgrad_plan(const lic_wgrad_args& a) {
  WgPlan p;
  const bool small = a.co <= 64 || a.ci <= 64;
  p.bm = small ? 64 : 128;
  p.bn = small ? 64 : 128;
  p.tiles_m = (a.co + p.bm - 1) / p.bm;
  p.tiles_n = (a.ci + p.bn - 1) / p.bn;
  p.K = a.n * a.mi * a.mj;
  const int bk = a.dtype == LIC_F16 ? 32 : 16;
  const int per_split = p.tiles_m * p.tiles_n * a.ntaps;
  const int max_split = std::max(1, (p.K + 8 * bk - 1) / (8 * bk));  // >= 8 K steps per work-group
  int ns = std::max(1, (2048 + per_split - 1) / per_split);
  ns = std::min(std::min(ns, max_split), 4096);
  int chunk = (p.K + ns - 1) / ns;
  chunk = (chunk + bk - 1) / bk * bk;
  p.nsplit = std::max(1, (p.K + chunk - 1) / chunk);
  p.chunk = chunk;
  return p;
}

static int wgrad_check(const lic_wgrad_args& a) {
  if (a.dtype != LIC_F32 && a.dtype != LIC_F16) return fail("wgrad: dtype must be LIC_F32 or LIC_F16");
  const int epc = a.dtype == LIC_F16 ? 8 : 4;
  if (!a.x || !a.dz || !a.dw) return fail("wgrad: null pointer");
  if (a.ci <= 0 || a.co <= 0 || a.n <= 0 || a.mi <= 0 || a.mj <= 0) return fail("wgrad: empty problem");
  if (a.ci % epc || a.co % epc || a.ldx % epc || a.ldz % epc)
    return fail("wgrad: channel counts / strides must be multiples of 16 bytes (pad the views)");
  if (((uintptr_t)a.x | (uintptr_t)a.dz) & 15) return fail("wgrad: views must be 16-byte aligned");
  if (a.ntaps <= 0 || a.ntaps > LIC_MAX_TAPS) return fail("wgrad: ntaps out of range");
  if (a.ci_out > a.ci || a.co_out > a.co || a.ci_out <= 0 || a.co_out <= 0) return fail("wgrad: bad ci_out / co_out");
  if (a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE) return fail("wgrad: prologue must be NONE or SQUARE");
  // lattice bounds (host-side shape check: every dz read is in range)
  if (a.oy0 + a.osy * (a.mi - 1) >= a.ho || a.ox0 + a.osx * (a.mj - 1) >= a.wo || a.oy0 < 0 || a.ox0 < 0)
    return fail("wgrad: output lattice exceeds the dz map");
  return 0;
}

template <typename T, int BM, int BN, int WM, int WN>
static void wgrad_launch(const lic_wgrad_args& a, const WgPlan& p, hipStream_t s) {
  dim3 grid(p.tiles_m * p.tiles_n, p.nsplit, a.ntaps);
  if (a.prologue == LIC_PRO_SQUARE)
    hipLaunchKernelGGL((wgrad_kernel<T, BM, BN, WM, WN, LIC_PRO_SQUARE>), grid, dim3(WM * WN * 64), 0, s, a, p.K,
                       p.chunk, p.tiles_n, a.ws);
  else
    hipLaunchKernelGGL((wgrad_kernel<T, BM, BN, WM, WN, LIC_PRO_NONE>), grid, dim3(WM * WN * 64), 0, s, a, p.K,
                       p.chunk, p.tiles_n, a.ws);
}

// ---------------------------------------------------------------------------- channel sums
constexpr int CS_CHUNKS = 256;

template <typename T>
__global__ void channel_sum_partial_kernel(const T* __restrict__ x, int ld, int npix, int c, int per,
                                           float* __restrict__ parts) {
  const int p0 = blockIdx.x * per, p1 = min(npix, p0 + per);
  for (int ch = threadIdx.x; ch < c; ch += blockDim.x) {
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += to_f(x[(int64_t)p * ld + ch]);
    parts[(int64_t)blockIdx.x * c + ch] = s;
  }
}

__global__ void channel_sum_reduce_kernel(const float* __restrict__ parts, int nparts, int c, float* __restrict__ out,
                                          int accumulate) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float s = 0.f;
  for (int k = 0; k < nparts; ++k) s += parts[(int64_t)k * c + ch];
  out[ch] = accumulate ? out[ch] + s : s;
}

// ---------------------------------------------------------------------------- elementwise
__device__ __forceinline__ float act_grad(float z, int act, float slope) {
  switch (act) {
    case LIC_ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case LIC_ACT_LRELU: return z > 0.f ? 1.f : slope;
    case LIC_ACT_GELU: {
      const float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752f));
      const float pdf = 0.39894228040143268f * expf(-0.5f * z * z);
      return cdf + z * pdf;
    }
    default: return 1.f;  // NONE; ROUND is straight-through (ste_round, net_ga.py:713-719)
  }
}

template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ z, int ldz, int npix, int c, int act, float slope,
                               T* __restrict__ y, int ldy) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  y[p * ldy + ch] = from_f<T>(apply_act(to_f(z[p * ldz + ch]), act, slope));
}

template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ z, int ldz, const T* __restrict__ dy, int lddy, int npix, int c,
                               int act, float slope, T* __restrict__ dz, int lddz) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  const float g = to_f(dy[p * lddy + ch]) * act_grad(to_f(z[p * ldz + ch]), act, slope);
  dz[p * lddz + ch] = from_f<T>(g);
}

// y = g * sigmoid(a) + r:  da = dy * g * s * (1 - s), dg = dy * s   (layers/layers.py:105-111)
template <typename T>
__global__ void gate_bwd_kernel(const T* __restrict__ av, int lda, const T* __restrict__ g, int ldg,
                                const T* __restrict__ dy, int lddy, int npix, int c, T* __restrict__ da, int ldda,
                                T* __restrict__ dg, int lddg) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  const float s = sigmoid_f(to_f(av[p * lda + ch]));
  const float d = to_f(dy[p * lddy + ch]);
  da[p * ldda + ch] = from_f<T>(d * to_f(g[p * ldg + ch]) * s * (1.f - s));
  if (dg) dg[p * lddg + ch] = from_f<T>(d * s);
}

// GDN family, y = x * n^p with n = beta' + Gamma' x^2 (p = -1/2 GDN, +1/2 IGDN):
//   dxd = dy * n^p,  u = dn = dy * x * p * n^(p-1)
template <typename T>
__global__ void gdn_bwd_elem_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ nrm, int ldn,
                                    const T* __restrict__ dy, int lddy, int npix, int c, int inverse,
                                    T* __restrict__ dxd, int lddxd, T* __restrict__ u, int ldu) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  const float n = to_f(nrm[p * ldn + ch]);
  const float d = to_f(dy[p * lddy + ch]);
  const float xv = to_f(x[p * ldx + ch]);
  const float sq = sqrtf(n);
  float npow, du;
  if (inverse) {  // x * sqrt(n)
    npow = sq;
    du = d * xv * 0.5f / sq;
  } else {        // x / sqrt(n)
    npow = 1.0f / sq;
    du = -0.5f * d * xv / (n * sq);
  }
  dxd[p * lddxd + ch] = from_f<T>(d * npow);
  u[p * ldu + ch] = from_f<T>(du);
}

// dx = dxd + 2 x t   (t = Gamma'^T u, the dgrad of the x^2 -> n 1x1 conv)
template <typename T>
__global__ void gdn_bwd_finish_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ tv, int ldt,
                                      const T* __restrict__ dxd, int lddxd, int npix, int c, T* __restrict__ dx,
                                      int lddx, int accumulate) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  float v = to_f(dxd[p * lddxd + ch]) + 2.f * to_f(x[p * ldx + ch]) * to_f(tv[p * ldt + ch]);
  if (accumulate) v += to_f(dx[p * lddx + ch]);
  dx[p * lddx + ch] = from_f<T>(v);
}

// q' = max(q, bound)^2 - pedestal:  dq = [q >= bound or g < 0] * g,  g = dq' * 2 max(q, bound)
__global__ void lower_bound_sq_bwd_kernel(const float* __restrict__ q, const float* __restrict__ dqe, int count,
                                          float bound, float* __restrict__ dq, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const float qv = q[i];
  const float g = dqe[i] * 2.f * fmaxf(qv, bound);
  const float r = (qv >= bound || g < 0.f) ? g : 0.f;
  dq[i] = accumulate ? dq[i] + r : r;
}

}  // namespace lic

using namespace lic;

#define TR_DISPATCH(dtype, NAME, ...)                                   \
  do {                                                                  \
    if ((dtype) == LIC_F32) {                                           \
      typedef float T;                                                  \
      __VA_ARGS__;                                                      \
    } else if ((dtype) == LIC_F16) {                                    \
      typedef half_t T;                                                 \
      __VA_ARGS__;                                                      \
    } else                                                              \
      return fail(std::string(NAME) + ": dtype must be LIC_F32 or LIC_F16"); \
  } while (0)

static inline unsigned tr_nblk(int64_t total) { return (unsigned)((total + 255) / 256); }

extern "C" int64_t lic_conv2d_wgrad_workspace(const lic_wgrad_args* a) {
  if (!a || wgrad_check(*a)) return -1;
  const WgPlan p = wgrad_plan(*a);
  return (int64_t)p.nsplit * a->ntaps * a->co * a->ci * (int64_t)sizeof(float);
}

extern "C" int lic_conv2d_wgrad(const lic_wgrad_args* ap, lic_stream_t stream) {
  if (!ap) return fail("wgrad: null args");
  const lic_wgrad_args& a = *ap;
  if (int e = wgrad_check(a)) return e;
  const WgPlan p = wgrad_plan(a);
  const int64_t need = (int64_t)p.nsplit * a.ntaps * a.co * a.ci * (int64_t)sizeof(float);
  if (!a.ws || a.ws_bytes < need)
    return fail("wgrad: workspace too small (" + std::to_string(a.ws_bytes) + " < " + std::to_string(need) + ")");
  hipStream_t s = (hipStream_t)stream;
  if (a.dtype == LIC_F16) {
    if (p.bm == 128) wgrad_launch<half_t, 128, 128, 2, 2>(a, p, s);
    else wgrad_launch<half_t, 64, 64, 2, 2>(a, p, s);
  } else {
    if (p.bm == 128) wgrad_launch<float, 128, 128, 2, 2>(a, p, s);
    else wgrad_launch<float, 64, 64, 2, 2>(a, p, s);
  }
  LIC_CHECK_LAUNCH();
  const int64_t total = (int64_t)a.ntaps * a.co_out * a.ci_out;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(tr_nblk(total)), dim3(256), 0, s, a.ws, p.nsplit, a.ntaps, a.co, a.ci,
                     a.co_out, a.ci_out, a.dw, a.s_co, a.s_ci, a.s_tap, a.accumulate);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t lic_channel_sum_workspace(int32_t c) { return (int64_t)CS_CHUNKS * c * (int64_t)sizeof(float); }

extern "C" int lic_channel_sum(int32_t dtype, const void* x, int32_t ldx, int32_t npix, int32_t c, float* ws,
                               int64_t ws_bytes, float* out, int32_t accumulate, lic_stream_t stream) {
  if (c <= 0) return 0;
  if (ws_bytes < lic_channel_sum_workspace(c)) return fail("channel_sum: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int per = std::max(1, (npix + CS_CHUNKS - 1) / CS_CHUNKS);
  const int nparts = std::max(1, (npix + per - 1) / per);
  const int threads = std::min(256, (c + 63) / 64 * 64);
  if (npix > 0) {
    TR_DISPATCH(dtype, "channel_sum",
                hipLaunchKernelGGL(channel_sum_partial_kernel<T>, dim3(nparts), dim3(threads), 0, s, (const T*)x, ldx,
                                   npix, c, per, ws));
    LIC_CHECK_LAUNCH();
  } else {
    hipMemsetAsync(ws, 0, (size_t)c * sizeof(float), s);
  }
  hipLaunchKernelGGL(channel_sum_reduce_kernel, dim3((c + 255) / 256), dim3(256), 0, s, ws, npix > 0 ? nparts : 1, c,
                     out, accumulate);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_act_fwd(int32_t dtype, const void* z, int32_t ldz, int32_t npix, int32_t c, int32_t act,
                           float slope, void* y, int32_t ldy, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "act_fwd",
              hipLaunchKernelGGL(act_fwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)z, ldz, npix, c, act, slope, (T*)y, ldy));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_act_bwd(int32_t dtype, const void* z, int32_t ldz, const void* dy, int32_t lddy, int32_t npix,
                           int32_t c, int32_t act, float slope, void* dz, int32_t lddz, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "act_bwd",
              hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)z, ldz, (const T*)dy, lddy, npix, c, act, slope, (T*)dz, lddz));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_gate_bwd(int32_t dtype, const void* a, int32_t lda, const void* g, int32_t ldg, const void* dy,
                            int32_t lddy, int32_t npix, int32_t c, void* da, int32_t ldda, void* dg, int32_t lddg,
                            lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "gate_bwd",
              hipLaunchKernelGGL(gate_bwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)a, lda, (const T*)g, ldg, (const T*)dy, lddy, npix, c, (T*)da, ldda,
                                 (T*)dg, lddg));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_gdn_bwd_elem(int32_t dtype, const void* x, int32_t ldx, const void* nrm, int32_t ldn,
                                const void* dy, int32_t lddy, int32_t npix, int32_t c, int32_t inverse, void* dxd,
                                int32_t lddxd, void* u, int32_t ldu, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "gdn_bwd_elem",
              hipLaunchKernelGGL(gdn_bwd_elem_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)x, ldx, (const T*)nrm, ldn, (const T*)dy, lddy, npix, c, inverse, (T*)dxd,
                                 lddxd, (T*)u, ldu));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_gdn_bwd_finish(int32_t dtype, const void* x, int32_t ldx, const void* t, int32_t ldt,
                                  const void* dxd, int32_t lddxd, int32_t npix, int32_t c, void* dx, int32_t lddx,
                                  int32_t accumulate, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "gdn_bwd_finish",
              hipLaunchKernelGGL(gdn_bwd_finish_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)x, ldx, (const T*)t, ldt, (const T*)dxd, lddxd, npix, c, (T*)dx, lddx,
                                 accumulate));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_lower_bound_sq_bwd(const float* q, const float* dq_eff, int32_t count, float bound, float* dq,
                                      int32_t accumulate, lic_stream_t stream) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(lower_bound_sq_bwd_kernel, dim3(tr_nblk(count)), dim3(256), 0, (hipStream_t)stream, q, dq_eff,
                     count, bound, dq, accumulate);
  LIC_CHECK_LAUNCH();
  return 0;
}
