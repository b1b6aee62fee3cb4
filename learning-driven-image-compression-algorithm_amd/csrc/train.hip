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
int wd_env(const char* name, int def);   // conv_split_wd.hip

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
  // Running (image, row, col) of this thread's first pixel of the next K step: decoded once
  // with divisions, then advanced by BK pixels per step and by one pixel per element with
  // carries (the per-element divisions made the kernel VALU-bound, ~8x the MFMA time).
  int cur_k = kbeg + pg * EPC, cur_b, cur_i, cur_j;
  {
    cur_b = cur_k / mij;
    const int rem = cur_k - cur_b * mij;
    cur_i = rem / a.mj;
    cur_j = rem - cur_i * a.mj;
  }
  auto step_pix = [&](int& b, int& i, int& j, int d) {
    j += d;
    while (j >= a.mj) {
      j -= a.mj;
      if (++i == a.mi) {
        i = 0;
        ++b;
      }
    }
  };
  auto gload = [&](int /*k0*/) {
    int b = cur_b, i = cur_i, j = cur_j;
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int k = cur_k + e;
      if (e) step_pix(b, i, j, 1);
      bool ok = ch_ok && k < kend;
      int64_t off = 0;
      if (ok) {
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
    cur_k += BK;
    step_pix(cur_b, cur_i, cur_j, BK);
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
            acc[i][j] = mfma_k16<T>(fa[i], fb[j], acc[i][j]);
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

// dw = sum over the splits; with wsb (tiled kernel's per-split bias sums [nsplit][co]) the threads
// past the weight elements also finish db[n], n < co_out
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int nsplit, int ntaps, int co, int ci, int co_out,
                                    int ci_out, float* __restrict__ dw, int64_t s_co, int64_t s_ci, int64_t s_tap,
                                    int accumulate, const float* __restrict__ wsb, float* __restrict__ db) {
  const int64_t total = (int64_t)ntaps * co_out * ci_out;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) {
    const int n = (int)(idx - total);
    if (!wsb || n >= co_out) return;
    float b0 = 0.f, b1 = 0.f;
    int k = 0;
    for (; k + 2 <= nsplit; k += 2) {
      b0 += wsb[(int64_t)k * co + n];
      b1 += wsb[(int64_t)(k + 1) * co + n];
    }
    if (k < nsplit) b0 += wsb[(int64_t)k * co + n];
    db[n] = accumulate ? db[n] + (b0 + b1) : b0 + b1;
    return;
  }
  const int c = (int)(idx % ci_out);
  const int64_t r = idx / ci_out;
  const int n = (int)(r % co_out);
  const int t = (int)(r / co_out);
  const int64_t stride = (int64_t)ntaps * co * ci;
  const float* p = ws + ((int64_t)t * co + n) * ci + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 4 <= nsplit; k += 4) {
    s0 += p[k * stride];
    s1 += p[(k + 1) * stride];
    s2 += p[(k + 2) * stride];
    s3 += p[(k + 3) * stride];
  }
  for (; k < nsplit; ++k) s0 += p[k * stride];
  const float s = (s0 + s1) + (s2 + s3);
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
  const int bk = a.dtype != LIC_F32 ? 32 : 16;
  const int per_split = p.tiles_m * p.tiles_n * a.ntaps;
  const int max_split = std::max(1, (p.K + 8 * bk - 1) / (8 * bk));  // >= 8 K steps per work-group
  int ns = std::max(1, (2048 + per_split - 1) / per_split);
  ns = std::min(std::min(ns, max_split), 64);
  int chunk = (p.K + ns - 1) / ns;
  chunk = (chunk + bk - 1) / bk * bk;
  p.nsplit = std::max(1, (p.K + chunk - 1) / chunk);
  p.chunk = chunk;
  return p;
}

static int wgrad_check(const lic_wgrad_args& a) {
  if (a.dtype != LIC_F32 && a.dtype != LIC_F16 && a.dtype != LIC_BF16)
    return fail("wgrad: dtype must be LIC_F32, LIC_F16 or LIC_BF16");
  const int epc = a.dtype != LIC_F32 ? 8 : 4;
  if (!a.x || !a.dz || !a.dw) return fail("wgrad: null pointer");
  if (a.ci <= 0 || a.co <= 0 || a.n <= 0 || a.mi <= 0 || a.mj <= 0) return fail("wgrad: empty problem");
  if (a.ci % epc || a.co % epc || a.ldx % epc || a.ldz % epc)
    return fail("wgrad: channel counts / strides must be multiples of 16 bytes (pad the views)");
  if (((uintptr_t)a.x | (uintptr_t)a.dz) & 15) return fail("wgrad: views must be 16-byte aligned");
  if (a.ntaps <= 0 || a.ntaps > LIC_MAX_TAPS) return fail("wgrad: ntaps out of range");
  if (a.ci_out > a.ci || a.co_out > a.co || a.ci_out <= 0 || a.co_out <= 0) return fail("wgrad: bad ci_out / co_out");
  if (a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE) return fail("wgrad: prologue must be NONE or SQUARE");
  if (a.db && (a.oy0 || a.ox0 || a.osy != 1 || a.osx != 1 || a.mi != a.ho || a.mj != a.wo))
    return fail("wgrad: db needs the lattice to be dz's full map");
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
// Both passes use 64 channels x 4 row groups per 256-thread block (lane = channel, coalesced
// 128-256 B rows; the 4 groups are folded in LDS), so no thread walks a long serial chain.
constexpr int CS_CHUNKS = 256;

template <typename T>
__global__ __launch_bounds__(256) void channel_sum_partial_kernel(const T* __restrict__ x, int ld, int npix, int c,
                                                                  int per, float* __restrict__ parts) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int ch = blockIdx.y * 64 + lane;
  const int p0 = blockIdx.x * per, p1 = min(npix, p0 + per);
  float s = 0.f;
  if (ch < c)
    for (int p = p0 + r; p < p1; p += 4) s += to_f(x[(int64_t)p * ld + ch]);
  red[r][lane] = s;
  __syncthreads();
  if (r == 0 && ch < c) parts[(int64_t)blockIdx.x * c + ch] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// 64 channels x 16 part groups per 1024-thread block, 4 independent loads in flight per
// thread: the serial chain per thread is nparts/64 adds (was nparts/4 dependent loads)
__global__ __launch_bounds__(1024) void channel_sum_reduce_kernel(const float* __restrict__ parts, int nparts, int c,
                                                                  float* __restrict__ out, int accumulate) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (ch < c) {
    int k = r;
    for (; k + 48 < nparts; k += 64) {
      s0 += parts[(int64_t)k * c + ch];
      s1 += parts[(int64_t)(k + 16) * c + ch];
      s2 += parts[(int64_t)(k + 32) * c + ch];
      s3 += parts[(int64_t)(k + 48) * c + ch];
    }
    for (; k < nparts; k += 16) s0 += parts[(int64_t)k * c + ch];
  }
  red[r][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (r == 0 && ch < c) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][lane];
    out[ch] = accumulate ? out[ch] + t : t;
  }
}

static inline void cs_reduce(const float* parts, int nparts, int c, float* out, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(channel_sum_reduce_kernel, dim3((c + 63) / 64), dim3(1024), 0, s, parts, nparts, c, out,
                     accumulate);
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


__device__ __forceinline__ double block_sum_f64_256(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

struct DwTaps { int8_t dy[LIC_MAX_TAPS]; int8_t dx[LIC_MAX_TAPS]; };

// ---------------------------------------------------------------------------- window attention bwd
// One 256-thread work-group per (image, window, head).  q, k, v, dO of the window are
// staged in LDS as fp32 (same roll / partition address arithmetic as the forward),
// the scores are recomputed in the forward's op order, then
//   D_i = sum_j P_ij (dO_i . v_j);  dV_j = sum_i P_ij dO_i;  dS_ij = P_ij (dO_i . v_j - D_i)
//   dQ_i = scale sum_j dS_ij k_j;   dK_j = scale sum_i dS_ij q_i
// and the relative-position-bias gradient is accumulated per work-group in LDS
// (one partial per (head, window, offset); deterministic second-pass reduce).
template <typename T>
__global__ __launch_bounds__(256) void win_attn_bwd_kernel(const lic_attn_args a, const T* __restrict__ dout,
                                                           int lddo, T* __restrict__ dqkv, int lddq,
                                                           float* __restrict__ tparts) {
  const int ws = a.ws, N = ws * ws, d = a.c / a.heads, dp = d + 1;
  const int R = (2 * ws - 1) * (2 * ws - 1);
  const int nwx = a.w / ws, nwy = a.h / ws;
  int bid = blockIdx.x;
  const int h = bid % a.heads;
  bid /= a.heads;
  const int win = bid;  // (b * nwy + wy) * nwx + wx
  const int wx = bid % nwx;
  bid /= nwx;
  const int wy = bid % nwy;
  const int b = bid / nwy;
  const int nwin = a.n * nwy * nwx;

  extern __shared__ float sm[];
  float* sq = sm;
  float* sk = sq + N * dp;
  float* sv = sk + N * dp;
  float* sdo = sv + N * dp;
  float* sP = sdo + N * dp;          // [N][N+1]
  float* sD = sP + N * (N + 1);      // [N]
  float* stab = sD + N;              // [R]
  const int tid = threadIdx.x;

  auto pix = [&](int t) -> int64_t {
    const int sy = wy * ws + t / ws, sx = wx * ws + t % ws;
    int py = sy + a.shift, px = sx + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return ((int64_t)b * a.h + py) * a.w + px;
  };
  const T* qkv = (const T*)a.qkv;
  for (int e = tid; e < N * d; e += 256) {
    const int t = e / d, c = e % d;
    const int64_t p = pix(t);
    const T* q = qkv + p * a.ldqkv + h * d + c;
    sq[t * dp + c] = to_f(q[0]);
    sk[t * dp + c] = to_f(q[a.c]);
    sv[t * dp + c] = to_f(q[2 * a.c]);
    sdo[t * dp + c] = to_f(dout[p * lddo + h * d + c]);
  }
  __syncthreads();

  const float scale = a.scale;
  auto reg_wba = [&](int y, int x) {
    const int ly = y < a.h - ws ? 0 : (y < a.h - a.shift ? 1 : 2);
    const int lx = x < a.w - ws ? 0 : (x < a.w - a.shift ? 1 : 2);
    return ly * 3 + lx;
  };
  const int split = ws - a.shift;
  const bool last_row = (wy == nwy - 1), last_col = (wx == nwx - 1);
  auto relidx = [&](int i, int j) {
    return (i / ws - j / ws + ws - 1) * (2 * ws - 1) + (i % ws - j % ws + ws - 1);
  };
  for (int e = tid; e < N * N; e += 256) {
    const int i = e / N, j = e % N;
    float dot = 0.f;
    for (int c = 0; c < d; ++c) {
      const float qv = a.scale_after ? sq[i * dp + c] : sq[i * dp + c] * scale;
      dot += qv * sk[j * dp + c];
    }
    if (a.scale_after) dot = dot * scale;
    float v = dot + a.table[relidx(i, j) * a.tab_sr + h * a.tab_sh];
    const int iy = i / ws, ix = i % ws, jy = j / ws, jx = j % ws;
    if (a.mask_kind == 1) {
      if (reg_wba(wy * ws + jy, wx * ws + jx) != reg_wba(wy * ws + iy, wx * ws + ix)) v += -100.0f;
    } else if (a.mask_kind == 2) {
      bool m = false;
      if (last_row && ((iy < split) != (jy < split))) m = true;
      if (last_col && ((ix < split) != (jx < split))) m = true;
      if (m) v = -INFINITY;
    }
    sP[i * (N + 1) + j] = v;
  }
  __syncthreads();
  if (tid < N) {
    float* row = sP + tid * (N + 1);
    float mx = -INFINITY;
    for (int j = 0; j < N; ++j) mx = fmaxf(mx, row[j]);
    float sum = 0.f;
    for (int j = 0; j < N; ++j) {
      row[j] = expf(row[j] - mx);
      sum += row[j];
    }
    const float inv = 1.0f / sum;
    for (int j = 0; j < N; ++j) row[j] *= inv;
  }
  __syncthreads();
  if (tid < N) {
    const float* row = sP + tid * (N + 1);
    float acc = 0.f;
    for (int j = 0; j < N; ++j) {
      float dpv = 0.f;
      for (int c = 0; c < d; ++c) dpv += sdo[tid * dp + c] * sv[j * dp + c];
      acc += row[j] * dpv;
    }
    sD[tid] = acc;
  }
  for (int e = tid; e < N * d; e += 256) {  // dV
    const int j = e / d, c = e % d;
    float acc = 0.f;
    for (int i = 0; i < N; ++i) acc += sP[i * (N + 1) + j] * sdo[i * dp + c];
    dqkv[pix(j) * lddq + 2 * a.c + h * d + c] = from_f<T>(acc);
  }
  __syncthreads();
  for (int e = tid; e < N * N; e += 256) {  // dS (in place of P)
    const int i = e / N, j = e % N;
    float dpv = 0.f;
    for (int c = 0; c < d; ++c) dpv += sdo[i * dp + c] * sv[j * dp + c];
    const float ds = sP[i * (N + 1) + j] * (dpv - sD[i]);
    sP[i * (N + 1) + j] = ds;
  }
  __syncthreads();
  // table gradient: every relative offset r sums its (i, j) pairs in a fixed order (deterministic;
  // an LDS atomicAdd here made training runs differ in the last bits)
  for (int r = tid; r < R; r += 256) {
    const int dy = r / (2 * ws - 1) - (ws - 1), dx = r % (2 * ws - 1) - (ws - 1);
    float acc = 0.f;
    for (int iy = max(0, dy); iy < min(ws, ws + dy); ++iy)
      for (int ix = max(0, dx); ix < min(ws, ws + dx); ++ix)
        acc += sP[(iy * ws + ix) * (N + 1) + (iy - dy) * ws + (ix - dx)];
    stab[r] = acc;
  }
  for (int e = tid; e < N * d; e += 256) {
    const int i = e / d, c = e % d;
    float aq = 0.f, ak = 0.f;
    for (int j = 0; j < N; ++j) {
      aq += sP[i * (N + 1) + j] * sk[j * dp + c];
      ak += sP[j * (N + 1) + i] * sq[j * dp + c];
    }
    const int64_t p = pix(i);
    dqkv[p * lddq + h * d + c] = from_f<T>(aq * scale);
    dqkv[p * lddq + a.c + h * d + c] = from_f<T>(ak * scale);
  }
  if (tparts)
    for (int r = tid; r < R; r += 256) tparts[((int64_t)h * nwin + win) * R + r] = stab[r];
}

// The 8x8-window case (N = 64 tokens, head dim D a multiple of 4: the a_model / s_model WBA at 64^2 and
// the slice loop's WMSA), round 6: the same math as win_attn_bwd_kernel with the O(N^2 d) products
// register-blocked -- each of the 256 threads owns a 4 x 4 block of (query i, key j) = (ib + 16 r,
// jb + 16 s), so one q / k row read (float4 along d) feeds 4 products instead of 1 and the 16 keys of a
// block row sit in 16 consecutive lanes (row max / sum / D by xor-shuffles); dP = dO V^T is computed
// ONCE (the generic kernel computes it twice, the D pass on 64 threads of 1536 serial products each);
// the table row of the head sits in LDS.  The dot products keep the generic kernel's order (sequential
// over the channel); the softmax sum and D are summed in a butterfly: last-bit differences from it.
template <typename T, int D>
__global__ __launch_bounds__(256) void win_attn_bwd64_kernel(const lic_attn_args a, const T* __restrict__ dout,
                                                             int lddo, T* __restrict__ dqkv, int lddq,
                                                             float* __restrict__ tparts) {
  constexpr int WS = 8, N = 64, DP = D + 4, R = 225, NP = N + 1, DC = D / 4;
  const int nwx = a.w / WS, nwy = a.h / WS;
  int bid = blockIdx.x;
  const int h = bid % a.heads;
  bid /= a.heads;
  const int win = bid;
  const int wx = bid % nwx;
  bid /= nwx;
  const int wy = bid % nwy;
  const int b = bid / nwy;
  const int nwin = a.n * nwy * nwx;

  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* sq = sm;                 // [N][DP]
  float* sk = sq + N * DP;
  float* sv = sk + N * DP;
  float* sdo = sv + N * DP;
  float* sP = sdo + N * DP;       // [N][NP]  P
  float* sS = sP + N * NP;        // [N][NP]  dS
  float* sbt = sS + N * NP;       // [R] this head's bias table
  float* stab = sbt + R;          // [R] table-gradient partials
  const int tid = threadIdx.x;

  auto pix = [&](int t) -> int64_t {
    const int sy = wy * WS + t / WS, sx = wx * WS + t % WS;
    int py = sy + a.shift, px = sx + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return ((int64_t)b * a.h + py) * a.w + px;
  };
  const T* qkv = (const T*)a.qkv;
  for (int e = tid; e < N * D; e += 256) {
    const int t = e / D, c = e % D;
    const int64_t p = pix(t);
    const T* q = qkv + p * a.ldqkv + h * D + c;
    sq[t * DP + c] = to_f(q[0]);
    sk[t * DP + c] = to_f(q[a.c]);
    sv[t * DP + c] = to_f(q[2 * a.c]);
    sdo[t * DP + c] = to_f(dout[p * lddo + h * D + c]);
  }
  for (int r = tid; r < R; r += 256) sbt[r] = a.table[r * a.tab_sr + h * a.tab_sh];
  __syncthreads();

  const float scale = a.scale;
  const int ib = tid >> 4, jb = tid & 15;
  const int split = WS - a.shift;
  const bool last_row = (wy == nwy - 1), last_col = (wx == nwx - 1);
  auto reg_wba = [&](int y, int x) {
    const int ly = y < a.h - WS ? 0 : (y < a.h - a.shift ? 1 : 2);
    const int lx = x < a.w - WS ? 0 : (x < a.w - a.shift ? 1 : 2);
    return ly * 3 + lx;
  };
  // ---- scores, P = softmax (rows i = ib + 16 r, keys j = jb + 16 s) ----
  float P[4][4], G[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) P[r][s2] = G[r][s2] = 0.f;
  for (int c = 0; c < D; c += 4) {
    float4 qr[4], kr[4], dr[4], vr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      qr[r] = *(const float4*)(sq + (ib + 16 * r) * DP + c);
      dr[r] = *(const float4*)(sdo + (ib + 16 * r) * DP + c);
      kr[r] = *(const float4*)(sk + (jb + 16 * r) * DP + c);
      vr[r] = *(const float4*)(sv + (jb + 16 * r) * DP + c);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float q4[4] = {qr[r].x, qr[r].y, qr[r].z, qr[r].w};
      const float d4[4] = {dr[r].x, dr[r].y, dr[r].z, dr[r].w};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const float k4[4] = {kr[s2].x, kr[s2].y, kr[s2].z, kr[s2].w};
        const float v4[4] = {vr[s2].x, vr[s2].y, vr[s2].z, vr[s2].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float qv = a.scale_after ? q4[e] : q4[e] * scale;
          P[r][s2] += qv * k4[e];          // the generic kernel's order: sequential over the channel
          G[r][s2] += d4[e] * v4[e];       // dP = dO . v
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = ib + 16 * r, iy = i / WS, ix = i % WS;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int j = jb + 16 * s2, jy = j / WS, jx = j % WS;
      float dot = P[r][s2];
      if (a.scale_after) dot = dot * scale;
      float v = dot + sbt[(iy - jy + WS - 1) * (2 * WS - 1) + (ix - jx + WS - 1)];
      if (a.mask_kind == 1) {
        if (reg_wba(wy * WS + jy, wx * WS + jx) != reg_wba(wy * WS + iy, wx * WS + ix)) v += -100.0f;
      } else if (a.mask_kind == 2) {
        bool m = false;
        if (last_row && ((iy < split) != (jy < split))) m = true;
        if (last_col && ((ix < split) != (jx < split))) m = true;
        if (m) v = -INFINITY;
      }
      P[r][s2] = v;
    }
    float mx = fmaxf(fmaxf(P[r][0], P[r][1]), fmaxf(P[r][2], P[r][3]));
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      P[r][s2] = expf(P[r][s2] - mx);
      sum += P[r][s2];
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
    float dsum = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      P[r][s2] *= inv;
      dsum += P[r][s2] * G[r][s2];
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) dsum += __shfl_xor(dsum, o);   // D_i = sum_j P_ij dP_ij
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int j = jb + 16 * s2;
      sP[i * NP + j] = P[r][s2];
      sS[i * NP + j] = P[r][s2] * (G[r][s2] - dsum);   // dS
    }
  }
  __syncthreads();
  // ---- table gradient: every relative offset sums its (i, j) pairs of dS in a fixed order ----
  for (int r = tid; r < R; r += 256) {
    const int dy = r / (2 * WS - 1) - (WS - 1), dx = r % (2 * WS - 1) - (WS - 1);
    float acc = 0.f;
    for (int iy = max(0, dy); iy < min(WS, WS + dy); ++iy)
      for (int ix = max(0, dx); ix < min(WS, WS + dx); ++ix)
        acc += sS[(iy * WS + ix) * NP + (iy - dy) * WS + (ix - dx)];
    stab[r] = acc;
  }
  // ---- dV_j = sum_i P_ij dO_i, dQ_i = scale sum_j dS_ij k_j, dK_j = scale sum_i dS_ij q_i (sequential
  // over i / j as the generic kernel); thread = (token t = tid / 4, channel quarter) ----
  {
    const int t = tid >> 2, c0 = (tid & 3) * DC;
    float av[DC], aq[DC], ak[DC];
#pragma unroll
    for (int e = 0; e < DC; ++e) av[e] = aq[e] = ak[e] = 0.f;
    for (int u = 0; u < N; ++u) {
      const float pt = sP[u * NP + t];        // P_{u t}: key t of query u
      const float st = sS[u * NP + t];        // dS_{u t}
      const float su = sS[t * NP + u];        // dS_{t u}
#pragma unroll
      for (int e = 0; e < DC; ++e) {
        av[e] += pt * sdo[u * DP + c0 + e];
        aq[e] += su * sk[u * DP + c0 + e];
        ak[e] += st * sq[u * DP + c0 + e];
      }
    }
    const int64_t p = pix(t);
#pragma unroll
    for (int e = 0; e < DC; ++e) {
      dqkv[p * lddq + 2 * a.c + h * D + c0 + e] = from_f<T>(av[e]);
      dqkv[p * lddq + h * D + c0 + e] = from_f<T>(aq[e] * scale);
      dqkv[p * lddq + a.c + h * D + c0 + e] = from_f<T>(ak[e] * scale);
    }
  }
  if (tparts) {
    __syncthreads();
    for (int r = tid; r < R; r += 256) tparts[((int64_t)h * nwin + win) * R + r] = stab[r];
  }
}

// Deterministic second pass of the table gradient, round 6: block (head, 16 offsets) x 16 window slices --
// slice w sums windows w, w + 16, ... in order, then the 16 slice sums are added in order (a fixed tree:
// the one-thread-per-offset loop over all windows ran 7 workgroups for up to 180 us).
__global__ __launch_bounds__(256) void attn_table_reduce16_kernel(const float* __restrict__ parts, int heads,
                                                                  int nwin, int R, float* __restrict__ dtab,
                                                                  int tab_sr, int tab_sh, int accumulate) {
  __shared__ float red[16][17];
  const int rl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int nrb = (R + 15) / 16;
  const int h = blockIdx.x / nrb, r = (blockIdx.x % nrb) * 16 + rl;
  float acc = 0.f;
  if (r < R) {
    const float* pp = parts + (int64_t)h * nwin * R + r;
    for (int k = sl; k < nwin; k += 16) acc += pp[(int64_t)k * R];
  }
  red[sl][rl] = acc;
  __syncthreads();
  if (sl == 0 && r < R) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][rl];
    float* o = dtab + r * tab_sr + h * tab_sh;
    *o = accumulate ? *o + s : s;
  }
}

__global__ void attn_table_reduce_kernel(const float* __restrict__ parts, int heads, int nwin, int R,
                                         float* __restrict__ dtab, int tab_sr, int tab_sh, int accumulate) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= heads * R) return;
  const int h = idx / R, r = idx % R;
  const float* p = parts + (int64_t)h * nwin * R + r;
  float s = 0.f;
  for (int k = 0; k < nwin; ++k) s += p[(int64_t)k * R];
  float* o = dtab + r * tab_sr + h * tab_sh;
  *o = accumulate ? *o + s : s;
}

// ---------------------------------------------------------------------------- LayerNorm bwd
// One wave per pixel (grid-stride), lane owns channels lane + 64 m.  dx = rstd (g - mean(g)
// - xhat mean(g xhat)), g = dy * w; dw / db accumulated per lane, then per block.
template <typename T, int CPL>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ x, int ldx,
                                                            const T* __restrict__ dy, int lddy, int npix, int c,
                                                            const float* __restrict__ wt, float eps,
                                                            T* __restrict__ dx, int lddx, float* __restrict__ parts) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dw[CPL], db[CPL];
#pragma unroll
  for (int m = 0; m < CPL; ++m) dw[m] = db[m] = 0.f;
  for (int64_t p = (int64_t)blockIdx.x * 4 + wave; p < npix; p += (int64_t)gridDim.x * 4) {
    const T* xp = x + p * ldx;
    const T* gp = dy + p * lddy;
    float xv[CPL], gv[CPL];
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int k = lane + 64 * m;
      xv[m] = k < c ? to_f(xp[k]) : 0.f;
      gv[m] = k < c ? to_f(gp[k]) : 0.f;
      s += xv[m];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / (float)c;
    float v = 0.f;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const float dd = lane + 64 * m < c ? xv[m] - mean : 0.f;
      v += dd * dd;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const float rstd = 1.0f / sqrtf(v / (float)c + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int k = lane + 64 * m;
      if (k < c) {
        const float xh = (xv[m] - mean) * rstd;
        const float g = gv[m] * wt[k];
        sg += g;
        sgx += g * xh;
        dw[m] += gv[m] * xh;
        db[m] += gv[m];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      sg += __shfl_xor(sg, o);
      sgx += __shfl_xor(sgx, o);
    }
    sg /= (float)c;
    sgx /= (float)c;
    T* op = dx + p * lddx;
#pragma unroll
    for (int m = 0; m < CPL; ++m) {
      const int k = lane + 64 * m;
      if (k < c) {
        const float xh = (xv[m] - mean) * rstd;
        op[k] = from_f<T>(rstd * (gv[m] * wt[k] - sg - xh * sgx));
      }
    }
  }
  __shared__ float red[4][2 * 64 * CPL];
#pragma unroll
  for (int m = 0; m < CPL; ++m) {
    red[wave][m * 64 + lane] = dw[m];
    red[wave][64 * CPL + m * 64 + lane] = db[m];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < c; k += 256) {
    const int m = k / 64, l = k % 64;
    float sw = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sw += red[q][m * 64 + l];
      sb += red[q][64 * CPL + m * 64 + l];
    }
    parts[(int64_t)blockIdx.x * 2 * c + k] = sw;
    parts[(int64_t)blockIdx.x * 2 * c + c + k] = sb;
  }
}

// ---------------------------------------------------------------------------- gate fwd
template <typename T>
__global__ void gate_fwd_kernel(const T* __restrict__ av, int lda, const T* __restrict__ g, int ldg,
                                const T* __restrict__ r, int ldr, int npix, int c, T* __restrict__ y, int ldy) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  float v = to_f(g[p * ldg + ch]) * sigmoid_f(to_f(av[p * lda + ch]));
  if (r) v += to_f(r[p * ldr + ch]);
  y[p * ldy + ch] = from_f<T>(v);
}

// ---------------------------------------------------------------------------- rate (train mode)
// compressai GaussianConditional.forward(y, scale, mu) with training=True: y~ = y + U(-1/2, 1/2)
// (counter-based hash noise: (seed, element index) -> uniform), L = Phi((1/2-|y~-mu|)/s) -
// Phi((-1/2-|y~-mu|)/s), s = LowerBound(scale, 0.11), L' = LowerBound(L, 1e-9); plus the
// ste_round forward yhat = rint(y - mu) + mu (net_ga.py:1053).
__device__ __forceinline__ float noise_u(uint64_t seed, uint64_t i) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f) - 0.5f;  // 24-bit uniform in [-1/2, 1/2)
}

template <typename T>
__global__ __launch_bounds__(256) void rate_train_fwd_kernel(const T* __restrict__ y, int ldy, const T* __restrict__ mu,
                                                             int ldmu, const T* __restrict__ sc, int ldsc, int npix,
                                                             int c, uint64_t seed, const uint64_t* seed_dev,
                                                             uint64_t seed_mul, float sbound, float lbound,
                                                             T* __restrict__ yhat, int ldyh, double* __restrict__ parts) {
  __shared__ double red[4];
  if (seed_dev) seed = seed_dev[0] * seed_mul + seed;   // graph replays: the step's seed lives on the device
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  if (idx < (int64_t)npix * c) {
    const int64_t p = idx / c;
    const int k = (int)(idx - p * c);
    const float yv = to_f(y[p * ldy + k]);
    const float m = to_f(mu[p * ldmu + k]);
    const float v = fabsf((yv + noise_u(seed, (uint64_t)idx)) - m);
    const float s = fmaxf(to_f(sc[p * ldsc + k]), sbound);
    const float cst = -0.70710678118654752440f;
    const float L = 0.5f * erfcf(cst * ((0.5f - v) / s)) - 0.5f * erfcf(cst * ((-0.5f - v) / s));
    acc = (double)logf(fmaxf(L, lbound));
    if (yhat) yhat[p * ldyh + k] = from_f<T>(rintf(yv - m) + m);
  }
  const double t = block_sum_f64_256(acc, red);
  if (threadIdx.x == 0) parts[blockIdx.x] = t;
}

template <typename T>
__global__ void rate_train_bwd_kernel(const T* __restrict__ y, int ldy, const T* __restrict__ mu, int ldmu,
                                      const T* __restrict__ sc, int ldsc, int npix, int c, uint64_t seed,
                                      const uint64_t* seed_dev, uint64_t seed_mul,
                                      float sbound, float lbound, const float* __restrict__ gout, float factor,
                                      T* __restrict__ dy, int lddy, T* __restrict__ dmu, int lddmu,
                                      T* __restrict__ dsc, int lddsc) {
  if (seed_dev) seed = seed_dev[0] * seed_mul + seed;   // graph replays: the step's seed lives on the device
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int k = (int)(idx - p * c);
  const float yv = to_f(y[p * ldy + k]);
  const float m = to_f(mu[p * ldmu + k]);
  const float val = (yv + noise_u(seed, (uint64_t)idx)) - m;
  const float v = fabsf(val);
  const float scr = to_f(sc[p * ldsc + k]);
  const float s = fmaxf(scr, sbound);
  const float cst = -0.70710678118654752440f;
  const float aa = (0.5f - v) / s, bb = (-0.5f - v) / s;
  const float L = 0.5f * erfcf(cst * aa) - 0.5f * erfcf(cst * bb);
  const float Lb = fmaxf(L, lbound);
  const float dLb = gout[0] * factor / Lb;                       // d(sum ln L') / dL'
  const float dL = (L >= lbound || dLb < 0.f) ? dLb : 0.f;       // LowerBound(L, 1e-9)
  const float pa = 0.39894228040143268f * expf(-0.5f * aa * aa);
  const float pb = 0.39894228040143268f * expf(-0.5f * bb * bb);
  const float dv = dL * (pb - pa) / s;
  const float dsv = -dL * (pa * (0.5f - v) + pb * (0.5f + v)) / (s * s);
  const float ds = (scr >= sbound || dsv < 0.f) ? dsv : 0.f;     // LowerBound(scale, 0.11)
  const float sgn = val > 0.f ? 1.f : (val < 0.f ? -1.f : 0.f);
  const float dval = dv * sgn;
  dy[p * lddy + k] = from_f<T>(dval);
  dmu[p * lddmu + k] = from_f<T>(-dval);
  dsc[p * lddsc + k] = from_f<T>(ds);
}

// ---------------------------------------------------------------------------- recon head (train)
// x~ = tanh(W_b x16) per image (batch_conv + tanh, net_ga.py:969-979,1092); MSE partials vs the
// NCHW fp32 image; backward: dpre = g*factor*(x~ - x)(1 - x~^2), dx16 = W_b^T dpre, dW_b partials.
template <typename T>
__global__ __launch_bounds__(256) void recon_train_fwd_kernel(const T* __restrict__ x16, int ldx, int hw, int cin,
                                                              const T* __restrict__ wgen, int ldw,
                                                              const float* __restrict__ img, float* __restrict__ xt,
                                                              double* __restrict__ parts) {
  __shared__ double red[4];
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  double acc = 0.0;
  if (p < hw) {
    const T* xr = x16 + ((int64_t)b * hw + p) * ldx;
    const T* wr = wgen + (int64_t)b * ldw;
    for (int o = 0; o < 3; ++o) {
      float v = 0.f;
      for (int cc = 0; cc < cin; ++cc) v += to_f(wr[o * cin + cc]) * to_f(xr[cc]);
      const float t = tanhf(v);
      const int64_t q = ((int64_t)b * 3 + o) * hw + p;
      if (xt) xt[q] = t;
      const float e = t - img[q];
      acc += (double)(e * e);
    }
  }
  const double t = block_sum_f64_256(acc, red);
  if (threadIdx.x == 0) parts[(int64_t)b * gridDim.x + blockIdx.x] = t;
}

template <typename T>
__global__ __launch_bounds__(256) void recon_train_bwd_kernel(const T* __restrict__ x16, int ldx, int hw, int cin,
                                                              const T* __restrict__ wgen, int ldw,
                                                              const float* __restrict__ img,
                                                              const float* __restrict__ gout, float factor,
                                                              T* __restrict__ dx16, int lddx,
                                                              float* __restrict__ wparts) {
  __shared__ float red[4][48];
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dpre[3] = {0.f, 0.f, 0.f};
  float xv[16];
  const bool ok = p < hw;
  const T* wr = wgen + (int64_t)b * ldw;
  if (ok) {
    const T* xr = x16 + ((int64_t)b * hw + p) * ldx;
    for (int cc = 0; cc < cin; ++cc) xv[cc] = to_f(xr[cc]);
    const float g = gout[0] * factor;
    for (int o = 0; o < 3; ++o) {
      float v = 0.f;
      for (int cc = 0; cc < cin; ++cc) v += to_f(wr[o * cin + cc]) * xv[cc];
      const float t = tanhf(v);
      const int64_t q = ((int64_t)b * 3 + o) * hw + p;
      dpre[o] = g * (t - img[q]) * (1.f - t * t);
    }
    T* dr = dx16 + ((int64_t)b * hw + p) * lddx;
    for (int cc = 0; cc < cin; ++cc) {
      float s = 0.f;
      for (int o = 0; o < 3; ++o) s += to_f(wr[o * cin + cc]) * dpre[o];
      dr[cc] = from_f<T>(s);
    }
  } else {
    for (int cc = 0; cc < 16; ++cc) xv[cc] = 0.f;
  }
  // dW_b[o][cc] partial over this block's pixels
  for (int k = 0; k < 3 * cin; ++k) {
    float v = ok ? dpre[k / cin] * xv[k % cin] : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * cin; k += 256)
    wparts[((int64_t)b * gridDim.x + blockIdx.x) * 3 * cin + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

__global__ void recon_wreduce_kernel(const float* __restrict__ wparts, int nblk, int n48, int B,
                                     float* __restrict__ dw) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * n48) return;
  const int b = idx / n48, k = idx % n48;
  float s = 0.f;
  for (int q = 0; q < nblk; ++q) s += wparts[((int64_t)b * nblk + q) * n48 + k];
  dw[idx] = s;
}

// ---------------------------------------------------------------------------- depthwise wgrad
// dW[c][t] = sum_pix dz[pix, c] * x[pix*s + tap_t, c] (groups = C conv, Syntax_Model's
// DepthwiseSeparableConv); one thread per (tap, channel) chunk of pixels, partials + reduce.
template <typename T>
__global__ void dw_wgrad_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ dz, int ldz, int n, int h,
                                int w, int ho, int wo, int c, int stride, int ntaps, const DwTaps tp, int per,
                                float* __restrict__ parts) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // ch * ntaps + t (torch [C, 1, kh, kw] order)
  if (idx >= ntaps * c) return;
  const int ch = idx / ntaps, t = idx % ntaps;
  const int K = n * ho * wo;
  const int k0 = blockIdx.y * per, k1 = min(K, k0 + per);
  const int ty = tp.dy[t], tx = tp.dx[t];
  float s = 0.f;
  for (int k = k0; k < k1; ++k) {
    const int b = k / (ho * wo), rem = k % (ho * wo), i = rem / wo, j = rem % wo;
    const int iy = i * stride + ty, ix = j * stride + tx;
    if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w)
      s += to_f(dz[(int64_t)k * ldz + ch]) * to_f(x[(((int64_t)b * h + iy) * w + ix) * ldx + ch]);
  }
  parts[(int64_t)blockIdx.y * ntaps * c + idx] = s;
}

// ---------------------------------------------------------------------------- small elementwise
// AdaptiveAvgPool2d(1) backward: dx[b, p, c] = dy[b, c] / hw
template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, int lddy, int hw, int c, int64_t total,
                                   T* __restrict__ dx, int lddx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  dx[p * lddx + ch] = from_f<T>(to_f(dy[(p / hw) * lddy + ch]) / (float)hw);
}

// y = r + 0.5 tanh(x) (LRP, net_ga.py:1060-1062); backward dx = dy * 0.5 (1 - tanh(x)^2), dr = dy
template <typename T>
__global__ void half_tanh_fwd_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ r, int ldr, int npix,
                                     int c, T* __restrict__ y, int ldy) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  y[p * ldy + ch] = from_f<T>(to_f(r[p * ldr + ch]) + 0.5f * tanhf(to_f(x[p * ldx + ch])));
}

template <typename T>
__global__ void half_tanh_bwd_kernel(const T* __restrict__ x, int ldx, const T* __restrict__ dy, int lddy, int npix,
                                     int c, T* __restrict__ dx, int lddx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)npix * c) return;
  const int64_t p = idx / c;
  const int ch = (int)(idx - p * c);
  const float t = tanhf(to_f(x[p * ldx + ch]));
  dx[p * lddx + ch] = from_f<T>(to_f(dy[p * lddy + ch]) * 0.5f * (1.f - t * t));
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
    } else if ((dtype) == LIC_BF16) {                                   \
      typedef bf16_t T;                                                 \
      __VA_ARGS__;                                                      \
    } else                                                              \
      return fail(std::string(NAME) + ": dtype must be LIC_F32, LIC_F16 or LIC_BF16"); \
  } while (0)

static inline unsigned tr_nblk(int64_t total) { return (unsigned)((total + 255) / 256); }

// wgrad_tr.hip: the tiled 16-bit kernel (all taps of a tap group per work-group, transpose reads)
namespace lic {
int wgrad_tr_nsplit(const lic_wgrad_args& a);
// Many wgrad_reduce_kernel launches in one (lic_wgrad_reduce_batch): block b finds its descriptor by
// binary search over the ascending first blocks and runs the same per-element sum (same order).
__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(const int64_t* __restrict__ desc, int n) {
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[(int64_t)mid * LIC_WGRAD_RED_DESC_WORDS + 14] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* d = desc + (int64_t)lo * LIC_WGRAD_RED_DESC_WORDS;
  const int64_t idx = (int64_t)(b - (int)d[14]) * 256 + threadIdx.x;
  const int ntaps = (int)d[8], co = (int)d[9], ci = (int)d[10], co_out = (int)d[11], ci_out = (int)d[12];
  const int64_t total = (int64_t)ntaps * co_out * ci_out;
  const float* wsb = (const float*)d[1];
  float* db = (float*)d[3];
  const int nsplit = (int)d[7], accumulate = (int)d[13];
  if (idx >= total) {
    const int nn = (int)(idx - total);
    if (!wsb || nn >= co_out) return;
    float b0 = 0.f, b1 = 0.f;
    int k = 0;
    for (; k + 2 <= nsplit; k += 2) {
      b0 += wsb[(int64_t)k * co + nn];
      b1 += wsb[(int64_t)(k + 1) * co + nn];
    }
    if (k < nsplit) b0 += wsb[(int64_t)k * co + nn];
    db[nn] = accumulate ? db[nn] + (b0 + b1) : b0 + b1;
    return;
  }
  const float* ws = (const float*)d[0];
  float* dw = (float*)d[2];
  const int c = (int)(idx % ci_out);
  const int64_t r = idx / ci_out;
  const int nn = (int)(r % co_out);
  const int t = (int)(r / co_out);
  const int64_t stride = (int64_t)ntaps * co * ci;
  const float* p = ws + ((int64_t)t * co + nn) * ci + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 4 <= nsplit; k += 4) {
    s0 += p[k * stride];
    s1 += p[(k + 1) * stride];
    s2 += p[(k + 2) * stride];
    s3 += p[(k + 3) * stride];
  }
  for (; k < nsplit; ++k) s0 += p[k * stride];
  const float sm = (s0 + s1) + (s2 + s3);
  float* o = dw + nn * d[4] + c * d[5] + t * d[6];
  *o = accumulate ? *o + sm : sm;
}

int wgrad_tr_launch(const lic_wgrad_args& a, hipStream_t s, int* nsplit);
}  // namespace lic

// workspace: [nsplit][tap][co][ci] fp32 partials, then (db requested) the bias partials: [nsplit][co]
// for the tiled kernel, the channel-sum parts [CS_CHUNKS][co] otherwise
static int64_t wgrad_ws_bytes(const lic_wgrad_args& a, int* nsplit_out, bool* tiled_out) {
  const int tr = wgrad_tr_nsplit(a);
  const int ns = tr ? tr : wgrad_plan(a).nsplit;
  if (nsplit_out) *nsplit_out = ns;
  if (tiled_out) *tiled_out = tr != 0;
  int64_t b = (int64_t)ns * a.ntaps * a.co * a.ci;
  if (a.db) b += (int64_t)(tr ? ns : CS_CHUNKS) * a.co;
  return b * (int64_t)sizeof(float);
}

extern "C" int64_t lic_conv2d_wgrad_workspace(const lic_wgrad_args* a) {
  if (!a || wgrad_check(*a)) return -1;
  return wgrad_ws_bytes(*a, nullptr, nullptr);
}

extern "C" int lic_conv2d_wgrad_partials(const lic_wgrad_args* ap, int32_t* nsplit_out, lic_stream_t stream) {
  if (!ap || !nsplit_out) return fail("wgrad partials: null args");
  const lic_wgrad_args& a = *ap;
  if (int e = wgrad_check(a)) return e;
  int nsplit = 0;
  bool tiled = false;
  const int64_t need = wgrad_ws_bytes(a, &nsplit, &tiled);
  if (!tiled) {   // the generic kernel: the whole wgrad now, nothing left to defer
    *nsplit_out = 0;
    return lic_conv2d_wgrad(ap, stream);
  }
  if (!a.ws || a.ws_bytes < need)
    return fail("wgrad partials: workspace too small (" + std::to_string(a.ws_bytes) + " < " + std::to_string(need) + ")");
  int ns = 0;
  if (int e = wgrad_tr_launch(a, (hipStream_t)stream, &ns)) return e;
  *nsplit_out = ns;
  return 0;
}

extern "C" int32_t lic_wgrad_reduce_blocks(const lic_wgrad_args* a) {
  if (!a) return -1;
  const int64_t total = (int64_t)a->ntaps * a->co_out * a->ci_out + (a->db ? a->co_out : 0);
  return (int32_t)((total + 255) / 256);
}

extern "C" int lic_wgrad_reduce_batch(const int64_t* desc, int32_t n, int32_t nblocks, lic_stream_t stream) {
  if (!desc || n <= 0 || nblocks <= 0) return fail("lic_wgrad_reduce_batch: need descriptors and blocks");
  hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, desc, n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(std::string("lic_wgrad_reduce_batch: ") + hipGetErrorString(e));
}

extern "C" int lic_conv2d_wgrad(const lic_wgrad_args* ap, lic_stream_t stream) {
  if (!ap) return fail("wgrad: null args");
  const lic_wgrad_args& a = *ap;
  if (int e = wgrad_check(a)) return e;
  const WgPlan p = wgrad_plan(a);
  int nsplit = 0;
  bool tiled = false;
  const int64_t need = wgrad_ws_bytes(a, &nsplit, &tiled);
  const int tr_ns = tiled ? nsplit : 0;
  if (!a.ws || a.ws_bytes < need)
    return fail("wgrad: workspace too small (" + std::to_string(a.ws_bytes) + " < " + std::to_string(need) + ")");
  hipStream_t s = (hipStream_t)stream;
  if (tr_ns) {
    int ns = 0;
    if (int e = wgrad_tr_launch(a, s, &ns)) return e;
  } else if (a.dtype == LIC_F16) {
    if (p.bm == 128) wgrad_launch<half_t, 128, 128, 2, 2>(a, p, s);
    else wgrad_launch<half_t, 64, 64, 2, 2>(a, p, s);
  } else if (a.dtype == LIC_BF16) {
    if (p.bm == 128) wgrad_launch<bf16_t, 128, 128, 2, 2>(a, p, s);
    else wgrad_launch<bf16_t, 64, 64, 2, 2>(a, p, s);
  } else {
    if (p.bm == 128) wgrad_launch<float, 128, 128, 2, 2>(a, p, s);
    else wgrad_launch<float, 64, 64, 2, 2>(a, p, s);
  }
  LIC_CHECK_LAUNCH();
  const int64_t total = (int64_t)a.ntaps * a.co_out * a.ci_out;
  float* const wsb = a.ws + (int64_t)nsplit * a.ntaps * a.co * a.ci;
  const bool fused_db = a.db && tiled;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(tr_nblk(total + (fused_db ? a.co_out : 0))), dim3(256), 0, s, a.ws,
                     nsplit, a.ntaps, a.co, a.ci, a.co_out, a.ci_out, a.dw, a.s_co, a.s_ci, a.s_tap, a.accumulate,
                     fused_db ? wsb : nullptr, a.db);
  LIC_CHECK_LAUNCH();
  if (a.db && !tiled) {   // generic kernel: the two-pass channel sum over dz
    const int npix = a.n * a.ho * a.wo;
    const int per = std::max(1, (npix + CS_CHUNKS - 1) / CS_CHUNKS);
    const int nparts = std::max(1, (npix + per - 1) / per);
    TR_DISPATCH(a.dtype, "wgrad db",
                hipLaunchKernelGGL(channel_sum_partial_kernel<T>, dim3(nparts, (a.co_out + 63) / 64), dim3(256), 0, s,
                                   (const T*)a.dz, a.ldz, npix, a.co_out, per, wsb));
    LIC_CHECK_LAUNCH();
    hipLaunchKernelGGL(channel_sum_reduce_kernel, dim3((a.co_out + 63) / 64), dim3(1024), 0, s, wsb, nparts, a.co_out,
                       a.db, a.accumulate);
    LIC_CHECK_LAUNCH();
  }
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
                hipLaunchKernelGGL(channel_sum_partial_kernel<T>, dim3(nparts, (c + 63) / 64), dim3(256), 0, s,
                                   (const T*)x, ldx, npix, c, per, ws));
    LIC_CHECK_LAUNCH();
  } else {
    (void)hipMemsetAsync(ws, 0, (size_t)c * sizeof(float), s);
  }
  cs_reduce(ws, npix > 0 ? nparts : 1, c, out, accumulate, s);
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

extern "C" int64_t lic_win_attn_bwd_workspace(const lic_attn_args* a) {
  if (!a || a->ws <= 0 || a->heads <= 0) return -1;
  const int R = (2 * a->ws - 1) * (2 * a->ws - 1);
  return (int64_t)a->heads * a->n * (a->h / a->ws) * (a->w / a->ws) * R * (int64_t)sizeof(float);
}

extern "C" int lic_win_attn_bwd(const lic_attn_args* ap, const void* dout, int32_t lddo, void* dqkv, int32_t lddq,
                                float* dtable, int32_t accumulate_table, float* ws, int64_t ws_bytes,
                                lic_stream_t stream) {
  if (!ap || !ap->qkv || !dout || !dqkv || !ap->table) return fail("attn_bwd: null tensor");
  const lic_attn_args& a = *ap;
  if (a.heads <= 0 || a.c % a.heads) return fail("attn_bwd: C % heads != 0");
  if (a.ws <= 0 || a.h % a.ws || a.w % a.ws) return fail("attn_bwd: H, W must be multiples of the window");
  if (a.shift < 0 || a.shift >= a.ws) return fail("attn_bwd: 0 <= shift < ws");
  if ((int64_t)a.n * a.h * a.w == 0) return 0;
  const int N = a.ws * a.ws, d = a.c / a.heads, R = (2 * a.ws - 1) * (2 * a.ws - 1);
  const size_t shm = (size_t)(4 * N * (d + 1) + N * (N + 1) + N + R) * sizeof(float);
  if (shm > 64 * 1024) return fail("attn_bwd: window x head_dim too large for LDS");
  const int64_t need = lic_win_attn_bwd_workspace(ap);
  if (dtable && (!ws || ws_bytes < need)) return fail("attn_bwd: workspace too small");
  const int nwin = a.n * (a.h / a.ws) * (a.w / a.ws);
  const int64_t blocks = (int64_t)nwin * a.heads;
  hipStream_t s = (hipStream_t)stream;
  float* tp = dtable ? ws : nullptr;
  // 8x8 windows with a head dim of 16 / 24 / 32: the register-blocked kernel (LIC_ATTN_BWD64=0: generic)
  static const int blk_on = wd_env("LIC_ATTN_BWD64", 1);
  bool done = false;
  if (blk_on && N == 64 && (d == 16 || d == 24 || d == 32)) {
    const size_t shm64 = (size_t)(4 * 64 * (d + 4) + 2 * 64 * 65 + 2 * 225) * sizeof(float);
#define ATTN64(DD)                                                                                             \
  if (d == DD) {                                                                                                 \
    TR_DISPATCH(a.dtype, "attn_bwd64", {                                                                        \
      const hipError_t ea = ensure_dyn_lds((const void*)win_attn_bwd64_kernel<T, DD>, (int)shm64);             \
      if (ea != hipSuccess) return fail(std::string("attn_bwd64: dynamic LDS: ") + hipGetErrorString(ea));      \
      hipLaunchKernelGGL((win_attn_bwd64_kernel<T, DD>), dim3((unsigned)blocks), dim3(256), shm64, s, a,         \
                         (const T*)dout, lddo, (T*)dqkv, lddq, tp);                                            \
    });                                                                                                          \
    done = true;                                                                                                 \
  }
    ATTN64(16)
    ATTN64(24)
    ATTN64(32)
#undef ATTN64
  }
  if (!done)
    TR_DISPATCH(a.dtype, "attn_bwd",
                hipLaunchKernelGGL(win_attn_bwd_kernel<T>, dim3((unsigned)blocks), dim3(256), shm, s, a,
                                   (const T*)dout, lddo, (T*)dqkv, lddq, tp));
  LIC_CHECK_LAUNCH();
  if (dtable) {
    const int nrb = (R + 15) / 16;
    hipLaunchKernelGGL(attn_table_reduce16_kernel, dim3((unsigned)(a.heads * nrb)), dim3(256), 0, s, ws, a.heads,
                       nwin, R, dtable, a.tab_sr, a.tab_sh, accumulate_table);
    LIC_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int64_t lic_layernorm_bwd_workspace(int32_t npix, int32_t c) {
  const int blocks = std::max(1, std::min(256, (npix + 3) / 4));
  return (int64_t)blocks * 2 * c * (int64_t)sizeof(float);
}

extern "C" int lic_layernorm_bwd(int32_t dtype, const void* x, int32_t ldx, const void* dy, int32_t lddy,
                                 int32_t npix, int32_t c, const float* weight, float eps, void* dx, int32_t lddx,
                                 float* dwb, int32_t accumulate, float* ws, int64_t ws_bytes, lic_stream_t stream) {
  if (npix <= 0 || c <= 0) return 0;
  if (c > 64 * 12) return fail("layernorm_bwd: C > 768");
  const int blocks = std::max(1, std::min(256, (npix + 3) / 4));
  if (ws_bytes < lic_layernorm_bwd_workspace(npix, c)) return fail("layernorm_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int cpl = (c + 63) / 64;
#define LNB(CPL)                                                                                                  \
  TR_DISPATCH(dtype, "layernorm_bwd",                                                                            \
              hipLaunchKernelGGL((layernorm_bwd_kernel<T, CPL>), dim3(blocks), dim3(256), 0, s, (const T*)x, ldx, \
                                 (const T*)dy, lddy, npix, c, weight, eps, (T*)dx, lddx, ws))
  if (cpl <= 2) LNB(2);
  else if (cpl <= 4) LNB(4);
  else if (cpl <= 8) LNB(8);
  else LNB(12);
#undef LNB
  LIC_CHECK_LAUNCH();
  cs_reduce(ws, blocks, 2 * c, dwb, accumulate, s);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_gate_fwd(int32_t dtype, const void* a, int32_t lda, const void* g, int32_t ldg, const void* r,
                            int32_t ldr, int32_t npix, int32_t c, void* y, int32_t ldy, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "gate_fwd",
              hipLaunchKernelGGL(gate_fwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)a, lda, (const T*)g, ldg, (const T*)r, ldr, npix, c, (T*)y, ldy));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int32_t lic_rate_train_parts(int32_t npix, int32_t c) { return (int32_t)tr_nblk((int64_t)npix * c); }

extern "C" int lic_rate_train_fwd(int32_t dtype, const void* y, int32_t ldy, const void* mu, int32_t ldmu,
                                  const void* scale, int32_t ldsc, int32_t npix, int32_t c, uint64_t seed,
                                  const uint64_t* seed_dev, uint64_t seed_mul,
                                  float scale_bound, float likelihood_bound, void* yhat, int32_t ldyh,
                                  double* partials, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "rate_train_fwd",
              hipLaunchKernelGGL(rate_train_fwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)y, ldy, (const T*)mu, ldmu, (const T*)scale, ldsc, npix, c, seed,
                                 seed_dev, seed_mul, scale_bound, likelihood_bound, (T*)yhat, ldyh, partials));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_rate_train_bwd(int32_t dtype, const void* y, int32_t ldy, const void* mu, int32_t ldmu,
                                  const void* scale, int32_t ldsc, int32_t npix, int32_t c, uint64_t seed,
                                  const uint64_t* seed_dev, uint64_t seed_mul,
                                  float scale_bound, float likelihood_bound, const float* gout, float factor,
                                  void* dy, int32_t lddy, void* dmu, int32_t lddmu, void* dscale, int32_t lddsc,
                                  lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "rate_train_bwd",
              hipLaunchKernelGGL(rate_train_bwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)y, ldy, (const T*)mu, ldmu, (const T*)scale, ldsc, npix, c, seed,
                                 seed_dev, seed_mul, scale_bound, likelihood_bound, gout, factor, (T*)dy, lddy, (T*)dmu, lddmu,
                                 (T*)dscale, lddsc));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int32_t lic_recon_train_blocks(int32_t hw) { return (hw + 255) / 256; }

extern "C" int lic_recon_train_fwd(int32_t dtype, const void* x16, int32_t ldx, int32_t n, int32_t hw, int32_t cin,
                                   const void* wgen, int32_t ldw, const float* img, float* xt, double* partials,
                                   lic_stream_t stream) {
  if (cin > 16 || cin <= 0) return fail("recon_train: cin must be 1..16");
  if (n <= 0 || hw <= 0) return 0;
  dim3 grid((hw + 255) / 256, n);
  TR_DISPATCH(dtype, "recon_train_fwd",
              hipLaunchKernelGGL(recon_train_fwd_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)x16,
                                 ldx, hw, cin, (const T*)wgen, ldw, img, xt, partials));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_recon_train_bwd(int32_t dtype, const void* x16, int32_t ldx, int32_t n, int32_t hw, int32_t cin,
                                   const void* wgen, int32_t ldw, const float* img, const float* gout, float factor,
                                   void* dx16, int32_t lddx, float* dw, float* ws, int64_t ws_bytes,
                                   lic_stream_t stream) {
  if (cin > 16 || cin <= 0) return fail("recon_train: cin must be 1..16");
  if (n <= 0 || hw <= 0) return 0;
  const int nblk = (hw + 255) / 256;
  if (ws_bytes < (int64_t)n * nblk * 3 * cin * (int64_t)sizeof(float)) return fail("recon_train_bwd: workspace");
  hipStream_t s = (hipStream_t)stream;
  TR_DISPATCH(dtype, "recon_train_bwd",
              hipLaunchKernelGGL(recon_train_bwd_kernel<T>, dim3(nblk, n), dim3(256), 0, s, (const T*)x16, ldx, hw,
                                 cin, (const T*)wgen, ldw, img, gout, factor, (T*)dx16, lddx, ws));
  LIC_CHECK_LAUNCH();
  hipLaunchKernelGGL(recon_wreduce_kernel, dim3((n * 3 * cin + 255) / 256), dim3(256), 0, s, ws, nblk, 3 * cin, n,
                     dw);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t lic_dwconv_wgrad_workspace(int32_t n, int32_t ho, int32_t wo, int32_t c, int32_t ntaps) {
  const int K = n * ho * wo;
  const int nsplit = std::max(1, std::min(256, K / 64));
  return (int64_t)nsplit * ntaps * c * (int64_t)sizeof(float);
}

extern "C" int lic_avgpool_bwd(int32_t dtype, const void* dy, int32_t lddy, int32_t n, int32_t hw, int32_t c,
                               void* dx, int32_t lddx, lic_stream_t stream) {
  const int64_t total = (int64_t)n * hw * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "avgpool_bwd",
              hipLaunchKernelGGL(avgpool_bwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)dy, lddy, hw, c, total, (T*)dx, lddx));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_half_tanh_fwd(int32_t dtype, const void* x, int32_t ldx, const void* r, int32_t ldr, int32_t npix,
                                 int32_t c, void* y, int32_t ldy, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "half_tanh_fwd",
              hipLaunchKernelGGL(half_tanh_fwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)x, ldx, (const T*)r, ldr, npix, c, (T*)y, ldy));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_half_tanh_bwd(int32_t dtype, const void* x, int32_t ldx, const void* dy, int32_t lddy,
                                 int32_t npix, int32_t c, void* dx, int32_t lddx, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (!total) return 0;
  TR_DISPATCH(dtype, "half_tanh_bwd",
              hipLaunchKernelGGL(half_tanh_bwd_kernel<T>, dim3(tr_nblk(total)), dim3(256), 0, (hipStream_t)stream,
                                 (const T*)x, ldx, (const T*)dy, lddy, npix, c, (T*)dx, lddx));
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_dwconv_wgrad(int32_t dtype, const void* x, int32_t ldx, const void* dz, int32_t ldz, int32_t n,
                                int32_t h, int32_t w, int32_t ho, int32_t wo, int32_t c, int32_t stride,
                                int32_t ntaps, const int8_t* dy_host, const int8_t* dx_host, float* dw, float* ws,
                                int64_t ws_bytes, lic_stream_t stream) {
  if (ntaps <= 0 || ntaps > LIC_MAX_TAPS) return fail("dwconv_wgrad: ntaps");
  const int K = n * ho * wo;
  if (K <= 0) return 0;
  const int nsplit = std::max(1, std::min(256, K / 64));
  const int per = (K + nsplit - 1) / nsplit;
  const int64_t need = (int64_t)nsplit * ntaps * c * (int64_t)sizeof(float);
  if (ws_bytes < need) return fail("dwconv_wgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  DwTaps tp;
  for (int t = 0; t < ntaps; ++t) { tp.dy[t] = dy_host[t]; tp.dx[t] = dx_host[t]; }
  dim3 grid((ntaps * c + 255) / 256, nsplit);
  TR_DISPATCH(dtype, "dwconv_wgrad",
              hipLaunchKernelGGL(dw_wgrad_kernel<T>, grid, dim3(256), 0, s, (const T*)x, ldx, (const T*)dz, ldz, n, h,
                                 w, ho, wo, c, stride, ntaps, tp, per, ws));
  LIC_CHECK_LAUNCH();
  cs_reduce(ws, nsplit, ntaps * c, dw, 0, s);
  LIC_CHECK_LAUNCH();
  return 0;
}
