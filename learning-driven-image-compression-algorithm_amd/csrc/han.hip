// HAN post-processing (reference model/han.py, called at
// net_ga.py:1096-1100): the non-convolution pieces.  Every 3x3 / 1x1 convolution of
// HAN runs on the MFMA conv kernels (lic_conv2d_fwd); these kernels are the
// HBM-bound glue around them:
//   ca_apply   CALayer + RCAB residual: out = r * sigmoid(W2 relu(W1 avg(r) + b1) + b2) + x
//   lam_gram / lam_apply   LAM_Module: per-image N x N Gram of the stacked group outputs,
//              softmax(max - energy), out_n = gamma * sum_m A[n][m] x_m + x_n
//   csam       CSAM_Module: out = x * (gamma * sigmoid(conv3d_3x3x3(x) + b)) + x, the 3-D
//              kernel sliding over (channel, y, x) of the NHWC map
// plus the generalised batch-conv reconstruction (lic_recon_fwd) that closes the path.
#include "lic_common.h"
#include <algorithm>

namespace lic {

__device__ __forceinline__ double block_sum_f64_256(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];  // valid in every thread
}

// Channel-vector mapping shared by the HAN glue kernels: a pixel's C channels are
// C/V vectors of 16 bytes (V = 8 fp16 / 4 fp32; V = 1 on the scalar path), tpp = C/V
// threads cover one pixel, 256/tpp pixels per block iteration; all index math is
// 32-bit (the host guarantees n*hw*ld < 2^31).
template <typename T, bool VEC>
struct ChanMap {
  static constexpr int V = VEC ? 16 / (int)sizeof(T) : 1;
  int tpp, ppi, cg, po;
  __device__ ChanMap(int c, int tid) {
    tpp = c / V;
    ppi = 256 / tpp;
    cg = tid % tpp;
    po = tid / tpp;
  }
};

template <typename T, bool VEC>
__device__ __forceinline__ void ld_chan(const T* p, float* f) {
  if constexpr (VEC) load_vec<T>(p, f);
  else f[0] = to_f(*p);
}

template <typename T, bool VEC>
__device__ __forceinline__ void st_chan(T* p, const float* f) {
  if constexpr (VEC) store_vec<T>(p, f);
  else *p = from_f<T>(f[0]);
}

// per-(image, pixel chunk) channel sums: grid (nchunk, n)
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void pool_partials_kernel(const T* __restrict__ x, int ldx, int hw, int c,
                                                            int nchunk, float* __restrict__ parts) {
  __shared__ float red[256 * 8];
  const ChanMap<T, VEC> m(c, threadIdx.x);
  constexpr int V = ChanMap<T, VEC>::V;
  const int b = blockIdx.y, k = blockIdx.x;
  const int per = (hw + nchunk - 1) / nchunk;
  const int p0 = k * per, p1 = min(hw, p0 + per);
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  if (m.po < m.ppi) {
    const T* xb = x + (b * hw) * ldx + m.cg * V;
    for (int p = p0 + m.po; p < p1; p += m.ppi) {
      float f[V];
      ld_chan<T, VEC>(xb + p * ldx, f);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += f[j];
    }
    // po-major staging: red[po * c + channel]
#pragma unroll
    for (int j = 0; j < V; ++j) red[m.po * c + m.cg * V + j] = acc[j];
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += 256) {
    float s = 0.f;
    for (int q = 0; q < m.ppi; ++q) s += red[q * c + ch];
    parts[(b * nchunk + k) * c + ch] = s;
  }
}

// CALayer weights: one workgroup per image reduces the pooling partials (all 256
// threads), runs the 2-layer MLP and writes y[b][c] (fp32) after the partials.
__global__ __launch_bounds__(256) void ca_weights_kernel(const float* __restrict__ parts, int nchunk, int hw, int c,
                                                         const float* __restrict__ w1, const float* __restrict__ b1,
                                                         const float* __restrict__ w2, const float* __restrict__ b2,
                                                         int cr, float* __restrict__ y) {
  __shared__ float pv[256], hid[32];
  __shared__ float part[4][256];
  const int b = blockIdx.x, tid = threadIdx.x;
  // thread (q4 = tid / 64, ch0 = tid % 64): channels ch0, ch0+64, ... over chunks q4, q4+4, ...
  const int q4 = tid >> 6, ch0 = tid & 63;
  for (int k = ch0; k < c; k += 64) {
    float s = 0.f;
    for (int q = q4; q < nchunk; q += 4) s += parts[(b * nchunk + q) * c + k];
    part[q4][k] = s;
  }
  __syncthreads();
  const float inv = 1.0f / (float)hw;
  for (int k = tid; k < c; k += 256) pv[k] = (part[0][k] + part[1][k] + part[2][k] + part[3][k]) * inv;
  __syncthreads();
  if (tid < cr) {
    float s = 0.f;
    for (int k = 0; k < c; ++k) s += w1[tid * c + k] * pv[k];
    s += b1[tid];
    hid[tid] = s > 0.f ? s : 0.f;
  }
  __syncthreads();
  for (int k = tid; k < c; k += 256) {
    float s = 0.f;
    for (int j = 0; j < cr; ++j) s += w2[k * cr + j] * hid[j];
    s += b2[k];
    y[b * c + k] = 1.0f / (1.0f + expf(-s));
  }
}

// CALayer + RCAB residual: out = r * y[b] + x; grid (chunks, n).
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ca_apply_kernel(const T* __restrict__ r, int ldr, const T* __restrict__ x,
                                                       int ldx, int hw, int c, const float* __restrict__ y,
                                                       T* __restrict__ out, int ldo) {
  const int b = blockIdx.y;
  const ChanMap<T, VEC> m(c, threadIdx.x);
  constexpr int V = ChanMap<T, VEC>::V;
  if (m.po >= m.ppi) return;
  const int per = (hw + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(hw, p0 + per);
  float yv[V];
#pragma unroll
  for (int j = 0; j < V; ++j) yv[j] = y[b * c + m.cg * V + j];
  for (int p = p0 + m.po; p < p1; p += m.ppi) {
    const int pix = b * hw + p;
    float fr[V], fx[V];
    ld_chan<T, VEC>(r + pix * ldr + m.cg * V, fr);
    ld_chan<T, VEC>(x + pix * ldx + m.cg * V, fx);
#pragma unroll
    for (int j = 0; j < V; ++j) fr[j] = __fadd_rn(__fmul_rn(fr[j], yv[j]), fx[j]);
    st_chan<T, VEC>(out + pix * ldo + m.cg * V, fr);
  }
}

// Gram partials: grid (nblk, n); each block sums x_i * x_j (i <= j < N) over its pixel
// range of one image and all C channels of each group (fp64 accumulation).
template <typename T, int N, bool VEC>
__global__ __launch_bounds__(256) void lam_gram_kernel(const T* __restrict__ x, int ldx, int hw, int C,
                                                       double* __restrict__ parts) {
  __shared__ double red[4];
  constexpr int NP = N * (N + 1) / 2;
  const ChanMap<T, VEC> m(C, threadIdx.x);
  constexpr int V = ChanMap<T, VEC>::V;
  const int b = blockIdx.y;
  double acc[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) acc[q] = 0.0;
  if (m.po < m.ppi) {
    const int per = (hw + gridDim.x - 1) / gridDim.x;
    const int p0 = blockIdx.x * per, p1 = min(hw, p0 + per);
    for (int p = p0 + m.po; p < p1; p += m.ppi) {
      const T* px = x + (b * hw + p) * ldx + m.cg * V;
      float v[N][V];
#pragma unroll
      for (int i = 0; i < N; ++i) ld_chan<T, VEC>(px + i * C, v[i]);
      int q = 0;
#pragma unroll
      for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = i; j < N; ++j) {
          float s = 0.f;
#pragma unroll
          for (int e = 0; e < V; ++e) s = fmaf(v[i][e], v[j][e], s);
          acc[q++] += (double)s;
        }
    }
  }
  double* dst = parts + ((int64_t)b * gridDim.x + blockIdx.x) * NP;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const double t = block_sum_f64_256(acc[q], red);
    if (threadIdx.x == 0) dst[q] = t;
  }
}

// One workgroup per image: reduce the Gram partials (NP sums spread over the waves,
// fixed order), softmax(max(E) - E) per row, A[b] (fp32 N x N) written after the partials.
template <int N>
__global__ __launch_bounds__(256) void lam_attn_kernel(const double* __restrict__ parts, int nblk,
                                                       float* __restrict__ A) {
  constexpr int NP = N * (N + 1) / 2;
  __shared__ double red[4];
  __shared__ double Es[NP];
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int q = 0; q < NP; ++q) {
    double s = 0.0;
    for (int k = tid; k < nblk; k += 256) s += parts[((int64_t)b * nblk + k) * NP + q];
    const double t = block_sum_f64_256(s, red);
    if (tid == 0) Es[q] = t;
  }
  __syncthreads();
  if (tid == 0) {
    double E[N][N];
    int q = 0;
    for (int i = 0; i < N; ++i)
      for (int j = i; j < N; ++j) {
        E[i][j] = E[j][i] = Es[q];
        ++q;
      }
    for (int i = 0; i < N; ++i) {
      float en[N];
      double mx = E[i][0];
      for (int j = 1; j < N; ++j) mx = E[i][j] > mx ? E[i][j] : mx;
      for (int j = 0; j < N; ++j) en[j] = (float)(mx - E[i][j]);        // energy_new
      float m2 = en[0];
      for (int j = 1; j < N; ++j) m2 = fmaxf(m2, en[j]);
      float sum = 0.f;
      for (int j = 0; j < N; ++j) {
        en[j] = expf(en[j] - m2);
        sum += en[j];
      }
      for (int j = 0; j < N; ++j) A[(b * N + i) * N + j] = en[j] / sum;
    }
  }
}

// grid (chunks, n): out_n = gamma * sum_m A[b][n][m] x_m + x_n over the block's pixels.
template <typename T, int N, bool VEC>
__global__ __launch_bounds__(256) void lam_apply_kernel(const T* __restrict__ x, int ldx, int hw, int C,
                                                        const float* __restrict__ Ag, const float* __restrict__ gamma,
                                                        T* __restrict__ out, int ldo) {
  __shared__ float A[N][N];
  const int b = blockIdx.y, tid = threadIdx.x;
  if (tid < N * N) A[tid / N][tid % N] = Ag[b * N * N + tid];
  __syncthreads();
  const ChanMap<T, VEC> m(C, tid);
  constexpr int V = ChanMap<T, VEC>::V;
  if (m.po >= m.ppi) return;
  const float g = gamma[0];
  const int per = (hw + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * per, p1 = min(hw, p0 + per);
  for (int p = p0 + m.po; p < p1; p += m.ppi) {
    const int pix = b * hw + p;
    const T* px = x + pix * ldx + m.cg * V;
    float v[N][V];
#pragma unroll
    for (int i = 0; i < N; ++i) ld_chan<T, VEC>(px + i * C, v[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < N; ++j) s += A[i][j] * v[j][e];
        o[e] = __fadd_rn(__fmul_rn(g, s), v[i][e]);
      }
      st_chan<T, VEC>(out + pix * ldo + i * C + m.cg * V, o);
    }
  }
}

// CSAM: params = {w[kd][kh][kw] (27), bias, gamma}
template <typename T>
__global__ __launch_bounds__(256) void csam_kernel(const T* __restrict__ x, int ldx, int n, int h, int w, int C,
                                                   const float* __restrict__ prm, T* __restrict__ out, int ldo) {
  __shared__ float wk[29];
  if (threadIdx.x < 29) wk[threadIdx.x] = prm[threadIdx.x];
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;   // host: n*h*w*C < 2^31
  if (e >= n * h * w * C) return;
  const int pix = e / C;
  const int k = e - pix * C;
  const int b = pix / (h * w);
  const int rem = pix - b * h * w;
  const int iy = rem / w, ix = rem - iy * w;
  float s = 0.f;
#pragma unroll
  for (int dd = 0; dd < 3; ++dd) {
    const int kc = k + dd - 1;
    if (kc < 0 || kc >= C) continue;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int yy = iy + dy - 1;
      if (yy < 0 || yy >= h) continue;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int xx = ix + dx - 1;
        if (xx < 0 || xx >= w) continue;
        s += wk[dd * 9 + dy * 3 + dx] * to_f(x[((b * h + yy) * w + xx) * ldx + kc]);
      }
    }
  }
  s += wk[27];
  const float sg = 1.0f / (1.0f + expf(-s));
  const float o = __fmul_rn(wk[28], sg);
  const float xv = to_f(x[pix * ldx + k]);
  out[pix * ldo + k] = from_f<T>(__fadd_rn(__fmul_rn(xv, o), xv));
}

// Per-image 1x1 "batch conv" (net_ga.py:969-979) with its finishing steps:
//   v = sum_c w[b][k][c] xtil[c]  (k < 3);  mode 1: v = tanh(v);  post: v = P v + p (1x1 3->3)
//   y (NHWC dtype, ycpad channels, zero padded) <- v;  x_rec (NCHW fp32) <- clamp(v, -1, 1)
//   parts[b][blk] <- sum (round(clamp((x_rec+1)*127.5)) - round((x+1)*127.5))^2   (x != NULL)
template <typename T>
__global__ __launch_bounds__(256) void recon_kernel(const T* __restrict__ xtil, int h, int w, int cin, int ldx,
                                                    int ldw, const T* __restrict__ wgen, int mode,
                                                    const float* __restrict__ post, const float* __restrict__ x,
                                                    float* __restrict__ xrec, double* __restrict__ parts,
                                                    int parts_per_img, T* __restrict__ y, int ldy, int ycpad) {
  __shared__ double red[4];
  __shared__ float ws[3 * 64];
  __shared__ float pm[12];
  const int b = blockIdx.y;
  for (int k = threadIdx.x; k < 3 * cin; k += 256) ws[k] = to_f(wgen[(int64_t)b * ldw + k]);
  if (post && threadIdx.x < 12) pm[threadIdx.x] = post[threadIdx.x];
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
    if (mode == 1) {
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] = tanhf(o[k]);
    }
    if (post) {
      float q[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) q[k] = pm[3 * k] * o[0] + pm[3 * k + 1] * o[1] + pm[3 * k + 2] * o[2] + pm[9 + k];
#pragma unroll
      for (int k = 0; k < 3; ++k) o[k] = q[k];
    }
    if (y) {
      T* yp = y + ((int64_t)b * hw + p) * ldy;
      for (int k = 0; k < ycpad; ++k) yp[k] = from_f<T>(k < 3 ? o[k] : 0.f);
    }
    if (xrec) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float t = fminf(fmaxf(o[k], -1.f), 1.f);
        const int64_t off = ((int64_t)b * 3 + k) * hw + p;
        xrec[off] = t;
        if (x) {
          const float gt = rintf(__fmul_rn(__fadd_rn(x[off], 1.f), 127.5f));
          float xh = __fmul_rn(__fadd_rn(t, 1.f), 127.5f);
          xh = rintf(fminf(fmaxf(xh, 0.f), 255.f));
          const float d = __fsub_rn(xh, gt);
          acc += (double)(d * d);
        }
      }
    }
  }
  if (x && parts) {
    const double t = block_sum_f64_256(acc, red);
    if (threadIdx.x == 0) parts[(int64_t)b * parts_per_img + blockIdx.x] = t;
  }
}

static unsigned chunks_for(int64_t total) {
  int64_t c = (total + 256 * 8 - 1) / (256 * 8);  // ~8 elements per thread
  if (c < 1) c = 1;
  if (c > 1024) c = 1024;
  return (unsigned)c;
}

}  // namespace lic

using namespace lic;

template <typename T>
static bool vec_ok(const void* p, int ld, int c) {
  constexpr int V = 16 / (int)sizeof(T);
  return ((uintptr_t)p % 16) == 0 && ld % V == 0 && c % V == 0 && c / V <= 256;
}

static bool fits32(int64_t n, int64_t hw, int64_t ld) { return n * hw * ld < (1LL << 31); }

extern "C" int lic_pool_partials(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t c,
                                 int32_t nchunk, float* parts, lic_stream_t stream) {
  if (n == 0 || hw == 0) return 0;
  if (c > 256 || nchunk < 1 || !fits32(n, hw, ldx)) return fail("pool_partials: needs c <= 256, n*hw*ld < 2^31");
  dim3 grid(nchunk, n);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LIC_F32) {
    if (vec_ok<float>(x, ldx, c))
      hipLaunchKernelGGL((pool_partials_kernel<float, true>), grid, dim3(256), 0, s, (const float*)x, ldx, hw, c,
                         nchunk, parts);
    else
      hipLaunchKernelGGL((pool_partials_kernel<float, false>), grid, dim3(256), 0, s, (const float*)x, ldx, hw, c,
                         nchunk, parts);
  } else if (dtype == LIC_F16) {
    if (vec_ok<half_t>(x, ldx, c))
      hipLaunchKernelGGL((pool_partials_kernel<half_t, true>), grid, dim3(256), 0, s, (const half_t*)x, ldx, hw, c,
                         nchunk, parts);
    else
      hipLaunchKernelGGL((pool_partials_kernel<half_t, false>), grid, dim3(256), 0, s, (const half_t*)x, ldx, hw, c,
                         nchunk, parts);
  } else if (dtype == LIC_BF16) {
    if (vec_ok<bf16_t>(x, ldx, c))
      hipLaunchKernelGGL((pool_partials_kernel<bf16_t, true>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, hw, c,
                         nchunk, parts);
    else
      hipLaunchKernelGGL((pool_partials_kernel<bf16_t, false>), grid, dim3(256), 0, s, (const bf16_t*)x, ldx, hw, c,
                         nchunk, parts);
  } else {
    return fail("pool_partials: bad dtype");
  }
  LIC_CHECK_LAUNCH();
  return 0;
}

template <typename T>
static void ca_launch(bool vec, dim3 grid, hipStream_t s, const void* r, int ldr, const void* x, int ldx, int hw,
                      int c, const float* y, void* out, int ldo) {
  if (vec)
    hipLaunchKernelGGL((ca_apply_kernel<T, true>), grid, dim3(256), 0, s, (const T*)r, ldr, (const T*)x, ldx, hw, c, y,
                       (T*)out, ldo);
  else
    hipLaunchKernelGGL((ca_apply_kernel<T, false>), grid, dim3(256), 0, s, (const T*)r, ldr, (const T*)x, ldx, hw, c,
                       y, (T*)out, ldo);
}

extern "C" int lic_ca_apply_fwd(int32_t dtype, const void* r, int32_t ldr, const void* x, int32_t ldx, int32_t n,
                                int32_t hw, int32_t c, float* parts, int32_t nchunk, const float* w1,
                                const float* b1, const float* w2, const float* b2, int32_t cr, void* out,
                                int32_t ldo, lic_stream_t stream) {
  if (n == 0 || hw == 0) return 0;
  if (c > 256 || cr > 32 || cr < 1) return fail("ca_apply: needs c <= 256 and 1 <= c/reduction <= 32");
  if (!fits32(n, hw, ldr) || !fits32(n, hw, ldx) || !fits32(n, hw, ldo)) return fail("ca_apply: map too large");
  hipStream_t s = (hipStream_t)stream;
  float* y = parts + (int64_t)n * nchunk * c;  // the caller's buffer holds n*(nchunk+1)*c floats
  hipLaunchKernelGGL(ca_weights_kernel, dim3(n), dim3(256), 0, s, parts, nchunk, hw, c, w1, b1, w2, b2, cr, y);
  dim3 grid((unsigned)std::min<int64_t>(256, std::max<int64_t>(1, (int64_t)hw / 256)), n);
  if (dtype == LIC_F32) {
    const bool v = vec_ok<float>(r, ldr, c) && vec_ok<float>(x, ldx, c) && vec_ok<float>(out, ldo, c);
    ca_launch<float>(v, grid, s, r, ldr, x, ldx, hw, c, y, out, ldo);
  } else if (dtype == LIC_F16) {
    const bool v = vec_ok<half_t>(r, ldr, c) && vec_ok<half_t>(x, ldx, c) && vec_ok<half_t>(out, ldo, c);
    ca_launch<half_t>(v, grid, s, r, ldr, x, ldx, hw, c, y, out, ldo);
  } else if (dtype == LIC_BF16) {
    const bool v = vec_ok<bf16_t>(r, ldr, c) && vec_ok<bf16_t>(x, ldx, c) && vec_ok<bf16_t>(out, ldo, c);
    ca_launch<bf16_t>(v, grid, s, r, ldr, x, ldx, hw, c, y, out, ldo);
  } else {
    return fail("ca_apply: bad dtype");
  }
  LIC_CHECK_LAUNCH();
  return 0;
}

template <typename T, int N, bool VEC>
static void lam_launch_t(const void* x, int ldx, int n, int hw, int C, double* parts, int nblk, const float* gamma,
                         void* out, int ldo, hipStream_t s) {
  float* A = (float*)(parts + (int64_t)n * nblk * (N * (N + 1) / 2));  // after the partials
  dim3 g1(nblk, n), g2((unsigned)std::min<int64_t>(256, std::max<int64_t>(1, (int64_t)hw / 256)), n);
  hipLaunchKernelGGL((lam_gram_kernel<T, N, VEC>), g1, dim3(256), 0, s, (const T*)x, ldx, hw, C, parts);
  hipLaunchKernelGGL((lam_attn_kernel<N>), dim3(n), dim3(256), 0, s, parts, nblk, A);
  hipLaunchKernelGGL((lam_apply_kernel<T, N, VEC>), g2, dim3(256), 0, s, (const T*)x, ldx, hw, C, A, gamma, (T*)out,
                     ldo);
}

template <int N>
static int lam_launch(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t C, double* parts,
                      int32_t nblk, const float* gamma, void* out, int32_t ldo, hipStream_t s) {
  if (dtype == LIC_F32) {
    if (vec_ok<float>(x, ldx, C) && vec_ok<float>(out, ldo, C))
      lam_launch_t<float, N, true>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
    else
      lam_launch_t<float, N, false>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
  } else if (dtype == LIC_F16) {
    if (vec_ok<half_t>(x, ldx, C) && vec_ok<half_t>(out, ldo, C))
      lam_launch_t<half_t, N, true>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
    else
      lam_launch_t<half_t, N, false>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
  } else if (dtype == LIC_BF16) {
    if (vec_ok<bf16_t>(x, ldx, C) && vec_ok<bf16_t>(out, ldo, C))
      lam_launch_t<bf16_t, N, true>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
    else
      lam_launch_t<bf16_t, N, false>(x, ldx, n, hw, C, parts, nblk, gamma, out, ldo, s);
  } else {
    return fail("lam: bad dtype");
  }
  LIC_CHECK_LAUNCH();
  return 0;
}

// per image: 256 blocks x NP fp64 Gram partials + N*N fp32 attention (in double slots)
extern "C" int32_t lic_lam_parts(int32_t ngroups) { return 256 * ngroups * (ngroups + 1) / 2 + ngroups * ngroups; }

extern "C" int lic_lam_fwd(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t ngroups,
                           int32_t c, double* parts, const float* gamma, void* out, int32_t ldo,
                           lic_stream_t stream) {
  if (n == 0 || hw == 0) return 0;
  if (out == x) return fail("lam: out must not alias x");
  if (c > 256 || !fits32(n, hw, ldx) || !fits32(n, hw, ldo)) return fail("lam: needs c <= 256, n*hw*ld < 2^31");
  const int nblk = 256;  // parts must hold n * lic_lam_parts(ngroups) doubles
  hipStream_t s = (hipStream_t)stream;
  switch (ngroups) {
    case 5: return lam_launch<5>(dtype, x, ldx, n, hw, c, parts, nblk, gamma, out, ldo, s);
    case 7: return lam_launch<7>(dtype, x, ldx, n, hw, c, parts, nblk, gamma, out, ldo, s);
    case 2: return lam_launch<2>(dtype, x, ldx, n, hw, c, parts, nblk, gamma, out, ldo, s);
    default: return fail("lam: ngroups must be 5 (HAN), 7 (HAN is_high) or 2");
  }
}

extern "C" int lic_csam_fwd(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t h, int32_t w, int32_t c,
                            const float* params, void* out, int32_t ldo, lic_stream_t stream) {
  const int64_t total = (int64_t)n * h * w * c;
  if (total == 0) return 0;
  if (out == x) return fail("csam: out must not alias x");
  if (!fits32(n, (int64_t)h * w, ldx) || !fits32(n, (int64_t)h * w, ldo) || !fits32(n, (int64_t)h * w, c))
    return fail("csam: map too large for 32-bit indexing");
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(csam_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, ldx, n, h, w, c, params,
                       (float*)out, ldo);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(csam_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)x, ldx, n, h, w, c, params,
                       (half_t*)out, ldo);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(csam_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)x, ldx, n, h, w, c, params,
                       (bf16_t*)out, ldo);
  else
    return fail("csam: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_recon_fwd(int32_t dtype, const void* xtil, int32_t n, int32_t h, int32_t w, int32_t cin,
                             int32_t ldx, const void* wgen, int32_t ldw, int32_t mode, const float* post,
                             const float* x, float* x_rec, double* sqerr_partials, int32_t parts_per_img, void* y,
                             int32_t ldy, int32_t ycpad, lic_stream_t stream) {
  if (cin > 64) return fail("recon: cin > 64");
  if (mode != 0 && mode != 1) return fail("recon: mode must be 0 (linear) or 1 (tanh)");
  if (y && (ycpad < 3 || ldy < ycpad)) return fail("recon: y needs >= 3 channels");
  if (x && !x_rec) return fail("recon: metrics need x_rec");
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(parts_per_img, n);
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(recon_kernel<float>, grid, dim3(256), 0, s, (const float*)xtil, h, w, cin, ldx, ldw,
                       (const float*)wgen, mode, post, x, x_rec, sqerr_partials, parts_per_img, (float*)y, ldy, ycpad);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(recon_kernel<half_t>, grid, dim3(256), 0, s, (const half_t*)xtil, h, w, cin, ldx, ldw,
                       (const half_t*)wgen, mode, post, x, x_rec, sqerr_partials, parts_per_img, (half_t*)y, ldy,
                       ycpad);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(recon_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)xtil, h, w, cin, ldx, ldw,
                       (const bf16_t*)wgen, mode, post, x, x_rec, sqerr_partials, parts_per_img, (bf16_t*)y, ldy,
                       ycpad);
  else
    return fail("recon: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}
