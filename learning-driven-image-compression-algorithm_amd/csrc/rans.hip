// Entropy coder: CDF tables and the Rans64 coder of
// compressai 1.2.x, restated for gfx950 (see include/lic.h).
//
// Layout: a latent [n, hw, ctot] (NHWC channel windows) is coded as n*ctot
// independent streams, one per (image, channel), symbols in raster order; each
// stream is exactly the compressai string of its symbol list, so one thread owns
// one stream (encode and decode are serial inside a stream; the parallelism is
// the stream count).  The coder is integer work on tiny data: it is bound by the
// dependent latency of each thread's symbol chain, not by HBM or the matrix cores.
//   encode: reverse pass over the symbols, words written backwards into a
//           per-stream scratch row, then one scan + copy launch packs the rows.
//   decode: each workgroup stages every CDF table into LDS (the Gaussian set of 64
//           tables is ~108 KB) and binary-searches it per symbol (compressai's
//           linear find_if returns the same index on a nondecreasing cdf).
#include "lic_common.h"

namespace lic {

constexpr int kPrec = 16;
constexpr uint32_t kBypassPrec = 4;
constexpr uint32_t kMaxBypass = (1u << kBypassPrec) - 1;
constexpr uint64_t kRansL = 1ull << 31;

// ---------------------------------------------------------------- tables
__device__ __forceinline__ float std_cumulative(float v) {
  // compressai _standardized_cumulative: 0.5 * erfc(-(2^-0.5) * v)
  return 0.5f * erfcf(-0.70710678118654752440f * v);
}

__global__ void gauss_pmf_kernel(const float* __restrict__ table, const int32_t* __restrict__ center, int ntab,
                                 int stride, float* __restrict__ pmf) {
  const int t = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntab) return;
  const int c = center[t];
  const int len = 2 * c + 1;
  if (k > len) return;
  const float s = table[t];
  float* row = pmf + (size_t)t * stride;
  if (k == len) {  // tail mass = 2 * lower[:, :1] (sample |0 - c| = c)
    row[k] = 2.0f * std_cumulative(__fdiv_rn(__fsub_rn(-0.5f, (float)c), s));
    return;
  }
  const float smp = (float)abs(k - c);
  const float upper = std_cumulative(__fdiv_rn(__fsub_rn(0.5f, smp), s));
  const float lower = std_cumulative(__fdiv_rn(__fsub_rn(-0.5f, smp), s));
  row[k] = __fsub_rn(upper, lower);
}

__device__ __forceinline__ float softplus_f(float v) { return v > 20.f ? v : log1pf(expf(v)); }

// EntropyBottleneck._logits_cumulative for filters (3,3,3,3) at one channel
__device__ float eb_logits(const float* p, float x) {
  const float* m0 = p;        // [3][1]
  const float* m1 = p + 3;    // [3][3]
  const float* m2 = p + 12;
  const float* m3 = p + 21;
  const float* m4 = p + 30;   // [1][3]
  const float* b = p + 33;    // b0[3] b1[3] b2[3] b3[3] b4[1]
  const float* f = p + 46;    // f0..f3 [3]
  float l[3], t[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    float v = __fmul_rn(softplus_f(m0[o]), x) + b[o];
    l[o] = v + tanhf(f[o]) * tanhf(v);
  }
  const float* ms[3] = {m1, m2, m3};
#pragma unroll
  for (int layer = 0; layer < 3; ++layer) {
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) v += softplus_f(ms[layer][o * 3 + i]) * l[i];
      v += b[3 * (layer + 1) + o];
      t[o] = v + tanhf(f[3 * (layer + 1) + o]) * tanhf(v);
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) l[o] = t[o];
  }
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) v += softplus_f(m4[i]) * l[i];
  return v + b[12];
}

__device__ __forceinline__ float sigmoid_exact(float v) { return 1.0f / (1.0f + expf(-v)); }

__global__ void eb_pmf_kernel(const float* __restrict__ params, const float* __restrict__ start,
                              const int32_t* __restrict__ length, int c, int stride, float* __restrict__ pmf) {
  const int ch = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const int len = length[ch];
  if (k > len) return;
  const float* p = params + (size_t)ch * LIC_EB_PARAMS;
  float* row = pmf + (size_t)ch * stride;
  if (k == len) {
    // tail = sigmoid(lower[:, 0, :1]) + sigmoid(-upper[:, 0, -1:]): compressai evaluates the
    // upper tail at the LAST column of the padded sample grid, k = max_length - 1 = stride - 2
    // for every channel (not at this channel's own pmf_length - 1)
    const float lo0 = eb_logits(p, __fsub_rn(start[ch] + 0.f, 0.5f));
    const float up1 = eb_logits(p, __fadd_rn(__fadd_rn((float)(stride - 2), start[ch]), 0.5f));
    row[k] = sigmoid_exact(lo0) + sigmoid_exact(-up1);
    return;
  }
  const float smp = __fadd_rn((float)k, start[ch]);
  const float lower = eb_logits(p, __fsub_rn(smp, 0.5f));
  const float upper = eb_logits(p, __fadd_rn(smp, 0.5f));
  const float sum = lower + upper;
  const float sign = sum > 0.f ? -1.f : (sum < 0.f ? 1.f : 0.f);
  row[k] = fabsf(sigmoid_exact(sign * upper) - sigmoid_exact(sign * lower));
}

constexpr int kCdfMax = 8192;  // entries per table handled by pmf_to_cdf_kernel

// compressai pmf_to_quantized_cdf, one workgroup (256 threads) per table, cdf in LDS
__global__ __launch_bounds__(256) void pmf_to_cdf_kernel(const float* __restrict__ pmf, const int32_t* __restrict__ nsym,
                                                         int stride, int precision, int32_t* __restrict__ cdf_out,
                                                         int cdf_stride, int32_t* __restrict__ status) {
  __shared__ uint32_t cdf[kCdfMax + 1];
  __shared__ uint64_t red[4];
  __shared__ uint32_t part[256];
  __shared__ int fail_flag;
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = nsym[t];
  const float* p = pmf + (size_t)t * stride;
  if (n + 1 > kCdfMax || n + 1 > cdf_stride || n < 1) {
    if (tid == 0) status[t] = 2;
    return;
  }
  const uint32_t one = 1u << precision;
  if (tid == 0) {
    cdf[0] = 0;
    fail_flag = 0;
  }
  for (int i = tid; i < n; i += 256) cdf[i + 1] = (uint32_t)roundf(p[i] * (float)one);
  __syncthreads();
  // total (fits 32 bits: n <= 8192 entries of <= 2^precision)
  uint64_t s = 0;
  for (int i = tid; i <= n; i += 256) s += cdf[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const uint32_t total = (uint32_t)(red[0] + red[1] + red[2] + red[3]);
  if (total == 0) {
    if (tid == 0) status[t] = 1;
    return;
  }
  for (int i = tid; i <= n; i += 256) cdf[i] = (uint32_t)(((uint64_t)one * cdf[i]) / total);
  __syncthreads();
  // inclusive prefix sum over n+1 entries: per-thread contiguous chunks
  const int per = (n + 1 + 255) / 256;
  const int lo = tid * per, hi = min(n + 1, lo + per);
  uint32_t acc = 0;
  for (int i = lo; i < hi; ++i) acc += cdf[i];
  part[tid] = acc;
  __syncthreads();
  if (tid == 0) {
    uint32_t run = 0;
    for (int k = 0; k < 256; ++k) {
      const uint32_t v = part[k];
      part[k] = run;
      run += v;
    }
  }
  __syncthreads();
  acc = part[tid];
  for (int i = lo; i < hi; ++i) {
    acc += cdf[i];
    cdf[i] = acc;
  }
  __syncthreads();
  if (tid == 0) cdf[n] = one;
  __syncthreads();
  // zero-frequency repair, in order (each step sees the previous steps' result)
  for (int i = 0; i < n; ++i) {
    if (cdf[i] != cdf[i + 1]) continue;  // uniform: every thread reads the same LDS words
    uint64_t best = ~0ull;
    for (int j = tid; j < n; j += 256) {
      const uint32_t f = cdf[j + 1] - cdf[j];
      if (f > 1) {
        const uint64_t key = ((uint64_t)f << 32) | (uint32_t)j;  // smallest freq, then smallest j
        best = key < best ? key : best;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t other = __shfl_xor(best, o);
      best = other < best ? other : best;
    }
    __syncthreads();
    if (lane == 0) red[wave] = best;
    __syncthreads();
    uint64_t b = red[0];
    for (int w = 1; w < 4; ++w) b = red[w] < b ? red[w] : b;
    if (b == ~0ull) {
      if (tid == 0) fail_flag = 1;
      break;
    }
    const int steal = (int)(uint32_t)b;
    if (steal < i) {
      for (int j = steal + 1 + tid; j <= i; j += 256) cdf[j] -= 1;
    } else {
      for (int j = i + 1 + tid; j <= steal; j += 256) cdf[j] += 1;
    }
    __syncthreads();
  }
  __syncthreads();
  int32_t* out = cdf_out + (size_t)t * cdf_stride;
  for (int i = tid; i <= n; i += 256) out[i] = (int32_t)cdf[i];
  if (tid == 0) status[t] = fail_flag;
}

template <typename T>
__global__ void gauss_indexes_kernel(const T* __restrict__ sc, int npix, int c, int ldsc,
                                     const float* __restrict__ table, int ntab, float bound, int32_t* __restrict__ idx,
                                     int ldidx) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)npix * c) return;
  const int64_t p = e / c;
  const int k = (int)(e - p * c);
  const float s = fmaxf(to_f(sc[p * ldsc + k]), bound);
  int v = ntab - 1;
  for (int t = 0; t < ntab - 1; ++t) v -= (s <= table[t]) ? 1 : 0;
  idx[p * ldidx + k] = v;
}

template <typename T>
__global__ void quantize_symbols_kernel(const T* __restrict__ z, int npix, int c, int ldz, const float* __restrict__ m,
                                        int32_t* __restrict__ sym, int ldsym) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)npix * c) return;
  const int64_t p = e / c;
  const int k = (int)(e - p * c);
  const float med = m ? m[k] : 0.f;
  sym[p * ldsym + k] = (int32_t)rintf(__fsub_rn(to_f(z[p * ldz + k]), med));
}

// ---------------------------------------------------------------- Rans64
__device__ __forceinline__ bool enc_put(uint64_t& x, uint32_t* row, int& ptr, uint32_t start, uint32_t freq) {
  const uint64_t x_max = ((kRansL >> kPrec) << 32) * freq;
  if (x >= x_max) {
    if (ptr <= 2) return false;
    row[--ptr] = (uint32_t)x;
    x >>= 32;
  }
  x = ((x / freq) << kPrec) + (x % freq) + start;
  return true;
}

__device__ __forceinline__ bool enc_put_bits(uint64_t& x, uint32_t* row, int& ptr, uint32_t val) {
  const uint32_t freq = 1u << (16 - kBypassPrec);
  const uint64_t x_max = ((kRansL >> 16) << 32) * freq;
  if (x >= x_max) {
    if (ptr <= 2) return false;
    row[--ptr] = (uint32_t)x;
    x >>= 32;
  }
  x = (x << kBypassPrec) | val;
  return true;
}

__global__ __launch_bounds__(64) void rans_encode_kernel(const lic_rans_args a) {
  const int sid = blockIdx.x * 64 + threadIdx.x;
  if (sid >= a.n * a.c) return;
  const int b = sid / a.c, ch = sid - b * a.c;
  const int gs = b * a.ctot + a.c0 + ch;
  uint32_t* row = a.scratch + (size_t)gs * a.cap;
  int ptr = a.cap;
  uint64_t x = kRansL;
  bool ok = true;
  // symbols are pushed forward (main symbol, bypass count chunks, raw chunks) and
  // encoded from the last push backwards
  for (int p = a.hw - 1; p >= 0 && ok; --p) {
    const int64_t r = (int64_t)b * a.hw + p;
    const int32_t ci = a.indexes ? a.indexes[r * a.ldidx + ch] : a.c0 + ch;
    if (ci < 0 || ci >= a.ncdf) {
      ok = false;
      break;
    }
    const int32_t* cdf = a.cdfs + (size_t)ci * a.cdf_stride;
    const int32_t max_value = a.cdf_sizes[ci] - 2;
    int32_t value = a.symbols[r * a.ldsym + ch] - a.offsets[ci];
    uint32_t raw = 0;
    if (value < 0) {
      raw = (uint32_t)(-2 * value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw = (uint32_t)(2 * (value - max_value));
      value = max_value;
    }
    if (value == max_value) {
      int nb = 0;
      while (nb < 8 && (raw >> (nb * kBypassPrec)) != 0) ++nb;
      for (int j = nb - 1; j >= 0 && ok; --j) ok = enc_put_bits(x, row, ptr, (raw >> (j * kBypassPrec)) & kMaxBypass);
      // count chunks were pushed as (kMaxBypass x q, rem): encode rem first
      const int q = nb / (int)kMaxBypass, rem = nb - q * (int)kMaxBypass;
      if (ok) ok = enc_put_bits(x, row, ptr, (uint32_t)rem);
      for (int j = 0; j < q && ok; ++j) ok = enc_put_bits(x, row, ptr, kMaxBypass);
    }
    if (ok) ok = enc_put(x, row, ptr, (uint32_t)cdf[value], (uint32_t)(cdf[value + 1] - cdf[value]));
  }
  if (!ok || ptr < 2) {
    a.lengths[gs] = -1;
    return;
  }
  row[--ptr] = (uint32_t)(x >> 32);
  row[--ptr] = (uint32_t)x;
  a.lengths[gs] = a.cap - ptr;
}

__global__ __launch_bounds__(1024) void rans_scan_kernel(const int32_t* __restrict__ len, int n,
                                                         uint32_t* __restrict__ off) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const uint32_t v = i < n ? (uint32_t)len[i] : 0u;
    uint32_t incl = v;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = carry_s;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    if (i < n) off[i] = before + incl - v;
    __syncthreads();
    if (tid == 1023) carry_s = before + incl;
    __syncthreads();
  }
  if (tid == 0) off[n] = carry_s;
}

__global__ __launch_bounds__(256) void rans_copy_kernel(const uint32_t* __restrict__ scratch, int cap,
                                                        const int32_t* __restrict__ len,
                                                        const uint32_t* __restrict__ off, uint32_t* __restrict__ out) {
  const int s = blockIdx.x;
  const int l = len[s];
  const uint32_t* src = scratch + (size_t)s * cap + (cap - l);
  uint32_t* dst = out + off[s];
  for (int k = threadIdx.x; k < l; k += 256) dst[k] = src[k];
}

constexpr int kDecLdsWords = 36 * 1024;  // <= 144 KB of CDF entries staged per workgroup
constexpr int kDecMaxStagedTables = 256;

// lds_words = dynamic LDS words of the launch (0: no staging).  The workgroup packs
// every table into LDS (table t at base[t]) when their total fits, else it reads the
// tables from global memory (uniform per workgroup).
template <typename T>
__global__ __launch_bounds__(64) void rans_decode_kernel(const lic_rans_args a, int lds_words) {
  extern __shared__ int32_t lds_cdf[];
  __shared__ int32_t base[kDecMaxStagedTables];
  __shared__ int stage_s;
  const int tid = threadIdx.x;
  if (tid == 0) {
    int tot = 0;
    const bool can = lds_words > 0 && a.ncdf <= kDecMaxStagedTables;
    for (int t = 0; can && t < a.ncdf; ++t) {
      base[t] = tot;
      tot += a.cdf_sizes[t];
    }
    stage_s = can && tot <= lds_words;
  }
  __syncthreads();
  const int stage = stage_s;
  if (stage) {
    for (int t = 0; t < a.ncdf; ++t) {
      const int sz = a.cdf_sizes[t];
      const int32_t* src = a.cdfs + (size_t)t * a.cdf_stride;
      for (int k = tid; k < sz; k += 64) lds_cdf[base[t] + k] = src[k];
    }
    __syncthreads();
  }
  const int sid = blockIdx.x * 64 + tid;
  if (sid >= a.n * a.c) return;
  const int b = sid / a.c, ch = sid - b * a.c;
  const int gs = b * a.ctot + a.c0 + ch;
  const uint32_t* ptr = a.words + a.offsets_w[gs];
  const uint32_t* end = a.words + a.offsets_w[gs + 1];
  bool ok = end - ptr >= 2;
  uint64_t x = 0;
  if (ok) {
    x = (uint64_t)ptr[0] | ((uint64_t)ptr[1] << 32);
    ptr += 2;
  }
  const float mch = a.mu_ch ? a.mu_ch[a.c0 + ch] : 0.f;
  for (int p = 0; p < a.hw; ++p) {
    const int64_t r = (int64_t)b * a.hw + p;
    int32_t out = 0;
    if (ok) {
      const int32_t ci = a.indexes ? a.indexes[r * a.ldidx + ch] : a.c0 + ch;
      if (ci < 0 || ci >= a.ncdf) {
        ok = false;
      } else {
        const int32_t* cdf = stage ? lds_cdf + base[ci] : a.cdfs + (size_t)ci * a.cdf_stride;
        const int32_t size = a.cdf_sizes[ci];
        const int32_t max_value = size - 2;
        const uint32_t cum = (uint32_t)(x & ((1u << kPrec) - 1));
        int lo = 0, hi = size;  // first entry > cum
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((uint32_t)cdf[mid] > cum) hi = mid;
          else lo = mid + 1;
        }
        int32_t s = lo - 1;
        if (s < 0 || s >= size - 1) {
          ok = false;
        } else {
          const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
          x = freq * (x >> kPrec) + (x & ((1u << kPrec) - 1)) - start;
          if (x < kRansL) {
            if (ptr >= end) ok = false;
            else x = (x << 32) | *ptr++;
          }
          int32_t value = s;
          if (ok && value == max_value) {
            auto get_bits = [&]() -> int32_t {
              const int32_t v = (int32_t)(x & kMaxBypass);
              x >>= kBypassPrec;
              if (x < kRansL) {
                if (ptr >= end) ok = false;
                else x = (x << 32) | *ptr++;
              }
              return v;
            };
            int32_t val = get_bits();
            int32_t nb = val;
            while (ok && val == (int32_t)kMaxBypass && nb <= 8) {
              val = get_bits();
              nb += val;
            }
            if (nb > 8) ok = false;
            int32_t raw = 0;
            for (int j = 0; j < nb && ok; ++j) raw |= get_bits() << (j * kBypassPrec);
            value = raw >> 1;
            value = (raw & 1) ? -value - 1 : value + max_value;
          }
          out = value + a.offsets[ci];
        }
      }
    }
    if (a.out_symbols) a.out_symbols[r * a.ldosym + ch] = out;
    if (a.yq) {
      const float mean = a.mu ? to_f(((const T*)a.mu)[r * a.ldmu + ch]) : mch;
      ((T*)a.yq)[r * a.ldyq + ch] = from_f<T>(__fadd_rn((float)out, mean));
    }
  }
  if (a.status) a.status[sid] = ok ? 0 : 1;
}

}  // namespace lic

using namespace lic;

extern "C" int lic_gauss_pmf(const float* scale_table, const int32_t* pmf_center, int32_t ntab, int32_t pmf_stride,
                             float* pmf, lic_stream_t stream) {
  if (ntab <= 0) return 0;
  // the longest row needs 2*c+2 entries; the launch covers pmf_stride entries per row
  dim3 grid((pmf_stride + 255) / 256, ntab);
  hipLaunchKernelGGL(gauss_pmf_kernel, grid, dim3(256), 0, (hipStream_t)stream, scale_table, pmf_center, ntab,
                     pmf_stride, pmf);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_eb_pmf(const float* params, const float* pmf_start, const int32_t* pmf_length, int32_t c,
                          int32_t pmf_stride, float* pmf, lic_stream_t stream) {
  if (c <= 0) return 0;
  dim3 grid((pmf_stride + 63) / 64, c);
  hipLaunchKernelGGL(eb_pmf_kernel, grid, dim3(64), 0, (hipStream_t)stream, params, pmf_start, pmf_length, c,
                     pmf_stride, pmf);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_pmf_to_cdf(const float* pmf, const int32_t* nsym, int32_t ntab, int32_t pmf_stride,
                              int32_t precision, int32_t* cdf, int32_t cdf_stride, int32_t* status,
                              lic_stream_t stream) {
  if (ntab <= 0) return 0;
  if (precision < 1 || precision > 16) return fail("pmf_to_cdf: precision must be in [1, 16]");
  hipLaunchKernelGGL(pmf_to_cdf_kernel, dim3(ntab), dim3(256), 0, (hipStream_t)stream, pmf, nsym, pmf_stride,
                     precision, cdf, cdf_stride, status);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_gauss_indexes(int32_t dtype, const void* scales, int32_t npix, int32_t c, int32_t ldsc,
                                 const float* scale_table, int32_t ntab, float bound, int32_t* idx, int32_t ldidx,
                                 lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (total == 0) return 0;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(gauss_indexes_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)scales, npix, c, ldsc,
                       scale_table, ntab, bound, idx, ldidx);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(gauss_indexes_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)scales, npix, c,
                       ldsc, scale_table, ntab, bound, idx, ldidx);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(gauss_indexes_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)scales, npix, c,
                       ldsc, scale_table, ntab, bound, idx, ldidx);
  else
    return fail("gauss_indexes: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_quantize_symbols(int32_t dtype, const void* z, int32_t npix, int32_t c, int32_t ldz,
                                    const float* medians, int32_t* sym, int32_t ldsym, lic_stream_t stream) {
  const int64_t total = (int64_t)npix * c;
  if (total == 0) return 0;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == LIC_F32)
    hipLaunchKernelGGL(quantize_symbols_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)z, npix, c, ldz,
                       medians, sym, ldsym);
  else if (dtype == LIC_F16)
    hipLaunchKernelGGL(quantize_symbols_kernel<half_t>, dim3(blocks), dim3(256), 0, s, (const half_t*)z, npix, c, ldz,
                       medians, sym, ldsym);
  else if (dtype == LIC_BF16)
    hipLaunchKernelGGL(quantize_symbols_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)z, npix, c, ldz,
                       medians, sym, ldsym);
  else
    return fail("quantize_symbols: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int32_t lic_rans_cap(int32_t hw) {
  // <= 16 bits per main symbol + 4 bits per bypass chunk (<= 1 count + 8 raw chunks
  // for 32-bit raw values) per symbol; +2 flush words, +2 slack
  return (int32_t)(((int64_t)hw * 52 + 31) / 32 + 4);
}

extern "C" int lic_rans_encode(const lic_rans_args* a, lic_stream_t stream) {
  if (!a) return fail("rans_encode: null args");
  const int64_t ns = (int64_t)a->n * a->c;
  if (ns == 0) return 0;
  if (!a->symbols || !a->cdfs || !a->cdf_sizes || !a->offsets || !a->scratch || !a->lengths)
    return fail("rans_encode: null argument");
  if (a->c0 < 0 || a->c0 + a->c > a->ctot) return fail("rans_encode: channel window outside ctot");
  if (a->cap < lic_rans_cap(a->hw)) return fail("rans_encode: scratch row smaller than lic_rans_cap(hw)");
  hipLaunchKernelGGL(rans_encode_kernel, dim3((unsigned)((ns + 63) / 64)), dim3(64), 0, (hipStream_t)stream, *a);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_rans_pack(const uint32_t* scratch, int32_t cap, const int32_t* lengths, int32_t nstreams,
                             uint32_t* offsets_w, uint32_t* out, lic_stream_t stream) {
  if (nstreams <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rans_scan_kernel, dim3(1), dim3(1024), 0, s, lengths, nstreams, offsets_w);
  LIC_CHECK_LAUNCH();
  hipLaunchKernelGGL(rans_copy_kernel, dim3(nstreams), dim3(256), 0, s, scratch, cap, lengths, offsets_w, out);
  LIC_CHECK_LAUNCH();
  return 0;
}

extern "C" int lic_rans_decode(const lic_rans_args* a, lic_stream_t stream) {
  if (!a) return fail("rans_decode: null args");
  const int64_t ns = (int64_t)a->n * a->c;
  if (ns == 0) return 0;
  if (!a->words || !a->offsets_w || !a->cdfs || !a->cdf_sizes || !a->offsets)
    return fail("rans_decode: null argument");
  if (a->c0 < 0 || a->c0 + a->c > a->ctot) return fail("rans_decode: channel window outside ctot");
  if (a->ncdf > 4096) return fail("rans_decode: too many tables");
  hipStream_t s = (hipStream_t)stream;
  const int64_t worst = (int64_t)a->ncdf * a->cdf_stride;
  const int lds_words = a->ncdf <= kDecMaxStagedTables ? (int)(worst < kDecLdsWords ? worst : kDecLdsWords) : 0;
  const size_t lds = (size_t)lds_words * sizeof(int32_t);
  const void* kern = a->dtype == LIC_F32   ? (const void*)rans_decode_kernel<float>
                     : a->dtype == LIC_BF16 ? (const void*)rans_decode_kernel<bf16_t>
                                            : (const void*)rans_decode_kernel<half_t>;
  const hipError_t ea = ensure_dyn_lds(kern, kDecLdsWords * 4);
  if (ea != hipSuccess) return fail(std::string("rans_decode: dynamic LDS attribute: ") + hipGetErrorString(ea));
  const dim3 grid((unsigned)((ns + 63) / 64));
  if (a->dtype == LIC_F32)
    hipLaunchKernelGGL(rans_decode_kernel<float>, grid, dim3(64), lds, s, *a, lds_words);
  else if (a->dtype == LIC_F16)
    hipLaunchKernelGGL(rans_decode_kernel<half_t>, grid, dim3(64), lds, s, *a, lds_words);
  else if (a->dtype == LIC_BF16)
    hipLaunchKernelGGL(rans_decode_kernel<bf16_t>, grid, dim3(64), lds, s, *a, lds_words);
  else
    return fail("rans_decode: bad dtype");
  LIC_CHECK_LAUNCH();
  return 0;
}
