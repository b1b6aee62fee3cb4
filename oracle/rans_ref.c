/* TEST INFRASTRUCTURE ONLY — CPU oracle for the entropy coder.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker.  The product path is csrc/rans.hip.
 *
 * The reference repository has no entropy coder: it only estimates the rate
 * (net_ga.py:1049 GaussianConditional likelihoods, :1104-1107 bpp).  Its entropy
 * models come from compressai (InterDigital; not vendored under /root/reference,
 * no lock file -> version unpinned, >= 1.1 implied by EntropyBottleneck._get_medians,
 * SURVEY.md 8(c)).  This file restates compressai 1.2.x's published coder:
 *   - pmf_to_quantized_cdf          cpp_exts/ops/ops.cpp
 *   - BufferedRansEncoder::encode_with_indexes / flush
 *                                   cpp_exts/rans/rans_interface.cpp (Rans64 of ryg_rans,
 *                                   precision 16, 4-bit bypass chunks for out-of-range values)
 *   - RansDecoder::decode_with_indexes
 *                                   cpp_exts/rans/rans_interface.cpp
 * Parity against compressai itself is UNPINNED (not importable here, no fixtures);
 * the GPU coder is checked bit-exact against this restatement and by round trips.
 *
 * Stream layout (lic bitstream): one independent compressai-style Rans64 string per
 * (image, channel) of a latent, symbols in raster (row-major) order.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define PRECISION 16
#define BYPASS_PRECISION 4
#define MAX_BYPASS_VAL ((1 << BYPASS_PRECISION) - 1)
#define RANS64_L (1ull << 31)

/* ops.cpp pmf_to_quantized_cdf: pmf (n floats, the last one the tail mass) -> cdf
 * (n + 1 entries) at `precision` bits; every symbol keeps a nonzero frequency by
 * stealing from the smallest frequency > 1.  Returns 0 or -1 (no symbol to steal from). */
int ref_pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf) {
  cdf[0] = 0;
  for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)roundf(pmf[i] * (float)(1 << precision));
  uint32_t total = 0;
  for (int i = 0; i <= n; ++i) total += cdf[i];
  if (total == 0) return -1;
  for (int i = 0; i <= n; ++i) cdf[i] = (uint32_t)(((uint64_t)(1u << precision) * cdf[i]) / total);
  for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
  cdf[n] = 1u << precision;
  for (int i = 0; i < n; ++i) {
    if (cdf[i] == cdf[i + 1]) {
      uint32_t best_freq = ~0u;
      int best_steal = -1;
      for (int j = 0; j < n; ++j) {
        uint32_t freq = cdf[j + 1] - cdf[j];
        if (freq > 1 && freq < best_freq) {
          best_freq = freq;
          best_steal = j;
        }
      }
      if (best_steal < 0) return -1;
      if (best_steal < i) {
        for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
      } else {
        for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
      }
    }
  }
  return 0;
}

/* ---- Rans64 (ryg_rans rans64.h as used by compressai) */
typedef struct {
  uint32_t start, range;
  int bypass;
} ref_sym;

static void enc_put(uint64_t* r, uint32_t** pptr, uint32_t start, uint32_t freq, uint32_t scale_bits) {
  uint64_t x = *r;
  uint64_t x_max = ((RANS64_L >> scale_bits) << 32) * freq;
  if (x >= x_max) {
    *pptr -= 1;
    **pptr = (uint32_t)x;
    x >>= 32;
  }
  *r = ((x / freq) << scale_bits) + (x % freq) + start;
}

static void enc_put_bits(uint64_t* r, uint32_t** pptr, uint32_t val, uint32_t nbits) {
  uint64_t x = *r;
  uint32_t freq = 1u << (16 - nbits);
  uint64_t x_max = ((RANS64_L >> 16) << 32) * freq;
  if (x >= x_max) {
    *pptr -= 1;
    **pptr = (uint32_t)x;
    x >>= 32;
  }
  *r = (x << nbits) | val;
}

/* rans_interface.cpp encode_with_indexes + flush for ONE string.
 * cdfs: [ncdf][cdf_stride] int32; cdf_sizes/offsets: [ncdf].
 * out: capacity `cap` 32-bit words; the string is written to the END of out and its
 * word count returned (-1 on overflow / bad index).  *first receives the word offset. */
int ref_rans_encode(const int32_t* symbols, const int32_t* indexes, int n, const int32_t* cdfs, int cdf_stride,
                    const int32_t* cdf_sizes, const int32_t* offsets, int ncdf, uint32_t* out, int cap, int* first) {
  ref_sym* syms = (ref_sym*)malloc(sizeof(ref_sym) * ((size_t)n * 12 + 1));
  size_t ns = 0;
  for (int i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    if (ci < 0 || ci >= ncdf) { free(syms); return -1; }
    const int32_t* cdf = cdfs + (size_t)ci * cdf_stride;
    const int32_t max_value = cdf_sizes[ci] - 2;
    int32_t value = symbols[i] - offsets[ci];
    uint32_t raw_val = 0;
    if (value < 0) {
      raw_val = (uint32_t)(-2 * value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw_val = (uint32_t)(2 * (value - max_value));
      value = max_value;
    }
    syms[ns++] = (ref_sym){(uint32_t)cdf[value], (uint32_t)(cdf[value + 1] - cdf[value]), 0};
    if (value == max_value) {
      int32_t n_bypass = 0;
      while (n_bypass < 8 && (raw_val >> (n_bypass * BYPASS_PRECISION)) != 0) ++n_bypass;
      int32_t val = n_bypass;
      while (val >= MAX_BYPASS_VAL) {
        syms[ns++] = (ref_sym){MAX_BYPASS_VAL, MAX_BYPASS_VAL + 1, 1};
        val -= MAX_BYPASS_VAL;
      }
      syms[ns++] = (ref_sym){(uint32_t)val, (uint32_t)val + 1, 1};
      for (int32_t j = 0; j < n_bypass; ++j) {
        const uint32_t v = (raw_val >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL;
        syms[ns++] = (ref_sym){v, v + 1, 1};
      }
    }
  }
  uint64_t rans = RANS64_L;
  uint32_t* ptr = out + cap;
  while (ns > 0) {
    const ref_sym s = syms[--ns];
    if (ptr - out < 4) { free(syms); return -1; }
    if (!s.bypass)
      enc_put(&rans, &ptr, s.start, s.range, PRECISION);
    else
      enc_put_bits(&rans, &ptr, s.start, BYPASS_PRECISION);
  }
  ptr -= 2;
  ptr[0] = (uint32_t)(rans >> 0);
  ptr[1] = (uint32_t)(rans >> 32);
  free(syms);
  *first = (int)(ptr - out);
  return (int)(out + cap - ptr);
}

static uint32_t dec_get_bits(uint64_t* r, const uint32_t** pptr, uint32_t n_bits) {
  uint64_t x = *r;
  uint32_t val = (uint32_t)(x & ((1u << n_bits) - 1));
  x >>= n_bits;
  if (x < RANS64_L) {
    x = (x << 32) | **pptr;
    *pptr += 1;
  }
  *r = x;
  return val;
}

/* rans_interface.cpp decode_with_indexes for ONE string of `nwords` words.
 * Returns 0, or -1 on a bad index / read past the string. */
int ref_rans_decode(const uint32_t* words, int nwords, const int32_t* indexes, int n, const int32_t* cdfs,
                    int cdf_stride, const int32_t* cdf_sizes, const int32_t* offsets, int ncdf, int32_t* out) {
  if (nwords < 2) return -1;
  const uint32_t* ptr = words;
  const uint32_t* end = words + nwords;
  uint64_t rans = (uint64_t)ptr[0] | ((uint64_t)ptr[1] << 32);
  ptr += 2;
  for (int i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    if (ci < 0 || ci >= ncdf) return -1;
    const int32_t* cdf = cdfs + (size_t)ci * cdf_stride;
    const int32_t size = cdf_sizes[ci];
    const int32_t max_value = size - 2;
    const uint32_t cum = (uint32_t)(rans & ((1u << PRECISION) - 1));
    int s = 0;
    while (s < size && (uint32_t)cdf[s] <= cum) ++s;  /* find_if(v > cum) */
    s -= 1;
    {
      const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
      uint64_t x = rans;
      x = freq * (x >> PRECISION) + (x & ((1u << PRECISION) - 1)) - start;
      if (x < RANS64_L) {
        if (ptr >= end) return -1;
        x = (x << 32) | *ptr++;
      }
      rans = x;
    }
    int32_t value = s;
    if (value == max_value) {
      if (ptr > end) return -1;
      int32_t val = (int32_t)dec_get_bits(&rans, &ptr, BYPASS_PRECISION);
      int32_t n_bypass = val;
      while (val == MAX_BYPASS_VAL) {
        val = (int32_t)dec_get_bits(&rans, &ptr, BYPASS_PRECISION);
        n_bypass += val;
      }
      int32_t raw_val = 0;
      for (int j = 0; j < n_bypass; ++j) {
        val = (int32_t)dec_get_bits(&rans, &ptr, BYPASS_PRECISION);
        raw_val |= val << (j * BYPASS_PRECISION);
      }
      if (ptr > end) return -1;
      value = raw_val >> 1;
      if (raw_val & 1)
        value = -value - 1;
      else
        value += max_value;
    }
    out[i] = value + offsets[ci];
  }
  return 0;
}
