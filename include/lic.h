/*
 * lic.h — C ABI of liblic.so, the MI355X (gfx950) kernels behind the
 * encode -> quantize -> decode hot path of the learned image codec
 * (reference: xiaobucc/learning-driven-image-compression-algorithm).
 *
 * The reference has no native plugin/FFI layer: its boundary is the PyTorch
 * nn.Module surface.  Every entry point below replaces the
 * L0 PyTorch op sequence of one reference layer, cited per function.  The
 * Python host modules in lic_amd/ (same class names and state_dict keys as the
 * reference) call these through ctypes (lic_amd/_ffi.py); INTEGRATION.md shows
 * the binding.
 *
 * Conventions
 *  - Activations are NHWC ("pixel-major", channels contiguous).  A view is
 *    (data, n, h, w, c, ld): `data` already points at the first channel of the
 *    view, `ld` is the element stride between consecutive pixels, so channel
 *    slices / concatenations (torch.cat, torch.split, chunk) are free.
 *  - dtype tag: LIC_F32 or LIC_F16 for activations and packed weights; biases,
 *    GDN/LayerNorm parameters, scales and metrics are always fp32.
 *  - All tensors are caller-owned device memory; the library never allocates,
 *    frees or retains.  Calls are asynchronous on the given stream and are safe
 *    under stream capture (hipGraph).  Errors: non-zero status +
 *    lic_last_error() (thread-local message).
 */
#ifndef LIC_H_
#define LIC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* lic_stream_t; /* hipStream_t */

enum lic_dtype { LIC_F32 = 0, LIC_F16 = 1, LIC_BF16 = 2 };
enum lic_act { LIC_ACT_NONE = 0, LIC_ACT_RELU = 1, LIC_ACT_LRELU = 2, LIC_ACT_GELU = 3, LIC_ACT_ROUND = 4 };
enum lic_prologue { LIC_PRO_NONE = 0, LIC_PRO_SQUARE = 1, LIC_PRO_ABS = 2 };
enum lic_epilogue {
  LIC_EPI_PLAIN = 0,     /* v = act(acc+bias) (+ r1)                                  */
  LIC_EPI_GATE = 1,      /* v = g * sigmoid(act(acc+bias) (+ r1)) + r2   (WNSA / SWAtten) */
  LIC_EPI_HALF_TANH = 2, /* v = r2 + 0.5*tanh(act(acc+bias))             (LRP)           */
  LIC_EPI_GDN_DIV = 3,   /* v = g / sqrt(acc+beta) (+ r1)      model/gdn.py GDN          */
  LIC_EPI_GDN_RSQRT = 4, /* v = g * rsqrt(acc+beta) (+ r1)     layers/gdn.py GDN          */
  LIC_EPI_GDN_SQRT = 5,  /* v = g * sqrt(acc+beta) (+ r1)      IGDN (both variants)       */
  LIC_EPI_RES_ACT = 6    /* v = act(acc+bias+r1)               compressai ResidualUnit    */
};

#define LIC_MAX_TAPS 64

/* One convolution launch in "tap" form.
 *   out[b, oy0 + osy*i, ox0 + osx*j, n]  for i < mi, j < mj, n < co
 *     = epilogue( bias[n] + sum_t sum_c pro(x[b, i*isy + dy[t], j*isx + dx[t], c]) * w[n][t][c] )
 * with x zero outside [0,h)x[0,w).  A standard conv (stride s, pads pt/pl) is
 * isy=isx=s, dy=ky-pt, dx=kx-pl; a transposed conv is up to s*s such launches,
 * one per output phase (sub-pixel decomposition).  w is packed
 * [copad][ntaps][cpad] in `dtype`, zero-padded (copad >= co, cpad >= ci/groups).
 * out_shuffle=2 writes channel n of pixel (y,x) to channel n/4 of pixel
 * (2y + (n>>1&1), 2x + (n&1)) (conv + nn.PixelShuffle(2)).
 * out_shuffle=3 (phase-major sub-pixel, all four phases of a stride-2 transposed
 * conv in one launch): with q = co/4, channel n = (2*ry + rx)*q + c of lattice
 * pixel (y,x) goes to channel c of pixel (2y + ry, 2x + rx).                  */
typedef struct lic_conv_args {
  int32_t dtype;
  /* input view */
  const void* x; int32_t n, h, w, ci, ldx;
  /* output view (h, w are the full output map) */
  void* y; int32_t ho, wo, co, ldy;
  void* y2; int32_t ldy2;            /* optional second destination (same values) */
  /* lattice */
  int32_t mi, mj, oy0, ox0, osy, osx, isy, isx;
  int32_t ntaps; int8_t dy[LIC_MAX_TAPS]; int8_t dx[LIC_MAX_TAPS];
  int32_t groups;                    /* 1, or ci for depthwise (direct kernel only) */
  /* weights */
  const void* wgt; int32_t cpad, copad;
  const float* bias;                 /* may be NULL */
  /* prologue / epilogue */
  int32_t prologue;                  /* lic_prologue, applied to x values */
  int32_t act; float slope;
  int32_t epi;
  const void* r1; int32_t ldr1;      /* views with the output's pixel geometry */
  const void* g;  int32_t ldg;
  const void* r2; int32_t ldr2;
  int32_t out_shuffle;               /* 0, 2 or 3 */
  int32_t force_direct;              /* testing: force the non-MFMA kernel */
  int32_t force_mfma_generic;        /* testing: skip the spatial-tile (halo) kernel */
  /* fp32 only, spatial-tile (k x k) launches; others use wgt (exact fp32):
   * 0 = exact fp32-input MFMA;
   * 2 = "fp32x6": three bf16 parts per operand (x = x0+x1+x2 exactly, split in LDS), six
   *     products x0w0+x0w1+x1w0+x0w2+x1w1+x2w0 on the bf16 matrix cores (dropped terms <= 2^-26
   *     relative); wgt_split = the weights as bf16 [copad][ntaps][cpad/16][w0 16 | w1 16 | w2 16];
   * 1 = "fp32x3": fp16 parts, x_hi*W1 + x_hi*W2 + x_lo*W1 (x_lo = fp16(x - fp16(x)), ~3e-7
   *     relative per product); wgt_split = fp16 [copad][ntaps][cpad/16][W1 16 | W2 16],
   *     W1 = fp16(w)*2^11, W2 = fp16((w - fp16(w))*2^11).
   * LIC_F16 / LIC_BF16 (mfma_mode 0): wgt_split is optional -- the same 16-bit weights as wgt in
   * MFMA-fragment order [copad/32][cpad/16][ntaps][64 lanes][8], lane = 32 * (channel half) +
   * (row % 32), one contiguous 1 KB per A fragment (the conv16 / conv16s kernels read it when given,
   * round 6); NULL = wgt only. */
  int32_t mfma_mode;
  const void* wgt_split;
} lic_conv_args;

/* Convolution / linear layer (nn.Conv2d, nn.ConvTranspose2d phase, nn.Linear as
 * 1x1) with fused epilogue.  Replaces F.conv2d + activation + residual chains,
 * e.g. net_ga.py:89-103 (ResidualBottleneck), layers/layers.py:36-54,105-111,
 * compressai ResidualBlock/ResidualBlockWithStride/AttentionBlock, and
 * F.conv2d(x**2, gamma, beta) + x*rsqrt/sqrt of layers/gdn.py:62-75 /
 * model/gdn.py:69-92 (prologue SQUARE + GDN epilogues).                        */
int lic_conv2d_fwd(const lic_conv_args* a, lic_stream_t stream);

/* GDN parameter reparametrisation: beta' = max(beta,beta_bound)^2 - pedestal,
 * gamma' = max(gamma,gamma_bound)^2 - pedestal, written as packed conv weight
 * [copad][1][cpad] (dtype) and fp32 bias.  model/gdn.py:69-84 (LowerBound
 * :11-28, evaluated on device — no per-call host tensor) and
 * ops/parametrizers.py:48-51 + ops/bound_ops.py:40-41.                          */
int lic_gdn_prepare(int32_t dtype, const float* beta, const float* gamma, int32_t c,
                    float beta_bound, float gamma_bound, float pedestal,
                    void* wgt_out, int32_t cpad, int32_t copad, float* beta_out,
                    lic_stream_t stream);

/* Shifted-window multi-head self-attention core over a qkv view (3C channels,
 * q|k|v, head-major inside each): roll(-shift) + window_partition + (q*scale)k^T
 * (or (qk^T)*scale) + relative-position bias + mask + softmax + AV +
 * window_reverse + roll(+shift).  Output view has C channels at the original
 * pixel positions (the proj Linear + residual is a following conv launch).
 *   WBA  (layers/win_attention.py:85-116,154-209): scale_after=0, mask_kind=1 (-100)
 *   WMSA (model/Block_unet.py:216-252):           scale_after=1, mask_kind=2 (-inf)
 * Bias table element (r = dy*(2ws-1)+dx, head h) at table[r*tab_sr + h*tab_sh]. */
typedef struct lic_attn_args {
  int32_t dtype;
  const void* qkv; int32_t n, h, w, c, ldqkv;
  void* out; int32_t ldo;
  int32_t heads, ws, shift;
  const float* table; int32_t tab_sr, tab_sh;
  int32_t mask_kind;   /* 0 none, 1 WBA regions (-100), 2 WMSA last row/col (-inf) */
  int32_t scale_after; /* 0: q*scale before dot, 1: dot*scale */
  float scale;         /* head_dim ** -0.5 (as the reference's Python float, cast to fp32) */
  int32_t force_valu;  /* 1: skip the MFMA kernel (ws 8, head_dim <= 32) - testing only */
  int32_t mfma_mode;   /* fp32 data: 0 exact fp32 MFMA; 2 "fp32x6": Q, K, V, P split into three bf16
                          parts, 6 part products per dot (as lic_conv_args.mfma_mode 2) (abi 4) */
} lic_attn_args;
int lic_win_attn_fwd(const lic_attn_args* a, lic_stream_t stream);

/* LayerNorm over channels (nn.LayerNorm(C), eps) per pixel.  net_ga.py:115-127. */
int lic_layernorm_fwd(int32_t dtype, const void* x, int32_t npix, int32_t c, int32_t ldx,
                      const float* weight, const float* bias, float eps,
                      void* y, int32_t ldy, lic_stream_t stream);

/* Gaussian-conditional quantisation + rate for one slice (compressai
 * GaussianConditional in 'dequantize' mode at net_ga.py:1049, ste_round at :1053):
 *   q = rint(y - mu)           -> symbols (int32, may be NULL)
 *   yq = q + mu                -> yq / yq2 (dtype views, may be NULL)
 *   L  = max(Phi((.5-|yq-mu|)/s) - Phi((-.5-|yq-mu|)/s), 1e-9), s = max(scale, .11)
 *   partial[blockIdx] = sum ln L (fp64), nblocks written to *nparts.            */
typedef struct lic_rate_args {
  int32_t dtype;
  int32_t npix, c;
  const void* y; int32_t ldy;
  const void* mu; int32_t ldmu;
  const void* scale; int32_t ldsc;
  void* yq; int32_t ldyq;
  void* yq2; int32_t ldyq2;
  int32_t* symbols; int32_t ldsym;
  float* likelihood; int32_t ldlik;  /* fp32 view, may be NULL */
  double* partials; int32_t max_parts;
  float scale_bound, likelihood_bound;
} lic_rate_args;
int lic_gauss_rate_fwd(const lic_rate_args* a, lic_stream_t stream);

/* z_hat = round(z - m[c]) + m[c] (EntropyBottleneck._get_medians path,
 * net_ga.py:996-1003).  Also used for ste/bypass rounding with m = NULL. */
int lic_quantize_median(int32_t dtype, const void* z, int32_t npix, int32_t c, int32_t ldz,
                        const float* medians, void* out, int32_t ldo, lic_stream_t stream);

/* Sum of fp64 partials -> bpp = sum / (-ln2 * num_pixels) written as fp32 [1]
 * and fp64 [1] (net_ga.py:1134). */
int lic_bpp_finalize(const double* partials, int32_t nparts, double num_pixels,
                     float* bpp_out, double* sum_out, lic_stream_t stream);

/* Syntax-generated per-image 1x1 head + tanh + clamp + 8-bit metrics:
 * net_ga.py:969-979 (batch_conv), :1092 (tanh), :1118 (clamp), :1137-1142.
 *   xt[b,o] = clamp(tanh(sum_c wgen[b*ldw + o*cin + c] * xtil[b,pix,c]), -1, 1)  (wgen in dtype)
 *   sqerr_partial[b][blk] = sum (round(clamp((xt+1)*127.5,0,255)) - round((x+1)*127.5))^2
 * x (reference input) and x_rec are NCHW fp32 [n,3,h,w]; xtil is an NHWC view. */
int lic_syntax_recon_fwd(int32_t dtype, const void* xtil, int32_t n, int32_t h, int32_t w,
                         int32_t cin, int32_t ldx, const void* wgen, int32_t ldw, const float* x,
                         float* x_rec, double* sqerr_partials, int32_t parts_per_img,
                         lic_stream_t stream);
/* v_mse[b] = sum/(3hw); v_psnr = mean_b 20 log10(255/sqrt(v_mse[b])). */
int lic_psnr_finalize(const double* sqerr_partials, int32_t n, int32_t parts_per_img,
                      double count, float* v_mse, float* v_psnr, lic_stream_t stream);

/* Layout / elementwise helpers. */
/* NCHW fp32 -> NHWC view of dtype (and back); channels [c, cpad) of the
 * destination are zero-filled (cpad = c for a plain conversion). */
int lic_nchw_to_nhwc(int32_t dtype, const float* x, int32_t n, int32_t c, int32_t h, int32_t w,
                     void* y, int32_t ldy, int32_t cpad, lic_stream_t stream);
/* Fused ResidualBottleneck(3) (net_ga.py:89-103 with N = 3: 1x1 3->1, GELU,
 * 3x3 1->1, GELU, 1x1 1->3, + x) in one pass; params = w1[3], b1, w2[9], b2,
 * w3[3], b3[3] (fp32).  Writes all ldy channels of each output pixel
 * (channels 3.. zero) so the 3->192 convolutions can run on MFMA. */
int lic_rb3_fwd(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t ldx,
                const float* params, void* y, int32_t ldy, lic_stream_t stream);
/* nblk (1..3) consecutive ResidualBottleneck(3) blocks in one launch (the a_model's first three,
 * net_ga.py:262-264): params = nblk x the 20 floats above; equals nblk lic_rb3_fwd launches (the
 * intermediate blocks rounded to dtype where those launches store them).  y must not alias x. */
int lic_rb3_chain_fwd(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t ldx,
                      const float* params, int32_t nblk, void* y, int32_t ldy, lic_stream_t stream);
int lic_nhwc_to_nchw(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t c,
                     int32_t ldx, float* y, lic_stream_t stream);
/* y = a + b (views, same geometry). */
int lic_add(int32_t dtype, const void* a, int32_t lda, const void* b, int32_t ldb, int32_t npix,
            int32_t c, void* y, int32_t ldy, lic_stream_t stream);
/* Copy a view (optionally casting dtype). */
int lic_copy(int32_t dtype_in, const void* x, int32_t ldx, int32_t npix, int32_t c,
             int32_t dtype_out, void* y, int32_t ldy, lic_stream_t stream);
/* Adaptive average pool to 1x1 (nn.AdaptiveAvgPool2d(1)) into a dtype row
 * y[b*ldy + c] (fp32 accumulation). */
int lic_avgpool(int32_t dtype, const void* x, int32_t n, int32_t hw, int32_t c, int32_t ldx,
                void* y, int32_t ldy, lic_stream_t stream);

/* ---- Entropy coder ---------------------------------
 * The reference only ESTIMATES the rate (net_ga.py:1049 likelihoods, :1104-1107
 * bpp) and never writes a bitstream.  These entry points are the coder of its
 * entropy models' library (compressai 1.2.x, unvendored): CDF tables built as
 * GaussianConditional.update / EntropyBottleneck.update do, and the Rans64 coder of
 * BufferedRansEncoder::encode_with_indexes / RansDecoder::decode_with_indexes
 * (precision 16, 4-bit bypass chunks for values outside a table).  A latent is
 * coded as independent streams, one per (image, channel), symbols in raster
 * order; each stream is exactly the compressai string of that symbol list.
 * CDF tables are [ntab][cdf_stride] int32 with cdf_sizes[t] = pmf length + 2
 * and offsets[t] = the symbol value of table entry 0.                          */

/* Gaussian pmfs of compressai GaussianConditional.update(): table t has
 * 2*pmf_center[t]+1 entries pmf[k] = Phi((.5-|k-c|)/s) - Phi((-.5-|k-c|)/s)
 * followed by the tail mass 2*Phi((-.5-c)/s); rows of pmf_stride floats. */
int lic_gauss_pmf(const float* scale_table, const int32_t* pmf_center, int32_t ntab, int32_t pmf_stride,
                  float* pmf, lic_stream_t stream);

/* Factorized-prior pmfs of compressai EntropyBottleneck.update() for the
 * default filters (3,3,3,3): params is [c][LIC_EB_PARAMS] fp32 per channel
 * (matrix0..4, bias0..4, factor0..3 flattened in that order, raw parameters:
 * softplus / tanh are applied here); pmf_start[c] = median - minima,
 * pmf_length[c] entries then the tail mass.  pmf_stride must be
 * max(pmf_length) + 1: the upper tail is evaluated at sample pmf_stride - 2 for
 * every channel, as compressai does on its padded sample grid. */
#define LIC_EB_PARAMS 58
int lic_eb_pmf(const float* params, const float* pmf_start, const int32_t* pmf_length, int32_t c,
               int32_t pmf_stride, float* pmf, lic_stream_t stream);

/* compressai pmf_to_quantized_cdf per table: nsym[t] pmf entries (tail included)
 * -> nsym[t]+1 cdf entries at `precision` bits.  status[t] = 0, or 1 when no
 * frequency could be stolen (degenerate pmf). */
int lic_pmf_to_cdf(const float* pmf, const int32_t* nsym, int32_t ntab, int32_t pmf_stride, int32_t precision,
                   int32_t* cdf, int32_t cdf_stride, int32_t* status, lic_stream_t stream);

/* GaussianConditional.build_indexes: idx = ntab-1 - #{t < ntab-1 : max(scale, bound) <= table[t]}. */
int lic_gauss_indexes(int32_t dtype, const void* scales, int32_t npix, int32_t c, int32_t ldsc,
                      const float* scale_table, int32_t ntab, float bound, int32_t* idx, int32_t ldidx,
                      lic_stream_t stream);

/* symbols = (int) round_half_even(z - m[c]) (EntropyModel.quantize(..., "symbols", medians));
 * medians may be NULL (0). */
int lic_quantize_symbols(int32_t dtype, const void* z, int32_t npix, int32_t c, int32_t ldz, const float* medians,
                         int32_t* sym, int32_t ldsym, lic_stream_t stream);

/* Streams: s = b * ctot + c0 + ch for image b < n, channel ch < c; hw symbols each
 * at pixel rows [b*hw, (b+1)*hw) of the channel-window views. */
typedef struct lic_rans_args {
  int32_t n, hw, c, ctot, c0;
  const int32_t* symbols; int32_t ldsym;      /* encode: input */
  const int32_t* indexes; int32_t ldidx;      /* NULL: table index = channel (c0 + ch) */
  const int32_t* cdfs; int32_t cdf_stride;
  const int32_t* cdf_sizes; const int32_t* offsets; int32_t ncdf;
  /* encode: per-stream scratch [n*ctot][cap] words; the string ends at the row end */
  uint32_t* scratch; int32_t cap; int32_t* lengths;   /* words, -1 = overflow / bad index */
  /* decode: stream s occupies words[offsets_w[s] .. offsets_w[s+1]) */
  const uint32_t* words; const uint32_t* offsets_w;
  int32_t dtype;                              /* of mu / yq */
  int32_t* out_symbols; int32_t ldosym;       /* decode outputs (each may be NULL) */
  const void* mu; int32_t ldmu;               /* per-element means (dtype) or NULL */
  const float* mu_ch;                         /* per-channel means (medians) or NULL */
  void* yq; int32_t ldyq;                     /* (float)symbol + mean, as lic_gauss_rate_fwd */
  int32_t* status;                            /* decode: [n*c] 0 ok, 1 = the stream ended early or
                                                 named an invalid table (rANS cannot detect other
                                                 corruption; reads never pass the stream's end) */
} lic_rans_args;
/* Upper bound of the words a stream of hw symbols can take (scratch row size). */
int32_t lic_rans_cap(int32_t hw);
int lic_rans_encode(const lic_rans_args* a, lic_stream_t stream);
/* Exclusive scan of lengths[nstreams] into offsets_w[nstreams+1] and copy of every
 * scratch string to out (capacity nstreams*cap words).  Lengths must be >= 0. */
int lic_rans_pack(const uint32_t* scratch, int32_t cap, const int32_t* lengths, int32_t nstreams,
                  uint32_t* offsets_w, uint32_t* out, lic_stream_t stream);
int lic_rans_decode(const lic_rans_args* a, lic_stream_t stream);

/* ---- HAN post-processing (model/han.py, net_ga.py:1096-1100).
 * The 3x3 / 1x1 convolutions of HAN run on lic_conv2d_fwd; these are the glue ops.  */

/* Per-(image, pixel chunk) channel sums of x (fp32): parts[(b*nchunk + k)*c + ch],
 * chunk k = pixels [k*ceil(hw/nchunk), ...).  The CALayer average pool in two
 * passes, so a 256x256 map is reduced by n*nchunk workgroups.                    */
int lic_pool_partials(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t c,
                      int32_t nchunk, float* parts, lic_stream_t stream);

/* CALayer + RCAB residual (han.py:97-113, :205-225):
 *   y = sigmoid(W2 relu(W1 mean + b1) + b2), mean = sum_k parts[b][k] / hw;  out = r * y + x
 * parts from lic_pool_partials(r), sized n*(nchunk+1)*c floats: y[b][c] is written after
 * the partials.  W1 [cr][c], W2 [c][cr] fp32. */
int lic_ca_apply_fwd(int32_t dtype, const void* r, int32_t ldr, const void* x, int32_t ldx, int32_t n,
                     int32_t hw, int32_t c, float* parts, int32_t nchunk, const float* w1,
                     const float* b1, const float* w2, const float* b2, int32_t cr, void* out,
                     int32_t ldo, lic_stream_t stream);

/* LAM_Module (han.py:124-150) over x = ngroups channel windows of c channels
 * (the NHWC image of the B x N x C x H x W stack):
 *   E = per-image Gram (fp64 partial sums), A = softmax(max(E) - E),
 *   out_n = gamma * sum_m A[n][m] x_m + x_n.
 * parts: n * lic_lam_parts(ngroups) doubles of scratch (Gram partials, then the
 * per-image attention matrices).  ngroups in {2, 5, 7}. */
int32_t lic_lam_parts(int32_t ngroups);
int lic_lam_fwd(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t hw, int32_t ngroups,
                int32_t c, double* parts, const float* gamma, void* out, int32_t ldo, lic_stream_t stream);

/* CSAM_Module (han.py:152-188): out = x * (gamma * sigmoid(conv3d(x) + bias)) + x with
 * the 3x3x3 Conv3d(1,1,3,1,1) sliding over (channel, y, x); params = {w[27], bias, gamma}. */
int lic_csam_fwd(int32_t dtype, const void* x, int32_t ldx, int32_t n, int32_t h, int32_t w, int32_t c,
                 const float* params, void* out, int32_t ldo, lic_stream_t stream);

/* Generalised reconstruction head (net_ga.py:969-979 batch_conv, :1092 tanh,
 * :1096-1100 HAN tail with add_mean, :1118/:1137-1141 metrics):
 *   v = W_b xtil (3 x cin per image), mode 1: tanh(v); post (fp32 [12], may be NULL):
 *   v = P v + p (row-major 3x3 then bias); y (NHWC dtype, ycpad channels, zero padded,
 *   may be NULL) <- v; x_rec (NCHW fp32, may be NULL) <- clamp(v, -1, 1); with x
 *   (NCHW fp32 input image) the squared 8-bit errors go to sqerr_partials.        */
int lic_recon_fwd(int32_t dtype, const void* xtil, int32_t n, int32_t h, int32_t w, int32_t cin,
                  int32_t ldx, const void* wgen, int32_t ldw, int32_t mode, const float* post,
                  const float* x, float* x_rec, double* sqerr_partials, int32_t parts_per_img, void* y,
                  int32_t ldy, int32_t ycpad, lic_stream_t stream);

/* ------------------------------------------------------------------ training path
 * Backward of the hot-path layers: the reference's
 * loss.backward() through Net.forward(x, 'train') — train_net_unet.py:177-200 and the
 * online encoder finetune eval_net.py:170-179.  Conv dgrad needs no entry point: it is
 * lic_conv2d_fwd over dz with transposed / tap-mirrored (stride 1) or transposed-conv
 * phase (stride 2) packed weights (lic_amd/autograd.py).                            */

/* Weight gradient of one conv launch (same tap / lattice form as lic_conv2d_fwd):
 *   dw[n*s_co + c*s_ci + t*s_tap] (+)= sum_{b,i,j} dz[b, oy0+osy*i, ox0+osx*j, n]
 *                                        * pro(x[b, i*isy+dy[t], j*isx+dx[t], c])
 * for n < co_out, c < ci_out (x zero outside the map; pro = identity or square, the
 * latter for GDN's dGamma = sum dn * x^2).  Replaces F.conv2d's / F.conv_transpose2d's
 * autograd weight gradient (torch.nn.grad.conv2d_weight) for every nn.Conv2d of
 * net_ga.py / net_unet_ha_hs.py / the layers/ modules and for GDN gamma (model/gdn.py:85-92,
 * layers/gdn.py:62-75).  MFMA implicit GEMM, K = output pixels split across
 * work-groups; fp32 partials in caller workspace (size: lic_conv2d_wgrad_workspace),
 * deterministic reduce.  ci, co, ldx, ldz multiples of 16 bytes; views 16-B aligned. */
typedef struct lic_wgrad_args {
  int32_t dtype;
  const void* x; int32_t n, h, w, ci, ldx;       /* forward input view                 */
  const void* dz; int32_t ho, wo, co, ldz;       /* grad at the conv output (pre-act)  */
  int32_t mi, mj, oy0, ox0, osy, osx, isy, isx;  /* lattice, as lic_conv_args          */
  int32_t ntaps; int8_t dy[LIC_MAX_TAPS]; int8_t dx[LIC_MAX_TAPS];
  int32_t prologue;                              /* LIC_PRO_NONE or LIC_PRO_SQUARE     */
  float* dw; int64_t s_co, s_ci, s_tap;          /* fp32 destination + element strides */
  int32_t co_out, ci_out, accumulate;
  float* ws; int64_t ws_bytes;
  float* db;           /* optional (NULL: none): fp32 bias gradient, db[n] (+)= sum of dz[., n] over the
                          lattice, n < co_out (accumulate as dw); the lattice must be dz's full map (abi 4) */
} lic_wgrad_args;
int64_t lic_conv2d_wgrad_workspace(const lic_wgrad_args* a);   /* bytes, -1 on bad args */
int lic_conv2d_wgrad(const lic_wgrad_args* a, lic_stream_t stream);

/* Deferred split-K reduce (a training step's weight gradients summed by ONE launch after the
 * backward; round 6).  lic_conv2d_wgrad_partials: when the tiled 16-bit kernel applies, launches
 * only its partial sums into a->ws and sets *nsplit (> 0): dw / db are NOT written until a
 * lic_wgrad_reduce_batch over a descriptor of this call runs; otherwise runs lic_conv2d_wgrad
 * whole and sets *nsplit = 0.  lic_wgrad_reduce_blocks(a): the call's 256-thread reduce blocks.
 * lic_wgrad_reduce_batch: `desc` is DEVICE memory holding n descriptors of
 * LIC_WGRAD_RED_DESC_WORDS int64 each,
 *   { ws, wsb (bias partials = ws + nsplit*ntaps*co*ci floats, or 0), dw, db (or 0), s_co, s_ci,
 *     s_tap, nsplit, ntaps, co, ci, co_out, ci_out, accumulate, first_block, 0 },
 * ascending first_block; the per-element sums are lic_conv2d_wgrad's (same order: bit-identical).
 * Replaces the per-layer reduce of train_net_unet.py:177-200's loss.backward(). */
#define LIC_WGRAD_RED_DESC_WORDS 16
int lic_conv2d_wgrad_partials(const lic_wgrad_args* a, int32_t* nsplit, lic_stream_t stream);
int32_t lic_wgrad_reduce_blocks(const lic_wgrad_args* a);
int lic_wgrad_reduce_batch(const int64_t* desc, int32_t n, int32_t nblocks, lic_stream_t stream);

/* Per-channel sum over pixels (bias / beta gradients): out[c] (+)= sum_p x[p*ldx + c].
 * fp32 out; workspace lic_channel_sum_workspace(c) bytes.                          */
int64_t lic_channel_sum_workspace(int32_t c);
int lic_channel_sum(int32_t dtype, const void* x, int32_t ldx, int32_t npix, int32_t c, float* ws,
                    int64_t ws_bytes, float* out, int32_t accumulate, lic_stream_t stream);

/* Activation forward / backward: y = act(z); dz = dy * act'(z) (nn.LeakyReLU,
 * nn.GELU (erf), nn.ReLU; ROUND is straight-through as ste_round, net_ga.py:713-719). */
int lic_act_fwd(int32_t dtype, const void* z, int32_t ldz, int32_t npix, int32_t c, int32_t act,
                float slope, void* y, int32_t ldy, lic_stream_t stream);
int lic_act_bwd(int32_t dtype, const void* z, int32_t ldz, const void* dy, int32_t lddy, int32_t npix,
                int32_t c, int32_t act, float slope, void* dz, int32_t lddz, lic_stream_t stream);

/* Gate y = g * sigmoid(a) + r (Win_noShift_Attention, layers/layers.py:105-111):
 * da = dy*g*s*(1-s), dg = dy*s (dg may be NULL); dr = dy needs no kernel.          */
int lic_gate_bwd(int32_t dtype, const void* a, int32_t lda, const void* g, int32_t ldg, const void* dy,
                 int32_t lddy, int32_t npix, int32_t c, void* da, int32_t ldda, void* dg, int32_t lddg,
                 lic_stream_t stream);

/* GDN / IGDN backward, y = x * n^p, n = beta' + Gamma' x^2 (p = -1/2, +1/2):
 *   elem:   dxd = dy * n^p,   u = dn = dy * x * p * n^(p-1)
 *   finish: dx (+)= dxd + 2 x t, with t = Gamma'^T u (lic_conv2d_fwd, transposed pack)
 * dGamma' = lic_conv2d_wgrad(dz=u, x, PRO_SQUARE), dbeta' = lic_channel_sum(u).
 * model/gdn.py:69-92 / :133-156, layers/gdn.py:62-75.                              */
int lic_gdn_bwd_elem(int32_t dtype, const void* x, int32_t ldx, const void* nrm, int32_t ldn,
                     const void* dy, int32_t lddy, int32_t npix, int32_t c, int32_t inverse, void* dxd,
                     int32_t lddxd, void* u, int32_t ldu, lic_stream_t stream);
int lic_gdn_bwd_finish(int32_t dtype, const void* x, int32_t ldx, const void* t, int32_t ldt,
                       const void* dxd, int32_t lddxd, int32_t npix, int32_t c, void* dx, int32_t lddx,
                       int32_t accumulate, lic_stream_t stream);

/* LowerBound + square reparametrisation backward (q' = max(q,bound)^2 - pedestal):
 * dq (+)= [q >= bound or g < 0] * g, g = dq' * 2 max(q, bound).  ops/bound_ops.py:25-28,
 * model/gdn.py:18-26, ops/parametrizers.py:45-49.  fp32, `count` elements.          */
int lic_lower_bound_sq_bwd(const float* q, const float* dq_eff, int32_t count, float bound, float* dq,
                           int32_t accumulate, lic_stream_t stream);

/* Weight pack into the conv launches' layout dst[copad][nty*ntx][cpad] (dtype, RNE) from an fp32
 * weight read through signed element strides: dst[o][ty*ntx+tx][c] = src[o*so + c*sc + ty*sy +
 * tx*sx] for o < no, c < nc, else 0.  One launch per pack: nn.Conv2d [co,ci,kh,kw] (so, sc, sy, sx
 * = its strides), the dgrad pack (transposed: so <-> sc; mirrored taps: src at the last tap,
 * sy, sx < 0), stride-s dgrad / ConvTranspose2d phases (sy = s*kw, ...).  The training path
 * re-packs every weight each step (reference train_net_unet.py:198-199: clip + opt.step, then the next forward). */
int lic_pack_taps(int32_t dtype, const float* src, int64_t so, int64_t sc, int64_t sy, int64_t sx, int32_t no,
                  int32_t nc, int32_t nty, int32_t ntx, void* dst, int32_t copad, int32_t cpad,
                  lic_stream_t stream);

/* Many lic_pack_taps in one launch (a training step's packs, replayed in a hipGraph): `desc` is
 * DEVICE memory holding n descriptors of LIC_PACK_DESC_WORDS int64 each,
 *   { src, dst, so, sc, sy, sx, no, nc, nty, ntx, copad, cpad, dtype, first_block, 0, 0 },
 * ascending first_block; descriptor i owns blocks [first_block_i, first_block_{i+1}) of
 * lic_pack_block_elems() elements each (ceil(copad*nty*ntx*cpad / that)); nblocks = the total.
 * The caller validates the descriptors (the library cannot read device memory on the host).      */
#define LIC_PACK_DESC_WORDS 16
int32_t lic_pack_block_elems(void);
int lic_pack_taps_batch(const int64_t* desc, int32_t n, int32_t nblocks, lic_stream_t stream);

/* Window-attention core backward (WBA layers/win_attention.py:85-116, WMSA
 * model/Block_unet.py:216-252): given the forward args `a` (qkv view, table, mask)
 * and dO (C channels per pixel), writes dqkv (3C channels: dq | dk | dv) and, if
 * dtable != NULL, the relative-position-bias gradient (same layout as a.table,
 * workspace lic_win_attn_bwd_workspace bytes).  Scores and softmax are recomputed
 * in the forward's op order; window <= 8x8, LDS-resident per (image, window, head). */
int64_t lic_win_attn_bwd_workspace(const lic_attn_args* a);
int lic_win_attn_bwd(const lic_attn_args* a, const void* dout, int32_t lddo, void* dqkv, int32_t lddq,
                     float* dtable, int32_t accumulate_table, float* ws, int64_t ws_bytes,
                     lic_stream_t stream);

/* nn.LayerNorm(C) backward (net_ga.py:115-127): dx, and dwb = [dweight(C) | dbias(C)]
 * fp32 (+)=; workspace lic_layernorm_bwd_workspace(npix, c) bytes; C <= 768.          */
int64_t lic_layernorm_bwd_workspace(int32_t npix, int32_t c);
int lic_layernorm_bwd(int32_t dtype, const void* x, int32_t ldx, const void* dy, int32_t lddy,
                      int32_t npix, int32_t c, const float* weight, float eps, void* dx, int32_t lddx,
                      float* dwb, int32_t accumulate, float* ws, int64_t ws_bytes, lic_stream_t stream);

/* Gate forward y = g * sigmoid(a) (+ r) (r may be NULL), the unfused form the training
 * path keeps `a` for (layers/layers.py:105-111, net_ga.py:153-174).               */
int lic_gate_fwd(int32_t dtype, const void* a, int32_t lda, const void* g, int32_t ldg, const void* r,
                 int32_t ldr, int32_t npix, int32_t c, void* y, int32_t ldy, lic_stream_t stream);

/* LRP refinement y = r + 0.5 tanh(x) (net_ga.py:1060-1062) and its backward
 * dx = dy * 0.5 (1 - tanh(x)^2) (dr = dy needs no kernel).                        */
int lic_half_tanh_fwd(int32_t dtype, const void* x, int32_t ldx, const void* r, int32_t ldr, int32_t npix,
                      int32_t c, void* y, int32_t ldy, lic_stream_t stream);
int lic_half_tanh_bwd(int32_t dtype, const void* x, int32_t ldx, const void* dy, int32_t lddy,
                      int32_t npix, int32_t c, void* dx, int32_t lddx, lic_stream_t stream);

/* nn.AdaptiveAvgPool2d(1) backward (Syntax_Model pooling, net_ga.py:627-646):
 * dx[b, p, c] = dy[b, c] / hw.                                                    */
int lic_avgpool_bwd(int32_t dtype, const void* dy, int32_t lddy, int32_t n, int32_t hw, int32_t c,
                    void* dx, int32_t lddx, lic_stream_t stream);

/* Training-mode GaussianConditional (compressai, net_ga.py:1049, mode 'train'):
 * y~ = y + U(-1/2,1/2) (counter-based noise from `seed` and the element index, so the
 * backward regenerates it), L' = LowerBound(Phi((1/2-|y~-mu|)/s) - Phi((-1/2-|y~-mu|)/s),
 * 1e-9), s = LowerBound(scale, 0.11); partials[block] = sum ln L' (fp64,
 * lic_rate_train_parts blocks); yhat (may be NULL) = rint(y-mu)+mu (ste_round forward).
 * bwd: with gout = dLoss/dbpp (device fp32 scalar) and factor = -1/(ln2 * num_pixels):
 * dy, dmu, dscale of factor * gout * sum ln L' (LowerBound gradient rules).
 * seed_dev (may be NULL): the noise seed is seed_dev[0] * seed_mul + seed, read on the device,
 * so a captured hipGraph of a training step draws a new stream per replay.        */
int32_t lic_rate_train_parts(int32_t npix, int32_t c);
int lic_rate_train_fwd(int32_t dtype, const void* y, int32_t ldy, const void* mu, int32_t ldmu,
                       const void* scale, int32_t ldsc, int32_t npix, int32_t c, uint64_t seed,
                       const uint64_t* seed_dev, uint64_t seed_mul,
                       float scale_bound, float likelihood_bound, void* yhat, int32_t ldyh,
                       double* partials, lic_stream_t stream);
int lic_rate_train_bwd(int32_t dtype, const void* y, int32_t ldy, const void* mu, int32_t ldmu,
                       const void* scale, int32_t ldsc, int32_t npix, int32_t c, uint64_t seed,
                       const uint64_t* seed_dev, uint64_t seed_mul,
                       float scale_bound, float likelihood_bound, const float* gout, float factor,
                       void* dy, int32_t lddy, void* dmu, int32_t lddmu, void* dscale, int32_t lddsc,
                       lic_stream_t stream);

/* Training reconstruction head: x~ = tanh(W_b x16) per image (batch_conv + tanh,
 * net_ga.py:969-979,1092), xt (NCHW fp32, may be NULL), per-(image, block) squared
 * error partials vs img (NCHW fp32) for nn.MSELoss (net_ga.py:1115).  bwd with
 * gout = dLoss/dmse (device scalar), factor = 2/(B*3*H*W): dx16 and dW_b (fp32
 * [n][3*cin]); workspace n * lic_recon_train_blocks(hw) * 3 * cin floats.          */
int32_t lic_recon_train_blocks(int32_t hw);
int lic_recon_train_fwd(int32_t dtype, const void* x16, int32_t ldx, int32_t n, int32_t hw, int32_t cin,
                        const void* wgen, int32_t ldw, const float* img, float* xt, double* partials,
                        lic_stream_t stream);
int lic_recon_train_bwd(int32_t dtype, const void* x16, int32_t ldx, int32_t n, int32_t hw, int32_t cin,
                        const void* wgen, int32_t ldw, const float* img, const float* gout, float factor,
                        void* dx16, int32_t lddx, float* dw, float* ws, int64_t ws_bytes,
                        lic_stream_t stream);

/* Depthwise (groups = C) conv weight gradient, dw fp32 in torch [C, 1, kh, kw] order
 * (Syntax_Model's DepthwiseSeparableConv, net_ga.py:613-619).  Tap offsets are host
 * arrays (copied into the kernel arguments).                                       */
int64_t lic_dwconv_wgrad_workspace(int32_t n, int32_t ho, int32_t wo, int32_t c, int32_t ntaps);
int lic_dwconv_wgrad(int32_t dtype, const void* x, int32_t ldx, const void* dz, int32_t ldz, int32_t n,
                     int32_t h, int32_t w, int32_t ho, int32_t wo, int32_t c, int32_t stride,
                     int32_t ntaps, const int8_t* dy, const int8_t* dx, float* dw, float* ws,
                     int64_t ws_bytes, lic_stream_t stream);

/* Patch (im2col) map of a small-channel input for one conv's taps (fp32):
 *   y[b, i, j, t*c + ch] = x[b, i*stride + dy[t], j*stride + dx[t], ch] (zero outside the map),
 *   channels [ntaps*c, cpad) zero; dy / dx host arrays, ntaps <= 32.  Lets the image's first conv
 *   (Cin 3, ResidualBlockWithStride.conv1 at net_ga.py:271) run as a 1x1 conv with K = 27 -> 32 instead
 *   of 9 taps of a 16-channel-padded input.                                        */
int lic_patches(int32_t dtype, const void* x, int32_t n, int32_t h, int32_t w, int32_t c, int32_t ldx,
                int32_t ho, int32_t wo, int32_t stride, int32_t ntaps, const int8_t* dy, const int8_t* dx,
                void* y, int32_t ldy, int32_t cpad, lic_stream_t stream);

/* compressai AttentionBlock ResidualUnit(N) in one launch, fp32 activations with fp32x6 split
 * products (mfma_mode 2):  y = relu(conv1x1_{N/2->N}(relu(conv3x3_{N/2->N/2}(relu(conv1x1_{N->N/2}(x)))))
 * + x), conv3x3 zero-padded by 1.  Replaces the three lic_conv2d_fwd launches of one ResidualUnit
 * (compressai layers.py AttentionBlock.ResidualUnit; SWAtten conv_a / conv_b at net_ga.py:118-136,
 * 6 per SWAtten).  w1s / w2s / w3s are the three convs' fp32x6 split packs in MFMA-fragment order
 * (lic_conv_args.wgt_split: conv[0] copad N/2 cpad N 1 tap, conv[2] copad N/2 cpad N/2 9 taps
 * row-major (dy, dx) = (-1..1, -1..1), conv[4] copad N cpad N/2 1 tap); b1 / b2 / b3 fp32 biases.
 * N = 128; h, w multiples of 8; x != y; views, weights and biases 16-B aligned (abi 5). */
typedef struct lic_resunit_args {
  int32_t dtype;                       /* LIC_F32 */
  const void* x; int32_t n, h, w, c, ldx;
  void* y; int32_t ldy;
  const void* w1s; const void* w2s; const void* w3s;
  const float* b1; const float* b2; const float* b3;
  int32_t mfma_mode;                   /* 2 */
} lic_resunit_args;
int lic_resunit_fwd(const lic_resunit_args* a, lic_stream_t stream);

/* fp32x6 WinBasedAttention in one launch (abi 6): qkv Linear + the shifted-window attention of
 * lic_win_attn_fwd (WBA: q*scale before the dot, mask_kind 1) without the qkv map in HBM, for
 * C = 192, 8 heads, 8x8 windows (the Win_noShift_Attention blocks at 64x64, layers/layers.py:87-102;
 * layers/win_attention.py:85-116,154-209).  proj_wsplit NULL: out = the attention output (C channels
 * per pixel) that the proj Linear consumes; else out = x + proj(attention) (the whole block, out !=
 * x).  Bit-identical to lic_conv2d_fwd(qkv, mfma_mode 2) + lic_win_attn_fwd(mfma_mode 2)
 * (+ lic_conv2d_fwd(proj, r1 = x)).  *_wsplit = fp32x6 split packs in MFMA-fragment order (qkv
 * [18][12][1][3][64][8], proj [6][12][1][3][64][8] bf16); biases fp32. */
typedef struct lic_wba_args {
  const float* x; int32_t n, h, w, c, ldx;   /* fp32 NHWC input (the block's x), c = 192 */
  float* out; int32_t ldo;                   /* fp32 NHWC attention output, c channels */
  int32_t heads, ws, shift, mask_kind;       /* 8, 8, shift, 1 */
  float scale;                               /* head_dim ** -0.5 */
  const float* table; int32_t tab_sr, tab_sh;
  const void* qkv_wsplit;
  const float* qkv_bias;
  const void* proj_wsplit;                   /* NULL: attention output only */
  const float* proj_bias;
} lic_wba_args;
int lic_wba_qkv_attn_fwd(const lic_wba_args* a, lic_stream_t stream);

/* 16-bit (fp16 / bf16) WinBasedAttention core in one launch (csrc/wba16.hip; ABI 7): the qkv Linear
 * (the 16-bit packed [3C][1][C] weights of its ConvPack, fp32 bias) + shifted-window attention with
 * the unfused launches' arithmetic (q, k, v rounded to the 16-bit type after the bias, the scale on
 * the fp32 dot); out = the C-channel attention output the proj Linear consumes.  C = 192, 8 heads,
 * 8x8 windows, H and W multiples of 8; x 16-B aligned rows of 8k elements, out 8-B aligned and not
 * overlapping x.
 * Replaces model/layers.py WinBasedAttention's qkv + attention (reference layers/win_attention.py:85-116). */
typedef struct lic_wba16_args {
  int32_t dtype;                             /* LIC_F16 or LIC_BF16 */
  const void* x; int32_t n, h, w, c, ldx;    /* NHWC input (the block's x), c = 192 */
  void* out; int32_t ldo;                    /* NHWC attention output, c channels */
  int32_t heads, ws, shift, mask_kind;       /* 8, 8, shift, 1 */
  float scale;                               /* head_dim ** -0.5 */
  const float* table; int32_t tab_sr, tab_sh;
  const void* qkv_w;                         /* [3C][1][C] packed weights, same dtype as x */
  const float* qkv_bias;                     /* [3C] */
} lic_wba16_args;
int lic_wba16_qkv_attn_fwd(const lic_wba16_args* a, lic_stream_t stream);

/* Library info.
 * LIC_ABI_VERSION changes whenever an entry point's parameter list or an args struct's layout
 * changes (3: lic_conv_args.mfma_mode / wgt_split, lic_rate_train_* seed_dev / seed_mul; 5:
 * lic_resunit_args / lic_resunit_fwd; 6: lic_wba_args / lic_wba_qkv_attn_fwd; 7: lic_wba16_args /
 * lic_wba16_qkv_attn_fwd).  A
 * caller compiled against this header checks lic_abi_version() == LIC_ABI_VERSION and
 * lic_args_size(k) == sizeof(...) once after loading the library (the Python host does, _ffi.load). */
#define LIC_ABI_VERSION 7
enum { LIC_ARGS_CONV = 0, LIC_ARGS_ATTN = 1, LIC_ARGS_RATE = 2, LIC_ARGS_RANS = 3, LIC_ARGS_WGRAD = 4,
       LIC_ARGS_RESUNIT = 5, LIC_ARGS_WBA = 6, LIC_ARGS_WBA16 = 7 };
const char* lic_last_error(void);
const char* lic_version(void);          /* "liblic <ver> gfx950 (abi N, src <source hash>)" */
/* Build provenance: the first 16 hex digits of the SHA-256 of the sources the library was built
 * from (csrc/ *.hip *.h Makefile in name order, then include/lic.h, concatenated).  The Python host
 * recomputes it from the tree and refuses a library built from other sources (_ffi.load). */
const char* lic_source_hash(void);
int32_t lic_abi_version(void);
int64_t lic_args_size(int32_t which);   /* sizeof the LIC_ARGS_* struct the library was built with, -1 if unknown */
int lic_device_arch(char* buf, int32_t len);

#ifdef __cplusplus
}
#endif
#endif /* LIC_H_ */
