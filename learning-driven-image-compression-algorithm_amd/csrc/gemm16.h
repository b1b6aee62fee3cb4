// 16-bit (fp16 / bf16) 1x1 convolution -- a GEMM over pixels -- on big maps, round 5 ("gemm16").
//
// The a_model's 1x1 layers (WinBasedAttention qkv 192->576 / proj 192->192, ResidualBottleneck
// 192->96 / 96->192, GDN's conv(x^2, gamma) + x*rsqrt epilogue, the 1x1 s2 skip) do 2*K flops per
// byte moved at K <= 192: they are HBM-bound, so the kernel is built to stream:
//   * a workgroup (4 waves) keeps the packed weights of its BN output channels in LDS for its
//     whole life ([K/16][BN][32 B], swizzled like conv16.h) -- loaded once, never re-streamed;
//   * the grid is persistent (one 8-wave workgroup per CU); each WAVE walks 32-pixel tiles on its own
//     (no barrier in the loop), loading a tile's activations straight into MFMA B-fragment
//     registers (lane = pixel, 16 B = 8 channels: one raw buffer load per 16-channel K step; rows
//     past the map read zeros through the buffer range) while the previous tile computes;
//   * transposed MFMA (A = weights from LDS, B = pixels); the x^2 prologue squares the fragments in
//     registers; the fused epilogue (bias, activation, residual / gate / GDN; lic_common.h) stages each
//     32 x 32 tile in a wave-private LDS slot and stores 16 B of consecutive channels per lane.
// MFMA is a quarter busy at the HBM rate: the bound is the bytes (x once, y once per N block).
#pragma once
#include <cstdio>
#include "conv16.h"

namespace lic {


// a wave's epilogue slot: 32 x 33 fp32 (general) or 32 rows of 208 B + 32 destinations (register path)
constexpr int G16_SLOT = 32 * 208 + 32 * 8;

struct G16Plan {
  int M;          // output lattice pixels (n * mi * mj)
  int ntiles;     // ceil(M / 32)
  int nblk;       // output-channel blocks (copad / BN)
  int wgs;        // workgroups per channel block
  unsigned xrec;  // bytes addressable from a.x
  unsigned wrec;  // bytes of the packed weights
  int fast_epi;   // 1: the register epilogue (g16_fast_epi_ok); 2: + GDN g from the fragments (g16_gx_ok)
};

// KT = 1: a 1x1 convolution, K step kk = input channels 16kk .. 16kk+15.  KT > 1: a small-Cin k x k
// convolution (the image's first layers: Cin 8 or 16, any stride) as an implicit GEMM without a halo:
// K step kk = tap kk's 16 channels, each lane loading its pixel's tap directly (the taps' re-reads of
// neighbouring pixels are L1 / L2 hits); channels 8..15 read zeros when Cin is 8.
// FAST: 0 = the shared epilogue (c16_epilogue), 1 = the register epilogue, 2 = the register epilogue of
// a GDN whose g is the layer's own input at the output pixel (g16_gx_ok): g is taken from this tile's
// B-fragment registers (the x^2 prologue squares a copy) instead of being loaded again.
template <typename T, int BN, int KST, int PRO, int KT = 1, int FAST = 0>
__global__ __launch_bounds__(512, 1) void gemm16_kernel(const lic_conv_args a, const G16Plan p) {
  // a wave computes 32 pixels x 96 channels (3 accumulator tiles); at BN = 192 two waves share each
  // pixel tile (its fragments are loaded twice, from L2 the second time)
  constexpr int NW = 8, WS = BN / 96, TN = 3, NSTREAM = NW / WS;
  static_assert(BN == 96 || BN == 192, "BN");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  float* sbias = (float*)(smem + KST * BN * 32);
  float* cts = sbias + BN;                 // NW epilogue slots (G16_SLOT bytes)
  int* rowpix_all = (int*)((char*)cts + NW * G16_SLOT);   // NW x 32 destination pixels

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int wc = wave % WS, wst = wave / WS;   // channel half, pixel stream
  const int nb = blockIdx.x % p.nblk;
  const int rank = blockIdx.x / p.nblk;
  const int n0 = nb * BN;

  // ---- weights of this channel block into LDS, once, by LDS-DMA (all pieces in flight together):
  // slot (kk, n, stored half ph) holds channel half ph ^ bit3(n) of K step kk; a 1-KB piece is 32
  // channels x 2 halves of one K step ----
  {
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.wgt, (short)0, (int)p.wrec, 0x00020000);
    const int wrow = a.ntaps * a.cpad;   // one output channel's packed weights [ntaps][cpad]
    const unsigned woff_lane = (unsigned)(((lane >> 1) * wrow + (((lane & 1) ^ ((lane >> 4) & 1)) * 8)) * 2);
    constexpr int NPIECE = KST * BN / 32;
    for (int P = wave; P < NPIECE; P += NW) {
      const int kk = P / (BN / 32), nq = P - kk * (BN / 32);
      c16_dma(wrs, smem + P * 1024, woff_lane, ((n0 + nq * 32) * wrow + (KT == 1 ? kk * 16 : kk * a.cpad)) * 2);
    }
    for (int n = tid; n < BN; n += NW * 64) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)p.xrec, 0x00020000);
  const int mij = a.mi * a.mj;
  const int dy0 = a.dy[0], dx0 = a.dx[0];
  // weight fragment: row n = j*32 + l32, logical half lh
  const int wlane = l32 * 32 + ((lh ^ ((l32 >> 3) & 1)) << 4) + wc * 96 * 32;
  float* ct = (float*)((char*)cts + wave * G16_SLOT);
  int* rowpix = rowpix_all + wave * 32;

  auto load_tile = [&](int t, u32x4(&xf)[KST]) __attribute__((always_inline)) {
    const int m = t * 32 + l32;
    if constexpr (KT == 1) {
      unsigned vo = 0x80000000u;   // past the map: out-of-range offsets read zeros
      if (m < p.M) {
        const int b = m / mij, rem = m - b * mij;
        const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
        const int iy = i * a.isy + dy0, ix = j * a.isx + dx0;
        vo = (unsigned)((((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + lh * 8) * 2);
      }
      // a ragged channel count (ci = 8 for the tap-mode first convs): the half past ci reads zeros, not
      // the next pixel's channels (the KT > 1 path guards the same way)
      const bool ragged = (a.ci & 15) != 0;
#pragma unroll
      for (int kk = 0; kk < KST; ++kk)
        xf[kk] = __builtin_amdgcn_raw_buffer_load_b128(
            xrs, ragged && kk * 16 + lh * 8 >= a.ci ? 0x80000000u : vo, kk * 32, 0);
    } else {
      int b = 0, iy0 = -(1 << 20), ix0 = 0;   // past the map: every tap out of the image
      if (m < p.M && lh * 8 < a.ci) {
        b = m / mij;
        const int rem = m - b * mij;
        const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
        iy0 = i * a.isy;
        ix0 = j * a.isx;
      }
#pragma unroll
      for (int kk = 0; kk < KST; ++kk) {
        const int iy = iy0 + a.dy[kk], ix = ix0 + a.dx[kk];
        const bool ok = (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
        const unsigned vo = ok ? (unsigned)((((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + lh * 8) * 2) : 0x80000000u;
        xf[kk] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, 0, 0);
      }
    }
  };

  // each wave walks its own tiles with one register set: the next tile's loads are issued as soon as
  // the MFMAs have consumed this tile's fragments, and land while the epilogue runs
  const int stride = p.wgs * NSTREAM;
  int t = __builtin_amdgcn_readfirstlane(rank * NSTREAM + wst);   // uniform: a scalar loop
  u32x4 xc[KST];
  if (t < p.ntiles) load_tile(t, xc);
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  // x^2 of 8 16-bit values, rounded once (the exact product rounded to T): fp16 by packed-f16 multiplies
  // (v_pk_mul_f16, 4 per fragment instead of 8 x convert / multiply / convert -- the VALU, not the
  // MFMA, bounded the GDN launches)
  auto square = [&](u32x4 v) __attribute__((always_inline)) -> u32x4 {
    if constexpr (std::is_same<T, half_t>::value) {
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
      h8 hv = __builtin_bit_cast(h8, v);
      hv = hv * hv;
      v = __builtin_bit_cast(u32x4, hv);
    } else {
      T* e = (T*)&v;
#pragma unroll
      for (int z = 0; z < 8; ++z) {
        const float f = to_f(e[z]);
        e[z] = from_f<T>(f * f);
      }
    }
    return v;
  };
  while (t < p.ntiles) {
    if constexpr (PRO == LIC_PRO_SQUARE && FAST != 2) {
#pragma unroll
      for (int kk = 0; kk < KST; ++kk) xc[kk] = square(xc[kk]);
    }
    floatx16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    // an opaque per-tile copy of the fragment base: the weight reads are loop-invariant, and
    // hoisting all KST*TN of them out of the tile loop would not fit the registers
    int wl = wlane;
    asm volatile("" : "+v"(wl));
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) {
      u32x4 xv = xc[kk];
      if constexpr (PRO == LIC_PRO_SQUARE && FAST == 2) xv = square(xv);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const u32x4 wf = *(const u32x4*)(smem + wl + (kk * BN + j * 32) * 32);
        acc[j] = mfma_k16<T>(wf, xv, acc[j]);
      }
    }
    const int tn = __builtin_amdgcn_readfirstlane(t + stride);
    const int m = t * 32 + l32;
    // register epilogue: its operands are fetched BEFORE the next tile's loads are issued (loads retire
    // in order: issued after them, waiting for an operand would wait for the whole next tile too)
    u32x2 og[TN][4], o1[TN][4];
    int64_t pix = 0;
    const bool pok = m < p.M;
    const int nw = n0 + wc * 96;
    const T* __restrict__ gg = (const T*)a.g;
    const T* __restrict__ r1g = (const T*)a.r1;
    if constexpr (FAST != 0) {
      if (pok) {
        const int b = m / mij, rem = m - b * mij;
        const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
        pix = ((int64_t)b * a.ho + a.oy0 + a.osy * i) * a.wo + a.ox0 + a.osx * j;
      }
      if constexpr (FAST == 2) {
        // g at channel n = nw + 32j + 8k + 4lh + e: K step n / 16 = KB + 2j + k/2, fragment half k & 1,
        // elements 4lh .. 4lh+3 of that half -- in this lane (half lh) or in its partner lane ^ 32
        auto gx = [&](auto kbc) __attribute__((always_inline)) {
          constexpr int KB = decltype(kbc)::value;
          const int partner = (lane ^ 32) << 2;
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const u32x4 x = xc[KB + 2 * j + h2];
              const unsigned own0 = lh ? x[2] : x[0], own1 = lh ? x[3] : x[1];
              const unsigned rc0 = (unsigned)__builtin_amdgcn_ds_bpermute(partner, (int)(lh ? x[0] : x[2]));
              const unsigned rc1 = (unsigned)__builtin_amdgcn_ds_bpermute(partner, (int)(lh ? x[1] : x[3]));
              const u32x2 own = {own0, own1}, rcv = {rc0, rc1};
              og[j][2 * h2] = lh ? rcv : own;       // half 0
              og[j][2 * h2 + 1] = lh ? own : rcv;   // half 1
            }
        };
        if constexpr (WS == 2) {
          if (wc == 0) gx(std::integral_constant<int, 0>{});
          else gx(std::integral_constant<int, 6>{});
        } else {
          gx(std::integral_constant<int, 0>{});
        }
      } else if (gg) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) og[j][k] = *(const u32x2*)(gg + pix * a.ldg + nw + j * 32 + 8 * k + 4 * lh);
      }
      if (r1g) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) o1[j][k] = *(const u32x2*)(r1g + pix * a.ldr1 + nw + j * 32 + 8 * k + 4 * lh);
      }
    }
    if (tn < p.ntiles) load_tile(tn, xc);
    if constexpr (FAST != 0) {
      // Register epilogue: bias, activation, GDN and residual on the accumulators as they stand (lane =
      // pixel, 4-channel runs), rounded, staged as 16-bit [pixel][96 channels] rows (208-B pitch) in the
      // wave's slot, stored as 16 B of consecutive channels per lane (six 1-KB stores per tile).
      // ~40 instructions per 32 x 32 tile against ~250 for lic_common.h's epilogue_run.
      char* stg = (char*)ct;
      const int epi = a.epi, act = a.act;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const floatx4 bv = *(const floatx4*)(sbias + wc * 96 + j * 32 + 8 * k + 4 * lh);
          float w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = acc[j][4 * k + e] + bv[e];
          if (FAST == 2 || gg) {
            // GDN / IGDN: g / sqrt(n), g * rsqrt(n) -> g * rsq(n); g * sqrt(n) -> g * n * rsq(n).  v_rsq_f32
            // (~1 ulp of fp32) instead of the IEEE sqrt + division sequences (~20 instructions an element):
            // the result is rounded to the 16-bit type (2^-11 / 2^-8) right after
            const T* ge = (const T*)&og[j][k];
            const bool sq = epi == LIC_EPI_GDN_SQRT;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float rs = __builtin_amdgcn_rsqf(w[e]);
              w[e] = to_f(ge[e]) * (sq ? w[e] * rs : rs);
            }
          } else if (act == LIC_ACT_GELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = gelu_f(w[e]);
          } else if (act == LIC_ACT_LRELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : w[e] * a.slope;
          } else if (act == LIC_ACT_RELU) {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : 0.f;
          }
          if (r1g) {
            const T* re = (const T*)&o1[j][k];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] += to_f(re[e]);
          }
          u32x2 raw;
          T* o = (T*)&raw;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = from_f<T>(w[e]);
          *(u32x2*)(stg + l32 * 208 + (j * 32 + 8 * k + 4 * lh) * 2) = raw;
        }
      }
      // destination of the tile's pixels, then the rows out as 16-B chunks (12 per pixel)
      if (lh == 0) ((int64_t*)(stg + 32 * 208))[l32] = pok ? pix : -1;
      wave_lds_sync();
      T* __restrict__ yg = (T*)a.y;
      T* __restrict__ y2g = (T*)a.y2;
#pragma unroll
      for (int h = 0; h < 6; ++h) {
        const int idx = lane + 64 * h, pr = idx / 12, c = idx - pr * 12;
        const u32x4 val = *(const u32x4*)(stg + pr * 208 + c * 16);
        const int64_t dp = ((const int64_t*)(stg + 32 * 208))[pr];
        if (dp >= 0) {
          *(u32x4*)(yg + dp * a.ldy + nw + c * 8) = val;
          if (y2g) *(u32x4*)(y2g + dp * a.ldy2 + nw + c * 8) = val;
        }
      }
      wave_lds_sync();
    } else {
      // destination pixels of the tile's 32 rows (wave-private; the previous tile's epilogue has
      // finished reading them: LDS requests of a wave complete in order)
      if (lh == 0) {
        int base = -1;
        if (m < p.M) {
          const int b = m / mij, rem = m - b * mij;
          const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
          int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
          if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
          base = (b * a.ho + oy) * a.wo + ox;
        }
        rowpix[l32] = base;
      }
      wave_lds_sync();
      // epilogue (lic_common.h): stage each 32x32 tile as [pixel][channel] in the wave's slot, finish
      // it with 16-B stores of consecutive channels, tile by tile
      auto stage = [&](int q) {
#pragma unroll
        for (int qq = 0; qq < TN; ++qq)
          if (qq == q) {
#pragma unroll
            for (int r = 0; r < 16; ++r) ct[l32 * 33 + 8 * (r >> 2) + 4 * lh + (r & 3)] = acc[qq][r];
          }
      };
      c16_epilogue<T, TN, TN, 0, 31>(a, ct, rowpix, n0 + wc * 96, sbias + wc * 96, lane, stage);
    }
    t = tn;
  }
}


// "Wide" gemm16 (round 6): each wave owns a 32-pixel tile x all 192 channels of its block (6 accumulator
// tiles) instead of two waves sharing every pixel tile with 96 channels each, so the CU runs 8 independent
// pixel streams (not 4, each loaded twice), and the next tile's K step kk is issued as soon as this tile's
// MFMAs of step kk have read it -- a whole K loop (72 MFMAs) ahead of its use instead of one epilogue.
// The HBM-bound 1x1s were latency-bound at one tile in flight per stream (3.9 TB/s).  The
// epilogue operands (r1 loads, or GDN's g from the fragments) are fetched before the first next-tile load
// (loads retire in order).  Register epilogue only (plain / + r1 / GDN with g = x); same arithmetic per
// output element as gemm16_kernel (the same MFMA sequence over the K steps): bit-identical.
template <typename T, int KST, int PRO, int FAST>
__global__ __launch_bounds__(512, 1) void gemm16w_kernel(const lic_conv_args a, const G16Plan p) {
  constexpr int NW = 8, BN = 192, TN = 6;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  float* sbias = (float*)(smem + KST * BN * 32);
  char* slots = (char*)(sbias + BN);
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;
  const int nb = blockIdx.x % p.nblk;
  const int rank = blockIdx.x / p.nblk;
  const int n0 = nb * BN;
  {
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.wgt, (short)0, (int)p.wrec, 0x00020000);
    const int wrow = a.ntaps * a.cpad;
    const unsigned woff_lane = (unsigned)(((lane >> 1) * wrow + (((lane & 1) ^ ((lane >> 4) & 1)) * 8)) * 2);
    constexpr int NPIECE = KST * BN / 32;
    for (int P = wave; P < NPIECE; P += NW) {
      const int kk = P / (BN / 32), nq = P - kk * (BN / 32);
      c16_dma(wrs, smem + P * 1024, woff_lane, ((n0 + nq * 32) * wrow + kk * 16) * 2);
    }
    for (int n = tid; n < BN; n += NW * 64) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)p.xrec, 0x00020000);
  const int mij = a.mi * a.mj;
  const int dy0 = a.dy[0], dx0 = a.dx[0];
  const int wlane = l32 * 32 + ((lh ^ ((l32 >> 3) & 1)) << 4);
  char* stg = slots + wave * G16_SLOT;
  auto voff = [&](int t) __attribute__((always_inline)) -> unsigned {
    const int m = t * 32 + l32;
    unsigned vo = 0x80000000u;   // past the map: out-of-range offsets read zeros
    if (m < p.M) {
      const int b = m / mij, rem = m - b * mij;
      const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
      vo = (unsigned)((((int64_t)(b * a.h + i * a.isy + dy0) * a.w + j * a.isx + dx0) * a.ldx + lh * 8) * 2);
    }
    return vo;
  };
  auto square = [&](u32x4 v) __attribute__((always_inline)) -> u32x4 {
    if constexpr (std::is_same<T, half_t>::value) {
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
      h8 hv = __builtin_bit_cast(h8, v);
      hv = hv * hv;
      v = __builtin_bit_cast(u32x4, hv);
    } else {
      T* e = (T*)&v;
#pragma unroll
      for (int z = 0; z < 8; ++z) {
        const float f = to_f(e[z]);
        e[z] = from_f<T>(f * f);
      }
    }
    return v;
  };

  const int stride = p.wgs * NW;
  int t = __builtin_amdgcn_readfirstlane(rank * NW + wave);
  u32x4 xc[KST];
  if (t < p.ntiles) {
    const unsigned vo = voff(t);
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) xc[kk] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, kk * 32, 0);
  }
  const T* __restrict__ r1g = (const T*)a.r1;
  T* __restrict__ yg = (T*)a.y;
  T* __restrict__ y2g = (T*)a.y2;
  while (t < p.ntiles) {
    const int tn = __builtin_amdgcn_readfirstlane(t + stride);
    const int m = t * 32 + l32;
    const bool pok = m < p.M;
    int64_t pix = 0;
    if (pok) {
      const int b = m / mij, rem = m - b * mij;
      const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
      pix = ((int64_t)b * a.ho + a.oy0 + a.osy * i) * a.wo + a.ox0 + a.osx * j;
    }
    // the epilogue operands, before the first next-tile load
    u32x2 oo[TN][4];
    // GDN g = x at channel n = 32j + 8k + 4lh + e: K step 2j + k/2, fragment half k & 1, elements 4lh..
    auto gx = [&](int j0) __attribute__((always_inline)) {
      const int partner = (lane ^ 32) << 2;
#pragma unroll
      for (int j = j0; j < j0 + 3; ++j)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const u32x4 x = xc[2 * j + h2];
          const unsigned own0 = lh ? x[2] : x[0], own1 = lh ? x[3] : x[1];
          const unsigned rc0 = (unsigned)__builtin_amdgcn_ds_bpermute(partner, (int)(lh ? x[0] : x[2]));
          const unsigned rc1 = (unsigned)__builtin_amdgcn_ds_bpermute(partner, (int)(lh ? x[1] : x[3]));
          const u32x2 own = {own0, own1}, rcv = {rc0, rc1};
          oo[j][2 * h2] = lh ? rcv : own;
          oo[j][2 * h2 + 1] = lh ? own : rcv;
        }
    };
    if constexpr (FAST == 2) {
      // the first half's g now; the second half's after the K loop (its K steps 6..11 are re-loaded for the
      // next tile only then): 24 live registers through the loop instead of 48
      gx(0);
    } else {
      if (r1g) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) oo[j][k] = *(const u32x2*)(r1g + pix * a.ldr1 + n0 + j * 32 + 8 * k + 4 * lh);
      }
    }
    floatx16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const bool more = tn < p.ntiles;
    const unsigned vn = more ? voff(tn) : 0x80000000u;
    int wl = wlane;
    asm volatile("" : "+v"(wl));
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) {
      const u32x4 xv = PRO == LIC_PRO_SQUARE ? square(xc[kk]) : xc[kk];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const u32x4 wf = *(const u32x4*)(smem + wl + (kk * BN + j * 32) * 32);
        acc[j] = mfma_k16<T>(wf, xv, acc[j]);
      }
      if (more && (FAST != 2 || kk < KST / 2)) xc[kk] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vn, kk * 32, 0);
    }
    if constexpr (FAST == 2) {
      gx(3);
      if (more) {
#pragma unroll
        for (int kk = KST / 2; kk < KST; ++kk) xc[kk] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vn, kk * 32, 0);
      }
    }
    // register epilogue, one 96-channel half at a time through the wave's slot
    const int epi = a.epi, act = a.act;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        const int j = 3 * hh + jj;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const floatx4 bv = *(const floatx4*)(sbias + j * 32 + 8 * k + 4 * lh);
          float w[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = acc[j][4 * k + e] + bv[e];
          if constexpr (FAST == 2) {
            const T* ge = (const T*)&oo[j][k];
            const bool sq = epi == LIC_EPI_GDN_SQRT;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float rs = __builtin_amdgcn_rsqf(w[e]);
              w[e] = to_f(ge[e]) * (sq ? w[e] * rs : rs);
            }
          } else {
            if (act == LIC_ACT_GELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = gelu_f(w[e]);
            } else if (act == LIC_ACT_LRELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : w[e] * a.slope;
            } else if (act == LIC_ACT_RELU) {
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = w[e] > 0.f ? w[e] : 0.f;
            }
            if (r1g) {
              const T* re = (const T*)&oo[j][k];
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] += to_f(re[e]);
            }
          }
          u32x2 raw;
          T* o = (T*)&raw;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = from_f<T>(w[e]);
          *(u32x2*)(stg + l32 * 208 + (jj * 32 + 8 * k + 4 * lh) * 2) = raw;
        }
      }
      if (lh == 0) ((int64_t*)(stg + 32 * 208))[l32] = pok ? pix : -1;
      wave_lds_sync();
#pragma unroll
      for (int h = 0; h < 6; ++h) {
        const int idx = lane + 64 * h, pr = idx / 12, c = idx - pr * 12;
        const u32x4 val = *(const u32x4*)(stg + pr * 208 + c * 16);
        const int64_t dp = ((const int64_t*)(stg + 32 * 208))[pr];
        if (dp >= 0) {
          *(u32x4*)(yg + dp * a.ldy + n0 + 96 * hh + c * 8) = val;
          if (y2g) *(u32x4*)(y2g + dp * a.ldy2 + n0 + 96 * hh + c * 8) = val;
        }
      }
      wave_lds_sync();
    }
    t = tn;
  }
}

template <typename T, int BN, int KST, int PRO, int KT>
void launch_g16(const lic_conv_args& a, const G16Plan& p, dim3 grid, int smem, hipStream_t s, int& status) {
  auto kern = p.fast_epi == 1 ? gemm16_kernel<T, BN, KST, PRO, KT, 1> : gemm16_kernel<T, BN, KST, PRO, KT, 0>;
  if constexpr (PRO == LIC_PRO_SQUARE && KT == 1 && BN == 192 && KST == 12)
    if (p.fast_epi == 2) kern = gemm16_kernel<T, BN, KST, PRO, KT, 2>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, smem);
  if (ea != hipSuccess) {
    status = fail(std::string("gemm16: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return;
  }
  hipLaunchKernelGGL(kern, grid, dim3(512), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("gemm16 launch: ") + hipGetErrorString(e));
}

// The register epilogue: PLAIN (any of none / relu / lrelu / gelu) or GDN_DIV / _RSQRT / _SQRT, optional
// r1, no r2; 16-B aligned outputs, 8-B aligned operands, whole 96-channel blocks, no pixel shuffle.
inline bool g16_fast_epi_ok(const lic_conv_args& a) {
  const bool gdn = a.epi == LIC_EPI_GDN_DIV || a.epi == LIC_EPI_GDN_RSQRT || a.epi == LIC_EPI_GDN_SQRT;
  auto al16 = [](const void* ptr, int ld) { return ptr == nullptr || (((uintptr_t)ptr & 15) == 0 && ld % 8 == 0); };
  auto al8 = [](const void* ptr, int ld) { return ptr == nullptr || (((uintptr_t)ptr & 7) == 0 && ld % 4 == 0); };
  return (a.epi == LIC_EPI_PLAIN || gdn) && (gdn == (a.g != nullptr)) && a.out_shuffle == 0 && a.co == a.copad &&
         a.act != LIC_ACT_ROUND && !(gdn && a.act != LIC_ACT_NONE) && al16(a.y, a.ldy) && al16(a.y2, a.ldy2) &&
         al8(a.r1, a.ldr1) && al8(a.g, a.ldg);
}

// FAST 2: a GDN (x^2 prologue) whose g is the layer input itself at the output pixel and channel --
// identity pixel map, Cin = Cout = 192 in one channel block -- so g is in the tile's fragments.
inline bool g16_gx_ok(const lic_conv_args& a) {
  return a.prologue == LIC_PRO_SQUARE && a.g == a.x && a.ldg == a.ldx && a.ci == 192 && a.cpad == 192 &&
         a.co == 192 && a.copad == 192 && a.ntaps == 1 && a.dy[0] == 0 && a.dx[0] == 0 && a.isy == 1 &&
         a.isx == 1 && a.oy0 == 0 && a.ox0 == 0 && a.osy == 1 && a.osx == 1 && a.ho == a.h && a.wo == a.w &&
         a.mi == a.h && a.mj == a.w;
}

// Returns 1 and launches when the gemm16 kernel applies; 0 to let the caller fall back.
template <typename T, int BN, int KST, int KT = 1>
int try_gemm16(const lic_conv_args& a, hipStream_t s, int& status) {
  // LIC_TRACE=1: name the condition that declines the launch (stderr)
#define G16_DECLINE(cond)                                                                     \
  if (cond) {                                                                                 \
    if (wd_env("LIC_TRACE", 0)) fprintf(stderr, "gemm16<%d,%d,%d> declines: %s\n", BN, KST, KT, #cond); \
    return 0;                                                                                 \
  }
  G16_DECLINE(a.ntaps != KT || a.copad % BN || a.out_shuffle != 0 || a.groups != 1)
  G16_DECLINE((a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE) || !c16_epi_supported(a))
  G16_DECLINE(a.ldx % 8 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt % 16))
  G16_DECLINE(KT == 1 && KST > 1 && (a.cpad != KST * 16 || a.ci != a.cpad))
  // one 16-channel chunk per tap: Cin 8 (channels 8..15 read as zeros) or 16 (a 16-channel view)
  G16_DECLINE((KT > 1 || KST == 1) && !(a.ci == 8 || (a.ci == 16 && a.ldx >= 16)))
  G16_DECLINE(KT > 1 && (KST != KT || a.prologue != LIC_PRO_NONE))
  const int64_t xbytes = ((int64_t)a.n * a.h * a.w - 1) * a.ldx * 2 + (int64_t)a.ci * 2;
  const int64_t M = (int64_t)a.n * a.mi * a.mj;
  G16_DECLINE(xbytes >= (1LL << 31) || M >= (1LL << 31) || (int64_t)a.n * a.ho * a.wo >= (1LL << 31))
#undef G16_DECLINE
  G16Plan p;
  p.M = (int)M;
  p.ntiles = (int)((M + 31) / 32);
  p.nblk = a.copad / BN;
  int wgs = 256 / p.nblk;   // one 8-wave workgroup per CU in all
  if (wgs < 1) wgs = 1;
  const int need = (p.ntiles + 8 / (BN / 96) - 1) / (8 / (BN / 96));
  if (wgs > need) wgs = need;
  p.wgs = wgs;
  p.xrec = (unsigned)xbytes;
  p.wrec = (unsigned)((int64_t)a.copad * a.ntaps * a.cpad * 2);
  const int smem = KST * BN * 32 + BN * 4 + 8 * G16_SLOT + 8 * 32 * 4;
  p.fast_epi = g16_fast_epi_ok(a) && wd_env("LIC_G16_FAST_EPI", 1) ? 1 : 0;
  if (p.fast_epi && g16_gx_ok(a) && wd_env("LIC_G16_GX", 1)) p.fast_epi = 2;
  dim3 grid((unsigned)(wgs * p.nblk));
  // the wide variant (gemm16w_kernel): 192-channel blocks of a 1x1, register epilogue with at most one
  // operand set (r1, or GDN's g = x); LIC_G16_WIDE=0 restores the two-waves-per-tile kernel (A/B)
  if constexpr (KT == 1 && BN == 192 && (KST == 12 || KST == 6)) {
    static const int wide_on = wd_env("LIC_G16_WIDE", 1);
    const bool gdn = a.g != nullptr;
    if (wide_on && ((p.fast_epi == 1 && !gdn) || (p.fast_epi == 2 && a.r1 == nullptr))) {
      int wg2 = 256 / p.nblk;
      if (wg2 < 1) wg2 = 1;
      const int need2 = (p.ntiles + 7) / 8;
      if (wg2 > need2) wg2 = need2;
      p.wgs = wg2;
      const int smem2 = KST * BN * 32 + BN * 4 + 8 * G16_SLOT;
      const dim3 grid2((unsigned)(wg2 * p.nblk));
      auto kern = p.fast_epi == 2 ? (a.prologue == LIC_PRO_SQUARE ? gemm16w_kernel<T, KST, LIC_PRO_SQUARE, 2>
                                                                  : gemm16w_kernel<T, KST, LIC_PRO_NONE, 2>)
                                  : (a.prologue == LIC_PRO_SQUARE ? gemm16w_kernel<T, KST, LIC_PRO_SQUARE, 1>
                                                                  : gemm16w_kernel<T, KST, LIC_PRO_NONE, 1>);
      const hipError_t ea = ensure_dyn_lds((const void*)kern, smem2);
      if (ea != hipSuccess) {
        status = fail(std::string("gemm16w: dynamic LDS attribute: ") + hipGetErrorString(ea));
        return 1;
      }
      hipLaunchKernelGGL(kern, grid2, dim3(512), smem2, s, a, p);
      hipError_t e = hipGetLastError();
      status = e == hipSuccess ? 0 : fail(std::string("gemm16w launch: ") + hipGetErrorString(e));
      return 1;
    }
  }
  if constexpr (KT > 1) launch_g16<T, BN, KST, LIC_PRO_NONE, KT>(a, p, grid, smem, s, status);
  else if (a.prologue == LIC_PRO_SQUARE) launch_g16<T, BN, KST, LIC_PRO_SQUARE, 1>(a, p, grid, smem, s, status);
  else launch_g16<T, BN, KST, LIC_PRO_NONE, 1>(a, p, grid, smem, s, status);
  return 1;
}

// Tile choice of the gemm16 kernel: 16-bit 1x1 convolutions with K in {96, 192} (or Cin 8 / 16) on
// maps of >= 4 K output pixels, and 3x3 convolutions of Cin 8 / 16 (the image's first layer).
// LIC_GEMM16=0 restores the previous kernels (A/B).
template <typename T>
int gemm16_dispatch_impl(const lic_conv_args& a, hipStream_t s, int& status) {
  static const int on = wd_env("LIC_GEMM16", 1);
  if (wd_env("LIC_TRACE", 0))
    fprintf(stderr, "gemm16 dispatch: n %d mi %d mj %d ci %d cpad %d co %d copad %d ntaps %d pro %d epi %d act %d\n", a.n,
            a.mi, a.mj, a.ci, a.cpad, a.co, a.copad, a.ntaps, a.prologue, a.epi, a.act);
  if (!on || a.force_mfma_generic || a.force_direct) return 0;
  if ((int64_t)a.n * a.mi * a.mj < 4096) return 0;
  if (a.ci <= 16) {   // the image's k x k layers and their 1x1 skips (one chunk per tap)
    if (a.copad % 192 != 0) return 0;
    if (a.ntaps == 9) return try_gemm16<T, 192, 9, 9>(a, s, status);
    if (a.ntaps == 1) return try_gemm16<T, 192, 1, 1>(a, s, status);
    return 0;
  }
  if (a.ntaps != 1) return 0;
  if (a.cpad == 192) {
    if (a.copad % 192 == 0) return try_gemm16<T, 192, 12>(a, s, status);
    if (a.copad % 96 == 0) return try_gemm16<T, 96, 12>(a, s, status);
  }
  if (a.cpad == 96) {
    if (a.copad % 192 == 0) return try_gemm16<T, 192, 6>(a, s, status);
    if (a.copad % 96 == 0) return try_gemm16<T, 96, 6>(a, s, status);
  }
  return 0;
}

}  // namespace lic
