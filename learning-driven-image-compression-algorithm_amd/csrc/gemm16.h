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
#include "conv16.h"

namespace lic {


struct G16Plan {
  int M;          // output lattice pixels (n * mi * mj)
  int ntiles;     // ceil(M / 32)
  int nblk;       // output-channel blocks (copad / BN)
  int wgs;        // workgroups per channel block
  unsigned xrec;  // bytes addressable from a.x
  unsigned wrec;  // bytes of the packed weights
};

template <typename T, int BN, int KST, int PRO>
__global__ __launch_bounds__(512, 1) void gemm16_kernel(const lic_conv_args a, const G16Plan p) {
  // a wave computes 32 pixels x 96 channels (3 accumulator tiles); at BN = 192 two waves share each
  // pixel tile (its fragments are loaded twice, from L2 the second time)
  constexpr int NW = 8, WS = BN / 96, TN = 3, NSTREAM = NW / WS;
  static_assert(BN == 96 || BN == 192, "BN");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  float* sbias = (float*)(smem + KST * BN * 32);
  float* cts = sbias + BN;                 // NW epilogue slots of 32 x 33 fp32
  int* rowpix_all = (int*)(cts + NW * 32 * 33);   // NW x 32 destination pixels

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
    const unsigned woff_lane = (unsigned)(((lane >> 1) * a.cpad + (((lane & 1) ^ ((lane >> 4) & 1)) * 8)) * 2);
    constexpr int NPIECE = KST * BN / 32;
    for (int P = wave; P < NPIECE; P += NW) {
      const int kk = P / (BN / 32), nq = P - kk * (BN / 32);
      c16_dma(wrs, smem + P * 1024, woff_lane, ((n0 + nq * 32) * a.cpad + kk * 16) * 2);
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
  float* ct = cts + wave * 32 * 33;
  int* rowpix = rowpix_all + wave * 32;

  auto load_tile = [&](int t, u32x4(&xf)[KST]) __attribute__((always_inline)) {
    const int m = t * 32 + l32;
    unsigned vo = 0x80000000u;   // past the map: out-of-range offsets read zeros
    if (m < p.M) {
      const int b = m / mij, rem = m - b * mij;
      const int i = rem / a.mj, j = rem - (rem / a.mj) * a.mj;
      const int iy = i * a.isy + dy0, ix = j * a.isx + dx0;
      vo = (unsigned)((((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + lh * 8) * 2);
    }
#pragma unroll
    for (int kk = 0; kk < KST; ++kk) xf[kk] = __builtin_amdgcn_raw_buffer_load_b128(xrs, vo, kk * 32, 0);
  };

  // each wave walks its own tiles with one register set: the next tile's loads are issued as soon as
  // the MFMAs have consumed this tile's fragments, and land while the epilogue runs
  const int stride = p.wgs * NSTREAM;
  int t = __builtin_amdgcn_readfirstlane(rank * NSTREAM + wst);   // uniform: a scalar loop
  u32x4 xc[KST];
  if (t < p.ntiles) load_tile(t, xc);
  while (t < p.ntiles) {
    if constexpr (PRO == LIC_PRO_SQUARE) {
#pragma unroll
      for (int kk = 0; kk < KST; ++kk) {
        T* e = (T*)&xc[kk];
#pragma unroll
        for (int z = 0; z < 8; ++z) {
          const float f = to_f(e[z]);
          e[z] = from_f<T>(f * f);
        }
      }
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
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const u32x4 wf = *(const u32x4*)(smem + wl + (kk * BN + j * 32) * 32);
        acc[j] = mfma_k16<T>(wf, xc[kk], acc[j]);
      }
    }
    const int tn = __builtin_amdgcn_readfirstlane(t + stride);
    if (tn < p.ntiles) load_tile(tn, xc);
    // destination pixels of the tile's 32 rows (wave-private; the previous tile's epilogue has
    // finished reading them: LDS requests of a wave complete in order)
    if (lh == 0) {
      const int m = t * 32 + l32;
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
    // epilogue (lic_common.h): stage each 32x32 tile as [pixel][channel] in the wave's slot, finish it
    // with 16-B stores of consecutive channels
    // one wave-private slot, tile by tile (stage(q) writes tile q as [pixel][channel])
    auto stage = [&](int q) {
#pragma unroll
      for (int qq = 0; qq < TN; ++qq)
        if (qq == q) {
#pragma unroll
          for (int r = 0; r < 16; ++r) ct[l32 * 33 + 8 * (r >> 2) + 4 * lh + (r & 3)] = acc[qq][r];
        }
    };
    c16_epilogue<T, TN, TN, 0>(a, ct, rowpix, n0 + wc * 96, sbias + wc * 96, lane, stage);
    t = tn;
  }
}

template <typename T, int BN, int KST, int PRO>
void launch_g16(const lic_conv_args& a, const G16Plan& p, dim3 grid, int smem, hipStream_t s, int& status) {
  const hipError_t ea = ensure_dyn_lds((const void*)gemm16_kernel<T, BN, KST, PRO>, smem);
  if (ea != hipSuccess) {
    status = fail(std::string("gemm16: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return;
  }
  hipLaunchKernelGGL((gemm16_kernel<T, BN, KST, PRO>), grid, dim3(512), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("gemm16 launch: ") + hipGetErrorString(e));
}

// Returns 1 and launches when the gemm16 kernel applies; 0 to let the caller fall back.
template <typename T, int BN, int KST>
int try_gemm16(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.ntaps != 1 || a.copad % BN || a.out_shuffle != 0 || a.groups != 1) return 0;
  if ((a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE) || !c16_epi_supported(a)) return 0;
  if (a.cpad != KST * 16 || a.ci != a.cpad || a.ldx % 8 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt % 16)) return 0;
  const int64_t xbytes = ((int64_t)a.n * a.h * a.w - 1) * a.ldx * 2 + (int64_t)a.ci * 2;
  const int64_t M = (int64_t)a.n * a.mi * a.mj;
  if (xbytes >= (1LL << 31) || M >= (1LL << 31) || (int64_t)a.n * a.ho * a.wo >= (1LL << 31)) return 0;
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
  p.wrec = (unsigned)((int64_t)a.copad * a.cpad * 2);
  const int smem = KST * BN * 32 + BN * 4 + 8 * 32 * 33 * 4 + 8 * 32 * 4;
  dim3 grid((unsigned)(wgs * p.nblk));
  if (a.prologue == LIC_PRO_SQUARE) launch_g16<T, BN, KST, LIC_PRO_SQUARE>(a, p, grid, smem, s, status);
  else launch_g16<T, BN, KST, LIC_PRO_NONE>(a, p, grid, smem, s, status);
  return 1;
}

// Tile choice of the gemm16 kernel: 16-bit 1x1 convolutions with K in {96, 192} on maps of
// >= 16 K output pixels.  LIC_GEMM16=0 restores the previous kernels (A/B).
template <typename T>
int gemm16_dispatch_impl(const lic_conv_args& a, hipStream_t s, int& status) {
  static const int on = wd_env("LIC_GEMM16", 1);
  if (!on || a.force_mfma_generic || a.force_direct || a.ntaps != 1) return 0;
  if ((int64_t)a.n * a.mi * a.mj < 16384) return 0;
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
