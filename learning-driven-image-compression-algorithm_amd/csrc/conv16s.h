// 16-bit (fp16 / bf16) k x k stride-1 convolution on SMALL maps, round 5 ("conv16s"): the 16 x 16
// latents of the a_model's Win_noShift_Attention (13 3x3 192 -> 192 per image and a 7x7) and of
// the slice loop, where conv16's 16 x 32-pixel tiles leave most of the chip idle (32 images x one
// tile) and the halo kernel's 8 x 8 tiles re-stage the weights through LDS behind a barrier per stage.
//
// One workgroup = 4 waves (one per SIMD) = a 4 x 16-pixel tile (two 32-pixel B fragments, each two
// tile rows) x BN = 32 CT output channels.  The reduction is split across the waves by input
// chunk (wave w takes the 16-channel chunks w, w+4, ...; all taps of each): every wave runs the
// whole pixel x channel tile on its own accumulators, so the launch has 4x the independent MFMA
// chains of a pixel-split tile and the weights are read once per workgroup.
//   * The tile's whole input halo, every chunk, is moved by LDS-DMA (buffer_load ... lds) up front:
//     chunk planes [HH x HWD px][32 B], 16-B halves XOR-swizzled by bit 3 of the halo column (as in
//     conv16: conflict-free fragment reads at every tap shift; a fragment address is a per-lane base
//     per tap column + compile-time immediates); out-of-image pixels are out-of-range offsets (zeros).
//   * Weights never touch LDS: the transposed GEMM's A fragments (32 output channels x 16 input
//     channels, 16 B a lane) are raw buffer loads from the packed [co][tap][cpad] weights (L2-resident:
//     every workgroup of a channel block reads the same bytes) into a ring of R register slots,
//     PD = R - 1 steps ahead of the MFMAs that use them.
//   * End: the 4 partial tiles meet in LDS (fixed summation order), each wave finishes CT*2/4 of the
//     32 x 32 tiles through the shared epilogue (lic_common.h epilogue_tile; every operand variant).
// (Included by conv16.h; not a standalone header.)
#pragma once

namespace lic {

struct C16sPlan {
  int tiles_x, tiles_y;
  int dymin, dxmin;
  int nchunks;        // cpad / 16
  int npieces;        // 1-KB LDS-DMA pieces of the halo (every chunk plane)
  int main_bytes;     // LDS before bias + destination pixels: max(halo, partial tiles)
  unsigned xrec, wrec;
  int frag;           // weights from a.wgt_split in MFMA-fragment order (conv16.h c16_frag_ok)
  int ws_co, ws_k, ws_tap, wl_row, wl_half;   // weight source strides (conv16.h c16_wstrides)
};

template <typename T, int MASK>
__device__ __forceinline__ void c16s_tile(const lic_conv_args& a, const float* ct, const int* rowpix, int n0, int lane,
                                          const float* sbias) {
  EpiOperands<T> o;
  epi_prefetch<T, MASK>(a, rowpix, n0, lane, o);
  epilogue_tile<T, MASK>(a, ct, rowpix, n0, lane, sbias, o);
}

// one staged 32 x 32 tile through the epilogue variant of the launch (uniform dispatch)
template <typename T>
__device__ __forceinline__ void c16s_finish(const lic_conv_args& a, const float* ct, const int* rowpix, int n0, int lane,
                                            const float* sbias) {
  if (!epi_vec_ok<T>(a)) {
    epilogue_tile_scalar<T>(a, ct, rowpix, n0, lane);
    return;
  }
  switch (epi_mask(a)) {
    case 0: c16s_tile<T, 0>(a, ct, rowpix, n0, lane, sbias); break;
    case EPI_R1: c16s_tile<T, EPI_R1>(a, ct, rowpix, n0, lane, sbias); break;
    case EPI_G: c16s_tile<T, EPI_G>(a, ct, rowpix, n0, lane, sbias); break;
    case EPI_G | EPI_R1: c16s_tile<T, EPI_G | EPI_R1>(a, ct, rowpix, n0, lane, sbias); break;
    case EPI_R2: c16s_tile<T, EPI_R2>(a, ct, rowpix, n0, lane, sbias); break;
    case EPI_G | EPI_R2: c16s_tile<T, EPI_G | EPI_R2>(a, ct, rowpix, n0, lane, sbias); break;
    default: c16s_tile<T, EPI_G | EPI_R1 | EPI_R2>(a, ct, rowpix, n0, lane, sbias); break;
  }
}

template <int KH, int KW, int CT>
struct C16sGeo {
  static constexpr int TH = 4, TW = 16, NW = 4, NT = NW * 64;
  static constexpr int BN = 32 * CT;
  static constexpr int NTAPS = KH * KW;
  static constexpr int HH = TH + KH - 1, HWD = TW + KW - 1, HPIX = HH * HWD;
  static constexpr int PLANE = HPIX * 32;           // one 16-channel chunk of the halo
  static constexpr int NQ = 2 * CT;                 // accumulator tiles per wave
  static constexpr int TILE = 32 * 33;              // staged fp32 tile (row stride 33)
  static constexpr int RED = NW * NQ * TILE * 4;    // the waves' partial tiles
  // weight ring: R slots (R divides the tap count, so a chunk starts at slot 0), prefetch distance R - 1:
  // (a 9-deep ring for 3x3 -- a whole chunk ahead -- was slower: 19.0 -> 22.9 us at 16x16, r05n)
  // (1x1: a 4-slot ring over the wave's chunks, the chunk loop unrolled by 4 so every slot is static)
  static constexpr int R = NTAPS == 1 ? 4 : (NTAPS % 7 == 0 ? 7 : (NTAPS % 4 == 0 ? 4 : (NTAPS % 3 == 0 ? 3 : 1)));
  static constexpr int PD = R - 1;
  static_assert(R > 1, "tap count");
};

template <typename T, int KH, int KW, int CT>
__global__ __launch_bounds__(256, 1) void conv16s_kernel(const lic_conv_args a, const C16sPlan p) {
  using Geo = C16sGeo<KH, KW, CT>;
  constexpr int NW = Geo::NW, TW = Geo::TW, TH = Geo::TH, HWD = Geo::HWD, HPIX = Geo::HPIX, PLANE = Geo::PLANE;
  constexpr int NTAPS = Geo::NTAPS, NQ = Geo::NQ, TILE = Geo::TILE, BN = Geo::BN, R = Geo::R, PD = Geo::PD;

  extern __shared__ __attribute__((aligned(1024))) char smem[];
  float* sbias = (float*)(smem + p.main_bytes);
  int* rowpix = (int*)(sbias + BN);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, lh = lane >> 5;

  int bid = blockIdx.x;
  const int tx_t = bid % p.tiles_x;
  bid /= p.tiles_x;
  const int ty_t = bid % p.tiles_y;
  const int b = bid / p.tiles_y;
  const int n0 = blockIdx.y * BN;
  const int i0 = ty_t * TH, j0 = tx_t * TW;
  const int iy0 = i0 + p.dymin, ix0 = j0 + p.dxmin;

  for (int n = tid; n < BN; n += Geo::NT) sbias[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
  for (int m = tid; m < TH * TW; m += Geo::NT) {
    const int i = i0 + m / TW, j = j0 + m % TW;
    int base = -1;
    if (i < a.mi && j < a.mj) {
      int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
      if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
      base = (b * a.ho + oy) * a.wo + ox;
    }
    rowpix[m] = base;
  }

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)p.xrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.frag ? a.wgt_split : a.wgt), (short)0, (int)p.wrec, 0x00020000);

  // ---- the whole halo by LDS-DMA: 16-B slot q = chunk q / (2 HPIX), halo pixel (q / 2) % HPIX, stored
  // half q & 1 = channel half (q & 1) ^ bit3(column) ----
  const int nslots = p.nchunks * HPIX * 2;
  for (int P = wave; P < p.npieces; P += NW) {
    const int q = P * 64 + lane;
    const int kc = q / (2 * HPIX), rem = q - kc * (2 * HPIX);
    const int hp = rem >> 1, r = hp / HWD, cc = hp - r * HWD;
    const int c = (rem & 1) ^ ((cc >> 3) & 1);
    const int iy = iy0 + r, ix = ix0 + cc;
    const bool ok = q < nslots && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    const unsigned off = ok ? (unsigned)((((int64_t)(b * a.h + iy) * a.w + ix) * a.ldx + kc * 16 + c * 8) * 2) : 0x80000000u;
    c16_dma(xrs, smem + P * 1024, off, 0);
  }

  // ---- weights: A fragment (tap t, chunk kc, channel tile i) = rows n0 + 32 i + l32, channels
  // 16 kc + 8 lh .. +7 (16 B): per-lane offset + scalar offset ----
  const unsigned wl = (unsigned)(l32 * p.wl_row + lh * p.wl_half);
  const int nchunks = p.nchunks;
  const int ncw = (nchunks - wave + NW - 1) / NW;   // this wave's chunks: wave, wave + NW, ...
  // the chunk order is rotated by the workgroup (a bijection of the chunks): the workgroups sharing an
  // L2 would otherwise read the same weight lines at the same moment
  const int rot = (int)(blockIdx.x % (unsigned)nchunks);
  auto chunk_of = [&](int cidx) __attribute__((always_inline)) {
    int kc = wave + NW * cidx;
    kc = kc < nchunks ? kc : nchunks - 1;   // past the wave's last chunk: a harmless re-read
    kc += rot;
    return kc < nchunks ? kc : kc - nchunks;
  };
  auto load_w = [&](int cidx, int t, u32x4(&f)[CT]) __attribute__((always_inline)) {
    const int kc = chunk_of(cidx);
#pragma unroll
    for (int i = 0; i < CT; ++i)
      f[i] = __builtin_amdgcn_raw_buffer_load_b128(wrs, wl, ((n0 >> 5) + i) * p.ws_co + t * p.ws_tap + kc * p.ws_k, 0);
  };

  // ---- B fragments: pixel l32 of fragment j = tile row 2j + (l32 >> 4), column l32 & 15 ----
  int hlane[KW];
#pragma unroll
  for (int dx = 0; dx < KW; ++dx) {
    const int col = (l32 & 15) + dx;
    hlane[dx] = ((l32 >> 4) * HWD + col) * 32 + ((lh ^ ((col >> 3) & 1)) << 4);
  }

  floatx16 acc[CT][2];
#pragma unroll
  for (int i = 0; i < CT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  u32x4 fw[R][CT];
#pragma unroll
  for (int q = 0; q < PD; ++q) {   // the first PD steps: taps of chunk 0 (1x1: chunks 0 .. PD-1)
    if constexpr (NTAPS == 1) load_w(q, 0, fw[q]);
    else load_w(0, q, fw[q]);
  }

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the halo; the first weights too)
  __syncthreads();

  if constexpr (NTAPS == 1) {
    // 1x1 (the slice loop's / hyper nets' Linears on 16x16 latents): one MFMA pair per chunk, the
    // weights of chunk + PD in flight
    for (int c0 = 0; c0 < ncw; c0 += R) {
      c16_static_for<0, R>([&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        const int cidx = c0 + u;
        if (cidx < ncw) {
          load_w(cidx + PD, 0, fw[(u + PD) % R]);
          const int hb0 = hlane[0] + chunk_of(cidx) * PLANE;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const u32x4 fbj = *(const u32x4*)(smem + hb0 + 2 * j * HWD * 32);
#pragma unroll
            for (int i = 0; i < CT; ++i) acc[i][j] = mfma_k16<T>(fw[u][i], fbj, acc[i][j]);
          }
        }
      });
    }
  } else
  for (int cidx = 0; cidx < ncw; ++cidx) {
    const int kc = chunk_of(cidx);
    int hb[KW];
#pragma unroll
    for (int dx = 0; dx < KW; ++dx) hb[dx] = hlane[dx] + kc * PLANE;
    auto load_b = [&](int t, int j) __attribute__((always_inline)) -> u32x4 {
      const int dy = t / KW, dx = t - (t / KW) * KW;
      return *(const u32x4*)(smem + hb[dx] + (2 * j + dy) * HWD * 32);
    };
    u32x4 fb[2][2];
    fb[0][0] = load_b(0, 0);
    fb[0][1] = load_b(0, 1);
    c16_static_for<0, NTAPS>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      constexpr int tn = t + PD;
      load_w(cidx + tn / NTAPS, tn % NTAPS, fw[tn % R]);
      if constexpr (t + 1 < NTAPS) {
        fb[(t + 1) & 1][0] = load_b(t + 1, 0);
        fb[(t + 1) & 1][1] = load_b(t + 1, 1);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < CT; ++i) acc[i][j] = mfma_k16<T>(fw[t % R][i], fb[t & 1][j], acc[i][j]);
    });
  }

  // ---- the partial tiles meet in LDS (over the halo), [pixel][channel] rows of 33 floats ----
  __syncthreads();
  float* part = (float*)smem + wave * (NQ * TILE);
  c16_static_for<0, NQ>([&](auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value, i = q % CT, j = q / CT;
#pragma unroll
    for (int r = 0; r < 16; ++r) part[q * TILE + l32 * 33 + 8 * (r >> 2) + 4 * lh + (r & 3)] = acc[i][j][r];
  });
  __syncthreads();
  // tile q (channel tile q % CT, fragment q / CT) is summed and finished by wave q % NW
  for (int q = wave; q < NQ; q += NW) {
    float* c0 = (float*)smem + q * TILE;
    for (int e = lane; e < TILE; e += 64) {
      float s = c0[e];
#pragma unroll
      for (int v = 1; v < NW; ++v) s += c0[v * NQ * TILE + e];
      c0[e] = s;
    }
    wave_lds_sync();
    const int i = q % CT, j = q / CT;
    c16s_finish<T>(a, c0, rowpix + 32 * j, n0 + 32 * i, lane, sbias + 32 * i);
  }
}

// Returns 1 and launches when the conv16s kernel applies; 0 to let the caller fall back.
template <typename T, int KH, int KW, int CT>
int try_conv16s(const lic_conv_args& a, hipStream_t s, int& status) {
  using Geo = C16sGeo<KH, KW, CT>;
  if (a.ntaps != KH * KW || a.copad % Geo::BN || a.isy != 1 || a.isx != 1) return 0;
  if (a.prologue != LIC_PRO_NONE || a.groups != 1) return 0;
  if (a.ci != a.cpad || a.cpad % 16 || a.ldx % 8 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt % 16)) return 0;
  for (int t = 0; t < a.ntaps; ++t)
    if (a.dy[t] != a.dy[0] + t / KW || a.dx[t] != a.dx[0] + t % KW) return 0;
  const int64_t xbytes = ((int64_t)a.n * a.h * a.w - 1) * a.ldx * 2 + (int64_t)a.ci * 2;
  const int64_t wbytes = (int64_t)a.copad * a.ntaps * a.cpad * 2;
  if (xbytes >= (1LL << 31) || wbytes >= (1LL << 31) || (int64_t)a.n * a.ho * a.wo >= (1LL << 31)) return 0;
  C16sPlan p;
  p.dymin = a.dy[0];
  p.dxmin = a.dx[0];
  p.tiles_y = (a.mi + Geo::TH - 1) / Geo::TH;
  p.tiles_x = (a.mj + Geo::TW - 1) / Geo::TW;
  p.nchunks = a.cpad / 16;
  p.npieces = (p.nchunks * Geo::HPIX * 2 + 63) / 64;
  const int halo = p.npieces * 1024;
  p.main_bytes = halo > Geo::RED ? halo : Geo::RED;
  const int smem = p.main_bytes + Geo::BN * 4 + Geo::TH * Geo::TW * 4;
  if (smem > 160 * 1024) return 0;
  p.xrec = (unsigned)xbytes;
  p.wrec = (unsigned)wbytes;
  p.frag = c16_frag_ok(a) ? 1 : 0;
  c16_wstrides(a, p);
  const int64_t blocks = (int64_t)a.n * p.tiles_y * p.tiles_x;
  dim3 grid((unsigned)blocks, a.copad / Geo::BN);
  auto kern = conv16s_kernel<T, KH, KW, CT>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, smem);
  if (ea != hipSuccess) {
    status = fail(std::string("conv16s: dynamic LDS attribute: ") + hipGetErrorString(ea));
    return 1;
  }
  hipLaunchKernelGGL(kern, grid, dim3(Geo::NT), smem, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("conv16s launch: ") + hipGetErrorString(e));
  return 1;
}

}  // namespace lic
