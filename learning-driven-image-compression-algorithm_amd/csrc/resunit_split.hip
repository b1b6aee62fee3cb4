// compressai AttentionBlock ResidualUnit, fused, fp32 activations with fp32x6 split products
// (conv_split.h): out = relu(conv1x1_{N/2->N}(relu(conv3x3_{N/2}(relu(conv1x1_{N->N/2}(x))))) + x)
// (reference: compressai/layers/layers.py AttentionBlock.ResidualUnit, called 6x per SWAtten at
// /root/reference/model/net_ga.py:118-136 and per Win_noShift_Attention at layers/layers.py:87-111).
//
// Why fused.  On the 16x16 latents of the slice loop (B x 256 px) each of the three convolutions is
// a grid of ~128 workgroups whose time is mostly latency (first loads, one barrier per chunk, the
// epilogue's round trip to HBM); 48 ResidualUnits per forward were 144 launches.  Here one
// workgroup owns an 8x8 output tile of one image and keeps every intermediate in LDS:
//   x halo 10x10 px x N ch  --split-->  3 bf16 planes            (the only activation read from HBM)
//   GEMM1  t1 = relu(W1 x + b1) on all 100 halo px (zero outside the image: conv3x3's padding)
//   GEMM2  t2 = relu(W2 * t1 + b2), 9 taps read as shifted windows of the t1 planes
//   GEMM3  out = relu(W3 t2 + b3 + x)  -> HBM
// Every GEMM is computed transposed (MFMA A = weights, rows = output channels; B = activations,
// columns = pixels): a lane's accumulator then holds 4-channel runs of ONE pixel, which the
// epilogues write straight into the next GEMM's split planes (ds_write_b64 per part) or, for the
// output, as float4 stores.  The split weights are the fragment-order packs of the three convs
// (functional.split_weights, the same bytes the per-conv kernels use): the "B operand" layout of
// conv_split.h is exactly the A layout of the transposed product.
// Summation order per output: chunks of 16 input channels in order, taps in order inside a chunk,
// the six part products smallest first, odd chunks split from -x with the running sum negated at
// each chunk start (the same bias cancellation as conv_split_wd.hip).
#include "conv_split.h"

namespace lic {

namespace {

constexpr int RU_HP = 128;   // halo pixel slots (10 x 10 = 100 used)

__device__ __forceinline__ int ru_swz(int hp, int half) { return hp * 32 + ((half ^ ((hp >> 3) & 1)) << 4); }

// One split GEMM over NSTEP (chunk, tap) steps: acc[i][j] += W(step)[i] . A(step)[j], weights
// from L2 by a ring of D+1 register slots (prefetch distance D), activation fragments from LDS one
// step ahead.  wload(s, slot) / aload(s, slot) fill [MT][3] / [NTT][3] fragments; NTAP steps per
// chunk; the running sum changes sign at every chunk start (odd chunks are split from -x).
template <int NSTEP, int NTAP, int MT, int NTT, int D, typename WL, typename AL>
__device__ __forceinline__ void ru_gemm(floatx16 (&acc)[MT][NTT], WL&& wload, AL&& aload) {
  using SM = SplitMode<2>;
  u32x4 wf[D + 1][MT][3];
  u32x4 af[2][NTT][3];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int q = 0; q < D; ++q)
    if (q < NSTEP) wload(q, wf[q]);
  aload(0, af[0]);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    if (s + D < NSTEP) wload(s + D, wf[(s + D) % (D + 1)]);
    if (s + 1 < NSTEP) aload(s + 1, af[(s + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
    if (s > 0 && s % NTAP == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTT; ++j) acc[i][j] = -acc[i][j];
    }
#pragma unroll
    for (int pr = SM::NPROD - 1; pr >= 0; --pr)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTT; ++j)
          acc[i][j] = mfma_k16<bf16_t>(wf[s % (D + 1)][i][SM::PB[pr]], af[s & 1][j][SM::PA[pr]], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

}  // namespace

// C = N input / output channels (128: the slice loop's SWAtten inter_dim); 4 waves, one workgroup
// per CU (LDS: x planes 96 KB + t1 planes 48 KB; t2 reuses the x planes)
template <int C>
__global__ __launch_bounds__(256, 1) void resunit_split_kernel(const lic_resunit_args a) {
  static_assert(C == 128, "wave assignment assumes N = 128 (2 / 4 m-tiles of 32 channels)");
  constexpr int C2 = C / 2;
  constexpr int KC1 = C / 16, KC2 = C2 / 16;
  constexpr int XPL = KC1 * RU_HP * 32;   // one part plane of the x halo (bytes)
  constexpr int T1PL = KC2 * RU_HP * 32;
  constexpr int T2PL = KC2 * 64 * 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const xs = smem;
  char* const t1s = smem + 3 * XPL;
  char* const t2s = smem;   // after GEMM1 (a barrier separates the last x read from the first t2 write)

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
  const int lrow = lane & 31, lhalf = lane >> 5;
  const int tiles_x = a.w >> 3, tiles_y = a.h >> 3;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int b = bid / tiles_y;
  const int hy0 = ty * 8 - 1, hx0 = tx * 8 - 1;   // halo origin (image coordinates)

  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)((int64_t)a.n * a.h * a.w * a.ldx * 4), 0x00020000);

  // ---- x halo -> three bf16 planes [part][chunk][halo px][16 ch]; zeros outside the image / px >= 100
  {
    constexpr int QPP = C / 4;                  // quads per pixel
    constexpr int Q = RU_HP * QPP / 256;        // quads per thread
    u32x4 h[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      const int qi = tid + i * 256, hp = qi / QPP, c4 = qi % QPP;
      const int hy = hp / 10, hx = hp - hy * 10, iy = hy0 + hy, ix = hx0 + hx;
      const bool ok = hp < 100 && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      const unsigned off = ok ? (unsigned)((((b * a.h + iy) * a.w + ix) * a.ldx + c4 * 4) * 4) : 0x80000000u;
      h[i] = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      const int qi = tid + i * 256, hp = qi / QPP, c4 = qi % QPP;
      const int k = c4 >> 2, q = c4 & 3;
      uint2 parts[3];
      split4<2>(make_float4(__uint_as_float(h[i].x), __uint_as_float(h[i].y), __uint_as_float(h[i].z),
                            __uint_as_float(h[i].w)),
                LIC_PRO_NONE, (k & 1) ? -1.f : 1.f, parts);
      const int off = k * RU_HP * 32 + ru_swz(hp, q >> 1) + (q & 1) * 8;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *(uint2*)(xs + pl * XPL + off) = parts[pl];
    }
  }

  // split-weight fragments (functional.split_weights: [copad/32][cpad/16][taps][3][64 lanes][16 B])
  auto wrsrc = [&](const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t w1r = wrsrc(a.w1s, (C2 / 32) * KC1 * 3 * 1024);
  const __amdgpu_buffer_rsrc_t w2r = wrsrc(a.w2s, (C2 / 32) * KC2 * 9 * 3 * 1024);
  const __amdgpu_buffer_rsrc_t w3r = wrsrc(a.w3s, (C / 32) * KC2 * 3 * 1024);
  auto frag = [&](const __amdgpu_buffer_rsrc_t& rs, int j, int k, int t, int nch, int ntap, int p) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (((j * nch + k) * ntap + t) * 3 + p) * 1024, 0);
  };
  __syncthreads();

  // ---- GEMM1: t1[64 ch][128 halo px]; wave: m-tile (wave & 1), n-tiles 2 (wave >> 1) + {0, 1}
  {
    const int mt = wave & 1;
    floatx16 acc[1][2];
    ru_gemm<KC1, 1, 1, 2, 4>(
        acc,
        [&](int s, u32x4(&w)[1][3]) {
#pragma unroll
          for (int p = 0; p < 3; ++p) w[0][p] = frag(w1r, mt, s, 0, KC1, 1, p);
        },
        [&](int s, u32x4(&f)[2][3]) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int hp = 32 * (2 * (wave >> 1) + j) + lrow;
#pragma unroll
            for (int p = 0; p < 3; ++p) f[j][p] = *(const u32x4*)(xs + p * XPL + s * RU_HP * 32 + ru_swz(hp, lhalf));
          }
        });
    const float os = (KC1 & 1) ? 1.f : -1.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int hp = 32 * (2 * (wave >> 1) + j) + lrow;
      const int hy = hp / 10, hx = hp - hy * 10, iy = hy0 + hy, ix = hx0 + hx;
      const bool ok = hp < 100 && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = 32 * mt + 8 * g + 4 * lhalf, kk = c0 >> 4;
        const float4 bb = *(const float4*)(a.b1 + c0);
        float4 v = make_float4(acc[0][j][4 * g] * os + bb.x, acc[0][j][4 * g + 1] * os + bb.y,
                               acc[0][j][4 * g + 2] * os + bb.z, acc[0][j][4 * g + 3] * os + bb.w);
        v = ok ? make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f))
               : make_float4(0.f, 0.f, 0.f, 0.f);
        uint2 parts[3];
        split4<2>(v, LIC_PRO_NONE, (kk & 1) ? -1.f : 1.f, parts);
        const int off = kk * RU_HP * 32 + ru_swz(hp, g & 1) + lhalf * 8;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *(uint2*)(t1s + pl * T1PL + off) = parts[pl];
      }
    }
  }
  __syncthreads();

  // ---- GEMM2: 3x3 conv on the t1 planes, t2[64 ch][64 px]; wave: m-tile (wave & 1), n-tile (wave >> 1)
  {
    const int mt = wave & 1, nt = wave >> 1;
    const int po = 32 * nt + lrow, oy = po >> 3, ox = po & 7;
    floatx16 acc[1][1];
    ru_gemm<KC2 * 9, 9, 1, 1, 5>(
        acc,
        [&](int s, u32x4(&w)[1][3]) {
#pragma unroll
          for (int p = 0; p < 3; ++p) w[0][p] = frag(w2r, mt, s / 9, s % 9, KC2, 9, p);
        },
        [&](int s, u32x4(&f)[1][3]) {
          const int k = s / 9, t = s % 9;
          const int hp = (oy + t / 3) * 10 + ox + t % 3;
#pragma unroll
          for (int p = 0; p < 3; ++p) f[0][p] = *(const u32x4*)(t1s + p * T1PL + k * RU_HP * 32 + ru_swz(hp, lhalf));
        });
    const float os = (KC2 & 1) ? 1.f : -1.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * mt + 8 * g + 4 * lhalf, kk = c0 >> 4;
      const float4 bb = *(const float4*)(a.b2 + c0);
      const float4 v = make_float4(fmaxf(acc[0][0][4 * g] * os + bb.x, 0.f), fmaxf(acc[0][0][4 * g + 1] * os + bb.y, 0.f),
                                   fmaxf(acc[0][0][4 * g + 2] * os + bb.z, 0.f), fmaxf(acc[0][0][4 * g + 3] * os + bb.w, 0.f));
      uint2 parts[3];
      split4<2>(v, LIC_PRO_NONE, (kk & 1) ? -1.f : 1.f, parts);
      const int off = kk * 64 * 32 + ru_swz(po, g & 1) + lhalf * 8;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *(uint2*)(t2s + pl * T2PL + off) = parts[pl];
    }
  }
  __syncthreads();

  // ---- GEMM3: out[128 ch][64 px] = relu(W3 t2 + b3 + x); wave: m-tiles 2 (wave & 1) + {0, 1}, n-tile (wave >> 1)
  {
    const int nt = wave >> 1;
    const int po = 32 * nt + lrow;
    floatx16 acc[2][1];
    ru_gemm<KC2, 1, 2, 1, 3>(
        acc,
        [&](int s, u32x4(&w)[2][3]) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p) w[i][p] = frag(w3r, 2 * (wave & 1) + i, s, 0, KC2, 1, p);
        },
        [&](int s, u32x4(&f)[1][3]) {
#pragma unroll
          for (int p = 0; p < 3; ++p) f[0][p] = *(const u32x4*)(t2s + p * T2PL + s * 64 * 32 + ru_swz(po, lhalf));
        });
    const float os = (KC2 & 1) ? 1.f : -1.f;
    const int y = ty * 8 + (po >> 3), xx = tx * 8 + (po & 7);
    const int64_t pix = ((int64_t)b * a.h + y) * a.w + xx;
    const float* xr = (const float*)a.x + pix * a.ldx;
    float* yr = (float*)a.y + pix * a.ldy;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = 32 * (2 * (wave & 1) + i) + 8 * g + 4 * lhalf;
        const float4 bb = *(const float4*)(a.b3 + c0);
        const float4 xv = *(const float4*)(xr + c0);
        const float4 v = make_float4(fmaxf(acc[i][0][4 * g] * os + bb.x + xv.x, 0.f),
                                     fmaxf(acc[i][0][4 * g + 1] * os + bb.y + xv.y, 0.f),
                                     fmaxf(acc[i][0][4 * g + 2] * os + bb.z + xv.z, 0.f),
                                     fmaxf(acc[i][0][4 * g + 3] * os + bb.w + xv.w, 0.f));
        *(float4*)(yr + c0) = v;
      }
  }
}

}  // namespace lic

extern "C" int lic_resunit_fwd(const lic_resunit_args* a, lic_stream_t stream) {
  using namespace lic;
  if (!a) return fail("resunit: null args");
  if (a->dtype != LIC_F32 || a->mfma_mode != 2) return fail("resunit: only fp32 activations with mfma_mode 2 (fp32x6)");
  if (!a->x || !a->y || !a->w1s || !a->w2s || !a->w3s || !a->b1 || !a->b2 || !a->b3) return fail("resunit: null tensor");
  if (a->c != 128) return fail("resunit: N (channels) must be 128");
  if (a->n < 1 || a->h < 8 || a->w < 8 || a->h % 8 || a->w % 8) return fail("resunit: map must be a positive multiple of 8x8");
  if (a->ldx % 4 || a->ldy % 4 || a->ldx < a->c || a->ldy < a->c || ((uintptr_t)a->x & 15) || ((uintptr_t)a->y & 15) ||
      ((uintptr_t)a->b1 & 15) || ((uintptr_t)a->b2 & 15) || ((uintptr_t)a->b3 & 15) || ((uintptr_t)a->w1s & 15) ||
      ((uintptr_t)a->w2s & 15) || ((uintptr_t)a->w3s & 15))
    return fail("resunit: views and weights must be 16-byte aligned (ld a multiple of 4)");
  if ((int64_t)a->n * a->h * a->w * a->ldx * 4 >= (1LL << 31)) return fail("resunit: input over 2 GB");
  if (a->x == a->y) return fail("resunit: in-place (x == y) is not supported: other tiles read x's halo");
  constexpr int C = 128;
  constexpr int smem = 3 * (C / 16) * RU_HP * 32 + 3 * (C / 32) * RU_HP * 32;
  auto kern = resunit_split_kernel<C>;
  const hipError_t ea = ensure_dyn_lds((const void*)kern, smem);
  if (ea != hipSuccess) return fail(std::string("resunit: dynamic LDS attribute: ") + hipGetErrorString(ea));
  const unsigned blocks = (unsigned)(a->n * (a->h / 8) * (a->w / 8));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), smem, (hipStream_t)stream, *a);
  LIC_CHECK_LAUNCH();
  return 0;
}
