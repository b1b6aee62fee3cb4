// 1x1 convolutions / nn.Linear in the split fp32 modes (lic_conv_args.mfma_mode 2 fp32x6 / 1 fp32x3;
// arithmetic and packed-weight layout: conv_split.h) as a register-streaming GEMM.
//
// A 1x1 conv has no halo to share, so nothing goes through LDS on the way in: every wave owns
// TM x 32 output pixels and TN x 32 output channels and, per 16-channel step,
//   * loads its A fragments as fp32 straight from the activation tensor (lane l: pixel l & 31,
//     channels 8(l >> 5) .. +7 = two 16-B raw buffer loads; out-of-range pixels / channels read
//     zeros) three steps ahead of use and splits them into the NPA 16-bit parts IN REGISTERS, one
//     step ahead, while the current step's MFMAs run -- the parts are the MFMA A operands as they
//     stand;
//   * loads its B fragments from the fragment-order weight pack (one contiguous 1 KB per part and
//     n-tile) one step ahead;
//   * issues NPROD x TM x TN MFMAs.
// No barrier, no LDS traffic in the loop; waves of a workgroup are independent (the workgroup
// only shares the epilogue's row table).  TM = TN = 2 (64 pixels x 64 channels per wave) fits
// two waves per SIMD (242 VGPRs); wider tiles at one wave per SIMD spill (the B and A rings must
// sit in arch VGPRs, only the accumulators go to AGPRs).  The chunk loop is unrolled by two (ring
// slots by parity): a six-way unroll made the compiler hoist loads across the copies and spill.
// Used for Win_noShift_Attention's qkv / proj Linear, the GDN / IGDN x^2 (prologue SQUARE)
// convolutions and the other 1x1 layers (net_ga.py:253-309, layers/layers.py:87-102).
#include "conv_halo.h"
#include "conv_split.h"

#ifndef G1_TN
#define G1_TN 2
#endif
#ifndef G1_NOEPI
#define G1_NOEPI 0
#endif
#ifndef G1_WPS
#define G1_WPS 2
#endif
#ifndef G1_AUX
#define G1_AUX 0
#endif
#ifndef G1_ALT
#define G1_ALT 1
#endif

namespace lic {

struct G1Plan {
  int M;              // output lattice pixels n * mi * mj
  int nchunks;        // cpad / 16
  int in_bytes;       // activation buffer extent for the raw buffer loads
};

template <int MODE, int TM, int TN>
__global__ __launch_bounds__(256, G1_WPS) void conv1x1_split_kernel(const lic_conv_args a, const G1Plan p) {
  using SM = SplitMode<MODE>;
  using T = typename SM::T;
  constexpr int NPA = SM::NPA, NPB = SM::NPB, NPROD = SM::NPROD;
  constexpr int WTM = 32 * TM, WTN = 32 * TN;

  __shared__ int rowpix_s[4 * WTM];
  __shared__ float sbias_s[WTN];
  __shared__ float ct_s[4][32 * 33];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar wave offsets (no waterfall loops)
  const int lrow = lane & 31, lhalf = lane >> 5;
  const int m0 = (blockIdx.x * 4 + wave) * WTM;
  const int n0 = blockIdx.y * WTN;
  const int mimj = a.mi * a.mj;

  for (int n = tid; n < WTN; n += 256) sbias_s[n] = (a.bias && n0 + n < a.co) ? a.bias[n0 + n] : 0.f;
  int* rowpix = rowpix_s + wave * WTM;
  for (int r = lane; r < WTM; r += 64) {
    const int m = m0 + r;
    int base = -1;
    if (m < p.M) {
      const int b = m / mimj, rem = m - b * mimj;
      const int i = rem / a.mj, j = rem - i * a.mj;
      int oy = a.oy0 + a.osy * i, ox = a.ox0 + a.osx * j;
      if (a.out_shuffle >= 2) { oy *= 2; ox *= 2; }
      base = (b * a.ho + oy) * a.wo + ox;
    }
    rowpix[r] = base;
  }
  __syncthreads();

  // A: element offset of this lane's pixel (row lrow of m-tile i) at channel 8 * lhalf, -1 = none
  int aoff[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + i * 32 + lrow;
    int off = -1;
    if (m < p.M) {
      const int b = m / mimj, rem = m - b * mimj;
      const int ii = rem / a.mj, jj = rem - ii * a.mj;
      const int iy = ii * a.isy + a.dy[0], ix = jj * a.isx + a.dx[0];
      if ((unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w)
        off = ((b * a.h + iy) * a.w + ix) * a.ldx + 8 * lhalf;
    }
    aoff[i] = off;
  }
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, p.in_bytes, 0x00020000);
  const int nch = p.nchunks;
  // raw fp32 A of chunk k (8 channels per lane and m-tile = two 16-B loads, unconditional; past the
  // last chunk: clamped, a harmless reload)
  auto load_a = [&](int k, u32x4(&ra)[TM][2]) {
    k = k < nch ? k : nch - 1;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = k * 16 + 8 * lhalf + 4 * h;
        const unsigned off = (aoff[i] >= 0 && c < a.ci) ? (unsigned)(aoff[i] + k * 16 + 4 * h) * 4u : 0x80000000u;
        ra[i][h] = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, G1_AUX);
      }
  };
  // B fragments of chunk k: n-tile (n0/32 + j), contiguous 1 KB per part.  Raw buffer loads with the
  // lane's 16 B as the only vector offset: the per-fragment offsets are scalar (no 64-bit vector
  // addresses held across the loop)
  const int ntiles = a.copad / 32;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.wgt_split, (short)0, (int)((int64_t)ntiles * nch * NPB * 1024), 0x00020000);
  auto load_b = [&](int k, u32x4(&fb)[NPB][TN]) {
    k = k < nch ? k : nch - 1;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int jj = n0 / 32 + j;
      jj = jj < ntiles ? jj : ntiles - 1;   // n-tiles past the pack: clamped (their outputs are masked)
#pragma unroll
      for (int pl = 0; pl < NPB; ++pl)
        fb[pl][j] = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, ((jj * nch + k) * NPB + pl) * 1024, G1_AUX);
    }
  };
  // raw -> parts (prologue, chunk sign); part pl of m-tile i as the MFMA A operand (8 x 16-bit)
  auto split_a = [&](const u32x4(&ra)[TM][2], int k, u32x4(&fa)[NPA][TM]) {
    const float sg = (G1_ALT && (k & 1)) ? -1.f : 1.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint2 parts[NPA];
        const u32x4 r = ra[i][h];
        split4<MODE>(make_float4(__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z), __uint_as_float(r.w)),
                     a.prologue, sg, parts);
#pragma unroll
        for (int pl = 0; pl < NPA; ++pl) {
          fa[pl][i][2 * h] = parts[pl].x;
          fa[pl][i][2 * h + 1] = parts[pl].y;
        }
      }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Software pipeline, unrolled by two (register sets by chunk parity): during chunk k the MFMAs read
  // the parts of chunk k (fa[k&1]) while the VALU splits the raw fp32 of chunk k+1 (ra[(k+1)&1],
  // loaded two chunks earlier) into fa[(k+1)&1] and reloads that raw slot with chunk k+3; B of
  // chunk k+1 is loaded into fb[(k+1)&1].  No scheduling barrier inside a chunk: the split's VALU
  // interleaves with the MFMAs.
  u32x4 ra[2][TM][2], fb[2][NPB][TN], fa[2][NPA][TM];
  load_a(0, ra[0]);
  load_a(1, ra[1]);
  load_b(0, fb[0]);
  split_a(ra[0], 0, fa[0]);
  load_a(2, ra[0]);

  auto chunk = [&](int k, auto u) {
    constexpr int U = decltype(u)::value;   // k & 1
#if G1_ALT
    if (k > 0)   // the running sum changes sign with the chunk's parts (conv_split_wd.hip)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = -acc[i][j];
#endif
    load_b(k + 1, fb[U ^ 1]);
#pragma unroll
    for (int pr = NPROD - 1; pr >= 0; --pr)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_k16<T>(fa[U][SM::PA[pr]][i], fb[U][SM::PB[pr]][j], acc[i][j]);
    split_a(ra[U ^ 1], k + 1, fa[U ^ 1]);
    load_a(k + 3, ra[U ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int k = 0; k < nch; k += 2) {
    chunk(k, std::integral_constant<int, 0>{});
    if (k + 1 >= nch) break;
    chunk(k + 1, std::integral_constant<int, 1>{});
  }

  const float oscale = (G1_ALT && nch > 0 && !(nch & 1)) ? -SM::scale : SM::scale;
  float* ct = ct_s[wave];
#if G1_NOEPI
  {
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) z += acc[i][j][r];
    if (z == 1234.5f) ((float*)a.y)[tid] = z;
    return;
  }
#endif
  epilogue_all<float, TM * TN, TN>(a, ct, rowpix, n0, sbias_s, lane, [&](int q) {
#pragma unroll
    for (int qq = 0; qq < TM * TN; ++qq)
      if (qq == q) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          ct[((r & 3) + 8 * (r >> 2) + 4 * lhalf) * 33 + lrow] = acc[qq / TN][qq % TN][r] * oscale;
      }
  });
}

template <int MODE, int TM, int TN>
static int try_split_1x1(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.ntaps != 1 || a.cpad % 16 || a.ci % 4 || a.ldx % 4 || ((uintptr_t)a.x % 16) || ((uintptr_t)a.wgt_split % 16))
    return 0;
  const int64_t in_elems = (int64_t)a.n * a.h * a.w * a.ldx;
  const int64_t M = (int64_t)a.n * a.mi * a.mj;
  if (in_elems * 4 >= (1LL << 31) || M >= (1LL << 31)) return 0;
  G1Plan p;
  p.M = (int)M;
  p.nchunks = a.cpad / 16;
  p.in_bytes = (int)(in_elems * 4);
  dim3 grid((unsigned)((M + 4 * 32 * TM - 1) / (4 * 32 * TM)), (a.copad + 32 * TN - 1) / (32 * TN));
  hipLaunchKernelGGL((conv1x1_split_kernel<MODE, TM, TN>), grid, dim3(256), 0, s, a, p);
  hipError_t e = hipGetLastError();
  status = e == hipSuccess ? 0 : fail(std::string("split 1x1 conv launch: ") + hipGetErrorString(e));
  return 1;
}

// Returns 1 and launches when the register-streaming 1x1 split GEMM applies, 0 otherwise.
int conv_split_1x1_dispatch(const lic_conv_args& a, hipStream_t s, int& status) {
  if (a.mfma_mode != 2 || !a.wgt_split || a.dtype != LIC_F32 || a.ntaps != 1) return 0;
  if (a.groups != 1 || a.force_direct || a.force_mfma_generic) return 0;
  if (a.prologue != LIC_PRO_NONE && a.prologue != LIC_PRO_SQUARE && a.prologue != LIC_PRO_ABS) return 0;
  const int64_t M = (int64_t)a.n * a.mi * a.mj;
  if (M < 2048) return 0;   // tiny maps: the LDS-staged kernels
  return try_split_1x1<2, 2, G1_TN>(a, s, status);
}

}  // namespace lic
