// 16-bit (fp16 / bf16) WinBasedAttention core in one launch: qkv Linear + shifted-window attention
// (layers/win_attention.py:85-116 qkv -> q k^T * scale + relative-position bias (+ -100 region mask),
// softmax, attn v; :154-209 roll / window partition / reverse as addressing), C = 192, 8 heads of 24
// channels, 8x8 windows: the a_model's Win_noShift_Attention blocks at 64x64 (layers/layers.py:87-102).
//
// Unfused, the qkv 1x1 writes a 3C map (151 MB per call at 64^2 x 32, fp16) that the attention kernel
// reads straight back.  Here persistent workgroups (8 waves, two per CU: 72 KB of LDS each) walk
// windows: the window's 64 x 192 activations go to LDS; per head group (heads 4g .. 4g+3) the qkv GEMM
// of the group's 288 channels (transposed: A = the packed [3C][C] weights streamed from L2, each
// fragment read once per window; B = token fragments from LDS) leaves q | k in LDS as [token][192]
// rows and v as V^T [channel][token] rows, rounded to the 16-bit type after the bias exactly as the
// unfused qkv launch stores them; then wave (head, query tile) runs that head's attention for 32
// queries with the fragments from LDS (the unfused kernel's arithmetic, csrc/attention_mfma.hip:
// S^T = K Q^T, scale and bias on the fp32 dot, softmax over the lane's registers + lane ^ 32,
// O^T = V^T P^T) and stores its 24 output channels.  The next window's activations are loaded into
// registers during the last attention phase; the other workgroup on the CU hides the barriers.
#include <type_traits>
#include "lic_common.h"

namespace lic {

namespace {

constexpr int W16_C = 192, W16_HEADS = 8, W16_D = 24, W16_WS = 8, W16_T = 64;
constexpr int W16_XS = 200;   // elements per token row of the x tile (400 B: conflict-free b128 reads)
constexpr int W16_QS = 200;   // elements per token row of the group's q | k (96 + 96 + 8)
constexpr int W16_VS = 72;    // elements per channel row of the group's V^T (64 + 8)
constexpr int W16_X = W16_T * W16_XS * 2;
constexpr int W16_QK = W16_T * W16_QS * 2;
constexpr int W16_V = 96 * W16_VS * 2;
constexpr int W16_TAB = W16_HEADS * 225 * 4;
constexpr int W16_LDS = W16_X + W16_QK + W16_V + W16_TAB;
constexpr int W16_R = 3, W16_PD = W16_R - 1;   // weight ring (12 K steps: R divides 12)
static_assert(2 * W16_LDS <= 160 * 1024, "LDS: two workgroups per CU");

}  // namespace

template <typename T>
__global__ __launch_bounds__(512, 4) void wba16_qkv_attn_kernel(const lic_wba16_args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xs = smem;                                       // [64 tokens][W16_XS]
  T* qk = (T*)(smem + W16_X);                            // [64 tokens][W16_QS]: q 0..95, k 96..191 of the group
  T* vt = (T*)(smem + W16_X + W16_QK);                   // [96 channels][W16_VS]: the group's V^T
  float* tab = (float*)(smem + W16_X + W16_QK + W16_V);  // [8 heads][225]

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int nwx = a.w / W16_WS, nwy = a.h / W16_WS;
  const int nwin = a.n * nwy * nwx;
  auto pix_of = [&](int win, int t) -> int {
    const int wx = win % nwx, r = win / nwx, wy = r % nwy, b = r / nwy;
    int py = wy * W16_WS + t / W16_WS + a.shift, px = wx * W16_WS + t % W16_WS + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return (b * a.h + py) * a.w + px;
  };
  for (int k = tid; k < W16_HEADS * 225; k += 512) {
    const int h = k / 225, e = k - h * 225;
    tab[k] = a.table[e * a.tab_sr + h * a.tab_sh];
  }

  // this thread's 3 x 16 B of a window: token f / 24, channels 8 (f % 24) ..
  const T* xg = (const T*)a.x;
  u32x4 xv[3];
  auto load_x = [&](int win) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int f = tid + 512 * i, t = f / 24, ch = (f % 24) * 8;
      xv[i] = *(const u32x4*)(xg + (int64_t)pix_of(win, t) * a.ldx + ch);
    }
  };
  if ((int)blockIdx.x < nwin) load_x(blockIdx.x);

  // qkv weights: packed [576][1][192] (the qkv Linear's ConvPack), A fragment of packed channel tile jt
  // and K step kk = rows 32 jt + lr, input channels 16 kk + 8 lh .. +7
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)a.qkv_w, (short)0, 576 * 192 * 2, 0x00020000);
  const unsigned wl = (unsigned)((lr * W16_C + 8 * lh) * 2);

  for (int win = blockIdx.x; win < nwin; win += gridDim.x) {
    const int wx = win % nwx, wy = (win / nwx) % nwy;
    // ---- A: the window's activations to LDS (their only reader, the previous window's last qkv
    // phase, ended at a barrier) ----
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int f = tid + 512 * i, t = f / 24, ch = (f % 24) * 8;
      *(u32x4*)(xs + t * (W16_XS * 2) + ch * 2) = xv[i];
    }
    for (int g = 0; g < 2; ++g) {
      __syncthreads();   // x written (g = 0); the previous attention phase done with q | k / V^T

      // ---- B: the group's 9 channel tiles (q, k, v x 3 of 32) x 2 token tiles = 18 tiles: wave w takes
      // local channel tile w for both token tiles (its weight fragments serve both), and the ninth
      // channel tile's two token tiles go to waves e and e + 1 (e = 0 for g = 0, 4 for g = 1) ----
      auto gemm = [&](auto ex_c) __attribute__((always_inline)) {
        constexpr int EX = decltype(ex_c)::value;   // 1: this wave also has tile (8, tx)
        constexpr int CNT = 1 + EX;
        const int e0 = 4 * g, tx = wave - e0;
        int jt[CNT], lt[CNT];
#pragma unroll
        for (int i = 0; i < CNT; ++i) {
          lt[i] = i == 0 ? wave : 8;
          jt[i] = (lt[i] / 3) * 6 + 3 * g + lt[i] % 3;
        }
        auto load_w = [&](int kk, u32x4(&f)[CNT]) __attribute__((always_inline)) {
#pragma unroll
          for (int i = 0; i < CNT; ++i)
            f[i] = __builtin_amdgcn_raw_buffer_load_b128(wrs, wl, (jt[i] * 32 * W16_C + 16 * kk) * 2, 0);
        };
        floatx16 acc[2], accx;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = accx[r] = 0.f;
        u32x4 fw[W16_R][CNT];
#pragma unroll
        for (int q = 0; q < W16_PD; ++q) load_w(q, fw[q]);
#pragma unroll
        for (int kk = 0; kk < 12; ++kk) {
          if (kk + W16_PD < 12) load_w(kk + W16_PD, fw[(kk + W16_PD) % W16_R]);
          u32x4 fx[2];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            fx[tt] = *(const u32x4*)(xs + (32 * tt + lr) * (W16_XS * 2) + (16 * kk + 8 * lh) * 2);
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) acc[tt] = mfma_k16<T>(fw[kk % W16_R][0], fx[tt], acc[tt]);
          if constexpr (EX) accx = mfma_k16<T>(fw[kk % W16_R][CNT - 1], tx ? fx[1] : fx[0], accx);
        }
        // + bias, rounded to T: lane (token 32 tt + lr) holds channels 32 jt + 8 q + 4 lh + (0..3)
        auto store = [&](const floatx16& c, int i, int tt) __attribute__((always_inline)) {
          const int which = lt[i] / 3;   // 0 q, 1 k, 2 v
          const int t = 32 * tt + lr;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int lc = 32 * (lt[i] % 3) + 8 * q + 4 * lh;   // channel within the group's q / k / v
            const floatx4 bv = *(const floatx4*)(a.qkv_bias + 32 * jt[i] + 8 * q + 4 * lh);
            T e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = from_f<T>(c[4 * q + k] + bv[k]);
            if (which < 2) {
              *(uint2*)(qk + t * W16_QS + 96 * which + lc) = *(const uint2*)e;
            } else {
#pragma unroll
              for (int k = 0; k < 4; ++k) vt[(lc + k) * W16_VS + t] = e[k];
            }
          }
        };
        store(acc[0], 0, 0);
        store(acc[1], 0, 1);
        if constexpr (EX) store(accx, CNT - 1, tx);
      };
      if (wave == 4 * g || wave == 4 * g + 1) gemm(std::integral_constant<int, 1>{});
      else gemm(std::integral_constant<int, 0>{});
      __syncthreads();
      // the next window's activations, consumed by its phase A (the attention phase issues no loads)
      if (g == 1 && win + (int)gridDim.x < nwin) load_x(win + gridDim.x);

      // ---- C: wave = (head 4g + hl, query tile ti) ----
      {
        const int hl = wave >> 1, ti = wave & 1, h = 4 * g + hl;
        u32x4 kf[2][2] = {}, qf[2] = {};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int ch = 16 * s + 8 * lh;
          if (ch >= W16_D) continue;
          qf[s] = *(const u32x4*)(qk + (32 * ti + lr) * W16_QS + hl * W16_D + ch);
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) kf[s][tj] = *(const u32x4*)(qk + (32 * tj + lr) * W16_QS + 96 + hl * W16_D + ch);
        }
        floatx16 S[2];   // [key tile], this wave's query tile
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[x][r] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int tj = 0; tj < 2; ++tj) S[tj] = mfma_k16<T>(kf[s][tj], qf[s], S[tj]);

        // scale + bias (+ region mask), softmax over the keys (rows) of query i (lane column):
        // register r of key tile tj is key 32 tj + 8 (r >> 2) + 4 lh + (r & 3)
        const int split = W16_WS - a.shift;
        const bool last_row = wy == nwy - 1, last_col = wx == nwx - 1;
        const bool mask_on = a.mask_kind != 0 && (last_row || last_col);
        auto reg_wba = [&](int y, int x) {
          const int ly = y < a.h - W16_WS ? 0 : (y < a.h - a.shift ? 1 : 2);
          const int lx = x < a.w - W16_WS ? 0 : (x < a.w - a.shift ? 1 : 2);
          return ly * 3 + lx;
        };
        constexpr float L2E = 1.4426950408889634f;
        const int i = 32 * ti + lr;
        const int iy = i / W16_WS, ix = i % W16_WS;
        const float* trow = &tab[h * 225 + (iy + W16_WS - 1) * 15 + (ix + W16_WS - 1) - 4 * lh];
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[tj][r] = S[tj][r] * a.scale + trow[-((4 * tj + (r >> 2)) * 15 + (r & 3))];
        if (mask_on) {
          const int my_reg = a.mask_kind == 1 ? reg_wba(wy * W16_WS + iy, wx * W16_WS + ix) : 0;
#pragma unroll
          for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int jy = 4 * tj + (r >> 2), jx = 4 * lh + (r & 3);
              if (a.mask_kind == 1) {
                if (reg_wba(wy * W16_WS + jy, wx * W16_WS + jx) != my_reg) S[tj][r] += -100.0f;
              } else if ((last_row && ((iy < split) != (jy < split))) || (last_col && ((ix < split) != (jx < split)))) {
                S[tj][r] = -INFINITY;
              }
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, S[tj][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mxl = mx * L2E;
        float sum = 0.f;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(S[tj][r], L2E, -mxl));
            S[tj][r] = e;
            sum += e;
          }
        sum += __shfl_xor(sum, 32);
        const float inv = 1.0f / sum;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) S[tj][r] *= inv;

        // O^T[c][i] = sum_j V^T[c][j] P^T[j][i]: lane (c = lr, half lh) reads V^T row c in the permuted
        // key order of P's registers (keys j0 .. j0+3 and j0+8 .. j0+11); rows c >= 24 read zeros
        floatx16 O;
#pragma unroll
        for (int r = 0; r < 16; ++r) O[r] = 0.f;
        const bool cok = lr < W16_D;
        const T* vrow = vt + (hl * W16_D + (cok ? lr : 0)) * W16_VS;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int j0 = 32 * tj + 16 * s2 + 4 * lh;
            u32x4 va = {0u, 0u, 0u, 0u};
            if (cok) {
              *(uint2*)&va = *(const uint2*)(vrow + j0);
              *((uint2*)&va + 1) = *(const uint2*)(vrow + j0 + 8);
            }
            u32x4 pb;
            T* pe = (T*)&pb;
#pragma unroll
            for (int e = 0; e < 8; ++e) pe[e] = from_f<T>(S[tj][8 * s2 + e]);
            O = mfma_k16<T>(va, pb, O);
          }
        // lane (query i, half lh) holds channels 8 q + 4 lh + (0..3) of head h (24 valid)
        T* op = (T*)a.out + (int64_t)pix_of(win, i) * a.ldo + h * W16_D;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int c0 = 8 * q + 4 * lh;
          if (c0 >= W16_D) continue;
          uint2 pk;
          T* e = (T*)&pk;
#pragma unroll
          for (int k = 0; k < 4; ++k) e[k] = from_f<T>(O[4 * q + k]);
          *(uint2*)(op + c0) = pk;
        }
      }
    }
    // (no barrier here: x was last read before the barrier that followed the g = 1 qkv phase, and the
    // next window's first qkv phase writes q | k / V^T only after its own barrier)
  }
}

}  // namespace lic

using namespace lic;

extern "C" int lic_wba16_qkv_attn_fwd(const lic_wba16_args* a, lic_stream_t stream) {
  if (!a) return fail("wba16: null args");
  if (a->dtype != LIC_F16 && a->dtype != LIC_BF16) return fail("wba16: dtype must be LIC_F16 or LIC_BF16");
  if (a->c != W16_C || a->heads != W16_HEADS || a->ws != W16_WS) return fail("wba16: needs C = 192, 8 heads, 8x8 windows");
  if (a->n < 1 || a->h < W16_WS || a->w < W16_WS || a->h % W16_WS || a->w % W16_WS) return fail("wba16: H and W must be multiples of 8");
  if (a->shift < 0 || a->shift >= W16_WS) return fail("wba16: shift out of range");
  if (!a->x || !a->out || !a->qkv_w || !a->qkv_bias || !a->table) return fail("wba16: null tensor");
  if ((uintptr_t)a->x % 16 || a->ldx % 8 || a->ldx < W16_C) return fail("wba16: x must be 16-byte aligned with rows of 8k elements");
  if ((uintptr_t)a->out % 8 || a->ldo % 4 || a->ldo < W16_C) return fail("wba16: out must be 8-byte aligned with rows of 4k elements");
  if ((uintptr_t)a->qkv_w % 16 || (uintptr_t)a->qkv_bias % 16) return fail("wba16: weights / bias must be 16-byte aligned");
  if ((int64_t)a->n * a->h * a->w * (int64_t)(a->ldx > a->ldo ? a->ldx : a->ldo) >= (1LL << 31))
    return fail("wba16: map too large for int32 indexing");
  {
    // persistent workgroups read the next window's x while others store their outputs: out may not
    // overlap x
    const int64_t npix = (int64_t)a->n * a->h * a->w;
    const uintptr_t x0 = (uintptr_t)a->x, x1 = x0 + (uintptr_t)(((npix - 1) * a->ldx + W16_C) * 2);
    const uintptr_t o0 = (uintptr_t)a->out, o1 = o0 + (uintptr_t)(((npix - 1) * a->ldo + W16_C) * 2);
    if (x0 < o1 && o0 < x1) return fail("wba16: out must not overlap x");
  }
  const int64_t nwin = (int64_t)a->n * (a->h / W16_WS) * (a->w / W16_WS);
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  const unsigned grid = (unsigned)(nwin < 2 * ncu ? nwin : 2 * ncu);   // two workgroups per CU
  hipStream_t s = (hipStream_t)stream;
  const void* kern = a->dtype == LIC_F16 ? (const void*)wba16_qkv_attn_kernel<half_t> : (const void*)wba16_qkv_attn_kernel<bf16_t>;
  const hipError_t ea = ensure_dyn_lds(kern, W16_LDS);
  if (ea != hipSuccess) return fail(std::string("wba16: dynamic LDS attribute: ") + hipGetErrorString(ea));
  if (a->dtype == LIC_F16) hipLaunchKernelGGL(wba16_qkv_attn_kernel<half_t>, dim3(grid), dim3(512), W16_LDS, s, *a);
  else hipLaunchKernelGGL(wba16_qkv_attn_kernel<bf16_t>, dim3(grid), dim3(512), W16_LDS, s, *a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(std::string("wba16 launch: ") + hipGetErrorString(e));
}
