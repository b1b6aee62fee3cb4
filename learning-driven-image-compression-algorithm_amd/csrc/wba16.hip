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

int wd_env(const char* name, int def);   // conv_split_wd.hip

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


// ---- v3 (round 6): head-group-stationary, weights in registers.  v2 streams the 221 KB of qkv weights
// from L2 for EVERY window through a 3-step register ring (24 dependent L2 round trips per window and
// wave: 129 us per call at 64^2 x 32 against a ~25 us MFMA / HBM floor).  Here a workgroup (one per CU)
// owns ONE head group g for the whole launch and each wave keeps ITS weight fragments -- local channel
// tile w, all 12 K steps (48 VGPRs; 96 for the two waves that also own tile 8's token tiles) -- in
// registers, loaded once.  Per window: the window's x (coalesced 16-B loads, prefetched one window
// ahead into registers as in v2) goes to LDS, the qkv GEMM reads its B fragments there, q | k / V^T go
// to their own LDS region, ONE barrier, the attention, ONE barrier (which also publishes the next
// window's x, written right after the attention).  The two workgroups of a window (g = 0, 1) sit on the
// same XCD (block ids b and b + 8) and walk the same window sequence, so the second read of x hits L2.
// (A first v3 read the x B fragments straight from global memory -- 32 pixels x 32 B per load, 12x over
// the same lines -- and took 204 us.)  The arithmetic is v2's (same MFMA sequence per tile, same
// rounding points): bit-identical outputs.
// diagnostic build only (-DW16_STAMP=1, tools/wba16_stamps.py): wave 0's per-phase cycle sums (s_memtime),
// written past the end of the output (the caller allocates room); outputs stay valid
#ifndef W16_STAMP
#define W16_STAMP 0
#endif
#if W16_STAMP
#define W16T(v)                                                                          \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#else
#define W16T(v)
#endif
constexpr int W16V3_TAB = 4 * 225 * 4;                   // the group's 4 heads of the bias table
constexpr int W16V3_BIAS = 288 * 4;                      // the group's q | k | v biases (fp32)
constexpr int W16V3_W8 = 12 * 1024;                      // local tile 8's weight fragments (the two ex waves)
constexpr int W16V3_LDS = W16_X + W16_QK + W16_V + W16V3_TAB + W16V3_BIAS + W16V3_W8;
static_assert(W16V3_LDS <= 160 * 1024, "LDS");

template <typename T>
__global__ __launch_bounds__(512, 2) void wba16_v3_kernel(const lic_wba16_args a, int npairs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* xs = smem;                                               // [64 tokens][W16_XS]
  T* qk = (T*)(smem + W16_X);                                    // [64 tokens][W16_QS]
  T* vt = (T*)(smem + W16_X + W16_QK);                           // [96 channels][W16_VS]
  float* tab = (float*)(smem + W16_X + W16_QK + W16_V);          // [4 heads][225]
  float* sbias = tab + 4 * 225;                                  // [9 local tiles][32]
  char* w8s = (char*)(sbias + 288);                              // [12 K steps][64 lanes][16 B]

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int bid = blockIdx.x;
  const int g = (bid >> 3) & 1;                 // head group; blocks b and b + 8 share an XCD
  const int pair = (bid >> 4) * 8 + (bid & 7);
  const int nwx = a.w / W16_WS, nwy = a.h / W16_WS;
  const int nwin = a.n * nwy * nwx;
  auto pix_of = [&](int win, int t) -> int {
    const int wx = win % nwx, r = win / nwx, wy = r % nwy, b = r / nwy;
    int py = wy * W16_WS + t / W16_WS + a.shift, px = wx * W16_WS + t % W16_WS + a.shift;
    if (py >= a.h) py -= a.h;
    if (px >= a.w) px -= a.w;
    return (b * a.h + py) * a.w + px;
  };
  if (pair >= nwin) return;

  // local channel tile lt (0..8) of group g: (lt / 3) = q / k / v, (lt % 3) = its 32-channel third
  auto jt_of = [&](int lt) { return (lt / 3) * 6 + 3 * g + lt % 3; };
  // GEMM tiles: wave w owns local tile w for both token tiles; tile 8's token tile tx goes to wave 4g + tx
  const int e0 = 4 * g;
  const bool ex = wave == e0 || wave == e0 + 1;
  const int tx = wave - e0;
  // ---- this wave's weight fragments, once: (tile, kk) lane (r, h) = row 32 jt + r, channels 16 kk + 8 h ----
  const T* wg = (const T*)a.qkv_w;
  u32x4 wf[12];
  {
    const T* src = wg + (32 * jt_of(wave) + lr) * W16_C + 8 * lh;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) wf[kk] = *(const u32x4*)(src + 16 * kk);
  }
  // local tile 8 (shared by the two ex waves) in LDS, fragment order
  for (int c = tid; c < 12 * 64; c += 512) {
    const int l = c & 63, kk = c >> 6;
    *(u32x4*)(w8s + c * 16) = *(const u32x4*)(wg + (32 * jt_of(8) + (l & 31)) * W16_C + 16 * kk + 8 * (l >> 5));
  }
  for (int k = tid; k < 4 * 225; k += 512) {
    const int hl = k / 225, e = k - hl * 225;
    tab[k] = a.table[e * a.tab_sr + (4 * g + hl) * a.tab_sh];
  }
  // the biases in LDS, then this wave's in registers (a global load per fragment in the store phase was
  // ~1/5 of the kernel: stamps)
  for (int k = tid; k < 288; k += 512) sbias[k] = a.qkv_bias[32 * jt_of(k / 32) + (k % 32)];

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
  auto store_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int f = tid + 512 * i, t = f / 24, ch = (f % 24) * 8;
      *(u32x4*)(xs + t * (W16_XS * 2) + ch * 2) = xv[i];
    }
  };
#if W16_STAMP
  unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, t6 = 0, tb = 0, te = 0;
  unsigned long long s_gemm = 0, s_store = 0, s_b1 = 0, s_next = 0, s_attn = 0, s_b2 = 0;
  unsigned long long ua = 0, ub = 0, uc = 0, ud = 0, s_a1 = 0, s_a2 = 0, s_a3 = 0, s_a4 = 0;
#endif
  W16T(tb);
  load_x(pair);
  store_x();
  if (pair + npairs < nwin) load_x(pair + npairs);
  __syncthreads();   // x of the first window, the table and the biases in LDS
  // the relative-position bias of this wave's (head, query tile) for this lane's 32 scores: the same for
  // every window (32 LDS reads per window before)
  const int hl_a = wave >> 1, ti_a = wave & 1;
  float rpb[2][16];
  {
    const int i = 32 * ti_a + lr, iy = i / W16_WS, ix = i % W16_WS;
    const float* trow = &tab[hl_a * 225 + (iy + W16_WS - 1) * 15 + (ix + W16_WS - 1) - 4 * lh];
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int r = 0; r < 16; ++r) rpb[tj][r] = trow[-((4 * tj + (r >> 2)) * 15 + (r & 3))];
  }
  floatx4 bw[4], b8[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bw[q] = *(const floatx4*)(sbias + 32 * wave + 8 * q + 4 * lh);
    b8[q] = *(const floatx4*)(sbias + 32 * 8 + 8 * q + 4 * lh);
  }
  W16T(t0);
#if W16_STAMP
  const unsigned long long t_pro = t0 - tb;
#endif

  for (int win = pair; win < nwin; win += npairs) {
    W16T(t1);
    const int wx = win % nwx, wy = (win / nwx) % nwy;
    floatx16 acc[2], accx;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = accx[r] = 0.f;
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) {
      u32x4 fx[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) fx[tt] = *(const u32x4*)(xs + (32 * tt + lr) * (W16_XS * 2) + (16 * kk + 8 * lh) * 2);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) acc[tt] = mfma_k16<T>(wf[kk], fx[tt], acc[tt]);
      if (ex) accx = mfma_k16<T>(*(const u32x4*)(w8s + kk * 1024 + lane * 16), tx ? fx[1] : fx[0], accx);
    }
    W16T(t2);
    // + bias, rounded to T: lane (token 32 tt + lr) holds channels 32 jt + 8 q + 4 lh + (0..3)
    auto store = [&](const floatx16& c, int lt, const floatx4(&bb)[4], int tt) __attribute__((always_inline)) {
      const int which = lt / 3;
      const int t = 32 * tt + lr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lc = 32 * (lt % 3) + 8 * q + 4 * lh;
        const floatx4 bv = bb[q];
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
    store(acc[0], wave, bw, 0);
    store(acc[1], wave, bw, 1);
    if (ex) store(accx, 8, b8, tx);
    W16T(t3);
    __syncthreads();   // q | k / V^T complete; every wave is done reading this window's x
    W16T(t4);

    // the next window's x to LDS (x is not read again this window) and the one after it into registers
    const bool more = win + npairs < nwin;
    if (more) {
      store_x();
      if (win + 2 * npairs < nwin) load_x(win + 2 * npairs);
    }
    W16T(t5);

    // ---- attention: wave = (head 4g + hl, query tile ti) (v2's arithmetic) ----
    {
      const int hl = wave >> 1, ti = wave & 1;
      u32x4 kf[2][2] = {}, qf[2] = {};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 16 * s + 8 * lh;
        if (ch >= W16_D) continue;
        qf[s] = *(const u32x4*)(qk + (32 * ti + lr) * W16_QS + hl * W16_D + ch);
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) kf[s][tj] = *(const u32x4*)(qk + (32 * tj + lr) * W16_QS + 96 + hl * W16_D + ch);
      }
      floatx16 S[2];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[x][r] = 0.f;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) S[tj] = mfma_k16<T>(kf[s][tj], qf[s], S[tj]);
      const int split = W16_WS - a.shift;
      const bool last_row = wy == nwy - 1, last_col = wx == nwx - 1;
      const bool mask_on = a.mask_kind != 0 && (last_row || last_col);
      constexpr float L2E = 1.4426950408889634f;
      const int i = 32 * ti + lr;
      const int iy = i / W16_WS, ix = i % W16_WS;
#pragma unroll
      for (int tj = 0; tj < 2; ++tj)
#pragma unroll
        for (int r = 0; r < 16; ++r) S[tj][r] = S[tj][r] * a.scale + rpb[tj][r];
      W16T(ua);
      if (mask_on) {
        // a key is in another region than the query iff the window is on the last window row and the two
        // lie on different sides of row `split`, or likewise for the last column (the regions of
        // layers/win_attention.py:160-181 / Block_unet.py:204-237 inside one window): -100 added (WBA) or
        // -inf (WMSA)
        const bool qy = iy < split, qx = ix < split;
        // key row jy = 4 tj + (r >> 2), key column jx = 4 lh + (r & 3): 8 row and 4 column flags
        unsigned rowd = 0, cold = 0;
#pragma unroll
        for (int jy = 0; jy < 8; ++jy) rowd |= (unsigned)(last_row && (qy != (jy < split))) << jy;
#pragma unroll
        for (int c = 0; c < 4; ++c) cold |= (unsigned)(last_col && (qx != ((4 * lh + c) < split))) << c;
        const float madd = a.mask_kind == 1 ? -100.0f : -INFINITY;
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool other = ((rowd >> (4 * tj + (r >> 2))) | (cold >> (r & 3))) & 1u;
            const float v = S[tj][r] + madd;   // (-inf + x = -inf)
            S[tj][r] = other ? v : S[tj][r];
          }
      }
      W16T(ub);
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
      W16T(uc);
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
      W16T(ud);
      T* op = (T*)a.out + (int64_t)pix_of(win, i) * a.ldo + (4 * g + hl) * W16_D;
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
    W16T(t6);
    __syncthreads();   // q | k / V^T read (the next stores may overwrite them); the next window's x in LDS
#if W16_STAMP
    W16T(te);
    s_gemm += t2 - t1; s_store += t3 - t2; s_b1 += t4 - t3; s_next += t5 - t4; s_attn += t6 - t5; s_b2 += te - t6;
    s_a1 += ua - t5; s_a2 += ub - ua; s_a3 += uc - ub; s_a4 += ud - uc;
#endif
  }
#if W16_STAMP
  if (tid == 0) {
    unsigned long long* o = (unsigned long long*)((T*)a.out + (size_t)a.n * a.h * a.w * a.ldo) + (size_t)blockIdx.x * 9;
    o[0] = t_pro; o[1] = s_gemm; o[2] = s_store; o[3] = s_b1; o[4] = s_next; o[5] = s_attn; o[6] = s_b2;
    o[7] = s_a1 | (s_a2 << 32);   // (two 32-bit sums: S + bias, mask)
    o[8] = s_a3 | (s_a4 << 32);   // (softmax, PV)
  }
#endif
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
  hipStream_t s = (hipStream_t)stream;
  // v3 (default): head-group-stationary workgroups, one per CU; LIC_WBA16_V=2 restores v2 (A/B)
  static const int ver = wd_env("LIC_WBA16_V", 3);
  if (ver == 3) {
    // window pairs: multiples of 8 so that the two head groups of a pair (blocks b, b + 8) share an XCD
    int64_t np = nwin < ncu / 2 ? nwin : ncu / 2;
    np = (np + 7) / 8 * 8;
    const void* kern3 = a->dtype == LIC_F16 ? (const void*)wba16_v3_kernel<half_t> : (const void*)wba16_v3_kernel<bf16_t>;
    const hipError_t e3 = ensure_dyn_lds(kern3, W16V3_LDS);
    if (e3 != hipSuccess) return fail(std::string("wba16: dynamic LDS attribute: ") + hipGetErrorString(e3));
    if (a->dtype == LIC_F16)
      hipLaunchKernelGGL(wba16_v3_kernel<half_t>, dim3((unsigned)(2 * np)), dim3(512), W16V3_LDS, s, *a, (int)np);
    else
      hipLaunchKernelGGL(wba16_v3_kernel<bf16_t>, dim3((unsigned)(2 * np)), dim3(512), W16V3_LDS, s, *a, (int)np);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(std::string("wba16 launch: ") + hipGetErrorString(e));
  }
  const unsigned grid = (unsigned)(nwin < 2 * ncu ? nwin : 2 * ncu);   // two workgroups per CU
  const void* kern = a->dtype == LIC_F16 ? (const void*)wba16_qkv_attn_kernel<half_t> : (const void*)wba16_qkv_attn_kernel<bf16_t>;
  const hipError_t ea = ensure_dyn_lds(kern, W16_LDS);
  if (ea != hipSuccess) return fail(std::string("wba16: dynamic LDS attribute: ") + hipGetErrorString(ea));
  if (a->dtype == LIC_F16) hipLaunchKernelGGL(wba16_qkv_attn_kernel<half_t>, dim3(grid), dim3(512), W16_LDS, s, *a);
  else hipLaunchKernelGGL(wba16_qkv_attn_kernel<bf16_t>, dim3(grid), dim3(512), W16_LDS, s, *a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(std::string("wba16 launch: ") + hipGetErrorString(e));
}
