// Weights-direct split convolutions on 8x8-px tiles (conv_split_wd.h): the 16x16 latents of the slice
// loop / hyper nets, 8-wide maps and the 4x4 hyper-prior maps.
#include "conv_split_wd.h"

namespace lic {

int wd_dispatch_small(const lic_conv_args& a, hipStream_t s, int& status) {
  // A/B switch (LIC_WD_SMALL1X1=0): 1x1 launches on small maps go to the register GEMM (conv_split_gemm.hip)
  const bool small1x1 = wd_env("LIC_WD_SMALL1X1", 1) != 0;
  auto blocks = [&](int th, int tw, int bn) {
    return (int64_t)a.n * ((a.mi + th - 1) / th) * ((a.mj + tw - 1) / tw) * (a.copad / bn);
  };
  // 8x8 px x 64 channel tiles, one 32x32 accumulator per wave, four waves per SIMD -- the grid is what
  // limits these launches.  32 output channels (the slice loop's per-slice mean / scale heads): 8x8 px
  // x 32 channel tiles of two waves, one 32x32 accumulator each.  (Maps down to 4x4 -- the hyper
  // prior's -- take the 8x8 tiles partly masked: latency-bound either way, and the exact-fp32 MFMA
  // chain they otherwise fall back to is 16x slower per product.)
  if (a.copad == 32 && a.mi >= 4 && a.mj >= 4) {
    if (a.ntaps == 1 && a.cpad % 32 == 0 && small1x1)
      return try_split_wd<2, 2, 8, 8, 32, 2, 1, 4, 2, 1>(a, s, status) || try_split_wd<2, 2, 8, 8, 32, 2, 1, 4, 2>(a, s, status);
    if (a.ntaps == 9) {
      if (try_split_wd<2, 9, 8, 8, 32, 2, 1, 4, 0, 1>(a, s, status)) return 1;
      return try_split_wd<2, 9, 8, 8, 32, 2, 1, 4>(a, s, status);
    }
  }
  // 1x1 convs below the big-map virtual-tap launches (< 64 K px: the 16x16 latents' Swin MLP 128 -> 512
  // and WBA qkv 192 -> 576, the 32x32 GDN / skip 1x1s) take these tiles too, whatever their channel
  // count (they went to the register GEMM at ~6 % of peak / 6).  A/B: LIC_WD_SMALL1X1_ALL=0
  const bool small1x1_all = a.ntaps == 1 && small1x1 && wd_env("LIC_WD_SMALL1X1_ALL", 1) != 0 &&
                            (int64_t)a.n * a.mi * a.mj < 65536;
  if (a.mi >= 4 && a.mj >= 4 && (blocks(16, 16, 64) < 256 || a.mi <= 8 || a.mj <= 8 || small1x1_all) &&
      blocks(8, 8, 64) >= 32) {
    if (a.ntaps == 1 && a.cpad % 32 == 0 && small1x1)
      return try_split_wd<2, 2, 8, 8, 64, 2, 2, 2, 2, 1>(a, s, status) || try_split_wd<2, 2, 8, 8, 64, 2, 2, 2, 2>(a, s, status);
    if (a.ntaps == 9) {
      // fewer workgroups than the GPU holds (the slice loop's cc / LRP transforms, B x 4 tiles x a few
      // channel blocks): two tap groups of 4 waves per workgroup, half the dependent chain per wave.
      // A/B: LIC_WD_TAPSPLIT=0
      // 96 output channels per workgroup (3 waves per tap group, three waves per SIMD) where the channel
      // count allows: the 16x16 latents' 192-channel 3x3s are 256 such workgroups -- one per CU -- instead
      // of 384 of 64 channels (half the CUs running two).  A/B: LIC_WD_BN96=0
      if (wd_env("LIC_WD_TAPSPLIT", 1) && wd_env("LIC_WD_BN96", 1) && a.copad % 96 == 0 && blocks(8, 8, 64) <= 512 &&
          try_split_wd<2, 9, 8, 8, 96, 2, 3, 1, 0, 1, 0, 3, 0, 2>(a, s, status))
        return 1;
      if (wd_env("LIC_WD_TAPSPLIT", 1) && blocks(8, 8, 64) <= 512 &&
          try_split_wd<2, 9, 8, 8, 64, 2, 2, 1, 0, 1, 0, 0, 0, 2>(a, s, status))
        return 1;
      if (try_split_wd<2, 9, 8, 8, 64, 2, 2, 2, 0, 1>(a, s, status)) return 1;
      return try_split_wd<2, 9, 8, 8, 64, 2, 2, 2>(a, s, status);
    }
    // one kernel row of a 7x7 (functional.kxk_row_packs): 8 x 14 halo
    if (a.ntaps == 7) {   // (96 channels per workgroup where the count allows, as for 3x3; bit-identical)
      if (wd_env("LIC_WD_BN96", 1) && a.copad % 96 == 0 && try_split_wd<2, 7, 8, 8, 96, 2, 3, 2, 0, 0, 0, 3>(a, s, status))
        return 1;
      return try_split_wd<2, 7, 8, 8, 64, 2, 2, 2>(a, s, status);
    }
    // stride-2 phases (5x5: 9/6/6/4 taps, 3x3: 4/2/2/1) and ConvT phases onto small maps: compile-time
    // tap grids (3x2 / 2x3 / 2x2 / 1x2 / 2x1) where the taps form one, else the general addressing
    if (a.ntaps == 6)
      return try_split_wd<2, 6, 8, 8, 64, 2, 2, 2, 0, 1, 2>(a, s, status) ||
             try_split_wd<2, 6, 8, 8, 64, 2, 2, 2, 0, 1, 3>(a, s, status) || try_split_wd<2, 6, 8, 8, 64, 2, 2, 2>(a, s, status);
    if (a.ntaps == 4)
      return try_split_wd<2, 4, 8, 8, 64, 2, 2, 2, 0, 1>(a, s, status) || try_split_wd<2, 4, 8, 8, 64, 2, 2, 2>(a, s, status);
    if (a.ntaps == 2)
      return try_split_wd<2, 2, 8, 8, 64, 2, 2, 2, 0, 1, 2>(a, s, status) ||
             try_split_wd<2, 2, 8, 8, 64, 2, 2, 2, 0, 1, 1>(a, s, status) || try_split_wd<2, 2, 8, 8, 64, 2, 2, 2>(a, s, status);
  }
  return 0;
}

}  // namespace lic
