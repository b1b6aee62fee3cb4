// Weights-direct split convolutions on 16x16-px tiles (conv_split_wd.h): the k x k convolutions, stride-2
// phases and transposed-conv phases of the 64x64 / 128x128 maps.
#include "conv_split_wd.h"

namespace lic {

int wd_dispatch_big(const lic_conv_args& a, hipStream_t s, int& status) {
  // 192 output channels per workgroup (8 waves, 4 x 2, two 32x32 x three accumulator tiles each): the
  // halo of a tile is read and split once instead of once per 64-channel block (3x3 @64^2 376.6 ->
  // 360.4 us; profiles/r04/wd_ab.txt).  A/B: LIC_WD_BN192=0 (64-channel blocks)
  const int bn192 = wd_env("LIC_WD_BN192", 1);
  auto blocks = [&](int th, int tw, int bn) {
    return (int64_t)a.n * ((a.mi + th - 1) / th) * ((a.mj + tw - 1) / tw) * (a.copad / bn);
  };
  if (!(a.mi > 8 && a.mj > 8 && blocks(16, 16, 64) >= 256)) return 0;
  switch (a.ntaps) {
    case 9:   // 3x3 grids (stride 1, stride-2 phases, ConvT phases): compile-time addressing (GEO 1), else general
      if (bn192 && a.copad == 192 && try_split_wd<2, 9, 16, 16, 192, 4, 2, 3, 0, 1, 0, 2, 2>(a, s, status)) return 1;
      // 96 channels (the ResidualBottleneck's 3x3 at 64^2): one 4-wave workgroup per tile instead of two
      // 64-channel blocks, the second half empty (per-element arithmetic unchanged).  A/B: LIC_WD_BN96=0
      if (a.copad == 96 && wd_env("LIC_WD_BN96", 1) && try_split_wd<2, 9, 16, 16, 96, 4, 1, 6, 0, 1, 0, 2, 2>(a, s, status))
        return 1;
      if (try_split_wd<2, 9, 16, 16, 64, 2, 2, 6, 0, 1>(a, s, status)) return 1;
      return try_split_wd<2, 9, 16, 16, 64, 2, 2, 6>(a, s, status);
    case 6:   // 3x2 / 2x3 phases (ConvT, stride-2); 192 channels per workgroup as for 3x3 (LIC_WD_BN192)
      if (bn192 && a.copad == 192 && (try_split_wd<2, 6, 16, 16, 192, 4, 2, 3, 0, 1, 2, 2, 2>(a, s, status) ||
                                      try_split_wd<2, 6, 16, 16, 192, 4, 2, 3, 0, 1, 3, 2, 2>(a, s, status)))
        return 1;
      return try_split_wd<2, 6, 16, 16, 64, 2, 2, 6, 0, 1, 2>(a, s, status) ||
             try_split_wd<2, 6, 16, 16, 64, 2, 2, 6, 0, 1, 3>(a, s, status) ||
             try_split_wd<2, 6, 16, 16, 64, 2, 2, 6>(a, s, status);
    case 4:   // 2x2 phases
      if (bn192 && a.copad == 192 && try_split_wd<2, 4, 16, 16, 192, 4, 2, 3, 0, 1, 0, 2, 2>(a, s, status)) return 1;
      return try_split_wd<2, 4, 16, 16, 64, 2, 2, 6, 0, 1>(a, s, status) || try_split_wd<2, 4, 16, 16, 64, 2, 2, 6>(a, s, status);
    case 2:   // 3x3 s2 phases 1x2 / 2x1
      return try_split_wd<2, 2, 16, 16, 64, 2, 2, 6, 0, 1, 2>(a, s, status) ||
             try_split_wd<2, 2, 16, 16, 64, 2, 2, 6, 0, 1, 1>(a, s, status) || try_split_wd<2, 2, 16, 16, 64, 2, 2, 6>(a, s, status);
    default: break;
  }
  return 0;
}

}  // namespace lic
