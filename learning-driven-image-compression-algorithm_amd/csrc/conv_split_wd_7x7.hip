// Weights-direct split convolutions: 7x7 on 16x16-px tiles, 8 waves, 22x22 halo (conv_split_wd.h).
#include "conv_split_wd.h"

namespace lic {

int wd_dispatch_7x7(const lic_conv_args& a, hipStream_t s, int& status) {
  const int bn192 = wd_env("LIC_WD_BN192", 1);   // 192 channels per workgroup: 1846.8 -> 1756.0 us (wd_ab.txt)
  const int64_t blocks = (int64_t)a.n * ((a.mi + 15) / 16) * ((a.mj + 15) / 16) * (a.copad / 64);
  if (!(a.mi > 8 && a.mj > 8 && blocks >= 256)) return 0;
  if (bn192 && a.copad == 192 && try_split_wd<2, 49, 16, 16, 192, 4, 2, 4, 0, 1, 0, 2, 2>(a, s, status)) return 1;
  return try_split_wd<2, 49, 16, 16, 64, 4, 2, 4, 0, 1>(a, s, status) || try_split_wd<2, 49, 16, 16, 64, 4, 2, 4>(a, s, status);
}

}  // namespace lic
