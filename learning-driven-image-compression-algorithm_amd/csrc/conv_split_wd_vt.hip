// Weights-direct split convolutions: 1x1 launches on big maps as "virtual taps" (conv_split_wd.h).
#include "conv_split_wd.h"

namespace lic {

int wd_dispatch_vt(const lic_conv_args& a, hipStream_t s, int& status) {
  // experiment switch LIC_WD_VT: 1 = 16x16 px x 192 on 8 waves; 2 = 16x16 px x 192 on 4 waves (one per SIMD)
  const int vt = wd_env("LIC_WD_VT", 0);
  if (vt == 1 && a.mi >= 16 && try_split_wd<2, 2, 16, 16, 192, 4, 2, 4, 2, 1, 0, 2, 2>(a, s, status)) return 1;
  if (vt == 2 && a.mi >= 16 && try_split_wd<2, 2, 16, 16, 192, 2, 2, 8, 2, 1, 0, 1, 2>(a, s, status)) return 1;
  // 8x16 px x 192 channels, two 16-channel chunks per barrier
  return try_split_wd<2, 2, 8, 16, 192, 2, 2, 4, 2, 1>(a, s, status) || try_split_wd<2, 2, 8, 16, 192, 2, 2, 4, 2>(a, s, status);
}

}  // namespace lic
