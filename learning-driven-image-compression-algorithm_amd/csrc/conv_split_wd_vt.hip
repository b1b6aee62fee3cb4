// Weights-direct split convolutions: 1x1 launches on big maps as "virtual taps" (conv_split_wd.h).
#include "conv_split_wd.h"

namespace lic {

int wd_dispatch_vt(const lic_conv_args& a, hipStream_t s, int& status) {
  // 8x16 px x 192 channels, two 16-channel chunks per barrier (16x16 px tiles on 8 waves or on 4 waves
  // at one per SIMD measured 1-40 % slower, profiles/r04/wd_ab.txt)
  return try_split_wd<2, 2, 8, 16, 192, 2, 2, 4, 2, 1>(a, s, status) || try_split_wd<2, 2, 8, 16, 192, 2, 2, 4, 2>(a, s, status);
}

}  // namespace lic
