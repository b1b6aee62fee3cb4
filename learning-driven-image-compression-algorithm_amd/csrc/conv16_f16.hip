// Instantiations of the conv16 kernel (conv16.h) for f16.
#include "conv16.h"

namespace lic {

template <typename T> int conv16_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
template <> int conv16_dispatch<half_t>(const lic_conv_args& a, hipStream_t s, int& status) {
  return conv16_dispatch_impl<half_t>(a, s, status);
}

}  // namespace lic
