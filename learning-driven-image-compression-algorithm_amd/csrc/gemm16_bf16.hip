// Instantiations of the gemm16 kernel (gemm16.h) for bf16.
#include "gemm16.h"

namespace lic {

template <typename T> int gemm16_dispatch(const lic_conv_args& a, hipStream_t s, int& status);
template <> int gemm16_dispatch<bf16_t>(const lic_conv_args& a, hipStream_t s, int& status) {
  return gemm16_dispatch_impl<bf16_t>(a, s, status);
}

}  // namespace lic
