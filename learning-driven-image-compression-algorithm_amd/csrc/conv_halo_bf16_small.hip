// Instantiations of the halo conv (conv_halo.h) for bf16: small tiles.
#include "conv_halo.h"

namespace lic {

template int try_halo<bf16_t, 16, 16, 64, 4, 2>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 16, 16, 32, 8, 1>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 8, 8, 64, 2, 2>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 8, 8, 32, 2, 1>(const lic_conv_args&, hipStream_t, int&);

}  // namespace lic
