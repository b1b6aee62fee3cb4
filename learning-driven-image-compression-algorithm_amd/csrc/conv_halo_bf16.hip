// Instantiations of the halo conv (conv_halo.h) for bf16: large tiles.
#include "conv_halo.h"

namespace lic {

template int try_halo<bf16_t, 32, 16, 192, 4, 2>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 32, 16, 64, 8, 1>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 16, 16, 192, 4, 2>(const lic_conv_args&, hipStream_t, int&);
template int try_halo<bf16_t, 16, 16, 128, 4, 2>(const lic_conv_args&, hipStream_t, int&);

}  // namespace lic
