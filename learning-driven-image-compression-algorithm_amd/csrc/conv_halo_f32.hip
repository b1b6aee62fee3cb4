// Instantiation of the halo conv (conv_halo.h) for f32.
#include "conv_halo.h"

namespace lic {

template int conv_halo_dispatch<float>(const lic_conv_args&, hipStream_t, int&);

}  // namespace lic
