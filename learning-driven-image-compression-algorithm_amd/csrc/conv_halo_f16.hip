// Instantiation of the halo conv (conv_halo.h) for f16.
#include "conv_halo.h"

namespace lic {

template int conv_halo_dispatch<half_t>(const lic_conv_args&, hipStream_t, int&);

}  // namespace lic
