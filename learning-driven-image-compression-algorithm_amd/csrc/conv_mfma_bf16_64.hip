// Instantiations of the generic implicit-GEMM conv (conv_mfma.h): bf16, BM = 64.
#include "conv_mfma.h"

namespace lic {

template int launch_mfma<bf16_t, 64, 192, 2, 2>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 64, 128, 2, 2>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 64, 96, 2, 1>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 64, 64, 2, 1>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 64, 32, 2, 1>(const lic_conv_args&, int, hipStream_t);

}  // namespace lic
