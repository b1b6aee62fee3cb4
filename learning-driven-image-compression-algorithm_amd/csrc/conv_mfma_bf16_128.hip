// Instantiations of the generic implicit-GEMM conv (conv_mfma.h): bf16, BM = 128.
#include "conv_mfma.h"

namespace lic {

template int launch_mfma<bf16_t, 128, 192, 2, 2>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 128, 128, 2, 2>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 128, 96, 4, 1>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 128, 64, 4, 1>(const lic_conv_args&, int, hipStream_t);
template int launch_mfma<bf16_t, 128, 32, 4, 1>(const lic_conv_args&, int, hipStream_t);

}  // namespace lic
