// Instantiation of the implicit-GEMM conv kernels for GEMM arithmetic mode 2
// (bf16 MFMA); one mode per translation unit keeps the build parallel.
#include "conv_gemm_kernel.h"

namespace vstk {
template void launch_prec<2>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
}  // namespace vstk
