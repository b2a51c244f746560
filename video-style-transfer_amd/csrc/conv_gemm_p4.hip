// Instantiation of the implicit-GEMM conv kernels for GEMM arithmetic mode 4
// (fp16 MFMA); one mode per translation unit keeps the build parallel.
#include "conv_gemm_kernel.h"

namespace vstk {
template void launch_prec<4>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
}  // namespace vstk
