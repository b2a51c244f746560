// one arithmetic mode of the halo-tiled 3x3 conv kernel per translation unit (conv_halo_kernel.h)
#include "conv_halo_kernel.h"

namespace vstk {
template void launch_halo_prec<1>(bool, int, int, dim3, hipStream_t, const ConvParams&);
}  // namespace vstk
