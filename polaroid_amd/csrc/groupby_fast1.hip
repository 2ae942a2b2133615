// Explicit instantiations of the fused group-by kernel's launches for
// 0 and 1 aggregated columns (groupby_kernels.hpp).
#define PLGPU_GB_FAST_TU
#include "groupby_kernels.hpp"

namespace plgpu {
template hipError_t launch_fast_nacc<0, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<0, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<1, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<1, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<1, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<1, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_part_fast_limbs<1>(const Plan&, int, hipStream_t);
template hipError_t launch_fast_nulls<0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nulls<1>(const Plan&, const DevProgram&, int, hipStream_t);
}  // namespace plgpu
