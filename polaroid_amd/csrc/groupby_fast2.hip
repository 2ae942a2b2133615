// Explicit instantiations of the fused group-by kernel's launches for
// 2 aggregated columns (groupby_kernels.hpp).
#define PLGPU_GB_FAST_TU
#include "groupby_kernels.hpp"

namespace plgpu {
template hipError_t launch_fast_nacc<2, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<2, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<2, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<2, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_part_fast_limbs<2>(const Plan&, int, hipStream_t);
template hipError_t launch_fast_pair<0, 2>(const Plan&, const DevProgram&, hipStream_t);
template hipError_t launch_fast_pair<1, 2>(const Plan&, const DevProgram&, hipStream_t);
template hipError_t launch_fast_pair<0, 3>(const Plan&, const DevProgram&, hipStream_t);
template hipError_t launch_fast_pair<1, 3>(const Plan&, const DevProgram&, hipStream_t);
template hipError_t launch_fast_nulls<2>(const Plan&, const DevProgram&, int, hipStream_t);
}  // namespace plgpu
