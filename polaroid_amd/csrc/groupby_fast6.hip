// Explicit instantiations of the fused group-by kernel's launches for
// 6 aggregated columns (groupby_kernels.hpp).
#define PLGPU_GB_FAST_TU
#include "groupby_kernels.hpp"

namespace plgpu {
template hipError_t launch_fast_nacc<6, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<6, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<6, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_fast_nacc<6, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
template hipError_t launch_part_fast_limbs<6>(const Plan&, int, hipStream_t);
template hipError_t launch_fast_nulls<6>(const Plan&, const DevProgram&, int, hipStream_t);
}  // namespace plgpu
