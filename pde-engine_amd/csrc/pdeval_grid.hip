// pdeval_grid.hip -- the lean grid pass (pdeval_grid.h) in its own translation unit: the hot
// kernel of the library builds (and is tuned) apart from the rest.
#include <hip/hip_runtime.h>

#include "pdeval_grid.h"
#include "pdeval_launch.h"

namespace pd {

void launch_grid(int problem, unsigned blocks, size_t lds, hipStream_t s, const KernelArgs& a,
                 int64_t* slow_list, int32_t* slow_count) {
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_FORCE_FREE>), dim3(blocks), dim3(256), lds, s, a,
                           slow_list, slow_count);
    else
        hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_KERR>), dim3(blocks), dim3(256), lds, s, a, slow_list,
                           slow_count);
}

}  // namespace pd
