// pdeval_grid.hip -- the lean grid pass (pdeval_grid.h) in its own translation unit: the hot
// kernel of the library builds (and is tuned) apart from the rest.
#include <hip/hip_runtime.h>

#include "pdeval_grid.h"
#include "pdeval_launch.h"

namespace pd {

void launch_grid(int problem, int64_t n, hipStream_t s, const KernelArgs& a,
                 int64_t* slow_list, int32_t* slow_count) {
    const unsigned blocks = (unsigned)((n + PD_GRID_WPB - 1) / PD_GRID_WPB);
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_FORCE_FREE>), dim3(blocks), dim3(64 * PD_GRID_WPB),
                           (grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 2>(PD_GRID_WPB)), s, a, slow_list, slow_count);
    else
        hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_KERR>), dim3(blocks), dim3(64 * PD_GRID_WPB),
                           (grid_lds<PDEVAL_PROBLEM_KERR, 2>(PD_GRID_WPB)), s, a, slow_list, slow_count);
}

size_t ptab_bytes(int problem, int nx, int ny) {
    return sizeof(double) * (problem == PDEVAL_PROBLEM_FORCE_FREE ? ptab_doubles<4>(nx, ny) : ptab_doubles<2>(nx, ny));
}

void launch_ptab(int problem, const double* gx, const double* gy, int nx, int ny, double* tab, hipStream_t s) {
    const unsigned blocks = (unsigned)(((int64_t)PTAB_N * (nx + ny) + 255) / 256);
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((ptab_kernel<4>), dim3(blocks), dim3(256), 0, s, gx, gy, nx, ny, tab);
    else
        hipLaunchKernelGGL((ptab_kernel<2>), dim3(blocks), dim3(256), 0, s, gx, gy, nx, ny, tab);
}

void launch_decode(int problem, int64_t n, hipStream_t s, const KernelArgs& a) {
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((decode_kernel<PDEVAL_PROBLEM_FORCE_FREE>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((decode_kernel<PDEVAL_PROBLEM_KERR>), dim3(blocks), dim3(256), 0, s, a);
}

void launch_grid_cplx(unsigned blocks, hipStream_t s, const KernelArgs& a, int64_t* slow_list, int32_t* slow_count) {
    hipLaunchKernelGGL(grid_cplx_kernel, dim3(blocks), dim3(64), (grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 2, cplx>(1)), s,
                       a, slow_list, slow_count);
}

void launch_grid_list(int problem, unsigned blocks, hipStream_t s, const KernelArgs& a,
                      int64_t* slow_list, int32_t* slow_count) {
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_FORCE_FREE>), dim3(blocks), dim3(64),
                           (grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 3>(1)), s, a, slow_list, slow_count);
    else
        hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_KERR>), dim3(blocks), dim3(64),
                           (grid_lds<PDEVAL_PROBLEM_KERR, 3>(1)), s, a, slow_list, slow_count);
}

}  // namespace pd
