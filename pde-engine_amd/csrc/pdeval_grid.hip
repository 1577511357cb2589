// pdeval_grid.hip -- the lean grid pass (pdeval_grid.h) in its own translation unit: the hot
// kernel of the library builds (and is tuned) apart from the rest.
#include <hip/hip_runtime.h>

#include "pdeval_grid.h"
#include "pdeval_launch.h"

namespace pd {

int grid_parts(int64_t n) {
    // waves per candidate of the lean grid passes: 1 for batches that fill the chip; small
    // batches split each candidate's 64 rows over up to 16 waves (~2k waves in flight)
    int p = 1;
    while (p < 16 && n * p * 2 <= 2048) p *= 2;
    return p;
}

void launch_grid(int problem, int64_t n, hipStream_t s, const KernelArgs& a,
                 int64_t* slow_list, int32_t* slow_count) {
    const int parts = grid_parts(n);
    const unsigned blocks = (unsigned)((n * parts + PD_GRID_WPB - 1) / PD_GRID_WPB);
    const size_t lff = grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 2>(PD_GRID_WPB), lk = grid_lds<PDEVAL_PROBLEM_KERR, 2>(PD_GRID_WPB);
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        if (a.prm.omega2 != 0.0)   // rotating field lines: the ROT instance (any parts)
            hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_FORCE_FREE, true, true>), dim3(blocks), dim3(64 * PD_GRID_WPB),
                               lff, s, a, slow_list, slow_count, parts);
        else if (parts > 1)
            hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_FORCE_FREE, true>), dim3(blocks), dim3(64 * PD_GRID_WPB), lff,
                               s, a, slow_list, slow_count, parts);
        else
            hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_FORCE_FREE, false>), dim3(blocks), dim3(64 * PD_GRID_WPB), lff,
                               s, a, slow_list, slow_count, 1);
    } else {
        if (parts > 1)
            hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_KERR, true>), dim3(blocks), dim3(64 * PD_GRID_WPB), lk, s, a,
                               slow_list, slow_count, parts);
        else
            hipLaunchKernelGGL((grid_kernel<PDEVAL_PROBLEM_KERR, false>), dim3(blocks), dim3(64 * PD_GRID_WPB), lk, s, a,
                               slow_list, slow_count, 1);
    }
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

void launch_grid_cplx(unsigned blocks, hipStream_t s, const KernelArgs& a, int64_t* slow_list, int32_t* slow_count,
                      int parts) {
    const size_t l = grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 2, cplx>(1);
    if (a.prm.omega2 != 0.0)
        hipLaunchKernelGGL((grid_cplx_kernel<true, true>), dim3(blocks), dim3(64), l, s, a, slow_list, slow_count, parts);
    else if (parts > 1)
        hipLaunchKernelGGL(grid_cplx_kernel<true>, dim3(blocks), dim3(64), l, s, a, slow_list, slow_count, parts);
    else
        hipLaunchKernelGGL(grid_cplx_kernel<false>, dim3(blocks), dim3(64), l, s, a, slow_list, slow_count, 1);
}

void launch_grid_list(int problem, unsigned blocks, hipStream_t s, const KernelArgs& a,
                      int64_t* slow_list, int32_t* slow_count, int parts) {
    const size_t lff = grid_lds<PDEVAL_PROBLEM_FORCE_FREE, 3>(1), lk = grid_lds<PDEVAL_PROBLEM_KERR, 3>(1);
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        if (a.prm.omega2 != 0.0)
            hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_FORCE_FREE, true, true>), dim3(blocks), dim3(64), lff, s,
                               a, slow_list, slow_count, parts);
        else if (parts > 1)
            hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_FORCE_FREE, true>), dim3(blocks), dim3(64), lff, s, a,
                               slow_list, slow_count, parts);
        else
            hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_FORCE_FREE, false>), dim3(blocks), dim3(64), lff, s, a,
                               slow_list, slow_count, 1);
    } else {
        if (parts > 1)
            hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_KERR, true>), dim3(blocks), dim3(64), lk, s, a,
                               slow_list, slow_count, parts);
        else
            hipLaunchKernelGGL((grid_list_kernel<PDEVAL_PROBLEM_KERR, false>), dim3(blocks), dim3(64), lk, s, a,
                               slow_list, slow_count, 1);
    }
}

}  // namespace pd
