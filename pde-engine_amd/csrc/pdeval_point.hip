// pdeval_point.hip -- the rare point-stage kernels (pdeval_point.h) in their own translation
// unit: the deep / complex list passes and the double-double tier.
#include <hip/hip_runtime.h>

#include "pdeval_launch.h"
#include "pdeval_point.h"

namespace pd {

void launch_point_list(int problem, int cplx, unsigned grid, hipStream_t s, const KernelArgs& a) {
    if (problem == PDEVAL_PROBLEM_FORCE_FREE) {
        if (cplx) hipLaunchKernelGGL((point_list_kernel<PDEVAL_PROBLEM_FORCE_FREE, pd::cplx>), dim3(grid), dim3(64), 0, s, a);
        else hipLaunchKernelGGL((point_list_kernel<PDEVAL_PROBLEM_FORCE_FREE, double>), dim3(grid), dim3(64), 0, s, a);
    } else {
        hipLaunchKernelGGL((point_list_kernel<PDEVAL_PROBLEM_KERR, double>), dim3(grid), dim3(64), 0, s, a);
    }
}

void launch_dd_point(int problem, int kind, unsigned grid, hipStream_t s, const KernelArgs& a, bool defer) {
    constexpr int FF = PDEVAL_PROBLEM_FORCE_FREE, KR = PDEVAL_PROBLEM_KERR;
    const size_t lds_ff = (size_t)nc(4) * 64 * sizeof(dd), lds_kr = (size_t)nc(2) * 64 * sizeof(dd);
    constexpr int M8 = PDEVAL_MAX_STACK;
    if (problem == FF) {
        if (kind == 0) {
            if (defer) hipLaunchKernelGGL((dd_point_kernel<FF, dd, 2, true>), dim3(grid), dim3(64), lds_ff, s, a);
            else hipLaunchKernelGGL((dd_point_kernel<FF, dd, 2>), dim3(grid), dim3(64), lds_ff, s, a);
        } else if (kind == 1) {
            if (defer) hipLaunchKernelGGL((dd_point_kernel<FF, dd, M8, true>), dim3(grid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((dd_point_kernel<FF, dd, M8>), dim3(grid), dim3(64), 0, s, a);
        } else {
            if (defer) hipLaunchKernelGGL((dd_point_kernel<FF, cdd, M8, true>), dim3(grid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((dd_point_kernel<FF, cdd, M8>), dim3(grid), dim3(64), 0, s, a);
        }
    } else {
        if (kind == 0) {
            if (defer) hipLaunchKernelGGL((dd_point_kernel<KR, dd, 2, true>), dim3(grid), dim3(64), lds_kr, s, a);
            else hipLaunchKernelGGL((dd_point_kernel<KR, dd, 2>), dim3(grid), dim3(64), lds_kr, s, a);
        } else if (kind == 1) {
            if (defer) hipLaunchKernelGGL((dd_point_kernel<KR, dd, M8, true>), dim3(grid), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((dd_point_kernel<KR, dd, M8>), dim3(grid), dim3(64), 0, s, a);
        }
    }
}

void launch_dd_apply(int problem, unsigned grid, hipStream_t s, const KernelArgs& a) {
    if (problem == PDEVAL_PROBLEM_FORCE_FREE)
        hipLaunchKernelGGL((dd_apply_kernel<PDEVAL_PROBLEM_FORCE_FREE>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dd_apply_kernel<PDEVAL_PROBLEM_KERR>), dim3(grid), dim3(256), 0, s, a);
}

void launch_point_eval(int problem, int tier, hipStream_t s, const KernelArgs& a, const int32_t* prog, int plen,
                       double* out, uint8_t* state) {
    constexpr int FF = PDEVAL_PROBLEM_FORCE_FREE, KR = PDEVAL_PROBLEM_KERR;
    if (problem == FF) {
        if (tier == 0) hipLaunchKernelGGL((point_eval_kernel<FF, double, double, false>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
        else if (tier == 1) hipLaunchKernelGGL((point_eval_kernel<FF, pd::cplx, double, false>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
        else if (tier == 2) hipLaunchKernelGGL((point_eval_kernel<FF, dd, dd, true>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
        else hipLaunchKernelGGL((point_eval_kernel<FF, cdd, dd, true>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
    } else {
        if (tier == 0) hipLaunchKernelGGL((point_eval_kernel<KR, double, double, false>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
        else hipLaunchKernelGGL((point_eval_kernel<KR, dd, dd, true>), dim3(1), dim3(64), 0, s, a, prog, plen, out, state);
    }
}

}  // namespace pd
