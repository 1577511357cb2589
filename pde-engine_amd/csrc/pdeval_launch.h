// pdeval_launch.h -- launchers of the rare point-stage kernels, compiled in their own
// translation unit (pdeval_point.hip: the double-double and complex kernels are large, and a
// separate unit builds in parallel with pdeval.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "pdeval_kernels.h"

namespace pd {
// point stage over a device list, one candidate per lane: cplx = 0 real (deep programs),
// 1 complex (force-free only)
void launch_point_list(int problem, int cplx, unsigned grid, hipStream_t s, const KernelArgs& a);
// double-double tier over a device list: kind 0 real programs of stack <= 2 (LDS stack),
// 1 deeper real programs, 2 complex (force-free only)
void launch_dd_point(int problem, int kind, unsigned grid, hipStream_t s, const KernelArgs& a);
// diagnostic: one program at the reference points in precision tier 0..3 (pdeval_point_eval)
void launch_point_eval(int problem, int tier, hipStream_t s, const KernelArgs& a, const int32_t* prog,
                       int plen, double* out, uint8_t* state);
}  // namespace pd
