// pdeval_launch.h -- launchers of kernels compiled in their own translation units: the rare
// point-stage kernels (pdeval_point.hip: the double-double and complex kernels are large) and
// the lean grid pass (pdeval_grid.hip); separate units build in parallel with pdeval.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "pdeval_kernels.h"

namespace pd {
// point stage over a device list, one candidate per lane: cplx = 0 real (deep programs),
// 1 complex (force-free only)
void launch_point_list(int problem, int cplx, unsigned grid, hipStream_t s, const KernelArgs& a);
// double-double tier over a device list: kind 0 real programs of stack <= 2 (LDS stack),
// 1 deeper real programs, 2 complex (force-free only)
// defer: the early tier's kernels (classes to a.ddps, dd_apply_kernel applies them)
void launch_dd_point(int problem, int kind, unsigned grid, hipStream_t s, const KernelArgs& a, bool defer = false);
void launch_dd_apply(int problem, unsigned grid, hipStream_t s, const KernelArgs& a);
// diagnostic: one program at the reference points in precision tier 0..3 (pdeval_point_eval)
void launch_point_eval(int problem, int tier, hipStream_t s, const KernelArgs& a, const int32_t* prog,
                       int plen, double* out, uint8_t* state);
// the lean grid passes (pdeval_grid.hip): pass 1 over all n candidates (one wave each, stack
// <= 2), pass 2 persistent over the stack-3 list a.list (64-thread blocks)
// the lean passes' coordinate-power tables (pdeval_grid.h ptab_kernel): size, and the build
// from the grid abscissae / ordinates of a context (once, at creation)
size_t ptab_bytes(int problem, int nx, int ny);
void launch_ptab(int problem, const double* gx, const double* gy, int nx, int ny, double* tab, hipStream_t s);
// decode every program for the lean passes (pdeval_grid.h decode_kernel) into a.dec
void launch_decode(int problem, int64_t n, hipStream_t s, const KernelArgs& a);
// waves per candidate of the lean grid passes for a batch of n (small batches split each
// candidate's rows over several waves, pdeval_grid.h grid_body)
int grid_parts(int64_t n);
void launch_grid(int problem, int64_t n, hipStream_t s, const KernelArgs& a,
                 int64_t* slow_list, int32_t* slow_count);
// the complex pass (force-free): persistent over the list a.list (L_CPLX), complex jets
void launch_grid_cplx(unsigned blocks, hipStream_t s, const KernelArgs& a, int64_t* slow_list, int32_t* slow_count,
                      int parts);
void launch_grid_list(int problem, unsigned blocks, hipStream_t s, const KernelArgs& a,
                      int64_t* slow_list, int32_t* slow_count, int parts);
// sort the batch by opcode sequence (pdeval_sort.hip): keys/idx hold 2 x n each, the
// permutation ends in idx + n
size_t sort_temp_bytes(int64_t cap);
int sort_batch(const int32_t* ops, const int64_t* offsets, int64_t n_words, int64_t n, uint64_t* keys,
               int32_t* idx, void* temp, size_t temp_bytes, hipStream_t s);
}  // namespace pd
