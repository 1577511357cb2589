// Host-only stand-in for <hip/hip_runtime.h>: lets tests/hostsim compile the device
// interpreter (pdeval_kernels.h / pdeval_tier2.h) as plain C++ for one lane, so its
// arithmetic can be checked on the CPU (test infrastructure; not a compatibility layer for
// the product, which is only ever built by hipcc for gfx950).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#define __host__
#define __device__
#define __global__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
#define __shared__
struct pd_dim3 { unsigned x = 0, y = 0, z = 0; };
static pd_dim3 threadIdx, blockIdx, blockDim, gridDim;
inline double __shfl_xor(double v, int, int) { return v; }
inline int __shfl_xor(int v, int, int) { return v; }
inline bool __any(bool v) { return v; }
inline unsigned long long __ballot(bool v) { return v ? 1ull : 0ull; }
inline unsigned long long __builtin_amdgcn_ballot_w64(bool v) { return v ? 1ull : 0ull; }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
inline double __builtin_amdgcn_rcp(double v) { return 1.0 / v; }   // (v_rcp_f64: ~1 ulp)
inline void __builtin_amdgcn_sched_barrier(int) {}
inline int atomicAdd(int32_t* p, int v) { int o = *p; *p += v; return o; }
inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { uint32_t o = *p; *p += v; return o; }
inline uint32_t atomicOr(uint32_t* p, uint32_t v) { uint32_t o = *p; *p |= v; return o; }
inline uint32_t atomicAnd(uint32_t* p, uint32_t v) { uint32_t o = *p; *p &= v; return o; }
inline unsigned long long atomicMax(unsigned long long* p, unsigned long long v) {
    unsigned long long o = *p; if (v > o) *p = v; return o; }
inline void __threadfence() {}
inline long long __double_as_longlong(double v) { long long r; __builtin_memcpy(&r, &v, 8); return r; }
inline double __longlong_as_double(long long v) { double r; __builtin_memcpy(&r, &v, 8); return r; }
inline double __hiloint2double(int hi, int lo) {
    uint64_t b = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
    double d;
    std::memcpy(&d, &b, 8);
    return d;
}
using std::fmax;
using std::isfinite;
#define __align__(n) __attribute__((aligned(n)))
// the kernels' dynamic LDS (not used by the simulation, which calls the interpreters only)
#define PD_HOST_SIM_LDS
