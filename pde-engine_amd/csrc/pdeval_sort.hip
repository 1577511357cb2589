// pdeval_sort.hip -- the order in which the one-candidate-per-lane kernels take the batch.
//
// Pass 0 and the double-double tier interpret a different program in every lane, so a wave
// executes the union of its lanes' opcode paths.  In the stream's own order neighbouring
// candidates share their opcode sequences; in a shuffled batch they do not, and the same step
// measured 113.5 ms against 107.4 ms (profiles/r02_bench_ff_order_*.log).  This unit sorts the
// batch by opcode sequence (a 60-bit key: the first ten opcodes, six bits each, first opcode
// most significant) into a permutation that pass 0 and the tier-B collect pass walk, so lanes
// of one wave take programs with a common prefix whatever the input order.  The sort is a
// rocPRIM/hipCUB radix sort on the launch stream with preallocated scratch: no host sync, so
// pdeval_validate_device stays graph-capturable.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include "pdeval_kernels.h"

namespace pd {

constexpr int kKeyOps = 10;   // opcodes in the key (6 bits each)

__global__ __launch_bounds__(256) void shape_key_kernel(const int32_t* ops, const int64_t* offsets, int64_t n_words,
                                                        int64_t n, uint64_t* keys, int32_t* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t beg = offsets[i], end = offsets[i + 1];
    uint64_t key = (1ull << (6 * kKeyOps)) - 1;   // malformed programs last
    if (beg >= 0 && end > beg && end <= n_words && end - beg < (1 << 24)) {
        key = 0;
        int64_t pc = beg + 1;
        int k = 0;
        for (; k < kKeyOps && pc < end; ++k) {
            const uint32_t w = (uint32_t)ops[pc];
            const uint32_t op = w & 0xffu;
            key = (key << 6) | (op & 63u);
            pc += op_has_imm(op) ? ((w & PDEVAL_IMM_DD) ? 5 : 3) : 1;
        }
        key <<= 6 * (kKeyOps - k);
    }
    keys[i] = key;
    idx[i] = (int32_t)i;
}

size_t sort_temp_bytes(int64_t cap) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, (int)cap, 0,
                                             6 * kKeyOps);
    return bytes;
}

// keys/idx: 2 x n each (in, out); the permutation ends in idx + n.  Returns a hipError_t.
int sort_batch(const int32_t* ops, const int64_t* offsets, int64_t n_words, int64_t n, uint64_t* keys,
               int32_t* idx, void* temp, size_t temp_bytes, hipStream_t s) {
    hipLaunchKernelGGL(shape_key_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ops, offsets, n_words, n,
                       keys, idx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    return (int)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys + n, idx, idx + n, (int)n, 0,
                                                   6 * kKeyOps, s);
}

}  // namespace pd
