// MT19937 pieces shared by the replay samplers (CPython random and numpy's legacy
// RandomState use the same generator, state layout (624 words + index) and tempering).
#pragma once
#include <stdint.h>

namespace dqnx {

constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_A = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    uint32_t y = (a & MT_UPPER) | (b & MT_LOWER);
    return (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}

// Block-parallel twist of the 624-word state in LDS (blockDim >= 624): the recurrence
// mt[k] = mt[k+397 or k-227] ^ mix(mt[k], mt[k+1]) has three dependency phases.
// Every thread of the block must call it.
__device__ __forceinline__ void mt_twist_block(uint32_t* mt, uint32_t* tmp) {
    const int tid = threadIdx.x;
    if (tid < 624) tmp[tid] = mt[tid];
    __syncthreads();
    if (tid < 227) mt[tid] = tmp[tid + 397] ^ mt_mix(tmp[tid], tmp[tid + 1]);
    __syncthreads();
    if (tid >= 227 && tid < 454) mt[tid] = mt[tid - 227] ^ mt_mix(tmp[tid], tmp[tid + 1]);
    __syncthreads();
    if (tid >= 454 && tid < 623) mt[tid] = mt[tid - 227] ^ mt_mix(tmp[tid], tmp[tid + 1]);
    if (tid == 623) mt[623] = mt[396] ^ mt_mix(tmp[623], mt[0]);
    __syncthreads();
}

// blk_new = twist(blk_old): CPython genrand_uint32's recurrence
//   new[k] = X ^ mix(old[k], old[k+1]),  X = old[k+397] (k < 227), new[k-227] (k >= 227).
// The dependency chain k -> k+227 -> k+454 stays inside thread k (< 227), in registers, so
// one barrier completes the twist; new[623] = new[396] ^ mix(old[623], new[0]) is done by
// thread 169, which owns new[396] and recomputes new[0] from `old`.
// Every thread of the block must call it.
__device__ __forceinline__ void mt_twist_into(const uint32_t* old, uint32_t* nw) {
    const int t = threadIdx.x;
    if (t < 227) {
        const uint32_t a0 = old[t + 397] ^ mt_mix(old[t], old[t + 1]);
        const uint32_t a1 = a0 ^ mt_mix(old[t + 227], old[t + 228]);
        nw[t] = a0;
        nw[t + 227] = a1;
        if (t < 169) nw[t + 454] = a1 ^ mt_mix(old[t + 454], old[t + 455]);
        if (t == 169) nw[623] = a1 ^ mt_mix(old[623], old[397] ^ mt_mix(old[0], old[1]));
    }
    __syncthreads();
}

// numpy MT block cache (learn.hpp, PerSampleArgs::npc): drop the blocks the last sample moved
// past, then twist forward until `target` blocks are held.  One workgroup (>= 227 threads);
// `mb` = LDS [2][624] + 2 ints.  Runs in a launch after the sample (no other reader or writer).
__device__ __forceinline__ void np_cache_extend(uint32_t* npc, const uint32_t* state, int target, uint32_t* mb) {
    const int tid = threadIdx.x, nt = blockDim.x;
    int* hdr = reinterpret_cast<int*>(mb + 2 * 624);
    uint32_t* blocks = npc + 64;
    if (tid == 0) {
        hdr[0] = (int)npc[0];
        hdr[1] = (int)npc[1];
    }
    __syncthreads();
    int cnt = hdr[0];
    const int sh = hdr[1];
    if (cnt <= 0 || sh >= cnt) {   // nothing usable: start again from the state block
        for (int j = tid; j < 624; j += nt) {
            const uint32_t x = state[j];
            mb[j] = x;
            blocks[j] = x;
        }
        cnt = 1;
    } else {
        // block b <- block b + sh in increasing b: a block is read before any lower block is written
        for (int b = 0; b < cnt - sh; b++)
            for (int j = tid; j < 624; j += nt) blocks[(int64_t)b * 624 + j] = blocks[(int64_t)(b + sh) * 624 + j];
        cnt -= sh;
        __syncthreads();   // (this thread's stores above are visible to its own loads; others' by the barrier)
        __threadfence_block();
        for (int j = tid; j < 624; j += nt) mb[j] = blocks[(int64_t)(cnt - 1) * 624 + j];
    }
    __syncthreads();
    int cur = 0;
    for (int b = cnt; b < target; b++) {
        mt_twist_into(mb + cur * 624, mb + (cur ^ 1) * 624);   // ends with a barrier
        cur ^= 1;
        for (int j = tid; j < 624; j += nt) blocks[(int64_t)b * 624 + j] = mb[cur * 624 + j];
    }
    if (tid == 0) {
        npc[0] = (uint32_t)(target > cnt ? target : cnt);
        npc[1] = 0u;
    }
}

}  // namespace dqnx
