// SumTree.update bookkeeping shared by the PER launches (per.hip) and the launches that host
// parts of it on the single-GPU PER learn step: the head kernel does k_per_prep's work for its
// samples, the weight-gradient launch runs k_per_prop's workgroups beside its tiles (fused.hip,
// learn.hip).  Exactness and ordering: per.hip's header.
#pragma once
#include "learn.hpp"

namespace dqnx {

constexpr int PER_TOP = 2047;   // nodes of depth <= 10, accumulated in LDS before the global atomics
constexpr int PER_GT = 256;     // threads per workgroup of the grid launches

// numpy: np.power(np.minimum(abs_td + eps, 1.0), alpha) on float32 (python floats are cast to
// float32).  The power is correctly rounded (float64 pow rounded once), which is what glibc's
// powf returns except in rare hard cases; numpy >= 1.22 on AVX-512 hosts may use SVML
// instead (within 1 ulp).  See DESIGN.md.
__device__ __forceinline__ float per_priority(float d, float eps, float alpha, float pmax) {
    float x = d + eps;
    x = (x > pmax) ? pmax : x;   // NaN propagates like np.minimum
    return (float)pow((double)x, (double)alpha);
}

// update i of a mode-0 chunk (update_batch_priorities, R:dqn/replay_memory.py:94-98): its leaf,
// new priority and the leaf's value before the chunk, and the slot's latest-writer tag (epoch + 1:
// k_per_update advances the epoch when it has consumed the chunk)
__device__ __forceinline__ void per_prep_item(const PerUpdateArgs& a, int i, float abs_td) {
    const int64_t base = a.cap - 1;
    const int64_t slot = (int64_t)a.slots[i];
    const int32_t L = (int32_t)(slot + base);
    a.wl[i] = L;
    a.wp[i] = per_priority(abs_td, a.eps, a.alpha, a.pmax);
    a.winit[i] = a.tree[L];
    const uint64_t e = (uint64_t)(*a.epoch + 1u);
    atomicMax((unsigned long long*)&a.last[slot], (unsigned long long)((e << 32) | (uint32_t)i));
}

// k_per_prop's body for updates [i0, i0 + blockDim.x): each slot's last update writes the final
// leaf and adds (final - old) to every ancestor, the top PER_TOP nodes summed in `topd` (LDS,
// PER_TOP doubles) first.  Exact in any order (per.hip's header).  Every thread of the workgroup
// calls it (barriers inside).
__device__ __forceinline__ void per_prop_block(const PerUpdateArgs& a, int i0, double* topd) {
    const int tid = threadIdx.x;
    for (int h = tid; h < PER_TOP; h += blockDim.x) topd[h] = 0.0;
    __syncthreads();
    const int i = i0 + tid;
    const int64_t base = a.cap - 1;
    if (i < a.n) {
        const int64_t L = a.wl[i];
        const uint64_t tag = ((uint64_t)*a.epoch << 32) | (uint32_t)i;
        if (a.last[L - base] == tag) {   // the slot's final value
            const double fin = (double)a.wp[i];
            a.tree[L] = fin;
            const double delta = fin - a.winit[i];
            if (delta != 0.0) {
                int64_t node = L;
                while (node > 0) {
                    node = (node - 1) >> 1;
                    if (node < PER_TOP) atomicAdd(&topd[node], delta);
                    else atomicAdd(&a.tree[node], delta);
                }
            }
        }
    }
    __syncthreads();
    for (int node = tid; node < PER_TOP && node < base; node += blockDim.x)
        if (topd[node] != 0.0) atomicAdd(&a.tree[node], topd[node]);
}

}  // namespace dqnx
