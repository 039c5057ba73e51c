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

// In-launch hand-off when one launch hosts the tracking workgroup and the prop workgroups
// (k_dw_adam16): the tracking workgroup publishes the chunk epoch it has just advanced to; the prop
// workgroups, dispatched after it (so it is resident or finished while they wait), spin until the
// word holds THEIR chunk's epoch, which they read from the latest-writer tag the head kernel left on
// the slot of their first update (epoch + 1 in the high word, per_prep_item).  A publish is tied to
// its launch, so nothing needs resetting between launches and a publish that arrives late (after a
// timed-out wait) can never satisfy the next launch's wait.  The wait is bounded: past ~2^21 sleeps
// the prop workgroups go on with DQNX_DEVERR_PER_HANDOFF in ctrl.error (a broken launch shape
// reports instead of hanging the queue; their tag check then writes no leaf, and the Agent raises).
__device__ __forceinline__ void per_track_publish(const PerUpdateArgs& a) {
    __syncthreads();
    if (threadIdx.x == 0) {   // after thread 0's leaf / ctrl / epoch stores (per_track_block)
        const uint32_t ep = *(volatile uint32_t*)a.epoch;   // thread 0 advanced it
        __threadfence();
        __hip_atomic_store(a.sync, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ void per_prop_wait(const PerUpdateArgs& a, int i0) {
    if (threadIdx.x == 0 && i0 < a.n) {
        const int64_t slot = (int64_t)a.wl[i0] - (a.cap - 1);
        const uint32_t want = (uint32_t)(a.last[slot] >> 32);   // written by the previous launch
        uint32_t spins = 0;
        while (__hip_atomic_load(a.sync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want) {
            __builtin_amdgcn_s_sleep(4);
            if (++spins == (1u << 21)) {
                __hip_atomic_store(&a.ctrl->error, (int32_t)DQNX_DEVERR_PER_HANDOFF, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    DQNX_STAMP_WG(a.stamps, 51);
}

// ---------------------------------------------------------------------------------------
// SumTree.update's max / min index tracking over a mode-0 or mode-1 chunk (k_per_update, or one
// workgroup of the weight-gradient launch on the single-GPU PER step).  NT threads, IPT
// consecutive items per thread (n <= NT * IPT <= PER_CHUNK).  The items are read from the
// k_per_prep hand-off (wl / wp) into registers; the few indexed lookups go to that hand-off too,
// so the body needs no more LDS than its scans (it fits beside any host kernel's tiles).
//
// SumTree.update(L, p) (R:dqn/utils/sum_tree.py:15-32):
//   max_p, min_p = tree[max_idx], tree[min_idx]; tree[L] = p
//   if p >= max_p: max_idx = L     elif L == max_idx: max_idx = argmax(leaves[:size])
//   if p <= min_p: min_idx = L     elif L == min_idx: min_idx = argmin(leaves[:size])
// Without rescans the tracked max value is the running max of the p's (prefix scan) and max_idx
// is the leaf of the last update with p >= running max before it; an update triggers a rescan
// iff it does not raise the max and writes the current max leaf.  The body scans for the first
// trigger, applies the updates before it to the leaves, does the rescan on the leaves as they
// stand after that update, and restarts after it.
// ---------------------------------------------------------------------------------------

// running max / min priority and the latest index at which each was (re)taken, with that
// update's leaf, scanned together: one pair of barriers for all of them
struct Track {
    float mx, mn;
    int lx, ln;   // update index (-1: none)
    int Lx, Ln;   // its leaf
};
// CARRY = false: the leaves are not scanned (looked up in the hand-off instead: fewer registers)
template <bool CARRY>
__device__ __forceinline__ Track track_op(const Track& a, const Track& b) {
    const bool bx = b.lx > a.lx, bn = b.ln > a.ln;
    return Track{fmaxf(a.mx, b.mx), fminf(a.mn, b.mn), bx ? b.lx : a.lx, bn ? b.ln : a.ln,
                 CARRY ? (bx ? b.Lx : a.Lx) : 0, CARRY ? (bn ? b.Ln : a.Ln) : 0};
}
template <bool CARRY>
__device__ __forceinline__ Track track_shfl_up(const Track& t, int d) {
    return Track{__shfl_up(t.mx, d, 64), __shfl_up(t.mn, d, 64), __shfl_up(t.lx, d, 64), __shfl_up(t.ln, d, 64),
                 CARRY ? __shfl_up(t.Lx, d, 64) : 0, CARRY ? __shfl_up(t.Ln, d, 64) : 0};
}

template <int NT>
struct PerTrackLds {
    Track sht[NT / 64];
    int shi[NT / 64];
    double shd[NT / 64];
    int64_t shl[NT / 64];
    int mx_i, mn_i, resx, resn;
    float mx_v, mn_v;
};

// exclusive scan over threads (thread order) and the block total; every thread must call
template <int NW, bool CARRY>
__device__ Track track_scan(const Track& v, Track* sh, Track* total) {
    const Track ident{-INFINITY, INFINITY, -1, -1, 0, 0};
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    Track x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Track y = track_shfl_up<CARRY>(x, d);
        if (lane >= d) x = track_op<CARRY>(y, x);
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    Track carry = ident, tot = ident;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        if (w == wid) carry = tot;
        tot = track_op<CARRY>(tot, sh[w]);
    }
    Track prev = track_shfl_up<CARRY>(x, 1);
    if (lane == 0) prev = ident;
    __syncthreads();
    *total = tot;
    return track_op<CARRY>(carry, prev);
}

template <int NW>
__device__ __forceinline__ int block_min_int(int v, int* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    int r = sh[0];
#pragma unroll
    for (int w = 1; w < NW; w++) r = sh[w] < r ? sh[w] : r;
    __syncthreads();
    return r;
}

// first index of the max (want_max) or min over leaves [base, base + n): np.argmax / np.argmin
__device__ int64_t block_arg_extreme(const double* tree, int64_t base, int64_t n, bool want_max, double* shv,
                                     int64_t* shi, double* out_val) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double bv = want_max ? -INFINITY : INFINITY;
    int64_t bi = INT64_MAX;
    for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
        const double v = tree[base + j];
        if (want_max ? (v > bv) : (v < bv)) {   // strided ascending j: first occurrence kept
            bv = v;
            bi = j;
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const double ov = __shfl_xor(bv, d, 64);
        const int64_t oi = __shfl_xor(bi, d, 64);
        const bool better = want_max ? (ov > bv || (ov == bv && oi < bi)) : (ov < bv || (ov == bv && oi < bi));
        if (better) {
            bv = ov;
            bi = oi;
        }
    }
    if (lane == 0) {
        shv[wid] = bv;
        shi[wid] = bi;
    }
    __syncthreads();
    double rv = shv[0];
    int64_t ri = shi[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
        const bool better = want_max ? (shv[w] > rv || (shv[w] == rv && shi[w] < ri))
                                     : (shv[w] < rv || (shv[w] == rv && shi[w] < ri));
        if (better) {
            rv = shv[w];
            ri = shi[w];
        }
    }
    __syncthreads();
    *out_val = rv;
    return ri;
}

// The tracking itself; every thread of the NT-thread workgroup calls it.  The n items are taken
// in super-chunks of NT * IPT (IPT bounds the registers the body adds to a host kernel), each
// scanned with the state the previous one left: the same sequential semantics.  Ends by storing
// the tracked indices and advancing the chunk epoch (thread 0).
// CARRY: each retaking update's leaf rides in the scans (no dependent hand-off lookups; more
// registers: the 1024-thread k_per_update keeps the lookups to stay within 128 VGPRs).
template <int NT, int IPT, bool CARRY = true>
__device__ void per_track_block(const PerUpdateArgs& a, PerTrackLds<NT>& sh) {
    static_assert(IPT % 4 == 0 && PER_CHUNK % (NT * IPT) == 0, "16-byte loads inside the PER_CHUNK hand-off");
    constexpr int NW = NT / 64, SC = NT * IPT;
    const int tid = threadIdx.x;
    DQNX_STAMP(a.stamps, 56);
    DQNX_STAMP_WG(a.stamps, 48);
    const int n = a.n;
    const int64_t base = a.cap - 1;
    // the tracked max / min leaves first (a dependent pair of round trips)
    int mx_i = (int)a.ctrl->per_max_idx, mn_i = (int)a.ctrl->per_min_idx;
    float mx_v = (float)a.tree[mx_i], mn_v = (float)a.tree[mn_i];
    int w = 0;   // updates [0, w) are written to the leaves (by the rescans so far)
    for (int c0 = 0; c0 < n; c0 += SC) {
        float pv[IPT];
        int32_t lv[IPT];
        {   // IPT consecutive items per thread (scan order); the tail past n is masked below
            const int4* wl4 = reinterpret_cast<const int4*>(a.wl + c0) + (IPT / 4) * tid;
            const float4* wp4 = reinterpret_cast<const float4*>(a.wp + c0) + (IPT / 4) * tid;
#pragma unroll
            for (int q = 0; q < IPT / 4; q++) {
                const int4 l4 = wl4[q];
                const float4 p4 = wp4[q];
                lv[4 * q] = l4.x; lv[4 * q + 1] = l4.y; lv[4 * q + 2] = l4.z; lv[4 * q + 3] = l4.w;
                pv[4 * q] = p4.x; pv[4 * q + 1] = p4.y; pv[4 * q + 2] = p4.z; pv[4 * q + 3] = p4.w;
            }
        }
#pragma unroll
        for (int k = 0; k < IPT; k++) {
            if (c0 + tid * IPT + k >= n) {
                lv[k] = -1;
                pv[k] = 0.f;
            }
        }
        DQNX_STAMP(a.stamps, 57);
        if (c0 == 0) DQNX_STAMP_WG(a.stamps, 49);
        int s = c0;   // updates [c0, s) of this super-chunk are folded into the state
        while (true) {
            // pass 1: the thread's max / min (for the scan)
            Track own{-INFINITY, INFINITY, -1, -1, 0, 0};
#pragma unroll
            for (int k = 0; k < IPT; k++) {
                const int i = c0 + tid * IPT + k;
                if (i >= s && i < n) {
                    own.mx = fmaxf(own.mx, pv[k]);
                    own.mn = fminf(own.mn, pv[k]);
                }
            }
            Track totv;
            const Track exv = track_scan<NW, CARRY>(own, sh.sht, &totv);
            // pass 2: which items (re)take the max / min, given the running values BEFORE each
            Track ownl{-INFINITY, INFINITY, -1, -1, 0, 0};
            {
                float rmx = fmaxf(mx_v, exv.mx), rmn = fminf(mn_v, exv.mn);
#pragma unroll
                for (int k = 0; k < IPT; k++) {
                    const int i = c0 + tid * IPT + k;
                    if (i >= s && i < n) {
                        if (pv[k] >= rmx) { ownl.lx = i; ownl.Lx = lv[k]; }
                        if (pv[k] <= rmn) { ownl.ln = i; ownl.Ln = lv[k]; }
                        rmx = fmaxf(rmx, pv[k]);
                        rmn = fminf(rmn, pv[k]);
                    }
                }
            }
            Track totl;
            const Track exl = track_scan<NW, CARRY>(ownl, sh.sht, &totl);
            // pass 3: the first item that rewrites the current max / min leaf without retaking it.
            // max_idx before update i is the leaf of the latest retaking item before it (the
            // thread's own item once one of its items retook), else the state entering the scan
            int curx = exl.lx >= 0 ? (CARRY ? exl.Lx : a.wl[exl.lx]) : mx_i;
            int curn = exl.ln >= 0 ? (CARRY ? exl.Ln : a.wl[exl.ln]) : mn_i;
            int mytrig = n;
            int cxb = 0, cnb = 0, tl = 0;
            float tp = 0.f, bx = 0.f, bn = 0.f;
            {
                float rmx = fmaxf(mx_v, exv.mx), rmn = fminf(mn_v, exv.mn);
#pragma unroll
                for (int k = 0; k < IPT; k++) {
                    const int i = c0 + tid * IPT + k;
                    if (i >= s && i < n) {
                        const bool fx = pv[k] >= rmx, fn = pv[k] <= rmn;
                        const bool trig = (!fx && lv[k] == curx) || (!fn && lv[k] == curn);
                        if (trig && mytrig == n) {
                            mytrig = i;
                            cxb = curx;
                            cnb = curn;
                            tl = lv[k];
                            tp = pv[k];
                            bx = rmx;
                            bn = rmn;
                        }
                        if (fx) curx = lv[k];
                        if (fn) curn = lv[k];
                        rmx = fmaxf(rmx, pv[k]);
                        rmn = fminf(rmn, pv[k]);
                    }
                }
            }
            if (!__syncthreads_or(mytrig < n)) {   // no rescan left: fold the scans into the state
                if (totl.lx >= 0) mx_i = CARRY ? totl.Lx : a.wl[totl.lx];
                if (totl.ln >= 0) mn_i = CARRY ? totl.Ln : a.wl[totl.ln];
                mx_v = fmaxf(mx_v, totv.mx);
                mn_v = fminf(mn_v, totv.mn);
                break;
            }
            const int istar = block_min_int<NW>(mytrig, sh.shi);
            if (mytrig == istar) {   // the owner of the first trigger applies that update
                const float p = tp;
                const int L = tl;
                sh.resx = 0;
                sh.resn = 0;
                if (p >= bx) { sh.mx_i = L; sh.mx_v = p; }
                else if (L == cxb) sh.resx = 1;
                else { sh.mx_i = cxb; sh.mx_v = bx; }
                if (p <= bn) { sh.mn_i = L; sh.mn_v = p; }
                else if (L == cnb) sh.resn = 1;
                else { sh.mn_i = cnb; sh.mn_v = bn; }
            }
            __syncthreads();
            // leaves as they stand after update istar, in update order (a slot written twice
            // keeps its later value)
            if (tid == 0)
                for (int j = w; j <= istar; j++) a.tree[a.wl[j]] = (double)a.wp[j];
            w = istar + 1;
            __threadfence_block();
            __syncthreads();
            const int64_t sz = a.mode == 1 ? min(a.size + istar + 1, a.cap) : a.ctrl->ring_size;
            if (sh.resx) {
                double v;
                const int64_t j = block_arg_extreme(a.tree, base, sz, true, sh.shd, sh.shl, &v);
                if (tid == 0) { sh.mx_i = (int)(j + base); sh.mx_v = (float)v; }
            }
            if (sh.resn) {
                double v;
                const int64_t j = block_arg_extreme(a.tree, base, sz, false, sh.shd, sh.shl, &v);
                if (tid == 0) { sh.mn_i = (int)(j + base); sh.mn_v = (float)v; }
            }
            __syncthreads();
            mx_i = sh.mx_i;
            mx_v = sh.mx_v;
            mn_i = sh.mn_i;
            mn_v = sh.mn_v;
            s = istar + 1;
            __syncthreads();
        }
    }
    DQNX_STAMP(a.stamps, 59);
    DQNX_STAMP_WG(a.stamps, 50);
    if (tid == 0) {
        a.ctrl->per_max_idx = mx_i;
        a.ctrl->per_min_idx = mn_i;
        *a.epoch += 1u;   // the chunk k_per_prep tagged; k_per_prop reads it back
    }
    DQNX_STAMP(a.stamps, 61);
}

}  // namespace dqnx
