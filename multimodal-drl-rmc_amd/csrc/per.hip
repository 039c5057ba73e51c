// Prioritised replay on the device: SumTree sampling and priority writes.
//
// Replaces ReplayMemoryPrioritized (R:dqn/replay_memory.py:43-98) over SumTree
// (R:dqn/utils/sum_tree.py:4-73).  The tree is the reference's own implicit heap of
// 2*cap-1 float64 nodes (leaves at [cap-1, 2cap-2]); a leaf's data index is the ring slot.
//
// Exactness argument used by k_per_update.  Every leaf holds a float32 priority
// p = min(|d| + 1e-4, 1)^0.6 in [2^-8, 1] (p >= 1e-4^0.6 = 0.00398 > 2^-8), or 0, or the
// push priority (a leaf value or 1.0).  Such values are integer multiples of 2^-31, and with
// cap <= 2^20 every partial sum stays below 2^21, so it needs at most 52 significant bits:
// every float64 addition the reference performs on the tree (`change`, `tree[parent] +=
// change`) is EXACT.  Internal node values are therefore exactly the sum of their leaves,
// independent of the order of the additions, and the kernel may apply all of a batch's
// leaf deltas in parallel (LDS / global float64 atomics) and still produce the reference's
// bits.  The order-dependent parts -- the max/min priority index tracking with its
// argmax/argmin rescans -- follow SumTree.update step by step (see k_per_update).
#include "learn.hpp"
#include "mt.hpp"
#include "per_common.hpp"

namespace dqnx {

constexpr int PER_NT = 1024;   // threads of the one-workgroup tracking kernel (256 x 32 items measured
                               // slower: serial per-item LDS lookups, strided LDS stores)

// ---------------------------------------------------------------------------------------
// sample_transitions (R:dqn/replay_memory.py:69-92): stratified proportional sampling.
// ceil(Bg / PER_SNT) workgroups, one sample per thread.  Every workgroup reads the numpy
// MT19937 state and walks the same sequence of twists (block-parallel, in LDS) up to the
// last of the 2*Bg words the legacy uniforms consume, tempering only the words of its own
// samples; the last workgroup to arrive at the ticket (so every other one has read the old
// state) writes the advanced state back.  The descent (get_leaf) reads the top PER_STOP
// nodes from LDS and the rest PER_LA levels per global round trip.
// ---------------------------------------------------------------------------------------
constexpr int PER_SNT = 256;     // samples (threads) per sampling workgroup: the descents' scattered
                                 // loads are texture-path bound, so spread them over more CUs
#ifndef DQNX_PER_STOP
#define DQNX_PER_STOP 8191
#endif
constexpr int PER_STOP = DQNX_PER_STOP;   // nodes of depth <= 12 (64 KiB of float64) cached per workgroup
constexpr int PER_LA = 4;        // tree levels fetched per dependent global round trip

// the chosen subtree's half of the first N nodes of a level fetched ahead:
// x[0 .. N/2) = r ? x[N/2 .. N) : x[0 .. N/2)
template <int N, int M>
__device__ __forceinline__ void per_narrow(double (&x)[M], bool r) {
    static_assert(N <= M, "narrow within the fetched level");
#pragma unroll
    for (int j = 0; j < N / 2; j++) x[j] = r ? x[j + N / 2] : x[j];
}

__global__ __launch_bounds__(PER_SNT) void k_per_sample(PerSampleArgs a) {
    __shared__ double top[PER_STOP];
    __shared__ uint32_t mtb[2][624];
    __shared__ uint32_t words[2 * PER_SNT];
    __shared__ int64_t s_step;
    __shared__ uint32_t s_pos;
    __shared__ int s_last, s_ccnt;
    const int spw = a.spw;   // samples per workgroup (<= PER_SNT; all PER_SNT threads load and twist)
    const int G = (a.Bg + spw - 1) / spw;
    if ((int)blockIdx.x >= G) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - G, gridDim.x - G);
        return;
    }
    const int tid = threadIdx.x, grp = blockIdx.x;
    DQNX_STAMP(a.stamps, 0);
    const int64_t len = 2 * a.cap - 1;
    const double total = a.tree[0];                        // SumTree.total_priority
    if (!(total > 0.0)) {   // every workgroup sees it: nobody arrives, the state stays untouched
        if (grp == 0 && tid == 0) atomicExch(&a.ctrl->error, DQNX_DEVERR_EMPTY_TREE);
        return;
    }
    const int64_t size = a.ctrl->ring_size;
    const int64_t min_idx = a.ctrl->per_min_idx;
    bool cmis = false;
    {   // every load in flight before the first LDS write (a plain loop waits on each one)
        constexpr int NQ = (PER_STOP + 2 * PER_SNT - 1) / (2 * PER_SNT);
        double2 tv[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int j = 2 * (tid + q * PER_SNT);
            // len is odd: a pair is whole, or only its first node exists (j = len - 1), or none
            tv[q] = j + 1 < len ? *reinterpret_cast<const double2*>(a.tree + j)
                                : make_double2(j < len ? a.tree[j] : 0.0, 0.0);
        }
        constexpr int NJ = (624 + PER_SNT - 1) / PER_SNT;
        uint32_t sw[NJ], cwv[NJ];
#pragma unroll
        for (int u = 0; u < NJ; u++) {   // the state block, and the cache's block 0 to check it against
            const int j = tid + u * PER_SNT < 624 ? tid + u * PER_SNT : 623;
            sw[u] = a.ctrl->np_mt[j];
            cwv[u] = a.npc ? a.npc[64 + j] : 0u;
        }
#pragma unroll
        for (int u = 0; u < NJ; u++) {
            if (tid + u * PER_SNT < 624) {
                mtb[0][tid + u * PER_SNT] = sw[u];
                cmis |= sw[u] != cwv[u];
            }
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int j = 2 * (tid + q * PER_SNT);
            if (j < PER_STOP) top[j] = tv[q].x;
            if (j + 1 < PER_STOP) top[j + 1] = tv[q].y;
        }
    }
    if (tid == 0) {
        s_pos = a.ctrl->np_mt[624];
        s_step = a.ctrl->agent_step;
        s_ccnt = a.npc ? (int)a.npc[0] : 0;
    }
    const double prob_min = a.tree[min_idx] / total;
    const bool cache_mismatch = __syncthreads_or(cmis ? 1 : 0) != 0;   // (the fields written back below are in LDS)
    if (tid == 0) {
        __threadfence();
        s_last = atomicAdd(a.ticket, 1) == G - 1;
    }
    const int64_t step = s_step;
    uint32_t pos = s_pos;
    DQNX_STAMP(a.stamps, 1);

    // the words of np.random.uniform calls i = 0..Bg-1: legacy double = 2 words each
    const int W = 2 * a.Bg;
    const int w0 = 2 * grp * spw, w1 = min(W, w0 + 2 * spw);
    // the block holding the last word (0 = the state block) and the index just past it
    const int bfin = ((int)pos + W - 1) / 624;
    const uint32_t nxfin = (uint32_t)(((int)pos + W - 1) % 624 + 1);
    const bool cached = a.npc && !cache_mismatch && s_ccnt >= bfin + 1;
    bool twisted = false;
    int cur = 0;
    if (cached) {   // word w of the call sits at cache position pos + w (blocks are contiguous)
        for (int w = w0 + tid; w < w1; w += PER_SNT) words[w - w0] = mt_temper(a.npc[64 + pos + w]);
    } else {
        for (int done = 0; done < W;) {
            if (pos >= 624) {
                mt_twist_into(mtb[cur], mtb[cur ^ 1]);   // ends with a barrier
                cur ^= 1;
                pos = 0;
                twisted = true;
            }
            const int take = min(624 - (int)pos, W - done);
            const int lo = max(done, w0), hi = min(done + take, w1);
            for (int w = lo + tid; w < hi; w += PER_SNT) words[w - w0] = mt_temper(mtb[cur][pos + (w - done)]);
            done += take;
            pos += (uint32_t)take;
        }
    }

    // beta = np.interp(step, [0, beta_inc], [beta_start, beta_end]) (numpy arr_interp, 2 points)
    const double x = (double)step;
    double beta;
    if (x >= a.beta_steps) beta = a.beta_end;
    else if (x <= 0.0) beta = a.beta_start;                // x < xp[0] -> left; x == xp[0] -> fp[0]
    else {
        const double slope = (a.beta_end - a.beta_start) / (a.beta_steps - 0.0);
        beta = slope * (x - 0.0) + a.beta_start;
    }
    const double seg = total / (double)a.Bg;               // priority_segment
    const double max_w = pow((double)size * prob_min, -beta);
    __syncthreads();
    DQNX_STAMP(a.stamps, 2);

    const int i = grp * spw + tid;
    if (tid < spw && i < a.Bg) {
        // legacy_double: (a >> 5, b >> 6) -> [0, 1); uniform = low + (high - low) * u
        const uint32_t wa = words[2 * tid] >> 5, wb = words[2 * tid + 1] >> 6;
        const double u = ((double)wa * 67108864.0 + (double)wb) / 9007199254740992.0;
        const double low = seg * (double)i, high = seg * (double)(i + 1);
        double v = low + (high - low) * u;
        // get_leaf (R:dqn/utils/sum_tree.py:42-61): the same comparisons, node by node
        int64_t p = 0, leaf = -1;
        double pval = top[0];
        while (true) {
            const int64_t left = 2 * p + 1;
            if (left >= len) { leaf = p; break; }
            if (left + 1 >= PER_STOP) break;
            const double tl = top[left];
            if (v <= tl) { p = left; pval = tl; }
            else { v -= tl; p = left + 1; pval = top[left + 1]; }
        }
        while (leaf < 0) {
            // the 2 + 4 + 8 + 16 nodes of the next PER_LA levels under p, in one round trip
            double l1[2], l2[4], l3[8], l4[16];
            const int64_t b1 = 2 * p + 1, b2 = 4 * p + 3, b3 = 8 * p + 7, b4 = 16 * p + 15;
            // 16-byte loads (a level's nodes are contiguous); past the end of the tree a pair
            // is clamped to the last two nodes (those values are never compared)
            auto ld2 = [&](int64_t n, double* d) {
                const double2 v = *reinterpret_cast<const double2*>(a.tree + (n + 1 < len ? n : len - 2));
                d[0] = v.x;
                d[1] = v.y;
            };
            if (len < 2) break;   // unreachable: a one-node tree is a leaf at the root
#pragma unroll
            for (int j = 0; j < 2; j += 2) ld2(b1 + j, l1 + j);
#pragma unroll
            for (int j = 0; j < 4; j += 2) ld2(b2 + j, l2 + j);
#pragma unroll
            for (int j = 0; j < 8; j += 2) ld2(b3 + j, l3 + j);
#pragma unroll
            for (int j = 0; j < 16; j += 2) ld2(b4 + j, l4 + j);
            // one level: the children of p are c[0], c[1]; the deeper levels keep the chosen half
            auto level = [&](const double* c) {
                const int64_t left = 2 * p + 1;
                if (left >= len) { leaf = p; return false; }
                const bool r = !(v <= c[0]);
                if (r) v -= c[0];
                pval = r ? c[1] : c[0];
                p = left + (r ? 1 : 0);
                return r;
            };
            bool r;
            do {
                r = level(l1); if (leaf >= 0) break;
                per_narrow<4>(l2, r); per_narrow<8>(l3, r); per_narrow<16>(l4, r);
                r = level(l2); if (leaf >= 0) break;
                per_narrow<4>(l3, r); per_narrow<8>(l4, r);
                r = level(l3); if (leaf >= 0) break;
                per_narrow<4>(l4, r);
                level(l4);
            } while (0);
        }
        const double prob = pval / total;
        const double w = pow((double)size * prob, -beta) / max_w;
        a.isw[i] = (float)w;
        const int32_t di = (int32_t)(leaf - (a.cap - 1));
        a.out_idx[i] = di;
        if (a.phys_out && i >= a.shard_begin && i < a.shard_begin + a.shard_len) a.phys_out[i - a.shard_begin] = di;
    }
    DQNX_STAMP(a.stamps, 3);
    if (s_last) {   // every other workgroup has read the old state: write the advanced one
        if (cached) {   // cache block bfin; the next extension drops the blocks before it
            if (bfin > 0)
                for (int j = tid; j < 624; j += PER_SNT) a.ctrl->np_mt[j] = a.npc[64 + 624 * bfin + j];
            if (tid == 0) a.npc[1] = (uint32_t)bfin;
        } else {
            if (twisted)
                for (int j = tid; j < 624; j += PER_SNT) a.ctrl->np_mt[j] = mtb[cur][j];
            if (tid == 0 && a.npc) a.npc[0] = 0u;   // the extension restarts from the new state
        }
        if (tid == 0) {
            a.ctrl->np_mt[624] = cached ? nxfin : pos;
            a.ctrl->per_beta = beta;
            a.ctrl->agent_step = step + a.n_env;   // the caller's agent.step advances once per learn
            *a.ticket = 0;
        }
    }
}

__device__ __forceinline__ uint32_t leaf_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// ---------------------------------------------------------------------------------------
// n <= PER_CHUNK SumTree.update calls in order: three launches.
//
// SumTree.update(L, p) (R:dqn/utils/sum_tree.py:15-32):
//   max_p, min_p = tree[max_idx], tree[min_idx]; tree[L] = p
//   if p >= max_p: max_idx = L     elif L == max_idx: max_idx = argmax(leaves[:size])
//   if p <= min_p: min_idx = L     elif L == min_idx: min_idx = argmin(leaves[:size])
//   ancestors += p - old
//
// k_per_prep (grid): leaf, priority (float64 pow) and old leaf value of every item; the
//   latest item writing each slot is found by a 64-bit atomicMax of (epoch << 32 | i) on a
//   per-slot word (tagged by a chunk epoch, so it never needs clearing).
// k_per_update (one workgroup): the max / min index tracking.  Without rescans the tracked
//   max value is the running max of the p's (prefix scan) and max_idx is the leaf of the last
//   update with p >= running max before it; an update triggers a rescan iff it does not
//   raise the max and writes the current max leaf.  The kernel scans for the first trigger,
//   applies the updates before it to the leaves, does the rescan on the leaves as they stand
//   after that update, and restarts after it.  Rescans are rare (the max / min leaf has to be
//   resampled), so the common case is one pass.
// k_per_prop (grid): every slot's last item writes the final leaf and adds its delta
//   (final - old) to the ancestors: float64 atomics, the top levels first summed per
//   workgroup in LDS.  Order-free: every addition is exact (file header).
// ---------------------------------------------------------------------------------------

__global__ __launch_bounds__(PER_GT) void k_per_prep(PerUpdateArgs a) {
    const int i = blockIdx.x * PER_GT + threadIdx.x;
    if (i >= a.n) return;
    const int64_t base = a.cap - 1;
    if (a.mode == 0) {
        per_prep_item(a, i, a.abs_td[i]);
        return;
    }
    const int64_t slot = (a.wptr + i) % a.cap;   // store_transitions: max_priority, or max_priority_high if 0
    const int32_t L = (int32_t)(slot + base);
    const double mv = a.tree[a.ctrl->per_max_idx];
    const float p = (mv == 0.0) ? a.pmax : (float)mv;
    a.wl[i] = L;
    a.wp[i] = p;
    a.winit[i] = a.tree[L];
    const uint64_t e = (uint64_t)(*a.epoch + 1u);
    atomicMax((unsigned long long*)&a.last[slot], (unsigned long long)((e << 32) | (uint32_t)i));
}

__global__ __launch_bounds__(PER_NT) void k_per_update(PerUpdateArgs a) {
    __shared__ PerTrackLds<PER_NT> sh;
    // one super-chunk; the leaf lookups instead of the carried leaves (128 VGPRs at 1024 threads)
    per_track_block<PER_NT, PER_CHUNK / PER_NT, false>(a, sh);
}

__global__ __launch_bounds__(PER_GT) void k_per_prop(PerUpdateArgs a) {
    __shared__ double topd[PER_TOP];
    per_prop_block(a, blockIdx.x * PER_GT, topd);
}

// ---------------------------------------------------------------------------------------
// numpy 1.21 mode (dqnx_config.per_numpy121).  update_batch_priorities hands SumTree.update a
// float32 (1,) array per sample (R:dqn/replay_memory.py:95-98); under numpy < 2's value-based
// casting `change = priority - tree[i]` and `tree[parent] += change` (R:dqn/utils/sum_tree.py:
// 18, 31-32) are computed in float32 (the float64 scalar is cast down), so the ancestors hold
// float32-rounded running sums and the ORDER of the updates matters.  Every node's sequence of
// additions is independent of every other node's, so:
//   k_per_chain<true>  (one workgroup): items sorted by (leaf, item); per leaf, in item order,
//                      change = f32(p - previous value of the leaf); the final p is written;
//   k_per_chain<false> (one workgroup per tree depth): items sorted by (ancestor at that depth,
//                      item); per ancestor, in item order, v = f32(f32(v) + change).
// Sorting is an LDS bitonic sort of (node << 13 | item) keys; a node's chain is one thread's
// sequential loop (the root's is the whole batch: B dependent adds).  The leaf max/min tracking
// (k_per_update) is unchanged: comparisons and leaves are the same under both numpy versions.
// ---------------------------------------------------------------------------------------
constexpr int PER_CHAIN_NT = 1024;

__device__ __forceinline__ void chain_sort(unsigned long long* keys, int N2) {
    for (int k = 2; k <= N2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < N2; i += PER_CHAIN_NT) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const unsigned long long x = keys[i], y = keys[ixj];
                    if ((x > y) == ((i & k) == 0)) {
                        keys[i] = y;
                        keys[ixj] = x;
                    }
                }
            }
            __syncthreads();
        }
}

template <bool LEAF>
__global__ __launch_bounds__(PER_CHAIN_NT) void k_per_chain(PerUpdateArgs a) {
    // LDS: keys [N2] (u64), then chg [n] (float; the ancestor pass reuses it for the chain starts),
    // then schg [n] (the changes in sorted order)
    extern __shared__ unsigned long long keys[];
    __shared__ int wave_cnt[PER_CHAIN_NT / 64];
    __shared__ int s_nst;
    const int n = a.n, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int N2 = 1;
    while (N2 < n) N2 <<= 1;
    float* chg = reinterpret_cast<float*>(keys + N2);
    const int depth = blockIdx.x;   // ancestor pass: the tree depth this workgroup owns
    for (int u = tid; u < N2; u += PER_CHAIN_NT) {
        unsigned long long k = ~0ull;
        if (u < n) {
            int64_t node = a.wl[u];
            if (!LEAF) {
                const int dn = 63 - __clzll((unsigned long long)(node + 1));   // depth of the leaf
                node = dn > depth ? ((node + 1) >> (dn - depth)) - 1 : -1;
                chg[u] = a.wchg[u];
            }
            if (node >= 0) k = ((unsigned long long)node << 13) | (unsigned)u;
        }
        keys[u] = k;
    }
    __syncthreads();
    chain_sort(keys, N2);
    if (LEAF) {
        for (int i = tid; i < n; i += PER_CHAIN_NT) {
            const unsigned long long k = keys[i];
            if (k == ~0ull) continue;
            const int64_t node = (int64_t)(k >> 13);
            if (i > 0 && (int64_t)(keys[i - 1] >> 13) == node) continue;   // not the start of a chain
            float prev = (float)a.winit[(int)(k & 8191u)];   // the leaf before this chunk
            for (int j = i; j < n && (int64_t)(keys[j] >> 13) == node; j++) {
                const int u = (int)(keys[j] & 8191u);
                const float p = a.wp[u];
                a.wchg[u] = p - prev;   // float32 subtraction
                prev = p;
            }
            a.tree[node] = (double)prev;
        }
        return;
    }
    // ---- ancestor pass ----
    // (1) the changes in sorted (node, item) order; (2) the chain starts, compacted in order (a block
    // scan over 8 consecutive positions per thread); (3) a WAVE per chain: 64 sorted changes per round
    // in the lanes, the node's float32 running sum carried through them in item order by readlane
    // (v = f32(v + change), the reference's sequence), so a chain costs ~2 instructions per update
    // instead of a dependent LDS round trip per update (the root's chain is the whole batch)
    float* schg = chg + n;
    for (int i = tid; i < n; i += PER_CHAIN_NT) {
        const unsigned long long k = keys[i];
        schg[i] = k == ~0ull ? 0.f : chg[(int)(k & 8191u)];
    }
    __syncthreads();
    constexpr int IPT = PER_CHUNK / PER_CHAIN_NT;   // positions per thread in the scan
    int flags = 0, cnt = 0;
#pragma unroll
    for (int q = 0; q < IPT; q++) {
        const int i = tid * IPT + q;
        bool st = false;
        if (i < n) {
            const unsigned long long k = keys[i];
            st = k != ~0ull && (i == 0 || (keys[i - 1] >> 13) != (k >> 13));
        }
        flags |= st ? (1 << q) : 0;
        cnt += st ? 1 : 0;
    }
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wave_cnt[wid] = incl;
    __syncthreads();   // (every schg / chg read above is done before the starts overwrite chg)
    int before = incl - cnt, total = 0;
#pragma unroll
    for (int w = 0; w < PER_CHAIN_NT / 64; w++) {
        const int c = wave_cnt[w];
        before += w < wid ? c : 0;
        total += c;
    }
    int* starts = reinterpret_cast<int*>(chg);
#pragma unroll
    for (int q = 0; q < IPT; q++)
        if (flags & (1 << q)) starts[before++] = tid * IPT + q;
    int nvalid = 0;   // positions holding a key (the no-ancestor keys sort last)
    if (tid == 0) s_nst = total;
    __syncthreads();
    const int nst = s_nst;
    {   // nvalid: the first position past the last valid key (binary search, every thread alike)
        int lo = 0, hi = n;
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (keys[m] != ~0ull) lo = m + 1;
            else hi = m;
        }
        nvalid = lo;
    }
    // short chains (deep levels: thousands of 1-3 update chains): a thread each, every tree value of
    // the thread's chains loaded before the first walk
    constexpr int LONG = 128, CPT = PER_CHUNK / PER_CHAIN_NT;
    {
        int c0[CPT], c1[CPT];
        int64_t nd[CPT];
        double tv[CPT];
#pragma unroll
        for (int k = 0; k < CPT; k++) {
            const int c = tid + k * PER_CHAIN_NT;
            c0[k] = c < nst ? starts[c] : 0;
            c1[k] = c < nst ? (c + 1 < nst ? starts[c + 1] : nvalid) : 0;
            if (c1[k] - c0[k] >= LONG) c1[k] = c0[k];   // a wave's below
            nd[k] = (int64_t)(keys[c0[k]] >> 13);
            tv[k] = c1[k] > c0[k] ? a.tree[nd[k]] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < CPT; k++) {
            if (c1[k] <= c0[k]) continue;
            float v = (float)tv[k];
            for (int j = c0[k]; j < c1[k]; j++) v = v + schg[j];
            a.tree[nd[k]] = (double)v;
        }
    }
    // long chains (the top levels; the root's is the whole batch): a wave each, 64 sorted changes per
    // round in the lanes, the running sum carried through them in item order by readlane
    for (int c = wid; c < nst; c += PER_CHAIN_NT / 64) {
        const int s0 = starts[c], e0 = c + 1 < nst ? starts[c + 1] : nvalid;
        if (e0 - s0 < LONG) continue;
        const int64_t node = (int64_t)(keys[s0] >> 13);
        float v = (float)a.tree[node];
        for (int j0 = s0; j0 < e0; j0 += 64) {
            const int len = min(64, e0 - j0);
            const float cv = lane < len ? schg[j0 + lane] : 0.f;
            const int cvi = __float_as_int(cv);
            for (int q = 0; q < len; q++) v = v + __int_as_float(__builtin_amdgcn_readlane(cvi, q));
        }
        if (lane == 0) a.tree[node] = (double)v;
    }
}

// the ancestor pass needs up to 128 KB of dynamic LDS: raise the limit once, outside any
// stream capture (dqnx_engine_create with per_numpy121)
int per_numpy121_init() {
    DQNX_HIP_CHECK(hipFuncSetAttribute((const void*)k_per_chain<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       PER_CHUNK * 16));
    DQNX_HIP_CHECK(hipFuncSetAttribute((const void*)k_per_chain<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       PER_CHUNK * 16));
    return DQNX_OK;
}

int launch_per_sample(const PerSampleArgs& a, hipStream_t s) {
    if (a.Bg < 1 || a.Bg > PER_MAX_B) return set_error(DQNX_EUNSUPPORTED, "PER batch %d outside [1, %d]", a.Bg, PER_MAX_B);
    if (a.spw < 1 || a.spw > PER_SNT) return set_error(DQNX_EINVAL, "PER samples per workgroup %d", a.spw);
    const int G = (a.Bg + a.spw - 1) / a.spw;
    DQNX_LAUNCH(k_per_sample, dim3(G + a.rl_blocks), dim3(PER_SNT), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_per_update(const PerUpdateArgs& a, hipStream_t s) {
    if (a.n < 0 || a.n > PER_CHUNK) return set_error(DQNX_EINVAL, "PER update chunk %d > %d", a.n, PER_CHUNK);
    if (a.n == 0) return DQNX_OK;
    const int g = (a.n + PER_GT - 1) / PER_GT;
    if ((a.skip & PER_SKIP_PREP) && (a.mode != 0 || a.numpy121))
        return set_error(DQNX_EINVAL, "PER update: the prep pass is hosted only for mode 0 without numpy121");
    if (!(a.skip & PER_SKIP_PREP)) DQNX_LAUNCH(k_per_prep, dim3(g), dim3(PER_GT), 0, s, a);
    DQNX_LAUNCH(k_per_update, dim3(1), dim3(PER_NT), 0, s, a);
    if (a.numpy121 && a.mode == 0) {   // float32 change / ancestor sums in update order
        int N2 = 1;
        while (N2 < a.n) N2 <<= 1;
        int depths = 0;   // internal depths 0 .. (deepest leaf depth - 1)
        while (((int64_t)1 << (depths + 1)) <= 2 * a.cap - 1) depths++;
        DQNX_LAUNCH(k_per_chain<true>, dim3(1), dim3(PER_CHAIN_NT), (size_t)N2 * 8, s, a);
        if (depths > 0)
            DQNX_LAUNCH(k_per_chain<false>, dim3(depths), dim3(PER_CHAIN_NT), (size_t)N2 * 8 + (size_t)a.n * 8, s, a);
    } else if (!(a.skip & PER_SKIP_PROP)) {
        DQNX_LAUNCH(k_per_prop, dim3(g), dim3(PER_GT), 0, s, a);
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
