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

namespace dqnx {

constexpr int PER_NT = 1024;
constexpr int PER_TOP = 2047;            // nodes of depth <= 10, cached / accumulated in LDS
constexpr int PER_IPT = PER_CHUNK / PER_NT;
constexpr int PER_HS = 2 * PER_CHUNK;    // leaf hash slots

// ---------------------------------------------------------------------------------------
// sample_transitions (R:dqn/replay_memory.py:69-92): stratified proportional sampling.
// One workgroup: the 2*Bg MT19937 words numpy's legacy uniform consumes are generated
// block-parallel (twist in LDS), then every sample descends the tree independently.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(PER_NT) void k_per_sample(PerSampleArgs a) {
    __shared__ uint32_t words[2 * PER_MAX_B];
    __shared__ double top[PER_TOP];
    __shared__ uint32_t mt[624], tmp[624];
    if (blockIdx.x > 0) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    const int tid = threadIdx.x;
    const int64_t len = 2 * a.cap - 1;
    const double total = a.tree[0];                        // SumTree.total_priority
    if (!(total > 0.0)) {
        if (tid == 0) atomicExch(&a.ctrl->error, DQNX_DEVERR_EMPTY_TREE);
        return;
    }
    const int64_t step = a.ctrl->agent_step;
    const int64_t size = a.ctrl->ring_size;
    const int64_t min_idx = a.ctrl->per_min_idx;
    for (int i = tid; i < PER_TOP && i < len; i += PER_NT) top[i] = a.tree[i];
    if (tid < 624) mt[tid] = a.ctrl->np_mt[tid];
    uint32_t pos = a.ctrl->np_mt[624];
    __syncthreads();

    // the words of np.random.uniform calls i = 0..Bg-1: legacy double = 2 words each
    const int W = 2 * a.Bg;
    bool twisted = false;
    for (int done = 0; done < W;) {
        if (pos >= 624) {
            mt_twist_block(mt, tmp);
            pos = 0;
            twisted = true;
        }
        const int take = min(624 - (int)pos, W - done);
        if (tid < take) words[done + tid] = mt_temper(mt[pos + tid]);
        done += take;
        pos += (uint32_t)take;
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
    const double prob_min = a.tree[min_idx] / total;
    const double max_w = pow((double)size * prob_min, -beta);
    __syncthreads();

    for (int i = tid; i < a.Bg; i += PER_NT) {
        // legacy_double: (a >> 5, b >> 6) -> [0, 1); uniform = low + (high - low) * u
        const uint32_t wa = words[2 * i] >> 5, wb = words[2 * i + 1] >> 6;
        const double u = ((double)wa * 67108864.0 + (double)wb) / 9007199254740992.0;
        const double low = seg * (double)i, high = seg * (double)(i + 1);
        double v = low + (high - low) * u;
        // get_leaf (R:dqn/utils/sum_tree.py:42-61)
        int64_t parent = 0, leaf;
        while (true) {
            const int64_t left = 2 * parent + 1;
            if (left >= len) {
                leaf = parent;
                break;
            }
            const double tl = left < PER_TOP ? top[left] : a.tree[left];
            if (v <= tl) {
                parent = left;
            } else {
                v -= tl;
                parent = left + 1;
            }
        }
        const double p = leaf < PER_TOP ? top[leaf] : a.tree[leaf];
        const double prob = p / total;
        const double w = pow((double)size * prob, -beta) / max_w;
        a.isw[i] = (float)w;
        const int32_t di = (int32_t)(leaf - (a.cap - 1));
        a.out_idx[i] = di;
        if (a.phys_out && i >= a.shard_begin && i < a.shard_begin + a.shard_len) a.phys_out[i - a.shard_begin] = di;
    }
    __syncthreads();
    if (twisted && tid < 624) a.ctrl->np_mt[tid] = mt[tid];
    if (tid == 0) {
        a.ctrl->np_mt[624] = pos;
        a.ctrl->per_beta = beta;
        a.ctrl->agent_step = step + a.n_env;   // the caller's agent.step advances once per learn
    }
}

// ---------------------------------------------------------------------------------------
// block scan / reduce helpers (1024 threads = 16 waves)
// ---------------------------------------------------------------------------------------
struct OpMaxF { __device__ float operator()(float x, float y) const { return fmaxf(x, y); } };
struct OpMinF { __device__ float operator()(float x, float y) const { return fminf(x, y); } };
struct OpMaxI { __device__ int operator()(int x, int y) const { return x > y ? x : y; } };
struct OpMinI { __device__ int operator()(int x, int y) const { return x < y ? x : y; } };

// exclusive scan over threads (thread order); every thread must call; sh: >= 16 entries
template <class T, class Op>
__device__ T block_exclusive(T v, T ident, Op op, T* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d, 64);
        if (lane >= d) x = op(x, y);
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    T carry = ident;
    for (int w = 0; w < wid; w++) carry = op(carry, sh[w]);
    T prev = __shfl_up(x, 1, 64);
    if (lane == 0) prev = ident;
    const T r = op(carry, prev);
    __syncthreads();
    return r;
}

template <class T, class Op>
__device__ T block_reduce(T v, Op op, T* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x = op(x, __shfl_xor(x, d, 64));
    if (lane == 0) sh[wid] = x;
    __syncthreads();
    T r = sh[0];
    for (int w = 1; w < (int)(blockDim.x >> 6); w++) r = op(r, sh[w]);
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

// numpy: np.power(np.minimum(abs_td + eps, 1.0), alpha) on float32 (python floats are cast to
// float32).  The power is correctly rounded (float64 pow rounded once), which is what glibc's
// powf returns except in rare hard cases; numpy >= 1.22 on AVX-512 hosts may use SVML
// instead (within 1 ulp).  See DESIGN.md.
__device__ __forceinline__ float per_priority(float d, float eps, float alpha, float pmax) {
    float x = d + eps;
    x = (x > pmax) ? pmax : x;   // NaN propagates like np.minimum
    return (float)pow((double)x, (double)alpha);
}

__device__ __forceinline__ uint32_t leaf_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// ---------------------------------------------------------------------------------------
// n <= PER_CHUNK SumTree.update calls in order, one workgroup.
//
// SumTree.update(L, p) (R:dqn/utils/sum_tree.py:15-32):
//   max_p, min_p = tree[max_idx], tree[min_idx]; tree[L] = p
//   if p >= max_p: max_idx = L     elif L == max_idx: max_idx = argmax(leaves[:size])
//   if p <= min_p: min_idx = L     elif L == min_idx: min_idx = argmin(leaves[:size])
//   ancestors += p - old
// Without rescans the tracked max value is the running max of the p's (prefix scan) and
// max_idx is the leaf of the last update with p >= running max before it; an update
// triggers a rescan iff it does not raise the max and writes the current max leaf.  The
// kernel scans for the first trigger, applies the updates before it as scans, does the
// rescan on the leaves as they stand after that update, and restarts after it.  Rescans
// are rare (the max / min leaf has to be resampled), so the common case is one pass.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(PER_NT) void k_per_update(PerUpdateArgs a) {
    __shared__ int32_t Ls[PER_CHUNK];
    __shared__ float Ps[PER_CHUNK];
    __shared__ int32_t hkey[PER_HS], hlast[PER_HS];
    __shared__ double topd[PER_TOP];
    __shared__ float shf[16];
    __shared__ int shi[16];
    __shared__ double shd[16];
    __shared__ int64_t shl[16];
    __shared__ int s_mx_i, s_mn_i, s_resx, s_resn;
    __shared__ float s_mx_v, s_mn_v;

    const int tid = threadIdx.x;
    const int n = a.n;
    const int64_t base = a.cap - 1;
    float mp = 0.f;
    if (a.mode == 1) {   // store_transitions: max_priority, or max_priority_high if 0
        const double mv = a.tree[a.ctrl->per_max_idx];
        mp = (mv == 0.0) ? a.pmax : (float)mv;
    }
    double init[PER_IPT];
    int hs[PER_IPT];
#pragma unroll
    for (int k = 0; k < PER_IPT; k++) {
        const int i = tid * PER_IPT + k;   // consecutive items per thread (scan order)
        init[k] = 0.0;
        hs[k] = -1;
        if (i < n) {
            int64_t slot;
            float p;
            if (a.mode == 0) {
                slot = a.slots[i];
                p = per_priority(a.abs_td[i], a.eps, a.alpha, a.pmax);
            } else {
                slot = (a.wptr + i) % a.cap;
                p = mp;
            }
            const int32_t L = (int32_t)(slot + base);
            Ls[i] = L;
            Ps[i] = p;
            init[k] = a.tree[L];
        }
    }
    for (int h = tid; h < PER_HS; h += PER_NT) {
        hkey[h] = -1;
        hlast[h] = -1;
    }
    for (int h = tid; h < PER_TOP; h += PER_NT) topd[h] = 0.0;
    int mx_i = (int)a.ctrl->per_max_idx, mn_i = (int)a.ctrl->per_min_idx;
    float mx_v = (float)a.tree[mx_i], mn_v = (float)a.tree[mn_i];
    __syncthreads();

    // last occurrence of every leaf in the batch (its final value)
#pragma unroll
    for (int k = 0; k < PER_IPT; k++) {
        const int i = tid * PER_IPT + k;
        if (i < n) {
            const int32_t L = Ls[i];
            int h = (int)(leaf_hash((uint32_t)L) & (PER_HS - 1));
            while (true) {
                const int32_t prev = atomicCAS(&hkey[h], -1, L);
                if (prev == -1 || prev == L) break;
                h = (h + 1) & (PER_HS - 1);
            }
            atomicMax(&hlast[h], i);
            hs[k] = h;
        }
    }
    __syncthreads();

    // ---- max / min index tracking, sequential semantics ----
    int s = 0;
    while (true) {
        float pv[PER_IPT];
        bool inr[PER_IPT];
        float lmx = -INFINITY, lmn = INFINITY;
#pragma unroll
        for (int k = 0; k < PER_IPT; k++) {
            const int i = tid * PER_IPT + k;
            inr[k] = i >= s && i < n;
            pv[k] = inr[k] ? Ps[i] : 0.f;
            if (inr[k]) {
                lmx = fmaxf(lmx, pv[k]);
                lmn = fminf(lmn, pv[k]);
            }
        }
        const float exmx = block_exclusive(lmx, -INFINITY, OpMaxF(), shf);
        const float exmn = block_exclusive(lmn, INFINITY, OpMinF(), shf);
        float rmx = fmaxf(mx_v, exmx), rmn = fminf(mn_v, exmn);   // running max / min before item
        bool fx[PER_IPT], fn[PER_IPT];
        float bmx[PER_IPT], bmn[PER_IPT];
        int lfx = -1, lfn = -1;
#pragma unroll
        for (int k = 0; k < PER_IPT; k++) {
            const int i = tid * PER_IPT + k;
            bmx[k] = rmx;
            bmn[k] = rmn;
            fx[k] = inr[k] && pv[k] >= rmx;
            fn[k] = inr[k] && pv[k] <= rmn;
            if (inr[k]) {
                rmx = fmaxf(rmx, pv[k]);
                rmn = fminf(rmn, pv[k]);
            }
            if (fx[k]) lfx = i;
            if (fn[k]) lfn = i;
        }
        const int exlx = block_exclusive(lfx, -1, OpMaxI(), shi);
        const int exln = block_exclusive(lfn, -1, OpMaxI(), shi);
        int lastx = exlx, lastn = exln;
        int mytrig = n;
        int cxb = 0, cnb = 0, tk = -1;
#pragma unroll
        for (int k = 0; k < PER_IPT; k++) {
            const int i = tid * PER_IPT + k;
            const int curx = lastx >= 0 ? Ls[lastx] : mx_i;   // max_idx before update i
            const int curn = lastn >= 0 ? Ls[lastn] : mn_i;
            const bool trig = inr[k] && ((!fx[k] && Ls[i] == curx) || (!fn[k] && Ls[i] == curn));
            if (trig && mytrig == n) {
                mytrig = i;
                cxb = curx;
                cnb = curn;
                tk = k;
            }
            if (fx[k]) lastx = i;
            if (fn[k]) lastn = i;
        }
        const int istar = block_reduce(mytrig, OpMinI(), shi);
        if (istar == n) {   // no rescan left: fold the scans into the state
            const float tmx = block_reduce(lmx, OpMaxF(), shf);
            const float tmn = block_reduce(lmn, OpMinF(), shf);
            const int tlx = block_reduce(lfx, OpMaxI(), shi);
            const int tln = block_reduce(lfn, OpMaxI(), shi);
            if (tlx >= 0) mx_i = Ls[tlx];
            if (tln >= 0) mn_i = Ls[tln];
            mx_v = fmaxf(mx_v, tmx);
            mn_v = fminf(mn_v, tmn);
            break;
        }
        if (mytrig == istar) {   // the owner of the first trigger applies that update
            const float p = pv[tk];
            const int L = Ls[istar];
            s_resx = 0;
            s_resn = 0;
            if (p >= bmx[tk]) { s_mx_i = L; s_mx_v = p; }
            else if (L == cxb) s_resx = 1;
            else { s_mx_i = cxb; s_mx_v = bmx[tk]; }
            if (p <= bmn[tk]) { s_mn_i = L; s_mn_v = p; }
            else if (L == cnb) s_resn = 1;
            else { s_mn_i = cnb; s_mn_v = bmn[tk]; }
        }
        __syncthreads();
        // leaves as they stand after update istar (earlier segments were written already)
        if (tid == 0)
            for (int j = s; j <= istar; j++) a.tree[Ls[j]] = (double)Ps[j];
        __threadfence_block();
        __syncthreads();
        const int64_t sz = a.mode == 1 ? min(a.size + istar + 1, a.cap) : a.ctrl->ring_size;
        if (s_resx) {
            double v;
            const int64_t j = block_arg_extreme(a.tree, base, sz, true, shd, shl, &v);
            if (tid == 0) { s_mx_i = (int)(j + base); s_mx_v = (float)v; }
        }
        if (s_resn) {
            double v;
            const int64_t j = block_arg_extreme(a.tree, base, sz, false, shd, shl, &v);
            if (tid == 0) { s_mn_i = (int)(j + base); s_mn_v = (float)v; }
        }
        __syncthreads();
        mx_i = s_mx_i;
        mx_v = s_mx_v;
        mn_i = s_mn_i;
        mn_v = s_mn_v;
        s = istar + 1;
        __syncthreads();
    }

    // ---- final leaf values and exact ancestor deltas ----
#pragma unroll
    for (int k = 0; k < PER_IPT; k++) {
        const int i = tid * PER_IPT + k;
        if (i < n && hlast[hs[k]] == i) {
            const int64_t L = Ls[i];
            const double fin = (double)Ps[i];
            a.tree[L] = fin;
            const double delta = fin - init[k];
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
    for (int node = tid; node < PER_TOP && node < base; node += PER_NT)
        if (topd[node] != 0.0) a.tree[node] += topd[node];
    if (tid == 0) {
        a.ctrl->per_max_idx = mx_i;
        a.ctrl->per_min_idx = mn_i;
    }
}

int launch_per_sample(const PerSampleArgs& a, hipStream_t s) {
    if (a.Bg < 1 || a.Bg > PER_MAX_B) return set_error(DQNX_EUNSUPPORTED, "PER batch %d outside [1, %d]", a.Bg, PER_MAX_B);
    hipLaunchKernelGGL(k_per_sample, dim3(1 + a.rl_blocks), dim3(PER_NT), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_per_update(const PerUpdateArgs& a, hipStream_t s) {
    if (a.n < 0 || a.n > PER_CHUNK) return set_error(DQNX_EINVAL, "PER update chunk %d > %d", a.n, PER_CHUNK);
    if (a.n == 0) return DQNX_OK;
    hipLaunchKernelGGL(k_per_update, dim3(1), dim3(PER_NT), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
