// Device-side uniform replay sampling, bit-exact with CPython random.sample on a deque.
//
// Replaces R:dqn/replay_memory.py:38-39 (ReplayMemoryNaive.sample_transitions ->
// random.sample(self.replay_buffer, self.batch_size)).  Algorithm restated from CPython
// Lib/random.py (Random.sample, _randbelow_with_getrandbits) and _randommodule.c
// (genrand_uint32); oracle: oracle/pyrandom.c.
//
// Set branch (n > setsize): draws are r = w >> (32 - bit_length(n)), rejected if r >= n,
// redrawn while already selected.  The accepted sequence is therefore the sequence of
// FIRST OCCURRENCES of valid candidates in the MT word stream.  One workgroup walks the
// stream in passes: a pass takes the rest of the current MT block plus as many freshly
// twisted blocks (up to SAMPLE_AHEAD; each twist = 3 dependency phases in LDS) as the
// expected number of draws needs, inserts every word's (value, stream position) into an
// LDS open-addressing table with a 64-bit atomicMin (earliest position per value), and a
// block-wide scan compacts first occurrences in stream order.  One pass normally covers the
// whole minibatch, so the hashing and scan barriers are paid once, not once per block.  The
// block holding the k-th acceptance and the index after it become the new MT state, so the
// state written back equals Python's random.getstate() after the call.
//
// Pool branch (n <= setsize, only while the buffer is tiny): sequential on one lane.
#include "learn.hpp"
#include "mt.hpp"

namespace dqnx {

// Serial genrand_uint32 on one lane (pool branch).
__device__ uint32_t mt_next_serial(uint32_t* mt, uint32_t& pos) {
    if (pos >= 624) {
        int kk;
        for (kk = 0; kk < 227; kk++) mt[kk] = mt[kk + 397] ^ mt_mix(mt[kk], mt[kk + 1]);
        for (; kk < 623; kk++) mt[kk] = mt[kk - 227] ^ mt_mix(mt[kk], mt[kk + 1]);
        mt[623] = mt[396] ^ mt_mix(mt[623], mt[0]);
        pos = 0;
    }
    return mt_temper(mt[pos++]);
}

__device__ __forceinline__ int bit_length64(uint64_t n) { return n ? 64 - __clzll((long long)n) : 0; }

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}



constexpr int SAMPLE_NT = 1024;   // threads of the sampler workgroup (>= 624: one MT word per lane)

constexpr int SAMPLE_AHEAD = 4;   // MT blocks twisted ahead per pass
constexpr int SAMPLE_WPT = 4;     // words per thread per pass: (624 * (1 + AHEAD)) / NT rounded up

template <int HS>  // hash slots (power of two)
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_uniform(SampleArgs a) {
    constexpr int NT = SAMPLE_NT, NW = NT / 64;
    __shared__ unsigned long long tab[HS];
    __shared__ uint32_t blk[SAMPLE_AHEAD + 1][624];   // [0] current block, [1..] twisted ahead
    __shared__ int wave_tot[NW];
    __shared__ int s_final;

    if (blockIdx.x > 0) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    DQNX_STAMP(a.stamps, 0);
    const int64_t n = a.n_dev ? *a.n_dev : a.n_val;
    const int k = a.k;
    if (k < 0 || (int64_t)k > n) {
        if (tid == 0) atomicExch(a.err, DQNX_DEVERR_SAMPLE_TOO_LARGE);
        return;
    }
    if (k == 0) return;
    int64_t phys_base = 0;
    if (a.phys_out) {
        const int64_t wptr = *a.wptr_dev;
        phys_base = wptr - n;
        if (phys_base < 0) phys_base += a.capacity;
    }
    if (tid < 624) blk[0][tid] = a.state[tid];
    uint32_t pos = a.state[624];

    if (n <= a.setsize) {
        // ---- pool branch: one lane, CPython order (only while the buffer is tiny) ----
        __syncthreads();
        if (tid == 0) {
            uint32_t* mt = blk[0];
            int32_t* pool = a.pool;
            for (int64_t i = 0; i < n; i++) pool[i] = (int32_t)i;
            for (int i = 0; i < k; i++) {
                const uint64_t m = (uint64_t)(n - i);
                const int bits = bit_length64(m);
                uint64_t r;
                do { r = mt_next_serial(mt, pos) >> (32 - bits); } while (r >= m);
                const int32_t j = pool[r];
                a.out[i] = j;
                if (a.phys_out && i >= a.shard_begin && i < a.shard_begin + a.shard_len) {
                    int64_t ps = phys_base + j;
                    if (ps >= a.capacity) ps -= a.capacity;
                    a.phys_out[i - a.shard_begin] = (int32_t)ps;
                }
                pool[r] = pool[n - i - 1];
            }
            for (int i = 0; i < 624; i++) a.state[i] = mt[i];
            a.state[624] = pos;
        }
        return;
    }

    // ---- set branch ----
    DQNX_STAMP(a.stamps, 1);
#pragma unroll
    for (int i = 0; i < HS / NT; i++) tab[tid + i * NT] = ~0ull;
    const int bits = bit_length64((uint64_t)n);
    const uint32_t shift = 32u - (uint32_t)bits;
    const float inv_accept = (float)((double)(1ull << bits) / (double)n);   // words per valid draw
    int accepted = 0;
    uint32_t spos0 = 0;      // stream position (since the call began) of blk[0][pos]
    int iter = 0;
    __syncthreads();
    while (true) {
        // ---- plan the pass: the rest of blk[0], then nb freshly twisted blocks ----
        const int avail = 624 - (int)pos;
        const int need = k - accepted;
        // expected words for `need` more acceptances (rejections + repeats), with margin
        const float est = need * inv_accept * (1.f + (float)(accepted + need) / (2.f * (float)n)) + 32.f + need / 16.f;
        int nb = (int)ceilf((est - (float)avail) / 624.f);
        const int room = (3 * HS / 4 - accepted - avail) / 624;   // keep the table <= 3/4 full
        nb = nb > room ? room : nb;
        nb = nb > SAMPLE_AHEAD ? SAMPLE_AHEAD : nb;
        nb = nb < (avail == 0 ? 1 : 0) ? 1 : nb;
        for (int j = 1; j <= nb; j++) mt_twist_into(blk[j - 1], blk[j]);
        if (iter == 0) DQNX_STAMP(a.stamps, 2);
        const int nwords = avail + 624 * nb;
        // ---- insert: thread t owns the contiguous words [t*m, t*m + m) of the pass ----
        const int m = (nwords + NT - 1) / NT;
        uint32_t cv[SAMPLE_WPT], hv[SAMPLE_WPT];
        bool val[SAMPLE_WPT];
        unsigned long long prev[SAMPLE_WPT];
#pragma unroll
        for (int u = 0; u < SAMPLE_WPT; u++) {   // first probe of every word, issued back to back
            const int w = tid * m + u;
            val[u] = false;
            cv[u] = 0;
            hv[u] = 0;
            prev[u] = ~0ull;
            if (u < m && w < nwords) {
                const int bw = (w < avail) ? 0 : 1 + (w - avail) / 624;
                const int ow = (w < avail) ? (int)pos + w : (w - avail) % 624;
                const uint32_t c = mt_temper(blk[bw][ow]) >> shift;
                if ((int64_t)c < n) {   // insert (value, stream position); earliest position wins
                    val[u] = true;
                    cv[u] = c;
                    hv[u] = hash_u32(c) & (HS - 1);
                    prev[u] = atomicCAS(&tab[hv[u]], ~0ull, ((unsigned long long)c << 32) | (spos0 + (uint32_t)w));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < SAMPLE_WPT; u++) {   // resolve: same value -> keep the minimum; else probe on
            if (!val[u] || prev[u] == ~0ull) continue;
            const unsigned long long key = ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u));
            uint32_t h = hv[u];
            unsigned long long pv = prev[u];
            while (true) {
                if ((uint32_t)(pv >> 32) == cv[u]) { atomicMin(&tab[h], key); break; }
                h = (h + 1) & (HS - 1);
                pv = atomicCAS(&tab[h], ~0ull, key);
                if (pv == ~0ull) break;
            }
            hv[u] = h;
        }
        if (tid == 0) s_final = -1;
        __syncthreads();
        if (iter == 0) DQNX_STAMP(a.stamps, 3);
        // ---- first occurrences, exclusive scan in stream (= thread, then u) order ----
        int cnt = 0;
        bool first[SAMPLE_WPT];
#pragma unroll
        for (int u = 0; u < SAMPLE_WPT; u++) {
            first[u] = val[u] && (uint32_t)(tab[hv[u]] & 0xffffffffull) == spos0 + (uint32_t)(tid * m + u);
            cnt += first[u] ? 1 : 0;
        }
        int incl = cnt;   // wave inclusive scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wave_tot[wid] = incl;
        __syncthreads();
        if (iter == 0) DQNX_STAMP(a.stamps, 4);
        int before = incl - cnt, total = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const int tw = wave_tot[w];
            before += (w < wid) ? tw : 0;
            total += tw;
        }
        int r = accepted + before;
#pragma unroll
        for (int u = 0; u < SAMPLE_WPT; u++) {
            if (!first[u]) continue;
            if (r < k) {
                const int32_t c = (int32_t)cv[u];
                a.out[r] = c;
                if (a.phys_out && r >= a.shard_begin && r < a.shard_begin + a.shard_len) {
                    int64_t ps = phys_base + (int64_t)c;
                    if (ps >= a.capacity) ps -= a.capacity;
                    a.phys_out[r - a.shard_begin] = (int32_t)ps;
                }
                if (r == k - 1) s_final = tid * m + u;   // word index of the k-th acceptance
            }
            r++;
        }
        __syncthreads();
        DQNX_STAMP(a.stamps, 5 + (iter < 9 ? iter : 9));
        iter++;
        accepted += total;
        if (accepted >= k) {
            // state after the k-th draw: the block holding that word, index just past it
            const int wf = s_final;
            const int bf = (wf < avail) ? 0 : 1 + (wf - avail) / 624;
            const uint32_t nx = (uint32_t)((wf < avail) ? (int)pos + wf + 1 : (wf - avail) % 624 + 1);
            if (bf > 0 && tid < 624) a.state[tid] = blk[bf][tid];
            if (tid == 0) a.state[624] = nx;
            break;
        }
        // the whole pass was consumed: continue from the last block's end
        spos0 += (uint32_t)nwords;
        if (nb > 0) {
            if (tid < 624) blk[0][tid] = blk[nb][tid];
            __syncthreads();
        }
        pos = 624;
    }
    (void)iter;
    DQNX_STAMP(a.stamps, 15);
}

// Logical positions (given by the caller) -> physical ring slots of the local shard.
__global__ void k_idx_to_phys(const int32_t* idx, int32_t* phys, int shard_begin, int n, const dqnx_ctrl* ctrl,
                              int64_t capacity, RelayoutArgs rl, int pblocks) {
    if ((int)blockIdx.x >= pblocks) {
        relayout_run(rl, blockIdx.x - pblocks, gridDim.x - pblocks);
        return;
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t size = ctrl->ring_size, wptr = ctrl->ring_wptr;
    const int64_t base = ((wptr - size) % capacity + capacity) % capacity;
    phys[i] = (int32_t)((base + idx[shard_begin + i]) % capacity);
}

int launch_idx_to_phys(const int32_t* idx, int32_t* phys, int shard_begin, int n, dqnx_ctrl* ctrl, int64_t capacity,
                       const RelayoutArgs* rl, int rl_blocks, hipStream_t s) {
    RelayoutArgs r = {};
    if (rl && rl_blocks > 0) r = *rl;
    else rl_blocks = 0;
    const int pb = (n + 255) / 256;
    hipLaunchKernelGGL(k_idx_to_phys, dim3(pb + 4 * rl_blocks), dim3(256), 0, s, idx, phys, shard_begin, n, ctrl,
                       capacity, r, pb);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int64_t sample_setsize(int64_t k) {
    int64_t setsize = 21;
    if (k > 5) {
        const double e = ceil(log((double)(k * 3)) / log(4.0));
        int64_t p = 1;
        for (int i = 0; i < (int)e; i++) p *= 4;
        setsize += p;
    }
    return setsize;
}

int sample_hash_slots(int32_t k) {
    // The table holds every value accepted so far plus one pass of words; the kernel caps a
    // pass at 3/4 of the table minus the accepted values, and a pass needs room for >= 1 block.
    int64_t need = 4 * ((int64_t)k + 624);   // load factor <= ~1/4 at the usual one-pass size
    int hs = 2048;
    while (hs < need && hs < 16384) hs <<= 1;
    if (4 * ((int64_t)k + 624) > 3 * (int64_t)hs) return -1;
    return hs;
}

int launch_sample_uniform(const SampleArgs& a, hipStream_t s) {
    const int hs = sample_hash_slots(a.k);
    if (hs < 0) return set_error(DQNX_EUNSUPPORTED, "sample: k=%d too large for the LDS table", a.k);
    switch (hs) {
        case 2048: hipLaunchKernelGGL(k_sample_uniform<2048>, dim3(1 + a.rl_blocks), dim3(SAMPLE_NT), 0, s, a); break;
        case 4096: hipLaunchKernelGGL(k_sample_uniform<4096>, dim3(1 + a.rl_blocks), dim3(SAMPLE_NT), 0, s, a); break;
        case 8192: hipLaunchKernelGGL(k_sample_uniform<8192>, dim3(1 + a.rl_blocks), dim3(SAMPLE_NT), 0, s, a); break;
        default: hipLaunchKernelGGL(k_sample_uniform<16384>, dim3(1 + a.rl_blocks), dim3(SAMPLE_NT), 0, s, a); break;
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx

extern "C" uint64_t dqnx_sample_scratch_bytes(int64_t n, int32_t k) {
    const int64_t ss = dqnx::sample_setsize(k);
    const int64_t m = n < ss ? n : ss;
    return (uint64_t)((m + 64) * sizeof(int32_t));
}

extern "C" int dqnx_sample_uniform(uint32_t* mt625, int64_t n, int32_t k, int32_t* out, void* scratch,
                                   int32_t* err, void* stream) {
    if (!mt625 || !out || !err || (k > 0 && !scratch) || n < 0 || k < 0)
        return dqnx::set_error(DQNX_EINVAL, "dqnx_sample_uniform: bad argument");
    if (n >= (int64_t)1 << 31) return dqnx::set_error(DQNX_EUNSUPPORTED, "dqnx_sample_uniform: n >= 2^31");
    dqnx::SampleArgs a = {};
    a.state = mt625;
    a.n_dev = nullptr;
    a.n_val = n;
    a.k = k;
    a.setsize = dqnx::sample_setsize(k);
    a.out = out;
    a.err = err;
    a.pool = (int32_t*)scratch;
    a.phys_out = nullptr;
    return dqnx::launch_sample_uniform(a, (hipStream_t)stream);
}
