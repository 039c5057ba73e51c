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
// stream one MT block (<= 624 words) at a time: the 624-word twist runs in 3 parallel
// phases in LDS, every lane tempers one word, inserts (value, stream position) into an
// LDS open-addressing table with a 64-bit atomicMin (keeps the earliest position per
// value), and a block-wide ballot scan compacts first occurrences in stream order.
// The position after the k-th acceptance becomes the new MT index, so the state written
// back equals Python's random.getstate() after the call.
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

template <int HS>  // hash slots (power of two)
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_uniform(SampleArgs a) {
    constexpr int NT = SAMPLE_NT, NW = NT / 64;
    __shared__ unsigned long long tab[HS];
    __shared__ uint32_t mt[624];
    __shared__ uint32_t tmp[624];
    __shared__ int wave_cnt[NW];
    __shared__ int s_newpos;

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
    if (tid < 624) mt[tid] = a.state[tid];
    uint32_t pos = a.state[624];

    if (n <= a.setsize) {
        // ---- pool branch: one lane, CPython order (only while the buffer is tiny) ----
        __syncthreads();
        if (tid == 0) {
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
    const uint32_t shift = 32u - (uint32_t)bit_length64((uint64_t)n);
    int accepted = 0;
    uint32_t consumed = 0;   // words consumed before the current MT block (stream position base)
    bool twisted = false;
    int iter = 0;
    __syncthreads();
    while (true) {
        if (pos >= 624) {   // parallel twist: 3 dependency phases (CPython genrand_uint32)
            mt_twist_block(mt, tmp);
            pos = 0;
            twisted = true;
        }
        const int avail = 624 - (int)pos;
        bool valid = false, first = false;
        uint32_t c = 0, sp = 0, h = 0;
        if (tid < avail) {
            c = mt_temper(mt[pos + tid]) >> shift;
            sp = consumed + (uint32_t)tid;
            valid = (int64_t)c < n;
            if (valid) {   // insert (value, stream position); keep the earliest position per value
                const unsigned long long key = ((unsigned long long)c << 32) | sp;
                h = hash_u32(c) & (HS - 1);
                while (true) {
                    const unsigned long long prev = atomicCAS(&tab[h], ~0ull, key);
                    if (prev == ~0ull) break;
                    if ((uint32_t)(prev >> 32) == c) { atomicMin(&tab[h], key); break; }
                    h = (h + 1) & (HS - 1);
                }
            }
        }
        if (tid == 0) s_newpos = -1;
        __syncthreads();
        if (valid) first = (uint32_t)(tab[h] & 0xffffffffull) == sp;   // h = the value's slot
        // block-wide exclusive scan of `first` in thread (= stream) order
        const unsigned long long bal = __ballot(first);
        const int wprefix = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wave_cnt[wid] = __popcll(bal);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const int cw = wave_cnt[w];
            before += (w < wid) ? cw : 0;
            total += cw;
        }
        if (first) {
            const int r = accepted + before + wprefix;
            if (r < k) {
                a.out[r] = (int32_t)c;
                if (a.phys_out && r >= a.shard_begin && r < a.shard_begin + a.shard_len) {
                    int64_t ps = phys_base + (int64_t)c;
                    if (ps >= a.capacity) ps -= a.capacity;
                    a.phys_out[r - a.shard_begin] = (int32_t)ps;
                }
                if (r == k - 1) s_newpos = (int)pos + tid + 1;
            }
        }
        __syncthreads();
        DQNX_STAMP(a.stamps, 2 + (iter < 12 ? iter : 12));
        iter++;
        accepted += total;
        if (accepted >= k) {
            pos = (uint32_t)s_newpos;
            break;
        }
        consumed += (uint32_t)avail;
        pos = 624;
    }
    (void)iter;
    if (twisted && tid < 624) a.state[tid] = mt[tid];
    if (tid == 0) a.state[624] = pos;
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
    int64_t need = 2 * ((int64_t)k + 624);
    int hs = 2048;
    while (hs < need && hs < 16384) hs <<= 1;
    if ((int64_t)k + 624 > (int64_t)(0.9 * hs)) return -1;
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
