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
#include "sample_pipe.hpp"

namespace dqnx {

constexpr int SAMPLE_NT = 1024;   // threads of the sampler workgroup
constexpr int SAMPLE_LDS_MAX_HS = 16384;      // largest LDS table of k_sample_uniform (128 KiB)

// k <= SAMPLE_FAST_MAX_K: the bitmap-dedup sampler (sample_pipe.hpp)
__global__ __launch_bounds__(SAMPLE_FAST_NT) void k_sample_fast(SampleArgs a) {
    __shared__ SampleFastUnion S;
    if (blockIdx.x > 0) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    sample_fast_body(a, S);
}

template <int HS>  // hash slots (power of two) in LDS
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_uniform(SampleArgs a) {
    __shared__ SampleLds<SAMPLE_NT, HS> S;
    if (blockIdx.x > 0) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    sample_uniform_body<SAMPLE_NT, HS>(a, S, S.tab);
}

template <int HS>  // hash slots (power of two) in global scratch (a.gtab): k beyond the LDS tables
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_uniform_g(SampleArgs a) {
    __shared__ SampleLdsBase<SAMPLE_NT> S;
    if (blockIdx.x > 0) {
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    sample_uniform_body<SAMPLE_NT, HS>(a, S, a.gtab);
}


// k beyond the LDS hash tables, population <= 2^20 (sample_bitmap_body): the dedup state in LDS
constexpr int SAMPLE_BITMAP_AH = 5, SAMPLE_BITMAP_BMX = 2048;   // 158.7 KiB of LDS: passes of 5 new blocks (4: 14 passes at k = 32768)
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_bitmap(SampleArgs a) {
    __shared__ SampleBitmapLds<SAMPLE_NT, SAMPLE_BITMAP_AH, SAMPLE_BITMAP_BMX> S;
    if (blockIdx.x > 0) {
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    sample_bitmap_body<SAMPLE_NT, SAMPLE_BITMAP_AH, SAMPLE_BITMAP_BMX>(a, S);
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
    DQNX_LAUNCH(k_idx_to_phys, dim3(pb + 4 * rl_blocks), dim3(256), 0, s, idx, phys, shard_begin, n, ctrl,
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

// LDS table of k_sample_uniform for k (the original rule), or -1 if k needs more than 16384 slots
static int lds_hash_slots(int32_t k) {
    // The table holds every value accepted so far plus one pass of words; the kernel caps a
    // pass at 3/4 of the table minus the accepted values, and a pass needs room for >= 1 block.
    int64_t need = 4 * ((int64_t)k + 624);   // load factor <= ~1/4 at the usual one-pass size
    int hs = 2048;
    while (hs < need && hs < SAMPLE_LDS_MAX_HS) hs <<= 1;
    if (need > 3 * (int64_t)hs) return -1;
    return hs;
}

// global table of k_sample_uniform_g (k beyond every LDS table)
static int global_hash_slots(int32_t k) {
    const int64_t need = 4 * ((int64_t)k + 624);
    int64_t hs = 2 * SAMPLE_LDS_MAX_HS;
    while (hs < need) hs <<= 1;
    return hs > ((int64_t)1 << 20) ? -1 : (int)hs;   // k > ~260 K: beyond any configured minibatch
}

int sample_hash_slots(int32_t k) {
    if (k <= SAMPLE_FAST_MAX_K) return SAMPLE_LDS_MAX_HS;
    const int hs = lds_hash_slots(k);
    return hs > 0 ? hs : global_hash_slots(k);
}

// smallest k routed to the fast sampler (DQNX_SAMPLER_FAST_MIN overrides, for measurements)
static int fast_min_k() {
    static const int v = tuning_knob("DQNX_SAMPLER_FAST_MIN", SAMPLE_FAST_MIN_K);
    return v;
}

int mt_cache_target_blocks(int32_t k, int64_t n) {
    if (k < fast_min_k() || k > SAMPLE_FAST_MAX_K || n <= k) return 0;   // the fast path only
    // the fast sampler's word estimate (sample_pipe.hpp) at population n, from a fully consumed
    // state block; + the state block itself
    int bits = 0;
    while (bits < 63 && ((int64_t)1 << bits) <= n) bits++;
    const double nf = (double)n, pf = nf / (double)((int64_t)1 << bits);
    const double D = nf * log1p((double)k / (nf - (double)k));
    const double words = D / pf + 8.0 * sqrt(D * (1.0 - pf)) / pf + 64.0;
    const int b = (int)ceil(words / 624.0) + 1;
    return b > MTC_MAX_BLOCKS ? MTC_MAX_BLOCKS : b;
}

uint64_t sample_table_bytes(int32_t k) {
    if (k <= SAMPLE_FAST_MAX_K || lds_hash_slots(k) > 0) return 0;
    const int hs = global_hash_slots(k);
    return hs > 0 ? (uint64_t)hs * 8 : 0;
}

int launch_sample_uniform(const SampleArgs& a_in, hipStream_t s) {
    SampleArgs a = a_in;
    a.test_flags = route_flag("DQNX_SAMPLER_FORCE_FALLBACK") ? 1 : 0;
    const dim3 grid(1 + a.rl_blocks);
    const int lhs = lds_hash_slots(a.k);
    if (a.k <= SAMPLE_FAST_MAX_K && (a.k >= fast_min_k() || route_flag("DQNX_SAMPLER_FAST") || a.test_flags) &&
        !route_flag("DQNX_SAMPLER_OLD")) {
        DQNX_LAUNCH(k_sample_fast, grid, dim3(SAMPLE_FAST_NT), 0, s, a);
    } else if (lhs > 0) {
        switch (lhs) {
            case 2048: DQNX_LAUNCH(k_sample_uniform<2048>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 4096: DQNX_LAUNCH(k_sample_uniform<4096>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 8192: DQNX_LAUNCH(k_sample_uniform<8192>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            default: DQNX_LAUNCH(k_sample_uniform<16384>, grid, dim3(SAMPLE_NT), 0, s, a); break;
        }
    } else if (a.capacity > 0 && a.capacity <= SAMPLE_BITMAP_MAX_N && !route_flag("DQNX_SAMPLER_GLOBAL")) {
        // k beyond the LDS tables over a replay of <= 2^20 slots: the LDS bitmap body (configs[3] weak
        // scaling at world 8: k = 32768, n = 10^6); DQNX_SAMPLER_GLOBAL keeps the global-table body
        DQNX_LAUNCH(k_sample_bitmap, grid, dim3(SAMPLE_NT), 0, s, a);
    } else {
        const int ghs = global_hash_slots(a.k);
        if (ghs < 0) return set_error(DQNX_EUNSUPPORTED, "sample: k=%d too large", a.k);
        if (!a.gtab) return set_error(DQNX_EINVAL, "sample: k=%d needs a global table", a.k);
        switch (ghs) {
            case 32768: DQNX_LAUNCH(k_sample_uniform_g<32768>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 65536: DQNX_LAUNCH(k_sample_uniform_g<65536>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 131072: DQNX_LAUNCH(k_sample_uniform_g<131072>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 262144: DQNX_LAUNCH(k_sample_uniform_g<262144>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            case 524288: DQNX_LAUNCH(k_sample_uniform_g<524288>, grid, dim3(SAMPLE_NT), 0, s, a); break;
            default: DQNX_LAUNCH(k_sample_uniform_g<1048576>, grid, dim3(SAMPLE_NT), 0, s, a); break;
        }
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx

// test-hook scratch: [n, n as the ring write pointer | MT block cache (empty) | pool | global table]
static uint64_t hook_pool_off() { return 256 + ((uint64_t)dqnx::mt_cache_words() * 4 + 255) / 256 * 256; }

extern "C" uint64_t dqnx_sample_scratch_bytes(int64_t n, int32_t k) {
    const int64_t ss = dqnx::sample_setsize(k);
    const int64_t m = n < ss ? n : ss;
    const uint64_t pool = ((uint64_t)((m + 64) * sizeof(int32_t)) + 255) / 256 * 256;
    return hook_pool_off() + pool + dqnx::sample_table_bytes(k);
}

extern "C" int dqnx_sample_uniform(uint32_t* mt625, int64_t n, int32_t k, int32_t* out, void* scratch,
                                   int32_t* err, void* stream) {
    if (!mt625 || !out || !err || (k > 0 && !scratch) || n < 0 || k < 0)
        return dqnx::set_error(DQNX_EINVAL, "dqnx_sample_uniform: bad argument");
    if (n >= (int64_t)1 << 31) return dqnx::set_error(DQNX_EUNSUPPORTED, "dqnx_sample_uniform: n >= 2^31");
    dqnx::SampleArgs a = {};
    a.state = mt625;
    a.k = k;
    a.setsize = dqnx::sample_setsize(k);
    a.out = out;
    a.err = err;
    char* sc = (char*)scratch;
    {   // the population size as the device-side ring size (the samplers read it from memory)
        const int64_t hv[2] = {n, n};
        hipError_t e = hipMemcpyAsync(sc, hv, sizeof(hv), hipMemcpyHostToDevice, (hipStream_t)stream);
        if (e == hipSuccess) e = hipMemsetAsync(sc + 256, 0, (size_t)dqnx::mt_cache_words() * 4, (hipStream_t)stream);
        if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);   // hv is on this stack frame
        if (e != hipSuccess) return dqnx::set_hip_error(e, "dqnx_sample_uniform staging", __FILE__, __LINE__);
    }
    a.n_dev = (const int64_t*)sc;
    a.n_val = n;
    a.capacity = n;   // (the population bound the routes check; no physical slots are written)
    a.wptr_dev = (const int64_t*)sc + 1;
    a.mtc = (uint32_t*)(sc + 256);
    a.mtc_blocks = 0;
    a.pool = (int32_t*)(sc + hook_pool_off());
    a.phys_out = nullptr;
    {
        const int64_t ss = a.setsize, m = n < ss ? n : ss;
        const uint64_t pool = ((uint64_t)((m + 64) * sizeof(int32_t)) + 255) / 256 * 256;
        a.gtab = dqnx::sample_table_bytes(k) ? (unsigned long long*)(sc + hook_pool_off() + pool) : nullptr;
    }
    return dqnx::launch_sample_uniform(a, (hipStream_t)stream);
}
