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
#include "sample_body.hpp"

namespace dqnx {

constexpr int SAMPLE_NT = 1024;   // threads of the sampler workgroup

template <int HS>  // hash slots (power of two)
__global__ __launch_bounds__(SAMPLE_NT) void k_sample_uniform(SampleArgs a) {
    __shared__ SampleLds<SAMPLE_NT, HS> S;
    if (blockIdx.x > 0) {   // spare workgroups: blocked weight copies for the fused plan
        relayout_run(a.rl, blockIdx.x - 1, gridDim.x - 1);
        return;
    }
    sample_uniform_body<SAMPLE_NT, HS>(a, S);
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
