// Fast uniform replay sampler: random.sample(deque, k) bit-exact with CPython
// (R:dqn/replay_memory.py:38-39; algorithm notes in sample.hip), for k <= SAMPLE_FAST_MAX_K.
//
// The set branch accepts the FIRST OCCURRENCES of valid candidates c = w >> (32 - bits), c < n,
// in the MT19937 word stream.  Measured on one MI355X CU (tools/sampler_micro.hip), a 64-bit LDS
// atomicCAS costs ~1.8 cycles per word and a 32-bit LDS atomicOr ~0.4, so the dedup no longer
// hashes every word into a (value, position) table:
//   1. one round: the rest of the state block plus nb freshly twisted blocks, nb sized for the
//      expected number of draws plus an 8-sigma margin (one round covers every n at k <= 4608);
//   2. every valid word sets its "seen" bit in an LDS bitmap indexed by c mod 2^19 (atomicOr);
//      a word that finds its bit already set (its value repeats, or shares the slot) enters a
//      small exact (value, earliest position) table (atomicCAS / atomicMin);
//   3. every other valid word looks its value up in that table: found means a later word
//      repeats it, and it enters the table too;
//      a word in the table is a first occurrence iff its position is the minimum of its value,
//      every other valid word is a first occurrence outright;
//   4. first occurrences are ranked in stream order: word g = t + 1024 u sits in row u, ranked
//      by ballot/mbcnt within the wave, earlier waves of the row, earlier rows.
// The block holding the k-th acceptance and the index just past it become the new state, i.e.
// Python's random.getstate() after the call.  A shortfall beyond the margin (never observed;
// probability far below 1e-12) falls back to k_sample_uniform's exact multi-pass body on the
// same LDS, from the unchanged input state.
#pragma once
#include "sample_body.hpp"

namespace dqnx {

constexpr int SAMPLE_FAST_NT = 1024;
constexpr int SAMPLE_FAST_NB = 22;                   // MT blocks in LDS: the state block + 21 twists
constexpr int SAMPLE_FAST_ROWS = (624 * SAMPLE_FAST_NB + SAMPLE_FAST_NT - 1) / SAMPLE_FAST_NT;   // 14
constexpr int SAMPLE_FAST_SLOTS = 1 << 19;           // seen-bitmap slots, 1 bit each (64 KiB)
constexpr int SAMPLE_FAST_XS = 4096;                 // exact table for contended words (32 KiB)
constexpr int SAMPLE_FAST_MAX_K = 4608;
// below this k the multi-pass kernel is as fast or faster (measured in context on MI355X at
// k = 1024: 7.3 vs 8.3 us; at k = 4096 the fast path wins, 13.7 vs 15.8 us)
constexpr int SAMPLE_FAST_MIN_K = 2048;

struct SampleFastLds {
    uint32_t bm[SAMPLE_FAST_SLOTS / 32];         // "seen" bit of slot c mod 2^19
    unsigned long long xt[SAMPLE_FAST_XS];       // (value << 32 | stream position), contended words only
    uint32_t blk[SAMPLE_FAST_NB][624];           // [0]: the input state block
    int row_wave[SAMPLE_FAST_ROWS][16];          // first occurrences per (row, wave)
    int s_final_g, s_short, s_total;
    int miss_w[16];
};
union SampleFastUnion {                          // the fallback reuses the same LDS
    SampleFastLds f;
    SampleLds<SAMPLE_FAST_NT, 16384> old;
};

// LDS-only barrier: no wait for this wave's global loads / stores (cross-wave data is all in LDS)
__device__ __forceinline__ void sample_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// twist_into with the LDS-only barrier (sample_body.hpp's form ends with __syncthreads)
__device__ __forceinline__ void mt_twist_into_lds(const uint32_t* old, uint32_t* nw) {
    const int t = threadIdx.x;
    if (t < 227) {
        const uint32_t a0 = old[t + 397] ^ mt_mix(old[t], old[t + 1]);
        const uint32_t a1 = a0 ^ mt_mix(old[t + 227], old[t + 228]);
        nw[t] = a0;
        nw[t + 227] = a1;
        if (t < 169) nw[t + 454] = a1 ^ mt_mix(old[t + 454], old[t + 455]);
        if (t == 169) nw[623] = a1 ^ mt_mix(old[623], old[397] ^ mt_mix(old[0], old[1]));
    }
    sample_lds_sync();
}

__device__ __forceinline__ bool sample_fast_path(const SampleArgs& a, SampleFastUnion& U);

__device__ __forceinline__ void sample_fast_body(const SampleArgs& a, SampleFastUnion& U) {
    if (!sample_fast_path(a, U)) {   // pool branch / error / k beyond the fast path / shortfall
        __syncthreads();
        sample_uniform_body<SAMPLE_FAST_NT, 16384>(a, U.old, U.old.tab);
    }
}

// Diagnostic builds: phase times kept in thread 0's registers and stored once at the end (a
// global store per phase would make every following barrier wait for it).
#ifdef DQNX_STAMPS
#define FAST_TS(i) do { if (tid == 0) ts[i] = (int64_t)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define FAST_TS(i) do { } while (0)
#endif

// true when the call is done; false: the caller runs the general body from the unchanged state
__device__ __forceinline__ bool sample_fast_path(const SampleArgs& a, SampleFastUnion& U) {
    SampleFastLds& S = U.f;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
#ifdef DQNX_STAMPS
    int64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    FAST_TS(0);
    // every global load of the call issued at once, unconditionally (the launcher guarantees
    // n_dev, wptr_dev and mtc are valid): a conditional load splits the block and the value it
    // feeds to a scalar gets waited for right there, serialising the round trips
    const int64_t n = gld(a.n_dev);
    const int64_t wptr = gld(a.wptr_dev);
    const uint32_t* src = a.state_in ? a.state_in : a.state;
    const uint32_t st_j = gld(src + (tid < 624 ? tid : 624));
    const int pos = (int)gld(src + 624);
    const int k = a.k;
    // the MT block cache (learn.hpp), fetched speculatively with the state: word f = tid + 1024 i
    // of the cached blocks (block f / 624, offset f % 624); block 0 must equal the state block
    constexpr int CW = (MTC_MAX_BLOCKS * 624 + SAMPLE_FAST_NT - 1) / SAMPLE_FAST_NT;
    const int cblocks = a.mtc_blocks;
    const int ccnt = (int)gld(a.mtc);
    const int clim = cblocks > 0 ? cblocks * 624 - 1 : 0;
    uint32_t cw[CW];
#pragma unroll
    for (int i = 0; i < CW; i++) {
        const int f = tid + SAMPLE_FAST_NT * i;
        cw[i] = (i * SAMPLE_FAST_NT < cblocks * 624) ? gld(a.mtc + 64 + (f < clim ? f : clim)) : 0u;
    }
    // LDS tables cleared while the loads are in flight (16-byte stores)
    {
        uint4* bm4 = reinterpret_cast<uint4*>(S.bm);
#pragma unroll
        for (int i = 0; i < SAMPLE_FAST_SLOTS / 128 / SAMPLE_FAST_NT; i++)
            bm4[tid + i * SAMPLE_FAST_NT] = make_uint4(0u, 0u, 0u, 0u);
        uint4* xt4 = reinterpret_cast<uint4*>(S.xt);
#pragma unroll
        for (int i = 0; i < SAMPLE_FAST_XS / 2 / SAMPLE_FAST_NT; i++)
            xt4[tid + i * SAMPLE_FAST_NT] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    if (k < 0 || (int64_t)k > n || k > SAMPLE_FAST_MAX_K || n <= a.setsize) return false;
    if (k == 0) return true;
    int64_t phys_base = 0;
    if (a.phys_out) {
        phys_base = wptr - n;
        if (phys_base < 0) phys_base += a.capacity;
    }
    if (tid < 624) S.blk[0][tid] = st_j;
    if (tid == 0) { S.s_final_g = -1; S.s_short = 0; }
    const int bits = bit_length64((uint64_t)n);
    const uint32_t shift = 32u - (uint32_t)bits;
    const int avail = 624 - pos;
    // words for k distinct draws: D = n ln(n / (n - k)) draws below n, each taking 1/p words
    // (p = n / 2^bits); margin 8 sigma of the negative binomial + 64
    int nb;
    {
        const float nf = (float)n, pf = nf / (float)(1ull << bits);
        const float D = nf * log1pf((float)k / (nf - (float)k));
        const float words = D / pf + 8.f * sqrtf(D * (1.f - pf)) / pf + 64.f;
        nb = (int)ceilf((words - (float)avail) / 624.f);
        nb = nb < 0 ? 0 : nb;
        nb = nb > SAMPLE_FAST_NB - 1 ? SAMPLE_FAST_NB - 1 : nb;
        if (avail == 0 && nb == 0) nb = 1;
    }
    const int nwords = avail + 624 * nb;
    // cache hit: block 0 equals the state block (tid < 624 holds its word in cw[0])
    {
        const unsigned long long mb = __ballot(tid < 624 && cw[0] != st_j);
        if (lane == 0) S.miss_w[wid] = mb != 0ull;
    }
    sample_lds_sync();
    bool miss = ccnt < 1 || cblocks < 1;
#pragma unroll
    for (int w = 0; w < 16; w++) miss = miss || S.miss_w[w];
    FAST_TS(1);
    int nbc = miss ? 0 : min(nb, min(ccnt, cblocks) - 1);   // blocks 1..nbc from the cache
    if (nbc > 0) {
#pragma unroll
        for (int i = 0; i < CW; i++) {
            const int f = tid + SAMPLE_FAST_NT * i, b = f / 624;
            if (b >= 1 && b <= nbc) S.blk[b][f - 624 * b] = cw[i];
        }
        sample_lds_sync();
    }
    for (int b = nbc + 1; b <= nb; b++) mt_twist_into_lds(S.blk[b - 1], S.blk[b]);   // ends with a barrier
    FAST_TS(2);

    // Every per-row phase below is a rolled loop whose per-word values are recomputed from the
    // blocks in LDS instead of kept in unrolled register arrays (compact code).  The blocks are
    // contiguous in LDS, so stream word g is simply blk_flat[pos + g].  The candidates are
    // uniform in [0, n), so their low bits index the bitmap and the table directly (no hash:
    // the sampler is VALU-bound on its one CU, every op per word counts).
    const uint32_t* bflat = &S.blk[0][0];
    auto word = [&](int g, uint32_t& c) -> bool {   // candidate of stream word g; valid?
        if (g >= nwords) return false;
        c = mt_temper(bflat[pos + g]) >> shift;
        return (int64_t)c < n;
    };
    // (value, stream position) into the exact table, keeping the earliest position per value
    auto xt_insert = [&](uint32_t c, uint32_t g) {
        const unsigned long long key = ((unsigned long long)c << 32) | g;
        uint32_t h = c & (SAMPLE_FAST_XS - 1);
        unsigned long long pv = atomicCAS(&S.xt[h], ~0ull, key);
        for (int probe = 0; probe < SAMPLE_FAST_XS && pv != ~0ull; probe++) {
            if ((uint32_t)(pv >> 32) == c) { atomicMin(&S.xt[h], key); break; }
            h = (h + 1) & (SAMPLE_FAST_XS - 1);
            pv = atomicCAS(&S.xt[h], ~0ull, key);
        }
    };
    auto xt_find = [&](uint32_t c) -> unsigned long long {   // the entry of value c, or ~0
        uint32_t h = c & (SAMPLE_FAST_XS - 1);
        for (int probe = 0; probe < SAMPLE_FAST_XS; probe++) {
            const unsigned long long pv = S.xt[h];
            if (pv == ~0ull || (uint32_t)(pv >> 32) == c) return pv;
            h = (h + 1) & (SAMPLE_FAST_XS - 1);
        }
        return ~0ull;
    };
    const int rows = (nwords + SAMPLE_FAST_NT - 1) / SAMPLE_FAST_NT;
    // ---- 2. seen bits; a word whose bit is already set enters the exact table (its value repeats
    //         or shares a bitmap slot with another value)
    uint32_t vmask = 0, cmask = 0, fmask = 0;
#pragma unroll 1
    for (int u = 0; u < rows; u++) {
        uint32_t c;
        const int g = tid + SAMPLE_FAST_NT * u;
        if (!word(g, c)) continue;
        vmask |= 1u << u;
        const uint32_t sl = c & (SAMPLE_FAST_SLOTS - 1);
        const uint32_t bit = 1u << (sl & 31);
        if (atomicOr(&S.bm[sl >> 5], bit) & bit) {
            cmask |= 1u << u;
            xt_insert(c, (uint32_t)g);
        }
    }
    sample_lds_sync();
    FAST_TS(3);
    // ---- 3. every other valid word: is its value in the table (a later word repeats it)?
#pragma unroll 1
    for (int u = 0; u < rows; u++) {
        if (!((vmask >> u) & 1) || ((cmask >> u) & 1)) continue;
        uint32_t c;
        const int g = tid + SAMPLE_FAST_NT * u;
        word(g, c);
        if (xt_find(c) != ~0ull) {
            cmask |= 1u << u;
            xt_insert(c, (uint32_t)g);
        }
    }
    sample_lds_sync();
    FAST_TS(4);
    // ---- 4. first occurrences (contended words: the earliest position of their value),
    //         counted per (row, wave)
#pragma unroll 1
    for (int u = 0; u < rows; u++) {
        bool f = (vmask >> u) & 1;
        if (f && ((cmask >> u) & 1)) {
            uint32_t c;
            const int g = tid + SAMPLE_FAST_NT * u;
            word(g, c);
            f = (uint32_t)(xt_find(c) & 0xffffffffull) == (uint32_t)g;
        }
        fmask |= (f ? 1u : 0u) << u;
        const unsigned long long bal = __ballot(f);
        if (lane == 0) S.row_wave[u][wid] = __popcll(bal);
    }
    for (int u = rows + (tid >> 4); u < SAMPLE_FAST_ROWS; u += SAMPLE_FAST_NT / 16)   // rows past the end
        S.row_wave[u][tid & 15] = 0;
    sample_lds_sync();
    // exclusive scan of the (row, wave) counts in that order = stream order (one wave)
    if (wid == 0) {
        constexpr int E = SAMPLE_FAST_ROWS * 16, PER = (E + 63) / 64;
        int* rw = &S.row_wave[0][0];
        int v[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int e = lane * PER + i;
            v[i] = e < E ? rw[e] : 0;
            sum += v[i];
        }
        int incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        int run = incl - sum;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int e = lane * PER + i;
            if (e < E) rw[e] = run;
            run += v[i];
        }
        if (lane == 63) S.s_total = incl;
    }
    sample_lds_sync();
    FAST_TS(5);
    if (S.s_total < k || (a.test_flags & 1)) return false;   // beyond the margin (uniform decision)
    int gfinal = -1;   // stream word of the k-th acceptance, known to the wave that holds it
#pragma unroll 1
    for (int u = 0; u < rows; u++) {
        const bool f = (fmask >> u) & 1;
        const unsigned long long bal = __ballot(f);
        const int r = S.row_wave[u][wid] +
                      (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (f && r < k) {
            uint32_t c;
            word(tid + SAMPLE_FAST_NT * u, c);
            a.out[r] = (int32_t)c;
            if (a.phys_out && r >= a.shard_begin && r < a.shard_begin + a.shard_len) {
                int64_t ps = phys_base + (int64_t)c;
                if (ps >= a.capacity) ps -= a.capacity;
                a.phys_out[r - a.shard_begin] = (int32_t)ps;
            }
        }
        const unsigned long long fin = __ballot(f && r == k - 1);
        if (fin) gfinal = wid * 64 + (__ffsll((long long)fin) - 1) + SAMPLE_FAST_NT * u;
    }
    FAST_TS(6);
    if (gfinal >= 0) {   // this wave: the state after the k-th draw (its block, index just past it)
        const int bf = (gfinal < avail) ? 0 : 1 + (gfinal - avail) / 624;
        const uint32_t nx = (uint32_t)((gfinal < avail) ? pos + gfinal + 1 : (gfinal - avail) - 624 * (bf - 1) + 1);
        if (bf > 0 || a.state_in)   // (drawn from state_in: `state` does not hold block 0 yet)
            for (int j = lane; j < 624; j += 64) a.state[j] = S.blk[bf][j];
        if (lane == 0) a.state[624] = nx;
        if (a.mtc_blocks > 0) {   // the cache for the next call: the new state block and the successors twisted here
            // (no fence: nothing reads the cache before this kernel has completed)
            const int keep = min(nb - bf + 1, a.mtc_blocks);
            for (int f = lane; f < keep * 624; f += 64) a.mtc[64 + f] = S.blk[bf + f / 624][f % 624];
            if (lane == 0) a.mtc[0] = (uint32_t)keep;
        }
    }
    FAST_TS(7);
#ifdef DQNX_STAMPS
    if (tid == 0 && a.stamps) {
        for (int i = 0; i < 8; i++) a.stamps[i] = ts[i];
        a.stamps[8] = nb;
        a.stamps[9] = nbc;
    }
#endif
    return true;
}

}  // namespace dqnx
