// The uniform replay sampler's body (sample.hip has the algorithm notes), templated on the
// workgroup size so other launches can host it (k_sample_uniform runs it with 1024 threads).
#pragma once
#include "learn.hpp"
#include "mt.hpp"

namespace dqnx {

// Serial genrand_uint32 on one lane (pool branch).
__device__ __forceinline__ uint32_t mt_next_serial(uint32_t* mt, uint32_t& pos) {
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

// threads -> MT blocks twisted ahead per pass (AH; default 4 at 1024 threads, 2 below) and words
// per thread per pass ((624 * (1 + AH)) / NT rounded up)
template <int NT>
constexpr int sample_default_ahead() { return NT >= 1024 ? 4 : 2; }
template <int NT, int AH = sample_default_ahead<NT>()>
struct SampleShape {
    static_assert(NT >= 256 && NT % 64 == 0, "the twist needs >= 227 threads");
    static constexpr int AHEAD = AH;
    static constexpr int WPT = (624 * (1 + AHEAD) + NT - 1) / NT;
};

template <int NT, int AH = sample_default_ahead<NT>()>
struct SampleLdsBase {
    uint32_t blk[AH + 1][624];   // [0] current block, [1..] twisted ahead
    int wave_tot[NT / 64];
    int s_final;
};
template <int NT, int HS>   // HS: hash slots (power of two) of a table in LDS
struct SampleLds : SampleLdsBase<NT> {
    unsigned long long tab[HS];
};

// `tab`: HS slots in LDS, or (k too large for LDS) in global memory, used by this one workgroup
// BMX > 0: `tab` is followed by a BMX-slot repeat table and a counter (the bitmap first pass)
template <int NT, int HS, int AH = sample_default_ahead<NT>(), int BMX = 0>
__device__ __forceinline__ void sample_uniform_body(const SampleArgs& a, SampleLdsBase<NT, AH>& S,
                                                    unsigned long long* tab) {
    constexpr int NW = NT / 64, AHEAD = SampleShape<NT, AH>::AHEAD, WPT = SampleShape<NT, AH>::WPT;
    static_assert(BMX == 0 || WPT <= 32, "the rolled bitmap pass keeps a thread's words in 32-bit masks");
    auto& blk = S.blk;
    int* wave_tot = S.wave_tot;
    int& s_final = S.s_final;
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
    const uint32_t pb32 = (uint32_t)phys_base, cap32 = (uint32_t)a.capacity;
    const uint32_t* src = a.state_in ? a.state_in : a.state;
    for (int j = tid; j < 624; j += NT) blk[0][j] = src[j];
    uint32_t pos = src[624];

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
    if (HS / NT <= 16) {
#pragma unroll
        for (int i = 0; i < HS / NT; i++) tab[tid + i * NT] = ~0ull;
    } else {
        for (int i = 0; i < HS / NT; i++) tab[tid + i * NT] = ~0ull;
        __threadfence_block();
    }
    if constexpr (BMX > 0) {
        for (int i = tid; i < BMX; i += NT) tab[HS + i] = ~0ull;
        if (tid == 0) *reinterpret_cast<int*>(tab + HS + BMX) = 0;
    }
    // the bitmap first pass: values fit the table's bits, and few repeats expected (~nwords^2 / 2n
    // pairs: n >= 32 k keeps them well under the repeat table's half)
    const bool bm_ok = BMX > 0 && a.bm_cap >= 0 && n <= (int64_t)HS * 64 && n >= 32ll * k;
    const int bm_cap = (a.bm_cap > 0 && a.bm_cap < BMX / 2) ? a.bm_cap : BMX / 2;
    (void)bm_ok;
    (void)bm_cap;
    const uint32_t n32 = (uint32_t)n;   // (n < 2^31: the engine's rings and the test hook refuse more)
    const int bits = bit_length64((uint64_t)n);
    const uint32_t shift = 32u - (uint32_t)bits;
    const float inv_accept = (float)((double)(1ull << bits) / (double)n);   // words per valid draw
    int accepted = 0;
    uint32_t spos0 = 0;      // stream position (since the call began) of blk[0][pos]
    int iter = 0;
    // The MT block cache (a.mtc, sample_pipe.hpp's layout: [0] blocks held, [64 + 624 b + o] block b,
    // block 0 = a state block): successors twisted ahead by an earlier launch (the update launch's
    // extension workgroup, or the previous call's own blocks).  Used only when its block 0 is this
    // call's state block; then the passes copy cached blocks instead of twisting them.
    int cache_next = 1, cache_left = 0;
    if (a.mtc && a.mtc_blocks > 0) {
        const int cnt = (int)a.mtc[0];
        bool mis = cnt < 2 || cnt > MTC_MAX_BLOCKS;   // (one block alone saves no twist: skip the compare)
        for (int j = tid; j < 624 && !mis; j += NT) mis = a.mtc[64 + j] != blk[0][j];   // (this thread's own words)
        // block-wide OR through the wave totals (no __syncthreads_or: it takes static LDS, which the
        // forward launch's 150 KB dynamic request leaves no room for)
        const unsigned long long wb = __ballot(mis);
        if (lane == 0) wave_tot[wid] = wb ? 1 : 0;
        __syncthreads();
        int any = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) any |= wave_tot[w];
        cache_left = any ? 0 : cnt - 1;
    }
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
        nb = nb > AHEAD ? AHEAD : nb;
        nb = nb < (avail == 0 ? 1 : 0) ? 1 : nb;
        {
            // cached blocks first: every load of them in flight at once (one round trip), then the stores
            const int nc = nb < cache_left ? nb : cache_left;
            if (nc > 0) {
                constexpr int CW = (AHEAD * 624 + NT - 1) / NT;   // cached words per thread, at most
                uint32_t cv[CW];
                const uint32_t* src = a.mtc + 64 + 624 * cache_next;
#pragma unroll
                for (int u = 0; u < CW; u++) {
                    const int f = tid + u * NT;
                    cv[u] = f < nc * 624 ? src[f] : 0u;
                }
#pragma unroll
                for (int u = 0; u < CW; u++) {
                    const int f = tid + u * NT;
                    if (f < nc * 624) blk[1 + f / 624][f % 624] = cv[u];
                }
                cache_next += nc;
                cache_left -= nc;
                __syncthreads();
            }
            for (int j = nc + 1; j <= nb; j++) mt_twist_into(blk[j - 1], blk[j]);   // each ends with a barrier
        }
        if (iter == 0) DQNX_STAMP(a.stamps, 2);
        const int nwords = avail + 624 * nb;
        // ---- insert: thread t owns the contiguous words [t*m, t*m + m) of the pass ----
        const int m = (nwords + NT - 1) / NT;
        // word w of the pass is blk[0][pos + w] read flat (blk[0][pos..624) then blocks 1..nb: avail = 624 - pos)
        const uint32_t* wflat = &blk[0][0] + pos;
        auto word_of = [&](int u, uint32_t& c) -> bool {   // word u of this thread: a valid candidate?
            const int w = tid * m + u;
            if (u >= m || w >= nwords) return false;
            c = mt_temper(wflat[w]) >> shift;
            return c < n32;
        };
        uint32_t cv[WPT], hv[WPT];
        bool val[WPT], first[WPT];
        bool hashed = true;
        // Rolled bitmap pass (a.bm_rolled): the same algorithm as the unrolled one below, with the
        // per-word flags in bit masks and the values recomputed from the LDS blocks, so the code the
        // workgroup runs once per launch stays a few hundred bytes (every instruction of this
        // workgroup is fetched cold: the forward's other workgroups run other code).
        bool rolled = false;
        uint32_t fmask = 0;
        if constexpr (BMX > 0) {
            if (bm_ok && iter == 0 && a.bm_rolled) {
                uint32_t* bm = reinterpret_cast<uint32_t*>(tab);
                unsigned long long* xt = tab + HS;
                int* xn = reinterpret_cast<int*>(tab + HS + BMX);
                uint32_t vmask = 0, cmask = 0;
#pragma unroll 1
                for (int u = 0; u < m; u++) {
                    uint32_t c;
                    if (!word_of(u, c)) continue;
                    vmask |= 1u << u;
                    const uint32_t bit = 1u << (c & 31u);
                    if ((atomicAnd(&bm[c >> 5], ~bit) & bit) != 0u) continue;
                    cmask |= 1u << u;
                    if (atomicAdd(xn, 1) >= bm_cap) continue;
                    const unsigned long long key = ((unsigned long long)c << 32) | (spos0 + (uint32_t)(tid * m + u));
                    uint32_t h = c & (BMX - 1);
                    while (true) {
                        const unsigned long long pv = atomicCAS(&xt[h], ~0ull, key);
                        if (pv == ~0ull) break;
                        if ((uint32_t)(pv >> 32) == c) { atomicMin(&xt[h], key); break; }
                        h = (h + 1) & (BMX - 1);
                    }
                }
                __syncthreads();
                const int nx = *xn;
                if (nx <= bm_cap) {
                    rolled = true;
                    hashed = false;
                    auto find = [&](uint32_t c) -> uint32_t {   // the slot of value c (or an empty one)
                        uint32_t h = c & (BMX - 1);
                        unsigned long long t = xt[h];
                        while (t != ~0ull && (uint32_t)(t >> 32) != c) {
                            h = (h + 1) & (BMX - 1);
                            t = xt[h];
                        }
                        return h;
                    };
                    if (nx > 0) {
#pragma unroll 1
                        for (int u = 0; u < m; u++) {
                            uint32_t c;
                            if (!((vmask >> u) & 1u) || ((cmask >> u) & 1u) || !word_of(u, c)) continue;
                            const uint32_t h = find(c);
                            if (xt[h] == ~0ull) continue;
                            cmask |= 1u << u;
                            atomicMin(&xt[h], ((unsigned long long)c << 32) | (spos0 + (uint32_t)(tid * m + u)));
                        }
                    }
#ifdef DQNX_STAMPS
                    if (a.stamps && tid == 0) a.stamps[13] = 2000 + nx;   // (diagnostic: the rolled pass ran)
#endif
                    if (tid == 0) s_final = -1;
                    __syncthreads();
                    if (iter == 0) DQNX_STAMP(a.stamps, 3);
                    fmask = vmask & ~cmask;
                    if (cmask) {
#pragma unroll 1
                        for (int u = 0; u < m; u++) {
                            uint32_t c;
                            if (!((cmask >> u) & 1u) || !word_of(u, c)) continue;
                            if ((uint32_t)(xt[find(c)] & 0xffffffffull) == spos0 + (uint32_t)(tid * m + u)) fmask |= 1u << u;
                        }
                    }
                } else {   // more repeats than the table takes: this pass on the hash table
                    for (int i = tid; i < HS; i += NT) tab[i] = ~0ull;
                    __syncthreads();
                }
            }
        }
        if (!rolled) {
#pragma unroll
        for (int u = 0; u < WPT; u++) {   // the candidates (tempered, scaled, range-checked)
            val[u] = false;
            cv[u] = 0;
            hv[u] = 0;
            uint32_t c = 0;
            if (word_of(u, c)) val[u] = true;
            cv[u] = c;
        }
        }
        if constexpr (BMX > 0) {
            if (bm_ok && iter == 0 && !a.bm_rolled) {
                // Bitmap first pass: bit c of the cleared table (all ones) is cleared by the first
                // word of value c to arrive; a word that finds it cleared repeats a value, and only
                // such words (then the words whose value they repeat) meet in the exact repeat table,
                // where the earliest stream position wins.  32-bit LDS atomics on ~k words instead
                // of 64-bit compare-and-swaps.  The repeat table is indexed by the value's low bits
                // (uniform: n >= 32 k); the pass is VALU-bound (8 waves on 4 SIMDs), so no hash.
                uint32_t* bm = reinterpret_cast<uint32_t*>(tab);
                unsigned long long* xt = tab + HS;
                int* xn = reinterpret_cast<int*>(tab + HS + BMX);
                bool xc[WPT];
                uint32_t old[WPT];
                DQNX_STAMP(a.stamps, 7);
#pragma unroll
                for (int u = 0; u < WPT; u++) {   // branch-free, so every atomic is in flight at once
                    const uint32_t bit = 1u << (cv[u] & 31u);   // (no word: an all-ones AND of a pad word)
                    uint32_t* p = val[u] ? &bm[cv[u] >> 5] : reinterpret_cast<uint32_t*>(xn + 1);
                    old[u] = atomicAnd(p, val[u] ? ~bit : ~0u);
                }
#pragma unroll
                for (int u = 0; u < WPT; u++) xc[u] = val[u] && (old[u] & (1u << (cv[u] & 31u))) == 0u;
                DQNX_STAMP(a.stamps, 8);
#pragma unroll
                for (int u = 0; u < WPT; u++) {
                    if (!xc[u] || atomicAdd(xn, 1) >= bm_cap) continue;
                    const unsigned long long key = ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u));
                    uint32_t h = cv[u] & (BMX - 1);
                    while (true) {   // (at most bm_cap <= BMX / 2 values: an empty slot exists)
                        const unsigned long long pv = atomicCAS(&xt[h], ~0ull, key);
                        if (pv == ~0ull) break;
                        if ((uint32_t)(pv >> 32) == cv[u]) { atomicMin(&xt[h], key); break; }
                        h = (h + 1) & (BMX - 1);
                    }
                    hv[u] = h;
                }
                DQNX_STAMP(a.stamps, 9);
                __syncthreads();
                const int nx = *xn;
                DQNX_STAMP(a.stamps, 10);
                if (nx <= bm_cap) {
                    hashed = false;
                    if (nx > 0) {
                        unsigned long long t[WPT];
                        uint32_t hp[WPT];
#pragma unroll
                        for (int u = 0; u < WPT; u++) {   // every first probe in flight at once
                            hp[u] = cv[u] & (BMX - 1);
                            t[u] = xt[hp[u]];
                        }
#pragma unroll
                        for (int u = 0; u < WPT; u++) {   // the first-arrived words of the repeated values
                            if (!val[u] || xc[u]) continue;
                            uint32_t h = hp[u];
                            while (t[u] != ~0ull && (uint32_t)(t[u] >> 32) != cv[u]) {
                                h = (h + 1) & (BMX - 1);
                                t[u] = xt[h];
                            }
                            if (t[u] == ~0ull) continue;
                            xc[u] = true;
                            hv[u] = h;
                            atomicMin(&xt[h], ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u)));
                        }
                    }
                    DQNX_STAMP(a.stamps, 11);
#ifdef DQNX_STAMPS
                    if (a.stamps && tid == 0) a.stamps[13] = 1000 + nx;   // (diagnostic: the bitmap pass ran, nx repeats)
#endif
                    if (tid == 0) s_final = -1;
                    __syncthreads();
                    if (iter == 0) DQNX_STAMP(a.stamps, 3);
#pragma unroll
                    for (int u = 0; u < WPT; u++)
                        first[u] = val[u] && (!xc[u] || (uint32_t)(xt[hv[u]] & 0xffffffffull) == spos0 + (uint32_t)(tid * m + u));
                } else {   // more repeats than the table takes: this pass on the hash table
                    for (int i = tid; i < HS; i += NT) tab[i] = ~0ull;
                    __syncthreads();
                }
            }
        }
        if (hashed) {   // (never with `rolled`)
        unsigned long long prev[WPT];
#pragma unroll
        for (int u = 0; u < WPT; u++) {   // first probe of every word, issued back to back
            prev[u] = ~0ull;
            if (val[u]) {   // insert (value, stream position); earliest position wins
                hv[u] = hash_u32(cv[u]) & (HS - 1);
                prev[u] = atomicCAS(&tab[hv[u]], ~0ull, ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u)));
            }
        }
#pragma unroll
        for (int u = 0; u < WPT; u++) {   // resolve: same value -> keep the minimum; else probe on
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
#pragma unroll
        for (int u = 0; u < WPT; u++) {
            // (an agent-scope load: a global table's lines must come from L2, where the atomics ran)
            const unsigned long long tv =
                val[u] ? __hip_atomic_load(&tab[hv[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
            first[u] = val[u] && (uint32_t)(tv & 0xffffffffull) == spos0 + (uint32_t)(tid * m + u);
        }
        }
        int cnt = 0;
        if (rolled) {
            cnt = __popc(fmask);
        } else {
#pragma unroll
            for (int u = 0; u < WPT; u++) cnt += first[u] ? 1 : 0;
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
        auto emit = [&](int u, uint32_t cu) {   // the r-th acceptance: word u of this thread, value cu
            if (r < k) {
                const int32_t c = (int32_t)cu;
                a.out[r] = c;
                if (a.phys_out && r >= a.shard_begin && r < a.shard_begin + a.shard_len) {
                    uint32_t ps = pb32 + (uint32_t)c;   // (< 2^32: both terms < capacity < 2^31)
                    if (ps >= cap32) ps -= cap32;
                    a.phys_out[r - a.shard_begin] = (int32_t)ps;
                }
                if (r == k - 1) s_final = tid * m + u;   // word index of the k-th acceptance
            }
            r++;
        };
        if (rolled) {
#pragma unroll 1
            for (int u = 0; u < m; u++) {
                uint32_t c;
                if (((fmask >> u) & 1u) && word_of(u, c)) emit(u, c);
            }
        } else {
#pragma unroll
            for (int u = 0; u < WPT; u++)
                if (first[u]) emit(u, cv[u]);
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
            if (bf > 0 || a.state_in)   // (drawn from state_in: `state` does not hold block 0 yet)
                for (int j = tid; j < 624; j += NT) a.state[j] = blk[bf][j];
            if (tid == 0) a.state[624] = nx;
            if (a.mtc && a.mtc_blocks > 0) {   // the cache for the next call: the new state block + its successors here
                const int keep = min(nb - bf + 1, a.mtc_blocks);
                for (int f = tid; f < keep * 624; f += NT) a.mtc[64 + f] = blk[bf + f / 624][f % 624];
                if (tid == 0) a.mtc[0] = (uint32_t)keep;
            }
            break;
        }
        // the whole pass was consumed: continue from the last block's end
        if (!hashed) {   // the next passes dedup on the hash table, seeded with this pass's first words
            for (int i = tid; i < HS; i += NT) tab[i] = ~0ull;
            __syncthreads();
            auto seed = [&](int u, uint32_t c) {
                const unsigned long long key = ((unsigned long long)c << 32) | (spos0 + (uint32_t)(tid * m + u));
                uint32_t h = hash_u32(c) & (HS - 1);
                while (atomicCAS(&tab[h], ~0ull, key) != ~0ull) h = (h + 1) & (HS - 1);
            };
            if (rolled) {
#pragma unroll 1
                for (int u = 0; u < m; u++) {
                    uint32_t c;
                    if (((fmask >> u) & 1u) && word_of(u, c)) seed(u, c);
                }
            } else {
#pragma unroll
                for (int u = 0; u < WPT; u++)
                    if (first[u]) seed(u, cv[u]);
            }
            __syncthreads();
        }
        spos0 += (uint32_t)nwords;
        if (nb > 0) {
            for (int j = tid; j < 624; j += NT) blk[0][j] = blk[nb][j];
            __syncthreads();
        }
        pos = 624;
    }
    (void)iter;
    DQNX_STAMP(a.stamps, 15);
}

// ---------------------------------------------------------------------------------------------
// Large minibatches over a population of at most 2^20 (the replay capacity): k beyond every LDS hash
// table (configs[3]'s weak-scaling global draw: k = 32,768 = 4096 rows x 8 ranks, n = 10^6), where
// the multi-pass body's (value, position) table would live in global memory (~205 us per draw on
// MI355X, one global atomicCAS per word).  The same first-occurrence semantics of random.sample's set
// branch (R:dqn/replay_memory.py:38-39), with the dedup state in LDS:
//   * a "seen" bit per value (2^20 bits = 128 KiB), set by every accepted draw and kept for the call;
//   * a pass = the rest of the current MT block + up to AH twisted blocks; a word whose bit was set by
//     an EARLIER pass repeats an accepted value and is dropped (read before any atomic of this pass);
//   * inside a pass, the word that finds its bit already set (atomicOr) repeats a value of the same
//     pass: such values go to a small (value, earliest position) table, every other word of the pass
//     probes it, and the earliest position wins.  A pass of W words repeats at most W / 2 distinct
//     values, and the table holds more than that: no overflow, no fallback;
//   * first occurrences are ranked in stream order by a block scan, as in sample_uniform_body.
template <int NT, int AH, int BMX>
struct SampleBitmapLds {
    SampleLdsBase<NT, AH> b;
    uint32_t bm[1 << 15];            // "seen" bit of every value < 2^20
    unsigned long long xt[BMX];      // (value << 32 | stream position): values repeated inside a pass
    int xn;                          // nonzero: the pass has a repeated value
};
constexpr int64_t SAMPLE_BITMAP_MAX_N = (int64_t)1 << 20;

// LDS-only workgroup barrier: the sampler's cross-thread data is all in LDS, so no wave waits here for
// its global stores (the minibatch it writes) to complete -- __syncthreads() would, once per pass
__device__ __forceinline__ void bm_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// mt_twist_into without its closing barrier (the caller ends it)
__device__ __forceinline__ void mt_twist_into_nowait(const uint32_t* old, uint32_t* nw) {
    const int t = threadIdx.x;
    if (t < 227) {
        const uint32_t a0 = old[t + 397] ^ mt_mix(old[t], old[t + 1]);
        const uint32_t a1 = a0 ^ mt_mix(old[t + 227], old[t + 228]);
        nw[t] = a0;
        nw[t + 227] = a1;
        if (t < 169) nw[t + 454] = a1 ^ mt_mix(old[t + 454], old[t + 455]);
        if (t == 169) nw[623] = a1 ^ mt_mix(old[623], old[397] ^ mt_mix(old[0], old[1]));
    }
}

template <int NT, int AH, int BMX>
__device__ __forceinline__ void sample_bitmap_body(const SampleArgs& a, SampleBitmapLds<NT, AH, BMX>& S) {
    static_assert(BMX > 624 * (AH + 1) / 2 && (BMX & (BMX - 1)) == 0, "a pass's repeated values fit the table");
    static_assert(NT >= 624, "one state word per thread");
    constexpr int NW = NT / 64, WPT = (624 * (AH + 1) + NT - 1) / NT;
    auto& blk = S.b.blk;
    int* wave_tot = S.b.wave_tot;
    int& s_final = S.b.s_final;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    // every global load of the call issued at once, unconditionally (a load whose value a branch needs
    // is waited for right there: three serialised round trips otherwise)
    const int64_t n = a.n_dev ? gld(a.n_dev) : a.n_val;
    const int64_t wptr0 = a.phys_out ? gld(a.wptr_dev) : 0;
    const uint32_t* src = a.state_in ? a.state_in : a.state;
    const uint32_t st_j = gld(src + (tid < 624 ? tid : 624));
    const uint32_t pos0 = gld(src + 624);
    const int k = a.k;
    if (k < 0 || (int64_t)k > n || n <= a.setsize || n > SAMPLE_BITMAP_MAX_N) {
        // errors and the pool branch (a replay still smaller than random.sample's setsize): the general
        // body (its set branch is never reached from here: n > 2^20 exceeds every routed capacity)
        sample_uniform_body<NT, 1024, AH, 0>(a, S.b, reinterpret_cast<unsigned long long*>(S.bm));
        return;
    }
    if (k == 0) return;
    DQNX_STAMP(a.stamps, 0);
    int64_t phys_base = 0;
    if (a.phys_out) {
        phys_base = wptr0 - n;
        if (phys_base < 0) phys_base += a.capacity;
    }
    const uint32_t pb32 = (uint32_t)phys_base, cap32 = (uint32_t)a.capacity;
    if (tid < 624) blk[0][tid] = st_j;
    uint32_t pos = pos0;
    {
        uint4* bm4 = reinterpret_cast<uint4*>(S.bm);
#pragma unroll
        for (int i = 0; i < (1 << 13) / NT; i++) bm4[tid + i * NT] = make_uint4(0u, 0u, 0u, 0u);
        for (int i = tid; i < BMX; i += NT) S.xt[i] = ~0ull;
        if (tid == 0) S.xn = 0;
    }
    bm_lds_sync();
    const uint32_t n32 = (uint32_t)n;
    const int bits = bit_length64((uint64_t)n);
    const uint32_t shift = 32u - (uint32_t)bits;
    const float inv_accept = (float)((double)(1ull << bits) / (double)n);   // words per valid draw
    int accepted = 0;
    uint32_t spos0 = 0;   // stream position (since the call began) of blk[0][pos]
    int pass = 0;
    DQNX_STAMP(a.stamps, 1);
    while (true) {
        const int avail = 624 - (int)pos;
        const int need = k - accepted;
        const float est = need * inv_accept * (1.f + (float)(accepted + need) / (2.f * (float)n)) + 32.f + need / 16.f;
        int nb = (int)ceilf((est - (float)avail) / 624.f);
        nb = nb > AH ? AH : nb;
        nb = nb < (avail == 0 ? 1 : 0) ? 1 : nb;
        for (int j = 1; j <= nb; j++) {   // block-parallel twists, each ended by an LDS-only barrier
            mt_twist_into_nowait(blk[j - 1], blk[j]);
            bm_lds_sync();
        }
        if (pass == 1) DQNX_STAMP(a.stamps, 2);
        const int nwords = avail + 624 * nb;
        const int m = (nwords + NT - 1) / NT;   // thread t owns the words [t m, t m + m) of the pass
        const uint32_t* wflat = &blk[0][0] + pos;
        uint32_t cv[WPT], hv[WPT];
        bool val[WPT], xc[WPT];
#pragma unroll
        for (int u = 0; u < WPT; u++) {   // the candidates; then drop repeats of earlier passes
            const int w = tid * m + u;
            const bool live = u < m && w < nwords;
            const uint32_t c = live ? mt_temper(wflat[w]) >> shift : 0u;
            cv[u] = c;
            val[u] = live && c < n32 && ((S.bm[c >> 5] >> (c & 31u)) & 1u) == 0u;
            hv[u] = 0;
        }
        bm_lds_sync();   // every earlier-pass read before this pass's first atomic
        if (pass == 1) DQNX_STAMP(a.stamps, 3);
#pragma unroll
        for (int u = 0; u < WPT; u++) {
            const uint32_t bit = 1u << (cv[u] & 31u);
            xc[u] = val[u] && (atomicOr(&S.bm[cv[u] >> 5], bit) & bit) != 0u;
        }
#pragma unroll
        for (int u = 0; u < WPT; u++) {   // values repeated inside the pass: (value, earliest position)
            if (!xc[u]) continue;
            const unsigned long long key = ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u));
            uint32_t h = cv[u] & (BMX - 1);
            while (true) {
                const unsigned long long pv = atomicCAS(&S.xt[h], ~0ull, key);
                if (pv == ~0ull) break;
                if ((uint32_t)(pv >> 32) == cv[u]) { atomicMin(&S.xt[h], key); break; }
                h = (h + 1) & (BMX - 1);
            }
            hv[u] = h;
            S.xn = 1;
        }
        if (tid == 0) s_final = -1;
        bm_lds_sync();
        if (pass == 1) DQNX_STAMP(a.stamps, 4);
        const int nx = S.xn;
        if (nx) {   // the other words of a repeated value (the one that set its bit first among them)
#pragma unroll
            for (int u = 0; u < WPT; u++) {
                if (!val[u] || xc[u]) continue;
                uint32_t h = cv[u] & (BMX - 1);
                unsigned long long t = S.xt[h];
                while (t != ~0ull && (uint32_t)(t >> 32) != cv[u]) {
                    h = (h + 1) & (BMX - 1);
                    t = S.xt[h];
                }
                if (t == ~0ull) continue;
                xc[u] = true;
                hv[u] = h;
                atomicMin(&S.xt[h], ((unsigned long long)cv[u] << 32) | (spos0 + (uint32_t)(tid * m + u)));
            }
            bm_lds_sync();
        }
        if (pass == 1) DQNX_STAMP(a.stamps, 5);
        bool first[WPT];
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < WPT; u++) {
            first[u] = val[u] && (!xc[u] || (uint32_t)(S.xt[hv[u]] & 0xffffffffull) == spos0 + (uint32_t)(tid * m + u));
            cnt += first[u] ? 1 : 0;
        }
        int incl = cnt;   // wave inclusive scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wave_tot[wid] = incl;
        bm_lds_sync();
        int before = incl - cnt, total = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const int tw = wave_tot[w];
            before += (w < wid) ? tw : 0;
            total += tw;
        }
        int r = accepted + before;
        if (pass == 1) DQNX_STAMP(a.stamps, 6);
#pragma unroll
        for (int u = 0; u < WPT; u++) {
            if (!first[u]) continue;
            if (r < k) {
                const int32_t c = (int32_t)cv[u];
                a.out[r] = c;
                if (a.phys_out && r >= a.shard_begin && r < a.shard_begin + a.shard_len) {
                    uint32_t ps = pb32 + (uint32_t)c;   // (< 2^32: both terms < capacity <= 2^20)
                    if (ps >= cap32) ps -= cap32;
                    a.phys_out[r - a.shard_begin] = (int32_t)ps;
                }
                if (r == k - 1) s_final = tid * m + u;   // word index of the k-th acceptance
            }
            r++;
        }
        bm_lds_sync();
        if (pass == 1) DQNX_STAMP(a.stamps, 7);
        pass++;
        accepted += total;
        if (accepted >= k) {   // state after the k-th draw: the block holding that word, index just past it
            const int wf = s_final;
            const int bf = (wf < avail) ? 0 : 1 + (wf - avail) / 624;
            const uint32_t nxp = (uint32_t)((wf < avail) ? (int)pos + wf + 1 : (wf - avail) % 624 + 1);
            if (bf > 0 || a.state_in)
                for (int j = tid; j < 624; j += NT) a.state[j] = blk[bf][j];
            if (tid == 0) a.state[624] = nxp;
            DQNX_STAMP(a.stamps, 15);
#ifdef DQNX_STAMPS
            if (a.stamps && blockIdx.x == 0 && tid == 0) a.stamps[14] = pass;
#endif
            break;
        }
        // the whole pass was consumed: clear the repeat table, continue from the last block's end
        if (nx) {
            for (int i = tid; i < BMX; i += NT) S.xt[i] = ~0ull;
            if (tid == 0) S.xn = 0;
        }
        spos0 += (uint32_t)nwords;
        if (nb > 0)
            for (int j = tid; j < 624; j += NT) blk[0][j] = blk[nb][j];
        bm_lds_sync();
        pos = 624;
    }
}

}  // namespace dqnx
