// Host-side mirror of the sampler's RNG stream position (include/dqnx.h: dqnx_rng_sample_words,
// dqnx_rng_advance).  No device work.
//
// The reference draws the minibatch inside Agent.learn() from the interpreter's global generators:
// CPython's `random.sample(deque, batch_size)` (R:dqn/replay_memory.py:38-39) and numpy's legacy
// `np.random.uniform` once per sample (R:dqn/replay_memory.py:79-80), so after learn() returns the
// caller's `random` / `np.random` have moved on.  On libdqnx the DEVICE sampler draws the minibatch
// (sample.hip / per.hip, bit-exact); these two functions only tell the host how far the draw moves
// the stream, so the drop-in Agent can advance its global generator at learn() time
// (random.getrandbits(32 * words) / np.random.random_sample(k)) without waiting for the GPU, and
// later check the device's returned state against `out625`.
//
// Stream layout: 624 MT19937 words + the position index, as random.getstate()[1] and
// np.random.get_state()[1:3] hold them.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/dqnx.h"
#include "common.hpp"

namespace {

constexpr int kN = 624, kM = 397;

struct Mt {
    uint32_t w[kN];
    uint32_t pos;

    void twist() {   // MT19937 regeneration of all 624 words (Matsumoto & Nishimura 1998)
        auto mix = [](uint32_t hi, uint32_t lo, uint32_t far) {
            const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
            return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        };
        // in place, in index order: words past i + 1 - 624 / i + 397 - 624 are read after their rewrite,
        // as in CPython's and numpy's genrand loops
        for (int i = 0; i < kN; i++) w[i] = mix(w[i], w[(i + 1) % kN], w[(i + kM) % kN]);
        pos = 0;
    }
    uint32_t next() {   // one tempered output
        if (pos >= kN) twist();
        uint32_t y = w[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        return y ^ (y >> 18);
    }
};

int bits_of(uint64_t n) {
    int b = 0;
    while (n) {
        b++;
        n >>= 1;
    }
    return b;
}

// Lib/random.py _randbelow_with_getrandbits: getrandbits(k) of one word for k <= 32, redrawn while
// >= n; returns the value, counts the words
uint64_t below(Mt& mt, uint64_t n, int64_t& words) {
    if (n == 0) return 0;
    const int k = bits_of(n);
    uint64_t r;
    do {
        r = mt.next() >> (32 - k);
        words++;
    } while (r >= n);
    return r;
}

bool load(Mt& mt, const uint32_t* s) {
    if (s[kN] > (uint32_t)kN) return false;
    memcpy(mt.w, s, sizeof(mt.w));
    mt.pos = s[kN];
    return true;
}

void store(const Mt& mt, uint32_t* out) {
    memcpy(out, mt.w, sizeof(mt.w));
    out[kN] = mt.pos;
}

}  // namespace

namespace dqnx {
int64_t sample_setsize(int64_t k);   // sample.hip: random.sample's set-vs-pool threshold
}

extern "C" int dqnx_rng_sample_words(const uint32_t* state625, int64_t n, int32_t k, uint32_t* out625,
                                     int64_t* words) {
    if (!state625 || !words) return dqnx::set_error(DQNX_EINVAL, "dqnx_rng_sample_words: null argument");
    if (k < 0 || (int64_t)k > n) return dqnx::set_error(DQNX_EINVAL, "Sample larger than population or is negative");
    if (n >= ((int64_t)1 << 32)) return dqnx::set_error(DQNX_EINVAL, "population beyond 2^32");
    Mt mt;
    if (!load(mt, state625)) return dqnx::set_error(DQNX_EINVAL, "MT index must be <= 624");
    int64_t w = 0;
    if (n <= dqnx::sample_setsize(k)) {
        // pool branch: j = randbelow(n - i); the draws' count does not depend on the pool contents
        for (int32_t i = 0; i < k; i++) (void)below(mt, (uint64_t)(n - i), w);
    } else {
        // set branch: redraw while j was already selected.  Open addressing over a power-of-two table
        // of >= 4k slots; a slot holds (generation << 32 | j) so the table is never cleared.
        static thread_local std::vector<uint64_t> table;
        static thread_local uint32_t gen = 0;
        size_t cap = 64;
        while (cap < (size_t)k * 4) cap <<= 1;
        if (table.size() < cap || ++gen == 0) {
            table.assign(std::max(cap, table.size()), 0);
            gen = 1;
        }
        const size_t mask = cap - 1;
        const uint64_t tag = (uint64_t)gen << 32;
        for (int32_t i = 0; i < k; i++) {
            while (true) {
                const uint64_t j = below(mt, (uint64_t)n, w);
                size_t h = (size_t)((j * 0x9E3779B97F4A7C15ull) >> 20) & mask;
                bool dup = false;
                while (true) {
                    const uint64_t v = table[h];
                    if ((v >> 32) != gen) {   // empty for this generation: insert
                        table[h] = tag | j;
                        break;
                    }
                    if ((v & 0xffffffffull) == j) {
                        dup = true;
                        break;
                    }
                    h = (h + 1) & mask;
                }
                if (!dup) break;
            }
        }
    }
    *words = w;
    if (out625) store(mt, out625);
    return DQNX_OK;
}

extern "C" int dqnx_rng_advance(const uint32_t* state625, int64_t words, uint32_t* out625) {
    if (!state625 || !out625 || words < 0) return dqnx::set_error(DQNX_EINVAL, "dqnx_rng_advance: bad argument");
    Mt mt;
    if (!load(mt, state625)) return dqnx::set_error(DQNX_EINVAL, "MT index must be <= 624");
    int64_t left = words;
    while (left > 0) {   // whole blocks skip the tempering
        if (mt.pos >= (uint32_t)kN) mt.twist();
        const int64_t take = std::min<int64_t>(left, kN - (int64_t)mt.pos);
        mt.pos += (uint32_t)take;
        left -= take;
    }
    store(mt, out625);
    return DQNX_OK;
}
