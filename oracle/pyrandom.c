/*
 * oracle/pyrandom.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C CPU restatement of the random-number arithmetic on the DQN learn-step
 * hot path of youcefMehamlia/Multimodal-DRL-RMC:
 *
 *   - R:dqn/replay_memory.py:38-39  ReplayMemoryNaive.sample_transitions ->
 *       CPython random.sample(deque, batch_size)   (CPython 3.7/3.10 Lib/random.py
 *       Random.sample + _randbelow_with_getrandbits, _randommodule.c genrand_uint32).
 *       Both branches are restated: the "pool" branch (n <= setsize) and the
 *       "set" branch (rejection + duplicate redraw).
 *   - R:dqn/replay_memory.py:79-80  ReplayMemoryPrioritized.sample_transitions ->
 *       numpy legacy RandomState.uniform(low, high) = low + (high-low)*random_sample(),
 *       random_sample = ((a>>5)*67108864 + (b>>6)) / 2^53 over two MT19937 words.
 *
 * The MT19937 state layout matches Python's random.getstate()[1]: 624 state words
 * followed by the position index (0..624).  numpy's get_state() keys/pos use the
 * same layout.
 *
 * Pinned by tests/test_oracle_sampler.py against CPython's own random.sample and
 * numpy's RandomState (the reference's dependencies) and against
 * tests/golden/sampler_*.npz, generated from the reference itself by
 * tests/golden/make_golden.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397
#define MATRIX_A 0x9908b0dfU
#define UPPER_MASK 0x80000000U
#define LOWER_MASK 0x7fffffffU

/* state[0..623] = mt words, state[624] = index (Python's mti). */
static uint32_t genrand_uint32(uint32_t *state) {
    static const uint32_t mag01[2] = {0x0U, MATRIX_A};
    uint32_t *mt = state;
    uint32_t y;
    if (state[MT_N] >= MT_N) { /* generate N words at one time (CPython _randommodule.c) */
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
            mt[kk] = mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
            mt[kk] = mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        y = (mt[MT_N - 1] & UPPER_MASK) | (mt[0] & LOWER_MASK);
        mt[MT_N - 1] = mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
        state[MT_N] = 0;
    }
    y = mt[state[MT_N]++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

uint32_t oracle_genrand_uint32(uint32_t *state) { return genrand_uint32(state); }

static int bit_length(uint64_t n) {
    int b = 0;
    while (n) { b++; n >>= 1; }
    return b;
}

/* Lib/random.py _randbelow_with_getrandbits(n); getrandbits(k<=32) = genrand>>(32-k). */
static uint64_t randbelow(uint32_t *state, uint64_t n) {
    if (n == 0) return 0;
    int k = bit_length(n);
    uint64_t r = genrand_uint32(state) >> (32 - k);
    while (r >= n) r = genrand_uint32(state) >> (32 - k);
    return r;
}

/* Lib/random.py Random.sample: setsize = 21 (+ 4**ceil(log(3k, 4)) if k > 5).
 * math.log(x, base) in CPython is log(x)/log(base) (loghelper). */
int64_t oracle_sample_setsize(int64_t k) {
    int64_t setsize = 21;
    if (k > 5) {
        double e = ceil(log((double)(k * 3)) / log(4.0));
        int64_t p = 1;
        for (int i = 0; i < (int)e; i++) p *= 4;
        setsize += p;
    }
    return setsize;
}

/* random.sample(range-like population of size n, k) -> out[k] positions.
 * Returns 0 on success, -1 if k > n (Python raises ValueError, consuming nothing). */
int oracle_random_sample(uint32_t *state, int64_t n, int64_t k, int64_t *out) {
    if (k < 0 || k > n) return -1;
    int64_t setsize = oracle_sample_setsize(k);
    if (n <= setsize) {
        int64_t *pool = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
        for (int64_t i = 0; i < n; i++) pool[i] = i;
        for (int64_t i = 0; i < k; i++) {
            int64_t j = (int64_t)randbelow(state, (uint64_t)(n - i));
            out[i] = pool[j];
            pool[j] = pool[n - i - 1];
        }
        free(pool);
    } else {
        /* open-addressing set of selected positions */
        int64_t cap = 16;
        while (cap < 4 * k + 16) cap <<= 1;
        int64_t *tab = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
        for (int64_t i = 0; i < cap; i++) tab[i] = -1;
        for (int64_t i = 0; i < k; i++) {
            for (;;) {
                int64_t j = (int64_t)randbelow(state, (uint64_t)n);
                uint64_t h = ((uint64_t)j * 0x9E3779B97F4A7C15ULL) >> 20;
                int64_t s = (int64_t)(h & (uint64_t)(cap - 1));
                int found = 0;
                while (tab[s] != -1) {
                    if (tab[s] == j) { found = 1; break; }
                    s = (s + 1) & (cap - 1);
                }
                if (found) continue;   /* while j in selected: redraw */
                tab[s] = j;
                out[i] = j;
                break;
            }
        }
        free(tab);
    }
    return 0;
}

/* numpy legacy RandomState.random_sample() (mt19937_next_double). */
double oracle_np_random_sample(uint32_t *state) {
    int32_t a = (int32_t)(genrand_uint32(state) >> 5);
    int32_t b = (int32_t)(genrand_uint32(state) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* numpy legacy RandomState.uniform(low, high) with scalar arguments:
 * range = high - low; low + range * random_sample(). */
double oracle_np_uniform(uint32_t *state, double low, double high) {
    volatile double range = high - low;
    volatile double u = oracle_np_random_sample(state);
    volatile double prod = range * u;
    return low + prod;
}
