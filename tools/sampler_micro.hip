// Diagnostic (tools/, not part of libdqnx): costs of the sampler's building blocks on one CU,
// timed with s_memtime inside one workgroup (median over launches):
//   twist:  one wave twists B MT19937 blocks in LDS (mt_twist_wave)
//   cas64:  1024 threads insert W words each into a 16384-slot LDS table (64-bit CAS + probing)
//   or32:   1024 threads set W hashed bits each in a 2^20-bit LDS bitmap (32-bit atomicOr, return)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#include "../multimodal-drl-rmc_amd/csrc/sample_pipe.hpp"

using namespace dqnx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

namespace dqnx {
int set_error(int code, const char*, ...) { return code; }
int set_hip_error(hipError_t e, const char*, const char*, int) { return 1000 + (int)e; }
}

__global__ __launch_bounds__(64) void k_twist(const uint32_t* st, uint32_t* out, int nb, long long* cyc) {
    __shared__ uint32_t blk[11][624];
    for (int j = threadIdx.x; j < 624; j += 64) blk[0][j] = st[j];
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 1; b <= nb; b++) mt_twist_wave(blk[b - 1], blk[b], threadIdx.x);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const long long t1 = __builtin_amdgcn_s_memtime();
    for (int j = threadIdx.x; j < 624; j += 64) out[j] = blk[nb][j];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the 1024-thread block twist of k_sample_uniform (3 barrier phases per block)
__global__ __launch_bounds__(1024) void k_twist_block(const uint32_t* st, uint32_t* out, int nb, long long* cyc) {
    __shared__ uint32_t blk[11][624];
    for (int j = threadIdx.x; j < 624; j += 1024) blk[0][j] = st[j];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 1; b <= nb; b++) mt_twist_into(blk[b - 1], blk[b]);
    const long long t1 = __builtin_amdgcn_s_memtime();
    for (int j = threadIdx.x; j < 624; j += 1024) out[j] = blk[nb][j];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(1024) void k_cas(uint32_t seed, int W, uint32_t n, int* out, long long* cyc) {
    __shared__ unsigned long long tab[16384];
    for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = ~0ull;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    int found = 0;
    for (int u = 0; u < W; u++) {
        const uint32_t pos = threadIdx.x * W + u;
        const uint32_t c = hash_u32(seed ^ (pos * 2654435761u)) % n;
        uint32_t h = hash_u32(c) & 16383;
        const unsigned long long key = ((unsigned long long)c << 32) | pos;
        unsigned long long pv = atomicCAS(&tab[h], ~0ull, key);
        for (int p = 0; p < 16384 && pv != ~0ull; p++) {
            if ((uint32_t)(pv >> 32) == c) { atomicMin(&tab[h], key); found++; break; }
            h = (h + 1) & 16383;
            pv = atomicCAS(&tab[h], ~0ull, key);
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (found) atomicAdd(out, found);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the same words, all first probes issued back to back (the samplers' form)
template <int W>
__global__ __launch_bounds__(1024) void k_cas_batched(uint32_t seed, uint32_t n, int* out, long long* cyc) {
    __shared__ unsigned long long tab[16384];
    for (int i = threadIdx.x; i < 16384; i += 1024) tab[i] = ~0ull;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t cv[W], hv[W];
    unsigned long long pv[W];
#pragma unroll
    for (int u = 0; u < W; u++) {
        const uint32_t pos = threadIdx.x * W + u;
        cv[u] = hash_u32(seed ^ (pos * 2654435761u)) % n;
        hv[u] = hash_u32(cv[u]) & 16383;
        pv[u] = atomicCAS(&tab[hv[u]], ~0ull, ((unsigned long long)cv[u] << 32) | pos);
    }
    int found = 0;
#pragma unroll
    for (int u = 0; u < W; u++) {
        const unsigned long long key = ((unsigned long long)cv[u] << 32) | (threadIdx.x * W + u);
        uint32_t h = hv[u];
        unsigned long long p = pv[u];
        for (int q = 0; q < 16384 && p != ~0ull; q++) {
            if ((uint32_t)(p >> 32) == cv[u]) { atomicMin(&tab[h], key); found++; break; }
            h = (h + 1) & 16383;
            p = atomicCAS(&tab[h], ~0ull, key);
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (found) atomicAdd(out, found);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int W>
__global__ __launch_bounds__(1024) void k_or32(uint32_t seed, uint32_t n, int* out, long long* cyc) {
    __shared__ uint32_t bm[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) bm[i] = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    uint32_t old[W], bit[W];
#pragma unroll
    for (int u = 0; u < W; u++) {
        const uint32_t pos = threadIdx.x * W + u;
        const uint32_t c = hash_u32(seed ^ (pos * 2654435761u)) % n;
        const uint32_t h = hash_u32(c) & 0xfffff;
        bit[u] = 1u << (h & 31);
        old[u] = atomicOr(&bm[h >> 5], bit[u]);
    }
    int found = 0;
#pragma unroll
    for (int u = 0; u < W; u++) found += (old[u] & bit[u]) ? 1 : 0;
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (found) atomicAdd(out, found);
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
long long median_cycles(F launch, long long* d_cyc, int reps = 21) {
    std::vector<long long> v;
    for (int r = 0; r < reps; r++) {
        launch();
        (void)hipDeviceSynchronize();
        long long c = 0;
        (void)hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
        v.push_back(c);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    uint32_t *st, *out;
    int* cnt;
    long long* cyc;
    CK(hipMalloc(&st, 625 * 4));
    CK(hipMalloc(&out, 625 * 4));
    CK(hipMalloc(&cnt, 4));
    CK(hipMalloc(&cyc, 64 * 8));
    std::vector<uint32_t> h(625);
    for (int i = 0; i < 625; i++) h[i] = 0x9e3779b9u * (i + 1);
    CK(hipMemcpy(st, h.data(), 625 * 4, hipMemcpyHostToDevice));
    for (int nb : {1, 2, 4, 8}) {
        const long long c1 = median_cycles([&] { hipLaunchKernelGGL(k_twist, dim3(1), dim3(64), 0, 0, st, out, nb, cyc); }, cyc);
        const long long c2 = median_cycles([&] { hipLaunchKernelGGL(k_twist_block, dim3(1), dim3(1024), 0, 0, st, out, nb, cyc); }, cyc);
        printf("twist %d blocks: one wave %lld cyc (%lld/block) | 1024-thread block twist %lld cyc (%lld/block)\n", nb, c1,
               c1 / nb, c2, c2 / nb);
    }
    for (int W : {1, 2, 4, 5}) {
        const long long c = median_cycles([&] { hipLaunchKernelGGL(k_cas, dim3(1), dim3(1024), 0, 0, 1234u, W, 1000000u, cnt, cyc); }, cyc);
        printf("cas64 serial: %d words/thread (%d words) %lld cyc, %.2f cyc/word\n", W, 1024 * W, c, (double)c / (1024 * W));
    }
#define CASB(W) { const long long c = median_cycles([&] { hipLaunchKernelGGL(k_cas_batched<W>, dim3(1), dim3(1024), 0, 0, 1234u, 1000000u, cnt, cyc); }, cyc); \
    printf("cas64 batched: %d words/thread (%d words) %lld cyc, %.2f cyc/word\n", W, 1024 * W, c, (double)c / (1024 * W)); }
    CASB(1) CASB(2) CASB(4) CASB(5)
#define ORB(W) { const long long c = median_cycles([&] { hipLaunchKernelGGL(k_or32<W>, dim3(1), dim3(1024), 0, 0, 1234u, 1000000u, cnt, cyc); }, cyc); \
    printf("or32 bitmap: %d words/thread (%d words) %lld cyc, %.2f cyc/word\n", W, 1024 * W, c, (double)c / (1024 * W)); }
    ORB(1) ORB(2) ORB(4) ORB(5)
    return 0;
}
