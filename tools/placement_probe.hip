// Diagnostic: where does the dispatcher put the workgroups of one launch?  Each workgroup spins for a
// while and records its XCC / SE / CU (s_getreg HW_ID, XCC_ID) and s_memtime start / end; the host
// prints how many distinct CUs were used and how many workgroups shared a CU at once.
//   hipcc --offload-arch=gfx950 -O2 tools/placement_probe.hip -o tools/placement_probe
//   tools/placement_probe <workgroups> <threads> <lds KB> <spin cycles>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ void probe(unsigned long long* out, int spin) {
    extern __shared__ float lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) lds[0] = 1.f;
    while ((long long)(__builtin_amdgcn_s_memtime() - t0) < spin) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        out[3 * blockIdx.x] = ((unsigned long long)(xcc & 0xf) << 32) | hw;
        out[3 * blockIdx.x + 1] = t0;
        out[3 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime() + (lds[0] > 2.f ? 1 : 0);
    }
}

int main(int argc, char** argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 192, nt = argc > 2 ? atoi(argv[2]) : 512;
    const int kb = argc > 3 ? atoi(argv[3]) : 0, spin = argc > 4 ? atoi(argv[4]) : 20000;
    unsigned long long* d;
    if (hipMalloc(&d, 3 * 8 * (size_t)nb) != hipSuccess) return 1;
    if (kb > 64) (void)hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(probe, dim3(nb), dim3(nt), (size_t)kb * 1024, 0, d, spin);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
    }
    std::vector<unsigned long long> h(3 * (size_t)nb);
    if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    std::map<unsigned long long, std::vector<int>> cu;   // (xcc, se, sh, cu) -> blocks
    for (int b = 0; b < nb; b++) {
        const unsigned long long v = h[3 * b];
        const unsigned hw = (unsigned)v, xcc = (unsigned)(v >> 32);
        const unsigned long long key = ((unsigned long long)xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) |
                                       ((hw >> 8) & 15);
        cu[key].push_back(b);
    }
    int maxc = 0;
    for (auto& kv : cu) {   // most workgroups overlapping in time on one CU
        auto& v = kv.second;
        for (int a : v) {
            int c = 0;
            for (int b : v) c += (h[3 * b + 1] < h[3 * a + 2] && h[3 * a + 1] < h[3 * b + 2]) ? 1 : 0;
            if (c > maxc) maxc = c;
        }
    }
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int b = 0; b < nb; b++) {
        if (h[3 * b + 1] < t0) t0 = h[3 * b + 1];
        if (h[3 * b + 2] > t1) t1 = h[3 * b + 2];
    }
    std::map<int, int> per_xcc;
    for (auto& kv : cu) per_xcc[(int)(kv.first >> 16)] += 1;
    printf("{\"workgroups\": %d, \"threads\": %d, \"lds_kb\": %d, \"distinct_cus\": %zu, \"max_concurrent_per_cu\": %d, "
           "\"span_ticks\": %llu, \"cus_per_xcc\": [", nb, nt, kb, cu.size(), maxc, t1 - t0);
    bool first = true;
    for (auto& kv : per_xcc) {
        printf("%s%d", first ? "" : ", ", kv.second);
        first = false;
    }
    printf("]}\n");
    return 0;
}
