// Diagnostic (tools/, not part of libdqnx): the cost of straight-line code at kernel start.
// A wave runs N independent-register VALU adds either as straight-line code (N instructions,
// 4 bytes each) or as a 16-instruction body looped N/16 times; thread 0 of every workgroup stamps
// s_memtime before and after, the host prints the mean cycles per workgroup.  If straight-line
// code costs far more than the loop, instruction fetch (cold instruction cache) bounds kernel
// prologues.  Build: hipcc --offload-arch=gfx950 -O3 tools/icache_probe.hip -o tools/icache_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

#define I1 "v_add_f32 %0, %0, %1\n"
#define I4 I1 I1 I1 I1
#define I16 I4 I4 I4 I4
#define I64 I16 I16 I16 I16
#define I256 I64 I64 I64 I64
#define I1024 I256 I256 I256 I256

__device__ __forceinline__ long long now() { return (long long)__builtin_amdgcn_s_memtime(); }

template <int K1024>
__global__ __launch_bounds__(256) void k_straight(long long* cyc, float* out, float y) {
    const long long t0 = now();
    float x = threadIdx.x;
#pragma unroll
    for (int k = 0; k < K1024; k++) asm volatile(I1024 : "+v"(x) : "v"(y));
    out[blockIdx.x * 256 + threadIdx.x] = x;
    const long long t1 = now();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_loop(long long* cyc, float* out, float y, int n16) {
    const long long t0 = now();
    float x = threadIdx.x;
    for (int k = 0; k < n16; k++) asm volatile(I16 : "+v"(x) : "v"(y));
    out[blockIdx.x * 256 + threadIdx.x] = x;
    const long long t1 = now();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
int run(const char* name, int blocks, long long* d, long long* h, F launch) {
    for (int rep = 0; rep < 3; rep++) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d, blocks * sizeof(long long), hipMemcpyDeviceToHost));
        double s = 0;
        long long mx = 0;
        for (int b = 0; b < blocks; b++) {
            s += h[b];
            mx = h[b] > mx ? h[b] : mx;
        }
        printf("%-22s blocks %4d rep %d: mean %8.0f max %8lld cycles\n", name, blocks, rep, s / blocks, mx);
    }
    return 0;
}

int main() {
    const int maxb = 1024;
    long long *d, h[maxb];
    float* out;
    CK(hipMalloc(&d, maxb * sizeof(long long)));
    CK(hipMalloc(&out, maxb * 256 * sizeof(float)));
    for (int blocks : {256, 768}) {
        run("straight 1024", blocks, d, h, [&] { k_straight<1><<<blocks, 256>>>(d, out, 1.f); });
        run("loop 1024", blocks, d, h, [&] { k_loop<<<blocks, 256>>>(d, out, 1.f, 64); });
        run("straight 4096", blocks, d, h, [&] { k_straight<4><<<blocks, 256>>>(d, out, 1.f); });
        run("loop 4096", blocks, d, h, [&] { k_loop<<<blocks, 256>>>(d, out, 1.f, 256); });
        run("straight 8192", blocks, d, h, [&] { k_straight<8><<<blocks, 256>>>(d, out, 1.f); });
        run("loop 8192", blocks, d, h, [&] { k_loop<<<blocks, 256>>>(d, out, 1.f, 512); });
    }
    return 0;
}
