// Per-kernel floor calibration on MI355X: back-to-back dependent launches captured in a
// hipGraph, average time per kernel.  Diagnostic only (tools/), not part of libdqnx.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(float* out) { (void)out; }
__global__ void k_store(float* out) { out[blockIdx.x * blockDim.x + threadIdx.x] = 1.f; }
__global__ void k_load_store(const float* in, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] * 2.f;
}
__global__ void k_dep2(const int* idx, const float* in, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[idx[i]] * 2.f;
}
__global__ void k_dep3(const int* idx, const float* in, const float* bias, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = in[idx[i]] * 2.f;
    out[i] = v + bias[(int)v & 1023];
}
__global__ __launch_bounds__(256) void k_lds_barrier(const float* in, float* out) {
    __shared__ float s[3072];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int j = threadIdx.x; j < 3072; j += 256) s[j] = in[(i + j) & 0xfffff];
    __syncthreads();
    out[i] = s[(threadIdx.x * 7) % 3072];
}

template <class F>
float time_graph(hipStream_t s, int reps, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int r = 0; r < reps; r++) launch(s);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    for (int it = 0; it < 5; it++) hipGraphLaunch(ge, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1e3f / (5 * reps);
}

int main() {
    const int N = 1 << 22;
    float *in, *out, *bias;
    int* idx;
    CK(hipMalloc(&in, N * 4));
    CK(hipMalloc(&out, N * 4));
    CK(hipMalloc(&bias, 4096 * 4));
    CK(hipMalloc(&idx, N * 4));
    std::vector<int> h(N);
    for (int i = 0; i < N; i++) h[i] = (int)((i * 2654435761u) % N);
    CK(hipMemcpy(idx, h.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemset(in, 0, N * 4));
    CK(hipMemset(bias, 0, 4096 * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int reps = 100;
    for (int blocks : {1, 64, 256, 768, 2048}) {
        printf("blocks=%4d  empty %.2f us | store %.2f | load+store %.2f | idx->load->store %.2f | +dep bias %.2f | lds+barrier %.2f\n",
               blocks,
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, out); }),
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_store, dim3(blocks), dim3(256), 0, st, out); }),
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_load_store, dim3(blocks), dim3(256), 0, st, in, out); }),
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_dep2, dim3(blocks), dim3(256), 0, st, idx, in, out); }),
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_dep3, dim3(blocks), dim3(256), 0, st, idx, in, bias, out); }),
               time_graph(s, reps, [&](hipStream_t st) { hipLaunchKernelGGL(k_lds_barrier, dim3(blocks), dim3(256), 0, st, in, out); }));
    }
    return 0;
}
