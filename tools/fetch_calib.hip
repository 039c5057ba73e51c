// Diagnostic (tools/, not part of libdqnx): calibrates rocprofv3 FETCH_SIZE on gfx950 for the
// access patterns of the implicit-conv band loads.  Each kernel reads exactly BYTES bytes of a
// 1 GiB buffer once (far beyond L2 / Infinity Cache reuse) and writes one float per workgroup:
//   k_wide   : 16 B per lane, a wave reads 1 KiB contiguous (the guide's "wide coalesced" case)
//   k_half64 : 16 B per lane, 4 lanes cover 64 B of a 128 B line, the other 64 B of every line
//              read by a later instruction of the same wave (the NHWC band with 16-channel
//              blocks of 32-channel pixels)
//   k_scalar : 4 B per lane, 64 lanes contiguous (the CHW band rows)
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr size_t BYTES = 1ull << 30;

__global__ void k_wide(const float4* p, float* out) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const size_t n = BYTES / 16;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (s.x + s.y + s.z + s.w == 1234.5f) out[blockIdx.x] = s.x;
}

// lane l of a wave reads 16 B: line = 16 lines per instruction, half h = instruction parity
__global__ void k_half64(const float4* p, float* out) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    const size_t lines = BYTES / 128;
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t l0 = wave * 16; l0 < lines; l0 += nwaves * 16) {
        for (int h = 0; h < 2; h++) {   // 64 B half h of each of the 16 lines
            const size_t line = l0 + (lane >> 2);
            const float4 v = p[line * 8 + h * 4 + (lane & 3)];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    if (s.x + s.y + s.z + s.w == 1234.5f) out[blockIdx.x] = s.x;
}

__global__ void k_scalar(const float* p, float* out) {
    float s = 0.f;
    const size_t n = BYTES / 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 1234.5f) out[blockIdx.x] = s;
}

int main() {
    float* buf;
    float* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, BYTES);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_wide, dim3(2048), dim3(256), 0, 0, (const float4*)buf, out);
        hipLaunchKernelGGL(k_half64, dim3(2048), dim3(256), 0, 0, (const float4*)buf, out);
        hipLaunchKernelGGL(k_scalar, dim3(2048), dim3(256), 0, 0, (const float*)buf, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("each kernel read %zu bytes per dispatch\n", BYTES);
    return 0;
}
