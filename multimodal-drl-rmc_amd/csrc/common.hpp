// Shared device/host helpers for libdqnx (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/dqnx.h"

namespace dqnx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][k=l>>4], B[k=l>>4][l&15];
// accumulator lane l holds C[(l>>4)*4 + r][l&15], r = 0..3.  Exact fp32 fmaf chain.
__device__ __forceinline__ floatx4 mfma16x16x4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 operands (DQNX_COMPUTE_BF16).  v_mfma_f32_16x16x32_bf16: lane l supplies
// A[l&15][8(l>>4) + j] and B[8(l>>4) + j][l&15], j = 0..7 (16 bytes each); the accumulator
// layout is the fp32 one above.  float -> bf16 is v_cvt_pk_bf16_f32 (round to nearest even,
// torch's Tensor.to(torch.bfloat16) on finite values).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t bf16_pack2(float lo, float hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)lo) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)hi) << 16);
}
__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ floatx4 mfma16x16x32bf16(u32x4 a, u32x4 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ float relu_f(float x) { return x > 0.f ? x : 0.f; }

// torch CPU ELU (alpha=scale=input_scale=1): x <= 0 ? expm1(x) : x
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }

// activation derivative from the activation OUTPUT h (threshold_backward / elu_backward
// with is_result=true): relu: h > 0 ? g : 0 ; elu: h > 0 ? g : g * (h + 1)
template <int ACT>
__device__ __forceinline__ float act_bwd(float g, float h) {
    if (ACT == DQNX_ACT_RELU) return h > 0.f ? g : 0.f;
    return h > 0.f ? g : g * (h + 1.f);
}

template <int ACT>
__device__ __forceinline__ float act_fwd(float x) {
    if (ACT == DQNX_ACT_RELU) return relu_f(x);
    return elu_f(x);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// Loads through the global address space.  A generic pointer the compiler cannot prove global
// (e.g. one fetched from a struct member) compiles to flat_load, which counts in lgkmcnt as
// well: the next s_waitcnt for a kernel-argument s_load then drains it, serialising round trips.
template <class T>
__device__ __forceinline__ T gld(const T* p) {
    return *(const __attribute__((address_space(1))) T*)p;
}


// Raw buffer descriptor for a wave-uniform base (bytes = the range; offsets at or past it read 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const float* base, uint32_t bytes) {
    const uint64_t b = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// XCD-aware block remap (CDNA guide T1): blocks are dealt round-robin over the 8 XCDs, so
// hand XCD x a CONTIGUOUS range of tiles (bijective for any total).  Speed only: placement
// never affects results.
__device__ __forceinline__ int xcd_remap(int L, int total) {
    const int per = total >> 3, rem = total & 7;
    const int x = L & 7, local = L >> 3;
    return x * per + (x < rem ? x : rem) + local;
}

#ifdef DQNX_STAMPS
#define DQNX_STAMP(ptr, i)                                                            \
    do {                                                                             \
        if ((ptr) && blockIdx.x == 0 && threadIdx.x == 0) (ptr)[i] = (int64_t)__builtin_amdgcn_s_memtime(); \
    } while (0)
// thread 0 of whichever workgroup runs it (a role hosted by one workgroup of a launch)
#define DQNX_STAMP_WG(ptr, i)                                                         \
    do {                                                                             \
        if ((ptr) && threadIdx.x == 0) (ptr)[i] = (int64_t)__builtin_amdgcn_s_memtime(); \
    } while (0)
// block `blk`, thread 0
#define DQNX_STAMP_BLK(ptr, i, blk)                                                   \
    do {                                                                             \
        if ((ptr) && blockIdx.x == (unsigned)(blk) && threadIdx.x == 0) (ptr)[i] = (int64_t)__builtin_amdgcn_s_memtime(); \
    } while (0)
// ... after this wave's loads and stores have completed (s_waitcnt vmcnt(0))
#define DQNX_STAMP_BLK_W(ptr, i, blk)                                                 \
    do {                                                                             \
        if ((ptr) && blockIdx.x == (unsigned)(blk)) {                                \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");              \
            if (threadIdx.x == 0) (ptr)[i] = (int64_t)__builtin_amdgcn_s_memtime();  \
        }                                                                            \
    } while (0)
#else
#define DQNX_STAMP(ptr, i) do { } while (0)
#define DQNX_STAMP_WG(ptr, i) do { } while (0)
#define DQNX_STAMP_BLK(ptr, i, blk) do { } while (0)
#define DQNX_STAMP_BLK_W(ptr, i, blk) do { } while (0)
#endif

}  // namespace dqnx

// Kernel-duration timing (dqnx_learn_step_timed, bench.py's roofline): while a pair of events is
// armed on this host thread, the NEXT kernel launched through DQNX_LAUNCH goes out through
// hipExtLaunchKernelGGL with the pair bound to its dispatch, so the events carry that dispatch's own
// begin / end timestamps (the packet's profiling signal, the source rocprofv3's kernel trace reads),
// not the time of marker packets around it.  Disarmed by that launch.
#include <hip/hip_ext.h>
namespace dqnx {
struct KernelTimer {
    hipEvent_t start = nullptr, stop = nullptr;
};
KernelTimer& kernel_timer();   // thread-local (engine.cpp)
}  // namespace dqnx
#define DQNX_LAUNCH(K, G, B, SH, S, ...)                                                         \
    do {                                                                                         \
        dqnx::KernelTimer& _kt = dqnx::kernel_timer();                                           \
        if (_kt.start || _kt.stop) {                                                             \
            const hipEvent_t _e0 = _kt.start, _e1 = _kt.stop;                                    \
            _kt.start = _kt.stop = nullptr;                                                      \
            hipExtLaunchKernelGGL(K, dim3(G), dim3(B), (std::uint32_t)(SH), S, _e0, _e1, 0u, __VA_ARGS__); \
        } else {                                                                                 \
            hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                     \
        }                                                                                        \
    } while (0)

#define DQNX_HIP_CHECK(expr)                                                    \
    do {                                                                        \
        hipError_t _e = (expr);                                                 \
        if (_e != hipSuccess) return dqnx::set_hip_error(_e, #expr, __FILE__, __LINE__); \
    } while (0)

namespace dqnx {
int set_error(int code, const char* fmt, ...);
int set_hip_error(hipError_t e, const char* expr, const char* file, int line);

// Host-side plan knobs (read when a plan is built, so tests can switch them per engine).
//  * route_knob / route_flag: choose between alternative kernel routes that are ALL parity-tested
//    (bitwise equal to the default, or within the stated tolerance of the same reference
//    arithmetic); the tests force each route through the environment.
//  * tuning_knob / tuning_flag: measurement-only parameters (tile, occupancy and threshold sweeps).
//    The shipped library uses the measured defaults; only the diagnostic build
//    (`make tuning`, -DDQNX_TUNING) reads them from the environment.
inline int route_knob(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}
inline bool route_flag(const char* name) { return getenv(name) != nullptr; }
#ifdef DQNX_TUNING
inline int tuning_knob(const char* name, int dflt) { return route_knob(name, dflt); }
inline bool tuning_flag(const char* name) { return route_flag(name); }
#else
inline int tuning_knob(const char*, int dflt) { return dflt; }
inline bool tuning_flag(const char*) { return false; }
#endif
}  // namespace dqnx
