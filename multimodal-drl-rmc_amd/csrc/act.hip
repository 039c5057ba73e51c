// Acting path: Network.actions(obses) as one launch.
//
//   DeepQNetwork.actions          R:dqn/network.py:67-74   argmax_a Q(s, a)
//   DuelingDeepQNetwork.actions   R:dqn/network.py:110-117 argmax_a A(s, a)  (advantage stream only)
//   called by Agent.choose_actions R:dqn/agent.py:92-99 once per env step with n_env rows.
//
// At n_env rows the forward is latency-bound: MLP-284 reads 428 KB of weights once and does
// 0.4 MFLOP per row.  What costs time is the number of dependent HBM round trips, so the
// kernel is shaped to keep that count at about one per layer:
//   * layer 1 (68 % of the weights) is spread over G = ceil(h0/16) workgroups of 16 waves, one
//     output neuron per wave: each lane issues its ceil(in/256) float4 loads of that weight row
//     at once, a wave butterfly reduces the row, lane r writes row r's activation to scratch;
//   * the last workgroup to finish layer 1 (agent-scope ticket, no spinning: every workgroup
//     exits) stages h0 into LDS and runs the remaining layers and the head, 8 neurons per wave
//     per pass with all of a pass's loads in flight before the first FMA;
//   * the argmax (first maximal index, like torch.argmax) is one thread per row.
// Rows are processed R = 1, 2 or 4 at a time per workgroup column (grid.y = row groups).
#include <algorithm>

#include "common.hpp"
#include "learn.hpp"

namespace dqnx {

namespace {

constexpr int kActThreads = 1024;
constexpr int kActWaves = kActThreads / kWave;
constexpr int kActU = 8;   // output neurons per wave per pass after layer 1

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// y[r][j] = act?(sum_k W[j][k] * x[r][k] + b[j]) for j < out, r < R; x, y in LDS (row stride ld).
// VEC: in % 4 == 0 and W 16-byte aligned -> float4 weight loads and LDS reads.
template <int R, int ACT, bool APPLY, bool VEC>
__device__ __forceinline__ void act_dense(const float* __restrict__ W, const float* __restrict__ b, int in, int out,
                                          const float* x, float* y, int ld) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    constexpr int V = VEC ? 4 : 1;
    const int nk = in / V;
    constexpr int U = R >= 4 ? kActU / 2 : kActU;   // 4 rows x 8 neurons would spill at 128 VGPRs
    for (int j0 = wave * U; j0 < out; j0 += kActWaves * U) {
        float acc[U][R];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < R; r++) acc[u][r] = 0.f;
        const float* wr[U];
#pragma unroll
        for (int u = 0; u < U; u++) wr[u] = W + (int64_t)min(j0 + u, out - 1) * in;   // clamped: valid reads, result dropped
        float bias[U];   // issued with the first weight loads, not after the reduction
#pragma unroll
        for (int u = 0; u < U; u++) bias[u] = b[min(j0 + u, out - 1)];
        for (int kv = lane; kv < nk; kv += kWave) {
            if (VEC) {
                float4 wv[U];
#pragma unroll
                for (int u = 0; u < U; u++) wv[u] = ld4(wr[u] + 4 * kv);
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const float4 xv = *reinterpret_cast<const float4*>(x + r * ld + 4 * kv);
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        acc[u][r] = fmaf(wv[u].x, xv.x, acc[u][r]);
                        acc[u][r] = fmaf(wv[u].y, xv.y, acc[u][r]);
                        acc[u][r] = fmaf(wv[u].z, xv.z, acc[u][r]);
                        acc[u][r] = fmaf(wv[u].w, xv.w, acc[u][r]);
                    }
                }
            } else {
                float wv[U];
#pragma unroll
                for (int u = 0; u < U; u++) wv[u] = wr[u][kv];
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const float xv = x[r * ld + kv];
#pragma unroll
                    for (int u = 0; u < U; u++) acc[u][r] = fmaf(wv[u], xv, acc[u][r]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                const float s = wave_sum(acc[u][r]);
                if (lane == r && j0 + u < out) {
                    const float v = s + bias[u];
                    y[r * ld + j0 + u] = APPLY ? act_fwd<ACT>(v) : v;
                }
            }
        }
    }
}

template <int R, int ACT, bool APPLY>
__device__ __forceinline__ void act_dense_any(const float* W, const float* b, int in, int out, const float* x,
                                              float* y, int ld) {
    if ((in & 3) == 0 && ((uintptr_t)W & 15) == 0)
        act_dense<R, ACT, APPLY, true>(W, b, in, out, x, y, ld);
    else
        act_dense<R, ACT, APPLY, false>(W, b, in, out, x, y, ld);
}

// Layer 1, one neuron per wave: h[r][j] = act(W[j] . x[r] + b[j]).  VEC as above (also needs D % 4 == 0).
template <int R, int ACT, bool VEC>
__device__ __forceinline__ void act_layer1_neuron(const float* __restrict__ W, const float* __restrict__ b, int in,
                                                  int j, const float* x, int ld, float* h, int ldh) {
    const int lane = threadIdx.x & (kWave - 1);
    constexpr int V = VEC ? 4 : 1;
    const int nk = in / V;
    const float* w = W + (int64_t)j * in;
    const float bias = b[j];
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.f;
    constexpr int P = VEC ? 4 : 8;   // loads of the row issued together per lane
    for (int k0 = lane; k0 < nk; k0 += P * kWave) {
        if (VEC) {
            float4 wv[P];
#pragma unroll
            for (int p = 0; p < P; p++) {
                const int kv = k0 + p * kWave;
                wv[p] = kv < nk ? ld4(w + 4 * kv) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int p = 0; p < P; p++) {
                const int kv = min(k0 + p * kWave, nk - 1);
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const float4 xv = *reinterpret_cast<const float4*>(x + r * ld + 4 * kv);
                    acc[r] = fmaf(wv[p].x, xv.x, acc[r]);
                    acc[r] = fmaf(wv[p].y, xv.y, acc[r]);
                    acc[r] = fmaf(wv[p].z, xv.z, acc[r]);
                    acc[r] = fmaf(wv[p].w, xv.w, acc[r]);
                }
            }
        } else {
            float wv[P];
#pragma unroll
            for (int p = 0; p < P; p++) {
                const int kv = k0 + p * kWave;
                wv[p] = kv < nk ? w[kv] : 0.f;
            }
#pragma unroll
            for (int p = 0; p < P; p++) {
                const int kv = min(k0 + p * kWave, nk - 1);
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] = fmaf(wv[p], x[r * ld + kv], acc[r]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const float s = wave_sum(acc[r]);
        if (lane == r) h[r * ldh + j] = act_fwd<ACT>(s + bias);
    }
}

template <int R, int ACT>
__global__ __launch_bounds__(kActThreads) void k_act_mlp(ActArgs a) {
    extern __shared__ float lds[];
    __shared__ int s_last;
    float* x = lds;
    float* y = lds + R * a.ld;
    const int grp = blockIdx.y;
    const int row0 = grp * R;
    const int nr = min(R, a.n - row0);
    const int tid = threadIdx.x;
    for (int i = tid; i < R * a.D; i += kActThreads) {
        const int r = i / a.D, k = i - r * a.D;
        x[r * a.ld + k] = r < nr ? a.obs[(int64_t)(row0 + r) * a.D + k] : 0.f;
    }
    __syncthreads();

    // ---- layer 1 slice: neurons [16 * blockIdx.x, +16), one per wave, into scratch
    const int h0 = a.out[0];
    float* hs = a.scratch + (int64_t)row0 * h0;   // [R][h0] of this row group
    {
        const int j = blockIdx.x * kActWaves + tid / kWave;
        const float* W = a.params + a.off[0];
        if (j < h0) {
            if ((a.D & 3) == 0 && (a.off[0] & 3) == 0 && (a.ld & 3) == 0)
                act_layer1_neuron<R, ACT, true>(W, W + (int64_t)h0 * a.D, a.D, j, x, a.ld, hs, h0);
            else
                act_layer1_neuron<R, ACT, false>(W, W + (int64_t)h0 * a.D, a.D, j, x, a.ld, hs, h0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (gridDim.x > 1) {
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t t = __hip_atomic_fetch_add(a.tickets - grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = t == gridDim.x - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                *(a.tickets - grp) = 0;   // ready for the next launch
            }
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
    }

    // ---- last arriver: h0 -> LDS, remaining layers, head, argmax
    for (int i = tid; i < R * h0; i += kActThreads) {
        const int r = i / h0, k = i - r * h0;
        x[r * a.ld + k] = hs[(int64_t)r * h0 + k];
    }
    __syncthreads();
    for (int l = 1; l < a.L; l++) {
        const float* W = a.params + a.off[l];
        act_dense_any<R, ACT, true>(W, W + (int64_t)a.out[l] * a.in[l], a.in[l], a.out[l], x, y, a.ld);
        __syncthreads();
        float* t = x; x = y; y = t;
    }
    const float* H = a.params + a.head_off;
    const int F = a.F, A = a.A;
    // dueling: only the advantage stream decides (R:dqn/network.py:110-117); fc_val is not evaluated
    const float* Wh = a.dueling ? H + F + 1 : H;
    act_dense_any<R, ACT, false>(Wh, Wh + (int64_t)A * F, F, A, x, y, a.ld);
    __syncthreads();
    if (tid < nr) {
        const int r = tid;
        const float* q = y + r * a.ld;
        int best = 0;
        float bv = q[0];
        for (int j = 0; j < A; j++) {
            const float v = q[j];
            if (a.values) a.values[(int64_t)(row0 + r) * A + j] = v;
            if (v > bv || (v != v && bv == bv)) { bv = v; best = j; }   // first max; NaN wins like torch
        }
        a.actions[row0 + r] = best;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (r == 0 && grp == 0 && gridDim.y == 1 && a.done_flag)
            __hip_atomic_store(a.done_flag, a.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The completion word for dqnx_act_host: system-scope release after the actions' stores, so the
// host sees the actions once it sees done_seq (fine-grained pinned memory)
__device__ __forceinline__ void act_signal(const ActArgs& a) {
    if (a.done_flag) __hip_atomic_store(a.done_flag, a.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Two hidden layers (the reference's MLP bodies): layer 2 is summed in parts where layer 1 is made.
// Workgroup w owns layer-1 neurons [16 w, 16 w + 16) (one per wave, as k_act_mlp) and also forms
// their share of every layer-2 pre-activation, p_w[r][o] = sum_{k < 16} W2[o][16 w + k] h1[r][16 w + k];
// the last workgroup to arrive sums the G shares in w order (+ b2, activation), then runs the head
// (advantage stream for dueling nets) and the first-max argmax.  Against k_act_mlp the tail after the
// hand-off no longer waits on a weight load of its own: layer 2's weights and the head's are fetched
// at the top of the kernel, beside layer 1's, and the hand-off moves G floats per layer-2 neuron.
// The shares go out as write-through (sc1) stores, so the producers need no release fence (the
// last arriver's acquire stays: cdna_hip_programming.md Guideline 16, the sc1 form of the recipe).
// This rests on gfx950 ISA behaviour, not on the HIP/C++ memory model: a relaxed agent-scope store
// lowers to `global_store ... sc1` (write-through to memory), every storing wave drains vmcnt before
// the workgroup barrier, and ONE lane then takes the relaxed agent-scope ticket; the workgroup whose
// ticket comes back last is the consumer -- row 1 of MI355X_MICROARCH.md's measured hand-off table
// ("ONE lane of each storing workgroup, for ALL that workgroup's stores ... an agent-scope atomic
// add").  A release RMW on the ticket would be the portable form; it lowers to buffer_wbl2 (an L2
// write-back per workgroup) on this chip, which the sc1 stores make redundant.
template <int R, int ACT>
__global__ __launch_bounds__(kActThreads) void k_act_mlp2(ActArgs a) {
    extern __shared__ float lds[];
    __shared__ int s_last;
    float* x = lds;                      // [R][ld] obs, later h2
    float* h1 = lds + R * a.ld;          // [R][16] this workgroup's layer-1 outputs, later Q [R][16]
    float* hw = h1 + R * 16;             // [A][F] head weights (last arriver)
    const int grp = blockIdx.y;
    const int row0 = grp * R;
    const int nr = min(R, a.n - row0);
    const int tid = threadIdx.x;
    const int G = gridDim.x;
    const int h0 = a.out[0], o1 = a.out[1], F = a.F, A = a.A;
    const int k0 = blockIdx.x * kActWaves;
    const int nk = min(kActWaves, h0 - k0);
    // (0) loads that do not depend on the observation, first: this thread's layer-2 weights (row
    //     o = tid, the workgroup's 16 columns) and bias, and a float4 of the head's weights
    const float* W2 = a.params + a.off[1];
    float w2[kActWaves];
#pragma unroll
    for (int k = 0; k < kActWaves; k++) w2[k] = (tid < o1 && k < nk) ? W2[(int64_t)tid * h0 + k0 + k] : 0.f;
    const float b2 = tid < o1 ? W2[(int64_t)o1 * h0 + tid] : 0.f;
    const float* Hh = a.params + a.head_off;
    const float* Wh = a.dueling ? Hh + F + 1 : Hh;   // advantage stream (R:dqn/network.py:110-117)
    const int nh4 = (A * F) >> 2;                     // (A * F % 4 == 0 and 16-byte rows: act2_ok)
    const float4 hwv = tid < nh4 ? ld4(Wh + 4 * tid) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float hb = tid < A ? Wh[(int64_t)A * F + tid] : 0.f;
    for (int i = tid; i < R * a.D; i += kActThreads) {
        const int r = i / a.D, k = i - r * a.D;
        x[r * a.ld + k] = r < nr ? a.obs[(int64_t)(row0 + r) * a.D + k] : 0.f;
    }
    __syncthreads();
    // (1) layer 1: neuron k0 + wave of every row into LDS
    {
        const int j = k0 + tid / kWave;
        const float* W = a.params + a.off[0];
        if (j < h0) {
            if ((a.D & 3) == 0 && (a.off[0] & 3) == 0 && (a.ld & 3) == 0)
                act_layer1_neuron<R, ACT, true>(W, W + (int64_t)h0 * a.D, a.D, j, x, a.ld, h1 - k0, 16);
            else
                act_layer1_neuron<R, ACT, false>(W, W + (int64_t)h0 * a.D, a.D, j, x, a.ld, h1 - k0, 16);
        }
    }
    __syncthreads();
    // (2) this workgroup's share of layer 2, written through (sc1) to memory
    float* part = a.scratch + (int64_t)grp * G * R * o1;   // [G][R][o1] of this row group
    if (tid < o1) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < kActWaves; k++) acc = fmaf(w2[k], h1[r * 16 + k], acc);
            __hip_atomic_store(part + ((int64_t)blockIdx.x * R + r) * o1 + tid, acc, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (G > 1) {
        if (tid == 0) {
            const uint32_t t = __hip_atomic_fetch_add(a.tickets - grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = t == (uint32_t)G - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                *(a.tickets - grp) = 0;   // ready for the next launch
            }
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
    }
    // (3) last arriver: h2 = act(sum of the shares in workgroup order + b2), the head, argmax
    if (tid < nh4) *reinterpret_cast<float4*>(hw + 4 * tid) = hwv;
    if (tid < o1) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            float z = 0.f;
            for (int w = 0; w < G; w++)
                z += __hip_atomic_load(part + ((int64_t)w * R + r) * o1 + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            x[r * a.ld + tid] = act_fwd<ACT>(z + b2);
        }
    }
    const float hbj = __shfl(hb, tid & 15, kWave);   // (bias of head output tid % 16, from lane tid % 16)
    __syncthreads();
    float* q = h1;
    if (tid < R * 16) {
        const int r = tid >> 4, j = tid & 15;
        if (j < A) {
            const float* xr = x + r * a.ld;
            const float* wr = hw + j * F;
            float acc = 0.f;
            for (int k = 0; k < F; k++) acc = fmaf(wr[k], xr[k], acc);
            q[r * 16 + j] = acc + hbj;
        }
    }
    __syncthreads();
    if (tid < nr) {
        const int r = tid;
        const float* qr = q + r * 16;
        int best = 0;
        float bv = qr[0];
        for (int j = 0; j < A; j++) {
            const float v = qr[j];
            if (a.values) a.values[(int64_t)(row0 + r) * A + j] = v;
            if (v > bv || (v != v && bv == bv)) { bv = v; best = j; }   // first max; NaN wins like torch
        }
        a.actions[row0 + r] = best;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (r == 0 && grp == 0 && gridDim.y == 1) act_signal(a);   // (one row group: n <= R)
    }
}

// ONE workgroup for the whole forward of n <= 2 rows (the agent's n_env): every weight of the net
// (MLP-284: 428 KB) is requested by the 1024 threads at once, straight into registers -- one CU's
// L2 / Infinity-Cache stream -- so the launch makes ONE dependent memory round trip plus the
// actions' store, where k_act_mlp2 makes three (layer 1 across 16 workgroups, the share hand-off,
// the head): no ticket, no acquire, no cross-workgroup hand-off.
//   layer 1: TPN1 = 1024 / h0 threads per neuron, thread (j, q) holds float4 q, q + TPN1, ... of row
//            j (consecutive lanes read consecutive 16 bytes), partial dot products per row summed
//            over the TPN1 lanes by xor shuffles;
//   layer 2: TPN2 = 1024 / h1 threads per neuron, float4 q, q + TPN2, ... of row o (loaded with
//            layer 1's weights);
//   head:    A rows (advantages for dueling nets, R:dqn/network.py:110-117) x F, one float4 per
//            thread, summed over the F / 4 lanes of a row.
// Compile-time register budget: W1S float4 of layer 1 and W2S of layer 2 per thread (act1_ok).
constexpr int kAct1Threads = 512;   // 2 waves per SIMD: 256 registers a lane for the weight slices
template <int TPN>
__device__ __forceinline__ float group_sum(float v) {   // over TPN consecutive lanes (power of two)
#pragma unroll
    for (int o = TPN / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
// G > 1 (DQNX_ACT1_G): the same over G workgroups on G CUs, workgroup g owning layer-1 neurons
// [g h0/G, (g+1) h0/G) and its share of every layer-2 pre-activation (k_act_mlp2's split, G-fold wider
// slices): each CU streams 1/G of the weights.  The shares go out write-through (sc1), every storing
// wave drains vmcnt, a barrier, ONE lane's agent-scope ticket; the workgroup whose ticket comes back last
// sums the shares in workgroup order with sc1 loads and runs bias + activation, the head and the argmax
// (MI355X_MICROARCH.md's measured hand-off table, first row).
template <int R, int ACT, int G, int TPN1, int TPN2, int W1S, int W2S>
__global__ __launch_bounds__(kAct1Threads) void k_act_mlp1(ActArgs a) {
    extern __shared__ float lds[];
    __shared__ int s_last;
    const int tid = threadIdx.x;
    const int D = a.D, h0 = a.out[0], h1 = a.out[1], F = a.F, A = a.A;
    const int n = a.n;
    const int h0g = h0 / G, g0 = (G > 1 ? (int)blockIdx.x : 0) * h0g;   // this workgroup's layer-1 neurons
    const int d4 = D >> 2, h04 = h0 >> 2, h0g4 = h0g >> 2;
    float4* x4 = reinterpret_cast<float4*>(lds);          // [R][d4] obs
    float* y1 = lds + R * D;                               // [R][h0g]
    float* y2 = y1 + R * h0g;                              // [R][h1]
    float* q = y2 + R * h1;                                // [R][16]
    const float* P = a.params;
    // (0) every load at once: layer 1's row slices, layer 2's, the head's float4, the biases, the obs
    const int jl = tid / TPN1, q1 = tid % TPN1, j = g0 + jl;
    const float4* W1 = reinterpret_cast<const float4*>(P + a.off[0]) + (int64_t)(jl < h0g ? j : 0) * d4;
    float4 w1[W1S];
#pragma unroll
    for (int i = 0; i < W1S; i++) {
        const int c = q1 + TPN1 * i;
        w1[i] = (c < d4 && jl < h0g) ? W1[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int o = tid / TPN2, q2 = tid % TPN2;
    const float4* W2 = reinterpret_cast<const float4*>(P + a.off[1]) + (int64_t)(o < h1 ? o : 0) * h04 + (g0 >> 2);
    float4 w2[W2S];
#pragma unroll
    for (int i = 0; i < W2S; i++) {
        const int c = q2 + TPN2 * i;
        w2[i] = (c < h0g4 && o < h1) ? W2[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float* Hh = P + a.head_off;
    const float* Wh = a.dueling ? Hh + F + 1 : Hh;   // advantage stream (R:dqn/network.py:110-117)
    // (the advantage rows start F + 1 floats into the head block: 4-byte aligned only -> scalar loads,
    // two consecutive elements of one row per thread, F / 2 lanes per row)
    const int hr = tid / (F / 2), hc = 2 * (tid % (F / 2));
    const float wh0 = hr < A ? Wh[(int64_t)hr * F + hc] : 0.f;
    const float wh1 = hr < A ? Wh[(int64_t)hr * F + hc + 1] : 0.f;
    const float b1 = jl < h0g ? P[a.off[0] + (int64_t)h0 * D + j] : 0.f;
    const float b2 = o < h1 ? P[a.off[1] + (int64_t)h1 * h0 + o] : 0.f;
    const float bh = hr < A ? Wh[(int64_t)A * F + hr] : 0.f;
    for (int e = tid; e < R * d4; e += kAct1Threads) {
        const int r = e / d4, c = e - r * d4;
        x4[e] = r < n ? reinterpret_cast<const float4*>(a.obs + (int64_t)r * D)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    // (1) layer 1 (this workgroup's neurons)
#pragma unroll
    for (int r = 0; r < R; r++) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < W1S; i++) {
            const int c = q1 + TPN1 * i;
            if (c < d4) {
                const float4 xv = x4[r * d4 + c];
                acc = fmaf(w1[i].x, xv.x, acc);
                acc = fmaf(w1[i].y, xv.y, acc);
                acc = fmaf(w1[i].z, xv.z, acc);
                acc = fmaf(w1[i].w, xv.w, acc);
            }
        }
        acc = group_sum<TPN1>(acc);
        if (q1 == 0 && jl < h0g) y1[r * h0g + jl] = act_fwd<ACT>(acc + b1);
    }
    __syncthreads();
    // (2) layer 2: the pre-activations (G == 1), or this workgroup's share of them
    const float4* y14 = reinterpret_cast<const float4*>(y1);
    float z[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < W2S; i++) {
            const int c = q2 + TPN2 * i;
            if (c < h0g4) {
                const float4 xv = y14[r * h0g4 + c];
                acc = fmaf(w2[i].x, xv.x, acc);
                acc = fmaf(w2[i].y, xv.y, acc);
                acc = fmaf(w2[i].z, xv.z, acc);
                acc = fmaf(w2[i].w, xv.w, acc);
            }
        }
        z[r] = group_sum<TPN2>(acc);
    }
    if constexpr (G > 1) {
        float* part = a.scratch;   // [G][R][h1] (one row group)
        if (q2 == 0 && o < h1) {
#pragma unroll
            for (int r = 0; r < R; r++)
                __hip_atomic_store(part + ((int64_t)blockIdx.x * R + r) * h1 + o, z[r], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const uint32_t t = __hip_atomic_fetch_add(a.tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = t == (uint32_t)G - 1;
            if (last) __hip_atomic_store(a.tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
        if (q2 == 0 && o < h1) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                float sum = 0.f;
#pragma unroll
                for (int w = 0; w < G; w++)
                    sum += __hip_atomic_load(part + ((int64_t)w * R + r) * h1 + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                z[r] = sum;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++)
        if (q2 == 0 && o < h1) y2[r * h1 + o] = act_fwd<ACT>(z[r] + b2);
    __syncthreads();
    // (3) the head: F / 2 lanes per output row (a power of two, <= 64: act1_ok)
#pragma unroll
    for (int r = 0; r < R; r++) {
        float acc = 0.f;
        if (hr < A) {
            acc = fmaf(wh0, y2[r * h1 + hc], acc);
            acc = fmaf(wh1, y2[r * h1 + hc + 1], acc);
        }
        for (int off = F / 4; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, kWave);
        if (hc == 0 && hr < A) q[r * 16 + hr] = acc + bh;
    }
    __syncthreads();
    if (tid < n) {
        const int r = tid;
        const float* qr = q + r * 16;
        int best = 0;
        float bv = qr[0];
        for (int jj = 0; jj < A; jj++) {
            const float v = qr[jj];
            if (a.values) a.values[(int64_t)r * A + jj] = v;
            if (v > bv || (v != v && bv == bv)) { bv = v; best = jj; }   // first max; NaN wins like torch
        }
        a.actions[r] = best;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (r == 0) act_signal(a);
    }
}

// k_act_mlp1 applies: n <= 2 rows, two hidden layers, widths dividing the 1024 threads into powers of
// two per neuron, every weight row a whole number of 16-byte pieces within the register budget, a
// head whose F / 4 lanes per row fit one wave.  (DQNX_ACT1=0: the multi-workgroup kernels.)
static bool act1_ok(const ActArgs& a, int G, int* tpn1, int* tpn2) {
    if (a.L != 2 || a.n > 4 || a.A > 16 || route_knob("DQNX_ACT1", 1) == 0) return false;
    const int D = a.D, h0 = a.out[0], h1 = a.out[1], F = a.F;
    if (D % 4 || h0 % (4 * G) || F % 4 || (a.off[0] & 3) || (a.off[1] & 3) || F != h1) return false;
    if (G > 1 && (!a.scratch || !a.tickets)) return false;
    auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
    const int h0g = h0 / G;
    if (!pow2(h0g) || !pow2(h1) || h0g > kAct1Threads || h1 > kAct1Threads) return false;
    const int t1 = kAct1Threads / h0g, t2 = kAct1Threads / h1;
    const int lpr = F / 2;   // head lanes per row
    if (!pow2(lpr) || lpr > kWave || a.A * lpr > kAct1Threads) return false;
    *tpn1 = t1;
    *tpn2 = t2;
    return true;
}

// k_act_mlp2 applies: two hidden layers, layer 2 on one thread per neuron, the head's advantage / Q
// rows as float4s of one pass (A * F % 4 == 0, 16-byte aligned, <= 4096 floats), A <= 16; with a
// completion word, one row group (act_signal stores it from row group 0)
static bool act2_ok(const ActArgs& a, int R) {
    const int64_t hoff = a.head_off + (a.dueling ? a.F + 1 : 0);
    return a.L == 2 && a.out[1] <= kActThreads && a.A <= 16 && (a.A * a.F) % 4 == 0 &&
           a.A * a.F <= 4 * kActThreads && (hoff & 3) == 0 && (a.done_flag == nullptr || a.n <= R) &&
           route_knob("DQNX_ACT2", 1) != 0;
}

template <int R, int ACT>
static int launch_act1(const ActArgs& a, int G, int t1, int t2, hipStream_t s) {
    const size_t lds = ((size_t)R * (a.D + a.out[0] / G + a.out[1] + 16)) * sizeof(float);
    const int s1 = (a.D / 4 + t1 - 1) / t1, s2 = (a.out[0] / G / 4 + t2 - 1) / t2;   // float4 slots per thread
#define ACT1(GG, T1, T2, S1, S2) DQNX_LAUNCH((k_act_mlp1<R, ACT, GG, T1, T2, S1, S2>), dim3(GG), dim3(kAct1Threads), lds, s, a)
    // the reference's MLP (R:env/custom_env/macro with lane/dqn_config.py:76-84): D -> 256 -> 128
    if (G == 1 && t1 == 2 && t2 == 4 && s2 <= 16) {
        if (s1 <= 8) ACT1(1, 2, 4, 8, 16);
        else if (s1 <= 16) ACT1(1, 2, 4, 16, 16);
        else if (s1 <= 24) ACT1(1, 2, 4, 24, 16);
        else if (s1 <= 36) ACT1(1, 2, 4, 36, 16);   // MLP-284: 71 float4 per row over 2 lanes
        else return -1;
    } else if (G == 4 && t1 == 8 && t2 == 4 && s2 <= 4) {   // 64 layer-1 neurons a workgroup
        if (s1 <= 4) ACT1(4, 8, 4, 4, 4);
        else if (s1 <= 8) ACT1(4, 8, 4, 8, 4);
        else if (s1 <= 12) ACT1(4, 8, 4, 12, 4);   // MLP-284: 71 float4 per row over 8 lanes
        else return -1;
    } else if (G == 8 && t1 == 16 && t2 == 4 && s2 <= 2) {   // 32 a workgroup
        if (s1 <= 8) ACT1(8, 16, 4, 8, 2);   // MLP-284: 71 float4 per row over 16 lanes
        else return -1;
    } else if (G == 2 && t1 == 4 && t2 == 4 && s2 <= 8) {   // 128 a workgroup
        if (s1 <= 8) ACT1(2, 4, 4, 8, 8);
        else if (s1 <= 18) ACT1(2, 4, 4, 18, 8);   // MLP-284: 71 float4 per row over 4 lanes
        else return -1;
    } else {
        return -1;
    }
#undef ACT1
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

template <int R>
int launch_act_r(const ActArgs& a, hipStream_t s) {
    if constexpr (R <= 2) {   // (4 rows of MLP-284's slices would spill the 256 registers)
        int t1 = 0, t2 = 0;
        // DQNX_ACT1_G: workgroups (CUs) the one-round-trip kernel spreads the weights over (1, 2 or 4)
        const int kg = route_knob("DQNX_ACT1_G", 4);
        for (int G : {kg == 1 || kg == 2 || kg == 4 || kg == 8 ? kg : 4, 1}) {
            if (a.n <= R && ((uintptr_t)a.obs & 15) == 0 && act1_ok(a, G, &t1, &t2)) {
                const int rc = a.act == DQNX_ACT_RELU ? launch_act1<R, DQNX_ACT_RELU>(a, G, t1, t2, s)
                                                       : launch_act1<R, DQNX_ACT_ELU>(a, G, t1, t2, s);
                if (rc != -1) return rc;
            }
        }
    }
    const dim3 grid((a.out[0] + kActWaves - 1) / kActWaves, (a.n + R - 1) / R);
    if (act2_ok(a, R)) {
        const size_t lds2 = ((size_t)R * a.ld + R * 16 + (size_t)a.A * a.F) * sizeof(float);
        if (a.act == DQNX_ACT_RELU)
            DQNX_LAUNCH((k_act_mlp2<R, DQNX_ACT_RELU>), grid, dim3(kActThreads), lds2, s, a);
        else
            DQNX_LAUNCH((k_act_mlp2<R, DQNX_ACT_ELU>), grid, dim3(kActThreads), lds2, s, a);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    const size_t lds = (size_t)2 * R * a.ld * sizeof(float);
    if (a.act == DQNX_ACT_RELU)
        DQNX_LAUNCH((k_act_mlp<R, DQNX_ACT_RELU>), grid, dim3(kActThreads), lds, s, a);
    else
        DQNX_LAUNCH((k_act_mlp<R, DQNX_ACT_ELU>), grid, dim3(kActThreads), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace

int act_rows_per_block(int n, int ld) {
    int R = n <= 1 ? 1 : (n == 2 ? 2 : 4);
    while (R > 1 && (size_t)2 * R * ld * sizeof(float) > kActMaxLds) R /= 2;
    return (size_t)2 * R * ld * sizeof(float) > kActMaxLds ? 0 : R;
}

uint64_t act_scratch_bytes(int n, int h0, int ld, int L, int out1) {
    const int R = act_rows_per_block(n, ld);
    if (R == 0 || n <= 0) return 0;
    const int64_t groups = (n + R - 1) / R;
    // per row group: k_act_mlp's [R][h0] layer-1 outputs, or k_act_mlp2's [G][R][out1] layer-2 shares
    const int64_t G = (h0 + kActWaves - 1) / kActWaves;
    const int64_t per = std::max<int64_t>((int64_t)R * h0, L >= 2 ? G * R * out1 : 0);
    return (uint64_t)groups * per * sizeof(float) + (uint64_t)groups * 4;
}

int launch_act(const ActArgs& a, hipStream_t s) {
    if (a.n <= 0) return DQNX_OK;
    switch (act_rows_per_block(a.n, a.ld)) {
        case 4: return launch_act_r<4>(a, s);
        case 2: return launch_act_r<2>(a, s);
        case 1: return launch_act_r<1>(a, s);
        default: return set_error(DQNX_EUNSUPPORTED, "dqnx_act: layer width %d does not fit LDS", a.ld);
    }
}

}  // namespace dqnx
