// Fused MLP learn-step kernels (gfx950): the whole forward of every stream in ONE launch and
// the Q head / TD target / Huber / dZ chain in one more.
//
//   k_mlp_fwd   one workgroup = 16 rows of one stream (online(s), online(s'), target(s')):
//               gather the rows from the replay ring into LDS, then every Linear layer and the
//               Q head in turn, activations kept in LDS between layers.  Writes only what the
//               backward needs: stream 0's activations and gathered rows, and the raw head
//               outputs [3][B][16] of every stream.
//   k_head_bwd  one workgroup = 16 samples (x nsplit column parts): dueling aggregate,
//               Double-DQN argmax / DQN max, y = r + (1-d)*gamma*q', Huber (mean, or
//               IS-weighted under PER), dHead, then dZ_L = (dHead W_head) (.) act'(H_L) and
//               dZ_{l-1} = (dZ_l W_l) (.) act'(H_{l-1}) down to layer 1, all in LDS.
// The weight gradients (split-K slabs, k_bwd_level) and Adam (k_adam) follow as two more
// launches: 5 launches per learn step instead of 7.
//
// Reference path (R: = /root/reference/):
//   DoubleAgent.learn R:dqn/agent.py:204-226, SimpleAgent.learn :166-185, PerDoubleAgent.learn
//   :245-272; DuelingDeepQNetwork.forward R:dqn/network.py:90-96 (aggregate :83);
//   DeepQNetwork.forward :61-65; MLP body R:env/custom_env/macro with lane/dqn_config.py:76-84.
//
// GEMM shape: M = 16 rows per workgroup, so every wave owns 16 output columns (one or two
// 16x16 tiles) and streams ITS weights straight from L2 into registers; nothing about W is
// shared between waves, so W never goes through LDS (cdna guide §5: "GEMV / M <= 16 ... load
// straight to VGPRs").  The weights are read from fragment-blocked copies (relayout.hpp):
// one coalesced 1 KiB buffer_load_dwordx4 per wave per 16x16x16 block.  The 16-row
// activation tile is shared by all waves and lives in LDS (row stride = 8 mod 64 floats:
// conflict-free ds_read_b128 fragments, MI355X_MICROARCH.md §LDS).
#include "learn.hpp"
#include "per_common.hpp"
#include "sample_body.hpp"

namespace dqnx {

constexpr int FW = FUSED_WAVES;
constexpr int FT = 64 * FW;
#ifndef DQNX_FPF
#define DQNX_FPF 4
#endif
#ifndef DQNX_FNB
#define DQNX_FNB 2   // measured: 3 and 4 sets are 0.9 / 2 us slower per forward at MLP-284 B=1024
#endif
#ifndef DQNX_FUSED_ORDER
#define DQNX_FUSED_ORDER 0   // gather issue order: 0 slots, W, rows; 1 W, slots, rows; 2 slots, rows, W
#endif
constexpr int FPF = DQNX_FPF;   // 16-deep chunks per group
constexpr int FNB = DQNX_FNB;   // register sets: FNB-1 groups of W in flight ahead of the MFMAs
constexpr int FGQ = 6;
// Gather registers sized to the row width: a gather slot holds one float4 of the 16 * MR-row input
// tile, so rows of <= 288 multiplied columns (MLP-284 both ways, MLP-14) need ceil(16 MR 72 / FT)
// slots -- 3 / 5 / 9 at MR 1 / 2 / 4 -- instead of the FGQ * MR the widest rows need (whose
// clamped dead loads also held 96 VGPRs at MR = 4 and kept the bf16 forward at 2 waves / SIMD).
constexpr int FWD_NARROW_Q4 = 72;
template <int MR, int GW>
__host__ __device__ constexpr int fwd_gather_slots() {
    return GW == 0 ? (16 * MR * FWD_NARROW_Q4 + FT - 1) / FT : FGQ * MR;
}
// bf16: slots of 8 bf16 (16 bytes) from the ring's bf16 copies, half as many
template <int MR, int GW>
__host__ __device__ constexpr int fwd_gather_slots16() {
    return GW == 0 ? (16 * MR * (FWD_NARROW_Q4 / 2) + FT - 1) / FT : (FGQ * MR + 1) / 2;
}
// The PER tracking workgroup hosted by k_dw_bf16 must not raise the tiles' register budget: 4 items
// per thread without the carried leaves stays within the 80 VGPRs of 6 waves / SIMD (8 items with
// them took 96-101 VGPRs, 4 waves / SIMD, and dw_all 23 -> 27.5 us at B=8192)
#ifndef DQNX_BF16_TRACK_IPT
#define DQNX_BF16_TRACK_IPT 4
#endif
#ifndef DQNX_BF16_TRACK_CARRY
#define DQNX_BF16_TRACK_CARRY false
#endif
#ifndef DQNX_DWB_WAVES
#define DQNX_DWB_WAVES 6
#endif     // float4 gather slots per thread (input tile <= FGQ * FT float4)

__host__ __device__ __forceinline__ int fused_stride(int K) { return ((K + 63) & ~63) + 8; }
__host__ __device__ __forceinline__ int fused_groups(int K) { return (K + 16 * FPF - 1) / (16 * FPF); }
// Chunks of one weight stream over K and MFMA groups of FPF chunks: 16-deep chunks (fp32) or
// 32-deep (bf16), K padded to a whole chunk only; chunks past nch in the last group are
// skipped (their A columns in LDS are not zeroed).  fp32 layer 1 of MLP-284: 18 chunks
// instead of the 20 of whole groups.
template <bool BF>
__host__ __device__ __forceinline__ int fwd_nch(int K) { return BF ? (K + 31) / 32 : (K + 15) / 16; }
template <bool BF>
__host__ __device__ __forceinline__ int fwd_groups(int K) { return (fwd_nch<BF>(K) + FPF - 1) / FPF; }

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also drains every outstanding
// global access of the wave (vmcnt(0)) -- here that would wait for the activation stores
// to HBM and for the weight prefetch in flight across the barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <class K>
static void allow_lds(K kern, size_t bytes) {
    if (bytes > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// ---- weight streams -------------------------------------------------------------------
// Buffer loads through a wave-uniform descriptor: they stay VMEM ops counted by vmcnt alone
// (a generic pointer that lost its address space becomes a flat load, and the compiler then
// drains vmcnt AND lgkmcnt at every use), and an out-of-range offset reads zeros without
// touching memory (the prefetch overrun past the last chunk needs no branch).
constexpr uint32_t kOOB = 0x80000000u;
// buffer op cache-policy operand: sc1 (write-through stores, L1-bypassing loads on gfx950)
constexpr int kCacheSC1 = 16;
constexpr int kPairSpinLimit = 1 << 20;   // paired forward: hand-off polls (s_sleep 1 each) before the error

__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// The output tiles a wave owns: tiles wid and wid + FW of the N/16 column tiles.
struct WaveCols {
    int n0[2];
    int tn;        // 0, 1 or 2 tiles
};
__device__ __forceinline__ WaveCols wave_cols(int N) {
    const int wid = threadIdx.x >> 6, nt = N >> 4;
    WaveCols c;
    c.n0[0] = wid * 16;
    c.n0[1] = (wid + FW) * 16;
    c.tn = (wid + FW < nt) ? 2 : (wid < nt ? 1 : 0);
    return c;
}

// One wave's stream over a fragment-blocked weight copy: chunk ch of column tile t is the
// 1 KiB at byte (t * nch + ch) * 1024, lane-ordered, so off[t] = (t * nch * 64 + lane) * 16.
struct WStream {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t off[2];
    int nch;
    int ng, rot;   // groups of FPF chunks; the group the stream starts at (DQNX_FWD_ROT)
};

// DQNX_FWD_ROT (measurement variant): a workgroup walks its stream's groups starting at group
// `rot` (its row tile mod the group count), so the CUs of an XCD request different weight blocks
// at any moment instead of all the same ones.  Changes the K accumulation order per row tile.
#ifndef DQNX_FWD_ROT
#define DQNX_FWD_ROT 0
#endif
// chunk s of the walk -> chunk of the stream (nch = past the end: an out-of-range fetch)
__device__ __forceinline__ int wchunk(const WStream& w, int s) {
#if DQNX_FWD_ROT
    const int g = s / FPF;
    if (g >= w.ng) return w.nch;
    const int gr = g + w.rot < w.ng ? g + w.rot : g + w.rot - w.ng;
    return gr * FPF + (s - g * FPF);
#else
    return s;
#endif
}

template <int TN>
__device__ __forceinline__ void bfetch(const WStream& w, int s, float4 (&d)[2]) {
    const int ch = wchunk(w, s);
#pragma unroll
    for (int t = 0; t < TN; t++) d[t] = bld4(w.rs, ch < w.nch ? w.off[t] + 1024u * ch : kOOB);
}

// Open the stream over the wave's tiles (column tile offset c0t) and issue groups 0..FNB-2.
// MAXTN: the most column tiles a wave of this kernel owns (1: the second register half is never used)
template <int MAXTN = 2>
__device__ __forceinline__ void stream_open(const float* blk, int ntiles, int nch, int c0t, const WaveCols& c,
                                            WStream& w, float4 (&wb)[FNB][FPF][2], int seed = 0) {
    const uint32_t lane = threadIdx.x & 63;
    w.rs = wave_rsrc(blk, (uint32_t)ntiles * nch * 1024u);
    w.nch = nch;
    w.ng = (nch + FPF - 1) / FPF;
    w.rot = DQNX_FWD_ROT ? seed % w.ng : 0;
    w.off[0] = ((uint32_t)(c0t + (c.tn >= 1 ? c.n0[0] >> 4 : 0)) * nch * 64u + lane) * 16u;
    w.off[1] = ((uint32_t)(c0t + (c.tn >= 2 ? c.n0[1] >> 4 : 0)) * nch * 64u + lane) * 16u;
    if (MAXTN >= 2 && c.tn == 2) {
#pragma unroll
        for (int u = 0; u + 1 < FNB; u++)
#pragma unroll
            for (int p = 0; p < FPF; p++) bfetch<2>(w, u * FPF + p, wb[u][p]);
    } else if (c.tn == 1) {
#pragma unroll
        for (int u = 0; u + 1 < FNB; u++)
#pragma unroll
            for (int p = 0; p < FPF; p++) bfetch<1>(w, u * FPF + p, wb[u][p]);
    }
}

// acc[t] += A[16][K-chunks ch0 ...] . B_t for one group of FPF chunks (A fragments from LDS).
// fp32: MFMA jj of a chunk consumes k = 16 ch + 4 (lane >> 4) + jj for both operands.
// bf16: one 16x16x32 MFMA per chunk, k = 32 ch + 8 (lane >> 4) + j; chunks >= nch skipped.
template <int TN, bool BF>
__device__ __forceinline__ void mma_group(const void* ap_, int ch0, int nch, const float4 (&w)[FPF][2],
                                          floatx4 (&acc)[2]) {
    if constexpr (!BF) {
        const float* ap = static_cast<const float*>(ap_);
        float4 av[FPF];
#pragma unroll
        for (int p = 0; p < FPF; p++) av[p] = *reinterpret_cast<const float4*>(ap + (ch0 + p) * 16);
#pragma unroll
        for (int p = 0; p < FPF; p++) {
            if (ch0 + p >= nch) break;
#pragma unroll
            for (int t = 0; t < TN; t++) acc[t] = mfma16x16x4(av[p].x, w[p][t].x, acc[t]);
#pragma unroll
            for (int t = 0; t < TN; t++) acc[t] = mfma16x16x4(av[p].y, w[p][t].y, acc[t]);
#pragma unroll
            for (int t = 0; t < TN; t++) acc[t] = mfma16x16x4(av[p].z, w[p][t].z, acc[t]);
#pragma unroll
            for (int t = 0; t < TN; t++) acc[t] = mfma16x16x4(av[p].w, w[p][t].w, acc[t]);
        }
    } else {
        const uint16_t* ap = static_cast<const uint16_t*>(ap_);
        u32x4 av[FPF];
#pragma unroll
        for (int p = 0; p < FPF; p++) av[p] = *reinterpret_cast<const u32x4*>(ap + (ch0 + p) * 32);
#pragma unroll
        for (int p = 0; p < FPF; p++) {
            if (ch0 + p >= nch) break;
#pragma unroll
            for (int t = 0; t < TN; t++) acc[t] = mfma16x16x32bf16(av[p], __builtin_bit_cast(u32x4, w[p][t]), acc[t]);
        }
    }
}

// acc = A[16][K] (LDS, stride sa) . B over ngroups groups (K zero padded to ngroups*64 on both
// sides).  B fragments rotate through FNB register sets by group: group g+FNB-1 is issued
// before group g is multiplied, so FNB-1 groups of MFMAs cover each L2 round trip.  Every
// fetch is unconditional (past the last chunk it reads the out-of-range offset), which keeps
// the compiler's vmcnt counts exact; only the MFMAs of missing groups are skipped.
template <int TN, bool BF>
__device__ __forceinline__ void wave_mma_t(const void* As, int sa, int ngroups, const WStream& w,
                                           float4 (&wb)[FNB][FPF][2], floatx4 (&acc)[2]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const void* ap = BF ? (const void*)(static_cast<const uint16_t*>(As) + i * sa + 8 * g)
                        : (const void*)(static_cast<const float*>(As) + i * sa + 4 * g);
#pragma unroll
    for (int t = 0; t < TN; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int grp = 0; grp < ngroups; grp += FNB) {
#pragma unroll
        for (int u = 0; u < FNB; u++) {
            const int ch = (grp + u) * FPF;
#pragma unroll
            for (int p = 0; p < FPF; p++) bfetch<TN>(w, ch + (FNB - 1) * FPF + p, wb[(u + FNB - 1) % FNB][p]);
            // pin the refill ahead of this group's MFMAs: left alone, the scheduler sinks the
            // loads below them and the prefetch distance collapses to ~0
            __builtin_amdgcn_sched_barrier(0);
            if (grp + u < ngroups) mma_group<TN, BF>(ap, wchunk(w, ch), w.nch, wb[u], acc);
        }
    }
}
template <bool BF, int MAXTN = 2>
__device__ __forceinline__ void wave_mma(const void* As, int sa, int ngroups, const WaveCols& c, const WStream& w,
                                         float4 (&wb)[FNB][FPF][2], floatx4 (&acc)[2]) {
    if (MAXTN >= 2 && c.tn == 2) wave_mma_t<2, BF>(As, sa, ngroups, w, wb, acc);
    else if (c.tn == 1) wave_mma_t<1, BF>(As, sa, ngroups, w, wb, acc);
}

// MR row tiles (16 * MR rows per workgroup, large batches): every weight fragment fetched
// from L2 feeds MR MFMAs, so the weight stream per row shrinks MR-fold.  A fragments are read
// per chunk (MR of them) to keep the register budget of MR accumulator sets.
template <int TN, bool BF, int MR>
__device__ __forceinline__ void mma_group_mr(const void* ap_, int rowoff, int ch0, int nch, const float4 (&w)[FPF][2],
                                             floatx4 (&acc)[MR][2]) {
#pragma unroll
    for (int p = 0; p < FPF; p++) {
        if (ch0 + p >= nch) break;
        if constexpr (!BF) {
            const float* ap = static_cast<const float*>(ap_);
            float4 av[MR];
#pragma unroll
            for (int m = 0; m < MR; m++) av[m] = *reinterpret_cast<const float4*>(ap + m * rowoff + (ch0 + p) * 16);
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int t = 0; t < TN; t++) acc[m][t] = mfma16x16x4(av[m].x, w[p][t].x, acc[m][t]);
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int t = 0; t < TN; t++) acc[m][t] = mfma16x16x4(av[m].y, w[p][t].y, acc[m][t]);
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int t = 0; t < TN; t++) acc[m][t] = mfma16x16x4(av[m].z, w[p][t].z, acc[m][t]);
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int t = 0; t < TN; t++) acc[m][t] = mfma16x16x4(av[m].w, w[p][t].w, acc[m][t]);
        } else {
            const uint16_t* ap = static_cast<const uint16_t*>(ap_);
            u32x4 av[MR];
#pragma unroll
            for (int m = 0; m < MR; m++) av[m] = *reinterpret_cast<const u32x4*>(ap + m * rowoff + (ch0 + p) * 32);
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int t = 0; t < TN; t++)
                    acc[m][t] = mfma16x16x32bf16(av[m], __builtin_bit_cast(u32x4, w[p][t]), acc[m][t]);
        }
    }
}
template <int TN, bool BF, int MR>
__device__ __forceinline__ void wave_mma_mr_t(const void* As, int sa, int ngroups, const WStream& w,
                                              float4 (&wb)[FNB][FPF][2], floatx4 (&acc)[MR][2]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const void* ap = BF ? (const void*)(static_cast<const uint16_t*>(As) + i * sa + 8 * g)
                        : (const void*)(static_cast<const float*>(As) + i * sa + 4 * g);
#pragma unroll
    for (int m = 0; m < MR; m++)
#pragma unroll
        for (int t = 0; t < TN; t++) acc[m][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int grp = 0; grp < ngroups; grp += FNB) {
#pragma unroll
        for (int u = 0; u < FNB; u++) {
            const int ch = (grp + u) * FPF;
#pragma unroll
            for (int p = 0; p < FPF; p++) bfetch<TN>(w, ch + (FNB - 1) * FPF + p, wb[(u + FNB - 1) % FNB][p]);
            __builtin_amdgcn_sched_barrier(0);
            if (grp + u < ngroups) mma_group_mr<TN, BF, MR>(ap, 16 * sa, wchunk(w, ch), w.nch, wb[u], acc);
        }
    }
}
template <bool BF, int MR, int MAXTN = 2>
__device__ __forceinline__ void wave_mma_rows(const void* As, int sa, int ngroups, const WaveCols& c, const WStream& w,
                                              float4 (&wb)[FNB][FPF][2], floatx4 (&acc)[MR][2]) {
    if constexpr (MR == 1) {
        wave_mma<BF, MAXTN>(As, sa, ngroups, c, w, wb, acc[0]);
    } else {
        if (c.tn == 2) wave_mma_mr_t<2, BF, MR>(As, sa, ngroups, w, wb, acc);
        else if (c.tn == 1) wave_mma_mr_t<1, BF, MR>(As, sa, ngroups, w, wb, acc);
    }
}

// =====================================================================================
// Forward: every layer + head raw outputs for one 16 * MR-row tile of one stream.
// LDS: buf0 = input tile [16][sx] (later hidden tiles / head partials), buf1 = hidden tiles.
// =====================================================================================
// NL (dense layers) is a template parameter so every per-layer kernel-argument access has a
// constant index: a runtime-indexed kernarg array element becomes a dependent global load
// with its own wait (eight of them serialised the head kernel's prologue).
// BF: bf16 activation tiles in LDS (row strides sx / sh in bf16 elements), bf16 blocked
// weights, 16x16x32 bf16 MFMAs; accumulation, bias, activation and the H stores stay fp32.
// PH (phase): 0 the whole forward; 1 only layer 1, its columns split over a.csplit
// workgroups per row tile, writing H_1 of every stream to HBM; 2 layers 2.. + head, reading
// H_1 back (the split-layer pair: twice or four times the workgroups on the widest GEMM).
// the paired forward (PH 3) needs two workgroups per CU resident (its 2 * tiles * streams grid exceeds
// the chip at B = 1024): 4 waves per SIMD, i.e. <= 128 VGPRs
template <int PH>
constexpr int fwd_waves() { return PH == 3 ? 4 : 1; }
template <int ACT, int NL, bool BF, int MR, int PH, int GW>
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(fwd_waves<PH>()))) void k_mlp_fwd(FusedFwdArgs a) {
    constexpr int RW = 16 * MR;          // rows per workgroup
    constexpr int GQ = BF ? fwd_gather_slots16<MR, GW>() : fwd_gather_slots<MR, GW>();   // gather slots per thread
    constexpr int LB = PH == 2 ? 1 : 0, LE = PH == 1 ? 1 : NL;   // layers of this launch
    constexpr int MTN = PH == 3 ? 1 : 2;   // column tiles per wave (paired forward: <= 128 columns a layer)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    // LDS tile b: pointer arithmetic on `lds` keeps the LDS address space visible to the
    // compiler (ds_read, not flat loads that share the vmcnt counter with the W stream)
#define FBUF(b) (lds + ((b) ? a.buf0 : 0))
    if (a.npc && blockIdx.x == 0) {   // PER: the next sample's numpy MT blocks, twisted ahead on their own CU
        np_cache_extend(a.npc, a.np_state, a.npc_blocks, reinterpret_cast<uint32_t*>(lds));
        return;
    }
    if (a.samp_shape && blockIdx.x == 0) {   // (dispatched first: it starts even when the grid exceeds the chip)
        // in-launch prefetch: the next step's random.sample (R:dqn/replay_memory.py:38-39) into the
        // staging slot.  It reads only the MT state and the ring's size / write pointer, which no
        // kernel of this step writes (the replay push is refused while a draw is pending).
#define FWD_SAMPLER(SH)                                                                              \
        do {                                                                                         \
            constexpr int AH = fwd_sample_ahead(SH);                                                 \
            static_assert(sizeof(SampleLdsBase<FT, AH>) <= (size_t)fwd_sample_tab_off(SH), "layout"); \
            sample_uniform_body<FT, fwd_sample_hs(SH), AH, fwd_sample_bmx(SH)>(                                          \
                a.samp, *reinterpret_cast<SampleLdsBase<FT, AH>*>(lds),                               \
                reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(lds) + fwd_sample_tab_off(SH))); \
        } while (0)
        if (a.samp_shape == 1) FWD_SAMPLER(1);
        else if (a.samp_shape == 2) FWD_SAMPLER(2);
        else FWD_SAMPLER(3);
#undef FWD_SAMPLER
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int nsp = PH == 1 ? a.csplit : (PH == 3 ? 2 : 1);
    const int bid = (int)blockIdx.x - ((a.samp_shape || a.npc) ? 1 : 0);
    const int T0 = xcd_remap(bid, a.tiles * a.nstreams * nsp);
    int part = T0 % nsp, T = T0 / nsp;   // the parts of one row tile are neighbours (one XCD)
    int z = T / a.tiles, tile = T - z * a.tiles;
    if constexpr (PH == 3) {   // the two parts of a row tile: blocks bid and bid ^ 8 (one XCD, tiles % 8 == 0)
        const int tp = a.tiles >> 3, L = bid >> 3, L2 = L >> 1;
        part = L & 1;
        z = L2 / tp;
        tile = (L2 - z * tp) * 8 + (bid & 7);
    } else if (PH != 1 && a.xcd_rows) {   // row tile t of every stream on XCD t % 8 (tiles % 8 == 0)
        const int tp = a.tiles >> 3, L = bid >> 3;
        z = L / tp;
        tile = (L - z * tp) * 8 + (bid & 7);
        part = 0;
    }
    const int s = a.stream_of[z];
    const int tgt = s == 2 ? 1 : 0;
    const int b0 = tile * RW, nb = min(RW, a.Bl - b0);
    const float* P = tgt ? a.tparams : a.params;
    const float* ring = (s == 0) ? a.ring_obs : a.ring_next;
    const bool keep = (s == 0);
    const int coff = (PH == 1 || PH == 3) ? part * (a.out[0] / nsp) : 0;   // layer-1 columns of this part

    if (PH != 2) DQNX_STAMP(a.stamps, 24);   // (slots 24-27: the layer-1 launch of a split forward)
    // the step's Adam scalars for the update launch: a dependent ctrl -> table chain on the last
    // thread of one workgroup, hidden under that workgroup's gather
    if (PH != 2 && a.adam_ctrl && T0 == a.tiles * a.nstreams * nsp - 1 && tid == FT - 1) adam_advance(a.adam_ctrl, a.ab);
    float4 wb[FNB][FPF][2];
    WStream ws;
    WaveCols c = wave_cols((PH == 1 || PH == 3) ? a.out[0] / nsp : a.out[LB]);
    if constexpr (PH == 2) {
        // H_1 rows of this stream, written by the split layer-1 launch -> LDS (zero past the batch)
        stream_open<MTN>(a.wblk[tgt][1], a.out[1] >> 4, fwd_nch<BF>(a.in[1]), 0, c, ws, wb, tile);
        const int N0 = a.out[0], q4 = N0 >> 2;
        const float* h1 = a.H[0] + (int64_t)s * a.Bl * N0;
        float4 hv[2 * MR];
#pragma unroll
        for (int j = 0; j < 2 * MR; j++) {
            const int q = tid + j * FT;
            const int r = q / q4, c4 = q - r * q4;
            const bool ok = r < nb && r < RW;
            float4 x = ld4(h1 + (int64_t)(b0 + (ok ? r : 0)) * N0 + 4 * c4);
            hv[j] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int j = 0; j < 2 * MR; j++) {
            const int q = tid + j * FT;
            const int r = q / q4, c4 = q - r * q4;
            if (r < RW) {
                if constexpr (BF)
                    *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(FBUF(0)) + r * a.sh + 4 * c4) =
                        make_uint2(bf16_pack2(hv[j].x, hv[j].y), bf16_pack2(hv[j].z, hv[j].w));
                else
                    *reinterpret_cast<float4*>(FBUF(0) + r * a.sh + 4 * c4) = hv[j];
            }
        }
    } else {

    // (0) gather the 16 ring rows -> LDS, zero beyond the batch / row; stream 0 keeps a copy.
    //     Issue order matters (vmcnt retires in order): ring slots first, then layer 1's
    //     weight stream (independent of the rows), then the dependent row loads.
    //     bf16: the rows come from the ring's bf16 copies (the replay push rounds them as the forward
    //     would: the same operands, half the gathered bytes, 16-byte pieces straight into the LDS tile);
    //     stream 0's fp32 copy for the weight gradient is those values widened (k_dw_bf16 rounds them
    //     to the same bf16 again).
    {
        const int kz = fwd_nch<BF>(a.in[0]) * (BF ? 32 : 16);   // columns multiplied
        constexpr int PW = BF ? 8 : 4;                            // elements per gather piece (16 bytes)
        const int qp = kz / PW;                                   // pieces per row
        const int rsp = BF ? (a.stride16 >> 3) : (a.ring_stride >> 2);   // pieces a ring row holds
        const int rs4 = a.ring_stride >> 2;
        // branch-free: every slot loads (clamped row / column) and selects zero afterwards,
        // so the loads issue back to back (one phys round trip, then one ring round trip)
        if (DQNX_FUSED_ORDER == 1) stream_open<MTN>(a.wblk[tgt][0], a.out[0] >> 4, fwd_nch<BF>(a.in[0]), coff >> 4, c, ws, wb, tile);
        int32_t slot[GQ];
#pragma unroll
        for (int j = 0; j < GQ; j++) {
            const int r = (tid + j * FT) / qp;
            slot[j] = a.phys[b0 + (r < nb ? r : nb - 1)];
        }
        // stream 0 also gathers the transition scalars for the head kernel (one contiguous
        // load there instead of a dependent phys -> ring chain)
        int32_t tslot = 0;
        const bool keep0 = keep && part == 0;   // one part writes the stream-0 copies
        if (keep0 && tid < nb) tslot = a.phys[b0 + tid];
        if (DQNX_FUSED_ORDER == 0) stream_open<MTN>(a.wblk[tgt][0], a.out[0] >> 4, fwd_nch<BF>(a.in[0]), coff >> 4, c, ws, wb, tile);
        u32x4 xv[GQ];
        const uint16_t* ring16 = BF ? ((s == 0) ? a.ring16_obs : a.ring16_next) : nullptr;
#pragma unroll
        for (int j = 0; j < GQ; j++) {
            const int q = tid + j * FT;
            const int r = q / qp, cp = q - r * qp;
            const bool ok = r < nb && cp < rsp;
            u32x4 x;
            if constexpr (BF)
                x = *reinterpret_cast<const u32x4*>(ring16 + (int64_t)slot[j] * a.stride16 + 8 * (ok ? cp : 0));
            else
                x = __builtin_bit_cast(u32x4, ld4(ring + (int64_t)slot[j] * a.ring_stride + 4 * (ok ? cp : 0)));
            if (!ok) x = u32x4{0u, 0u, 0u, 0u};
            xv[j] = x;
        }
        if (DQNX_FUSED_ORDER == 2) stream_open<MTN>(a.wblk[tgt][0], a.out[0] >> 4, fwd_nch<BF>(a.in[0]), coff >> 4, c, ws, wb, tile);
        // after the row loads are in flight: the transition scalars' own round trip overlaps them
        if (keep0 && tid < nb)
            a.trans[b0 + tid] = make_float4(__int_as_float(a.act[tslot]), a.rew[tslot], a.done[tslot], 0.f);
#pragma unroll
        for (int j = 0; j < GQ; j++) {
            const int q = tid + j * FT;
            const int r = q / qp, cp = q - r * qp;
            if (r < RW) {
                if constexpr (BF) {
                    *reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(FBUF(0)) + r * a.sx + 8 * cp) = xv[j];
                    if (keep0 && r < nb && cp < rsp) {   // widened: bf16 -> fp32 is exact
                        float* dst = a.xcopy + (int64_t)(b0 + r) * a.ring_stride + 8 * cp;
                        const u32x4 w = xv[j];
                        if (2 * cp < rs4)
                            *reinterpret_cast<float4*>(dst) = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                                                          __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
                        if (2 * cp + 1 < rs4)
                            *reinterpret_cast<float4*>(dst + 4) = make_float4(__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                                                                              __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u));
                    }
                } else {
                    *reinterpret_cast<float4*>(FBUF(0) + r * a.sx + 4 * cp) = __builtin_bit_cast(float4, xv[j]);
                    if (keep0 && r < nb && cp < rs4)
                        *reinterpret_cast<float4*>(a.xcopy + (int64_t)(b0 + r) * a.ring_stride + 4 * cp) =
                            __builtin_bit_cast(float4, xv[j]);
                }
            }
        }
    }
    }   // PH != 2
    if (PH != 2) DQNX_STAMP(a.stamps, 25);
    lds_barrier();
    if (PH != 2) DQNX_STAMP(a.stamps, 26);

    int cur = 0;
#pragma unroll
    for (int l = LB; l < LE; l++) {
        const int K = a.in[l], N = a.out[l];
        const float* bias_p = P + a.woff[l] + (int64_t)N * K + (l == 0 ? coff : 0);
        float bias[2];
#pragma unroll
        for (int t = 0; t < 2; t++) bias[t] = bias_p[(t < c.tn ? c.n0[t] : 0) + i];   // branch-free
        floatx4 acc[MR][2];
        wave_mma_rows<BF, MR, MTN>(FBUF(cur), l == 0 ? a.sx : a.sh, fwd_groups<BF>(K), c, ws, wb, acc);
        DQNX_STAMP(a.stamps, 27 + 2 * l);
        const WaveCols cl = c;
        // the paired forward's part 1 ends after layer 1: it publishes its H_1 half (below)
        const bool pub = PH == 3 && l == 0 && part == 1;
        // next layer's weight stream in flight during the epilogue + barrier
        if (l + 1 < LE && !pub) {
            c = wave_cols(a.out[l + 1]);
            stream_open<MTN>(a.wblk[tgt][l + 1], a.out[l + 1] >> 4, fwd_nch<BF>(a.in[l + 1]), 0, c, ws, wb, tile);
        }
        float* Hs = FBUF(cur ^ 1);
        // H to HBM: stream 0 (the backward's operands); the split layer 1 writes every stream's; the
        // paired forward's part 1 writes its half from the LDS tile, 16 bytes a lane (below)
        float* Hg = (PH == 1) ? a.H[0] + (int64_t)s * a.Bl * N : ((keep && !pub) ? a.H[l] : nullptr);
        // bf16 + DQNX_DWB_T=1 (k_dw_bf16d): stream 0's H_l also as a slab-transposed copy (4 consecutive samples per lane: 8 bytes)
        uint16_t* Ht = (BF && PH == 0 && keep) ? a.HT16[l] : nullptr;
#pragma unroll
        for (int t = 0; t < MTN; t++) {
            if (t >= cl.tn) continue;
            const int col = cl.n0[t] + i;
#pragma unroll
            for (int m = 0; m < MR; m++) {
                float vv[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int rr = 16 * m + 4 * g + r;
                    const float v = act_fwd<ACT>(acc[m][t][r] + bias[t]);
                    vv[r] = v;
                    if constexpr (PH != 1) {
                        if constexpr (BF) reinterpret_cast<uint16_t*>(Hs)[rr * a.sh + col] = bf16_bits(v);
                        else Hs[rr * a.sh + col] = v;
                    }
                    if (Hg && rr < nb) Hg[(int64_t)(b0 + rr) * N + coff + col] = v;
                }
                if (Ht && 16 * m + 4 * g < nb)   // (copies need whole 32-row blocks: nb % 32 == 0)
                    *reinterpret_cast<uint2*>(Ht + tcopy_index(b0 + 16 * m + 4 * g, col, N, a.tkb)) =
                        make_uint2(bf16_pack2(vv[0], vv[1]), bf16_pack2(vv[2], vv[3]));
            }
        }
        if constexpr (BF && PH == 0) {
            // stream 0's input rows as a slab-transposed copy, from the bf16 input tile (still in buffer 0 until
            // layer 2's epilogue), while layer 2's weight stream is in flight: 8 rows of a column per piece
            if (l == 0 && keep && a.xT16) {
                const int C = a.in[0];
                const uint16_t* xs = reinterpret_cast<const uint16_t*>(FBUF(0));
                for (int q = tid; q < 2 * MR * C; q += FT) {
                    const int ph = q / C, cc = q - ph * C;
                    if (8 * ph >= nb) continue;
                    const uint16_t* col = xs + 8 * ph * a.sx + cc;
                    uint32_t w[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) w[j] = (uint32_t)col[(2 * j) * a.sx] | ((uint32_t)col[(2 * j + 1) * a.sx] << 16);
                    *reinterpret_cast<uint4*>(a.xT16 + tcopy_index(b0 + 8 * ph, cc, C, a.tkb)) = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
        }
        if constexpr (PH == 1) return;
        if constexpr (PH == 3 && !BF) {
            if (l == 0) {
                // H_1 halves of the row tile: part 1 publishes (write-through sc1 16-byte stores of its LDS
                // half, every storing wave drained, then ONE lane's sc1 flag store behind a workgroup
                // barrier); part 0's polling lane matches the flag with sc1 loads, and after a barrier every
                // wave loads the half with sc1 loads into its tile (MI355X_MICROARCH.md, the measured
                // hand-off table's first row).  Stream 0's half is also the backward's H_1.
                uint32_t* flag = a.pair_flags + (z * a.tiles + tile);
                const int hw = N >> 1, q4 = hw >> 2;
                float* Hx = a.H[0] + (int64_t)s * a.Bl * N + (int64_t)b0 * N;   // [nb][N] of this stream
                const __amdgpu_buffer_rsrc_t xr = wave_rsrc(Hx, (uint32_t)nb * N * 4u);   // rows past nb: dropped / 0
                lds_barrier();
                if (pub) {
                    for (int q = tid; q < 16 * q4; q += FT) {
                        const int r = q / q4, c4 = q - r * q4;
                        const u32x4 v = *reinterpret_cast<const u32x4*>(Hs + r * a.sh + 4 * c4);
                        __builtin_amdgcn_raw_buffer_store_b128(v, xr, (uint32_t)(r * N + hw + 4 * c4) * 4u, 0, kCacheSC1);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    lds_barrier();
                    if (tid == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return;
                }
                if (tid == 0) {
                    int spins = 0;
                    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                        if (++spins > kPairSpinLimit) {   // (never expected: the partner is dispatched right behind)
                            if (a.err) __hip_atomic_store(a.err, (int32_t)DQNX_DEVERR_FWD_PAIR_HANDOFF, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // zero for the next launch
                }
                lds_barrier();
                for (int q = tid; q < 16 * q4; q += FT) {
                    const int r = q / q4, c4 = q - r * q4;
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, (uint32_t)(r * N + hw + 4 * c4) * 4u, 0, kCacheSC1);
                    *reinterpret_cast<u32x4*>(Hs + r * a.sh + hw + 4 * c4) = v;
                }
            }
        }
        lds_barrier();
        DQNX_STAMP(a.stamps, 28 + 2 * l);
        cur ^= 1;
    }

    // head: raw[o] = H_L . W_head[o] + b_head[o], o < NH; K = F split over the waves
    if constexpr (PH != 1) {
        const int F = a.F;
        const int A = a.head_kind == DQNX_HEAD_DUELING ? a.NH - 1 : a.NH;
        const float* hw = P + a.head_off + head_w_off(a.head_kind, i < a.NH ? i : 0, F);
        floatx4 acc[MR];
#pragma unroll
        for (int m = 0; m < MR; m++) acc[m] = floatx4{0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {   // head weights rounded to bf16 here (fp32 master copy)
            const uint16_t* hs = reinterpret_cast<const uint16_t*>(FBUF(cur)) + i * a.sh + 8 * g;
            for (int ck = wid; ck < (F >> 5); ck += FW) {
                const float4 w0 = ld4(hw + ck * 32 + 8 * g), w1 = ld4(hw + ck * 32 + 8 * g + 4);
                u32x4 wv = {bf16_pack2(w0.x, w0.y), bf16_pack2(w0.z, w0.w), bf16_pack2(w1.x, w1.y), bf16_pack2(w1.z, w1.w)};
                if (i >= a.NH) wv = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                for (int m = 0; m < MR; m++)
                    acc[m] = mfma16x16x32bf16(*reinterpret_cast<const u32x4*>(hs + 16 * m * a.sh + ck * 32), wv, acc[m]);
            }
        } else {
            const float* hs = FBUF(cur) + i * a.sh + 4 * g;
            for (int ck = wid; ck < (F >> 4); ck += FW) {
                float4 wv = ld4(hw + ck * 16 + 4 * g);
                if (i >= a.NH) wv = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int m = 0; m < MR; m++) {
                    const float4 av = *reinterpret_cast<const float4*>(hs + 16 * m * a.sh + ck * 16);
                    acc[m] = mfma16x16x4(av.x, wv.x, acc[m]);
                    acc[m] = mfma16x16x4(av.y, wv.y, acc[m]);
                    acc[m] = mfma16x16x4(av.z, wv.z, acc[m]);
                    acc[m] = mfma16x16x4(av.w, wv.w, acc[m]);
                }
            }
        }
        DQNX_STAMP(a.stamps, 36);
        float* part = FBUF(cur ^ 1);   // [FW][RW rows][16 outputs]
#pragma unroll
        for (int m = 0; m < MR; m++)
#pragma unroll
            for (int r = 0; r < 4; r++) part[(wid * RW + 16 * m + 4 * g + r) * 16 + i] = acc[m][r];
        float hb = 0.f;
        if ((tid & 15) < a.NH) hb = P[a.head_off + head_b_off(a.head_kind, tid & 15, F, A)];
        lds_barrier();
        for (int e = tid; e < RW * 16; e += FT) {   // FT is a multiple of 16: o == tid & 15
            const int b = e >> 4, o = e & 15;
            float v = part[b * 16 + o];
#pragma unroll
            for (int w = 1; w < FW; w++) v += part[(w * RW + b) * 16 + o];
            v = (o < a.NH) ? v + hb : 0.f;
            if (b < nb) a.raw[((int64_t)s * a.Bl + b0 + b) * 16 + o] = v;
        }
    }
    DQNX_STAMP(a.stamps, 37);
#undef FBUF
}

// =====================================================================================
// Head / TD / Huber / dZ chain for 16 samples.
// dZ_{l-1} = (dZ_l W_l) (.) act'(H_{l-1}): B[k][n] = W_l[k][n], read from the chain-blocked
// copy of W_l (relayout.hpp, kind 1).
// =====================================================================================
constexpr int HB_SD = 264;   // LDS row stride of fp32 dZ tiles (width <= 256)
constexpr int HB_SDH = 272;  // LDS row stride of bf16 dZ tiles (bf16 elements, 32 bytes mod 256)

// BF: the chain's dZ tiles are rounded to bf16 in LDS and multiplied by bf16 blocked weights
// (fp32 accumulate); dZ_L = dHead W_head (K = 16) and every global dZ stay fp32.
template <int ACT, int NL, bool BF>
__global__ __launch_bounds__(FT) void k_head_bwd(HeadBwdArgs a) {
    __shared__ __attribute__((aligned(16))) float dzs[2][16 * HB_SD];
    __shared__ float dh[16][17];
    __shared__ float lossv[16];
    const int tid = threadIdx.x, lane = tid & 63;
    const int i = lane & 15, g = lane >> 4;
    // nsplit workgroups per 16-sample tile: each recomputes the (cheap) head part and takes
    // 1/nsplit of the columns of the LAST dZ of the chain (dZ_1, the widest)
    int tile = blockIdx.x / a.nsplit, part = blockIdx.x - tile * a.nsplit;
    if (a.xcd_rows) {   // tile t on the XCD whose L2 holds the forward's outputs of its row tile t / xcd_mr
        const int xh = blockIdx.x & 7, k = blockIdx.x >> 3;
        const int kt = k / a.nsplit, mr = a.xcd_mr;
        tile = ((kt / mr) * 8 + ((xh - a.xcd_shift) & 7)) * mr + (kt - (kt / mr) * mr);
        part = k - kt * a.nsplit;
    }
    const bool lead = part == 0;
    const int b0 = tile * 16, nb = min(16, a.Bl - b0);
    const int A = a.A, NH = a.NH, F = a.F;
    constexpr int L = NL;
    const bool use1 = a.algo != DQNX_ALGO_DQN;
    const float* Wh = a.params + a.head_off;
    DQNX_STAMP(a.stamps, 40);

    // chain level l: dZ_{l-1}[16][cols] = dZ_l[16][K] . W_l[K][cols], cols = this part's range
    float4 wb[FNB][FPF][2];
    float hm[2][4];
    WStream ws;
    WaveCols cw;
    int coff = 0, ldn = 0;
    auto setup = [&](int l) {
        const int K = a.out[l], N = a.in[l];
        const int nparts = (l == 1) ? a.nsplit : 1;
        const int np_ = N / nparts;
        coff = (l == 1) ? part * np_ : 0;
        ldn = N;
        cw = wave_cols(np_);
        stream_open(a.wblkT[l], N >> 4, fwd_nch<BF>(K), coff >> 4, cw, ws, wb);
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                hm[t][r] = a.H[l - 1][(int64_t)(b0 + (4 * g + r < nb ? 4 * g + r : nb - 1)) * N + coff +
                                      (t < cw.tn ? cw.n0[t] : 0) + i];
    };
    // (0) every independent load first.  Head part: lane (b, j) = (tid >> 4, tid & 15) of
    //     waves 0-3 owns head slot j of sample b and reads its raw outputs straight into
    //     registers (coalesced rows); all waves: the head weights for dZ_L and H_L for its mask;
    //     then the first chain level's weight stream.  Branch-free clamped loads throughout.
    const int hb = tid >> 4, hj = tid & 15;
    const int hbc = hb < nb ? hb : nb - 1;
    float r0 = 0.f, r1 = 0.f, r2 = 0.f, wis = 1.f;
    float4 tr = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < 256) {
        const int64_t base = (int64_t)(b0 + hbc) * 16 + hj;
        r0 = a.raw[base];
        r1 = a.raw[(int64_t)a.Bl * 16 + base];   // online(s') (Double) / unused (DQN)
        r2 = a.raw[(int64_t)2 * a.Bl * 16 + base];
        tr = a.trans[b0 + hbc];
        if (a.isw) wis = a.isw[b0 + hbc];
    }
    const WaveCols cF = wave_cols(F);
    float whv[2][4], hmask[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int o = 4 * g + jj;
            // rows o >= NH meet dh == 0, samples >= nb are never stored, tiles >= tn unused
            const int col = (t < cF.tn ? cF.n0[t] : 0) + i;
            whv[t][jj] = Wh[head_w_off(a.head_kind, o < NH ? o : 0, F) + col];
            hmask[t][jj] = a.H[L - 1][(int64_t)(b0 + (4 * g + jj < nb ? 4 * g + jj : nb - 1)) * F + col];
        }
    if (L >= 2) setup(L - 1);
    DQNX_STAMP(a.stamps, 41);

    // (1) head part in registers, 16 lanes per sample, shuffles within the lane group:
    //     Q = V + (A - mean A) (R:dqn/network.py:83,90-96), Double-DQN argmax of online(s') /
    //     DQN max of target(s'), y = r + (1-d)*gamma*q' (R:dqn/agent.py:172-181, 209-216),
    //     SmoothL1 value / gradient (mean, or IS-weighted 'none' under PER, :259-267), dHead.
    if (tid < 256) {
        const bool duel = a.head_kind == DQNX_HEAD_DUELING;
        auto qval = [&](float r) {   // Q of this lane's action slot j (valid for j < A)
            if (!duel) return r;
            const float v = __shfl(r, 0, 16);
            const float adv = __shfl(r, hj + 1 < 16 ? hj + 1 : 15, 16);
            float sum = (hj >= 1 && hj <= A) ? r : 0.f;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) sum += __shfl_xor(sum, m, 16);
            const float mean = sum / (float)A;
            return v + (adv - mean);
        };
        const float q0 = qval(r0), q1 = qval(r1), q2 = qval(r2);
        float qn;
        if (!use1) {   // target(s').max(1)
            float mx = hj < A ? q2 : -INFINITY;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 16));
            qn = mx;
        } else {       // argmax online(s') (first maximum), gather target(s')
            float bv = hj < A ? q1 : -INFINITY;
            int bi = hj;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) {
                const float ov = __shfl_xor(bv, m, 16);
                const int oi = __shfl_xor(bi, m, 16);
                if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
            }
            qn = __shfl(q2, bi, 16);
        }
        int act = __float_as_int(tr.x);
        if (act < 0 || act >= A) act = 0;
        const float rew = tr.y, done = tr.z;
        const float t1 = 1.f - done;
        const float t2 = t1 * a.gamma;
        const float t3 = t2 * qn;
        const float y = rew + t3;
        const float qa = __shfl(q0, act, 16);
        const float x = qa - y;                        // smooth_l1: input - target
        const float zabs = fabsf(x);
        const float l = zabs < 1.f ? (0.5f * zabs) * zabs / 1.f : zabs - 0.5f;
        float gq, lb;
        if (a.isw) {
            const float go = a.inv_bg * wis;
            gq = x <= -1.f ? -go : (x >= 1.f ? go : (x * go) / 1.f);
            lb = wis * l;
        } else {
            gq = x <= -1.f ? -a.inv_bg : (x >= 1.f ? a.inv_bg : (a.inv_bg * x) / 1.f);
            lb = l;
        }
        const float gmean = (-gq) / (float)A;
        float d = 0.f;
        if (hj < NH) {
            if (duel) d = (hj == 0) ? gq : ((hj - 1 == act ? gq : 0.f) + gmean);
            else d = (hj == act) ? gq : 0.f;
        }
        const bool real = hb < nb;
        if (!real) { d = 0.f; lb = 0.f; }
        dh[hb][hj] = d;
        if (hj == 0) lossv[hb] = lb;
        if (lead && real) {
            const int64_t qrow = (int64_t)(b0 + hb) * A + hj;
            if (hj < A) {
                a.Q[qrow] = q0;
                if (use1) a.Q[(int64_t)a.Bl * A + qrow] = q1;
                a.Q[(int64_t)2 * a.Bl * A + qrow] = q2;
            }
            a.dhead[(int64_t)(b0 + hb) * 16 + hj] = d;
            if (a.dheadT16) a.dheadT16[tcopy_index(b0 + hb, hj, 16, a.tkb)] = bf16_bits(d);
            if (hj == 0) {
                const int gb = b0 + hb;
                a.td[gb] = y;
                a.td[a.Bl + gb] = qa;
                a.td[2 * a.Bl + gb] = zabs;
                if (a.abs_td_out) a.abs_td_out[gb] = zabs;
                if (a.pp_on) per_prep_item(a.pp, gb, zabs);   // SumTree.update bookkeeping of this sample
            }
        }
    }
    if (blockIdx.x == 0 && tid == 320 && a.ctrl) adam_advance(a.ctrl, a.ab);
    lds_barrier();
    DQNX_STAMP(a.stamps, 44);
    if (lead && tid == 256) {   // loss partial of the tile, sample order
        float sacc = 0.f;
        for (int b = 0; b < 16; b++) sacc += lossv[b];
        a.loss_partial[tile] = sacc;
    }

    // (4) dZ_L = (dHead W_head) (.) act'(H_L): K = 16 head rows, one MFMA group per tile
    int cur = 0;
    {
        float* dz = dzs[cur];
        float* dzg = a.dZ[L - 1];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            if (t >= cF.tn) continue;
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int jj = 0; jj < 4; jj++) acc = mfma16x16x4(dh[i][4 * g + jj], whv[t][jj], acc);
            const int col = cF.n0[t] + i;
            float vv[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int rr = 4 * g + r;
                const float v = act_bwd<ACT>(acc[r], hmask[t][r]);
                vv[r] = v;
                if constexpr (BF) reinterpret_cast<uint16_t*>(dz)[rr * HB_SDH + col] = bf16_bits(v);
                else dz[rr * HB_SD + col] = v;
                if (lead && rr < nb) dzg[(int64_t)(b0 + rr) * F + col] = v;
            }
            if (lead && a.dZT16[L - 1] && 4 * g < nb)   // slab-transposed copy for k_dw_bf16d
                *reinterpret_cast<uint2*>(a.dZT16[L - 1] + tcopy_index(b0 + 4 * g, col, F, a.tkb)) =
                    make_uint2(bf16_pack2(vv[0], vv[1]), bf16_pack2(vv[2], vv[3]));
        }
    }

    DQNX_STAMP(a.stamps, 45);
    // (5) dZ chain down to layer 1
#pragma unroll
    for (int l = L - 1; l >= 1; l--) {
        if (l < L - 1) setup(l);
        floatx4 acc[2];
        lds_barrier();   // dZ_l tile complete in LDS
        DQNX_STAMP(a.stamps, 46 + 3 * (L - 1 - l));
        wave_mma<BF>(dzs[cur], BF ? HB_SDH : HB_SD, fwd_groups<BF>(a.out[l]), cw, ws, wb, acc);
        DQNX_STAMP(a.stamps, 47 + 3 * (L - 1 - l));
        float* dz = dzs[cur ^ 1];
        float* dzg = a.dZ[l - 1];
        const bool store = lead || l == 1;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            if (t >= cw.tn) continue;
            const int col = cw.n0[t] + i;
            float vv[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int rr = 4 * g + r;
                const float v = act_bwd<ACT>(acc[t][r], hm[t][r]);
                vv[r] = v;
                if (l > 1) {   // the last level's tile feeds nothing
                    if constexpr (BF) reinterpret_cast<uint16_t*>(dz)[rr * HB_SDH + col] = bf16_bits(v);
                    else dz[rr * HB_SD + col] = v;
                }
                if (store && rr < nb) dzg[(int64_t)(b0 + rr) * ldn + coff + col] = v;
            }
            if (store && a.dZT16[l - 1] && 4 * g < nb)
                *reinterpret_cast<uint2*>(a.dZT16[l - 1] + tcopy_index(b0 + 4 * g, coff + col, ldn, a.tkb)) =
                    make_uint2(bf16_pack2(vv[0], vv[1]), bf16_pack2(vv[2], vv[3]));
        }
        cur ^= 1;
    }
    DQNX_STAMP(a.stamps, 55);
}

// =====================================================================================
// Weight gradients in bf16 (DQNX_COMPUTE_BF16): partial[slice] = bf16(dZ)^T [bf16(X) | 1],
// fp32 accumulate, the same split-K slabs and flat layouts as k_bwd_level (the Adam pass is
// shared).  32 x 32 or 64 x 64 output tiles, 4 waves, K (samples) in passes of KT.  Operands are read as fp32 rows [k][cols], rounded, and stored TRANSPOSED in LDS
// ([col][k], k contiguous) so an MFMA fragment (8 consecutive k of one column) is one
// ds_read_b128; a column stride of KT/2 + 4 dwords makes those reads and the paired-k stores
// conflict-free.
// =====================================================================================
#ifndef DQNX_DWB_KT64
// samples per pass of the 64 x 64 tiles (configs[4]: 512-sample split-K slices).  Measured round 6,
// B = 8192 PER bf16 (gpurun_out r06g): 32 -> dw_all 29.1 us, 64 -> 26.6, 128 -> 36.0 (2 waves / SIMD),
// 64 with two passes in flight 28.2; the chunks still accumulate in k order (bitwise the same sums)
#define DQNX_DWB_KT64 64
#endif
#ifndef DQNX_DWB_PIPE
#define DQNX_DWB_PIPE 0   // 1: two passes in flight, two LDS buffers (measured equal: 27.7 vs 26.4 us at B=8192)
#endif
#ifndef DQNX_DWB_KT32
#define DQNX_DWB_KT32 128
#endif
// LDS column stride in dwords (2 bf16 each) for KT samples per pass: KT/2 + 4, i.e. 4 mod 16
// dwords (b128 fragment reads of 16 consecutive columns hit distinct banks).
template <int KT>
struct DwbShape {
    static constexpr int SD = KT / 2 + 4;
    static constexpr int KP = KT / 2;   // k pairs per pass
};

// rows [k0, k0 + KT) x cols [c0, c0 + BT) of a [K][ld] operand; pair index q = (column group of
// 4) * KP + k pair, q = tid + 256 u.  Column j reads 0 past `ncols`, or 1.0 at j == aug.
template <int BT, int KT>
struct DwbStage {
    static constexpr int KP = KT / 2, NQ = KP * (BT / 4), NU = NQ / 256 > 0 ? NQ / 256 : 1;
};
template <int BT, int KT>
__device__ __forceinline__ void dwb_stage(const float* base, int ld, int ncols, int aug, int c0, int k0, int kend,
                                          float4 (&v)[DwbStage<BT, KT>::NU][2]) {
    constexpr int KP = DwbStage<BT, KT>::KP, NQ = DwbStage<BT, KT>::NQ, NU = DwbStage<BT, KT>::NU;
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int q = threadIdx.x + 256 * u;
        const int kp = q % KP, cg = q / KP;
        const int c = c0 + 4 * cg;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int k = k0 + 2 * kp + h;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < NQ && k < kend) {
                const float* row = base + (int64_t)k * ld;
                if (c + 3 < ncols) {
                    x = ld4(row + c);
                } else if ((c <= aug && aug < c + 4) || c < ncols) {   // the group holding the edge
                    float e[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) e[j] = (c + j < ncols) ? row[c + j] : (c + j == aug ? 1.f : 0.f);
                    x = make_float4(e[0], e[1], e[2], e[3]);
                }
            }
            v[u][h] = x;
        }
    }
}
template <int BT, int KT>
__device__ __forceinline__ void dwb_store(uint32_t* dst, const float4 (&v)[DwbStage<BT, KT>::NU][2]) {
    constexpr int KP = DwbStage<BT, KT>::KP, SD = DwbShape<KT>::SD, NQ = DwbStage<BT, KT>::NQ,
                  NU = DwbStage<BT, KT>::NU;
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int q = threadIdx.x + 256 * u;
        if (q >= NQ) continue;
        const int kp = q % KP, cg = q / KP;
        uint32_t* p = dst + (4 * cg) * SD + kp;
        p[0 * SD] = bf16_pack2(v[u][0].x, v[u][1].x);
        p[1 * SD] = bf16_pack2(v[u][0].y, v[u][1].y);
        p[2 * SD] = bf16_pack2(v[u][0].z, v[u][1].z);
        p[3 * SD] = bf16_pack2(v[u][0].w, v[u][1].w);
    }
}

// BM x BN output tile (rows = dZ columns, cols = X columns + the ones column), 4 waves in a 2 x 2
// grid of (BM/2) x (BN/2) wave tiles of 16x16 MFMA tiles, KT samples per pass.  Larger tiles read
// fewer operand bytes per MFMA: 64 x 64 moves 16 KiB of fp32 rows per 4 MFMAs a wave, 128 x 128
// 32 KiB per 16 (configs[4]: 8192 samples, 32 split-K slices).
template <int BM, int BN>
constexpr int dwb_waves() {
    return BM * BN >= 128 * 128 ? 2 : BM * BN >= 128 * 64 ? 3 : (DQNX_DWB_PIPE ? 4 : DQNX_DWB_WAVES);
}
template <int BM, int BN, int KT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(dwb_waves<BM, BN>()))) void k_dw_bf16(BwdArgs a) {
    static_assert((BM == 32 || BM == 64 || BM == 128) && (BN == 32 || BN == 64 || BN == 128), "tile");
    static_assert(KT % 32 == 0, "whole MFMA chunks");
    constexpr int TM = BM / 32, TN = BN / 32, SD = DwbShape<KT>::SD;
    constexpr int NUA = DwbStage<BM, KT>::NU, NUB = DwbStage<BN, KT>::NU;
    static_assert((KT / 2) * (BM / 4) <= 256 * NUA && (KT / 2) * (BN / 4) <= 256 * NUB, "pairs per thread");
    constexpr int NB = DQNX_DWB_PIPE ? 2 : 1;   // LDS pass buffers
    __shared__ __attribute__((aligned(16))) uint32_t lds[NB * (BM + BN) * SD];
    uint32_t* la = lds;            // dZ columns (rows m of the gradient tile)
    uint32_t* lb = lds + BM * SD;  // X columns (+ ones)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int wm = wid >> 1, wn = wid & 1;
    if (a.ptrack && blockIdx.x == 0) {   // k_per_update's tracking (single-GPU PER step; dispatched
        // first so it starts under any grid size; its prop workgroups run in the Adam launch)
        static_assert(sizeof(lds) >= sizeof(PerTrackLds<256>), "tracking scratch");
        auto& tl = *reinterpret_cast<PerTrackLds<256>*>(lds);
        per_track_block<256, DQNX_BF16_TRACK_IPT, DQNX_BF16_TRACK_CARRY>(a.pprop, tl);
        return;
    }
    int b = (int)blockIdx.x - a.ptrack;
    {   // workgroups past the tiles: k_per_prop's (single-GPU PER step; independent of the gradients)
        int tiles = 0;
        for (int p = 0; p < a.ndw; p++) tiles += a.dw[p].blocks;
        if (b >= tiles) {
            if constexpr (sizeof(lds) >= PER_TOP * sizeof(double)) {
                per_prop_block(a.pprop, (b - tiles) * 256, reinterpret_cast<double*>(lds));
            } else {
                __shared__ double topd[PER_TOP];
                per_prop_block(a.pprop, (b - tiles) * 256, topd);
            }
            return;
        }
    }
    int p = 0;
    while (p + 1 < a.ndw && b >= a.dw[p].blocks) { b -= a.dw[p].blocks; p++; }
    const DwProblem& d = a.dw[p];
    b = xcd_remap(b, d.blocks);
    const int bx = b % d.grid_x;
    const int t2 = b / d.grid_x;
    const int by = t2 % d.grid_y, bz = t2 / d.grid_y;
    const int m0 = by * BM, n0 = bx * BN;
    const int kb = bz * a.kslice;
    const int ke = min(a.Bl, kb + a.kslice);
    floatx4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
        for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int ncz = d.out < d.ldz ? d.out : d.ldz;   // dZ columns that exist (head: ldz 16 >= NH)
    auto mma_pass = [&](const uint32_t* pa, const uint32_t* pb) {
#pragma unroll
        for (int ch = 0; ch < KT / 32; ch++) {
            u32x4 fa[TM], fb[TN];
#pragma unroll
            for (int t = 0; t < TM; t++)
                fa[t] = *reinterpret_cast<const u32x4*>(pa + (wm * 16 * TM + t * 16 + i) * SD + 16 * ch + 4 * g);
#pragma unroll
            for (int t = 0; t < TN; t++)
                fb[t] = *reinterpret_cast<const u32x4*>(pb + (wn * 16 * TN + t * 16 + i) * SD + 16 * ch + 4 * g);
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int tn = 0; tn < TN; tn++) acc[tm][tn] = mfma16x16x32bf16(fa[tm], fb[tn], acc[tm][tn]);
        }
    };
    float4 va[NUA][2], vb[NUB][2];
    dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, kb, ke, va);
    dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, kb, ke, vb);
    if constexpr (DQNX_DWB_PIPE) {
        // two passes in flight in registers, two LDS buffers, one barrier per pass: while pass p's
        // fragments are multiplied out of buffer p & 1, pass p+1 goes into the other buffer and
        // pass p+2's rows are loading
        uint32_t* la1 = lds + (BM + BN) * SD;
        uint32_t* lb1 = la1 + BM * SD;
        float4 wa[NUA][2], wb2[NUB][2];
        dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, kb + KT, ke, wa);
        dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, kb + KT, ke, wb2);
        dwb_store<BM, KT>(la, va);
        dwb_store<BN, KT>(lb, vb);
        dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, kb + 2 * KT, ke, va);
        dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, kb + 2 * KT, ke, vb);
        __syncthreads();
        for (int k0 = kb; k0 < ke; k0 += 2 * KT) {
            mma_pass(la, lb);                                // pass k0 (buffer 0)
            if (k0 + KT >= ke) break;
            dwb_store<BM, KT>(la1, wa);                      // pass k0 + KT -> buffer 1
            dwb_store<BN, KT>(lb1, wb2);
            dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, k0 + 3 * KT, ke, wa);
            dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, k0 + 3 * KT, ke, wb2);
            __syncthreads();
            mma_pass(la1, lb1);                              // pass k0 + KT (buffer 1)
            if (k0 + 2 * KT >= ke) break;
            // buffer 0's readers (pass k0) all passed the barrier above
            dwb_store<BM, KT>(la, va);                       // pass k0 + 2 KT -> buffer 0
            dwb_store<BN, KT>(lb, vb);
            dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, k0 + 4 * KT, ke, va);
            dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, k0 + 4 * KT, ke, vb);
            __syncthreads();
        }
    } else {
        for (int k0 = kb; k0 < ke; k0 += KT) {
            __syncthreads();   // previous pass's fragments read
            dwb_store<BM, KT>(la, va);
            dwb_store<BN, KT>(lb, vb);
            __syncthreads();
            if (k0 + KT < ke) {   // next pass in flight during this one's MFMAs
                dwb_stage<BM, KT>(d.dZ, d.ldz, ncz, -1, m0, k0 + KT, ke, va);
                dwb_stage<BN, KT>(d.X, d.ldx, d.in, d.in, n0, k0 + KT, ke, vb);
            }
            mma_pass(la, lb);
        }
    }
    // rows beyond `out` / columns beyond `in` (+1) of the tile are not stored
    float* part = d.partial + (int64_t)bz * d.pstride;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + wn * 16 * TN + tn * 16 + i;
        if (col > d.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wm * 16 * TM + tm * 16 + 4 * g + r;
                if (row >= d.out) continue;
                int64_t o;
                if (d.head_kind < 0) o = (col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row;
                else o = (col < d.in) ? head_w_off(d.head_kind, row, d.in) + col : head_b_off(d.head_kind, row, d.in, d.A);
                part[o] = acc[tm][tn][r];
            }
    }
}

// Opt-in (DQNX_DWB_T=1): the same weight gradients from slab-transposed bf16 copies that the forward
// (stream 0's rows and activations) and the head kernel (dZ_l, dHead) write beside their fp32 outputs,
// the MFMA fragments loaded straight into registers (no LDS, no barrier): lane (i, g) of a wave fetches
// samples 32 ch + 8 g .. + 7 of its tile row / column i as one 16-byte load, DWT_STAGES chunks ahead of
// the MFMAs that use them.  The fragments, their k order and the slabs are k_dw_bf16's (bitwise equal,
// test_gpu_bf16_t16_dw_bit_identical).  Measured at configs[4] (rocprofv3, profiles/r05/): 30.2 us
// against k_dw_bf16's 28.1, and the copies cost the forward 3.3 us and the head 1.8; an LDS-DMA variant
// (every operand row of a slice staged by global_load_lds at once) took 45-48 us.  Block 0's stamps
// (tools/stamps_dw.py): ~7.5 K cycles per 4 chunks of 16-byte loads, i.e. ~3 us per round trip while
// all 528 tiles load at once -- the launch is bound by the memory system's queueing, not by how a tile
// stages its operands, so k_dw_bf16 stays the default.
#ifndef DQNX_DWT_STAGES
#define DQNX_DWT_STAGES 4
#endif
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_dw_bf16d(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dlds[];   // (PER tracking / prop scratch only)
    constexpr int TM = BM / 32, TN = BN / 32, NS = DQNX_DWT_STAGES;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int wm = wid >> 1, wn = wid & 1;
    if (a.ptrack && blockIdx.x == 0) {
        auto& tl = *reinterpret_cast<PerTrackLds<256>*>(dlds);
        per_track_block<256, DQNX_BF16_TRACK_IPT, DQNX_BF16_TRACK_CARRY>(a.pprop, tl);
        return;
    }
    int b = (int)blockIdx.x - a.ptrack;
    {
        int tiles = 0;
        for (int p = 0; p < a.ndw; p++) tiles += a.dw[p].blocks;
        if (b >= tiles) {
            per_prop_block(a.pprop, (b - tiles) * 256, reinterpret_cast<double*>(dlds));
            return;
        }
    }
    int p = 0;
    while (p + 1 < a.ndw && b >= a.dw[p].blocks) { b -= a.dw[p].blocks; p++; }
    const DwProblem& d = a.dw[p];
    DQNX_STAMP(a.stamps, 57);
    b = xcd_remap(b, d.blocks);
    const int bx = b % d.grid_x;
    const int t2 = b / d.grid_x;
    const int by = t2 % d.grid_y, bz = t2 / d.grid_y;
    const int m0 = by * BM, n0 = bx * BN;
    const int kb = bz * a.kslice;
    const int ke = min(a.Bl, kb + a.kslice);
    const int KB = a.kslice;
    const int ncz = d.out < d.cz ? d.out : d.cz;
    // this lane's TM dZ columns and TN X columns; missing ones read a valid address and are replaced
    const uint16_t* ap[TM];
    const uint16_t* bp[TN];
    uint32_t afill[TM], bfill[TN];   // 0: load; else the constant bf16 pair to use (zero: 1, ones: 0x3F803F80)
#pragma unroll
    for (int t = 0; t < TM; t++) {
        const int c = m0 + wm * 16 * TM + t * 16 + i;
        const bool have = c < ncz;
        ap[t] = d.dZT + tcopy_index(kb, have ? c : 0, d.cz, KB) + 8 * g;
        afill[t] = have ? 0u : 1u;
    }
#pragma unroll
    for (int t = 0; t < TN; t++) {
        const int c = n0 + wn * 16 * TN + t * 16 + i;
        const bool have = c < d.in;
        bp[t] = d.XT + tcopy_index(kb, have ? c : 0, d.cx, KB) + 8 * g;
        bfill[t] = have ? 0u : (c == d.in ? 0x3F803F80u : 1u);
    }
    floatx4 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
        for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int nch = (ke - kb) >> 5;
    u32x4 fa[NS][TM], fb[NS][TN];
    auto fetch = [&](int ch, u32x4 (&xa)[TM], u32x4 (&xb)[TN]) {
        const int cc = ch < nch ? ch : nch - 1;   // (clamped: past the last chunk a valid, unused load)
#pragma unroll
        for (int t = 0; t < TM; t++) xa[t] = *reinterpret_cast<const u32x4*>(ap[t] + 32 * cc);
#pragma unroll
        for (int t = 0; t < TN; t++) xb[t] = *reinterpret_cast<const u32x4*>(bp[t] + 32 * cc);
    };
#pragma unroll
    for (int st = 0; st < NS - 1; st++) fetch(st, fa[st], fb[st]);
    for (int c0 = 0; c0 < nch; c0 += NS) {
#pragma unroll
        for (int st = 0; st < NS; st++) {
            const int ch = c0 + st;
            fetch(ch + NS - 1, fa[(st + NS - 1) % NS], fb[(st + NS - 1) % NS]);
            __builtin_amdgcn_sched_barrier(0);
            if (ch < nch) {
                u32x4 xa[TM], xb[TN];
#pragma unroll
                for (int t = 0; t < TM; t++) {
                    const uint32_t f = afill[t] == 1u ? 0u : afill[t];
                    xa[t] = afill[t] ? u32x4{f, f, f, f} : fa[st][t];
                }
#pragma unroll
                for (int t = 0; t < TN; t++) {
                    const uint32_t f = bfill[t] == 1u ? 0u : bfill[t];
                    xb[t] = bfill[t] ? u32x4{f, f, f, f} : fb[st][t];
                }
#pragma unroll
                for (int tm = 0; tm < TM; tm++)
#pragma unroll
                    for (int tn = 0; tn < TN; tn++) acc[tm][tn] = mfma16x16x32bf16(xa[tm], xb[tn], acc[tm][tn]);
            }
        }
        if (c0 == 0) DQNX_STAMP(a.stamps, 58);
    }
    DQNX_STAMP(a.stamps, 59);
    float* part = d.partial + (int64_t)bz * d.pstride;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + wn * 16 * TN + tn * 16 + i;
        if (col > d.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + wm * 16 * TM + tm * 16 + 4 * g + r;
                if (row >= d.out) continue;
                int64_t o;
                if (d.head_kind < 0) o = (col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row;
                else o = (col < d.in) ? head_w_off(d.head_kind, row, d.in) + col : head_b_off(d.head_kind, row, d.in, d.A);
                part[o] = acc[tm][tn][r];
            }
    }
#ifdef DQNX_STAMPS
    DQNX_STAMP(a.stamps, 60);
    if (a.stamps && threadIdx.x == 0) {   // the last workgroup's end, and how many workgroups ran
        atomicMax(reinterpret_cast<unsigned long long*>(a.stamps + 61), (unsigned long long)__builtin_amdgcn_s_memtime());
        atomicAdd(reinterpret_cast<unsigned long long*>(a.stamps + 62), 1ull);
    }
#endif
}

// Tile shape (BM x BN): 64 x 64 when that still gives >= 512 workgroups (large batches: fewer operand
// re-reads), else 32 x 32 (B=1024: 132 workgroups of 64 x 64 left the chip idle).  DQNX_DWB_SHAPE
// (tuning builds): 1 = 32 x 32, 2 = 64 x 64, 3 = 128 x 128, 4 = 128 x 64.
struct DwbTile { int bm, bn; };
static DwbTile dw_bf16_tile(const BwdArgs& a) {
    static const int shape = tuning_knob("DQNX_DWB_SHAPE", 0);
    if (shape == 1) return {32, 32};
    if (shape == 2) return {64, 64};
    if (shape == 3) return {128, 128};
    if (shape == 4) return {128, 64};
    int n64 = 0;
    for (int p = 0; p < a.ndw; p++)
        n64 += ((a.dw[p].in + 1 + 63) / 64) * ((a.dw[p].out + 63) / 64) * a.dw_slices;
    return n64 >= 512 ? DwbTile{64, 64} : DwbTile{32, 32};
}

void dw_bf16_grid(BwdArgs& a) {
    const DwbTile t = dw_bf16_tile(a);
    for (int p = 0; p < a.ndw; p++) {
        DwProblem& d = a.dw[p];
        d.grid_x = (d.in + 1 + t.bn - 1) / t.bn;
        d.grid_y = (d.out + t.bm - 1) / t.bm;
        d.blocks = d.grid_x * d.grid_y * a.dw_slices;
    }
}

bool dw_bf16t_supported(const BwdArgs& a) {
    const DwbTile t = dw_bf16_tile(a);
    return a.kslice % 32 == 0 && a.Bl % 32 == 0 && ((t.bm == 64 && t.bn == 64) || (t.bm == 32 && t.bn == 32));
}

int launch_dw_bf16(const BwdArgs& a, hipStream_t s) {
    int blocks = a.pprop_wgs + a.ptrack;   // (+ k_per_prop's workgroups: 256 updates each, after the
                                            // tiles; + the tracking workgroup, block 0)
    if (a.ptrack && a.pprop.n > PER_CHUNK) return set_error(DQNX_EINVAL, "dw_bf16: PER tracking chunk %d", a.pprop.n);
    for (int p = 0; p < a.ndw; p++) blocks += a.dw[p].blocks;
    if (a.t16) {
        const DwbTile t = dw_bf16_tile(a);
        if (a.kslice % 32 || a.Bl % 32)
            return set_error(DQNX_EUNSUPPORTED, "dw_bf16d: slices / batch a multiple of 32 samples");
        for (int p = 0; p < a.ndw; p++)
            if (!a.dw[p].dZT || !a.dw[p].XT) return set_error(DQNX_EINVAL, "dw_bf16d: copy operand missing");
        // (the attribute only past 64 KB, and exactly the bytes requested: a failed hipFuncSetAttribute
        // -- static LDS + a 160 KB maximum -- would be the launch's hipGetLastError)
        const size_t shd = sizeof(PerTrackLds<256>) > PER_TOP * sizeof(double) ? sizeof(PerTrackLds<256>) : PER_TOP * sizeof(double);
        if (t.bm == 64 && t.bn == 64) DQNX_LAUNCH((k_dw_bf16d<64, 64>), dim3(blocks), dim3(256), shd, s, a);
        else if (t.bm == 32 && t.bn == 32) DQNX_LAUNCH((k_dw_bf16d<32, 32>), dim3(blocks), dim3(256), shd, s, a);
        else return set_error(DQNX_EUNSUPPORTED, "dw_bf16d: %dx%d tiles", t.bm, t.bn);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    for (int p = 0; p < a.ndw; p++)   // 16-byte row loads
        if (a.dw[p].ldx % 4 || a.dw[p].ldz % 4)
            return set_error(DQNX_EUNSUPPORTED, "bf16 weight gradients need row strides that are multiples of 4");
    // measured: 64 x 64 tiles best with 32-sample passes (64: +1.7 us, 128: +6 us at B=8192);
    // 32 x 32 tiles with 128-sample passes (the fp32 kernel's depth)
    const DwbTile t = dw_bf16_tile(a);
    if (t.bm == 128 && t.bn == 128) DQNX_LAUNCH((k_dw_bf16<128, 128, 32>), dim3(blocks), dim3(256), 0, s, a);
    else if (t.bm == 128) DQNX_LAUNCH((k_dw_bf16<128, 64, 32>), dim3(blocks), dim3(256), 0, s, a);
    else if (t.bm == 64) DQNX_LAUNCH((k_dw_bf16<64, 64, DQNX_DWB_KT64>), dim3(blocks), dim3(256), 0, s, a);
    else DQNX_LAUNCH((k_dw_bf16<32, 32, DQNX_DWB_KT32>), dim3(blocks), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// ---- host side ------------------------------------------------------------------------
bool fused_fwd_plan(FusedFwdArgs& a, int obs_dim, bool bf16, int mr) {
    if (mr != 1 && mr != 2 && mr != 4) return false;
    if (a.L < 1 || a.L > FUSED_MAX_L || a.NH > 16) return false;
    for (int l = 0; l < a.L; l++)
        if (a.out[l] % 64 || a.out[l] > 256) return false;
    if (a.F != a.out[a.L - 1]) return false;
    a.bf16 = bf16 ? 1 : 0;
    const int kz = bf16 ? fwd_nch<true>(obs_dim) * 32 : fwd_nch<false>(obs_dim) * 16;
    if (16 * (kz / 4) > FGQ * FT) return false;   // gather slots (per 16 rows)
    a.gw = kz / 4 <= FWD_NARROW_Q4 ? 0 : 1;
    if (a.gw && mr != 1) return false;   // wide rows: 16-row tiles only
    const int rw = 16 * mr;
    a.mr = mr;
    int wmax = 0;
    for (int l = 0; l < a.L; l++) wmax = a.out[l] > wmax ? a.out[l] : wmax;
    int t0, t1;   // tile sizes in floats
    if (bf16) {   // stride = an odd multiple of 32 bytes mod 256 (conflict-free b128 fragment reads)
        // 16-row tiles read the A fragments of a whole group before skipping the chunks past nch, so
        // their rows cover the last group; MR > 1 stops at nch (bf16 MLP-284 at MR = 4: 86 -> 74 KB
        // of LDS, two workgroups per CU)
        a.sx = (mr == 1 ? fwd_groups<true>(obs_dim) * FPF : fwd_nch<true>(obs_dim)) * 32 + 16;
        a.sh = ((wmax + 127) & ~127) + 16;
        t0 = rw * a.sx / 2;
        t1 = rw * a.sh / 2;
    } else {
        a.sx = fused_stride(kz);
        a.sh = fused_stride(wmax);
        t0 = rw * a.sx;
        t1 = rw * a.sh;
    }
    int b0 = t0 > t1 ? t0 : t1, b1 = t1;
    if (b0 < FW * rw * 16) b0 = FW * rw * 16;   // head partials [FW][rw][16]
    if (b1 < FW * rw * 16) b1 = FW * rw * 16;
    a.buf0 = (b0 + 3) & ~3;
    a.buf1 = (b1 + 3) & ~3;
    for (int l = 0; l < a.L; l++) a.kpad[l] = bf16 ? fwd_nch<true>(a.in[l]) * 32 : fwd_nch<false>(a.in[l]) * 16;
    return (a.buf0 + a.buf1) * 4 <= (mr == 1 ? 64 : 160) * 1024;
}

int fused_wblk_bytes(bool bf16, int rows, int kpad) { return rows * kpad * (bf16 ? 2 : 4); }

// Occupancy: a workgroup streams every weight of its stream at the MFMA rate of ONE CU, so two
// workgroups sharing a CU (the dispatcher packs up to 4 of these onto one CU while others sit
// idle: 192 workgroups at B = 1024 on 256 CUs) double that CU's time and set the kernel's tail.
// DQNX_FUSED_LDS_MIN pads the LDS request so only one fits per CU.
#ifndef DQNX_FUSED_LDS_MIN
#define DQNX_FUSED_LDS_MIN 0
#endif
#ifndef DQNX_HEAD_LDS_PAD
#define DQNX_HEAD_LDS_PAD 0
#endif

int launch_fused_fwd(const FusedFwdArgs& a, int act, hipStream_t s) {
    if (a.phase != 0 && (a.L < 2 || a.mr != (a.phase == 1 ? a.mr : 1) ||
                         (a.phase == 1 && (a.csplit < 1 || a.out[0] % (16 * a.csplit)))))
        return set_error(DQNX_EUNSUPPORTED, "split forward: L >= 2, 16-row tiles (layer 1: 16, 32 or 64), layer 1 width / parts a multiple of 16");
    bool pair_ok = a.L >= 2 && a.mr == 1 && !a.bf16 && !a.gw && a.xcd_rows && a.tiles % 8 == 0 && a.out[0] % 32 == 0 &&
                   a.out[0] <= 32 * FW && a.pair_flags;
    for (int l = 1; l < a.L; l++) pair_ok = pair_ok && a.out[l] <= 16 * FW;   // one column tile per wave
    if (a.phase == 3 && !pair_ok)
        return set_error(DQNX_EUNSUPPORTED, "paired forward: fp32, L >= 2, 16-row tiles, tiles %% 8 == 0, layer 1 width a "
                                            "multiple of 32 and <= %d, later layers <= %d wide", 32 * FW, 16 * FW);
    if (a.gw && (a.phase != 0 || a.mr != 1))
        return set_error(DQNX_EUNSUPPORTED, "fused forward: rows wider than %d columns take the one-launch 16-row plan", 4 * FWD_NARROW_Q4);
    if (a.samp_shape && (a.phase == 2 || a.samp_shape > 3 || a.samp.k > FWD_SAMPLE_MAX_K ||
                         (a.samp_shape == 1 && a.samp.k > 2048)))
        return set_error(DQNX_EUNSUPPORTED, "forward sampler workgroup: whole forward or layer-1 launch, k <= %d", FWD_SAMPLE_MAX_K);
    if (a.bf16 && a.phase != 2 && (!a.ring16_obs || !a.ring16_next || a.stride16 % 8 || a.stride16 < a.in[0]))
        return set_error(DQNX_EUNSUPPORTED, "bf16 forward: needs the ring's bf16 copies (16-byte rows)");
    if (a.npc && (a.samp_shape || a.phase == 2 || a.npc_blocks > NPC_MAX_BLOCKS))
        return set_error(DQNX_EUNSUPPORTED, "forward MT-cache workgroup: not with the sampler workgroup / phase 2");
    const dim3 grid(a.tiles * a.nstreams * (a.phase == 1 ? a.csplit : (a.phase == 3 ? 2 : 1)) +
                    ((a.samp_shape || a.npc) ? 1 : 0)), block(FT);
    size_t shm = (size_t)(a.buf0 + a.buf1) * 4;
    if (shm < (size_t)DQNX_FUSED_LDS_MIN) shm = DQNX_FUSED_LDS_MIN;
    if (shm < (size_t)a.lds_min) shm = (size_t)a.lds_min;
    if (a.samp_shape && shm < (size_t)fwd_sample_lds_bytes(a.samp_shape)) shm = fwd_sample_lds_bytes(a.samp_shape);
    if (a.npc && shm < (size_t)(2 * 624 + 2) * 4) shm = (2 * 624 + 2) * 4;
#define FUSED_FWD_GW(ACTV, NLV, BFV, MRV, PHV, GWV)                                                  \
    do {                                                                                             \
        if (shm > 64 * 1024) allow_lds(k_mlp_fwd<ACTV, NLV, BFV, MRV, PHV, GWV>, 160 * 1024);        \
        DQNX_LAUNCH((k_mlp_fwd<ACTV, NLV, BFV, MRV, PHV, GWV>), grid, block, shm, s, a);      \
    } while (0)
#define FUSED_FWD_MR(ACTV, NLV, BFV, MRV, PHV)                                                       \
    do {                                                                                             \
        if constexpr (MRV == 1 && PHV == 0) {                                                        \
            if (a.gw) { FUSED_FWD_GW(ACTV, NLV, BFV, 1, 0, 1); break; }                             \
        }                                                                                            \
        FUSED_FWD_GW(ACTV, NLV, BFV, MRV, PHV, 0);                                                   \
    } while (0)
#define FUSED_FWD_BF(ACTV, NLV, BFV)                                                                 \
    do {                                                                                             \
        if (a.phase == 1) {                                                                          \
            if constexpr (NLV >= 2) {                                                                \
                if (a.mr == 4) FUSED_FWD_MR(ACTV, NLV, BFV, 4, 1);                                   \
                else if (a.mr == 2) FUSED_FWD_MR(ACTV, NLV, BFV, 2, 1);                              \
                else FUSED_FWD_MR(ACTV, NLV, BFV, 1, 1);                                             \
            }                                                                                        \
        }                                                                                            \
        else if (a.phase == 2) { if constexpr (NLV >= 2) FUSED_FWD_MR(ACTV, NLV, BFV, 1, 2); }        \
        else if (a.phase == 3) { if constexpr (NLV >= 2 && !BFV) FUSED_FWD_GW(ACTV, NLV, BFV, 1, 3, 0); } \
        else if (a.mr == 4) FUSED_FWD_MR(ACTV, NLV, BFV, 4, 0);                                      \
        else if (a.mr == 2) FUSED_FWD_MR(ACTV, NLV, BFV, 2, 0);                                      \
        else FUSED_FWD_MR(ACTV, NLV, BFV, 1, 0);                                                     \
    } while (0)
#define FUSED_FWD_CASE(ACTV, NLV)                                                                    \
    do {                                                                                             \
        if (a.bf16) FUSED_FWD_BF(ACTV, NLV, true);                                                   \
        else FUSED_FWD_BF(ACTV, NLV, false);                                                         \
    } while (0)
    const bool relu = act == DQNX_ACT_RELU;
    switch (a.L) {
        case 1: if (relu) FUSED_FWD_CASE(DQNX_ACT_RELU, 1); else FUSED_FWD_CASE(DQNX_ACT_ELU, 1); break;
        case 2: if (relu) FUSED_FWD_CASE(DQNX_ACT_RELU, 2); else FUSED_FWD_CASE(DQNX_ACT_ELU, 2); break;
        case 3: if (relu) FUSED_FWD_CASE(DQNX_ACT_RELU, 3); else FUSED_FWD_CASE(DQNX_ACT_ELU, 3); break;
        default: return set_error(DQNX_EUNSUPPORTED, "fused forward: %d dense layers", a.L);
    }
#undef FUSED_FWD_CASE
#undef FUSED_FWD_BF
#undef FUSED_FWD_MR
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_head_bwd(const HeadBwdArgs& a, int act, hipStream_t s) {
    const dim3 grid(((a.Bl + 15) / 16) * a.nsplit), block(FT);
    const size_t pad = DQNX_HEAD_LDS_PAD;   // dynamic LDS on top of the static tiles (occupancy knob)
#define HEAD_BWD_CASE(ACTV, NLV)                                                                     \
    do {                                                                                             \
        if (a.bf16) {                                                                                \
            if (pad > 64 * 1024) allow_lds(k_head_bwd<ACTV, NLV, true>, 120 * 1024);                 \
            DQNX_LAUNCH((k_head_bwd<ACTV, NLV, true>), grid, block, pad, s, a);               \
        } else {                                                                                     \
            if (pad > 64 * 1024) allow_lds(k_head_bwd<ACTV, NLV, false>, 120 * 1024);                \
            DQNX_LAUNCH((k_head_bwd<ACTV, NLV, false>), grid, block, pad, s, a);              \
        }                                                                                            \
    } while (0)
    const bool relu = act == DQNX_ACT_RELU;
    switch (a.L) {
        case 1: if (relu) HEAD_BWD_CASE(DQNX_ACT_RELU, 1); else HEAD_BWD_CASE(DQNX_ACT_ELU, 1); break;
        case 2: if (relu) HEAD_BWD_CASE(DQNX_ACT_RELU, 2); else HEAD_BWD_CASE(DQNX_ACT_ELU, 2); break;
        case 3: if (relu) HEAD_BWD_CASE(DQNX_ACT_RELU, 3); else HEAD_BWD_CASE(DQNX_ACT_ELU, 3); break;
        default: return set_error(DQNX_EUNSUPPORTED, "fused head: %d dense layers", a.L);
    }
#undef HEAD_BWD_CASE
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
