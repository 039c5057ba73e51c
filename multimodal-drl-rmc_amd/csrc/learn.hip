// DQN learn-step kernels (dense part): forward Linear layers, the fused Q-head /
// TD-target / Huber / head-backward kernel, backward levels (dX and split-K dW) and the
// fused Adam + soft-target-update pass.
//
// Reference path (R: = /root/reference/):
//   DoubleAgent.learn      R:dqn/agent.py:204-226   (online(s'), argmax, target(s'), gather,
//                                                    TD target, online(s), gather, Huber, bwd, Adam)
//   SimpleAgent.learn      R:dqn/agent.py:166-185   (max over target(s'))
//   PerDoubleAgent.learn   R:dqn/agent.py:245-272   (IS-weighted Huber, |delta| for priorities)
//   DuelingDeepQNetwork    R:dqn/network.py:77-96   (Q = V + (A - mean A))
//   DeepQNetwork           R:dqn/network.py:50-65
//   MLP body               R:env/custom_env/macro with lane/dqn_config.py:76-84
//   Adam                   torch.optim.Adam single-tensor step (R:env/dqn_config.py:176)
//   soft target update     R:dqn/agent.py:105-110
#include "gemm_lds.hpp"
#include "gemm_sk.hpp"
#include "learn.hpp"
#include "per_common.hpp"
#include "mt.hpp"

namespace dqnx {

// =====================================================================================
// Forward Linear: C[s] = act(A[s] W[s]^T + b[s]) for up to 3 "streams" (blockIdx.z):
// online(obs), online(next_obs), target(next_obs).  Layer 1 gathers A rows from the
// replay ring through the sampled physical slots (no materialised minibatch), and
// stream 0's first column tile also writes the gathered rows to `xcopy` for layer-1 dW.
// =====================================================================================
// Tile engine: DQNX_GEMM_SK=1 selects the wave-split-K engine (gemm_sk.hpp), default the
// LDS-staged engine (gemm_lds.hpp).  Configs are compile-time (tools/variants_*.txt sweeps).
#ifndef DQNX_GEMM_SK
#define DQNX_GEMM_SK 0
#endif
#ifndef DQNX_FWD_BM
#define DQNX_FWD_BM 16
#endif
#ifndef DQNX_FWD_BN
#define DQNX_FWD_BN 64
#endif
#ifndef DQNX_FWD_KT
#define DQNX_FWD_KT 128
#endif
#ifndef DQNX_FWD_WM
#define DQNX_FWD_WM 1
#endif
#ifndef DQNX_BWD_BM
#define DQNX_BWD_BM 32
#endif
#ifndef DQNX_BWD_BN
#define DQNX_BWD_BN 32
#endif
#ifndef DQNX_BWD_KT
#define DQNX_BWD_KT 128
#endif
#ifndef DQNX_BWD_WM
#define DQNX_BWD_WM 2
#endif
constexpr int FWD_BM = DQNX_FWD_BM, FWD_BN = DQNX_FWD_BN, BWD_BM = DQNX_BWD_BM, BWD_BN = DQNX_BWD_BN;


// Engine adapter: G::run leaves tile element rows [ro + tm*16 + 4g + r], cols [co + tn*16 + i]
// in acc[tm][tn][r] of the waves for which owner() is true.
template <int BM, int BN, int KT, int WM, int LA, int LB, bool VA, bool VB>
struct Engine {
#if DQNX_GEMM_SK
    using G = TileGemmSK<BM, BN, 4, (KT < 64 ? KT : 64), LA, LB, VA, VB>;
    __device__ __forceinline__ static int ro() { return 0; }
    __device__ __forceinline__ static int co() { return 0; }
    __device__ __forceinline__ static bool owner() { return (threadIdx.x >> 6) == 0; }
#else
    using G = TileGemm<BM, BN, KT, WM, 4 / WM, LA, LB, VA, VB>;
    __device__ __forceinline__ static int ro() { return ((threadIdx.x >> 6) / (4 / WM)) * G::TM * 16; }
    __device__ __forceinline__ static int co() { return ((threadIdx.x >> 6) % (4 / WM)) * G::TN * 16; }
    __device__ __forceinline__ static bool owner() { return true; }
#endif
    static constexpr int TM = G::TM, TN = G::TN, LDS_FLOATS = G::LDS_FLOATS > 0 ? G::LDS_FLOATS : 1;
};

// =====================================================================================
// Forward Linear: C[s] = act(A[s] W[s]^T + b[s]) for up to 3 "streams":
// online(obs), online(next_obs), target(next_obs).  Layer 1 gathers A rows from the
// replay ring through the sampled physical slots (no materialised minibatch), and
// stream 0's first column tile also writes the gathered rows to `xcopy` for layer-1 dW.
// =====================================================================================
// GATHER: first layer (operand rows gathered from the replay ring through the sampled
// physical rows); hidden layers read the previous activation rows in order.
// ULOAD (dense rows, no gather, K % 4 == 0): unconditional operand loads (gemm_common.hpp)
template <int ACT, bool VECB, bool GATHER, bool ULOAD = false>
__global__ __launch_bounds__(256) void k_linear_fwd(FwdArgs args) {
    constexpr int LAY = ULOAD ? L_ROWS_KU : L_ROWS_K;
    using E = Engine<FWD_BM, FWD_BN, DQNX_FWD_KT, DQNX_FWD_WM, LAY, LAY, true, VECB>;
    constexpr int TM = E::TM, TN = E::TN;
    __shared__ __attribute__((aligned(16))) float lds[E::LDS_FLOATS];
    // tiles ordered (stream, m-tile, n-tile) with n fastest; each XCD gets a contiguous
    // range, so the n-tiles that re-read one m-tile's gathered rows share an L2.
    const int ntn = (args.N + FWD_BN - 1) / FWD_BN, ntm = (args.M + FWD_BM - 1) / FWD_BM;
    const int T = xcd_remap(blockIdx.x, ntn * ntm * args.nprob);
    const int z = T / (ntn * ntm), rem = T - z * ntn * ntm;
    const int tm_ = rem / ntn, tn_ = rem - tm_ * ntn;
    const FwdProblem& P = args.p[z];
    const int lane = threadIdx.x & 63;
    const int i = lane & 15, g = lane >> 4;
    const int m0 = tm_ * FWD_BM, n0 = tn_ * FWD_BN;
    const int M = args.M, N = args.N, K = args.K;
    const int Kpad = (K + 3) & ~3;   // ring / activation rows are zero padded to a multiple of 4
    float bias[TN];                  // epilogue operands fetched before the main loop
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + E::co() + tn * 16 + i;
        bias[tn] = col < N ? P.bias[col] : 0.f;
    }
    Operand A{P.A, P.lda, GATHER ? P.phys : nullptr, M, Kpad, -1, (GATHER && P.xcopy && tn_ == 0) ? P.xcopy : nullptr, P.lda};
    Operand B{P.W, K, nullptr, N, K, -1, nullptr, 0};
    floatx4 acc[TM][TN];
    E::G::run(lds, A, B, m0, n0, 0, Kpad, acc);
    if (!E::owner()) return;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + E::co() + tn * 16 + i;
        if (col >= N) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + E::ro() + tm * 16 + 4 * g + r;
                if (row < M) P.C[(int64_t)row * args.ldc + col] = act_fwd<ACT>(acc[tm][tn][r] + bias[tn]);
            }
    }
}

// Large-K forward (a 128x128 tile re-reads each weight row ntm = M/128 times instead of M/16):
// split-K over ksplit chunks, raw sums to `partial`, then k_linear_fwd_reduce.
// ksplit == 1 (the conv GEMMs: M = B*Ho*Wo rows, N = Cout): bias + activation epilogue straight
// into C.  A 128-row tile loads each weight K-slab once per 128 rows instead of once per 16.
// The per-element accumulation order (K ascending, 16-deep MFMA chunks) is the one of the
// 16x64 kernel, so both give bit-identical outputs.
template <int ACT, bool VECB, int BM, int BN, int WM, int KT = FWD_BIG_KT, int LAYA = L_ROWS_K, int LAYB = L_ROWS_K,
          int PF = 1>
__global__ __launch_bounds__(256) void k_linear_fwd_big(FwdArgs args) {
    constexpr int WN = 4 / WM;
    using G = TileGemm<BM, BN, KT, WM, WN, LAYA, LAYB, true, VECB>;
    constexpr int TM = G::TM, TN = G::TN;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    const int M = args.M, N = args.N, K = args.K;
    const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
    const int tiles = ntn * ntm * args.nprob;
    // chunk-major order: an XCD's contiguous range shares one K chunk of A and W in its L2
    const int T = xcd_remap(blockIdx.x, tiles * args.ksplit);
    const int sl = T / tiles, T2 = T - sl * tiles;
    const int z = T2 / (ntn * ntm), rem = T2 - z * ntn * ntm;
    const int tm_ = rem / ntn, tn_ = rem - tm_ * ntn;
    const FwdProblem& P = args.p[z];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
    const int Kpad = (K + 3) & ~3;
    const int kb = sl * args.kchunk, ke = min(Kpad, kb + args.kchunk);
    Operand A{P.A, P.lda, nullptr, M, Kpad, -1, nullptr, P.lda};
    Operand B{P.W, K, nullptr, N, K, -1, nullptr, 0};
    floatx4 acc[TM][TN];
    DQNX_STAMP(args.stamps, 53);
    if constexpr (PF == 2) G::run2(lds, A, B, m0, n0, kb, ke, acc);
    else G::run(lds, A, B, m0, n0, kb, ke, acc);
    DQNX_STAMP(args.stamps, 54);
    const int ro = (wid / WN) * TM * 16, co = (wid % WN) * TN * 16;
    if (args.ksplit == 1) {
#pragma unroll
        for (int tn = 0; tn < TN; tn++) {
            const int col = n0 + co + tn * 16 + i;
            if (col >= N) continue;
            const float bv = P.bias[col];
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = m0 + ro + tm * 16 + 4 * g + r;
                    if (row < M) P.C[(int64_t)row * args.ldc + col] = act_fwd<ACT>(acc[tm][tn][r] + bv);
                }
        }
        return;
    }
    float* part = args.partial + ((int64_t)sl * args.nprob + z) * M * N;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + co + tn * 16 + i;
        if (col >= N) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + ro + tm * 16 + 4 * g + r;
                if (row < M) part[(int64_t)row * N + col] = acc[tm][tn][r];
            }
    }
    DQNX_STAMP(args.stamps, 55);
}

template <int ACT>
__global__ __launch_bounds__(256) void k_linear_fwd_reduce(FwdArgs args) {
    const int M = args.M, N = args.N;
    const int64_t per = (int64_t)M * N, total = per * args.nprob;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int z = (int)(t / per);
        const int64_t e = t - (int64_t)z * per;
        const int row = (int)(e / N), col = (int)(e - (int64_t)row * N);
        float s = args.partial[((int64_t)0 * args.nprob + z) * per + e];
        for (int sl = 1; sl < args.ksplit; sl++) s += args.partial[((int64_t)sl * args.nprob + z) * per + e];
        args.p[z].C[(int64_t)row * args.ldc + col] = act_fwd<ACT>(s + args.p[z].bias[col]);
    }
}

// Conv dX role on 128x64 tiles (dCol = dZ W, no mask: col2im applies the previous conv's ELU'),
// for convs whose M = B*Ho*Wo rows fill the chip: the 32x32 dx role re-reads the weight per 32
// rows and dZ per 32 columns.  Same K order as the 32x32 role: bit-identical dCol.
template <bool VECW>
__global__ __launch_bounds__(256) void k_conv_dx_big(BwdArgs a) {
    constexpr int BM = 128, BN = 64, WM = 2, WN = 2;
    using G = TileGemm<BM, BN, FWD_BIG_KT, WM, WN, L_ROWS_K, L_K_ROWS, true, VECW>;
    constexpr int TM = G::TM, TN = G::TN;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    const int ntn = (a.in + BN - 1) / BN, ntm = (a.Bl + BM - 1) / BM;
    const int T = xcd_remap(blockIdx.x, ntn * ntm);
    const int tm_ = T / ntn, tn_ = T - tm_ * ntn;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
    Operand A{a.dZ, a.out, nullptr, a.Bl, a.out, -1, nullptr, 0};
    Operand B{a.W, a.in, nullptr, a.in, a.out, -1, nullptr, 0};
    floatx4 acc[TM][TN];
    G::run(lds, A, B, m0, n0, 0, a.out, acc);
    const int ro = (wid / WN) * TM * 16, co = (wid % WN) * TN * 16;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + co + tn * 16 + i;
        if (col >= a.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + ro + tm * 16 + 4 * g + r;
                if (row < a.Bl) a.dZprev[(int64_t)row * a.in + col] = acc[tm][tn][r];
            }
    }
}

// Conv dW (partial[s] = dZ^T [X | 1] over the pixels of slice s) on 64x128 tiles for large
// convs: the 32x32 role re-reads the column matrix X per 32 output channels and dZ per 32
// columns.  Its own launch; the slab layout and the Adam-side slab sum are unchanged.
__global__ __launch_bounds__(256) void k_conv_dw_big(BwdArgs a) {
    constexpr int BM = 64, BN = 128, WM = 2, WN = 2;
    using G = TileGemm<BM, BN, FWD_BIG_KT, WM, WN, L_K_ROWS, L_K_ROWS, true, true>;
    constexpr int TM = G::TM, TN = G::TN;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    const DwProblem& d = a.dw[0];
    const int ntn = (d.in + 1 + BN - 1) / BN, ntm = (d.out + BM - 1) / BM;
    const int T = xcd_remap(blockIdx.x, ntn * ntm * a.dw_slices);
    const int bz = T / (ntn * ntm), rem = T - bz * ntn * ntm;
    const int by = rem / ntn, bx = rem - by * ntn;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int m0 = by * BM, n0 = bx * BN;
    const int kb = bz * a.kslice, ke = min(a.Bl, kb + a.kslice);
    Operand A{d.dZ, d.ldz, nullptr, d.out, a.Bl, -1, nullptr, 0};
    Operand B{d.X, d.ldx, nullptr, d.in, a.Bl, d.in, nullptr, 0};
    floatx4 acc[TM][TN];
    G::run(lds, A, B, m0, n0, kb, ke, acc);
    const int ro = (wid / WN) * TM * 16, co = (wid % WN) * TN * 16;
    float* part = d.partial + (int64_t)bz * d.pstride;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + co + tn * 16 + i;
        if (col > d.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + ro + tm * 16 + 4 * g + r;
                if (row >= d.out) continue;
                part[col < d.in ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row] = acc[tm][tn][r];
            }
    }
}

int conv_dw_big_tiles(int in, int out) { return ((in + 1 + 127) / 128) * ((out + 63) / 64); }

int launch_conv_dw_big(const BwdArgs& a, hipStream_t s) {
    const dim3 grid(conv_dw_big_tiles(a.dw[0].in, a.dw[0].out) * a.dw_slices);
    DQNX_LAUNCH(k_conv_dw_big, grid, dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int conv_dx_big_tiles(int Bl, int in) { return ((in + 63) / 64) * ((Bl + 127) / 128); }

int launch_conv_dx_big(const BwdArgs& a, hipStream_t s) {
    const dim3 grid(conv_dx_big_tiles(a.Bl, a.in));
    if (a.in % 4 == 0) DQNX_LAUNCH((k_conv_dx_big<true>), grid, dim3(256), 0, s, a);
    else DQNX_LAUNCH((k_conv_dx_big<false>), grid, dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// =====================================================================================
// Backward level: independent GEMMs in one launch.
//   dx role:  dZprev = (dZ W) (.) act'(Hprev)      [Bl x in], K = out
//   dw role:  partial[s] = dZ^T [Xprev | 1]        [out x (in+1)], K = samples of slice s
// =====================================================================================
// VECW: the dx role's weight rows (length `in`) allow float4 loads (in % 4 == 0).
// Hprev == null: no activation mask (conv dX columns before col2im).
// U: unconditional operand loads (gemm_common.hpp); the dx role's weight rows as float4 (VECW) or
// float2 pairs
template <int ACT, bool VECW, bool U = false, int TS = BWD_BM>
__global__ __launch_bounds__(256) void k_bwd_level(BwdArgs a) {
    constexpr int BWD_BM = TS, BWD_BN = TS;   // (shadows the default tile edge)
    constexpr int KT = TS == 64 ? 64 : DQNX_BWD_KT;   // 64 x 64 tiles: 64-deep passes (36 KB of LDS)
    using EX = Engine<BWD_BM, BWD_BN, KT, DQNX_BWD_WM, U ? L_ROWS_KU : L_ROWS_K,
                      U ? (VECW ? L_K_ROWSU : L_K_ROWS2) : L_K_ROWS, true, VECW>;
    using EW = Engine<BWD_BM, BWD_BN, KT, DQNX_BWD_WM, U ? L_K_ROWSU : L_K_ROWS, U ? L_K_ROWSU : L_K_ROWS, true, true>;
    constexpr int TM = EX::TM, TN = EX::TN;
    constexpr int LF = EX::LDS_FLOATS > EW::LDS_FLOATS ? EX::LDS_FLOATS : EW::LDS_FLOATS;
    __shared__ __attribute__((aligned(16))) float lds[LF];
    const int lane = threadIdx.x & 63;
    const int i = lane & 15, g = lane >> 4;
    int b = blockIdx.x;
    floatx4 acc[TM][TN];
    if (b < a.dx_blocks) {
        const int T = xcd_remap(b, a.dx_blocks);
        const int bx = T % a.dx_grid_x, by = T / a.dx_grid_x;
        const int m0 = by * BWD_BM, n0 = bx * BWD_BN;
        float hm[TM][TN][4];   // activation values for the mask, fetched before the main loop
#pragma unroll
        for (int tn = 0; tn < TN; tn++)
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int col = n0 + EX::co() + tn * 16 + i, row = m0 + EX::ro() + tm * 16 + 4 * g + r;
                    hm[tm][tn][r] = !a.Hprev ? 1.f   // act_bwd(g, h > 0) == g
                                    : (col < a.in && row < a.Bl) ? a.Hprev[(int64_t)row * a.ldh + col] : 0.f;
                }
        Operand A{a.dZ, a.out, nullptr, a.Bl, a.out, -1, nullptr, 0};
        Operand B{a.W, a.in, nullptr, a.in, a.out, -1, nullptr, 0};
        EX::G::run(lds, A, B, m0, n0, 0, a.out, acc);
        if (!EX::owner()) return;
#pragma unroll
        for (int tn = 0; tn < TN; tn++) {
            const int col = n0 + EX::co() + tn * 16 + i;
            if (col >= a.in) continue;
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = m0 + EX::ro() + tm * 16 + 4 * g + r;
                    if (row < a.Bl) a.dZprev[(int64_t)row * a.in + col] = act_bwd<ACT>(acc[tm][tn][r], hm[tm][tn][r]);
                }
        }
        return;
    }
    b -= a.dx_blocks;
    int p = 0;
    while (p + 1 < a.ndw && b >= a.dw[p].blocks) { b -= a.dw[p].blocks; p++; }
    const DwProblem& d = a.dw[p];
    // dW tiles ordered (slice, m, n) so one XCD re-reads one slice of dZ / X rows
    b = xcd_remap(b, d.blocks);
    const int bx = b % d.grid_x;
    const int t2 = b / d.grid_x;
    const int by = t2 % d.grid_y, bz = t2 / d.grid_y;
    const int m0 = by * BWD_BM, n0 = bx * BWD_BN;
    const int kb = bz * a.kslice;
    const int ke = min(a.Bl, kb + a.kslice);
    Operand A{d.dZ, d.ldz, nullptr, d.out, a.Bl, -1, nullptr, 0};
    Operand B{d.X, d.ldx, nullptr, d.in, a.Bl, d.in, nullptr, 0};
    EW::G::run(lds, A, B, m0, n0, kb, ke, acc);
    if (!EW::owner()) return;
    float* part = d.partial + (int64_t)bz * d.pstride;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + EW::co() + tn * 16 + i;
        if (col > d.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + EW::ro() + tm * 16 + 4 * g + r;
                if (row >= d.out) continue;
                int64_t o;
                if (d.head_kind < 0) o = (col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row;
                else o = (col < d.in) ? head_w_off(d.head_kind, row, d.in) + col : head_b_off(d.head_kind, row, d.in, d.A);
                part[o] = acc[tm][tn][r];
            }
    }
}

// =====================================================================================
// Fused head kernel: one workgroup = 16 samples, 256 threads.
//   (0) stage H_L of the 3 streams and both heads' weights in LDS (one round trip)
//   (1) head Linear for the 3 streams on MFMA (waves 0..2)
//   (2) thread (b, j): Q[s][b][j] (dueling aggregate V + (A - mean A))
//   (3) thread (b, 0): Double-DQN argmax / DQN max, TD target y = r + ((1-d)*gamma)*q',
//       q(s,a), Huber (beta=1) value and gradient (mean or IS-weighted 'none' reduction)
//   (4) thread (b, o): d(head outputs)
//   (5) MFMA: dH = dHead . W_head -> dZ_L = dH (.) act'(H_L);  dW_head partial = dHead^T H_L;
//       bias and loss partials in fixed order.
// =====================================================================================
template <int ACT, int F>
__global__ __launch_bounds__(256) void k_head(HeadArgs a) {
    constexpr int TS = 16, QS = 17;
    constexpr int SF = F + 8, F4 = F / 4;
    constexpr int NHQ = 3 * TS * F4, NWQ = 2 * 16 * F4, NQ = (NHQ + NWQ + 255) / 256;
    __shared__ __attribute__((aligned(16))) float dyn[5 * 16 * SF];
    __shared__ float raw[3][TS][QS];
    __shared__ float qv[3][TS][QS];
    __shared__ float dh[TS][20];
    __shared__ float gsh[TS], lossv[TS], rsh[TS], dsh[TS], wsh[TS];
    __shared__ int ash[TS];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int b0 = blockIdx.x * TS;
    const int A = a.A, NH = a.NH, Bl = a.Bl;
    const int nb = min(TS, Bl - b0);
    const bool use1 = a.algo != DQNX_ALGO_DQN;
    float* Hs = dyn;                    // [3][TS][SF]
    float* Wh = dyn + 3 * TS * SF;      // [2][16][SF] online, target (rows >= NH zero)
    DQNX_STAMP(a.stamps, 16);

    // (0) stage: every load issued before the first wait
    {
        float4 v[NQ];
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < NHQ) {
                const int s = q / (TS * F4), rem = q - s * TS * F4, b = rem / F4, c = 4 * (rem - b * F4);
                if (b < nb && (s != 1 || use1)) x = ld4(a.H + ((int64_t)s * Bl + b0 + b) * F + c);
            } else if (q < NHQ + NWQ) {
                const int q2 = q - NHQ;
                const int w = q2 / (16 * F4), rem = q2 - w * 16 * F4, o = rem / F4, c = 4 * (rem - o * F4);
                if (o < NH) x = ld4((w ? a.Wt : a.Wo) + head_w_off(a.head_kind, o, F) + c);
            }
            v[j] = x;
        }
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            if (q < NHQ) {
                const int s = q / (TS * F4), rem = q - s * TS * F4, b = rem / F4, c = 4 * (rem - b * F4);
                *reinterpret_cast<float4*>(Hs + (s * TS + b) * SF + c) = v[j];
            } else if (q < NHQ + NWQ) {
                const int q2 = q - NHQ;
                const int w = q2 / (16 * F4), rem = q2 - w * 16 * F4, o = rem / F4, c = 4 * (rem - o * F4);
                *reinterpret_cast<float4*>(Wh + (w * 16 + o) * SF + c) = v[j];
            }
        }
        if (tid < TS) {
            const int b = tid;
            int act = 0;
            float rew = 0.f, done = 0.f, w = 1.f;
            if (b < nb) {
                const int slot = a.phys[b0 + b];
                act = a.act[slot];
                rew = a.rew[slot];
                done = a.done[slot];
                if (a.isw) w = a.isw[b0 + b];
                if (act < 0 || act >= A) act = 0;
            }
            ash[b] = act;
            rsh[b] = rew;
            dsh[b] = done;
            wsh[b] = w;
        }
    }
    __syncthreads();
    DQNX_STAMP(a.stamps, 17);

    // (1) head outputs per stream: raw[s] = H_s . W^T + b
    if (wid < 3 && (wid != 1 || use1)) {
        const int s = wid;
        const float* hs = Hs + s * TS * SF;
        const float* wh = Wh + (s == 2 ? 16 : 0) * SF;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int kk = 0; kk < F; kk += 16) {
            const float4 av = *reinterpret_cast<const float4*>(hs + i * SF + kk + 4 * g);
            const float4 bv = *reinterpret_cast<const float4*>(wh + i * SF + kk + 4 * g);
            acc = mfma16x16x4(av.x, bv.x, acc);
            acc = mfma16x16x4(av.y, bv.y, acc);
            acc = mfma16x16x4(av.z, bv.z, acc);
            acc = mfma16x16x4(av.w, bv.w, acc);
        }
        const float* W = (s == 2) ? a.Wt : a.Wo;
        const float bias = (i < NH) ? W[head_b_off(a.head_kind, i, F, A)] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; r++) raw[s][4 * g + r][i] = acc[r] + bias;
    }
    __syncthreads();

    // (2) Q values, thread (b, j)
    {
        const int b = tid >> 4, j = tid & 15;
        for (int s = 0; s < 3; s++) {
            if (s == 1 && !use1) continue;
            float q = 0.f;
            if (a.head_kind == DQNX_HEAD_DUELING) {
                float sum = 0.f;
                for (int jj = 0; jj < A; jj++) sum += raw[s][b][1 + jj];
                const float mean = sum / (float)A;
                if (j < A) q = raw[s][b][0] + (raw[s][b][1 + j] - mean);
            } else if (j < A) {
                q = raw[s][b][j];
            }
            qv[s][b][j] = q;
            if (j < A && b < nb) a.Q[((int64_t)s * Bl + b0 + b) * A + j] = q;
        }
    }
    __syncthreads();
    DQNX_STAMP(a.stamps, 18);

    // (3) per-sample TD target / Huber, thread (b, 0)
    if (tid < TS) {
        const int b = tid;
        float gq = 0.f, lb = 0.f;
        if (b < nb) {
            float qn;
            if (!use1) {                                   // target(s').max(1) (R:dqn/agent.py:172-173)
                qn = qv[2][b][0];
                for (int j = 1; j < A; j++) qn = qv[2][b][j] > qn ? qv[2][b][j] : qn;
            } else {                                       // argmax online(s'), gather target(s') (:210-214)
                int best = 0;
                float bq = qv[1][b][0];
                for (int j = 1; j < A; j++)
                    if (qv[1][b][j] > bq) { bq = qv[1][b][j]; best = j; }
                qn = qv[2][b][best];
            }
            // targets = rews + (1 - dones) * gamma * q'   (R:dqn/agent.py:216)
            const float t1 = 1.f - dsh[b];
            const float t2 = t1 * a.gamma;
            const float t3 = t2 * qn;
            const float y = rsh[b] + t3;
            const float qa = qv[0][b][ash[b]];
            const float x = qa - y;                        // smooth_l1: input - target
            const float z = fabsf(x);
            const float l = z < 1.f ? (0.5f * z) * z / 1.f : z - 0.5f;
            if (a.isw) {                                   // PER: mean(w * huber_none) (R:dqn/agent.py:267)
                const float go = a.inv_bg * wsh[b];
                gq = x <= -1.f ? -go : (x >= 1.f ? go : (x * go) / 1.f);
                lb = wsh[b] * l;
            } else {                                       // SmoothL1Loss(mean): norm = 1/B
                gq = x <= -1.f ? -a.inv_bg : (x >= 1.f ? a.inv_bg : (a.inv_bg * x) / 1.f);
                lb = l;
            }
            const int gb = b0 + b;
            a.td[gb] = y;
            a.td[Bl + gb] = qa;
            a.td[2 * Bl + gb] = z;
            if (a.abs_td_out) a.abs_td_out[gb] = z;
        }
        gsh[b] = gq;
        lossv[b] = lb;
    }
    __syncthreads();

    // (4) d(head outputs), thread (b, o)
    {
        const int b = tid >> 4, o = tid & 15;
        const float gq = gsh[b];
        const int act = ash[b];
        float d = 0.f;
        if (o < NH) {
            if (a.head_kind == DQNX_HEAD_DUELING)
                d = (o == 0) ? gq : ((o - 1 == act ? gq : 0.f) + (-gq) / (float)A);   // V / A - mean(A) bwd
            else
                d = (o == act) ? gq : 0.f;
        }
        dh[b][o] = d;
    }
    __syncthreads();
    DQNX_STAMP(a.stamps, 19);

    // (5) dH = dHead . W_head (online), dZ_L = dH (.) act'(H_L)   [TS x F], K = 16 head rows;
    //     dHead rows go to global for the head-weight gradient (bwd level L)
    if (tid < TS * 4) {
        const int b = tid >> 2, q = tid & 3;
        if (b < nb)
            *reinterpret_cast<float4*>(a.dhead + (int64_t)(b0 + b) * 16 + 4 * q) =
                make_float4(dh[b][4 * q], dh[b][4 * q + 1], dh[b][4 * q + 2], dh[b][4 * q + 3]);
    }
    constexpr int ftiles = F / 16;
    for (int t = wid; t < ftiles; t += 4) {
        const int f0 = t * 16;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {   // A[b][o] = dh[b][o]; B[o][f] = Wh_online[o][f]
            const int o = 4 * g + jj;
            acc = mfma16x16x4(dh[i][o], Wh[o * SF + f0 + i], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int b = 4 * g + r;
            if (b < nb) a.dZ[(int64_t)(b0 + b) * F + f0 + i] = act_bwd<ACT>(acc[r], Hs[b * SF + f0 + i]);
        }
    }
    if (tid == 64) {
        float s = 0.f;
        for (int b = 0; b < TS; b++) s += lossv[b];
        a.loss_partial[blockIdx.x] = s;
    }
    // (6) dZ_{L-1} = (dZ_L W_L) (.) act'(H_{L-1}) for this tile's samples: [TS x in_prev], K = F.
    //     The tile's dZ_L rows were just stored by this workgroup (never cached before: no
    //     stale L1 lines); the block fence + barrier order them before the reads.
    if (a.dZprev) {
        using GP = TileGemm<16, 256, 32, 1, 4, L_ROWS_K, L_K_ROWS, true, true>;
        __shared__ __attribute__((aligned(16))) float lds2[GP::LDS_FLOATS];
        __threadfence_block();
        __syncthreads();
        Operand Ao{a.dZ, F, nullptr, Bl, F, -1, nullptr, 0};
        Operand Bo{a.W_last, a.in_prev, nullptr, a.in_prev, F, -1, nullptr, 0};
        for (int n0 = 0; n0 < a.in_prev; n0 += 256) {
            float hm[GP::TN][4];   // mask operands fetched before the GEMM
#pragma unroll
            for (int tn = 0; tn < GP::TN; tn++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int col = n0 + (wid * GP::TN + tn) * 16 + i, b = 4 * g + r;
                    hm[tn][r] = (col < a.in_prev && b < nb) ? a.Hprev[(int64_t)(b0 + b) * a.in_prev + col] : 0.f;
                }
            floatx4 acc2[GP::TM][GP::TN];
            GP::run(lds2, Ao, Bo, b0, n0, 0, F, acc2);
#pragma unroll
            for (int tn = 0; tn < GP::TN; tn++) {
                const int col = n0 + (wid * GP::TN + tn) * 16 + i;
                if (col >= a.in_prev) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int b = 4 * g + r;
                    if (b < nb)
                        a.dZprev[(int64_t)(b0 + b) * a.in_prev + col] = act_bwd<ACT>(acc2[0][tn][r], hm[tn][r]);
                }
            }
            __syncthreads();
        }
    }
    // Adam step counter of this learn step (read by the Adam pass, a later launch)
    if (blockIdx.x == 0 && tid == 128 && a.ctrl) adam_advance(a.ctrl, a.ab);
    DQNX_STAMP(a.stamps, 20);
}

// =====================================================================================
// Adam (+ soft target update).  Gradient of each flat element = fixed-order sum of its
// segment's split-K / per-tile partial slabs (deterministic, no atomics).
//   m.lerp_(g, 1-b1)                 -> m + w*(g - m) as the vectorised fmadd
//   v.mul_(b2).addcmul_(g, g, 1-b2)  -> v*b2 + ((1-b2)*g)*g
//   denom = sqrt(v)/sqrt(bc2) + eps ; p += (-lr/bc1 * m) / denom
//   target = (tau*n_env)*p + (1 - tau*n_env)*target
// mode 0: partials -> grads only; 1: partials -> grads + Adam; 2: grads -> Adam.
// =====================================================================================
// The uniform sampler's MT block cache (learn.hpp): twist the last cached block forward until
// the cache holds `target` blocks.  One 256-thread workgroup; blocks ping-pong through LDS.
__device__ __forceinline__ void mt_cache_extend(uint32_t* mtc, int target) {
    __shared__ uint32_t mb[2][624];
    __shared__ int s_cnt;
    const int tid = threadIdx.x;
    if (tid == 0) s_cnt = (int)mtc[0];
    __syncthreads();
    const int cnt = s_cnt;
    if (cnt <= 0 || cnt >= target) return;
    uint32_t* blocks = mtc + 64;
    for (int j = tid; j < 624; j += blockDim.x) mb[0][j] = blocks[(int64_t)(cnt - 1) * 624 + j];
    __syncthreads();
    int cur = 0;
    for (int b = cnt; b < target; b++) {
        mt_twist_into(mb[cur], mb[cur ^ 1]);   // ends with a barrier
        cur ^= 1;
        for (int j = tid; j < 624; j += blockDim.x) blocks[(int64_t)b * 624 + j] = mb[cur][j];
    }
    if (tid == 0) mtc[0] = (uint32_t)target;   // read by a later kernel only: no fence needed
}

// Position of W_l[r][q] in its fragment-blocked copies (relayout.hpp): fp32 fwd blocks are
// [t = r/16][c = q/16][g = q%16/4][i = r%16][j = q%4] with c < kpad/16; chain blocks the same with
// the roles of r and q exchanged (c < out/16).  bf16 blocks are 16 x 32: c = q/32, g = q%32/8,
// j = q%8, 8 elements per 16-byte unit.
__device__ __forceinline__ int64_t blk_pos(int r, int q, int nch, bool bf16) {
    if (!bf16) return 4 * ((((int64_t)(r >> 4) * nch + (q >> 4)) * 64) + ((q & 15) >> 2) * 16 + (r & 15)) + (q & 3);
    return 8 * ((((int64_t)(r >> 4) * nch + (q >> 5)) * 64) + ((q & 31) >> 3) * 16 + (r & 15)) + (q & 7);
}

__device__ __forceinline__ void blk_store(float* base, int64_t pos, float v, bool bf16) {
    if (bf16) reinterpret_cast<uint16_t*>(base)[pos] = bf16_bits(v);
    else base[pos] = v;
}

// The Adam launch's extra workgroups, BEFORE the element blocks (dispatched first, so they overlap
// the element pass instead of trailing it: at B=4096 the trailing copy cost ~4 us): the sampler's
// MT block cache (a.mtc), then the in-launch prefetch's copy of the staged minibatch over the
// compute slot (a.pf_nidx > 0; every reader of the step's minibatch ran in earlier launches).
__device__ __forceinline__ int adam_extra_count(const AdamArgs& a) {
    return (a.mtc ? 1 : 0) + (a.pf_nidx > 0 ? 1 : 0) + a.pprop_wgs;
}
__device__ __forceinline__ bool adam_extra_wg(const AdamArgs& a) {
    if ((int)blockIdx.x >= adam_extra_count(a)) return false;
    const int x = (int)blockIdx.x - (a.mtc ? 1 : 0) - (a.pf_nidx > 0 ? 1 : 0);
    if (x >= 0) {   // k_per_prop's workgroups (the tree; independent of the parameter update)
        __shared__ double topd[PER_TOP];
        per_prop_block(a.pprop, x * blockDim.x, topd);
    } else if (a.mtc && blockIdx.x == 0) {
        mt_cache_extend(a.mtc, a.mtc_blocks);
    } else {
        for (int q = threadIdx.x; q < a.pf_nidx; q += blockDim.x) a.pf_idx_dst[q] = a.pf_idx_src[q];
        for (int q = threadIdx.x; q < a.pf_nphys; q += blockDim.x) a.pf_phys_dst[q] = a.pf_phys_src[q];
    }
    return true;
}

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    if (adam_extra_wg(a)) return;   // the sampler-cache / staged-minibatch workgroups
    const int eb = (int)blockIdx.x - adam_extra_count(a);   // element block
    const int64_t P = a.n_params;
    const int64_t stride = (int64_t)(gridDim.x - adam_extra_count(a)) * blockDim.x;
    float step_size = 0.f, bc2s = 1.f;
    if (a.mode != 0) {   // this step's scalars, stored by the head kernel (adam_advance)
        step_size = a.ctrl->adam_step_size;
        bc2s = a.ctrl->adam_bc2_sqrt;
    }
    for (int64_t e = a.e0 + (int64_t)eb * blockDim.x + threadIdx.x; e < P; e += stride) {
        // every load of this element is issued before the first use (one round trip)
        float m = 0.f, v = 0.f, p = 0.f, tg = 0.f;
        if (a.mode != 0) {
            m = a.m[e];
            v = a.v[e];
            p = a.p[e];
            if (a.soft) tg = a.target[e];
        }
        float gsum;
        if (a.mode == 2) {
            gsum = a.grads[e];
        } else {
            // the element's segment by static-index selects (a kernel-argument array indexed by a
            // per-lane value would be copied to scratch)
            AdamSegment sg = a.seg[0];
#pragma unroll
            for (int q = 1; q < kMaxSeg; q++)
                if (q < a.nseg && e >= a.seg[q].off) sg = a.seg[q];
            const float* pp = sg.partial + (e - sg.off);
            // fixed-order sum of the slabs: slab 0, then 16 / 4 / 1 per round trip, every load of a
            // round unconditional
            const int64_t ps = sg.pstride;
            gsum = pp[0];
            int u = 1;
            if (sg.wide) {   // k_adam4's wide order: 8 strided partials, then its xor butterfly
                float part[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {   // lanes past the segment's slabs add zeros, as in k_adam4
                    float t = j < sg.S ? pp[(int64_t)j * ps] : 0.f;
                    for (int w = j + 8; w < sg.S; w += 8) t += pp[(int64_t)w * ps];
                    part[j] = t;
                }
                gsum = ((part[0] + part[4]) + (part[2] + part[6])) + ((part[1] + part[5]) + (part[3] + part[7]));
                u = sg.S;
            }
            for (; u + 16 <= sg.S; u += 16) {
                float pv[16];
#pragma unroll
                for (int j = 0; j < 16; j++) pv[j] = pp[(int64_t)(u + j) * ps];
#pragma unroll
                for (int j = 0; j < 16; j++) gsum += pv[j];
            }
            for (; u + 4 <= sg.S; u += 4) {
                float pv[4];
#pragma unroll
                for (int j = 0; j < 4; j++) pv[j] = pp[(int64_t)(u + j) * ps];
#pragma unroll
                for (int j = 0; j < 4; j++) gsum += pv[j];
            }
            for (; u < sg.S; u++) gsum += pp[(int64_t)u * ps];
            a.grads[e] = gsum;
        }
        if (a.mode == 0) continue;
        m = fmaf(a.w1, gsum - m, m);
        v = v * a.beta2;
        v = v + (a.c2 * gsum) * gsum;
        const float denom = sqrtf(v) / bc2s + a.eps;
        p = p + (step_size * m) / denom;
        a.m[e] = m;
        a.v[e] = v;
        a.p[e] = p;
        if (a.soft) tg = a.tau * p + a.one_minus_tau * tg;
        if (a.soft) a.target[e] = tg;
#pragma unroll
        for (int l = 0; l < 3; l++) {   // the blocked copies of a dense-layer weight
            if (l >= a.nblk) continue;
            const AdamArgs::BlkLayer& L = a.blk[l];
            const int64_t le64 = e - L.woff;
            if (le64 < 0 || le64 >= (int64_t)L.out * L.in) continue;
            // row / column by a float reciprocal, corrected by one step (le < 2^24: exact enough)
            const int le = (int)le64;
            int r = (int)((float)le * L.inv_in);
            r -= (r * L.in > le) ? 1 : 0;
            r += ((r + 1) * L.in <= le) ? 1 : 0;
            const int q = le - r * L.in;
            const bool bf = a.blk_bf16 != 0;
            const int64_t pf = blk_pos(r, q, L.kpad / (bf ? 32 : 16), bf);
            blk_store(L.fwd_online, pf, p, bf);
            if (a.soft) blk_store(L.fwd_target, pf, tg, bf);
            if (L.chain) blk_store(L.chain, blk_pos(q, r, L.out / (bf ? 32 : 16), bf), p, bf);
        }
    }
    if (a.mode != 2 && eb == 0 && threadIdx.x < 64 && a.loss_partial) {   // one wave, fixed order
        float s = 0.f;
        for (int j = threadIdx.x; j < a.n_loss_partial; j += 64) s += a.loss_partial[j];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (threadIdx.x == 0) {
            const float loss = s / (float)a.batch_global;
            a.grads[P] = loss;     // all-reduced with the gradient under DP
            a.ctrl->loss = loss;
        }
    }
    if (a.mode == 2 && a.with_loss && eb == 0 && threadIdx.x == 0) a.ctrl->loss = a.grads[P];
}

// k_adam on float4s: every segment offset / slab stride a multiple of 4 and no blocked copies
// (launch_adam checks); 4 consecutive elements per thread per pass, so a thread keeps 4x the
// bytes in flight of the scalar kernel (the (4,84,84) variant updates 29 M parameters).  The
// same per-element arithmetic, the same fixed slab order.
//
// Wide segments (a.wide_end > e0: the leading segments with many split-K slabs, i.e. the micro
// CNN's conv weight gradients, 24..128 slabs at the HEAD net's B=256): ADAM_WIDE lanes share one
// float4, lane j summing slabs j, j + ADAM_WIDE, ... in order, then a fixed xor butterfly over the
// lanes (every lane ends with the same bits).  One round trip of slab loads instead of S / 16
// dependent rounds: the slab sum of conv 2 (128 slabs) was the launch's critical path.
static_assert(ADAM_WIDE == 8, "k_adam's scalar wide sum assumes 8 lanes");
__device__ __forceinline__ void adam4_compute(const AdamArgs& a, const float4& g, float4& m, float4& v, float4& p,
                                              float4& tg, float step_size, float bc2s) {
    auto upd = [&](float& mk, float& vk, float& pk, float& tk, float gk) {
        mk = fmaf(a.w1, gk - mk, mk);
        vk = vk * a.beta2;
        vk = vk + (a.c2 * gk) * gk;
        const float denom = sqrtf(vk) / bc2s + a.eps;
        pk = pk + (step_size * mk) / denom;
        if (a.soft) tk = a.tau * pk + a.one_minus_tau * tk;
    };
    upd(m.x, v.x, p.x, tg.x, g.x);
    upd(m.y, v.y, p.y, tg.y, g.y);
    upd(m.z, v.z, p.z, tg.z, g.z);
    upd(m.w, v.w, p.w, tg.w, g.w);
}
__device__ __forceinline__ void adam4_update(const AdamArgs& a, int64_t e, int nv, float4 g, float4 m, float4 v,
                                             float4& p, float4& tg, float step_size, float bc2s, bool store_g) {
    auto st = [&](float* base, const float4& x) {
        if (nv == 4) {
            *reinterpret_cast<float4*>(base + e) = x;
            return;
        }
        base[e] = x.x;
        if (nv > 1) base[e + 1] = x.y;
        if (nv > 2) base[e + 2] = x.z;
    };
    if (store_g) st(a.grads, g);
    if (a.mode == 0) return;
    adam4_compute(a, g, m, v, p, tg, step_size, bc2s);
    st(a.m, m);
    st(a.v, v);
    st(a.p, p);
    if (a.soft) st(a.target, tg);
}

__device__ __forceinline__ AdamSegment adam_segment_of(const AdamArgs& a, int64_t e) {
    // static-index selects (a kernel-argument array indexed by a per-lane value goes to scratch)
    AdamSegment sg = a.seg[0];
#pragma unroll
    for (int q = 1; q < kMaxSeg; q++)
        if (q < a.nseg && e >= a.seg[q].off) sg = a.seg[q];
    return sg;
}

// an out-of-range write skipped: sticky ctrl.error (the first site to report wins), raised by the host
// at its next synchronisation point (dqn.engine.raise_device_error)
__device__ __forceinline__ void adam_bounds_error(const AdamArgs& a, int site) {
    if (a.ctrl) __hip_atomic_store(&a.ctrl->error, (int32_t)site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_adam4(AdamArgs a) {
    if (adam_extra_wg(a)) return;   // the sampler-cache / staged-minibatch workgroups
    const int eb = (int)blockIdx.x - adam_extra_count(a);   // element block
    const int64_t P = a.n_params, P4 = (P + 3) >> 2;   // e0 is a multiple of 4 (launch_adam)
    if (eb == 0) {
        if (a.mode != 2 && threadIdx.x < 64 && a.loss_partial) {   // one wave, fixed order
            float s = 0.f;
            for (int j = threadIdx.x; j < a.n_loss_partial; j += 64) s += a.loss_partial[j];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
            if (threadIdx.x == 0) {
                const float loss = s / (float)a.batch_global;
                a.grads[P] = loss;
                a.ctrl->loss = loss;
            }
        }
        if (a.mode == 2 && a.with_loss && threadIdx.x == 0) a.ctrl->loss = a.grads[P];
    }
    float step_size = 0.f, bc2s = 1.f;
    if (a.mode != 0) {
        step_size = a.ctrl->adam_step_size;
        bc2s = a.ctrl->adam_bc2_sqrt;
    }
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t w0 = a.e0 >> 2, w4 = a.wide_end > a.e0 ? ((a.wide_end - a.e0) >> 2) : 0;
    const int wide_blocks = (int)((w4 * ADAM_WIDE + 255) / 256);
    if (eb < wide_blocks) {   // ---- wide segments: ADAM_WIDE lanes per float4 ----
        const int64_t gid = (int64_t)eb * 256 + threadIdx.x;
        const int64_t e4 = w0 + gid / ADAM_WIDE;
        const int j = (int)(gid % ADAM_WIDE);
        const bool live = e4 < w0 + w4;
        const int64_t e = (live ? e4 : w0) << 2;
        float4 m = z4, v = z4, p = z4, tg = z4;
        const bool perms = a.mode == 1 && a.nperm > 0;
        // with the permuted copies every lane of the group loads the operands (one transaction per
        // group) and computes the same update, so the stores below spread over the 8 lanes
        if (a.mode != 0 && (j == 0 || perms) && live) {
            m = ld4(a.m + e);
            v = ld4(a.v + e);
            p = ld4(a.p + e);
            if (a.soft || perms) tg = ld4(a.target + e);
        }
        const AdamSegment sg = adam_segment_of(a, e);
        const float* q4 = sg.partial + (e - sg.off);
        const int64_t ps = sg.pstride;
        float4 g = z4;
        const int cnt = live && j < sg.S ? (sg.S - j + ADAM_WIDE - 1) / ADAM_WIDE : 0;   // slabs j, j + W, ...
        if (cnt > 0 && cnt <= 4) {   // (up to 32 slabs: one round trip of 4 loads instead of 16, 12 of
                                     // them clamped; cnt = 0: slab j may not exist, nothing is loaded)
            float4 pv[4];
#pragma unroll
            for (int q = 0; q < 4; q++) pv[q] = ld4(q4 + (int64_t)(j + (q < cnt ? q : 0) * ADAM_WIDE) * ps);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (q >= cnt) break;
                if (q == 0) {
                    g = pv[q];
                } else {
                    g.x += pv[q].x; g.y += pv[q].y; g.z += pv[q].z; g.w += pv[q].w;
                }
            }
        }
        for (int u0 = 0; cnt > 4 && u0 < cnt; u0 += 16) {
            float4 pv[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {   // addresses clamped to slab j: the loads stay unconditional
                const int u = u0 + q < cnt ? u0 + q : 0;
                pv[q] = ld4(q4 + (int64_t)(j + u * ADAM_WIDE) * ps);
            }
#pragma unroll
            for (int q = 0; q < 16; q++) {
                if (u0 + q >= cnt) break;
                if (u0 + q == 0) {
                    g = pv[q];
                } else {
                    g.x += pv[q].x; g.y += pv[q].y; g.z += pv[q].z; g.w += pv[q].w;
                }
            }
        }
#pragma unroll
        for (int o = ADAM_WIDE / 2; o >= 1; o >>= 1) {   // (x + y == y + x: all lanes agree)
            g.x += __shfl_xor(g.x, o);
            g.y += __shfl_xor(g.y, o);
            g.z += __shfl_xor(g.z, o);
            g.w += __shfl_xor(g.w, o);
        }
        // bounds check (the bucketed DP step): a wide float4 lies inside this launch's
        // element range [e0, n_params) -- a DP bucket's range -- or its stores are skipped and the
        // sticky ctrl.error names the site (a write into another bucket's range would race with that
        // bucket's Adam on the other stream)
        if (live && (e < a.e0 || e + 4 > a.n_params)) {
            if (j == 0) adam_bounds_error(a, DQNX_DEVERR_BOUNDS_ADAM_WIDE);
            return;
        }
        if (live && !perms) {
            if (j == 0) adam4_update(a, e, 4, g, m, v, p, tg, step_size, bc2s, true);
        } else if (live) {
            // every lane: the same update; lane j < 4 writes element j's three permuted copies, lanes
            // 4..7 the float4s of grads / m / v / p (+ target)
            adam4_compute(a, g, m, v, p, tg, step_size, bc2s);
            if (j < 4) {
                const float pv = j == 0 ? p.x : j == 1 ? p.y : j == 2 ? p.z : p.w;
                const float tv = j == 0 ? tg.x : j == 1 ? tg.y : j == 2 ? tg.z : tg.w;
#pragma unroll
                for (int l = 0; l < 2; l++) {
                    if (l >= a.nperm) continue;
                    const AdamArgs::PermLayer& L = a.perm[l];
                    const int K = L.Ci * 9;
                    const int64_t le = e + j - L.woff;
                    if (le < 0 || le >= (int64_t)L.Co * K) continue;   // (a layer's bias is not permuted)
                    const int co = (int)le / K, r = (int)le - co * K, ci = r / 9, t = r - ci * 9;
                    if (e + j >= a.n_params) {   // (a permuted copy of an element outside this range)
                        adam_bounds_error(a, DQNX_DEVERR_BOUNDS_ADAM_PERM);
                        continue;
                    }
                    L.p0[(co * 9 + t) * L.Ci + ci] = pv;
                    L.p1[(co * 9 + t) * L.Ci + ci] = tv;
                    L.pT[(ci * 9 + t) * L.Co + co] = pv;
                }
            } else if (j == 4) {
                *reinterpret_cast<float4*>(a.grads + e) = g;
                *reinterpret_cast<float4*>(a.m + e) = m;
            } else if (j == 5) {
                *reinterpret_cast<float4*>(a.v + e) = v;
            } else if (j == 6) {
                *reinterpret_cast<float4*>(a.p + e) = p;
            } else if (a.soft) {
                *reinterpret_cast<float4*>(a.target + e) = tg;
            }
        }
        return;
    }
    const int nb = eb - wide_blocks;
    const int64_t stride = (int64_t)(gridDim.x - adam_extra_count(a) - wide_blocks) * blockDim.x;
    for (int64_t e4 = w0 + w4 + (int64_t)nb * blockDim.x + threadIdx.x; e4 < P4; e4 += stride) {
        const int64_t e = e4 << 2;
        const int nv = (int)min((int64_t)4, P - e);   // 4 except in the last vector
        float4 m = z4, v = z4, p = z4, tg = z4, g = z4;
        auto ld = [&](const float* base) {   // the last vector may be partial (no dynamic indexing)
            if (nv == 4) return ld4(base + e);
            return make_float4(base[e], nv > 1 ? base[e + 1] : 0.f, nv > 2 ? base[e + 2] : 0.f, 0.f);
        };
        if (a.mode != 0) {
            m = ld(a.m);
            v = ld(a.v);
            p = ld(a.p);
            if (a.soft) tg = ld(a.target);
        }
        if (a.mode == 2) {
            g = ld(a.grads);
        } else {
            const AdamSegment sg = adam_segment_of(a, e);
            const float* pp = sg.partial + (e - sg.off) - e;   // ld() adds e back
            if (nv == 4) {
                // slab 0, then 16 / 4 / 1 slabs per round trip, every load of a round unconditional
                // (a conditional load would make the compiler wait for all of them before the
                // first add)
                const float* q4 = pp + e;
                const int64_t ps = sg.pstride;
                g = ld4(q4);
                int u = 1;
                for (; u + 16 <= sg.S; u += 16) {
                    float4 pv[16];
#pragma unroll
                    for (int j = 0; j < 16; j++) pv[j] = ld4(q4 + (int64_t)(u + j) * ps);
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        g.x += pv[j].x; g.y += pv[j].y; g.z += pv[j].z; g.w += pv[j].w;
                    }
                }
                for (; u + 4 <= sg.S; u += 4) {
                    float4 pv[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) pv[j] = ld4(q4 + (int64_t)(u + j) * ps);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        g.x += pv[j].x; g.y += pv[j].y; g.z += pv[j].z; g.w += pv[j].w;
                    }
                }
                for (; u < sg.S; u++) {
                    const float4 x = ld4(q4 + (int64_t)u * ps);
                    g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
                }
            } else {   // the last, partial vector
                for (int u = 0; u < sg.S; u++) {
                    const float4 x = ld(pp + (int64_t)u * sg.pstride);
                    if (u == 0) {
                        g = x;
                    } else {
                        g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w;
                    }
                }
            }
        }
        adam4_update(a, e, nv, g, m, v, p, tg, step_size, bc2s, a.mode != 2);
    }
}

// =====================================================================================
// Fused plan, fp32: weight gradients + Adam (+ soft update, + blocked copies) in one launch.
// One 512-thread workgroup per 16 x 16 parameter tile of a dense layer or the head; its 8 waves
// split the minibatch, every wave streams its rows of dZ and X straight into MFMA operands
// (an element of either feeds exactly one v_mfma_f32_16x16x4_f32 of a 16 x 16 tile, so nothing
// is staged in LDS), and the 8 partial tiles are summed through LDS in wave order: the gradient
// is final inside the workgroup (deterministic, no split-K slabs, no separate optimizer pass).
// Tiles with i-block 0 also sum dZ's column (the bias).  The epilogue is k_adam's per-element
// arithmetic, and writes the tile's fwd- / chain-blocked copies (one 16 x 16 block each), so
// the next step's forward needs no rebuild.  Reference: loss.backward() + optimizer.step()
// (R:dqn/agent.py:224-226), soft update R:dqn/agent.py:105-110.
// =====================================================================================
__device__ __forceinline__ int64_t dw16_index(const DwAdam16Layer& d, int row, int col) {
    if (d.head_kind < 0) return d.poff + ((col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row);
    return d.poff + ((col < d.in) ? (int64_t)head_w_off(d.head_kind, row, d.in) + col
                                  : (int64_t)head_b_off(d.head_kind, row, d.in, d.A));
}

// R: 16-row blocks of W per workgroup (a tile is 16 R x 16; every X element loaded feeds R MFMAs)
template <int DW16_NW, int U, int R>   // waves per tile; k-steps (4 rows each) per register set, two sets in flight
__global__ __launch_bounds__(64 * DW16_NW) void k_dw_adam16(DwAdam16Args a) {
    __shared__ floatx4 red[DW16_NW][R][64];
    __shared__ float redb[DW16_NW][R][64];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int i = lane & 15, g = lane >> 4;
    if ((int)blockIdx.x >= a.tiles) {   // extra workgroups: PER tracking, sampler cache, the staged-minibatch copy, PER prop
        const int x = (int)blockIdx.x - a.tiles - a.ptrack - (a.mtc ? 1 : 0) - (a.pf_nidx > 0 ? 1 : 0);
        if (x >= 0) {   // k_per_prop's body over 64 * DW16_NW updates (the red table as its LDS)
            if constexpr (sizeof(red) >= PER_TOP * sizeof(double)) {   // (launch_dw_adam16: 32 x 16 tiles only)
                if (a.ptrack) per_prop_wait(a.pprop, x * 64 * DW16_NW);   // the tracking workgroup of this launch first
                per_prop_block(a.pprop, x * 64 * DW16_NW, reinterpret_cast<double*>(&red[0][0][0]));
                DQNX_STAMP_WG(a.pprop.stamps, 52);
            }
        } else if (a.ptrack && (int)blockIdx.x == a.tiles) {   // k_per_update's tracking (dispatched
            // right after the tiles, before the prop workgroups that wait for it)
            if constexpr (sizeof(red) >= sizeof(PerTrackLds<64 * DW16_NW>)) {
                auto& tl = *reinterpret_cast<PerTrackLds<64 * DW16_NW>*>(&red[0][0][0]);
                per_track_block<64 * DW16_NW, 4>(a.pprop, tl);
                per_track_publish(a.pprop);
            }
        } else if (a.mtc && (int)blockIdx.x == a.tiles + a.ptrack) {
            mt_cache_extend(a.mtc, a.mtc_blocks);
        } else {
            // in-launch prefetch: the forward launch drew the next minibatch into the staging slot;
            // nothing after this launch reads the compute slot of this step, so it takes the new one
            for (int q = tid; q < a.pf_nidx; q += blockDim.x) a.pf_idx_dst[q] = a.pf_idx_src[q];
            for (int q = tid; q < a.pf_nphys; q += blockDim.x) a.pf_phys_dst[q] = a.pf_phys_src[q];
        }
        return;
    }
    DQNX_STAMP(a.stamps, 56);
    const int T = xcd_remap(blockIdx.x, a.tiles);
    // the tile's layer: every first-tile index read at once, then one (scalar) load of the layer
    // (a chain of per-layer selects serialises a kernel-argument round trip per layer)
    int li = 0;
#pragma unroll
    for (int q = 1; q <= DQNX_MAX_DENSE; q++) li += (q < a.nl && T >= a.L[q].t0) ? 1 : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const DwAdam16Layer d = a.L[li];
    const int t = T - d.t0;
    const int ob = t / d.ti, ib = t - ob * d.ti;
    const int o0 = ob * 16 * R, i0 = ib * 16;

    // (0) this thread's parameters: slot q = tid + j NT of the tile's 256 R weights (q < 256 R) and
    //     16 R biases (q = 256 R + row, tiles with ib == 0), with their optimizer state, fetched
    //     before the K loop so the latency hides under it
    constexpr int NW_ = 256 * R, NT = 64 * DW16_NW, NS = (NW_ + 16 * R + NT - 1) / NT;
    int row[NS], col[NS];
    bool own[NS];
    int64_t e[NS];
    float p[NS], m[NS], v[NS], tg[NS], ga[NS];
    const bool apply = a.mode == 3;   // the gradient is in `grads` already (all-reduced): no K loop
#pragma unroll
    for (int j = 0; j < NS; j++) {
        const int q = tid + j * NT;
        ga[j] = 0.f;
        if (q < NW_) {
            row[j] = o0 + (q >> 4);
            col[j] = i0 + (q & 15);
            own[j] = row[j] < d.out && col[j] < d.in;
        } else {
            row[j] = o0 + q - NW_;
            col[j] = d.in;
            own[j] = ib == 0 && q < NW_ + 16 * R && row[j] < d.out;
        }
        e[j] = own[j] ? dw16_index(d, row[j], col[j]) : 0;
        p[j] = m[j] = v[j] = tg[j] = 0.f;
        if (own[j] && a.mode) {
            p[j] = gld(a.p + e[j]);
            m[j] = gld(a.m + e[j]);
            v[j] = gld(a.v + e[j]);
            if (a.soft) tg[j] = gld(a.target + e[j]);
            if (apply) ga[j] = gld(a.grads + e[j]);
        }
    }
    const float step_size = gld(&a.ctrl->adam_step_size), bc2s = gld(&a.ctrl->adam_bc2_sqrt);
    DQNX_STAMP(a.stamps, 57);

    // (1) dW tile = dZ[:, o0:o0+16]^T X[:, i0:i0+16] over this wave's rows; lane (i, g) supplies
    //     dZ[b][o0 + i] and X[b][i0 + i] of row b = 4 s + g at k-step s.  Loads go through
    //     wave-uniform buffer descriptors bounded at Bl rows: rows past the batch read zero
    //     without a branch.  Columns past the layer are clamped (their accumulator rows /
    //     columns are never stored).  A wave owns a multiple of 2U k-steps, so the loop has no
    //     tail.
    const int nsteps = apply ? 0 : (a.Bl + 3) >> 2;
    const int spw = ((nsteps + DW16_NW - 1) / DW16_NW + 2 * U - 1) / (2 * U) * (2 * U);
    const int s0 = wid * spw;
    const int iters = s0 < nsteps ? spw / (2 * U) : 0;
    const __amdgpu_buffer_rsrc_t zr = wave_rsrc(d.dZ, (uint32_t)a.Bl * d.ldz * 4u);
    const __amdgpu_buffer_rsrc_t xr = wave_rsrc(d.X, (uint32_t)a.Bl * d.ldx * 4u);
    uint32_t zo[R];
#pragma unroll
    for (int r = 0; r < R; r++) zo[r] = (uint32_t)((4 * s0 + g) * d.ldz + min(o0 + 16 * r + i, d.out - 1)) * 4u;
    uint32_t xo = (uint32_t)((4 * s0 + g) * d.ldx + min(i0 + i, d.in - 1)) * 4u;
    const uint32_t zs = 16u * d.ldz, xs = 16u * d.ldx;   // bytes per k-step (4 rows)
    floatx4 acc[R];
    float bs[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
        bs[r] = 0.f;
    }
    float za[R][U], xa[U], zb[R][U], xb[U];
    auto load = [&](float (*z)[U], float* x) {
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
            for (int r = 0; r < R; r++)
                z[r][u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(zr, zo[r] + u * zs, 0, 0));
            x[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, xo + u * xs, 0, 0));
        }
#pragma unroll
        for (int r = 0; r < R; r++) zo[r] += U * zs;
        xo += U * xs;
    };
    auto comp = [&](const float (*z)[U], const float* x) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < R; r++) {
                acc[r] = mfma16x16x4(z[r][u], x[u], acc[r]);
                bs[r] += z[r][u];
            }
    };
    if (iters > 0) {
        load(za, xa);
        for (int it = 0;; it++) {
            load(zb, xb);
            __builtin_amdgcn_sched_barrier(0);
            comp(za, xa);
            __builtin_amdgcn_sched_barrier(0);
            if (it + 1 == iters) {   // (wave-uniform) no prefetch past the wave's rows
                comp(zb, xb);
                break;
            }
            load(za, xa);
            __builtin_amdgcn_sched_barrier(0);
            comp(zb, xb);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    DQNX_STAMP(a.stamps, 58);
#pragma unroll
    for (int r = 0; r < R; r++) {
        red[wid][r][lane] = acc[r];
        redb[wid][r][lane] = bs[r];
    }
    __syncthreads();

    DQNX_STAMP(a.stamps, 59);
    // (2) fixed-order sum of the wave partials, then k_adam's per-element update
#pragma unroll
    for (int j = 0; j < NS; j++) {
        if (!own[j]) continue;
        const int q = tid + j * NT;
        float gsum;
        if (apply) {
            gsum = ga[j];
        } else if (q < NW_) {   // row block r = q / 256 of the tile; the same order for every R
            const float* rf = reinterpret_cast<const float*>(&red[0][0][0]) + (q >> 8) * 256;
            const int qq = q & 255, rr = qq >> 4, off = ((rr >> 2) * 16 + (qq & 15)) * 4 + (rr & 3);
            gsum = rf[off];
#pragma unroll
            for (int w = 1; w < DW16_NW; w++) gsum += rf[w * 256 * R + off];
        } else {   // bias: lanes (i = row, g = 0..3) of every wave, wave-major
            const int rb = (q - NW_) >> 4, rr = (q - NW_) & 15;
            gsum = redb[0][rb][rr];
#pragma unroll
            for (int k = 1; k < 4 * DW16_NW; k++) gsum += redb[k >> 2][rb][(k & 3) * 16 + rr];
        }
        if (!apply) a.grads[e[j]] = gsum;
        if (!a.mode) continue;
        float mk = fmaf(a.w1, gsum - m[j], m[j]);
        float vk = v[j] * a.beta2;
        vk = vk + (a.c2 * gsum) * gsum;
        const float denom = sqrtf(vk) / bc2s + a.eps;
        const float pk = p[j] + (step_size * mk) / denom;
        a.m[e[j]] = mk;
        a.v[e[j]] = vk;
        a.p[e[j]] = pk;
        float tk = 0.f;
        if (a.soft) {
            tk = a.tau * pk + a.one_minus_tau * tg[j];
            a.target[e[j]] = tk;
        }
        if (q < NW_ && d.fwd_online) {   // the tile's blocks of the forward / dZ-chain copies
            const int64_t pf = blk_pos(row[j], col[j], d.nch_fwd, false);
            d.fwd_online[pf] = pk;
            if (a.soft) d.fwd_target[pf] = tk;
            if (d.chain) d.chain[blk_pos(col[j], row[j], d.nch_chain, false)] = pk;
        }
    }
    DQNX_STAMP(a.stamps, 60);
    if (apply && T == 0 && tid == 0) a.ctrl->loss = a.grads[a.n_params];   // (the all-reduced loss slot)
    if (!apply && T == 0 && wid == DW16_NW - 1 && a.loss_partial) {   // one wave, k_adam's fixed order
        float s = 0.f;
        for (int j = lane; j < a.n_loss_partial; j += 64) s += a.loss_partial[j];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) {
            const float loss = s / (float)a.batch_global;
            a.grads[a.n_params] = loss;
            a.ctrl->loss = loss;
        }
    }
}

int launch_dw_adam16(const DwAdam16Args& a, hipStream_t s) {
    static const int var = tuning_knob("DQNX_DW16_VAR", 0);
    if ((a.pprop_wgs || a.ptrack) && (a.rows16 != 2 || var != 0))
        return set_error(DQNX_EUNSUPPORTED, "dw_adam16: PER workgroups with the default 32 x 16 tiles only");
    if (a.ptrack && (a.pprop.n > PER_CHUNK || !a.pprop.sync || a.pprop_wgs < 1))
        return set_error(DQNX_EINVAL, "dw_adam16: PER tracking workgroup needs its prop workgroups and hand-off words");
    const dim3 grid(a.tiles + a.ptrack + (a.mtc ? 1 : 0) + (a.pf_nidx > 0 ? 1 : 0) + a.pprop_wgs);
    if (a.rows16 == 2) {
        switch (var) {   // measurement variants (waves per tile, k-steps per register set)
            case 7: DQNX_LAUNCH((k_dw_adam16<16, 4, 2>), grid, dim3(1024), 0, s, a); break;
            case 8: DQNX_LAUNCH((k_dw_adam16<8, 4, 2>), grid, dim3(512), 0, s, a); break;
            default: DQNX_LAUNCH((k_dw_adam16<8, 8, 2>), grid, dim3(512), 0, s, a); break;
        }
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    if (a.rows16 != 1) return set_error(DQNX_EINVAL, "dw_adam16: %d row blocks per tile", a.rows16);
    switch (var) {   // measurement variants (waves per tile, k-steps per register set)
        case 1: DQNX_LAUNCH((k_dw_adam16<4, 8, 1>), grid, dim3(256), 0, s, a); break;
        case 2: DQNX_LAUNCH((k_dw_adam16<16, 4, 1>), grid, dim3(1024), 0, s, a); break;
        case 3: DQNX_LAUNCH((k_dw_adam16<8, 4, 1>), grid, dim3(512), 0, s, a); break;
        case 4: DQNX_LAUNCH((k_dw_adam16<4, 16, 1>), grid, dim3(256), 0, s, a); break;
        case 5: DQNX_LAUNCH((k_dw_adam16<8, 16, 1>), grid, dim3(512), 0, s, a); break;
        case 6: DQNX_LAUNCH((k_dw_adam16<16, 8, 1>), grid, dim3(1024), 0, s, a); break;
        default: DQNX_LAUNCH((k_dw_adam16<8, 8, 1>), grid, dim3(512), 0, s, a); break;
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// two int32 arrays copied in one launch (the side-stream prefetch's staged minibatch over the compute
// slot: the sampled positions and their ring slots)
__global__ __launch_bounds__(256) void k_copy_i32x2(int32_t* __restrict__ d0, const int32_t* __restrict__ s0, int n0,
                                                    int32_t* __restrict__ d1, const int32_t* __restrict__ s1, int n1) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n0 + n1; i += gridDim.x * 256) {
        if (i < n0) d0[i] = s0[i];
        else d1[i - n0] = s1[i - n0];
    }
}
int launch_copy_i32x2(int32_t* d0, const int32_t* s0, int n0, int32_t* d1, const int32_t* s1, int n1, hipStream_t s) {
    const int n = n0 + n1;
    if (n <= 0) return DQNX_OK;
    const int blocks = std::min((n + 255) / 256, 256);
    DQNX_LAUNCH(k_copy_i32x2, dim3(blocks), dim3(256), 0, s, d0, s0, n0, d1, s1, n1);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

__global__ void k_soft_update(float* __restrict__ target, const float* __restrict__ p, int64_t n, float tau,
                              float omt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride)
        target[e] = tau * p[e] + omt * target[e];
}

// Replay push: rows [0, n) of the staged batch go to slots (wptr + i) % capacity.
__global__ void k_replay_push(PushArgs a) {
    const int row = blockIdx.x;
    if (row >= a.n) return;
    const int64_t slot = (a.wptr + row) % a.capacity;
    float* o = a.ring_obs + slot * a.stride;
    float* no = a.ring_next + slot * a.stride;
    const float* so = a.obs + (int64_t)row * a.obs_dim;
    const float* sn = a.next_obs + (int64_t)row * a.obs_dim;
    for (int j = threadIdx.x; j < a.obs_dim; j += blockDim.x) {
        o[j] = so[j];
        no[j] = sn[j];
    }
    if (a.ring16_obs) {   // bf16 engines: the rows' bf16 copies (RNE, as the forward rounds them), pad zero
        uint16_t* o16 = a.ring16_obs + slot * a.stride16;
        uint16_t* n16 = a.ring16_next + slot * a.stride16;
        for (int j = threadIdx.x; j < a.stride16; j += blockDim.x) {
            o16[j] = j < a.obs_dim ? bf16_bits(so[j]) : (uint16_t)0;
            n16[j] = j < a.obs_dim ? bf16_bits(sn[j]) : (uint16_t)0;
        }
    }
    if (threadIdx.x == 0) {
        a.ring_act[slot] = a.act[row];
        a.ring_rew[slot] = a.rew[row];
        a.ring_done[slot] = a.done[row] ? 1.f : 0.f;
    }
    if (row == 0 && threadIdx.x == 0) {
        a.ctrl->ring_size = a.new_size;
        a.ctrl->ring_wptr = a.new_wptr;
    }
}


// =====================================================================================
// host-side launchers
// =====================================================================================
// DQNX_FWD_ULOAD=1: the unconditional loader for dense rows (bit-identical; measured no faster on
// the HEAD net's dense 2 in round 5: opt-in)
template <int ACT, bool VECB>
static void launch_fwd_gather(const FwdArgs& a, dim3 grid, hipStream_t s) {
    bool u = VECB && !a.p[0].phys && a.K % 4 == 0 && route_knob("DQNX_FWD_ULOAD", 0) != 0;
    for (int z = 0; z < a.nprob; z++)
        u = u && a.p[z].lda % 4 == 0 && ((uintptr_t)a.p[z].A & 15) == 0 && ((uintptr_t)a.p[z].W & 15) == 0;
    if (a.p[0].phys) DQNX_LAUNCH((k_linear_fwd<ACT, VECB, true>), grid, dim3(256), 0, s, a);
    else if (u) DQNX_LAUNCH((k_linear_fwd<ACT, true, false, true>), grid, dim3(256), 0, s, a);
    else DQNX_LAUNCH((k_linear_fwd<ACT, VECB, false>), grid, dim3(256), 0, s, a);
}

int launch_linear_fwd(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s) {
    FwdArgs a2 = args;
    a2.nprob = nprob;
    dim3 grid(((args.N + FWD_BN - 1) / FWD_BN) * ((args.M + FWD_BM - 1) / FWD_BM) * nprob);
    if (act == DQNX_ACT_RELU) {
        if (vecb) launch_fwd_gather<DQNX_ACT_RELU, true>(a2, grid, s);
        else launch_fwd_gather<DQNX_ACT_RELU, false>(a2, grid, s);
    } else {
        if (vecb) launch_fwd_gather<DQNX_ACT_ELU, true>(a2, grid, s);
        else launch_fwd_gather<DQNX_ACT_ELU, false>(a2, grid, s);
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int fwd_big_ksplit(int M, int N, int K, int nprob, int64_t partial_floats, int* kchunk) {
    const int tiles = ((N + FWD_BIG_BN - 1) / FWD_BIG_BN) * ((M + FWD_BIG_BM - 1) / FWD_BIG_BM) * nprob;
    const int Kpad = (K + 3) & ~3;
    int S = std::max(1, std::min((512 + tiles - 1) / tiles, Kpad / (8 * FWD_BIG_KT)));
    while (S > 1 && (int64_t)S * nprob * M * N > partial_floats) S--;
    int kc = (Kpad + S - 1) / S;
    kc = (kc + FWD_BIG_KT - 1) / FWD_BIG_KT * FWD_BIG_KT;
    S = (Kpad + kc - 1) / kc;
    *kchunk = kc;
    return S;
}

template <int BM, int BN, int WM>
static void launch_fwd_big_t(const FwdArgs& a, int act, bool vecb, hipStream_t s) {
    const int tiles = ((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM) * a.nprob;
    const dim3 grid(tiles * a.ksplit);
    if (act == DQNX_ACT_RELU) {
        if (vecb) DQNX_LAUNCH((k_linear_fwd_big<DQNX_ACT_RELU, true, BM, BN, WM>), grid, dim3(256), 0, s, a);
        else DQNX_LAUNCH((k_linear_fwd_big<DQNX_ACT_RELU, false, BM, BN, WM>), grid, dim3(256), 0, s, a);
    } else {
        if (vecb) DQNX_LAUNCH((k_linear_fwd_big<DQNX_ACT_ELU, true, BM, BN, WM>), grid, dim3(256), 0, s, a);
        else DQNX_LAUNCH((k_linear_fwd_big<DQNX_ACT_ELU, false, BM, BN, WM>), grid, dim3(256), 0, s, a);
    }
}

int launch_linear_fwd_big(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s) {
    FwdArgs a2 = args;
    a2.nprob = nprob;
    if (a2.ksplit < 1) a2.ksplit = 1;
    if (a2.ksplit == 1) a2.kchunk = (args.K + 3) & ~3;
    // tile width follows N (conv Cout 32 / 64): no MFMA work on padding columns
    if (a2.ksplit == 1 && args.N <= 32) launch_fwd_big_t<128, 32, 4>(a2, act, vecb, s);
    else if (a2.ksplit == 1 && args.N <= 64) launch_fwd_big_t<128, 64, 2>(a2, act, vecb, s);
    else launch_fwd_big_t<FWD_BIG_BM, FWD_BIG_BN, 2>(a2, act, vecb, s);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

constexpr int FWD_SPLIT_T = 64, FWD_SPLIT_KT = 64;
int fwd_split_ksplit(int M, int N, int K, int nprob, int n_cu, int* kchunk) {
    const int tiles = ((N + FWD_SPLIT_T - 1) / FWD_SPLIT_T) * ((M + FWD_SPLIT_T - 1) / FWD_SPLIT_T) * nprob;
    const int Kpad = (K + 3) & ~3;
    // slabs: whole KT passes (a slab's last pass must not run into the next slab's K range)
    int S = std::max(1, std::min(2 * n_cu / tiles, Kpad / (2 * FWD_SPLIT_KT)));
    int kc = (Kpad + S - 1) / S;
    kc = (kc + FWD_SPLIT_KT - 1) / FWD_SPLIT_KT * FWD_SPLIT_KT;
    S = (Kpad + kc - 1) / kc;
    *kchunk = kc;
    return S;
}

template <int ACT>
static void launch_fwd_split_t(const FwdArgs& a2, bool vecb, dim3 grid, hipStream_t s) {
    constexpr int T = FWD_SPLIT_T, KT = FWD_SPLIT_KT;
    // unconditional operand loads (exact vmcnt waits): A = the dense input rows (float4), B = the
    // weight rows as float4, or as float2 pairs where the rows are only 8-byte aligned (the HEAD
    // net's K = 1358); odd strides keep the scalar loader
    bool a4 = route_knob("DQNX_F1_ULOAD", 1) != 0, b2 = a4 && !vecb && a2.K % 2 == 0;
    for (int z = 0; z < a2.nprob; z++) {
        a4 = a4 && a2.p[z].lda % 4 == 0 && ((uintptr_t)a2.p[z].A & 15) == 0;
        b2 = b2 && ((uintptr_t)a2.p[z].W & 7) == 0;
    }
    // ... optionally with two passes in flight (DQNX_F1_PF=2)
    const bool pf2 = route_knob("DQNX_F1_PF", 1) == 2;   // (measured 1 us slower at the HEAD net: opt-in)
    if (a4 && vecb && pf2) DQNX_LAUNCH((k_linear_fwd_big<ACT, true, T, T, 2, KT, L_ROWS_KU, L_ROWS_KU, 2>), grid, dim3(256), 0, s, a2);
    else if (a4 && b2 && pf2) DQNX_LAUNCH((k_linear_fwd_big<ACT, false, T, T, 2, KT, L_ROWS_KU, L_ROWS_K2, 2>), grid, dim3(256), 0, s, a2);
    else if (a4 && vecb) DQNX_LAUNCH((k_linear_fwd_big<ACT, true, T, T, 2, KT, L_ROWS_KU, L_ROWS_KU>), grid, dim3(256), 0, s, a2);
    else if (a4 && b2) DQNX_LAUNCH((k_linear_fwd_big<ACT, false, T, T, 2, KT, L_ROWS_KU, L_ROWS_K2>), grid, dim3(256), 0, s, a2);
    else if (vecb) DQNX_LAUNCH((k_linear_fwd_big<ACT, true, T, T, 2, KT>), grid, dim3(256), 0, s, a2);
    else DQNX_LAUNCH((k_linear_fwd_big<ACT, false, T, T, 2, KT>), grid, dim3(256), 0, s, a2);
}
int launch_linear_fwd_split(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s) {
    FwdArgs a2 = args;
    a2.nprob = nprob;
    constexpr int T = FWD_SPLIT_T;
    const int tiles = ((a2.N + T - 1) / T) * ((a2.M + T - 1) / T) * nprob;
    const dim3 grid(tiles * a2.ksplit);
    if (act == DQNX_ACT_RELU) launch_fwd_split_t<DQNX_ACT_RELU>(a2, vecb, grid, s);
    else launch_fwd_split_t<DQNX_ACT_ELU>(a2, vecb, grid, s);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_linear_fwd_reduce(const FwdArgs& args, int nprob, int act, hipStream_t s) {
    FwdArgs a2 = args;
    a2.nprob = nprob;
    int64_t g = ((int64_t)args.M * args.N * nprob + 255) / 256;
    if (g > 4096) g = 4096;
    if (act == DQNX_ACT_RELU) DQNX_LAUNCH((k_linear_fwd_reduce<DQNX_ACT_RELU>), dim3((unsigned)g), dim3(256), 0, s, a2);
    else DQNX_LAUNCH((k_linear_fwd_reduce<DQNX_ACT_ELU>), dim3((unsigned)g), dim3(256), 0, s, a2);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

void bwd_level_grid(BwdArgs& a) {
    const int BM = a.ts ? a.ts : BWD_BM, BN = a.ts ? a.ts : BWD_BN;
    if (a.dZprev) {
        a.dx_grid_x = (a.in + BN - 1) / BN;
        a.dx_blocks = a.dx_grid_x * ((a.Bl + BM - 1) / BM);
    } else {
        a.dx_grid_x = 1;
        a.dx_blocks = 0;
    }
    for (int p = 0; p < a.ndw; p++) {
        DwProblem& d = a.dw[p];
        d.grid_x = (d.in + 1 + BN - 1) / BN;
        d.grid_y = (d.out + BM - 1) / BM;
        d.blocks = d.grid_x * d.grid_y * a.dw_slices;
    }
}

template <int ACT>
static void launch_bwd_level_t(const BwdArgs& a, int blocks, hipStream_t s) {
    const bool vw = (a.in % 4) == 0;
    // unconditional loads where every operand meets its loader's alignment: dZ / X rows as float4
    // (row strides multiples of 4, 16-byte bases), the dx role's weight rows as float4 or pairs
    bool u = route_knob("DQNX_BWD_ULOAD", 1) != 0 && (vw || (a.in % 2 == 0 && ((uintptr_t)a.W & 7) == 0));
    if (a.dx_blocks) u = u && a.out % 4 == 0 && ((uintptr_t)a.dZ & 15) == 0 && (!vw || ((uintptr_t)a.W & 15) == 0);
    for (int p = 0; p < a.ndw; p++)
        u = u && a.dw[p].ldz % 4 == 0 && a.dw[p].ldx % 4 == 0 && ((uintptr_t)a.dw[p].dZ & 15) == 0 &&
            ((uintptr_t)a.dw[p].X & 15) == 0;
    if (a.ts == 64 && u && vw) DQNX_LAUNCH((k_bwd_level<ACT, true, true, 64>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.ts == 64 && u) DQNX_LAUNCH((k_bwd_level<ACT, false, true, 64>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.ts == 64 && vw) DQNX_LAUNCH((k_bwd_level<ACT, true, false, 64>), dim3(blocks), dim3(256), 0, s, a);
    else if (a.ts == 64) DQNX_LAUNCH((k_bwd_level<ACT, false, false, 64>), dim3(blocks), dim3(256), 0, s, a);
    else if (u && vw) DQNX_LAUNCH((k_bwd_level<ACT, true, true>), dim3(blocks), dim3(256), 0, s, a);
    else if (u) DQNX_LAUNCH((k_bwd_level<ACT, false, true>), dim3(blocks), dim3(256), 0, s, a);
    else if (vw) DQNX_LAUNCH((k_bwd_level<ACT, true>), dim3(blocks), dim3(256), 0, s, a);
    else DQNX_LAUNCH((k_bwd_level<ACT, false>), dim3(blocks), dim3(256), 0, s, a);
}
int launch_bwd_level(const BwdArgs& a, int act, hipStream_t s) {
    int blocks = a.dx_blocks;
    for (int p = 0; p < a.ndw; p++) blocks += a.dw[p].blocks;
    if (act == DQNX_ACT_RELU) launch_bwd_level_t<DQNX_ACT_RELU>(a, blocks, s);
    else launch_bwd_level_t<DQNX_ACT_ELU>(a, blocks, s);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

template <int F>
static void launch_head_f(const HeadArgs& a, int act, int tiles, hipStream_t s) {
    if (act == DQNX_ACT_RELU) DQNX_LAUNCH((k_head<DQNX_ACT_RELU, F>), dim3(tiles), dim3(256), 0, s, a);
    else DQNX_LAUNCH((k_head<DQNX_ACT_ELU, F>), dim3(tiles), dim3(256), 0, s, a);
}

bool head_supported(int F) { return F == 64 || F == 128 || F == 256; }

int launch_head(const HeadArgs& a, int act, hipStream_t s) {
    const int tiles = (a.Bl + 15) / 16;
    switch (a.F) {
        case 64: launch_head_f<64>(a, act, tiles, s); break;
        case 128: launch_head_f<128>(a, act, tiles, s); break;
        case 256: launch_head_f<256>(a, act, tiles, s); break;
        default: return set_error(DQNX_EUNSUPPORTED, "head input width %d not in {64,128,256}", a.F);
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// the float4 kernel when every segment is 4-aligned (offsets, slab strides, pointers) and no
// blocked copies ride along; DQNX_ADAM_VEC=0 keeps the scalar kernel
static bool adam_vec_ok(const AdamArgs& a) {
    if (tuning_knob("DQNX_ADAM_VEC", 1) == 0) return false;
    if (a.nblk || a.e0 % 4) return false;
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!al(a.p) || !al(a.m) || !al(a.v) || !al(a.grads) || (a.target && !al(a.target))) return false;
    for (int i = 0; i < a.nseg; i++)
        if (a.seg[i].off % 4 || (a.mode != 2 && (a.seg[i].pstride % 4 || !al(a.seg[i].partial)))) return false;
    return true;
}

bool adam_writes_perms(const AdamArgs& a) {
    if (a.nperm <= 0 || a.mode != 1 || a.e0 != 0 || !adam_vec_ok(a)) return false;
    int64_t end = 0;   // the wide prefix must cover every perm layer
    for (int q = 0; q < a.nseg && a.seg[q].wide; q++) end = q + 1 < a.nseg ? a.seg[q + 1].off : a.n_params;
    for (int l = 0; l < a.nperm; l++)
        if (a.perm[l].woff + (int64_t)a.perm[l].Co * a.perm[l].Ci * 9 > end) return false;
    return end % 4 == 0;
}

int launch_adam(const AdamArgs& a_in, hipStream_t s) {
    AdamArgs a = a_in;
    if (!adam_writes_perms(a)) a.nperm = 0;
    const bool vec = adam_vec_ok(a);
    // the wide prefix (k_adam4): the leading segments of the range with >= ADAM_WIDE_MIN_S slabs
    a.wide_end = 0;
    if (vec && a.mode != 2) {
        int q = 0;
        while (q + 1 < a.nseg && a.seg[q + 1].off <= a.e0) q++;
        int64_t end = a.e0;
        for (; q < a.nseg && a.seg[q].wide; q++) end = q + 1 < a.nseg ? a.seg[q + 1].off : a.n_params;
        if (end > a.n_params) end = a.n_params;
        if (end > a.e0 && end % 4 == 0) a.wide_end = end;
    }
    const int64_t wide4 = a.wide_end > a.e0 ? (a.wide_end - a.e0) / 4 : 0;
    const int64_t items = vec ? (a.n_params - a.e0 + 3) / 4 - wide4 : a.n_params - a.e0;
    int blocks = (int)((items + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    blocks += (int)((wide4 * 8 + 255) / 256);   // ADAM_WIDE lanes per wide float4
    if (a.mtc) blocks++;   // + the sampler-cache workgroup
    if (a.pf_nidx > 0) blocks++;   // + the staged-minibatch copy
    blocks += a.pprop_wgs;         // + k_per_prop's workgroups (256 updates each)
    if (vec) DQNX_LAUNCH(k_adam4, dim3(blocks), dim3(256), 0, s, a);
    else DQNX_LAUNCH(k_adam, dim3(blocks), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_soft_update(float* target, const float* p, int64_t n, float tau, float omt, hipStream_t s) {
    int blocks = (int)((n + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    DQNX_LAUNCH(k_soft_update, dim3(blocks), dim3(256), 0, s, target, p, n, tau, omt);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_replay_push(const PushArgs& a, hipStream_t s) {
    if (a.n <= 0) return DQNX_OK;
    DQNX_LAUNCH(k_replay_push, dim3(a.n), dim3(128), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
