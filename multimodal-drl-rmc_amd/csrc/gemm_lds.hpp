// LDS-staged fp32 MFMA GEMM tiles for the learn step's small GEMMs (gfx950).
//
// A 256-thread workgroup stages a K pass of its A and B tiles in LDS with every lane's
// float4 loads issued before the first wait (full-line, lane-contiguous loads: one
// round trip per pass), prefetches the next pass into registers while the current one is
// multiplied, and reads MFMA fragments from LDS:
//   ROWS_K image [rows][KT+8]  (K contiguous)  -> one ds_read_b128 per fragment
//   K_ROWS image [KT][cols+4]  (K strided)     -> four ds_read_b32 per fragment
// (paddings chosen conflict-free for the b128 / b32 lane groups of MI355X_MICROARCH §LDS).
// MFMA jj of a 16-deep chunk consumes k = kk + 4*(lane>>4) + jj for both operands.
// Measured against the wave-split-K engine (gemm_sk.hpp) in profiles/r01_*: this one is
// faster for every GEMM of the MLP learn step (fragment-shaped global loads cost more
// than the LDS round trip).
#pragma once
#include "gemm_common.hpp"

namespace dqnx {

template <int R, int KT, bool VEC>
struct StageRowsK {
    static constexpr int S = KT + 8;                 // LDS row stride (floats)
    static constexpr int Q4 = KT / 4;                // float4 per row
    static constexpr int NQ = (R * Q4 + 255) / 256;  // float4 slots per thread
    static constexpr int LDS_FLOATS = R * S;
    float4 v[NQ];

    __device__ __forceinline__ void load(const Operand& o, int r0, int kb) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < R * Q4) {
                const int r = q / Q4, k = kb + 4 * (q - r * Q4);
                const int gr = r0 + r;
                if (gr < o.nrows && k < o.K) {
                    const int64_t row = o.gather ? (int64_t)o.gather[gr] : (int64_t)gr;
                    const float* p = o.base + row * o.ld + k;
                    if (VEC) {
                        x = ld4(p);
                    } else {
                        x.x = p[0];
                        x.y = (k + 1 < o.K) ? p[1] : 0.f;
                        x.z = (k + 2 < o.K) ? p[2] : 0.f;
                        x.w = (k + 3 < o.K) ? p[3] : 0.f;
                    }
                }
            }
            v[j] = x;
        }
    }
    __device__ __forceinline__ void store(float* lds, const Operand& o, int r0, int kb) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            if (q < R * Q4) {
                const int r = q / Q4, c = 4 * (q - r * Q4);
                *reinterpret_cast<float4*>(lds + r * S + c) = v[j];
                if (o.copy && r0 + r < o.nrows && kb + c < o.K)
                    *reinterpret_cast<float4*>(o.copy + (int64_t)(r0 + r) * o.ldcopy + kb + c) = v[j];
            }
        }
    }
    __device__ __forceinline__ void frag(const float* lds, int rw, int kk, float (&f)[4]) const {
        const int lane = threadIdx.x & 63;
        const float4 x = *reinterpret_cast<const float4*>(lds + (rw + (lane & 15)) * S + kk + 4 * (lane >> 4));
        f[0] = x.x; f[1] = x.y; f[2] = x.z; f[3] = x.w;
    }
};

template <int C, int KT, bool VEC = true>
struct StageKRows {
    static constexpr int S = C + 4;
    static constexpr int C4 = C / 4;
    static constexpr int NQ = (KT * C4 + 255) / 256;
    static constexpr int LDS_FLOATS = KT * S;
    float4 v[NQ];

    __device__ __forceinline__ void load(const Operand& o, int c0, int kb) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < KT * C4) {
                const int kr = q / C4, c = c0 + 4 * (q - kr * C4);
                const int k = kb + kr;
                if (k < o.K && c < o.nrows) {
                    const float* p = o.base + (int64_t)k * o.ld + c;
                    if (VEC) {   // row stride and column count multiples of 4
                        x = ld4(p);
                    } else {
                        x.x = p[0];
                        x.y = (c + 1 < o.nrows) ? p[1] : 0.f;
                        x.z = (c + 2 < o.nrows) ? p[2] : 0.f;
                        x.w = (c + 3 < o.nrows) ? p[3] : 0.f;
                    }
                }
            }
            v[j] = x;
        }
    }
    __device__ __forceinline__ void store(float* lds, const Operand&, int, int) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j;
            if (q < KT * C4) {
                const int kr = q / C4, c = 4 * (q - kr * C4);
                *reinterpret_cast<float4*>(lds + kr * S + c) = v[j];
            }
        }
    }
    __device__ __forceinline__ void frag(const float* lds, int cw, int kk, float (&f)[4], int col_abs, int aug) const {
        const int lane = threadIdx.x & 63;
        const float* p = lds + (kk + 4 * (lane >> 4)) * S + cw + (lane & 15);
        if (col_abs == aug) {
            f[0] = f[1] = f[2] = f[3] = 1.f;
        } else {
            f[0] = p[0]; f[1] = p[S]; f[2] = p[2 * S]; f[3] = p[3 * S];
        }
    }
};

// ROWS_K image, unconditional loads (L_ROWS_KU: float4, L_ROWS_K2: float2 pairs)
template <int R, int KT, bool PAIR>
struct StageRowsKU : StageRowsK<R, KT, true> {
    using Base = StageRowsK<R, KT, true>;
    using Base::NQ;
    using Base::Q4;
    __device__ __forceinline__ void load(const Operand& o, int r0, int kb) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j, qc = q < R * Q4 ? q : 0;
            const int r = qc / Q4, k = kb + 4 * (qc - r * Q4), gr = r0 + r;
            const int grc = min(gr, o.nrows - 1);
            const float* row = o.base + (int64_t)grc * o.ld;
            const bool v = q < R * Q4 && gr < o.nrows;
            float4 x;
            // an element outside the operand reads offset 0 of the row instead (any valid address)
            if (PAIR) {   // pairs (k, k+1), (k+2, k+3); K even: a pair is wholly in or out
                const bool vl = v && k < o.K, vh = v && k + 2 < o.K;
                const float2 lo = *reinterpret_cast<const float2*>(row + (vl ? k : 0));
                const float2 hi = *reinterpret_cast<const float2*>(row + (vh ? k + 2 : 0));
                x = make_float4(vl ? lo.x : 0.f, vl ? lo.y : 0.f, vh ? hi.x : 0.f, vh ? hi.y : 0.f);
            } else {
                const bool vk = v && k < o.K;
                const float4 y = ld4(row + (vk ? k : 0));
                x = vk ? y : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            this->v[j] = x;
        }
    }
};

// K_ROWS image, unconditional loads (L_K_ROWSU: float4 as StageKRows<VEC = true>, L_K_ROWS2:
// float2 pairs, ld and the column count even)
template <int C, int KT, bool PAIR>
struct StageKRowsU : StageKRows<C, KT, true> {
    using Base = StageKRows<C, KT, true>;
    using Base::NQ;
    using Base::C4;
    __device__ __forceinline__ void load(const Operand& o, int c0, int kb) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int j = 0; j < NQ; j++) {
            const int q = tid + 256 * j, qc = q < KT * C4 ? q : 0;
            const int kr = qc / C4, c = c0 + 4 * (qc - kr * C4), k = kb + kr;
            const bool v = q < KT * C4 && k < o.K;
            const float* row = o.base + (int64_t)(v ? k : 0) * o.ld;
            float4 x;
            if (PAIR) {
                const bool vl = v && c < o.nrows, vh = v && c + 2 < o.nrows;
                const float2 lo = *reinterpret_cast<const float2*>(row + (vl ? c : 0));
                const float2 hi = *reinterpret_cast<const float2*>(row + (vh ? c + 2 : 0));
                x = make_float4(vl ? lo.x : 0.f, vl ? lo.y : 0.f, vh ? hi.x : 0.f, vh ? hi.y : 0.f);
            } else {
                const bool vc = v && c < o.nrows;
                const float4 y = ld4(row + (vc ? c : 0));
                x = vc ? y : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            this->v[j] = x;
        }
    }
};

template <int LAYOUT, int R, int KT, bool VEC>
struct Stage;
template <int R, int KT, bool VEC>
struct Stage<L_ROWS_K, R, KT, VEC> : StageRowsK<R, KT, VEC> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int, int) const {
        this->frag(lds, rw, kk, f);
    }
};
template <int R, int KT, bool VEC>
struct Stage<L_ROWS_KU, R, KT, VEC> : StageRowsKU<R, KT, false> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int, int) const {
        this->frag(lds, rw, kk, f);
    }
};
template <int R, int KT, bool VEC>
struct Stage<L_ROWS_K2, R, KT, VEC> : StageRowsKU<R, KT, true> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int, int) const {
        this->frag(lds, rw, kk, f);
    }
};
template <int R, int KT, bool VEC>
struct Stage<L_K_ROWSU, R, KT, VEC> : StageKRowsU<R, KT, false> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int col_abs,
                                          int aug) const {
        this->frag(lds, rw, kk, f, col_abs, aug);
    }
};
template <int R, int KT, bool VEC>
struct Stage<L_K_ROWS2, R, KT, VEC> : StageKRowsU<R, KT, true> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int col_abs,
                                          int aug) const {
        this->frag(lds, rw, kk, f, col_abs, aug);
    }
};
template <int R, int KT, bool VEC>
struct Stage<L_K_ROWS, R, KT, VEC> : StageKRows<R, KT, VEC> {
    __device__ __forceinline__ void fragx(const float* lds, int rw, int kk, float (&f)[4], int col_abs,
                                          int aug) const {
        this->frag(lds, rw, kk, f, col_abs, aug);
    }
};

// Workgroup tile: BM x BN outputs, 4 waves as WM x WN, each wave TM x TN 16x16 sub-tiles,
// K range [kbeg, kend) in passes of KT.  acc[tm][tn] lane l holds
// C[m0 + (wm*TM + tm)*16 + 4*(l>>4) + r][n0 + (wn*TN + tn)*16 + (l&15)], r = 0..3.
template <int BM, int BN, int KT, int WM, int WN, int LA, int LB, bool VA, bool VB>
struct TileGemm {
    static constexpr int TM = BM / (WM * 16), TN = BN / (WN * 16);
    static_assert(WM * WN == 4, "4 waves per workgroup");
    static_assert(TM * 16 * WM == BM && TN * 16 * WN == BN, "tile shape");
    static_assert(KT % 16 == 0, "KT multiple of 16");
    using SA = Stage<LA, BM, KT, VA>;
    using SB = Stage<LB, BN, KT, VB>;
    static constexpr int LDS_FLOATS = SA::LDS_FLOATS + SB::LDS_FLOATS;

    __device__ __forceinline__ static void run(float* lds, const Operand& A, const Operand& B, int m0, int n0,
                                               int kbeg, int kend, floatx4 (&acc)[TM][TN]) {
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int wm = wid / WN, wn = wid % WN;
        float* la = lds;
        float* lb = lds + SA::LDS_FLOATS;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
        SA sa;
        SB sb;
        int kb = kbeg;
        if (kb >= kend) return;
        sa.load(A, m0, kb);
        sb.load(B, n0, kb);
        sa.store(la, A, m0, kb);
        sb.store(lb, B, n0, kb);
        __syncthreads();
        while (true) {
            const int klen = min(KT, kend - kb);
            const int kn = kb + KT;
            const bool more = kn < kend;
            if (more) {   // next pass in flight while this one is multiplied
                sa.load(A, m0, kn);
                sb.load(B, n0, kn);
            }
            for (int kk = 0; kk < klen; kk += 16) {
                float a[TM][4], b[TN][4];
#pragma unroll
                for (int tm = 0; tm < TM; tm++) sa.fragx(la, (wm * TM + tm) * 16, kk, a[tm], -1, -2);
#pragma unroll
                for (int tn = 0; tn < TN; tn++) {
                    const int cw = (wn * TN + tn) * 16;
                    sb.fragx(lb, cw, kk, b[tn], n0 + cw + (lane & 15), B.aug);
                }
#pragma unroll
                for (int jj = 0; jj < 4; jj++)
#pragma unroll
                    for (int tm = 0; tm < TM; tm++)
#pragma unroll
                        for (int tn = 0; tn < TN; tn++)
                            acc[tm][tn] = mfma16x16x4(a[tm][jj], b[tn][jj], acc[tm][tn]);
            }
            if (!more) break;
            __syncthreads();
            sa.store(la, A, m0, kn);
            sb.store(lb, B, n0, kn);
            __syncthreads();
            kb = kn;
        }
    }

    // run() with two passes in flight: pass k+2's loads are issued before pass k is multiplied and
    // stored to LDS only after pass k+1 (two register sets under fixed names, the loop unrolled by
    // two).  Same LDS image per pass and same MFMA order: bit-identical to run().
    __device__ __forceinline__ static void mma_pass(const float* la, const float* lb, const SA& sa, const SB& sb,
                                                    const Operand& B, int n0, int klen, floatx4 (&acc)[TM][TN]) {
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int wm = wid / WN, wn = wid % WN;
        for (int kk = 0; kk < klen; kk += 16) {
            float a[TM][4], b[TN][4];
#pragma unroll
            for (int tm = 0; tm < TM; tm++) sa.fragx(la, (wm * TM + tm) * 16, kk, a[tm], -1, -2);
#pragma unroll
            for (int tn = 0; tn < TN; tn++) {
                const int cw = (wn * TN + tn) * 16;
                sb.fragx(lb, cw, kk, b[tn], n0 + cw + (lane & 15), B.aug);
            }
#pragma unroll
            for (int jj = 0; jj < 4; jj++)
#pragma unroll
                for (int tm = 0; tm < TM; tm++)
#pragma unroll
                    for (int tn = 0; tn < TN; tn++) acc[tm][tn] = mfma16x16x4(a[tm][jj], b[tn][jj], acc[tm][tn]);
        }
    }
    __device__ __forceinline__ static void run2(float* lds, const Operand& A, const Operand& B, int m0, int n0,
                                                int kbeg, int kend, floatx4 (&acc)[TM][TN]) {
        float* la = lds;
        float* lb = lds + SA::LDS_FLOATS;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
        SA a0, a1;
        SB b0, b1;
        int kb = kbeg;
        if (kb >= kend) return;
        a0.load(A, m0, kb);
        b0.load(B, n0, kb);
        if (kb + KT < kend) {
            a1.load(A, m0, kb + KT);
            b1.load(B, n0, kb + KT);
        }
        a0.store(la, A, m0, kb);
        b0.store(lb, B, n0, kb);
        __syncthreads();
        while (true) {
            // LDS: pass kb; set 1: pass kb + KT (if any); set 0 <- pass kb + 2 KT
            if (kb + 2 * KT < kend) {
                a0.load(A, m0, kb + 2 * KT);
                b0.load(B, n0, kb + 2 * KT);
            }
            mma_pass(la, lb, a1, b1, B, n0, min(KT, kend - kb), acc);
            if (kb + KT >= kend) break;
            __syncthreads();
            a1.store(la, A, m0, kb + KT);
            b1.store(lb, B, n0, kb + KT);
            __syncthreads();
            kb += KT;
            // LDS: pass kb; set 0: pass kb + KT (if any); set 1 <- pass kb + 2 KT
            if (kb + 2 * KT < kend) {
                a1.load(A, m0, kb + 2 * KT);
                b1.load(B, n0, kb + 2 * KT);
            }
            mma_pass(la, lb, a0, b0, B, n0, min(KT, kend - kb), acc);
            if (kb + KT >= kend) break;
            __syncthreads();
            a0.store(la, A, m0, kb + KT);
            b0.store(lb, B, n0, kb + KT);
            __syncthreads();
            kb += KT;
        }
    }
};

}  // namespace dqnx
