// Wave-split-K fp32 MFMA tiles for the learn step's latency-bound GEMMs (gfx950).
//
// Measured (profiles/r01_*): with LDS-staged K passes the small GEMMs of a learn step sit
// on a chain of dependent global round trips (row index -> row data -> LDS -> MFMA chain
// -> next pass), and bigger per-wave tiles only made it worse.  Here a workgroup of NWV
// waves owns one BM x BN output tile and splits K across its waves: each wave loads its
// WHOLE K range for the whole tile straight into registers (every load issued before the
// first wait, one round trip per KW-deep round), runs TM*TN independent accumulator chains
// (pipelined MFMA issue), and the waves' partial tiles are summed through LDS in a fixed
// order (w = 0, 1, ..., NWV-1), so results are deterministic.  Wave 0 ends with the tile.
//
// Fragment convention (v_mfma_f32_16x16x4_f32): inside a 16-deep chunk, MFMA jj of lane
// group g = lane>>4 consumes k = k0 + 4g + jj for both operands; accumulator lane l holds
// C[4*(l>>4) + r][l&15], r = 0..3.
#pragma once
#include "gemm_common.hpp"

namespace dqnx {

template <int T, int LAYOUT, bool VEC>
struct FragLoader;

template <int T, bool VEC>
struct FragLoader<T, L_ROWS_K, VEC> {
    const float* rp[T];
    float* cp[T];
    __device__ __forceinline__ void init(const Operand& o, int r0) {
        const int i = threadIdx.x & 15;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = r0 + t * 16 + i;
            if (r < o.nrows) {
#ifdef DQNX_ABLATE_NOGATHER   // timing-only build: rows in order instead of gathered
                const int64_t row = (int64_t)r;
#else
                const int64_t row = o.gather ? (int64_t)o.gather[r] : (int64_t)r;
#endif
                rp[t] = o.base + row * o.ld;
                cp[t] = o.copy ? o.copy + (int64_t)r * o.ldcopy : nullptr;
            } else {
                rp[t] = nullptr;
                cp[t] = nullptr;
            }
        }
    }
    __device__ __forceinline__ void load(const Operand& o, int k0, int kend, float (&f)[T][4]) const {
        const int k = k0 + 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
        for (int t = 0; t < T; t++) {
            if (VEC) {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (rp[t] && k < kend) v = ld4(rp[t] + k);
                f[t][0] = v.x; f[t][1] = v.y; f[t][2] = v.z; f[t][3] = v.w;
            } else {
#pragma unroll
                for (int jj = 0; jj < 4; jj++) f[t][jj] = (rp[t] && k + jj < kend) ? rp[t][k + jj] : 0.f;
            }
        }
    }
    __device__ __forceinline__ void copy_out(int k0, int kend, const float (&f)[T][4]) const {
        const int k = k0 + 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
        for (int t = 0; t < T; t++)
            if (cp[t] && k < kend) *reinterpret_cast<float4*>(cp[t] + k) = make_float4(f[t][0], f[t][1], f[t][2], f[t][3]);
    }
};

template <int T, bool VEC>
struct FragLoader<T, L_K_ROWS, VEC> {
    int col[T];
    bool ok[T], one[T];
    __device__ __forceinline__ void init(const Operand& o, int c0) {
        const int i = threadIdx.x & 15;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int c = c0 + t * 16 + i;
            col[t] = c;
            one[t] = (c == o.aug);
            ok[t] = (c < o.nrows) && !one[t];
        }
    }
    __device__ __forceinline__ void load(const Operand& o, int k0, int kend, float (&f)[T][4]) const {
        const int kb = k0 + 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int k = kb + jj;
            const bool kv = k < kend;
            const float* row = o.base + (int64_t)k * o.ld;
#pragma unroll
            for (int t = 0; t < T; t++) f[t][jj] = (kv && ok[t]) ? row[col[t]] : ((kv && one[t]) ? 1.f : 0.f);
        }
    }
    __device__ __forceinline__ void copy_out(int, int, const float (&)[T][4]) const {}
};

// BM x BN tile, NWV waves, K split across waves in ranges of kq (multiple of 16); each wave
// issues its loads in rounds of KW (<= KW/16 chunks in registers at once).
template <int BM, int BN, int NWV, int KW, int LA, int LB, bool VA, bool VB>
struct TileGemmSK {
    static constexpr int TM = BM / 16, TN = BN / 16, NC = KW / 16;
    static_assert(BM % 16 == 0 && BN % 16 == 0 && KW % 16 == 0, "tile shape");
    static constexpr int LDS_FLOATS = (NWV - 1) * TM * TN * 4 * 64;   // partial tiles of waves 1..NWV-1

    // On return, wave 0's acc holds the full tile sum (fixed order); other waves' acc is junk.
    __device__ __forceinline__ static void run(float* lds, const Operand& A, const Operand& B, int m0, int n0,
                                               int kbeg, int kend, floatx4 (&acc)[TM][TN]) {
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
        const int span = kend - kbeg;
        const int kq = ((span + NWV - 1) / NWV + 15) & ~15;
        const int wb = kbeg + wid * kq;
        const int we = min(kend, wb + kq);
        if (wb < we) {
            FragLoader<TM, LA, VA> la;
            FragLoader<TN, LB, VB> lb;
            la.init(A, m0);
            lb.init(B, n0);
            for (int rb = wb; rb < we; rb += KW) {
                float a[NC][TM][4], b[NC][TN][4];
#ifdef DQNX_ABLATE_NOLOAD   // timing-only build: no global operand loads
#pragma unroll
                for (int c = 0; c < NC; c++) {
#pragma unroll
                    for (int t = 0; t < TM; t++)
#pragma unroll
                        for (int jj = 0; jj < 4; jj++) a[c][t][jj] = (float)(lane + c + jj + rb);
#pragma unroll
                    for (int t = 0; t < TN; t++)
#pragma unroll
                        for (int jj = 0; jj < 4; jj++) b[c][t][jj] = (float)(lane - c + jj + rb);
                }
#else
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    la.load(A, rb + 16 * c, we, a[c]);
                    lb.load(B, rb + 16 * c, we, b[c]);
                }
#endif
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    if (A.copy) la.copy_out(rb + 16 * c, we, a[c]);
#ifdef DQNX_ABLATE_NOMFMA   // timing-only build: operands kept live, no MFMA
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
#pragma unroll
                        for (int tm = 0; tm < TM; tm++)
#pragma unroll
                            for (int tn = 0; tn < TN; tn++) asm volatile("" ::"v"(a[c][tm][jj]), "v"(b[c][tn][jj]));
#else
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
#pragma unroll
                        for (int tm = 0; tm < TM; tm++)
#pragma unroll
                            for (int tn = 0; tn < TN; tn++)
                                acc[tm][tn] = mfma16x16x4(a[c][tm][jj], b[c][tn][jj], acc[tm][tn]);
#endif
                }
            }
        }
        if (NWV > 1) {
            if (wid > 0) {
                float* p = lds + (wid - 1) * TM * TN * 4 * 64;
#pragma unroll
                for (int tm = 0; tm < TM; tm++)
#pragma unroll
                    for (int tn = 0; tn < TN; tn++)
#pragma unroll
                        for (int r = 0; r < 4; r++) p[((tm * TN + tn) * 4 + r) * 64 + lane] = acc[tm][tn][r];
            }
            __syncthreads();
            if (wid == 0) {
#pragma unroll
                for (int w = 1; w < NWV; w++) {
                    const float* p = lds + (w - 1) * TM * TN * 4 * 64;
#pragma unroll
                    for (int tm = 0; tm < TM; tm++)
#pragma unroll
                        for (int tn = 0; tn < TN; tn++)
#pragma unroll
                            for (int r = 0; r < 4; r++) acc[tm][tn][r] += p[((tm * TN + tn) * 4 + r) * 64 + lane];
                }
            }
        }
    }
};

}  // namespace dqnx
