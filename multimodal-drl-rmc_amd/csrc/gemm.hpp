// fp32 MFMA tile machinery for the small GEMMs of the DQN learn step (gfx950).
//
// One wave owns TM x TN sub-tiles of 16x16 outputs and walks K in chunks of 16 with
// v_mfma_f32_16x16x4_f32 (exact fp32 fmaf chains, 64 FLOP/clk/SIMD = the fp32 peak).
// Inside a 16-deep chunk, MFMA jj (0..3) of lane group g = lane>>4 consumes
// k = k0 + 4*g + jj for BOTH operands, so a K-contiguous operand is one float4 per lane
// (16-B loads) and a K-strided operand is 4 scalar loads whose 16-lane groups are
// 64-B contiguous.  Operands are read straight from global memory (L1/L2 resident at
// these sizes) with a 2-deep register pipeline; no LDS round trip (the GEMV/small-M
// row of the CDNA guide's "glds vs register staging" table).
#pragma once
#include "common.hpp"

namespace dqnx {

// ---- operand whose K index runs along a row (X[m][k], W[n][k]) ----------------------
// Fragment element (t, jj) = row(base + t*16 + (lane&15))[k0 + 4g + jj].
template <int T, bool VEC>
struct RowsK {
    const float* ptr[T];
    float* cpy[T];   // optional row copy target (layer-1 input materialisation)
    int K;
    __device__ __forceinline__ void set_dense(const float* base, int ld, int row0, int nrows, int K_) {
        const int i = threadIdx.x & 15;
        K = K_;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int r = row0 + t * 16 + i;
            ptr[t] = (r < nrows) ? base + (int64_t)r * ld : nullptr;
            cpy[t] = nullptr;
        }
    }
    __device__ __forceinline__ void load(int k0, float (&f)[T][4]) const {
        const int k = k0 + 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
        for (int t = 0; t < T; t++) {
            if (VEC) {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ptr[t] && k < K) v = ld4(ptr[t] + k);
                if (cpy[t] && k < K) *reinterpret_cast<float4*>(cpy[t] + k) = v;
                f[t][0] = v.x; f[t][1] = v.y; f[t][2] = v.z; f[t][3] = v.w;
            } else {
#pragma unroll
                for (int jj = 0; jj < 4; jj++)
                    f[t][jj] = (ptr[t] && k + jj < K) ? ptr[t][k + jj] : 0.f;
            }
        }
    }
};

// ---- operand whose K index runs down rows (S[k][col]): dZ^T, W as [K][N], X as [K][N] ----
// Fragment element (t, jj) = S[k0 + 4g + jj][col0 + t*16 + (lane&15)]; column == aug -> 1.0
// (the appended ones-column that turns a bias gradient into one more GEMM column).
template <int T>
struct StridedK {
    const float* base;
    int ld, K;
    int col[T];
    bool ok[T], one[T];
    __device__ __forceinline__ void set(const float* b, int ld_, int K_, int col0, int ncols, int aug) {
        const int i = threadIdx.x & 15;
        base = b; ld = ld_; K = K_;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const int c = col0 + t * 16 + i;
            col[t] = c;
            one[t] = (c == aug);
            ok[t] = (c < ncols) && !one[t];
        }
    }
    __device__ __forceinline__ void load(int k0, float (&f)[T][4]) const {
        const int kb = k0 + 4 * ((threadIdx.x & 63) >> 4);
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int k = kb + jj;
            const bool kv = k < K;
            const float* row = base + (int64_t)k * ld;
#pragma unroll
            for (int t = 0; t < T; t++)
                f[t][jj] = (kv && ok[t]) ? row[col[t]] : ((kv && one[t]) ? 1.f : 0.f);
        }
    }
};

template <int TM, int TN>
__device__ __forceinline__ void mma_chunk(const float (&a)[TM][4], const float (&b)[TN][4],
                                          floatx4 (&acc)[TM][TN]) {
#pragma unroll
    for (int jj = 0; jj < 4; jj++)
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) acc[tm][tn] = mfma16x16x4(a[tm][jj], b[tn][jj], acc[tm][tn]);
}

// acc += sum_{k in [kbeg, kend)} A[.][k] * B[k][.], chunks of 16, 2-deep register pipeline.
template <int TM, int TN, class LA, class LB>
__device__ __forceinline__ void mfma_loop(const LA& A, const LB& B, int kbeg, int kend,
                                          floatx4 (&acc)[TM][TN]) {
    if (kbeg >= kend) return;
    float a0[TM][4], b0[TN][4], a1[TM][4], b1[TN][4];
    int k = kbeg;
    A.load(k, a0);
    B.load(k, b0);
    while (true) {
        const int k1 = k + 16;
        const bool h1 = k1 < kend;
        if (h1) { A.load(k1, a1); B.load(k1, b1); }
        mma_chunk<TM, TN>(a0, b0, acc);
        if (!h1) break;
        const int k2 = k1 + 16;
        const bool h2 = k2 < kend;
        if (h2) { A.load(k2, a0); B.load(k2, b0); }
        mma_chunk<TM, TN>(a1, b1, acc);
        if (!h2) break;
        k = k2;
    }
}

template <int TM, int TN>
__device__ __forceinline__ void zero_acc(floatx4 (&acc)[TM][TN]) {
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
        for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
}

}  // namespace dqnx
