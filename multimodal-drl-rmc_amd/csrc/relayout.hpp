// Fragment-blocked weight copies for the fused MLP kernels (fused.hip).
//
// An M = 16 GEMM tile streams every weight once per workgroup; in torch's [out][in] layout a
// wave's MFMA B fragments (16 rows x 16 B per quarter-wave) touch 16 cache lines per 256 B,
// and the texture path, not the MFMA, sets the pace.  The blocked copies store each
// 16 x 16 fragment block in the exact lane order of one wave-instruction, so a fragment
// load is 1 KiB contiguous:
//   fwd   (W [N][K], B[k][n] = W[n][k]):   blk[t][c][g*16 + i][j] = W[16t + i][16c + 4g + j]
//         (K zero padded to kpad, a multiple of 64)
//   chain (W [K][N], B[k][n] = W[k][n]):   blk[t][c][g*16 + i][j] = W[16c + 4g + j][16t + i]
// bf16 (DQNX_COMPUTE_BF16) copies hold 16 x 32 blocks, 8 bf16 (RNE) per lane, the operand
// order of v_mfma_f32_16x16x32_bf16:
//   fwd16   blk[t][c][g*16 + i][j] = bf16(W[16t + i][32c + 8g + j])   (K zero padded to 32)
//   chain16 blk[t][c][g*16 + i][j] = bf16(W[32c + 8g + j][16t + i])
// Every job is indexed in 16-byte units (one lane's fragment) in both precisions.
// The copies are rebuilt at the start of every learn step by spare workgroups of the
// sampler launch (the weights may change between steps through the torch views of the
// parameter arena), never by the critical path.
#pragma once
#include "common.hpp"

namespace dqnx {

constexpr int RELAYOUT_MAX_JOBS = 9;
struct RelayoutJob {
    const float* src;   // torch layout [rows][cols]
    float* dst;
    int rows, cols;
    int kind;           // 0 fwd (tiles over rows, chunks over cols padded to kpad), 1 chain (tiles over cols,
                        // chunks over rows); 2 / 3 the same in bf16
    int nch;            // chunks per tile
    int64_t q0;         // first 16-byte unit of this job in the concatenated index space
};
struct RelayoutArgs {
    RelayoutJob job[RELAYOUT_MAX_JOBS];
    int njobs;
    int64_t total_q;
};

__device__ __forceinline__ void relayout_run(const RelayoutArgs& r, int blk, int nblk) {
    const int64_t stride = (int64_t)nblk * blockDim.x;
    for (int64_t q = (int64_t)blk * blockDim.x + threadIdx.x; q < r.total_q; q += stride) {
        int j = 0;
#pragma unroll
        for (int u = 1; u < RELAYOUT_MAX_JOBS; u++)
            if (u < r.njobs && q >= r.job[u].q0) j = u;
        const RelayoutJob& jb = r.job[j];
        const int64_t lq = q - jb.q0;
        const int lane = (int)(lq & 63), i = lane & 15, g = lane >> 4;
        const int64_t rest = lq >> 6;
        const int c = (int)(rest % jb.nch), t = (int)(rest / jb.nch);
        const int n = 16 * t + i;
        if (jb.kind < 2) {
            const int k = 16 * c + 4 * g;
            float v[4];
            if (jb.kind == 0) {
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = (k + u < jb.cols) ? jb.src[(int64_t)n * jb.cols + k + u] : 0.f;
            } else {
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = jb.src[(int64_t)(k + u) * jb.cols + n];
            }
            *reinterpret_cast<float4*>(jb.dst + 4 * lq) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
            const int k = 32 * c + 8 * g;
            uint32_t w[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                float v0, v1;
                if (jb.kind == 2) {
                    v0 = (k + 2 * u < jb.cols) ? jb.src[(int64_t)n * jb.cols + k + 2 * u] : 0.f;
                    v1 = (k + 2 * u + 1 < jb.cols) ? jb.src[(int64_t)n * jb.cols + k + 2 * u + 1] : 0.f;
                } else {
                    v0 = (k + 2 * u < jb.rows) ? jb.src[(int64_t)(k + 2 * u) * jb.cols + n] : 0.f;
                    v1 = (k + 2 * u + 1 < jb.rows) ? jb.src[(int64_t)(k + 2 * u + 1) * jb.cols + n] : 0.f;
                }
                w[u] = bf16_pack2(v0, v1);
            }
            *reinterpret_cast<uint4*>(jb.dst + 4 * lq) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

}  // namespace dqnx
