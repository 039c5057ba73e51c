// Weight gradients + optimizer in ONE launch (the last kernel of a learn step).
//
// Every parameter tile (dW of each dense layer and of the Q head, each with its bias as a
// ones column) is one 512-thread workgroup that owns the FULL sample range: its 8 waves
// split the minibatch (wave-split-K engine, gemm_sk.hpp) and their partial tiles are summed
// through LDS in a fixed order, so gradients are deterministic and final inside the
// workgroup.  The epilogue applies torch's single-tensor Adam and the tau soft update
// (R:dqn/agent.py:105-110) to the tile's parameters directly: no split-K slabs, no
// separate optimizer pass.  Reference: loss.backward() + optimizer.step()
// (R:dqn/agent.py:224-226) followed by update_target_network() (R:train.py:101).
#include "gemm_sk.hpp"
#include "learn.hpp"

namespace dqnx {

__device__ __forceinline__ int64_t dw_param_index(const DwAdamProblem& d, int row, int col) {
    if (d.head_kind < 0)
        return d.poff + ((col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.out * d.in + row);
    if (d.head_kind == DQNX_HEAD_DUELING)   // [fc_val.w (F) | fc_val.b | fc_adv.w (A*F) | fc_adv.b (A)]
        return d.poff + ((col < d.in) ? (row == 0 ? col : d.in + 1 + (int64_t)(row - 1) * d.in + col)
                                      : (row == 0 ? d.in : d.in + 1 + (int64_t)d.A * d.in + (row - 1)));
    return d.poff + ((col < d.in) ? (int64_t)row * d.in + col : (int64_t)d.A * d.in + row);   // fc_out
}

constexpr int DW_BM = 32, DW_BN = 32, DW_NWV = 8, DW_KW = 64;

__global__ __launch_bounds__(64 * DW_NWV) void k_dw_adam(DwAdamArgs a) {
    using G = TileGemmSK<DW_BM, DW_BN, DW_NWV, DW_KW, L_K_ROWS, L_K_ROWS, true, true>;
    constexpr int TM = G::TM, TN = G::TN;
    __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    int b = blockIdx.x, p = 0;
    while (p + 1 < a.npr && b >= a.pr[p].blocks) { b -= a.pr[p].blocks; p++; }
    const DwAdamProblem& d = a.pr[p];
    const int m0 = (b / d.grid_x) * DW_BM, n0 = (b % d.grid_x) * DW_BN;

    // The tile's optimizer state is fetched into LDS before the GEMM (its latency hides
    // under the K loop); wave 0, which ends up owning the tile, reads it back afterwards.
    __shared__ float st[4][DW_BM * DW_BN];   // p, m, v, target
    if (a.mode) {
        for (int q = tid; q < DW_BM * DW_BN; q += 64 * DW_NWV) {
            const int row = m0 + q / DW_BN, col = n0 + q % DW_BN;
            if (row < d.out && col <= d.in) {
                const int64_t e = dw_param_index(d, row, col);
                st[0][q] = a.p[e];
                st[1][q] = a.m[e];
                st[2][q] = a.v[e];
                st[3][q] = a.soft ? a.target[e] : 0.f;
            }
        }
    }
    Operand A{d.dZ, d.ldz, nullptr, d.out, a.Bl, -1, nullptr, 0};
    Operand B{d.X, d.ldx, nullptr, d.in, a.Bl, d.in, nullptr, 0};
    floatx4 acc[TM][TN];
    G::run(lds, A, B, m0, n0, 0, a.Bl, acc);
    if (wid != 0) return;

    float step_size = 0.f, bc2s = 1.f;
    if (a.mode) {
        const int64_t t = a.ctrl->adam_step;
        if (t >= 1 && t <= a.adam_table_len) {
            step_size = a.adam_table[2 * (t - 1)];
            bc2s = a.adam_table[2 * (t - 1) + 1];
        } else {
            step_size = (float)(-(a.lrd / (1.0 - pow(a.beta1d, (double)t))));
            bc2s = (float)pow(1.0 - pow(a.beta2d, (double)t), 0.5);
        }
    }
#pragma unroll
    for (int tm = 0; tm < TM; tm++)
#pragma unroll
        for (int tn = 0; tn < TN; tn++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int rl = tm * 16 + 4 * g + r, cl = tn * 16 + i;
                const int row = m0 + rl, col = n0 + cl;
                if (row >= d.out || col > d.in) continue;
                const int64_t e = dw_param_index(d, row, col);
                const float gsum = acc[tm][tn][r];
                a.grads[e] = gsum;
                if (!a.mode) continue;
                const int q = rl * DW_BN + cl;
                // torch _single_tensor_adam (see k_adam in learn.hip for the op-by-op mapping)
                float m = st[1][q], v = st[2][q], pv = st[0][q];
                m = fmaf(a.w1, gsum - m, m);
                v = v * a.beta2;
                v = v + (a.c2 * gsum) * gsum;
                const float denom = sqrtf(v) / bc2s + a.eps;
                pv = pv + (step_size * m) / denom;
                a.m[e] = m;
                a.v[e] = v;
                a.p[e] = pv;
                if (a.soft) a.target[e] = a.tau * pv + a.one_minus_tau * st[3][q];
            }
    if (blockIdx.x == 0 && lane == 0 && a.loss_partial) {
        float s = 0.f;
        for (int j = 0; j < a.n_loss_partial; j++) s += a.loss_partial[j];
        const float loss = s / (float)a.batch_global;
        a.grads[a.n_params] = loss;     // all-reduced with the gradient under DP
        a.ctrl->loss = loss;
    }
}

void dw_adam_grid(DwAdamArgs& a) {
    for (int p = 0; p < a.npr; p++) {
        DwAdamProblem& d = a.pr[p];
        d.grid_x = (d.in + 1 + DW_BN - 1) / DW_BN;
        d.blocks = d.grid_x * ((d.out + DW_BM - 1) / DW_BM);
    }
}

int launch_dw_adam(const DwAdamArgs& a, hipStream_t s) {
    int blocks = 0;
    for (int p = 0; p < a.npr; p++) blocks += a.pr[p].blocks;
    DQNX_LAUNCH(k_dw_adam, dim3(blocks), dim3(64 * DW_NWV), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
