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
#include "gemm.hpp"
#include "learn.hpp"

namespace dqnx {

// =====================================================================================
// Forward Linear: C[s] = act(A[s] W[s]^T + b[s]) for up to 3 "streams" (blockIdx.z):
// online(obs), online(next_obs), target(next_obs).  Layer 1 gathers A rows from the
// replay ring through the sampled physical slots (no materialised minibatch), and
// stream 0 also writes the gathered rows to `xcopy` for the dW of layer 1.
// =====================================================================================
template <int TM, int TN, int WM, int WN, int ACT, bool VECB>
__global__ __launch_bounds__(256) void k_linear_fwd(FwdArgs args) {
    const FwdProblem& P = args.p[blockIdx.z];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int i = lane & 15, g = lane >> 4;
    const int m0 = blockIdx.y * (WM * TM * 16) + wm * TM * 16;
    const int n0 = blockIdx.x * (WN * TN * 16) + wn * TN * 16;
    const int M = args.M, N = args.N, K = args.K;

    RowsK<TM, true> A;
    if (P.phys) {
        A.K = K;
#pragma unroll
        for (int t = 0; t < TM; t++) {
            const int r = m0 + t * 16 + i;
            A.ptr[t] = (r < M) ? P.A + (int64_t)P.phys[r] * P.lda : nullptr;
            A.cpy[t] = (P.xcopy && blockIdx.x == 0 && wn == 0 && r < M) ? P.xcopy + (int64_t)r * P.lda : nullptr;
        }
    } else {
        A.set_dense(P.A, P.lda, m0, M, K);
    }
    RowsK<TN, VECB> B;
    B.set_dense(P.W, K, n0, N, K);

    floatx4 acc[TM][TN];
    zero_acc<TM, TN>(acc);
    mfma_loop<TM, TN>(A, B, 0, K, acc);

#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + tn * 16 + i;
        if (col >= N) continue;
        const float bias = P.bias[col];
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + tm * 16 + 4 * g + r;
                if (row < M) P.C[(int64_t)row * args.ldc + col] = act_fwd<ACT>(acc[tm][tn][r] + bias);
            }
    }
}

// =====================================================================================
// Backward level: two independent GEMMs in one launch.
//   dx role:  dZprev = (dZ W) (.) act'(Hprev)      [Bl x in], K = out
//   dw role:  partial[s] = dZ^T [Xprev | 1]        [out x (in+1)], K = samples of slice s
// =====================================================================================
template <int ACT>
__global__ __launch_bounds__(256) void k_bwd_level(BwdArgs a) {
    constexpr int TM = 1, TN = 2, WM = 2, WN = 2;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int i = lane & 15, g = lane >> 4;
    int b = blockIdx.x;
    if (b < a.dx_blocks) {
        const int bx = b % a.dx_grid_x, by = b / a.dx_grid_x;
        const int m0 = by * (WM * TM * 16) + wm * TM * 16;
        const int n0 = bx * (WN * TN * 16) + wn * TN * 16;
        RowsK<TM, true> A;
        A.set_dense(a.dZ, a.out, m0, a.Bl, a.out);
        StridedK<TN> B;
        B.set(a.W, a.in, a.out, n0, a.in, -1);
        floatx4 acc[TM][TN];
        zero_acc<TM, TN>(acc);
        mfma_loop<TM, TN>(A, B, 0, a.out, acc);
#pragma unroll
        for (int tn = 0; tn < TN; tn++) {
            const int col = n0 + tn * 16 + i;
            if (col >= a.in) continue;
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = m0 + tm * 16 + 4 * g + r;
                    if (row < a.Bl)
                        a.dZprev[(int64_t)row * a.in + col] =
                            act_bwd<ACT>(acc[tm][tn][r], a.Hprev[(int64_t)row * a.ldh + col]);
                }
        }
        return;
    }
    b -= a.dx_blocks;
    const int bx = b % a.dw_grid_x;
    const int t2 = b / a.dw_grid_x;
    const int by = t2 % a.dw_grid_y, bz = t2 / a.dw_grid_y;
    const int m0 = by * (WM * TM * 16) + wm * TM * 16;   // out rows
    const int n0 = bx * (WN * TN * 16) + wn * TN * 16;   // in cols (+ ones column)
    const int kb = bz * a.kslice;
    const int ke = min(a.Bl, kb + a.kslice);
    StridedK<TM> A;
    A.set(a.dZ, a.out, ke, m0, a.out, -1);
    StridedK<TN> B;
    B.set(a.X, a.ldx, ke, n0, a.in, a.in);
    floatx4 acc[TM][TN];
    zero_acc<TM, TN>(acc);
    mfma_loop<TM, TN>(A, B, kb, ke, acc);
    float* part = a.partial + (int64_t)bz * a.pstride;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int col = n0 + tn * 16 + i;
        if (col > a.in) continue;
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + tm * 16 + 4 * g + r;
                if (row >= a.out) continue;
                const int64_t o = (col < a.in) ? (int64_t)row * a.in + col : (int64_t)a.out * a.in + row;
                part[o] = acc[tm][tn][r];
            }
    }
}

// =====================================================================================
// Fused head kernel: one workgroup = 16 samples.
//   (1) head Linear(s) for the 3 streams on MFMA (waves 0..2)
//   (2) per sample: dueling aggregate, Double-DQN argmax / DQN max, TD target
//       y = r + ((1-d)*gamma)*q', q(s,a), Huber (beta=1) value and gradient (mean or
//       IS-weighted 'none' reduction), dQ -> d(head outputs)
//   (3) dH = dHead . W_head, dZ_L = dH (.) act'(H_L); head-weight gradient partial of the
//       16 samples; loss partial.
// =====================================================================================
__device__ __forceinline__ int head_w_off(int kind, int o, int F) {
    // dueling: [fc_val.w (F) | fc_val.b | fc_adv.w (A*F) | fc_adv.b (A)], o = 0 val, 1..A adv
    // linear:  [fc_out.w (A*F) | fc_out.b (A)]
    return kind == DQNX_HEAD_DUELING ? (o == 0 ? 0 : F + 1 + (o - 1) * F) : o * F;
}
__device__ __forceinline__ int head_b_off(int kind, int o, int F, int A) {
    return kind == DQNX_HEAD_DUELING ? (o == 0 ? F : F + 1 + A * F + (o - 1)) : A * F + o;
}

template <int ACT>
__global__ __launch_bounds__(256) void k_head(HeadArgs a) {
    constexpr int TS = 16;
    __shared__ float raw[3][TS][17];
    __shared__ float dh[TS][17];
    __shared__ float lossv[TS];
    extern __shared__ __attribute__((aligned(16))) float dyn[];
    float* Hl = dyn;                       // [TS][F]   last hidden of stream 0 (online, obs)
    float* Wl = dyn + TS * a.F;            // [NH][F]   online head weights

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, g = lane >> 4;
    const int b0 = blockIdx.x * TS;
    const int F = a.F, A = a.A, NH = a.NH, Bl = a.Bl;
    const int nb = min(TS, Bl - b0);

    // stage H_L(stream 0) tile and the online head weights into LDS
    for (int idx = tid; idx < TS * F; idx += 256) {
        const int b = idx / F, f = idx - b * F;
        Hl[idx] = (b < nb) ? a.H[(int64_t)(b0 + b) * F + f] : 0.f;
    }
    for (int idx = tid; idx < NH * F; idx += 256) {
        const int o = idx / F, f = idx - o * F;
        Wl[idx] = a.Wo[head_w_off(a.head_kind, o, F) + f];
    }

    // (1) head outputs for the streams this algorithm needs
    if (wid < 3 && !(wid == 1 && a.algo == DQNX_ALGO_DQN)) {
        const int s = wid;
        const float* W = (s == 2) ? a.Wt : a.Wo;
        const float* Hs = a.H + (int64_t)s * Bl * F;
        const int row = b0 + i;
        const float* arow = (row < Bl) ? Hs + (int64_t)row * F : nullptr;
        const float* brow = (i < NH) ? W + head_w_off(a.head_kind, i, F) : nullptr;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < F; k0 += 16) {
            const int k = k0 + 4 * g;
            float4 av = make_float4(0.f, 0.f, 0.f, 0.f), bv = av;
            if (arow && k < F) av = ld4(arow + k);
            if (brow && k < F) bv = ld4(brow + k);
            acc = mfma16x16x4(av.x, bv.x, acc);
            acc = mfma16x16x4(av.y, bv.y, acc);
            acc = mfma16x16x4(av.z, bv.z, acc);
            acc = mfma16x16x4(av.w, bv.w, acc);
        }
        const float bias = (i < NH) ? W[head_b_off(a.head_kind, i, F, A)] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; r++) raw[s][4 * g + r][i] = acc[r] + bias;
    }
    __syncthreads();

    // (2) per-sample TD / loss / head gradient
    if (tid < TS) {
        const int b = tid;
        float dho[17];
        float lb = 0.f;
        if (b < nb) {
            const int gb = b0 + b;
            const int slot = a.phys[gb];
            const int act = a.act[slot];
            const float rew = a.rew[slot], done = a.done[slot];
            float q[3][16];
            for (int s = 0; s < 3; s++) {
                if (s == 1 && a.algo == DQNX_ALGO_DQN) continue;
                if (a.head_kind == DQNX_HEAD_DUELING) {
                    const float v = raw[s][b][0];
                    float sum = 0.f;
                    for (int j = 0; j < A; j++) sum += raw[s][b][1 + j];
                    const float mean = sum / (float)A;
                    for (int j = 0; j < A; j++) q[s][j] = v + (raw[s][b][1 + j] - mean);
                } else {
                    for (int j = 0; j < A; j++) q[s][j] = raw[s][b][j];
                }
                for (int j = 0; j < A; j++) a.Q[((int64_t)s * Bl + gb) * A + j] = q[s][j];
            }
            float qn;
            if (a.algo == DQNX_ALGO_DQN) {        // target(s').max(1)  (R:dqn/agent.py:172-173)
                qn = q[2][0];
                for (int j = 1; j < A; j++) qn = q[2][j] > qn ? q[2][j] : qn;
            } else {                               // argmax online(s'), gather target(s') (:210-214)
                int best = 0;
                float bq = q[1][0];
                for (int j = 1; j < A; j++)
                    if (q[1][j] > bq) { bq = q[1][j]; best = j; }
                qn = q[2][best];
            }
            // targets = rews + (1 - dones) * gamma * q'    (R:dqn/agent.py:216)
            const float t1 = 1.f - done;
            const float t2 = t1 * a.gamma;
            const float t3 = t2 * qn;
            const float y = rew + t3;
            const float qa = q[0][act];
            const float x = qa - y;               // smooth_l1: input - target
            const float z = fabsf(x);
            const float l = z < 1.f ? (0.5f * z) * z / 1.f : z - 0.5f;
            float gq;
            if (a.isw) {                          // PER: mean(w * huber_none)  (R:dqn/agent.py:267)
                const float w = a.isw[gb];
                const float go = a.inv_bg * w;    // MeanBackward (1/B) then MulBackward (* w)
                gq = x <= -1.f ? -go : (x >= 1.f ? go : (x * go) / 1.f);
                lb = w * l;
            } else {                              // SmoothL1Loss(mean): norm = 1/B
                gq = x <= -1.f ? -a.inv_bg : (x >= 1.f ? a.inv_bg : (a.inv_bg * x) / 1.f);
                lb = l;
            }
            a.td[gb] = y;
            a.td[Bl + gb] = qa;
            a.td[2 * Bl + gb] = z;
            if (a.head_kind == DQNX_HEAD_DUELING) {
                const float nm = (-gq) / (float)A;    // mean backward of -sum(dQ)
                dho[0] = gq;                          // dV = sum_a dQ
                for (int j = 0; j < A; j++) dho[1 + j] = (j == act ? gq : 0.f) + nm;
            } else {
                for (int j = 0; j < A; j++) dho[j] = (j == act) ? gq : 0.f;
            }
        } else {
            for (int o = 0; o < NH; o++) dho[o] = 0.f;
        }
        for (int o = 0; o < NH; o++) dh[b][o] = dho[o];
        lossv[b] = lb;
    }
    __syncthreads();

    // (3a) loss partial (fixed order)
    if (tid == 0) {
        float s = 0.f;
        for (int b = 0; b < TS; b++) s += lossv[b];
        a.loss_partial[blockIdx.x] = s;
    }
    // (3b) dH_L and dZ_L = dH_L (.) act'(H_L)
    for (int idx = tid; idx < TS * F; idx += 256) {
        const int b = idx / F, f = idx - b * F;
        if (b >= nb) continue;
        float s = 0.f;
        if (a.head_kind == DQNX_HEAD_DUELING) {
            for (int o = 1; o < NH; o++) s += dh[b][o] * Wl[o * F + f];
            s = dh[b][0] * Wl[f] + s;
        } else {
            for (int o = 0; o < NH; o++) s += dh[b][o] * Wl[o * F + f];
        }
        a.dZ[(int64_t)(b0 + b) * F + f] = act_bwd<ACT>(s, Hl[idx]);
    }
    // (3c) head weight / bias gradient partial of this tile
    float* part = a.head_partial + (int64_t)blockIdx.x * a.head_params;
    for (int idx = tid; idx < NH * F; idx += 256) {
        const int o = idx / F, f = idx - o * F;
        float s = 0.f;
        for (int b = 0; b < TS; b++) s += dh[b][o] * Hl[b * F + f];
        part[head_w_off(a.head_kind, o, F) + f] = s;
    }
    if (tid < NH) {
        float s = 0.f;
        for (int b = 0; b < TS; b++) s += dh[b][tid];
        part[head_b_off(a.head_kind, tid, F, A)] = s;
    }
    // Adam scalars of this step (read by the Adam pass, a later launch)
    if (blockIdx.x == 0 && tid == 0 && a.ctrl) {
        const int64_t t = a.ctrl->adam_step + 1;
        a.ctrl->adam_step = t;
        const double bc1 = 1.0 - pow((double)a.beta1, (double)t);
        const double bc2 = 1.0 - pow((double)a.beta2, (double)t);
        const double step_size = (double)a.lr / bc1;
        a.ctrl->adam_step_size = (float)(-step_size);
        a.ctrl->adam_bc2_sqrt = (float)sqrt(bc2);
    }
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
__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    const int64_t P = a.n_params;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < P; e += stride) {
        float gsum;
        if (a.mode == 2) {
            gsum = a.grads[e];
        } else {
            int sgi = 0;
#pragma unroll 1
            for (int q = 1; q < a.nseg; q++)
                if (e >= a.seg[q].off) sgi = q;
            const AdamSegment sg = a.seg[sgi];
            const float* pp = sg.partial + (e - sg.off);
            gsum = pp[0];
#pragma unroll 1
            for (int s = 1; s < sg.S; s++) gsum += pp[(int64_t)s * sg.pstride];
            a.grads[e] = gsum;
        }
        if (a.mode == 0) continue;
        const float step_size = a.ctrl->adam_step_size;
        const float bc2s = a.ctrl->adam_bc2_sqrt;
        float m = a.m[e], v = a.v[e], p = a.p[e];
        m = fmaf(a.w1, gsum - m, m);
        v = v * a.beta2;
        v = v + (a.c2 * gsum) * gsum;
        const float denom = sqrtf(v) / bc2s + a.eps;
        p = p + (step_size * m) / denom;
        a.m[e] = m;
        a.v[e] = v;
        a.p[e] = p;
        if (a.soft) a.target[e] = a.tau * p + a.one_minus_tau * a.target[e];
    }
    if (a.mode != 2 && blockIdx.x == 0 && threadIdx.x == 0 && a.loss_partial) {
        float s = 0.f;
        for (int j = 0; j < a.n_loss_partial; j++) s += a.loss_partial[j];
        const float loss = s / (float)a.batch_global;
        a.grads[P] = loss;     // all-reduced with the gradient under DP
        a.ctrl->loss = loss;
    }
    if (a.mode == 2 && blockIdx.x == 0 && threadIdx.x == 0) a.ctrl->loss = a.grads[P];
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
int launch_linear_fwd(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s) {
    constexpr int TM = 1, TN = 2, WM = 2, WN = 2;
    dim3 grid((args.N + WN * TN * 16 - 1) / (WN * TN * 16), (args.M + WM * TM * 16 - 1) / (WM * TM * 16), nprob);
    if (act == DQNX_ACT_RELU) {
        if (vecb) hipLaunchKernelGGL((k_linear_fwd<TM, TN, WM, WN, DQNX_ACT_RELU, true>), grid, dim3(256), 0, s, args);
        else hipLaunchKernelGGL((k_linear_fwd<TM, TN, WM, WN, DQNX_ACT_RELU, false>), grid, dim3(256), 0, s, args);
    } else {
        if (vecb) hipLaunchKernelGGL((k_linear_fwd<TM, TN, WM, WN, DQNX_ACT_ELU, true>), grid, dim3(256), 0, s, args);
        else hipLaunchKernelGGL((k_linear_fwd<TM, TN, WM, WN, DQNX_ACT_ELU, false>), grid, dim3(256), 0, s, args);
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

void bwd_level_grid(BwdArgs& a) {
    constexpr int BM = 32, BN = 64;
    if (a.dZprev) {
        a.dx_grid_x = (a.in + BN - 1) / BN;
        a.dx_blocks = a.dx_grid_x * ((a.Bl + BM - 1) / BM);
    } else {
        a.dx_grid_x = 1;
        a.dx_blocks = 0;
    }
    a.dw_grid_x = (a.in + 1 + BN - 1) / BN;
    a.dw_grid_y = (a.out + BM - 1) / BM;
}

int launch_bwd_level(const BwdArgs& a, int nslices, int act, hipStream_t s) {
    const int blocks = a.dx_blocks + a.dw_grid_x * a.dw_grid_y * nslices;
    if (act == DQNX_ACT_RELU) hipLaunchKernelGGL(k_bwd_level<DQNX_ACT_RELU>, dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_bwd_level<DQNX_ACT_ELU>, dim3(blocks), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_head(const HeadArgs& a, int act, hipStream_t s) {
    const int tiles = (a.Bl + 15) / 16;
    const size_t lds = (size_t)(16 + a.NH) * a.F * sizeof(float);
    if (act == DQNX_ACT_RELU) hipLaunchKernelGGL(k_head<DQNX_ACT_RELU>, dim3(tiles), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_head<DQNX_ACT_ELU>, dim3(tiles), dim3(256), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_adam(const AdamArgs& a, hipStream_t s) {
    int blocks = (int)((a.n_params + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_soft_update(float* target, const float* p, int64_t n, float tau, float omt, hipStream_t s) {
    int blocks = (int)((n + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_soft_update, dim3(blocks), dim3(256), 0, s, target, p, n, tau, omt);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_replay_push(const PushArgs& a, hipStream_t s) {
    if (a.n <= 0) return DQNX_OK;
    hipLaunchKernelGGL(k_replay_push, dim3(a.n), dim3(128), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
