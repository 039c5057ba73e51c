// Acting path of the two-stream network (TwoStreamHybridNetwork, R:env/dqn_config.py:66-143):
// Network.actions (DuelingDeepQNetwork R:dqn/network.py:110-117: argmax of the advantage stream;
// DeepQNetwork :67-74: argmax of Q) at n_env rows, called by Agent.choose_actions
// (R:dqn/agent.py:92-99) every env step.
//
// Per row the body is 3 small convs (2 -> 32 -> 64 -> 64 channels on the 2x27x5 micro grid) and
// a 1358 -> 512 -> 256 dense stream: ~6 MFLOP and 3.5 MB of weights, so the time is set by the
// number of dependent round trips, not by FLOPs.  One launch per conv, each a grid of
// (output channel x row) workgroups that stage the row's input image and the channel's weights
// in LDS and split every output pixel's K = Ci*kh*kw sum over as many threads as fit (fixed-order
// reduction); conv 3 writes its CHW output straight into the dense input F = cat(flatten(conv3),
// macro) (R:env/dqn_config.py:135-138).  The dense stream and the head are then the MLP acting
// kernel (act.hip) on F.
#include "common.hpp"
#include "learn.hpp"

namespace dqnx {

namespace {

constexpr int kConvThreads = 256;

__global__ __launch_bounds__(kConvThreads) void k_act_conv(ActConvArgs a) {
    extern __shared__ float lds[];
    const int c = blockIdx.x, r = blockIdx.y, tid = threadIdx.x;
    const int HWi = a.Hi * a.Wi, img = a.Ci * HWi, K = a.Ci * a.kh * a.kw, P = a.Ho * a.Wo;
    float* x = lds;            // [Ci][Hi][Wi] of row r
    float* w = lds + img;      // [Ci][kh][kw] of channel c
    float* part = w + K;       // [S][P] partial sums
    const float* src = a.in + (int64_t)r * a.in_stride + a.in_off;
    for (int i = tid; i < img; i += kConvThreads) x[i] = src[i];
    const float* Wc = a.W + (int64_t)c * K;
    for (int i = tid; i < K; i += kConvThreads) w[i] = Wc[i];
    const float bias = a.b[c];
    if (a.macro && c == 0)   // the dense input's macro tail: F[r][Co*P ..] = obs[r][0 .. macro_len)
        for (int i = tid; i < a.macro_len; i += kConvThreads)
            a.out[(int64_t)r * a.out_stride + (int64_t)a.Co * P + i] = a.macro[(int64_t)r * a.macro_stride + i];
    __syncthreads();
    // output pixel p = t % P, input-channel slice s = t / P of S slices (fixed order: slice 0
    // first); within a slice the sum runs over (ci, i, j) like torch's weight row, with the
    // padding bounds hoisted out of the channel loop
    const int S = max(1, min(kConvThreads / P, a.Ci));
    const int cper = (a.Ci + S - 1) / S;
    for (int t = tid; t < S * P; t += kConvThreads) {
        const int p = t % P, s = t / P;
        const int ho = p / a.Wo, wo = p - ho * a.Wo;
        const int c0 = s * cper, c1 = min(a.Ci, c0 + cper);
        const int h0 = ho * a.sh - a.ph, w0 = wo * a.sw - a.pw;
        const int i0 = max(0, -h0), i1 = min(a.kh, a.Hi - h0), j0 = max(0, -w0), j1 = min(a.kw, a.Wi - w0);
        const int khw = a.kh * a.kw;
        float acc = 0.f;
        for (int ci = c0; ci < c1; ci++) {
            const float* xc = x + ci * HWi + h0 * a.Wi + w0;
            const float* wc = w + ci * khw;
            for (int i = i0; i < i1; i++)
                for (int j = j0; j < j1; j++) acc = fmaf(xc[i * a.Wi + j], wc[i * a.kw + j], acc);
        }
        part[s * P + p] = acc;
    }
    __syncthreads();
    for (int p = tid; p < P; p += kConvThreads) {
        float v = part[p];
        for (int s = 1; s < S; s++) v += part[s * P + p];
        a.out[(int64_t)r * a.out_stride + a.out_off + (int64_t)c * P + p] = elu_f(v + bias);
    }
}

}  // namespace

size_t act_conv_lds_bytes(const ActConvArgs& a) {
    const int P = a.Ho * a.Wo, K = a.Ci * a.kh * a.kw;
    const int S = std::max(1, std::min(kConvThreads / std::max(P, 1), a.Ci));
    return (size_t)(a.Ci * a.Hi * a.Wi + K + S * P) * sizeof(float);
}

int launch_act_conv(const ActConvArgs& a, hipStream_t s) {
    if (a.n <= 0) return DQNX_OK;
    const size_t lds = act_conv_lds_bytes(a);
    if (lds > 64 * 1024 || a.Ho * a.Wo > kConvThreads * 64)
        return set_error(DQNX_EUNSUPPORTED, "dqnx_act: conv layer too large for the acting kernel (%zu B LDS)", lds);
    DQNX_LAUNCH(k_act_conv, dim3(a.Co, a.n), dim3(kConvThreads), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
