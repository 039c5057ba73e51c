// Implicit-GEMM convolutions of the two-stream hybrid Q-network's micro CNN
// (TwoStreamHybridNetwork, R:env/dqn_config.py:92-101 / 126-138) for large occupancy grids
// (the stacked (4,84,84) variant): forward, data gradient and weight gradient as MFMA GEMMs
// whose A / B operands are read from an image band staged in LDS -- no column matrix is ever
// written to HBM (the explicit im2col / col2im path of conv.hip moves 3.8 GB per step on conv 2).
//
// Forward (k_conv_ig, CIG_EPI_NHWC / CIG_EPI_FLAT):
//   C[(b, ho, wo)][co] = act(sum_{i, j, ci} X[b][ho*sh - ph + i][wo*sw - pw + j][ci] W[co][ci][i][j] + bias)
//   A workgroup owns TR output rows (full width) of one image and all Cout columns.  The input
//   rows they touch (NR = (TR-1)*sh + kh) are staged channel block by channel block into LDS as
//   [row][col][ch] with a zero halo, so an A fragment is one ds_read_b128 at
//   band[(pixel position + tap offset) * CS + 4*(lane>>4)] -- the tap offset is a constant per
//   16-deep K chunk.  The weights are read as float4 straight from a permuted copy
//   [co][tap][ci] (L1/L2 resident, one chunk ahead).  The last conv writes
//   cat(flatten_CHW(conv), macro) (R:env/dqn_config.py:135-138) directly (CIG_EPI_FLAT).
// Data gradient (k_conv_ig, CIG_EPI_DX): the transposed conv, split into the (sh x sw) output
//   phases of a strided conv (sub-pixel decomposition): in phase (a, c) only the taps with
//   (a + ph - i) % sh == 0 and (c + pw - j) % sw == 0 contribute, each from a fixed offset of
//   the dZ band, so every phase is again a dense GEMM (K = its taps x Cout) over the staged dZ
//   band with weights [ci][tap][co]; the epilogue applies the previous conv's ELU' (torch's
//   elu_backward on the activation output), which col2im did before.
// Weight gradient (k_conv_dw_ig): per slice of output row groups,
//   partial[s][co][(ci, i, j)] = sum_pixels dZ[p][co] X[pixel + tap][ci], plus db[co] = sum dZ,
//   in the split-K slab layout the Adam pass sums in fixed order (learn.hip).  X is staged per
//   row group; dZ is read per lane (4 pixels per MFMA k-group) one chunk ahead.
// Accumulation orders are fixed (deterministic), not the explicit path's: parity with torch is
// by tolerance, like the explicit path.
#include <map>
#include <mutex>

#include "learn.hpp"

namespace dqnx {

namespace {

// x / d and x % d for 0 <= x < 2^22 via a float reciprocal and one correction step
__device__ __forceinline__ void divmod_f(int x, int d, float inv, int& q, int& r) {
    q = (int)((float)x * inv);
    r = x - q * d;
    if (r < 0) { q--; r += d; } else if (r >= d) { q++; r -= d; }
}

// Band staging in two halves, so a workgroup can have the NEXT band's global loads in flight
// while it multiplies the current one: stage_load issues a thread's loads into registers,
// stage_store writes them to band[(row * WP + col) * CS + ch] (zeros outside the image).  Work
// is dealt by lines that are uniform per wave (no per-element divisions), lanes along the
// contiguous source dimension:
//   NHWC source (cstride 1): line = band row, WP*CB/4 float4 per line (pixels x channel quads);
//   CHW source (pixels fastest): line = (channel, band row), WP floats per line.
// The host keeps every band within NQ float4 (NHWC) / 4*NQ floats (CHW) per thread.
constexpr int NQ = 12;    // float4 per thread, NHWC sources
constexpr int NQS = 12;   // floats per thread, CHW sources
struct Stage {
    const float* srcb;
    int r0, c0, ch0;
};
template <bool VEC>
struct StageRegs {
    static constexpr int N = VEC ? NQ : NQS;
    float4 v[VEC ? NQ : 1];
    float f[VEC ? 1 : NQS];

    __device__ __forceinline__ void load(const CigSource& S, const Stage& st, int NR, int WP, int CB, int RS = 1) {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (VEC) {
            const int q4s = CB == 64 ? 4 : CB == 32 ? 3 : CB == 16 ? 2 : (CB == 8 ? 1 : 0);   // log2(CB / 4)
            const int per_line = WP << q4s;              // float4 per band row
            const int lpr = (per_line + 63) >> 6;        // 64-lane passes per row
            const int nlines = NR * lpr;
#pragma unroll
            for (int u = 0; u < N; u++) {
                const int li = wid + 4 * u;              // (row, pass), wave-uniform
                const int rr = li / lpr, h = li - rr * lpr;
                const int j = 64 * h + lane;
                const int cc = j >> q4s, q = j & ((1 << q4s) - 1);
                const int r = st.r0 + rr * RS, w = st.c0 + cc;
                v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (li < nlines && j < per_line && r >= 0 && r < S.H && w >= 0 && w < S.W)
                    v[u] = ld4(st.srcb + (int64_t)(r * S.W + w) * S.pstride + st.ch0 + 4 * q);
            }
        } else {
            const int lpr = (WP + 63) >> 6;
            const int nlines = CB * NR * lpr;
#pragma unroll
            for (int u = 0; u < N; u++) {
                const int li = wid + 4 * u;              // (channel, row, pass), wave-uniform
                const int ch = li / (NR * lpr), rem = li - ch * (NR * lpr);
                const int rr = rem / lpr, h = rem - rr * lpr;
                const int cc = 64 * h + lane;
                const int r = st.r0 + rr * RS, w = st.c0 + cc;
                f[u] = 0.f;
                if (li < nlines && cc < WP && r >= 0 && r < S.H && w >= 0 && w < S.W)
                    f[u] = st.srcb[(int64_t)(r * S.W + w) * S.pstride + (int64_t)(st.ch0 + ch) * S.cstride];
            }
        }
    }
    __device__ __forceinline__ void store(float* band, int NR, int WP, int CB, int CS) const {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (VEC) {
            const int q4s = CB == 64 ? 4 : CB == 32 ? 3 : CB == 16 ? 2 : (CB == 8 ? 1 : 0);
            const int per_line = WP << q4s;
            const int lpr = (per_line + 63) >> 6;
            const int nlines = NR * lpr;
#pragma unroll
            for (int u = 0; u < N; u++) {
                const int li = wid + 4 * u;
                const int rr = li / lpr, h = li - rr * lpr;
                const int j = 64 * h + lane;
                const int cc = j >> q4s, q = j & ((1 << q4s) - 1);
                if (li < nlines && j < per_line) *reinterpret_cast<float4*>(band + (rr * WP + cc) * CS + 4 * q) = v[u];
            }
        } else {
            const int lpr = (WP + 63) >> 6;
            const int nlines = CB * NR * lpr;
#pragma unroll
            for (int u = 0; u < N; u++) {
                const int li = wid + 4 * u;
                const int ch = li / (NR * lpr), rem = li - ch * (NR * lpr);
                const int rr = rem / lpr, h = rem - rr * lpr;
                const int cc = 64 * h + lane;
                if (li < nlines && cc < WP) band[(rr * WP + cc) * CS + ch] = f[u];
            }
        }
    }
};

__device__ __forceinline__ const float* image_base(const CigSource& S, int z, int b) {
    const int64_t row = S.phys ? (int64_t)S.phys[b] : (int64_t)b;
    return S.base[z] + row * S.bstride + S.off;
}

// Forward / data-gradient GEMM, persistent: workgroup w takes tiles w, w + grid, ... in the
// order (stream, class, image, row tile), tile = TR class rows of one image (full width) x all N
// output channels.  4 waves as WM x WN, wave tile TM x TN 16x16 fragments (BN = WN*TN*16 = N).
// Per channel block the band is stored to LDS from registers, then the loads of the NEXT band
// (the next block, or block 0 of the next tile) are issued before this block's MFMAs, so HBM
// reads overlap the math instead of every workgroup of the chip staging in lockstep.
// C4: 4-channel input (the stacked frames): a 16-deep K chunk is 4 taps x 4 channels, lane
// group g takes tap 4*chunk + g.  Otherwise a chunk is one tap x 16 channels of the block.
template <int TM, int TN, int WM, bool C4, int EPI, bool VEC>
__global__ __launch_bounds__(256, 2) void k_conv_ig(ConvIgArgs a) {
    constexpr int WN = 4 / WM;
    extern __shared__ __attribute__((aligned(16))) float band[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid - (wid / WN) * WN;
    const int g = lane >> 4, i16 = lane & 15;
    const int per_cls = a.Bl * a.maxtiles, per_z = a.nclass * per_cls;
    const int total = a.nstreams * a.nclass * per_cls;
    const int C = a.src.C, CB = C4 ? 4 : a.CB;
    const int ncb = C / CB;
    const floatx4* band4 = reinterpret_cast<const floatx4*>(band);   // native vectors: one ds_read_b128
    const int CS4 = a.CS >> 2;
    const bool relu = a.act == DQNX_ACT_RELU;

    auto decode = [&](int T, int& z, int& cl, int& b, int& tile) {
        z = T / per_z;
        int rem = T - z * per_z;
        cl = rem / per_cls;
        rem -= cl * per_cls;
        b = rem / a.maxtiles;
        tile = rem - b * a.maxtiles;
    };
    auto next_valid = [&](int T) {   // first tile >= T of this workgroup's sequence that exists
        for (; T < total; T += gridDim.x) {
            int z, cl, b, tile;
            decode(T, z, cl, b, tile);
            if (tile < a.cls[cl].tiles) break;
        }
        return T;
    };
    const int ngrp = a.ngrp, nstage = ncb * ngrp;   // stage s = (channel block, row group)
    auto stage_of = [&](int T, int s) {
        int z, cl, b, tile;
        decode(T, z, cl, b, tile);
        const CigClass& K = a.cls[cl];
        const int cbk = s / ngrp, grp = s - cbk * ngrp;
        return Stage{image_base(a.src, z, b), tile * a.TR * a.SRM + K.rmin + grp, K.cmin, cbk * CB};
    };
    auto nr_of = [&](int s) { return ngrp > 1 ? a.gnr[s % ngrp] : a.NR; };

    int T = next_valid(blockIdx.x);
    if (T >= total) return;
    StageRegs<VEC> pre;   // the next band, loaded while the current one is multiplied
    pre.load(a.src, stage_of(T, 0), nr_of(0), a.WP, CB, a.RS);
    while (true) {
        int z, cl, b, tile;
        decode(T, z, cl, b, tile);
        const CigClass& K = a.cls[cl];
        const int Wq = K.Wq;
        const float invWq = 1.f / (float)Wq;
        const int y0 = tile * a.TR;
        const int mvalid = min(a.TR, K.Hq - y0) * Wq;
        const int Tn = next_valid(T + gridDim.x);

        if (EPI == CIG_EPI_FLAT && tile == 0) {   // torch.cat([micro, macro], dim=1) + zero padding
            float* F = a.out[z] + (int64_t)b * a.ob;
            const float* mac = a.ring[z] + (int64_t)a.phys[b] * a.ring_stride;
            for (int col = a.flat_cols + tid; col < a.strideF; col += 256)
                F[col] = col < a.flat_cols + a.macro_len ? mac[col - a.flat_cols] : 0.f;
        }

        int ppos4[TM];   // band position of this lane's A row (float4 units), per fragment
#pragma unroll
        for (int tm = 0; tm < TM; tm++) {
            int q = (wm * TM + tm) * 16 + i16;
            if (q >= mvalid) q = 0;
            int yl, xq;
            divmod_f(q, Wq, invWq, yl, xq);
            ppos4[tm] = (yl * a.RM * a.WP + xq * a.CM) * CS4;
        }
        const float* Wz = a.W[z];
        const float* wrow[TN];
#pragma unroll
        for (int tn = 0; tn < TN; tn++) wrow[tn] = Wz + (int64_t)((wn * TN + tn) * 16 + i16) * a.Kw;
        floatx4 acc[TM][TN];
#pragma unroll
        for (int tm = 0; tm < TM; tm++)
#pragma unroll
            for (int tn = 0; tn < TN; tn++) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
        // C^T = W X^T: the weights are the MFMA's A operand (rows = output channels), the band
        // pixels its B operand, so a lane's accumulator holds 4 consecutive channels of one pixel
        // (acc[tm][tn][r] = channel (wn*TN + tn)*16 + 4g + r of pixel (wm*TM + tm)*16 + i16):
        // NHWC outputs leave as float4 stores
        auto mma = [&](const floatx4 (&av)[TM], const float4 (&bq)[TN]) {
#pragma unroll
            for (int tm = 0; tm < TM; tm++)
#pragma unroll
                for (int tn = 0; tn < TN; tn++) {
                    acc[tm][tn] = mfma16x16x4(bq[tn].x, av[tm][0], acc[tm][tn]);
                    acc[tm][tn] = mfma16x16x4(bq[tn].y, av[tm][1], acc[tm][tn]);
                    acc[tm][tn] = mfma16x16x4(bq[tn].z, av[tm][2], acc[tm][tn]);
                    acc[tm][tn] = mfma16x16x4(bq[tn].w, av[tm][3], acc[tm][tn]);
                }
        };
        // stage s = (channel block cbk, row group grp): taps i = gi0 + ii*gdi (ii < gni), all j;
        // chunk r of a stage = (tap, sub): A at band4[ppos + toff*CS/4 + 4*sub + g], weights at
        // wtap*C + cbk*CB + 16*sub + 4g (uniform integer math, no table loads)
        const int nsub_s = C4 ? 0 : (CB == 64 ? 2 : CB == 32 ? 1 : 0);
        int cbk = 0, gi0 = K.i0, gdi = K.di, gni = K.ni, ntaps = K.ntaps, per_blk = 0;
        auto set_stage = [&](int s) {
            cbk = s / ngrp;
            const int grp = s - cbk * ngrp;
            gi0 = ngrp > 1 ? grp : K.i0;
            gdi = ngrp > 1 ? a.SRM : K.di;
            gni = ngrp > 1 ? a.gni[grp] : K.ni;
            ntaps = gni * K.nj;
            per_blk = C4 ? (ntaps + 3) >> 2 : ntaps << nsub_s;
        };
        auto chunk = [&](int r, int& aoff4, int& woff, bool& bv) {
            if (C4) {   // lane group g: tap 4r + g, its 4 channels
                const int t = 4 * r + g;
                bv = t < ntaps;
                const int ii = t / K.nj, jj = t - ii * K.nj;
                aoff4 = bv ? (K.o0 + ii * K.oi + jj * K.oj) * CS4 : 0;
                woff = ((gi0 + ii * gdi) * K.kw + K.j0 + jj * K.dj) * 4;
            } else {
                const int ti = r >> nsub_s, sub = r & ((1 << nsub_s) - 1);
                const int ii = ti / K.nj, jj = ti - ii * K.nj;
                bv = true;
                aoff4 = (K.o0 + ii * K.oi + jj * K.oj) * CS4 + 4 * sub + g;
                woff = ((gi0 + ii * gdi) * K.kw + K.j0 + jj * K.dj) * C + cbk * CB + 16 * sub + 4 * g;
            }
        };
        auto bload = [&](int r, float4 (&bb)[TN]) {
            int aoff4, woff;
            bool bv;
            chunk(r, aoff4, woff, bv);
#pragma unroll
            for (int tn = 0; tn < TN; tn++) bb[tn] = bv ? ld4(wrow[tn] + woff) : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        // one chunk: the next chunk's weights into `nxt` while `cur` is multiplied (two named
        // register sets, chunk loop unrolled by 2: no copies, so the wait for `cur` does not
        // also wait for the prefetch)
        auto step = [&](int r, const float4 (&cur)[TN], float4 (&nxt)[TN]) {
            int aoff4, woff;
            bool bv;
            chunk(r, aoff4, woff, bv);
            if (r + 1 < per_blk) bload(r + 1, nxt);
            // keep the prefetch at the top of the chunk: under register pressure the scheduler
            // otherwise sinks it below the MFMAs, exposing the L2 latency at every chunk
            __builtin_amdgcn_sched_barrier(0);
            floatx4 av[TM];
#pragma unroll
            for (int tm = 0; tm < TM; tm++) av[tm] = band4[ppos4[tm] + aoff4];
            mma(av, cur);
        };
        for (int s = 0; s < nstage; s++) {
            set_stage(s);
            float4 b0[TN], b1[TN];
            bload(0, b0);
            __syncthreads();   // the previous stage's A reads are done
            pre.store(band, nr_of(s), a.WP, CB, a.CS);
            __syncthreads();
            if (s + 1 < nstage) pre.load(a.src, stage_of(T, s + 1), nr_of(s + 1), a.WP, CB, a.RS);
            else if (Tn < total) pre.load(a.src, stage_of(Tn, 0), nr_of(0), a.WP, CB, a.RS);
            int r = 0;
            for (; r + 1 < per_blk; r += 2) {
                step(r, b0, b1);
                step(r + 1, b1, b0);
            }
            if (r < per_blk) step(r, b0, b1);
        }

        // epilogue: lane holds pixel q = (wm*TM + tm)*16 + i16, channels n = (wn*TN + tn)*16 + 4g + r.
        // VALU here costs 4 cycles per instruction per wave against 32 per MFMA: the forward
        // uses the tile's linear pixel index (a tile is whole class rows of one image, no
        // divisions) and 32-bit offsets inside the image
        float* outb = a.out[z] + (int64_t)b * a.ob;
        if (EPI == CIG_EPI_DX) {   // NHWC (och 1): float4 of Hprev in, float4 out
            const float* hb = a.Hprev + (int64_t)b * a.ob;
#pragma unroll
            for (int tm = 0; tm < TM; tm++) {
                const int q = (wm * TM + tm) * 16 + i16;
                int yl, xq;
                divmod_f(min(q, mvalid - 1), Wq, invWq, yl, xq);
                const int o = (a.ymul * (y0 + yl) + K.a) * a.orow + (a.xmul * xq + K.c) * a.opix;
                float4 h[TN];
#pragma unroll
                for (int tn = 0; tn < TN; tn++) h[tn] = ld4(hb + o + (wn * TN + tn) * 16 + 4 * g);
                if (q >= mvalid) continue;
#pragma unroll
                for (int tn = 0; tn < TN; tn++) {
                    float d[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float v = acc[tm][tn][r], hv = (&h[tn].x)[r];
                        d[r] = relu ? (hv > 0.f ? v : 0.f) : (hv > 0.f ? v : v * (hv + 1.f));
                    }
                    *reinterpret_cast<float4*>(outb + o + (wn * TN + tn) * 16 + 4 * g) = make_float4(d[0], d[1], d[2], d[3]);
                }
            }
        } else {
            float bias[TN][4];
#pragma unroll
            for (int tn = 0; tn < TN; tn++)
#pragma unroll
                for (int r = 0; r < 4; r++) bias[tn][r] = a.bias[z][(wn * TN + tn) * 16 + 4 * g + r];
            outb += (int64_t)y0 * Wq * a.opix;   // the tile's first pixel
#pragma unroll
            for (int tm = 0; tm < TM; tm++) {
                const int q = (wm * TM + tm) * 16 + i16;
                if (q >= mvalid) continue;
#pragma unroll
                for (int tn = 0; tn < TN; tn++) {
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float x = acc[tm][tn][r] + bias[tn][r];
                        // ELU as exp(x) - 1 (v_exp_f32): within ~1e-7 absolute of expm1, the
                        // parity tolerance is 1e-5
                        v[r] = x > 0.f ? x : (relu ? 0.f : __expf(x) - 1.f);
                    }
                    const int n0 = (wn * TN + tn) * 16 + 4 * g;
                    if (EPI == CIG_EPI_NHWC) {
                        *reinterpret_cast<float4*>(outb + q * a.opix + n0) = make_float4(v[0], v[1], v[2], v[3]);
                    } else {   // CHW flatten: consecutive lanes on consecutive pixels of a channel row
#pragma unroll
                        for (int r = 0; r < 4; r++) outb[q + (n0 + r) * a.och] = v[r];
                    }
                }
            }
        }
        T = Tn;
        if (T >= total) break;
    }
}

// Weight gradient.  Workgroup = (slice of output row groups, input channel block); waves
// (wm, ks): wm picks 16 output channels (A rows), the KS = 4/WM waves of one wm split the
// pixel chunks and are summed in LDS at the end (fixed order).  Columns n = tap * CB + ch.
template <int TN, int WM, bool VEC>
__global__ __launch_bounds__(256, 2) void k_conv_dw_ig(ConvDwIgArgs a) {
    constexpr int KS = 4 / WM;
    extern __shared__ __attribute__((aligned(16))) float band[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid % WM, ks = wid / WM;
    const int g = lane >> 4, i16 = lane & 15;
    const int ncb = a.C / a.CB;
    const int T = xcd_remap(blockIdx.x, gridDim.x);
    const int s = T / ncb, cbk = T - s * ncb;
    const int co = wm * 16 + i16;   // this lane's A row
    int coff[TN];
    bool cval[TN];
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        const int n = tn * 16 + i16;
        const int ti = n / a.CB, ch = n - ti * a.CB;
        cval[tn] = ti < a.ntaps;
        const int i = ti / a.kw, j = ti - i * a.kw;
        coff[tn] = cval[tn] ? (i * a.WP + j) * a.CS + ch : 0;
    }
    floatx4 acc[TN];
#pragma unroll
    for (int tn = 0; tn < TN; tn++) acc[tn] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;
    const float invWo = 1.f / (float)a.Wo;
    const int gend = min((s + 1) * a.gps, a.Bl * a.G);
    auto stage_of = [&](int gi) {
        const int b = gi / a.G, grp = gi - b * a.G;
        return Stage{image_base(a.X, 0, b), grp * a.RB * a.sh - a.ph, -a.pw, cbk * a.CB};
    };
    StageRegs<VEC> pre;   // the next row group's X band, loaded while this one is multiplied
    if (s * a.gps < gend) pre.load(a.X, stage_of(s * a.gps), a.NR, a.WP, a.CB);
    for (int gi = s * a.gps; gi < gend; gi++) {
        const int b = gi / a.G, grp = gi - b * a.G;
        const int ho0 = grp * a.RB;
        const int npix = min(a.RB, a.Ho - ho0) * a.Wo;
        __syncthreads();   // the previous group's band reads are done
        pre.store(band, a.NR, a.WP, a.CB, a.CS);
        __syncthreads();
        if (gi + 1 < gend) pre.load(a.X, stage_of(gi + 1), a.NR, a.WP, a.CB);
        const float* dzb = a.dZ + (int64_t)b * a.dzb + (int64_t)co * a.dzc + (int64_t)ho0 * a.Wo * a.dzp;
        const int nck = (npix + 15) >> 4;
        float av[4];
        int pp[4];
        auto fetch = [&](int ck, float (&A)[4], int (&P)[4]) {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int u = ck * 16 + 4 * g + jj;
                int r, wo;
                divmod_f(u, a.Wo, invWo, r, wo);
                const bool v = u < npix;
                A[jj] = v ? dzb[(int64_t)u * a.dzp] : 0.f;
                P[jj] = v ? (r * a.sh * a.WP + wo * a.sw) * a.CS : 0;
            }
        };
        // dZ of the next two chunks in flight while this one is multiplied
        float a1[4], a2[4];
        int p1[4], p2[4];
        if (ks < nck) fetch(ks, av, pp);
        if (ks + KS < nck) fetch(ks + KS, a1, p1);
        for (int ck = ks; ck < nck; ck += KS) {
            if (ck + 2 * KS < nck) fetch(ck + 2 * KS, a2, p2);
            __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of this chunk's work
            float bv[TN][4];
#pragma unroll
            for (int tn = 0; tn < TN; tn++)
#pragma unroll
                for (int jj = 0; jj < 4; jj++) bv[tn][jj] = cval[tn] ? band[pp[jj] + coff[tn]] : 0.f;
            bsum += (av[0] + av[1]) + (av[2] + av[3]);
#pragma unroll
            for (int jj = 0; jj < 4; jj++)
#pragma unroll
                for (int tn = 0; tn < TN; tn++) acc[tn] = mfma16x16x4(av[jj], bv[tn][jj], acc[tn]);
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                av[jj] = a1[jj]; pp[jj] = p1[jj];
                a1[jj] = a2[jj]; p1[jj] = p2[jj];
            }
        }
    }
    __syncthreads();   // band reads done before the KS reduce reuses it
    // bias: sum over the 4 lane groups, then over the KS waves
    bsum += __shfl_xor(bsum, 16);
    bsum += __shfl_xor(bsum, 32);
    if (KS > 1) {   // ks > 0 waves hand their sums to ks = 0 through LDS (band is free now)
        float* red = band;
        if (ks > 0) {
            float* dst = red + ((ks - 1) * WM + wm) * (TN * 4 + 1) * 64;
#pragma unroll
            for (int tn = 0; tn < TN; tn++)
#pragma unroll
                for (int r = 0; r < 4; r++) dst[(tn * 4 + r) * 64 + lane] = acc[tn][r];
            dst[TN * 4 * 64 + lane] = bsum;
        }
        __syncthreads();
        if (ks > 0) return;
        for (int k2 = 1; k2 < KS; k2++) {
            const float* src = red + ((k2 - 1) * WM + wm) * (TN * 4 + 1) * 64;
#pragma unroll
            for (int tn = 0; tn < TN; tn++)
#pragma unroll
                for (int r = 0; r < 4; r++) acc[tn][r] += src[(tn * 4 + r) * 64 + lane];
            bsum += src[TN * 4 * 64 + lane];
        }
    }
    float* part = a.partial + (int64_t)s * a.pstride;
    const int taps_all = a.K / a.C;
#pragma unroll
    for (int tn = 0; tn < TN; tn++) {
        if (!cval[tn]) continue;
        const int n = tn * 16 + i16;
        const int ti = n / a.CB, ch = n - ti * a.CB;
        const int ci = cbk * a.CB + ch;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int orow = wm * 16 + 4 * g + r;
            part[(int64_t)orow * a.K + ci * taps_all + ti] = acc[tn][r];
        }
    }
    if (cbk == 0 && g == 0) part[(int64_t)a.Co * a.K + co] = bsum;
}

__global__ __launch_bounds__(256) void k_conv_perm(ConvPermArgs a) {
    const ConvPermJob& J = a.job[blockIdx.y];
    const int total = J.Co * J.Ci * J.taps;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
        int co, ci, t;
        if (J.mode == 0) {   // dst [co][t][ci]
            ci = e % J.Ci;
            const int r = e / J.Ci;
            t = r % J.taps;
            co = r / J.taps;
        } else {             // dst [ci][t][co]
            co = e % J.Co;
            const int r = e / J.Co;
            t = r % J.taps;
            ci = r / J.taps;
        }
        J.dst[e] = J.src[((int64_t)co * J.Ci + ci) * J.taps + t];
    }
}

// dF (rows in CHW-flatten order, R:env/dqn_config.py:135-137) -> the last conv's dZ in NHWC,
// as an LDS-tiled transpose: workgroup (b, 64-pixel tile) reads C rows of 64 pixels (coalesced
// along pixels) and writes 64 pixels x C channels (coalesced along channels).  A copy.
__global__ __launch_bounds__(256) void k_unflatten_tiled(UnflattenArgs a) {
    __shared__ float tile[64 * 65];
    const int HoWo = a.Ho * a.Wo, nt = (HoWo + 63) / 64;
    const int b = blockIdx.x / nt, p0 = (blockIdx.x - b * nt) * 64;
    const int np = min(64, HoWo - p0);
    const float* src = a.dF + (int64_t)b * a.ldf + p0;
    float* dst = a.dZ + ((int64_t)b * HoWo + p0) * a.C;
    for (int c0 = 0; c0 < a.C; c0 += 64) {
        const int nc = min(64, a.C - c0);
        for (int t = threadIdx.x; t < 64 * nc; t += 256) {
            const int c = t >> 6, p = t & 63;
            if (p < np) tile[c * 65 + p] = src[(int64_t)(c0 + c) * HoWo + p];
        }
        __syncthreads();
        for (int t = threadIdx.x; t < np * nc; t += 256) {
            const int p = t / nc, c = t - p * nc;
            dst[(int64_t)p * a.C + c0 + c] = tile[c * 65 + p];
        }
        __syncthreads();
    }
}

// persistent grid: the workgroups that fit the chip at once (occupancy by registers and LDS),
// at most one per tile; DQNX_CIG_OCC overrides the workgroups per CU
int persistent_grid(const void* fn, size_t lds, int64_t tiles) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int> occ_cache;
    static int cus = 0;
    int occ = 0;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!cus) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                cus = 256;
        }
        auto it = occ_cache.find({fn, lds});
        if (it != occ_cache.end()) {
            occ = it->second;
        } else {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, lds) != hipSuccess || occ < 1) occ = 1;
            occ_cache[{fn, lds}] = occ;
        }
    }
    occ = std::max(1, tuning_knob("DQNX_CIG_OCC", occ));
    return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, (int64_t)occ * cus));
}

template <class KernelT>
int launch_persistent(KernelT fn, const ConvIgArgs& a, size_t lds, hipStream_t s) {
    const int64_t tiles = (int64_t)a.nstreams * a.nclass * a.Bl * a.maxtiles;
    const int grid = persistent_grid(reinterpret_cast<const void*>(fn), lds, tiles);
    DQNX_LAUNCH(fn, dim3(grid), dim3(256), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

template <int TM, int TN, int WM>
int launch_tile(const ConvIgArgs& a, int epi, size_t lds, bool c4, hipStream_t s) {
    const bool vec = a.src.cstride == 1;
    if (c4) {   // the stacked frames, CHW ring rows
        if (vec) return set_error(DQNX_EUNSUPPORTED, "conv_ig: 4-channel NHWC source");
        if (epi == CIG_EPI_NHWC) return launch_persistent(k_conv_ig<TM, TN, WM, true, CIG_EPI_NHWC, false>, a, lds, s);
        if (epi == CIG_EPI_FLAT) return launch_persistent(k_conv_ig<TM, TN, WM, true, CIG_EPI_FLAT, false>, a, lds, s);
        return set_error(DQNX_EUNSUPPORTED, "conv_ig: 4-channel data gradient");
    }
    if (!vec) return set_error(DQNX_EUNSUPPORTED, "conv_ig: CHW source with C %d", a.src.C);
    if (epi == CIG_EPI_DX) return launch_persistent(k_conv_ig<TM, TN, WM, false, CIG_EPI_DX, true>, a, lds, s);
    if (epi == CIG_EPI_NHWC) return launch_persistent(k_conv_ig<TM, TN, WM, false, CIG_EPI_NHWC, true>, a, lds, s);
    return launch_persistent(k_conv_ig<TM, TN, WM, false, CIG_EPI_FLAT, true>, a, lds, s);
}

}  // namespace

size_t conv_ig_lds_bytes(const ConvIgArgs& a) { return (size_t)a.NR * a.WP * a.CS * sizeof(float); }

bool conv_ig_supported(int N, int BM, int C) {
    if (N != 32 && N != 64) return false;
    if (BM != 64 && BM != 128 && BM != 256) return false;
    return C == 4 || C % 16 == 0;
}

int launch_conv_ig(const ConvIgArgs& a, int epi, hipStream_t s) {
    if (!conv_ig_supported(a.N, a.BM, a.src.C)) return set_error(DQNX_EUNSUPPORTED, "conv_ig: N %d BM %d C %d", a.N, a.BM, a.src.C);
    const size_t lds = conv_ig_lds_bytes(a);
    if (lds > 160 * 1024) return set_error(DQNX_EUNSUPPORTED, "conv_ig: band of %zu B exceeds LDS", lds);
    const bool c4 = a.src.C == 4;
    if (a.N == 32) {
        if (a.BM == 256) return launch_tile<4, 2, 4>(a, epi, lds, c4, s);
        if (a.BM == 128) return launch_tile<2, 2, 4>(a, epi, lds, c4, s);
        return launch_tile<1, 2, 4>(a, epi, lds, c4, s);
    }
    if (a.BM == 256) return launch_tile<8, 2, 2>(a, epi, lds, c4, s);
    if (a.BM == 128) return launch_tile<4, 2, 2>(a, epi, lds, c4, s);
    return launch_tile<4, 1, 1>(a, epi, lds, c4, s);
}

size_t conv_dw_ig_lds_bytes(const ConvDwIgArgs& a) {
    const size_t bandf = (size_t)a.NR * a.WP * a.CS;
    const size_t redf = (size_t)4 * (a.TN * 4 + 1) * 64;
    return (bandf > redf ? bandf : redf) * sizeof(float);
}

int launch_conv_dw_ig(const ConvDwIgArgs& a, hipStream_t s) {
    const size_t lds = conv_dw_ig_lds_bytes(a);
    if (lds > 160 * 1024) return set_error(DQNX_EUNSUPPORTED, "conv_dw_ig: band of %zu B exceeds LDS", lds);
    const dim3 grid((unsigned)((int64_t)a.slices * (a.C / a.CB)));
    const bool vec = a.X.cstride == 1;
    if (a.Co == 64 && a.TN == 9 && vec) DQNX_LAUNCH((k_conv_dw_ig<9, 4, true>), grid, dim3(256), lds, s, a);
    else if (a.Co == 32 && a.TN == 9 && vec) DQNX_LAUNCH((k_conv_dw_ig<9, 2, true>), grid, dim3(256), lds, s, a);
    else if (a.Co == 64 && a.TN == 3 && !vec) DQNX_LAUNCH((k_conv_dw_ig<3, 4, false>), grid, dim3(256), lds, s, a);
    else if (a.Co == 32 && a.TN == 3 && !vec) DQNX_LAUNCH((k_conv_dw_ig<3, 2, false>), grid, dim3(256), lds, s, a);
    else return set_error(DQNX_EUNSUPPORTED, "conv_dw_ig: Co %d TN %d", a.Co, a.TN);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_unflatten_tiled(const UnflattenArgs& a, hipStream_t s) {
    const int nt = (a.Ho * a.Wo + 63) / 64;
    DQNX_LAUNCH(k_unflatten_tiled, dim3((unsigned)((int64_t)a.Bl * nt)), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_conv_perm(const ConvPermArgs& a, hipStream_t s) {
    if (a.njobs <= 0) return DQNX_OK;
    DQNX_LAUNCH(k_conv_perm, dim3(64, a.njobs), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
