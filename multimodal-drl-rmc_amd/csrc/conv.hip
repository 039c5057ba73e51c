// Data movement of the two-stream hybrid Q-network (TwoStreamHybridNetwork,
// R:env/dqn_config.py:66-143): im2col / col2im around the MFMA GEMMs that carry the
// convolutions, and the flatten + concat in front of the dense stream.
//
// Layouts.  The obs row is [macro (macro_len) | micro grid (c,h,w) flattened CHW]
// (R:env/dqn_config.py:126-133).  Conv activations are kept in GEMM layout
// [rows = (b, ho, wo)][channels] (NHWC), so a conv is C[m][n] = A[m][k] W[n][k] with
// k = (ci, i, j): torch's weight [Cout][Cin][kh][kw] is already row n = output channel,
// K-contiguous, so the weight needs no permutation.  The dense stream's input is
// cat(flatten_CHW(last conv), macro) (:135-138), materialised as F[b][strideF].
#include "learn.hpp"

namespace dqnx {

// One wave per output row (z, b, ho, wo): the row's decomposition is computed once, the 64
// lanes write 64 consecutive columns (coalesced), 32-bit index math throughout.
__global__ __launch_bounds__(256) void k_im2col_rows(Im2colArgs a) {
    const int lane = threadIdx.x & 63;
    const int rows = a.M * a.nstreams;
    const int HoWo = a.Ho * a.Wo, KK = a.kh * a.kw;
    const int wave0 = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
    for (int r = wave0; r < rows; r += nwaves) {
        const int z = r / a.M, m = r - z * a.M;
        const int b = m / HoWo, p = m - b * HoWo;
        const int ho = p / a.Wo, wo = p - ho * a.Wo;
        const int h0 = ho * a.sh - a.ph, w0 = wo * a.sw - a.pw;
        const float* ring = a.ring[z];
        const float* src = a.src[z];
        const int64_t rbase = ring ? (int64_t)a.phys[b] * a.ring_stride + a.ring_off : 0;
        float* out = a.col[z] + (int64_t)m * a.Kstride;
        for (int kk = lane; kk < a.Kstride; kk += 64) {
            float v = 0.f;
            if (kk < a.K) {
                const int ci = kk / KK, rr = kk - ci * KK;
                const int i = rr / a.kw, j = rr - i * a.kw;
                const int h = h0 + i, w = w0 + j;
                if (h >= 0 && h < a.Hi && w >= 0 && w < a.Wi) {
                    if (ring) v = ring[rbase + (ci * a.Hi + h) * a.Wi + w];   // CHW micro grid
                    else v = src[((int64_t)(b * a.Hi + h) * a.Wi + w) * a.Ci + ci];   // NHWC
                }
            }
            out[kk] = v;
        }
    }
}

// Small K (conv 1: Cin*9 = 18 or 36, where a wave per row leaves most lanes idle): one thread
// per element (z, b, ho, wo, k) of the column matrices, k fastest, stores coalesced.  Reads: the micro grid straight from the ring (conv 1, CHW) or
// the previous conv's NHWC activations.
__global__ __launch_bounds__(256) void k_im2col_flat(Im2colArgs a) {
    const int64_t rows = (int64_t)a.M * a.nstreams;
    const int64_t total = rows * a.Kstride;
    const int HoWo = a.Ho * a.Wo, KK = a.kh * a.kw;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / a.Kstride;
        const int kk = (int)(t - r * a.Kstride);
        const int z = (int)(r / a.M), m = (int)(r - (int64_t)z * a.M);
        float v = 0.f;
        if (kk < a.K) {
            const int b = m / HoWo, p = m - b * HoWo;
            const int ho = p / a.Wo, wo = p - ho * a.Wo;
            const int ci = kk / KK, rr = kk - ci * KK;
            const int i = rr / a.kw, j = rr - i * a.kw;
            const int h = ho * a.sh - a.ph + i, w = wo * a.sw - a.pw + j;
            if (h >= 0 && h < a.Hi && w >= 0 && w < a.Wi) {
                const float* ring = a.ring[z];
                if (ring) v = ring[(int64_t)a.phys[b] * a.ring_stride + a.ring_off + (ci * a.Hi + h) * a.Wi + w];   // CHW
                else v = a.src[z][((int64_t)(b * a.Hi + h) * a.Wi + w) * a.Ci + ci];                              // NHWC
            }
        }
        a.col[z][(int64_t)m * a.Kstride + kk] = v;
    }
}

// One workgroup per output image row (z, b, ho): the kh input rows it reads (all Ci channels,
// all Wi columns, zeros outside the image) are staged once into LDS as [i][ci][w] with
// coalesced global reads, then the Wo output rows -- one contiguous [Wo][Kstride] block of the
// column matrix -- are written with consecutive threads on consecutive addresses.  The
// row-per-wave kernel above reads the NHWC source at a 4*Ci-byte stride across lanes (k runs
// over (ci, i, j)), i.e. about one cache line per element; here every input byte of the row
// band is read once per band.  Bit-identical output (a copy).
// Channel groups (grid.x = rows * G): workgroup g of a row stages channels [g*Cg, (g+1)*Cg) only
// and writes their column range [g*Cg*KK, ...) of each of the Wo rows (the last group also
// the zero padding up to Kstride), keeping the band at <= 32 KB.
__global__ __launch_bounds__(256) void k_im2col_lds(Im2colArgs a, int G) {
    extern __shared__ float band[];   // [kh][Cg][Wi], then the per-column table
    const int HoWo = a.Ho * a.Wo, KK = a.kh * a.kw;
    const int Bl = a.M / HoWo;
    const int blk = blockIdx.x / G, grp = blockIdx.x - (blockIdx.x / G) * G;
    const int z = blk / (Bl * a.Ho);
    const int rem = blk - z * Bl * a.Ho;
    const int b = rem / a.Ho, ho = rem - b * a.Ho;
    const int hbase = ho * a.sh - a.ph;
    const int Cg = a.Ci / G, c0 = grp * Cg;
    const int kk0 = c0 * KK, kk1 = grp == G - 1 ? a.Kstride : (c0 + Cg) * KK, Wk = kk1 - kk0;
    const int CW = Cg * a.Wi;
    const int nband = a.kh * CW;
    int* tab = reinterpret_cast<int*>(band + nband);   // local column -> (band offset of (i, ci, w=j) << 8) | j, or -1
    const int tid = threadIdx.x;
    // index math is incremental (one division per thread up front): at these sizes the
    // per-element divisions, not the bytes, were the cost
    for (int kl = tid; kl < Wk; kl += 256) {
        const int kk = kk0 + kl;
        int v = -1;
        if (kk < a.K) {
            const int ci = kk / KK - c0, rr = kk - (ci + c0) * KK;
            const int i = rr / a.kw, j = rr - i * a.kw;
            v = (((i * Cg + ci) * a.Wi + j) << 8) | j;
        }
        tab[kl] = v;
    }
    const float* ring = a.ring[z];
    for (int i = 0; i < a.kh; i++) {
        const int h = hbase + i;
        const bool inside = h >= 0 && h < a.Hi;
        float* dst = band + i * CW;
        if (ring) {   // conv 1: CHW micro grid inside the ring row, w fastest
            const float* src = ring + (int64_t)a.phys[b] * a.ring_stride + a.ring_off + h * a.Wi + (int64_t)c0 * a.Hi * a.Wi;
            const int sw_ = 256 / a.Wi, sr = 256 - sw_ * a.Wi;
            int ci = tid / a.Wi, w = tid - ci * a.Wi;
            for (int t = tid; t < CW; t += 256) {
                dst[t] = inside ? src[ci * a.Hi * a.Wi + w] : 0.f;
                ci += sw_; w += sr;
                if (w >= a.Wi) { w -= a.Wi; ci++; }
            }
        } else {      // NHWC activations, ci fastest (coalesced), transposed into [ci][w]
            const float* src = a.src[z] + ((int64_t)(b * a.Hi + h) * a.Wi) * a.Ci + c0;
            const int sw_ = 256 / Cg, sc = 256 - sw_ * Cg;
            int w = tid / Cg, ci = tid - w * Cg;
            for (int t = tid; t < CW; t += 256) {
                dst[ci * a.Wi + w] = inside ? src[(int64_t)w * a.Ci + ci] : 0.f;
                w += sw_; ci += sc;
                if (ci >= Cg) { ci -= Cg; w++; }
            }
        }
    }
    __syncthreads();
    float* out = a.col[z] + ((int64_t)b * HoWo + (int64_t)ho * a.Wo) * a.Kstride + kk0;
    if ((Wk & 3) == 0 && (kk0 & 3) == 0 && (a.Kstride & 3) == 0) {   // 16-byte stores
        const int W4 = Wk >> 2, total = a.Wo * W4;
        const int so = 256 / W4, sk = 256 - so * W4;
        int wo = tid / W4, q = tid - wo * W4;
        for (int t = tid; t < total; t += 256) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int e = tab[4 * q + u];
                const int w = wo * a.sw - a.pw + (e & 255);
                v[u] = (e >= 0 && w >= 0 && w < a.Wi) ? band[(e >> 8) + wo * a.sw - a.pw] : 0.f;
            }
            *reinterpret_cast<float4*>(out + (int64_t)wo * a.Kstride + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
            wo += so; q += sk;
            if (q >= W4) { q -= W4; wo++; }
        }
        return;
    }
    const int total = a.Wo * Wk;
    const int so = 256 / Wk, sk = 256 - so * Wk;
    int wo = tid / Wk, kl = tid - wo * Wk;
    for (int t = tid; t < total; t += 256) {
        const int e = tab[kl];
        const int w = wo * a.sw - a.pw + (e & 255);
        out[(int64_t)wo * a.Kstride + kl] = (e >= 0 && w >= 0 && w < a.Wi) ? band[(e >> 8) + wo * a.sw - a.pw] : 0.f;
        wo += so; kl += sk;
        if (kl >= Wk) { kl -= Wk; wo++; }
    }
}

// flatten_CHW as a tiled transpose: workgroup (z, b, tile) reads 64 pixels x C channels of the
// NHWC activations (one contiguous block) into LDS and writes them channel-major (64-float runs
// of F); the extra tile per (z, b) writes the macro features and the zero padding.  The
// element-wise kernel above reads NHWC at a C-float stride across lanes.  Same values.
__global__ __launch_bounds__(256) void k_flatten_concat_tiled(FlattenArgs a) {
    __shared__ float tile[64 * 129];
    const int HoWo = a.Ho * a.Wo, C = a.C, CHW = C * HoWo;
    const int ntiles = (HoWo + 63) / 64;
    const int per_b = ntiles + 1;
    const int z = blockIdx.x / (a.Bl * per_b);
    const int rem = blockIdx.x - z * a.Bl * per_b;
    const int b = rem / per_b, tt = rem - b * per_b;
    float* F = a.F[z] + (int64_t)b * a.strideF;
    if (tt == ntiles) {   // torch.cat([micro, macro], dim=1) + zero padding to strideF
        const float* mac = a.ring[z] + (int64_t)a.phys[b] * a.ring_stride;
        for (int col = CHW + threadIdx.x; col < a.strideF; col += 256)
            F[col] = col < CHW + a.macro_len ? mac[col - CHW] : 0.f;
        return;
    }
    const int hw0 = tt * 64, nhw = min(64, HoWo - hw0);
    const float* src = a.Hc[z] + ((int64_t)b * HoWo + hw0) * C;
    for (int t = threadIdx.x; t < nhw * C; t += 256) {
        const int hl = t / C, c = t - hl * C;
        tile[hl * (C + 1) + c] = src[t];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < 64 * C; t += 256) {
        const int c = t >> 6, hl = t & 63;
        if (hl < nhw) F[(int64_t)c * HoWo + hw0 + hl] = tile[hl * (C + 1) + c];
    }
}

__global__ __launch_bounds__(256) void k_flatten_concat(FlattenArgs a) {
    const int64_t per = (int64_t)a.Bl * a.strideF;
    const int64_t total = per * a.nstreams;
    const int HoWo = a.Ho * a.Wo, CHW = a.C * HoWo;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int z = (int)(t / per);
        const int64_t rem = t - (int64_t)z * per;
        const int b = (int)(rem / a.strideF);
        const int col = (int)(rem - (int64_t)b * a.strideF);
        float v = 0.f;
        if (col < CHW) {                  // processed_micro_4d.flatten(start_dim=1): (c, h, w)
            const int c = col / HoWo, hw = col - c * HoWo;
            v = a.Hc[z][((int64_t)b * HoWo + hw) * a.C + c];
        } else if (col < CHW + a.macro_len) {   // torch.cat([micro, macro], dim=1)
            v = a.ring[z][(int64_t)a.phys[b] * a.ring_stride + (col - CHW)];
        }
        a.F[z][(int64_t)b * a.strideF + col] = v;
    }
}

// dF (CHW-flatten order, already masked by the conv's activation) -> dZ rows (NHWC)
__global__ __launch_bounds__(256) void k_unflatten(UnflattenArgs a) {
    const int HoWo = a.Ho * a.Wo;
    const int64_t total = (int64_t)a.Bl * HoWo * a.C;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(t % a.C);
        const int64_t mrow = t / a.C;
        const int b = (int)(mrow / HoWo), hw = (int)(mrow - (int64_t)b * HoWo);
        a.dZ[t] = a.dF[(int64_t)b * a.ldf + (int64_t)c * HoWo + hw];
    }
}

// dX (NHWC) = col2im(dCol), gather form (fixed (i, j) order, deterministic), then the
// previous conv's activation backward: dZprev = act'(Hprev) (.) dX.
template <int ACT>
__global__ __launch_bounds__(256) void k_col2im(Col2imArgs a) {
    const int total = a.Bl * a.Hi * a.Wi * a.Ci;
    const int KK = a.kh * a.kw;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int ci = t % a.Ci;
        int q = t / a.Ci;
        const int w = q % a.Wi;
        q /= a.Wi;
        const int h = q % a.Hi;
        const int b = q / a.Hi;
        float s = 0.f;
        for (int i = 0; i < a.kh; i++) {
            const int hh = h + a.ph - i;
            if (hh < 0 || hh % a.sh) continue;
            const int ho = hh / a.sh;
            if (ho >= a.Ho) continue;
            for (int j = 0; j < a.kw; j++) {
                const int ww = w + a.pw - j;
                if (ww < 0 || ww % a.sw) continue;
                const int wo = ww / a.sw;
                if (wo >= a.Wo) continue;
                const int64_t m = ((int64_t)b * a.Ho + ho) * a.Wo + wo;
                s += a.dcol[m * a.ldcol + (ci * KK + i * a.kw + j)];
            }
        }
        a.dZprev[t] = act_bwd<ACT>(s, a.Hprev[t]);
    }
}

// k_col2im for the reference's 3x3 / padding-1 convs with strides SH x SW fixed at compile time
// and a power-of-two channel count: the per-element index math of the generic kernel (runtime
// divisions and remainders by Ci, Wi, Hi, the strides) was its cost, not its bytes.  Same (i, j)
// order, same sums.
template <int ACT, int SH, int SW>
__global__ __launch_bounds__(256) void k_col2im_3x3(Col2imArgs a, int ci_shift) {
    const int total = a.Bl * a.Hi * a.Wi * a.Ci;
    const int cmask = a.Ci - 1;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int ci = t & cmask;
        const int q = t >> ci_shift;
        const int bh = q / a.Wi, w = q - bh * a.Wi;
        const int b = bh / a.Hi, h = bh - b * a.Hi;
        const float* dc = a.dcol + ci * 9;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const int hh = h + 1 - i;
            if (hh < 0 || hh % SH) continue;
            const int ho = hh / SH;
            if (ho >= a.Ho) continue;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const int ww = w + 1 - j;
                if (ww < 0 || ww % SW) continue;
                const int wo = ww / SW;
                if (wo >= a.Wo) continue;
                const int64_t m = ((int64_t)b * a.Ho + ho) * a.Wo + wo;
                s += dc[m * a.ldcol + i * 3 + j];
            }
        }
        a.dZprev[t] = act_bwd<ACT>(s, a.Hprev[t]);
    }
}

template <int SH, int SW>
static void launch_col2im_3x3(const Col2imArgs& a, int act, int shift, dim3 g, hipStream_t s) {
    if (act == DQNX_ACT_RELU) DQNX_LAUNCH((k_col2im_3x3<DQNX_ACT_RELU, SH, SW>), g, dim3(256), 0, s, a, shift);
    else DQNX_LAUNCH((k_col2im_3x3<DQNX_ACT_ELU, SH, SW>), g, dim3(256), 0, s, a, shift);
}

static dim3 grid_for(int64_t total) {
    int64_t g = (total + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return dim3((unsigned)g);
}

int im2col_mode() {
    static int mode = -1;   // DQNX_IM2COL: 0 = flat/row kernels only, 1 = LDS band kernel where it fits (default)
    if (mode < 0) {
        mode = tuning_knob("DQNX_IM2COL", 1);
    }
    return mode;
}

int launch_im2col(const Im2colArgs& a, hipStream_t s) {
    // channel groups: the smallest G dividing Ci whose band fits 32 KB
    int G = 1;
    while (G < a.Ci && ((size_t)a.kh * (a.Ci / G) * a.Wi * sizeof(float) > 32 * 1024 || a.Ci % G)) G++;
    const size_t band = (size_t)a.kh * (a.Ci / G) * a.Wi * sizeof(float) + (size_t)a.Kstride * sizeof(int);
    // the band kernel pays off when one output image row is a large block (the (4,84,84)
    // variant); the (2,27,5) grid's rows are a few KB and stay on the kernels below.
    // measured on the (4,84,84) variant, B=256: conv 1 819 -> 263 us, conv 2 2102 -> 1156 us
    if (im2col_mode() == 1 && band <= 64 * 1024 && a.M % (a.Ho * a.Wo) == 0 && a.Wo * a.Kstride >= 2048 &&
        a.kw < 256 && (size_t)a.kh * a.Ci * a.Wi < (1u << 23)) {
        const int64_t g = (int64_t)a.nstreams * (a.M / (a.Ho * a.Wo)) * a.Ho * G;
        DQNX_LAUNCH(k_im2col_lds, dim3((unsigned)g), dim3(256), band, s, a, G);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    if (a.Kstride < 64) {   // measured: conv 1 (K 18 / 36) 30 -> 15 us / 1.40 -> 0.82 ms; K >= 288 slower
        int64_t g = ((int64_t)a.M * a.nstreams * a.Kstride + 255) / 256;
        if (g > 16384) g = 16384;
        DQNX_LAUNCH(k_im2col_flat, dim3((unsigned)g), dim3(256), 0, s, a);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    int64_t g = ((int64_t)a.M * a.nstreams + 3) / 4;   // 4 rows (waves) per block
    if (g > 8192) g = 8192;
    DQNX_LAUNCH(k_im2col_rows, dim3((unsigned)g), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_flatten_concat(const FlattenArgs& a, hipStream_t s) {
    // (4,84,84) B=256: 395 -> 67 us; the (2,27,5) net's 21-pixel maps keep the element-wise form
    if (im2col_mode() == 1 && a.C <= 128 && a.Ho * a.Wo >= 256) {
        const int64_t g = (int64_t)a.nstreams * a.Bl * ((a.Ho * a.Wo + 63) / 64 + 1);
        DQNX_LAUNCH(k_flatten_concat_tiled, dim3((unsigned)g), dim3(256), 0, s, a);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    DQNX_LAUNCH(k_flatten_concat, grid_for((int64_t)a.Bl * a.strideF * a.nstreams), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_unflatten(const UnflattenArgs& a, hipStream_t s) {
    DQNX_LAUNCH(k_unflatten, grid_for((int64_t)a.Bl * a.Ho * a.Wo * a.C), dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

int launch_col2im(const Col2imArgs& a, int act, hipStream_t s) {
    const dim3 g = grid_for((int64_t)a.Bl * a.Hi * a.Wi * a.Ci);
    const bool pow2 = a.Ci > 0 && (a.Ci & (a.Ci - 1)) == 0;
    if (im2col_mode() == 1 && pow2 && a.kh == 3 && a.kw == 3 && a.ph == 1 && a.pw == 1 && a.sh <= 2 && a.sw <= 2) {
        int shift = 0;
        while ((1 << shift) < a.Ci) shift++;
        if (a.sh == 1 && a.sw == 1) launch_col2im_3x3<1, 1>(a, act, shift, g, s);
        else if (a.sh == 2 && a.sw == 1) launch_col2im_3x3<2, 1>(a, act, shift, g, s);
        else if (a.sh == 1 && a.sw == 2) launch_col2im_3x3<1, 2>(a, act, shift, g, s);
        else launch_col2im_3x3<2, 2>(a, act, shift, g, s);
        DQNX_HIP_CHECK(hipGetLastError());
        return DQNX_OK;
    }
    if (act == DQNX_ACT_RELU) DQNX_LAUNCH(k_col2im<DQNX_ACT_RELU>, g, dim3(256), 0, s, a);
    else DQNX_LAUNCH(k_col2im<DQNX_ACT_ELU>, g, dim3(256), 0, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
