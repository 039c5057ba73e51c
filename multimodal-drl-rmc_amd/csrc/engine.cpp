// libdqnx host side: network planning, arena layout, the C ABI of include/dqnx.h, the
// learn-step launch sequence and its hipGraph capture/replay.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <dlfcn.h>
#include <cmath>
#include <functional>
#include <map>
#include <tuple>
#include <string>
#include <vector>

#include "learn.hpp"

namespace dqnx {

KernelTimer& kernel_timer() {   // (DQNX_LAUNCH, common.hpp)
    static thread_local KernelTimer t;
    return t;
}

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int set_hip_error(hipError_t e, const char* expr, const char* file, int line) {
    snprintf(g_err, sizeof(g_err), "%s failed: %s (%s:%d)", expr, hipGetErrorString(e), file, line);
    return DQNX_ERR_HIP + (int)e;
}

// ------------------------------------------------------------------------------------
// network planning (host only)
// ------------------------------------------------------------------------------------
struct LayerPlan {
    int in, out;        // Linear in/out features
    int64_t off;        // flat offset of the weight ([out][in]); bias follows at off + out*in
};

struct ConvPlan {
    int Ci, Hi, Wi, Co, Ho, Wo, kh, kw, sh, sw, ph, pw;
    int K, Kstride;     // K = Ci*kh*kw (torch weight row), Kstride = K rounded up to 4
    int64_t off;        // flat offset of the weight [Co][Ci][kh][kw]; bias follows
};

struct NetPlan {
    std::vector<dqnx_param_info> params;
    std::vector<ConvPlan> conv;     // two-stream micro CNN (empty for MLP)
    int macro_len = 0, strideF = 0; // two-stream: dense input = cat(flatten(conv), macro)
    std::vector<LayerPlan> dense;   // body Linear layers
    int F = 0;                      // body output features
    int NH = 0;                     // head rows (dueling: 1 + A)
    int64_t head_off = 0, head_params = 0, P = 0;
};

static void add_param(NetPlan& np, const std::string& name, std::vector<int> shape) {
    dqnx_param_info pi;
    memset(&pi, 0, sizeof(pi));
    snprintf(pi.name, sizeof(pi.name), "%s", name.c_str());
    pi.offset = np.P;
    pi.ndim = (int32_t)shape.size();
    int64_t n = 1;
    for (size_t i = 0; i < shape.size(); i++) {
        pi.shape[i] = shape[i];
        n *= shape[i];
    }
    pi.numel = n;
    np.P += n;
    np.params.push_back(pi);
}

static int plan_net(const dqnx_net_desc* d, NetPlan& np) {
    np = NetPlan();
    if (!d) return set_error(DQNX_EINVAL, "net desc is null");
    if (d->obs_dim <= 0 || d->n_actions <= 0) return set_error(DQNX_EINVAL, "obs_dim/n_actions must be > 0");
    if (d->n_dense < 1 || d->n_dense > DQNX_MAX_DENSE) return set_error(DQNX_EINVAL, "n_dense out of range");
    if (d->head != DQNX_HEAD_DUELING && d->head != DQNX_HEAD_LINEAR) return set_error(DQNX_EINVAL, "bad head kind");
    int in;
    if (d->kind == DQNX_NET_MLP) {
        in = d->obs_dim;
        for (int l = 0; l < d->n_dense; l++) {
            const int out = d->dense[l];
            if (out <= 0) return set_error(DQNX_EINVAL, "dense width must be > 0");
            LayerPlan lp{in, out, np.P};
            add_param(np, "net." + std::to_string(2 * l) + ".weight", {out, in});
            add_param(np, "net." + std::to_string(2 * l) + ".bias", {out});
            np.dense.push_back(lp);
            in = out;
        }
    } else if (d->kind == DQNX_NET_TWO_STREAM) {
        if (d->n_conv < 1 || d->n_conv > DQNX_MAX_CONV) return set_error(DQNX_EINVAL, "n_conv out of range");
        if (d->macro_len + d->micro_c * d->micro_h * d->micro_w != d->obs_dim)
            return set_error(DQNX_EINVAL, "obs_dim != macro_len + c*h*w");
        int c = d->micro_c, h = d->micro_h, w = d->micro_w;
        for (int l = 0; l < d->n_conv; l++) {
            const int f = d->conv_out[l], kh = d->conv_kh[l], kw = d->conv_kw[l];
            if (f <= 0 || kh <= 0 || kw <= 0 || d->conv_sh[l] <= 0 || d->conv_sw[l] <= 0)
                return set_error(DQNX_EINVAL, "bad conv layer %d", l);
            ConvPlan cp;
            cp.Ci = c; cp.Hi = h; cp.Wi = w; cp.Co = f; cp.kh = kh; cp.kw = kw;
            cp.sh = d->conv_sh[l]; cp.sw = d->conv_sw[l]; cp.ph = kh / 2; cp.pw = kw / 2;   // padding k//2
            cp.off = np.P;
            add_param(np, "net.cnn_stream." + std::to_string(2 * l) + ".weight", {f, c, kh, kw});
            add_param(np, "net.cnn_stream." + std::to_string(2 * l) + ".bias", {f});
            h = (h + 2 * (kh / 2) - kh) / d->conv_sh[l] + 1;
            w = (w + 2 * (kw / 2) - kw) / d->conv_sw[l] + 1;
            if (h <= 0 || w <= 0) return set_error(DQNX_EINVAL, "conv layer %d output is empty", l);
            cp.Ho = h; cp.Wo = w;
            cp.K = c * kh * kw;
            cp.Kstride = (cp.K + 3) & ~3;
            np.conv.push_back(cp);
            c = f;
        }
        in = c * h * w + d->macro_len;
        np.macro_len = d->macro_len;
        np.strideF = (in + 3) & ~3;
        for (int l = 0; l < d->n_dense; l++) {
            const int out = d->dense[l];
            LayerPlan lp{in, out, np.P};
            add_param(np, "net.dense_stream." + std::to_string(2 * l) + ".weight", {out, in});
            add_param(np, "net.dense_stream." + std::to_string(2 * l) + ".bias", {out});
            np.dense.push_back(lp);
            in = out;
        }
    } else {
        return set_error(DQNX_EINVAL, "bad net kind");
    }
    np.F = in;
    np.head_off = np.P;
    if (d->head == DQNX_HEAD_DUELING) {
        add_param(np, "fc_val.weight", {1, in});
        add_param(np, "fc_val.bias", {1});
        add_param(np, "fc_adv.weight", {d->n_actions, in});
        add_param(np, "fc_adv.bias", {d->n_actions});
        np.NH = 1 + d->n_actions;
    } else {
        add_param(np, "fc_out.weight", {d->n_actions, in});
        add_param(np, "fc_out.bias", {d->n_actions});
        np.NH = d->n_actions;
    }
    np.head_params = np.P - np.head_off;
    return DQNX_OK;
}

constexpr int BWD_TILE = 32;   // k_bwd_level dW tile edge (DQNX_BWD_BM = DQNX_BWD_BN = 32)

// conv dW on 64x128 tiles (k_conv_dw_big) for convs of at least 64K output pixels per step and
// a K of at least 127 (the (4,84,84) variant, B=256: conv 2 605 -> 421 us, conv 3 278 -> 226 us;
// conv 1, K = 36, was slower on 128-wide tiles, 108 -> 382 us); DQNX_CONV_DW_BIG=0 keeps
// k_bwd_level's 32x32 role
// (environment knobs are read when a plan is built, so tests can switch them per engine)
static bool conv_dw_big(int64_t rows, int K) {
    const int mode = tuning_knob("DQNX_CONV_DW_BIG", 1);
    return mode != 0 && rows >= 65536 && K >= 127;
}

// DQNX_FWD_BIG=0 keeps every dense forward on the 16x64-tile kernel (A/B measurements)
static bool fwd_big_mode() {
    return route_knob("DQNX_FWD_BIG", 1) != 0;
}

static inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// head split-K slabs padded to 4 floats, so every slab stride allows the float4 Adam pass
static inline int64_t head_pstride(const NetPlan& np) { return (int64_t)align_up((uint64_t)np.head_params, 4); }

// ---- implicit-GEMM conv geometry (conv_ig.hip) ----
// Row tile of TR class rows (full width) on a BM-row workgroup tile: the BM of 256 / 128 / 64
// wasting the fewest padded rows, the larger on ties ((4,84,84) convs 1/2: 3 x 84 rows on 256;
// conv 3: 3 x 42 on 128; conv 3's data-gradient phases: 3 x 21 on 64 -- all 98.4 % full).
static bool cig_tile(int Hq, int Wq, int& BM, int& TR) {
    double best = 0;
    BM = 0;
    for (int bm : {256, 128, 64}) {
        int tr = bm / Wq;
        if (tr < 1) continue;
        tr = std::min(tr, Hq);
        const int tiles = (Hq + tr - 1) / tr;
        const double eff = (double)Hq * Wq / ((double)tiles * bm);
        if (eff > best + 0.01) { best = eff; BM = bm; TR = tr; }
    }
    return BM > 0;
}

// channels staged per pass: all of them when the band stays <= 50 KB (fewer restages), else
// 32 or 16; LDS floats per pixel CB + 4 (16-byte aligned rows for the float4 stage / b128 reads)
// a band must fit the kernels' staging registers: 256 threads x NQ float4 (NHWC sources) or
// x 4*NQ floats (CHW sources)
// (lines of one band row / one channel row, dealt round-robin to the 4 waves: conv_ig.hip)
static bool cig_stage_fits(int NR, int WP, int CB, bool vec) {
    constexpr int NQ = 12, NQS = 12;   // conv_ig.hip: float4 / floats per thread
    if (vec) return (int64_t)NR * ((WP * (CB / 4) + 63) / 64) <= 4 * NQ;
    return (int64_t)CB * NR * ((WP + 63) / 64) <= 4 * NQS;
}
static int cig_cb(int C, int NR, int WP, bool vec) {
    if (C == 4) return 4;
    size_t cap = 50 * 1024;   // DQNX_CIG_LDS_KB: band budget (a larger band means fewer workgroups per CU)
    cap = (size_t)tuning_knob("DQNX_CIG_LDS_KB", 50) * 1024;
    for (int cb : {64, 32})
        if (C % cb == 0 && (size_t)NR * WP * (cb + 4) * 4 <= cap && cig_stage_fits(NR, WP, cb, vec)) return cb;
    return 16;
}
static int cig_cs(int CB) { return CB == 4 ? 4 : CB + 4; }

// forward of conv cp: one class, band = the input rows of TR output rows
static bool cig_fwd_geom(const ConvPlan& cp, int Bl, bool first, ConvIgArgs& a) {
    memset(&a, 0, sizeof(a));
    if (!cig_tile(cp.Ho, cp.Wo, a.BM, a.TR)) return false;
    if (!conv_ig_supported(cp.Co, a.BM, cp.Ci)) return false;
    a.Bl = Bl;
    a.nclass = 1;
    a.CM = cp.sw;
    a.WP = (cp.Wo - 1) * cp.sw + cp.kw;
    a.SRM = cp.sh;
    CigClass& k = a.cls[0];
    k.ni = cp.kh; k.nj = cp.kw; k.i0 = k.j0 = 0; k.di = k.dj = 1; k.kw = cp.kw;
    k.o0 = 0; k.oi = a.WP; k.oj = 1;
    // DQNX_CIG_GROUPS=0 (tuning): stride-2 forwards stage all rows at once
    if (cp.sh == 2 && cp.Ci != 4 && tuning_knob("DQNX_CIG_GROUPS", 1) != 0) {   // row-parity groups: band rows compact, one group per parity
        a.ngrp = 2;
        a.RM = 1;
        a.RS = 2;
        a.NR = 0;
        for (int p = 0; p < 2; p++) {
            a.gni[p] = p < cp.kh ? (cp.kh - 1 - p) / 2 + 1 : 0;
            a.gnr[p] = a.TR + std::max(a.gni[p], 1) - 1;
            a.NR = std::max(a.NR, a.gnr[p]);
        }
    } else {
        a.ngrp = 1;
        a.RM = cp.sh;
        a.RS = 1;
        a.NR = (a.TR - 1) * cp.sh + cp.kh;
    }
    a.N = cp.Co;
    const bool vec = cp.Ci != 4 && !first;   // the first conv stages CHW ring rows
    a.CB = cig_cb(cp.Ci, a.NR, a.WP, vec);
    a.CS = cig_cs(a.CB);
    if (!cig_stage_fits(a.NR, a.WP, a.CB, vec)) return false;
    k.Hq = cp.Ho;
    k.Wq = cp.Wo;
    k.tiles = (cp.Ho + a.TR - 1) / a.TR;
    k.ntaps = cp.kh * cp.kw;
    k.rmin = -cp.ph;
    k.cmin = -cp.pw;
    a.maxtiles = k.tiles;
    a.Kw = cp.kh * cp.kw * cp.Ci;
    a.ymul = a.xmul = 1;
    a.src.H = cp.Hi;
    a.src.W = cp.Wi;
    a.src.C = cp.Ci;
    return conv_ig_lds_bytes(a) <= 160 * 1024;
}

// data gradient of conv cp (into the previous conv's NHWC dZ): one class per output phase
// (a, c): taps i = i0 + ii*sh with (a + ph - i) % sh == 0 read dZ row yq + (a + ph - i)/sh, i.e.
// band row ni-1-ii above the class origin; columns alike
static bool cig_dx_geom(const ConvPlan& cp, int Bl, bool last, ConvIgArgs& a) {
    memset(&a, 0, sizeof(a));
    if (cp.sh * cp.sw > 4 || cp.Co % 16) return false;
    const int Hq0 = (cp.Hi + cp.sh - 1) / cp.sh, Wq0 = (cp.Wi + cp.sw - 1) / cp.sw;
    if (!cig_tile(Hq0, Wq0, a.BM, a.TR)) return false;
    if (!conv_ig_supported(cp.Ci, a.BM, cp.Co)) return false;
    a.Bl = Bl;
    a.RM = a.CM = 1;
    a.SRM = a.RS = a.ngrp = 1;
    int nr = 0, wp = 0;
    for (int pa = 0; pa < cp.sh; pa++)
        for (int pc = 0; pc < cp.sw; pc++) {
            const int Hq = (cp.Hi - pa + cp.sh - 1) / cp.sh, Wq = (cp.Wi - pc + cp.sw - 1) / cp.sw;
            if (Hq <= 0 || Wq <= 0) continue;
            CigClass& k = a.cls[a.nclass++];
            k.a = pa;
            k.c = pc;
            k.Hq = Hq;
            k.Wq = Wq;
            k.tiles = (Hq + a.TR - 1) / a.TR;
            k.i0 = ((pa + cp.ph) % cp.sh);
            k.j0 = ((pc + cp.pw) % cp.sw);
            k.ni = k.i0 < cp.kh ? (cp.kh - 1 - k.i0) / cp.sh + 1 : 0;
            k.nj = k.j0 < cp.kw ? (cp.kw - 1 - k.j0) / cp.sw + 1 : 0;
            k.di = cp.sh; k.dj = cp.sw; k.kw = cp.kw;
            k.ntaps = k.ni * k.nj;
            // source row of tap ii: yq + (pa + ph - i0)/sh - ii; the band starts at its minimum
            const int rtop = (pa + cp.ph - k.i0) / cp.sh, ctop = (pc + cp.pw - k.j0) / cp.sw;
            k.rmin = k.ni ? rtop - (k.ni - 1) : 0;
            k.cmin = k.nj ? ctop - (k.nj - 1) : 0;
            nr = std::max(nr, a.TR + std::max(k.ni, 1) - 1);
            wp = std::max(wp, Wq + std::max(k.nj, 1) - 1);
            a.maxtiles = std::max(a.maxtiles, k.tiles);
        }
    a.NR = nr;
    a.WP = wp;
    for (int q = 0; q < a.nclass; q++) {
        CigClass& k = a.cls[q];
        k.o0 = (std::max(k.ni, 1) - 1) * a.WP + std::max(k.nj, 1) - 1;
        k.oi = -a.WP;
        k.oj = -1;
    }
    a.N = cp.Ci;
    (void)last;                                 // every dZ source is NHWC (the last conv's via k_unflatten_tiled)
    a.CB = cig_cb(cp.Co, a.NR, a.WP, true);
    a.CS = cig_cs(a.CB);
    if (!cig_stage_fits(a.NR, a.WP, a.CB, true)) return false;
    a.Kw = cp.kh * cp.kw * cp.Co;
    a.ymul = cp.sh;
    a.xmul = cp.sw;
    a.src.H = cp.Ho;
    a.src.W = cp.Wo;
    a.src.C = cp.Co;
    a.nstreams = 1;
    return conv_ig_lds_bytes(a) <= 160 * 1024;
}

// weight gradient of conv cp: row groups of RB output rows (X band <= 64 KB, pixel chunks as
// full as possible), slices of gps groups sized for ~512 workgroups over the channel blocks
static bool cig_dw_geom(const ConvPlan& cp, int Bl, bool first, ConvDwIgArgs& d) {
    memset(&d, 0, sizeof(d));
    d.Bl = Bl; d.Ho = cp.Ho; d.Wo = cp.Wo;
    d.Co = cp.Co; d.C = cp.Ci; d.CB = cp.Ci == 4 ? 4 : 16;
    d.CS = cp.Ci == 4 ? 5 : 20;
    d.ntaps = cp.kh * cp.kw; d.kw = cp.kw;
    d.sh = cp.sh; d.sw = cp.sw; d.ph = cp.ph; d.pw = cp.pw;
    d.K = cp.K;
    d.TN = (d.ntaps * d.CB + 15) / 16;
    if ((d.Co != 32 && d.Co != 64) || (d.TN != 3 && d.TN != 9) || d.C % d.CB) return false;
    d.WP = (cp.Wo - 1) * cp.sw + cp.kw;
    double best = 0;
    for (int rb = 8; rb >= 1; rb--) {
        const int nr = (rb - 1) * cp.sh + cp.kh;
        if ((size_t)nr * d.WP * d.CS * 4 > 64 * 1024 || rb > cp.Ho || !cig_stage_fits(nr, d.WP, d.CB, !first)) continue;
        const int G = (cp.Ho + rb - 1) / rb;
        // useful pixels over MFMA pixel slots (16-pixel chunks per group)
        const double slots = (double)(G - 1) * ((rb * cp.Wo + 15) / 16 * 16) + ((cp.Ho - (G - 1) * rb) * cp.Wo + 15) / 16 * 16;
        const double eff = (double)cp.Ho * cp.Wo / slots;
        if (eff > best + 0.005) { best = eff; d.RB = rb; d.NR = nr; }
    }
    if (!d.RB) return false;
    d.G = (cp.Ho + d.RB - 1) / d.RB;
    const int groups = Bl * d.G, ncb = d.C / d.CB;
    const int target = std::max(1, std::min(groups, 512 / ncb));
    d.gps = (groups + target - 1) / target;
    d.slices = (groups + d.gps - 1) / d.gps;
    d.pstride = (int64_t)cp.Co * cp.K + cp.Co;
    return conv_dw_ig_lds_bytes(d) <= 64 * 1024;
}

// implicit-GEMM convs for every conv of a large micro grid (DQNX_CONV_IG=0: explicit path)
static bool conv_ig_plan(const NetPlan& np, int Bl) {
    if (np.conv.empty()) return false;
    if (route_knob("DQNX_CONV_IG", 1) == 0) return false;
    if ((int64_t)np.conv[0].Hi * np.conv[0].Wi < 1024) return false;   // the (2,27,5) grid keeps the explicit kernels
    for (size_t l = 0; l < np.conv.size(); l++) {
        ConvIgArgs f;
        ConvDwIgArgs d;
        const bool first = l == 0, last = l + 1 == np.conv.size();
        if (!cig_fwd_geom(np.conv[l], Bl, first, f) || !cig_dw_geom(np.conv[l], Bl, first, d)) return false;
        if (l > 0 && !cig_dx_geom(np.conv[l], Bl, last, f)) return false;
    }
    return true;
}

// the micro-CNN geometry of a two-stream net (micro.hip): every conv 3x3 with padding 1
static bool micro_geom(const NetPlan& np, MicroConv* c) {
    const int NC = (int)np.conv.size();
    if (NC < 2 || NC > MICRO_MAX_CONV) return false;
    for (int l = 0; l < NC; l++) {
        const ConvPlan& cp = np.conv[l];
        if (cp.kh != 3 || cp.kw != 3 || cp.ph != 1 || cp.pw != 1) return false;
        MicroConv& m = c[l];
        memset(&m, 0, sizeof(m));
        m.Ci = cp.Ci; m.Hi = cp.Hi; m.Wi = cp.Wi; m.Co = cp.Co; m.Ho = cp.Ho; m.Wo = cp.Wo;
        m.sh = cp.sh; m.sw = cp.sw;
        m.woff = cp.off;
        // LDS floats per pixel: Co + 8 (b128 reads conflict-free); DQNX_MICRO_PIXPAD=4: Co + 4 (also
        // conflict-free for the stride-2 taps; measured equal, kept for the LDS counter comparison)
        m.cs = cp.Co + (route_knob("DQNX_MICRO_PIXPAD", 8) == 4 ? 4 : 8);
    }
    return true;
}

struct KStep {
    std::string name;
    double flops = 0, bytes = 0;
    std::function<int(hipStream_t)> run;
};

}  // namespace dqnx

using namespace dqnx;

struct dqnx_engine {
    dqnx_config cfg;
    NetPlan np;
    int Bg = 0, Bl = 0, shard_begin = 0, stride = 0, tiles = 0;
    int Bs = 0;              // positions the sampler draws: Bg, or Bl with rank-local sampling
    bool local_sampling = false;
    int64_t setsize = 0;
    std::vector<int> slices;          // split-K slabs per dense layer
    std::vector<int> kslice;
    uint64_t off[DQNX_BUF_COUNT] = {0}, bytes[DQNX_BUF_COUNT] = {0};
    uint64_t total = 0;
    // workspace sub-regions (byte offsets from the arena base)
    uint64_t ws_phys = 0, ws_pool = 0, ws_xobs = 0, ws_head_part = 0, ws_loss_part = 0, ws_stage = 0;
    uint64_t ws_ring16[2] = {0, 0};   // bf16 engines: [cap][stride16] bf16 copies of obs / next_obs
    int stride16 = 0;
    uint64_t ws_npc = 0;   // numpy MT block cache (PER, fused plan)
    uint64_t ws_pairflag = 0;   // paired forward: [3][tiles] H_1 hand-off words
    uint64_t ws_adam_tab = 0, ws_stamps = 0, ws_dhead = 0, ws_raw = 0, ws_trans = 0, ws_gtab = 0, ws_mtc = 0, ws_per_ticket = 0, ws_per_wl = 0, ws_per_wp = 0, ws_per_winit = 0, ws_per_last = 0, ws_per_wchg = 0;
    // fused plan: fragment-blocked weight copies [online fwd | target fwd | online chain] per layer
    uint64_t ws_wblk[2][FUSED_MAX_L] = {{0}}, ws_wblkT[FUSED_MAX_L] = {0};
    std::vector<uint64_t> ws_H, ws_dZ, ws_part;
    // bf16 weight gradients from T16 copies (k_dw_bf16t): stream 0's rows / H_l and dZ_l / dHead in bf16
    bool dwt = false;
    uint64_t ws_xT16 = 0, ws_dheadT16 = 0;
    std::vector<uint64_t> ws_HT16, ws_dZT16;
    // two-stream CNN: per conv layer im2col [3][M][Kstride], activations [3][M][Co],
    // dZ [M][Co], split-K partial slabs; dense input F [3][Bl][strideF] and its gradient
    std::vector<uint64_t> ws_col, ws_Hc, ws_dZc, ws_cpart;
    std::vector<int> cslices, ckslice;
    uint64_t ws_F = 0, ws_dF = 0, ws_dcol = 0, ws_fpart = 0;
    int f1_ksplit = 0, f1_kchunk = 0;   // conv nets' dense 1 forward: split-K slabs (0: the 16 x 64 kernel)
    // implicit-GEMM convs (conv_ig.hip): no column matrices; permuted weight copies per conv
    // ([co][tap][ci] online / target, [ci][tap][co] online), the last conv writes F directly
    bool conv_ig = false;
    std::vector<uint64_t> ws_wperm0, ws_wperm1, ws_wpermT;
    // micro-CNN plan (micro.hip): the reference HEAD net's convs on a small grid, activations on
    // chip (forward: S samples per workgroup; data gradients: dx_S; weight gradients: dw plan)
    bool micro = false;
    int micro_S = 1, micro_lds = 0, micro_dx_S = 1, micro_dx_lds = 0;
    int micro_lds_d[MICRO_MAX_CONV] = {0, 0, 0};
    MicroDwArgs micro_dw;
    int stage_rows = 0;
    char* arena = nullptr;
    int64_t ring_size = 0, ring_wptr = 0;   // host mirror of the ring state (pushes are host-driven)
    bool graphs = false;   // eager launches by default (dqnx_engine_set_graphs)
    std::map<int, hipGraphExec_t> graph_cache;
    hipStream_t capture_stream = nullptr;
    std::map<int, std::vector<KStep>> steps_cache;
    std::map<int, DwAdam16Args> dw16_cache;   // the fused plan's k_dw_adam16 launch of each cached plan
    int building_key = 0;                     // (the plan key steps_for is building)
    // drop-in Agent fast path (dqnx_agent_*, small host pushes): engine-owned pinned blocks + events
    uint32_t* ag_rng_pin = nullptr;           // [2][625] staged RNG states (alternating)
    uint32_t* ag_rng_zc = nullptr;            // [625] fine-grained pinned block the sampler reads in place
    bool ag_zc_launch = false;                // (set around the learn step of an agent launch)
    bool ag_zc_used = false;                  // the block is read by an agent launch not yet known done
    hipEvent_t ag_rng_ev[2] = {nullptr, nullptr};
    bool ag_rng_live[2] = {false, false};
    int ag_slot = 0, ag_which = -1;
    uint32_t ag_expect[625];                  // host mirror of the staged draw's post-draw state
    bool ag_expect_live = false;
    dqnx_ctrl* ag_ctrl_pin = nullptr;         // control block read back after each agent launch
    hipEvent_t ag_ctrl_ev = nullptr;
    bool ag_ctrl_live = false;
    bool ag_check_live = false;               // the pending readback is to be checked against ag_check
    int ag_check_which = 0;
    uint32_t ag_check[625];
    char* push_pin = nullptr;                 // small host pushes: one pinned block, one H2D
    hipEvent_t push_ev = nullptr;
    bool push_live = false;
    int bucket_key = -1;                      // the GRADS_ONLY plan of the bucketed step in flight
    bool bucket_prefetch = false;
    std::map<std::tuple<int, int, void*, void*>, hipGraphExec_t> timed_cache;
    hipStream_t side_stream = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    hipEvent_t ev_sampled[2] = {nullptr, nullptr}, ev_computed[2] = {nullptr, nullptr};
    bool pf_computed_valid[2] = {false, false};
    // step plan: 2 = fused MLP plan (default where supported: one forward launch for every
    // layer + head, one head/TD/dZ-chain launch, one split-K dW launch, Adam); 0 = per-layer
    // forward + split-K backward levels + Adam pass (two-stream nets); 1 = head kernel also
    // makes dZ_{L-1}, one full-K dW + Adam launch
    int bwd_plan = 0;
    int mtc_blocks = 0;     // uniform sampler's MT block cache (fused plan only; 0 = off)
    bool wblk_dirty = true; // the fused plan's blocked weight copies must be rebuilt before the next step
    // the micro-CNN plan's permuted conv weight copies (k_conv_perm) are stale: the next step launches
    // conv_perm (an Adam pass that writes them -- adam_writes_perms -- makes them current)
    bool perm_dirty = true;
    FusedFwdArgs fplan;     // LDS geometry of the fused plan (valid when bwd_plan == 2)
    int fsplit = 1;         // layer-1 column parts of the split forward (1: one forward launch)
    int fsplit_mr = 1;      // 16-row blocks per workgroup of the split forward's layer-1 launch
    int fpair = 0;          // DQNX_FWD_PAIR=1: one forward launch, layer 1's columns over 2 partner workgroups
    bool pf_valid = false;   // a prefetched minibatch for the next step sits in slot pf_slot
    bool pf_inlaunch = false;   // ... drawn by the previous step's forward launch (fused plan)
    int n_cu = 256;             // compute units of the device (hipDeviceAttributeMultiprocessorCount)
    hipStream_t pf_stream = nullptr;   // ... on this stream
    int pf_slot = 0;
};

namespace {

template <class T>
T* at(dqnx_engine* e, uint64_t byte_off) {
    return reinterpret_cast<T*>(e->arena + byte_off);
}

dqnx_ctrl* ctrl_of(dqnx_engine* e) { return at<dqnx_ctrl>(e, e->off[DQNX_BUF_CTRL]); }

int layout(dqnx_engine* e) {
    const dqnx_config& c = e->cfg;
    const NetPlan& np = e->np;
    const int L = (int)np.dense.size();
    const int A = c.net.n_actions;
    const int64_t P = np.P;
    uint64_t cur = 0;
    auto region = [&](int which, uint64_t nbytes) {
        cur = align_up(cur, 256);
        e->off[which] = cur;
        e->bytes[which] = nbytes;
        cur += nbytes;
    };
    region(DQNX_BUF_PARAMS, P * 4);
    region(DQNX_BUF_TARGET_PARAMS, P * 4);
    region(DQNX_BUF_GRADS, (P + 1) * 4);
    region(DQNX_BUF_ADAM_M, P * 4);
    region(DQNX_BUF_ADAM_V, P * 4);
    region(DQNX_BUF_CTRL, sizeof(dqnx_ctrl));
    const uint64_t cap = (uint64_t)c.capacity;
    region(DQNX_BUF_RING_OBS, cap * e->stride * 4);
    region(DQNX_BUF_RING_NEXT_OBS, cap * e->stride * 4);
    region(DQNX_BUF_RING_ACT, cap * 4);
    region(DQNX_BUF_RING_REW, cap * 4);
    region(DQNX_BUF_RING_DONE, cap * 4);
    region(DQNX_BUF_SUMTREE, c.algo == DQNX_ALGO_PER_DOUBLE ? (2 * cap - 1) * 8 : 0);
    region(DQNX_BUF_BATCH_IDX, (uint64_t)2 * e->Bg * 4);   // [slot][Bg]: slot 1 is the prefetch buffer
    region(DQNX_BUF_Q, (uint64_t)3 * e->Bl * A * 4);
    region(DQNX_BUF_TD, (uint64_t)3 * e->Bl * 4);
    region(DQNX_BUF_IS_WEIGHTS, (uint64_t)e->Bg * 4);
    region(DQNX_BUF_PER_ABS_TD, c.algo == DQNX_ALGO_PER_DOUBLE ? (uint64_t)e->Bg * 4 : 0);
    // workspace
    cur = align_up(cur, 256);
    e->off[DQNX_BUF_WORKSPACE] = cur;
    auto sub = [&](uint64_t nbytes) {
        cur = align_up(cur, 256);
        uint64_t o = cur;
        cur += nbytes;
        return o;
    };
    e->ws_phys = sub((uint64_t)2 * e->Bl * 4);
    e->ws_pool = sub((uint64_t)(e->setsize + 64) * 4);
    e->ws_gtab = sub(sample_table_bytes(e->Bs));   // 0 unless the minibatch exceeds the LDS tables
    e->mtc_blocks = (e->bwd_plan == 2 && c.algo != DQNX_ALGO_PER_DOUBLE && !tuning_flag("DQNX_NO_MT_CACHE"))
                        ? mt_cache_target_blocks(e->Bs, c.capacity) : 0;
    e->ws_mtc = sub((uint64_t)mt_cache_words() * 4);   // always valid for the sampler's loads
    e->ws_xobs = sub((uint64_t)e->Bl * e->stride * 4);
    if (e->bwd_plan == 2 && e->fplan.bf16) {   // the bf16 forward gathers these (csrc/fused.hip)
        e->stride16 = (c.net.obs_dim + 7) & ~7;
        e->ws_ring16[0] = sub(cap * e->stride16 * 2);
        e->ws_ring16[1] = sub(cap * e->stride16 * 2);
    }
    e->ws_H.assign(L, 0);
    e->ws_dZ.assign(L, 0);
    e->ws_part.assign(L, 0);
    for (int l = 0; l < L; l++) {
        const int w = np.dense[l].out;
        e->ws_H[l] = sub((uint64_t)3 * e->Bl * w * 4);
        e->ws_dZ[l] = sub((uint64_t)e->Bl * w * 4);
        const uint64_t lp = (uint64_t)np.dense[l].out * np.dense[l].in + np.dense[l].out;
        e->ws_part[l] = sub((uint64_t)e->slices[l] * lp * 4);
    }
    e->ws_head_part = sub((uint64_t)e->slices[L - 1] * head_pstride(np) * 4);
    e->ws_dhead = sub((uint64_t)e->Bl * 16 * 4);
    e->ws_HT16.assign(L, 0);
    e->ws_dZT16.assign(L, 0);
    if (e->dwt) {
        const uint64_t rows = (uint64_t)e->slices[0] * e->kslice[0];   // whole slices (tcopy_index)
        e->ws_xT16 = sub(rows * np.dense[0].in * 2);
        for (int l = 0; l < L; l++) {
            e->ws_HT16[l] = sub(rows * np.dense[l].out * 2);
            e->ws_dZT16[l] = sub(rows * np.dense[l].out * 2);
        }
        e->ws_dheadT16 = sub(rows * 16 * 2);
    }
    e->ws_raw = sub((uint64_t)3 * e->Bl * 16 * 4);
    e->ws_trans = sub((uint64_t)e->Bl * 16);
    if (e->bwd_plan == 2) {
        for (int l = 0; l < L; l++) {
            const bool bf = e->fplan.bf16 != 0;
            const uint64_t fwd = (uint64_t)fused_wblk_bytes(bf, np.dense[l].out, e->fplan.kpad[l]);
            e->ws_wblk[0][l] = sub(fwd);
            e->ws_wblk[1][l] = sub(fwd);
            if (l >= 1) e->ws_wblkT[l] = sub((uint64_t)fused_wblk_bytes(bf, np.dense[l].in, np.dense[l].out));
        }
    }
    e->ws_adam_tab = sub((uint64_t)kAdamTable * 2 * 4);
    e->ws_stamps = sub(64 * 8);
    if (e->fpair) e->ws_pairflag = sub((uint64_t)3 * ((e->Bl + 15) / 16) * 4);
    e->ws_per_ticket = sub(128);   // k_per_sample arrival counter (zero between launches); [16]: PER chunk
                                   // epoch; [20]: the in-launch tracking -> prop hand-off word
    // numpy MT block cache: only where the fused forward launch keeps it extended
    if (c.algo == DQNX_ALGO_PER_DOUBLE && e->bwd_plan == 2 && e->fsplit <= 1 && !route_flag("DQNX_NO_NP_CACHE") &&
        np_cache_blocks(e->Bg) <= NPC_MAX_BLOCKS)
        e->ws_npc = sub((uint64_t)np_cache_words() * 4);
    if (c.algo == DQNX_ALGO_PER_DOUBLE) {   // k_per_prep / k_per_update / k_per_prop hand-offs
        e->ws_per_wl = sub((uint64_t)PER_CHUNK * 4);
        e->ws_per_wp = sub((uint64_t)PER_CHUNK * 4);
        e->ws_per_winit = sub((uint64_t)PER_CHUNK * 8);
        e->ws_per_last = sub((uint64_t)c.capacity * 8);
        e->ws_per_wchg = sub((uint64_t)PER_CHUNK * 4);
    }
    e->ws_loss_part = sub((uint64_t)e->tiles * 4);
    e->stage_rows = 1024;
    e->ws_stage = sub((uint64_t)e->stage_rows * (2 * (uint64_t)c.net.obs_dim + 3) * 4 + 256);
    const int NC = (int)np.conv.size();
    e->ws_col.assign(NC, 0);
    e->ws_Hc.assign(NC, 0);
    e->ws_dZc.assign(NC, 0);
    e->ws_cpart.assign(NC, 0);
    uint64_t dcol_max = 0;
    e->ws_wperm0.assign(NC, 0);
    e->ws_wperm1.assign(NC, 0);
    e->ws_wpermT.assign(NC, 0);
    for (int l = 0; l < NC; l++) {
        const ConvPlan& cp = np.conv[l];
        const uint64_t M = (uint64_t)e->Bl * cp.Ho * cp.Wo;
        const bool last = l == NC - 1;
        if (!e->conv_ig && !e->micro) e->ws_col[l] = sub(3 * M * cp.Kstride * 4);
        // the implicit path's last conv writes F; the micro plan keeps stream 0's outputs only
        if (!((e->conv_ig || e->micro) && last)) e->ws_Hc[l] = sub((e->micro ? 1 : 3) * M * cp.Co * 4);
        e->ws_dZc[l] = sub(M * cp.Co * 4);
        e->ws_cpart[l] = sub((uint64_t)e->cslices[l] * ((uint64_t)cp.Co * cp.K + cp.Co) * 4);
        if (!e->conv_ig && !e->micro && l > 0 && M * cp.K * 4 > dcol_max) dcol_max = M * cp.K * 4;
        if (e->conv_ig || e->micro) {
            e->ws_wperm0[l] = sub((uint64_t)cp.Co * cp.K * 4);
            e->ws_wperm1[l] = sub((uint64_t)cp.Co * cp.K * 4);
            if (l > 0) e->ws_wpermT[l] = sub((uint64_t)cp.Co * cp.K * 4);
        }
    }
    if (NC) {
        e->ws_F = sub((uint64_t)3 * e->Bl * np.strideF * 4);
        e->ws_dF = sub((uint64_t)e->Bl * np.dense[0].in * 4);
        if (e->f1_ksplit) e->ws_fpart = sub((uint64_t)e->f1_ksplit * 3 * e->Bl * np.dense[0].out * 4);
        if (dcol_max) e->ws_dcol = sub(dcol_max);
    }
    cur = align_up(cur, 256);
    e->bytes[DQNX_BUF_WORKSPACE] = cur - e->off[DQNX_BUF_WORKSPACE];
    e->total = cur;
    return DQNX_OK;
}

int check_bound(const dqnx_engine* e) {
    if (!e) return set_error(DQNX_EINVAL, "engine is null");
    if (!e->arena) return set_error(DQNX_ESTATE, "engine arena not bound");
    return DQNX_OK;
}

// ---- the learn-step launch sequence ----------------------------------------------------
// One learn step = an ordered list of kernel launches.  Each entry carries its name and
// algorithmic FLOPs / bytes (for the roofline of DESIGN.md) so a sub-range can be captured
// and timed on its own (dqnx_learn_step_timed).


PerSampleArgs per_sample_args(dqnx_engine* e, int32_t* idx, int32_t* phys) {
    const dqnx_config& c = e->cfg;
    PerSampleArgs pa;
    memset(&pa, 0, sizeof(pa));
    pa.tree = at<double>(e, e->off[DQNX_BUF_SUMTREE]);
    pa.cap = c.capacity;
    pa.ctrl = ctrl_of(e);
    pa.Bg = e->Bg;
    pa.shard_begin = e->shard_begin;
    pa.shard_len = e->Bl;
    pa.out_idx = idx;
    pa.phys_out = phys;
    pa.isw = at<float>(e, e->off[DQNX_BUF_IS_WEIGHTS]);
    pa.beta_start = c.per_beta_start;
    pa.beta_end = c.per_beta_end;
    pa.beta_steps = c.per_beta_steps;
    pa.n_env = c.n_env;
    pa.stamps = at<int64_t>(e, e->ws_stamps);
    pa.ticket = at<int32_t>(e, e->ws_per_ticket);
    pa.npc = e->ws_npc ? at<uint32_t>(e, e->ws_npc) : nullptr;   // extended by the fused forward
    // samples per workgroup: the descents' scattered tree loads are texture-path bound, so with the
    // MT blocks cached (no per-workgroup twists) fewer samples per workgroup spread them wider
    // (measured on MI355X: B=1024 per_sample 17.3 / 14.8 / 13.5 us at 256 / 128 / 64 per workgroup,
    // step 68.2 -> 63.2 us; bf16 B=8192 step 120.0 / 116.6 / 117.9 us)
    pa.spw = e->Bg <= 2048 ? 64 : 128;
    {
        const int x = tuning_knob("DQNX_PER_SPW", pa.spw);
        if (x == 64 || x == 128 || x == 256) pa.spw = x;
    }
    return pa;
}

PerUpdateArgs per_update_args(dqnx_engine* e) {
    const dqnx_config& c = e->cfg;
    PerUpdateArgs ua;
    memset(&ua, 0, sizeof(ua));
    ua.tree = at<double>(e, e->off[DQNX_BUF_SUMTREE]);
    ua.cap = c.capacity;
    ua.ctrl = ctrl_of(e);
    ua.eps = (float)c.per_eps;
    ua.alpha = (float)c.per_alpha;
    ua.pmax = (float)c.per_max_priority;
    ua.stamps = at<int64_t>(e, e->ws_stamps);
    ua.wl = at<int32_t>(e, e->ws_per_wl);
    ua.wp = at<float>(e, e->ws_per_wp);
    ua.winit = at<double>(e, e->ws_per_winit);
    ua.last = at<uint64_t>(e, e->ws_per_last);
    ua.epoch = at<uint32_t>(e, e->ws_per_ticket) + 16;
    ua.sync = at<uint32_t>(e, e->ws_per_ticket) + 20;
    ua.numpy121 = c.per_numpy121;
    ua.wchg = at<float>(e, e->ws_per_wchg);
    return ua;
}

// update_batch_priorities over n (slot, |delta|) pairs in order, in PER_CHUNK launches.
// size: the ring size at the time (the rescan range); read from the host mirror.
int enqueue_per_update_pairs(dqnx_engine* e, const int32_t* slots, const float* abs_td, int n, hipStream_t s) {
    for (int o = 0; o < n; o += PER_CHUNK) {
        PerUpdateArgs ua = per_update_args(e);
        ua.mode = 0;
        ua.n = std::min(PER_CHUNK, n - o);
        ua.slots = slots + o;
        ua.abs_td = abs_td + o;
        int rc = launch_per_update(ua, s);   // mode 0 reads the ring size on the device
        if (rc) return rc;
    }
    return DQNX_OK;
}

int enqueue_per_update(dqnx_engine* e, const int32_t* idx, hipStream_t s) {
    return enqueue_per_update_pairs(e, idx, at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]), e->Bg, s);
}

AdamBias adam_bias_args(dqnx_engine* e) {
    AdamBias b;
    b.table = at<float>(e, e->ws_adam_tab);
    b.len = kAdamTable;
    b.lrd = e->cfg.lr;
    b.beta1d = e->cfg.beta1;
    b.beta2d = e->cfg.beta2;
    return b;
}

// The fused plan's blocked weight copies, written by the Adam pass next to every weight.
// Opt-in (DQNX_ADAM_BLK=1): the Adam pass writes the blocked copies next to every weight, so
// the sampler launch rebuilds them only after host-side writes (dqnx_params_modified).  Measured
// on MI355X (MLP-284, B = 1024): Adam 4.1 -> 6.6 us (three scattered stores per weight) while the
// rebuild by spare workgroups of the sampler launch costs the sampler ~0.4 us, so the default
// keeps the per-step rebuild.  (Adam's row/column split needs out * in < 2^24.)
bool adam_keeps_blk(const dqnx_engine* e) {
    if (e->bwd_plan != 2) return false;
    if (route_knob("DQNX_ADAM_BLK", 0) == 0) return false;
    for (const LayerPlan& lp : e->np.dense)
        if ((int64_t)lp.out * lp.in >= ((int64_t)1 << 24)) return false;
    return true;
}

// Fused plan, fp32: every dW over the full (local) minibatch + Adam + blocked copies in one
// launch (k_dw_adam16) instead of split-K slabs + the Adam pass, up to 2048 rows per GPU.
// Measured on MI355X, MLP-284: B = 1024 step 46.8 -> 43.7 us (dW + Adam 8.5 + 5.1 -> 10.6 us);
// at B = 4096 the slabs win (18.7 + 6.7 vs 26.3 us: the full-K tiles re-read dZ and X from L2
// per 16 x 16 tile, the split-K slices spread the rows over more workgroups).
// DQNX_DW_ADAM16=0 / 1 forces the slab plan / this kernel.  GRADS_ONLY steps run it in
// gradient mode (so world-1 DP equals the single-GPU step bitwise).
bool dw_adam16_on(const dqnx_engine* e, int flags) {
    (void)flags;
    if (e->bwd_plan != 2 || e->fplan.bf16) return false;
    if (route_flag("DQNX_DW_ADAM16")) {
        if (route_knob("DQNX_DW_ADAM16", 1) == 0) return false;
    } else if (e->Bl > 2048) {
        return false;
    }
    for (const LayerPlan& lp : e->np.dense)
        if (lp.out % 16) return false;   // chain blocks tile `out` by 16
    return e->np.NH <= 16;
}

// the weight update of a step with these flags keeps the fused plan's blocked copies current
static bool blk_kept(const dqnx_engine* e, int flags) {
    // (a GRADS_ONLY step: the update is dqnx_apply_grads' Adam pass)
    if (flags & DQNX_STEP_GRADS_ONLY) return adam_keeps_blk(e);
    return adam_keeps_blk(e) || dw_adam16_on(e, flags);
}

// force: this Adam pass writes the blocked copies although the engine does not keep them by
// default (a prefetching step has no sampler launch whose spare workgroups would rebuild them)
void fill_blk_layers(dqnx_engine* e, AdamArgs& aa, bool force = false) {
    aa.nblk = 0;
    if (!adam_keeps_blk(e) && !(force && e->bwd_plan == 2)) return;
    for (const LayerPlan& lp : e->np.dense)
        if ((int64_t)lp.out * lp.in >= ((int64_t)1 << 24)) return;
    const NetPlan& np = e->np;
    aa.blk_bf16 = e->fplan.bf16 ? 1 : 0;
    for (int l = 0; l < (int)np.dense.size() && l < 3; l++) {
        AdamArgs::BlkLayer& B = aa.blk[aa.nblk++];
        B.woff = np.dense[l].off;
        B.in = np.dense[l].in;
        B.out = np.dense[l].out;
        B.inv_in = 1.0f / (float)B.in;
        B.kpad = e->fplan.kpad[l];

        B.fwd_online = at<float>(e, e->ws_wblk[0][l]);
        B.fwd_target = at<float>(e, e->ws_wblk[1][l]);
        B.chain = l >= 1 ? at<float>(e, e->ws_wblkT[l]) : nullptr;
    }
}

// The Adam launch of a plan step; one that writes the micro plan's permuted conv copies marks them
// current when it is enqueued (launch order = execution order on the step's stream)
static std::function<int(hipStream_t)> adam_run(dqnx_engine* e, const AdamArgs& aa) {
    const bool perms = adam_writes_perms(aa);
    return [=](hipStream_t s) {
        const int rc = launch_adam(aa, s);
        if (!rc && perms) e->perm_dirty = false;
        return rc;
    };
}

// Gradient reduction (fixed-order sum of the split-K slabs) + Adam (+ soft update).
KStep adam_kstep(dqnx_engine* e, int flags, AdamArgs* args_out = nullptr) {
    const dqnx_config& c = e->cfg;
    const NetPlan& np = e->np;
    const int L = (int)np.dense.size();
    const int NC = (int)np.conv.size();
    dqnx_ctrl* ctrl = ctrl_of(e);
    float* params = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    float* tparams = at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]);
    AdamArgs aa;
    memset(&aa, 0, sizeof(aa));
    aa.nseg = 0;
    double part_elems = 0;
    for (int l = 0; l < NC; l++) {   // segments in flat-offset order: convs, dense, head
        const ConvPlan& cp = np.conv[l];
        AdamSegment& sg = aa.seg[aa.nseg++];
        sg.off = cp.off;
        sg.partial = at<float>(e, e->ws_cpart[l]);
        sg.pstride = (int64_t)cp.Co * cp.K + cp.Co;
        sg.S = e->cslices[l];
        sg.wide = sg.S >= ADAM_WIDE_MIN_S || e->micro;   // micro plan: every conv (its permuted copies)
        part_elems += (double)sg.S * sg.pstride;
    }
    for (int l = 0; l < L; l++) {
        AdamSegment& sg = aa.seg[aa.nseg++];
        sg.off = np.dense[l].off;
        sg.partial = at<float>(e, e->ws_part[l]);
        sg.pstride = (int64_t)np.dense[l].out * np.dense[l].in + np.dense[l].out;
        sg.S = e->slices[l];
        sg.wide = sg.S >= ADAM_WIDE_MIN_S;
        part_elems += (double)sg.S * sg.pstride;
    }
    {
        AdamSegment& sg = aa.seg[aa.nseg++];
        sg.off = np.head_off;
        sg.partial = at<float>(e, e->ws_head_part);
        sg.pstride = head_pstride(np);
        sg.S = e->slices[L - 1];
        sg.wide = sg.S >= ADAM_WIDE_MIN_S;
        part_elems += (double)sg.S * sg.pstride;
    }
    aa.mode = (flags & DQNX_STEP_GRADS_ONLY) ? 0 : 1;
    aa.soft = (flags & DQNX_STEP_SOFT_UPDATE) ? 1 : 0;
    aa.n_params = np.P;
    aa.p = params;
    aa.m = at<float>(e, e->off[DQNX_BUF_ADAM_M]);
    aa.v = at<float>(e, e->off[DQNX_BUF_ADAM_V]);
    aa.grads = at<float>(e, e->off[DQNX_BUF_GRADS]);
    aa.target = tparams;
    aa.ctrl = ctrl;
    aa.w1 = (float)(1.0 - c.beta1);          // Python: exp_avg.lerp_(grad, 1 - beta1)
    aa.beta2 = (float)c.beta2;
    aa.c2 = (float)(1.0 - c.beta2);
    aa.eps = (float)c.adam_eps;
    aa.tau = (float)(c.tau * c.n_env);      // (tau * n_env) * online + (1 - tau * n_env) * target
    aa.one_minus_tau = (float)(1.0 - c.tau * c.n_env);
    aa.adam_table = at<float>(e, e->ws_adam_tab);
    aa.adam_table_len = kAdamTable;
    aa.beta1d = c.beta1;
    aa.beta2d = c.beta2;
    aa.lrd = c.lr;
    aa.loss_partial = at<float>(e, e->ws_loss_part);
    aa.n_loss_partial = e->tiles;
    aa.batch_global = e->Bg;
    aa.with_loss = 1;
    fill_blk_layers(e, aa);
    if (e->mtc_blocks && !(flags & DQNX_STEP_GIVEN_INDICES)) {   // keep the sampler's MT blocks ahead
        aa.mtc = at<uint32_t>(e, e->ws_mtc);
        aa.mtc_blocks = e->mtc_blocks;
    }
    if (e->micro && aa.mode == 1) {   // the permuted copies of convs 2.. next to the updated weights
        for (int l = 1; l < NC && aa.nperm < 2; l++) {
            const ConvPlan& cp = np.conv[l];
            AdamArgs::PermLayer& P = aa.perm[aa.nperm++];
            P.woff = cp.off;
            P.Co = cp.Co;
            P.Ci = cp.Ci;
            P.p0 = at<float>(e, e->ws_wperm0[l]);
            P.p1 = at<float>(e, e->ws_wperm1[l]);
            P.pT = at<float>(e, e->ws_wpermT[l]);
        }
        if (NC - 1 > 2) aa.nperm = 0;
    }
    KStep k;
    k.name = aa.mode ? "adam_fused" : "grad_reduce";
    const double P = (double)np.P;
    // read partials; write g; Adam: read p,m,v (+target), write p,m,v (+target)
    k.bytes = 4.0 * (part_elems + P + (aa.mode ? 6.0 * P + (aa.soft ? 2.0 * P : 0.0) : 0.0));
    k.flops = aa.mode ? 12.0 * P : 0.0;
    k.run = adam_run(e, aa);
    if (args_out) *args_out = aa;
    return k;
}


// Blocked weight copies for the fused plan (relayout.hpp), rebuilt by spare workgroups of
// the sampler launch at the start of every step.
RelayoutArgs relayout_args(dqnx_engine* e, int* blocks) {
    RelayoutArgs r;
    memset(&r, 0, sizeof(r));
    *blocks = 0;
    if (e->bwd_plan != 2) return r;
    const NetPlan& np = e->np;
    float* params = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    float* tparams = at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]);
    int64_t q = 0;
    auto add = [&](const float* src, float* dst, int rows, int cols, int kind, int nch, int64_t nq) {
        RelayoutJob& j = r.job[r.njobs++];
        j.src = src; j.dst = dst; j.rows = rows; j.cols = cols; j.kind = kind; j.nch = nch; j.q0 = q;
        q += nq;
    };
    const bool bf = e->fplan.bf16 != 0;
    const int kc = bf ? 32 : 16, per_q = bf ? 8 : 4;   // K per chunk, elements per 16-byte unit
    for (int l = 0; l < (int)np.dense.size(); l++) {
        const LayerPlan& lp = np.dense[l];
        const int kp = e->fplan.kpad[l];
        const int64_t nq = (int64_t)lp.out * kp / per_q;
        add(params + lp.off, at<float>(e, e->ws_wblk[0][l]), lp.out, lp.in, bf ? 2 : 0, kp / kc, nq);
        add(tparams + lp.off, at<float>(e, e->ws_wblk[1][l]), lp.out, lp.in, bf ? 2 : 0, kp / kc, nq);
        if (l >= 1) add(params + lp.off, at<float>(e, e->ws_wblkT[l]), lp.out, lp.in, bf ? 3 : 1, lp.out / kc,
                        (int64_t)lp.out * lp.in / per_q);
    }
    r.total_q = q;
    int b = (int)((q + 1023) / 1024);
    *blocks = b < 1 ? 1 : (b > 64 ? 64 : b);
    return r;
}

// The single-GPU PER step's SumTree update split over the launches that run anyway (round 3): the
// head kernel does k_per_prep's work, the weight-gradient launch (k_dw_adam16 on 32 x 16 tiles, or
// k_dw_bf16) runs k_per_prop's workgroups, leaving the order-dependent k_per_update launch.  Not
// under DP (the |delta| of other shards arrive by all-gather), not in numpy-1.21 mode (k_per_chain),
// not on the fp32 slab plan.  DQNX_PER_FUSED=0: the three launches.  With the tracking in the
// gradient launch too (per_track_inlaunch, the default) no PER launch is left: k_dw_adam16 runs
// the tracking workgroup and its prop workgroups wait for it in the same launch; k_dw_bf16 runs
// the tracking workgroup and the Adam launch after it the prop workgroups.
bool dw_adam16_on(const dqnx_engine* e, int flags);
static bool per_fused_update(const dqnx_engine* e, int flags) {
    if (e->cfg.algo != DQNX_ALGO_PER_DOUBLE || (flags & DQNX_STEP_GRADS_ONLY) || e->cfg.per_numpy121) return false;
    if (e->bwd_plan != 2 || e->Bg > PER_CHUNK || route_knob("DQNX_PER_FUSED", 1) == 0) return false;
    if (e->fplan.bf16) return true;
    return dw_adam16_on(e, flags) && route_knob("DQNX_DW16_R", 2) == 2;
}
static bool per_track_inlaunch(const dqnx_engine* e, int flags) {
    return per_fused_update(e, flags) && route_knob("DQNX_PER_TRACK_INLAUNCH", 1) != 0;
}

// Fused MLP plan (bwd_plan 2): forward of every layer + head in one launch, head / TD /
// dZ chain in one launch, every dW in one split-K launch, then the Adam pass.
void build_fused_steps(dqnx_engine* e, int flags, int32_t* idx, int32_t* phys, std::vector<KStep>& ks,
                       const SampleArgs* sample_next) {
    const dqnx_config& c = e->cfg;
    const NetPlan& np = e->np;
    const int L = (int)np.dense.size();
    const int A = c.net.n_actions;
    const int act = c.net.activation;
    dqnx_ctrl* ctrl = ctrl_of(e);
    float* params = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    float* tparams = at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]);
    const double Bl = e->Bl;
    const bool dbl = c.algo != DQNX_ALGO_DQN;
    const int nstreams = dbl ? 3 : 2;
    double body_flops = 0, wbytes = 0;   // per stream: 2 * in * out summed; weight bytes
    for (int l = 0; l < L; l++) {
        body_flops += 2.0 * np.dense[l].in * np.dense[l].out;
        wbytes += (e->fplan.bf16 ? 2.0 : 4.0) * np.dense[l].in * np.dense[l].out + 4.0 * np.dense[l].out;
    }
    // row tile t of every stream (and the head's tile t) on XCD t % 8: the head kernel then reads
    // the forward's outputs from its own XCD's L2 (16-row tiles, tiles % 8 == 0).  Measured at
    // B=1024: head_bwd 7.2 -> 6.6 us, the forward unchanged; DQNX_XCD_ROWS=0 keeps xcd_remap's order
    const int ftiles = (e->Bl + 15) / 16;
    // (row tiles of 16 * mr rows: the head kernel's 16-sample tiles follow their row tile's XCD)
    const int frows = 16 * e->fplan.mr;
    const bool xcd_rows = route_knob("DQNX_XCD_ROWS", 1) != 0 && ftiles % 8 == 0 &&
                          (e->fplan.mr == 1 || (route_knob("DQNX_XCD_ROWS_MR", 1) != 0 && e->Bl % frows == 0 &&
                                                (e->Bl / frows) % 8 == 0));
    // 2. forward (R:dqn/agent.py:209-214 / 172-173 streams, R:dqn/network.py:61-65, 90-96)
    {
        FusedFwdArgs fa = e->fplan;
        fa.Bl = e->Bl;
        fa.tiles = (e->Bl + 16 * fa.mr - 1) / (16 * fa.mr);
        fa.nstreams = nstreams;
        for (int l = 0; l < L; l++) fa.woff[l] = np.dense[l].off;
        fa.head_off = np.head_off;
        fa.head_kind = c.net.head;
        fa.stream_of[0] = 0;
        fa.stream_of[1] = dbl ? 1 : 2;
        fa.stream_of[2] = 2;
        fa.params = params;
        fa.tparams = tparams;
        fa.ring_obs = at<float>(e, e->off[DQNX_BUF_RING_OBS]);
        fa.ring_next = at<float>(e, e->off[DQNX_BUF_RING_NEXT_OBS]);
        fa.ring_stride = e->stride;
        fa.ring16_obs = e->stride16 ? at<uint16_t>(e, e->ws_ring16[0]) : nullptr;
        fa.ring16_next = e->stride16 ? at<uint16_t>(e, e->ws_ring16[1]) : nullptr;
        fa.stride16 = e->stride16;
        fa.phys = phys;
        fa.xcopy = at<float>(e, e->ws_xobs);
        for (int l = 0; l < L; l++) fa.H[l] = at<float>(e, e->ws_H[l]);   // stream-0 third of [3][Bl][w]
        if (e->dwt) {   // + the T16 copies k_dw_bf16t reads
            fa.xT16 = at<uint16_t>(e, e->ws_xT16);
            fa.tkb = e->kslice[0];
            for (int l = 0; l < L; l++) fa.HT16[l] = at<uint16_t>(e, e->ws_HT16[l]);
        }
        fa.raw = at<float>(e, e->ws_raw);
        fa.trans = at<float4>(e, e->ws_trans);
        fa.act = at<int32_t>(e, e->off[DQNX_BUF_RING_ACT]);
        fa.rew = at<float>(e, e->off[DQNX_BUF_RING_REW]);
        fa.done = at<float>(e, e->off[DQNX_BUF_RING_DONE]);
        for (int l = 0; l < L; l++) {
            fa.wblk[0][l] = at<float>(e, e->ws_wblk[0][l]);
            fa.wblk[1][l] = at<float>(e, e->ws_wblk[1][l]);
        }
        fa.stamps = at<int64_t>(e, e->ws_stamps);
        fa.xcd_rows = xcd_rows ? 1 : 0;
        fa.lds_min = 1024 * tuning_knob("DQNX_FWD_LDSKB", 0);
        fa.adam_ctrl = ctrl;   // (the head kernel below gets no ctrl: the forward stores the scalars)
        if (e->ws_npc && c.algo == DQNX_ALGO_PER_DOUBLE && !(e->fsplit > 1 && L >= 2 && fa.mr == 1)) {
            fa.npc = at<uint32_t>(e, e->ws_npc);   // the next PER sample's MT blocks, twisted ahead
            fa.np_state = ctrl->np_mt;
            fa.npc_blocks = np_cache_blocks(e->Bg);
        }
        fa.ab = adam_bias_args(e);
        if (e->fpair && e->ws_pairflag && xcd_rows && L >= 2 && fa.mr == 1 && !fa.bf16 && fa.gw == 0) {
            fa.phase = 3;   // (the row tiles keep their XCDs: the head kernel's mapping is unchanged)
            fa.csplit = 2;
            fa.pair_flags = at<uint32_t>(e, e->ws_pairflag);
            fa.err = &ctrl->error;
        }
        if (sample_next) {   // + the next step's minibatch into the staging slot (in-launch prefetch)
            // the one-pass shape only when the row tiles leave a CU idle (its LDS allows one
            // workgroup per CU); else the 3-block passes, whose LDS keeps two per CU
            const int wgs = fa.tiles * nstreams * (fa.phase == 3 ? 2 : 1) + 1;
            fa.samp_shape = sample_next->k <= 2048 ? 1 : (wgs <= e->n_cu ? 3 : 2);
            fa.samp = *sample_next;
#ifdef DQNX_STAMPS
            fa.samp.stamps = at<int64_t>(e, e->ws_stamps);   // (diagnostic builds: the sampler's slots 0-15)
#else
            fa.samp.stamps = nullptr;
#endif
        }
        KStep k;
        k.name = sample_next ? "mlp_fwd+sample" : "mlp_fwd";
        k.flops = nstreams * Bl * (body_flops + 2.0 * np.NH * np.F);
        // gathered rows in, stream-0 rows + activations + raw heads out, online + target weights
        double hsum = 0;
        for (int l = 0; l < L; l++) hsum += np.dense[l].out;
        k.bytes = 4.0 * (nstreams * Bl * np.dense[0].in + Bl * np.dense[0].in + Bl * hsum + 3.0 * Bl * 16)
                  + 2.0 * (wbytes + 4.0 * np.head_params);
        if (e->fsplit > 1 && L >= 2 && fa.mr == 1) {
            // layer 1 on csplit workgroups per (16 * fsplit_mr)-row tile, then layers 2.. + head (H_1
            // via HBM); the sampler workgroup (in-launch prefetch) rides in the layer-1 launch
            const double w0 = (double)np.dense[0].in * np.dense[0].out;
            FusedFwdArgs f1 = fa, f2 = fa;
            f1.phase = 1;
            f1.csplit = e->fsplit;
            f1.xcd_rows = 0;   // (the layer-2 launch places row tile t on XCD t % 8 for the head kernel)
            f1.lds_min = 1024 * tuning_knob("DQNX_FWD_L1_LDSKB", 0);
            f2.lds_min = 1024 * tuning_knob("DQNX_FWD_L2_LDSKB", 0);
            if (e->fsplit_mr > 1) {
                FusedFwdArgs t = e->fplan;
                fused_fwd_plan(t, c.net.obs_dim, e->fplan.bf16 != 0, e->fsplit_mr);
                f1.mr = t.mr;
                f1.sx = t.sx;
                f1.sh = t.sh;
                f1.buf0 = t.buf0;
                f1.buf1 = t.buf1;
                f1.tiles = (e->Bl + 16 * f1.mr - 1) / (16 * f1.mr);
            }
            if (sample_next) {
                const int wgs = f1.tiles * nstreams * f1.csplit + 1;
                f1.samp_shape = sample_next->k <= 2048 ? 1 : (wgs <= e->n_cu ? 3 : 2);
            }
            f2.phase = 2;
            f2.samp_shape = 0;
            f2.adam_ctrl = nullptr;   // (the layer-1 launch stores the step's Adam scalars)
            KStep k1, k2;
            k1.name = sample_next ? "mlp_fwd_l1+sample" : "mlp_fwd_l1";
            k1.flops = nstreams * Bl * 2.0 * w0;
            k1.bytes = 4.0 * (nstreams * Bl * (np.dense[0].in + np.dense[0].out) + Bl * np.dense[0].in)
                       + 2.0 * (e->fplan.bf16 ? 2.0 : 4.0) * w0;
            k1.run = [=](hipStream_t s) { return launch_fused_fwd(f1, act, s); };
            k2.name = "mlp_fwd_rest";
            k2.flops = k.flops - k1.flops;
            k2.bytes = 4.0 * (nstreams * Bl * np.dense[0].out + Bl * (hsum - np.dense[0].out) + 3.0 * Bl * 16)
                       + 2.0 * (wbytes - (e->fplan.bf16 ? 2.0 : 4.0) * w0 + 4.0 * np.head_params);
            k2.run = [=](hipStream_t s) { return launch_fused_fwd(f2, act, s); };
            ks.push_back(k1);
            ks.push_back(k2);
        } else {
            k.run = [=](hipStream_t s) { return launch_fused_fwd(fa, act, s); };
            ks.push_back(k);
        }
    }
    // 3. head / TD / Huber / dZ chain (R:dqn/agent.py:209-221; PER :259-267)
    {
        HeadBwdArgs ha;
        memset(&ha, 0, sizeof(ha));
        ha.L = L;
        ha.Bl = e->Bl;
        ha.nsplit = 1;
        ha.bf16 = e->fplan.bf16;
        // dZ_1's columns over nsplit workgroups per 16-sample tile: the largest of 4, 2 that keeps
        // tiles * nsplit <= 256 (one workgroup per CU).  Measured at MLP-284: B=1024 head 6.5 ->
        // 6.0 us with 4 parts; B=4096 best unsplit (9.2 vs 9.5 with 2, 13.8 with 4)
        for (int v : {4, 2})
            if (ha.nsplit == 1 && L >= 2 && np.dense[0].out % (v * 16) == 0 && e->tiles * v <= 256) ha.nsplit = v;
        if (route_flag("DQNX_HEAD_SPLIT")) {
            const int v = route_knob("DQNX_HEAD_SPLIT", 1);
            if (v == 1 || ((v == 2 || v == 4) && L >= 2 && np.dense[0].out % (v * 16) == 0)) ha.nsplit = v;
        }
        ha.A = A;
        ha.NH = np.NH;
        ha.F = np.F;
        ha.head_kind = c.net.head;
        ha.algo = c.algo;
        for (int l = 0; l < L; l++) {
            ha.in[l] = np.dense[l].in;
            ha.out[l] = np.dense[l].out;
            ha.woff[l] = np.dense[l].off;
            ha.H[l] = at<float>(e, e->ws_H[l]);
            ha.dZ[l] = at<float>(e, e->ws_dZ[l]);
        }
        ha.head_off = np.head_off;
        ha.inv_bg = (float)(1.0 / (double)e->Bg);
        ha.gamma = (float)c.gamma;
        ha.params = params;
        ha.raw = at<float>(e, e->ws_raw);
        ha.trans = at<float4>(e, e->ws_trans);
        ha.phys = phys;
        ha.act = at<int32_t>(e, e->off[DQNX_BUF_RING_ACT]);
        ha.rew = at<float>(e, e->off[DQNX_BUF_RING_REW]);
        ha.done = at<float>(e, e->off[DQNX_BUF_RING_DONE]);
        ha.isw = (c.algo == DQNX_ALGO_PER_DOUBLE) ? at<float>(e, e->off[DQNX_BUF_IS_WEIGHTS]) + e->shard_begin : nullptr;
        ha.abs_td_out = (c.algo == DQNX_ALGO_PER_DOUBLE) ? at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]) + e->shard_begin
                                                         : nullptr;
        ha.Q = at<float>(e, e->off[DQNX_BUF_Q]);
        ha.td = at<float>(e, e->off[DQNX_BUF_TD]);
        ha.dhead = at<float>(e, e->ws_dhead);
        if (e->dwt) {
            for (int l = 0; l < L; l++) ha.dZT16[l] = at<uint16_t>(e, e->ws_dZT16[l]);
            ha.dheadT16 = at<uint16_t>(e, e->ws_dheadT16);
            ha.tkb = e->kslice[0];
        }
        ha.loss_partial = at<float>(e, e->ws_loss_part);
        ha.ctrl = nullptr;   // the forward launch stores the step's Adam scalars
        ha.xcd_rows = xcd_rows ? 1 : 0;
        ha.xcd_mr = e->fplan.mr;
        ha.xcd_shift = (sample_next || (e->ws_npc && c.algo == DQNX_ALGO_PER_DOUBLE)) ? 1 : 0;   // forward's block 0
        for (int l = 1; l < L; l++) ha.wblkT[l] = at<float>(e, e->ws_wblkT[l]);
        ha.ab = adam_bias_args(e);
        ha.stamps = at<int64_t>(e, e->ws_stamps);
        if (per_fused_update(e, flags)) {   // the single-GPU PER step: k_per_prep's work per sample here
            ha.pp = per_update_args(e);
            ha.pp.mode = 0;
            ha.pp.n = e->Bg;
            ha.pp.slots = idx;
            ha.pp.abs_td = at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]);
            ha.pp_on = 1;
        }
        KStep k;
        k.name = "head_bwd";
        double dzf = 2.0 * Bl * 16 * np.F, dzb = 0;
        for (int l = L - 1; l >= 1; l--) {
            dzf += 2.0 * Bl * np.dense[l].out * np.dense[l].in;
            dzb += 4.0 * (np.dense[l].out * (double)np.dense[l].in + 2.0 * Bl * np.dense[l].in);
        }
        k.flops = dzf;
        k.bytes = 4.0 * (3.0 * Bl * 16 + 2.0 * Bl * np.F + 16.0 * Bl + 3.0 * Bl * A + 6.0 * Bl) + dzb
                  + 4.0 * np.head_params;
        k.run = [=](hipStream_t s) { return launch_head_bwd(ha, act, s); };
        ks.push_back(k);
    }
    // 3b. PER priorities (single GPU; under DP after the all-gather, in dqnx_apply_grads).  Fused:
    //     the head kernel did k_per_prep's work, the gradient launch below runs k_per_prop's
    //     workgroups beside its tiles, so only the order-dependent tracking launch remains here
    PerUpdateArgs pua;
    const bool per_fused = per_fused_update(e, flags);
    const bool per_track = per_track_inlaunch(e, flags);
    if (per_fused) {
        pua = per_update_args(e);
        pua.mode = 0;
        pua.n = e->Bg;
        pua.slots = idx;
        pua.abs_td = at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]);
        pua.skip = PER_SKIP_PREP | PER_SKIP_PROP;
    }
    if (c.algo == DQNX_ALGO_PER_DOUBLE && !(flags & DQNX_STEP_GRADS_ONLY) && !per_track) {
        KStep k;
        k.name = "per_update";
        k.bytes = e->Bg * (4.0 + 4.0 + 8.0 * 2.0 * 21.0);
        if (per_fused) k.run = [=](hipStream_t s) { return launch_per_update(pua, s); };
        else k.run = [=](hipStream_t s) { return enqueue_per_update(e, idx, s); };
        ks.push_back(k);
    }
    // 4. every weight gradient: split-K slabs of dZ_l^T [X_l | 1] and dHead^T [H_L | 1]
    {
        BwdArgs ba;
        memset(&ba, 0, sizeof(ba));
        ba.Bl = e->Bl;
        ba.kslice = e->kslice[0];
        ba.dw_slices = e->slices[0];
        double flops = 0, bytes = 0;
        for (int l = L - 1; l >= 0; l--) {   // widest problems last: the grid tail is the head
            const LayerPlan lp = np.dense[l];
            DwProblem& d = ba.dw[ba.ndw++];
            d.dZ = at<float>(e, e->ws_dZ[l]);
            d.ldz = lp.out;
            if (l > 0) {
                d.X = at<float>(e, e->ws_H[l - 1]);
                d.ldx = lp.in;
            } else {
                d.X = at<float>(e, e->ws_xobs);
                d.ldx = e->stride;
            }
            d.in = lp.in;
            d.out = lp.out;
            d.partial = at<float>(e, e->ws_part[l]);
            d.pstride = (int64_t)lp.out * lp.in + lp.out;
            d.head_kind = -1;
            if (e->dwt) {
                d.dZT = at<uint16_t>(e, e->ws_dZT16[l]);
                d.cz = lp.out;
                d.XT = at<uint16_t>(e, l > 0 ? e->ws_HT16[l - 1] : e->ws_xT16);
                d.cx = lp.in;
            }
            flops += 2.0 * Bl * lp.out * (lp.in + 1.0);
            bytes += 4.0 * (Bl * (lp.out + lp.in) + ba.dw_slices * (lp.out * (lp.in + 1.0)));
        }
        {
            DwProblem& h = ba.dw[ba.ndw++];
            h.dZ = at<float>(e, e->ws_dhead);
            h.ldz = 16;
            if (e->dwt) {
                h.dZT = at<uint16_t>(e, e->ws_dheadT16);
                h.cz = 16;
                h.XT = at<uint16_t>(e, e->ws_HT16[L - 1]);
                h.cx = np.F;
            }
            h.X = at<float>(e, e->ws_H[L - 1]);
            h.ldx = np.F;
            h.in = np.F;
            h.out = np.NH;
            h.partial = at<float>(e, e->ws_head_part);
            h.pstride = head_pstride(np);
            h.head_kind = c.net.head;
            h.A = A;
            flops += 2.0 * Bl * np.NH * (np.F + 1.0);
            bytes += 4.0 * (16.0 * Bl + Bl * np.F + ba.dw_slices * (double)np.head_params);
        }
        if (dw_adam16_on(e, flags)) {   // full-minibatch 16 x 16 tiles + Adam + blocked copies
            DwAdam16Args da;
            memset(&da, 0, sizeof(da));
            int tiles = 0;
            // 32 x 16 tiles: every X element loaded feeds two MFMAs, half the workgroups (216 at
            // MLP-284: one per CU).  Measured at B=1024: 11.8 -> 10.35 us in context, bitwise equal
            // to the 16 x 16 tiles (DQNX_DW16_R=1 selects those)
            const int rows16 = route_knob("DQNX_DW16_R", 2) == 1 ? 1 : 2;
            da.rows16 = rows16;
            auto add = [&](const DwProblem& p, int64_t poff, int l) {
                DwAdam16Layer& d = da.L[da.nl++];
                d.dZ = p.dZ;
                d.ldz = p.ldz;
                d.X = p.X;
                d.ldx = p.ldx;
                d.in = p.in;
                d.out = p.out;
                d.poff = poff;
                d.head_kind = p.head_kind;
                d.A = p.A;
                d.ti = (p.in + 15) / 16;
                d.t0 = tiles;
                tiles += d.ti * ((p.out + 16 * rows16 - 1) / (16 * rows16));
                if (l >= 0) {
                    d.fwd_online = at<float>(e, e->ws_wblk[0][l]);
                    d.fwd_target = at<float>(e, e->ws_wblk[1][l]);
                    d.chain = l >= 1 ? at<float>(e, e->ws_wblkT[l]) : nullptr;
                    d.nch_fwd = e->fplan.kpad[l] / 16;
                    d.nch_chain = np.dense[l].out / 16;
                }
            };
            for (int q = 0; q < ba.ndw; q++) {   // dense layers last-first, then the head
                const int l = q < L ? L - 1 - q : -1;
                add(ba.dw[q], l >= 0 ? np.dense[l].off : np.head_off, l);
            }
            AdamArgs aa;
            adam_kstep(e, flags, &aa);
            da.tiles = tiles;
            da.Bl = e->Bl;
            da.mode = aa.mode;
            da.soft = aa.soft;
            da.n_params = np.P;
            da.p = aa.p;
            da.m = aa.m;
            da.v = aa.v;
            da.grads = aa.grads;
            da.target = aa.target;
            da.ctrl = aa.ctrl;
            da.w1 = aa.w1;
            da.beta2 = aa.beta2;
            da.c2 = aa.c2;
            da.eps = aa.eps;
            da.tau = aa.tau;
            da.one_minus_tau = aa.one_minus_tau;
            da.loss_partial = aa.loss_partial;
            da.n_loss_partial = aa.n_loss_partial;
            da.batch_global = aa.batch_global;
            da.mtc = aa.mtc;
            da.mtc_blocks = aa.mtc_blocks;
            da.stamps = at<int64_t>(e, e->ws_stamps);
            if (sample_next) {   // the staged minibatch becomes the compute slot's (in-launch prefetch)
                da.pf_idx_src = sample_next->out;
                da.pf_idx_dst = idx;
                da.pf_nidx = e->Bg;
                da.pf_phys_src = sample_next->phys_out;
                da.pf_phys_dst = phys;
                da.pf_nphys = e->Bl;
                // (da.mtc kept: the extension workgroup twists the next draw's MT blocks ahead for the
                // forward's sampler body, which reads them from the cache instead of twisting)
            }
            if (per_fused) {
                da.pprop = pua;
                da.pprop_wgs = (e->Bg + 511) / 512;
                da.ptrack = per_track ? 1 : 0;
            }
            const double P = (double)np.P;
            KStep k;
            k.name = da.mode ? "dw_adam16" : "dw16_grads";
            k.flops = flops + (da.mode ? 12.0 * P : 0.0);
            // dZ / X rows once; p, m, v read and written, grads written (+ target read and
            // written); the blocked copies: fwd online (+ fwd target), chain for l >= 1
            double ops = Bl * (16.0 + np.F), blk = 0;
            for (int l = 0; l < L; l++) {
                const double w = (double)np.dense[l].out * np.dense[l].in;
                ops += Bl * (np.dense[l].out + np.dense[l].in);
                blk += w * (da.soft ? 2.0 : 1.0) + (l >= 1 ? w : 0.0);
            }
            k.bytes = 4.0 * (ops + (da.mode ? 7.0 * P + (da.soft ? 2.0 * P : 0.0) + blk : P));
            k.run = [=](hipStream_t s) { return launch_dw_adam16(da, s); };
            ks.push_back(k);
            e->dw16_cache[e->building_key] = da;   // (the bucketed DP step launches subsets of it)
            return;
        }
        if (e->fplan.bf16) {   // bf16 operands, fp32 slabs: the same Adam pass follows
            dw_bf16_grid(ba);
            ba.t16 = e->dwt && dw_bf16t_supported(ba) ? 1 : 0;
            ba.stamps = at<int64_t>(e, e->ws_stamps);
            if (per_fused) {   // tracking in this launch, prop in the Adam launch; or prop here
                ba.pprop = pua;
                ba.ptrack = per_track ? 1 : 0;
                ba.pprop_wgs = per_track ? 0 : (e->Bg + 255) / 256;
            }
            KStep k;
            k.name = "dw_all";
            k.flops = flops;
            k.bytes = bytes;
            k.run = [=](hipStream_t s) { return launch_dw_bf16(ba, s); };
            ks.push_back(k);
        } else {                // split-K slabs of every dW, then the Adam pass sums them
            bwd_level_grid(ba);
            KStep k;
            k.name = "dw_all";
            k.flops = flops;
            k.bytes = bytes;
            k.run = [=](hipStream_t s) { return launch_bwd_level(ba, act, s); };
            ks.push_back(k);
        }
        if (sample_next) {   // the Adam launch's last workgroup takes the staged minibatch over
            AdamArgs aa;
            KStep k = adam_kstep(e, flags, &aa);
            aa.pf_idx_src = sample_next->out;
            aa.pf_idx_dst = idx;
            aa.pf_nidx = e->Bg;
            aa.pf_phys_src = sample_next->phys_out;
            aa.pf_phys_dst = phys;
            aa.pf_nphys = e->Bl;
            // (aa.mtc kept: the forward's sampler body reads the blocks its extension twists ahead)
            fill_blk_layers(e, aa, true);   // ... and the next step has no sampler launch to rebuild them
            if (per_track) {
                aa.pprop = pua;
                aa.pprop_wgs = (e->Bg + 255) / 256;
            }
            k.run = [=](hipStream_t s) { return launch_adam(aa, s); };
            ks.push_back(k);
            return;
        }
        if (per_track) {   // the prop workgroups after the gradient launch's tracking
            AdamArgs aa;
            KStep k = adam_kstep(e, flags, &aa);
            aa.pprop = pua;
            aa.pprop_wgs = (e->Bg + 255) / 256;
            k.run = adam_run(e, aa);
            ks.push_back(k);
            return;
        }
        ks.push_back(adam_kstep(e, flags));
    }
}

// key = flags | (slot << 8) | KEY_RELAYOUT: `slot` selects the (sampled indices, physical rows)
// buffer pair; KEY_RELAYOUT = the sampler launch also rebuilds the fused plan's blocked weight
// copies (only after the weights changed outside the Adam pass, which keeps them current).
constexpr int KEY_RELAYOUT = 0x40;
// KEY_SAMPLE_NEXT (in-launch prefetch; the compute slot is 0): no sampler launch at the front (slot
// 0 holds the minibatch the previous step drew); one more workgroup of the forward launch draws the
// next step's minibatch into the staging slot 1, and the last launch copies it over slot 0
constexpr int KEY_SAMPLE_NEXT = 0x80;
// KEY_AGENT_RNG: the sampler launch draws from the drop-in Agent's pinned state block in place
// (dqnx_agent_launch, uniform replay) instead of the control block an upload copy filled
constexpr int KEY_AGENT_RNG = 0x4000;

SampleArgs uniform_sample_args(dqnx_engine* e, int32_t* idx, int32_t* phys) {
    dqnx_ctrl* ctrl = ctrl_of(e);
    SampleArgs sa;
    memset(&sa, 0, sizeof(sa));
    sa.state = ctrl->py_mt;
    sa.n_dev = &ctrl->ring_size;
    sa.k = e->Bs;
    sa.setsize = e->setsize;
    sa.out = idx;
    sa.err = &ctrl->error;
    sa.pool = at<int32_t>(e, e->ws_pool);
    sa.phys_out = phys;
    sa.shard_begin = e->shard_begin;
    sa.shard_len = e->Bl;
    sa.wptr_dev = &ctrl->ring_wptr;
    sa.capacity = e->cfg.capacity;
    sa.stamps = at<int64_t>(e, e->ws_stamps);
    sa.gtab = sample_table_bytes(e->Bs) ? at<unsigned long long>(e, e->ws_gtab) : nullptr;
    sa.mtc = at<uint32_t>(e, e->ws_mtc);
    sa.mtc_blocks = e->mtc_blocks;
    sa.bm_cap = route_knob("DQNX_SAMPLER_BM_CAP", 0);
    sa.bm_rolled = route_knob("DQNX_SAMPLER_ROLLED", 0);
    return sa;
}

// The fused plan's forward launch can host the next step's sampler workgroup: uniform replay, the
// engine draws its own indices, the whole forward is one launch, and k fits the multi-pass sampler
// body's LDS table.  The step's last launch (k_dw_adam16, or the slab plan's Adam pass) copies the
// staged minibatch over the compute slot.
// The micro-CNN plan's forward launch hosts it the same way (k_micro_fwd block 0, k <= 2048), and
// its Adam / gradient-reduce launch copies the staged minibatch.
bool inlaunch_prefetch_ok(const dqnx_engine* e, int flags) {
    if (tuning_flag("DQNX_PF_SIDE")) return false;   // measurements: the side-stream pipeline instead
    if (e->cfg.algo == DQNX_ALGO_PER_DOUBLE || (flags & DQNX_STEP_GIVEN_INDICES)) return false;
    if (e->bwd_plan == 2) return e->Bs <= FWD_SAMPLE_MAX_K;
    return e->bwd_plan == 0 && e->micro && e->Bs <= MICRO_SAMPLE_MAX_K;
}
// the fused plan's blocked weight copies need a rebuild launch before the next step
static bool relayout_due(const dqnx_engine* e) { return e->bwd_plan == 2 && e->wblk_dirty; }

std::vector<KStep> build_learn_steps(dqnx_engine* e, int key) {
    const int flags = key & 0x3f;
    const int slot = (key >> 8) & 1;
    std::vector<KStep> ks;
    const dqnx_config& c = e->cfg;
    const NetPlan& np = e->np;
    const int L = (int)np.dense.size();
    const int A = c.net.n_actions;
    const int act = c.net.activation;
    dqnx_ctrl* ctrl = ctrl_of(e);
    float* params = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    float* tparams = at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]);
    int32_t* idx = at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]) + (size_t)slot * e->Bg;
    int32_t* phys = at<int32_t>(e, e->ws_phys) + (size_t)slot * e->Bl;
    const double Bl = e->Bl;
    const double Bg_ = e->Bg;

    // 1. sample (R:dqn/replay_memory.py:38-39; PER :69-92)
    int rl_blocks = 0;
    RelayoutArgs rl = relayout_args(e, &rl_blocks);
    if (!(key & KEY_RELAYOUT)) {
        rl.njobs = 0;
        rl.total_q = 0;
        rl_blocks = 0;
    }
    if (c.algo == DQNX_ALGO_PER_DOUBLE) {
        PerSampleArgs pa = per_sample_args(e, idx, phys);
        pa.rl = rl;
        pa.rl_blocks = rl_blocks;
        KStep k;
        k.name = "per_sample";
        k.bytes = 2.0 * 625 * 4 + 8.0 * Bg_ * 22 + 8.0 * e->Bg + 4.0 * Bl;
        k.run = [=](hipStream_t s) { return launch_per_sample(pa, s); };
        ks.push_back(k);
    } else if (flags & DQNX_STEP_GIVEN_INDICES) {
        KStep k;
        k.name = "idx_to_phys";
        k.bytes = 8.0 * Bl;
        k.run = [=](hipStream_t s) {
            return launch_idx_to_phys(idx, phys, e->shard_begin, e->Bl, ctrl, c.capacity, &rl, rl_blocks, s);
        };
        ks.push_back(k);
    } else if (!(key & KEY_SAMPLE_NEXT)) {
        SampleArgs sa = uniform_sample_args(e, idx, phys);
        sa.rl = rl;
        sa.rl_blocks = rl_blocks;
        if (key & KEY_AGENT_RNG) sa.state_in = e->ag_rng_zc;
        KStep k;
        k.name = "sample_uniform";
        k.bytes = 2.0 * 625 * 4 + 4.0 * e->Bs + 4.0 * Bl;
        k.run = [=](hipStream_t s) { return launch_sample_uniform(sa, s); };
        ks.push_back(k);
    }

    if (e->bwd_plan == 2) {
        SampleArgs nxt;
        const bool sample_next = (key & KEY_SAMPLE_NEXT) != 0;
        if (sample_next)   // the staging slot (the compute slot is slot 0)
            nxt = uniform_sample_args(e, at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]) + (size_t)e->Bg,
                                      at<int32_t>(e, e->ws_phys) + (size_t)e->Bl);
        build_fused_steps(e, flags, idx, phys, ks, sample_next ? &nxt : nullptr);
        return ks;
    }

    // 2. forward layers: streams 0 online(obs), 1 online(next) [double], 2 target(next)
    const bool dbl = c.algo != DQNX_ALGO_DQN;
    const int nstreams = dbl ? 3 : 2;
    const int NC = (int)np.conv.size();
    const float* ring_obs = at<float>(e, e->off[DQNX_BUF_RING_OBS]);
    const float* ring_next = at<float>(e, e->off[DQNX_BUF_RING_NEXT_OBS]);
    if (NC && e->conv_ig) {   // 2a'. implicit-GEMM convs, the last one writing F (conv_ig.hip)
        ConvPermArgs pa;
        memset(&pa, 0, sizeof(pa));
        double pbytes = 0;
        for (int l = 0; l < NC; l++) {
            const ConvPlan& cp = np.conv[l];
            const int taps = cp.kh * cp.kw;
            pa.job[pa.njobs++] = ConvPermJob{params + cp.off, at<float>(e, e->ws_wperm0[l]), cp.Co, cp.Ci, taps, 0};
            pa.job[pa.njobs++] = ConvPermJob{tparams + cp.off, at<float>(e, e->ws_wperm1[l]), cp.Co, cp.Ci, taps, 0};
            if (l > 0) pa.job[pa.njobs++] = ConvPermJob{params + cp.off, at<float>(e, e->ws_wpermT[l]), cp.Co, cp.Ci, taps, 1};
            pbytes += 8.0 * cp.Co * cp.K * (l > 0 ? 3 : 2);
        }
        {
            KStep k;
            k.name = "conv_perm";
            k.bytes = pbytes;
            k.run = [=](hipStream_t s) { return launch_conv_perm(pa, s); };
            ks.push_back(k);
        }
        for (int l = 0; l < NC; l++) {
            const ConvPlan cp = np.conv[l];
            const bool last = l == NC - 1;
            ConvIgArgs ca;
            cig_fwd_geom(cp, e->Bl, l == 0, ca);
            ca.act = act;
            CigSource& S = ca.src;
            if (l == 0) {   // the micro grid straight from the ring rows (CHW after the macro features)
                S.phys = phys;
                S.bstride = e->stride;
                S.off = np.macro_len;
                S.pstride = 1;
                S.cstride = cp.Hi * cp.Wi;
            } else {
                S.bstride = (int64_t)cp.Hi * cp.Wi * cp.Ci;
                S.pstride = cp.Ci;
                S.cstride = 1;
            }
            int z = 0;
            for (int st = 0; st < 3; st++) {
                if (st == 1 && !dbl) continue;
                S.base[z] = l == 0 ? (st == 0 ? ring_obs : ring_next)
                                   : at<float>(e, e->ws_Hc[l - 1]) + (int64_t)st * e->Bl * cp.Hi * cp.Wi * cp.Ci;
                ca.W[z] = at<float>(e, st == 2 ? e->ws_wperm1[l] : e->ws_wperm0[l]);
                ca.bias[z] = (st == 2 ? tparams : params) + cp.off + (int64_t)cp.Co * cp.K;
                if (last) {
                    ca.out[z] = at<float>(e, e->ws_F) + (int64_t)st * e->Bl * np.strideF;
                    ca.ring[z] = st == 0 ? ring_obs : ring_next;
                } else {
                    ca.out[z] = at<float>(e, e->ws_Hc[l]) + (int64_t)st * e->Bl * cp.Ho * cp.Wo * cp.Co;
                }
                z++;
            }
            ca.nstreams = z;
            if (last) {   // F[b] = cat(flatten_CHW(conv), macro) (R:env/dqn_config.py:135-138)
                ca.ob = np.strideF;
                ca.orow = cp.Wo;
                ca.opix = 1;
                ca.och = cp.Ho * cp.Wo;
                ca.phys = phys;
                ca.ring_stride = e->stride;
                ca.macro_len = np.macro_len;
                ca.flat_cols = cp.Co * cp.Ho * cp.Wo;
                ca.strideF = np.strideF;
            } else {
                ca.ob = (int64_t)cp.Ho * cp.Wo * cp.Co;
                ca.orow = cp.Wo * cp.Co;
                ca.opix = cp.Co;
                ca.och = 1;
            }
            const double M = (double)e->Bl * cp.Ho * cp.Wo;
            KStep k;
            k.name = "conv_fwd_c" + std::to_string(l + 1);
            k.flops = 2.0 * nstreams * M * cp.Co * cp.K;
            k.bytes = 4.0 * (nstreams * (Bl * (double)cp.Ci * cp.Hi * cp.Wi + M * cp.Co) + 2.0 * cp.Co * (cp.K + 1.0));
            const int epi = last ? CIG_EPI_FLAT : CIG_EPI_NHWC;
            k.run = [=](hipStream_t s) { return launch_conv_ig(ca, epi, s); };
            ks.push_back(k);
        }
    }
    // micro-CNN plan: conv weights of the step in the kernels' layouts, then ONE launch for every
    // conv of every stream (micro.hip)
    MicroConv mconv[MICRO_MAX_CONV];
    if (NC && e->micro) {
        micro_geom(np, mconv);
        int x0 = 0, zero = 0;
        micro_fwd_layout(mconv, NC, e->micro_S, &x0, &zero);
        ConvPermArgs pa;
        memset(&pa, 0, sizeof(pa));
        double pbytes = 0;
        for (int l = 1; l < NC; l++) {   // conv 1 reads the torch layout directly
            const ConvPlan& cp = np.conv[l];
            pa.job[pa.njobs++] = ConvPermJob{params + cp.off, at<float>(e, e->ws_wperm0[l]), cp.Co, cp.Ci, 9, 0};
            pa.job[pa.njobs++] = ConvPermJob{tparams + cp.off, at<float>(e, e->ws_wperm1[l]), cp.Co, cp.Ci, 9, 0};
            pa.job[pa.njobs++] = ConvPermJob{params + cp.off, at<float>(e, e->ws_wpermT[l]), cp.Co, cp.Ci, 9, 1};
            mconv[l].wp[0] = at<float>(e, e->ws_wperm0[l]);
            mconv[l].wp[1] = at<float>(e, e->ws_wperm1[l]);
            mconv[l].wT = at<float>(e, e->ws_wpermT[l]);
            pbytes += 8.0 * cp.Co * cp.K * 3;
        }
        for (int l = 0; l < NC; l++) {
            mconv[l].hc = l + 1 < NC ? at<float>(e, e->ws_Hc[l]) : nullptr;
            mconv[l].dz = at<float>(e, e->ws_dZc[l]);
        }
        {
            KStep k;
            k.name = "conv_perm";
            k.bytes = pbytes;
            // eager: only while the copies are stale (the last step's Adam pass wrote them otherwise);
            // a captured graph always holds the launch (its replays may follow any update)
            k.run = [=](hipStream_t s) {
                hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                DQNX_HIP_CHECK(hipStreamIsCapturing(s, &cs));
                if (!e->perm_dirty && cs == hipStreamCaptureStatusNone) return (int)DQNX_OK;
                return launch_conv_perm(pa, s);
            };
            ks.push_back(k);
        }
        MicroFwdArgs ma;
        memset(&ma, 0, sizeof(ma));
        for (int l = 0; l < NC; l++) ma.c[l] = mconv[l];
        ma.nc = NC;
        ma.Bl = e->Bl;
        ma.S = e->micro_S;
        ma.groups = (e->Bl + ma.S - 1) / ma.S;
        int z = 0;
        for (int st = 0; st < 3; st++) {
            if (st == 1 && !dbl) continue;
            ma.stream_of[z] = st;
            ma.F[z] = at<float>(e, e->ws_F) + (int64_t)st * e->Bl * np.strideF;
            z++;
        }
        ma.nstreams = z;
        ma.params = params;
        ma.tparams = tparams;
        ma.ring_obs = ring_obs;
        ma.ring_next = ring_next;
        ma.ring_stride = e->stride;
        ma.macro_len = np.macro_len;
        ma.phys = phys;
        ma.strideF = np.strideF;
        const ConvPlan& cl = np.conv[NC - 1];
        ma.flat_cols = cl.Co * cl.Ho * cl.Wo;
        ma.x0 = x0;
        ma.zero = zero;
        ma.lds_floats = e->micro_lds;
        if (key & KEY_SAMPLE_NEXT) {   // + the next step's minibatch into the staging slot (in-launch prefetch)
            ma.samp_on = 1;
            ma.samp = uniform_sample_args(e, at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]) + (size_t)e->Bg,
                                          at<int32_t>(e, e->ws_phys) + (size_t)e->Bl);
            ma.samp.stamps = nullptr;
        }
#ifdef DQNX_STAMPS
        ma.stamps = at<int64_t>(e, e->ws_stamps);
#endif
        double flops = 0, bytes = 0;
        for (int l = 0; l < NC; l++) {
            const ConvPlan& cp = np.conv[l];
            flops += 2.0 * nstreams * Bl * cp.Ho * cp.Wo * (double)cp.Co * cp.K;
            bytes += 4.0 * 2.0 * (cp.Co * (double)cp.K + cp.Co) + (l + 1 < NC ? 4.0 * Bl * cp.Ho * cp.Wo * cp.Co : 0.0);
        }
        bytes += 4.0 * nstreams * Bl * (np.conv[0].Ci * np.conv[0].Hi * np.conv[0].Wi + np.strideF);
        KStep k;
        k.name = ma.samp_on ? "micro_fwd+sample" : "micro_fwd";
        k.flops = flops;
        k.bytes = bytes;
        k.run = [=](hipStream_t s) { return launch_micro_fwd(ma, s); };
        ks.push_back(k);
    }
    if (!e->conv_ig && !e->micro) {
    // 2a. two-stream micro CNN (R:env/dqn_config.py:92-101, forward :126-133): im2col + MFMA GEMM
    for (int l = 0; l < NC; l++) {
        const ConvPlan cp = np.conv[l];
        const int M = e->Bl * cp.Ho * cp.Wo;
        Im2colArgs ia;
        memset(&ia, 0, sizeof(ia));
        FwdArgs fa;
        memset(&fa, 0, sizeof(fa));
        fa.M = M;
        fa.N = cp.Co;
        fa.K = cp.K;
        fa.ldc = cp.Co;
        int np_ = 0;
        for (int st = 0; st < 3; st++) {
            if (st == 1 && !dbl) continue;
            float* col = at<float>(e, e->ws_col[l]) + (int64_t)st * M * cp.Kstride;
            if (l == 0) {
                ia.ring[np_] = st == 0 ? ring_obs : ring_next;
            } else {
                ia.src[np_] = at<float>(e, e->ws_Hc[l - 1]) + (int64_t)st * e->Bl * cp.Hi * cp.Wi * cp.Ci;
            }
            ia.col[np_] = col;
            FwdProblem& p = fa.p[np_++];
            p.W = (st == 2 ? tparams : params) + cp.off;
            p.bias = p.W + (int64_t)cp.Co * cp.K;
            p.C = at<float>(e, e->ws_Hc[l]) + (int64_t)st * M * cp.Co;
            p.A = col;
            p.lda = cp.Kstride;
        }
        ia.nstreams = np_;
        ia.phys = phys;
        ia.ring_stride = e->stride;
        ia.ring_off = np.macro_len;
        ia.Ci = cp.Ci; ia.Hi = cp.Hi; ia.Wi = cp.Wi; ia.Ho = cp.Ho; ia.Wo = cp.Wo;
        ia.kh = cp.kh; ia.kw = cp.kw; ia.sh = cp.sh; ia.sw = cp.sw; ia.ph = cp.ph; ia.pw = cp.pw;
        ia.K = cp.K; ia.Kstride = cp.Kstride; ia.M = M;
        {
            KStep k;
            k.name = "im2col_c" + std::to_string(l + 1);
            // algorithmic: write the column matrix once, read the source image once
            k.bytes = 4.0 * nstreams * ((double)M * cp.Kstride + (double)Bl * cp.Ci * cp.Hi * cp.Wi);
            k.run = [=](hipStream_t s) { return launch_im2col(ia, s); };
            ks.push_back(k);
        }
        KStep k;
        k.name = "conv_fwd_c" + std::to_string(l + 1);
        k.flops = 2.0 * nstreams * (double)M * cp.Co * cp.K;
        k.bytes = 4.0 * (nstreams * (double)M * (cp.Kstride + cp.Co) + 2.0 * cp.Co * (cp.K + 1.0));
        const bool vecb = (cp.K % 4) == 0;
        const int nps = np_;
        // conv GEMMs with enough rows to fill the chip with 128-row tiles (weight slab loaded once per
        // 128 rows): (4,84,84) B=256 convs 1-3 1538/1849/717 -> 408/1228/546 us; (2,27,5) conv 1
        // 31.6 -> 12.8 us, conv 3 (126 tiles) was slower on 128-row tiles and stays on 16 x 64
        if (fwd_big_mode() && (int64_t)((fa.M + 127) / 128) * np_ >= 256) {
            fa.ksplit = 1;
            k.run = [=](hipStream_t s) { return launch_linear_fwd_big(fa, nps, act, vecb, s); };
        } else {
            k.run = [=](hipStream_t s) { return launch_linear_fwd(fa, nps, act, vecb, s); };
        }
        ks.push_back(k);
    }
    if (NC) {   // 2b. cat(flatten_CHW(conv), macro) (R:env/dqn_config.py:135-138)
        const ConvPlan cl = np.conv[NC - 1];
        FlattenArgs fl;
        memset(&fl, 0, sizeof(fl));
        int z = 0;
        for (int st = 0; st < 3; st++) {
            if (st == 1 && !dbl) continue;
            fl.Hc[z] = at<float>(e, e->ws_Hc[NC - 1]) + (int64_t)st * e->Bl * cl.Ho * cl.Wo * cl.Co;
            fl.ring[z] = st == 0 ? ring_obs : ring_next;
            fl.F[z] = at<float>(e, e->ws_F) + (int64_t)st * e->Bl * np.strideF;
            z++;
        }
        fl.nstreams = z;
        fl.phys = phys;
        fl.ring_stride = e->stride;
        fl.macro_len = np.macro_len;
        fl.C = cl.Co; fl.Ho = cl.Ho; fl.Wo = cl.Wo;
        fl.Bl = e->Bl;
        fl.strideF = np.strideF;
        KStep k;
        k.name = "flatten_concat";
        k.bytes = 4.0 * nstreams * Bl * 2.0 * np.strideF;
        k.run = [=](hipStream_t s) { return launch_flatten_concat(fl, s); };
        ks.push_back(k);
    }
    }
    for (int l = 0; l < L; l++) {
        const LayerPlan lp = np.dense[l];
        FwdArgs fa;
        memset(&fa, 0, sizeof(fa));
        fa.M = e->Bl;
        fa.N = lp.out;
        fa.K = lp.in;
        fa.ldc = lp.out;
        float* H = at<float>(e, e->ws_H[l]);
        int np_ = 0;
        for (int st = 0; st < 3; st++) {
            if (st == 1 && !dbl) continue;
            FwdProblem& p = fa.p[np_++];
            const bool tgt = st == 2;
            p.W = (tgt ? tparams : params) + lp.off;
            p.bias = p.W + (int64_t)lp.out * lp.in;
            p.C = H + (int64_t)st * e->Bl * lp.out;
            if (l == 0 && NC) {
                p.A = at<float>(e, e->ws_F) + (int64_t)st * e->Bl * np.strideF;
                p.lda = np.strideF;
            } else if (l == 0) {
                p.A = at<float>(e, e->off[st == 0 ? DQNX_BUF_RING_OBS : DQNX_BUF_RING_NEXT_OBS]);
                p.lda = e->stride;
                p.phys = phys;
                p.xcopy = (st == 0) ? at<float>(e, e->ws_xobs) : nullptr;
            } else {
                const int w = np.dense[l - 1].out;
                p.A = at<float>(e, e->ws_H[l - 1]) + (int64_t)st * e->Bl * w;
                p.lda = w;
            }
        }
        KStep k;
        k.name = "linear_fwd_l" + std::to_string(l + 1);
        k.flops = 2.0 * nstreams * Bl * lp.out * lp.in;
        // unique bytes: input rows, weights (online + target), outputs (+ layer-1 row copy)
        k.bytes = 4.0 * (nstreams * Bl * lp.in + 2.0 * (lp.out * (double)lp.in + lp.out) + nstreams * Bl * lp.out
                         + (l == 0 && !NC ? Bl * lp.in : 0.0));
        const bool vecb = (lp.in % 4) == 0;
        // large-K layers that read dense rows (not the ring gather): 128x128 tiles + split-K into
        // the layer's dW partial slabs (free until the backward), then an ordered reduce
        const uint64_t part_floats = (uint64_t)e->slices[l] * ((uint64_t)lp.out * lp.in + lp.out);
        int kchunk = 0;
        const int ksplit = fwd_big_ksplit(e->Bl, lp.out, lp.in, np_, (int64_t)part_floats, &kchunk);
        if (l == 0 && NC && e->f1_ksplit) {
            fa.ksplit = e->f1_ksplit;
            fa.kchunk = e->f1_kchunk;
            fa.partial = at<float>(e, e->ws_fpart);
#ifdef DQNX_STAMPS
            fa.stamps = at<int64_t>(e, e->ws_stamps);
#endif
            k.run = [=](hipStream_t s) { return launch_linear_fwd_split(fa, np_, act, vecb, s); };
            ks.push_back(k);
            KStep kr;
            kr.name = k.name + "_reduce";
            kr.bytes = 4.0 * ((double)fa.ksplit + 1) * np_ * Bl * lp.out;
            kr.run = [=](hipStream_t s) { return launch_linear_fwd_reduce(fa, np_, act, s); };
            ks.push_back(kr);
            continue;
        }
        const int big_min_k = tuning_knob("DQNX_FWD_BIG_MINK", 8192);
        if ((l > 0 || NC) && lp.in >= big_min_k && e->Bl >= 64 && fwd_big_mode() &&
            (uint64_t)ksplit * np_ * e->Bl * lp.out <= part_floats) {
            fa.ksplit = ksplit;
            fa.kchunk = kchunk;
            fa.partial = at<float>(e, e->ws_part[l]);
            k.run = [=](hipStream_t s) { return launch_linear_fwd_big(fa, np_, act, vecb, s); };
            ks.push_back(k);
            KStep kr;
            kr.name = k.name + "_reduce";
            kr.bytes = 4.0 * ((double)ksplit + 1) * np_ * Bl * lp.out;
            kr.run = [=](hipStream_t s) { return launch_linear_fwd_reduce(fa, np_, act, s); };
            ks.push_back(kr);
            continue;
        }
        k.run = [=](hipStream_t s) { return launch_linear_fwd(fa, np_, act, vecb, s); };
        ks.push_back(k);
    }

    // 3. head + TD + Huber + head backward (R:dqn/agent.py:209-221, R:dqn/network.py:90-96)
    {
        HeadArgs ha;
        memset(&ha, 0, sizeof(ha));
        ha.Bl = e->Bl;
        ha.F = np.F;
        ha.A = A;
        ha.NH = np.NH;
        ha.head_kind = c.net.head;
        ha.algo = c.algo;
        ha.head_params = (int)np.head_params;
        ha.inv_bg = (float)(1.0 / (double)e->Bg);
        ha.gamma = (float)c.gamma;
        ha.H = at<float>(e, e->ws_H[L - 1]);
        ha.Wo = params + np.head_off;
        ha.Wt = tparams + np.head_off;
        ha.phys = phys;
        ha.act = at<int32_t>(e, e->off[DQNX_BUF_RING_ACT]);
        ha.rew = at<float>(e, e->off[DQNX_BUF_RING_REW]);
        ha.done = at<float>(e, e->off[DQNX_BUF_RING_DONE]);
        ha.isw = (c.algo == DQNX_ALGO_PER_DOUBLE) ? at<float>(e, e->off[DQNX_BUF_IS_WEIGHTS]) + e->shard_begin : nullptr;
        ha.abs_td_out = (c.algo == DQNX_ALGO_PER_DOUBLE) ? at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]) + e->shard_begin
                                                         : nullptr;
        ha.Q = at<float>(e, e->off[DQNX_BUF_Q]);
        ha.td = at<float>(e, e->off[DQNX_BUF_TD]);
        ha.dZ = at<float>(e, e->ws_dZ[L - 1]);
        ha.dhead = at<float>(e, e->ws_dhead);
        if (L >= 2 && e->bwd_plan == 1) {
            ha.W_last = params + np.dense[L - 1].off;
            ha.Hprev = at<float>(e, e->ws_H[L - 2]);
            ha.dZprev = at<float>(e, e->ws_dZ[L - 2]);
            ha.in_prev = np.dense[L - 1].in;
        }
        ha.loss_partial = at<float>(e, e->ws_loss_part);
        ha.ctrl = ctrl;
        ha.beta1 = (float)c.beta1;
        ha.beta2 = (float)c.beta2;
        ha.lr = (float)c.lr;
        ha.ab = adam_bias_args(e);
        ha.stamps = at<int64_t>(e, e->ws_stamps);
        KStep k;
        k.name = "head_td_loss";
        const double F = np.F, NH = np.NH;
        k.flops = 2.0 * Bl * NH * F * (nstreams + 2.0);
        k.bytes = 4.0 * (nstreams * Bl * F + 2.0 * np.head_params + Bl * F + e->tiles * (double)np.head_params
                         + 3.0 * Bl * A + 6.0 * Bl);
        k.run = [=](hipStream_t s) { return launch_head(ha, act, s); };
        ks.push_back(k);
    }

    // 3b. PER priorities (R:dqn/agent.py:263-265): single GPU here; under DP after the
    //     all-gather of |delta|, in dqnx_apply_grads
    if (c.algo == DQNX_ALGO_PER_DOUBLE && !(flags & DQNX_STEP_GRADS_ONLY)) {
        KStep k;
        k.name = "per_update";
        k.bytes = Bg_ * (4.0 + 4.0 + 8.0 * 2.0 * 21.0);
        k.run = [=](hipStream_t s) { return enqueue_per_update(e, idx, s); };
        ks.push_back(k);
    }

    if (e->bwd_plan == 0) {
    // 4. backward levels L..1: dX of the level below + split-K dW of this level
    //    (level L also computes the head-weight gradient from the head kernel's dHead)
    for (int l = L - 1; l >= 0; l--) {
        const LayerPlan lp = np.dense[l];
        BwdArgs ba;
        memset(&ba, 0, sizeof(ba));
        ba.dZ = at<float>(e, e->ws_dZ[l]);
        ba.Bl = e->Bl;
        ba.in = lp.in;
        ba.out = lp.out;
        ba.W = params + lp.off;
        ba.kslice = e->kslice[l];
        ba.dw_slices = e->slices[l];
        DwProblem& d = ba.dw[ba.ndw++];
        d.dZ = ba.dZ;
        d.ldz = lp.out;
        d.in = lp.in;
        d.out = lp.out;
        d.head_kind = -1;
        if (l > 0) {
            ba.Hprev = at<float>(e, e->ws_H[l - 1]);   // stream 0 rows
            ba.ldh = lp.in;
            ba.dZprev = at<float>(e, e->ws_dZ[l - 1]);
            d.X = ba.Hprev;
            d.ldx = lp.in;
        } else if (NC) {   // dense input F = cat(conv features, macro): dF, masked by the conv's ELU
            ba.Hprev = at<float>(e, e->ws_F);
            ba.ldh = np.strideF;
            ba.dZprev = at<float>(e, e->ws_dF);
            d.X = ba.Hprev;
            d.ldx = np.strideF;
        } else {
            d.X = at<float>(e, e->ws_xobs);
            d.ldx = e->stride;
        }
        d.partial = at<float>(e, e->ws_part[l]);
        d.pstride = (int64_t)lp.out * lp.in + lp.out;
        const bool dx = l > 0 || NC;
        double flops = 2.0 * Bl * lp.out * (lp.in + 1.0) + (dx ? 2.0 * Bl * lp.out * lp.in : 0.0);
        double bytes = 4.0 * (Bl * lp.out + Bl * lp.in + ba.dw_slices * (lp.out * (lp.in + 1.0))
                              + (dx ? lp.out * (double)lp.in + 2.0 * Bl * lp.in : 0.0));
        // very large levels (the (4,84,84) variant's 56,462 -> 512 dense 1): 64 x 64 tiles, a quarter of
        // the 32 x 32 workgroups with four times the MFMAs per operand pass: its backward level 434 ->
        // 351 us; the HEAD net's 1358 -> 512 keeps 32 x 32 (16.1 us; 25.9 with 64 x 64: ~1 workgroup per
        // CU, latency-bound).  DQNX_BWD_TS=32 / 64 forces the edge
        const int bts = route_knob("DQNX_BWD_TS", 0);
        if (bts == 64 || (bts == 0 && (int64_t)(lp.in + 1) * lp.out >= ((int64_t)4 << 20) && e->Bl >= 64)) ba.ts = 64;
        if (l == L - 1) {   // head weight gradient: dHead^T [H_L | 1]
            DwProblem& h = ba.dw[ba.ndw++];
            h.dZ = at<float>(e, e->ws_dhead);
            h.ldz = 16;
            h.X = at<float>(e, e->ws_H[L - 1]);
            h.ldx = np.F;
            h.in = np.F;
            h.out = np.NH;
            h.partial = at<float>(e, e->ws_head_part);
            h.pstride = head_pstride(np);
            h.head_kind = c.net.head;
            h.A = A;
            flops += 2.0 * Bl * np.NH * (np.F + 1.0);
            bytes += 4.0 * (16.0 * Bl + ba.dw_slices * (double)np.head_params);
        }
        bwd_level_grid(ba);
        KStep k;
        k.name = "linear_bwd_l" + std::to_string(l + 1);
        k.flops = flops;
        k.bytes = bytes;
        k.run = [=](hipStream_t s) { return launch_bwd_level(ba, act, s); };
        ks.push_back(k);
    }

    // 4b'. implicit-GEMM conv backward, last conv first: dW (+ db) slabs, then the data gradient
    //      with the previous conv's activation derivative in its epilogue
    if (NC && e->conv_ig) {
        for (int l = NC - 1; l >= 0; l--) {
            const ConvPlan cp = np.conv[l];
            const bool last = l == NC - 1;
            const double M = (double)e->Bl * cp.Ho * cp.Wo;
            // this conv's dZ (NHWC): for the last conv dF (CHW-flatten rows, masked by the dense
            // layer's dx role) transposed, else what the next conv's data gradient wrote
            if (last) {
                UnflattenArgs ua;
                ua.dF = at<float>(e, e->ws_dF);
                ua.ldf = np.dense[0].in;
                ua.dZ = at<float>(e, e->ws_dZc[l]);
                ua.Bl = e->Bl;
                ua.C = cp.Co; ua.Ho = cp.Ho; ua.Wo = cp.Wo;
                KStep k;
                k.name = "unflatten";
                k.bytes = 8.0 * M * cp.Co;
                k.run = [=](hipStream_t s) { return launch_unflatten_tiled(ua, s); };
                ks.push_back(k);
            }
            const float* dZ = at<float>(e, e->ws_dZc[l]);
            const int64_t dzb = (int64_t)cp.Ho * cp.Wo * cp.Co;
            const int dzp = cp.Co, dzc = 1;
            ConvDwIgArgs d;
            cig_dw_geom(cp, e->Bl, l == 0, d);
            CigSource& X = d.X;
            X.H = cp.Hi; X.W = cp.Wi; X.C = cp.Ci;
            if (l == 0) {
                X.base[0] = ring_obs;
                X.phys = phys;
                X.bstride = e->stride;
                X.off = np.macro_len;
                X.pstride = 1;
                X.cstride = cp.Hi * cp.Wi;
            } else {
                X.base[0] = at<float>(e, e->ws_Hc[l - 1]);   // stream 0
                X.bstride = (int64_t)cp.Hi * cp.Wi * cp.Ci;
                X.pstride = cp.Ci;
                X.cstride = 1;
            }
            d.dZ = dZ;
            d.dzb = dzb;
            d.dzp = dzp;
            d.dzc = dzc;
            d.partial = at<float>(e, e->ws_cpart[l]);
            {
                KStep k;
                k.name = "conv_dw_c" + std::to_string(l + 1);
                k.flops = 2.0 * M * cp.Co * (cp.K + 1.0);
                k.bytes = 4.0 * (M * cp.Co + Bl * (double)cp.Ci * cp.Hi * cp.Wi + (double)d.slices * d.pstride);
                k.run = [=](hipStream_t s) { return launch_conv_dw_ig(d, s); };
                ks.push_back(k);
            }
            if (l == 0) continue;
            const ConvPlan pp = np.conv[l - 1];
            ConvIgArgs ca;
            cig_dx_geom(cp, e->Bl, last, ca);
            ca.act = act;
            ca.src.base[0] = dZ;
            ca.src.bstride = dzb;
            ca.src.pstride = dzp;
            ca.src.cstride = dzc;
            ca.W[0] = at<float>(e, e->ws_wpermT[l]);
            ca.out[0] = at<float>(e, e->ws_dZc[l - 1]);
            ca.Hprev = at<float>(e, e->ws_Hc[l - 1]);   // stream 0
            ca.ob = (int64_t)pp.Ho * pp.Wo * pp.Co;
            ca.orow = pp.Wo * pp.Co;
            ca.opix = pp.Co;
            ca.och = 1;
            KStep k;
            k.name = "conv_dx_c" + std::to_string(l + 1);
            k.flops = 2.0 * M * cp.Co * cp.K;
            k.bytes = 4.0 * (M * cp.Co + 2.0 * Bl * pp.Ho * pp.Wo * pp.Co + (double)cp.Co * cp.K);
            k.run = [=](hipStream_t s) { return launch_conv_ig(ca, CIG_EPI_DX, s); };
            ks.push_back(k);
        }
    }
    // 4b''. micro-CNN backward: data gradients of every conv (one launch, stream 0), then every
    //       conv's weight gradient as split-K slabs (one launch)
    if (NC && e->micro) {
        MicroDxArgs xa;
        memset(&xa, 0, sizeof(xa));
        for (int l = 0; l < NC; l++) xa.c[l] = mconv[l];
        xa.nc = NC;
        xa.Bl = e->Bl;
        xa.S = e->micro_dx_S;
        xa.groups = (e->Bl + xa.S - 1) / xa.S;
        xa.dF = at<float>(e, e->ws_dF);
        xa.ldf = np.dense[0].in;
        micro_dx_layout(mconv, NC, xa.S, xa.lds_d, &xa.zero);
        micro_dx_waves(xa);
        xa.lds_floats = e->micro_dx_lds;
#ifdef DQNX_STAMPS
        xa.stamps = at<int64_t>(e, e->ws_stamps);
#endif
        double xf = 0, xb = 0;
        for (int l = 1; l < NC; l++) {
            const ConvPlan& cp = np.conv[l];
            xf += 2.0 * Bl * cp.Ho * cp.Wo * (double)cp.Co * cp.K;
            xb += 4.0 * (Bl * cp.Ho * cp.Wo * (double)cp.Co + 2.0 * Bl * cp.Hi * cp.Wi * cp.Ci + cp.Co * (double)cp.K);
        }
        KStep kx;
        kx.name = "micro_dx";
        kx.flops = xf;
        kx.bytes = xb;
        kx.run = [=](hipStream_t s) { return launch_micro_dx(xa, s); };
        ks.push_back(kx);
        MicroDwArgs da = e->micro_dw;
        da.ring_obs = ring_obs;
        da.stamps = at<int64_t>(e, e->ws_stamps);
        da.err = &ctrl_of(e)->error;
        da.phys = phys;
        da.ring_stride = e->stride;
        da.macro_len = np.macro_len;
        double wf = 0, wb = 0;
        for (int l = 0; l < NC; l++) {
            const ConvPlan& cp = np.conv[l];
            MicroDwLayer& L = da.L[l];
            L.D = at<float>(e, e->ws_dZc[l]);
            L.X = l > 0 ? at<float>(e, e->ws_Hc[l - 1]) : nullptr;
            L.partial = at<float>(e, e->ws_cpart[l]);
            wf += 2.0 * Bl * cp.Ho * cp.Wo * (double)cp.Co * (cp.K + 1.0);
            wb += 4.0 * (Bl * cp.Ho * cp.Wo * (double)cp.Co + Bl * (double)cp.Ci * cp.Hi * cp.Wi + (double)L.slices * L.pstride);
        }
        KStep kw;
        kw.name = "micro_dw";
        kw.flops = wf;
        kw.bytes = wb;
        kw.run = [=](hipStream_t s) { return launch_micro_dw(da, s); };
        ks.push_back(kw);
    }
    // 4b. micro CNN backward: unflatten dF, then per conv (last first) dW + dX columns, col2im
    if (NC && !e->conv_ig && !e->micro) {
        {
            const ConvPlan cl = np.conv[NC - 1];
            UnflattenArgs ua;
            ua.dF = at<float>(e, e->ws_dF);
            ua.ldf = np.dense[0].in;
            ua.dZ = at<float>(e, e->ws_dZc[NC - 1]);
            ua.Bl = e->Bl;
            ua.C = cl.Co; ua.Ho = cl.Ho; ua.Wo = cl.Wo;
            KStep k;
            k.name = "unflatten";
            k.bytes = 8.0 * Bl * cl.Co * cl.Ho * cl.Wo;
            k.run = [=](hipStream_t s) { return launch_unflatten(ua, s); };
            ks.push_back(k);
        }
        for (int l = NC - 1; l >= 0; l--) {
            const ConvPlan cp = np.conv[l];
            const int M = e->Bl * cp.Ho * cp.Wo;
            BwdArgs ba;
            memset(&ba, 0, sizeof(ba));
            ba.dZ = at<float>(e, e->ws_dZc[l]);
            ba.Bl = M;
            ba.in = cp.K;
            ba.out = cp.Co;
            ba.W = params + cp.off;
            ba.kslice = e->ckslice[l];
            ba.dw_slices = e->cslices[l];
            // dCol = dZ W (no mask here: col2im applies the previous conv's ELU'); on 128x64 tiles in
            // its own launch when that fills the chip, else as the dx role of the level
            const bool dx_big = l > 0 && fwd_big_mode() && conv_dx_big_tiles(M, cp.K) >= 256;
            BwdArgs bdx;
            if (l > 0) {
                ba.Hprev = nullptr;
                ba.dZprev = at<float>(e, e->ws_dcol);
                bdx = ba;
                if (dx_big) ba.dZprev = nullptr;
            }
            DwProblem& d = ba.dw[ba.ndw++];
            d.dZ = ba.dZ;
            d.ldz = cp.Co;
            d.X = at<float>(e, e->ws_col[l]);   // stream 0 columns
            d.ldx = cp.Kstride;
            d.in = cp.K;
            d.out = cp.Co;
            d.partial = at<float>(e, e->ws_cpart[l]);
            d.pstride = (int64_t)cp.Co * cp.K + cp.Co;
            d.head_kind = -1;
            bwd_level_grid(ba);
            KStep k;
            k.name = "conv_bwd_c" + std::to_string(l + 1);
            k.flops = 2.0 * M * cp.Co * (cp.K + 1.0) + (l > 0 ? 2.0 * M * cp.Co * (double)cp.K : 0.0);
            k.bytes = 4.0 * ((double)M * (cp.Co + cp.Kstride) + ba.dw_slices * (double)d.pstride
                             + (l > 0 ? (double)M * cp.K + cp.Co * (double)cp.K : 0.0));
            const bool dw_big = conv_dw_big(M, cp.K);
            if (dw_big) {   // dx role (if any) runs as conv_dx_c* or stays in a level launch
                BwdArgs bw = ba;
                if (ba.dZprev) {    // small dx: keep it in its own level launch without the dW role
                    BwdArgs bl = ba;
                    bl.ndw = 0;
                    bwd_level_grid(bl);
                    KStep kl;
                    kl.name = "conv_dxs_c" + std::to_string(l + 1);
                    kl.flops = 2.0 * M * cp.Co * (double)cp.K;
                    kl.bytes = 4.0 * ((double)M * cp.K + (double)M * cp.Co + cp.Co * (double)cp.K);
                    kl.run = [=](hipStream_t s) { return launch_bwd_level(bl, act, s); };
                    ks.push_back(kl);
                }
                k.run = [=](hipStream_t s) { return launch_conv_dw_big(bw, s); };
            } else {
                k.run = [=](hipStream_t s) { return launch_bwd_level(ba, act, s); };
            }
            if (dx_big || dw_big) {   // the conv_bwd launch is the dW GEMM alone
                k.flops = 2.0 * M * cp.Co * (cp.K + 1.0);
                k.bytes = 4.0 * ((double)M * (cp.Co + cp.Kstride) + ba.dw_slices * (double)d.pstride);
            }
            ks.push_back(k);
            if (dx_big) {
                KStep kx;
                kx.name = "conv_dx_c" + std::to_string(l + 1);
                kx.flops = 2.0 * M * cp.Co * (double)cp.K;
                kx.bytes = 4.0 * ((double)M * cp.K + (double)M * cp.Co + cp.Co * (double)cp.K);
                kx.run = [=](hipStream_t s) { return launch_conv_dx_big(bdx, s); };
                ks.push_back(kx);
            }
            if (l > 0) {
                const ConvPlan pp = np.conv[l - 1];
                Col2imArgs ca;
                ca.dcol = at<float>(e, e->ws_dcol);
                ca.ldcol = cp.K;
                ca.Hprev = at<float>(e, e->ws_Hc[l - 1]);      // stream 0
                ca.dZprev = at<float>(e, e->ws_dZc[l - 1]);
                ca.Bl = e->Bl;
                ca.Ci = cp.Ci; ca.Hi = cp.Hi; ca.Wi = cp.Wi; ca.Ho = cp.Ho; ca.Wo = cp.Wo;
                ca.kh = cp.kh; ca.kw = cp.kw; ca.sh = cp.sh; ca.sw = cp.sw; ca.ph = cp.ph; ca.pw = cp.pw;
                KStep k2;
                k2.name = "col2im_c" + std::to_string(l + 1);
                k2.bytes = 4.0 * ((double)M * cp.K + 2.0 * Bl * pp.Ho * pp.Wo * pp.Co);
                k2.run = [=](hipStream_t s) { return launch_col2im(ca, act, s); };
                ks.push_back(k2);
            }
        }
    }

    // 5. gradient reduction + Adam (+ soft update); with the in-launch prefetch its extra workgroup
    //    copies the staged minibatch over the compute slot (every reader of slot 0 ran before)
    if (key & KEY_SAMPLE_NEXT) {
        AdamArgs aa;
        KStep k = adam_kstep(e, flags, &aa);
        aa.pf_idx_src = at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]) + (size_t)e->Bg;
        aa.pf_idx_dst = idx;
        aa.pf_nidx = e->Bg;
        aa.pf_phys_src = at<int32_t>(e, e->ws_phys) + (size_t)e->Bl;
        aa.pf_phys_dst = phys;
        aa.pf_nphys = e->Bl;
        aa.mtc = nullptr;   // the forward's sampler body draws from the MT state itself
        aa.mtc_blocks = 0;
        k.run = adam_run(e, aa);
        ks.push_back(k);
    } else {
        ks.push_back(adam_kstep(e, flags));
    }
    } else {
    // 4. dZ of levels below L-1 (deeper MLPs only; the head kernel produced dZ_L and dZ_{L-1})
    for (int l = L - 2; l >= 1; l--) {
        const LayerPlan lp = np.dense[l];
        BwdArgs ba;
        memset(&ba, 0, sizeof(ba));
        ba.dZ = at<float>(e, e->ws_dZ[l]);
        ba.Bl = e->Bl;
        ba.in = lp.in;
        ba.out = lp.out;
        ba.W = params + lp.off;
        ba.Hprev = at<float>(e, e->ws_H[l - 1]);
        ba.ldh = lp.in;
        ba.dZprev = at<float>(e, e->ws_dZ[l - 1]);
        ba.ndw = 0;
        ba.dw_slices = 1;
        ba.kslice = e->Bl;
        bwd_level_grid(ba);
        KStep k;
        k.name = "linear_dx_l" + std::to_string(l + 1);
        k.flops = 2.0 * Bl * lp.out * lp.in;
        k.bytes = 4.0 * (Bl * lp.out + lp.out * (double)lp.in + 2.0 * Bl * lp.in);
        k.run = [=](hipStream_t s) { return launch_bwd_level(ba, act, s); };
        ks.push_back(k);
    }

    // 5. all weight gradients (full minibatch per tile) + Adam (+ soft update) in one launch
    {
        DwAdamArgs da;
        memset(&da, 0, sizeof(da));
        double flops = 0, bytes = 0;
        for (int l = 0; l < L; l++) {
            const LayerPlan lp = np.dense[l];
            DwAdamProblem& d = da.pr[da.npr++];
            d.dZ = at<float>(e, e->ws_dZ[l]);
            d.ldz = lp.out;
            if (l > 0) {
                d.X = at<float>(e, e->ws_H[l - 1]);   // stream 0 rows
                d.ldx = lp.in;
            } else {
                d.X = at<float>(e, e->ws_xobs);
                d.ldx = e->stride;
            }
            d.in = lp.in;
            d.out = lp.out;
            d.poff = lp.off;
            d.head_kind = -1;
            flops += 2.0 * Bl * lp.out * (lp.in + 1.0);
            bytes += 4.0 * Bl * (lp.out + lp.in);
        }
        {
            DwAdamProblem& d = da.pr[da.npr++];
            d.dZ = at<float>(e, e->ws_dhead);
            d.ldz = 16;
            d.X = at<float>(e, e->ws_H[L - 1]);
            d.ldx = np.F;
            d.in = np.F;
            d.out = np.NH;
            d.poff = np.head_off;
            d.head_kind = c.net.head;
            d.A = A;
            flops += 2.0 * Bl * np.NH * (np.F + 1.0);
            bytes += 4.0 * Bl * (16.0 + np.F);
        }
        dw_adam_grid(da);
        da.Bl = e->Bl;
        da.mode = (flags & DQNX_STEP_GRADS_ONLY) ? 0 : 1;
        da.soft = (flags & DQNX_STEP_SOFT_UPDATE) ? 1 : 0;
        da.n_params = np.P;
        da.p = params;
        da.m = at<float>(e, e->off[DQNX_BUF_ADAM_M]);
        da.v = at<float>(e, e->off[DQNX_BUF_ADAM_V]);
        da.grads = at<float>(e, e->off[DQNX_BUF_GRADS]);
        da.target = tparams;
        da.ctrl = ctrl;
        da.w1 = (float)(1.0 - c.beta1);          // Python: exp_avg.lerp_(grad, 1 - beta1)
        da.beta2 = (float)c.beta2;
        da.c2 = (float)(1.0 - c.beta2);
        da.eps = (float)c.adam_eps;
        da.tau = (float)(c.tau * c.n_env);
        da.one_minus_tau = (float)(1.0 - c.tau * c.n_env);
        da.adam_table = at<float>(e, e->ws_adam_tab);
        da.adam_table_len = kAdamTable;
        da.beta1d = c.beta1;
        da.beta2d = c.beta2;
        da.lrd = c.lr;
        da.loss_partial = at<float>(e, e->ws_loss_part);
        da.n_loss_partial = e->tiles;
        da.batch_global = e->Bg;
        const double P = (double)np.P;
        bytes += 4.0 * (P + (da.mode ? 6.0 * P + (da.soft ? 2.0 * P : 0.0) : 0.0));
        flops += da.mode ? 12.0 * P : 0.0;
        KStep k;
        k.name = da.mode ? "dw_adam" : "dw_grads";
        k.flops = flops;
        k.bytes = bytes;
        k.run = [=](hipStream_t s) { return launch_dw_adam(da, s); };
        ks.push_back(k);
    }
    }
    return ks;
}

int enqueue_range(const std::vector<KStep>& ks, int a, int b, hipStream_t s) {
    for (int i = a; i < b; i++) {
        int rc = ks[i].run(s);
        if (rc) return rc;
    }
    return DQNX_OK;
}

// dqnx_apply_grads on the fused plan: k_dw_adam16 in apply mode (mode 3: Adam from `grads`, no K
// loop) over every parameter tile, dense layers last-first then the head, writing the blocked copies
static DwAdam16Args apply_dw16_args(dqnx_engine* e, const AdamArgs& aa) {
    const dqnx_config& c = e->cfg;
    DwAdam16Args da;
    memset(&da, 0, sizeof(da));
    const NetPlan& np = e->np;
    const int L = (int)np.dense.size();
    da.rows16 = 2;
    int tiles = 0;
    for (int q = 0; q <= L; q++) {   // dense layers last-first, then the head (any tiling: elementwise)
        const int l = q < L ? L - 1 - q : -1;
        DwAdam16Layer& d = da.L[da.nl++];
        d.in = l >= 0 ? np.dense[l].in : np.F;
        d.out = l >= 0 ? np.dense[l].out : np.NH;
        d.poff = l >= 0 ? np.dense[l].off : np.head_off;
        d.head_kind = l >= 0 ? -1 : c.net.head;
        d.A = c.net.n_actions;
        d.ti = (d.in + 15) / 16;
        d.t0 = tiles;
        tiles += d.ti * ((d.out + 31) / 32);
        if (l >= 0) {
            d.fwd_online = at<float>(e, e->ws_wblk[0][l]);
            d.fwd_target = at<float>(e, e->ws_wblk[1][l]);
            d.chain = l >= 1 ? at<float>(e, e->ws_wblkT[l]) : nullptr;
            d.nch_fwd = e->fplan.kpad[l] / 16;
            d.nch_chain = np.dense[l].out / 16;
        }
        d.dZ = aa.grads;   // (no K loop: never read)
        d.X = aa.grads;
        d.ldz = d.ldx = 1;
    }
    da.tiles = tiles;
    da.Bl = 0;
    da.mode = 3;
    da.soft = aa.soft;
    da.n_params = np.P;
    da.p = aa.p;
    da.m = aa.m;
    da.v = aa.v;
    da.grads = aa.grads;
    da.target = aa.target;
    da.ctrl = aa.ctrl;
    da.w1 = aa.w1;
    da.beta2 = aa.beta2;
    da.c2 = aa.c2;
    da.eps = aa.eps;
    da.tau = aa.tau;
    da.one_minus_tau = aa.one_minus_tau;
    da.batch_global = e->Bg;
    da.stamps = at<int64_t>(e, e->ws_stamps);
    return da;
}

// The layers q of a k_dw_adam16 launch with bit q of `mask` set (a.L order), as a launch of their own:
// the same per-tile arithmetic, tiles renumbered.  `first`: this launch computes the loss (tile 0 of
// the gradient mode); `last`: it hosts the step's extra workgroups (PER, MT cache, staged minibatch).
static DwAdam16Args dw16_subset(const DwAdam16Args& a, uint32_t mask, bool first, bool last) {
    DwAdam16Args b = a;
    b.nl = 0;
    int tiles = 0;
    for (int q = 0; q < a.nl; q++) {
        const int nt = (q + 1 < a.nl ? a.L[q + 1].t0 : a.tiles) - a.L[q].t0;
        if (!((mask >> q) & 1u)) continue;
        DwAdam16Layer d = a.L[q];
        d.t0 = tiles;
        tiles += nt;
        b.L[b.nl++] = d;
    }
    b.tiles = tiles;
    if (!first) {
        b.loss_partial = nullptr;
        b.n_loss_partial = 0;
    }
    if (!last) {
        b.mtc = nullptr;
        b.mtc_blocks = 0;
        b.pf_nidx = b.pf_nphys = 0;
        b.pprop_wgs = 0;
        b.ptrack = 0;
    }
    return b;
}

int enqueue_apply(dqnx_engine* e, int flags, hipStream_t s) {
    const bool keep_blk = (flags & 0x200) != 0;   // (a prefetched minibatch is pending: no sampler launch next)
    const dqnx_config& c = e->cfg;
    // priorities from the all-gathered |delta| (DP); k_per_prop's workgroups ride in the Adam launch
    // below (DQNX_PER_FUSED=0: its own launch)
    PerUpdateArgs pua;
    memset(&pua, 0, sizeof(pua));
    const bool prop_in_adam = c.algo == DQNX_ALGO_PER_DOUBLE && !c.per_numpy121 && e->Bg <= PER_CHUNK &&
                              route_knob("DQNX_PER_FUSED", 1) != 0;
    if (prop_in_adam) {
        pua = per_update_args(e);
        pua.mode = 0;
        pua.n = e->Bg;
        pua.slots = at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]);
        pua.abs_td = at<float>(e, e->off[DQNX_BUF_PER_ABS_TD]);
        pua.skip = PER_SKIP_PROP;
        int rc = launch_per_update(pua, s);
        if (rc) return rc;
    } else if (c.algo == DQNX_ALGO_PER_DOUBLE) {
        int rc = enqueue_per_update(e, at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]), s);
        if (rc) return rc;
    }
    AdamArgs aa;
    memset(&aa, 0, sizeof(aa));
    aa.nseg = 0;
    aa.mode = 2;
    aa.soft = (flags & DQNX_STEP_SOFT_UPDATE) ? 1 : 0;
    aa.n_params = e->np.P;
    aa.p = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    aa.m = at<float>(e, e->off[DQNX_BUF_ADAM_M]);
    aa.v = at<float>(e, e->off[DQNX_BUF_ADAM_V]);
    aa.grads = at<float>(e, e->off[DQNX_BUF_GRADS]);
    aa.target = at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]);
    aa.ctrl = ctrl_of(e);
    aa.w1 = (float)(1.0 - c.beta1);          // Python: exp_avg.lerp_(grad, 1 - beta1)
    aa.beta2 = (float)c.beta2;
    aa.c2 = (float)(1.0 - c.beta2);
    aa.eps = (float)c.adam_eps;
    aa.tau = (float)(c.tau * c.n_env);      // (tau * n_env) * online + (1 - tau * n_env) * target
    aa.one_minus_tau = (float)(1.0 - c.tau * c.n_env);
    aa.adam_table = at<float>(e, e->ws_adam_tab);
    aa.adam_table_len = kAdamTable;
    aa.beta1d = c.beta1;
    aa.beta2d = c.beta2;
    aa.lrd = c.lr;
    aa.batch_global = e->Bg;
    aa.with_loss = 1;
    if (keep_blk && dw_adam16_on(e, DQNX_STEP_GRADS_ONLY) && route_knob("DQNX_APPLY_TILES", 1) != 0) {
        // fused plan: k_dw_adam16 in apply mode -- 32 x 16 parameter tiles, the same per-element
        // update as k_adam, and each tile's blocked copies as (near-)contiguous blocks instead of
        // k_adam's per-element scattered stores (the DP shard step's last launch)
        DwAdam16Args da = apply_dw16_args(e, aa);
        if (prop_in_adam) {
            da.pprop = pua;
            da.pprop_wgs = (e->Bg + 511) / 512;
        }
        if (e->mtc_blocks > 0 && !prop_in_adam && (flags & 0x400)) {   // the next step's in-forward draw reads its MT blocks from the cache
            da.mtc = at<uint32_t>(e, e->ws_mtc);
            da.mtc_blocks = e->mtc_blocks;
        }
        return launch_dw_adam16(da, s);
    }
    fill_blk_layers(e, aa, keep_blk);
    if (prop_in_adam) {
        aa.pprop = pua;
        aa.pprop_wgs = (e->Bg + 255) / 256;
    }
    return launch_adam(aa, s);
}

// Capture `fn` (enqueueing on the given stream) into an executable graph.
template <class Fn>
int capture(dqnx_engine* e, Fn fn, hipGraphExec_t* out) {
    if (!e->capture_stream) DQNX_HIP_CHECK(hipStreamCreateWithFlags(&e->capture_stream, hipStreamNonBlocking));
    DQNX_HIP_CHECK(hipStreamBeginCapture(e->capture_stream, hipStreamCaptureModeThreadLocal));
    int rc = fn(e->capture_stream);
    hipGraph_t graph = nullptr;
    hipError_t ce = hipStreamEndCapture(e->capture_stream, &graph);
    if (rc) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
    }
    if (ce != hipSuccess) return set_hip_error(ce, "hipStreamEndCapture", __FILE__, __LINE__);
    hipError_t ie = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ie != hipSuccess) return set_hip_error(ie, "hipGraphInstantiate", __FILE__, __LINE__);
    return DQNX_OK;
}

// Capture `fn` into a graph once per key, then replay on the caller's stream.
template <class Fn>
int run_graphed(dqnx_engine* e, int key, hipStream_t s, Fn fn) {
    if (!e->graphs) return fn(s);
    auto it = e->graph_cache.find(key);
    if (it == e->graph_cache.end()) {
        hipGraphExec_t exec = nullptr;
        int rc = capture(e, fn, &exec);
        if (rc) return rc;
        it = e->graph_cache.emplace(key, exec).first;
    }
    DQNX_HIP_CHECK(hipGraphLaunch(it->second, s));
    return DQNX_OK;
}

void drop_graphs(dqnx_engine* e) {
    for (auto& kv : e->graph_cache) (void)hipGraphExecDestroy(kv.second);
    e->graph_cache.clear();
    for (auto& kv : e->timed_cache) (void)hipGraphExecDestroy(kv.second);
    e->timed_cache.clear();
    e->steps_cache.clear();
    e->dw16_cache.clear();
}

const std::vector<KStep>& steps_for(dqnx_engine* e, int key) {
    auto it = e->steps_cache.find(key);
    if (it == e->steps_cache.end()) {
        e->building_key = key;
        it = e->steps_cache.emplace(key, build_learn_steps(e, key)).first;
    }
    return it->second;
}

// ---- bucketed DP step (conv nets): the GRADS_ONLY step cut where a layer's
// weight gradient is complete.  Bucket 0 = dense layers + head + the loss slot (complete after
// the dense backward), then one bucket per conv, last conv first; each a contiguous flat range,
// so the caller all-reduces bucket b while the engine computes the remaining backward.
struct DpBucket {
    int k0, k1;              // kernels [k0, k1) of the GRADS_ONLY plan
    int64_t first, count;    // parameter range [first, first + count) (bucket 0: + the loss slot)
};

int dp_buckets(dqnx_engine* e, std::vector<DpBucket>& out) {
    out.clear();
    const NetPlan& np = e->np;
    const int NC = (int)np.conv.size();
    const std::vector<KStep>& ks = steps_for(e, DQNX_STEP_GRADS_ONLY);
    // the last kernel is the whole-gradient slab sum, or (fused plan, k_dw_adam16 in gradient
    // mode) the kernel that writes the gradient itself
    const bool direct = ks.back().name == "dw16_grads";
    const int nk = (int)ks.size() - (direct ? 0 : 1);
    auto find = [&](const std::string& nm, int from) {
        for (int k = from; k < nk; k++)
            if (ks[k].name == nm) return k;
        return -1;
    };
    if (direct && NC == 0 && np.dense.size() >= 2 && route_knob("DQNX_MLP_BUCKETS", 1) != 0) {
        // fused MLP plan: bucket 0 = every gradient but layer 1's (the step up to the head kernel plus
        // the dW tiles of layers 2.. and the head: one k_dw_adam16 launch), bucket 1 = layer 1's dW
        // tiles (a second launch), so bucket 0's all-reduce and Adam run under them.  Layer 1's weight
        // and bias lead the flat vector.  (k ranges: dqnx_learn_step_bucket splits the last launch.)
        const int64_t cut = np.dense[1].off;
        out.push_back({0, nk, cut, np.P - cut});
        out.push_back({nk, nk, 0, cut});
        return DQNX_OK;
    }
    if (NC == 0 || direct) {
        if (direct && NC) return set_error(DQNX_EUNSUPPORTED, "dp buckets: fused dW plan with convs");
        out.push_back({0, nk, 0, np.P});
        return DQNX_OK;
    }
    if (e->micro) {   // micro-CNN plan: every conv's gradient comes out of one launch (micro_dw)
        const int kx = find("micro_dx", 0), kw = find("micro_dw", 0);
        if (kx < 0 || kw < kx) return set_error(DQNX_EUNSUPPORTED, "dp buckets: no micro conv backward in the plan");
        out.push_back({0, kx, np.dense[0].off, np.P - np.dense[0].off});
        out.push_back({kx, nk, np.conv[0].off, np.dense[0].off - np.conv[0].off});
        return DQNX_OK;
    }
    int cut = find("unflatten", 0);
    if (cut < 0) return set_error(DQNX_EUNSUPPORTED, "dp buckets: no conv backward in the plan");
    out.push_back({0, cut, np.dense[0].off, np.P - np.dense[0].off});
    for (int l = NC - 1; l >= 0; l--) {
        // the bucket closes after the last kernel that READS this conv's weights: the implicit
        // path's data gradient reads the permuted copy made at the step's start, so its bucket
        // closes at the dW kernel; the explicit path's dX GEMM (conv_dx / conv_dxs / the level
        // kernel's dx role) reads the live weights, which the bucket's Adam must not update first
        const std::string tag = "_c" + std::to_string(l + 1);
        int k = -1;
        if (e->conv_ig) {
            k = find("conv_dw" + tag, cut);
        } else {
            for (int q = cut; q < nk; q++) {
                const std::string& nm = ks[q].name;
                if (nm.rfind("conv_", 0) == 0 && nm.size() > tag.size() &&
                    nm.compare(nm.size() - tag.size(), tag.size(), tag) == 0)
                    k = q;
            }
        }
        if (k < 0) return set_error(DQNX_EUNSUPPORTED, "dp buckets: no weight gradient kernel for conv %d", l + 1);
        const ConvPlan& cp = np.conv[l];
        out.push_back({cut, k + 1, cp.off, (int64_t)cp.Co * cp.K + cp.Co});
        cut = k + 1;
    }
    if (cut != nk) {   // kernels after conv 1's dW (none in either conv path) go with the last bucket
        out.back().k1 = nk;
    }
    return DQNX_OK;
}

}  // namespace

// ======================================================================================
// C ABI
// ======================================================================================
extern "C" {

const char* dqnx_last_error(void) { return g_err; }
int32_t dqnx_abi_version(void) { return DQNX_ABI_VERSION; }

int dqnx_net_param_count(const dqnx_net_desc* net, int64_t* n_params, int32_t* n_tensors) {
    NetPlan np;
    int rc = plan_net(net, np);
    if (rc) return rc;
    if (n_params) *n_params = np.P;
    if (n_tensors) *n_tensors = (int32_t)np.params.size();
    return DQNX_OK;
}

int dqnx_net_param_info(const dqnx_net_desc* net, int32_t index, dqnx_param_info* out) {
    NetPlan np;
    int rc = plan_net(net, np);
    if (rc) return rc;
    if (!out || index < 0 || index >= (int32_t)np.params.size())
        return set_error(DQNX_EINVAL, "param index %d out of range", index);
    *out = np.params[index];
    return DQNX_OK;
}

void dqnx_config_defaults(dqnx_config* c) {
    if (!c) return;
    const dqnx_net_desc keep = c->net;
    memset(c, 0, sizeof(*c));
    c->net = keep;
    c->algo = DQNX_ALGO_DOUBLE;
    c->batch = 32;
    c->world_size = 1;
    c->rank = 0;
    c->capacity = 1000000;
    c->gamma = 0.99;
    c->lr = 1e-4;
    c->beta1 = 0.9;
    c->beta2 = 0.999;
    c->adam_eps = 1e-8;
    c->tau = 1e-3;
    c->n_env = 1;
    c->per_eps = 1e-4;
    c->per_alpha = 0.6;
    c->per_max_priority = 1.0;
    c->per_beta_start = 0.4;
    c->per_beta_end = 1.0;
    c->per_beta_steps = 2e6;
}

int dqnx_engine_create(const dqnx_config* cfg, dqnx_engine** out) {
    if (!cfg || !out) return set_error(DQNX_EINVAL, "null argument");
    *out = nullptr;
    dqnx_engine* e = new dqnx_engine();
    e->cfg = *cfg;
    int rc = plan_net(&cfg->net, e->np);
    if (rc) { delete e; return rc; }
    const dqnx_config c = *cfg;   // a copy: the error paths below read it after `delete e`
    if (c.algo < DQNX_ALGO_DQN || c.algo > DQNX_ALGO_PER_DOUBLE) { delete e; return set_error(DQNX_EINVAL, "bad algo"); }
    if (c.algo == DQNX_ALGO_PER_DOUBLE && c.per_numpy121) {
        rc = per_numpy121_init();
        if (rc) { delete e; return rc; }
    }
    if (c.algo == DQNX_ALGO_PER_DOUBLE) {
        // exact float64 tree sums need cap <= 2^20 (see per.hip); one sampler workgroup <= PER_MAX_B
        if (c.capacity > ((int64_t)1 << 20)) { delete e; return set_error(DQNX_EUNSUPPORTED, "PER capacity > 2^20"); }
        if (c.batch > PER_MAX_B) { delete e; return set_error(DQNX_EUNSUPPORTED, "PER batch > %d", PER_MAX_B); }
    }
    if (c.batch <= 0 || c.world_size <= 0 || c.rank < 0 || c.rank >= c.world_size || c.batch % c.world_size)
        { delete e; return set_error(DQNX_EINVAL, "batch must be a positive multiple of world_size"); }
    if (c.capacity <= 0 || c.capacity >= ((int64_t)1 << 31)) { delete e; return set_error(DQNX_EINVAL, "capacity out of range"); }
    if (e->np.NH > 16) { delete e; return set_error(DQNX_EUNSUPPORTED, "head with more than 16 outputs"); }
    if (!head_supported(e->np.F)) {
        const int F = e->np.F;   // (read before the delete: found by the ASan plan check)
        delete e;
        return set_error(DQNX_EUNSUPPORTED, "head input width %d not in {64,128,256}", F);
    }
    for (size_t l = 0; l < e->np.dense.size(); l++)
        if (e->np.dense[l].out % 4) { delete e; return set_error(DQNX_EUNSUPPORTED, "hidden widths must be multiples of 4"); }
    if (sample_hash_slots(c.batch) < 0) { delete e; return set_error(DQNX_EUNSUPPORTED, "batch too large for the sampler"); }
    {
        FusedFwdArgs& fp = e->fplan;
        memset(&fp, 0, sizeof(fp));
        fp.L = (int)e->np.dense.size();
        for (int l = 0; l < fp.L && l < FUSED_MAX_L; l++) {
            fp.in[l] = e->np.dense[l].in;
            fp.out[l] = e->np.dense[l].out;
        }
        fp.NH = e->np.NH;
        fp.F = e->np.F;
        if (c.compute_dtype != DQNX_COMPUTE_FP32 && c.compute_dtype != DQNX_COMPUTE_BF16)
            { delete e; return set_error(DQNX_EINVAL, "bad compute_dtype %d", c.compute_dtype); }
        const bool bf = c.compute_dtype == DQNX_COMPUTE_BF16;
        const bool fused_ok = c.net.kind == DQNX_NET_MLP && fused_fwd_plan(fp, c.net.obs_dim, bf, 1);
        e->bwd_plan = fused_ok ? 2 : 0;
        if (route_flag("DQNX_BWD_PLAN")) {
            const int want = route_knob("DQNX_BWD_PLAN", 2);
            if (want == 0 || (want == 1 && c.net.kind == DQNX_NET_MLP) || (want == 2 && fused_ok)) e->bwd_plan = want;
        }
        if (bf && e->bwd_plan != 2) {   // bf16 lives in the fused MLP kernels only
            delete e;
            return set_error(DQNX_EUNSUPPORTED, "bf16 compute needs the fused MLP plan (MLP, widths multiple of 64 <= 256, <= 3 layers)");
        }
    }
    {   // the current device's compute units: the plans below size their grids (and the conv dW /
        // dense-1 split-K slab counts, hence their fixed summation order) from it.  Without a visible
        // device (host-only plan checks) the MI355X's 256 stays.
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            e->n_cu = cus;
        (void)hipGetLastError();
    }
    e->Bg = c.batch;
    e->Bl = c.batch / c.world_size;
    e->local_sampling = c.local_sampling && c.world_size > 1;
    if (e->local_sampling && c.algo == DQNX_ALGO_PER_DOUBLE) {
        delete e;   // the replicated SumTree needs every rank to apply the same ordered updates
        return set_error(DQNX_EUNSUPPORTED, "rank-local sampling is for uniform replay (PER samples globally)");
    }
    e->shard_begin = e->local_sampling ? 0 : c.rank * e->Bl;
    e->Bs = e->local_sampling ? e->Bl : e->Bg;
    e->stride = (int)align_up((uint64_t)c.net.obs_dim, 4);
    e->tiles = (e->Bl + 15) / 16;
    if (e->bwd_plan == 2) {
        // forward rows per workgroup.  bf16: the largest of 4, 2 (x16) that still gives every
        // CU a workgroup (each weight fragment streamed from L2 then feeds mr MFMAs): 30.5 ->
        // 26.2 us at B=8192.  fp32 is MFMA-bound per CU and gains nothing (B=4096: 37.8 us at
        // mr 1, 43.8 at 2, 41.0 at 4), so it keeps 16-row workgroups.
        const int nst = c.algo == DQNX_ALGO_DQN ? 2 : 3;
        int mr = 1;
        if (e->fplan.bf16)
            for (int cand : {4, 2})
                if (mr == 1 && ((e->Bl + 16 * cand - 1) / (16 * cand)) * nst >= 256) mr = cand;
        mr = route_knob("DQNX_FWD_MR", mr);
        FusedFwdArgs trial = e->fplan;
        if (mr != 1 && fused_fwd_plan(trial, c.net.obs_dim, e->fplan.bf16 != 0, mr)) e->fplan = trial;
        // opt-in (DQNX_FWD_SPLIT=2|4): layer 1 in a launch of its own over 2 or 4 column parts
        // per row tile.  Measured slower (B=1024: layer 1 alone 12.1 us on 384 workgroups vs
        // 15.7 us for the whole one-launch forward; step 47.7 vs 45.2 us): the weight bytes
        // streamed from L2 stay the same in total, so more workgroups do not help
        if (e->fplan.mr == 1 && e->fplan.gw == 0 && e->np.dense.size() >= 2) {
            if (route_flag("DQNX_FWD_SPLIT")) {
                const int w = route_knob("DQNX_FWD_SPLIT", 1);
                if (w <= 1) e->fsplit = 1;
                else if (e->np.dense[0].out % (16 * w) == 0) e->fsplit = w;
            }
            // opt-in (DQNX_FWD_PAIR=1, fp32): the one-launch forward with layer 1's columns over two
            // partner workgroups of one XCD and an in-launch sc1 hand-off of the H_1 halves (fused.hip)
            bool pair_ok = e->np.dense[0].out % 32 == 0 && e->np.dense[0].out <= 32 * FUSED_WAVES;
            for (size_t l = 1; l < e->np.dense.size(); l++) pair_ok = pair_ok && e->np.dense[l].out <= 16 * FUSED_WAVES;
            if (e->fsplit <= 1 && !e->fplan.bf16 && route_knob("DQNX_FWD_PAIR", 0) != 0 && pair_ok) e->fpair = 1;
            if (e->fsplit > 1) {   // layer 1's row tiles: 32 rows (each weight fragment feeds 2 MFMAs)
                const int m = route_knob("DQNX_FWD_L1_MR", 2);
                FusedFwdArgs t2 = e->fplan;
                if ((m == 2 || m == 4) && fused_fwd_plan(t2, c.net.obs_dim, e->fplan.bf16 != 0, m)) e->fsplit_mr = m;
            }
        }
    }
    e->setsize = sample_setsize(e->Bs);
    const int L = (int)e->np.dense.size();
    e->slices.assign(L, 1);
    e->kslice.assign(L, e->Bl);
    // minibatch rows per split-K slice of the weight gradients.  bf16 (configs[4], B=8192): 512 rows
    // = 16 slabs, the Adam pass sums half the partials (step 94-96 -> 92 us, profiles/r04/dw_bf16_shapes.json)
    int dw_rows = (e->bwd_plan == 2 && e->fplan.bf16) ? 512 : 256;
    dw_rows = std::max(16, tuning_knob("DQNX_DW_ROWS", dw_rows));
    for (int l = 0; l < L; l++) {
        int S = e->Bl / dw_rows;
        if (S < 1) S = 1;
        if (S > 32) S = 32;
        int ks = (int)align_up((uint64_t)((e->Bl + S - 1) / S), 16);
        S = (e->Bl + ks - 1) / ks;
        e->slices[l] = S;
        e->kslice[l] = ks;
    }
    // opt-in (DQNX_DWB_T=1): bf16 weight gradients from slab-transposed copies written by the forward
    // (the one-launch plan) and the head kernel (k_dw_bf16d; measured slower at configs[4], fused.hip);
    // whole 32-sample chunks
    e->dwt = e->bwd_plan == 2 && e->fplan.bf16 && !(e->fsplit > 1 && e->fplan.mr == 1) && e->Bl % 32 == 0 &&
             e->kslice[0] % 32 == 0 && e->kslice[0] <= 512 && route_knob("DQNX_DWB_T", 0) != 0;
    const int NC = (int)e->np.conv.size();
    e->cslices.assign(NC, 1);
    e->ckslice.assign(NC, 1);
    e->conv_ig = conv_ig_plan(e->np, e->Bl);
    if (NC && route_knob("DQNX_MICRO_CNN", 1) != 0) {   // DQNX_MICRO_CNN=0 keeps the per-layer conv kernels
        MicroConv mc[MICRO_MAX_CONV];
        const int nst = c.algo == DQNX_ALGO_DQN ? 2 : 3;
        int S = 0, lf = 0, dS = 0, dlf = 0, lds_d[MICRO_MAX_CONV];
        if (micro_geom(e->np, mc) && micro_plan(mc, NC, e->Bl, nst, e->n_cu, &S, &lf) &&
            micro_dx_plan(mc, NC, e->Bl, &dS, lds_d, &dlf)) {
            MicroDwArgs& d = e->micro_dw;
            memset(&d, 0, sizeof(d));
            d.nc = NC;
            d.Bl = e->Bl;
            for (int l = 0; l < NC; l++) {
                MicroDwLayer& L = d.L[l];
                L.Ci = mc[l].Ci; L.Hi = mc[l].Hi; L.Wi = mc[l].Wi; L.Co = mc[l].Co; L.Ho = mc[l].Ho; L.Wo = mc[l].Wo;
                L.sh = mc[l].sh; L.sw = mc[l].sw;
            }
            if (micro_dw_plan(d, e->n_cu) == DQNX_OK) {
                e->micro = true;
                e->conv_ig = false;
                e->micro_S = S;
                e->micro_lds = lf;
                e->micro_dx_S = dS;
                e->micro_dx_lds = dlf;
                for (int l = 0; l < NC; l++) e->micro_lds_d[l] = lds_d[l];
            }
        }
    }
    if (NC && route_knob("DQNX_F1_SPLITK", 1) != 0) {   // dense 1 (K = F) as 64 x 64 split-K tiles
        const int nst = c.algo == DQNX_ALGO_DQN ? 2 : 3;
        e->f1_ksplit = fwd_split_ksplit(e->Bl, e->np.dense[0].out, e->np.dense[0].in, nst, e->n_cu, &e->f1_kchunk);
    }
    // conv dW workgroups to aim for: the (4,84,84) conv 1 ([32 x 37] tile grid 2 x 1) had only
    // 64 workgroups at the old 32-slice cap; DQNX_CONV_DW_WGS=0 restores that rule
    int dw_wgs = 1024;
    dw_wgs = std::max(0, tuning_knob("DQNX_CONV_DW_WGS", dw_wgs));
    for (int l = 0; l < NC; l++) {   // split-K over the conv's output pixels (b, ho, wo)
        const ConvPlan& cq = e->np.conv[l];
        const int rows = e->Bl * cq.Ho * cq.Wo;
        int S = rows / 512;
        if (S < 1) S = 1;
        if (S > 32) S = 32;
        const bool big = conv_dw_big(rows, cq.K);
        const int tiles = big ? conv_dw_big_tiles(cq.K, cq.Co)
                              : ((cq.K + 1 + BWD_TILE - 1) / BWD_TILE) * ((cq.Co + BWD_TILE - 1) / BWD_TILE);
        if (dw_wgs > 0) S = std::max(S, std::min({rows / 512, (dw_wgs + tiles - 1) / tiles, 256}));
        int ks = (int)align_up((uint64_t)((rows + S - 1) / S), 16);
        S = (rows + ks - 1) / ks;
        e->cslices[l] = S;
        e->ckslice[l] = ks;
        if (e->conv_ig) {   // slices of output row groups (k_conv_dw_ig)
            ConvDwIgArgs d;
            cig_dw_geom(cq, e->Bl, l == 0, d);
            e->cslices[l] = d.slices;
        }
        if (e->micro) e->cslices[l] = e->micro_dw.L[l].slices;   // sample slices of k_micro_dw
        if (e->np.conv[l].Co % 4) { delete e; return set_error(DQNX_EUNSUPPORTED, "conv channels must be multiples of 4"); }
    }
    layout(e);
    *out = e;
    return DQNX_OK;
}

int dqnx_engine_destroy(dqnx_engine* e) {
    if (!e) return DQNX_OK;
    drop_graphs(e);
    if (e->capture_stream) (void)hipStreamDestroy(e->capture_stream);
    if (e->side_stream) {
        (void)hipStreamSynchronize(e->side_stream);
        (void)hipStreamDestroy(e->side_stream);
    }
    for (int i = 0; i < 2; i++) {
        if (e->ev_sampled[i]) (void)hipEventDestroy(e->ev_sampled[i]);
        if (e->ev_computed[i]) (void)hipEventDestroy(e->ev_computed[i]);
    }
    if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
    if (e->join_ev) (void)hipEventDestroy(e->join_ev);
    for (int i = 0; i < 2; i++)
        if (e->ag_rng_ev[i]) (void)hipEventDestroy(e->ag_rng_ev[i]);
    if (e->ag_ctrl_ev) {
        (void)hipEventSynchronize(e->ag_ctrl_ev);
        (void)hipEventDestroy(e->ag_ctrl_ev);
    }
    if (e->push_ev) {
        (void)hipEventSynchronize(e->push_ev);
        (void)hipEventDestroy(e->push_ev);
    }
    if (e->ag_rng_pin) (void)hipHostFree(e->ag_rng_pin);
    if (e->ag_rng_zc) (void)hipHostFree(e->ag_rng_zc);
    if (e->ag_ctrl_pin) (void)hipHostFree(e->ag_ctrl_pin);
    if (e->push_pin) (void)hipHostFree(e->push_pin);
    delete e;
    return DQNX_OK;
}

int dqnx_engine_arena_bytes(const dqnx_engine* e, uint64_t* bytes) {
    if (!e || !bytes) return set_error(DQNX_EINVAL, "null argument");
    *bytes = e->total;
    return DQNX_OK;
}

int dqnx_engine_buffer(const dqnx_engine* e, int32_t which, uint64_t* offset, uint64_t* bytes) {
    if (!e || which < 0 || which >= DQNX_BUF_COUNT) return set_error(DQNX_EINVAL, "bad buffer id %d", which);
    if (offset) *offset = e->off[which];
    if (bytes) *bytes = e->bytes[which];
    return DQNX_OK;
}

int dqnx_engine_obs_stride(const dqnx_engine* e, int32_t* stride) {
    if (!e || !stride) return set_error(DQNX_EINVAL, "null argument");
    *stride = e->stride;
    return DQNX_OK;
}

int dqnx_params_modified(dqnx_engine* e) {
    if (!e) return set_error(DQNX_EINVAL, "null engine");
    e->perm_dirty = true;
    e->wblk_dirty = true;
    return DQNX_OK;
}

int dqnx_engine_bind(dqnx_engine* e, void* arena, uint64_t bytes) {
    if (!e || !arena) return set_error(DQNX_EINVAL, "null argument");
    if (bytes < e->total) return set_error(DQNX_EINVAL, "arena too small: %llu < %llu", (unsigned long long)bytes,
                                           (unsigned long long)e->total);
    if (((uintptr_t)arena) % 256) return set_error(DQNX_EINVAL, "arena must be 256-byte aligned");
    drop_graphs(e);
    e->arena = (char*)arena;
    e->perm_dirty = true;
    e->wblk_dirty = true;
    return DQNX_OK;
}

int dqnx_engine_set_graphs(dqnx_engine* e, int32_t enabled) {
    if (!e) return set_error(DQNX_EINVAL, "null engine");
    e->graphs = enabled != 0;
    if (!e->graphs) drop_graphs(e);
    return DQNX_OK;
}

int dqnx_engine_reset(dqnx_engine* e, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int ids[] = {DQNX_BUF_GRADS, DQNX_BUF_ADAM_M, DQNX_BUF_ADAM_V, DQNX_BUF_CTRL, DQNX_BUF_RING_OBS,
                       DQNX_BUF_RING_NEXT_OBS, DQNX_BUF_RING_ACT, DQNX_BUF_RING_REW, DQNX_BUF_RING_DONE,
                       DQNX_BUF_SUMTREE, DQNX_BUF_BATCH_IDX, DQNX_BUF_Q, DQNX_BUF_TD, DQNX_BUF_IS_WEIGHTS,
                       DQNX_BUF_WORKSPACE, DQNX_BUF_PER_ABS_TD};
    for (int id : ids)
        if (e->bytes[id]) DQNX_HIP_CHECK(hipMemsetAsync(e->arena + e->off[id], 0, e->bytes[id], s));
    // SumTree.max/min_priority_index start at capacity - 1 (R:dqn/utils/sum_tree.py:12-13)
    dqnx_ctrl init;
    memset(&init, 0, sizeof(init));
    init.per_max_idx = e->cfg.capacity - 1;
    init.per_min_idx = e->cfg.capacity - 1;
    DQNX_HIP_CHECK(hipMemcpyAsync(&ctrl_of(e)->per_max_idx, &init.per_max_idx, 2 * sizeof(int64_t),
                                  hipMemcpyHostToDevice, s));
    // Adam bias corrections, computed like torch's _single_tensor_adam does on the host:
    // step_size = lr / (1 - beta1**t), bias_correction2**0.5 (Python float pow = libm pow)
    {
        std::vector<float> tab((size_t)kAdamTable * 2);
        const dqnx_config& c = e->cfg;
        for (int t = 1; t <= kAdamTable; t++) {
            const double bc1 = 1.0 - std::pow(c.beta1, (double)t);
            const double bc2 = 1.0 - std::pow(c.beta2, (double)t);
            tab[2 * (t - 1)] = (float)(-(c.lr / bc1));
            tab[2 * (t - 1) + 1] = (float)std::pow(bc2, 0.5);
        }
        DQNX_HIP_CHECK(hipMemcpyAsync(e->arena + e->ws_adam_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, s));
        DQNX_HIP_CHECK(hipStreamSynchronize(s));
    }
    e->ring_size = 0;
    e->ring_wptr = 0;
    e->pf_valid = false;
    e->pf_inlaunch = false;
    e->wblk_dirty = true;
    e->perm_dirty = true;   // the workspace memset above zeroed the permuted conv weight copies too
    return DQNX_OK;
}

constexpr int kPinnedPushRows = 64;   // host pushes up to this many rows take the pinned one-copy path

int dqnx_replay_push(dqnx_engine* e, const float* obs, const int32_t* act, const float* rew, const uint8_t* done,
                     const float* next_obs, int32_t n, int32_t src_on_device, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!obs || !act || !rew || !done || !next_obs)))
        return set_error(DQNX_EINVAL, "dqnx_replay_push: bad argument");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "replay push while a prefetched minibatch is pending");
    hipStream_t s = (hipStream_t)stream;
    const int D = e->cfg.net.obs_dim;
    if (!src_on_device && n > 0 && n <= kPinnedPushRows && (int64_t)n <= e->cfg.capacity) {
        // the env loop's n_env rows (Agent.store_transitions): packed into one pinned, fine-grained
        // (host-coherent) block that the push kernel reads in place over the fabric: no copy call, no
        // host wait (the block is reused once the event after its previous push kernel has passed)
        const size_t fb = (size_t)n * D * 4;
        if (!e->push_pin) {
            DQNX_HIP_CHECK(hipHostMalloc((void**)&e->push_pin, (size_t)kPinnedPushRows * (8 * (size_t)D + 9) + 64,
                                         hipHostMallocCoherent));
            DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->push_ev, hipEventDisableTiming));
        }
        if (e->push_live) DQNX_HIP_CHECK(hipEventSynchronize(e->push_ev));
        char* h = e->push_pin;
        memcpy(h, obs, fb);
        memcpy(h + fb, next_obs, fb);
        memcpy(h + 2 * fb, act, (size_t)n * 4);
        memcpy(h + 2 * fb + 4 * (size_t)n, rew, (size_t)n * 4);
        memcpy(h + 2 * fb + 8 * (size_t)n, done, (size_t)n);
        rc = dqnx_replay_push(e, (const float*)h, (const int32_t*)(h + 2 * fb), (const float*)(h + 2 * fb + 4 * (size_t)n),
                              (const uint8_t*)(h + 2 * fb + 8 * (size_t)n), (const float*)(h + fb), n, 1, stream);
        if (rc) return rc;
        DQNX_HIP_CHECK(hipEventRecord(e->push_ev, s));
        e->push_live = true;
        return DQNX_OK;
    }
    int done_rows = 0;
    while (done_rows < n) {
        const bool per = e->cfg.algo == DQNX_ALGO_PER_DOUBLE;
        int m = src_on_device ? n - done_rows : std::min(n - done_rows, e->stage_rows);
        // PER: every add is a SumTree.update in order; chunks never wrap onto themselves
        if (per) m = (int)std::min<int64_t>(std::min(m, PER_CHUNK), e->cfg.capacity);
        PushArgs pa;
        memset(&pa, 0, sizeof(pa));
        if (src_on_device) {
            pa.obs = obs + (int64_t)done_rows * D;
            pa.next_obs = next_obs + (int64_t)done_rows * D;
            pa.act = act + done_rows;
            pa.rew = rew + done_rows;
            pa.done = done + done_rows;
        } else {
            char* st = e->arena + e->ws_stage;
            float* so = (float*)st;
            float* sn = so + (int64_t)e->stage_rows * D;
            int32_t* sa = (int32_t*)(sn + (int64_t)e->stage_rows * D);
            float* sr = (float*)(sa + e->stage_rows);
            uint8_t* sd = (uint8_t*)(sr + e->stage_rows);
            DQNX_HIP_CHECK(hipMemcpyAsync(so, obs + (int64_t)done_rows * D, (size_t)m * D * 4, hipMemcpyHostToDevice, s));
            DQNX_HIP_CHECK(hipMemcpyAsync(sn, next_obs + (int64_t)done_rows * D, (size_t)m * D * 4, hipMemcpyHostToDevice, s));
            DQNX_HIP_CHECK(hipMemcpyAsync(sa, act + done_rows, (size_t)m * 4, hipMemcpyHostToDevice, s));
            DQNX_HIP_CHECK(hipMemcpyAsync(sr, rew + done_rows, (size_t)m * 4, hipMemcpyHostToDevice, s));
            DQNX_HIP_CHECK(hipMemcpyAsync(sd, done + done_rows, (size_t)m, hipMemcpyHostToDevice, s));
            pa.obs = so;
            pa.next_obs = sn;
            pa.act = sa;
            pa.rew = sr;
            pa.done = sd;
        }
        const int64_t cap = e->cfg.capacity;
        pa.n = m;
        pa.obs_dim = D;
        pa.stride = e->stride;
        pa.wptr = e->ring_wptr;
        pa.capacity = cap;
        pa.new_wptr = (e->ring_wptr + m) % cap;
        pa.new_size = std::min<int64_t>(e->ring_size + m, cap);
        pa.ring_obs = at<float>(e, e->off[DQNX_BUF_RING_OBS]);
        pa.ring_next = at<float>(e, e->off[DQNX_BUF_RING_NEXT_OBS]);
        pa.ring_act = at<int32_t>(e, e->off[DQNX_BUF_RING_ACT]);
        pa.ring_rew = at<float>(e, e->off[DQNX_BUF_RING_REW]);
        pa.ring_done = at<float>(e, e->off[DQNX_BUF_RING_DONE]);
        pa.ctrl = ctrl_of(e);
        pa.ring16_obs = e->stride16 ? at<uint16_t>(e, e->ws_ring16[0]) : nullptr;
        pa.ring16_next = e->stride16 ? at<uint16_t>(e, e->ws_ring16[1]) : nullptr;
        pa.stride16 = e->stride16;
        if (m > cap) {
            // only the last `cap` rows survive; push them alone
            const int skip = (int)(m - cap);
            e->ring_wptr = (e->ring_wptr + skip) % cap;
            e->ring_size = std::min<int64_t>(e->ring_size + skip, cap);
            pa.obs += (int64_t)skip * D;
            pa.next_obs += (int64_t)skip * D;
            pa.act += skip;
            pa.rew += skip;
            pa.done += skip;
            pa.n = (int)cap;
            pa.wptr = e->ring_wptr;
            pa.new_wptr = (e->ring_wptr + cap) % cap;
            pa.new_size = cap;
        }
        if (per) {   // Agent.store_transitions -> SumTree.add(max_priority) x m (R:dqn/replay_memory.py:56-67)
            PerUpdateArgs ua = per_update_args(e);
            ua.mode = 1;
            ua.n = pa.n;
            ua.wptr = pa.wptr;
            ua.size = e->ring_size;
            rc = launch_per_update(ua, s);
            if (rc) return rc;
        }
        rc = launch_replay_push(pa, s);
        if (rc) return rc;
        e->ring_wptr = pa.new_wptr;
        e->ring_size = pa.new_size;
        done_rows += m;
        if (!src_on_device) DQNX_HIP_CHECK(hipStreamSynchronize(s));  // staging buffer reuse
    }
    return DQNX_OK;
}

int dqnx_rng_set(dqnx_engine* e, int32_t which, const uint32_t* state625, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!state625 || (which != DQNX_RNG_PY && which != DQNX_RNG_NP)) return set_error(DQNX_EINVAL, "bad argument");
    if (state625[624] > 624) return set_error(DQNX_EINVAL, "MT index must be <= 624");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "rng_set while a prefetched minibatch is pending");
    hipStream_t s = (hipStream_t)stream;
    uint32_t* dst = which == DQNX_RNG_PY ? ctrl_of(e)->py_mt : ctrl_of(e)->np_mt;
    DQNX_HIP_CHECK(hipMemcpyAsync(dst, state625, 625 * 4, hipMemcpyHostToDevice, s));
    DQNX_HIP_CHECK(hipStreamSynchronize(s));
    return DQNX_OK;
}

int dqnx_rng_get(dqnx_engine* e, int32_t which, uint32_t* state625, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!state625 || (which != DQNX_RNG_PY && which != DQNX_RNG_NP)) return set_error(DQNX_EINVAL, "bad argument");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t* src = which == DQNX_RNG_PY ? ctrl_of(e)->py_mt : ctrl_of(e)->np_mt;
    if (e->pf_valid && e->pf_inlaunch) DQNX_HIP_CHECK(hipStreamSynchronize(e->pf_stream));
    else if (e->pf_valid) DQNX_HIP_CHECK(hipStreamWaitEvent(s, e->ev_sampled[e->pf_slot], 0));
    DQNX_HIP_CHECK(hipMemcpyAsync(state625, src, 625 * 4, hipMemcpyDeviceToHost, s));
    DQNX_HIP_CHECK(hipStreamSynchronize(s));
    return DQNX_OK;
}

int dqnx_rng_set_async(dqnx_engine* e, int32_t which, const uint32_t* state625, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!state625 || (which != DQNX_RNG_PY && which != DQNX_RNG_NP)) return set_error(DQNX_EINVAL, "bad argument");
    if (state625[624] > 624) return set_error(DQNX_EINVAL, "MT index must be <= 624");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "rng_set while a prefetched minibatch is pending");
    uint32_t* dst = which == DQNX_RNG_PY ? ctrl_of(e)->py_mt : ctrl_of(e)->np_mt;
    DQNX_HIP_CHECK(hipMemcpyAsync(dst, state625, 625 * 4, hipMemcpyHostToDevice, (hipStream_t)stream));
    return DQNX_OK;
}

int dqnx_rng_get_async(dqnx_engine* e, int32_t which, uint32_t* state625, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!state625 || (which != DQNX_RNG_PY && which != DQNX_RNG_NP)) return set_error(DQNX_EINVAL, "bad argument");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "rng_get_async while a prefetched minibatch is pending");
    const uint32_t* src = which == DQNX_RNG_PY ? ctrl_of(e)->py_mt : ctrl_of(e)->np_mt;
    DQNX_HIP_CHECK(hipMemcpyAsync(state625, src, 625 * 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return DQNX_OK;
}

int dqnx_ctrl_get_async(dqnx_engine* e, void* dst, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!dst) return set_error(DQNX_EINVAL, "null argument");
    DQNX_HIP_CHECK(hipMemcpyAsync(dst, ctrl_of(e), sizeof(dqnx_ctrl), hipMemcpyDeviceToHost, (hipStream_t)stream));
    return DQNX_OK;
}

// Prefetch pipeline (DQNX_STEP_PREFETCH): the sampler runs on the engine's side stream,
// one step ahead, into the other (idx, phys) slot.  Ordering, all by events:
//   side: wait computed[nxt] (step t-1 read slot nxt) -> sample(t+1) into nxt -> sampled[nxt]
//   main: wait sampled[cur] -> compute(t) on slot cur -> computed[cur]
// The sampler is the only writer of ctrl->py_mt and the slots, so results are bit-identical
// to sequential steps.
static int pf_events(dqnx_engine* e) {
    if (!e->side_stream) {
        // the highest priority the device offers: the side stream's sampler workgroup (one workgroup with
        // up to 154 KiB of LDS) is placed ahead of the remaining workgroups of the step's forward instead of
        // waiting for a CU to drain (measured round 6: the side draw otherwise started near the forward's end)
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo) {
            DQNX_HIP_CHECK(hipStreamCreateWithPriority(&e->side_stream, hipStreamNonBlocking, hi));
        } else {
            DQNX_HIP_CHECK(hipStreamCreateWithFlags(&e->side_stream, hipStreamNonBlocking));
        }
    }
    for (int i = 0; i < 2; i++) {
        if (!e->ev_sampled[i]) DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->ev_sampled[i], hipEventDisableTiming));
        if (!e->ev_computed[i]) DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->ev_computed[i], hipEventDisableTiming));
    }
    if (!e->fork_ev) DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming));
    return DQNX_OK;
}

static int pf_sample(dqnx_engine* e, int base, int slot) {
    const std::vector<KStep>& ks = steps_for(e, base | (slot << 8));
    return run_graphed(e, 0x10000 | (slot << 8), e->side_stream,
                       [&](hipStream_t cs) { return enqueue_range(ks, 0, 1, cs); });
}

// In-launch prefetch (fused plan): step t computes on slot cur, and its k_dw_adam16 launch draws
// step t+1's minibatch into slot cur ^ 1 with one more workgroup.  Same stream, so ordering is
// the launch order: the draw reads the MT state only after step t-1's draw wrote it, and step t+1
// reads the slot after the launch that filled it.  Results are bitwise those of sequential steps
// (the sample depends only on the MT state and the ring, which push / rng_set refuse to change
// while a minibatch is pending).
// The fused plan's blocked weight copies rebuilt by a launch of their own (a step whose minibatch
// was drawn ahead has no sampler launch whose spare workgroups would do it)
static int enqueue_relayout(dqnx_engine* e, hipStream_t s) {
    int blocks = 0;
    RelayoutArgs rl = relayout_args(e, &blocks);
    return launch_idx_to_phys(nullptr, nullptr, 0, 0, ctrl_of(e), e->cfg.capacity, &rl, blocks, s);
}

static int inlaunch_prologue(dqnx_engine* e, int base, hipStream_t s) {
    const int key0 = base | (relayout_due(e) ? KEY_RELAYOUT : 0);
    const std::vector<KStep>& ks0 = steps_for(e, key0);
    int rc = run_graphed(e, 0x80000 | key0, s, [&](hipStream_t cs) { return enqueue_range(ks0, 0, 1, cs); });
    if (rc) return rc;
    e->wblk_dirty = false;
    e->pf_valid = true;
    e->pf_inlaunch = true;
    e->pf_stream = s;
    return DQNX_OK;
}

static int learn_step_inlaunch(dqnx_engine* e, int base, bool prefetch, hipStream_t s) {
    int rc = DQNX_OK;
    if (e->pf_valid && s != e->pf_stream) {   // the pending draw was enqueued on another stream
        DQNX_HIP_CHECK(hipStreamSynchronize(e->pf_stream));
    }
    if (!e->pf_valid) {   // prologue: this step's minibatch by the sampler launch (+ relayout if dirty)
        rc = inlaunch_prologue(e, base, s);
        if (rc) return rc;
    } else if (relayout_due(e)) {   // weights changed outside a blocked-copy-keeping update
        rc = enqueue_relayout(e, s);
        if (rc) return rc;
        e->wblk_dirty = false;
    }
    const int key = base | (prefetch ? KEY_SAMPLE_NEXT : 0);
    const std::vector<KStep>& ks = steps_for(e, key);
    rc = run_graphed(e, key | 0x20000, s,
                     [&](hipStream_t cs) { return enqueue_range(ks, prefetch ? 0 : 1, (int)ks.size(), cs); });
    if (rc) return rc;
    // the slab plan's Adam pass (and a GRADS_ONLY step's later dqnx_apply_grads) leaves the blocked
    // copies behind: the next step rebuilds them first (with no sampler launch to host it)
    // (a prefetching step's update keeps them: k_dw_adam16 always, the slab plan's Adam pass when it
    // draws ahead; a GRADS_ONLY step's dqnx_apply_grads decides for itself)
    if (!blk_kept(e, base) && !(prefetch && !(base & DQNX_STEP_GRADS_ONLY))) e->wblk_dirty = true;
    if (!prefetch) {   // consumed the pending minibatch; nothing drawn ahead
        e->pf_valid = false;
        e->pf_inlaunch = false;
        return DQNX_OK;
    }
    e->pf_stream = s;   // dqnx_rng_get synchronises it (an event record per step cost ~10 us of queue time)
    return DQNX_OK;
}

// Side-stream prefetch on the fused plan, where the in-launch draw does not fit (k beyond the forward's
// sampler workgroup: configs[3] weak scaling, every rank drawing the global 32768): step t computes on
// slot 0 on the caller's stream while the engine's side stream draws step t+1's minibatch into slot 1
// (the sampler reads only the MT state and the ring's size / write pointer, which no kernel of a step
// writes); once step t's kernels are done with slot 0 the side stream copies slot 1 over it, and the
// step's last act on the caller's stream is to wait for that -- every step (and any captured sequence
// of them) is self-contained, the draw hidden under the step's compute.  The blocked weight copies (no
// sampler launch in the step to rebuild them) are rebuilt on the caller's stream when stale.  Bitwise
// equal to sequential steps (test_gpu_side_prefetch_bit_identical).
// Only for draws long enough to pay for the pipeline (a copy launch, a cross-queue wait and the draw's
// workgroup slowing the forward beside it): rank 0's weak shard (4096 rows) replayed as GraphedDPStep
// replays it measured 117.5 us drawn ahead vs 111.7 us with the draw as its own launch at k = 8192,
// 116.9 vs 117.4 at 16384, 117.7 vs 145.2 at 32768.
static bool side_fused_ok(const dqnx_engine* e, int base) {
    return e->bwd_plan == 2 && e->cfg.algo != DQNX_ALGO_PER_DOUBLE && !(base & DQNX_STEP_GIVEN_INDICES) &&
           !inlaunch_prefetch_ok(e, base) && route_knob("DQNX_PF_SIDE_FUSED", 1) != 0 &&
           e->Bs > route_knob("DQNX_PF_SIDE_MIN_K", 8192);
}

// Side-stream prefetch (fused plan, k past the forward's sampler workgroup): the pending minibatch
// always sits in slot 1.  A step first copies slot 1 over the compute slot 0 on the caller's stream
// (one small launch), then forks the side stream there and draws step t+1 into slot 1 beside its own
// compute, so the caller's stream never waits on the side stream after the compute: only the next
// step's copy waits for that draw, which has had the whole step to finish.  (A first version copied at
// the END of the step on the side stream: two cross-queue hops and two copy launches between the
// compute and the DP apply launch, ~39 us per step at configs[3]'s weak shard.)
static int side_fused_prologue(dqnx_engine* e, int base, hipStream_t s) {
    int rc = pf_events(e);
    if (rc) return rc;
    // (kernel 0 = the sampler launch, slot 1; its spare workgroups rebuild stale blocked copies)
    const int key1 = base | (1 << 8) | (relayout_due(e) ? KEY_RELAYOUT : 0);
    const std::vector<KStep>& ks1 = steps_for(e, key1);
    rc = run_graphed(e, 0x80000 | key1, s, [&](hipStream_t cs) { return enqueue_range(ks1, 0, 1, cs); });
    if (rc) return rc;
    if (key1 & KEY_RELAYOUT) e->wblk_dirty = false;
    DQNX_HIP_CHECK(hipEventRecord(e->ev_sampled[1], s));
    e->pf_slot = 1;
    e->pf_valid = true;
    e->pf_inlaunch = false;
    e->pf_stream = s;
    return DQNX_OK;
}

static int learn_step_side_fused(dqnx_engine* e, int base, bool prefetch, hipStream_t s) {
    int rc = DQNX_OK;
    if (!e->pf_valid) {   // this step's minibatch, drawn on the caller's stream
        rc = side_fused_prologue(e, base, s);
        if (rc) return rc;
    }
    // the pending minibatch (slot 1) over the compute slot, once its draw is done
    DQNX_HIP_CHECK(hipStreamWaitEvent(s, e->ev_sampled[1], 0));
    int32_t* idx = at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]);
    int32_t* phys = at<int32_t>(e, e->ws_phys);
    if (relayout_due(e)) {   // (an apply with a draw pending rewrites the blocked copies itself)
        rc = enqueue_relayout(e, s);
        if (rc) return rc;
        e->wblk_dirty = false;
    }
    // the copy and this step's compute launches as one graph (a separate copy launch ahead of the
    // graph measured a ~7 us hop between them); step t+1's draw forks once the copy has read slot 1
    const std::vector<KStep>& ks = steps_for(e, base);
    const int key = base | 0x20000 | 0x10000000;
    auto copy = [&](hipStream_t cs) { return launch_copy_i32x2(idx, idx + e->Bg, e->Bg, phys, phys + e->Bl, e->Bl, cs); };
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    DQNX_HIP_CHECK(hipStreamIsCapturing(s, &cst));
    if (prefetch && cst == hipStreamCaptureStatusNone && route_knob("DQNX_SIDE_EXTEV", 1) != 0) {
        // eager: the fork and the draw's completion recorded by the copy's and the sampler's own
        // dispatches (hipExtLaunchKernelGGL's stop event) -- no marker packet of their own
        KernelTimer& kt = kernel_timer();
        kt.start = nullptr;
        kt.stop = e->fork_ev;
        rc = copy(s);
        kt.stop = nullptr;
        if (rc) return rc;
        DQNX_HIP_CHECK(hipStreamWaitEvent(e->side_stream, e->fork_ev, 0));
        kt.stop = e->ev_sampled[1];
        rc = enqueue_range(steps_for(e, base | (1 << 8)), 0, 1, e->side_stream);
        kt.stop = nullptr;
        if (rc) return rc;
        rc = run_graphed(e, key, s, [&](hipStream_t cs) { return enqueue_range(ks, 1, (int)ks.size(), cs); });
    } else if (prefetch) {
        rc = run_graphed(e, key | 0x8000000, s, copy);
        if (rc) return rc;
        DQNX_HIP_CHECK(hipEventRecord(e->fork_ev, s));
        DQNX_HIP_CHECK(hipStreamWaitEvent(e->side_stream, e->fork_ev, 0));
        rc = pf_sample(e, base, 1);
        if (rc) return rc;
        DQNX_HIP_CHECK(hipEventRecord(e->ev_sampled[1], e->side_stream));
        if (route_knob("DQNX_SIDE_GRAPH", 1) != 0)
            rc = run_graphed(e, key, s, [&](hipStream_t cs) { return enqueue_range(ks, 1, (int)ks.size(), cs); });
        else
            rc = enqueue_range(ks, 1, (int)ks.size(), s);
    } else {
        rc = run_graphed(e, key | 0x4000000, s, [&](hipStream_t cs) {
            int r = copy(cs);
            return r ? r : enqueue_range(ks, 1, (int)ks.size(), cs);
        });
    }
    if (rc) return rc;
    if (!blk_kept(e, base)) e->wblk_dirty = true;
    if (!prefetch) {   // consumed the pending minibatch; nothing drawn ahead
        e->pf_valid = false;
        return DQNX_OK;
    }
    // a captured graph may not end with the side draw unjoined: join it at the step's end there, after
    // the Adam pass (GRADS_ONLY: at the end of dqnx_apply_grads) -- the same graph edges as leaving it
    // to the next step's copy, whose wait the join then duplicates; eager steps leave it running
    if (cst == hipStreamCaptureStatusActive && !(base & DQNX_STEP_GRADS_ONLY))
        DQNX_HIP_CHECK(hipStreamWaitEvent(s, e->ev_sampled[1], 0));
    e->pf_slot = 1;
    e->pf_stream = s;
    return DQNX_OK;
}

int dqnx_learn_step(dqnx_engine* e, int32_t flags, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (e->cfg.algo == DQNX_ALGO_PER_DOUBLE && (flags & DQNX_STEP_GIVEN_INDICES))
        return set_error(DQNX_EUNSUPPORTED, "PER learn step samples its own minibatch");
    // PER: step t+1's sample depends on step t's priority update, so nothing is drawn ahead.
    // Fused plan: the last launch of step t (k_dw_adam16) hosts step t+1's sampler workgroup
    // (in-launch prefetch, same stream, no events); where it cannot (k past the multi-pass
    // sampler, slab plan), nothing is drawn ahead.  Per-layer plan: a side-stream pipeline.
    const int base = flags & (DQNX_STEP_SOFT_UPDATE | DQNX_STEP_GIVEN_INDICES | DQNX_STEP_GRADS_ONLY);
    const bool inl = inlaunch_prefetch_ok(e, base);
    const bool side = side_fused_ok(e, base);
    const bool prefetch = (flags & DQNX_STEP_PREFETCH) && !(flags & DQNX_STEP_GIVEN_INDICES) &&
                          e->cfg.algo != DQNX_ALGO_PER_DOUBLE && (e->bwd_plan != 2 || inl || side);
    if (e->ring_size < e->Bs && !(flags & DQNX_STEP_GIVEN_INDICES) && !e->pf_valid)
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    if (e->pf_valid && (flags & DQNX_STEP_GIVEN_INDICES))
        return set_error(DQNX_ESTATE, "given-indices step while a prefetched minibatch is pending");
    if (e->pf_valid && e->pf_inlaunch) return learn_step_inlaunch(e, base, prefetch, s);
    if (prefetch && inl) return learn_step_inlaunch(e, base, true, s);
    if (!prefetch && !e->pf_valid) {
        // the weights changed outside the Adam pass: this step's sampler launch rebuilds the copies
        const int key = base | ((e->bwd_plan == 2 && (e->wblk_dirty || !blk_kept(e, base))) ? KEY_RELAYOUT : 0) |
                        (e->ag_zc_launch ? KEY_AGENT_RNG : 0);
        const std::vector<KStep>& ks = steps_for(e, key);
        rc = run_graphed(e, key, s, [&](hipStream_t cs) { return enqueue_range(ks, 0, (int)ks.size(), cs); });
        if (!rc) e->wblk_dirty = !blk_kept(e, base);   // stale again after an update that does not keep them
        return rc;
    }
    if (e->bwd_plan == 2) return learn_step_side_fused(e, base, prefetch, s);
    rc = pf_events(e);
    if (rc) return rc;
    if (!e->pf_valid) {   // prologue: this step's minibatch, ordered after everything on s
        DQNX_HIP_CHECK(hipEventRecord(e->fork_ev, s));
        DQNX_HIP_CHECK(hipStreamWaitEvent(e->side_stream, e->fork_ev, 0));
        rc = pf_sample(e, base, 0);
        if (rc) return rc;
        DQNX_HIP_CHECK(hipEventRecord(e->ev_sampled[0], e->side_stream));
        e->pf_slot = 0;
        e->pf_valid = true;
        e->pf_computed_valid[0] = e->pf_computed_valid[1] = false;
    }
    const int cur = e->pf_slot, nxt = cur ^ 1;
    // compute this step on slot `cur`
    DQNX_HIP_CHECK(hipStreamWaitEvent(s, e->ev_sampled[cur], 0));
    const std::vector<KStep>& ks = steps_for(e, base | (cur << 8));
    rc = run_graphed(e, base | (cur << 8) | 0x20000, s,
                     [&](hipStream_t cs) { return enqueue_range(ks, 1, (int)ks.size(), cs); });
    if (rc) return rc;
    DQNX_HIP_CHECK(hipEventRecord(e->ev_computed[cur], s));
    e->pf_computed_valid[cur] = true;
    if (!prefetch) {   // consumed the pending minibatch; nothing drawn ahead
        e->pf_valid = false;
        return DQNX_OK;
    }
    // draw the next step's minibatch into slot `nxt` once step t-1 no longer reads it
    if (e->pf_computed_valid[nxt]) DQNX_HIP_CHECK(hipStreamWaitEvent(e->side_stream, e->ev_computed[nxt], 0));
    rc = pf_sample(e, base, nxt);
    if (rc) return rc;
    DQNX_HIP_CHECK(hipEventRecord(e->ev_sampled[nxt], e->side_stream));
    e->pf_slot = nxt;
    return DQNX_OK;
}

// `count` consecutive learn steps as ONE graph (pure learning loops, e.g. several learn steps
// per environment step): the first step's minibatch is drawn by the sampler launch, every
// later one by the previous step's forward launch (in-launch prefetch), the last step draws
// nothing ahead.  Bitwise equal to `count` dqnx_learn_step calls, and nothing is pending after
// the call.  Configurations without the in-launch sampler (PER, the slab / per-layer plans,
// k past the multi-pass sampler) run the steps one by one.
int dqnx_learn_steps(dqnx_engine* e, int32_t flags, int32_t count, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (count < 1 || count > 256) return set_error(DQNX_EINVAL, "learn_steps: count %d not in [1, 256]", count);
    if (flags & (DQNX_STEP_PREFETCH | DQNX_STEP_GIVEN_INDICES | DQNX_STEP_GRADS_ONLY))
        return set_error(DQNX_EINVAL, "learn_steps: flags may only hold DQNX_STEP_SOFT_UPDATE");
    hipStream_t s = (hipStream_t)stream;
    const int base = flags & DQNX_STEP_SOFT_UPDATE;
    if (e->pf_valid || !inlaunch_prefetch_ok(e, base)) {
        for (int i = 0; i < count; i++) {
            rc = dqnx_learn_step(e, base, stream);
            if (rc) return rc;
        }
        return DQNX_OK;
    }
    if (e->ring_size < e->Bs)
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    const int first = base | (relayout_due(e) ? KEY_RELAYOUT : 0);
    rc = run_graphed(e, 0x40000000 | (count << 12) | first, s, [&](hipStream_t cs) {
        const std::vector<KStep>& k0 = steps_for(e, first);   // slot 0: sampler (+ relayout) + step
        int r = enqueue_range(k0, 0, 1, cs);
        const bool kept = blk_kept(e, base);
        for (int i = 0; i < count && !r; i++) {
            const bool last = i == count - 1;
            (void)kept;   // every step before the last draws ahead, and its update keeps the copies
            const std::vector<KStep>& ks = steps_for(e, base | (last ? 0 : KEY_SAMPLE_NEXT));
            if (!r) r = enqueue_range(ks, last ? 1 : 0, (int)ks.size(), cs);
        }
        return r;
    });
    if (!rc) e->wblk_dirty = !blk_kept(e, base);
    return rc;
}

// The plan the timing entry points describe: flags & 7, and with DQNX_STEP_PREFETCH (where the
// in-launch prefetch applies) the steady-state step of a prefetching loop -- no sampler launch,
// the last launch draws the next minibatch (into slot 1; timing runs leave the state stale).
static int timing_key(const dqnx_engine* e, int32_t flags) {
    const int base = flags & 7;
    if ((flags & DQNX_STEP_PREFETCH) && inlaunch_prefetch_ok(e, base)) return base | KEY_SAMPLE_NEXT;
    return base;
}

int dqnx_prefetch_begin(dqnx_engine* e, int32_t flags, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    const int base = flags & (DQNX_STEP_SOFT_UPDATE | DQNX_STEP_GRADS_ONLY);
    const bool side = side_fused_ok(e, base);
    if (e->pf_valid || e->cfg.algo == DQNX_ALGO_PER_DOUBLE || (!inlaunch_prefetch_ok(e, base) && !side))
        return DQNX_OK;   // a draw is pending already, or this configuration does not draw ahead
    if (e->ring_size < e->Bs)
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    if (side) return side_fused_prologue(e, base, (hipStream_t)stream);
    return inlaunch_prologue(e, base, (hipStream_t)stream);
}

int dqnx_learn_kernel_count(dqnx_engine* e, int32_t flags, int32_t* n) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!n) return set_error(DQNX_EINVAL, "null argument");
    *n = (int32_t)steps_for(e, timing_key(e, flags)).size();
    return DQNX_OK;
}

int dqnx_learn_kernel_info(dqnx_engine* e, int32_t flags, int32_t i, char* name, int32_t name_len, double* flops,
                           double* bytes) {
    int rc = check_bound(e);
    if (rc) return rc;
    const std::vector<KStep>& ks = steps_for(e, timing_key(e, flags));
    if (i < 0 || i >= (int32_t)ks.size()) return set_error(DQNX_EINVAL, "kernel index %d out of range", i);
    if (name && name_len > 0) snprintf(name, (size_t)name_len, "%s", ks[i].name.c_str());
    if (flops) *flops = ks[i].flops;
    if (bytes) *bytes = ks[i].bytes;
    return DQNX_OK;
}

int dqnx_learn_step_timed(dqnx_engine* e, int32_t flags, int32_t kernel_index, void* ev_start, void* ev_stop,
                          void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!ev_start || !ev_stop) return set_error(DQNX_EINVAL, "null event");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "timed step with a prefetched minibatch pending");
    if (e->ring_size < e->Bs && !(flags & DQNX_STEP_GIVEN_INDICES))
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    // the plan kernel_count / kernel_info / step_omit describe (with DQNX_STEP_PREFETCH: the
    // steady-state step of a prefetching loop; the draw it makes is left stale, as step_omit's)
    const int key = timing_key(e, flags);
    const std::vector<KStep>& ks = steps_for(e, key);
    const int n = (int)ks.size();
    if (kernel_index < 0 || kernel_index >= n) return set_error(DQNX_EINVAL, "kernel index out of range");
    hipStream_t s = (hipStream_t)stream;
    // eager launches (HIP cannot time events recorded inside a graph).  The event pair is bound to
    // the timed kernel's own dispatch (DQNX_LAUNCH through hipExtLaunchKernelGGL, common.hpp): the
    // events carry that dispatch's begin / end timestamps, as rocprofv3's kernel trace does, with no
    // marker packets between the kernels of the step
    rc = enqueue_range(ks, 0, kernel_index, s);
    if (rc) return rc;
    KernelTimer& kt = kernel_timer();
    kt.start = (hipEvent_t)ev_start;
    kt.stop = (hipEvent_t)ev_stop;
    rc = enqueue_range(ks, kernel_index, kernel_index + 1, s);
    const bool unused = kt.start != nullptr;
    kt.start = kt.stop = nullptr;
    if (rc) return rc;
    if (unused) return set_error(DQNX_EUNSUPPORTED, "kernel %d (%s) launches nothing through DQNX_LAUNCH", kernel_index,
                                 ks[kernel_index].name.c_str());
    return enqueue_range(ks, kernel_index + 1, n, s);
}

// Timing aid: one learn step as a graph with kernel `omit_index` left out (-1: none).  The
// difference of event-timed runs with and without a kernel is that kernel's in-context
// cost per launch (bench.py roofline).  The omitted kernel's outputs are stale, so the
// engine state afterwards is for timing only.
int dqnx_learn_step_omit(dqnx_engine* e, int32_t flags, int32_t omit_index, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (e->pf_valid) return set_error(DQNX_ESTATE, "timing step with a prefetched minibatch pending");
    if (e->ring_size < e->Bs && !(flags & DQNX_STEP_GIVEN_INDICES))
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    const int base = timing_key(e, flags);
    const std::vector<KStep>& ks = steps_for(e, base);
    const int n = (int)ks.size();
    if (omit_index < -1 || omit_index >= n) return set_error(DQNX_EINVAL, "kernel index out of range");
    return run_graphed(e, base | 0x40000 | ((omit_index + 1) << 20), (hipStream_t)stream, [&](hipStream_t cs) {
        for (int i = 0; i < n; i++) {
            if (i == omit_index) continue;
            int r = ks[i].run(cs);
            if (r) return r;
        }
        return (int)DQNX_OK;
    });
}

int dqnx_per_sample(dqnx_engine* e, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (e->cfg.algo != DQNX_ALGO_PER_DOUBLE) return set_error(DQNX_ESTATE, "engine is not PER");
    const PerSampleArgs pa = per_sample_args(e, at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]), at<int32_t>(e, e->ws_phys));
    return launch_per_sample(pa, (hipStream_t)stream);
}

int dqnx_per_update_priorities(dqnx_engine* e, const int32_t* slots, const float* abs_td, int32_t n, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (e->cfg.algo != DQNX_ALGO_PER_DOUBLE) return set_error(DQNX_ESTATE, "engine is not PER");
    if (n < 0 || (n && (!slots || !abs_td))) return set_error(DQNX_EINVAL, "bad argument");
    return enqueue_per_update_pairs(e, slots, abs_td, n, (hipStream_t)stream);
}

int dqnx_set_agent_step(dqnx_engine* e, int64_t step_times_n_env, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    const int64_t v = step_times_n_env;
    DQNX_HIP_CHECK(hipMemcpyAsync(&ctrl_of(e)->agent_step, &v, sizeof(v), hipMemcpyHostToDevice, (hipStream_t)stream));
    DQNX_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));   // `v` is on this stack frame
    return DQNX_OK;
}

int dqnx_events_create(int32_t n, void** events) {
    if (n < 0 || (n && !events)) return set_error(DQNX_EINVAL, "bad argument");
    for (int i = 0; i < n; i++) {
        hipEvent_t ev;
        DQNX_HIP_CHECK(hipEventCreate(&ev));
        events[i] = (void*)ev;
    }
    return DQNX_OK;
}

int dqnx_events_destroy(int32_t n, void** events) {
    for (int i = 0; i < n; i++)
        if (events && events[i]) (void)hipEventDestroy((hipEvent_t)events[i]);
    return DQNX_OK;
}

int dqnx_event_elapsed(void* start, void* stop, float* ms) {
    if (!start || !stop || !ms) return set_error(DQNX_EINVAL, "null argument");
    DQNX_HIP_CHECK(hipEventSynchronize((hipEvent_t)stop));
    DQNX_HIP_CHECK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return DQNX_OK;
}

int dqnx_prefetch_stream(dqnx_engine* e, void* stream) {
    if (!e) return set_error(DQNX_EINVAL, "null engine");
    e->pf_stream = (hipStream_t)stream;   // where replays of a captured prefetching step run
    return DQNX_OK;
}

int dqnx_apply_grads(dqnx_engine* e, int32_t flags, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    // with an in-launch prefetch pending the next step has no sampler launch: this pass writes the
    // fused plan's blocked copies itself (measured 2.4-2.6 us per DP shard step faster than a
    // relayout launch); otherwise the next sampler launch rebuilds them for free
    // (the side-stream pipeline too: its next step has no sampler launch on the compute stream)
    const bool keep = e->bwd_plan == 2 && e->pf_valid && (e->pf_inlaunch || route_knob("DQNX_SIDE_APPLY_KEEP", 1) != 0);
    const int key = 0x100 | (flags & DQNX_STEP_SOFT_UPDATE) | (keep ? 0x200 : 0) | (keep && e->pf_inlaunch ? 0x400 : 0);
    const int rc2 = run_graphed(e, key, (hipStream_t)stream, [&](hipStream_t s) { return enqueue_apply(e, key, s); });
    if (rc2) return rc2;
    if (e->bwd_plan == 2 && e->pf_valid && !e->pf_inlaunch && e->side_stream) {   // (learn_step_side_fused: the captured join)
        hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
        DQNX_HIP_CHECK(hipStreamIsCapturing((hipStream_t)stream, &cst));
        if (cst == hipStreamCaptureStatusActive) DQNX_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, e->ev_sampled[1], 0));
    }
    e->perm_dirty = true;   // (mode 2: the conv weights change without their permuted copies)
    if (keep) e->wblk_dirty = false;                          // every blocked copy rewritten from the new weights
    else if (!adam_keeps_blk(e)) e->wblk_dirty = true;        // this Adam pass leaves the blocked copies behind
    return DQNX_OK;
}

int dqnx_dp_bucket_count(dqnx_engine* e, int32_t* n) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!n) return set_error(DQNX_EINVAL, "null argument");
    std::vector<DpBucket> b;
    rc = dp_buckets(e, b);
    if (rc) return rc;
    *n = (int32_t)b.size();
    return DQNX_OK;
}

int dqnx_dp_bucket_info(dqnx_engine* e, int32_t bucket, int64_t* first, int64_t* count) {
    int rc = check_bound(e);
    if (rc) return rc;
    std::vector<DpBucket> b;
    rc = dp_buckets(e, b);
    if (rc) return rc;
    if (bucket < 0 || bucket >= (int32_t)b.size()) return set_error(DQNX_EINVAL, "bucket %d out of range", bucket);
    if (first) *first = b[bucket].first;
    if (count) *count = b[bucket].count + (bucket == 0 ? 1 : 0);   // bucket 0 carries the loss slot
    return DQNX_OK;
}

// the fused MLP plan's two buckets (dp_buckets): the dW tiles of every layer but layer 1 / of layer 1
// (a.L order of the plan's k_dw_adam16 launch: dense layers last-first, then the head)
static uint32_t mlp_bucket_mask(const dqnx_engine* e, int bucket) {
    const uint32_t l1 = 1u << ((int)e->np.dense.size() - 1);
    return bucket == 0 ? ~l1 : l1;
}

static int learn_step_bucket_mlp(dqnx_engine* e, int32_t flags, int32_t bucket, hipStream_t s) {
    const int base = DQNX_STEP_GRADS_ONLY;
    int rc = DQNX_OK;
    if (bucket == 1) {   // layer 1's dW tiles (+ the step's extra workgroups: the staged-minibatch copy)
        auto it = e->dw16_cache.find(e->bucket_key);
        if (e->bucket_key < 0 || it == e->dw16_cache.end())
            return set_error(DQNX_ESTATE, "dp bucket 1 before bucket 0 of the same step");
        rc = launch_dw_adam16(dw16_subset(it->second, mlp_bucket_mask(e, 1), false, true), s);
        if (rc) return rc;
        const bool pf_path = (e->bucket_key & KEY_SAMPLE_NEXT) || e->pf_valid;
        if (pf_path) {   // learn_step_inlaunch's bookkeeping
            if (!blk_kept(e, base)) e->wblk_dirty = true;
            if (!e->bucket_prefetch) {
                e->pf_valid = false;
                e->pf_inlaunch = false;
            } else {
                e->pf_stream = s;
            }
        }
        e->bucket_key = -1;
        return DQNX_OK;
    }
    const bool prefetch = (flags & DQNX_STEP_PREFETCH) != 0;
    const bool inl = inlaunch_prefetch_ok(e, base);
    if ((prefetch || e->pf_valid) && !(inl && (!e->pf_valid || e->pf_inlaunch)))
        return set_error(DQNX_EUNSUPPORTED, "bucketed step: the in-launch prefetch does not apply here");
    int key, k0;
    if (prefetch || e->pf_valid) {   // the in-launch pipeline (learn_step_inlaunch)
        if (e->pf_valid && s != e->pf_stream) DQNX_HIP_CHECK(hipStreamSynchronize(e->pf_stream));
        if (!e->pf_valid) {
            rc = inlaunch_prologue(e, base, s);
            if (rc) return rc;
        } else if (relayout_due(e)) {
            rc = enqueue_relayout(e, s);
            if (rc) return rc;
            e->wblk_dirty = false;
        }
        key = base | (prefetch ? KEY_SAMPLE_NEXT : 0);
        k0 = prefetch ? 0 : 1;
    } else {
        key = base | ((e->wblk_dirty || !blk_kept(e, base)) ? KEY_RELAYOUT : 0);
        k0 = 0;
    }
    const std::vector<KStep>& ks = steps_for(e, key);
    auto it = e->dw16_cache.find(key);
    if (ks.empty() || ks.back().name != "dw16_grads" || it == e->dw16_cache.end())
        return set_error(DQNX_ESTATE, "dp buckets: plan mismatch");
    rc = enqueue_range(ks, k0, (int)ks.size() - 1, s);
    if (rc) return rc;
    rc = launch_dw_adam16(dw16_subset(it->second, mlp_bucket_mask(e, 0), true, false), s);
    if (rc) return rc;
    if (!(prefetch || e->pf_valid)) e->wblk_dirty = false;   // (the sampler launch rebuilt the copies)
    e->bucket_key = key;
    e->bucket_prefetch = prefetch;
    return DQNX_OK;
}

int dqnx_learn_step_bucket(dqnx_engine* e, int32_t flags, int32_t bucket, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (flags & DQNX_STEP_GIVEN_INDICES) return set_error(DQNX_EUNSUPPORTED, "bucketed steps sample their own minibatch");
    std::vector<DpBucket> b;
    rc = dp_buckets(e, b);
    if (rc) return rc;
    if (bucket < 0 || bucket >= (int32_t)b.size()) return set_error(DQNX_EINVAL, "bucket %d out of range", bucket);
    if (bucket == 0 && e->ring_size < e->Bs && !e->pf_valid)
        return set_error(DQNX_EINVAL, "Sample larger than population: %lld < %d", (long long)e->ring_size, e->Bs);
    const bool mlp2 = b.size() == 2 && e->np.conv.empty();
    if (mlp2) return learn_step_bucket_mlp(e, flags, bucket, s);
    if (flags & DQNX_STEP_PREFETCH)
        return set_error(DQNX_EUNSUPPORTED, "bucketed conv-net steps sample their own minibatch, without prefetch");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "a prefetched minibatch is pending");
    // the plan of a plain GRADS_ONLY step (blocked-weight rebuild as that step decides)
    const int key = DQNX_STEP_GRADS_ONLY | ((e->bwd_plan == 2 && (e->wblk_dirty || !blk_kept(e, DQNX_STEP_GRADS_ONLY))) ? KEY_RELAYOUT : 0);
    const std::vector<KStep>& ks = steps_for(e, key);
    const std::vector<KStep>& k0 = steps_for(e, DQNX_STEP_GRADS_ONLY);
    if (ks.size() != k0.size()) return set_error(DQNX_ESTATE, "dp buckets: plan mismatch");
    rc = enqueue_range(ks, b[bucket].k0, b[bucket].k1, s);
    if (rc) return rc;
    if (bucket == 0) e->wblk_dirty = false;
    if (ks.back().name == "dw16_grads") return DQNX_OK;   // it wrote the gradient and the loss
    AdamArgs aa;
    adam_kstep(e, DQNX_STEP_GRADS_ONLY, &aa);   // mode 0: this bucket's slab sums into DQNX_BUF_GRADS
    aa.e0 = b[bucket].first;
    aa.n_params = b[bucket].first + b[bucket].count;
    aa.with_loss = bucket == 0;
    if (bucket != 0) {
        aa.loss_partial = nullptr;
        aa.mtc = nullptr;
    }
    return launch_adam(aa, s);
}

int dqnx_apply_grads_bucket(dqnx_engine* e, int32_t flags, int32_t bucket, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    std::vector<DpBucket> b;
    rc = dp_buckets(e, b);
    if (rc) return rc;
    if (bucket < 0 || bucket >= (int32_t)b.size()) return set_error(DQNX_EINVAL, "bucket %d out of range", bucket);
    const dqnx_config& c = e->cfg;
    if (bucket == 0 && c.algo == DQNX_ALGO_PER_DOUBLE) {   // the tree update, once per step
        rc = enqueue_per_update(e, at<int32_t>(e, e->off[DQNX_BUF_BATCH_IDX]), s);
        if (rc) return rc;
    }
    e->perm_dirty = true;
    const bool mlp2 = b.size() == 2 && e->np.conv.empty();
    if (mlp2 && e->bwd_plan == 2 && e->pf_valid && e->pf_inlaunch && dw_adam16_on(e, DQNX_STEP_GRADS_ONLY) &&
        route_knob("DQNX_APPLY_TILES", 1) != 0) {
        // as dqnx_apply_grads with a draw pending: k_dw_adam16 apply tiles writing the blocked copies
        // (the next step has no sampler launch to rebuild them), this bucket's layers only
        AdamArgs aa;
        adam_kstep(e, DQNX_STEP_GRADS_ONLY, &aa);
        aa.mode = 2;
        aa.soft = (flags & DQNX_STEP_SOFT_UPDATE) ? 1 : 0;
        rc = launch_dw_adam16(dw16_subset(apply_dw16_args(e, aa), mlp_bucket_mask(e, bucket), true, true), s);
        if (rc) return rc;
        if (bucket == (int32_t)b.size() - 1) e->wblk_dirty = false;   // every blocked copy rewritten
        return DQNX_OK;
    }
    if (!adam_keeps_blk(e)) e->wblk_dirty = true;
    AdamArgs aa;
    adam_kstep(e, DQNX_STEP_GRADS_ONLY, &aa);
    aa.mode = 2;
    aa.soft = (flags & DQNX_STEP_SOFT_UPDATE) ? 1 : 0;
    aa.loss_partial = nullptr;
    aa.mtc = nullptr;
    aa.e0 = b[bucket].first;
    aa.n_params = b[bucket].first + b[bucket].count;
    aa.with_loss = bucket == 0;
    return launch_adam(aa, s);
}

int dqnx_soft_update(dqnx_engine* e, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    e->perm_dirty = true;
    e->wblk_dirty = true;   // the target copies change outside the Adam pass
    const float tau = (float)((double)e->cfg.tau * e->cfg.n_env);
    const float omt = (float)(1.0 - (double)e->cfg.tau * e->cfg.n_env);
    return launch_soft_update(at<float>(e, e->off[DQNX_BUF_TARGET_PARAMS]), at<float>(e, e->off[DQNX_BUF_PARAMS]),
                              e->np.P, tau, omt, (hipStream_t)stream);
}

int dqnx_hard_update(dqnx_engine* e, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    e->perm_dirty = true;
    e->wblk_dirty = true;
    DQNX_HIP_CHECK(hipMemcpyAsync(e->arena + e->off[DQNX_BUF_TARGET_PARAMS], e->arena + e->off[DQNX_BUF_PARAMS],
                                  (size_t)e->np.P * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return DQNX_OK;
}

// acting kernel geometry of a network (host only).  A two-stream net acts as its convs (one
// launch each, act_hybrid.hip) followed by the MLP acting kernel on F = cat(flatten(conv), macro).
static int act_plan_build(const dqnx_net_desc* net, NetPlan& np, ActArgs& a);

// act_plan for the acting path's every call (choose_actions: one per env step): the plans of the last
// few network descriptions this thread acted with, keyed by the description's bytes (planning a net --
// param layout, names -- costs ~3.4 us of host time, and dqnx_act_host / dqnx_agent_choose need it
// three times per call).  *npp points into the cache: valid until this thread plans 4 other nets.
static int act_plan(const dqnx_net_desc* net, const NetPlan** npp, ActArgs& a) {
    struct Entry {
        bool used = false;
        dqnx_net_desc desc;
        NetPlan np;
        ActArgs a;
        int rc = 0;
    };
    static thread_local Entry cache[4];
    static thread_local int next = 0;
    if (!net) return set_error(DQNX_EINVAL, "null net");
    for (Entry& en : cache) {
        if (en.used && !memcmp(&en.desc, net, sizeof(dqnx_net_desc))) {
            if (en.rc) {   // (re-raise its error message)
                NetPlan tmp;
                return act_plan_build(net, tmp, a);
            }
            *npp = &en.np;
            a = en.a;
            return DQNX_OK;
        }
    }
    Entry& en = cache[next];
    next = (next + 1) & 3;
    en.used = true;
    memcpy(&en.desc, net, sizeof(dqnx_net_desc));
    en.np = NetPlan();
    en.rc = act_plan_build(net, en.np, en.a);
    if (en.rc) return en.rc;
    *npp = &en.np;
    a = en.a;
    return DQNX_OK;
}

static int act_plan_build(const dqnx_net_desc* net, NetPlan& np, ActArgs& a) {
    int rc = plan_net(net, np);
    if (rc) return rc;
    memset(&a, 0, sizeof(a));
    a.D = net->kind == DQNX_NET_MLP ? net->obs_dim : np.dense[0].in;
    a.L = (int)np.dense.size(); a.A = net->n_actions; a.F = np.F;
    if (a.L > kActMaxDense) return set_error(DQNX_EUNSUPPORTED, "dqnx_act: more than %d dense layers", kActMaxDense);
    a.dueling = net->head == DQNX_HEAD_DUELING; a.act = net->activation;
    a.ld = std::max(a.D, a.A);
    for (int l = 0; l < a.L; l++) {
        a.in[l] = np.dense[l].in; a.out[l] = np.dense[l].out; a.off[l] = np.dense[l].off;
        a.ld = std::max(a.ld, a.out[l]);
    }
    a.ld = (a.ld + 3) & ~3;   // float4 LDS rows
    a.head_off = np.head_off;
    for (const ConvPlan& cp : np.conv) {   // each conv's row image + one channel's weights in LDS
        ActConvArgs ca;
        memset(&ca, 0, sizeof(ca));
        ca.Ci = cp.Ci; ca.Hi = cp.Hi; ca.Wi = cp.Wi; ca.Ho = cp.Ho; ca.Wo = cp.Wo; ca.kh = cp.kh; ca.kw = cp.kw;
        if (act_conv_lds_bytes(ca) > 64 * 1024)
            return set_error(DQNX_EUNSUPPORTED, "dqnx_act: conv input %dx%dx%d too large for the acting kernel",
                             cp.Ci, cp.Hi, cp.Wi);
    }
    return DQNX_OK;
}

// two-stream scratch: conv outputs of every conv but the last, F [n][D]; the MLP part follows
static uint64_t act_conv_scratch_bytes(const NetPlan& np, int n, int D) {
    uint64_t b = 0;
    for (size_t l = 0; l + 1 < np.conv.size(); l++)
        b += (uint64_t)n * np.conv[l].Co * np.conv[l].Ho * np.conv[l].Wo * 4;
    b += (uint64_t)n * D * 4;
    return (b + 255) / 256 * 256;
}

uint64_t dqnx_act_scratch_bytes(const dqnx_net_desc* net, int32_t n) {
    const NetPlan* npp = nullptr;
    ActArgs a;
    if (act_plan(net, &npp, a)) return 0;
    const NetPlan& np = *npp;
    const uint64_t mlp = act_scratch_bytes(n, a.out[0], a.ld, a.L, a.L >= 2 ? a.out[1] : 0);
    if (!mlp) return 0;
    return (net->kind == DQNX_NET_MLP ? 0 : act_conv_scratch_bytes(np, n, a.D)) + mlp;
}

// done_flag: the MLP acting kernel stores done_seq there (system scope) after the actions (dqnx_act_host)
static int act_impl(const dqnx_net_desc* net, const float* params, const float* obs, int32_t n, int32_t* actions,
                    float* values, void* scratch, uint64_t scratch_bytes, void* stream, uint32_t* done_flag,
                    uint32_t done_seq, bool* signals = nullptr);

int dqnx_act(const dqnx_net_desc* net, const float* params, const float* obs, int32_t n, int32_t* actions,
             float* values, void* scratch, uint64_t scratch_bytes, void* stream) {
    return act_impl(net, params, obs, n, actions, values, scratch, scratch_bytes, stream, nullptr, 0);
}

static int act_impl(const dqnx_net_desc* net, const float* params, const float* obs, int32_t n, int32_t* actions,
                    float* values, void* scratch, uint64_t scratch_bytes, void* stream, uint32_t* done_flag,
                    uint32_t done_seq, bool* signals) {
    const NetPlan* npp = nullptr;
    ActArgs a;
    if (signals) *signals = false;
    int rc = act_plan(net, &npp, a);
    if (rc) return rc;
    const NetPlan& np = *npp;
    if (n < 0 || (n > 0 && (!params || !obs || !actions || !scratch)))
        return set_error(DQNX_EINVAL, "dqnx_act: bad argument");
    const int R = n > 0 ? act_rows_per_block(n, a.ld) : 1;
    if (R == 0) return set_error(DQNX_EUNSUPPORTED, "dqnx_act: layer width %d does not fit LDS", a.ld);
    a.params = params; a.obs = obs; a.actions = actions; a.values = values; a.n = n;
    // the acting kernels store the completion word from row group 0 only when the launch has ONE row
    // group (n <= R rows per workgroup: R halves for inputs wider than 2048 / 4096 floats)
    a.done_flag = (net->kind == DQNX_NET_MLP && n <= R) ? done_flag : nullptr;
    if (signals) *signals = a.done_flag != nullptr && n > 0;
    a.done_seq = done_seq;
    if (n == 0) return DQNX_OK;
    const uint64_t need = dqnx_act_scratch_bytes(net, n);
    if (scratch_bytes < need || (scratch_bytes & 3) || ((uintptr_t)scratch & 15))
        return set_error(DQNX_EINVAL, "dqnx_act: scratch of %llu bytes too small or misaligned for n=%d",
                         (unsigned long long)scratch_bytes, n);
    char* sc = (char*)scratch;
    hipStream_t s = (hipStream_t)stream;
    if (net->kind == DQNX_NET_TWO_STREAM) {   // the conv stack, rows' CHW images through scratch
        const int NC = (int)np.conv.size();
        const float* in = obs;
        int64_t in_stride = net->obs_dim;
        int in_off = np.macro_len;   // the micro grid viewed as (c, h, w) (R:env/dqn_config.py:126-128)
        char* cur = sc;
        float* F = nullptr;
        {
            uint64_t b = 0;
            for (int l = 0; l + 1 < NC; l++) b += (uint64_t)n * np.conv[l].Co * np.conv[l].Ho * np.conv[l].Wo * 4;
            F = (float*)(sc + b);
        }
        for (int l = 0; l < NC; l++) {
            const ConvPlan& cp = np.conv[l];
            ActConvArgs ca;
            memset(&ca, 0, sizeof(ca));
            ca.in = in; ca.in_stride = in_stride; ca.in_off = in_off;
            ca.W = params + cp.off; ca.b = ca.W + (int64_t)cp.Co * cp.K;
            ca.n = n; ca.Ci = cp.Ci; ca.Hi = cp.Hi; ca.Wi = cp.Wi; ca.Co = cp.Co; ca.Ho = cp.Ho; ca.Wo = cp.Wo;
            ca.kh = cp.kh; ca.kw = cp.kw; ca.sh = cp.sh; ca.sw = cp.sw; ca.ph = cp.ph; ca.pw = cp.pw;
            if (l + 1 < NC) {
                ca.out = (float*)cur;
                ca.out_stride = (int64_t)cp.Co * cp.Ho * cp.Wo;
                cur += (uint64_t)n * ca.out_stride * 4;
            } else {   // flatten(conv) ++ macro = the dense input F (R:env/dqn_config.py:135-138)
                ca.out = F;
                ca.out_stride = a.D;
                ca.macro = obs;
                ca.macro_stride = net->obs_dim;
                ca.macro_len = np.macro_len;
            }
            rc = launch_act_conv(ca, s);
            if (rc) return rc;
            in = ca.out; in_stride = ca.out_stride; in_off = 0;
        }
        a.obs = F;
        const uint64_t cb = act_conv_scratch_bytes(np, n, a.D);
        sc += cb;
        scratch_bytes -= cb;
    }
    // activations from the start, tickets from the END (ticket g at bytes - 4(g+1)): a larger
    // call's activations never reach a smaller call's tickets, so every ticket word only ever
    // holds counts that the last arriver returns to zero, whatever n the buffer last served.
    a.scratch = (float*)sc;
    a.tickets = (uint32_t*)(sc + scratch_bytes) - 1;   // ticket g = tickets[-g]
    return launch_act(a, s);
}

// ---- drop-in Agent fast path ------------------------------------------------------------
int dqnx_rng_sample_words(const uint32_t* state625, int64_t n, int32_t k, uint32_t* out625, int64_t* words);
int dqnx_rng_advance(const uint32_t* state625, int64_t words, uint32_t* out625);

// the caller's state into the engine's pinned staging slot for the next dqnx_agent_launch
static int agent_pin_state(dqnx_engine* e, int32_t which, const uint32_t* state625) {
    if (!e->ag_rng_pin) {
        DQNX_HIP_CHECK(hipHostMalloc((void**)&e->ag_rng_pin, 2 * 625 * 4, hipHostMallocDefault));
        for (int i = 0; i < 2; i++) DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->ag_rng_ev[i], hipEventDisableTiming));
    }
    const int i = e->ag_slot ^= 1;
    if (e->ag_rng_live[i]) {   // that block's previous upload has run (two launches ago: long passed)
        DQNX_HIP_CHECK(hipEventSynchronize(e->ag_rng_ev[i]));
        e->ag_rng_live[i] = false;
    }
    memcpy(e->ag_rng_pin + 625 * i, state625, 625 * 4);
    e->ag_which = which;
    return DQNX_OK;
}

int dqnx_agent_stage_rng(dqnx_engine* e, int32_t which, const uint32_t* state625, int64_t* words) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (!state625 || !words || (which != DQNX_RNG_PY && which != DQNX_RNG_NP)) return set_error(DQNX_EINVAL, "bad argument");
    if (state625[624] > 624) return set_error(DQNX_EINVAL, "MT index must be <= 624");
    if (e->pf_valid) return set_error(DQNX_ESTATE, "agent stage while a prefetched minibatch is pending");
    if (which == DQNX_RNG_PY) {   // random.sample(deque, batch_size): refused like CPython (k > n)
        rc = dqnx_rng_sample_words(state625, e->ring_size, e->Bs, e->ag_expect, words);
    } else {                      // np.random.uniform once per sample: 2 words each
        *words = 2 * (int64_t)e->Bg;
        rc = dqnx_rng_advance(state625, *words, e->ag_expect);
    }
    if (rc) return rc;
    rc = agent_pin_state(e, which, state625);
    if (rc) return rc;
    e->ag_expect_live = true;
    return DQNX_OK;
}

static int agent_launch_impl(dqnx_engine* e, int32_t flags, void* stream, int* prev_rc);

int dqnx_agent_learn_mt(dqnx_engine* e, uint32_t* mt, int32_t* pos, int32_t flags, void* stream, int64_t* words) {
    if (!mt || !pos || !words) return set_error(DQNX_EINVAL, "bad argument");
    if (*pos < 0 || *pos > 624) return set_error(DQNX_EINVAL, "MT position must be in [0, 624]");
    uint32_t s625[625];
    memcpy(s625, mt, 624 * 4);
    s625[624] = (uint32_t)*pos;
    int rc;
    if (flags & DQNX_AGENT_LAUNCH) {
        // the device only needs the state BEFORE the draw: stage it and launch first, then walk the draw
        // on the host while the GPU runs the step (the walk of a 1024-row draw is ~7 us)
        rc = check_bound(e);
        if (rc) return rc;
        if (e->pf_valid) return set_error(DQNX_ESTATE, "agent stage while a prefetched minibatch is pending");
        if ((int64_t)e->Bs > e->ring_size) return set_error(DQNX_EINVAL, "Sample larger than population or is negative");
        rc = agent_pin_state(e, DQNX_RNG_PY, s625);
        if (rc) return rc;
        e->ag_expect_live = false;   // (the check below is armed after the walk)
        int prev_rc;
        rc = agent_launch_impl(e, flags & ~DQNX_AGENT_LAUNCH, stream, &prev_rc);
        if (rc) return rc;
        rc = dqnx_rng_sample_words(s625, e->ring_size, e->Bs, e->ag_check, words);
        if (rc) return rc;
        e->ag_check_live = true;
        e->ag_check_which = DQNX_RNG_PY;
        memcpy(mt, e->ag_check, 624 * 4);   // the caller's generator moves past the draw
        *pos = (int32_t)e->ag_check[624];
        return prev_rc;   // the launched step's draw is mirrored; the previous step's checks raise
    }
    rc = dqnx_agent_stage_rng(e, DQNX_RNG_PY, s625, words);
    if (rc) return rc;
    // the caller's generator moves past the draw now (what random.sample would have consumed)
    memcpy(mt, e->ag_expect, 624 * 4);
    *pos = (int32_t)e->ag_expect[624];
    return DQNX_OK;
}

// the checks of a completed control-block readback: sticky device error, then the device sampler's
// RNG state against the host mirror of the draw
static int agent_check_ctrl(dqnx_engine* e, dqnx_ctrl* out) {
    const dqnx_ctrl* c = e->ag_ctrl_pin;
    if (out) memcpy(out, c, sizeof(dqnx_ctrl));
    const bool check = e->ag_check_live;
    e->ag_check_live = false;
    if (c->error) return set_error(DQNX_EDEVICE, "device error %d", c->error);
    if (check) {
        const uint32_t* got = e->ag_check_which == DQNX_RNG_PY ? c->py_mt : c->np_mt;
        if (memcmp(got, e->ag_check, sizeof(e->ag_check)))
            return set_error(DQNX_EDEVICE, "the device sampler's RNG state differs from the host mirror of the draw");
    }
    return DQNX_OK;
}

// *prev_rc: the checks of the previous step's unread readback (this step is launched either way)
static int agent_launch_impl(dqnx_engine* e, int32_t flags, void* stream, int* prev_rc) {
    *prev_rc = DQNX_OK;
    int rc = check_bound(e);
    if (rc) return rc;
    if (e->ag_which < 0) return set_error(DQNX_ESTATE, "dqnx_agent_launch without a staged RNG state");
    hipStream_t s = (hipStream_t)stream;
    const int i = e->ag_slot;
    // uniform replay, no draw pending: the sampler launch reads the staged state in place from a
    // fine-grained pinned block (no upload copy call); other configurations upload it into ctrl
    const bool zc = e->ag_which == DQNX_RNG_PY && !e->pf_valid && e->cfg.algo != DQNX_ALGO_PER_DOUBLE &&
                    route_knob("DQNX_AGENT_ZC", 1) != 0;
    if (zc) {
        if (!e->ag_rng_zc) DQNX_HIP_CHECK(hipHostMalloc((void**)&e->ag_rng_zc, 625 * 4, hipHostMallocCoherent));
        if (e->ag_zc_used) DQNX_HIP_CHECK(hipEventSynchronize(e->ag_ctrl_ev));   // its last reader has run
        memcpy(e->ag_rng_zc, e->ag_rng_pin + 625 * i, 625 * 4);
        e->ag_zc_launch = true;
        rc = dqnx_learn_step(e, flags & (DQNX_STEP_SOFT_UPDATE | DQNX_STEP_GRADS_ONLY), stream);
        e->ag_zc_launch = false;
        if (rc) return rc;
        e->ag_zc_used = true;
    } else {
        uint32_t* dst = e->ag_which == DQNX_RNG_PY ? ctrl_of(e)->py_mt : ctrl_of(e)->np_mt;
        DQNX_HIP_CHECK(hipMemcpyAsync(dst, e->ag_rng_pin + 625 * i, 625 * 4, hipMemcpyHostToDevice, s));
        DQNX_HIP_CHECK(hipEventRecord(e->ag_rng_ev[i], s));
        e->ag_rng_live[i] = true;
        rc = dqnx_learn_step(e, flags & (DQNX_STEP_SOFT_UPDATE | DQNX_STEP_GRADS_ONLY), stream);
        if (rc) return rc;
    }
    if (!e->ag_ctrl_pin) {
        DQNX_HIP_CHECK(hipHostMalloc((void**)&e->ag_ctrl_pin, sizeof(dqnx_ctrl), hipHostMallocDefault));
        DQNX_HIP_CHECK(hipEventCreateWithFlags(&e->ag_ctrl_ev, hipEventDisableTiming));
    }
    if (e->ag_ctrl_live) {   // the previous step's readback was never read: check it before it is overwritten
        DQNX_HIP_CHECK(hipEventSynchronize(e->ag_ctrl_ev));
        e->ag_ctrl_live = false;
        *prev_rc = agent_check_ctrl(e, nullptr);
    }
    DQNX_HIP_CHECK(hipMemcpyAsync(e->ag_ctrl_pin, ctrl_of(e), sizeof(dqnx_ctrl), hipMemcpyDeviceToHost, s));
    DQNX_HIP_CHECK(hipEventRecord(e->ag_ctrl_ev, s));
    e->ag_ctrl_live = true;
    e->ag_check_live = e->ag_expect_live;
    e->ag_check_which = e->ag_which;
    memcpy(e->ag_check, e->ag_expect, sizeof(e->ag_check));
    e->ag_expect_live = false;
    e->ag_which = -1;
    return DQNX_OK;
}

int dqnx_agent_launch(dqnx_engine* e, int32_t flags, void* stream) {
    int prev_rc;
    const int rc = agent_launch_impl(e, flags, stream, &prev_rc);
    return rc ? rc : prev_rc;
}

int dqnx_agent_quiesce(dqnx_engine* e) {
    if (!e) return set_error(DQNX_EINVAL, "null engine");
    // the waits agent_launch_impl would make (the previous step's unread control-block readback, the
    // last reader of the zero-copy RNG block), made here instead: callers reach this through a binding
    // that releases the GIL, so dqnx_agent_learn_mt (GIL held) finds them complete
    if (e->ag_ctrl_ev && (e->ag_ctrl_live || e->ag_zc_used)) DQNX_HIP_CHECK(hipEventSynchronize(e->ag_ctrl_ev));
    return DQNX_OK;
}

int dqnx_agent_readback(dqnx_engine* e, int32_t wait, dqnx_ctrl* out) {
    if (!e) return set_error(DQNX_EINVAL, "null engine");
    if (!e->ag_ctrl_live) return 0;
    if (wait) {
        DQNX_HIP_CHECK(hipEventSynchronize(e->ag_ctrl_ev));
    } else {
        const hipError_t q = hipEventQuery(e->ag_ctrl_ev);
        if (q == hipErrorNotReady) return 0;
        if (q != hipSuccess) return set_hip_error(q, "hipEventQuery", __FILE__, __LINE__);
    }
    e->ag_ctrl_live = false;
    const int rc = agent_check_ctrl(e, out);
    return rc ? rc : 1;
}

uint64_t dqnx_act_host_scratch_bytes(const dqnx_net_desc* net, int32_t n) {
    const uint64_t a = dqnx_act_scratch_bytes(net, n);
    if (!a || !net || n < 0) return 0;
    return a + ((uint64_t)n * net->obs_dim * 4 + 255) / 256 * 256 + ((uint64_t)n * 4 + 255) / 256 * 256;
}

// dqnx_act_host in two halves: the launch (obs into the pinned block, one acting launch sequence) and
// the wait (the completion word polled, or the stream synchronised), with the host free in between
// (dqnx_agent_choose draws the epsilon-greedy words there)
struct ActHostCall {
    char* pin = nullptr;
    int32_t* pa = nullptr;
    volatile uint32_t* flag = nullptr;
    uint32_t want_seq = 0;
    bool signals = false, direct = false;
    int32_t n = 0;
    hipStream_t s = nullptr;
};

static int act_host_launch(const dqnx_net_desc* net, const float* params, const float* obs_host, int32_t n,
                           void* scratch, uint64_t scratch_bytes, void* stream, ActHostCall& c) {
    if (!net || (n > 0 && (!params || !obs_host || !scratch))) return set_error(DQNX_EINVAL, "bad argument");
    if (n <= 0) return n == 0 ? DQNX_OK : set_error(DQNX_EINVAL, "n < 0");
    const uint64_t need = dqnx_act_host_scratch_bytes(net, n);
    if (!need) return set_error(DQNX_EUNSUPPORTED, "dqnx_act_host: network not supported by the acting kernel");
    if (scratch_bytes < need) return set_error(DQNX_EINVAL, "dqnx_act_host: scratch too small (%llu < %llu)",
                                                (unsigned long long)scratch_bytes, (unsigned long long)need);
    const uint64_t ob = ((uint64_t)n * net->obs_dim * 4 + 255) / 256 * 256, ab = ((uint64_t)n * 4 + 255) / 256 * 256;
    // obs and actions at the START, the acting scratch after them: dqnx_act keeps its arrival tickets at
    // the END of the scratch it is given, which is then the end of the caller's buffer for every n (a
    // call's obs never lands on the tickets another n's call uses; tests/test_gpu_act.py)
    char* sc = (char*)scratch;
    float* d_obs = (float*)sc;
    int32_t* d_act = (int32_t*)(sc + ob);
    void* act_sc = sc + ob + ab;
    const uint64_t act_bytes = scratch_bytes - ob - ab;
    // pinned staging, per thread, grown as needed: [obs n x D][actions n][completion word]
    static thread_local char* pin = nullptr;
    static thread_local size_t pin_bytes = 0;
    static thread_local uint32_t seq = 0;
    const size_t flag_at = ((size_t)n * net->obs_dim * 4 + (size_t)n * 4 + 63) / 64 * 64;
    const size_t want = flag_at + 64;
    hipStream_t s = (hipStream_t)stream;
    if (pin_bytes < want) {
        if (pin) {
            DQNX_HIP_CHECK(hipStreamSynchronize(s));
            (void)hipHostFree(pin);
            pin = nullptr;
            pin_bytes = 0;
        }
        DQNX_HIP_CHECK(hipHostMalloc((void**)&pin, want, hipHostMallocCoherent));
        pin_bytes = want;
    }
    c.pin = pin;
    c.n = n;
    c.s = s;
    c.pa = (int32_t*)(pin + (size_t)n * net->obs_dim * 4);
    memcpy(pin, obs_host, (size_t)n * net->obs_dim * 4);
    if (net->kind == DQNX_NET_MLP) {
        // one launch: the acting kernel reads the obs from and writes the actions to the pinned,
        // fine-grained block in place (no copy calls) and then a completion word, which the host
        // polls instead of synchronising the stream (the wake-up of a stream synchronisation costs
        // more than the kernel); a kernel that never signals ends the poll after ~0.5 s, and the
        // stream synchronisation then reports its error
        c.direct = true;
        c.flag = (volatile uint32_t*)(pin + flag_at);
        c.want_seq = ++seq ? seq : ++seq;   // (never 0)
        *c.flag = 0;   // (a grown or reused block never holds a stale word, whatever its sequence)
        return act_impl(net, params, (const float*)pin, n, c.pa, nullptr, act_sc, act_bytes, stream,
                        (uint32_t*)(pin + flag_at), c.want_seq, &c.signals);
    }
    DQNX_HIP_CHECK(hipMemcpyAsync(d_obs, pin, (size_t)n * net->obs_dim * 4, hipMemcpyHostToDevice, s));
    int rc = act_impl(net, params, d_obs, n, d_act, nullptr, act_sc, act_bytes, stream, nullptr, 0);
    if (rc) return rc;
    DQNX_HIP_CHECK(hipMemcpyAsync(c.pa, d_act, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    return DQNX_OK;
}

static int act_host_wait(ActHostCall& c) {
    if (c.n <= 0) return DQNX_OK;
    // poll only a launch that stores the word (one row group); any other waits on the stream
    bool seen = false;
    if (c.direct && c.signals && route_knob("DQNX_ACT_POLL", 1) != 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t it = 0;; it++) {
            if (__atomic_load_n(c.flag, __ATOMIC_ACQUIRE) == c.want_seq) { seen = true; break; }
            if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) break;
            __builtin_ia32_pause();
        }
    }
    if (!seen) DQNX_HIP_CHECK(hipStreamSynchronize(c.s));
    return DQNX_OK;
}

int dqnx_act_host(const dqnx_net_desc* net, const float* params, const float* obs_host, int32_t n,
                  int32_t* actions_host, void* scratch, uint64_t scratch_bytes, void* stream) {
    if (n > 0 && !actions_host) return set_error(DQNX_EINVAL, "bad argument");
    ActHostCall c;
    int rc = act_host_launch(net, params, obs_host, n, scratch, scratch_bytes, stream, c);
    if (rc || n <= 0) return rc;
    rc = act_host_wait(c);
    if (rc) return rc;
    memcpy(actions_host, c.pa, (size_t)n * 4);
    return DQNX_OK;
}

// The GIL, when the caller holds it (DQNX_CHOOSE_GIL_HELD): released around the GPU wait through the
// interpreter's own PyEval_SaveThread / PyEval_RestoreThread, looked up in the process (no link-time
// dependency on libpython; absent outside a Python process, where the flag is not passed)
struct GilRelease {
    void* ts = nullptr;
    void (*restore)(void*) = nullptr;
    explicit GilRelease(bool held) {
        if (!held) return;
        static void* (*save_fn)() = (void* (*)())dlsym(RTLD_DEFAULT, "PyEval_SaveThread");
        static void (*restore_fn)(void*) = (void (*)(void*))dlsym(RTLD_DEFAULT, "PyEval_RestoreThread");
        if (save_fn && restore_fn) {
            restore = restore_fn;
            ts = save_fn();
        }
    }
    ~GilRelease() {
        if (restore) restore(ts);
    }
};

// CPython's random.random() (genrand_res53) and randint(0, m - 1) = randrange(m) = _randbelow(m)
// (getrandbits(m.bit_length()) redrawn while >= m, Lib/random.py), on the caller's live MT19937
static inline uint32_t py_mt_next(uint32_t* w, int32_t* pos) {
    if (*pos >= 624) {
        for (int i = 0; i < 624; i++) {   // CPython genrand_uint32's regeneration, in index order
            const uint32_t y = (w[i] & 0x80000000u) | (w[(i + 1) % 624] & 0x7fffffffu);
            w[i] = w[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        *pos = 0;
    }
    uint32_t y = w[(*pos)++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    return y ^ (y >> 18);
}

int dqnx_agent_choose(dqnx_engine* e, const float* obs_host, int32_t n, double epsilon, uint32_t* mt, int32_t* pos,
                      int32_t* actions_out, void* scratch, uint64_t scratch_bytes, int32_t flags, void* stream) {
    int rc = check_bound(e);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!obs_host || !actions_out)) || !mt || !pos) return set_error(DQNX_EINVAL, "bad argument");
    if (*pos < 0 || *pos > 624) return set_error(DQNX_EINVAL, "MT position must be in [0, 624]");
    if (n > DQNX_CHOOSE_MAX_ENVS) return set_error(DQNX_EINVAL, "n > %d environments", DQNX_CHOOSE_MAX_ENVS);
    const float* params = at<float>(e, e->off[DQNX_BUF_PARAMS]);
    ActHostCall c;
    rc = act_host_launch(&e->cfg.net, params, obs_host, n, scratch, scratch_bytes, stream, c);
    if (rc) return rc;
    // while the acting kernel runs: R:dqn/agent.py:95-97 for every env, in env order, on the live
    // generator (the draws do not depend on the greedy actions)
    int32_t rnd[DQNX_CHOOSE_MAX_ENVS];
    bool take[DQNX_CHOOSE_MAX_ENVS];
    const uint32_t m = (uint32_t)e->cfg.net.n_actions;
    int k = 0;
    while (k < 32 && ((uint64_t)1 << k) <= m) k++;   // m.bit_length()
    for (int i = 0; i < n; i++) {
        const uint32_t a = py_mt_next(mt, pos) >> 5, b = py_mt_next(mt, pos) >> 6;
        const double u = ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
        take[i] = u <= epsilon;
        if (take[i]) {
            uint32_t r;
            do {
                r = k ? py_mt_next(mt, pos) >> (32 - k) : 0;
            } while (r >= m && m > 0);
            rnd[i] = (int32_t)r;
        }
    }
    int prev_rc = DQNX_OK;
    {
        GilRelease gil((flags & DQNX_CHOOSE_GIL_HELD) != 0);
        rc = act_host_wait(c);
        // the last agent step's control block (its readback ran before the acting kernel on this stream)
        if (!rc && e->ag_ctrl_live) {
            const hipError_t q = hipEventSynchronize(e->ag_ctrl_ev);
            if (q != hipSuccess) rc = set_hip_error(q, "hipEventSynchronize", __FILE__, __LINE__);
        }
    }
    if (rc) return rc;
    if (e->ag_ctrl_live) {
        e->ag_ctrl_live = false;
        prev_rc = agent_check_ctrl(e, nullptr);
    }
    for (int i = 0; i < n; i++) actions_out[i] = take[i] ? rnd[i] : c.pa[i];
    return prev_rc;
}

int dqnx_debug_stamps(dqnx_engine* e, int64_t* out64, void* stream) {
#ifdef DQNX_STAMPS
    int rc = check_bound(e);
    if (rc) return rc;
    DQNX_HIP_CHECK(hipMemcpyAsync(out64, e->arena + e->ws_stamps, 64 * 8, hipMemcpyDeviceToHost, (hipStream_t)stream));
    DQNX_HIP_CHECK(hipMemsetAsync(e->arena + e->ws_stamps, 0, 64 * 8, (hipStream_t)stream));
    DQNX_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    return DQNX_OK;
#else
    (void)e; (void)out64; (void)stream;
    return set_error(DQNX_EUNSUPPORTED, "not a -DDQNX_STAMPS build");
#endif
}

}  // extern "C"
