// Micro-CNN kernels (gfx950) for the reference's HEAD Q-network body, TwoStreamHybridNetwork
// (R:env/dqn_config.py:66-143, network_config :148-193): 3x3 convs (padding 1, ELU) over the
// (2,27,5) micro grid viewed from x[:, 14:] (R:env/dqn_config.py:126-128), then
// cat(flatten_CHW(conv), macro) (:135-138).  The grid is small (2x27x5 -> 32x27x5 -> 64x14x5 ->
// 64x7x3), so a sample's whole activation stack fits in LDS, and the per-layer plan's column
// matrices, flatten / unflatten and col2im launches (102 us of the 355 us B=256 step) disappear:
//
//   k_micro_fwd  one workgroup = S samples of one stream (online(s), online(s'), target(s')):
//                conv 1 straight from the gathered ring rows, then conv 2, conv 3, each image in
//                LDS (NHWC) for the next; written out only where the backward reads them (stream
//                0's conv outputs) and as the dense input F = cat(flatten_CHW(last conv), macro).
//   k_micro_dx   one workgroup = S samples of stream 0: the data gradients, last conv first, each
//                strided conv split into its sub-pixel phases (a phase's pixels meet only the taps
//                that reach them, so no MFMA multiplies a structural zero), the previous conv's
//                ELU' in the epilogue; each dZ image stays in LDS for the next level and is written
//                out (NHWC) for the weight gradients.
//   k_micro_dw   weight + bias gradients of every conv in one launch: a workgroup = one 16-channel
//                co tile of one conv over a slice of samples, all 9 taps x every ci tile, each
//                sample's dZ / input images staged in LDS with the next sample's loads in flight;
//                one split-K slab per slice, summed in fixed slice order by the Adam pass.
//
// GEMM orientation: rows (the MFMA's A side) are output channels, columns are pixels, so a lane's
// accumulator holds 4 consecutive channels of one pixel and NHWC images are written as float4.
// Every contraction is v_mfma_f32_16x16x4_f32 (an exact fp32 fmaf chain, MI355X_MICROARCH.md §F32);
// sums run in a fixed order (no atomics): results are bitwise reproducible run to run.
#include "learn.hpp"
#include "sample_body.hpp"

namespace dqnx {

constexpr int MW = 4;          // waves per workgroup
constexpr int MTH = 64 * MW;   // threads per workgroup
constexpr int MNT = 8;         // pixel tiles per wave and conv (accumulator sets) the kernels carry
constexpr int MNT_FWD = 6;     // ... in the forward (3 workgroups per CU: <= 168 VGPRs without spills)
constexpr int MICRO_ZERO = 80; // zero floats at the end of LDS: out-of-range taps read 16 ci/co of them

__device__ __forceinline__ void micro_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float4 lds4(const float* lds, int off) { return *reinterpret_cast<const float4*>(lds + off); }

// ---- host-side geometry ------------------------------------------------------------------
static int mfma_tiles_fwd(const MicroConv* c, int nc, int S) {   // 16x16x4 MFMAs of one workgroup
    int n = 0;
    for (int l = 0; l < nc; l++) {
        const int Nt = (S * c[l].Ho * c[l].Wo + 15) / 16, Mt = c[l].Co / 16;
        const int ksteps = l == 0 ? (c[0].Ci * 9 + 3) / 4 : 9 * c[l].Ci / 4;
        n += Mt * Nt * ksteps;
    }
    return n;
}
static int max_tiles_per_wave_fwd(const MicroConv* c, int nc, int S) {
    int m = 0;
    for (int l = 0; l < nc; l++) {
        const int Nt = (S * c[l].Ho * c[l].Wo + 15) / 16, nst = MW / (c[l].Co / 16);
        m = std::max(m, (Nt + nst - 1) / nst);
    }
    return m;
}
static bool micro_geom_ok(const MicroConv* c, int nc) {
    if (nc < 2 || nc > MICRO_MAX_CONV) return false;
    for (int l = 0; l < nc; l++) {
        const int Mt = c[l].Co / 16;
        if (c[l].Co % 16 || Mt < 1 || Mt > MW || MW % Mt) return false;
        if (c[l].sh < 1 || c[l].sh > 2 || c[l].sw < 1 || c[l].sw > 2) return false;
        if (c[l].Ho != (c[l].Hi - 1) / c[l].sh + 1 || c[l].Wo != (c[l].Wi - 1) / c[l].sw + 1) return false;
        if (l > 0 && (c[l].Ci % 16 || c[l].Ci != c[l - 1].Co || c[l].Hi != c[l - 1].Ho || c[l].Wi != c[l - 1].Wo)) return false;
        if (l > 0 && (c[l].Ci / 16 > MW || MW % (c[l].Ci / 16))) return false;   // data-gradient row tiles
    }
    return c[0].Ci * 9 <= 64;
}
static int fwd_lds_floats(const MicroConv* c, int nc, int S, int* x0, int* zero, int* offs) {
    int cur = 0;
    for (int l = 0; l + 1 < nc; l++) {
        offs[l] = cur;
        cur += S * c[l].Ho * c[l].Wo * c[l].cs;
    }
    *x0 = cur;
    cur += (S * c[0].Ci * c[0].Hi * c[0].Wi + 3) & ~3;
    *zero = cur;
    return cur + MICRO_ZERO;
}

static int dx_lds_floats(const MicroConv* c, int nc, int S, int* lds_d, int* zero);
int micro_fwd_layout(MicroConv* c, int nc, int S, int* x0, int* zero) {
    int offs[MICRO_MAX_CONV] = {0, 0, 0};
    const int lf = fwd_lds_floats(c, nc, S, x0, zero, offs);
    for (int l = 0; l + 1 < nc; l++) c[l].lds = offs[l];
    return lf;
}
int micro_dx_layout(const MicroConv* c, int nc, int S, int* lds_d, int* zero) { return dx_lds_floats(c, nc, S, lds_d, zero); }

bool micro_plan(const MicroConv* convs, int nc, int Bl, int nstreams, int n_cu, int* S_out, int* lds_floats) {
    if (!micro_geom_ok(convs, nc)) return false;
    // pick S (samples per workgroup) for the shortest estimated time: the busiest CU runs
    // ceil(workgroups / CUs) workgroups back to back at the MFMA rate.  (2,27,5) at B=256 x 3
    // streams: S = 1 (768 workgroups, 3 per CU, 2682 MFMAs each) beats S = 3 (258 workgroups:
    // two CUs would run two, 6596 each) and S = 2.
    double best = 1e30;
    int bestS = 0;
    for (int S = 1; S <= 3; S++) {
        int x0, zero, offs[MICRO_MAX_CONV];
        const int lf = fwd_lds_floats(convs, nc, S, &x0, &zero, offs);
        if ((size_t)lf * 4 > 160 * 1024 || max_tiles_per_wave_fwd(convs, nc, S) > MNT_FWD) continue;
        const int wgs = nstreams * ((Bl + S - 1) / S);
        const double t = (double)((wgs + n_cu - 1) / n_cu) * mfma_tiles_fwd(convs, nc, S);
        if (t < best - 1e-9) { best = t; bestS = S; *lds_floats = lf; }
    }
    if (!bestS) return false;
    *S_out = bestS;
    return true;
}

// data-gradient workgroups: S samples of stream 0, dZ images of convs 1..nc-1 in LDS
static int dx_lds_floats(const MicroConv* c, int nc, int S, int* lds_d, int* zero) {
    int cur = 0;
    for (int l = 0; l < nc; l++) lds_d[l] = -1;
    for (int l = 1; l < nc; l++) {   // dZ of conv l (conv 1's dZ goes to HBM only)
        lds_d[l] = cur;
        cur += S * c[l].Ho * c[l].Wo * c[l].cs;
    }
    *zero = cur;
    return cur + MICRO_ZERO;
}
// data gradients: a wave owns (sub-pixel phase, a contiguous run of that phase's pixel tiles, a
// contiguous run of its ci row tiles): the phase's taps' weights are read by that phase's waves
// only, and a wave carries (row tiles) x (pixel tiles) independent accumulators.  Each phase's
// tiles x rows are split over its waves, the phases' splits chosen to minimise the busiest SIMD's
// MFMAs (wave w on SIMD w % 4), then the busiest wave's.  8 waves per workgroup (the default at
// one sample per workgroup: one workgroup per CU at B = 256, so 2 waves per SIMD hide each other's
// LDS / weight latency); DQNX_MDX_WAVES=4 keeps 4.
constexpr int MNT_DX = 4;      // pixel tiles per wave and level in the data-gradient kernel ...
constexpr int MACC_DX = 8;     // ... and row x pixel accumulator tiles (5 tiles spill)
constexpr int MWD_MAX = 8;     // waves per data-gradient workgroup (max)
static int dx_phase_tiles(const MicroConv& L, int ph, int S, int* taps) {
    const int pa = ph / L.sw, pc = ph - pa * L.sw;
    const int Hq = (L.Hi - pa + L.sh - 1) / L.sh, Wq = (L.Wi - pc + L.sw - 1) / L.sw;
    const int i0 = (pa + 1) % L.sh, j0 = (pc + 1) % L.sw;
    *taps = ((2 - i0) / L.sh + 1) * ((2 - j0) / L.sw + 1);
    return (S * Hq * Wq + 15) / 16;
}
static bool dx_assign(const MicroConv& L, int S, int nw, int* asg) {   // asg[nw]; nt = 0: idle wave
    const int nph = L.sh * L.sw, MT = L.Ci / 16;
    if (nph > nw || nph > 4) return false;
    int tiles[4], taps[4];
    for (int p = 0; p < nph; p++) tiles[p] = dx_phase_tiles(L, p, S, &taps[p]);
    // per phase: (tile split ts, row split rs) options
    struct Opt { int ts, rs; };
    std::vector<Opt> opts[4];
    for (int p = 0; p < nph; p++)
        for (int rs = 1; rs <= MT; rs *= 2) {
            if (MT % rs) continue;
            for (int ts = 1; ts <= std::min(tiles[p], nw); ts++) {
                const int nt = (tiles[p] + ts - 1) / ts;
                if (ts * rs <= nw && nt <= MNT_DX && nt * (MT / rs) <= MACC_DX) opts[p].push_back({ts, rs});
            }
        }
    for (int p = 0; p < nph; p++)
        if (opts[p].empty()) return false;
    long best = -1;
    int bw[MWD_MAX * 2], nbw = 0;
    int idx[4] = {0, 0, 0, 0};
    while (true) {
        int waves = 0;
        for (int p = 0; p < nph; p++) waves += opts[p][idx[p]].ts * opts[p][idx[p]].rs;
        if (waves <= nw) {
            // the waves (encoded) and their costs (MFMA k-steps: tiles x taps x rows)
            int enc[MWD_MAX], cost[MWD_MAX], n = 0;
            for (int p = 0; p < nph; p++) {
                const Opt o = opts[p][idx[p]];
                for (int j = 0; j < o.ts; j++) {
                    const int t0 = tiles[p] * j / o.ts, t1 = tiles[p] * (j + 1) / o.ts;
                    for (int r = 0; r < o.rs; r++) {
                        const int mw = MT / o.rs;
                        enc[n] = p | (t0 << 4) | ((t1 - t0) << 12) | ((r * mw) << 16) | (mw << 20);
                        cost[n++] = (t1 - t0) * taps[p] * mw;
                    }
                }
            }
            // heaviest first, each onto the least loaded SIMD with a free slot
            int order[MWD_MAX];
            for (int i = 0; i < n; i++) order[i] = i;
            std::sort(order, order + n, [&](int x, int y) { return cost[x] > cost[y] || (cost[x] == cost[y] && x < y); });
            int load[4] = {0, 0, 0, 0}, used[4] = {0, 0, 0, 0}, slot[MWD_MAX];
            const int per = nw / 4;
            for (int i = 0; i < n; i++) {
                int sbest = -1;
                for (int sd = 0; sd < 4; sd++)
                    if (used[sd] < per && (sbest < 0 || load[sd] < load[sbest])) sbest = sd;
                slot[order[i]] = sbest + 4 * used[sbest];
                used[sbest]++;
                load[sbest] += cost[order[i]];
            }
            int mx = 0, mwv = 0;
            for (int sd = 0; sd < 4; sd++) mx = std::max(mx, load[sd]);
            for (int i = 0; i < n; i++) mwv = std::max(mwv, cost[i]);
            const long key = (long)mx * 4096 + mwv;
            if (best < 0 || key < best) {
                best = key;
                nbw = nw;
                for (int w = 0; w < nw; w++) bw[w] = 0;   // idle: nt = 0
                for (int i = 0; i < n; i++) bw[slot[i]] = enc[i];
            }
        }
        int p = 0;
        while (p < nph && ++idx[p] == (int)opts[p].size()) idx[p++] = 0;
        if (p == nph) break;
    }
    if (best < 0) return false;
    for (int w = 0; w < nbw; w++) asg[w] = bw[w];
    return true;
}
static int dx_waves_knob() { return route_knob("DQNX_MDX_WAVES", 8) == 4 ? 4 : 8; }
bool micro_dx_plan(const MicroConv* convs, int nc, int Bl, int* S_out, int* lds_d, int* lds_floats) {
    if (!micro_geom_ok(convs, nc)) return false;
    (void)Bl;
    const int nw = dx_waves_knob();
    for (int S = 1; S <= 3; S++) {   // S = 1: one workgroup per sample (B = 256: one per CU)
        int zero, asg[MWD_MAX];
        const int lf = dx_lds_floats(convs, nc, S, lds_d, &zero);
        bool ok = (size_t)lf * 4 <= 160 * 1024;
        for (int l = 1; l < nc && ok; l++) ok = dx_assign(convs[l], S, nw, asg) && convs[l].Ci / 16 <= 4;
        if (ok) {
            *S_out = S;
            *lds_floats = lf;
            return true;
        }
    }
    return false;
}
void micro_dx_waves(MicroDxArgs& a) {
    a.nw = dx_waves_knob();
    for (int l = 1; l < a.nc; l++) dx_assign(a.c[l], a.S, a.nw, a.wasg[l]);
}

// weight gradients.  convs 2..: a workgroup = (ci tile, slice of samples), wave w owns co tile w
// (its 9 taps), the samples of a slice pass through LDS G at a time (dZ, the input image's ci tile
// with a zero border), the next stage's loads in flight.  conv 1: a workgroup = (up to MW
// (co tile, im2col column tile) pairs, slice), one sample at a time (micro_dw_first).
constexpr int DW_CSD = 16;    // extra floats per staged dZ pixel (convs 2..: Co + 16, b32 reads conflict-free)
constexpr int DW1_KS_MAX = 36, DW1_IMG_MAX = 1024;   // conv 1 body limits (micro_dw_first)
static int dw_per_sample_floats(const MicroDwLayer& L) {   // convs 2..
    const int PP = (L.Hi + 2) * (L.Wi + 2);
    return L.Ho * L.Wo * (L.Co + DW_CSD) + PP * 16;
}
static int dw_mfma_per_sample_wave(const MicroDwLayer& L, bool first) {   // MFMAs of one wave
    const int ks = (L.Ho * L.Wo + 3) / 4;
    return first ? ks : ks * 9;
}
static int dw_lds_floats(const MicroDwLayer& L, bool first, int G) {   // conv 1: G = samples per workgroup
    if (first) return 2 * ((L.Ci * (L.Hi + 2) * (L.Wi + 2) + 3) & ~3) + G;
    return 2 * ((G * dw_per_sample_floats(L) + 3) & ~3) + MICRO_ZERO;
}
constexpr int DW_DQ = 7;      // float4 of the staged dZ per thread and stage
constexpr int DW_XQ = 4;      // float4 of the staged input per thread and stage
int micro_dw_plan(MicroDwArgs& a, int n_cu) {
    // per conv: column tiles and the LDS stage size G; slices (below) = split-K slabs of the conv,
    // summed by the Adam pass in slice order
    for (int l = 0; l < a.nc; l++) {
        MicroDwLayer& L = a.L[l];
        const bool first = l == 0;
        const int Mt = L.Co / 16;
        if (!first && Mt > MW) return DQNX_EUNSUPPORTED;
        L.nct = first ? (L.Ci * 9 + 15) / 16 : L.Ci / 16;
        const int Pq = L.Ho * L.Wo, Pin = L.Hi * L.Wi;
        L.G = 0;
        if (first) {   // one sample per LDS stage, the dZ fragments in registers
            if ((Pq + 3) / 4 > DW1_KS_MAX || L.Ci * Pin > DW1_IMG_MAX || L.Ci * (L.Hi + 2) * (L.Wi + 2) >= 16384)
                return DQNX_EUNSUPPORTED;   // (16-bit byte offsets of the image pixels)
            L.G = 1;
        }
        // convs 2..: the largest stage (<= 8 samples) whose two buffers fit 80 KB (two workgroups
        // per CU) and whose loads fit the staging registers
        for (int G = 8; G >= 1 && !L.G; G--) {
            const bool regs = G * Pq * L.Co / 4 <= DW_DQ * MTH && G * Pin * 4 <= DW_XQ * MTH;
            if (regs && dw_lds_floats(L, false, G) * 4 <= 80 * 1024) L.G = G;
        }
        if (!L.G) return DQNX_EUNSUPPORTED;
        L.wo_mul = (65536 + L.Wo - 1) / L.Wo;
        for (int q = 0; q < Pq + 4; q++)
            if (((q * L.wo_mul) >> 16) != q / L.Wo) return DQNX_EUNSUPPORTED;
    }
    // samples per workgroup: minimise the makespan of the slowest workgroup, all workgroups resident
    // at once (two per CU).  Workgroup cost model (cycles): a fixed start (launch ramp, maps,
    // borders, the first loads), a per-stage latency (barriers, the exposed part of the next
    // stage's loads) and the MFMAs of one wave, two waves sharing a SIMD.
    auto wg_per_slice = [&](int l) {
        const MicroDwLayer& L = a.L[l];
        return l == 0 ? (L.nct * (L.Co / 16) + MW - 1) / MW : L.nct;
    };
    // (constants fitted to the per-conv timings of tools/dwexp.sh on the HEAD net: ~14K cycles of
    // start, MFMA issue ~1.5x the two-wave pipe time; conv 1 ~4.8K cycles per sample, refitted in
    // round 5 (tools/variants/mdw_spw3.txt: 11 samples per slice 30.7 us, 6-8 samples 26.5 us))
    auto cost = [&](int l, int spw) {
        const MicroDwLayer& L = a.L[l];
        if (l == 0) return 14000.0 + 4800.0 * spw;
        return 14000.0 + 2500.0 * ((spw + L.G - 1) / L.G) + 1.5 * 64.0 * dw_mfma_per_sample_wave(L, false) * spw;
    };
    auto spw_for = [&](int l, double T) {   // the most samples per workgroup within makespan T (0: none)
        int lo = 0, hi = a.Bl;
        while (lo < hi) {
            const int m = (lo + hi + 1) / 2;
            if (cost(l, m) <= T) lo = m;
            else hi = m - 1;
        }
        return lo;
    };
    auto wgs_at = [&](double T) {
        int64_t n = 0;
        for (int l = 0; l < a.nc; l++) {
            const int spw = spw_for(l, T);
            if (!spw) return (int64_t)1 << 40;
            n += (int64_t)((a.Bl + spw - 1) / spw) * wg_per_slice(l);
        }
        return n;
    };
    double Tlo = 0, Thi = 0;
    for (int l = 0; l < a.nc; l++) Thi = std::max(Thi, cost(l, a.Bl));
    if (wgs_at(Thi) <= 2 * n_cu)
        for (int it = 0; it < 60; it++) {
            const double m = 0.5 * (Tlo + Thi);
            if (wgs_at(m) <= 2 * n_cu) Thi = m;
            else Tlo = m;
        }
    int wg = 0, lf = 0;
    for (int l = 0; l < a.nc; l++) {
        MicroDwLayer& L = a.L[l];
        const bool first = l == 0;
        int spw = std::max(1, spw_for(l, Thi));
        spw = std::max(1, std::min(route_knob(l == 0 ? "DQNX_MDW_SPW0" : l == 1 ? "DQNX_MDW_SPW1" : "DQNX_MDW_SPW2", spw), a.Bl));
        L.skip = (tuning_knob("DQNX_MDW_SKIP", 0) >> l) & 1;
        L.spw = spw;
        L.slices = (a.Bl + spw - 1) / spw;
        L.wg0 = wg;
        wg += L.slices * wg_per_slice(l);
        L.pstride = (int64_t)L.Co * L.Ci * 9 + L.Co;
        lf = std::max(lf, dw_lds_floats(L, first, first ? L.spw : L.G));
        if (!first) lf = std::max(lf, MW * 16 * 144);   // the slab store's transpose rows
    }
    a.wgs = wg;
    a.lds_floats = lf;
    return (size_t)lf * 4 <= 160 * 1024 ? DQNX_OK : DQNX_EUNSUPPORTED;
}

// =====================================================================================
// Shared implicit-GEMM chunk loop
// =====================================================================================
// acc[t] += sum over nch 16-deep chunks of A (weights, float4 per lane from `wrow`) x B (float4
// per lane from LDS).  Chunk ch belongs to tap ch >> lcpt; `base_of(t, tap)` is tile t's LDS float
// offset of that tap (its 16-column block at +16*(ch & cpm)), `woff(ch)` the chunk's weight offset.
// Compile-time NTW: every tile's 4 MFMAs per chunk are independent chains interleaved across the
// tiles.
template <int NTW, class BaseFn, class WFn>
__device__ __forceinline__ void igemm_chunks(const float* lds, const float* wrow, int nch, int lcpt, BaseFn base_of,
                                             WFn woff, floatx4 (&acc)[NTW]) {
    // Register rings without copies (a copy of an in-flight load waits for it): weights in 4 named
    // slots (chunk ch in slot ch % 4, loaded two chunks ahead), B fragments in 2 named sets (chunk ch
    // in set ch % 2, loaded one chunk ahead); the loop is unrolled by 4 so every slot is a fixed
    // register set.  The chunk count is padded to a multiple of 4 with null taps (base_of returns the
    // zero block for a tap past the last; their weights are re-read in range) and every load is
    // unconditional, so the compiler's vmcnt / lgkmcnt waits stay exact.
    const int cpm = (1 << lcpt) - 1;
    const int n4 = (nch + 3) & ~3;
    int bs[NTW];
    float4 b0[NTW], b1[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        bs[t] = base_of(t, 0);
        b0[t] = lds4(lds, bs[t]);
        b1[t] = b0[t];
    }
    float4 w0 = ld4(wrow + woff(0));
    float4 w1 = ld4(wrow + woff(min(1, nch - 1)));
    float4 w2 = w1, w3 = w1;
    auto step = [&](int ch, const float4& wc, float4& wl, const float4 (&bc)[NTW], float4 (&bn)[NTW]) {
        const int nx = ch + 1;
        if ((nx & cpm) == 0) {
#pragma unroll
            for (int t = 0; t < NTW; t++) bs[t] = base_of(t, nx >> lcpt);
        }
        const int co = (nx & cpm) * 16;
#pragma unroll
        for (int t = 0; t < NTW; t++) bn[t] = lds4(lds, bs[t] + co);
        wl = ld4(wrow + woff(min(nx + 1, nch - 1)));
        // keep the loads ahead of this chunk's MFMAs: left alone, the scheduler sinks them below,
        // and the next chunk's MFMAs then wait for their full latency
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NTW; t++) acc[t] = mfma16x16x4(wc.x, bc[t].x, acc[t]);
#pragma unroll
        for (int t = 0; t < NTW; t++) acc[t] = mfma16x16x4(wc.y, bc[t].y, acc[t]);
#pragma unroll
        for (int t = 0; t < NTW; t++) acc[t] = mfma16x16x4(wc.z, bc[t].z, acc[t]);
#pragma unroll
        for (int t = 0; t < NTW; t++) acc[t] = mfma16x16x4(wc.w, bc[t].w, acc[t]);
    };
    for (int ch = 0; ch < n4; ch += 4) {
        step(ch, w0, w2, b0, b1);
        step(ch + 1, w1, w3, b1, b0);
        step(ch + 2, w2, w0, b0, b1);
        step(ch + 3, w3, w1, b1, b0);
    }
}

// igemm_chunks with MT row tiles per wave: row tile m's weights at wrow + m * wstr (MT float4
// per chunk, the same 4-slot ring), acc[m][t] += A_m x B_t
template <int MT, int NTW, class BaseFn, class WFn>
__device__ __forceinline__ void igemm_chunks_m(const float* lds, const float* wrow, int wstr, int nch, int lcpt,
                                               BaseFn base_of, WFn woff, floatx4 (&acc)[MT][NTW]) {
    const int cpm = (1 << lcpt) - 1;
    const int n4 = (nch + 3) & ~3;
    int bs[NTW];
    float4 b0[NTW], b1[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        bs[t] = base_of(t, 0);
        b0[t] = lds4(lds, bs[t]);
        b1[t] = b0[t];
    }
    float4 w0[MT], w1[MT], w2[MT], w3[MT];
#pragma unroll
    for (int m = 0; m < MT; m++) {
        w0[m] = ld4(wrow + m * wstr + woff(0));
        w1[m] = ld4(wrow + m * wstr + woff(min(1, nch - 1)));
        w2[m] = w1[m];
        w3[m] = w1[m];
    }
    auto step = [&](int ch, const float4 (&wc)[MT], float4 (&wl)[MT], const float4 (&bc)[NTW], float4 (&bn)[NTW]) {
        const int nx = ch + 1;
        if ((nx & cpm) == 0) {
#pragma unroll
            for (int t = 0; t < NTW; t++) bs[t] = base_of(t, nx >> lcpt);
        }
        const int co = (nx & cpm) * 16;
#pragma unroll
        for (int t = 0; t < NTW; t++) bn[t] = lds4(lds, bs[t] + co);
        const int wo = woff(min(nx + 1, nch - 1));
#pragma unroll
        for (int m = 0; m < MT; m++) wl[m] = ld4(wrow + m * wstr + wo);
        __builtin_amdgcn_sched_barrier(0);   // the loads ahead of this chunk's MFMAs
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int t = 0; t < NTW; t++) acc[m][t] = mfma16x16x4(wc[m].x, bc[t].x, acc[m][t]);
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int t = 0; t < NTW; t++) acc[m][t] = mfma16x16x4(wc[m].y, bc[t].y, acc[m][t]);
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int t = 0; t < NTW; t++) acc[m][t] = mfma16x16x4(wc[m].z, bc[t].z, acc[m][t]);
#pragma unroll
        for (int m = 0; m < MT; m++)
#pragma unroll
            for (int t = 0; t < NTW; t++) acc[m][t] = mfma16x16x4(wc[m].w, bc[t].w, acc[m][t]);
    };
    for (int ch = 0; ch < n4; ch += 4) {
        step(ch, w0, w2, b0, b1);
        step(ch + 1, w1, w3, b1, b0);
        step(ch + 2, w2, w0, b0, b1);
        step(ch + 3, w3, w1, b1, b0);
    }
}

// tiles of this wave: pixel tiles n0, n0 + nst, ... below Nt
__device__ __forceinline__ int wave_tiles(int Nt, int n0, int nst) { return Nt > n0 ? (Nt - n0 + nst - 1) / nst : 0; }

#define MICRO_DISPATCH6(ntw, CALL)                \
    switch (ntw) {                                \
        case 1: CALL(1); break;                   \
        case 2: CALL(2); break;                   \
        case 3: CALL(3); break;                   \
        case 4: CALL(4); break;                   \
        case 5: CALL(5); break;                   \
        case 6: CALL(6); break;                   \
        default: break;                           \
    }
#define MICRO_DISPATCH(ntw, CALL)                 \
    switch (ntw) {                                \
        case 7: CALL(7); break;                   \
        case 8: CALL(8); break;                   \
        default: MICRO_DISPATCH6(ntw, CALL) break; \
    }

// =====================================================================================
// Forward
// =====================================================================================
// bias + ELU of 4 consecutive channels.  ELU as exp(x) - 1 (v_exp_f32, a few VALU ops instead of
// the ~25 of expm1f): within ~1.2e-7 absolute of torch CPU's expm1 (x <= 0 only), the parity
// tolerance is 1e-5 -- as conv_ig.hip's epilogue
__device__ __forceinline__ float elu_fast(float x) { return x > 0.f ? x : __expf(x) - 1.f; }
__device__ __forceinline__ float4 bias_elu(const floatx4& a, const float4& b) {
    return make_float4(elu_fast(a[0] + b.x), elu_fast(a[1] + b.y), elu_fast(a[2] + b.z), elu_fast(a[3] + b.w));
}

// conv 1: K = Ci*9 <= 64 in torch order k = (ci, i, j); A = W straight from the parameters, B
// gathered per k-step from the CHW images (scalar LDS reads, zero outside the grid).  The lane's
// weights (k = 4 st + g, zero past K0) and bias are loaded with the input images (conv1_weights).
constexpr int MICRO_C1_KS = 16;   // k-steps of conv 1: Ci*9 <= 64
__device__ __forceinline__ void conv1_weights(const MicroConv& L, const float* P, int mt, float (&wv)[MICRO_C1_KS],
                                              float4& bv4) {
    const int lane = threadIdx.x & 63, i16 = lane & 15, g = lane >> 4, K0 = L.Ci * 9;
    const float* W = P + L.woff + (int64_t)(mt * 16 + i16) * K0;
#pragma unroll
    for (int st = 0; st < MICRO_C1_KS; st++) {
        const int k = 4 * st + g;
        const float w = W[k < K0 ? k : K0 - 1];   // unconditional (vmcnt)
        wv[st] = k < K0 ? w : 0.f;
    }
    const float* bias = P + L.woff + (int64_t)L.Co * K0 + mt * 16 + 4 * g;
    bv4 = make_float4(bias[0], bias[1], bias[2], bias[3]);
}
template <int NTW>
__device__ __forceinline__ void micro_conv1(const MicroFwdArgs& a, const MicroConv& L, float* lds, const float (&wv)[MICRO_C1_KS],
                                            float4 bv4, bool keep, int b0, int ns, int mt, int n0, int nst) {
    const int lane = threadIdx.x & 63, i16 = lane & 15, g = lane >> 4;
    const int Pq = L.Ho * L.Wo, img = L.Ci * L.Hi * L.Wi, HW = L.Hi * L.Wi, K0 = L.Ci * 9, ks = (K0 + 3) >> 2;
    const int npx = a.S * Pq;
    int r0[NTW], c0[NTW], xb[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (n0 + t * nst) * 16 + i16;
        const bool v = p < npx;
        const int sb = v ? p / Pq : 0, q = p - sb * Pq;
        const int ho = q / L.Wo, wo = q - ho * L.Wo;
        r0[t] = v ? ho * L.sh - 1 : -1000;
        c0[t] = wo * L.sw - 1;
        xb[t] = a.x0 + sb * img;
    }
    floatx4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < MICRO_C1_KS; st++) {
        if (st < ks) {
            const int k = 4 * st + g;
            const float av = wv[st];
            const int ci = k / 9, tap = k - 9 * ci, ti = tap / 3, tj = tap - 3 * ti;
            float bv[NTW];
#pragma unroll
            for (int t = 0; t < NTW; t++) {
                const int r = r0[t] + ti, c = c0[t] + tj;
                const bool ok = k < K0 && (unsigned)r < (unsigned)L.Hi && (unsigned)c < (unsigned)L.Wi;
                bv[t] = lds[ok ? xb[t] + ci * HW + r * L.Wi + c : a.zero];
            }
#pragma unroll
            for (int t = 0; t < NTW; t++) acc[t] = mfma16x16x4(av, bv[t], acc[t]);
        }
    }
    const int co0 = mt * 16 + 4 * g;
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (n0 + t * nst) * 16 + i16;
        if (p >= npx) continue;
        const int sb = p / Pq, q = p - sb * Pq;
        const float4 v = bias_elu(acc[t], bv4);
        *reinterpret_cast<float4*>(lds + L.lds + p * L.cs + co0) = v;
        if (keep && sb < ns) *reinterpret_cast<float4*>(L.hc + ((int64_t)(b0 + sb) * Pq + q) * L.Co + co0) = v;
    }
}

// conv l >= 1: C[co][p] = sum_(tap, ci) Wperm[co][tap][ci] * act_{l-1}[src(p, tap)][ci]
template <bool LAST, int NTW>
__device__ __forceinline__ void micro_conv(const MicroFwdArgs& a, const MicroConv& L, const MicroConv& Lp, float* lds,
                                           const float* P, int tgt, bool keep, int b0, int ns, float* F, int mt, int n0,
                                           int nst) {
    const int lane = threadIdx.x & 63, i16 = lane & 15, g = lane >> 4;
    const int Pq = L.Ho * L.Wo, Pin = L.Hi * L.Wi, npx = a.S * Pq;
    const int cpt = L.Ci >> 4, lcpt = cpt == 4 ? 2 : (cpt == 2 ? 1 : (cpt == 1 ? 0 : 3));
    int rb[NTW], cb[NTW], ib[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (n0 + t * nst) * 16 + i16;
        const bool v = p < npx;
        const int sb = v ? p / Pq : 0, q = p - sb * Pq;
        const int ho = q / L.Wo, wo = q - ho * L.Wo;
        rb[t] = v ? ho * L.sh - 1 : -1000;
        cb[t] = wo * L.sw - 1;
        ib[t] = sb * Pin;
    }
    const float* wrow = L.wp[tgt] + (int64_t)(mt * 16 + i16) * 9 * L.Ci + 4 * g;
    floatx4 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto base_of = [&](int t, int tap) {
        const int ti = tap / 3, tj = tap - 3 * ti;
        const int r = rb[t] + ti, c = cb[t] + tj;
        const bool ok = tap < 9 && (unsigned)r < (unsigned)L.Hi && (unsigned)c < (unsigned)L.Wi;
        return ok ? Lp.lds + (ib[t] + r * L.Wi + c) * Lp.cs + 4 * g : a.zero + 4 * g;
    };
    auto woff = [&](int ch) { return ch * 16; };   // [co][tap][ci]: chunk ch at tap*Ci + 16*cc = 16*ch
    igemm_chunks<NTW>(lds, wrow, 9 * cpt, lcpt, base_of, woff, acc);
    const int co0 = mt * 16 + 4 * g;
    const float* bias = P + L.woff + (int64_t)L.Co * L.Ci * 9 + co0;
    const float4 bv4 = make_float4(bias[0], bias[1], bias[2], bias[3]);
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (n0 + t * nst) * 16 + i16;
        if (p >= npx) continue;
        const int sb = p / Pq, q = p - sb * Pq;
        const float4 v = bias_elu(acc[t], bv4);
        if constexpr (LAST) {   // F row: flatten_CHW (R:env/dqn_config.py:135-137)
            if (sb < ns) {
                float* f = F + (int64_t)(b0 + sb) * a.strideF + (int64_t)co0 * Pq + q;
                f[0] = v.x;
                f[Pq] = v.y;
                f[2 * Pq] = v.z;
                f[3 * Pq] = v.w;
            }
        } else {
            *reinterpret_cast<float4*>(lds + L.lds + p * L.cs + co0) = v;
            if (keep && sb < ns) *reinterpret_cast<float4*>(L.hc + ((int64_t)(b0 + sb) * Pq + q) * L.Co + co0) = v;
        }
    }
}

// the sampler workgroup's LDS: the 3-block MT window, then a 4096-slot (value, position) table
constexpr int MICRO_SAMP_AH = 2, MICRO_SAMP_HS = 4096;
constexpr int MICRO_SAMP_TAB = ((int)sizeof(SampleLdsBase<MTH, MICRO_SAMP_AH>) + 63) / 64 * 64;
constexpr int MICRO_SAMP_LDS = MICRO_SAMP_TAB + 8 * MICRO_SAMP_HS;

template <int NC>
__global__ __launch_bounds__(MTH, 3) void k_micro_fwd(MicroFwdArgs a) {   // 3 waves per SIMD: 3 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (a.samp_on && blockIdx.x == 0) {
        // in-launch prefetch: the next step's random.sample (R:dqn/replay_memory.py:38-39) into the
        // staging slot.  It reads only the MT state and the ring's size / write pointer, which no
        // kernel of this step writes (push / rng_set are refused while a draw is pending).
        sample_uniform_body<MTH, MICRO_SAMP_HS, MICRO_SAMP_AH>(
            a.samp, *reinterpret_cast<SampleLdsBase<MTH, MICRO_SAMP_AH>*>(lds),
            reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(lds) + MICRO_SAMP_TAB));
        return;
    }
    const int bid = (int)blockIdx.x - (a.samp_on ? 1 : 0);
    const int sblk = a.samp_on ? 1 : 0;   // diagnostic stamps: the first compute workgroup
    DQNX_STAMP_BLK(a.stamps, 40, sblk);
    const int tid = threadIdx.x, wid = tid >> 6;
#ifdef DQNX_STAMPS
    if (a.stamps && blockIdx.x == (unsigned)sblk && (tid & 63) == 0) a.stamps[56 + wid] = (int64_t)__builtin_amdgcn_s_memtime();
#endif
    const int z = bid / a.groups, grp = bid - z * a.groups;
    const int s = a.stream_of[z];
    const int tgt = s == 2 ? 1 : 0;
    const bool keep = s == 0;
    const float* P = tgt ? a.tparams : a.params;
    const float* ring = s == 0 ? a.ring_obs : a.ring_next;
    float* F = a.F[z];
    const int b0 = grp * a.S, ns = min(a.S, a.Bl - b0);

    // (0) the micro grids of the S gathered rows -> LDS (CHW, zero past the batch); the F row tail
    //     = the macro features + zero padding (R:env/dqn_config.py:138: cat([cnn_out, macro])).
    //     One round of loads: the rows' offsets (uniform), then every grid / tail element of this
    //     thread's first batch and conv 1's weights are in flight together before any store.
    const MicroConv& C0 = a.c[0];
    const int c1_mt = wid % (C0.Co >> 4);
    float c1w[MICRO_C1_KS];
    float4 c1b;
    {
        const int img = C0.Ci * C0.Hi * C0.Wi, tot = a.S * img, tail = a.strideF - a.flat_cols, ttot = ns * tail;
        int64_t ro[3];
#pragma unroll
        for (int sb = 0; sb < 3; sb++) ro[sb] = (int64_t)a.phys[b0 + min(sb, ns - 1)] * a.ring_stride;
        auto row = [&](int sb) { return sb == 0 ? ro[0] : (sb == 1 ? ro[1] : ro[2]); };
        constexpr int GE = 4;   // grid elements per thread and batch
        auto gload = [&](int base, float (&v)[GE]) {
#pragma unroll
            for (int j = 0; j < GE; j++) {
                const int e = min(base + tid + j * MTH, tot - 1), sb = e / img;
                const float x = ring[row(sb) + a.macro_len + (e - sb * img)];   // unconditional (vmcnt)
                v[j] = sb < ns ? x : 0.f;
            }
        };
        auto gstore = [&](int base, const float (&v)[GE]) {
#pragma unroll
            for (int j = 0; j < GE; j++)
                if (base + tid + j * MTH < tot) lds[a.x0 + base + tid + j * MTH] = v[j];
        };
        auto tload = [&](int e) {
            if (tail == 0 || a.macro_len == 0) return 0.f;
            const int ec = min(e, max(ttot - 1, 0)), sb = ec / tail, m = ec - sb * tail;
            const float x = ring[row(sb) + min(m, a.macro_len - 1)];
            return m < a.macro_len ? x : 0.f;
        };
        auto tstore = [&](int e, float v) {
            if (e < ttot) {
                const int sb = e / tail, m = e - sb * tail;
                F[(int64_t)(b0 + sb) * a.strideF + a.flat_cols + m] = v;
            }
        };
        float v[GE];
        gload(0, v);
        const float tv = tload(tid);
        conv1_weights(C0, P, c1_mt, c1w, c1b);
        gstore(0, v);
        tstore(tid, tv);
        for (int base = GE * MTH; base < tot; base += GE * MTH) {   // grids past one batch (larger S)
            gload(base, v);
            gstore(base, v);
        }
        for (int e = tid + MTH; e < ttot; e += MTH) tstore(e, tload(e));
        if (tid < MICRO_ZERO) lds[a.zero + tid] = 0.f;
    }
    micro_barrier();
    DQNX_STAMP_BLK(a.stamps, 41, sblk);
    {   // (1) conv 1
        const MicroConv& L = a.c[0];
        const int Mt = L.Co >> 4, nst = MW / Mt, n0 = wid / Mt, mt = wid - n0 * Mt;
        const int ntw = wave_tiles((a.S * L.Ho * L.Wo + 15) >> 4, n0, nst);
#define C1(N) micro_conv1<N>(a, L, lds, c1w, c1b, keep, b0, ns, mt, n0, nst)
        MICRO_DISPATCH6(ntw, C1)
#undef C1
    }
    micro_barrier();
    DQNX_STAMP_BLK(a.stamps, 42, sblk);
    // (2) convs 2 .. NC, each from the previous conv's LDS image (constant layer indices)
    auto conv = [&](const MicroConv& L, const MicroConv& Lp, bool last) {
        const int Mt = L.Co >> 4, nst = MW / Mt, n0 = wid / Mt, mt = wid - n0 * Mt;
        const int ntw = wave_tiles((a.S * L.Ho * L.Wo + 15) >> 4, n0, nst);
        if (!last) {
#define CM(N) micro_conv<false, N>(a, L, Lp, lds, P, tgt, keep, b0, ns, F, mt, n0, nst)
            MICRO_DISPATCH6(ntw, CM)
#undef CM
            micro_barrier();
        } else {
#define CL(N) micro_conv<true, N>(a, L, Lp, lds, P, tgt, keep, b0, ns, F, mt, n0, nst)
            MICRO_DISPATCH6(ntw, CL)
#undef CL
        }
    };
    if constexpr (NC == 2) {
        conv(a.c[1], a.c[0], true);
    } else {
        conv(a.c[1], a.c[0], false);
        DQNX_STAMP_BLK(a.stamps, 43, sblk);
        conv(a.c[2], a.c[1], true);
    }
    DQNX_STAMP_BLK(a.stamps, 44, sblk);
}

int launch_micro_fwd(const MicroFwdArgs& a, hipStream_t s) {
    if (a.samp_on && a.samp.k > MICRO_SAMPLE_MAX_K)
        return set_error(DQNX_EUNSUPPORTED, "micro forward sampler workgroup: k <= %d", MICRO_SAMPLE_MAX_K);
    const dim3 grid(a.nstreams * a.groups + (a.samp_on ? 1 : 0));
    size_t lds = (size_t)a.lds_floats * 4;
    if (a.samp_on && lds < (size_t)MICRO_SAMP_LDS) lds = MICRO_SAMP_LDS;
    if (a.nc == 3) DQNX_LAUNCH(k_micro_fwd<3>, grid, dim3(MTH), lds, s, a);
    else DQNX_LAUNCH(k_micro_fwd<2>, grid, dim3(MTH), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// =====================================================================================
// Data gradients (stream 0): dZ_{l-1} = convT_l(dZ_l) (.) ELU'(h_{l-1}), l = NC-1 .. 1
// =====================================================================================
// Sub-pixel phases: an input pixel (r, c) of conv l with r % sh == pa, c % sw == pc is reached by
// the taps i = i0 + sh*u (i0 = (pa + 1) % sh), j = j0 + sw*v, from output pixel
// (yq + (pa + 1 - i0)/sh - u, xq + (pc + 1 - j0)/sw - v) where r = pa + sh*yq, c = pc + sw*xq.
// GEMM: rows = ci (A = W^T [ci][tap][co] from the mode-1 copy), columns = the phase's pixels,
// K = its taps x co (B = dZ_l image from LDS, float4 over co).
template <int MT, int NTW>
__device__ __forceinline__ void micro_dx_phase(const MicroDxArgs& a, const MicroConv& L, const MicroConv& Lp, float* lds,
                                               int l, int b0, int ns, int pa, int pc, int t0, int m0) {
    const int lane = threadIdx.x & 63, i16 = lane & 15, g = lane >> 4;
    const int Pq = L.Ho * L.Wo, Pin = L.Hi * L.Wi;
    const int Hq = (L.Hi - pa + L.sh - 1) / L.sh, Wq = (L.Wi - pc + L.sw - 1) / L.sw, HWq = Hq * Wq;
    const int i0 = (pa + 1) % L.sh, j0 = (pc + 1) % L.sw;
    const int ni = (2 - i0) / L.sh + 1, nj = (2 - j0) / L.sw + 1;
    const int npx = a.S * HWq;
    const int cpt = L.Co >> 4, lcpt = cpt == 4 ? 2 : (cpt == 2 ? 1 : (cpt == 1 ? 0 : 3));
    int yb[NTW], xb[NTW], ob[NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (t0 + t) * 16 + i16;
        const bool v = p < npx;
        const int sb = v ? p / HWq : 0, m = p - sb * HWq;
        const int yq = m / Wq, xq = m - yq * Wq;
        yb[t] = v ? yq + (pa + 1 - i0) / L.sh : -1000;
        xb[t] = xq + (pc + 1 - j0) / L.sw;
        ob[t] = sb * Pq;
    }
    const float* wrow = L.wT + (int64_t)(m0 * 16 + i16) * 9 * L.Co + 4 * g;   // row tile m: + m * 16 * 9 * Co
    const int ldz = a.lds_d[l];
    floatx4 acc[MT][NTW];
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
        for (int t = 0; t < NTW; t++) acc[m][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto base_of = [&](int t, int tu) {
        const int u = tu / nj, v = tu - u * nj;
        const int yo = yb[t] - u, xo = xb[t] - v;
        const bool ok = u < ni && (unsigned)yo < (unsigned)L.Ho && (unsigned)xo < (unsigned)L.Wo;
        return ok ? ldz + (ob[t] + yo * L.Wo + xo) * L.cs + 4 * g : a.zero + 4 * g;
    };
    auto woff = [&](int ch) {
        const int tu = ch >> lcpt, u = tu / nj, v = tu - u * nj;
        return ((i0 + L.sh * u) * 3 + j0 + L.sw * v) * L.Co + (ch & (cpt - 1)) * 16;
    };
    // conv l-1's outputs for the epilogue's ELU', loaded ahead of the GEMM (unconditional: pixels
    // outside re-read the tile's first valid one)
    int pixo[NTW], hrow[NTW];
    float4 hv[MT][NTW];
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        const int p = (t0 + t) * 16 + i16;
        const bool v = p < npx && p / HWq < ns;
        const int pc_ = v ? p : 0;
        const int sb = pc_ / HWq, mm = pc_ - sb * HWq;
        const int yq = mm / Wq, xq = mm - yq * Wq;
        pixo[t] = v ? sb * Pin + (pa + L.sh * yq) * L.Wi + pc + L.sw * xq : -1;
        hrow[t] = b0 * Pin + sb * Pin + (pa + L.sh * yq) * L.Wi + pc + L.sw * xq;
#pragma unroll
        for (int m = 0; m < MT; m++) hv[m][t] = ld4(Lp.hc + (int64_t)hrow[t] * L.Ci + (m0 + m) * 16 + 4 * g);
    }
    igemm_chunks_m<MT, NTW>(lds, wrow, 16 * 9 * L.Co, ni * nj * cpt, lcpt, base_of, woff, acc);
    // epilogue: ELU' of conv l-1's output (torch elu_backward on the result)
#pragma unroll
    for (int t = 0; t < NTW; t++) {
        if (pixo[t] < 0) continue;
#pragma unroll
        for (int m = 0; m < MT; m++) {
            const int ci0 = (m0 + m) * 16 + 4 * g;
            const int64_t go = (int64_t)hrow[t] * L.Ci + ci0;
            const float4 h = hv[m][t];
            const float4 d = make_float4(act_bwd<DQNX_ACT_ELU>(acc[m][t][0], h.x), act_bwd<DQNX_ACT_ELU>(acc[m][t][1], h.y),
                                         act_bwd<DQNX_ACT_ELU>(acc[m][t][2], h.z), act_bwd<DQNX_ACT_ELU>(acc[m][t][3], h.w));
            *reinterpret_cast<float4*>(Lp.dz + go) = d;
            if (l - 1 >= 1) *reinterpret_cast<float4*>(lds + a.lds_d[l - 1] + pixo[t] * Lp.cs + ci0) = d;
        }
    }
}

template <int NC, int NW>
__global__ __launch_bounds__(64 * NW) void k_micro_dx(MicroDxArgs a) {
    constexpr int MTH = 64 * NW;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    DQNX_STAMP(a.stamps, 47);
    const int tid = threadIdx.x, wid = tid >> 6;
    const int b0 = blockIdx.x * a.S, ns = min(a.S, a.Bl - b0);
    // (0) dZ of the last conv: the dF rows (flatten_CHW order) -> LDS (NHWC) and the HBM copy
    {   // batches of DE elements per thread, every load of a batch in flight before its stores
        const MicroConv& L = a.c[NC - 1];
        const int Pq = L.Ho * L.Wo, per = L.Co * Pq, tot = a.S * per;
        constexpr int DE = 8;
        for (int base = 0; base < tot; base += DE * MTH) {
            float v[DE];
#pragma unroll
            for (int j = 0; j < DE; j++) {
                const int e = min(base + tid + j * MTH, tot - 1), sb = e / per;
                const float x = a.dF[(int64_t)(b0 + min(sb, ns - 1)) * a.ldf + (e - sb * per)];   // unconditional (vmcnt)
                v[j] = sb < ns ? x : 0.f;
            }
#pragma unroll
            for (int j = 0; j < DE; j++) {
                const int e = base + tid + j * MTH;
                if (e >= tot) break;
                const int sb = e / per, rem = e - sb * per, co = rem / Pq, q = rem - co * Pq;
                if (sb < ns) L.dz[((int64_t)(b0 + sb) * Pq + q) * L.Co + co] = v[j];
                lds[a.lds_d[NC - 1] + (sb * Pq + q) * L.cs + co] = v[j];
            }
        }
        if (tid < MICRO_ZERO) lds[a.zero + tid] = 0.f;
    }
    micro_barrier();
    DQNX_STAMP(a.stamps, 48);
    // levels NC-1 .. 1 (constant layer indices); this wave's (phase, tile run) from the host plan
    auto level = [&](const MicroConv& L, const MicroConv& Lp, int l) {
        const int w = a.wasg[l][wid], ph = w & 15, t0 = (w >> 4) & 255, nt = (w >> 12) & 15;
        const int m0 = (w >> 16) & 15, mt = (w >> 20) & 15;
        const int pa = ph / L.sw, pc = ph - pa * L.sw;
#define DX(M, N) micro_dx_phase<M, N>(a, L, Lp, lds, l, b0, ns, pa, pc, t0, m0)
#define DXN(M)                      \
    switch (nt) {                   \
        case 1: DX(M, 1); break;    \
        case 2: DX(M, 2); break;    \
        case 3: DX(M, 3); break;    \
        case 4: DX(M, 4); break;    \
        default: break;             \
    }
        if (mt == 4) {   // at most MACC_DX / 4 tiles (host plan)
            switch (nt) {
                case 1: DX(4, 1); break;
                case 2: DX(4, 2); break;
                default: break;
            }
        } else if (mt == 2) {
            DXN(2)
        } else {
            DXN(1)
        }
#undef DXN
#undef DX
    };
    if constexpr (NC == 3) {
        level(a.c[2], a.c[1], 2);
        micro_barrier();
        DQNX_STAMP(a.stamps, 49);
    }
    level(a.c[1], a.c[0], 1);
    DQNX_STAMP(a.stamps, 50);
}

int launch_micro_dx(const MicroDxArgs& a, hipStream_t s) {
    const dim3 grid(a.groups);
    const size_t lds = (size_t)a.lds_floats * 4;
    if (a.nw == 8) {
        if (a.nc == 3) DQNX_LAUNCH((k_micro_dx<3, 8>), grid, dim3(512), lds, s, a);
        else DQNX_LAUNCH((k_micro_dx<2, 8>), grid, dim3(512), lds, s, a);
    } else {
        if (a.nc == 3) DQNX_LAUNCH((k_micro_dx<3, 4>), grid, dim3(256), lds, s, a);
        else DQNX_LAUNCH((k_micro_dx<2, 4>), grid, dim3(256), lds, s, a);
    }
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

// =====================================================================================
// Weight gradients: dW_l[co][ci][i][j] = sum_(b,q) dZ_l[b][q][co] * X_l[b][src(q,i,j)][ci],
// db_l[co] = sum dZ_l[b][q][co], over one slice of samples per workgroup
// =====================================================================================
// LDS per buffer: D [G][Ho*Wo][16] (the co tile) | X with a zero border: [G][(Hi+2)*(Wi+2)][16]
// (the ci tile; 16 floats per pixel: the two pixels of a ds_read_b32 lane group sit 16 banks
// apart) or, for conv 1, CHW planes [G][Ci][Hi+2][Wi+2]; the output tiles are the 9 taps of the
// ci tile (conv 1: one 16-column tile of the (ci, i, j) columns in torch order).
// floor(n / d) for 0 <= n < 2^22, d >= 1: v_rcp_f32 estimate, one correction step (a handful of
// VALU ops instead of the ~25 of an integer division by a runtime divisor)
__device__ __forceinline__ int udiv(int n, int d) {
    int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
    const int r = n - q * d;
    return q + (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
}

// convs 2..: workgroup = (ci tile ct, slice); wave w < Co/16 owns co tile w and its 9 tap tiles
__device__ __forceinline__ void micro_dw_body_ci(const MicroDwArgs& a, const MicroDwLayer& L, int rel, float* lds) {
    constexpr int NT = 9;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, i16 = lane & 15, g = lane >> 4;
    const int Mt = L.Co >> 4, ct = rel % L.nct, slice = rel / L.nct;
    const int mt = wid < Mt ? wid : 0;
    const bool active = wid < Mt;
    const int s0 = slice * L.spw, s1 = min(a.Bl, s0 + L.spw);
    const int Pq = L.Ho * L.Wo, Pin = L.Hi * L.Wi, G = L.G;
    const int PW = L.Wi + 2, PP = (L.Hi + 2) * PW;
    const int csD = L.Co + DW_CSD, dper = Pq * csD, xper = PP * 16;
    const int dsz = G * dper;
    const int bufsz = (dsz + G * xper + 3) & ~3, zero = 2 * bufsz;
    const int ks = (Pq + 3) >> 2;
    const int sblk = L.wg0;   // diagnostic stamps: this conv's first workgroup (conv 2: slots 53..58, conv 3: 0..5)
    const int sb_ = &L == &a.L[1] ? 53 : 0;
    DQNX_STAMP_BLK(a.stamps, sb_, sblk);
    for (int bb = 0; bb < 2; bb++)   // zero borders of both buffers
        for (int e = tid; e < G * xper; e += MTH) lds[bb * bufsz + dsz + e] = 0.f;
    if (tid < MICRO_ZERO) lds[zero + tid] = 0.f;
    int toff[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) toff[t] = dsz + ((t / 3) * PW + t % 3) * 16 + i16;
    // stage-invariant staging maps (sample of the stage: G = unused)
    const int c4 = L.Co >> 2;
    int dgg[DW_DQ], dsrc[DW_DQ], ddst[DW_DQ], xgg[DW_XQ], xsrc[DW_XQ], xdst[DW_XQ];
#pragma unroll
    for (int j = 0; j < DW_DQ; j++) {
        const int e = tid + j * MTH, gg = udiv(e, Pq * c4), rem = e - gg * Pq * c4, px = udiv(rem, c4), q4 = rem - px * c4;
        dgg[j] = gg < G ? gg : G;
        dsrc[j] = rem * 4;
        ddst[j] = gg * dper + px * csD + 4 * q4;
    }
#pragma unroll
    for (int j = 0; j < DW_XQ; j++) {
        const int e = tid + j * MTH, gg = udiv(e, Pin * 4), rem = e - gg * Pin * 4, pix = rem >> 2, part = rem & 3;
        const int r = udiv(pix, L.Wi), c = pix - r * L.Wi;
        xgg[j] = gg < G ? gg : G;
        xsrc[j] = pix * L.Ci + ct * 16 + 4 * part;
        xdst[j] = dsz + gg * xper + ((r + 1) * PW + c + 1) * 16 + 4 * part;
    }
    float4 dr[DW_DQ], xr[DW_XQ];
    auto gload = [&](int sb0) {
        const int nG = min(G, s1 - sb0);
#pragma unroll
        for (int j = 0; j < DW_DQ; j++)
            dr[j] = dgg[j] < nG ? ld4(L.D + (int64_t)(sb0 + dgg[j]) * Pq * L.Co + dsrc[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < DW_XQ; j++)
            xr[j] = xgg[j] < nG ? ld4(L.X + (int64_t)(sb0 + xgg[j]) * Pin * L.Ci + xsrc[j]) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto sstore = [&](int buf) {
        float* B = lds + buf * bufsz;
#pragma unroll
        for (int j = 0; j < DW_DQ; j++)
            if (dgg[j] < G) *reinterpret_cast<float4*>(B + ddst[j]) = dr[j];
#pragma unroll
        for (int j = 0; j < DW_XQ; j++)
            if (xgg[j] < G) *reinterpret_cast<float4*>(B + xdst[j]) = xr[j];
    };
    floatx4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float dbias = 0.f;
    DQNX_STAMP_BLK(a.stamps, sb_ + 1, sblk);
    gload(s0);
    micro_barrier();   // borders / zeros before the first store
    sstore(0);
    micro_barrier();
    DQNX_STAMP_BLK(a.stamps, sb_ + 2, sblk);
    int cur = 0;
    for (int sb0 = s0; sb0 < s1; sb0 += G) {
        const int cb = cur * bufsz, nG = min(G, s1 - sb0), T = nG * ks;
        if (sb0 + G < s1) gload(sb0 + G);   // the next stage in flight during this one's MFMAs
        if (active) {
            // step j = (sample j / ks, pixel 4 (j % ks) + g); the next step's operands are read while
            // this step's MFMAs issue (two named sets, no copies); steps past the stage read zeros
            int lg_ = 0, lst = 0;
            auto load = [&](int j, float& av, float (&bv)[NT]) {
                const int gg = lg_, px = 4 * lst + g;
                if (++lst == ks) {
                    lst = 0;
                    lg_++;
                }
                const bool okp = j < T && px < Pq;
                av = lds[okp ? cb + gg * dper + px * csD + mt * 16 + i16 : zero];
                const int ho = (px * L.wo_mul) >> 16, wo = px - ho * L.Wo;
                const int pb = okp ? (ho * L.sh * PW + wo * L.sw) * 16 + cb + gg * xper : cb;
#pragma unroll
                for (int t = 0; t < NT; t++) bv[t] = lds[pb + toff[t]];
            };
            auto mm = [&](float av, const float (&bv)[NT]) {
#pragma unroll
                for (int t = 0; t < NT; t++) acc[t] = mfma16x16x4(av, bv[t], acc[t]);
            };
            float a0, a1, v0[NT], v1[NT];
            load(0, a0, v0);
            for (int j = 0; j < T; j += 2) {
                load(j + 1, a1, v1);
                __builtin_amdgcn_sched_barrier(0);   // the next step's reads ahead of these MFMAs
                mm(a0, v0);
                load(j + 2, a0, v0);
                __builtin_amdgcn_sched_barrier(0);
                if (j + 1 < T) mm(a1, v1);
            }
            if (ct == 0)   // db partials: pixels q = g, g + 4, ... of every sample of the stage
                for (int gg = 0; gg < nG; gg++)
                    for (int q = g; q < Pq; q += 4) dbias += lds[cb + gg * dper + q * csD + mt * 16 + i16];
        }
        micro_barrier();   // every read of the other buffer's previous stage is done
        if (sb0 == s0) DQNX_STAMP_BLK(a.stamps, sb_ + 3, sblk);
        if (sb0 + G < s1) {
            sstore(cur ^ 1);
            micro_barrier();
        }
        cur ^= 1;
    }
    DQNX_STAMP_BLK(a.stamps, sb_ + 4, sblk);
    if (!active) return;
    // bounds check: the tile's slab rows lie inside its conv's [slices][Co*Ci*9 + Co]
    if (slice >= L.slices || mt * 16 + 16 > L.Co || ct * 16 + 16 > L.Ci ||
        (int64_t)L.Co * L.Ci * 9 + L.Co > L.pstride) {
        if (lane == 0 && a.err) __hip_atomic_store(a.err, (int32_t)DQNX_DEVERR_BOUNDS_MICRO_DW, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    float* part = L.partial + (int64_t)slice * L.pstride;
    // the wave's 16 co x (16 ci x 9 taps) outputs are 16 runs of 144 contiguous floats of the slab
    // ([co][ci][i][j]): transposed through the wave's own LDS rows (the stages' buffers are free
    // after the loop's last barrier), then written as whole float4s
    {
        float* w = lds + wid * 16 * 144;
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int r = 0; r < 4; r++) w[(4 * g + r) * 144 + i16 * 9 + t] = acc[t][r];
        float* dst = part + ((int64_t)(mt * 16) * L.Ci + ct * 16) * 9;
#pragma unroll
        for (int j = 0; j < 9; j++) {   // 16 rows x 36 float4 = 576 = 9 per lane
            const int q = lane + 64 * j, row = q / 36, c4 = q - row * 36;
            *reinterpret_cast<float4*>(dst + (int64_t)row * L.Ci * 9 + 4 * c4) = *reinterpret_cast<const float4*>(w + row * 144 + 4 * c4);
        }
    }
    if (ct == 0) {   // the 4 lane groups' partial column sums, in group order
        float sb = __shfl(dbias, i16, 64);
        sb += __shfl(dbias, 16 + i16, 64);
        sb += __shfl(dbias, 32 + i16, 64);
        sb += __shfl(dbias, 48 + i16, 64);
        if (g == 0) part[(int64_t)L.Co * L.Ci * 9 + mt * 16 + i16] = sb;
    }
    DQNX_STAMP_BLK(a.stamps, sb_ + 5, sblk);
}

// conv 1: workgroup = (group of up to MW (co tile, im2col column tile) pairs, slice of samples);
// wave w owns one tile and every k-step of it.  Per sample: the wave's dZ fragments come straight
// from global memory into registers (a sample ahead), the input image (Ci x Hi x Wi, zero
// border) through LDS (double buffered, one barrier per sample); four accumulators rotate over
// the k-steps (summed in order at the end) and db rides on the dZ fragments already loaded.
constexpr int DW1_KS = 36;    // k-steps (4 pixels each) per sample: conv 1 Ho*Wo <= 144
constexpr int DW1_XE = 4;     // image floats per thread: Ci*Hi*Wi <= 1024
__device__ __forceinline__ void micro_dw_first(const MicroDwArgs& a, const MicroDwLayer& L, int rel, float* lds) {
    DQNX_STAMP(a.stamps, 24);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, i16 = lane & 15, g = lane >> 4;
    const int Mt = L.Co >> 4, nt = Mt * L.nct, ngr = (nt + MW - 1) / MW;
    const int tg = rel % ngr, slice = rel / ngr;
    const int tile = tg * MW + wid;
    const bool active = tile < nt;
    const int tl = active ? tile : 0, mt = tl % Mt, ct = tl / Mt;
    const int s0 = slice * L.spw, ns = min(a.Bl, s0 + L.spw) - s0;
    const int Pq = L.Ho * L.Wo, Pin = L.Hi * L.Wi, img = L.Ci * Pin, K0 = L.Ci * 9;
    const int PW = L.Wi + 2, PP = (L.Hi + 2) * PW;
    const int xb = (L.Ci * PP + 3) & ~3;    // one image buffer; two of them, then the zero block
    for (int e = tid; e < 2 * xb; e += MTH) lds[e] = 0.f;   // borders stay zero
    int* rows = reinterpret_cast<int*>(lds + 2 * xb);        // the slice's ring rows (phys)
    for (int e = tid; e < ns; e += MTH) rows[e] = a.phys[s0 + e];
    // this lane's im2col column n = (ci, tap) -> image offset; columns past K0 read zeros
    const int n = ct * 16 + i16, nc_ = n < K0 ? n : 0;
    const int ci = udiv(nc_, 9), tap = nc_ - 9 * ci, ti = udiv(tap, 3), tj = tap - 3 * ti;
    const int toff = ci * PP + ti * PW + tj;
    // per k-step: the image offset (bytes) of this lane's pixel 4 st + g, two 16-bit offsets per
    // register (pixels past Pq: offset 0, A = 0 there, any finite B)
    uint32_t pb2[DW1_KS / 2];
#pragma unroll
    for (int h = 0; h < DW1_KS / 2; h++) {
        uint32_t v = 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int px = 4 * (2 * h + u) + g;
            const int ho = (px * L.wo_mul) >> 16, wo = px - ho * L.Wo;
            v |= (uint32_t)(px < Pq ? 4 * (ho * L.sh * PW + wo * L.sw + toff) : 0) << (16 * u);   // 0: zero corner
        }
        pb2[h] = v;
    }
    // image staging map: element e = tid + j*MTH of the CHW micro grid -> LDS interior
    int xdst[DW1_XE];
#pragma unroll
    for (int j = 0; j < DW1_XE; j++) {
        const int e = tid + j * MTH, c_ = udiv(e, Pin), rc = e - c_ * Pin, r = udiv(rc, L.Wi), c = rc - r * L.Wi;
        xdst[j] = e < img ? c_ * PP + (r + 1) * PW + c + 1 : -1;
    }
    float xr[DW1_XE];
    auto xload = [&](int j) {   // slice sample j's image -> registers (ring row from LDS: no global round trip)
        const float* src = a.ring_obs + (int64_t)rows[j] * a.ring_stride + a.macro_len;
#pragma unroll
        for (int j = 0; j < DW1_XE; j++) xr[j] = src[min(tid + j * MTH, img - 1)];   // unconditional (vmcnt)
    };
    auto xstore = [&](int buf) {
#pragma unroll
        for (int j = 0; j < DW1_XE; j++)
            if (xdst[j] >= 0) lds[buf * xb + xdst[j]] = xr[j];
    };
    // dZ fragments: unconditional loads (a conditional load would make the compiler wait for
    // every load in flight before the MFMAs); pixels past Pq re-read pixel Pq - 1 and meet the
    // image's zero corner (pb2 = 0) in the MFMA, and are masked out of db
    const float* Dw = L.D + mt * 16 + i16;   // this lane's dZ column
    const int kv = (Pq - g + 3) >> 2;        // k-steps whose pixel 4 st + g is inside the image
    auto aload = [&](int b, float (&av)[DW1_KS]) {
        const float* d = Dw + (int64_t)b * Pq * L.Co;
#pragma unroll
        for (int st = 0; st < DW1_KS; st++) av[st] = d[(int64_t)min(4 * st + g, Pq - 1) * L.Co];
    };
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    float dbias = 0.f;
    auto compute = [&](int buf, const float (&av)[DW1_KS]) {
        const char* X = reinterpret_cast<const char*>(lds + buf * xb);
#pragma unroll
        for (int st = 0; st < DW1_KS; st++) {   // steps past ks: every pixel outside, B = 0
            const uint32_t o = st & 1 ? pb2[st >> 1] >> 16 : pb2[st >> 1] & 0xffffu;
            acc[st & 3] = mfma16x16x4(av[st], *reinterpret_cast<const float*>(X + o), acc[st & 3]);
            dbias += st < kv ? av[st] : 0.f;
        }
    };
    DQNX_STAMP(a.stamps, 25);
    float a0[DW1_KS], a1[DW1_KS];
    micro_barrier();   // borders zeroed and rows staged before their use
    // every load unconditional (ns >= 1; inactive waves re-read tile 0's fragments, the last
    // sample's prefetch re-reads it): a load under a branch makes the compiler's vmcnt waits
    // assume it was skipped, i.e. wait for the loads issued after it
    xload(0);
    aload(s0, a0);
    xstore(0);
    micro_barrier();
    DQNX_STAMP(a.stamps, 27);
    // sample j: image in buffer j & 1, dZ fragments in a0 (even j) / a1 (odd j)
    for (int j = 0; j < ns; j += 2) {
        const int j1 = min(j + 1, ns - 1), j2 = min(j + 2, ns - 1);
        xload(j1);
        aload(s0 + j1, a1);
        if (active) compute(0, a0);
        if (j + 1 < ns) xstore(1);
        micro_barrier();
        if (j + 1 >= ns) break;
        xload(j2);
        aload(s0 + j2, a0);
        if (active) compute(1, a1);
        if (j + 2 < ns) xstore(0);
        micro_barrier();
    }
    DQNX_STAMP(a.stamps, 36);
    if (!active) return;
    float* part = L.partial + (int64_t)slice * L.pstride;
    const int co = mt * 16 + 4 * g;
    if (n < K0)
#pragma unroll
        for (int r = 0; r < 4; r++)
            part[(int64_t)(co + r) * K0 + n] = ((acc[0][r] + acc[1][r]) + acc[2][r]) + acc[3][r];
    if (ct == 0) {   // the 4 lane groups' partial column sums, in group order
        float sb = __shfl(dbias, i16, 64);
        sb += __shfl(dbias, 16 + i16, 64);
        sb += __shfl(dbias, 32 + i16, 64);
        sb += __shfl(dbias, 48 + i16, 64);
        if (g == 0) part[(int64_t)L.Co * K0 + mt * 16 + i16] = sb;
    }
    DQNX_STAMP(a.stamps, 39);
}

template <int NC>
__global__ __launch_bounds__(MTH, 2) void k_micro_dw(MicroDwArgs a) {   // 2 waves per SIMD: 2 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int bid = blockIdx.x;
    if (a.L[NC >= 3 && bid >= a.L[2].wg0 ? 2 : bid >= a.L[1].wg0 ? 1 : 0].skip) return;
    if (NC >= 3 && bid >= a.L[2].wg0) micro_dw_body_ci(a, a.L[2], bid - a.L[2].wg0, lds);
    else if (bid >= a.L[1].wg0) micro_dw_body_ci(a, a.L[1], bid - a.L[1].wg0, lds);
    else micro_dw_first(a, a.L[0], bid, lds);
}

int launch_micro_dw(const MicroDwArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.lds_floats * 4;
    if (a.nc == 3) DQNX_LAUNCH(k_micro_dw<3>, dim3(a.wgs), dim3(MTH), lds, s, a);
    else DQNX_LAUNCH(k_micro_dw<2>, dim3(a.wgs), dim3(MTH), lds, s, a);
    DQNX_HIP_CHECK(hipGetLastError());
    return DQNX_OK;
}

}  // namespace dqnx
