// Kernel argument structs and launchers shared by learn.hip / conv.hip / engine.cpp.
#pragma once
#include "common.hpp"
#include "relayout.hpp"

namespace dqnx {

// Flat offsets inside the Q-head parameter block (torch named_parameters order):
//   dueling: [fc_val.w (F) | fc_val.b | fc_adv.w (A*F) | fc_adv.b (A)], o = 0 val, 1..A adv
//   linear:  [fc_out.w (A*F) | fc_out.b (A)]
__host__ __device__ __forceinline__ int head_w_off(int kind, int o, int F) {
    return kind == DQNX_HEAD_DUELING ? (o == 0 ? 0 : F + 1 + (o - 1) * F) : o * F;
}
__host__ __device__ __forceinline__ int head_b_off(int kind, int o, int F, int A) {
    return kind == DQNX_HEAD_DUELING ? (o == 0 ? F : F + 1 + A * F + (o - 1)) : A * F + o;
}

// torch single-tensor Adam's per-step scalars for step t (R:env/dqn_config.py:176):
// step_size = -(lr / (1 - beta1**t)), bias_correction2**0.5, from the host-libm table for
// t <= len (the same pow the CPU reference calls), device libm beyond.  The head kernel of a
// step advances t and stores both in dqnx_ctrl, so the optimizer pass reads them in the
// same round trip as its operands.
struct AdamBias {
    const float* table;
    int len;
    double lrd, beta1d, beta2d;
};
__device__ __forceinline__ void adam_bias(int64_t t, const AdamBias& b, float& step_size, float& bc2s) {
    if (t >= 1 && t <= b.len) {
        step_size = b.table[2 * (t - 1)];
        bc2s = b.table[2 * (t - 1) + 1];
    } else {
        step_size = (float)(-(b.lrd / (1.0 - pow(b.beta1d, (double)t))));
        bc2s = (float)pow(1.0 - pow(b.beta2d, (double)t), 0.5);
    }
}
__device__ __forceinline__ void adam_advance(dqnx_ctrl* ctrl, const AdamBias& b) {
    const int64_t t = ctrl->adam_step + 1;
    float ss, bc;
    adam_bias(t, b, ss, bc);
    ctrl->adam_step = t;
    ctrl->adam_step_size = ss;
    ctrl->adam_bc2_sqrt = bc;
}

// PER priority writes with SumTree.update's sequential semantics (R:dqn/utils/sum_tree.py:15-32):
// mode 0 = update_batch_priorities (R:dqn/replay_memory.py:94-98),
// mode 1 = store_transitions' adds at the current max priority (R:dqn/replay_memory.py:56-67).
struct PerUpdateArgs {
    double* tree;
    int64_t cap;
    dqnx_ctrl* ctrl;          // per_max_idx / per_min_idx (read + written)
    int32_t mode;
    int32_t n;                // updates in this launch (<= PER_CHUNK)
    const int32_t* slots;     // mode 0: [n] ring slots, in batch order
    const float* abs_td;      // mode 0: [n] |targets - q(s,a)|
    int64_t wptr, size;       // mode 1: ring write pointer / size before this chunk (mode 0 reads ctrl)
    float eps, alpha, pmax;   // numpy float32 arithmetic on the python-float constants
    int64_t* stamps;          // diagnostic builds (-DDQNX_STAMPS): slots 56..63
    // workspace shared by the three launches of one chunk (k_per_prep, k_per_update, k_per_prop)
    int32_t* wl;              // [PER_CHUNK] leaf (tree index) of item i
    float* wp;                // [PER_CHUNK] its new priority
    double* winit;            // [PER_CHUNK] the leaf's value before the chunk
    uint64_t* last;           // [cap] (epoch << 32 | i) of the latest item writing the slot
    uint32_t* epoch;          // chunk counter (tags `last`; zero after reset, like `last`)
    // numpy 1.21 arithmetic (dqnx_config.per_numpy121, mode 0 only): `change` and every
    // ancestor sum rounded to float32, applied in update order (k_per_chain)
    int32_t numpy121;
    float* wchg;              // [PER_CHUNK] float32 change of item i
    // single-GPU PER learn step: k_per_prep's work done by the head kernel for its samples
    // (PER_SKIP_PREP) and k_per_prop's workgroups run beside the weight-gradient tiles (PER_SKIP_PROP)
    int32_t skip;
    // the tracking workgroup -> prop workgroups hand-off inside one launch (k_dw_adam16 hosting
    // both): the chunk epoch the tracking workgroup last advanced to (per_track_publish)
    uint32_t* sync;
};
constexpr int PER_SKIP_PREP = 1, PER_SKIP_PROP = 2, PER_SKIP_TRACK = 4;

struct FwdProblem {
    const float* A;        // dense rows, or the replay ring (layer 1, phys != null)
    int lda;
    const int32_t* phys;   // physical ring slot per row (layer 1) or null
    const float* W;        // [N][K] (torch Linear weight)
    const float* bias;     // [N]
    float* C;              // [M][ldc]
    float* xcopy;          // layer 1 stream 0: materialised gathered rows (ld = lda) or null
};
struct FwdArgs {
    FwdProblem p[3];
    int M, N, K, ldc;
    int nprob;
    // large-K layers (k_linear_fwd_big): K split into ksplit chunks of kchunk columns; chunk s of
    // problem z writes its raw sums to partial[(s * nprob + z) * M * N ...], a second launch adds
    // them in chunk order (deterministic), then bias and activation
    int ksplit, kchunk;
    float* partial;
    int64_t* stamps;           // diagnostic builds: launch_linear_fwd_split's workgroup 0 (slots 53..55)
};

// One split-K weight-gradient GEMM: partial[s] = dZ^T [X | 1] over the samples of slice s.
// Partials are written in the flat parameter layout of the layer: plain Linear
// ([W (out x in) | b (out)]) or, for head_kind >= 0, the Q-head layout
// ([fc_val.w | fc_val.b | fc_adv.w | fc_adv.b] or [fc_out.w | fc_out.b]).
struct DwProblem {
    const float* dZ;       // [Bl][ldz]
    int ldz;
    const float* X;        // [Bl][ldx] layer input rows (stream 0)
    int ldx;
    int in, out;
    float* partial;        // [slices][pstride]
    int64_t pstride;
    int head_kind;         // -1 plain Linear layout, else dqnx_head_kind
    int A;                 // actions (head layout)
    int grid_x, grid_y, blocks;   // filled by bwd_level_grid
    // k_dw_bf16d (BwdArgs::t16, opt-in DQNX_DWB_T=1): the same operands as bf16 copies in the slab-transposed layout (tcopy_index):
    // dZ with cz columns, X with cx columns; X's column `in` is the ones column (the bias), not stored
    const uint16_t* dZT;
    const uint16_t* XT;
    int cz, cx;
};
// Slab-transposed layout of a bf16 operand with C columns over the minibatch, KB = the weight
// gradients' split-K slice (kslice): element (sample b, column c) at ((b / KB) * C + c) * KB + b % KB --
// one column's samples of one slice contiguous (whole cache lines for k_dw_bf16d's 16-byte fragment
// loads; a first layout of 16-sample blocks, [b/16][C][16], left 32 bytes used per line touched).
__host__ __device__ __forceinline__ int64_t tcopy_index(int64_t b, int c, int C, int KB) {
    return ((b / KB) * C + c) * KB + b % KB;
}
struct BwdArgs {
    // dx role (skipped when dZprev == null): dZprev = (dZ W) (.) act'(Hprev)
    const float* dZ;       // [Bl][out]
    const float* W;        // [out][in]
    const float* Hprev;    // [Bl][ldh]
    int ldh;
    float* dZprev;         // [Bl][in]
    int in, out;
    // dw roles
    DwProblem dw[4];       // dW of up to 3 dense layers + the head in one launch (fused plan)
    int ndw;
    int Bl, kslice, dw_slices;
    int dx_blocks, dx_grid_x;
    int ts;                // k_bwd_level tile edge: 0 = DQNX_BWD_BM (32), or 64 (large layers: a quarter of the
                           // workgroups, four times the MFMAs per operand pass; set before bwd_level_grid)
    int t16;               // bf16 weight gradients from the slab-transposed copies (k_dw_bf16d) instead of fp32 rows
    int64_t* stamps;       // diagnostic builds (-DDQNX_STAMPS): k_dw_bf16d's slots 57..62
    int pprop_wgs;         // k_dw_bf16: + workgroups running k_per_prop's body (single-GPU PER step)
    int ptrack;            // k_dw_bf16: + block 0 running k_per_update's tracking (its prop in the Adam launch)
    PerUpdateArgs pprop;
};

struct HeadArgs {
    int Bl, F, A, NH, head_kind, algo, head_params;
    float inv_bg;          // float(1.0 / global batch)
    float gamma;
    const float* H;        // [3][Bl][F] last hidden activations
    const float* Wo;       // online head params (flat, torch order)
    const float* Wt;       // target head params
    const int32_t* phys;   // [Bl] ring slots
    const int32_t* act;
    const float* rew;
    const float* done;
    const float* isw;      // [Bl] PER IS weights of the local shard or null
    float* abs_td_out;     // PER: [Bl] |targets - q(s,a)| into the global [Bg] array (shard offset) or null
    float* Q;              // [3][Bl][A]
    float* td;             // [3][Bl]: y, q(s,a), |y - q(s,a)|
    float* dZ;             // [Bl][F]
    float* dhead;          // [Bl][16] d(head outputs), consumed by the head dW
    // dZ of the layer below the last hidden layer (L >= 2): dZprev = (dZ_L W_L) (.) act'(H_{L-1})
    const float* W_last;   // W_L [F][in_prev]
    const float* Hprev;    // H_{L-1} stream 0 [Bl][in_prev]
    float* dZprev;         // [Bl][in_prev] or null (L == 1)
    int in_prev;
    float* loss_partial;   // [tiles]
    dqnx_ctrl* ctrl;       // Adam step bookkeeping (block 0) or null
    float beta1, beta2, lr;
    AdamBias ab;
    int64_t* stamps;       // diagnostic builds (-DDQNX_STAMPS)
};

constexpr int kMaxSeg = 10;
constexpr int ADAM_WIDE = 8;          // k_adam4: lanes per float4 of a wide segment
constexpr int ADAM_WIDE_MIN_S = 24;   // k_adam4: segments with this many split-K slabs or more take the wide path
constexpr int kAdamTable = 1 << 20;   // precomputed Adam bias corrections (steps 1..2^20)
struct AdamSegment {
    int64_t off;           // first flat element of the segment
    const float* partial;  // slab 0 of the segment's partials
    int64_t pstride;       // elements between slabs
    int S;                 // number of slabs
    int wide;              // summed ADAM_WIDE-strided (k_adam4's wide path; the scalar kernel the same order)
};
struct AdamArgs {
    AdamSegment seg[kMaxSeg];
    int nseg;
    int mode;              // 0 partials->grads, 1 partials->grads+adam, 2 grads->adam
    int soft;
    int64_t n_params;      // elements [e0, n_params) are processed (e0 = 0 except for DP buckets)
    int64_t e0;
    int64_t wide_end;      // k_adam4: [e0, wide_end) = segments summed by ADAM_WIDE lanes per float4 (launch_adam)
    int with_loss;         // the range ends at the loss slot grads[n_params] (mode 2: publish it)
    float* p;
    float* m;
    float* v;
    float* grads;          // [n_params + 1] (last = loss)
    float* target;
    dqnx_ctrl* ctrl;
    float w1, beta2, c2, eps, tau, one_minus_tau;
    const float* loss_partial;
    int n_loss_partial;
    int batch_global;
    const float* adam_table;   // [t-1] = {-lr/bc1, bc2**0.5} for t <= adam_table_len (host libm)
    int adam_table_len;
    double beta1d, beta2d, lrd;
    uint32_t* mtc;         // uniform sampler's MT block cache, extended by an extra workgroup (or null)
    int mtc_blocks;
    // fused plan: the fragment-blocked weight copies (relayout.hpp) written next to every updated
    // weight, so they never need a rebuild launch (nblk = 0: none)
    int nblk;
    struct BlkLayer {
        int64_t woff;      // flat offset of W_l [out][in]
        int in, out, kpad;
        float inv_in;      // 1 / in
        float* fwd_online; // fwd-blocked online W_l
        float* fwd_target; // fwd-blocked target W_l (soft update)
        float* chain;      // chain-blocked online W_l (l >= 1) or null
    } blk[3];
    int blk_bf16;
    // in-launch prefetch: the minibatch the forward drew into the staging slot replaces this
    // step's (one more workgroup; pf_nidx = 0: none)
    const int32_t* pf_idx_src;
    int32_t* pf_idx_dst;
    int pf_nidx;
    const int32_t* pf_phys_src;
    int32_t* pf_phys_dst;
    int pf_nphys;
    // micro-CNN plan: the permuted weight copies of convs 2.. (k_conv_perm's layouts) written next to
    // every updated conv weight by the wide path (mode 1), so the next step needs no conv_perm launch
    int pprop_wgs;         // + workgroups running k_per_prop's body (DP apply: after the all-gathered update)
    PerUpdateArgs pprop;
    int nperm;
    struct PermLayer {
        int64_t woff;      // flat offset of W [Co][Ci][3][3]
        int Co, Ci;
        float* p0;         // [Co][9][Ci] online
        float* p1;         // [Co][9][Ci] target
        float* pT;         // [Ci][9][Co] online
    } perm[2];
};
// launch_adam writes AdamArgs::perm (the float4 kernel's wide path covers every perm layer)
bool adam_writes_perms(const AdamArgs& a);

// Full-K weight gradients of every layer + Adam (+ soft update) in one launch.
struct DwAdamProblem {
    const float* dZ;       // [Bl][ldz]
    int ldz;
    const float* X;        // [Bl][ldx]
    int ldx;
    int in, out;           // gradient tile space: out x (in + 1 ones column)
    int64_t poff;          // flat offset of this layer's parameters
    int head_kind;         // -1 plain Linear layout, else dqnx_head_kind
    int A;
    int grid_x, blocks;
};
struct DwAdamArgs {
    DwAdamProblem pr[DQNX_MAX_DENSE + 1];
    int npr;
    int Bl;
    int mode;              // 0: write grads only (DP all-reduce follows), 1: grads + Adam
    int soft;
    int64_t n_params;
    float* p;
    float* m;
    float* v;
    float* grads;          // [n_params + 1] (last = loss)
    float* target;
    dqnx_ctrl* ctrl;
    float w1, beta2, c2, eps, tau, one_minus_tau;
    const float* loss_partial;
    int n_loss_partial;
    int batch_global;
    const float* adam_table;
    int adam_table_len;
    double beta1d, beta2d, lrd;
};

struct PushArgs {
    const float* obs;
    const float* next_obs;
    const int32_t* act;
    const float* rew;
    const uint8_t* done;
    int n, obs_dim, stride;
    int64_t wptr, capacity, new_size, new_wptr;
    float* ring_obs;
    float* ring_next;
    int32_t* ring_act;
    float* ring_rew;
    float* ring_done;
    dqnx_ctrl* ctrl;
    uint16_t* ring16_obs;        // bf16 engines: the rows' bf16 copies too (null: none)
    uint16_t* ring16_next;
    int stride16;
};

struct SampleArgs {
    uint32_t* state;          // [625] the advanced state is written here
    const uint32_t* state_in; // [625] the state drawn from, when not `state` (null: `state`): the drop-in
                              // Agent's pinned fine-grained host block, read in place (no upload copy)
    const int64_t* n_dev;     // population size from device (ring size) or null
    int64_t n_val;
    int32_t k;
    int64_t setsize;
    int32_t* out;             // [k] logical positions
    int32_t* err;             // sticky error word
    int32_t* pool;            // pool-branch scratch [>= setsize]
    // optional: physical ring slots of the local shard  phys = (wptr - size + j) mod cap
    int32_t* phys_out;        // [shard_len] or null
    int32_t shard_begin, shard_len;
    const int64_t* wptr_dev;
    int64_t capacity;
    int64_t* stamps;          // diagnostic builds (-DDQNX_STAMPS)
    RelayoutArgs rl;          // fused plan: blocked weight copies, built by blocks 1.. of the launch
    int rl_blocks;
    unsigned long long* gtab; // k too large for an LDS table: sample_table_bytes(k) of global scratch
    int test_flags;           // tests only (DQNX_SAMPLER_FORCE_FALLBACK): 1 = take the fast path's fallback
    uint32_t* mtc;            // MT block cache (mt_cache_words), or null: [0] = blocks held, [64 + 624 b + o]
    int mtc_blocks;           // blocks the cache is kept at (the state's block + its successors)
    int bm_cap;               // bitmap first pass (hosts with a repeat table): repeated words it takes
                              // before falling back to the hash table; 0 = half the table, < 0 = off
                              // (tests: DQNX_SAMPLER_BM_CAP)
    int bm_rolled;            // the bitmap pass in rolled loops (DQNX_SAMPLER_ROLLED, 0/1)
};
// Fused plan (fp32): every weight gradient over the FULL minibatch on 16 x 16 parameter tiles,
// then Adam, the soft update and the fragment-blocked weight copies of the tile, in one launch
// (k_dw_adam16, learn.hip).  A tile is exactly one 16 x 16 block of the fwd- and chain-blocked
// copies (relayout.hpp).
struct DwAdam16Layer {
    const float* dZ;       // [Bl][ldz]
    int ldz;
    const float* X;        // [Bl][ldx] layer input rows (stream 0)
    int ldx;
    int in, out;
    int64_t poff;          // flat offset of W ([out][in]; the bias follows, or the head layout)
    int head_kind;         // -1 plain Linear, else dqnx_head_kind
    int A;
    int ti;                // 16-column blocks along `in`
    int t0;                // first tile of this layer in the grid (tiles: ti x ceil(out / (16 rows16)))
    float* fwd_online;     // fwd-blocked copies (null: the layer has none)
    float* fwd_target;
    float* chain;          // chain-blocked online copy (null: none)
    int nch_fwd, nch_chain;   // kpad / 16, out / 16
};
struct DwAdam16Args {
    DwAdam16Layer L[DQNX_MAX_DENSE + 1];
    int nl;
    int tiles;             // parameter tiles (+ 1 workgroup for the MT cache when mtc)
    int rows16;            // 16-row blocks of W per tile (1: 16 x 16 tiles; 2: 32 x 16)
    int Bl;
    int mode;              // 0: gradients (+ loss) only, the DP all-reduce and Adam pass follow; 1: + Adam;
                           // 3: Adam from `grads` (dqnx_apply_grads after the all-reduce: no K loop)
    int soft;
    int64_t n_params;
    float* p;
    float* m;
    float* v;
    float* grads;          // [n_params + 1] (last = loss)
    float* target;
    dqnx_ctrl* ctrl;
    float w1, beta2, c2, eps, tau, one_minus_tau;
    const float* loss_partial;
    int n_loss_partial;
    int batch_global;
    uint32_t* mtc;
    int mtc_blocks;
    int64_t* stamps;       // diagnostic builds (-DDQNX_STAMPS): slots 56..61
    // in-launch prefetch (DQNX_STEP_PREFETCH): one more workgroup copies the minibatch the forward
    // launch drew into the staging slot over this step's (pf_nidx = 0: none)
    const int32_t* pf_idx_src;
    int32_t* pf_idx_dst;
    int pf_nidx;
    const int32_t* pf_phys_src;
    int32_t* pf_phys_dst;
    int pf_nphys;
    int pprop_wgs;         // + workgroups running k_per_prop's body (single-GPU PER step; 0: none)
    int ptrack;            // + one workgroup running k_per_update's tracking first; the prop
                           //   workgroups then wait for it (pprop.sync)
    PerUpdateArgs pprop;
};

// MT block cache: the state block of the uniform sampler and its twisted successors, kept ahead
// by the Adam launch of the previous step (k_adam's extra workgroup), so the next sample reads the
// blocks it consumes instead of twisting them on its critical path.  Valid by construction: cache
// block b+1 is always twist(cache block b), and it is used only when cache block 0 equals the
// state block the caller hands in.
constexpr int MTC_MAX_BLOCKS = 22;
constexpr int64_t mt_cache_words() { return 64 + (int64_t)MTC_MAX_BLOCKS * 624; }
int mt_cache_target_blocks(int32_t k, int64_t n);   // blocks a sample of k from n consumes (+ margin)

// PER sampling: ReplayMemoryPrioritized.sample_transitions (R:dqn/replay_memory.py:69-92)
constexpr int PER_MAX_B = 8192;     // largest global minibatch k_per_sample handles
constexpr int PER_CHUNK = 8192;     // priority updates per k_per_update launch
struct PerSampleArgs {
    const double* tree;       // [2*cap-1] SumTree (R:dqn/utils/sum_tree.py)
    int64_t cap;
    dqnx_ctrl* ctrl;          // np_mt (advanced), ring_size, per_min_idx, agent_step (read, += n_env)
    int32_t Bg;               // global minibatch
    int32_t shard_begin, shard_len;
    int32_t* out_idx;         // [Bg] sampled data indices (= ring slots = leaf - (cap-1))
    int32_t* phys_out;        // [shard_len] ring slots of this rank's shard
    float* isw;               // [Bg] importance weights (float32, like T.as_tensor(..., float32))
    double beta_start, beta_end, beta_steps;
    int32_t n_env;
    RelayoutArgs rl;          // fused plan: blocked weight copies, built by blocks 1.. of the launch
    int rl_blocks;
    int64_t* stamps;          // diagnostic builds (-DDQNX_STAMPS): slots 0..7
    int32_t* ticket;          // arrival counter of the sampling workgroups, zero between launches
    uint32_t* npc;            // numpy MT block cache (np_cache_words; null: twist every block here)
    int spw;                  // samples (descents) per workgroup
};
// numpy MT block cache (PER, fused plan): [0] blocks held, [1] block the state moved to in the last
// sample (the extension shifts the cache down by it), [64 + 624 b + o] block b (0 = the state block).
// PER sampling consumes 2 Bg words; without the cache every sampling workgroup twists all of those
// blocks in sequence (26 at Bg = 8192).  One extra workgroup of the forward launch (which runs
// after the sample) twists the next sample's blocks ahead, off the critical path.
constexpr int NPC_MAX_BLOCKS = 29;   // (624 + 2 PER_MAX_B - 1) / 624 + 1 at PER_MAX_B = 8192
constexpr int64_t np_cache_words() { return 64 + (int64_t)NPC_MAX_BLOCKS * 624; }
__host__ __device__ constexpr int np_cache_blocks(int Bg) { return (624 + 2 * Bg - 1) / 624 + 1; }


// ---- two-stream hybrid network data movement (conv.hip) ----
struct Im2colArgs {
    int nstreams;
    const float* ring[3];     // first conv: ring (obs / next_obs) per stream, else null
    const int32_t* phys;      // [Bl] ring slots (first conv)
    int64_t ring_stride;      // floats per ring row
    int ring_off;             // micro grid offset inside the row (= macro_len)
    const float* src[3];      // later convs: NHWC activations [Bl*Hi*Wi][Ci] per stream
    float* col[3];            // [M][Kstride] per stream, k = (ci, i, j), zero padded
    int Ci, Hi, Wi, Ho, Wo, kh, kw, sh, sw, ph, pw;
    int K, Kstride, M;
};
struct FlattenArgs {
    int nstreams;
    const float* Hc[3];       // last conv NHWC [Bl*Ho*Wo][C]
    const float* ring[3];     // macro source rows per stream
    const int32_t* phys;
    int64_t ring_stride;
    int macro_len, C, Ho, Wo, Bl, strideF;
    float* F[3];              // [Bl][strideF] = cat(flatten_CHW(conv), macro), zero padded
};
struct UnflattenArgs {
    const float* dF;          // [Bl][ldf], CHW-flatten order
    int ldf;
    float* dZ;                // [Bl*Ho*Wo][C]
    int Bl, C, Ho, Wo;
};
struct Col2imArgs {
    const float* dcol;        // [Bl*Ho*Wo][ldcol], k = (ci, i, j)
    int ldcol;
    const float* Hprev;       // [Bl*Hi*Wi][Ci] activation output of the previous conv
    float* dZprev;            // [Bl*Hi*Wi][Ci]
    int Bl, Ci, Hi, Wi, Ho, Wo, kh, kw, sh, sw, ph, pw;
};
// ---- fused MLP plan (fused.hip): one forward launch for every layer + the Q head, one
//      head / TD / dZ-chain launch per 16-sample tile ----
constexpr int FUSED_MAX_L = 3;
#ifndef DQNX_FUSED_WAVES
#define DQNX_FUSED_WAVES 8
#endif
constexpr int FUSED_WAVES = DQNX_FUSED_WAVES;   // waves per workgroup of both fused kernels
struct FusedFwdArgs {
    int L, Bl, tiles, nstreams;
    int in[FUSED_MAX_L], out[FUSED_MAX_L];
    int64_t woff[FUSED_MAX_L];   // flat offset of W_l ([out][in]); the bias follows
    int64_t head_off;
    int head_kind, NH, F;
    int stream_of[3];            // logical stream of grid slice z: 0 online(s), 1 online(s'), 2 target(s')
    const float* params;
    const float* tparams;
    const float* ring_obs;
    const float* ring_next;
    int ring_stride;             // floats per ring row (obs_dim rounded up to 4)
    // bf16 compute: the rows as bf16 copies (RNE of the fp32 rows, written by the replay push), which is
    // all the bf16 GEMMs read of them; the forward gathers these (half the bytes), bitwise the same operands
    const uint16_t* ring16_obs;
    const uint16_t* ring16_next;
    int stride16;                // bf16 elements per ring16 row (obs_dim rounded up to 8: 16-byte rows)
    const int32_t* phys;         // [Bl] physical ring slots
    float* xcopy;                // [Bl][ring_stride] stream-0 gathered rows (layer-1 dW operand)
    float* H[FUSED_MAX_L];       // stream-0 activations [Bl][out_l]
    uint16_t* xT16;              // bf16 + DQNX_DWB_T=1: stream 0's rows / activations as slab-transposed
    uint16_t* HT16[FUSED_MAX_L]; // copies (tcopy_index, slice length tkb), or null
    int tkb;
    float* raw;                  // [3][Bl][16] head outputs per logical stream
    float4* trans;               // [Bl] stream 0: {act (int bits), rew, done, 0} of each sampled slot
    const int32_t* act;          // replay ring columns (gathered for `trans`)
    const float* rew;
    const float* done;
    int bf16;                    // DQNX_COMPUTE_BF16: bf16 LDS tiles, bf16 blocked weights, bf16 MFMA
    int mr;                      // 16-row tiles per workgroup (1, 2 or 4; `tiles` counts 16*mr-row tiles)
    int gw;                      // gather width class: 0 rows of <= 288 multiplied columns (FWD_NARROW_Q4
                                 // float4), 1 wider (whole forward, 16-row tiles only)
    int phase;                   // 0 whole forward; 1 layer 1 split over csplit parts; 2 layers 2.. + head;
                                 // 3 whole forward, layer 1's columns over 2 partner workgroups of one XCD
                                 // (in-launch H_1 hand-off, DQNX_FWD_PAIR)
    int csplit;
    uint32_t* pair_flags;        // phase 3: [nstreams * tiles] hand-off words (zero between launches)
    int32_t* err;                // phase 3: dqnx_ctrl.error (hand-off timeout)
    int sx, sh;                  // LDS row strides (elements: floats, or bf16 under bf16) of the input / hidden tiles
    int buf0, buf1;              // LDS buffer sizes (floats)
    int kpad[FUSED_MAX_L];       // layer inputs zero padded to kpad (blocked copies): fp32 a multiple of 64, bf16 of 32
    const float* wblk[2][FUSED_MAX_L];   // fragment-blocked W_l of the online / target net (relayout.hpp)
    int64_t* stamps;             // diagnostic builds (-DDQNX_STAMPS): slots 24..39
    // in-launch prefetch (DQNX_STEP_PREFETCH, uniform replay): one more workgroup (the last)
    // draws the NEXT step's minibatch into the staging slot with the multi-pass sampler body, on
    // a CU the row tiles leave idle (samp_shape: its LDS shape, fwd_sample_*; 0 = no sampler workgroup)
    int samp_shape;
    SampleArgs samp;
    // this step's Adam scalars (adam_advance), stored by one otherwise idle thread while its
    // workgroup gathers, off the head kernel's critical path (null: the head kernel stores them)
    int xcd_rows;                // row tile t of every stream on XCD t % 8 (the head kernel follows)
    dqnx_ctrl* adam_ctrl;
    AdamBias ab;
    // PER: block 0 (dispatched first) twists the numpy MT block cache ahead for the next sample
    uint32_t* npc;
    const uint32_t* np_state;   // ctrl->np_mt (the state the cache must start from)
    int npc_blocks;
    int lds_min;                 // dynamic LDS request floor in bytes (placement knob: > 80 KB = one workgroup per CU)
};
// The forward's sampler workgroup (512 threads), three LDS shapes (FusedFwdArgs::samp_shape):
//   1: k <= 2048, passes of 3 MT blocks into a 4096-slot table (40 KB, no more than the forward's
//      own tiles);
//   2: k <= FWD_SAMPLE_MAX_K, passes of 3 blocks into 8192 slots (72 KB: two forward workgroups per
//      CU still fit, for grids larger than the chip);
//   3: k <= FWD_SAMPLE_MAX_K, ONE pass of 9 blocks into 16384 slots (150 KB: one workgroup per CU,
//      only when the forward's grid leaves a CU idle), so k = 4096 takes one pass instead of three;
//      the same 128 KB serve as an exact 2^20-bit "seen" bitmap for a first pass with n <= 2^20
//      (+ a 512-slot table for the repeated values, sample_body.hpp)
constexpr int FWD_SAMPLE_MAX_K = 4608;
constexpr int MICRO_SAMPLE_MAX_K = 2048;   // k_micro_fwd's sampler workgroup (256 threads, 4096 slots)
__host__ __device__ constexpr int fwd_sample_ahead(int shape) { return shape == 3 ? 8 : 2; }
__host__ __device__ constexpr int fwd_sample_hs(int shape) { return shape == 1 ? 4096 : shape == 2 ? 8192 : 16384; }
// LDS of that workgroup: the sampler's MT blocks / scan words, then the hash table (8-byte slots)
__host__ __device__ constexpr int fwd_sample_tab_off(int shape) {
    return (((fwd_sample_ahead(shape) + 1) * 624 + 16) * 4 + 63) / 64 * 64;
}
__host__ __device__ constexpr int fwd_sample_bmx(int shape) { return shape == 3 ? 512 : 0; }   // repeat-table slots
__host__ __device__ constexpr int fwd_sample_lds_bytes(int shape) {
    return fwd_sample_tab_off(shape) + 8 * fwd_sample_hs(shape) + (fwd_sample_bmx(shape) ? 8 * fwd_sample_bmx(shape) + 64 : 0);
}
struct HeadBwdArgs {
    int L, Bl, A, NH, F, head_kind, algo;
    int nsplit;                  // workgroups per 16-sample tile (split the last dZ's columns)
    int xcd_rows;                // tile t's workgroups on the XCD the forward ran row tile t on
    int xcd_shift;               // ... whose workgroups the forward's extra block 0 shifted by one
    int xcd_mr;                  // ... of 16 * xcd_mr rows (the forward's row-tile height)
    int bf16;                    // DQNX_COMPUTE_BF16: dZ chain on bf16 operands (LDS tiles + wblkT)
    int in[FUSED_MAX_L], out[FUSED_MAX_L];
    int64_t woff[FUSED_MAX_L], head_off;
    float inv_bg, gamma;
    const float* params;
    const float* raw;            // [3][Bl][16]
    const float4* trans;         // [Bl] {act, rew, done, 0} gathered by the forward (stream 0)
    const int32_t* phys;
    const int32_t* act;
    const float* rew;
    const float* done;
    const float* isw;
    float* abs_td_out;
    float* Q;                    // [3][Bl][A]
    float* td;                   // [3][Bl]
    const float* H[FUSED_MAX_L]; // stream-0 activations
    float* dZ[FUSED_MAX_L];      // [Bl][out_l]
    float* dhead;                // [Bl][16]
    uint16_t* dZT16[FUSED_MAX_L];   // bf16 + DQNX_DWB_T=1: slab-transposed copies of dZ_l / dHead (or null)
    uint16_t* dheadT16;
    int tkb;                     // their slice length (tcopy_index)
    float* loss_partial;         // [tiles]
    dqnx_ctrl* ctrl;
    const float* wblkT[FUSED_MAX_L];     // chain-blocked online W_l, l >= 1 (relayout.hpp)
    AdamBias ab;
    int64_t* stamps;             // diagnostic builds (-DDQNX_STAMPS): slots 40..55
    int pp_on;                   // single-GPU PER: k_per_prep's work for this kernel's samples
    PerUpdateArgs pp;
};
bool fused_fwd_plan(FusedFwdArgs& a, int obs_dim, bool bf16, int mr);   // fills sx/sh/buf/kpad; false if unsupported
int fused_wblk_bytes(bool bf16, int rows, int kpad);          // one blocked weight copy
int launch_fused_fwd(const FusedFwdArgs& a, int act, hipStream_t s);
int launch_head_bwd(const HeadBwdArgs& a, int act, hipStream_t s);
void dw_bf16_grid(BwdArgs& a);                               // 64x64 tiles of k_dw_bf16
int launch_dw_bf16(const BwdArgs& a, hipStream_t s);          // bf16 split-K weight gradients
bool dw_bf16t_supported(const BwdArgs& a);                   // k_dw_bf16d fits (after dw_bf16_grid)

// ---- implicit-GEMM convolutions (conv_ig.hip): the (4,84,84) variant's convs without
//      materialised column matrices ----
// One output class of a conv GEMM: the forward has one; the data gradient of a strided conv has
// one per (row, column) phase (sub-pixel decomposition), each with its own tap subset.
struct CigClass {
    int a, c;                 // output image offsets: y = ymul * yq + a, x = xmul * xq + c
    int Hq, Wq, tiles;        // class grid, row tiles of TR class rows
    int ntaps;                // = ni * nj
    int rmin, cmin;           // band origin relative to (yq * RM, xq * CM) in source pixels
    // tap (ii, jj) of the ni x nj tap grid: weight tap (i0 + ii*di) * kw + (j0 + jj*dj), at LDS
    // pixel offset o0 + ii*oi + jj*oj inside the band (uniform integer math, no table loads)
    int ni, nj, i0, j0, di, dj, kw;
    int o0, oi, oj;
};
// A staged image: element (b, r, w, ch) at base[z] + (phys ? phys[b] : b) * bstride + off
// + (r * W + w) * pstride + ch * cstride (NHWC: pstride = C, cstride = 1; CHW: pstride = 1).
struct CigSource {
    const float* base[3];
    const int32_t* phys;
    int64_t bstride, off;
    int pstride, cstride;
    int H, W, C;
};
enum { CIG_EPI_NHWC = 0, CIG_EPI_FLAT = 1, CIG_EPI_DX = 2 };
struct ConvIgArgs {
    int nstreams, Bl, nclass, maxtiles;
    int TR, RM, CM, NR, WP;   // tile = TR class rows; band NR x WP source pixels; RM band rows per class row
    // source rows per class row (SRM) and the staging row step (RS).  A stride-2 forward stages its
    // band in two row-parity groups (ngrp 2: group p holds source rows r0 + p + 2k compactly, gnr[p]
    // of them, and the taps i = p + 2 ii, ii < gni[p]), so every stage reads whole pixels (all
    // channels of a 128-B line at once) and each source row once
    int SRM, RS, ngrp;
    int gnr[2], gni[2];
    int BM, act;              // tile rows (64 / 128 / 256; TR * Wq <= BM), activation
    int N, CB, CS;            // GEMM columns, channels staged per pass, LDS floats per pixel
    CigSource src;
    CigClass cls[4];
    const float* W[3];        // permuted weights [N][kh*kw][C] per stream
    int Kw;                   // = kh*kw*C
    const float* bias[3];     // forward only
    float* out[3];            // element (b, y, x, n) at out + b*ob + y*orow + x*opix + n*och
    int64_t ob;
    int ymul, xmul, orow, opix, och;
    const float* Hprev;       // DX: the previous conv's activation output, same layout as out
    // FLAT: F row tail cat(..., macro) + zero padding, written by each image's tile-0 workgroup
    const float* ring[3];
    const int32_t* phys;
    int64_t ring_stride;
    int macro_len, flat_cols, strideF;
};
size_t conv_ig_lds_bytes(const ConvIgArgs& a);
bool conv_ig_supported(int N, int BM, int C);
int launch_conv_ig(const ConvIgArgs& a, int epi, hipStream_t s);
// conv dW + db over slices of output row groups: partial[s] = [dZ^T X | dZ^T 1] in torch order
struct ConvDwIgArgs {
    int Bl, Ho, Wo, RB, G, gps, slices;   // RB output rows per group, G groups per image, gps groups per slice
    int Co, C, CB, CS, ntaps, kw, sh, sw, ph, pw, NR, WP;
    int TN;                   // column tiles: 16 * TN >= ntaps * CB
    CigSource X;              // stream-0 conv input
    const float* dZ;          // element (b, p, co) at dZ + b*dzb + p*dzp + co*dzc
    int64_t dzb;
    int dzp, dzc;
    float* partial;
    int64_t pstride;
    int K;                    // C * kh * kw
};
size_t conv_dw_ig_lds_bytes(const ConvDwIgArgs& a);
int launch_conv_dw_ig(const ConvDwIgArgs& a, hipStream_t s);
// weight relayouts for the implicit convs: mode 0 [co][ci][t] -> [co][t][ci] (forward),
// mode 1 -> [ci][t][co] (data gradient)
struct ConvPermJob {
    const float* src;
    float* dst;
    int Co, Ci, taps, mode;
};
struct ConvPermArgs {
    int njobs;
    ConvPermJob job[12];
};
int launch_conv_perm(const ConvPermArgs& a, hipStream_t s);
int launch_unflatten_tiled(const UnflattenArgs& a, hipStream_t s);

// ---- micro-CNN plan (micro.hip): the reference HEAD net's convs on its small micro grid
//      (TwoStreamHybridNetwork, R:env/dqn_config.py:66-143: 3x3 convs, padding 1, ELU) with the
//      whole per-sample activations on chip -- no column matrices, no flatten / col2im launches ----
constexpr int MICRO_MAX_CONV = 3;
struct MicroConv {
    int Ci, Hi, Wi, Co, Ho, Wo, sh, sw;
    int64_t woff;              // flat offset of W [Co][Ci][3][3] (the bias follows)
    const float* wp[2];        // l >= 1: [Co][9][Ci] copies of the online / target W (k_conv_perm mode 0)
    const float* wT;           // l >= 1: [Ci][9][Co] copy of the online W (mode 1, data gradient)
    int cs;                    // LDS floats per pixel of this conv's output image (Co + 8: b128 reads conflict-free; Co + 4 knob)
    int lds;                   // LDS float offset of this conv's output images [S][Ho*Wo][cs]
    float* hc;                 // l < nc - 1: stream-0 output (ELU applied), NHWC [Bl][Ho*Wo][Co]
    float* dz;                 // stream-0 dZ of this conv's output (ELU' applied), NHWC [Bl][Ho*Wo][Co]
};
struct MicroFwdArgs {
    MicroConv c[MICRO_MAX_CONV];
    int nc, Bl, S, groups;     // samples per workgroup, workgroups per stream
    int nstreams, stream_of[3];
    const float* params;
    const float* tparams;
    const float* ring_obs;
    const float* ring_next;
    int ring_stride, macro_len;
    const int32_t* phys;
    float* F[3];               // per grid slice: [Bl][strideF] = cat(flatten_CHW(last conv), macro), zero padded
    int strideF, flat_cols;
    int x0;                    // LDS float offset of the input images [S][Ci*Hi*Wi] (CHW, as in the ring row)
    int zero;                  // LDS float offset of 16 zeros (out-of-range taps read them)
    int lds_floats;
    // in-launch prefetch: block 0 (dispatched first) draws the NEXT step's minibatch into the
    // staging slot with the 256-thread sampler body (k <= 2048: 3-block passes into 4096 LDS slots)
    int samp_on;
    SampleArgs samp;
    int64_t* stamps;           // diagnostic builds: slots 40..46 (first compute workgroup's phases, launch span)
};
struct MicroDxArgs {           // data gradients, last conv down to conv 2's input (stream 0)
    MicroConv c[MICRO_MAX_CONV];
    int nc, Bl, S, groups;
    const float* dF;           // [Bl][ldf] CHW-flatten dZ of the last conv (ELU' applied by the dense dx role)
    int ldf;
    int lds_d[MICRO_MAX_CONV]; // LDS float offset of each conv's dZ images [S][Ho*Wo][c.cs]
    int zero;
    int lds_floats;
    int nw;                    // waves per workgroup (4 or 8)
    int wasg[MICRO_MAX_CONV][8];   // per level, per wave: phase | first tile << 4 | tiles << 12 | first row tile << 16 | row tiles << 20
    int64_t* stamps;           // diagnostic builds: slots 47..52
};
struct MicroDwLayer {
    int Ci, Hi, Wi, Co, Ho, Wo, sh, sw;
    const float* D;            // dZ NHWC [Bl][Ho*Wo][Co] (stream 0)
    const float* X;            // input NHWC [Bl][Hi*Wi][Ci] (l >= 1), null for conv 1 (CHW ring rows)
    float* partial;            // [slices][Co*Ci*9 + Co], torch order [co][ci][i][j] then the bias
    int64_t pstride;
    int spw, slices, wg0;      // samples per slice, slices, first workgroup of this conv
    int G;                     // samples per LDS stage (the next stage's loads in flight)
    int skip;                  // tuning builds only: workgroups of this conv return at once (timing)
    int nct;                   // column tiles: Ci/16 ci tiles (l >= 1), ceil(Ci*9/16) (conv 1, torch column order)
    int wo_mul;                // q / Wo == (q * wo_mul) >> 16 for every pixel q < Ho*Wo + 4 (host-checked)
};
struct MicroDwArgs {
    MicroDwLayer L[MICRO_MAX_CONV];
    int nc, Bl, wgs;
    const float* ring_obs;     // conv 1 input: the micro grid of the gathered obs rows
    const int32_t* phys;
    int ring_stride, macro_len;
    int lds_floats;
    int64_t* stamps;           // diagnostic builds (-DDQNX_STAMPS): slots 24..39 (conv 1 workgroup 0)
    int32_t* err;              // &ctrl.error: a bounds check that skipped a slab store reports there
};
// plans (host): false if the net is outside what the micro kernels implement
bool micro_plan(const MicroConv* convs, int nc, int Bl, int nstreams, int n_cu, int* S, int* lds_floats);
bool micro_dx_plan(const MicroConv* convs, int nc, int Bl, int* S, int* lds_d, int* lds_floats);
void micro_dx_waves(MicroDxArgs& a);   // fills wasg (after micro_dx_plan accepted the net)
int micro_dw_plan(MicroDwArgs& a, int n_cu);
int micro_fwd_layout(MicroConv* c, int nc, int S, int* x0, int* zero);        // sets c[l].lds; LDS floats
int micro_dx_layout(const MicroConv* c, int nc, int S, int* lds_d, int* zero); // LDS floats   // fills spw / slices / wg0 / cs / lds; returns slices per conv via a
int launch_micro_fwd(const MicroFwdArgs& a, hipStream_t s);
int launch_micro_dx(const MicroDxArgs& a, hipStream_t s);
int launch_micro_dw(const MicroDwArgs& a, hipStream_t s);

int launch_im2col(const Im2colArgs& a, hipStream_t s);
int launch_flatten_concat(const FlattenArgs& a, hipStream_t s);
int launch_unflatten(const UnflattenArgs& a, hipStream_t s);
int launch_col2im(const Col2imArgs& a, int act, hipStream_t s);

int launch_per_sample(const PerSampleArgs& a, hipStream_t s);
int launch_per_update(const PerUpdateArgs& a, hipStream_t s);
int per_numpy121_init();

int launch_linear_fwd(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s);
// large-K dense layers (the (4,84,84) variant's 56,462 -> 512): 128x128 tiles, split-K
constexpr int FWD_BIG_BM = 128, FWD_BIG_BN = 128, FWD_BIG_KT = 32;
int fwd_big_ksplit(int M, int N, int K, int nprob, int64_t partial_floats, int* kchunk);
int launch_linear_fwd_big(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s);
// conv nets' dense 1 (M = Bl rows per stream, K = F): 64 x 64 tiles split over K into slabs
// (about two workgroups per CU), reduced in slab order by launch_linear_fwd_reduce
int fwd_split_ksplit(int M, int N, int K, int nprob, int n_cu, int* kchunk);
int launch_linear_fwd_split(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s);
int launch_linear_fwd_reduce(const FwdArgs& args, int nprob, int act, hipStream_t s);
int conv_dx_big_tiles(int Bl, int in);
int conv_dw_big_tiles(int in, int out);
int launch_conv_dw_big(const BwdArgs& a, hipStream_t s);
int launch_conv_dx_big(const BwdArgs& a, hipStream_t s);
void bwd_level_grid(BwdArgs& a);
int launch_bwd_level(const BwdArgs& a, int act, hipStream_t s);
int launch_head(const HeadArgs& a, int act, hipStream_t s);
bool head_supported(int F);
int launch_adam(const AdamArgs& a, hipStream_t s);
void dw_adam_grid(DwAdamArgs& a);
int launch_dw_adam(const DwAdamArgs& a, hipStream_t s);
int launch_dw_adam16(const DwAdam16Args& a, hipStream_t s);
// acting path (act.hip): Network.actions for MLP nets, one launch
constexpr int kActMaxDense = DQNX_MAX_DENSE;
constexpr size_t kActMaxLds = 64 * 1024;
struct ActArgs {
    const float* params;    // flat fp32 vector, named_parameters order
    const float* obs;       // [n][D]
    int32_t* actions;       // [n]
    float* values;          // [n][A] or null: Q (linear head) / advantages (dueling), the argmaxed values
    uint32_t* tickets;      // layer-1 arrival counter of row group g at tickets[-g] (zero between launches)
    float* scratch;         // [row groups * R][h0] layer-1 activations
    int n, D, L, A, F, dueling, act, ld;   // ld: LDS row stride (max layer width)
    int in[kActMaxDense], out[kActMaxDense];
    int64_t off[kActMaxDense];
    int64_t head_off;
    // dqnx_act_host: the last arriver stores done_seq here (system scope, after the actions) and the
    // host polls it instead of synchronising the stream (null: no flag)
    uint32_t* done_flag;
    uint32_t done_seq;
};
// two-stream acting: one conv layer over n rows (act_hybrid.hip); images CHW, rows strided
struct ActConvArgs {
    const float* in;  int64_t in_stride;  int in_off;    // input image of row r: in + r*in_stride + in_off
    const float* W;   const float* b;                    // [Co][Ci][kh][kw], [Co]
    float* out;       int64_t out_stride; int out_off;   // output [Co][Ho][Wo] of row r
    const float* macro; int64_t macro_stride; int macro_len;   // last conv: copy macro features after its output
    int n, Ci, Hi, Wi, Co, Ho, Wo, kh, kw, sh, sw, ph, pw;
};
size_t act_conv_lds_bytes(const ActConvArgs& a);
int launch_act_conv(const ActConvArgs& a, hipStream_t s);
int act_rows_per_block(int n, int ld);
uint64_t act_scratch_bytes(int n, int h0, int ld, int L, int out1);
int launch_act(const ActArgs& a, hipStream_t s);
int launch_soft_update(float* target, const float* p, int64_t n, float tau, float omt, hipStream_t s);
int launch_copy_i32x2(int32_t* d0, const int32_t* s0, int n0, int32_t* d1, const int32_t* s1, int n1, hipStream_t s);
int launch_replay_push(const PushArgs& a, hipStream_t s);

int launch_sample_uniform(const SampleArgs& a, hipStream_t s);
int launch_idx_to_phys(const int32_t* idx, int32_t* phys, int shard_begin, int n, dqnx_ctrl* ctrl, int64_t capacity,
                       const RelayoutArgs* rl, int rl_blocks, hipStream_t s);
int64_t sample_setsize(int64_t k);
int sample_hash_slots(int32_t k);            // hash slots of the sampler for k (LDS or global table)
uint64_t sample_table_bytes(int32_t k);      // global scratch the sampler needs for k (0: none)

}  // namespace dqnx
