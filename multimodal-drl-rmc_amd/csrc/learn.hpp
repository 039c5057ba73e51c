// Kernel argument structs and launchers shared by learn.hip / conv.hip / engine.cpp.
#pragma once
#include "common.hpp"

namespace dqnx {

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
};

struct BwdArgs {
    // dx role (skipped when dZprev == null)
    const float* W;        // [out][in]
    const float* Hprev;    // activations of the previous layer, stream 0 [Bl][ldh]
    int ldh;
    float* dZprev;         // [Bl][in]
    // dw role
    const float* X;        // layer input rows [Bl][ldx] (stream 0)
    int ldx;
    float* partial;        // [slices][out*in + out]
    int64_t pstride;
    int kslice;
    // shared
    const float* dZ;       // [Bl][out]
    int Bl, in, out;
    // grid bookkeeping (bwd_level_grid)
    int dx_blocks, dx_grid_x, dw_grid_x, dw_grid_y;
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
    float* Q;              // [3][Bl][A]
    float* td;             // [3][Bl]: y, q(s,a), |y - q(s,a)|
    float* dZ;             // [Bl][F]
    float* head_partial;   // [tiles][head_params]
    float* loss_partial;   // [tiles]
    dqnx_ctrl* ctrl;       // Adam step bookkeeping (block 0) or null
    float beta1, beta2, lr;
};

constexpr int kMaxSeg = 10;
struct AdamSegment {
    int64_t off;           // first flat element of the segment
    const float* partial;  // slab 0 of the segment's partials
    int64_t pstride;       // elements between slabs
    int S;                 // number of slabs
};
struct AdamArgs {
    AdamSegment seg[kMaxSeg];
    int nseg;
    int mode;              // 0 partials->grads, 1 partials->grads+adam, 2 grads->adam
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
};

struct SampleArgs {
    uint32_t* state;          // [625]
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
};

int launch_linear_fwd(const FwdArgs& args, int nprob, int act, bool vecb, hipStream_t s);
void bwd_level_grid(BwdArgs& a);
int launch_bwd_level(const BwdArgs& a, int nslices, int act, hipStream_t s);
int launch_head(const HeadArgs& a, int act, hipStream_t s);
int launch_adam(const AdamArgs& a, hipStream_t s);
int launch_soft_update(float* target, const float* p, int64_t n, float tau, float omt, hipStream_t s);
int launch_replay_push(const PushArgs& a, hipStream_t s);

int launch_sample_uniform(const SampleArgs& a, hipStream_t s);
int launch_idx_to_phys(const int32_t* idx, int32_t* phys, int shard_begin, int n, dqnx_ctrl* ctrl, int64_t capacity, hipStream_t s);
int64_t sample_setsize(int64_t k);
int sample_hash_slots(int32_t k);

}  // namespace dqnx
