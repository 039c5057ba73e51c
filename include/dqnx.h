/*
 * dqnx.h -- C ABI of the MI355X-native DQN learn-step engine (libdqnx.so).
 *
 * Drop-in boundary for the hot path of youcefMehamlia/Multimodal-DRL-RMC
 * (R: = /root/reference/).  The reference has no FFI: its "operator API" is the
 * duck-typed Python of dqn.agent / dqn.network / dqn.replay_memory, which the
 * Python host shim (multimodal-drl-rmc_amd/dqn/) keeps, calling the entry points
 * below through ctypes.  Each entry point names the reference interface it
 * replaces.  Plain C: pointers, sizes, enums; no torch types.  Streams are
 * hipStream_t passed as void*.  All device work is enqueued on the caller's
 * stream; nothing here synchronises unless its comment says so.
 *
 * Error convention: every function returns int (0 = DQNX_OK, < 0 = invalid
 * argument/state, > 0 = DQNX_ERR_HIP + hipError_t).  dqnx_last_error() returns a
 * thread-local message for the last failure.  No C++ exception crosses the ABI.
 *
 * Memory: the engine owns no device memory.  The caller allocates ONE device arena
 * of dqnx_engine_arena_bytes() bytes and binds it; dqnx_engine_buffer() gives the
 * offset of every region inside it (parameters, Adam moments, replay ring, SumTree,
 * control block, workspace), so a host framework can view them (the Python shim
 * makes torch views so state_dict()/load_state_dict() keep working).
 */
#ifndef DQNX_H
#define DQNX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQNX_ABI_VERSION 3

/* ---- status codes ---------------------------------------------------------------- */
#define DQNX_OK 0
#define DQNX_EINVAL (-1)      /* bad argument */
#define DQNX_ESTATE (-2)      /* call not valid in the engine's current state (e.g. unbound) */
#define DQNX_EUNSUPPORTED (-3)/* configuration outside what the engine implements */
#define DQNX_EDEVICE (-4)     /* device-side sticky error word was set (see dqnx_ctrl.error) */
#define DQNX_ERR_HIP 1000     /* DQNX_ERR_HIP + hipError_t */

/* ---- enums ------------------------------------------------------------------------- */
enum dqnx_net_kind { DQNX_NET_MLP = 0, DQNX_NET_TWO_STREAM = 1 };
enum dqnx_head_kind { DQNX_HEAD_LINEAR = 0, DQNX_HEAD_DUELING = 1 };
enum dqnx_activation { DQNX_ACT_RELU = 0, DQNX_ACT_ELU = 1 };
/* Arithmetic of the network GEMMs.  FP32 is the reference's (parity within 1e-5).  BF16
 * (BASELINE config 5): forward and dZ-chain GEMM operands rounded to bf16 (RNE), fp32
 * accumulate; bias, activations, TD target, Huber, weight gradients, Adam and the master
 * weights stay fp32.  MLP networks only. */
enum dqnx_compute_dtype { DQNX_COMPUTE_FP32 = 0, DQNX_COMPUTE_BF16 = 1 };
/* Learner algorithm = which Agent.learn() runs:
 *   DQNX_ALGO_DQN        SimpleAgent.learn          R:dqn/agent.py:166-185  (DQNAgent)
 *   DQNX_ALGO_DOUBLE     DoubleAgent.learn          R:dqn/agent.py:204-226  (DoubleDQNAgent,
 *                                                                            DuelingDoubleDQNAgent)
 *   DQNX_ALGO_PER_DOUBLE PerDoubleAgent.learn       R:dqn/agent.py:245-272  (PerDuelingDoubleDQNAgent) */
enum dqnx_algo { DQNX_ALGO_DQN = 0, DQNX_ALGO_DOUBLE = 1, DQNX_ALGO_PER_DOUBLE = 2 };

/* ---- network description (replaces nn_conf_func / network_config) ----------------
 * MLP:        R:env/custom_env/macro with lane/dqn_config.py:58-104
 *             nn.Sequential(Linear(D,h0), act, Linear(h0,h1), act, ...)
 * TWO_STREAM: TwoStreamHybridNetwork R:env/dqn_config.py:66-143 (network_config :148-193)
 * heads:      DeepQNetwork fc_out (R:dqn/network.py:50-65), DuelingDeepQNetwork
 *             fc_val/fc_adv + aggregate (R:dqn/network.py:77-96). */
#define DQNX_MAX_DENSE 6
#define DQNX_MAX_CONV 4
typedef struct dqnx_net_desc {
    int32_t kind;              /* dqnx_net_kind */
    int32_t head;              /* dqnx_head_kind */
    int32_t activation;        /* dqnx_activation of the body (MLP: ReLU, hybrid: ELU) */
    int32_t obs_dim;           /* D: length of one flat observation */
    int32_t n_actions;         /* A */
    int32_t n_dense;           /* number of body Linear layers (MLP) / dense_stream layers */
    int32_t dense[DQNX_MAX_DENSE];
    /* TWO_STREAM only: obs = [macro (macro_len) | micro grid viewed as (c,h,w)] */
    int32_t macro_len;
    int32_t micro_c, micro_h, micro_w;
    int32_t n_conv;
    int32_t conv_out[DQNX_MAX_CONV], conv_kh[DQNX_MAX_CONV], conv_kw[DQNX_MAX_CONV];
    int32_t conv_sh[DQNX_MAX_CONV], conv_sw[DQNX_MAX_CONV];
} dqnx_net_desc;

/* One parameter tensor of the flat parameter vector, in torch named_parameters()
 * order (= state_dict order, = the order Adam iterates).  Names are the reference's
 * state_dict keys (e.g. "net.0.weight", "fc_adv.bias"). */
typedef struct dqnx_param_info {
    char name[48];
    int64_t offset;            /* element offset in the flat fp32 vector */
    int64_t numel;
    int32_t ndim;
    int32_t shape[4];
} dqnx_param_info;

/* Total fp32 parameter count and tensor count of a network (host only, no GPU). */
int dqnx_net_param_count(const dqnx_net_desc* net, int64_t* n_params, int32_t* n_tensors);
int dqnx_net_param_info(const dqnx_net_desc* net, int32_t index, dqnx_param_info* out);

/* ---- engine configuration (replaces the Agent constructor kwargs, R:dqn/agent.py:19-52,
 *      with the hyper-parameters of R:env/dqn_config.py:26-56) -------------------- */
typedef struct dqnx_config {
    dqnx_net_desc net;
    int32_t algo;              /* dqnx_algo */
    int32_t batch;             /* global minibatch = batch_size (k of random.sample) */
    int32_t world_size;        /* data-parallel ranks (1 = single GPU) */
    int32_t rank;              /* this rank: processes samples [rank*batch/world, (rank+1)*batch/world) */
    int64_t capacity;          /* buffer_size (deque maxlen / SumTree capacity) */
    /* hyper-parameters are doubles, like the reference's Python floats; the engine casts
     * them to fp32 exactly where torch does (tensor * Python float). */
    double gamma;              /* discount */
    double lr;                 /* Adam lr */
    double beta1, beta2, adam_eps;  /* torch.optim.Adam defaults 0.9, 0.999, 1e-8 */
    double tau;                /* target_soft_update_tau */
    int32_t n_env;             /* soft update uses tau*n_env (R:dqn/agent.py:108-109) */
    int32_t local_sampling;    /* world_size > 1, uniform replay only: 0 = every rank draws the same
                                  global minibatch of `batch` (bit-exact with one GPU) and takes its
                                  shard; 1 = each rank draws its own batch/world_size positions from
                                  its own RNG stream (plain data parallelism; O(batch/world) sampling) */
    /* ReplayMemoryPrioritized constants (R:dqn/replay_memory.py:49-54) */
    double per_eps, per_alpha, per_max_priority;
    double per_beta_start, per_beta_end, per_beta_steps;   /* beta = interp(step,[0,steps],[start,end]) */
    int32_t compute_dtype;     /* dqnx_compute_dtype (ABI 2) */
    int32_t per_numpy121;      /* PER tree arithmetic of the reference's pinned numpy 1.21: 0 (default) =
                                  numpy >= 2 (NEP 50: `change` and the ancestor sums in float64, exact);
                                  1 = numpy 1.21 value-based casting: update_batch_priorities' float32
                                  `change` and float32-rounded ancestor sums, applied in update order
                                  (R:dqn/utils/sum_tree.py:18, 31-32; R:bin/environment.yml pins 1.21) */
} dqnx_config;

/* Fill cfg with the reference's HYPER_PARAMS defaults for the given network. */
void dqnx_config_defaults(dqnx_config* cfg);

/* ---- device control block (lives in the arena; layout is ABI) ------------------- */
typedef struct dqnx_ctrl {
    uint32_t py_mt[625];       /* CPython random state: random.getstate()[1] (624 words + index) */
    uint32_t np_mt[625];       /* numpy legacy RandomState: get_state()[1] keys + [2] pos */
    int64_t ring_size;         /* len(replay deque) / SumTree.size */
    int64_t ring_wptr;         /* next physical write slot (SumTree.data_pointer) */
    int64_t adam_step;         /* torch Adam state['step'] (same for every tensor) */
    int64_t agent_step;        /* agent.step * n_env handed to PER sample_transitions */
    int64_t per_max_idx;       /* SumTree.max_priority_index (tree index) */
    int64_t per_min_idx;       /* SumTree.min_priority_index (tree index) */
    float loss;                /* loss of the last learn step (global batch mean) */
    int32_t error;             /* sticky device error code, 0 = ok */
    float adam_step_size;      /* -lr / bias_correction1 of the current step (fp32) */
    float adam_bc2_sqrt;       /* sqrt(bias_correction2) of the current step (fp32) */
    double per_beta;           /* beta used by the last PER sample */
    int64_t reserved[8];
} dqnx_ctrl;

/* device error codes written to dqnx_ctrl.error */
#define DQNX_DEVERR_SAMPLE_TOO_LARGE 1   /* random.sample: k > n (ValueError) */
#define DQNX_DEVERR_EMPTY_TREE 2         /* PER sample with total priority 0 */
#define DQNX_DEVERR_PER_HANDOFF 3        /* internal: a PER update hand-off inside one launch timed out */
#define DQNX_DEVERR_FWD_PAIR_HANDOFF 4   /* internal: the paired-column forward's H_1 hand-off timed out */
/* internal: a write outside its range was skipped (bounds checks on the DP-bucket write paths) */
#define DQNX_DEVERR_BOUNDS_ADAM_WIDE 16  /*   k_adam4 wide path: a float4 outside [e0, n_params) of the launch */
#define DQNX_DEVERR_BOUNDS_ADAM_PERM 17  /*   k_adam4 wide path: a permuted conv-weight copy outside the range */
#define DQNX_DEVERR_BOUNDS_MICRO_DW 18   /*   k_micro_dw: a split-K slab tile outside its conv's slabs */

/* ---- engine lifetime --------------------------------------------------------------- */
typedef struct dqnx_engine dqnx_engine;

int dqnx_engine_create(const dqnx_config* cfg, dqnx_engine** out);
int dqnx_engine_destroy(dqnx_engine* e);
/* Bytes of the single device arena the engine needs (host only). */
int dqnx_engine_arena_bytes(const dqnx_engine* e, uint64_t* bytes);

/* Arena regions. */
enum dqnx_buffer {
    DQNX_BUF_PARAMS = 0,       /* online network flat fp32 params (named_parameters order) */
    DQNX_BUF_TARGET_PARAMS,    /* target network flat params */
    DQNX_BUF_GRADS,            /* flat fp32 gradient of the last learn step (all-reduced under DP) */
    DQNX_BUF_ADAM_M,           /* Adam exp_avg */
    DQNX_BUF_ADAM_V,           /* Adam exp_avg_sq */
    DQNX_BUF_CTRL,             /* dqnx_ctrl */
    DQNX_BUF_RING_OBS,         /* [capacity][obs_stride] fp32 */
    DQNX_BUF_RING_NEXT_OBS,    /* [capacity][obs_stride] fp32 */
    DQNX_BUF_RING_ACT,         /* [capacity] int32 */
    DQNX_BUF_RING_REW,         /* [capacity] fp32 */
    DQNX_BUF_RING_DONE,        /* [capacity] fp32 (0/1) */
    DQNX_BUF_SUMTREE,          /* [2*capacity-1] fp64 (PER only, else 0 bytes) */
    DQNX_BUF_BATCH_IDX,        /* [2][batch] int32: sampled logical replay positions / tree leaves;
                                  slot 0 unless DQNX_STEP_PREFETCH alternates the slots */
    DQNX_BUF_Q,                /* [3][batch_local][n_actions] fp32: Q online(s), online(s'), target(s') */
    DQNX_BUF_TD,               /* [3][batch_local] fp32: targets y, q(s,a), |y - q(s,a)| */
    DQNX_BUF_IS_WEIGHTS,       /* [batch] fp32 PER importance weights */
    DQNX_BUF_WORKSPACE,        /* everything else (activations, partial slabs, scratch) */
    DQNX_BUF_PER_ABS_TD,       /* [batch] fp32 |targets - q(s,a)| of the GLOBAL minibatch (PER only):
                                  each rank's learn step writes its shard; under DP the caller
                                  all-gathers it in place before dqnx_apply_grads */
    DQNX_BUF_COUNT
};
int dqnx_engine_buffer(const dqnx_engine* e, int32_t which, uint64_t* offset, uint64_t* bytes);
/* Row stride (in floats) of the replay observation rings (>= obs_dim, multiple of 4). */
int dqnx_engine_obs_stride(const dqnx_engine* e, int32_t* stride);
/* Bind the caller-allocated arena (device pointer, 256-byte aligned). */
int dqnx_engine_bind(dqnx_engine* e, void* arena, uint64_t bytes);
/* The caller wrote the parameters (DQNX_BUF_PARAMS / DQNX_BUF_TARGET_PARAMS) directly, e.g. a
 * checkpoint load through state_dict() views (R:dqn/network.py:37-47, R:dqn/agent.py:112-121):
 * the next learn step rebuilds the engine's derived weight layouts.  Host only, no device work.
 * (dqnx_soft_update / dqnx_hard_update / dqnx_engine_reset imply it.) */
int dqnx_params_modified(dqnx_engine* e);
/* Zero Adam moments, ring state, tree, control block (params untouched); stream-ordered. */
int dqnx_engine_reset(dqnx_engine* e, void* stream);
/* Use hipGraph capture/replay for learn steps (default OFF: measured on MI355X / ROCm 7.2, every
 * hipGraphLaunch leaves ~8.5 us between the previous graph's last kernel and its first one, while
 * back-to-back kernel launches on one stream leave ~0; eager steps are 3-4 us faster at every
 * configuration measured -- MLP B=1024 / 4096, PER, bf16 B=8192, two-stream). */
int dqnx_engine_set_graphs(dqnx_engine* e, int32_t enabled);

/* ---- replay ring: replaces ReplayMemoryNaive/Prioritized.store_transitions
 *      (R:dqn/replay_memory.py:30-36, :56-67) via Agent.store_transitions (R:dqn/agent.py:80-84).
 * Appends n transitions (evicting the oldest when full).  Pointers are host memory
 * (src_on_device = 0; up to 64 rows are copied into an engine-owned pinned block at once and sent
 * with one async copy -- the caller's arrays are free on return; larger pushes are copied with
 * hipMemcpyAsync and the call synchronises the stream) or device memory (src_on_device = 1).  obs rows are
 * obs_dim floats, contiguous.  done: 0/1 bytes.  Under PER new leaves get the current
 * max priority (1.0 when the tree is empty), exactly as the reference. */
int dqnx_replay_push(dqnx_engine* e, const float* obs, const int32_t* act, const float* rew,
                     const uint8_t* done, const float* next_obs, int32_t n, int32_t src_on_device,
                     void* stream);

/* ---- prioritised replay (DQNX_ALGO_PER_DOUBLE) ------------------------------------
 * The SumTree lives in DQNX_BUF_SUMTREE with the reference's layout (leaf of ring slot s
 * = tree index s + capacity - 1); its max/min priority indices in dqnx_ctrl.
 * dqnx_per_sample: ReplayMemoryPrioritized.sample_transitions(step) (R:dqn/replay_memory.py:69-92)
 *   -> ring slots into DQNX_BUF_BATCH_IDX slot 0, IS weights into DQNX_BUF_IS_WEIGHTS; consumes
 *   numpy global-state words from dqnx_ctrl.np_mt and advances dqnx_ctrl.agent_step by n_env.
 *   A PER learn step does this itself.
 * dqnx_per_update_priorities: update_batch_priorities(tree_indices, abs_td_errors)
 *   (R:dqn/replay_memory.py:94-98) for n (ring slot, |delta|) pairs in device memory, in order.
 *   A PER learn step does this itself (after the all-gather under DP: dqnx_apply_grads).
 * dqnx_set_agent_step: the `self.step * self.n_env` the next PER sample interpolates beta from
 *   (R:dqn/agent.py:247). */
int dqnx_per_sample(dqnx_engine* e, void* stream);
int dqnx_per_update_priorities(dqnx_engine* e, const int32_t* slots, const float* abs_td, int32_t n, void* stream);
int dqnx_set_agent_step(dqnx_engine* e, int64_t step_times_n_env, void* stream);

/* ---- RNG state exchange (Python random / numpy legacy global state) -------------- */
enum dqnx_rng { DQNX_RNG_PY = 0, DQNX_RNG_NP = 1 };
/* Upload 625 words (624 + index) into the control block (host pointer; stream-ordered,
 * the copy is complete when this returns). */
int dqnx_rng_set(dqnx_engine* e, int32_t which, const uint32_t* state625, void* stream);
/* Download 625 words; synchronises the stream. */
int dqnx_rng_get(dqnx_engine* e, int32_t which, uint32_t* state625, void* stream);
/* The same two copies, stream-ordered and WITHOUT a synchronisation: `state625` must be pinned
 * (page-locked) host memory that the caller keeps unchanged (set) / does not read (get) until the
 * copy has executed (e.g. an event recorded after it).  The drop-in Agent uses them to hand the
 * sampler's RNG to and from Python's global `random` / numpy state without a host round trip per
 * learn() (dqn/agent.py).  Same argument checks as dqnx_rng_set / dqnx_rng_get; refused while a
 * prefetched minibatch is pending. */
int dqnx_rng_set_async(dqnx_engine* e, int32_t which, const uint32_t* state625, void* stream);
int dqnx_rng_get_async(dqnx_engine* e, int32_t which, uint32_t* state625, void* stream);

/* The whole control block (both RNG states, ring size, loss, sticky error, ...) into PINNED host memory
 * (sizeof(dqnx_ctrl) bytes), stream-ordered and without a synchronisation: the drop-in Agent reads it
 * back after each launched learn step and checks the sticky error and its RNG mirror (below) at its
 * next synchronisation point, so a device error reaches the caller without a host round trip per step. */
int dqnx_ctrl_get_async(dqnx_engine* e, void* dst, void* stream);

/* ---- host-side RNG stream mirror (host only, no device work) -----------------------------------
 * The reference draws the minibatch inside Agent.learn() from the interpreter's global generators
 * (R:dqn/replay_memory.py:38-39 random.sample; :79-80 np.random.uniform once per sample), so the
 * caller's `random` / `np.random` have moved on when learn() returns.  The device sampler draws the
 * minibatch; these tell the host how far that draw moves the stream, so the Agent advances its global
 * generator at learn() time without waiting for the GPU (R:dqn/agent.py:204-226 stays synchronous
 * from the caller's view) and checks the device's returned state against `out625` later.
 * dqnx_rng_sample_words: the 32-bit words CPython's random.sample(population of n, k) consumes from
 *   `state625` (its _randbelow rejections and the set branch's duplicate redraws depend on the values,
 *   so the stream is walked); `out625` (may be NULL) receives the state after the draw.  k > n returns
 *   DQNX_EINVAL with random.sample's ValueError message.
 * dqnx_rng_advance: `out625` = `state625` advanced by `words` MT19937 outputs (numpy's legacy uniform
 *   takes two per draw). */
int dqnx_rng_sample_words(const uint32_t* state625, int64_t n, int32_t k, uint32_t* out625, int64_t* words);
int dqnx_rng_advance(const uint32_t* state625, int64_t words, uint32_t* out625);

/* ---- the learn step: replaces Agent.learn() (R:dqn/agent.py:166-185 / 204-226 /
 *      245-272) and, with DQNX_STEP_SOFT_UPDATE, the following
 *      Agent.update_target_network() soft update (R:dqn/agent.py:105-110; caller
 *      R:train.py:99-101).
 * Stream-ordered; returns without synchronising.  Reads ring size/RNG/step from the
 * control block, so consecutive calls need no host round trip. */
#define DQNX_STEP_SOFT_UPDATE 0x1   /* fuse the tau soft update into the Adam pass */
#define DQNX_STEP_GIVEN_INDICES 0x2 /* skip sampling: use DQNX_BUF_BATCH_IDX as written by caller */
#define DQNX_STEP_GRADS_ONLY 0x4    /* stop after writing DQNX_BUF_GRADS (DP: all-reduce, then apply) */
#define DQNX_STEP_PREFETCH 0x8      /* pure learning loops: also draw the NEXT step's minibatch,
                                       overlapped with this step's compute (fused MLP plan: by one
                                       more workgroup of the last launch; per-layer plan: on a
                                       side stream).
                                       Results are bit-identical to sequential steps; while a
                                       prefetched minibatch is pending, dqnx_replay_push and
                                       dqnx_rng_set return DQNX_ESTATE and dqnx_rng_get already
                                       reflects the prefetched draw.  A step without the flag
                                       consumes the pending minibatch. */
int dqnx_learn_step(dqnx_engine* e, int32_t flags, void* stream);
/* Same-stream rule for DQNX_STEP_PREFETCH: the engine remembers the stream of the step that
 * left a draw pending; dqnx_rng_get synchronises THAT stream, and a later step on another
 * stream synchronises it first.  A caller that captures prefetching steps into its own graph
 * (dqn.data_parallel.GraphedDPStep) must replay the graph on the capture's stream or call
 * dqnx_prefetch_stream() with the replay stream before dqnx_rng_get. */
int dqnx_prefetch_stream(dqnx_engine* e, void* stream);
/* Draw the first minibatch of a prefetching loop now (no-op when a draw is pending or the
 * configuration does not draw ahead), so that the next DQNX_STEP_PREFETCH step can be captured
 * into a caller's graph without its prologue (dqn.data_parallel.GraphedDPStep). */
int dqnx_prefetch_begin(dqnx_engine* e, int32_t flags, void* stream);
/* `count` (1..256) consecutive learn steps, bitwise equal to `count` dqnx_learn_step(flags) calls
 * (flags: 0 or DQNX_STEP_SOFT_UPDATE).  Replaces a loop of Agent.learn() +
 * update_target_network() with no host work in between (R:train.py:99-101 repeated, e.g. several
 * gradient steps per environment step).  Uniform replay on the fused MLP plan runs them as ONE
 * graph in which step i's last launch also draws step i+1's minibatch; other configurations
 * run the steps one by one.  Nothing is pending afterwards. */
int dqnx_learn_steps(dqnx_engine* e, int32_t flags, int32_t count, void* stream);
/* Adam (+ optional soft update) from DQNX_BUF_GRADS: second half of a GRADS_ONLY step. */
int dqnx_apply_grads(dqnx_engine* e, int32_t flags, void* stream);
/* ---- bucketed data-parallel step (conv nets) -----------------------
 * The DQNX_STEP_GRADS_ONLY step cut where a layer's weight gradient is complete, so the caller
 * can all-reduce a finished bucket (on a side stream) while the engine runs the rest of the
 * backward, and apply Adam to it before the last bucket arrives.  Bucket 0 = dense layers +
 * Q head + the loss slot (done after the dense backward), then one bucket per conv, last conv
 * first.  The fused MLP plan (up to 2048 rows per GPU): bucket 0 = every layer but layer 1 + the
 * head + the loss slot, bucket 1 = layer 1 (its weight-gradient tiles as a launch of their own); the
 * slab plan's MLP has one bucket.  Each bucket is a contiguous range of DQNX_BUF_GRADS /
 * DQNX_BUF_PARAMS.  Enqueue dqnx_learn_step_bucket for b = 0, 1, ... in order on one stream;
 * dqnx_apply_grads_bucket(b) after bucket b's all-reduce (bucket 0's also applies the PER tree
 * update).  Together they equal dqnx_learn_step(GRADS_ONLY) + dqnx_apply_grads, bit for bit.
 * Replaces the single all-reduce of dqn/data_parallel.py's unbucketed step (no reference call
 * site: the reference trains on one device). */
int dqnx_dp_bucket_count(dqnx_engine* e, int32_t* n);
int dqnx_dp_bucket_info(dqnx_engine* e, int32_t bucket, int64_t* first, int64_t* count);
int dqnx_learn_step_bucket(dqnx_engine* e, int32_t flags, int32_t bucket, void* stream);
int dqnx_apply_grads_bucket(dqnx_engine* e, int32_t flags, int32_t bucket, void* stream);
/* Agent.update_target_network (R:dqn/agent.py:101-110): soft (tau*n_env) or hard copy. */
int dqnx_soft_update(dqnx_engine* e, void* stream);
int dqnx_hard_update(dqnx_engine* e, void* stream);

/* ---- acting path: replaces Network.actions (DeepQNetwork R:dqn/network.py:67-74: argmax of Q;
 *      DuelingDeepQNetwork R:dqn/network.py:110-117: argmax of the advantage stream only), as
 *      called by Agent.choose_actions (R:dqn/agent.py:92-99) before the epsilon-greedy override.
 * Stateless: `params` is a device fp32 vector in the layout of dqnx_net_param_info (the engine's
 * DQNX_BUF_PARAMS / DQNX_BUF_TARGET_PARAMS, or any flat copy).  obs: device [n][obs_dim];
 * actions: device int32[n] (first maximal index, like torch.argmax); values: device [n][n_actions]
 * or NULL (receives the argmaxed values: Q, or the advantages for a dueling head).  scratch:
 * 16-byte aligned device buffer of scratch_bytes >= dqnx_act_scratch_bytes(net, n) bytes (a
 * multiple of 4), zero-filled before its first use; every call leaves it ready for the next, so
 * calls with any n up to its size may share it on one stream.  MLP nets: one launch.  Two-stream
 * nets (TwoStreamHybridNetwork, R:env/dqn_config.py:66-143): one launch per conv layer, then the
 * dense stream + head as for an MLP on cat(flatten(conv), macro).  Stream-ordered, no sync. */
uint64_t dqnx_act_scratch_bytes(const dqnx_net_desc* net, int32_t n);
int dqnx_act(const dqnx_net_desc* net, const float* params, const float* obs, int32_t n, int32_t* actions,
             float* values, void* scratch, uint64_t scratch_bytes, void* stream);

/* ---- drop-in Agent fast path: one host call per agent method (R:train.py:88-108) ---------------
 * dqnx_agent_stage_rng: Agent.learn()'s draw source -- snapshot `state625` (the caller's
 *   random.getstate()[1], or numpy's legacy keys + pos under PER) into the engine's pinned staging
 *   block for the next dqnx_agent_launch, and return in *words the MT19937 outputs the device draw will
 *   consume (the host advances its generator by them, dqnx_rng_sample_words / dqnx_rng_advance).  The
 *   post-draw state is remembered and checked against the device's at dqnx_agent_readback.  Uniform
 *   replay with fewer stored transitions than the batch: DQNX_EINVAL with random.sample's ValueError
 *   text (R:dqn/replay_memory.py:39).  Host only.
 * dqnx_agent_launch: the staged state's upload, dqnx_learn_step(flags) (DQNX_STEP_SOFT_UPDATE allowed),
 *   then the control block into an engine-owned pinned copy with an event; stream-ordered, no wait.
 * dqnx_agent_readback: 1 when the last launch's control block has arrived (wait = 1 blocks until it
 *   has), copied to `out` (may be NULL); 0 when none is pending or (wait = 0) it has not arrived yet;
 *   DQNX_EDEVICE when it carries a sticky device error (dqnx_ctrl.error) or its RNG state differs from
 *   the host mirror (dqnx_last_error() says which).
 * dqnx_act_host: dqnx_act with HOST obs [n][obs_dim] and HOST actions [n]: the obs through pinned
 *   memory into the END of `scratch` (dqnx_act_host_scratch_bytes(net, n) bytes, zero-filled before
 *   its first use), one launch sequence, the actions back; synchronises `stream` (Network.actions,
 *   R:dqn/network.py:67-74, 110-117). */
int dqnx_agent_stage_rng(dqnx_engine* e, int32_t which, const uint32_t* state625, int64_t* words);
int dqnx_agent_launch(dqnx_engine* e, int32_t flags, void* stream);
/* dqnx_agent_learn_mt: Agent.learn() on the caller's LIVE generator, uniform replay: `mt` = its 624
 *   MT19937 state words and `*pos` its output position (CPython's RandomObject holds them as
 *   `int index; uint32_t state[624]`: the drop-in passes the addresses inside random._inst after
 *   checking the layout against random.getstate()).  Staged as dqnx_agent_stage_rng(DQNX_RNG_PY)
 *   stages mt + pos, then advanced IN PLACE past the words the draw consumes (*words), i.e. the
 *   generator is left where random.sample(deque, batch_size) leaves it (R:dqn/replay_memory.py:39);
 *   with DQNX_AGENT_LAUNCH in flags, dqnx_agent_launch(flags without it) follows in the same call.
 *   One library call per learn() instead of getstate + stage + getrandbits + launch. */
#define DQNX_AGENT_LAUNCH 0x100
int dqnx_agent_learn_mt(dqnx_engine* e, uint32_t* mt, int32_t* pos, int32_t flags, void* stream, int64_t* words);
int dqnx_agent_readback(dqnx_engine* e, int32_t wait, dqnx_ctrl* out);
/* dqnx_agent_quiesce: waits for what dqnx_agent_launch / dqnx_agent_learn_mt would wait on before
 *   launching (the previous step's unread control-block readback); no state changes.  The drop-in
 *   calls it, with the GIL released, before a dqnx_agent_learn_mt (GIL held) whose previous readback
 *   is still unread, so no other Python thread is blocked for the length of a GPU wait. */
int dqnx_agent_quiesce(dqnx_engine* e);
/* dqnx_agent_choose: Agent.choose_actions(obses) (R:dqn/agent.py:92-99) in ONE call, MLP nets on the
 *   engine's online parameters: the greedy actions of the n HOST rows at obs_host (dqnx_act_host's
 *   launch: the advantage stream for dueling nets, R:dqn/network.py:110-117), and -- while the acting
 *   kernel runs -- for every env i in order: u = random.random() from the caller's LIVE MT19937 (mt =
 *   its 624 words, *pos its index, advanced in place as dqnx_agent_learn_mt does: CPython's
 *   genrand_res53, 2 words); if u <= epsilon, actions[i] = random.randint(0, n_actions - 1)
 *   (_randbelow: getrandbits(n_actions.bit_length()) redrawn while >= n_actions).  Then the wait for
 *   the kernel and the last agent step's control-block checks (as dqnx_agent_readback(wait = 1)).
 *   `scratch` as dqnx_act_host's (dqnx_act_host_scratch_bytes(&cfg.net, n)); n <= DQNX_CHOOSE_MAX_ENVS.
 *   flags & DQNX_CHOOSE_GIL_HELD: the caller holds the Python GIL (it must, for the in-place generator
 *   update); the GIL is released around the GPU wait (PyEval_SaveThread / PyEval_RestoreThread of the
 *   running interpreter). */
#define DQNX_CHOOSE_MAX_ENVS 256
#define DQNX_CHOOSE_GIL_HELD 0x1
int dqnx_agent_choose(dqnx_engine* e, const float* obs_host, int32_t n, double epsilon, uint32_t* mt, int32_t* pos,
                      int32_t* actions_out, void* scratch, uint64_t scratch_bytes, int32_t flags, void* stream);
uint64_t dqnx_act_host_scratch_bytes(const dqnx_net_desc* net, int32_t n);
int dqnx_act_host(const dqnx_net_desc* net, const float* params, const float* obs_host, int32_t n,
                  int32_t* actions_host, void* scratch, uint64_t scratch_bytes, void* stream);

/* ---- kernel-level timing (bench.py roofline) ---------------------------------------
 * A learn step is an ordered list of kernel launches (sample, linear_fwd_l1.., head_td_loss,
 * linear_bwd_lL..l1, adam_fused).  dqnx_learn_step_timed runs one whole step exactly like
 * dqnx_learn_step but records ev_start/ev_stop (hipEvent_t) around kernel `kernel_index`
 * on `stream` (the sub-ranges before/after it are graph-replayed separately).
 * kernel_count / kernel_info / step_omit with DQNX_STEP_PREFETCH describe the steady-state step
 * of a prefetching loop where the in-launch prefetch applies (no sampler launch; the last
 * launch, "dw_adam16+sample", also draws the next minibatch). */
int dqnx_learn_kernel_count(dqnx_engine* e, int32_t flags, int32_t* n);
int dqnx_learn_kernel_info(dqnx_engine* e, int32_t flags, int32_t index, char* name, int32_t name_len,
                           double* algorithmic_flops, double* algorithmic_bytes);
int dqnx_learn_step_timed(dqnx_engine* e, int32_t flags, int32_t kernel_index, void* ev_start, void* ev_stop,
                          void* stream);
/* Timing aid (bench.py roofline): one learn step (graph-launched when graphs are on), with kernel
 * `omit_index` (as numbered by dqnx_learn_kernel_info; -1 = none) left out.  Engine state
 * afterwards is meant for timing only. */
int dqnx_learn_step_omit(dqnx_engine* e, int32_t flags, int32_t omit_index, void* stream);

int dqnx_events_create(int32_t n, void** events);      /* hipEventCreate x n */
int dqnx_events_destroy(int32_t n, void** events);
int dqnx_event_elapsed(void* start, void* stop, float* ms);   /* synchronises `stop` */

/* ---- sampler (test hook): random.sample positions on device.
 * R:dqn/replay_memory.py:38-39.  mt625: device uint32[625] (advanced in place);
 * n: population size; k: sample size; out: device int32[k].  scratch: device buffer of
 * dqnx_sample_scratch_bytes(n, k) bytes.  err: device int32 (set to 1 if k > n).
 * BLOCKING and not capturable: it stages n into `scratch` from a host stack value and
 * synchronises `stream` before the launch.  Learn steps never call it (their samplers read the
 * ring size from the control block, stream-ordered). */
uint64_t dqnx_sample_scratch_bytes(int64_t n, int32_t k);
int dqnx_sample_uniform(uint32_t* mt625, int64_t n, int32_t k, int32_t* out, void* scratch,
                        int32_t* err, void* stream);

/* ---- misc ------------------------------------------------------------------------ */
const char* dqnx_last_error(void);
int32_t dqnx_abi_version(void);
/* Diagnostic builds only (-DDQNX_STAMPS): copy the 64 s_memtime phase stamps written by
 * block 0 of the sampler / head kernels (synchronises).  Returns DQNX_EUNSUPPORTED in
 * production builds. */
int dqnx_debug_stamps(dqnx_engine* e, int64_t* out64, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DQNX_H */
