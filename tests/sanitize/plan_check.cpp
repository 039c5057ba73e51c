// Host-only sanitizer driver for libdqnx's host engine (SURVEY.md §5 "race detection /
// sanitizers": ASan / UBSan builds of the C++ host side).  Built by `make -C
// multimodal-drl-rmc_amd sanitize` from host-only objects (--offload-host-only, no device code)
// with -fsanitize=address,undefined, and run by tests/test_sanitize.py on the CPU.
//
// It drives every host-side planning path of include/dqnx.h without a GPU: network planning
// and parameter tables, engine creation (arena layout, kernel plans for every network family,
// algorithm, dtype, batch and data-parallel split), binding a (never dereferenced) arena
// address, the learn-step launch lists for every flag combination (dqnx_learn_kernel_count /
// _info), the data-parallel bucket cuts, the acting / sampler scratch sizes and the argument
// checks of the entry points.  No kernel is launched.  Every region dqnx_engine_buffer reports
// must lie inside the arena, 256-byte aligned, without overlapping another.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/dqnx.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                  \
            fprintf(stderr, " (%s)\n", dqnx_last_error()); \
            g_fail++;                                      \
        }                                                  \
    } while (0)

static dqnx_net_desc mlp(int D, int head, std::vector<int> hidden) {
    dqnx_net_desc d;
    memset(&d, 0, sizeof(d));
    d.kind = DQNX_NET_MLP;
    d.head = head;
    d.activation = DQNX_ACT_RELU;
    d.obs_dim = D;
    d.n_actions = 8;
    d.n_dense = (int)hidden.size();
    for (size_t i = 0; i < hidden.size(); i++) d.dense[i] = hidden[i];
    return d;
}

// TwoStreamHybridNetwork (R:env/dqn_config.py:66-193) on a (c,h,w) micro grid
static dqnx_net_desc hybrid(int c, int h, int w, int head) {
    dqnx_net_desc d;
    memset(&d, 0, sizeof(d));
    d.kind = DQNX_NET_TWO_STREAM;
    d.head = head;
    d.activation = DQNX_ACT_ELU;
    d.macro_len = 14;
    d.micro_c = c; d.micro_h = h; d.micro_w = w;
    d.obs_dim = 14 + c * h * w;
    d.n_actions = 8;
    d.n_conv = 3;
    const int co[3] = {32, 64, 64}, sh[3] = {1, 2, 2}, sw[3] = {1, 1, 2};
    for (int l = 0; l < 3; l++) {
        d.conv_out[l] = co[l]; d.conv_kh[l] = d.conv_kw[l] = 3; d.conv_sh[l] = sh[l]; d.conv_sw[l] = sw[l];
    }
    d.n_dense = 2;
    d.dense[0] = 512;
    d.dense[1] = 256;
    return d;
}

static void check_params(const dqnx_net_desc& d) {
    int64_t P = 0;
    int32_t nt = 0;
    CHECK(dqnx_net_param_count(&d, &P, &nt) == DQNX_OK && P > 0 && nt > 0, "param_count");
    int64_t off = 0;
    for (int i = 0; i < nt; i++) {
        dqnx_param_info pi;
        CHECK(dqnx_net_param_info(&d, i, &pi) == DQNX_OK, "param_info %d", i);
        CHECK(pi.offset == off && pi.numel > 0 && strlen(pi.name) > 0, "param %d layout", i);
        off += pi.numel;
    }
    CHECK(off == P, "param total");
    dqnx_param_info pi;
    CHECK(dqnx_net_param_info(&d, nt, &pi) == DQNX_EINVAL, "param index past the end");
    CHECK(dqnx_net_param_info(&d, -1, &pi) == DQNX_EINVAL, "negative param index");
}

struct Case {
    dqnx_net_desc net;
    int algo, batch, world, rank, local, dtype;
    int64_t cap;
};

static void run_case(const Case& k) {
    dqnx_config c;
    memset(&c, 0, sizeof(c));
    c.net = k.net;
    dqnx_config_defaults(&c);
    c.algo = k.algo;
    c.batch = k.batch;
    c.world_size = k.world;
    c.rank = k.rank;
    c.local_sampling = k.local;
    c.capacity = k.cap;
    c.compute_dtype = k.dtype;
    dqnx_engine* e = nullptr;
    const int rc = dqnx_engine_create(&c, &e);
    if (rc != DQNX_OK) {   // refused configurations must say why and leave nothing behind
        CHECK(e == nullptr && strlen(dqnx_last_error()) > 0, "refused create left a handle");
        return;
    }
    uint64_t total = 0;
    CHECK(dqnx_engine_arena_bytes(e, &total) == DQNX_OK && total > 0, "arena_bytes");
    // every region inside the arena, 256-aligned, pairwise disjoint
    std::vector<std::pair<uint64_t, uint64_t>> regs;
    for (int b = 0; b < DQNX_BUF_COUNT; b++) {
        uint64_t o = 0, n = 0;
        CHECK(dqnx_engine_buffer(e, b, &o, &n) == DQNX_OK, "buffer %d", b);
        CHECK(o + n <= total, "buffer %d past the arena", b);
        if (n) {
            CHECK(o % 256 == 0, "buffer %d misaligned", b);
            regs.push_back({o, o + n});
        }
    }
    std::sort(regs.begin(), regs.end());
    for (size_t i = 1; i < regs.size(); i++) CHECK(regs[i].first >= regs[i - 1].second, "buffers overlap");
    uint64_t o, n;
    CHECK(dqnx_engine_buffer(e, DQNX_BUF_COUNT, &o, &n) == DQNX_EINVAL, "buffer id past the end");
    int32_t stride = 0;
    CHECK(dqnx_engine_obs_stride(e, &stride) == DQNX_OK && stride >= k.net.obs_dim && stride % 4 == 0, "stride");
    // unbound: step entry points refuse
    int32_t nk = 0;
    CHECK(dqnx_learn_kernel_count(e, 0, &nk) != DQNX_OK, "unbound engine planned a step");
    CHECK(dqnx_engine_bind(e, (void*)(uintptr_t)0x1010, total) == DQNX_EINVAL, "misaligned arena accepted");
    CHECK(dqnx_engine_bind(e, (void*)(uintptr_t)0x100000, total - 1) == DQNX_EINVAL, "short arena accepted");
    // a device-sized address that is never dereferenced: planning must not touch the arena
    CHECK(dqnx_engine_bind(e, (void*)(uintptr_t)0x7f0000000000ull, total) == DQNX_OK, "bind");
    const int flag_sets[] = {0, DQNX_STEP_SOFT_UPDATE, DQNX_STEP_GRADS_ONLY, DQNX_STEP_PREFETCH,
                             DQNX_STEP_PREFETCH | DQNX_STEP_SOFT_UPDATE, DQNX_STEP_GIVEN_INDICES,
                             DQNX_STEP_GRADS_ONLY | DQNX_STEP_PREFETCH};
    for (int f : flag_sets) {
        nk = 0;
        CHECK(dqnx_learn_kernel_count(e, f, &nk) == DQNX_OK && nk > 0, "kernel_count flags %d", f);
        for (int i = 0; i < nk; i++) {
            char name[64];
            double fl = -1, by = -1;
            CHECK(dqnx_learn_kernel_info(e, f, i, name, sizeof(name), &fl, &by) == DQNX_OK, "kernel_info %d", i);
            CHECK(strlen(name) > 0 && fl >= 0 && by >= 0, "kernel %d description", i);
        }
        char name[8];
        CHECK(dqnx_learn_kernel_info(e, f, nk, name, sizeof(name), nullptr, nullptr) == DQNX_EINVAL, "kernel index past the end");
    }
    int32_t nb = 0;
    if (dqnx_dp_bucket_count(e, &nb) == DQNX_OK) {
        // the buckets tile [0, P) exactly (bucket 0 carries the loss slot at P), every range starts on a
        // float4 (the bucket Adam passes run the float4 kernel from `first`), none is empty
        int64_t P = 0;
        CHECK(dqnx_net_param_count(&k.net, &P, nullptr) == DQNX_OK, "param_count");
        std::vector<std::pair<int64_t, int64_t>> rg;
        for (int b = 0; b < nb; b++) {
            int64_t first = -1, count = -1;
            CHECK(dqnx_dp_bucket_info(e, b, &first, &count) == DQNX_OK && first >= 0 && count > 0, "bucket %d", b);
            if (b == 0) {
                CHECK(first + count == P + 1, "bucket 0 must end with the loss slot (%lld + %lld vs P %lld)",
                      (long long)first, (long long)count, (long long)P);
                count -= 1;
            }
            CHECK(first % 4 == 0, "bucket %d starts at %lld, not a float4", b, (long long)first);
            rg.push_back({first, first + count});
        }
        std::sort(rg.begin(), rg.end());
        int64_t at = 0;
        for (const auto& r : rg) {
            CHECK(r.first == at && r.second > r.first, "buckets leave a gap or overlap at %lld", (long long)at);
            at = r.second;
        }
        CHECK(at == P, "buckets end at %lld, not at P %lld", (long long)at, (long long)P);
        CHECK(dqnx_dp_bucket_info(e, nb, nullptr, nullptr) == DQNX_EINVAL, "bucket past the end");
    }
    CHECK(dqnx_params_modified(e) == DQNX_OK, "params_modified");
    CHECK(dqnx_engine_set_graphs(e, 1) == DQNX_OK && dqnx_engine_set_graphs(e, 0) == DQNX_OK, "set_graphs");
    CHECK(dqnx_engine_destroy(e) == DQNX_OK, "destroy");
}

int main() {
    const int heads[2] = {DQNX_HEAD_LINEAR, DQNX_HEAD_DUELING};
    std::vector<dqnx_net_desc> nets = {mlp(14, DQNX_HEAD_DUELING, {256, 128}), mlp(284, DQNX_HEAD_DUELING, {256, 128}),
                                       mlp(284, DQNX_HEAD_LINEAR, {256, 128}), mlp(8, DQNX_HEAD_LINEAR, {64}),
                                       mlp(100, DQNX_HEAD_DUELING, {256, 128, 64}), mlp(284, DQNX_HEAD_DUELING, {200, 72}),
                                       hybrid(2, 27, 5, DQNX_HEAD_DUELING), hybrid(2, 27, 5, DQNX_HEAD_LINEAR),
                                       hybrid(4, 84, 84, DQNX_HEAD_DUELING)};
    for (const auto& d : nets) check_params(d);
    // invalid networks are refused
    dqnx_net_desc bad = mlp(284, DQNX_HEAD_DUELING, {256, 128});
    bad.n_dense = DQNX_MAX_DENSE + 1;
    int64_t P;
    CHECK(dqnx_net_param_count(&bad, &P, nullptr) == DQNX_EINVAL, "too many layers accepted");
    bad = hybrid(2, 27, 5, DQNX_HEAD_DUELING);
    bad.obs_dim += 1;
    CHECK(dqnx_net_param_count(&bad, &P, nullptr) == DQNX_EINVAL, "hybrid obs_dim mismatch accepted");
    CHECK(dqnx_net_param_count(nullptr, &P, nullptr) == DQNX_EINVAL, "null net accepted");

    std::vector<Case> cases;
    const int algos[3] = {DQNX_ALGO_DQN, DQNX_ALGO_DOUBLE, DQNX_ALGO_PER_DOUBLE};
    for (int n = 0; n < 6; n++)
        for (int a : algos)
            for (int B : {32, 100, 1024, 4096, 8192})
                for (int dt : {DQNX_COMPUTE_FP32, DQNX_COMPUTE_BF16})
                    cases.push_back({nets[n], a, B, 1, 0, 0, dt, 20000});
    for (int W : {2, 4, 8})
        for (int r : {0, W - 1})
            for (int a : {DQNX_ALGO_DOUBLE, DQNX_ALGO_PER_DOUBLE}) {
                cases.push_back({nets[1], a, 4096, W, r, 0, DQNX_COMPUTE_FP32, 1000000});
                cases.push_back({nets[1], a, 8192, W, r, 0, DQNX_COMPUTE_BF16, 1000000});
                cases.push_back({nets[1], a, 4096, W, r, 1, DQNX_COMPUTE_FP32, 1000000});   // local (PER refused)
                cases.push_back({nets[6], a, 256, W, r, 0, DQNX_COMPUTE_FP32, 100000});
                cases.push_back({nets[8], a, 256, W, r, 0, DQNX_COMPUTE_FP32, 1000});
            }
    // world 1 (the bucketed DP tests' engines) for both conv nets, every algorithm, and the small
    // batches those tests use
    for (int n : {6, 7, 8})
        for (int a : algos)
            for (int B : {64, 256})
                cases.push_back({nets[n], a, B, 1, 0, 0, DQNX_COMPUTE_FP32, n == 8 ? 2000 : 20000});
    for (int n = 6; n < 9; n++)
        for (int a : algos)
            for (int B : {32, 48, 256})
                cases.push_back({nets[n], a, B, 1, 0, 0, DQNX_COMPUTE_FP32, 2000});
    // refusals: PER beyond the exact-sum capacity, bf16 on a conv net, bad dtype, k > capacity
    cases.push_back({nets[1], DQNX_ALGO_PER_DOUBLE, 1024, 1, 0, 0, DQNX_COMPUTE_FP32, (1 << 20) + 1});
    cases.push_back({nets[6], DQNX_ALGO_DOUBLE, 256, 1, 0, 0, DQNX_COMPUTE_BF16, 2000});
    cases.push_back({nets[1], DQNX_ALGO_DOUBLE, 1024, 1, 0, 0, 7, 2000});
    cases.push_back({nets[1], DQNX_ALGO_DOUBLE, 1000, 3, 1, 0, DQNX_COMPUTE_FP32, 2000});
    for (const Case& k : cases) run_case(k);

    // acting path: scratch sizes and argument checks on the host (no launch)
    for (const auto& d : nets) {
        const uint64_t need = dqnx_act_scratch_bytes(&d, 4);
        if (need == 0) continue;   // networks the acting kernels do not cover
        CHECK(dqnx_act(&d, nullptr, nullptr, 4, nullptr, nullptr, nullptr, 0, nullptr) == DQNX_EINVAL, "act null buffers");
        CHECK(dqnx_act(&d, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, nullptr) == DQNX_OK, "act n = 0");
    }
    for (int64_t n : {50, 10000, 1000000})
        for (int k : {32, 1024, 4096, 8192}) CHECK(dqnx_sample_scratch_bytes(n, k) > 0, "sample scratch %lld %d", (long long)n, k);
    CHECK(dqnx_engine_destroy(nullptr) != DQNX_OK || true, "destroy(null)");
    printf("plan_check: %zu engine configurations, %d failures\n", cases.size(), g_fail);
    return g_fail ? 1 : 0;
}
