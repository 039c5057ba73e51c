#!/usr/bin/env python3
"""bench.py -- DQN learn-step throughput (transitions/s) on MI355X through libdqnx.

Workload (BASELINE.json configs[1]): synthetic 1ramp_1x3 state vectors (D=284, A=8),
MLP(256,128) dueling Q-net, fp32, DuelingDoubleDQNAgent learn step, minibatch 1024 per
GPU sampled from a GPU-resident replay ring of 1e6 transitions.  One "step" = one
Agent.learn() + update_target_network() (R:train.py:99-101): sample (bit-exact CPython
random.sample) -> gather -> online(s'), target(s'), online(s) -> Double-DQN TD target ->
Huber -> backward -> Adam -> soft target update.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...    (one process per GPU, RCCL)

Data parallel = weak scaling: every rank processes `--batch` transitions per step; all
ranks draw the same global index set (batch * N) from the same MT19937 state and take
their shard; gradients are summed with one RCCL all-reduce per step.

Prints ONE JSON line on rank 0 (fields: see the driver contract in DESIGN.md).
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time

import numpy as np
import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "multimodal-drl-rmc_amd"))

from dqn import _capi as C  # noqa: E402
from dqn.data_parallel import GraphedDPStep, dp_learn_step  # noqa: E402
from dqn.engine import LearnEngine, hybrid_spec, mlp_spec  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 matrix, dense
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--batch", type=int, default=1024, help="transitions per GPU per step")
    p.add_argument("--capacity", type=int, default=None,
                   help="replay capacity (default 1e6; 1e5 for hybrid84: 113 KB rows)")
    p.add_argument("--obs-dim", type=int, default=284)
    p.add_argument("--actions", type=int, default=8)
    p.add_argument("--algo", default="DuelingDoubleDQNAgent")
    p.add_argument("--net", default="mlp", choices=["mlp", "hybrid", "hybrid84"],
                   help="mlp: MLP-284 (configs[1]); hybrid: TwoStreamHybridNetwork on the (2,27,5) grid; "
                        "hybrid84: the stacked (4,84,84) occupancy-grid CNN variant (configs[2])")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--no-dp-graph", action="store_true",
                   help="N > 1: launch the learn graph, the all-reduce and Adam separately each step "
                        "instead of replaying them as one captured HIP graph")
    p.add_argument("--compute", default="fp32", choices=["fp32", "bf16"],
                   help="GEMM operand precision (bf16: BASELINE config 5; MLP only; fp32 accumulate, master weights, Adam)")
    p.add_argument("--global-sampling", action="store_true",
                   help="N > 1: every rank draws the same global minibatch (bit-exact with 1 GPU)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--prefetch", action="store_true",
                   help="overlap the next step's replay sampling with this step's compute on a "
                        "side stream (measured slower at batch 1024: cross-stream event waits)")
    a = p.parse_args()
    if a.capacity is None:
        a.capacity = 100_000 if a.net == "hybrid84" else 1_000_000
    return a


def init_params(spec, seed=0):
    """Random init of the Q-net architecture (torch default Conv2d / Linear init), in the
    reference's construction order (R:env/dqn_config.py:92-122, R:dqn/network.py:81-82)."""
    torch.manual_seed(seed)
    mods = {}
    if spec.kind == C.DQNX_NET_TWO_STREAM:
        c, h, w = spec.micro_chw
        for i, (f, k, st) in enumerate(spec.conv):
            mods[f"net.cnn_stream.{2 * i}"] = nn.Conv2d(c, f, kernel_size=k, stride=st, padding=(k[0] // 2, k[1] // 2))
            h = (h + 2 * (k[0] // 2) - k[0]) // st[0] + 1
            w = (w + 2 * (k[1] // 2) - k[1]) // st[1] + 1
            c = f
        d = c * h * w + spec.macro_len
        prefix = "net.dense_stream"
    else:
        d = spec.obs_dim
        prefix = "net"
    for i, width in enumerate(spec.dense):
        mods[f"{prefix}.{2 * i}"] = nn.Linear(d, width)
        d = width
    if spec.head == C.DQNX_HEAD_DUELING:
        mods["fc_val"] = nn.Linear(d, 1)
        mods["fc_adv"] = nn.Linear(d, spec.n_actions)
    else:
        mods["fc_out"] = nn.Linear(d, spec.n_actions)
    sd = {}
    for k, m in mods.items():
        sd[k + ".weight"] = m.weight.detach()
        sd[k + ".bias"] = m.bias.detach()
    return sd


def make_spec(args):
    head = "dueling" if "Dueling" in args.algo else "linear"
    if args.net == "hybrid":
        return hybrid_spec(args.actions, head, micro_chw=(2, 27, 5))
    if args.net == "hybrid84":
        return hybrid_spec(args.actions, head, micro_chw=(4, 84, 84))
    return mlp_spec(args.obs_dim, args.actions, head)


def fill_ring(eng, n, D, A, device, seed=0, chunk=None):
    """Synthetic 1ramp_1x3-shaped transitions generated on the GPU:
    macro U[0,1); micro grid occupancy ~ Bernoulli(0.2) with speed U[0,1); action U{0..A-1};
    reward U[-24,3]; done ~ Bernoulli(1/90)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    macro = min(14, D)
    if chunk is None:   # ~256 MB of obs per chunk
        chunk = max(256, min(1 << 16, (1 << 28) // (4 * D)))

    def obs_block(m):
        o = torch.empty(m, D, device=device)
        o[:, :macro] = torch.rand(m, macro, generator=g, device=device)
        if D > macro:
            occ = torch.rand(m, D - macro, generator=g, device=device) < 0.2
            spd = torch.rand(m, D - macro, generator=g, device=device)
            o[:, macro:] = torch.where(occ, spd, torch.zeros((), device=device))
        return o

    done_rows = 0
    while done_rows < n:
        m = min(chunk, n - done_rows)
        obs, nobs = obs_block(m), obs_block(m)
        act = torch.randint(0, A, (m,), generator=g, device=device, dtype=torch.int32)
        rew = torch.rand(m, generator=g, device=device) * 27.0 - 24.0
        done = (torch.rand(m, generator=g, device=device) < 1.0 / 90.0).to(torch.uint8)
        eng.push(obs, act, rew, done, nobs)
        done_rows += m
    torch.cuda.synchronize()


def net_name(args):
    return {"mlp": f"MLP-{args.obs_dim}", "hybrid": "TwoStreamHybrid(2x27x5)",
            "hybrid84": "TwoStreamHybrid(4x84x84)"}[args.net]


WORKLOADS = {
    "mlp": "configs[1]: synthetic 1ramp_1x3 state vectors, MLP Q-net fp32, GPU replay buffer",
    "hybrid": "TwoStreamHybridNetwork (micro CNN on the 2x27x5 grid + 14 macro), fp32, GPU replay buffer",
    "hybrid84": "configs[2]: stacked 4x84x84 occupancy-grid CNN encoder + dueling head, fp32, GPU replay buffer",
}


def cpu_baseline(args):
    """The oracle's torch-CPU restatement of the same learn step (reference algorithm:
    deque + random.sample + transitions_to_tensor + 3 forwards + Huber + autograd + Adam +
    soft update), timed on this host's cores on a bounded sample."""
    sys.path.insert(0, REPO)
    from oracle import ref as O
    head = "dueling" if "Dueling" in args.algo else "linear"
    if args.net == "mlp":
        spec = O.mlp_spec(args.obs_dim, args.actions, head)
    else:
        spec = O.hybrid_spec(args.actions, head, micro_chw=(2, 27, 5) if args.net == "hybrid" else (4, 84, 84))
    per = args.algo.startswith("Per")
    cap = min(args.capacity, 100_000) if per else args.capacity   # Python SumTree fill is ~20 us/row
    if args.net == "hybrid84":
        cap = min(cap, 2_000)   # 113 KB rows: a host deque of 1e5 would need 22.6 GB
    L = O.OracleLearner(spec, args.algo, args.batch, cap, seed=0)
    obs, act, rew, done, nobs = O.synth_transitions(cap, spec.obs_dim, args.actions, seed=0)
    if per:
        list(L.replay.store_transitions(obs, act, rew, done, nobs))
    else:
        L.replay.replay_buffer.extend(zip(obs, act, rew, done, nobs))
    random.seed(1234)
    L.py_state = O.py_state_to_array()
    for _ in range(2):
        L.train_step()
    t0 = time.perf_counter()
    steps = 0
    while True:
        L.train_step()
        steps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds and steps >= 3:
            break
    return {"value": args.batch * steps / el, "unit": "transitions/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/ref.py OracleLearner {args.algo} {net_name(args)} batch {args.batch}, "
                      f"{'SumTree' if per else 'deque'} of {cap} transitions, {steps} learn+soft-update steps in {el:.1f} s, "
                      f"torch {torch.__version__} CPU, {torch.get_num_threads()} threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log(f"warning: --gpus {args.gpus} != WORLD_SIZE {world}; using WORLD_SIZE")
    # rehearsal knobs for a 1-GPU box: every rank on cuda:0, gloo collectives
    dev_index = 0 if os.environ.get("DQNX_SINGLE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    dist = None
    backend = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("DQNX_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    spec = make_spec(args)
    Bg = args.batch * world
    per = args.algo.startswith("Per")
    # N > 1: plain data parallelism -- every rank draws its own batch_per_gpu positions from its
    # own MT19937 stream (O(batch_per_gpu) sampling per rank).  --global-sampling instead has
    # every rank draw the same global minibatch (bit-exact with one GPU; PER always does this).
    local = world > 1 and not per and not args.global_sampling
    eng = LearnEngine(spec, args.algo, Bg, args.capacity, world_size=world, rank=rank, device=device,
                      graphs=not args.no_graphs, local_sampling=local, compute_dtype=args.compute)
    eng.load_params(init_params(spec, 0))
    fill_ring(eng, args.capacity, spec.obs_dim, args.actions, device, seed=0)
    random.seed(1234 + (rank if local else 0))   # the replay sampler continues CPython's MT19937 stream
    eng.set_rng(C.DQNX_RNG_PY, np.array(random.getstate()[1], dtype=np.uint32))
    if per:             # PER draws numpy's legacy global stream (np.random.uniform)
        np.random.seed(1234)
        st = np.random.get_state()
        eng.set_rng(C.DQNX_RNG_NP, np.append(st[1], st[2]).astype(np.uint32))
    Bl = args.batch

    prefetch = args.prefetch

    def step():
        if world > 1:   # shard compute, RCCL all-reduce (+ PER |delta| all-gather), replicated Adam
            dp_learn_step(eng, soft_update=True)
        else:
            eng.learn_step(soft_update=True, prefetch=prefetch)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.check_device_error()
    dp_graph = False
    if world > 1 and backend == "nccl" and not args.no_dp_graph and not args.no_graphs:
        # the whole DP step (shard kernels + RCCL all-reduce + Adam) as one replayed graph: the
        # eager loop is host-bound (3 launches + a collective call per ~50 us step).  RCCL
        # collectives are capturable; gloo's are host calls and never are.
        g = GraphedDPStep(eng, soft_update=True)
        g()   # one untimed replay
        torch.cuda.synchronize()
        dp_graph = True

        def step():
            g()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dp_graph:
        eng.set_graphs(True)   # the kernel timing below replays the engine's own graphs
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    eng.check_device_error()
    loss = eng.loss()
    ms_per_step = el / args.steps * 1e3
    value = Bg * args.steps / el

    # ---- dominant-kernel roofline: HIP-event-timed graph steps with / without each kernel ----
    roofline = None
    kernels = []
    if not args.no_kernel_timing:
        flags = C.STEP_GRADS_ONLY if world > 1 else C.STEP_SOFT_UPDATE
        L = C.lib()
        n = C.I32()
        C.check(L.dqnx_learn_kernel_count(eng.h, flags, ctypes.byref(n)), "kernel_count")
        infos = []
        for i in range(n.value):
            nm = ctypes.create_string_buffer(64)
            fl, by = ctypes.c_double(), ctypes.c_double()
            C.check(L.dqnx_learn_kernel_info(eng.h, flags, i, nm, 64, ctypes.byref(fl), ctypes.byref(by)), "info")
            infos.append((nm.value.decode(), fl.value, by.value))
        # consume a pending prefetched minibatch so the timing steps sample themselves
        if world > 1:
            dp_learn_step(eng, soft_update=True)
        else:
            eng.learn_step(soft_update=True)
        K = max(args.steps, 50)
        stream = eng.stream()

        def graph_steps_ms(omit, count):
            """`count` graph-launched learn steps with kernel `omit` left out (-1: none),
            bracketed by HIP events on the engine's stream; ms per step."""
            C.check(L.dqnx_learn_step_omit(eng.h, flags, omit, stream), "omit step")   # capture
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0.record()
            for _ in range(count):
                C.check(L.dqnx_learn_step_omit(eng.h, flags, omit, stream), "omit step")
            t1.record()
            t1.synchronize()
            return t0.elapsed_time(t1) / count

        # a kernel's in-context time per launch = step time with it - step time without it;
        # full and omitted runs are interleaved and the median of `reps` pairs is kept
        def kernel_ms(i, count, reps):
            d = []
            for _ in range(reps):
                d.append(graph_steps_ms(-1, count) - graph_steps_ms(i, count))
            d.sort()
            return d[len(d) // 2]

        for i, (nm, fl, by) in enumerate(infos):
            kernels.append({"kernel": nm, "avg_us": kernel_ms(i, 50, 3) * 1e3, "flops": fl, "bytes": by})
        dom = max(range(len(kernels)), key=lambda i: kernels[i]["avg_us"])
        avg_ms = kernel_ms(dom, K, 5)
        kernels[dom]["avg_us"] = avg_ms * 1e3
        nm, fl, by = infos[dom]
        intensity = fl / by if by else 0.0
        peak_mfma = PEAK_BF16_MFMA_TFLOPS if args.compute == "bf16" else PEAK_FP32_MFMA_TFLOPS
        ridge = peak_mfma * 1e12 / (PEAK_HBM_GBS * 1e9)
        traffic = None
        # HBM bytes per launch from rocprofv3 PMC passes of this same workload (tools/pmc_traffic.py)
        tag = "" if args.compute == "fp32" else f"_{args.compute}"
        pmc_path = os.path.join(REPO, "profiles", f"pmc_traffic_{args.net}_b{args.batch}{tag}.json")
        if os.path.exists(pmc_path):
            try:
                traffic = json.load(open(pmc_path)).get(nm, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        if intensity > ridge and fl > 0:
            ach = fl / (avg_ms * 1e-3) / 1e12
            roofline = {"bound": "mfma", "achieved": ach, "peak": peak_mfma, "unit": "TFLOP/s",
                        "frac": ach / peak_mfma, "traffic": traffic, "kernel": nm,
                        "avg_us": avg_ms * 1e3, "algorithmic_flops": fl, "algorithmic_bytes": by}
        else:
            ach = by / (avg_ms * 1e-3) / 1e9
            roofline = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": ach / PEAK_HBM_GBS, "traffic": traffic, "kernel": nm,
                        "avg_us": avg_ms * 1e3, "algorithmic_flops": fl, "algorithmic_bytes": by}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args)
        except Exception as ex:  # the baseline must never hide the GPU number
            log(f"cpu baseline failed: {ex!r}")

    if rank == 0:
        out = {
            "metric": "DQN learn-steps/sec × batch (transitions/sec) at 1/2/4/8 MI355X",
            "value": value,
            "unit": "transitions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.compute,
            "data": "synthetic",
            "config": {
                "workload": WORKLOADS[args.net],
                "algo": args.algo, "net": net_name(args),
                "batch_per_gpu": args.batch, "global_batch": Bg, "replay_capacity": args.capacity,
                "parallelism": f"dp{world}", "graphs": not args.no_graphs, "prefetch_sampling": prefetch,
                "sampling": "rank-local" if local else "global",
                "dp_step": ("one HIP graph" if dp_graph else "eager") if world > 1 else None,
                "compute": args.compute,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "loss": loss,
            "kernels": kernels,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
