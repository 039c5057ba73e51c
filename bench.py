#!/usr/bin/env python3
"""bench.py -- DQN learn-step throughput (transitions/s) on MI355X through libdqnx.

One "step" = one Agent.learn() + update_target_network() (R:train.py:99-101): sample
(bit-exact CPython random.sample) -> gather -> online(s'), target(s'), online(s) ->
Double-DQN TD target -> Huber -> backward -> Adam -> soft target update, on synthetic
1ramp_1x3-shaped transitions (D=284, A=8) in a GPU-resident replay ring of 1e6.

Workloads (BASELINE.json configs):
  * N = 1 (default): configs[1] -- MLP(256,128) dueling Q-net fp32, DuelingDoubleDQNAgent,
    minibatch 1024.  The line also carries `configs3_n1` (the same learn step at configs[3]'s
    global minibatch 4096 on this one GPU: the N = 1 point of the strong-scaling series) and
    `projection_w8` (the rank-0 shard step of a world_size = 8 engine -- 512 rows + the global
    4096-draw sampling + Adam -- timed here; the all-reduce is the only missing term).
  * N > 1 (torchrun, one process per GPU, RCCL over xGMI): configs[3] strong scaling --
    global minibatch 4096 (--global-batch), 4096/N rows per rank, every rank drawing the SAME
    global index set from the same MT19937 state (reference-exact random.sample semantics),
    one gradient all-reduce per step, the whole DP step replayed as one HIP graph.  The line
    also carries `weak` (4096 rows per rank, same semantics).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0 (fields: see the driver contract in DESIGN.md section 5).
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
from dqn.data_parallel import GraphedDPStep, dp_learn_step, dp_learn_step_bucketed  # noqa: E402
from dqn.data_parallel import capture as dp_capture  # noqa: E402
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
    p.add_argument("--batch", type=int, default=None,
                   help="minibatch of a one-GPU run (default 1024, configs[1]); rows per rank with --scaling weak "
                        "(default 4096)")
    p.add_argument("--global-batch", type=int, default=4096,
                   help="N > 1, --scaling strong: global minibatch sharded over the ranks (configs[3]: 4096)")
    p.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                   help="N > 1: strong = fixed global minibatch (configs[3]); weak = --batch rows per rank")
    p.add_argument("--capacity", type=int, default=None,
                   help="replay capacity (default 1e6; 1e5 for hybrid84: 113 KB rows)")
    p.add_argument("--obs-dim", type=int, default=284)
    p.add_argument("--actions", type=int, default=8)
    p.add_argument("--algo", default="DuelingDoubleDQNAgent")
    p.add_argument("--net", default="mlp", choices=["mlp", "hybrid", "hybrid84"],
                   help="mlp: MLP-284 (configs[1]/[3]/[4]); hybrid: TwoStreamHybridNetwork on the (2,27,5) grid; "
                        "hybrid84: the stacked (4,84,84) occupancy-grid CNN variant (configs[2])")
    p.add_argument("--graphs", action="store_true",
                   help="replay every learn step as a captured HIP graph (default: eager launches, 3-4 us per "
                        "step faster on MI355X / ROCm 7.2: each hipGraphLaunch adds ~8.5 us between graphs)")
    p.add_argument("--no-graphs", action="store_true", help="(the default; kept for old command lines)")
    p.add_argument("--dp-graph-steps", type=int, default=4,
                   help="N > 1: DP steps captured back to back into the one replayed graph (every hipGraphLaunch "
                        "leaves ~8.5 us before its first kernel); the timed K steps are K // this replays plus "
                        "the remainder as eager steps")
    p.add_argument("--no-dp-graph", action="store_true",
                   help="N > 1: launch the learn graph, the all-reduce and Adam separately each step "
                        "instead of replaying them as one captured HIP graph")
    p.add_argument("--compute", default="fp32", choices=["fp32", "bf16"],
                   help="GEMM operand precision (bf16: BASELINE config 5; MLP only; fp32 accumulate, master weights, Adam)")
    p.add_argument("--local-sampling", action="store_true",
                   help="N > 1, uniform replay: each rank draws its own rows from its own MT stream (plain data "
                        "parallelism; NOT the reference's random.sample semantics)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-buckets", action="store_true",
                   help="conv nets under DP: one gradient all-reduce instead of per-layer buckets")
    p.add_argument("--mlp-buckets", action="store_true",
                   help="MLP under DP: two gradient buckets (every layer but layer 1, then layer 1), bucket 0's "
                        "all-reduce and Adam on a side stream under layer 1's dW tiles (default: one all-reduce; "
                        "DESIGN.md section 6 has the latency model)")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="seconds per CPU-baseline leg")
    p.add_argument("--no-kernel-timing", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the secondary measurements (configs3_n1 / projection_w8 / weak)")
    p.add_argument("--chain", type=int, default=1,
                   help="N = 1: learn steps per engine call (dqnx_learn_steps: one graph, each step's "
                        "minibatch drawn inside the previous step's last launch); 1 = one Agent.learn() per call")
    p.add_argument("--no-prefetch", action="store_true",
                   help="N = 1, uniform replay: do not draw step t+1's minibatch inside step t's last launch "
                        "(DQNX_STEP_PREFETCH; on by default for this pure learning loop)")
    p.add_argument("--prefetch", action="store_true", help="(the default; kept for old command lines)")
    p.add_argument("--per-numpy121", action="store_true",
                   help="PER: the SumTree arithmetic of the reference's pinned numpy 1.21 (float32 change and "
                        "ancestor sums in update order, k_per_chain) instead of numpy >= 2's float64")
    a = p.parse_args()
    if a.capacity is None:
        a.capacity = 100_000 if a.net == "hybrid84" else 1_000_000
    a.prefetch = not a.no_prefetch
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


def workload_name(args, world):
    """Which BASELINE.json config a line measures."""
    per = args.algo.startswith("Per")
    if args.net == "hybrid84":
        return "configs[2]: stacked 4x84x84 occupancy-grid CNN encoder + dueling head, fp32, GPU replay buffer"
    if args.net == "hybrid":
        return ("TwoStreamHybridNetwork (micro CNN on the 2x27x5 grid + 14 macro; the reference HEAD net), "
                "fp32, GPU replay buffer")
    if per or args.compute == "bf16":
        return (f"configs[4]: prioritised replay (GPU sum-tree) + double/dueling DQN, {args.compute} compute, "
                f"MLP Q-net, synthetic 1ramp_1x3 state vectors")
    if world > 1 and args.scaling == "strong":
        return "configs[3]: MLP Q-net fp32, global minibatch sharded DP over the GPUs, RCCL grad all-reduce over xGMI"
    if world > 1:
        return "configs[3] weak-scaling variant: MLP Q-net fp32, fixed minibatch per GPU, RCCL grad all-reduce"
    return "configs[1]: synthetic 1ramp_1x3 state vectors, MLP Q-net fp32, GPU replay buffer, 1 GPU"


# ----------------------------------------------------------------------------------------
# CPU baseline: the oracle (torch-CPU restatement of the reference learn step)
# ----------------------------------------------------------------------------------------
def cpu_info():
    """CPU model and core counts of this host (lscpu), and the CPUs this process may use."""
    model, phys = None, None
    try:
        import subprocess
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        cores = {tuple(l.split(",")) for l in out.splitlines() if l and not l.startswith("#")}
        phys = len(cores) or None
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except Exception:
        usable = os.cpu_count()
    # the CPU share: the cgroup v2 quota (cpu.max "quota period"), else OMP_NUM_THREADS
    share, source = None, None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            share, source = max(1, int(int(q) // int(per))), f"/sys/fs/cgroup/cpu.max {q} {per}"
    except Exception:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if share is None and (omp or "").isdigit():
        share, source = int(omp), f"OMP_NUM_THREADS={omp}"
    return {"model": model, "physical_cores": phys, "usable_cpus": usable, "omp_num_threads": omp,
            "cpu_share": share, "cpu_share_source": source}


def cpu_baseline(args, batch):
    """The oracle learner (deque + random.sample + transitions_to_tensor + 3 forwards + Huber +
    autograd + Adam + soft update) timed on this host's cores on bounded samples: every
    combination of {all usable physical cores, 8 threads} x {capacity 1e5, 1e6} (BASELINE.md
    section 3; deque sampling is O(n)).  `value` is the all-cores run at the GPU run's capacity."""
    sys.path.insert(0, REPO)
    from oracle import ref as O
    info = cpu_info()
    head = "dueling" if "Dueling" in args.algo else "linear"
    if args.net == "mlp":
        spec = O.mlp_spec(args.obs_dim, args.actions, head)
    else:
        spec = O.hybrid_spec(args.actions, head, micro_chw=(2, 27, 5) if args.net == "hybrid" else (4, 84, 84))
    per = args.algo.startswith("Per")
    caps = sorted({min(args.capacity, 100_000), args.capacity})
    if per:
        caps = [min(args.capacity, 100_000)]   # the Python SumTree fill is ~20 us per row
    if args.net == "hybrid84":
        caps = [2_000]                          # 113 KB rows: a host deque of 1e5 would need 22.6 GB
    ncap = max(caps)
    obs, act, rew, done, nobs = O.synth_transitions(ncap, spec.obs_dim, args.actions, seed=0)
    # thread counts: all physical cores the affinity mask allows, the
    # process's CPU share (the cgroup quota / OMP_NUM_THREADS the box sets), and 8; the headline is the
    # fastest run at the bench capacity (threads beyond the share only get throttled by the quota)
    phys = min(x for x in (info["physical_cores"], info["usable_cpus"]) if x) if any(
        (info["physical_cores"], info["usable_cpus"])) else torch.get_num_threads()
    share = info["cpu_share"] or phys
    threads = sorted({phys, share, 8}, reverse=True)
    runs = []
    saved = torch.get_num_threads()
    for cap in caps:
        L = O.OracleLearner(spec, args.algo, batch, cap, seed=0)
        if per:
            list(L.replay.store_transitions(obs[:cap], act[:cap], rew[:cap], done[:cap], nobs[:cap]))
        else:
            L.replay.replay_buffer.extend(zip(obs[:cap], act[:cap], rew[:cap], done[:cap], nobs[:cap]))
        for th in threads:
            torch.set_num_threads(th)
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
            runs.append({"threads": th, "capacity": cap, "value": batch * steps / el, "steps": steps,
                         "seconds": round(el, 2)})
        del L
    torch.set_num_threads(saved)
    at_cap = [r for r in runs if r["capacity"] == min(args.capacity, ncap)] or runs
    main_run = max(at_cap, key=lambda r: r["value"])
    return {"value": main_run["value"], "unit": "transitions/s", "cores": main_run["threads"], "kind": "port",
            "sample": f"oracle/ref.py OracleLearner {args.algo} {net_name(args)} batch {batch}, "
                      f"{'SumTree' if per else 'deque'} of {main_run['capacity']} transitions, {main_run['steps']} "
                      f"learn+soft-update steps in {main_run['seconds']} s, torch {torch.__version__} CPU, "
                      f"{main_run['threads']} threads on {info['model']} ({info['physical_cores']} physical cores "
                      f"on the host, {info['usable_cpus']} in the affinity mask, CPU share {info['cpu_share']} "
                      f"from {info['cpu_share_source']}); the fastest of the runs at {threads} threads",
            "cpu": info, "threads_run": threads, "runs": runs}


# ----------------------------------------------------------------------------------------
# GPU measurements
# ----------------------------------------------------------------------------------------
def set_rngs(eng, per, rank_seed=0):
    random.seed(1234 + rank_seed)   # the replay sampler continues CPython's MT19937 stream
    eng.set_rng(C.DQNX_RNG_PY, np.array(random.getstate()[1], dtype=np.uint32))
    if per:                         # PER draws numpy's legacy global stream (np.random.uniform)
        np.random.seed(1234)
        st = np.random.get_state()
        eng.set_rng(C.DQNX_RNG_NP, np.append(st[1], st[2]).astype(np.uint32))


def make_engine(args, spec, batch_global, world, rank, device, local=False):
    eng = LearnEngine(spec, args.algo, batch_global, args.capacity, world_size=world, rank=rank, device=device,
                      graphs=args.graphs, local_sampling=local, compute_dtype=args.compute,
                      per_numpy121=getattr(args, "per_numpy121", False))
    eng.load_params(init_params(spec, 0))
    fill_ring(eng, args.capacity, spec.obs_dim, args.actions, device, seed=0)
    set_rngs(eng, args.algo.startswith("Per"), rank if local else 0)
    return eng


def timed_steps(step, steps, dist, device, chain=1):
    """`steps` steps bracketed by barrier + synchronize on both sides; max over ranks (s).
    chain > 1: step(c) runs c learn steps per call (steps // chain calls + the remainder)."""
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if chain > 1:
        for _ in range(steps // chain):
            step(chain)
        if steps % chain:
            step(steps % chain)
    else:
        for _ in range(steps):
            step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def run_learner(args, eng, world, backend, steps, warmup, dist, device, dp=None):
    """Warm up, then time `steps` learn steps (single GPU: the engine's graph; DP: the whole DP
    step as one HIP graph over RCCL).  Returns (seconds, dp_graph)."""
    # conv nets exchange per-layer gradient buckets on a side stream, overlapped with the rest of
    # the backward (dp_learn_step_bucketed); the MLP's 428 KB gradient stays one all-reduce
    dp = world > 1 if dp is None else dp   # the data-parallel step (DQNX_BENCH_FORCE_DP: also at world 1)
    bucketed = dp and ((args.net != "mlp" and not args.no_buckets) or (args.net == "mlp" and args.mlp_buckets))
    if bucketed and args.net == "mlp" and len(eng.dp_buckets()) < 2:
        bucketed = False   # (past 2048 rows per GPU the MLP's gradient comes from the slab plan: one bucket)

    chain = args.chain if not dp else 1

    # pure learning loop, uniform replay: step t+1's minibatch is drawn inside step t's forward launch
    # (bucketed conv nets sample their own minibatch; the bucketed MLP step prefetches like the plain one)
    prefetch = args.prefetch and not args.algo.startswith("Per") and (not bucketed or args.net == "mlp")

    def step(count=1):
        if dp:   # shard compute, RCCL all-reduce (+ PER |delta| all-gather), replicated Adam
            if bucketed:
                dp_learn_step_bucketed(eng, soft_update=True, prefetch=prefetch)
            else:
                dp_learn_step(eng, soft_update=True, prefetch=prefetch)
        elif chain > 1:
            eng.learn_steps(count, soft_update=True)
        else:
            eng.learn_step(soft_update=True, prefetch=prefetch)
    for _ in range(warmup):
        step(chain)
    torch.cuda.synchronize()
    eng.check_device_error()
    dp_graph = False
    # (PER shard steps too: the ~3x slower graphed PER steps of round 3 were the one-GPU projection's
    # stale |delta| shards, not the graphs -- tools/c5_graph_diag.py)
    if dp and backend == "nccl" and not args.no_dp_graph:
        # the whole DP step (shard kernels + RCCL all-reduce + Adam) as one replayed graph: the
        # eager loop is host-bound (3 launches + a collective call per ~50 us step).  RCCL
        # collectives are capturable; gloo's are host calls and never are.
        gs = max(1, args.dp_graph_steps)
        g = GraphedDPStep(eng, soft_update=True, bucketed=bucketed, prefetch=prefetch, steps=gs)
        g()   # one untimed replay
        torch.cuda.synchronize()
        dp_graph = True
        eager_step = step

        def step(count=1):   # count steps: whole replays, the remainder eagerly
            for _ in range(count // gs):
                g()
            for _ in range(count % gs):
                eager_step()
        chain = gs
    el = timed_steps(step, steps, dist, device, chain)
    if prefetch and (dp or chain == 1):   # consume the minibatch drawn ahead (none pending after)
        if dp and bucketed:
            dp_learn_step_bucketed(eng, soft_update=True)
        elif dp:
            dp_learn_step(eng, soft_update=True)
        else:
            eng.learn_step(soft_update=True)
    if dp_graph:
        eng.set_graphs(args.graphs)   # GraphedDPStep switched the engine's own graphs off
    eng.check_device_error()
    return el, dp_graph


def kernel_infos(eng, flags):
    L = C.lib()
    n = C.I32()
    C.check(L.dqnx_learn_kernel_count(eng.h, flags, ctypes.byref(n)), "kernel_count")
    infos = []
    for i in range(n.value):
        nm = ctypes.create_string_buffer(64)
        fl, by = ctypes.c_double(), ctypes.c_double()
        C.check(L.dqnx_learn_kernel_info(eng.h, flags, i, nm, 64, ctypes.byref(fl), ctypes.byref(by)), "info")
        infos.append((nm.value.decode(), fl.value, by.value))
    return infos


def kernel_times(eng, flags, count=50, reps=5, only=None):
    """In-context time per launch of every kernel of a learn step: K graph-launched steps with
    and without the kernel (dqnx_learn_step_omit), bracketed by HIP events recorded on the
    engine's own stream; the median of `reps` interleaved pairs.  Returns [(name, us, flops, bytes)]."""
    L = C.lib()
    infos = kernel_infos(eng, flags)
    stream = eng.stream()
    hs = torch.cuda.current_stream(eng.device)   # the engine launches on this stream: events go there too

    def graph_steps_ms(omit):
        C.check(L.dqnx_learn_step_omit(eng.h, flags, omit, stream), "omit step")   # capture
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record(hs)
        for _ in range(count):
            C.check(L.dqnx_learn_step_omit(eng.h, flags, omit, stream), "omit step")
        t1.record(hs)
        t1.synchronize()
        return t0.elapsed_time(t1) / count

    out = []
    for i, (nm, fl, by) in enumerate(infos):
        if only is not None and nm not in only:
            continue
        d = sorted(graph_steps_ms(-1) - graph_steps_ms(i) for _ in range(reps))
        out.append((nm, d[len(d) // 2] * 1e3, fl, by))
    return out


def kernel_event_us(eng, flags, name, count=100):
    """Average launch duration of kernel `name` of the learn step, measured live with a HIP event pair
    recorded on the engine's stream immediately before and after that one launch (dqnx_learn_step_timed:
    every other kernel of the step is enqueued eagerly around it, so the pair brackets the kernel alone),
    over `count` steps; the host enqueues all of them before reading the events.  This is the quantity
    rocprofv3's kernel trace reports (dispatch begin to end), unlike kernel_times' with / without
    difference.  Returns (mean_us, median_us)."""
    L = C.lib()
    infos = kernel_infos(eng, flags)
    idx = next(i for i, k in enumerate(infos) if k[0] == name)
    stream = eng.stream()
    ev = (ctypes.c_void_p * (2 * count))()
    C.check(L.dqnx_events_create(2 * count, ev), "events_create")
    try:
        for _ in range(5):   # warm: the same launches as the timed ones
            C.check(L.dqnx_learn_step_timed(eng.h, flags, idx, ev[0], ev[1], stream), "timed step")
        torch.cuda.synchronize()
        for j in range(count):
            C.check(L.dqnx_learn_step_timed(eng.h, flags, idx, ev[2 * j], ev[2 * j + 1], stream), "timed step")
        us = []
        for j in range(count):
            ms = ctypes.c_float()
            C.check(L.dqnx_event_elapsed(ev[2 * j], ev[2 * j + 1], ctypes.byref(ms)), "event_elapsed")
            us.append(ms.value * 1e3)
    finally:
        torch.cuda.synchronize()
        L.dqnx_events_destroy(2 * count, ev)
    us.sort()
    return sum(us) / len(us), us[len(us) // 2]


ROCPROF_ROUND = "r06"


def rocprof_avg_us(stats_name, kernel):
    """The committed rocprofv3 --kernel-trace --stats summary of this same bench command
    (profiles/<round>/kernel_stats_<workload>.csv): average duration (us) of the kernel whose name
    contains k_<kernel> (the engine's kernel names are k_<timing name>), or None."""
    path = os.path.join(REPO, "profiles", ROCPROF_ROUND, f"kernel_stats_{stats_name}.csv")
    if not os.path.exists(path):
        return None, None
    import csv
    tname = kernel.split("+")[0]
    # timing names whose kernel function is named otherwise; the implicit-GEMM convs (configs[2]) share
    # one kernel template, one instantiation per conv: the dominant conv_fwd_c2 is the k_conv_ig
    # instantiation with the largest total time
    alias = {"dw_all": ("k_dw_bf16", "k_bwd_level"), "adam_fused": ("k_adam4", "k_adam")}
    bases = alias.get(tname, ("k_" + tname,))
    key = "TotalDurationNs" if tname.startswith("conv_fwd_c") else "Calls"
    if tname.startswith("conv_fwd_c"):
        bases = ("k_conv_ig",)
    best = None
    with open(path) as f:
        rows = list(csv.DictReader(f))
    for base in bases:
        for row in rows:
            nm = row.get("Name", "").replace("(anonymous namespace)::", "")
            short = nm.split("(")[0].split("<")[0].split("::")[-1].strip()
            if short == base and (best is None or float(row[key]) > float(best[key])):
                best = row
        if best is not None:
            break
    if best is None:
        return None, path
    return float(best["AverageNs"]) / 1e3, os.path.relpath(path, REPO)


def pmc_traffic(args, batch_tag):
    """The committed rocprofv3 PMC traffic passes of this workload (profiles/pmc_traffic_*.json):
    {kernel: hbm bytes per launch} (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction), or {}."""
    tag = "" if args.compute == "fp32" else f"_{args.compute}"
    pmc_path = os.path.join(REPO, "profiles", f"pmc_traffic_{args.net}_b{batch_tag}{tag}.json")
    if not os.path.exists(pmc_path):
        return {}
    try:
        pmc = json.load(open(pmc_path))
        return {k: v["hbm_bytes_per_launch"] for k, v in pmc.items() if isinstance(v, dict) and "hbm_bytes_per_launch" in v}
    except Exception:
        return {}


def roofline_of(args, kern, batch_tag, incontext_us=None, stats_name=None, step_kernels=None):
    """roofline object for the dominant kernel: achieved algorithmic FLOP/s (or B/s) against the
    MI355X peak of the compute dtype, plus both fractions.  kern = (name, avg_us, flops, bytes) with
    avg_us the kernel's average launch duration measured live by HIP events around the launch
    (kernel_event_us).  `traffic` = HBM bytes per launch from the committed rocprofv3 PMC passes of the
    same workload; `traffic_ratio` = traffic / algorithmic bytes (per launch and, over every kernel of
    the step the passes cover, per step).  `rocprof` = the committed kernel-trace average of the same
    kernel (profiles/<round>/kernel_stats_<stats_name>.csv) and the fraction it gives."""
    nm, us_live, fl, by = kern
    peak_mfma = PEAK_BF16_MFMA_TFLOPS if args.compute == "bf16" else PEAK_FP32_MFMA_TFLOPS
    # the duration behind achieved / frac (reproducible from profiles/): the committed
    # rocprofv3 kernel-trace average of this workload's kernel when there is one, else the live
    # event-bound measurement; both are on the line (avg_us_events, frac_live)
    rp_us, rp_path = rocprof_avg_us(stats_name, nm) if stats_name else (None, None)
    us = rp_us or us_live
    pmc = pmc_traffic(args, batch_tag)
    traffic = pmc.get(nm, pmc.get(nm.split("+")[0]))
    sec = us * 1e-6
    mfma_ach = fl / sec / 1e12 if fl else 0.0
    hbm_ach = by / sec / 1e9
    mfma_frac = mfma_ach / peak_mfma
    hbm_frac = hbm_ach / PEAK_HBM_GBS
    ridge = peak_mfma * 1e12 / (PEAK_HBM_GBS * 1e9)
    intensity = fl / (traffic or by) if (traffic or by) else 0.0
    # the bound from the measured limiter: a kernel is HBM-bound only when its MEASURED traffic (PMC,
    # else its algorithmic bytes) streams at >= half the HBM peak or it does no math; otherwise its
    # roof is the MFMA peak of the compute dtype, whatever bounds it below that (LDS, L2->VGPR, latency:
    # DESIGN.md section 3), and `frac` says how far below it runs
    hbm_measured_frac = ((traffic or by) / sec / 1e9) / PEAK_HBM_GBS
    mfma_bound = fl > 0 and hbm_measured_frac < 0.5
    common = {"traffic": traffic, "kernel": nm, "avg_us": us,
              "avg_us_source": (f"rocprofv3 --kernel-trace --stats average ({rp_path})" if rp_us else
                                "HIP events bound to the launch's dispatch (kernel_event_us)"),
              "avg_us_events": us_live,
              "algorithmic_flops": fl, "algorithmic_bytes": by,
              "traffic_ratio": (traffic / by) if (traffic and by) else None,
              "mfma_frac": mfma_frac, "hbm_frac": hbm_frac, "hbm_measured_frac": hbm_measured_frac,
              "intensity_flop_per_byte": intensity, "ridge_flop_per_byte": ridge}
    if incontext_us is not None:   # the step-time difference with / without the kernel (kernel_times)
        common["avg_us_incontext_omit"] = incontext_us
    if step_kernels:
        covered = [(k[0], k[3]) for k in step_kernels if pmc.get(k[0], pmc.get(k[0].split("+")[0])) is not None]
        if covered:
            t = sum(pmc.get(n, pmc.get(n.split("+")[0])) for n, _ in covered)
            b = sum(b for _, b in covered)
            common["traffic_step"] = t
            common["algorithmic_bytes_step"] = b
            common["traffic_ratio_step"] = t / b if b else None
            common["traffic_step_kernels"] = [n for n, _ in covered]
    frac_live = (fl / (us_live * 1e-6) / 1e12 / peak_mfma) if mfma_bound else (by / (us_live * 1e-6) / 1e9 / PEAK_HBM_GBS)
    common["frac_live"] = frac_live
    if rp_us:
        common["rocprof"] = {"avg_us": rp_us, "file": rp_path, "events_over_rocprof": us_live / rp_us}
    if mfma_bound:
        return dict({"bound": "mfma", "achieved": mfma_ach, "peak": peak_mfma, "unit": "TFLOP/s",
                     "frac": mfma_frac}, **common)
    return dict({"bound": "hbm", "achieved": hbm_ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": hbm_frac},
                **common)


def dominant_roofline(args, eng, flags, batch_tag, stats_name, count=50, reps=5, ev_count=200):
    """Every kernel's in-context time (kernel_times), the dominant one picked by it, then that kernel's
    average launch duration from HIP event pairs (kernel_event_us) for the roofline.
    Returns (kernels list, roofline)."""
    ks = kernel_times(eng, flags, count=count, reps=reps)
    dom = max(ks, key=lambda k: k[1])
    mean_us, med_us = kernel_event_us(eng, flags, dom[0], count=ev_count)
    kernels = [{"kernel": k[0], "avg_us_incontext_omit": k[1], "flops": k[2], "bytes": k[3]} for k in ks]
    for k in kernels:
        if k["kernel"] == dom[0]:
            k["avg_us_events"] = mean_us
            k["median_us_events"] = med_us
    roof = roofline_of(args, (dom[0], mean_us, dom[2], dom[3]), batch_tag, incontext_us=dom[1],
                       stats_name=stats_name, step_kernels=ks)
    roof["median_us_events"] = med_us
    return kernels, roof


ALLREDUCE_EST_US = 20.0   # assumed RCCL all-reduce of the 428 KB MLP-284 gradient over 8 xGMI-linked GPUs


def shard_td_exchange(eng):
    """Stand-in, on one GPU, for the |delta| all-gather of a PER shard step: the other ranks' shards of
    `per_abs_td` get this rank's |delta| (one small copy kernel).  Without it the ordered priority update
    of the projection writes stale |delta| for 7/8 of the minibatch, and the degenerate priorities it
    leaves (most sampled leaves at the minimum) make the SumTree max / min rescans run nearly every step
    after a few hundred steps (profiles/r04/c5_dynamics.json): the projection would time a state no
    real world-8 run reaches."""
    W = eng.world_size
    if W > 1 and eng.per_abs_td.numel():
        n = eng.batch // W
        td = eng.per_abs_td
        td[n:].view(W - 1, n).copy_(td[:n].unsqueeze(0).expand(W - 1, n))


def graphed_shard_steps(eng, args, steps, device, prefetch=None):
    """`steps` GRADS_ONLY shard steps (+ apply_grads) replayed --dp-graph-steps per captured graph, as
    GraphedDPStep runs them under torchrun (the collective left out; PER: shard_td_exchange in its place).
    Returns (seconds, steps per graph)."""
    prefetch = args.prefetch if prefetch is None else prefetch
    gs = max(1, args.dp_graph_steps)
    eng.set_graphs(False)
    if prefetch:
        eng.prefetch_prologue()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with dp_capture(g):
        for _ in range(gs):
            eng.learn_step(grads_only=True, prefetch=prefetch)
            shard_td_exchange(eng)
            eng.apply_grads(soft_update=True)
    for _ in range(max(2, args.warmup // gs)):
        g.replay()
    n = max(1, steps // gs)
    el = timed_steps(lambda: g.replay(), n, None, device)
    if prefetch:   # the replays ran on this stream: dqnx_rng_get / the next step wait on it
        C.check(C.lib().dqnx_prefetch_stream(eng.h, eng.stream()), "prefetch_stream")
        eng.learn_step(grads_only=True)   # consume the pending draw
        eng.apply_grads(soft_update=True)
    torch.cuda.synchronize()
    eng.check_device_error()
    eng.set_graphs(args.graphs)
    del g
    return el * steps / (n * gs), gs


def single_gpu_extras(args, spec, device):
    """configs[3] points measured on this one GPU:
    * configs3_n1: the learn step at the global minibatch 4096 (strong-scaling N = 1 point);
    * projection_w8: the rank-0 shard step of a world_size = 8 engine (512 rows, the global
      4096-draw sampler, Adam + soft update) -- every term of the 8-GPU step but the all-reduce."""
    out = {}
    Bg = args.global_batch
    eng = make_engine(args, spec, Bg, 1, 0, device)
    el, _ = run_learner(args, eng, 1, None, max(args.steps, 50), args.warmup, None, device)
    ks = kernel_times(eng, C.STEP_SOFT_UPDATE, count=50, reps=3, only={"sample_uniform", "mlp_fwd"})
    steps = max(args.steps, 50)
    out["configs3_n1"] = {"value": Bg * steps / el, "ms_per_step": el / steps * 1e3, "batch": Bg,
                          "kernels": [{"kernel": k[0], "avg_us": k[1]} for k in ks]}
    del eng
    torch.cuda.empty_cache()
    W = 8
    eng = make_engine(args, spec, Bg, W, 0, device)

    def shard_step(prefetch=args.prefetch):   # what each rank runs around the all-reduce
        eng.learn_step(grads_only=True, prefetch=prefetch)
        eng.apply_grads(soft_update=True)
    for _ in range(args.warmup):
        shard_step()
    el_eager = timed_steps(shard_step, steps, None, device)
    shard_step(prefetch=False)   # consume the pending draw
    # the way the N > 1 bench runs it: --dp-graph-steps shard steps per replayed graph (GraphedDPStep
    # without the collective)
    el, gs = graphed_shard_steps(eng, args, steps, device)
    seq = {}
    if args.prefetch:   # the same shard step with the sampler launch on the critical path
        for _ in range(args.warmup):
            shard_step(prefetch=False)
        el_seq = timed_steps(lambda: shard_step(prefetch=False), steps, None, device)
        seq = {"shard_step_us_sampler_launch": el_seq / steps * 1e6}
    ks = kernel_times(eng, C.STEP_GRADS_ONLY, count=50, reps=3)
    samp = next((k[1] for k in ks if k[0] == "sample_uniform"), None)
    kpf = kernel_times(eng, C.STEP_GRADS_ONLY | C.STEP_PREFETCH, count=50, reps=3) if args.prefetch else []
    out["projection_w8"] = dict({
        "rows_per_rank": Bg // W, "global_batch": Bg, "shard_step_us": el / steps * 1e6,
        "shard_step_us_eager": el_eager / steps * 1e6, "steps_per_graph": gs,
        "prefetch_sampling": args.prefetch,
        "global_sampling_us": samp,
        "tr_per_s_without_allreduce": Bg / (el / steps),
        "kernels": [{"kernel": k[0], "avg_us": k[1]} for k in ks],
        "kernels_prefetch": [{"kernel": k[0], "avg_us": k[1]} for k in kpf],
        "note": "rank 0 of world_size 8 on one GPU: 512-row shard + grad reduce + Adam/soft update, the global "
                "4096-draw sampler inside the forward launch (prefetch) or as its own launch, replayed "
                f"{gs} steps per captured graph like the N>1 bench (shard_step_us_eager: one host call per "
                "launch); add the RCCL all-reduce of the 428 KB gradient for the 8-GPU step"}, **seq)
    # Amdahl bound of 8-GPU strong scaling at global 4096: the one-GPU step
    # over 8 x (the shard step + an all-reduce estimate).  The all-reduce term is an assumption
    # (RCCL ring over xGMI, 428 KB fp32 gradient: latency-dominated), not a measurement.
    t1 = out["configs3_n1"]["ms_per_step"] * 1e3
    shard = out["projection_w8"]["shard_step_us"]
    out["projection_w8"]["efficiency_bound"] = {
        "without_allreduce": t1 / (W * shard),
        "with_allreduce": t1 / (W * (shard + ALLREDUCE_EST_US)),
        "allreduce_estimate_us": ALLREDUCE_EST_US, "one_gpu_step_us": t1}
    del eng
    torch.cuda.empty_cache()
    out["projection_w8_weak"] = weak_projection(args, spec, device, t1)
    return out


def sampler_route(k, capacity):
    """Which random.sample kernel the engine launches for k draws (csrc/sample.hip launch_sample_uniform)."""
    if 2048 <= k <= 4608:
        return "k_sample_fast (one-round draw, bitmap dedup, MT block cache; csrc/sample_pipe.hpp)"
    need = 4 * (k + 624)
    hs = 2048
    while hs < need and hs < 16384:
        hs <<= 1
    if need <= 3 * hs:
        return f"k_sample_uniform<{hs}> (one 1024-thread workgroup, LDS hash table of {hs} slots)"
    if capacity <= (1 << 20):
        return ("k_sample_bitmap (one 1024-thread workgroup: a seen-bit per value of the <= 2^20 population in LDS, "
                "passes of up to 5 MT blocks, in-pass repeats resolved in a small LDS table; csrc/sample_body.hpp)")
    hs = 32768
    while hs < need:
        hs <<= 1
    return (f"k_sample_uniform_g<{hs}> (one 1024-thread workgroup, multi-pass body, a {hs}-slot (value, position) "
            "hash table in global memory)")


def weak_projection(args, spec, device, t1_us, W=8, rows=4096):
    """Weak scaling (4096 rows per rank, global minibatch 32768 at world 8), rank 0 of a world_size = 8
    engine on one GPU: every rank draws the SAME global 32768-sample random.sample (bit-exact with one
    GPU, R:dqn/replay_memory.py:38-39) and computes its 4096-row shard, then Adam + soft update.  The
    efficiency bound is the one-GPU 4096-row step (configs3_n1) over the shard step (+ the all-reduce
    estimate); the sampler's route and cost at k = 32768 are measured as its own launch."""
    Bg = rows * W
    eng = make_engine(args, spec, Bg, W, 0, device)
    steps = max(args.steps // 2, 50)

    def shard_step(prefetch=args.prefetch):
        eng.learn_step(grads_only=True, prefetch=prefetch)
        eng.apply_grads(soft_update=True)
    for _ in range(args.warmup):
        shard_step()
    el_pf = timed_steps(shard_step, steps, None, device)
    shard_step(prefetch=False)   # consume the pending draw
    for _ in range(max(2, args.warmup // 2)):
        shard_step(prefetch=False)
    el_seq = timed_steps(lambda: shard_step(prefetch=False), steps, None, device)
    el_g, gs = graphed_shard_steps(eng, args, steps, device)   # as GraphedDPStep replays it under torchrun
    ks = kernel_times(eng, C.STEP_GRADS_ONLY, count=30, reps=3)
    samp = next((k for k in ks if k[0].startswith("sample")), None)
    samp_ev = kernel_event_us(eng, C.STEP_GRADS_ONLY, samp[0], count=50) if samp else None
    kpf = kernel_times(eng, C.STEP_GRADS_ONLY | C.STEP_PREFETCH, count=30, reps=3) if args.prefetch else []
    del eng
    torch.cuda.empty_cache()
    shard_pf, shard_seq, shard_g = el_pf / steps * 1e6, el_seq / steps * 1e6, el_g / steps * 1e6
    shard = min(shard_pf, shard_seq, shard_g)
    return {"rows_per_rank": rows, "global_batch": Bg, "world": W,
            "shard_step_us": shard, "shard_step_us_prefetch": shard_pf, "shard_step_us_sampler_launch": shard_seq,
            "shard_step_us_graphed": shard_g, "graph_steps": gs,
            "one_gpu_step_us_4096": t1_us,
            "sampler": {"kernel": samp[0] if samp else None, "k": Bg,
                        "route": sampler_route(Bg, args.capacity),
                        "avg_us_events": samp_ev[0] if samp_ev else None,
                        "avg_us_incontext_omit": samp[1] if samp else None},
            "kernels": [{"kernel": k[0], "avg_us": k[1]} for k in ks],
            "kernels_prefetch": [{"kernel": k[0], "avg_us": k[1]} for k in kpf],
            "efficiency_bound": {"without_allreduce": t1_us / shard,
                                 "with_allreduce": t1_us / (shard + ALLREDUCE_EST_US),
                                 "allreduce_estimate_us": ALLREDUCE_EST_US},
            "note": "weak scaling: per-GPU work fixed at 4096 rows; efficiency = one-GPU 4096-row step time / "
                    "world-8 shard step time (each rank still draws the global 32768-sample random.sample, the "
                    "replicated O(B_global) term); the all-reduce term is an estimate, the driver's 8-GPU node "
                    "measures it"}


def head_net_extra(args, device):
    """The reference's HEAD net (TwoStreamHybridNetwork on the (2,27,5) grid + 14 macro features,
    R:env/dqn_config.py:66-193, the net bin/train.sh trains), DuelingDouble fp32, B=256, in the same
    learning loop as the headline (eager, in-launch prefetch), with its dominant kernel's roofline."""
    import copy
    a = copy.copy(args)
    a.net, a.batch = "hybrid", 256
    spec = make_spec(a)
    eng = make_engine(a, spec, 256, 1, 0, device)
    steps = max(args.steps, 100)
    el, _ = run_learner(a, eng, 1, None, steps, args.warmup, None, device)
    flags = C.STEP_SOFT_UPDATE | (C.STEP_PREFETCH if a.prefetch else 0)
    kernels, roof = dominant_roofline(a, eng, flags, 256, "hybrid_b256", count=50, reps=3, ev_count=200)
    out = {"value": 256 * steps / el, "unit": "transitions/s", "ms_per_step": el / steps * 1e3, "batch": 256,
           "net": net_name(a), "algo": a.algo, "dtype": "fp32", "kernels": kernels, "roofline": roof}
    del eng
    torch.cuda.empty_cache()
    return out


def configs0_extra(args, device):
    """configs[0]: the reference's CPU plumbing case -- MLP Q-net, batch 32 (HYPER_PARAMS['bs'],
    R:env/dqn_config.py:37) -- timed both ways on this box: the oracle learner (torch CPU restatement of
    the reference learn step) on the host cores at MLP-284 and MLP-14, and the same learn step on the
    GPU engine (uniform replay, DuelingDouble, the learning loop of the headline), where B = 32 is pure
    launch latency."""
    import copy
    out = {"batch": 32, "replay_capacity": 100_000}
    for D in (284, 14):
        a = copy.copy(args)
        a.obs_dim, a.batch, a.capacity = D, 32, 100_000
        spec = make_spec(a)
        eng = make_engine(a, spec, 32, 1, 0, device)
        steps = max(args.steps, 200)
        el, _ = run_learner(a, eng, 1, None, steps, max(args.warmup, 20), None, device)
        row = {"gpu": {"value": 32 * steps / el, "unit": "transitions/s", "ms_per_step": el / steps * 1e3}}
        del eng
        torch.cuda.empty_cache()
        if not args.no_cpu_baseline:
            try:
                a.cpu_seconds = min(args.cpu_seconds, 3.0)
                cb = cpu_baseline(a, 32)
                row["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
            except Exception as ex:   # the baseline must never hide the GPU number
                log(f"configs0 cpu baseline failed: {ex!r}")
        out[f"mlp{D}"] = row
    return out


def configs2_extra(args, device):
    """configs[2] as BASELINE.json states it: the stacked 4x84x84 occupancy-grid CNN encoder + dueling
    head (TwoStreamHybridNetwork on a (4,84,84) micro grid, R:env/dqn_config.py:97-143: the class is
    shape-generic), DuelingDouble fp32, B=256, replay capacity 1e5 resident in HBM (113 KB rows), in the
    same learning loop as the headline, with its dominant kernel's roofline (traffic from the committed
    PMC passes) and the oracle's CPU baseline on a 2e3-transition deque (a 1e5 host deque of these rows
    would need 22.6 GB)."""
    import copy
    a = copy.copy(args)
    a.net, a.batch, a.capacity = "hybrid84", 256, 100_000
    spec = make_spec(a)
    eng = make_engine(a, spec, 256, 1, 0, device)
    steps = max(args.steps, 20)
    el, _ = run_learner(a, eng, 1, None, steps, max(2, min(args.warmup, 5)), None, device)
    flags = C.STEP_SOFT_UPDATE | (C.STEP_PREFETCH if a.prefetch else 0)
    kernels, roof = dominant_roofline(a, eng, flags, 256, "hybrid84_b256", count=6, reps=3, ev_count=20)
    out = {"value": 256 * steps / el, "unit": "transitions/s", "ms_per_step": el / steps * 1e3, "steps": steps,
           "batch": 256, "replay_capacity": a.capacity, "net": net_name(a), "algo": a.algo, "dtype": "fp32",
           "workload": workload_name(a, 1), "kernels": kernels, "roofline": roof}
    del eng
    torch.cuda.empty_cache()
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(a, 256)
        except Exception as ex:   # the baseline must never hide the GPU number
            log(f"configs2 cpu baseline failed: {ex!r}")
    return out


def c5_projection(args, device):
    """configs[4] (PER + DuelingDouble, bf16 compute, global minibatch 8192): the one-GPU step, and
    the rank-0 shard step of a world_size = 8 engine (1024 rows; the replicated O(B_global) PER
    sampler and tree update included, the |delta| all-gather and gradient all-reduce not)."""
    import copy
    a = copy.copy(args)
    a.algo, a.compute = "PerDuelingDoubleDQNAgent", "bf16"
    spec = make_spec(a)
    Bg, W = 8192, 8
    steps = max(args.steps // 2, 50)
    eng = make_engine(a, spec, Bg, 1, 0, device)
    el1, _ = run_learner(a, eng, 1, None, steps, args.warmup, None, device)
    kernels1, roof1 = dominant_roofline(a, eng, C.STEP_SOFT_UPDATE, Bg, "mlp_b8192_bf16", count=30, reps=3,
                                        ev_count=100)
    del eng
    torch.cuda.empty_cache()
    eng = make_engine(a, spec, Bg, W, 0, device)

    def shard_step():
        eng.learn_step(grads_only=True)
        shard_td_exchange(eng)              # (the |delta| all-gather's output)
        eng.apply_grads(soft_update=True)   # Adam + the PER tree update of all 8192 |delta|
    for _ in range(args.warmup):
        shard_step()
    el_eager = timed_steps(shard_step, steps, None, device)
    el, gs = graphed_shard_steps(eng, a, steps, device, prefetch=False)
    ks = kernel_times(eng, C.STEP_GRADS_ONLY, count=30, reps=3)
    del eng
    torch.cuda.empty_cache()
    # (round 3 measured these graphed PER shard steps at ~3x the eager time: an artefact of the
    # projection, which wrote stale |delta| for 7/8 of the minibatch until shard_td_exchange; the
    # faster of the two is the projection, both are reported)
    t1, shard_g, shard_e = el1 / steps * 1e6, el / steps * 1e6, el_eager / steps * 1e6
    shard = min(shard_g, shard_e)
    return {"one_gpu_step_us": t1, "one_gpu_value": Bg * steps / el1, "one_gpu_kernels": kernels1,
            "one_gpu_roofline": roof1, "rows_per_rank": Bg // W,
            "shard_step_us": shard, "shard_step_us_eager": shard_e, "shard_step_us_graph": shard_g,
            "steps_per_graph": gs,
            "tr_per_s_without_collectives": Bg / (shard * 1e-6),
            "kernels": [{"kernel": k[0], "avg_us": k[1]} for k in ks],
            "efficiency_bound": {"without_collectives": t1 / (W * shard),
                                 "with_allreduce": t1 / (W * (shard + ALLREDUCE_EST_US)),
                                 "allreduce_estimate_us": ALLREDUCE_EST_US},
            "note": "rank 0 of world_size 8 on one GPU: the 1024-row shard's GRADS_ONLY step (every rank draws the "
                    "same global 8192 PER sample) + apply_grads (Adam, soft update, the ordered priority update "
                    "of all 8192 |delta| on every tree replica), the other ranks' |delta| shards filled from "
                    "rank 0's by one copy kernel in place of the all-gather; add the |delta| all-gather (32 KB) "
                    "and the 428 KB gradient all-reduce for the 8-GPU step"}


def dropin_loop(args, device, batch=1024, iters=200, warmup=20):
    """The drop-in path a reference user runs (R:train.py:88-108): `Agents.DuelingDoubleDQNAgent`
    on the macro-lane MLP, one env row per iteration (n_env = 1):
    choose_actions -> store_transitions -> learn -> update_target_network, timed per call on the
    host clock, the stream synchronised only before the clock stops (as in train.py, where the next
    choose_actions waits for the GPU).  The default Agent: learn() stages the RNG (host mirror of the
    draw) and launches the step at once, update_target_network() enqueues the soft update;
    `deferred_fused`: DQNX_AGENT_DEFER=1 (learn() recorded, launched by update_target_network with the
    soft update fused into the Adam pass).  The replay is pre-filled through the engine (synthetic
    rows, like the headline line)."""
    import tempfile

    import torch.optim as optim
    from dqn import Agents

    class Box:
        shape = (args.obs_dim,)

    def net_conf(space):   # R:env/custom_env/macro with lane/dqn_config.py:58-104 (MLP, ReLU, Adam)
        act = nn.ReLU()
        return (nn.Sequential(nn.Linear(space.shape[0], 256), act, nn.Linear(256, 128), act), 128, optim.Adam,
                nn.SmoothL1Loss)

    def run(defer, graphs=False, inplace=True):
        os.environ["DQNX_AGENT_DEFER"] = "1" if defer else "0"
        os.environ["DQNX_AGENT_GRAPHS"] = "1" if graphs else "0"
        os.environ["DQNX_AGENT_MT_INPLACE"] = "1" if inplace else "0"
        tmp = tempfile.mkdtemp(prefix="dqnx_dropin_")
        agent = Agents.DuelingDoubleDQNAgent(
            n_env=1, lr=1e-4, gamma=0.99, epsilon_start=1.0, epsilon_min=0.05, epsilon_decay=2e6,
            epsilon_exp_decay=False, nn_conf_func=net_conf, input_dim=Box(), output_dim=args.actions,
            batch_size=batch, min_buffer_size=batch, buffer_size=args.capacity, update_target_frequency=30000,
            target_soft_update=True, target_soft_update_tau=1e-3, save_frequency=10 ** 9, log_frequency=10 ** 9,
            save_dir=tmp + "/", log_dir=tmp + "/", load=False, algo="DuelingDoubleDQNAgent",
            gpu=str(device.index or 0))
        fill_ring(agent.engine, min(args.capacity, 100_000), args.obs_dim, args.actions, device, seed=0)
        rng = np.random.default_rng(0)
        obs = rng.random((iters + warmup + 1, args.obs_dim), dtype=np.float32)
        random.seed(1234)
        phases = {"choose_actions": 0.0, "store_transitions": 0.0, "learn": 0.0, "update_target_network": 0.0}
        t_start = None
        for t in range(iters + warmup):
            if t == warmup:
                agent.flush()
                torch.cuda.synchronize(device)
                t_start = time.perf_counter()
            agent.step = t
            t0 = time.perf_counter()
            a = agent.choose_actions(obs[t:t + 1])
            t1 = time.perf_counter()
            agent.store_transitions(obs[t:t + 1], a, [0.5], [False], obs[t + 1:t + 2], None)
            t2 = time.perf_counter()
            agent.learn()
            t3 = time.perf_counter()
            agent.update_target_network()
            t4 = time.perf_counter()
            if t >= warmup:
                phases["choose_actions"] += t1 - t0
                phases["store_transitions"] += t2 - t1
                phases["learn"] += t3 - t2
                phases["update_target_network"] += t4 - t3
        agent.flush()
        torch.cuda.synchronize(device)
        t_all = time.perf_counter() - t_start
        # choose_actions with no learn step in flight (R:train.py's loop with a real env: env.step -- 40
        # TraCI simulation steps, R:env/custom_env/rl_controller.py:211-250 -- runs between learn() and
        # the next choose_actions, so the step has finished): host obs in, action list out
        idle = []
        for t in range(100):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            agent.choose_actions(obs[t:t + 1])
            idle.append(time.perf_counter() - t0)
        idle.sort()
        del agent
        torch.cuda.empty_cache()
        return {"us_per_iteration": t_all / iters * 1e6, "learn_tr_per_s": batch * iters / t_all,
                "phases_us": {k: v / iters * 1e6 for k, v in phases.items()},
                "choose_actions_idle_us": {"median": idle[len(idle) // 2] * 1e6, "p10": idle[len(idle) // 10] * 1e6,
                                           "p90": idle[(9 * len(idle)) // 10] * 1e6}}

    keys = ("DQNX_AGENT_DEFER", "DQNX_AGENT_GRAPHS", "DQNX_AGENT_MT_INPLACE")
    saved = {k: os.environ.get(k) for k in keys}
    try:
        now = run(False)
        dfr = run(True)
        grf = run(False, graphs=True)
        port = run(False, inplace=False)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return dict(now, batch=batch, n_env=1, iterations=iters, deferred_fused=dfr, graphed_step=grf,
                portable_rng=port,
                note="Agents.DuelingDoubleDQNAgent through the R:train.py:88-108 call sequence on the MLP-284 "
                     "macro-lane net; host clock per call; the top-level numbers are the default agent (learn() "
                     "stages random._inst in place and launches the step in one library call), `deferred_fused` "
                     "DQNX_AGENT_DEFER=1, `graphed_step` the learn step as one HIP graph launch "
                     "(DQNX_AGENT_GRAPHS=1), `portable_rng` the getstate / getrandbits hand-off "
                     "(DQNX_AGENT_MT_INPLACE=0); phases_us.choose_actions includes waiting for the learn step "
                     "launched in the previous iteration (no env.step in this loop), choose_actions_idle_us is "
                     "the call with the GPU idle, as after a real env.step")


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
    # DQNX_BENCH_FORCE_DP=1 (rehearsal on a one-GPU box): the N > 1 code path -- process group,
    # GraphedDPStep over RCCL, global-batch sharding -- at world size 1
    dpmode = world > 1 or os.environ.get("DQNX_BENCH_FORCE_DP") == "1"
    if dpmode:
        import torch.distributed as dist
        backend = os.environ.get("DQNX_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    spec = make_spec(args)
    per = args.algo.startswith("Per")
    if not dpmode:
        Bg = args.batch or 1024
        scaling = "strong"
    elif args.scaling == "strong":
        Bg = args.global_batch
        scaling = "strong"
    else:
        Bg = (args.batch or 4096) * world
        scaling = "weak"
    if Bg % world:
        raise SystemExit(f"global batch {Bg} is not a multiple of {world} ranks")
    Bl = Bg // world
    local = dpmode and args.local_sampling and not per
    eng = make_engine(args, spec, Bg, world, rank, device, local=local)
    el, dp_graph = run_learner(args, eng, world, backend, args.steps, args.warmup, dist, device, dp=dpmode)
    loss = eng.loss()
    ms_per_step = el / args.steps * 1e3
    value = Bg * args.steps / el

    # ---- dominant-kernel roofline: HIP-event-timed graph steps with / without each kernel ----
    roofline = None
    kernels = []
    if not args.no_kernel_timing:
        flags = C.STEP_GRADS_ONLY if dpmode else C.STEP_SOFT_UPDATE
        if args.prefetch and not per:   # the plan the timed loop ran (steady state: no sampler launch)
            flags |= C.STEP_PREFETCH
        tag = "" if args.compute == "fp32" else f"_{args.compute}"
        kernels, roofline = dominant_roofline(args, eng, flags, Bl, f"{args.net}_b{Bl}{tag}")

    extras = {}
    if not args.no_extras and args.net == "mlp" and not per and args.compute == "fp32":
        del eng
        torch.cuda.empty_cache()
        if not dpmode:
            extras = single_gpu_extras(args, spec, device)
            for name, fn in (("configs0", configs0_extra), ("head_net", head_net_extra), ("configs2", configs2_extra),
                             ("configs4_projection_w8", c5_projection), ("dropin_loop", dropin_loop)):
                try:
                    extras[name] = fn(args, device)
                except Exception as ex:   # an extra must never hide the headline number
                    log(f"{name} failed: {ex!r}")
                torch.cuda.empty_cache()
        elif scaling == "strong":   # the weak-scaling companion line: 4096 rows per rank
            weng = make_engine(args, spec, 4096 * world, world, rank, device, local=local)
            wel, _ = run_learner(args, weng, world, backend, args.steps, args.warmup, dist, device, dp=dpmode)
            extras["weak"] = {"value": 4096 * world * args.steps / wel, "ms_per_step": wel / args.steps * 1e3,
                              "batch_per_gpu": 4096, "global_batch": 4096 * world}
            del weng

    cpu = None
    if rank == 0 and not dpmode and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, Bg)
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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.compute,
            "data": "synthetic",
            "config": {
                "workload": workload_name(args, world),
                "algo": args.algo, "net": net_name(args),
                "batch_per_gpu": Bl, "global_batch": Bg, "replay_capacity": args.capacity,
                "parallelism": f"dp{world}", "graphs": args.graphs, "prefetch_sampling": args.prefetch and not per and (world == 1 or args.net == "mlp"),
                "steps_per_call": args.chain if not dpmode else 1,
                "sampling": "rank-local" if local else "global (reference-exact random.sample on every rank)",
                "dp_step": (((f"one HIP graph per {args.dp_graph_steps} steps" if dp_graph else "eager launches")
                             + (", per-layer gradient buckets" if ((args.net != "mlp" and not args.no_buckets)
                                                                  or (args.net == "mlp" and args.mlp_buckets)) else ""))
                            if dpmode else None),
                "compute": args.compute,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "loss": loss,
            "kernels": kernels,
        }
        out.update(extras)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
