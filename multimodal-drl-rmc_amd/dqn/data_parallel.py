"""Data-parallel learn step: one process per GPU, minibatch sharded, one gradient all-reduce
(SURVEY.md §8(e)).

Every rank runs the same sampler on the same RNG state, so all ranks draw the identical
global minibatch (bit-exact with one GPU). Rank r then computes samples
[r*B/W, (r+1)*B/W) with `DQNX_STEP_GRADS_ONLY`. The loss is a mean over the GLOBAL batch
(the engine scales by 1/B_global), so the SUM of the shard gradients is the full-batch
gradient. Everything after that is identical on every rank:

* one all-reduce (sum) of the flat gradient buffer (+ the loss slot) moves the gradient;
* PER only: one all-gather of the shards' |δ| gives every rank the ordered priority update
  for its tree replica (R:dqn/agent.py:263-265);
* `dqnx_apply_grads` (Adam + soft update, and the PER tree update) runs on every rank.

With backend "nccl" (RCCL on ROCm) the collectives run over xGMI. The same code runs under
"gloo" for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(batch: int, world: int, rank: int):
    per = batch // world
    return rank * per, (rank + 1) * per


def dp_learn_step(engine, soft_update: bool = True, group=None, prefetch: bool = False):
    """One data-parallel learn step (+ soft target update) on `engine` (a LearnEngine built
    with world_size / rank).  Collectives are enqueued on the current stream.
    prefetch=True (pure learning loops, uniform replay): the shard's forward launch also draws the
    NEXT step's global minibatch (DQNX_STEP_PREFETCH), so the O(B_global) sampler leaves the
    critical path; a step with prefetch=False consumes the pending draw."""
    if prefetch:
        engine.learn_step(grads_only=True, prefetch=True)
    else:
        engine.learn_step(grads_only=True)
    exchange(engine, group)
    engine.apply_grads(soft_update=soft_update)


def exchange(engine, group=None):
    """The exchange step between the shard gradients and the optimizer."""
    dist.all_reduce(engine.grads, op=dist.ReduceOp.SUM, group=group)
    if engine.per_abs_td.numel():
        _gather_abs_td(engine, group)


def dp_learn_step_bucketed(engine, soft_update: bool = True, group=None, comm_stream=None, prefetch: bool = False):
    """The data-parallel step with per-layer gradient buckets.  The engine's backward completes the
    gradient in buckets (engine.dp_buckets()): conv nets -- dense layers + head + loss first, then
    each conv, last conv first; the fused MLP plan -- every gradient but layer 1's (one launch of
    dW tiles), then layer 1's.  Bucket b's all-reduce and its Adam run on `comm_stream` while the
    engine computes bucket b+1's backward on the current stream.  No parameter the remaining backward
    reads is updated early: a conv's data gradient reads the permuted weight copy made at the start
    of the step, dF was computed before bucket 0 closed, and the MLP's layer-1 dW tiles read only dZ_1
    and the gathered rows.  The kernels' per-element sums are dp_learn_step's; the all-reduce of a
    bucket sums each element in the order its ring chunking gives it, so at world > 2 an element may
    round differently than in the one-buffer all-reduce (an ulp; world 2 is bit-identical), while every
    rank still receives the same sum.  prefetch (MLP, uniform replay): as dp_learn_step's.

    On CPU tensors (gloo rehearsals) the buckets run in the same order on one thread."""
    buckets = engine.dp_buckets()
    cuda = engine.grads.is_cuda
    main = torch.cuda.current_stream(engine.grads.device) if cuda else None
    comm = (comm_stream or torch.cuda.Stream(engine.grads.device)) if cuda else None
    for b, (first, count) in enumerate(buckets):
        if prefetch and b == 0:
            engine.learn_step_bucket(b, prefetch=True)   # on the main stream
        else:
            engine.learn_step_bucket(b)
        if cuda:
            comm.wait_stream(main)
            ctx = torch.cuda.stream(comm)
        else:
            ctx = _nullctx()
        with ctx:
            dist.all_reduce(engine.grads[first:first + count], op=dist.ReduceOp.SUM, group=group)
            if b == 0 and engine.per_abs_td.numel():
                _gather_abs_td(engine, group)
            engine.apply_grads_bucket(b, soft_update=soft_update)
    if cuda:
        main.wait_stream(comm)


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _gather_abs_td(engine, group):
    world = engine.world_size
    b0, b1 = shard_bounds(engine.batch, world, engine.rank)
    parts = list(engine.per_abs_td.chunk(world))
    mine = engine.per_abs_td[b0:b1].clone()
    dist.all_gather(parts, mine, group=group)


CAPTURE_MODE = "thread_local"


def capture(graph):
    """torch.cuda.graph(graph) in "thread_local" capture mode -- the mode every capture of this package
    uses: the capture restricts only the capturing thread, not ProcessGroupNCCL's watchdog thread, which
    polls the events of eager collectives (hipEventQuery) every ~100 ms.

    Round 5 tested whether such a poll inside a capture explains round 4's two aborts of
    test_gpu_graphed_bucketed_dp_step (SIGABRT from WorkNCCL::finishedGPUExecutionInternal, a HIP error
    returned to the watchdog's event query).  tools/capture_watchdog_check.py holds an eager all-reduce's
    work incomplete in the watchdog's list across a capture held open for 0.6 s: in "global" and
    "thread_local" mode, with and without a captured collective on the same process group's stream, the
    process survives (gpurun_out r05a / r05k).  So the watchdog poll is not that cause;
    tests/test_gpu_dp.py::test_gpu_capture_tolerates_watchdog_polls keeps the condition covered."""
    return torch.cuda.graph(graph, capture_error_mode=CAPTURE_MODE)


class GraphedDPStep:
    """The whole data-parallel step -- the shard's learn kernels, the RCCL all-reduce (+ the
    PER |delta| all-gather), Adam + soft update -- captured once into one HIP graph
    (torch.cuda.CUDAGraph) and replayed: one host launch per step instead of a learn-graph
    launch, a collective call and an optimizer launch, so the GPU never waits on the host.

    The step state (RNG, ring size, Adam step, SumTree) lives on the device, so replays
    continue the same sequence of steps as eager dp_learn_step calls (transitions pushed in
    between are seen: the samplers read the ring size on the device).  Run at least one eager
    dp_learn_step first (communicator warm-up).  The engine's own per-step graphs are switched
    off: its kernels become nodes of this graph.
    """

    def __init__(self, engine, soft_update: bool = True, group=None, bucketed: bool = False, prefetch: bool = False,
                 steps: int = 1):
        """prefetch=True: capture the prefetching step (each replay computes on the minibatch the
        previous one drew and draws the next; see dp_learn_step).  The first draw is made here,
        before the capture; run one dp_learn_step(prefetch=False) after the last replay to
        consume the pending draw.
        steps: DP steps captured back to back into the one graph (a replay = `steps` steps).
        Every hipGraphLaunch leaves ~8.5 us before its first kernel on MI355X / ROCm 7.2; inside
        a graph consecutive kernels start back to back.
        Replays run on the caller's current stream; with prefetch each replay re-points the
        engine's pending-draw stream there (dqnx_prefetch_stream), so dqnx_rng_get waits on the
        stream that holds the draw."""
        self.steps = int(steps)
        self.engine = engine
        engine.set_graphs(False)
        self.graph = torch.cuda.CUDAGraph()
        self.comm = torch.cuda.Stream(engine.grads.device) if bucketed else None
        if prefetch:
            engine.prefetch_prologue()
        torch.cuda.synchronize()
        with capture(self.graph):
            for _ in range(self.steps):
                if bucketed:   # the side stream forks and joins inside the capture
                    dp_learn_step_bucketed(engine, soft_update=soft_update, group=group, comm_stream=self.comm,
                                           prefetch=prefetch)
                else:
                    dp_learn_step(engine, soft_update=soft_update, group=group, prefetch=prefetch)
        torch.cuda.synchronize()
        # the captured steps recorded torch's capture stream as the pending draw's stream; replays
        # run on the caller's current stream, which dqnx_rng_get must synchronise instead
        self._prefetch = prefetch

    def __call__(self):
        self.graph.replay()
        if self._prefetch:
            import ctypes
            from . import _capi as C
            C.check(C.lib().dqnx_prefetch_stream(self.engine.h, ctypes.c_void_p(
                torch.cuda.current_stream(self.engine.grads.device).cuda_stream)), "prefetch_stream")
