#!/bin/bash
# World-1 RCCL rehearsals of the N > 1 path on a one-GPU box: graphed / prefetching DP steps vs eager
# (bitwise), then bench.py's DP code path (process group, GraphedDPStep over RCCL, 4 steps per
# replay, prefetch) at world size 1 with the configs[3] global minibatch.
set -u
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
MASTER_PORT=29611 timeout -k 10 300 python tools/dp_graph_check.py DuelingDoubleDQNAgent 512 > gpurun_out/dpg.log 2>&1 || { tail -5 gpurun_out/dpg.log; exit 1; }
tail -1 gpurun_out/dpg.log
DQNX_BENCH_FORCE_DP=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 \
    bench.py --gpus 1 --steps 200 --warmup 20 --no-extras > gpurun_out/dp1_bench.json 2> gpurun_out/dp1_bench.err || { tail -5 gpurun_out/dp1_bench.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/dp1_bench.json').read().strip().splitlines()[-1])
print('force-dp world1', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us', d['config']['dp_step'], d['config']['batch_per_gpu'], [(k['kernel'],round(k['avg_us'],2)) for k in d['kernels']])"
DQNX_BENCH_FORCE_DP=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29615 \
    bench.py --gpus 1 --steps 200 --warmup 20 --no-extras --no-kernel-timing --dp-graph-steps 1 > gpurun_out/dp1_bench_g1.json 2> gpurun_out/dp1_bench_g1.err || { tail -5 gpurun_out/dp1_bench_g1.err; exit 1; }
python -c "
import json
d=json.loads(open('gpurun_out/dp1_bench_g1.json').read().strip().splitlines()[-1])
print('force-dp world1, 1 step per graph', round(d['value']/1e6,2), 'M tr/s', round(d['ms_per_step']*1e3,2), 'us')"
