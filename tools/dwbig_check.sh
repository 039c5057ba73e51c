set -u
mkdir -p gpurun_out/dw
timeout -k 10 300 python -u -m pytest tests/test_gpu_hybrid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dw/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/dw/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  DQNX_CONV_DW_BIG=$m timeout -k 10 200 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dw/h84_$m.json 2>/dev/null || exit $?
done
python -c "
import json
for n in ('h84_0','h84_1'):
    d=json.load(open(f'gpurun_out/dw/{n}.json'))
    print(n, round(d['value']), round(d['ms_per_step']*1e3,1), {k['kernel']:round(k['avg_us'],1) for k in d['kernels'] if 'bwd' in k['kernel'] or 'dx' in k['kernel'] or 'adam' in k['kernel']})
"
