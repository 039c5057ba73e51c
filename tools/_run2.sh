set -u
mkdir -p gpurun_out/r04j
export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1
timeout -k 10 120 python tools/stamps_fused.py 8192 bf16 > gpurun_out/r04j/stamps_8192_bf16.txt 2>&1 || { tail -5 gpurun_out/r04j/stamps_8192_bf16.txt; exit 1; }
grep "fwd total\|head_bwd total" gpurun_out/r04j/stamps_8192_bf16.txt | tail -4
timeout -k 10 120 python tools/stamps_fused.py 1024 > gpurun_out/r04j/stamps_1024.txt 2>&1 || { tail -5 gpurun_out/r04j/stamps_1024.txt; exit 1; }
tail -4 gpurun_out/r04j/stamps_1024.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04j/bench.json 2> gpurun_out/r04j/bench.err || { tail -5 gpurun_out/r04j/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r04j/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k in ('configs0','configs2','dropin_loop','head_net','configs4_projection_w8','projection_w8','configs3_n1'):
    v=d.get(k); print(k, json.dumps({kk:vv for kk,vv in (v or {}).items() if kk not in ('kernels','note')})[:700])
"
for mr in 4 2; do
  DQNX_FWD_MR=$mr timeout -k 10 240 python bench.py --algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r04j/c4_mr$mr.json 2> gpurun_out/r04j/c4_mr$mr.err || { tail -5 gpurun_out/r04j/c4_mr$mr.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r04j/c4_mr$mr.json').read().strip().splitlines()[-1])
print('mr=$mr', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], json.dumps(d.get('kernels_us', d.get('roofline',{}).get('kernels','')))[:600])
"
done
for v in base fnb3 fnb4fpf2 fnb3fpf2 fpf8; do
  lib=multimodal-drl-rmc_amd/dqn/_lib/var/libdqnx_$v.so; [ $v = base ] && lib=multimodal-drl-rmc_amd/dqn/_lib/libdqnx.so
  DQNX_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-extras --no-cpu-baseline > gpurun_out/r04j/var_$v.json 2> gpurun_out/r04j/var_$v.err || { tail -3 gpurun_out/r04j/var_$v.err; exit 1; }
  DQNX_LIB=$PWD/$lib timeout -k 10 200 python bench.py --algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 --steps 30 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/r04j/var_c4_$v.json 2> gpurun_out/r04j/var_c4_$v.err || { tail -3 gpurun_out/r04j/var_c4_$v.err; exit 1; }
  python -c "
import json
for f in ('var_$v','var_c4_$v'):
    d=json.loads(open('gpurun_out/r04j/'+f+'.json').read().strip().splitlines()[-1])
    print(f, round(d['ms_per_step']*1e3,2), [(k['kernel'],round(k['avg_us'],2)) for k in d.get('kernels',[])])
"
done
