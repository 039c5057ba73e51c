set -u
mkdir -p gpurun_out/h2
for k in 8192 1024; do
  DQNX_FWD_BIG_MINK=$k timeout -k 10 200 python bench.py --net hybrid --batch 256 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/h2/h_$k.json 2>gpurun_out/h2/h_$k.err || exit $?
  DQNX_FWD_BIG_MINK=$k timeout -k 10 200 python bench.py --net hybrid --batch 1024 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/h2/hb_$k.json 2>gpurun_out/h2/hb_$k.err || exit $?
done
python - <<'PY'
import json
for n in ("h_8192","h_1024","hb_8192","hb_1024"):
    d=json.load(open(f"gpurun_out/h2/{n}.json"))
    print(n, round(d["value"]), round(d["ms_per_step"]*1e3,1), {k["kernel"]:round(k["avg_us"],1) for k in d["kernels"] if "linear" in k["kernel"]})
PY
