set -u
mkdir -p gpurun_out/hyb
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hybrid.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hyb/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/hyb/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do export DQNX_FWD_BIG=$m; export DQNX_CONV_DW_WGS=$((m*1024));
  DQNX_IM2COL=$m timeout -k 10 200 python bench.py --net hybrid --batch 256 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/hyb/h_$m.json 2>gpurun_out/hyb/h_$m.err || exit $?
  DQNX_IM2COL=$m timeout -k 10 300 python bench.py --net hybrid84 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hyb/h84_$m.json 2>gpurun_out/hyb/h84_$m.err || exit $?
done
python - <<'PY'
import json
for n in ("h_0","h_1","h84_0","h84_1"):
    d=json.load(open(f"gpurun_out/hyb/{n}.json"))
    ks={k["kernel"]:round(k["avg_us"],1) for k in d.get("kernels",[]) if "im2col" in k["kernel"] or "conv" in k["kernel"] or "linear_fwd" in k["kernel"] or "dx" in k["kernel"] or "col2im" in k["kernel"] or "adam" in k["kernel"] or "flatten" in k["kernel"]}
    print(n, round(d["value"]), round(d["ms_per_step"]*1e3,1), ks)
PY
