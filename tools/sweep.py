"""GPU-box sweep: for each libdqnx variant run bench (value) and a rocprofv3 kernel trace."""
import csv, collections, glob, json, os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out", "sweep")
os.makedirs(OUT, exist_ok=True)
libs = sorted(glob.glob(os.path.join(REPO, "multimodal-drl-rmc_amd/dqn/_lib/var/libdqnx_*.so")))
extra = sys.argv[1:]
summary = []
# optional runtime knobs: SWEEP_ENVS="tag:K=V,K2=V2;tag2:K=V" crosses every library with every set
envsets = [("", {})]
if os.environ.get("SWEEP_ENVS"):
    envsets = []
    for item in os.environ["SWEEP_ENVS"].split(";"):
        tag, _, kv = item.partition(":")
        envsets.append((tag, dict(p.split("=", 1) for p in kv.split(",") if p)))
runs = [(lib, tag, ev) for lib in libs for tag, ev in envsets]
for lib, tag, ev in runs:
    name = os.path.basename(lib)[8:-3] + (("+" + tag) if tag else "")
    env = dict(os.environ, DQNX_LIB=lib, **ev)
    r = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline",
                        "--no-kernel-timing", "--steps", "400"] + extra, env=env, capture_output=True, text=True)
    if r.returncode != 0:
        print(name, "bench failed rc", r.returncode, r.stderr[-500:], flush=True)
        if r.returncode >= 124: sys.exit(r.returncode)
        continue
    val = json.loads(r.stdout.strip().splitlines()[-1])
    d = os.path.join(OUT, name)
    r2 = subprocess.run(["timeout", "-k", "10", "240", "rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d,
                         "-o", "run", "--", sys.executable, os.path.join(REPO, "bench.py"), "--no-cpu-baseline",
                         "--no-kernel-timing", "--steps", "100", "--warmup", "10"] + extra,
                        env=env, capture_output=True, text=True)
    ks = {}
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if r2.returncode == 0 and tr:
        dd = collections.defaultdict(list)
        for row in csv.DictReader(open(tr[0])):
            if "dqnx" not in row["Kernel_Name"] or "push" in row["Kernel_Name"]:
                continue
            key = row["Kernel_Name"].split("(")[0].split("::")[-1][:24] + "/" + row["Grid_Size_X"]
            dd[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
        for k, v in dd.items():
            v.sort()
            ks[k] = round(v[len(v) // 2], 2)
    elif r2.returncode >= 124:
        print(name, "rocprof rc", r2.returncode, flush=True); sys.exit(r2.returncode)
    line = {"variant": name, "Mtr_s": round(val["value"] / 1e6, 3), "us_step": round(val["ms_per_step"] * 1e3, 2), "kernels_us": ks}
    summary.append(line)
    print(json.dumps(line), flush=True)
json.dump(summary, open(os.path.join(OUT, "summary.json"), "w"), indent=1)
