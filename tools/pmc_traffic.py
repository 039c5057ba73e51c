"""Per-kernel HBM traffic per dispatch from rocprofv3 --pmc passes (tools/pmc.sh with
tools/pmc_traffic_groups.txt) -> profiles/pmc_traffic_<net>_b<batch>.json, read by bench.py's roofline.

hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, per MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KB) reads exactly half the bytes of a wide (16 B/lane) coalesced read on gfx950,
WRITE_SIZE (KB) is exact for 16-B stores.  Kernel names map to bench.py's step names."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

NAMES = [   # (substring of the HIP kernel name, bench step name); the first match wins
    # the HEAD net's micro-CNN plan (micro.hip) and its ELU dense layers
    ("k_micro_fwd", "micro_fwd"),
    ("k_micro_dx", "micro_dx"),
    ("k_micro_dw", "micro_dw"),
    ("k_linear_fwd_big<1, false, 64, 64, 2, 64>", "linear_fwd_l1"),
    ("k_linear_fwd<1, true, false>", "linear_fwd_l2"),
    ("k_bwd_level<1, true>", "linear_bwd_l2"),
    ("k_bwd_level<1, false>", "linear_bwd_l1"),
    ("k_mlp_fwd", "mlp_fwd"),
    ("k_head_bwd", "head_bwd"),
    ("k_linear_fwd<0, true, true>", "linear_fwd_l1"),
    ("k_linear_fwd<0, true, false>", "linear_fwd_l2"),
    ("k_sample_uniform", "sample_uniform"),
    ("k_head<", "head_td_loss"),
    ("k_bwd_level<", "dw_all"),
    ("k_dw_adam16", "dw_adam16"),
    ("k_dw_bf16", "dw_all"),
    ("k_adam", "adam_fused"),
    ("k_per_sample", "per_sample"),
    ("k_per_update", "per_update"),
    ("k_per_prep", "per_update_prep"),
    ("k_per_prop", "per_update_prop"),
    # (4,84,84) variant, implicit-GEMM convs (conv_ig.hip)
    ("k_conv_perm", "conv_perm"),
    ("k_conv_ig<4, 2, 4, true, 0, false>", "conv_fwd_c1"),
    ("k_conv_ig<8, 2, 2, false, 0, true>", "conv_fwd_c2"),
    ("k_conv_ig<4, 2, 2, false, 1, true>", "conv_fwd_c3"),
    ("k_conv_ig<4, 2, 2, false, 2, true>", "conv_dx_c3"),
    ("k_conv_ig<4, 2, 4, false, 2, true>", "conv_dx_c2"),
    ("k_conv_dw_ig<3, 2, false>", "conv_dw_c1"),
    ("k_unflatten_tiled", "unflatten"),
    ("k_linear_fwd_reduce", "linear_fwd_l1_reduce"),
    ("k_adam4", "adam_fused"),
]


# kernels launched more than once per step under one name: bench step names in dispatch order
CYCLES = [
    ("k_im2col_lds", ["im2col_c1", "im2col_c2", "im2col_c3"]),   # (4,84,84) variant
    ("k_linear_fwd_big<1, true, 128, 64", ["conv_fwd_c2", "conv_fwd_c3"]),   # explicit path
    ("k_conv_dw_ig<9, 4, true>", ["conv_dw_c3", "conv_dw_c2"]),              # implicit path, last conv first
]


def bench_name(kernel):
    for sub, nm in NAMES:
        if sub in kernel:
            return nm
    return None


def main(root="gpurun_out/pmc", out="profiles/pmc_traffic_mlp_b1024.json"):
    vals = defaultdict(lambda: defaultdict(list))   # bench name -> counter -> per-dispatch values
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        cyc = defaultdict(list)   # (cycle index, counter) -> rows
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            ci = next((i for i, (sub, _) in enumerate(CYCLES) if sub in kn), None)
            if ci is not None:
                cyc[(ci, r["Counter_Name"])].append(r)
                continue
            nm = bench_name(kn)
            if nm is None:
                continue
            vals[nm][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for (ci, cn), rows in cyc.items():
            names = CYCLES[ci][1]
            rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
            for i, r in enumerate(rows):
                vals[names[i % len(names)]][cn].append(float(r["Counter_Value"]))
    res = {}
    for nm, cs in vals.items():
        d = {k: sum(v) / len(v) for k, v in cs.items()}
        e = {"dispatches": max(len(v) for v in cs.values()), **{k + "_avg": v for k, v in d.items()}}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and d["TCC_HIT_sum"] + d["TCC_MISS_sum"] > 0:
            e["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        res[nm] = e
    res["_note"] = ("per-dispatch averages over every dispatch of the bench run (timed + timing steps); "
                    "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE half-count correction)")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:])
