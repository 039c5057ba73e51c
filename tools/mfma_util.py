"""MFMA utilisation per kernel from a rocprofv3 --pmc pass of tools/pmc_groups_mfma.txt
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, ...) -> profiles/mfma_util_<name>.json.

Per dispatch (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy SIMD cycles summed
over every SIMD of the chip; GRBM_GUI_ACTIVE is the GPU-busy cycle count summed over the 8 XCDs):
  mfma_busy_frac       = MFMA_BUSY / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)   (busy share at the chip's own clock)
  mfma_busy_frac_2400  = MFMA_BUSY / (1024 SIMDs * duration * 2.4 GHz)    (against the nominal clock)
duration = the dispatch's own End - Start timestamps in the counter pass, or, when a kernel-trace
stats CSV of the same command is given, its AverageNs (counters serialise dispatches).
usage: python tools/mfma_util.py <pmc dir> <out.json> [kernel_stats.csv]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import bench_name  # noqa: E402

N_SIMD = 1024   # 256 CUs x 4 SIMDs


def main(root, out, stats=None):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            nm = bench_name(kn) or kn.split("(")[0].replace("void ", "")[:60]
            key = (nm, r.get("Grid_Size", ""))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            did = (f, r.get("Dispatch_Id"))
            if did not in seen and r.get("Start_Timestamp"):
                seen.add(did)
                durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    avg_ns, rows_of = {}, defaultdict(int)
    if stats:   # kernel-trace means, used only for names that map to ONE kernel at ONE grid size
        for r in csv.DictReader(open(stats)):
            nm = bench_name(r["Name"])
            if nm:
                avg_ns[nm] = float(r["AverageNs"])
                rows_of[nm] += 1
    grids_of = defaultdict(set)
    for (nm, grid) in vals:
        grids_of[nm].add(grid)
    avg_ns = {k: v for k, v in avg_ns.items() if rows_of[k] == 1 and len(grids_of[k]) == 1}
    res = {}
    for (nm, grid), cs in vals.items():
        d = {k: sum(v) / len(v) for k, v in cs.items()}
        e = {"grid": grid, "dispatches": max(len(v) for v in cs.values()), **{k + "_avg": v for k, v in d.items()}}
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES")
        if busy is not None:
            if d.get("GRBM_GUI_ACTIVE"):
                e["mfma_busy_frac"] = busy * 8.0 / (N_SIMD * d["GRBM_GUI_ACTIVE"])
            dur = avg_ns.get(nm, 0) * 1e-9 or (sum(durs[(nm, grid)]) / len(durs[(nm, grid)]) if durs[(nm, grid)] else 0)
            if dur > 0:
                e["duration_us"] = dur * 1e6
                e["duration_source"] = "kernel-trace AverageNs" if nm in avg_ns else "counter-pass timestamps"
                e["mfma_busy_frac_2400"] = busy / (N_SIMD * dur * 2.4e9)
        key = nm if nm not in res else f"{nm}@{grid}"
        res[key] = e
    res["_note"] = ("per-dispatch averages; mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                    "GRBM_GUI_ACTIVE / 8); mfma_busy_frac_2400 uses the duration at 2.4 GHz")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:])
