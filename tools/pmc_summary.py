"""Summarise rocprofv3 --pmc passes (tools/pmc.sh): mean counter value per dispatch for each
libdqnx kernel, plus its VGPR / AGPR / LDS / scratch allocation."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(list)
info = {}
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "dqnx" not in k or "push" in k:
            continue
        name = k.split("(")[0].replace("void ", "").replace("dqnx::", "")
        vals[(name, row["Counter_Name"])].append(float(row["Counter_Value"]))
        info[name] = (row["VGPR_Count"], row["Accum_VGPR_Count"], row["SGPR_Count"], row["LDS_Block_Size"],
                      row["Scratch_Size"], row["Grid_Size"], row["Workgroup_Size"])
names = sorted({n for n, _ in vals})
for n in names:
    v, a, sg, lds, scr, grid, wg = info[n]
    print(f"{n}: vgpr {v} agpr {a} sgpr {sg} lds {lds} scratch {scr} grid {grid} wg {wg}")
    for (nn, c), xs in sorted(vals.items()):
        if nn == n:
            print(f"    {c:32s} {sum(xs) / len(xs):14.1f}  (n={len(xs)})")
