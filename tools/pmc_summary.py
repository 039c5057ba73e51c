"""Per-kernel averages of rocprofv3 --pmc counters (any groups), keyed by kernel name and grid
size (launches of one template at different shapes stay apart).
usage: python tools/pmc_summary.py gpurun_out/pmcX [filter-substring]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(dqnx::[A-Za-z]*Args\).*$", "", name).replace("void ", "")
    return name.replace("dqnx::", "").replace("(anonymous namespace)::", "")


def main(root, filt=""):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if filt and filt not in kn:
                continue
            key = (short(kn), r.get("Grid_Size", r.get("Grid_Size_X", "")))
            vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key in sorted(vals):
        cs = vals[key]
        n = max(len(v) for v in cs.values())
        print(f"{key[0]}  grid={key[1]}  dispatches~{n}")
        for c in sorted(cs):
            v = cs[c]
            print(f"    {c:32s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
