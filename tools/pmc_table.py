"""Per-kernel table of PMC counters from tools/gpu_pmc.sh output (sums per
dispatch, averaged over dispatches).   python tools/pmc_table.py gpurun_out/TAG [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "k_"
vals = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    per = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(path)):
        key = (int(r["Dispatch_Id"]), r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        meta[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    for (d, c), v in per.items():
        vals[meta[d]][c].append(v)
for k, cs in vals.items():
    if filt not in k:
        continue
    print(k.replace("(anonymous namespace)::", "")[:90])
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v) / len(v):16.1f}")
