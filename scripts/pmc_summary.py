"""Summarise rocprofv3 counter-collection CSVs for the tube_step kernel (per-dispatch means)."""
import csv, glob, json, os, sys
from collections import defaultdict

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "tube_step_kernel"
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
out = {c: sum(v) / len(v) for c, v in vals.items()}
print(json.dumps(out, indent=1))
