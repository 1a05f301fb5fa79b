"""Per-launch durations of the dominant kernel from a rocprofv3 --kernel-trace run of bench.py, the
warm-up launches excluded by index: the figure bench.py's roofline `achieved` is computed from (HIP events
around the same launches), reproducible from the committed trace.
usage: python scripts/trace_summary.py TRACE_DIR OUT.json --warmup W [--kernel tube_fast_kernel]
                                       [--batch B] [--algo-bytes BYTES_PER_LAUNCH]"""
import argparse
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("out")
ap.add_argument("--warmup", type=int, required=True)
ap.add_argument("--timed-last", type=int, default=0,
                help="take the LAST K launches as the timed ones (bench.py warms up until the clock is stable, "
                     "so the warm-up count varies; its timed steps are the last --steps launches)")
ap.add_argument("--kernel", default="fk::tube_fast_kernel")  # f32 (fk64:: is the f64 leg)
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--algo-bytes", type=float, default=274324.0 * 65536)
a = ap.parse_args()
rows = []
for f in glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if a.kernel in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:100]))
rows.sort()
d = [(e - s) * 1e-6 for s, e, _ in rows]  # ms
timed = d[-a.timed_last:] if a.timed_last > 0 else d[a.warmup:]
if a.timed_last > 0:
    a.warmup = len(d) - len(timed)
mean = sum(timed) / len(timed)
res = {"kernel": rows[0][2] if rows else a.kernel, "launches": len(d), "warmup_excluded": a.warmup,
       "timed_launches": len(timed), "mean_ms": mean, "min_ms": min(timed), "max_ms": max(timed),
       "per_launch_ms": [round(x, 5) for x in d], "batch": a.batch, "algo_bytes_per_launch": a.algo_bytes,
       "achieved_GBs": a.algo_bytes / (mean * 1e-3) / 1e9, "frac_of_8TBs": a.algo_bytes / (mean * 1e-3) / 8e12}
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "per_launch_ms"}))
