"""Summarise a scripts/prof_pmc.sh output directory into the JSON bench.py reads (profiles/*pmc*.json).

usage: python scripts/pmc_summary.py gpurun_out/prof_TAG OUT.json [--batch B]

Per-dispatch means of every counter for the tube-step kernel (tube_fast_kernel, the specialised paper
configuration, or the generic tube_step_kernel -- whichever the bench launched), plus the HBM bytes per launch:
  raw = FETCH_SIZE + WRITE_SIZE (KiB -> bytes), and the calibrated figure, where FETCH / WRITE are each
  divided by the ratio measured/known on the known-byte launch of scripts/pmc_calib.py (the tube kernel's
  16-byte / 8-byte per-lane record pattern through one buffer resource, past the Infinity Cache).
  MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reads 1/2 of wide 16-B/lane streams; other widths must be
  calibrated -- this does it for ours.
The summary records the sha256 of the library the passes ran (bench.py refuses a summary of another
build for its roofline `traffic` field)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


# the f32 headline kernel only: dtmpc::fk:: (the f64 instantiation is dtmpc::fk64::, the generic f64 one
# tube_step_kernel<double>; a default bench run launches both in its secondary legs)
TUBE_KERNELS = ("fk::tube_fast_kernel", "tube_step_kernel<float")


def _match(name, kern):
    return any(k in name for k in kern) if isinstance(kern, tuple) else kern in name


SKIP = 0  # --skip N: drop each pass's first N dispatches of the kernel (a leg's warm-up launch of another size)


def counters(root, kern, sub="*"):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, sub, "run_counter_collection.csv")) + \
            glob.glob(os.path.join(root, sub, "*", "run_counter_collection.csv")):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if not _match(r["Kernel_Name"], kern):
                continue
            per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        keep = sorted({d for d, _ in per})[SKIP:]
        for (d, c), v in per.items():
            if d in keep:
                vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}


def kernel_stats(root, kern):
    for f in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if _match(r["Name"], kern):
                return {"name": r["Name"][:120], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                        "max_ns": float(r["MaxNs"])}
    return None


def main():
    global SKIP
    root, out = sys.argv[1], sys.argv[2]
    SKIP = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 65536
    # --kernel SUBSTR / --workload NAME: another kernel of the run, e.g. the f64 leg (fk64::tube_fast_kernel,
    # workload tube_f64: bench.py's tube_f64 roofline reads it; its record loads are all 16 B per lane, the
    # width the calibration launch's reads mostly have)
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else TUBE_KERNELS
    workload = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "tube"
    tube = {k: v for sub in ("fetch", "write", "sq1", "sq2", "tcc") for k, v in counters(root, kern, sub).items()}
    cal_f = counters(root, "record_stream_kernel", "cal_fetch")
    cal_w = counters(root, "record_stream_kernel", "cal_write")
    N = 50
    Bc = 262144
    known_r = known_w = Bc * ((N + 1) * 16 + N * 8)
    ks = kernel_stats(root, kern)
    import hashlib

    lib = os.environ.get("DTMPC_LIBRARY") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "differentiable-tube-mpc_amd", "diff_tube_mpc_strict_pt",
                                                          "libdtmpc.so")
    res = {"kernel": (ks or {}).get("name", "tube step") + " (7 alphas: 6 rolled out + alpha = 0 from the current tape)",
           "workload": workload, "batch": batch, "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "counters_per_dispatch": tube, "kernel_trace": ks}
    if "FETCH_SIZE" in tube and "WRITE_SIZE" in tube:
        raw = 1024.0 * (tube["FETCH_SIZE"] + tube["WRITE_SIZE"])
        res["tube_step_bytes_raw"] = raw
        res["tube_step_bytes_per_launch"] = raw
        if cal_f.get("FETCH_SIZE") and cal_w.get("WRITE_SIZE"):
            rf = 1024.0 * cal_f["FETCH_SIZE"] / known_r
            rw = 1024.0 * cal_w["WRITE_SIZE"] / known_w
            res["calibration"] = {"kernel": "record_stream_kernel", "batch": Bc, "known_read_bytes": known_r,
                                  "known_write_bytes": known_w, "fetch_measured_over_known": rf,
                                  "write_measured_over_known": rw}
            res["tube_step_bytes_per_launch"] = 1024.0 * (tube["FETCH_SIZE"] / rf + tube["WRITE_SIZE"] / rw)
            res["tube_step_read_bytes"] = 1024.0 * tube["FETCH_SIZE"] / rf
            res["tube_step_write_bytes"] = 1024.0 * tube["WRITE_SIZE"] / rw
        # round 5: every leg's kernel (tube step, standalone iLQR, receding driver) under one key
        res["kernel_bytes_per_launch"] = res["tube_step_bytes_per_launch"]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
