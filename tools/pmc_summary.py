"""Summarise a tools/profile_bench.sh output directory for one kernel.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring] [rows]

Prints per-launch averages of every collected counter, the kernel's mean
duration from the trace, and HBM traffic per launch with the gfx950
FETCH_SIZE correction (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the
bytes of a wide coalesced read; both counters are in KiB).  With `rows`, also
writes <dir>/traffic.json for bench.py.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "gb_kernel"
rows = int(float(sys.argv[3])) if len(sys.argv) > 3 else None
vals = defaultdict(list)
for f in glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = []
for f in glob.glob(os.path.join(d, "trace", "run_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {k: statistics.mean(v) for k, v in sorted(vals.items())}
for k, v in out.items():
    print(f"{k:28s} {v:16.4g}")
if dur:
    print(f"{'duration_ms (trace, mean)':28s} {statistics.mean(dur):16.4f}  n={len(dur)}")
if "FETCH_SIZE" in out:
    rd = out["FETCH_SIZE"] * 1024 * 2
    wr = out.get("WRITE_SIZE", 0.0) * 1024
    print(f"{'HBM read bytes (x2 corr.)':28s} {rd:16.4g}")
    print(f"{'HBM write bytes':28s} {wr:16.4g}")
    if rows:
        t = {"rows": rows, "kernel": kern, "hbm_bytes_per_launch": rd + wr, "fetch_kib": out["FETCH_SIZE"],
             "write_kib": out.get("WRITE_SIZE", 0.0), "correction": "FETCH_SIZE x2 (gfx950, 16B/lane reads)",
             "duration_ms": statistics.mean(dur) if dur else None}
        json.dump(t, open(os.path.join(d, "traffic.json"), "w"), indent=1)
if "SQ_WAVE_CYCLES" in out:
    w = out["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_ANY"):
        if k in out:
            print(f"{k + ' / WAVE_CYCLES':40s} {out[k] / w:8.3f}")
