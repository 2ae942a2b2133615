"""Cross-check a bench line against the rocprofv3 runs of the same lease
(tools/bench_profile.sh output):

    python tools/bench_evidence.py gpurun_out/<tag> [--out profiles/<name>]

For every leg's roofline kernel (headline gb_fast_kernel, vwap / std legs,
sort: aos_gather_kernel, join: jn_probe_match_kernel) it reports
  - kernel_ms of the plain bench line (HIP events, bench.json),
  - kernel_ms of the profiled run's own line (trace.json),
  - the rocprofv3 kernel-trace mean of the same launches (trace/),
  - frac recomputed from the trace mean at the line's algorithmic bytes,
    and its distance from the line's frac,
  - HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes (pmc1 /
    pmc2; KiB; FETCH_SIZE doubled for the wide streaming kernels per
    MI355X_MICROARCH.md "HBM", raw for random-access kernels, whose
    correction is uncalibrated),
and checks that no kernel mean exceeds its step.  With --out it writes
<out>.json and <out>.md, and profiles/traffic.json for the headline.
"""
import argparse
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

HBM_PEAK = 8000.0

# leg -> (kernel-name regex over the trace, algorithmic bytes / launch key, streaming?)
# gb_fast_kernel's last two template arguments: VAR (0 none, 1 the variance
# triple, 2 / 3 the product pair) and PACK (0: a key column,
# 1: integer key columns packed in the kernel, 2: String key codes).  The
# keys leg runs its Categorical case and then its (symbol, day) case on the
# PACK = 1 variant with equal launch counts: "first" / "second" half of that
# kernel's launches in trace order.
LEGS = {
    "headline": (r"gb_fast_kernel<4, 1, true, 2, 2, false, false, false, [05], 0, false>", "headline", True),
    "vwap": (r"gb_fast_kernel<2, 1, true, 2, 2, false, false, false, 2, 0, false>", "vwap", True),
    "std": (r"gb_fast_kernel<3, 1, true, 2, 2, false, false, false, [14], 0, false>", "std", True),
    "keys_categorical": (r"gb_fast_kernel<4, 1, true, 2, 2, false, false, false, [05], 1, false>", "keys_categorical",
                         ("first", True)),
    "keys_string": (r"gb_fast_kernel<4, 1, true, 2, 2, false, false, false, [05], 2, false>", "keys_string", True),
    "keys_sym_day": (r"gb_fast_kernel<4, 1, true, 2, 2, false, false, false, [05], 1, false>", "keys_sym_day",
                     ("second", True)),
    "sort": (r"aos_gather_kernel<8>", "sort", False),
    "sort_pack": (r"aos_pack_kernel<8>", "sort_pack", True),
    "rolling": (r"rl_wave_kernel<4, false, false>", "rolling", True),
    "join": (r"rj_match_kernel<", "join", False),
    "join_emit": (r"jn_take_emit_kernel<2, 1>", "join_emit", True),
    "filter": (r"filter_(scatter8|fused8)_kernel", "filter", True),
    "filter_mask": (r"filter_mask_kernel", "filter_mask", True),
}

# many_groups leg, largest G: its kernels run once or twice per step (one
# launch per scatter level, each level its own template instance); the
# line's kernel_ms is the per-step sum, so the trace side is the sum over
# the kernel's instances of the mean of their last timed launches.  No other
# leg launches these instances.
# (null-free instances only: the nulls leg runs the NUL = true ones; the
# partitioned join runs <0, false, true, false>, the keyless-predicate form)
MG_KERNELS = {"count": r"gbp_count_kernel<(1, false|0, true), true, false>",
              "scatter": r"gbp_scatter_kernel<(1, false|0, true), true, false>",
              "aggregate": r"gb_fast_kernel<\d+, 0, true, 2, 2, (true|false), true, false, 0, 0, false>"}


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def line_view(d):
    """leg -> (kernel_ms, algorithmic bytes per launch, step ms, line frac)."""
    out = {}
    r = d["roofline"]
    rows = d["config"]["rows_per_gpu"]
    out["headline"] = (r["kernel_ms"], r["bytes_per_row"] * rows, d["ms_per_step"], r["frac"])
    for leg in ("vwap", "std"):
        if leg in d:
            L = d[leg]
            out[leg] = (L["kernel_ms"], L["bytes_per_row"] * L["rows"], L["ms_per_step"], L["frac"])
    if "sort" in d:
        L = d["sort"]
        for key, sub in (("sort", L["roofline"]), ("sort_pack", L["pack"]), ("rolling", L["rolling"])):
            if sub.get("kernel_ms"):
                out[key] = (sub["kernel_ms"], sub["algorithmic_GB"] * 1e9, L["ms_per_step"], sub["frac"])
    rows = d["config"]["rows_per_gpu"]
    for case in ("categorical", "string", "sym_day"):
        K = d.get("keys", {}).get(case)
        if K and K.get("kernel_ms"):
            out["keys_" + case] = (K["kernel_ms"], K["bytes_per_row"] * rows, K["ms_per_step"], K["frac"])
    if "join" in d:
        L = d["join"]
        for key, sub in (("join", L["roofline"]), ("join_emit", L["emit"])):
            if sub.get("kernel_ms"):
                out[key] = (sub["kernel_ms"], sub["algorithmic_GB"] * 1e9, L["ms_per_step"], sub["frac"])
    if "filter" in d:
        L = d["filter"]
        for key, sub in (("filter", L["roofline"]), ("filter_mask", L.get("mask"))):
            if sub and sub.get("kernel_ms"):
                out[key] = (sub["kernel_ms"], sub["algorithmic_GB"] * 1e9, L["ms_per_step"], sub["frac"])
    return out


def mg_view(d):
    """many_groups, largest G -> {part: (per-step kernel ms, algorithmic bytes, step ms, frac, launches/step)}."""
    mg = d.get("many_groups") or {}
    gs = [int(g) for g in mg if g.isdigit()]
    if not gs:
        return None, {}
    g = str(max(gs))
    L = mg[g]
    out = {}
    for part in MG_KERNELS:
        sub = L.get(part) or {}
        if sub.get("kernel_ms"):
            out[part] = (sub["kernel_ms"], sub["algorithmic_GB"] * 1e9, L["ms_per_step"], sub["frac"])
    return g, out


def trace_durations(path):
    dur = defaultdict(list)
    for r in csv.DictReader(open(path)):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return dur


def pick(table, pattern):
    rx = re.compile(pattern)
    vals = []
    names = []
    for name, v in table.items():
        if rx.search(name):
            vals += v
            names.append(name)
    return vals, names


def counters(path):
    c = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        c[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    d = args.dir
    plain = last_json(os.path.join(d, "bench.json"))
    prof = last_json(os.path.join(d, "trace.json"))
    lp, lq = line_view(plain), line_view(prof)
    tr = trace_durations(os.path.join(d, "trace", "run_kernel_trace.csv"))
    fetch = counters(os.path.join(d, "pmc1", "run_counter_collection.csv"))
    write = counters(os.path.join(d, "pmc2", "run_counter_collection.csv"))
    rows = []
    for leg, (pat, _, streaming) in LEGS.items():
        if leg not in lp:
            continue
        half = None
        if isinstance(streaming, tuple):
            half, streaming = streaming
        k_plain, algo, step_plain, frac_plain = lp[leg]
        k_prof = lq.get(leg, (None,) * 4)[0]
        step_prof = lq.get(leg, (None,) * 4)[2]
        durs, names = pick(tr, pat)
        if half:
            durs = durs[: len(durs) // 2] if half == "first" else durs[len(durs) // 2:]
        # the profiled run's timed launches are the last ones of the leg
        # (warmup launches come first); the mean over all of them is reported too
        tmean = statistics.mean(durs) if durs else None
        fvals, _ = pick({k: v["FETCH_SIZE"] for k, v in fetch.items() if "FETCH_SIZE" in v}, pat)
        wvals, _ = pick({k: v["WRITE_SIZE"] for k, v in write.items() if "WRITE_SIZE" in v}, pat)
        if half:
            fvals = fvals[: len(fvals) // 2] if half == "first" else fvals[len(fvals) // 2:]
            wvals = wvals[: len(wvals) // 2] if half == "first" else wvals[len(wvals) // 2:]
        rd = statistics.mean(fvals) * 1024 * (2 if streaming else 1) if fvals else None
        wr = statistics.mean(wvals) * 1024 if wvals else None
        row = {
            "leg": leg, "kernel": names[0] if names else pat, "launches_traced": len(durs),
            "algorithmic_bytes": algo,
            "line_kernel_ms": k_plain, "line_frac": frac_plain, "line_step_ms": step_plain,
            "profiled_line_kernel_ms": k_prof, "profiled_step_ms": step_prof,
            "trace_mean_ms": round(tmean, 4) if tmean else None,
            "trace_frac": round(algo / (tmean * 1e-3) / 1e9 / HBM_PEAK, 4) if tmean else None,
            "hbm_read_bytes": rd, "hbm_write_bytes": wr,
            "read_correction": "FETCH_SIZE x 2 (wide streaming reads, gfx950)" if streaming
            else "FETCH_SIZE raw (random access: uncalibrated)",
        }
        if tmean:
            row["trace_vs_line_pct"] = round(100 * (tmean - k_plain) / k_plain, 2)
            row["trace_vs_profiled_line_pct"] = round(100 * (tmean - k_prof) / k_prof, 2) if k_prof else None
            row["frac_diff_pct"] = round(100 * (row["trace_frac"] - frac_plain) / frac_plain, 2)
            row["kernel_mean_within_step"] = tmean <= (step_prof or step_plain) and k_plain <= step_plain
        if rd is not None and wr is not None:
            row["hbm_bytes_per_launch"] = rd + wr
            row["traffic_over_algorithmic"] = round((rd + wr) / algo, 4)
        rows.append(row)
    g, mgp = mg_view(plain)
    _, mgq = mg_view(prof)
    steps = None
    if g:
        L = plain["many_groups"][g]
        steps = max(1, L["kernels"].get("gb_finalize_kernel", {}).get("launches", 2))
    for part, (pat, streaming) in ((k, (v, True)) for k, v in MG_KERNELS.items()):
        if part not in mgp:
            continue
        k_plain, algo, step_plain, frac_plain = mgp[part]
        k_prof = mgq.get(part, (None,) * 4)[0]
        rx = re.compile(pat)
        tsum = fsum = wsum = 0.0
        names = []
        for name, v in tr.items():
            if rx.search(name) and v:
                names.append(name)
                tsum += statistics.mean(v[-steps:])
                fv = fetch.get(name, {}).get("FETCH_SIZE", [])
                wv = write.get(name, {}).get("WRITE_SIZE", [])
                fsum += statistics.mean(fv[-steps:]) * 1024 * 2 if fv else 0.0
                wsum += statistics.mean(wv[-steps:]) * 1024 if wv else 0.0
        if not names:
            continue
        row = {"leg": f"many_groups_{g}_{part}", "kernel": " + ".join(n.split("(")[0] for n in names),
               "launches_traced": steps, "algorithmic_bytes": algo, "line_kernel_ms": k_plain,
               "line_frac": frac_plain, "line_step_ms": step_plain, "profiled_line_kernel_ms": k_prof,
               "trace_mean_ms": round(tsum, 4), "trace_frac": round(algo / (tsum * 1e-3) / 1e9 / HBM_PEAK, 4),
               "hbm_read_bytes": fsum, "hbm_write_bytes": wsum,
               "read_correction": "FETCH_SIZE x 2 (wide streaming reads, gfx950); per step: sum over the "
                                  "kernel's instances of the mean of their last timed launches"}
        row["trace_vs_line_pct"] = round(100 * (tsum - k_plain) / k_plain, 2)
        row["trace_vs_profiled_line_pct"] = round(100 * (tsum - k_prof) / k_prof, 2) if k_prof else None
        row["frac_diff_pct"] = round(100 * (row["trace_frac"] - frac_plain) / frac_plain, 2)
        row["kernel_mean_within_step"] = tsum <= step_plain
        row["hbm_bytes_per_launch"] = fsum + wsum
        row["traffic_over_algorithmic"] = round((fsum + wsum) / algo, 4)
        rows.append(row)
    hdr = ("| leg | kernel | line kernel ms (HIP events) | trace mean ms | trace vs line | profiled run's line ms "
           "| trace vs profiled line | line frac | trace frac | HBM bytes / launch (PMC) | / algorithmic | mean <= step |")
    md = [f"Bench evidence from `{d}` (plain run, then the same command under rocprofv3 in the same lease).  "
          "The profiled run's own line (HIP events of the traced launches) checks the timer; the plain line "
          "checks run-to-run agreement.", "",
          hdr, "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        md.append(f"| {r['leg']} | `{r['kernel'][:70]}` | {r['line_kernel_ms']} | {r['trace_mean_ms']} | "
                  f"{r.get('trace_vs_line_pct')} % | {r.get('profiled_line_kernel_ms')} | "
                  f"{r.get('trace_vs_profiled_line_pct')} % | {r['line_frac']} | {r['trace_frac']} | "
                  f"{(r.get('hbm_bytes_per_launch') or 0) / 1e9:.3f} GB | {r.get('traffic_over_algorithmic')} | "
                  f"{r.get('kernel_mean_within_step')} |")
    print("\n".join(md))
    if args.out:
        json.dump({"dir": d, "plain_line": {"value": plain["value"], "ms_per_step": plain["ms_per_step"]},
                   "legs": rows}, open(args.out + ".json", "w"), indent=1)
        open(args.out + ".md", "w").write("\n".join(md) + "\n")
        h = next((r for r in rows if r["leg"] == "headline"), None)
        if h and h.get("hbm_bytes_per_launch"):
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            json.dump({"rows": plain["config"]["rows_per_gpu"], "kernel": h["kernel"],
                       "hbm_bytes_per_launch": h["hbm_bytes_per_launch"], "correction": h["read_correction"],
                       "duration_ms": h["trace_mean_ms"], "source": args.out + ".json"},
                      open(os.path.join(root, "profiles", "traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
