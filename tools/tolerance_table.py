"""Measured deviation of the GPU's float results from the reference's own
fold orders (DESIGN.md "Float tolerance against the reference").

The GPU's f64 group-by sums and rolling sums are exact (the correctly
rounded sum of the values, bit-identical to the oracle's SUM_EXACT /
ROLLING_EXACT leg in every parity test), so their distance from the
reference is the reference's own rounding error, measured here against the
oracle's restatements of the reference's folds:

  kahan    polars-core/src/frame/group_by/aggregations/mod.rs:581 agg_sum
           (KahanSum per group, row order; polars-utils/src/kahan_sum.rs)
  naive    polars-expr/src/reduce/sum.rs:103 SumReducer (a left fold from
           +0.0, row order; one thread)
  morsel   the streaming engine's order: the same fold per morsel of
           100,000 rows, then the morsel partials folded in order
  window   polars-compute/src/rolling/sum.rs:7 SumWindow (Kahan add /
           subtract while sliding)

    python tools/tolerance_table.py [--rows-per-group 1500000] [--json out]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

MORSEL = 100_000


def datasets(n, rng):
    return {
        "same-sign (prices 10..490)": rng.uniform(10, 490, n),
        "mixed-sign (N(0, 100))": rng.standard_normal(n) * 100,
        "mixed-sign, 40 binades": rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n)),
    }


def ulps(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|a - b| in units of b's last place (b = the exact value)."""
    sp = np.spacing(np.abs(b))
    return np.abs(a - b) / np.where(sp > 0, sp, np.finfo(np.float64).tiny)


def morsel_fold(key, x, groups):
    out = {g: 0.0 for g in groups}
    for m0 in range(0, len(x), MORSEL):
        k, v = key[m0:m0 + MORSEL], x[m0:m0 + MORSEL]
        for g in groups:
            sel = v[k == g]
            if sel.size:
                out[g] = out[g] + float(np.add.accumulate(np.concatenate([[0.0], sel]))[-1])
    return np.array([out[g] for g in groups])


def group_rows(rows_per_group: int, ngroups: int = 4, seed: int = 7):
    rng = np.random.default_rng(seed)
    n = rows_per_group * ngroups
    key = rng.integers(0, ngroups, n).astype(np.int64)
    res = []
    for name, x in datasets(n, rng).items():
        k, kv, outs = None, None, {}
        for mode, tag in ((O.SUM_EXACT, "exact"), (O.SUM_KAHAN, "kahan"), (O.SUM_NAIVE, "naive")):
            k, kv, o = O.group_by_agg(O.HostCol(key), [O.HostCol(x)], [(4, 0, 1)], [("sum", 0), ("mean", 0)], n,
                                      mode)
            outs[tag] = (o[0][0], o[1][0])
        outs["morsel"] = (morsel_fold(key, x, list(k)), None)
        absum = np.array([np.abs(x[key == g]).sum() for g in k])
        ex_s, ex_m = outs["exact"]
        row = {"data": name, "rows_per_group": int(np.bincount(key).min())}
        for tag in ("kahan", "naive", "morsel"):
            s, m = outs[tag]
            row[f"sum_{tag}_ulp"] = float(ulps(s, ex_s).max())
            row[f"sum_{tag}_rel_abs"] = float((np.abs(s - ex_s) / absum).max())
            if m is not None:
                row[f"mean_{tag}_ulp"] = float(ulps(m, ex_m).max())
        res.append(row)
    return res


def rolling_rows(n: int = 1_000_000, seed: int = 11):
    rng = np.random.default_rng(seed)
    res = []
    for name, x in datasets(n, rng).items():
        for w in (3, 20, 200):
            hc = O.HostCol(x)
            ev, eok = O.rolling(hc, "sum", w, w, False, O.ROLLING_EXACT)
            rv, rok = O.rolling(hc, "sum", w, w, False, O.ROLLING_REFERENCE)
            e, r = ev[eok], rv[rok]
            mv, mok = O.rolling(O.HostCol(np.abs(x)), "sum", w, w, False, O.ROLLING_EXACT)
            mag = mv[mok]  # exact window sums of |x|
            res.append({"data": name, "window": w, "rows": n, "window_ulp": float(ulps(r, e).max()),
                        "window_rel_abs": float((np.abs(r - e) / mag).max())})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows-per-group", type=int, default=1_500_000)
    ap.add_argument("--rolling-rows", type=int, default=1_000_000)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    g = group_rows(args.rows_per_group)
    r = rolling_rows(args.rolling_rows)
    print("| data | rows/group | sum vs kahan ulp | vs naive ulp | vs morsel ulp | naive rel. to sum|x| | "
          "mean vs kahan ulp | mean vs naive ulp |")
    print("|---|---|---|---|---|---|---|---|")
    for x in g:
        print(f"| {x['data']} | {x['rows_per_group']:,} | {x['sum_kahan_ulp']:.3g} | {x['sum_naive_ulp']:.3g} | "
              f"{x['sum_morsel_ulp']:.3g} | {x['sum_naive_rel_abs']:.2e} | {x['mean_kahan_ulp']:.3g} | "
              f"{x['mean_naive_ulp']:.3g} |")
    print()
    print("| data | window | rolling sum vs SumWindow ulp | rel. to window sum|x| |")
    print("|---|---|---|---|")
    for x in r:
        print(f"| {x['data']} | {x['window']} | {x['window_ulp']:.3g} | {x['window_rel_abs']:.2e} |")
    if args.json:
        json.dump({"group_by": g, "rolling": r}, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
