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
  pairwise polars-compute/src/float_sum.rs sum_arr_as_f64 (16-lane stripes,
           128-value pairwise blocks): the in-memory engine's keyless
           select(x.sum()) / x.mean() (ChunkAgg::sum, aggregate/mod.rs:68,94)
  welford  polars-compute/src/moment.rs VarState.insert_one per row
           (reduce/var_std.rs:89), one state per thread / morsel, combined:
           the streaming group-by's var / std
  chunked  moment.rs:641 var (VarState::new per 128 values, combined): the
           in-memory keyless x.var() / x.std()

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


def group_rows(rows_per_group: int, ngroups: int = 4, seed: int = 7, morsel: bool = True):
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
        if morsel:
            outs["morsel"] = (morsel_fold(key, x, list(k)), None)
        absum = np.array([np.abs(x[key == g]).sum() for g in k])
        ex_s, ex_m = outs["exact"]
        row = {"data": name, "rows_per_group": int(np.bincount(key).min())}
        for tag in ("kahan", "naive", "morsel"):
            if tag not in outs:
                continue
            s, m = outs[tag]
            row[f"sum_{tag}_ulp"] = float(ulps(s, ex_s).max())
            row[f"sum_{tag}_rel_abs"] = float((np.abs(s - ex_s) / absum).max())
            if m is not None:
                row[f"mean_{tag}_ulp"] = float(ulps(m, ex_m).max())
        res.append(row)
    return res


def keyless_rows(n: int = 6_000_000, seed: int = 5):
    """select(x.sum()) / select(x.mean()) over one chunk: the reference's
    pairwise float_sum against the exact sum the GPU returns (and the mean
    as that sum / count, each rounded once)."""
    rng = np.random.default_rng(seed)
    res = []
    for name, x in datasets(n, rng).items():
        ex = math.fsum(x)
        ref = O.float_sum(x)
        row = {"data": name, "rows": n,
               "sum_pairwise_ulp": float(ulps(np.array([ref]), np.array([ex]))[0]),
               "sum_pairwise_rel_abs": abs(ref - ex) / float(np.abs(x).sum()),
               "mean_pairwise_ulp": float(ulps(np.array([ref / n]), np.array([ex / n]))[0])}
        res.append(row)
    return res


def exact_var(x: np.ndarray, ddof: int = 1) -> float:
    """The exact variance of the stored values, rounded once: x as integers
    over their common lowest exponent, n * sum(x^2) - sum(x)^2 in Python
    integers, divided as a Fraction."""
    from fractions import Fraction

    m, e = np.frexp(x)
    mi = (m * 2.0 ** 53).astype(np.int64)  # exact: |m| in [0.5, 1)
    e = e.astype(np.int64) - 53
    lo = int(e.min())
    s1 = s2 = 0
    for a, b in zip(mi.tolist(), (e - lo).tolist()):
        v = a << b
        s1 += v
        s2 += v * v
    n = x.shape[0]
    num = n * s2 - s1 * s1
    return float(Fraction(num, n * (n - ddof)) * Fraction(2) ** (2 * lo))


def var_rows(n: int = 300_000, ngroups: int = 4, seed: int = 9):
    """var(ddof=1) per group (streaming Welford, one thread and per morsel)
    and keyless (chunked VarState) against the exact variance, which the
    GPU's fused pass returns within ~2 ULP (tests/test_gpu_var_std.py)."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, ngroups, n * ngroups)
    res = []
    sets = dict(datasets(n * ngroups, rng))
    sets["mean 1e6, spread 3 (prices)"] = 1e6 + rng.standard_normal(n * ngroups) * 3.0
    for name, x in sets.items():
        worst = {"welford": 0.0, "welford_morsel": 0.0}
        for g in range(ngroups):
            sel = np.nonzero(key == g)[0]
            xs = x[sel]
            ex = exact_var(xs)
            w1 = O.var_welford(xs)
            wm = O.var_welford(xs, sel // MORSEL)
            worst["welford"] = max(worst["welford"], float(ulps(np.array([w1]), np.array([ex]))[0]))
            worst["welford_morsel"] = max(worst["welford_morsel"], float(ulps(np.array([wm]), np.array([ex]))[0]))
        exk = exact_var(x)
        ck = O.var_chunked(x)
        res.append({"data": name, "rows_per_group": int(np.bincount(key).min()),
                    "var_welford_ulp": worst["welford"], "var_welford_morsel_ulp": worst["welford_morsel"],
                    "keyless_rows": int(x.shape[0]),
                    "var_keyless_chunked_ulp": float(ulps(np.array([ck]), np.array([exk]))[0])})
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
    ap.add_argument("--groups", type=int, default=4)
    ap.add_argument("--group-only", action="store_true",
                    help="only the group-by table (e.g. at configs[1]'s 1e8 rows: --rows-per-group 1000000 --groups 100)")
    args = ap.parse_args()
    g = group_rows(args.rows_per_group, args.groups, morsel=args.groups <= 4)
    if args.group_only:
        print("| data | rows/group | groups | sum vs kahan ulp | vs naive ulp | naive rel. to sum|x| | mean vs kahan ulp |")
        print("|---|---|---|---|---|---|---|")
        for x in g:
            print(f"| {x['data']} | {x['rows_per_group']:,} | {args.groups} | {x['sum_kahan_ulp']:.3g} | "
                  f"{x['sum_naive_ulp']:.3g} | {x['sum_naive_rel_abs']:.2e} | {x['mean_kahan_ulp']:.3g} |")
        if args.json:
            json.dump({"group_by": g, "groups": args.groups}, open(args.json, "w"), indent=1)
        return
    r = rolling_rows(args.rolling_rows)
    k = keyless_rows()
    v = var_rows()
    print("| data | rows/group | sum vs kahan ulp | vs naive ulp | vs morsel ulp | naive rel. to sum|x| | "
          "mean vs kahan ulp | mean vs naive ulp |")
    print("|---|---|---|---|---|---|---|---|")
    for x in g:
        print(f"| {x['data']} | {x['rows_per_group']:,} | {x['sum_kahan_ulp']:.3g} | {x['sum_naive_ulp']:.3g} | "
              f"{x.get('sum_morsel_ulp', float('nan')):.3g} | {x['sum_naive_rel_abs']:.2e} | {x['mean_kahan_ulp']:.3g} | "
              f"{x['mean_naive_ulp']:.3g} |")
    print()
    print("| data | window | rolling sum vs SumWindow ulp | rel. to window sum|x| |")
    print("|---|---|---|---|")
    for x in r:
        print(f"| {x['data']} | {x['window']} | {x['window_ulp']:.3g} | {x['window_rel_abs']:.2e} |")
    print()
    print("| data | rows | select sum vs pairwise float_sum ulp | rel. to sum|x| | select mean ulp |")
    print("|---|---|---|---|---|")
    for x in k:
        print(f"| {x['data']} | {x['rows']:,} | {x['sum_pairwise_ulp']:.3g} | {x['sum_pairwise_rel_abs']:.2e} | "
              f"{x['mean_pairwise_ulp']:.3g} |")
    print()
    print("| data | rows/group | group var vs Welford ulp (one thread) | per morsel | keyless var vs chunked ulp |")
    print("|---|---|---|---|---|")
    for x in v:
        print(f"| {x['data']} | {x['rows_per_group']:,} | {x['var_welford_ulp']:.3g} | "
              f"{x['var_welford_morsel_ulp']:.3g} | {x['var_keyless_chunked_ulp']:.3g} |")
    if args.json:
        json.dump({"group_by": g, "rolling": r, "keyless": k, "var": v}, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
