"""CPU: pin the oracle (oracle/polars_oracle.c) before trusting it.

* against the golden fixtures transcribed from the reference's own tests;
* the exact-sum leg against CPython's math.fsum;
* the Kahan leg (the reference's GroupByExec fold) within 1 ULP of exact on
  same-sign data, the naive leg (the streaming reducer) within Higham's
  bound gamma_{n-1} * sum|x|.
"""

import math

import numpy as np
import pytest

from conftest import check_rolling_case, load_golden, unhex
from oracle import oracle as O

OPS = dict(eq=20, ne=21, lt=22, le=23, gt=24, ge=25, eq_missing=26, ne_missing=27)


def _fcol(vals):
    valid = np.array([v is not None for v in vals], dtype=bool)
    arr = np.array([0.0 if v is None else v for v in vals], dtype=np.float64)
    return O.HostCol(arr, None if valid.all() else valid)


def test_compare_truth_table_scalar_and_column():
    g = load_golden("compare_total_order.json")
    assert len(g["cases"]) == 81
    for case in g["cases"]:
        lhs, rhs = unhex(case["lhs"]), unhex(case["rhs"])
        lcol = _fcol([lhs, 0.0])
        rcol = _fcol([rhs, 0.0])
        for opname, exp in case["expected"].items():
            # column vs column
            dt, v, valid = O.eval_program([lcol, rcol], [(1, 0, 0), (1, 1, 0), (OPS[opname], 0, 0)], 2)
            got = bool(v[0]) if valid[0] else None
            assert got == exp, (lhs, rhs, opname)
            # column vs scalar literal (pl.col("l") <op> rhs)
            lit = (5, 4, 0) if rhs is None else (2, 0, rhs)
            dt, v, valid = O.eval_program([lcol], [(1, 0, 0), lit, (OPS[opname], 0, 0)], 2)
            got = bool(v[0]) if valid[0] else None
            assert got == exp, (lhs, rhs, opname, "scalar")


def _case_cols(case):
    cols, names = [], []
    for name, spec in case["cols"].items():
        vals = unhex(spec["values"]) if spec["dtype"] == "f64" else spec["values"]
        valid = np.array([v is not None for v in vals], dtype=bool)
        dt = np.float64 if spec["dtype"] == "f64" else np.int64
        fill = 0.0 if dt is np.float64 else 0
        arr = np.array([fill if v is None else v for v in vals], dtype=dt)
        cols.append(O.HostCol(arr, None if valid.all() else valid))
        names.append(name)
    return cols, names


def _same(a, b):
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, float) or isinstance(b, float):
        if math.isnan(a) or math.isnan(b):
            return math.isnan(a) and math.isnan(b)
    return a == b


@pytest.mark.parametrize("mode", [O.SUM_KAHAN, O.SUM_NAIVE, O.SUM_EXACT])
def test_group_by_golden(mode):
    for case in load_golden("group_by_cases.json")["cases"]:
        cols, names = _case_cols(case)
        key = O.HostCol(np.array(case["key"], dtype=np.int64))
        aggs = [(a[0], names.index(a[1])) for a in case["aggs"]]
        keys, kvalid, outs = O.group_by_agg(key, cols, None, aggs, len(case["key"]), mode)
        order = np.argsort(keys, kind="stable") if case.get("sort_by_key") else np.arange(len(keys))
        assert keys[order].tolist() == case["expected"]["key"], case["name"]
        for a, (vals, valid) in zip(case["aggs"], outs):
            outname = a[2] if len(a) > 2 else a[1]
            exp = unhex(case["expected"][outname])
            got = [v if ok else None for v, ok in zip(vals[order].tolist(), valid[order].tolist())]
            assert all(_same(x, y) for x, y in zip(got, exp)), (case["name"], outname, got, exp)


def test_filter_golden():
    for case in load_golden("filter_cases.json")["cases"]:
        names = list(case["cols"])
        cols = []
        for nm in names:
            vals = case["cols"][nm]
            valid = np.array([v is not None for v in vals], dtype=bool)
            arr = np.array([0 if v is None else v for v in vals], dtype=np.int64)
            cols.append(O.HostCol(arr, None if valid.all() else valid))
        n = len(case["cols"][names[0]])
        # predicates of the fixtures, as postfix programs
        progs = {
            "lit(True) | (col('column_0') == 1)": [(4, 0, 1), (1, 0, 0), (3, 0, 1), (20, 0, 0), (31, 0, 0)],
            "(col('a') > 2) | lit(False)": [(1, 0, 0), (3, 0, 2), (24, 0, 0), (4, 0, 0), (31, 0, 0)],
            "lit(True)": [(1, 0, 0), (34, 0, 0), (1, 0, 0), (33, 0, 0), (31, 0, 0)],  # x.is_not_null() | x.is_null()
            "col('a').is_null()": [(1, 0, 0), (33, 0, 0)],
            "col('a') <= 2": [(1, 0, 0), (3, 0, 2), (23, 0, 0)],
        }
        prog = progs[case["predicate"]]
        if "expected_mask" in case:
            dt, v, valid = O.eval_program(cols, prog, n)
            assert [bool(x) for x in v] == case["expected_mask"]
            continue
        outs = [O.filter_column(cols, prog, n, i) for i in range(len(cols))]
        rows = [list(r) for r in zip(*[[x if ok else None for x, ok in zip(v.tolist(), va.tolist())]
                                       for v, va in outs])] if outs else []
        assert rows == case["expected_rows"], case["name"]


@pytest.mark.parametrize("seed", range(5))
def test_fsum_matches_math_fsum(seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(5000) * 10.0 ** rng.integers(-30, 30, 5000)
    x[::97] = -x[::89][: len(x[::97])]
    assert O.fsum(x) == math.fsum(x)


def _ulp_diff(a: float, b: float) -> int:
    ia = np.array(a).view(np.int64).item()
    ib = np.array(b).view(np.int64).item()
    return abs(ia - ib)


@pytest.mark.parametrize("seed", range(3))
def test_sum_modes_bounds(seed):
    rng = np.random.default_rng(100 + seed)
    n = 20000
    key = rng.integers(0, 50, n).astype(np.int64)
    v = rng.uniform(1.0, 1000.0, n)
    kc, vc = O.HostCol(key), O.HostCol(v)
    res = {m: O.group_by_agg(kc, [vc], None, [("sum", 0)], n, m) for m in (0, 1, 2)}
    k0 = res[2][0]
    for m in (0, 1):
        assert (res[m][0] == k0).all()
    for gi, kv in enumerate(k0):
        exact = res[2][2][0][0][gi]
        assert exact == math.fsum(v[key == kv])
        assert _ulp_diff(res[0][2][0][0][gi], exact) <= 1           # Kahan
        cnt = int((key == kv).sum())
        bound = (cnt - 1) * 2.0 ** -53 / (1 - (cnt - 1) * 2.0 ** -53) * np.abs(v[key == kv]).sum()
        assert abs(res[1][2][0][0][gi] - exact) <= bound           # naive (Higham)


def test_baseline_matches_group_by():
    rng = np.random.default_rng(7)
    n = 50000
    key = rng.integers(0, 100, n).astype(np.int64)
    a, b = rng.uniform(0, 100, n), rng.uniform(0, 100, n)
    g, chk = O.baseline_filter_groupby_sum(key, a, 50.0, [a, b], threads=4)
    sel = a > 50.0
    assert g == len(np.unique(key[sel]))
    assert abs(chk - (a[sel].sum() + b[sel].sum())) < 1e-6 * chk


# ------------------------------------------------------------------ joins
def _golden_join_pairs(case):
    lname = case.get("left_on", case.get("on"))
    rname = case.get("right_on", case.get("on"))
    lv = case["left"][lname]
    rv = case["right"][rname]
    lk = O.HostCol(np.array([0 if v is None else v for v in lv], np.int64), np.array([v is not None for v in lv]))
    rk = O.HostCol(np.array([0 if v is None else v for v in rv], np.int64), np.array([v is not None for v in rv]))
    return O.join_inner(lk, rk, case["args"].get("nulls_equal", False))


def test_oracle_join_golden():
    """The oracle's inner join reproduces every join assertion transcribed
    from operations/test_join.py (tests/golden/join_cases.json)."""
    for case in load_golden("join_cases.json")["cases"]:
        li, ri = _golden_join_pairs(case)
        if "raises" in case:
            lname = case.get("left_on", case.get("on"))
            lvals, rvals = case["left"][lname], case["right"][case.get("right_on", lname)]
            v = case["args"]["validate"]
            left_unique = len(set(lvals)) == len(lvals)
            right_unique = len(set(rvals)) == len(rvals)
            ok = {"m:m": True, "1:m": left_unique, "m:1": right_unique, "1:1": left_unique and right_unique}[v]
            assert ok != case["raises"], case["name"]
            continue
        if "expected_height" in case:
            assert len(li) == case["expected_height"], case["name"]
            continue
        lname = case.get("on")
        order = case["args"].get("maintain_order")
        if order in ("right", "right_left"):
            perm = np.lexsort((li, ri))
            li, ri = li[perm], ri[perm]
        rows = []
        for a, b in zip(li, ri):
            row = {k: v[a] for k, v in case["left"].items()}
            row.update({k: v[b] for k, v in case["right"].items() if k != lname})
            rows.append(row)
        if "expected_column" in case:
            (cname, exp), = case["expected_column"].items()
            assert [r[cname] for r in rows] == exp, case["name"]
            continue
        exp = case["expected"]
        cols = list(exp)
        got = [tuple(r[c] for c in cols) for r in rows]
        want = list(zip(*[exp[c] for c in cols]))
        if not case["ordered"]:
            key = lambda t: tuple((x is None, x if x is not None else 0) for x in t)  # noqa: E731
            got, want = sorted(got, key=key), sorted(want, key=key)
        assert got == want, case["name"]


# ------------------------------------------------------------ sort / rolling
def _host(vals):
    isf = any(isinstance(v, float) for v in vals if v is not None)
    dt = np.float64 if isf else np.int64
    arr = np.array([0 if v is None else v for v in vals], dt)
    valid = np.array([v is not None for v in vals], bool)
    return O.HostCol(arr, None if valid.all() else valid), arr, valid


def _same_val(a, b):
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b


def test_oracle_sort_golden():
    """Stable TotalOrd arg-sort reproduces operations/test_sort.py."""
    for case in load_golden("sort_cases.json")["cases"]:
        vals = [unhex(v) if isinstance(v, str) else v for v in case["values"]]
        col, arr, valid = _host(vals)
        a = case["args"]
        idx = O.arg_sort(col, a.get("descending", False), a.get("nulls_last", False))
        if "expected_arg_sort" in case:
            assert idx.tolist() == case["expected_arg_sort"], case["name"]
        else:
            exp = [unhex(v) if isinstance(v, str) else v for v in case["expected_sorted"]]
            got = [vals[i] for i in idx]
            assert all(_same_val(g, e) for g, e in zip(got, exp)), case["name"]


def test_oracle_rolling_golden():
    """The restated SumWindow / MeanWindow / MinMaxWindow / MomentWindow
    reproduce every transcribed rolling assertion; the exact mode agrees on
    these cases."""
    for case in load_golden("rolling_cases.json")["cases"]:
        vals = [unhex(v) if isinstance(v, str) else v for v in case["values"]]
        col, _, _ = _host(vals)
        for mode in (O.ROLLING_REFERENCE, O.ROLLING_EXACT):
            if case["kind"] in ("var", "std"):
                out, ok = O.rolling_var(col, case["window"], case["min"], case["center"], case["ddof"],
                                        case["kind"] == "std", mode)
            else:
                out, ok = O.rolling(col, case["kind"], case["window"], case["min"], case["center"], mode)
            got = [v.item() if k else None for v, k in zip(out, ok)]
            check_rolling_case(got, case, mode)


def test_oracle_rolling_var_exact_is_the_exact_rational():
    """The exact mode of or_rolling_var is (RN(c sum x^2 - (sum x)^2) / c) /
    (c - ddof) with the numerator rounded once from the exact rational
    (Fractions), over values spanning 1e-320 .. 1e300, zeros, nulls and
    centred windows; std is its square root."""
    from fractions import Fraction

    rng = np.random.default_rng(3)
    n = 1500
    x = rng.uniform(10, 500, n) * rng.choice([1.0, -1.0], n)
    x[::97] = rng.standard_normal(x[::97].shape[0]) * 1e-200
    x[5] = 1e300
    x[700:705] = [3e-320, 1e-310, 0.0, -2e-315, 5e-324]
    valid = rng.random(n) > 0.1

    def tof(f):
        try:
            return float(f)
        except OverflowError:
            return math.inf

    for w, ms, center, ddof in ((20, 5, False, 1), (7, 1, True, 0), (64, 64, False, 2)):
        for std in (False, True):
            out, ok = O.rolling_var(O.HostCol(x, valid), w, ms, center, ddof, std, O.ROLLING_EXACT)
            for i in range(n):
                if center:
                    right = (w + 1) // 2
                    s, e = max(0, i - (w - right)), min(n, i + right)
                else:
                    s, e = max(0, i + 1 - w), i + 1
                vals = [Fraction(float(t)) for t, v in zip(x[s:e], valid[s:e]) if v]
                c = len(vals)
                if c < ms or c <= ddof:
                    assert not ok[i], (w, i)
                    continue
                ref = (tof(c * sum(t * t for t in vals) - sum(vals) ** 2) / c) / (c - ddof)
                if std:
                    ref = math.sqrt(ref)
                assert ok[i] and (out[i] == ref or (math.isinf(ref) and math.isinf(out[i]))), (w, i, out[i], ref)


def test_oracle_rolling_reference_vs_exact_ulp():
    """How far the reference's Kahan sliding window (mode 0) is from the
    exact window sum (mode 1, what the GPU computes).  The sliding state
    carries rounding from the whole column, so the two differ by more than
    the usual 1 ULP on small windows: measured max relative difference
    (to the window's sum of |x|) 1.4e-13 at w=3 on 2e5 rows, 2.1e-13 on 2e6
    rows; for w >= 20, <= 1 ULP (sum) / 2 ULP (mean, one more rounding).
    The GPU parity tests use these bounds against mode 0 and bit-exactness
    against mode 1."""
    rng = np.random.default_rng(0)
    n = 200_000
    x = rng.uniform(10, 500, n) * np.exp(0.02 * rng.standard_normal(n))
    cs = np.concatenate([[0.0], np.cumsum(np.abs(x))])
    i = np.arange(n)
    for w in (3, 20, 257):
        mag = cs[i + 1] - cs[np.maximum(0, i + 1 - w)]
        for kind in ("sum", "mean"):
            r, rv = O.rolling(O.HostCol(x), kind, w, 1, False, O.ROLLING_REFERENCE)
            e, ev = O.rolling(O.HostCol(x), kind, w, 1, False, O.ROLLING_EXACT)
            assert np.array_equal(rv, ev)
            if w >= 20:
                d = np.abs(r.view(np.int64) - e.view(np.int64))
                assert d.max() <= (1 if kind == "sum" else 2), (w, kind, d.max())
            else:
                scale = mag if kind == "sum" else mag / np.minimum(i + 1, w)
                assert (np.abs(r - e) / scale).max() <= 1e-12, (w, kind)


def _spec_arr(spec):
    """Fixture column -> (numpy values, validity or None)."""
    vals = unhex(spec["values"]) if spec["dtype"] == "f64" else spec["values"]
    valid = np.array([v is not None for v in vals], dtype=bool)
    dt = np.float64 if spec["dtype"] == "f64" else np.int64
    arr = np.array([(0.0 if dt is np.float64 else 0) if v is None else v for v in vals], dtype=dt)
    return arr, (None if valid.all() else valid)


def test_group_by_multi_golden():
    """Multi-key fixtures (tests/golden/group_by_multi_cases.json) through the
    row-encoding restatement (oracle.group_by_agg_multi)."""
    for case in load_golden("group_by_multi_cases.json")["cases"]:
        keys = [_spec_arr(s) for s in case["keys"].values()]
        cols, names = _case_cols(case)
        aggs = [(a[0], names.index(a[1])) for a in case["aggs"]]
        okeys, outs = O.group_by_agg_multi(keys, cols, None, aggs, len(keys[0][0]))
        knames = list(case["keys"])
        order = np.arange(len(okeys[0][0]))
        if "sort_by" in case:
            order = np.argsort(okeys[knames.index(case["sort_by"])][0], kind="stable")
        for kn, (v, m) in zip(knames, okeys):
            got = [x if ok else None for x, ok in zip(v[order].tolist(), m[order].tolist())]
            assert got == case["expected"][kn], (case["name"], kn, got)
        for a, (v, m) in zip(case["aggs"], outs):
            exp = unhex(case["expected"][a[2]])
            got = [x if ok else None for x, ok in zip(v[order].tolist(), m[order].tolist())]
            assert all(_same(x, y) for x, y in zip(got, exp)), (case["name"], a, got, exp)


def test_group_by_multi_matches_tuple_dict():
    """The multi-key restatement against a plain dict of tuples (nulls, -0.0
    / NaN keys, predicate-free)."""
    rng = np.random.default_rng(3)
    n = 3000
    a = rng.integers(0, 4, n).astype(np.int64)
    av = rng.random(n) > 0.2
    b = rng.choice(np.array([0.0, -0.0, np.nan, 1.5]), n)
    c = rng.random(n) < 0.5
    x = rng.standard_normal(n)
    okeys, outs = O.group_by_agg_multi([(a, av), (b, None), (c, None)], [O.HostCol(x)], None,
                                       [("sum", 0), ("len", 0)], n)
    exp = {}
    for i in range(n):
        t = (int(a[i]) if av[i] else None, "nan" if np.isnan(b[i]) else float(b[i]) + 0.0, bool(c[i]))
        exp.setdefault(t, []).append(x[i])
    got = {}
    for g in range(len(okeys[0][0])):
        bv = okeys[1][0][g]
        t = (int(okeys[0][0][g]) if okeys[0][1][g] else None, "nan" if np.isnan(bv) else float(bv) + 0.0,
             bool(okeys[2][0][g]))
        got[t] = (outs[0][0][g], int(outs[1][0][g]))
    assert set(got) == set(exp)
    for t, xs in exp.items():
        assert got[t] == (math.fsum(xs), len(xs))


def _keys_of(frame, names):
    out = []
    for nm in names:
        vals = frame[nm]
        valid = np.array([v is not None for v in vals], dtype=bool)
        arr = np.array([0 if v is None else v for v in vals], dtype=np.int64)
        out.append((arr, None if valid.all() else valid))
    return out


def _join_multi_rows(case, li, ri):
    """Output rows (dicts) of a multi-key fixture join: left columns, then the
    right non-key columns (suffix `_right` on a name clash)."""
    rows = []
    for a, b in zip(li, ri):
        row = {k: v[a] for k, v in case["left"].items()}
        for k, v in case["right"].items():
            if k not in case["on"]:
                row[k + "_right" if k in row else k] = v[b]
        rows.append(row)
    return rows


def test_join_multi_golden():
    """Multi-key join fixtures (tests/golden/join_multi_cases.json) through
    the row-encoding restatement (oracle.join_inner_multi)."""
    for case in load_golden("join_multi_cases.json")["cases"]:
        neq = case["args"].get("nulls_equal", False)
        li, ri = O.join_inner_multi(_keys_of(case["left"], case["on"]), _keys_of(case["right"], case["on"]), neq)
        if "expected_height" in case:
            assert len(li) == case["expected_height"], case["name"]
            continue
        rows = _join_multi_rows(case, li, ri)
        if "post_filter" in case:
            c, op, v = case["post_filter"]
            assert op == "<="
            rows = [r for r in rows if r[c] is not None and r[c] <= v]
        exp = case["expected"]
        assert [tuple(r[c] for c in exp) for r in rows] == list(zip(*exp.values())), case["name"]


def test_join_multi_matches_nested_loop():
    rng = np.random.default_rng(8)
    nl, nr = 400, 300
    la, ra = rng.integers(0, 5, nl), rng.integers(0, 5, nr)
    lb, rb = rng.integers(0, 4, nl), rng.integers(0, 4, nr)
    lbv, rbv = rng.random(nl) > 0.2, rng.random(nr) > 0.2
    for neq in (False, True):
        li, ri = O.join_inner_multi([(la, None), (lb, lbv)], [(ra, None), (rb, rbv)], neq)
        exp = sorted((i, j) for i in range(nl) for j in range(nr)
                     if la[i] == ra[j] and ((lbv[i] and rbv[j] and lb[i] == rb[j]) or
                                            (neq and not lbv[i] and not rbv[j])))
        assert sorted(zip(li.tolist(), ri.tolist())) == exp


def _frame_cols(frame, names):
    return [(np.array([0 if v is None else v for v in frame[nm]], dtype=np.int64),
             np.array([v is not None for v in frame[nm]], dtype=bool)) for nm in names]


def test_sort_multi_golden():
    """Multi-column sort fixtures (tests/golden/sort_multi_cases.json)."""
    for case in load_golden("sort_multi_cases.json")["cases"]:
        k = len(case["by"])
        desc = case["args"].get("descending", False)
        nl = case["args"].get("nulls_last", False)
        desc = desc if isinstance(desc, list) else [desc] * k
        nl = nl if isinstance(nl, list) else [nl] * k
        perm = O.arg_sort_multi(_frame_cols(case["frame"], case["by"]), desc, nl)
        for c, exp in case["expected"].items():
            assert [case["frame"][c][i] for i in perm] == exp, (case["name"], c)


def test_sort_multi_matches_python_sorted():
    rng = np.random.default_rng(4)
    n = 2000
    a = rng.choice(np.array([0.0, -0.0, 1.0, np.nan, -np.inf]), n)
    b = rng.integers(0, 5, n)
    bv = rng.random(n) > 0.3
    for da, db, nla, nlb in [(False, False, False, False), (True, False, True, False), (False, True, False, True),
                             (True, True, True, True)]:
        perm = O.arg_sort_multi([(a, None), (b, bv)], [da, db], [nla, nlb])

        def key(i):
            x = a[i]
            ka = (2 if np.isnan(x) else 1, 0.0 if np.isnan(x) else x + 0.0)
            ka = (-ka[0], -ka[1]) if da else ka
            kb = (0, 0) if not bv[i] else (1, -int(b[i]) if db else int(b[i]))
            kb = (kb[0] if not nlb else 1 - kb[0], kb[1])
            return (ka, kb, i)
        assert perm.tolist() == sorted(range(n), key=key)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_baseline_sort_rolling_matches_oracle(threads):
    """bench.py's configs[2] cpu_baseline computes the reference's result:
    the stable sort permutation applied to every column, and rolling_mean
    equal to the oracle's restatement of the Kahan sliding window."""
    rng = np.random.default_rng(threads)
    n = 50_003
    key = rng.integers(0, 5_000, n).astype(np.int64)  # many ties: stability matters
    cols = [rng.integers(0, 1 << 20, n).astype(np.int64) for _ in range(4)] + \
           [100 + rng.random(n) * 50 for _ in range(4)]
    outs, roll, _ = O.baseline_sort_rolling(key, cols, 4, 20, threads)
    perm = np.argsort(key, kind="stable")
    for c, o in zip(cols, outs):
        assert np.array_equal(o.view(c.dtype), c[perm])
    want, valid = O.rolling(O.HostCol(cols[4][perm]), "mean", 20)
    assert np.array_equal(roll[valid].view(np.uint64), want[valid].view(np.uint64))


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_baseline_join_inner_matches_oracle(threads):
    """bench.py's configs[3] cpu_baseline: the inner join's pairs equal the
    oracle's (as a multiset; within a thread's probe chunk in row order),
    duplicate build keys included."""
    rng = np.random.default_rng(10 + threads)
    nb, npr = 3_000, 40_000
    bk = rng.permutation(6_000)[:nb].astype(np.int64)
    bk[:50] = bk[50:100]  # duplicate build keys
    bv = rng.random(nb)
    pk = rng.integers(0, 6_000, npr).astype(np.int64)
    pv = rng.random(npr)
    ok, opv, obv = O.baseline_join_inner(pk, pv, bk, bv, threads)
    li, ri = O.join_inner(O.HostCol(pk), O.HostCol(bk))
    want = sorted(zip(pk[li].tolist(), pv[li].tolist(), bv[ri].tolist()))
    assert sorted(zip(ok.tolist(), opv.tolist(), obv.tolist())) == want


def _float_sum_spec(x, valid=None):
    """An independent Python reading of float_sum.rs sum_arr_as_f64, to pin
    the C restatement's lane / block order (no reference fixture covers it)."""
    x = [float(v) if valid is None or valid[i] else 0.0 for i, v in enumerate(x)]
    rem = len(x) % 128

    def block(b):
        lanes = [0.0] * 16
        for c in range(0, 128, 16):
            for j in range(16):
                lanes[j] = lanes[j] + b[c + j]
        w = 16
        while w > 4:
            for j in range(w // 2):
                lanes[j] = lanes[j] + lanes[w // 2 + j]
            w //= 2
        return (lanes[0] + lanes[2]) + (lanes[1] + lanes[3])

    def pairwise(a):
        if len(a) == 128:
            return block(a)
        left = (len(a) // 128 // 2) * 128
        return pairwise(a[:left]) + pairwise(a[left:])

    main = pairwise(x[rem:]) if len(x) > rem else 0.0
    rest = -0.0
    for v in x[:rem]:
        rest = rest + v
    return main + rest


@pytest.mark.parametrize("n", [0, 1, 127, 128, 129, 255, 256, 384, 1000, 5 * 128 + 17, 20_000])
def test_float_sum_restatement(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))
    valid = rng.random(n) > 0.2
    for v in (None, valid):
        got = O.float_sum(x, v)
        want = _float_sum_spec(x, v)
        assert np.float64(got).view(np.uint64) == np.float64(want).view(np.uint64)
    # exact inputs: integers below 2^40 sum exactly in any order
    xi = rng.integers(-2**40, 2**40, n).astype(np.float64)
    assert O.float_sum(xi) == float(xi.astype(np.int64).sum())


def test_variance_restatements():
    """Welford (insert_one / combine) and the chunked VarState give the
    textbook variance on exact data and agree with numpy to rounding."""
    x = np.arange(1, 1001, dtype=np.float64)
    assert O.var_welford(x) == pytest.approx(float(np.var(x, ddof=1)), rel=1e-15)
    assert O.var_chunked(x, 0) == pytest.approx(float(np.var(x)), rel=1e-15)
    part = np.arange(1000) // 100
    assert O.var_welford(x, part) == pytest.approx(float(np.var(x, ddof=1)), rel=1e-15)
    assert math.isnan(O.var_welford(x[:1], None, 1)) and O.var_welford(x[:1], None, 0) == 0.0


def test_one_correction_division_by_window_length():
    """rolling.hip rw_div: a full window's mean as q0 = RN(a y), r = a - w q0
    (exact, one fma), q = RN(q0 + r y) with y = RN(1 / w) equals RN(a / w)
    for every a whose quotient stays normal (Markstein's theorem; w is an
    integer, so its significand is never all ones).  Checked here with
    exact rationals over random a (|a| from 2^-900 to 2^990, the kernel's
    guard) and every w up to 1024."""
    import random
    from fractions import Fraction as Fr

    rnd = random.Random(7)
    for w in list(range(1, 1025)) + [rnd.randint(1025, 1 << 24) for _ in range(64)]:
        y = 1.0 / w
        for _ in range(24):
            e = rnd.choice([rnd.randint(-60, 60), rnd.randint(-900, 990)])
            a = ((rnd.getrandbits(52) | (1 << 52)) * 2.0 ** (e - 52)) * rnd.choice([1.0, -1.0])
            q0 = a * y
            r = Fr(a) - Fr(w) * Fr(q0)
            assert Fr(float(r)) == r  # the fma's remainder is exact
            assert float(Fr(q0) + r * Fr(y)) == float(Fr(a) / w), (a, w)


def test_fsum_exact_through_intermediate_overflow():
    """The oracle's exact sum stays correctly rounded when its partials
    overflow on the way (where math.fsum raises): the exact rational sum,
    rounded once, or +-inf beyond the largest double."""
    from fractions import Fraction

    def exact(xs):
        f = sum((Fraction(v) for v in xs), Fraction(0))
        try:
            return float(f)
        except OverflowError:
            return math.inf if f > 0 else -math.inf

    big = 1.7e308
    cases = [[big, big, -big], [big, big], [-big, -big], [1e308, 1e308, -1e308, -1e308, 1e-300],
             [big, big, -big, -big, 2.0 ** -1074], [big] * 3 + [-big] * 2 + [1.0]]
    rng = np.random.default_rng(5)
    for _ in range(200):
        n = int(rng.integers(2, 12))
        xs = rng.uniform(-1, 1, n) * 1.79e308
        xs[rng.random(n) < 0.3] *= 2.0 ** -int(rng.integers(0, 1100))
        cases.append(list(xs))
    for xs in cases:
        got = O.fsum(np.array(xs, dtype=np.float64))
        want = exact(xs)
        assert got == want and math.copysign(1, got) == math.copysign(1, want) or (got == 0 and want == 0), (xs, got, want)
