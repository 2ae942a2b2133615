"""Aggregations over computed inputs and global reductions (CPU).

Pins the oracle's restatement (oracle.group_by_agg_inputs: each input
program evaluated by the elementwise restatement or_eval, then aggregated;
key None = select(aggs), one output row even with no selected row) against
the cases transcribed from the reference's tests in
tests/golden/reduce_cases.json.  var / std are checked with the test's own
exact two-pass formula (math.fsum), which the GPU path computes too.  The
GPU side of the same cases is in tests/test_gpu_reduce.py.
"""

import math

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O
from polaroid_amd import _native as N
from polaroid_amd.expr import col, lit, lower, when

from conftest import load_golden, unhex

CASES = load_golden("reduce_cases.json")["cases"]
NP = {"i64": np.int64, "f64": np.float64, "f32": np.float32, "bool": np.bool_, "i32": np.int32}


def host_cols(case):
    names = list(case["cols"])
    cols = []
    for nm in names:
        spec = case["cols"][nm]
        vals = unhex(spec["values"])
        valid = np.array([v is not None for v in vals], bool)
        arr = np.array([0 if v is None else v for v in vals], dtype=NP[spec["dtype"]])
        cols.append(O.HostCol(arr, None if valid.all() else valid))
    return names, cols


def parse_aggs(case):
    """[(kind, input expr or None for len, out name, ddof)]."""
    out = []
    for text, name in case["aggs"]:
        e = eval(text, {"pl": pl, "col": col, "lit": lit, "when": when})
        base = e.args[0] if e.kind == "alias" else e
        if base.kind == "len":
            out.append(("len", None, name, None))
        else:
            out.append((base.op, base.args[0], name, base.value if base.op in ("var", "std") else None))
    return out


def oracle_case(case):
    """Run a case through the oracle: {out name: (values, valid)} (+ 'key')."""
    names, cols = host_cols(case)
    n = len(next(iter(case["cols"].values()))["values"])
    schema = {nm: c.code for nm, c in zip(names, cols)}
    idx = {nm: i for i, nm in enumerate(names)}
    aggs = parse_aggs(case)
    inputs, specs = [], []
    for kind, x, name, ddof in aggs:
        if kind == "len":
            specs.append(("len", 0))
            continue
        if kind in ("var", "std"):
            continue
        if x.kind == "col":
            specs.append((kind, idx[x.value]))
        else:
            inputs.append(lower(x, idx, schema))
            specs.append((kind, len(cols) + len(inputs) - 1))
    key = None if case["key"] is None else O.HostCol(np.array(case["key"], np.int64))
    keys, kvalid, outs = O.group_by_agg_inputs(key, cols, None, inputs, specs, n)
    res = {"key": keys}
    it = iter(outs)
    for kind, x, name, ddof in aggs:
        if kind in ("var", "std"):
            res[name] = var_std(case, cols, idx, x, kind, ddof, keys if key is not None else None)
        else:
            res[name] = next(it)
    return res


def var_std(case, cols, idx, x, kind, ddof, keys):
    """Exact two-pass var / std per group (the GPU's formula: mean from the
    exact sum, squared deviations summed exactly, one division)."""
    assert x.kind == "col"
    c = cols[idx[x.value]]
    n = c.c.length
    vals = np.unpackbits(c.buf, bitorder="little")[:n].astype(np.float64) if c.code == O.BOOL else c.buf.astype(
        np.float64)
    valid = np.ones(n, bool) if c.vbuf is None else np.unpackbits(c.vbuf, bitorder="little")[:n].astype(bool)
    gid = np.zeros(n, np.int64) if keys is None else np.array(case["key"], np.int64)
    groups = [0] if keys is None else list(keys)
    out, ok = [], []
    for g in groups:
        v = vals[(gid == g) & valid]
        if v.size <= ddof:
            out.append(0.0)
            ok.append(False)
            continue
        m = math.fsum(v) / v.size
        r = math.fsum((v - m) * (v - m)) / (v.size - ddof)
        out.append(math.sqrt(r) if kind == "std" else r)
        ok.append(True)
    return np.array(out), np.array(ok)


def check(case, res, order=None):
    exp = case["expected"]
    tol = case.get("tol", {})
    keys = res["key"]
    if "key" in exp:
        o = np.argsort(keys, kind="stable") if case.get("sort_by_key") or order is None else order
        assert keys[o].tolist() == exp["key"]
    else:
        o = np.arange(len(keys))
    for name, want in exp.items():
        if name == "key":
            continue
        want = unhex(want)
        vals, valid = res[name]
        got = [None if not valid[i] else vals[i].item() for i in o]
        assert len(got) == len(want), (name, got, want)
        for g, w in zip(got, want):
            if w is None:
                assert g is None, (name, got, want)
            elif isinstance(w, float):
                assert g is not None
                if name in tol:
                    assert math.isclose(g, w, rel_tol=tol[name]), (name, g, w)
                else:
                    assert float(g) == w, (name, g, w)
            else:
                assert int(g) == w, (name, got, want)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_reductions_match_reference(case):
    check(case, oracle_case(case))


def test_oracle_empty_selection_row():
    """No selected row: one row, sum / len / count 0, the rest null."""
    a = O.HostCol(np.array([1.5, 2.5, -1.0]))
    prog = [(N.OP["COL"], 0, 0), (N.OP["LIT_F64"], 0, 100.0), (N.OP["GT"], 0, 0)]
    keys, kvalid, outs = O.group_by_agg_inputs(None, [a], prog, [], [("sum", 0), ("len", 0), ("count", 0),
                                                                   ("mean", 0), ("min", 0), ("first", 0)], 3)
    assert keys.shape[0] == 1
    assert [bool(v[0]) for _, v in outs] == [True, True, True, False, False, False]
    assert outs[0][0][0] == 0.0 and outs[1][0][0] == 0 and outs[2][0][0] == 0


def test_oracle_derived_input_is_elementwise_then_exact():
    """(a * b).sum() per group = the exact sum of the IEEE products, and a
    Boolean input sums as counts."""
    rng = np.random.default_rng(5)
    n = 5000
    a, b = rng.standard_normal(n) * 1e3, rng.standard_normal(n)
    k = rng.integers(0, 7, n).astype(np.int64)
    prog = [(N.OP["COL"], 0, 0), (N.OP["COL"], 1, 0), (N.OP["MUL"], 0, 0)]
    gt = [(N.OP["COL"], 0, 0), (N.OP["LIT_F64"], 0, 0.0), (N.OP["GT"], 0, 0)]
    keys, _, outs = O.group_by_agg_inputs(O.HostCol(k), [O.HostCol(a), O.HostCol(b)], None, [prog, gt],
                                          [("sum", 2), ("sum", 3)], n)
    for i, g in enumerate(keys):
        m = k == g
        assert outs[0][0][i] == math.fsum(a[m] * b[m])
        assert outs[1][0][i] == int((a[m] > 0).sum())
    assert outs[1][0].dtype == np.int64  # integer results as int64 bits (the caller narrows to UInt32)
