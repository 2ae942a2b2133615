"""The polars GPU-engine plugin (polaroid_amd/polars_engine.py) against a
model of the reference's NodeTraverser: the IR / expression node classes of
crates/polars-python/src/lazyframe/visitor/{nodes,expr_nodes}.rs with the
same class and attribute names, and the traverser methods of
crates/polars-python/src/lazyframe/visit.rs (view_current_node, get_node,
set_node, view_expression, get_schema, set_udf).  polars itself is not
installed here, so polars DataFrames are modelled by their Arrow export.
"""

import math

import numpy as np
import pyarrow as pa
import pytest

import polaroid_amd as pl
from polaroid_amd import polars_engine as PE


# ---------------------------------------------------------------- IR model
class _Enum:
    def __init__(self, cls, name):
        self.s = f"{cls}.{name}"

    def __str__(self):
        return self.s


def _node(kind, **kw):
    return type(kind, (), {})() if not kw else type(kind, (), kw)()


class PyExprIR:
    def __init__(self, node, output_name):
        self.node, self.output_name = node, output_name


class FakePolarsDF:
    def __init__(self, table):
        self.table = table

    def to_arrow(self):
        return self.table


class FakeNT:
    def __init__(self, table):
        self.lp, self.ex, self.schemas = [], [], []
        self.root = None
        self.udf = None
        self.table = table

    # builders
    def e(self, kind, **kw):
        self.ex.append(_node(kind, **kw))
        return len(self.ex) - 1

    def p(self, kind, schema, **kw):
        self.lp.append(_node(kind, **kw))
        self.schemas.append(schema)
        self.root = len(self.lp) - 1
        return self.root

    def col(self, name):
        return self.e("Column", name=name)

    def lit(self, v):
        return self.e("Literal", value=v, dtype=None)

    def bin(self, l, op, r):
        return self.e("BinaryExpr", left=l, op=_Enum("Operator", op), right=r)

    # NodeTraverser API
    def view_current_node(self):
        return self.lp[self.root]

    def get_node(self):
        return self.root

    def set_node(self, n):
        self.root = n

    def view_expression(self, n):
        return self.ex[n]

    def get_schema(self):
        return {k: None for k in self.schemas[self.root]}

    def set_udf(self, fn, is_pure=False):
        self.udf = fn


def _table(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 13, n).astype(np.int64)
    v = rng.standard_normal(n) * 10
    w = rng.integers(-100, 100, n).astype(np.int64)
    vmask = rng.random(n) < 0.1
    return pa.table({"k": pa.array(k), "v": pa.array(v, mask=vmask), "w": pa.array(w)}), k, v, w, ~vmask


def _filter_groupby_ir(table):
    """df.lazy().filter((v > 0.5) | (w == 3)).group_by("k").agg(v.sum(), w.mean(), len())"""
    nt = FakeNT(table)
    scan = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    pred = nt.bin(nt.bin(nt.col("v"), "Gt", nt.lit(0.5)), "Or", nt.bin(nt.col("w"), "Eq", nt.lit(3)))
    filt = nt.p("Filter", ["k", "v", "w"], input=scan, predicate=PyExprIR(pred, "v"))
    key = nt.col("k")
    a1 = nt.e("Agg", name="sum", arguments=[nt.col("v")], options=None)
    a2 = nt.e("Agg", name="mean", arguments=[nt.col("w")], options=None)
    a3 = nt.e("Len")
    a4 = nt.e("Agg", name="count", arguments=[nt.col("v")], options=False)
    opts = _node("GroupbyOptions", slice=None, dynamic=None, rolling=None)
    nt.p("GroupBy", ["k", "v", "w", "len", "cnt"], input=filt, keys=[PyExprIR(key, "k")],
         aggs=[PyExprIR(a1, "v"), PyExprIR(a2, "w"), PyExprIR(a3, "len"), PyExprIR(a4, "cnt")], apply=None,
         maintain_order=True, options=opts)
    return nt


def test_translate_filter_group_by():
    table = _table()[0]
    nt = _filter_groupby_ir(table)
    root = nt.root
    plan = PE.translate(nt)
    assert nt.root == root  # traverser restored
    assert plan[0] == "group_by" and plan[2] == "k" and plan[4] is True
    assert [a.output_name() for a in plan[3]] == ["v", "w", "len", "cnt"]
    assert plan[1][0] == "filter" and plan[1][1][0] == "polars_scan"
    assert repr(plan[1][2]).count("v") == 1


def test_unsupported_leaves_plan_to_polars():
    table = _table()[0]
    nt = _filter_groupby_ir(table)
    nt.lp[nt.root].aggs.append(PyExprIR(nt.e("Agg", name="median", arguments=[nt.col("v")], options=None),
                                        "med"))
    PE.execute_with_polaroid(nt, None)
    assert nt.udf is None
    with pytest.raises(pl.InvalidOperationError):
        PE.execute_with_polaroid(nt, None, config={"raise_on_fail": True})
    # NaN-propagating min (nan_min) is outside the path too
    nt2 = _filter_groupby_ir(table)
    nt2.lp[nt2.root].aggs[0] = PyExprIR(nt2.e("Agg", name="min", arguments=[nt2.col("v")], options=True), "v")
    with pytest.raises(PE.Unsupported):
        PE.translate(nt2)


def test_accepted_query_installs_udf():
    nt = _filter_groupby_ir(_table()[0])
    PE.execute_with_polaroid(nt, None)
    assert callable(nt.udf)


@pytest.mark.gpu
def test_udf_runs_on_gpu_and_matches(gpu):
    table, k, v, w, vvalid = _table(200_000, 3)
    nt = _filter_groupby_ir(table)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    assert out.column_names == ["k", "v", "w", "len", "cnt"]
    sel = ((v > 0.5) & vvalid) | (w == 3)
    keys = out.column("k").to_pylist()
    # maintain_order: first-occurrence order of the selected rows
    first = list(dict.fromkeys(k[sel].tolist()))
    assert keys == first
    for i, kk in enumerate(keys):
        m = sel & (k == kk)
        assert out.column("v")[i].as_py() == math.fsum(v[m & vvalid])
        assert out.column("w")[i].as_py() == float(w[m].sum()) / int(m.sum())
        assert out.column("len")[i].as_py() == int(m.sum())
        assert out.column("cnt")[i].as_py() == int((m & vvalid).sum())


def test_translate_join_and_sort():
    table = _table()[0]
    nt = FakeNT(table)
    left = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    right = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    j = nt.p("Join", ["k", "v", "w", "v_right", "w_right"], input_left=left, input_right=right,
             left_on=[PyExprIR(nt.col("k"), "k")], right_on=[PyExprIR(nt.col("k"), "k")],
             options=("inner", False, None, "_right", True, "left"))
    nt.p("Sort", ["k", "v", "w", "v_right", "w_right"], input=j, by_column=[PyExprIR(nt.col("w"), "w")],
         sort_options=(False, [True], [True]), slice=None)
    plan = PE.translate(nt)
    assert plan[0] == "sort" and plan[2] == "w" and plan[3] is True and plan[4] is True
    jn = plan[1]
    assert jn[0] == "join" and jn[3] == "k" and jn[4] == "k" and jn[5] == "_right" and jn[8] == "left"
    assert jn[1][0] == "polars_scan" and jn[2][0] == "polars_scan"
    # every equi-join type translates (coalesce arrives resolved); cross joins
    # and IE joins (a tuple `how`) stay on polars
    for how, co in (("left", True), ("right", True), ("full", False), ("semi", True), ("anti", True)):
        nt.lp[j].options = (how, True, None, "_r", co, "left_right")
        jn = PE.translate(nt)[1]
        assert jn[9] == how and jn[10] is co and jn[7] is True and jn[8] == "left_right" and jn[5] == "_r"
    for how in ("cross", ("ie_join", "lt", None)):
        nt.lp[j].options = (how, False, None, "_right", True, "none")
        with pytest.raises(PE.Unsupported):
            PE.translate(nt)


@pytest.mark.gpu
def test_udf_join_sort_on_gpu(gpu):
    table, k, v, w, vvalid = _table(20_000, 5)
    right = pa.table({"k": pa.array(np.arange(13, dtype=np.int64)), "z": pa.array(np.arange(13) * 1.5)})
    nt = FakeNT(table)
    left = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    rs = nt.p("DataFrameScan", ["k", "z"], df=FakePolarsDF(right), projection=None, selection=None)
    j = nt.p("Join", ["k", "v", "w", "z"], input_left=left, input_right=rs,
             left_on=[PyExprIR(nt.col("k"), "k")], right_on=[PyExprIR(nt.col("k"), "k")],
             options=("inner", False, None, "_right", True, "left"))
    nt.p("Sort", ["k", "v", "w", "z"], input=j, by_column=[PyExprIR(nt.col("w"), "w")],
         sort_options=(True, [False], [False]), slice=None)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    order = np.argsort(w, kind="stable")
    assert out.column("w").to_pylist() == w[order].tolist()
    assert out.column("z").to_pylist() == (k[order] * 1.5).tolist()


def test_translate_multi_key_group_by():
    table = _table()[0]
    nt = _filter_groupby_ir(table)
    nt.lp[nt.root].keys.append(PyExprIR(nt.col("w"), "w"))
    plan = PE.translate(nt)
    assert plan[0] == "group_by" and plan[2] == ("k", "w")
    # a computed key stays on polars
    nt.lp[nt.root].keys[1] = PyExprIR(nt.bin(nt.col("w"), "Plus", nt.lit(1)), "w")
    with pytest.raises(PE.Unsupported):
        PE.translate(nt)


@pytest.mark.gpu
def test_udf_multi_key_group_by_on_gpu(gpu):
    table, k, v, w, vvalid = _table(50_000, 8)
    nt = _filter_groupby_ir(table)
    nt.lp[nt.root].keys.append(PyExprIR(nt.col("w"), "w"))
    nt.schemas[nt.root] = ["k", "w", "v", "w_mean", "len", "cnt"]
    nt.lp[nt.root].aggs[1] = PyExprIR(nt.e("Agg", name="mean", arguments=[nt.col("w")], options=None), "w_mean")
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    sel = ((v > 0.5) & vvalid) | (w == 3)
    first = list(dict.fromkeys(zip(k[sel].tolist(), w[sel].tolist())))
    assert list(zip(out.column("k").to_pylist(), out.column("w").to_pylist())) == first
    for i, (kk, ww) in enumerate(first):
        m = sel & (k == kk) & (w == ww)
        assert out.column("v")[i].as_py() == math.fsum(v[m & vvalid])
        assert out.column("len")[i].as_py() == int(m.sum())


def test_translate_multi_key_join():
    table = _table()[0]
    nt = FakeNT(table)
    left = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    right = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    nt.p("Join", ["k", "v", "w", "v_right"], input_left=left, input_right=right,
         left_on=[PyExprIR(nt.col("k"), "k"), PyExprIR(nt.col("w"), "w")],
         right_on=[PyExprIR(nt.col("k"), "k"), PyExprIR(nt.col("w"), "w")],
         options=("inner", True, None, "_right", True, "none"))
    plan = PE.translate(nt)
    assert plan[0] == "join" and plan[3] == ("k", "w") and plan[4] == ("k", "w") and plan[7] is True


def test_translate_multi_column_sort():
    table = _table()[0]
    nt = FakeNT(table)
    scan = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    nt.p("Sort", ["k", "v", "w"], input=scan, by_column=[PyExprIR(nt.col("k"), "k"), PyExprIR(nt.col("w"), "w")],
         sort_options=(True, [False, True], [True, False]), slice=None)
    plan = PE.translate(nt)
    assert plan[0] == "sort" and plan[2] == ("k", "w") and plan[3] == (True, False) and plan[4] == (False, True)
    # a broadcast single flag applies to every column
    nt.lp[nt.root].sort_options = (False, [True], [False])
    plan = PE.translate(nt)
    assert plan[3] == (False, False) and plan[4] == (True, True)
