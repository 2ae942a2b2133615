"""The polars GPU-engine plugin (polaroid_amd/polars_engine.py) against a
model of the reference's NodeTraverser: the IR / expression node classes of
crates/polars-python/src/lazyframe/visitor/{nodes,expr_nodes}.rs with the
same class and attribute names, and the traverser methods of
crates/polars-python/src/lazyframe/visit.rs (view_current_node, get_node,
set_node, view_expression, get_schema, set_udf).  polars itself is not
installed here, so `DataFrameScan.df` is modelled as the reference's
PyDataFrame: `to_arrow(compat_level)` with no default, returning one Arrow
RecordBatch per chunk (crates/polars-python/src/dataframe/export.rs:80-99),
and `get_schema` hands out dtype objects whose str() is polars' dtype repr.
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


class FakePyDataFrame:
    """Model of the reference's PyDataFrame (DataFrameScan.df, visitor/nodes.rs:190)."""

    def __init__(self, table, chunk_rows=None):
        self.table = table
        self.chunk_rows = chunk_rows
        self.calls = []

    def to_arrow(self, compat_level):  # export.rs:80: no default for compat_level
        if not isinstance(compat_level, (bool, int)):
            raise TypeError("'compat_level' argument accepts int or bool")  # conversion/mod.rs:1574
        self.calls.append(compat_level)
        t = self.table
        if compat_level is False or compat_level == 0:  # CompatLevel::oldest: large_string, no views
            t = t.cast(pa.schema([pa.field(f.name, pa.large_string() if f.type == pa.string() else f.type)
                                  for f in t.schema]))
        return t.to_batches(max_chunksize=self.chunk_rows)


FakePolarsDF = FakePyDataFrame


class _DType:
    """A polars DataType as the visitor returns it (only its repr matters here)."""

    def __init__(self, s):
        self.s = s

    def __str__(self):
        return self.s

    __repr__ = __str__


_ARROW_TO_POLARS = {pa.int64(): "Int64", pa.int32(): "Int32", pa.uint32(): "UInt32", pa.float64(): "Float64",
                    pa.bool_(): "Boolean", pa.string(): "String", pa.large_string(): "String",
                    pa.timestamp("ns"): "Datetime(time_unit='ns', time_zone=None)", pa.float32(): "Float32",
                    pa.list_(pa.int64()): "List(Int64)"}


class FakeNT:
    def __init__(self, table):
        self.lp, self.ex, self.schemas = [], [], []
        self.root = None
        self.udf = None
        self.table = table
        self.dtypes = {}
        if table is not None:
            self.add_dtypes(table)

    def add_dtypes(self, table):
        for f in table.schema:
            if pa.types.is_dictionary(f.type):
                self.dtypes[f.name] = "Categorical"
            else:
                self.dtypes[f.name] = _ARROW_TO_POLARS.get(f.type, str(f.type))

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
        return {k: _DType(self.dtypes.get(k, "Float64")) for k in self.schemas[self.root]}

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


# ------------------------------------------------------------ scan binding
def test_scan_calls_to_arrow_with_compat_level_and_takes_batches():
    table = _table(1000)[0]
    df = FakePyDataFrame(table, chunk_rows=300)
    batches = PE.scan_batches(df)
    assert df.calls == [False] and len(batches) == 4
    assert all(isinstance(b, pa.RecordBatch) for b in batches)

    class Wrapped:  # a polars DataFrame: its PyDataFrame is `_df`
        _df = df

    assert len(PE.scan_batches(Wrapped())) == 4


def test_unsupported_scan_dtype_falls_back_without_error():
    table = _table()[0]
    nt = _filter_groupby_ir(table)
    nt.dtypes["w"] = "List(Int64)"
    PE.execute_with_polaroid(nt, None)  # polars keeps the query: no UDF, no error
    assert nt.udf is None
    with pytest.raises(pl.InvalidOperationError):
        PE.execute_with_polaroid(nt, None, config={"raise_on_fail": True})
    # a projection that leaves the column out is fine
    nt2 = _filter_groupby_ir(table)
    nt2.dtypes["x"] = "Decimal(precision=10, scale=2)"
    nt2.schemas[0] = ["k", "v", "w", "x"]
    nt2.lp[0].projection = ["k", "v", "w"]
    PE.execute_with_polaroid(nt2, None)
    assert callable(nt2.udf)


def _enum_nt():
    cats = pa.array(["zeta", "alpha", "mid"])
    e = pa.DictionaryArray.from_arrays(pa.array([0, 1, 2, 0, 1], pa.uint32()), cats)
    table = pa.table({"e": e, "v": pa.array([1.0, 2.0, 3.0, 4.0, 5.0])})
    nt = FakeNT(table)
    nt.dtypes["e"] = "Enum(categories=['zeta', 'alpha', 'mid'])"
    scan = nt.p("DataFrameScan", ["e", "v"], df=FakePyDataFrame(table), projection=None, selection=None)
    return nt, scan


def test_enum_ordered_uses_stay_on_polars():
    # Enum orders by category index (logical/categorical.rs:58, sort/categorical.rs:74),
    # the GPU handles it as strings: sort / ordered comparisons / min / max go to polars
    nt, scan = _enum_nt()
    nt.p("Sort", ["e", "v"], input=scan, by_column=[PyExprIR(nt.col("e"), "e")],
         sort_options=(False, [False], [False]), slice=None)
    with pytest.raises(PE.Unsupported, match="Enum"):
        PE.translate(nt)
    nt, scan = _enum_nt()
    nt.p("Filter", ["e", "v"], input=scan, predicate=PyExprIR(nt.bin(nt.col("e"), "Lt", nt.lit("mid")), "e"))
    with pytest.raises(PE.Unsupported, match="Enum"):
        PE.translate(nt)
    nt, scan = _enum_nt()
    a = nt.e("Agg", name="max", arguments=[nt.col("e")], options=False)
    opts = _node("GroupbyOptions", slice=None, dynamic=None, rolling=None)
    nt.p("GroupBy", ["v", "e"], input=scan, keys=[PyExprIR(nt.col("v"), "v")], aggs=[PyExprIR(a, "e")],
         apply=None, maintain_order=True, options=opts)
    with pytest.raises(PE.Unsupported, match="Enum"):
        PE.translate(nt)
    # equality on an Enum is order-free and stays on the GPU path
    nt, scan = _enum_nt()
    nt.p("Filter", ["e", "v"], input=scan, predicate=PyExprIR(nt.bin(nt.col("e"), "Eq", nt.lit("mid")), "e"))
    assert PE.translate(nt)[0] == "filter"


@pytest.mark.gpu
def test_udf_multi_chunk_scan_on_gpu(gpu):
    """Chunks of 777 rows: validity and Boolean bits land at bit offsets that
    are not byte aligned; strings are rebased per chunk; a dictionary column
    is unified across chunks."""
    rng = np.random.default_rng(11)
    n = 10_000
    k = rng.integers(0, 9, n).astype(np.int64)
    v = rng.standard_normal(n)
    vmask = rng.random(n) < 0.2
    b = rng.random(n) < 0.5
    bmask = rng.random(n) < 0.1
    sym = np.array(["AAPL", "MSFT", "", "GOOGLEPLEX_LONG_NAME", "Ä€"])[rng.integers(0, 5, n)]
    smask = rng.random(n) < 0.15
    table = pa.table({"k": pa.array(k), "v": pa.array(v, mask=vmask), "b": pa.array(b, mask=bmask),
                      "s": pa.array(sym.tolist(), mask=smask), "w": pa.array(k.astype(np.int32) * 3)})
    nt = FakeNT(table)
    nt.p("DataFrameScan", ["k", "v", "b", "s", "w"], df=FakePyDataFrame(table, chunk_rows=777), projection=None,
         selection=None)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    for name in ("k", "v", "b", "s", "w"):
        assert out.column(name).to_pylist() == table.column(name).to_pylist(), name


@pytest.mark.gpu
def test_from_arrow_sliced_chunks(gpu):
    rng = np.random.default_rng(5)
    base = pa.array(rng.standard_normal(5000), mask=rng.random(5000) < 0.3)
    bools = pa.array(rng.random(5000) < 0.5, mask=rng.random(5000) < 0.3)
    strs = pa.array([None if i % 7 == 0 else "x" * (i % 13) for i in range(5000)], pa.large_string())
    for arr in (base, bools, strs):
        chunks = [arr.slice(3, 100), arr.slice(1001, 1), arr.slice(0, 0), arr.slice(2000, 2999), arr.slice(13, 64)]
        ca = pa.chunked_array(chunks, type=arr.type)
        s = pl.Series.from_arrow("x", ca)
        assert s.to_list() == ca.to_pylist()
        assert s.null_count() == ca.null_count
    # all-valid chunk next to a chunk with nulls: the column gets a validity
    ca = pa.chunked_array([pa.array([1, 2, 3], pa.int64()), pa.array([None, 5], pa.int64())])
    assert pl.Series.from_arrow("y", ca).to_list() == [1, 2, 3, None, 5]
    # an empty frame of batches keeps its columns
    df = pl.DataFrame.from_batches([pa.record_batch({"a": pa.array([], pa.int64())})])
    assert df.height == 0 and df.columns == ["a"]


def test_column_cache_keys_and_eviction():
    """The resident-column cache (CPU side): the same Arrow chunks give the
    same key, other buffers another; LRU eviction by bytes."""
    a = pa.array(np.arange(1000, dtype=np.int64))
    b = pa.array(np.arange(1000, dtype=np.int64))
    ka, kb = PE.ColumnCache.key([a], a.type), PE.ColumnCache.key([b], b.type)
    assert ka == PE.ColumnCache.key([a], a.type) and ka != kb
    assert PE.ColumnCache.key([a.slice(10, 20)], a.type) != ka  # offset / length are part of the key
    c = PE.ColumnCache(capacity=20_000)
    c.put(ka, "A", [a], 8_000)
    c.put(kb, "B", [b], 8_000)
    assert c.get(ka) == "A"  # A is now most recent
    k3 = PE.ColumnCache.key([pa.array([1.0])], pa.float64())
    c.put(k3, "C", [], 8_000)  # over capacity: B (least recent) goes
    assert c.get(kb) is None and c.get(ka) == "A" and c.get(k3) == "C"
    assert c.bytes == 16_000 and c.hits == 3 and c.misses == 1
    c.put(("big",), "X", [], 50_000)  # larger than the whole cache: not kept
    assert c.get(("big",)) is None


@pytest.mark.gpu
def test_udf_reuses_resident_columns(gpu):
    """A second query over the same frame takes its columns from the device
    cache (no re-upload) and gives the same result; another frame misses."""
    PE.column_cache().clear()
    rng = np.random.default_rng(2)
    n = 50_000
    table = pa.table({"k": pa.array(rng.integers(0, 50, n)), "v": pa.array(rng.standard_normal(n))})
    pydf = FakePyDataFrame(table)
    outs = []
    for _ in range(2):
        nt = FakeNT(table)
        scan = nt.p("DataFrameScan", ["k", "v"], df=pydf, projection=None, selection=None)
        nt.p("Filter", ["k", "v"], input=scan, predicate=PyExprIR(nt.bin(nt.col("v"), "Gt", nt.lit(0.0)), "v"))
        PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
        outs.append(nt.udf(None, None, None, False))
    assert outs[0].equals(outs[1])
    c = PE.column_cache()
    assert c.hits >= 2 and c.misses == 2  # k and v uploaded once
    want = table.filter(pa.compute.greater(table.column("v"), 0.0))
    assert outs[0].column("v").to_pylist() == want.column("v").to_pylist()
    # a different frame: new buffers, new keys
    t2 = pa.table({"k": pa.array(rng.integers(0, 50, n)), "v": pa.array(rng.standard_normal(n))})
    nt = FakeNT(t2)
    nt.p("DataFrameScan", ["k", "v"], df=FakePyDataFrame(t2), projection=None, selection=None)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    assert out.column("v").to_pylist() == t2.column("v").to_pylist() and c.misses == 4
    # device_cache_bytes = 0 turns the cache off
    nt = FakeNT(t2)
    nt.p("DataFrameScan", ["k", "v"], df=FakePyDataFrame(t2), projection=None, selection=None)
    PE.execute_with_polaroid(nt, None, config={"device_cache_bytes": 0}, to_frame=lambda t: t)
    assert nt.udf(None, None, None, False).column("k").to_pylist() == t2.column("k").to_pylist()
    PE.column_cache().capacity = 32 << 30


def _vwap_ir(table, select=False):
    """group_by("k").agg((v * w).sum(), (v - 1.0).mean(), when(w > 0).then(v).otherwise(0.0).sum())
    -- the aggregation inputs the reference pre-aggregates (general.rs:303-356
    can_pre_agg) -- or, with `select`, filter(w > 0).select(the same aggs, len())."""
    nt = FakeNT(table)
    scan = nt.p("DataFrameScan", ["k", "v", "w"], df=FakePolarsDF(table), projection=None, selection=None)
    vw = nt.bin(nt.col("v"), "Multiply", nt.col("w"))
    vm1 = nt.bin(nt.col("v"), "Minus", nt.lit(1.0))
    tern = nt.e("Ternary", predicate=nt.bin(nt.col("w"), "Gt", nt.lit(0)), truthy=nt.col("v"), falsy=nt.lit(0.0))
    a1 = nt.e("Agg", name="sum", arguments=[vw], options=None)
    a2 = nt.e("Agg", name="mean", arguments=[vm1], options=None)
    a3 = nt.e("Agg", name="sum", arguments=[tern], options=None)
    if select:
        filt = nt.p("Filter", ["k", "v", "w"], input=scan,
                    predicate=PyExprIR(nt.bin(nt.col("w"), "Gt", nt.lit(0)), "w"))
        nt.p("Select", ["vw", "vm1", "pos", "len"], input=filt,
             expr=[PyExprIR(a1, "vw"), PyExprIR(a2, "vm1"), PyExprIR(a3, "pos"), PyExprIR(nt.e("Len"), "len")])
        return nt
    opts = _node("GroupbyOptions", slice=None, dynamic=None, rolling=None)
    nt.p("GroupBy", ["k", "vw", "vm1", "pos"], input=scan, keys=[PyExprIR(nt.col("k"), "k")],
         aggs=[PyExprIR(a1, "vw"), PyExprIR(a2, "vm1"), PyExprIR(a3, "pos")], apply=None, maintain_order=True,
         options=opts)
    return nt


def test_translate_aggregations_over_expressions_and_select():
    table = _table()[0]
    plan = PE.translate(_vwap_ir(table))
    assert plan[0] == "group_by" and [a.output_name() for a in plan[3]] == ["vw", "vm1", "pos"]
    assert plan[3][0].args[0].args[0].kind == "bin"  # (v * w).sum(): an input expression
    plan = PE.translate(_vwap_ir(table, select=True))
    assert plan[0] == "select" and plan[1][0] == "filter"
    assert [a.output_name() for a in plan[2]] == ["vw", "vm1", "pos", "len"]
    # a select mixing aggregations and elementwise expressions stays on polars
    nt = _vwap_ir(table, select=True)
    nt.lp[nt.root].expr.append(PyExprIR(nt.col("v"), "v"))
    with pytest.raises(PE.Unsupported):
        PE.translate(nt)


def _typed_agg_ir(agg_name, arg, dtypes, select=True):
    """select(<agg>(arg)) or group_by("k").agg(<agg>(arg)) over a scan whose
    columns have the given polars dtypes; `arg` builds the argument node."""
    table = _table()[0]
    nt = FakeNT(table)
    nt.dtypes.update(dtypes)
    cols = ["k", "v", "w"] + [c for c in dtypes if c not in ("k", "v", "w")]
    scan = nt.p("DataFrameScan", cols, df=FakePolarsDF(table), projection=None, selection=None)
    a = nt.e("Agg", name=agg_name, arguments=[arg(nt)], options=None)
    if select:
        nt.p("Select", ["out"], input=scan, expr=[PyExprIR(a, "out")])
    else:
        opts = _node("GroupbyOptions", slice=None, dynamic=None, rolling=None)
        nt.p("GroupBy", ["k", "out"], input=scan, keys=[PyExprIR(nt.col("k"), "k")], aggs=[PyExprIR(a, "out")],
             apply=None, maintain_order=False, options=opts)
    return nt


@pytest.mark.parametrize("select", [True, False])
def test_aggregations_the_device_lacks_stay_on_polars(select):
    """Input dtypes the device aggregations do not take are refused at
    translate time, so polars runs those queries (no UDF, no collect-time
    error): min / max / first / last of Boolean (column or comparison),
    anything over String / Categorical, sum / mean of Datetime / Date, mean
    of Duration.  The supported neighbours still translate."""
    refused = [
        ("max", lambda nt: nt.col("b"), {"b": "Boolean"}),
        ("first", lambda nt: nt.col("b"), {"b": "Boolean"}),
        ("min", lambda nt: nt.bin(nt.col("v"), "Gt", nt.lit(0.5)), {}),
        ("min", lambda nt: nt.col("s"), {"s": "String"}),
        ("count", lambda nt: nt.col("s"), {"s": "Categorical"}),
        ("mean", lambda nt: nt.col("t"), {"t": "Datetime(time_unit='us', time_zone=None)"}),
        ("sum", lambda nt: nt.col("d"), {"d": "Date"}),
        ("mean", lambda nt: nt.col("u"), {"u": "Duration(time_unit='ns')"}),
    ]
    for name, arg, dt in refused:
        nt = _typed_agg_ir(name, arg, dt, select)
        with pytest.raises(PE.Unsupported):
            PE.translate(nt)
        PE.execute_with_polaroid(nt, None)
        assert nt.udf is None, (name, dt)
    accepted = [
        ("sum", lambda nt: nt.col("b"), {"b": "Boolean"}),
        ("mean", lambda nt: nt.bin(nt.col("v"), "Gt", nt.lit(0.5)), {}),
        ("max", lambda nt: nt.col("t"), {"t": "Datetime(time_unit='us', time_zone=None)"}),
        ("sum", lambda nt: nt.col("u"), {"u": "Duration(time_unit='ns')"}),
        ("sum", lambda nt: nt.col("v"), {}),
    ]
    for name, arg, dt in accepted:
        nt = _typed_agg_ir(name, arg, dt, select)
        PE.translate(nt)
        PE.execute_with_polaroid(nt, None)
        assert callable(nt.udf), (name, dt)


@pytest.mark.gpu
def test_udf_aggregations_over_expressions_on_gpu(gpu):
    table, k, v, w, vvalid = _table(100_000, 21)
    nt = _vwap_ir(table)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    keys = out.column("k").to_pylist()
    assert keys == list(dict.fromkeys(k.tolist()))
    for i, kk in enumerate(keys):
        m = (k == kk) & vvalid
        assert out.column("vw")[i].as_py() == math.fsum(v[m] * w[m])
        assert out.column("vm1")[i].as_py() == math.fsum(v[m] - 1.0) / int(m.sum())
        pos = np.where(w[k == kk] > 0, v[k == kk], 0.0)
        assert out.column("pos")[i].as_py() == math.fsum(pos[vvalid[k == kk]])
    nt = _vwap_ir(table, select=True)
    PE.execute_with_polaroid(nt, None, to_frame=lambda t: t)
    out = nt.udf(None, None, None, False)
    assert out.num_rows == 1
    sel = w > 0
    m = sel & vvalid
    assert out.column("vw")[0].as_py() == math.fsum(v[m] * w[m])
    assert out.column("len")[0].as_py() == int(sel.sum())
