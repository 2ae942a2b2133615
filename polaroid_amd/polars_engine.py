"""Polars GPU-engine plugin: `lf.collect(engine="gpu")` executed on MI355X.

The reference dispatches `collect(engine="gpu")` through a post-optimisation
callback (py-polars/src/polars/lazyframe/frame.py:208 `_gpu_engine_callback`,
which hands `cudf_polars.execute_with_cudf` to Rust; the callback receives a
`NodeTraverser` over the optimised IR, crates/polars-python/src/lazyframe/
general.rs:47 `post_opt_callback`).  The callback may replace the root
subtree with a Python UDF via `NodeTraverser.set_udf`
(crates/polars-python/src/lazyframe/visit.rs:158), which polars turns into a
`PythonScan` node that the in-memory engine calls as
`fn(with_columns, predicate, n_rows, should_time)`
(crates/polars-mem-engine/src/executors/scan/python_scan.rs:91).

`execute_with_polaroid` has the same signature and contract as
`execute_with_cudf`: it translates the IR (node classes of
crates/polars-python/src/lazyframe/visitor/nodes.rs, expression classes of
.../visitor/expr_nodes.rs) for the hot path — DataFrameScan, Filter,
Select/HStack of arithmetic + comparisons, GroupBy on one integer key with
sum/mean/min/max/count/len/first/last/std/var, inner / left / right / full / semi / anti Join
on 1..8 key columns, Sort by 1..8 columns — into a polaroid_amd plan and installs a UDF that
runs it through libpolaroid_gpu.so.  A query outside that path is left to
polars' own engine unless `raise_on_fail` is set (the reference GPU engine's
behaviour).  Once accepted, nothing falls back: a missing HIP library or a
device error raises.
"""

from __future__ import annotations

from typing import Any, Callable

from . import _native as N
from .expr import Expr, col, lit
from .frame import DataFrame, LazyFrame

__all__ = ["ColumnCache", "column_cache", "execute_with_polaroid", "Unsupported", "translate"]


class Unsupported(Exception):
    """The IR is outside the GPU hot path."""


def _name(obj) -> str:
    return type(obj).__name__


def _enum_name(v) -> str:
    s = str(v)
    return s.rsplit(".", 1)[-1]


_BINOPS: dict[str, Callable[[Expr, Expr], Expr]] = {
    "Eq": lambda a, b: a == b, "NotEq": lambda a, b: a != b, "Lt": lambda a, b: a < b,
    "LtEq": lambda a, b: a <= b, "Gt": lambda a, b: a > b, "GtEq": lambda a, b: a >= b,
    "EqValidity": lambda a, b: a.eq_missing(b), "NotEqValidity": lambda a, b: a.ne_missing(b),
    "Plus": lambda a, b: a + b, "Minus": lambda a, b: a - b, "Multiply": lambda a, b: a * b,
    "TrueDivide": lambda a, b: a / b, "And": lambda a, b: a & b, "Or": lambda a, b: a | b,
    "LogicalAnd": lambda a, b: a & b, "LogicalOr": lambda a, b: a | b,
    "FloorDivide": lambda a, b: a // b, "Modulus": lambda a, b: a % b, "Xor": lambda a, b: a ^ b,
    "Divide": lambda a, b: a._bin("div", b),  # Operator::Divide (legacy_div)
}

_ORDERED_CMP = frozenset({"Lt", "LtEq", "Gt", "GtEq"})

_BOOLFUNCS: dict[str, Callable[[Expr], Expr]] = {
    "IsNull": lambda a: a.is_null(), "IsNotNull": lambda a: a.is_not_null(), "IsNan": lambda a: a.is_nan(),
    "IsFinite": lambda a: a.is_finite(), "Not": lambda a: ~a,
}


def _dtype_kind(dt) -> str:
    """Name of a polars DataType as the visitor hands it over
    (`Int64`, `Datetime(time_unit='ns', time_zone=None)`, `Enum(categories=...)`)."""
    s = str(dt) if dt is not None else "?"
    return s.split("(", 1)[0].split("[", 1)[0].strip()


# dtypes whose columns the GPU path takes (anything else stays on polars)
SUPPORTED_DTYPES = frozenset({"Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32", "UInt64", "Float32",
                              "Float64", "Boolean", "String", "Categorical", "Enum", "Datetime", "Date",
                              "Duration"})


def _dtype_obj(dt):
    """A visitor dtype (its repr) -> polaroid_amd DataType, or None."""
    from . import frame as F

    kind = _dtype_kind(dt)
    if hasattr(F, kind) and isinstance(getattr(F, kind), F.DataType) and not kind.startswith("_"):
        return getattr(F, kind)
    s = str(dt)
    unit = next((u for u in ("ns", "us", "ms") if f"'{u}'" in s), None)
    if kind == "Datetime" and unit:
        tz = None
        if "time_zone=" in s:
            tzs = s.split("time_zone=", 1)[1].rstrip(")").strip()
            tz = None if tzs in ("None", "") else tzs.strip("'\"")
        return F.Datetime(unit, tz)
    if kind == "Duration" and unit:
        return F.Duration(unit)
    return None


class _Translator:
    def __init__(self, nt):
        self.nt = nt
        # Enum columns order by category index, not lexically (logical/
        # categorical.rs:58 uses_lexical_ordering; sort/categorical.rs:74):
        # the GPU handles them as strings, so ordered uses stay on polars
        self.enums: set[str] = set()

    # ---------------------------------------------------------- expressions
    def _is_enum(self, node: int) -> bool:
        e = self.view(node)
        return _name(e) == "Column" and str(e.name) in self.enums

    def view(self, node: int):
        try:
            return self.nt.view_expression(node)
        except NotImplementedError as exc:  # e.g. rolling expressions (expr_nodes.rs:1192)
            raise Unsupported(str(exc)) from exc

    def expr(self, node: int) -> Expr:
        e = self.view(node)
        k = _name(e)
        if k == "Column":
            return col(str(e.name))
        if k == "Literal":
            v = e.value
            import datetime as _dt

            if v is None or isinstance(v, (bool, int, float, str, _dt.date, _dt.timedelta)):
                # str: String comparisons; temporal values: converted against
                # the column they meet (frame._prepare).  A typed literal
                # (lit(1, dtype=Int8)) keeps its dtype through a cast.
                out = lit(v)
                dt = _dtype_obj(getattr(e, "dtype", None))
                if dt is not None and isinstance(v, (int, float)) and not isinstance(v, bool) \
                        and not _dtype_kind(getattr(e, "dtype", None)).startswith("Unknown") and not dt.logical:
                    out = out.cast(dt, strict=False)
                return out
            raise Unsupported(f"literal {v!r}")
        if k == "BinaryExpr":
            op = _enum_name(e.op)
            if op not in _BINOPS:
                raise Unsupported(f"operator {op}")
            if op in _ORDERED_CMP and (self._is_enum(e.left) or self._is_enum(e.right)):
                raise Unsupported("ordered comparison on an Enum column (category order)")
            return _BINOPS[op](self.expr(e.left), self.expr(e.right))
        if k == "Cast":
            # options: 0 strict, 1 non-strict, 2 overflowing (expr_nodes.rs:305)
            dt = _dtype_obj(e.dtype)
            if dt is None or dt is getattr(__import__("polaroid_amd.frame", fromlist=["String"]), "String"):
                raise Unsupported(f"cast to {e.dtype}")
            opt = int(getattr(e, "options", 0) or 0)
            return self.expr(e.expr).cast(dt, strict=opt == 0, wrap_numerical=opt == 2)
        if k == "Ternary":  # when(predicate).then(truthy).otherwise(falsy) (expr_nodes.rs:367)
            from .expr import when

            return when(self.expr(e.predicate)).then(self.expr(e.truthy)).otherwise(self.expr(e.falsy))
        if k == "Function":
            fd = e.function_data
            fname = _enum_name(fd[0]) if isinstance(fd, tuple) and fd else _enum_name(fd)
            if fname == "Abs":
                return abs(self.expr(e.input[0]))
            if fname == "Negate":
                return -self.expr(e.input[0])
            if fname in _BOOLFUNCS and len(e.input) == 1:
                return _BOOLFUNCS[fname](self.expr(e.input[0]))
            if fname == "fill_null" and len(e.input) == 2:  # FunctionExpr::FillNull (expr_nodes.rs:1191)
                return self.expr(e.input[0]).fill_null(self.expr(e.input[1]))
            if fname == "IsBetween" and len(e.input) == 3:  # (IsBetween, closed) (expr_nodes.rs:1112)
                closed = str(fd[1]) if isinstance(fd, tuple) and len(fd) > 1 else "both"
                return self.expr(e.input[0]).is_between(self.expr(e.input[1]), self.expr(e.input[2]), closed)
            if fname == "IsIn" and len(e.input) == 2:  # (IsIn, nulls_equal) (expr_nodes.rs:1116)
                other = self.view(e.input[1])
                vals = getattr(other, "value", None)
                if _name(other) != "Literal" or vals is None:
                    raise Unsupported("is_in over a non-literal collection")
                vals = vals.to_list() if hasattr(vals, "to_list") else list(vals)
                nulls_equal = bool(fd[1]) if isinstance(fd, tuple) and len(fd) > 1 else False
                try:
                    return self.expr(e.input[0]).is_in(vals, nulls_equal=nulls_equal)
                except N.InvalidOperationError as exc:
                    raise Unsupported(str(exc)) from exc
            raise Unsupported(f"function {fname}")
        raise Unsupported(f"expression {k}")

    def input_schema(self, input_node: int) -> dict:
        """Output schema of plan node `input_node` (visit.rs get_schema at that
        node); the traverser is restored."""
        here = self.nt.get_node()
        self.nt.set_node(input_node)
        try:
            return dict(self.nt.get_schema())
        finally:
            self.nt.set_node(here)

    _CMP_OPS = frozenset({"Eq", "NotEq", "Lt", "LtEq", "Gt", "GtEq", "EqValidity", "NotEqValidity"})
    _LOGIC_OPS = frozenset({"And", "Or", "LogicalAnd", "LogicalOr", "Xor"})

    def expr_kind(self, node: int, schema: dict) -> str:
        """The dtype kind an expression yields (`Boolean`, `String`, `Datetime`,
        `Duration`, ...; `?` when the translator cannot tell), enough to keep
        the aggregations the device path lacks on polars."""
        e = self.view(node)
        k = _name(e)
        if k == "Column":
            kind = _dtype_kind(schema.get(str(e.name)))
            return "String" if kind in ("Categorical", "Enum") else kind
        if k == "Literal":
            v = e.value
            return "Boolean" if isinstance(v, bool) else "String" if isinstance(v, str) else "?"
        if k == "Cast":
            return _dtype_kind(e.dtype)
        if k == "BinaryExpr":
            op = _enum_name(e.op)
            if op in self._CMP_OPS:
                return "Boolean"
            a, b = self.expr_kind(e.left, schema), self.expr_kind(e.right, schema)
            if op in self._LOGIC_OPS:
                return "Boolean" if "Boolean" in (a, b) else a
            if "Datetime" in (a, b) or "Date" in (a, b):
                # Datetime - Datetime = Duration, Datetime +- Duration = Datetime
                return "Duration" if op == "Minus" and a == b else ("Datetime" if "Datetime" in (a, b) else "Date")
            return "Duration" if "Duration" in (a, b) else "?"
        if k == "Ternary":
            return self.expr_kind(e.truthy, schema)
        if k == "Function":
            fd = e.function_data
            fname = _enum_name(fd[0]) if isinstance(fd, tuple) and fd else _enum_name(fd)
            if fname in _BOOLFUNCS or fname in ("IsBetween", "IsIn"):
                return "Boolean"
            if e.input:
                return self.expr_kind(e.input[0], schema)
        return "?"

    def agg(self, node: int, key: str | None, schema: dict | None = None) -> Expr:
        """IRAggExpr (expr_nodes.rs) -> an aggregation over a column or over an
        elementwise expression (the inputs the reference's partitionable
        group-by pre-aggregates, plans/aexpr/properties/general.rs:303-356
        can_pre_agg).  `key` None: a select of aggregations.  `schema` (the
        input node's) gates the input dtypes the device aggregations lack --
        String inputs, min / max / first / last of Boolean, sum / mean of
        Date / Datetime and mean of Duration -- so those queries stay on
        polars instead of failing at collect time."""
        e = self.view(node)
        k = _name(e)
        if k == "Len":
            if key is None:
                from .expr import len as len_

                return len_()
            return col(key).len()
        if k != "Agg":
            raise Unsupported(f"aggregation expression {k}")
        name = str(e.name)
        if len(e.arguments) != 1:
            raise Unsupported("multi-argument aggregation")
        if name in ("min", "max") and self._is_enum(e.arguments[0]):
            raise Unsupported(f"{name} of an Enum column (category order)")
        if schema is not None:
            kind = self.expr_kind(e.arguments[0], schema)
            if kind == "String":
                raise Unsupported(f"{name} of a String / Categorical input")
            if kind == "Boolean" and name in ("min", "max", "first", "last"):
                raise Unsupported(f"{name} of a Boolean input")
            if kind in ("Date", "Datetime", "Time") and name in ("sum", "mean", "std", "var"):
                raise Unsupported(f"{name} of a {kind} input")
            if kind == "Duration" and name in ("mean", "std", "var"):
                raise Unsupported(f"{name} of a Duration input")
        arg = self.nt.view_expression(e.arguments[0])
        if _name(arg) == "Column":
            c = col(str(arg.name))
            if name in ("min", "max") and str(arg.name) in self.enums:
                raise Unsupported(f"{name} of an Enum column (category order)")
        else:
            c = self.expr(e.arguments[0])  # raises Unsupported outside the elementwise path
        if name in ("sum", "mean"):
            return getattr(c, name)()
        if name in ("min", "max"):
            if e.options:  # propagate_nans=True (nan_min / nan_max)
                raise Unsupported(f"{name} with NaN propagation")
            return getattr(c, name)()
        if name == "count":
            return c.len() if e.options else c.count()
        if name in ("first", "last"):  # IRAggExpr::First / Last (expr_nodes.rs:677,687)
            return getattr(c, name)()
        if name in ("std", "var"):  # IRAggExpr::Std / Var, options = ddof (expr_nodes.rs:737,742)
            return getattr(c, name)(int(e.options))
        raise Unsupported(f"aggregation {name}")

    # ---------------------------------------------------------------- plans
    def plan(self) -> tuple:
        """Translate the subtree at the traverser's current node."""
        node = self.nt.view_current_node()
        k = _name(node)
        if k == "DataFrameScan":
            if getattr(node, "selection", None) is not None:
                raise Unsupported("scan predicate")
            proj = node.projection
            schema = dict(self.nt.get_schema())  # the scan's output schema (visit.rs get_schema)
            names = list(schema) if proj is None else list(proj)
            for nm in names:
                kind = _dtype_kind(schema.get(nm))
                if kind not in SUPPORTED_DTYPES:
                    raise Unsupported(f"column {nm!r} of dtype {schema.get(nm)}")
                if kind == "Enum":
                    self.enums.add(nm)
            return ("polars_scan", node.df, None if proj is None else list(proj), schema)
        if k == "Join":
            # options: (how, nulls_equal, slice, suffix, coalesce, maintain_order), nodes.rs:536
            how, nulls_equal, slc, suffix, coalesce, order = node.options
            if not isinstance(how, str) or how not in ("inner", "left", "right", "full", "semi", "anti"):
                raise Unsupported(f"{how} join")
            if slc is not None:
                raise Unsupported("join slice")
            if not 1 <= len(node.left_on) <= 8 or len(node.left_on) != len(node.right_on):
                raise Unsupported("join key count")
            names = []
            for side in (node.left_on, node.right_on):
                ks = [self.nt.view_expression(e.node) for e in side]
                if any(_name(x) != "Column" for x in ks):
                    raise Unsupported("join keys must be plain columns")
                ks = [str(x.name) for x in ks]
                names.append(ks[0] if len(ks) == 1 else tuple(ks))
            left = self.child(node.input_left)
            right = self.child(node.input_right)
            order = str(order).lower()
            # coalesce arrives resolved for the join type (JoinCoalesce::coalesce)
            return ("join", left, right, names[0], names[1], str(suffix), "m:m", bool(nulls_equal),
                    order if order in ("none", "left", "right", "left_right", "right_left") else "none",
                    how, bool(coalesce))
        if k == "Sort":
            if node.slice is not None:
                raise Unsupported("sort slice")
            if not 1 <= len(node.by_column) <= 8:
                raise Unsupported("sort by more than 8 columns")
            bys = [self.nt.view_expression(e.node) for e in node.by_column]
            if any(_name(b) != "Column" for b in bys):
                raise Unsupported("sort by an expression")
            _maintain, nulls_last, descending = node.sort_options
            k = len(bys)
            # the visitor gives one flag per column, or a single broadcast flag
            desc = [bool(descending[i if len(descending) == k else 0]) for i in range(k)]
            nl = [bool(nulls_last[i if len(nulls_last) == k else 0]) for i in range(k)]
            child = self.child(node.input)
            if any(str(b.name) in self.enums for b in bys):
                raise Unsupported("sort by an Enum column (category order)")
            if k == 1:
                return ("sort", child, str(bys[0].name), desc[0], nl[0])
            return ("sort", child, tuple(str(b.name) for b in bys), tuple(desc), tuple(nl))
        if k in ("Filter", "Select", "HStack", "GroupBy", "SimpleProjection"):
            child = self.child(node.input)
            if k == "Filter":
                return ("filter", child, self.expr(node.predicate.node))
            if k == "SimpleProjection":
                names = list(self.nt.get_schema().keys())
                return ("select", child, [col(n) for n in names])
            if k == "Select" and node.expr and all(_name(self.view(ei.node)) in ("Agg", "Len") for ei in node.expr):
                # select(aggregations): a global reduction on the GPU
                ins = self.input_schema(node.input)
                return ("select", child, [self.agg(ei.node, None, ins).alias(ei.output_name) for ei in node.expr])
            if k in ("Select", "HStack"):
                exprs = node.expr if k == "Select" else node.exprs
                out = []
                for ei in exprs:
                    x = self.expr(ei.node)
                    out.append(x if x.output_name() == ei.output_name else x.alias(ei.output_name))
                return ("select" if k == "Select" else "with_columns", child, out)
            # GroupBy
            opts = node.options
            if getattr(opts, "dynamic", None) is not None or getattr(opts, "rolling", None) is not None:
                raise Unsupported("dynamic / rolling group-by")
            if getattr(opts, "slice", None) is not None:
                raise Unsupported("group-by slice")
            if not 1 <= len(node.keys) <= 8:
                raise Unsupported("group-by on more than 8 keys")
            names = []
            for ki in node.keys:
                kx = self.nt.view_expression(ki.node)
                if _name(kx) != "Column" or str(kx.name) != ki.output_name:
                    raise Unsupported("group-by key must be a plain column")
                names.append(str(kx.name))
            key = names[0] if len(names) == 1 else tuple(names)
            aggs = []
            ins = self.input_schema(node.input)
            for ai in node.aggs:
                a = self.agg(ai.node, names[0], ins)
                aggs.append(a.alias(ai.output_name))
            return ("group_by", child, key, aggs, bool(node.maintain_order))
        raise Unsupported(f"plan node {k}")

    def child(self, input_node: int) -> tuple:
        here = self.nt.get_node()
        self.nt.set_node(input_node)
        try:
            return self.plan()
        finally:
            self.nt.set_node(here)


def translate(nt) -> tuple:
    """IR at `nt`'s current node -> polaroid_amd plan tuple (raises Unsupported)."""
    return _Translator(nt).plan()


# PyDataFrame.to_arrow(compat_level): 0 / False = CompatLevel::oldest, whose
# export uses large_string / large_binary instead of the view types
# (crates/polars-python/src/conversion/mod.rs:1559 PyCompatLevel).
_COMPAT_OLDEST = False


def scan_batches(df) -> list:
    """RecordBatches of a DataFrameScan's frame.  In the reference
    `DataFrameScan.df` is a PyDataFrame (visitor/nodes.rs:190) whose
    `to_arrow(compat_level)` returns one RecordBatch per chunk
    (dataframe/export.rs:80-99); a wrapped polars DataFrame is unwrapped to
    its PyDataFrame first (wrap_df's inverse, py-polars/src/polars/_utils/
    wrap.py:12)."""
    pydf = getattr(df, "_df", df)
    return list(pydf.to_arrow(_COMPAT_OLDEST))


class ColumnCache:
    """Device-resident scan columns, so repeated queries over the same frame
    do not re-upload it over the host link.

    A column's key is its Arrow type and the (address, size) of every buffer
    of every chunk, plus each chunk's offset and length: polars exports a
    primitive column zero-copy, so an unchanged frame gives the same key.
    The entry holds a reference to the chunks, so their host memory cannot
    be freed and reused by other data while the entry lives (no false hit);
    polars' buffers are immutable (a write to a shared buffer copies it).
    Entries are evicted least recently used beyond `capacity` bytes."""

    def __init__(self, capacity: int = 32 << 30):
        from collections import OrderedDict

        self.capacity = capacity
        self._d: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.bytes = 0
        self.hits = 0
        self.misses = 0

    @staticmethod
    def key(chunks: list, atype) -> tuple:
        parts: list = [str(atype)]
        for c in chunks:
            bufs = list(c.buffers())
            if hasattr(c, "dictionary"):  # Categorical / Enum: the dictionary's buffers too
                bufs += list(c.dictionary.buffers())
            parts.append((c.offset, len(c), tuple(None if b is None else (b.address, b.size) for b in bufs)))
        return tuple(parts)

    def get(self, key: tuple):
        e = self._d.get(key)
        if e is None:
            self.misses += 1
            return None
        self._d.move_to_end(key)
        self.hits += 1
        return e[0]

    def put(self, key: tuple, series, chunks: list, nbytes: int) -> None:
        if nbytes > self.capacity:
            return
        self._d[key] = (series, chunks, nbytes)
        self.bytes += nbytes
        self._evict()

    def _evict(self) -> None:
        while self.bytes > self.capacity and self._d:
            _, (_, _, nb) = self._d.popitem(last=False)
            self.bytes -= nb

    def resize(self, capacity: int) -> None:
        """New capacity in bytes; entries beyond it are released now (their
        device memory returns to the pool), least recently used first."""
        self.capacity = max(0, int(capacity))
        self._evict()

    def clear(self) -> None:
        self._d.clear()
        self.bytes = 0
        self.hits = 0
        self.misses = 0


_COLUMN_CACHE = ColumnCache()


def column_cache() -> ColumnCache:
    return _COLUMN_CACHE


def _scan_frame(batches: list, names: list, cache: "ColumnCache | None") -> DataFrame:
    """The projected columns of the scanned batches on the device, each
    taken from the resident cache or ingested chunk by chunk."""
    from .frame import _ingest_chunks

    cols = []
    for nm in names:
        i = batches[0].schema.get_field_index(nm)
        if i < 0:
            raise N.ComputeError(f"column {nm!r} not found in the scanned batches")
        atype = batches[0].schema.field(i).type
        chunks = [b.column(i) for b in batches]
        key = ColumnCache.key(chunks, atype) if cache is not None else None
        s = cache.get(key) if cache is not None else None
        if s is None:
            s = _ingest_chunks(nm, chunks, atype, sync=False)
            if cache is not None:
                cache.put(key, s, chunks, sum(c.nbytes for c in chunks))
        cols.append(s.alias(nm))
    N.check(N.lib().plgpu_synchronize(None))  # every column's copies issued: one wait
    return DataFrame(cols)


def _bind_scans(node: tuple, cache: "ColumnCache | None" = None) -> tuple:
    """Upload the scanned frames (RecordBatch chunks -> HBM), or find their
    columns resident in `cache`."""
    if node[0] == "polars_scan":
        _, df, proj, schema = node
        batches = scan_batches(df)
        names = proj if proj is not None else list(schema)
        if not batches:
            return ("scan", _empty_frame(names, schema))
        return ("scan", _scan_frame(batches, names, cache))
    if node[0] == "join":
        return (node[0], _bind_scans(node[1], cache), _bind_scans(node[2], cache)) + tuple(node[3:])
    return (node[0], _bind_scans(node[1], cache)) + tuple(node[2:])


def _empty_frame(names: list, schema: dict) -> DataFrame:
    """A zero-row frame with the scan's dtypes (to_arrow gives no batch)."""
    import pyarrow as pa

    from .frame import Series, _arrow_logical

    cols = []
    for nm in names:
        kind = _dtype_kind(schema.get(nm))
        dt = _dtype_obj(schema.get(nm))
        if kind in ("Categorical", "Enum"):
            t = pa.large_string()
        elif dt is not None:
            t = _arrow_logical(dt)
        else:
            raise Unsupported(f"column {nm!r} of dtype {schema.get(nm)}")
        cols.append(Series.from_arrow(nm, pa.array([], t)))
    return DataFrame(cols)


def _to_polars(table):
    import polars  # the caller is polars itself, so it is importable there

    return polars.from_arrow(table)


def run_plan(plan: tuple, n_rows: int | None = None, to_frame=None, cache: "ColumnCache | None" = None):
    """Execute a translated plan on the GPU; returns a polars DataFrame (or
    whatever `to_frame` makes of the result's Arrow table)."""
    N.lib()  # fail loudly when the HIP library is missing
    lf = LazyFrame(_bind_scans(plan, cache))
    out = lf.collect()
    table = out.to_arrow()
    if n_rows is not None:
        table = table.slice(0, n_rows)
    return (to_frame or _to_polars)(table)


def _restore_dtypes(df, schema: dict):
    """Categorical / Enum columns run on the GPU as their strings (the
    dictionary gathered on the device); the result gets the dtype the plan's
    schema names back."""
    cols = getattr(df, "columns", None)
    if not schema or cols is None or not hasattr(df, "with_columns"):
        return df
    casts = []
    for name, dt in schema.items():
        if name in cols and str(dt).startswith(("Categorical", "Enum")) and str(df.schema[name]) != str(dt):
            import polars

            casts.append(polars.col(name).cast(dt))
    return df.with_columns(casts) if casts else df


def _config_flag(config: Any, name: str, default: bool = False) -> bool:
    """Read a flag from a polars GPUEngine (attribute) or a plain dict."""
    if config is None:
        return default
    if isinstance(config, dict):
        return bool(config.get(name, default))
    return bool(getattr(config, name, default))


def execute_with_polaroid(nt, duration_since_start: int | None = None, *, config: Any = None,
                          to_frame=None) -> None:
    """Post-optimisation callback with `cudf_polars.execute_with_cudf`'s
    signature.  Installs a GPU UDF at the root when the query is on the hot
    path; otherwise leaves the plan untouched (or raises with
    `raise_on_fail`)."""
    try:
        plan = translate(nt)
        schema = dict(nt.get_schema()) if hasattr(nt, "get_schema") else {}
    except Unsupported as exc:
        if _config_flag(config, "raise_on_fail"):
            raise N.InvalidOperationError(f"query is not supported by the MI355X engine: {exc}") from exc
        return
    N.lib()  # a GPU plan was accepted: the HIP library must be present
    # scanned columns stay resident between queries unless the engine config
    # sets device_cache_bytes = 0 (any other value resizes the cache)
    cache_bytes = None
    if isinstance(config, dict):
        cache_bytes = config.get("device_cache_bytes")
    elif config is not None:
        cache_bytes = getattr(config, "device_cache_bytes", None)
    cache = _COLUMN_CACHE
    if cache_bytes is not None:
        cache.resize(int(cache_bytes))
        if cache.capacity <= 0:
            cache.clear()
            cache = None

    def _udf(with_columns, predicate, n_rows, should_time=False):
        try:
            res = run_plan(plan, n_rows, to_frame, cache)
        except N.OutOfMemoryError:
            if cache is None or not len(cache._d):
                raise
            # resident columns of earlier queries hold the memory this one
            # needs: release them and run once more (scans re-upload)
            cache.clear()
            res = run_plan(plan, n_rows, to_frame, cache)
        df = _restore_dtypes(res, schema)
        if with_columns is not None:
            df = df.select(with_columns)
        if should_time:
            return df, []
        return df

    nt.set_udf(_udf)
