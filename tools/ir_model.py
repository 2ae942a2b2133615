"""A minimal model of the reference's NodeTraverser for driving the plugin
without polars (which is not installed in this image): the IR / expression
node classes of crates/polars-python/src/lazyframe/visitor/{nodes,
expr_nodes}.rs with their class and attribute names, and the traverser
methods of crates/polars-python/src/lazyframe/visit.rs the plugin calls
(view_current_node, get_node, set_node, view_expression, get_schema,
set_udf).  `DataFrameScan.df` models PyDataFrame.to_arrow(compat_level)
(crates/polars-python/src/dataframe/export.rs:80-99): one RecordBatch per
chunk.  Used by bench.py's plugin leg; tests/test_polars_engine.py has the
fuller model its tests need.
"""

from __future__ import annotations


class _Enum:
    def __init__(self, cls: str, name: str):
        self.s = f"{cls}.{name}"

    def __str__(self):
        return self.s


def _node(kind: str, **kw):
    return type(kind, (), kw)()


class ExprIR:
    def __init__(self, node: int, output_name: str):
        self.node, self.output_name = node, output_name


class ArrowFrame:
    """PyDataFrame stand-in over a pyarrow Table cut into `chunk_rows` batches."""

    def __init__(self, table, chunk_rows: int | None = None):
        self.table, self.chunk_rows = table, chunk_rows

    def to_arrow(self, compat_level):
        return self.table.to_batches(max_chunksize=self.chunk_rows)


class _DType:
    def __init__(self, s: str):
        self.s = s

    def __str__(self):
        return self.s


class Traverser:
    def __init__(self, dtypes: dict[str, str]):
        self.lp, self.ex, self.schemas = [], [], []
        self.root = None
        self.udf = None
        self.dtypes = dtypes

    def e(self, kind: str, **kw) -> int:
        self.ex.append(_node(kind, **kw))
        return len(self.ex) - 1

    def p(self, kind: str, schema: list[str], **kw) -> int:
        self.lp.append(_node(kind, **kw))
        self.schemas.append(schema)
        self.root = len(self.lp) - 1
        return self.root

    def col(self, name: str) -> int:
        return self.e("Column", name=name)

    def lit(self, v) -> int:
        return self.e("Literal", value=v, dtype=None)

    def bin(self, left: int, op: str, right: int) -> int:
        return self.e("BinaryExpr", left=left, op=_Enum("Operator", op), right=right)

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
        return {k: _DType(self.dtypes[k]) for k in self.schemas[self.root]}

    def set_udf(self, fn, is_pure=False):
        self.udf = fn


def filter_group_by_sum(table, key: str, pred_col: str, threshold: float, sum_cols: list[str],
                        chunk_rows: int | None = None) -> Traverser:
    """IR of lf.filter(pred_col > threshold).group_by(key).agg(c.sum() for c in sum_cols)."""
    names = table.column_names
    nt = Traverser({f.name: {"int64": "Int64", "double": "Float64"}[str(f.type)] for f in table.schema})
    scan = nt.p("DataFrameScan", names, df=ArrowFrame(table, chunk_rows), projection=None, selection=None)
    pred = nt.bin(nt.col(pred_col), "Gt", nt.lit(threshold))
    filt = nt.p("Filter", names, input=scan, predicate=ExprIR(pred, pred_col))
    aggs = [ExprIR(nt.e("Agg", name="sum", arguments=[nt.col(c)], options=None), c) for c in sum_cols]
    opts = _node("GroupbyOptions", slice=None, dynamic=None, rolling=None)
    nt.p("GroupBy", [key] + sum_cols, input=filt, keys=[ExprIR(nt.col(key), key)], aggs=aggs, apply=None,
         maintain_order=False, options=opts)
    return nt
