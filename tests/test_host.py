"""CPU: host-side logic of the Python mirror (expression lowering, plan
shape, error behaviour) — nothing here touches the device."""

import pytest

import polaroid_amd as pl
from polaroid_amd import _native as N
from polaroid_amd.expr import lower


def test_lower_simple_comparison():
    prog = lower(pl.col("close") > 100.0, {"close": 0}, {"close": N.F64})
    assert prog == [(N.OP["COL"], 0, 0), (N.OP["LIT_F64"], 0, 100.0), (N.OP["GT"], 0, 0)]


def test_lower_arith_and_logic():
    e = ((pl.col("a") * 2 + pl.col("b")) / 3 >= 1) & ~pl.col("c").is_null()
    prog = lower(e, {"a": 0, "b": 1, "c": 2}, {"a": N.I64, "b": N.F64, "c": N.F64})
    ops = [p[0] for p in prog]
    assert ops == [N.OP[o] for o in ("COL", "LIT_I64", "MUL", "COL", "ADD", "LIT_I64", "TRUEDIV", "LIT_I64",
                                     "GE", "COL", "IS_NULL", "NOT", "AND")]


def test_null_literal_is_untyped():
    # the native lowering gives an untyped null the other operand's type
    prog = lower(pl.col("x") == None, {"x": 0}, {"x": N.F64})  # noqa: E711
    assert prog[1] == (N.OP["LIT_NULL"], 0, 0)


def test_reverse_operands():
    prog = lower(1.5 < pl.col("x"), {"x": 0}, {"x": N.F64})
    assert prog == [(N.OP["COL"], 0, 0), (N.OP["LIT_F64"], 0, 1.5), (N.OP["GT"], 0, 0)]


def test_unknown_column_is_compute_error():
    with pytest.raises(pl.ComputeError):
        lower(pl.col("nope") > 1, {}, {})


def test_agg_in_row_context_is_invalid():
    with pytest.raises(pl.InvalidOperationError):
        lower(pl.col("x").sum() > 1, {"x": 0}, {"x": N.F64})


def test_expr_truthiness_is_ambiguous():
    with pytest.raises(TypeError):
        bool(pl.col("a") > 1)


def test_output_names_follow_polars():
    assert (pl.col("a") + pl.col("b")).output_name() == "a"
    assert pl.col("a").sum().alias("s").output_name() == "s"
    assert pl.len().output_name() == "len"
    assert pl.sum("v").output_name() == "v"


def test_plan_pushes_filter_into_group_by():
    lf = pl.LazyFrame(("scan", pl.DataFrame({}))).filter(pl.col("close") > 1.0).group_by("sym").agg(
        pl.col("close").sum())
    text = lf.explain()
    assert text.splitlines()[0].startswith("AGGREGATE")
    assert "FILTER" in text


def test_group_by_key_validation():
    lf = pl.LazyFrame(("scan", pl.DataFrame({})))
    g = lf.group_by("a", "b")  # several keys: a tuple in the plan node
    assert g._key == ("a", "b")
    assert lf.group_by("a")._key == "a"
    with pytest.raises(pl.InvalidOperationError):
        lf.group_by(pl.col("a") + 1)
    with pytest.raises(pl.InvalidOperationError):
        lf.group_by(*[f"k{i}" for i in range(9)])
    with pytest.raises(pl.DuplicateError):
        lf.group_by("a", "a")
