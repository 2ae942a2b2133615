"""Generate the golden fixtures in tests/golden/ from the reference's own tests.

The reference (polars, Rust + py-polars) cannot be built or imported in this
image (no rustc; `import polars` fails), so each fixture transcribes the
inputs and expected outputs a reference test asserts, citing the test by
file:line (paths relative to /root/reference/py-polars/tests/unit).  Floats
are stored as float.hex() strings so NaN / -0.0 / inf survive JSON exactly;
None is null.

    python tests/golden/make_golden.py      # rewrites the *.json files
"""

from __future__ import annotations

import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def fx(v):
    """Encode a value: floats as hex strings, everything else as-is."""
    if isinstance(v, float):
        return v.hex()
    if isinstance(v, list):
        return [fx(x) for x in v]
    return v


# ---------------------------------------------------------------------------
# 1. Total-order comparison truth table.
#    operations/test_comparison.py:206-245 states the rule the reference is
#    checked against: "normal < nan, nan == nan, nulls propagate" for the
#    plain operators and "null < normal < nan, nan == nan, null == null" for
#    eq_missing / ne_missing; :340-350 lists INTERESTING_FLOAT_VALUES and
#    :353-370 runs every (lhs, rhs) pair as `pl.col("l") <op> rhs`.
INTERESTING = [0.0, -0.0, -1.0, 1.0, -float("nan"), float("nan"), -float("inf"), float("inf"), None]


def _ordering(lhs, rhs, missing):
    if lhs is None or rhs is None:
        if not missing:
            return None
        if lhs is None and rhs is None:
            return "="
        return "<" if lhs is None else ">"
    ln, rn = math.isnan(lhs), math.isnan(rhs)
    if ln and rn:
        return "="
    if ln or lhs > rhs:
        return ">"
    if rn or lhs < rhs:
        return "<"
    return "="


def compare_table():
    rows = []
    for lhs in INTERESTING:
        for rhs in INTERESTING:
            ref = _ordering(lhs, rhs, False)
            miss = _ordering(lhs, rhs, True)
            exp = {
                "eq": None if ref is None else ref == "=",
                "ne": None if ref is None else ref != "=",
                "lt": None if ref is None else ref == "<",
                "le": None if ref is None else ref in "<=",
                "gt": None if ref is None else ref == ">",
                "ge": None if ref is None else ref in ">=",
                "eq_missing": miss == "=",
                "ne_missing": miss != "=",
            }
            rows.append({"lhs": fx(lhs), "rhs": fx(rhs), "expected": exp})
    return {"source": "py-polars/tests/unit/operations/test_comparison.py:206-245,340-370",
            "cases": rows}


# ---------------------------------------------------------------------------
# 2. Group-by cases with the expected outputs the reference asserts.
#    Keys that the reference test writes as strings are mapped to Int64
#    codes in first-occurrence order (the path under test groups integer
#    keys); the code -> label map is kept in "key_labels".
def group_by_cases():
    cases = []
    cases.append({
        "name": "test_group_by_sum",
        "source": "operations/test_group_by.py:30-51",
        "key": [0, 1, 0, 1, 1, 2], "key_labels": ["a", "b", "c"],
        "cols": {"b": {"dtype": "i64", "values": [1, 2, 3, 4, 5, 6]}},
        "aggs": [["sum", "b"]], "maintain_order": True,
        "expected": {"key": [0, 1, 2], "b": [4, 11, 6]},
    })
    cases.append({
        "name": "test_group_by_count",
        "source": "operations/test_group_by.py:53-67",
        "key": [0, 0, 1, 1, 1], "key_labels": ["a", "b"],
        "cols": {"a": {"dtype": "i64", "values": [1, 2, 3, 4, 5]}},
        "aggs": [["count", "a"]], "maintain_order": True,
        "expected": {"key": [0, 1], "a": [2, 3]},
    })
    cases.append({
        "name": "test_group_by_mean_by_dtype[Float64]",
        "source": "operations/test_group_by.py:80,141-160",
        "key": [0, 0, 0, 1], "key_labels": ["a", "b"],
        "cols": {"Float64": {"dtype": "f64", "values": fx([1.0, 2.0, 3.0, 4.0])}},
        "aggs": [["mean", "Float64"]], "maintain_order": True,
        "expected": {"key": [0, 1], "Float64": fx([2.0, 4.0])},
    })
    cases.append({
        "name": "test_group_by_mean_by_dtype[Int64-like]",
        "source": "operations/test_group_by.py:73-79,141-160",
        "key": [0, 0, 0, 1], "key_labels": ["a", "b"],
        "cols": {"Int64": {"dtype": "i64", "values": [1, 2, 3, 4]}},
        "aggs": [["mean", "Int64"]], "maintain_order": True,
        "expected": {"key": [0, 1], "Int64": fx([2.0, 4.0])},
    })
    a = [1] * 10 + [2] * 10 + [3] * 10
    b = [1] * 10 + [None] * 20
    cases.append({
        "name": "test_partitioned_group_by_nulls_mean_21838",
        "source": "operations/test_group_by.py:1109-1117",
        "key": a,
        "cols": {"b": {"dtype": "i64", "values": b}},
        "aggs": [["mean", "b"]], "maintain_order": False, "sort_by_key": True,
        "expected": {"key": [1, 2, 3], "b": fx([1.0, None, None])},
    })
    nan, inf = float("nan"), float("inf")
    groups = ["both nan", "both nan", "nan and 5", "nan and 5", "nan and null", "nan and null",
              "both none", "both none", "both inf", "both inf", "inf and null", "inf and null"]
    labels = list(dict.fromkeys(groups))
    vals = [nan, nan, nan, 5.0, nan, None, None, None, inf, inf, inf, None]
    cases.append({
        "name": "test_nan_inf_aggregation",
        "source": "operations/aggregation/test_aggregations.py:523-560",
        "key": [labels.index(g) for g in groups], "key_labels": labels,
        "cols": {"value": {"dtype": "f64", "values": fx(vals)}},
        "aggs": [["min", "value", "min"], ["max", "value", "max"], ["mean", "value", "mean"]],
        "maintain_order": True,
        "expected": {
            "key": list(range(6)),
            "min": fx([nan, 5.0, nan, None, inf, inf]),
            "max": fx([nan, 5.0, nan, None, inf, inf]),
            "mean": fx([nan, nan, nan, None, inf, inf]),
        },
    })
    cases.append({
        "name": "test_group_by_wildcard (first)",
        "source": "operations/test_group_by.py:760-770 (keys a == b, so one key is equivalent)",
        "key": [1, 2],
        "cols": {"a": {"dtype": "i64", "values": [1, 2]}},
        "aggs": [["first", "a", "a_agg"]], "maintain_order": True,
        "expected": {"key": [1, 2], "a_agg": [1, 2]},
    })
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 2b. Multi-key group-by cases.  String / date keys of the reference tests are
#     label-encoded into integers (tuple equality is unchanged by a
#     bijection); a list aggregation (`agg(pl.col("c"))`) is checked through
#     its per-group lengths (`len`).
def group_by_multi_cases():
    cases = []
    cases.append({
        "name": "test_nan_in_group_by_agg",
        "source": "datatypes/test_float.py:8-18",
        "keys": {"bar": {"dtype": "i64", "values": [0, 0, 0, 0]},
                 "key": {"dtype": "i64", "values": [0, 0, 0, 0], "labels": ["a"]}},
        "cols": {"value": {"dtype": "f64", "values": fx([18.58, 18.78, float("nan"), 18.63])}},
        "aggs": [["max", "value", "max"], ["min", "value", "min"]], "maintain_order": False,
        "expected": {"bar": [0], "key": [0], "max": fx([18.78]), "min": fx([18.58])},
    })
    cases.append({
        "name": "test_group_by_partitioned_ending_cast",
        "source": "operations/test_group_by.py:968-973",
        "keys": {"a": {"dtype": "i64", "values": [1] * 5}, "b": {"dtype": "i64", "values": [1] * 5}},
        "cols": {"a": {"dtype": "i64", "values": [1] * 5}},
        "aggs": [["len", "a", "num"]], "maintain_order": False,
        "expected": {"a": [1], "b": [1], "num": [5]},
    })
    cases.append({
        "name": "test_group_by_with_null",
        "source": "operations/test_group_by.py:1080-1089",
        "keys": {"a": {"dtype": "i64", "values": [None, None, None, None]},
                 "b": {"dtype": "i64", "values": [1, 1, 2, 2]}},
        "cols": {"c": {"dtype": "i64", "values": [0, 1, 2, 3], "labels": ["x", "y", "z", "u"]}},
        "aggs": [["len", "c", "c_len"]], "maintain_order": True,
        "expected": {"a": [None, None], "b": [1, 2], "c_len": [2, 2]},
    })
    cases.append({
        "name": "test_streaming_literal_group_by_mean",
        "source": "streaming/test_streaming.py:100-118",
        "keys": {"x": {"dtype": "i64", "values": [0, 0], "labels": ["constant"]},
                 "y": {"dtype": "i64", "values": [0, 1], "labels": ["a", "b"]}},
        "cols": {"z": {"dtype": "i64", "values": [1, 2]}},
        "aggs": [["mean", "z", "z"]], "maintain_order": False, "sort_by": "y",
        "expected": {"x": [0, 0], "y": [0, 1], "z": fx([1.0, 2.0])},
    })
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 3. Filter cases.
def filter_cases():
    cases = []
    cases.append({
        "name": "test_simplify_expression_lit_true_4376",
        "source": "operations/test_filter.py:17-25",
        # pl.DataFrame([[1, 4, 7], [2, 5, 8], [3, 6, 9]]) builds columns from the inner lists
        "cols": {"column_0": [1, 4, 7], "column_1": [2, 5, 8], "column_2": [3, 6, 9]},
        "predicate": "lit(True) | (col('column_0') == 1)",
        "expected_rows": [[1, 2, 3], [4, 5, 6], [7, 8, 9]],
    })
    cases.append({
        "name": "test_binary_simplification_5971",
        "source": "operations/test_filter.py:157-164",
        "cols": {"a": [1, 2, 3, 4]},
        "predicate": "(col('a') > 2) | lit(False)",
        "expected_mask": [False, False, True, True],
    })
    cases.append({
        "name": "test_filter_19771",
        "source": "operations/test_filter.py:314-316",
        "cols": {"a": [None, None]},
        "predicate": "lit(True)",
        "expected_rows": [[None], [None]],
    })
    cases.append({
        "name": "test_filter_on_empty[Int32]",
        "source": "operations/test_filter.py:93-110",
        "cols": {"a": []},
        "predicate": "col('a').is_null()",
        "expected_rows": [],
    })
    cases.append({
        "name": "test_filter_horizontal_selector_15428",
        "source": "operations/test_filter.py:262-266",
        "cols": {"a": [1, 2, 3]},
        "predicate": "col('a') <= 2",
        "expected_rows": [[1], [2]],
    })
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 4. Inner joins on one integer key (operations/test_join.py).  Each case:
#    left / right columns, the join arguments, and what the test asserts:
#    `expected` rows (as a multiset unless `ordered`), `expected_height`, or
#    `raises` for a validation error.
def join_cases():
    cases = []
    cases.append({
        "name": "test_join_negative_integers",
        "source": "operations/test_join.py:129-151",
        "left": {"a": [-1, -6, -3, 0]},
        "right": {"a": [-6, -1, -4, -2, 0], "b": [-6, -1, -4, -2, 0]},
        "on": "a", "args": {},
        "expected": {"a": [-6, -1, 0], "b": [-6, -1, 0]}, "ordered": False,
    })
    for order, exp in (("left", [2, 1, 1, 1, 1]), ("right", [1, 1, 1, 1, 2])):
        cases.append({
            "name": f"test_join_preserve_order_inner[{order}]",
            "source": "operations/test_join.py:1284-1305",
            "left": {"a": [None, 2, 1, 1, 5]},
            "right": {"a": [1, 1, None, 2], "b": [6, 7, 8, 9]},
            "on": "a", "args": {"maintain_order": order},
            "expected_column": {"a": exp},
        })
    for order in ("none", "left_right", "right_left"):
        cases.append({
            "name": f"test_join_null_equal[{order}] with_null",
            "source": "operations/test_join.py:1916-1931",
            "left": {"x": [1, None, None], "y": [1, 2, 3]},
            "right": {"x": [1, None], "z": [1, 2]},
            "on": "x", "args": {"nulls_equal": True, "maintain_order": order},
            "expected": {"x": [1, None, None], "y": [1, 2, 3], "z": [1, 2, 2]},
            "ordered": order != "none",
        })
    cases.append({
        "name": "test_join_null_equal without_null",
        "source": "operations/test_join.py:1932-1935",
        "left": {"x": [1, None, None], "y": [1, 2, 3]},
        "right": {"x": [1, 3], "z": [1, 3]},
        "on": "x", "args": {"nulls_equal": True},
        "expected": {"x": [1], "y": [1], "z": [1]}, "ordered": True,
    })
    # joining on four identical columns == joining on one of them
    col = [None if a % 6 == 0 else a for a in range(138)]
    for neq, h in ((True, 644), (False, 115)):
        cases.append({
            "name": f"test_join_4_columns_with_validity[nulls_equal={neq}]",
            "source": "operations/test_join.py:978-997 (b = c = d = a, so one key is equivalent)",
            "left": {"a": col}, "right": {"a": col},
            "on": "a", "args": {"nulls_equal": neq},
            "expected_height": h,
        })
    cases.append({
        "name": "test_join eager a=foo",
        "source": "operations/test_join.py:268-279 (integer key columns only)",
        "left": {"a": [1, 2, 1, 1]}, "right": {"foo": [1, 1, 1]},
        "left_on": "a", "right_on": "foo", "args": {},
        "expected_height": 9,
    })
    # validation: (unique, duplicate) frames of the test, on "id"
    frames = {
        "short_unique": [1, 2, 3, 4], "short_duplicate": [1, 2, 3, 1],
        "long_unique": [1, 2, 3, 4, 5], "long_duplicate": [1, 2, 3, 1, 5],
    }
    for u, d in (("long_unique", "long_duplicate"), ("long_unique", "short_duplicate"),
                 ("short_unique", "long_duplicate")):
        for left, right, validate, raises in (
                (u, d, "1:m", False), (d, u, "1:m", True), (u, d, "1:1", True), (d, u, "1:1", True),
                (u, d, "m:1", True), (d, u, "m:1", False), (d, u, "m:m", False), (u, d, "m:m", False)):
            cases.append({
                "name": f"test_join_validation[{left} x {right}, {validate}]",
                "source": "operations/test_join.py:713-796",
                "left": {"id": frames[left]}, "right": {"id": frames[right]},
                "on": "id", "args": {"validate": validate},
                "raises": raises,
            })
    cases.append({
        "name": "test_join_empties[inner]",
        "source": "operations/test_join.py:1079-1084",
        "left": {"col2": []}, "right": {"col2": []},
        "on": "col2", "args": {},
        "expected_height": 0,
    })
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 4b. Multi-key inner joins (string columns label-encoded into integers).
def join_multi_cases():
    cases = []
    col = [None if a % 6 == 0 else a for a in range(138)]
    for neq, h in ((True, 644), (False, 115)):
        cases.append({
            "name": f"test_join_4_columns_with_validity[nulls_equal={neq}]",
            "source": "operations/test_join.py:975-995",
            "left": {"a": col, "b": col, "c": col, "d": col},
            "right": {"a": col, "b": col, "c": col, "d": col},
            "on": ["a", "b", "c", "d"], "args": {"nulls_equal": neq},
            "expected_height": h, "expected_width": 4,
        })
    cases.append({
        "name": "test_join_concat_projection_pd_case_7071 (join part)",
        "source": "operations/test_join.py:660-670",
        "left": {"id": [1, 2], "value": [100, 200]},
        "right": {"id": [1, 3], "value": [100, 300]},
        "on": ["id", "value"], "args": {},
        "expected": {"id": [1], "value": [100]},
    })
    cases.append({
        "name": "test_join_filter_pushdown_inner_join",
        "source": "operations/test_join.py:2179-2200",
        "left": {"a": [1, 2, 3, 4, 5], "b": [1, 2, 3, 4, None], "c": [0, 1, 2, 3, 4]},
        "right": {"a": [1, 2, 3, 4, 5], "b": [1, 2, 3, None, 5], "c": [0, 1, 2, 3, 4]},
        "labels": {"c": ["a", "b", "c", "d", "e"], "c_right": ["A", "B", "C", "D", "E"]},
        "on": ["a", "b"], "args": {"maintain_order": "left_right"},
        "post_filter": ["b", "<=", 2],
        "expected": {"a": [1, 2], "b": [1, 2], "c": [0, 1], "c_right": [0, 1]},
    })
    return {"cases": cases}

# ---------------------------------------------------------------------------
# 4c. Left / right / full / semi / anti joins (operations/test_join.py).
#     String payloads and nested keys are label-encoded into integers (the
#     encoding keeps equality and order, which is all the joins look at).
#     Each case: left / right columns, `on` (one name or a list), `how`,
#     `args`, and `expected` columns compared in order when `ordered`
#     (first `prefix` rows only when the test slices), as a multiset of
#     rows otherwise; `columns` = the asserted output column order.
def join_types_cases():
    cases = []
    # test_semi_anti_join: payload ["f", "i", None] -> [0, 1, None]
    la = {"key": [1, 2, 3], "payload": [0, 1, None]}
    rb = {"key": [3, 4, 5, None]}
    for how, exp in (("anti", {"key": [1, 2], "payload": [0, 1]}), ("semi", {"key": [3], "payload": [None]})):
        cases.append({"name": f"test_semi_anti_join[{how}]", "source": "operations/test_join.py:27-48",
                      "left": la, "right": rb, "on": "key", "how": how, "args": {},
                      "expected": exp, "ordered": True, "columns": ["key", "payload"]})
    # b: ["a", "b", "c", "a"] / ["c", "c", "d", "e"] -> a=0, b=1, c=2, d=3, e=4
    la = {"a": [1, 2, 3, 1], "b": [0, 1, 2, 0], "payload": [10, 20, 30, 40]}
    rb = {"a": [3, 3, 4, 5], "b": [2, 2, 3, 4]}
    for how, exp in (("anti", {"a": [1, 2, 1], "b": [0, 1, 0], "payload": [10, 20, 40]}),
                     ("semi", {"a": [3], "b": [2], "payload": [30]})):
        cases.append({"name": f"test_semi_anti_join multi-key[{how}]", "source": "operations/test_join.py:50-65",
                      "left": la, "right": rb, "on": ["a", "b"], "how": how, "args": {},
                      "expected": exp, "ordered": True, "columns": ["a", "b", "payload"]})
    # test_join_sorted_fast_paths_null
    l1 = {"x": [0, 0, 1]}
    r1 = {"x": [0, None], "y": [0, 1]}
    for how, exp, cols in (("inner", {"x": [0, 0], "y": [0, 0]}, ["x", "y"]),
                           ("left", {"x": [0, 0, 1], "y": [0, 0, None]}, ["x", "y"]),
                           ("anti", {"x": [1]}, ["x"]),
                           ("semi", {"x": [0, 0]}, ["x"]),
                           ("full", {"x": [0, 0, 1, None], "x_right": [0, 0, None, None], "y": [0, 0, None, 1]},
                            ["x", "x_right", "y"])):
        cases.append({"name": f"test_join_sorted_fast_paths_null[{how}]", "source": "operations/test_join.py:674-691",
                      "left": l1, "right": r1, "on": "x", "how": how, "args": {},
                      "expected": exp, "ordered": how != "full", "columns": cols})
    # test_join_preserve_order_left / _full
    l2 = {"a": [None, 2, 1, 1, 5]}
    r2 = {"a": [1, None, 2, 6], "b": [6, 7, 8, 9]}
    for how, order, col, exp, prefix in (
            ("left", "none", "a", [None, 2, 1, 1, 5], None),
            ("left", "left", "a", [None, 2, 1, 1, 5], None),
            ("left", "left_right", "a", [None, 2, 1, 1, 5], None),
            ("left", "right", "a", [1, 1, 2, None, 5], 5),
            ("left", "right_left", "a", [1, 1, 2, None, 5], None),
            ("right", "left", "a", [2, 1, 1, None, 6], None),
            ("right", "right", "a", [1, 1, None, 2, 6], None),
            ("full", "left", "a", [None, 2, 1, 1, 5], 5),
            ("full", "right", "a", [1, 1, None, 2, None], 5),
            ("full", "left_right", "a_right", [None, 2, 1, 1, None, None, 6], None),
            ("full", "right_left", "a", [1, 1, None, 2, None, None, 5], None)):
        src = "operations/test_join.py:1311-1373" if how != "full" else "operations/test_join.py:1376-1421"
        case = {"name": f"test_join_preserve_order_{'full' if how == 'full' else 'left'}[{how}, {order}]",
                "source": src, "left": l2, "right": r2, "on": "a", "how": how,
                "args": {"maintain_order": order}, "expected": {col: exp}, "ordered": True}
        if prefix:
            case["prefix"] = prefix
        cases.append(case)
    # test_join_null_equal: left and full parts
    lhs = {"x": [1, None, None], "y": [1, 2, 3]}
    with_null = {"x": [1, None], "z": [1, 2]}
    without_null = {"x": [1, 3], "z": [1, 3]}
    for order in ("none", "left_right", "right_left"):
        src = "operations/test_join.py:1933-1985"
        cases.append({"name": f"test_join_null_equal[{order}] left with_null", "source": src,
                      "left": lhs, "right": with_null, "on": "x", "how": "left",
                      "args": {"nulls_equal": True, "maintain_order": order},
                      "expected": {"x": [1, None, None], "y": [1, 2, 3], "z": [1, 2, 2]},
                      "ordered": order != "none"})
        cases.append({"name": f"test_join_null_equal[{order}] left without_null", "source": src,
                      "left": lhs, "right": without_null, "on": "x", "how": "left",
                      "args": {"nulls_equal": True, "maintain_order": order},
                      "expected": {"x": [1, None, None], "y": [1, 2, 3], "z": [1, None, None]},
                      "ordered": order != "none"})
        cases.append({"name": f"test_join_null_equal[{order}] full coalesce with_null", "source": src,
                      "left": lhs, "right": with_null, "on": "x", "how": "full",
                      "args": {"nulls_equal": True, "coalesce": True, "maintain_order": order},
                      "expected": {"x": [1, None, None], "y": [1, 2, 3], "z": [1, 2, 2]},
                      "ordered": order != "none"})
        if order == "left_right":
            exp = {"x": [1, None, None, None], "x_right": [1, None, None, 3], "y": [1, 2, 3, None],
                   "z": [1, None, None, 3]}
        else:
            exp = {"x": [1, None, None, None], "x_right": [1, 3, None, None], "y": [1, None, 2, 3],
                   "z": [1, 3, None, None]}
        cases.append({"name": f"test_join_null_equal[{order}] full without_null", "source": src,
                      "left": lhs, "right": without_null, "on": "x", "how": "full",
                      "args": {"nulls_equal": True, "maintain_order": order},
                      "expected": exp, "ordered": order != "none"})
    # test_join_on_nested: the nested key values data[0..3] -> 1..4
    lhs = {"a": [1, 2, 3], "b": [1, 2, 3]}
    rhs = {"a": [4, 2], "c": [4, 2]}
    src = "operations/test_join.py:1776-1836"
    for how, order, exp, cols in (
            ("left", "left", {"a": [1, 2, 3], "b": [1, 2, 3], "c": [None, 2, None]}, ["a", "b", "c"]),
            ("right", "right", {"b": [None, 2], "a": [4, 2], "c": [4, 2]}, ["b", "a", "c"]),
            ("inner", None, {"a": [2], "b": [2], "c": [2]}, ["a", "b", "c"]),
            ("full", "left_right", {"a": [1, 2, 3, None], "b": [1, 2, 3, None], "a_right": [None, 2, None, 4],
                                    "c": [None, 2, None, 4]}, ["a", "b", "a_right", "c"]),
            ("semi", None, {"a": [2], "b": [2]}, ["a", "b"]),
            ("anti", "left", {"a": [1, 3], "b": [1, 3]}, ["a", "b"])):
        args = {} if order is None else {"maintain_order": order}
        cases.append({"name": f"test_join_on_nested[{how}]", "source": src, "left": lhs, "right": rhs,
                      "on": "a", "how": how, "args": args, "expected": exp, "ordered": True, "columns": cols})
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 5. Sorting (operations/test_sort.py).  `values` of one column; expected
#    arg-sort or sorted values for (descending, nulls_last).
def sort_cases():
    cases = []
    a = [1.0, 2.0, 3.0, None, None]
    cases.append({"name": "test_arg_sort_nulls[nulls_last=True]", "source": "operations/test_sort.py:213-221",
                  "values": a, "args": {"nulls_last": True}, "expected_arg_sort": [0, 1, 2, 3, 4]})
    cases.append({"name": "test_arg_sort_nulls[nulls_last=False]", "source": "operations/test_sort.py:213-221",
                  "values": a, "args": {"nulls_last": False}, "expected_arg_sort": [3, 4, 0, 1, 2]})
    cases.append({"name": "test_arg_sort_nulls sorted values", "source": "operations/test_sort.py:223-227",
                  "values": a, "args": {"nulls_last": False}, "expected_sorted": [None, None, 1.0, 2.0, 3.0]})
    cases.append({"name": "test_sort_nans_3740", "source": "operations/test_sort.py:299-315",
                  "values": [0.0, None, float("nan"), float("-inf"), float("inf")], "args": {},
                  "expected_arg_sort": [1, 3, 0, 4, 2]})   # keys [2, 4, 1, 5, 3] - 1
    cases.append({"name": "test_arg_sort_rank_nans", "source": "operations/test_sort.py:517-531",
                  "values": [1.0, float("nan")], "args": {}, "expected_arg_sort": [0, 1]})
    cases.append({"name": "test_sort_series_nulls_last", "source": "operations/test_sort.py:951-963",
                  "values": [1, None, 3], "args": {"nulls_last": True}, "expected_sorted": [1, 3, None]})
    x = [1, 3, None, 2, None]
    for descending in (True, False):
        for nulls_last in (True, False):
            sentinel = 100 if descending ^ nulls_last else -100
            ref = sorted(x, key=lambda k: sentinel if k is None else k, reverse=descending)
            cases.append({"name": f"test_sort_descending_nulls_last[{descending}-{nulls_last}]",
                          "source": "operations/test_sort.py:979-1001",
                          "values": x, "args": {"descending": descending, "nulls_last": nulls_last},
                          "expected_sorted": ref})
    cases.append({"name": "test_sort_descending", "source": "operations/test_sort.py:801-806",
                  "values": [1, 2, 3], "args": {"descending": True}, "expected_sorted": [3, 2, 1]})
    return {"cases": cases}


# 5b. Multi-column sort (frames of operations/test_sort.py; `expected` holds
#     the sorted columns; string/datetime columns label-encoded in order).
def sort_multi_cases():
    cases = []
    x, y = [None, 1, None, 3], [3, 2, None, 1]
    for nl, desc, ex, ey in (([False, True], False, [None, None, 1, 3], [3, None, 2, 1]),
                             ([True, False], False, [1, 3, None, None], [2, 1, None, 3]),
                             ([True, False], True, [3, 1, None, None], [1, 2, None, 3]),
                             ([False, True], True, [None, None, 3, 1], [3, None, 1, 2]),
                             ([False, True], [True, False], [None, None, 3, 1], [3, None, 1, 2])):
        cases.append({"name": f"test_expr_sort_by_multi_nulls_last[{nl}-{desc}]",
                      "source": "operations/test_sort.py:158-188",
                      "frame": {"x": x, "y": y}, "by": ["x", "y"],
                      "args": {"nulls_last": nl, "descending": desc},
                      "expected": {"x": ex, "y": ey}})
    cases.append({"name": "test_sort_by[b, c]", "source": "operations/test_sort.py:76-100",
                  "frame": {"a": [1, 2, 3, 4, 5], "b": [1, 1, 1, 2, 2], "c": [2, 3, 1, 2, 1]},
                  "by": ["b", "c"], "args": {"maintain_order": True},
                  "expected": {"a": [3, 1, 2, 5, 4]}})
    cases.append({"name": "test_sort_dates_multiples", "source": "operations/test_sort.py:48-72",
                  "frame": {"date": [0, 0, 1, 1, 2], "values": [5, 4, 3, 2, 1]},
                  "labels": {"date": ["2021-01-01 00:00:00", "2021-01-02 00:00:00", "2021-01-03 00:00:00"]},
                  "by": ["date", "values"], "args": {}, "expected": {"values": [4, 5, 2, 3, 1]}})
    cases.append({"name": "test_sort_descending (2 columns)", "source": "operations/test_sort.py:801-809",
                  "frame": {"a": [1, 2, 3], "b": [4, 5, 6]}, "by": ["a", "b"], "args": {"descending": [True, True]},
                  "expected": {"a": [3, 2, 1], "b": [6, 5, 4]}})
    fx_, fy = [1, 3, None, 2, None], [1, 3, 0, 2, 0]
    for descending in (True, False):
        for nulls_last in (True, False):
            sentinel = 100 if descending ^ nulls_last else -100
            rx = sorted(fx_, key=lambda k: sentinel if k is None else k, reverse=descending)
            ry = sorted(fy, key=lambda k: sentinel if k == 0 else k, reverse=descending)
            cases.append({"name": f"test_sort_descending_nulls_last[x,y-{descending}-{nulls_last}]",
                          "source": "operations/test_sort.py:979-1001",
                          "frame": {"x": fx_, "y": fy}, "by": ["x", "y"],
                          "args": {"descending": descending, "nulls_last": nulls_last},
                          "expected": {"x": rx, "y": ry}})
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 6. Fixed-window rolling sum / mean (operations/rolling/test_rolling.py,
#    lazyframe/test_lazyframe.py, polars-compute rolling/no_nulls/sum.rs
#    unit test).  `expected` with None for null outputs.
def rolling_cases():
    nan = float("nan")
    cases = []
    cases.append({"name": "test_rolling_infinity", "source": "operations/rolling/test_rolling.py:288-292",
                  "values": [float("-inf"), 5.0, 5.0], "kind": "mean", "window": 2, "min": None, "center": False,
                  "expected": [None, float("-inf"), 5.0]})
    cases.append({"name": "test_rolling_ints mean", "source": "operations/rolling/test_rolling.py:873-891",
                  "values": [1, 2, 3, 2, 1], "kind": "mean", "window": 2, "min": None, "center": False,
                  "expected": [None, 1.5, 2.5, 2.5, 1.5]})
    cases.append({"name": "test_rolling_ints sum", "source": "operations/rolling/test_rolling.py:881-889",
                  "values": [1, 2, 3, 2, 1], "kind": "sum", "window": 2, "min": None, "center": False,
                  "expected": [None, 3, 5, 5, 3]})
    for kind, ms, exp in (("mean", 1, [1.0, 1.5, 2.0, 3.0, 4.0]), ("mean", None, [None, None, 2.0, 3.0, 4.0]),
                          ("sum", 1, [1, 3, 6, 9, 12]), ("sum", None, [None, None, 6, 9, 12])):
        cases.append({"name": f"test_rolling fruits_cars A rolling_{kind}(3, min_samples={ms})",
                      "source": "lazyframe/test_lazyframe.py:734-763",
                      "values": [1, 2, 3, 4, 5], "kind": kind, "window": 3, "min": ms, "center": False,
                      "expected": exp})
    v = [1.0, 2.0, 3.0, 4.0]
    for w, ms, center, exp in ((2, 2, False, [None, 3.0, 5.0, 7.0]), (2, 1, False, [1.0, 3.0, 5.0, 7.0]),
                               (4, 1, False, [1.0, 3.0, 6.0, 10.0]), (4, 1, True, [3.0, 6.0, 10.0, 9.0]),
                               (4, 4, True, [None, None, 10.0, None])):
        cases.append({"name": f"test_rolling_sum(w={w}, min={ms}, center={center})",
                      "source": "crates/polars-compute/src/rolling/no_nulls/sum.rs:69-96",
                      "values": v, "kind": "sum", "window": w, "min": ms, "center": center, "expected": exp})
    cases.append({"name": "test_rolling_sum nan", "source": "crates/polars-compute/src/rolling/no_nulls/sum.rs:98-117",
                  "values": [1.0, 2.0, 3.0, nan, 5.0, 6.0, 7.0], "kind": "sum", "window": 3, "min": 3,
                  "center": False, "expected": [None, None, 6.0, nan, nan, nan, 18.0]})
    stab = [0.0, 290.57, 107.0, 172.0, 124.25, 304.0, 379.5, 347.35, 1516.41, 386.12, 226.5, 294.62, 125.5,
            0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0]
    cases.append({"name": "test_rolling_sum_stability_11146 (last value)",
                  "source": "operations/rolling/test_rolling.py:1476-1510",
                  "values": stab, "kind": "mean", "window": 8, "min": 1, "center": False, "expected_last": 0.0})
    # rolling_min / rolling_max (MinMaxWindow, NaN propagates)
    src = "operations/rolling/test_rolling.py:322-362 (sorted data; the shuffled half needs polars' RNG)"
    cols = {"col1": [0, 1, 2, 3, 4, 5, 6], "col2": [6, 5, 4, 3, 2, 1, 0],
            "col1_nulls": [None, None, 2, 3, 4, 5, 6], "col2_nulls": [None, None, 4, 3, 2, 1, 0]}
    emin = {"col1": [None, None, 0, 1, 2, 3, 4], "col2": [None, None, 4, 3, 2, 1, 0],
            "col1_nulls": [None, None, None, None, 2, 3, 4], "col2_nulls": [None, None, None, None, 2, 1, 0]}
    emax = {"col1": [None, None, 2, 3, 4, 5, 6], "col2": [None, None, 6, 5, 4, 3, 2],
            "col1_nulls": [None, None, None, None, 4, 5, 6], "col2_nulls": [None, None, None, None, 4, 3, 2]}
    for kind, exp in (("min", emin), ("max", emax)):
        for name, vals in cols.items():
            cases.append({"name": f"test_rolling_extrema {name} rolling_{kind}(3)", "source": src,
                          "values": vals, "kind": kind, "window": 3, "min": None, "center": False,
                          "expected": exp[name]})
    for kind, exp in (("min", [None, 1, 2, 2, 1]), ("max", [None, 2, 3, 3, 2])):
        cases.append({"name": f"test_rolling_ints rolling_{kind}(2)", "source": "operations/rolling/test_rolling.py:873-880",
                      "values": [1, 2, 3, 2, 1], "kind": kind, "window": 2, "min": None, "center": False,
                      "expected": exp})
    for kind in ("min", "max"):
        cases.append({"name": f"test_rolling_nan rolling_{kind}(3): 2 nulls, 5 NaN-or-null",
                      "source": "operations/rolling/test_rolling.py:924-933",
                      "values": [1.0, 2.0, 3.0, nan, 5.0, 6.0, 7.0], "kind": kind, "window": 3, "min": None,
                      "center": False, "expected_null_count": 2, "expected_nan_or_null": 5})
    # rolling_var / rolling_std (MomentWindow<VarianceMoment>; round 5).
    # `approx`: the reference test compares with pytest.approx (rel 1e-6).
    vsrc = "crates/polars-compute/src/rolling/no_nulls/moment.rs:104-133 (test_rolling_var)"
    for ddof, ms, exp in ((1, 2, [None, 8.0, 2.0, 0.5]), (0, 2, [None, 4.0, 1.0, 0.25]),
                          (1, 1, [None, 8.0, 2.0, 0.5])):
        cases.append({"name": f"test_rolling_var(w=2, min={ms}, ddof={ddof})", "source": vsrc,
                      "values": [1.0, 5.0, 3.0, 4.0], "kind": "var", "window": 2, "min": ms, "center": False,
                      "ddof": ddof, "expected": exp})
    cases.append({"name": "test_rolling_var_numerical_stability_5197",
                  "source": "operations/rolling/test_rolling.py:626-640",
                  "values": [1.2] * 4 + [3.3] * 7, "kind": "var", "window": 5, "min": None, "center": False,
                  "ddof": 1, "approx": True,
                  "expected": [None] * 4 + [0.882, 1.3229999999999997, 1.3229999999999997, 0.8819999999999983,
                                            0.0, 0.0, 0.0]})
    for kind, ddof, exp in (("std", 1, 0.7071067811865476), ("var", 1, 0.5), ("std", 0, 0.5), ("var", 0, 0.25)):
        cases.append({"name": f"test_rolling_ints rolling_{kind}(2, ddof={ddof})[1]",
                      "source": "operations/rolling/test_rolling.py:893-896",
                      "values": [1, 2, 3, 2, 1], "kind": kind, "window": 2, "min": None, "center": False,
                      "ddof": ddof, "approx": True, "expected_at": [1, exp]})
    cases.append({"name": "test_rolling_std_nulls_min_samples_1_20076",
                  "source": "operations/rolling/test_rolling.py:956-961",
                  "values": [1, 2, None, 4], "kind": "std", "window": 3, "min": 1, "center": False, "ddof": 1,
                  "expected": [None, 0.7071067811865476, 0.7071067811865476, 1.4142135623730951]})
    cases.append({"name": "test_rolling_var_zero_weight", "source": "operations/test_rolling.py:632-636",
                  "values": [1.0, None, 1.0, 2.0], "kind": "var", "window": 2, "min": None, "center": False,
                  "ddof": 1, "expected": [None, None, None, 0.5]})
    for kind in ("var", "std"):
        cases.append({"name": f"test_rolling_var_stability_12905 rolling_{kind}(12, min_samples=2).sum() == 0",
                      "source": "operations/rolling/test_rolling_fixed.py:4-7",
                      "values": [36743.6] * 10, "kind": kind, "window": 12, "min": 2, "center": False, "ddof": 1,
                      "expected_sum": 0.0})
        cases.append({"name": f"test_rolling fruits_cars A rolling_{kind}(3)",
                      "source": "lazyframe/test_lazyframe.py:747-763 (.round(1))",
                      "values": [1, 2, 3, 4, 5], "kind": kind, "window": 3, "min": None, "center": False, "ddof": 1,
                      "round": 1, "expected": [None, None, 1.0, 1.0, 1.0]})
        cases.append({"name": f"test_rolling fruits_cars A rolling_{kind}(3, min_samples=1)[0] is null",
                      "source": "lazyframe/test_lazyframe.py:768-775",
                      "values": [1, 2, 3, 4, 5], "kind": kind, "window": 3, "min": 1, "center": False, "ddof": 1,
                      "expected_at": [0, None]})
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 9. Arithmetic / casts / bitwise / when-then over typed columns (round 2:
#    dtype breadth).  Each case: typed input columns, an expression in the
#    polaroid_amd DSL (evaluated with `pl` and `col` in scope), what the
#    reference test asserts (`expected` values, `expected_dtype`, or
#    `raises`), and `approx` where the test compares with assert_*_equal's
#    default float tolerance.
INT_DTYPES = ["Int8", "Int16", "Int32", "Int64", "UInt8", "UInt16", "UInt32", "UInt64"]


def arith_cases():
    cases = []

    def add(name, source, cols, expr, **kw):
        cases.append(dict(name=name, source=source, cols=cols, expr=expr, **kw))

    add("test_floor_divide", "series/test_series.py:1128-1133", {"a": ["Int64", [1, 2, 3]]},
        "col('a') // 2", expected=[0, 1, 1], expected_dtype="Int64")
    add("test_true_divide", "series/test_series.py:1136-1141", {"a": ["Int64", [1, 2]]},
        "col('a') / 2", expected=fx([0.5, 1.0]), expected_dtype="Float64")
    add("test_true_divide rtruediv", "series/test_series.py:1143-1147", {"a": ["Int64", [1, 2]]},
        "2 / col('a')", expected=fx([2.0, 1.0]), expected_dtype="Float64", expected_name="literal")
    add("test_floor_divide (float by 0.5)", "dataframe/test_df.py:3091-3095", {"x": ["Float64", [10.4]]},
        "col('x') // 0.5", expected=fx([10.4 // 0.5]), expected_dtype="Float64")
    add("test_float_floor_divide", "lazyframe/test_lazyframe.py:877-882", {"x": ["Float64", [10.4]]},
        "col('x') // 0.5", expected=fx([10.4 // 0.5]), expected_dtype="Float64")
    add("test_integer_divide_scalar_zero_lhs_19142 //", "operations/arithmetic/test_arithmetic.py:847-849",
        {"b": ["Int64", [1, 0]]}, "lit(0) // col('b')", expected=[0, None], expected_dtype="Int64",
        expected_name="literal")
    add("test_integer_divide_scalar_zero_lhs_19142 %", "operations/arithmetic/test_arithmetic.py:850",
        {"b": ["Int64", [1, 0]]}, "lit(0) % col('b')", expected=[0, None], expected_dtype="Int64",
        expected_name="literal")
    add("test_neg_overflow_wrapping", "operations/arithmetic/test_neg.py:49-52", {"a": ["Int8", [-128]]},
        "-col('a')", expected=[-128], expected_dtype="Int8")
    add("test_neg_unsigned_int", "operations/arithmetic/test_neg.py:55-60", {"a": ["UInt8", [1, 2, 3]]},
        "-col('a')", raises="InvalidOperationError")
    add("test_literal_subtract_schema_13284", "operations/arithmetic/test_arithmetic.py:659-666",
        {"a": ["UInt8", [23, 30]]}, "col('a') - lit(1)", expected=[22, 29], expected_dtype="UInt8")
    for dt in INT_DTYPES:
        for op, val, odt in (("//", 5, dt), ("+", 12, dt), ("-", 8, dt), ("*", 20, dt), ("/", 5.0, "Float64")):
            add(f"test_int_operator_stability[{dt}] {op}", "operations/arithmetic/test_arithmetic.py:668-675",
                {"a": [dt, [10]]}, f"col('a') {op} 2", expected=fx([val]), expected_dtype=odt)
    add("test_literal_no_upcast fma", "operations/arithmetic/test_arithmetic.py:224-238",
        {"a": ["Float32", [1.0, 2.0, 3.0]]}, "col('a') * -5 + 2", expected=fx([-3.0, -8.0, -13.0]),
        expected_dtype="Float32")
    add("test_literal_no_upcast fsm", "operations/arithmetic/test_arithmetic.py:224-238",
        {"a": ["Float32", [1.0, 2.0, 3.0]]}, "2 - col('a') * 5", expected=fx([-3.0, -8.0, -13.0]),
        expected_dtype="Float32", expected_name="literal")
    add("test_literal_no_upcast fms", "operations/arithmetic/test_arithmetic.py:224-238",
        {"a": ["Float32", [1.0, 2.0, 3.0]]}, "col('a') * 5 - 2", expected=fx([3.0, 8.0, 13.0]),
        expected_dtype="Float32")
    add("test_bitwise_6311 step 1", "operations/arithmetic/test_arithmetic.py:254-267",
        {"col1": ["Int64", [0, 1, 2, 3]], "flag": ["Int64", [0, 0, 0, 0]]},
        "pl.when((col('col1') < 1) | (col('col1') >= 3)).then(col('flag') | 2).otherwise(col('flag'))",
        expected=[2, 0, 0, 2], expected_dtype="Int64", expected_name="flag")
    add("test_bitwise_6311 step 2", "operations/arithmetic/test_arithmetic.py:254-267",
        {"col1": ["Int64", [0, 1, 2, 3]], "flag": ["Int64", [2, 0, 0, 2]]},
        "pl.when(col('col1') > -1).then(col('flag') | 4).otherwise(col('flag'))",
        expected=[6, 4, 4, 6], expected_dtype="Int64", expected_name="flag")
    add("test_modulo a % 2", "sql/test_numeric.py:38-70",
        {"a": ["Float64", [1.5, None, 3.0, 13 / 3, 5.0]]}, "col('a') % 2",
        expected=fx([1.5, None, 1.0, 1 / 3, 1.0]), expected_dtype="Float64", approx=True)
    add("test_modulo b % 3", "sql/test_numeric.py:38-70", {"b": ["Int64", [6, 7, 8, 9, 10]]}, "col('b') % 3",
        expected=[0, 1, 2, 0, 1], expected_dtype="Int64")
    add("test_modulo MOD(c, 4)", "sql/test_numeric.py:38-70", {"c": ["Int64", [11, 12, 13, 14, 15]]},
        "col('c') % 4", expected=[3, 0, 1, 2, 3], expected_dtype="Int64")
    add("test_modulo MOD(d, 5.5)", "sql/test_numeric.py:38-70",
        {"d": ["Float64", [16.5, 17.0, 18.5, None, 20.0]]}, "col('d') % 5.5",
        expected=fx([0.0, 0.5, 2.0, None, 3.5]), expected_dtype="Float64", approx=True)
    add("test_float_truediv_output_type f32/f32", "operations/arithmetic/test_arithmetic.py:925-931",
        {"f32": ["Float32", [1.0]], "f64": ["Float64", [2.0]]}, "col('f32') / col('f32')",
        expected=fx([1.0]), expected_dtype="Float32")
    add("test_float_truediv_output_type f32/f64", "operations/arithmetic/test_arithmetic.py:932-934",
        {"f32": ["Float32", [1.0]], "f64": ["Float64", [2.0]]}, "col('f32') / col('f64')",
        expected=fx([0.5]), expected_dtype="Float64")
    add("test_lit_cast_arithmetic_23677", "operations/test_cast.py:1032-1036", {"a": ["Float32", [1.0]]},
        "col('a') / lit(1).cast(pl.Int32)", expected=fx([1.0]), expected_dtype="Float64")
    strict_int = [(-1, "Int8", "UInt8", None), (-1, "Int16", "UInt16", None), (-1, "Int32", "UInt32", None),
                  (-1, "Int64", "UInt64", None), (2 ** 7, "UInt8", "Int8", None), (2 ** 15, "UInt16", "Int16", None),
                  (2 ** 31, "UInt32", "Int32", None), (2 ** 63, "UInt64", "Int64", None),
                  (2 ** 7 - 1, "UInt8", "Int8", 2 ** 7 - 1), (2 ** 15 - 1, "UInt16", "Int16", 2 ** 15 - 1),
                  (2 ** 31 - 1, "UInt32", "Int32", 2 ** 31 - 1), (2 ** 63 - 1, "UInt64", "Int64", 2 ** 63 - 1)]
    for v, a, b, exp in strict_int:
        add(f"test_cast_int[{v}-{a}-{b}]", "operations/test_cast.py:247-269", {"a": [a, [v]]},
            f"col('a').cast(pl.{b}, strict=False)", expected=[exp], expected_dtype=b)
        if exp is None:
            add(f"test_strict_cast_int[{v}-{a}-{b}]", "operations/test_cast.py:206-244", {"a": [a, [v]]},
                f"col('a').cast(pl.{b})", raises="InvalidOperationError")
        else:
            add(f"test_strict_cast_int[{v}-{a}-{b}]", "operations/test_cast.py:206-244", {"a": [a, [v]]},
                f"col('a').cast(pl.{b})", expected=[exp], expected_dtype=b)
    add("test_overflowing_cast_literals_21023", "operations/test_cast.py:747-763", {"a": ["Int64", [128]]},
        "col('a').cast(pl.Int8, wrap_numerical=True)", expected=[-128], expected_dtype="Int8")
    return {"cases": cases}


# ---------------------------------------------------------------------------
# 12. Aggregations over computed inputs and global reductions (select(aggs)).
#     Each aggregation is an expression string of the polars API (evaluated
#     with col / lit / when in scope); `key` None is a select, else group ids
#     (string keys label-encoded).  `tol`: relative tolerance for an output the
#     reference itself compares approximately or computes with a different
#     rounding (Welford var / std, np.isclose).
def reduce_cases():
    cases = []
    cases.append({
        "name": "test_boolean_aggs (select)",
        "source": "operations/aggregation/test_aggregations.py:30-42",
        "cols": {"bool": {"dtype": "bool", "values": [True, False, None, True]}},
        "key": None,
        "aggs": [["col('bool').mean()", "mean"], ["col('bool').std()", "std"], ["col('bool').var()", "var"]],
        "expected": {"mean": fx([0.6666666666666666]), "std": fx([0.5773502691896258]),
                     "var": fx([0.33333333333333337])},
        "tol": {"std": 1e-12, "var": 1e-12},
    })
    cases.append({
        "name": "test_boolean_aggs (group_by literal key)",
        "source": "operations/aggregation/test_aggregations.py:44-49 (group_by(pl.lit(1)): one group)",
        "cols": {"bool": {"dtype": "bool", "values": [True, False, None, True]}},
        "key": [1, 1, 1, 1],
        "aggs": [["col('bool').mean()", "mean"]],
        "expected": {"key": [1], "mean": fx([0.6666666666666666])},
    })
    cases.append({
        "name": "test_sum_empty_and_null_set (select)",
        "source": "operations/aggregation/test_aggregations.py:441-445",
        "cols": {"a": {"dtype": "f32", "values": [None, None, None]}, "b": {"dtype": "i64", "values": [1, 1, 1]}},
        "key": None,
        "aggs": [["col('a').sum()", "a"]],
        "expected": {"a": fx([0.0])},
    })
    cases.append({
        "name": "test_sum_empty_and_null_set (group_by)",
        "source": "operations/aggregation/test_aggregations.py:441-446",
        "cols": {"a": {"dtype": "f32", "values": [None, None, None]}, "b": {"dtype": "i64", "values": [1, 1, 1]}},
        "key": [1, 1, 1],
        "aggs": [["col('a').sum()", "a"]],
        "expected": {"key": [1], "a": fx([0.0])},
    })
    cases.append({
        "name": "test_empty_agg_22005",
        "source": "operations/aggregation/test_aggregations.py:940-946",
        "cols": {"a": {"dtype": "i64", "values": []}},
        "key": None,
        "aggs": [["col('a').sum()", "a"]],
        "expected": {"a": [0]},
    })
    cases.append({
        "name": "test_group_by_when_then_no_aggregation_predicate",
        "source": "operations/test_group_by.py:1039-1053",
        "cols": {"val": {"dtype": "i64", "values": [-3, -2, 1, 4, -3, 5]}},
        "key": [0, 0, 1, 1, 0, 0], "key_labels": ["aa", "bb"],
        "aggs": [["when(col('val') >= 0).then(col('val')).sum()", "pos"],
                 ["when(col('val') < 0).then(col('val')).sum()", "neg"]],
        "sort_by_key": True,
        "expected": {"key": [0, 1], "pos": [5, 5], "neg": [-8, 0]},
    })
    ids = [130352432, 130352277, 130352611, 130352833, 130352305, 130352258, 130352764, 130352475, 130352368,
           130352346]
    cases.append({
        "name": "test_min_max_2850",
        "source": "operations/aggregation/test_aggregations.py:705-733",
        "cols": {"id": {"dtype": "i64", "values": ids}},
        "key": None,
        "aggs": [["col('id').min()", "min"], ["col('id').max()", "max"]],
        "expected": {"min": [130352258], "max": [130352833]},
    })
    cases.append({
        "name": "test_cse_expr_selection_context (d1)",
        "source": "test_cse.py:211-226 (derived = (a * b).sum(), aliased d1)",
        "cols": {"a": {"dtype": "i64", "values": [1, 2, 3, 4]}, "b": {"dtype": "i64", "values": [1, 2, 3, 4]},
                 "c": {"dtype": "i64", "values": [1, 2, 3, 4]}},
        "key": None,
        "aggs": [["(col('a') * col('b')).sum()", "d1"]],
        "expected": {"d1": [30]},
    })
    cases.append({
        "name": "test_mean_overflow",
        "source": "operations/aggregation/test_aggregations.py:298-302 (Series.mean, np.isclose)",
        "cols": {"a": {"dtype": "i64", "values": [9_223_372_036_854_775_800, 100]}},
        "key": None,
        "aggs": [["col('a').mean()", "a"]],
        "expected": {"a": fx([4.611686018427388e18])},
        "tol": {"a": 1e-9},
    })
    return {"cases": cases}


def categorical_cases():
    """Group-by on Categorical keys: the groups, their first-occurrence order
    (maintain_order) and sizes the reference's tests assert."""
    cases = []
    # operations/test_group_by.py:903-957 test_perfect_hash_table_null_values:
    # a Categorical with nulls grouped with maintain_order; `groups` is the
    # expected key column and the expected agg lists' lengths are the sizes
    values = ["3", "41", "17", "5", "26", "27", "43", "45", "41", "13", "45", "48", "17", "22", "31", "25", "28",
              "13", "7", "26", "17", "4", "43", "47", "30", "28", "8", "27", "6", "7", "26", "11", "37", "29", "49",
              "20", "29", "28", "23", "9", None, "38", "19", "7", "38", "3", "30", "37", "41", "5", "16", "26", "31",
              "6", "25", "11", "17", "31", "31", "20", "26", None, "39", "10", "38", "4", "39", "15", "13", "35",
              "38", "11", "39", "11", "48", "36", "18", "11", "34", "16", "28", "9", "37", "8", "17", "48", "44",
              "28", "25", "30", "37", "30", "18", "12", None, "27", "10", "3", "16", "27", "6"]
    groups = ["3", "41", "17", "5", "26", "27", "43", "45", "13", "48", "22", "31", "25", "28", "7", "4", "47", "30",
              "8", "6", "11", "37", "29", "49", "20", "23", "9", None, "38", "19", "16", "39", "10", "15", "35", "36",
              "18", "34", "44", "12"]
    sizes = [3, 3, 5, 2, 5, 4, 2, 2, 3, 3, 1, 4, 3, 5, 3, 2, 1, 4, 2, 3, 5, 4, 2, 1, 2, 1, 2, 3, 4, 1, 3, 3, 2, 1,
             1, 1, 2, 1, 1, 1]
    cases.append({"name": "perfect_hash_table_null_values",
                  "source": "operations/test_group_by.py:903-957",
                  "key": values, "maintain_order": True, "groups": groups, "len": sizes})
    # datatypes/test_categorical.py:104-118 test_unset_sorted_on_append: two
    # Categorical frames concatenated without rechunking (two chunks, the
    # dictionaries unified), group_by("key").len() == [4, 4]
    cases.append({"name": "unset_sorted_on_append",
                  "source": "datatypes/test_categorical.py:104-118",
                  "chunks": [["a", "a", "b", "b"], ["a", "a", "b", "b"]], "vals": [1, 3, 2, 4, 5, 7, 6, 8],
                  "maintain_order": False, "groups": ["a", "b"], "len": [4, 4]})
    # operations/test_group_by.py:608-626 test_group_by_custom_agg_empty_list:
    # an empty Categorical key grouped: no rows (and a Categorical key column)
    cases.append({"name": "empty_categorical_key",
                  "source": "operations/test_group_by.py:608-626",
                  "key": [], "maintain_order": False, "groups": [], "len": []})
    return {"cases": cases}


def main():
    for name, obj in (("categorical_cases.json", categorical_cases()),("compare_total_order.json", compare_table()),
                      ("group_by_cases.json", group_by_cases()),
                      ("group_by_multi_cases.json", group_by_multi_cases()),
                      ("filter_cases.json", filter_cases()),
                      ("join_cases.json", join_cases()),
                      ("join_multi_cases.json", join_multi_cases()),
                      ("join_types_cases.json", join_types_cases()),
                      ("sort_cases.json", sort_cases()),
                      ("sort_multi_cases.json", sort_multi_cases()),
                      ("rolling_cases.json", rolling_cases()),
                      ("arith_cases.json", arith_cases()),
                      ("reduce_cases.json", reduce_cases())):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1, sort_keys=False)
            f.write("\n")


if __name__ == "__main__":
    main()
