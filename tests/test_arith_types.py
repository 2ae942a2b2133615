"""Typed arithmetic, casts, bitwise ops and when/then/otherwise (CPU).

Pins the oracle's typed expression evaluator (oracle/polars_oracle.c
eval_row: supertypes, dynamic literals, wrapping at the dtype's width,
floor division / modulo, scalar-divisor forms, non-strict casts) against the
cases transcribed from the reference's own tests in
tests/golden/arith_cases.json, and checks that the executor's static typing
(plgpu_expr_dtype: the native lowering, run on the host) gives every case
the dtype the reference asserts.  The GPU side of the same cases is in
tests/test_gpu_dtypes.py.
"""

import ctypes as C
import math
import zlib

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O
from polaroid_amd import _native as N
from polaroid_amd.expr import col, lit, lower, to_instr_array

from conftest import load_golden, unhex

CASES = load_golden("arith_cases.json")["cases"]
NP = {"Int8": np.int8, "Int16": np.int16, "Int32": np.int32, "Int64": np.int64, "UInt8": np.uint8,
      "UInt16": np.uint16, "UInt32": np.uint32, "UInt64": np.uint64, "Float32": np.float32, "Float64": np.float64}
CODE = {"Int8": N.I8, "Int16": N.I16, "Int32": N.I32, "Int64": N.I64, "UInt8": N.U8, "UInt16": N.U16,
        "UInt32": N.U32, "UInt64": N.U64, "Float32": N.F32, "Float64": N.F64, "Boolean": N.BOOL}
NAME = {v: k for k, v in CODE.items()}


def host_cols(case):
    names = list(case["cols"])
    cols = []
    for nm in names:
        dt, vals = case["cols"][nm]
        vals = unhex(vals)
        valid = np.array([v is not None for v in vals], bool)
        arr = np.array([0 if v is None else v for v in vals], dtype=NP[dt])
        cols.append(O.HostCol(arr, None if valid.all() else valid))
    return names, cols


def program(case):
    expr = eval(case["expr"], {"pl": pl, "col": col, "lit": lit})
    names = list(case["cols"])
    schema = {nm: CODE[case["cols"][nm][0]] for nm in names}
    return expr, lower(expr, {nm: i for i, nm in enumerate(names)}, schema)


def static_dtype(case, prog):
    names = list(case["cols"])
    cols = (N.Column * max(1, len(names)))()
    for i, nm in enumerate(names):
        cols[i].dtype = CODE[case["cols"][nm][0]]
    out = C.c_int32(0)
    rc = N.lib().plgpu_expr_dtype(cols, len(names), to_instr_array(prog), len(prog), C.byref(out))
    return rc, out.value


def same(got, want, approx):
    if want is None:
        return got is None
    if got is None:
        return False
    if isinstance(want, float):
        if math.isnan(want):
            return math.isnan(got)
        if approx:
            return math.isclose(got, want, rel_tol=1e-5, abs_tol=1e-8)
        return float(got) == want and math.copysign(1, got) == math.copysign(1, want)
    return int(got) == want


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_and_static_types_match_reference(case):
    names, cols = host_cols(case)
    nrows = len(unhex(case["cols"][names[0]][1]))
    expr, prog = program(case)
    raises = case.get("raises")
    strict_fail = raises and ".cast(" in case["expr"]
    if raises and not strict_fail:
        # an ill-typed program: the oracle refuses it, and so does the lowering
        with pytest.raises(ValueError):
            O.eval_program(cols, prog, nrows)
        assert static_dtype(case, prog)[0] == N.ERR_INVALID
        return
    dt, vals, valid = O.eval_program(cols, prog, nrows)
    if strict_fail:
        # polars raises for a strict cast that meets a value that does not
        # fit; the evaluator's non-strict result has the null that triggers it
        assert not valid.all()
        return
    assert NAME[dt] == case["expected_dtype"], case["name"]
    rc, sdt = static_dtype(case, prog)
    assert rc == 0 and NAME[sdt] == case["expected_dtype"], case["name"]
    got = [v.item() if ok else None for v, ok in zip(vals, valid)]
    want = unhex(case["expected"])
    assert all(same(g, w, case.get("approx")) for g, w in zip(got, want)), (case["name"], got, want)
    assert expr.output_name() == case.get("expected_name", names[0])


# -------------------------------------------------- supertype matrix (CPU)
# polars-core/src/utils/supertype.rs:146 rows for column + column
SUPER = {
    ("Int8", "UInt8"): "Int16", ("Int8", "UInt16"): "Int32", ("Int8", "UInt32"): "Int64",
    ("Int8", "UInt64"): "Float64", ("Int8", "Float32"): "Float32", ("Int16", "UInt16"): "Int32",
    ("Int16", "Float32"): "Float32", ("Int32", "UInt32"): "Int64", ("Int32", "Float32"): "Float64",
    ("Int64", "UInt64"): "Float64", ("Int64", "Float32"): "Float64", ("UInt8", "UInt32"): "UInt32",
    ("UInt16", "UInt64"): "UInt64", ("Float32", "UInt8"): "Float32", ("Float32", "UInt16"): "Float32",
    ("Float32", "UInt32"): "Float64", ("Float32", "Float64"): "Float64", ("Int16", "UInt8"): "Int16",
    ("Int32", "UInt16"): "Int32", ("Int64", "UInt32"): "Int64",
}


@pytest.mark.parametrize("pair", sorted(SUPER), ids=[f"{a}+{b}" for a, b in sorted(SUPER)])
def test_column_supertypes(pair):
    a, b = pair
    case = {"cols": {"a": [a, [1]], "b": [b, [1]]}, "expr": "col('a') + col('b')"}
    _, prog = program(case)
    rc, dt = static_dtype(case, prog)
    assert rc == 0 and NAME[dt] == SUPER[pair]
    # symmetric
    case = {"cols": {"a": [b, [1]], "b": [a, [1]]}, "expr": "col('a') + col('b')"}
    _, prog = program(case)
    assert NAME[static_dtype(case, prog)[1]] == SUPER[pair]


# supertype.rs:463: a dynamic int literal takes the smallest type holding it
LIT = [("Int8", 1, "Int8"), ("Int8", 1000, "Int16"), ("Int8", -100000, "Int32"), ("UInt8", 1, "UInt8"),
       ("UInt8", -1, "Int16"), ("UInt8", 300, "UInt16"), ("UInt64", 5, "UInt64"), ("UInt64", -5, "Int64"),
       ("Int32", 2 ** 40, "Int64"), ("Float32", 7, "Float32"), ("Int64", 2.5, "Float64"),
       ("Float32", 2.5, "Float32"), ("UInt32", 2 ** 33, "UInt64")]


@pytest.mark.parametrize("dt,v,want", LIT)
def test_dynamic_literal_types(dt, v, want):
    case = {"cols": {"a": [dt, [1]]}, "expr": f"col('a') + {v!r}"}
    _, prog = program(case)
    rc, got = static_dtype(case, prog)
    assert rc == 0 and NAME[got] == want


def _rand(dt, n, rng):
    if dt.startswith("Float"):
        x = rng.standard_normal(n) * 100
        x[rng.random(n) < 0.05] = np.nan
        x[rng.random(n) < 0.02] = 0.0
        return x.astype(NP[dt])
    info = np.iinfo(NP[dt])
    return rng.integers(info.min, info.max, n, dtype=NP[dt], endpoint=True)


@pytest.mark.parametrize("dt", list(NP))
@pytest.mark.parametrize("op", ["//", "%", "+", "-", "*", "/"])
def test_oracle_ops_vs_numpy_semantics(dt, op):
    """The oracle's per-dtype arithmetic against numpy's (same wrapping,
    floor and modulo conventions as Rust's wrapping_* / floor_divmod for
    integers; IEEE for floats), with x // 0 and x % 0 null."""
    rng = np.random.default_rng(zlib.crc32(f"{dt},{op}".encode()))
    n = 2000
    a, b = _rand(dt, n, rng), _rand(dt, n, rng)
    if not dt.startswith("Float"):
        b[:50] = 0
    case = {"cols": {"a": [dt, [0]], "b": [dt, [0]]}, "expr": f"col('a') {op} col('b')"}
    _, prog = program(case)
    dt_out, vals, valid = O.eval_program([O.HostCol(a), O.HostCol(b)], prog, n)
    with np.errstate(all="ignore"):
        if dt.startswith("Float"):
            f = {"+": np.add, "-": np.subtract, "*": np.multiply, "/": np.divide,
                 "//": lambda x, y: np.floor(x / y), "%": lambda x, y: x - y * np.floor(x / y)}[op]
            want = f(a, b)
            assert np.array_equal(vals.view(np.uint8).reshape(n, -1), want.astype(vals.dtype).view(np.uint8).reshape(n, -1)) \
                or np.array_equal(np.isnan(vals), np.isnan(want)) and np.array_equal(vals[~np.isnan(vals)], want[~np.isnan(want)])
        elif op == "/":
            want = a.astype(np.float64) / b.astype(np.float64)
            m = ~np.isnan(want)
            assert np.array_equal(vals[m], want[m])
        else:
            nz = b != 0
            if op in ("//", "%"):
                assert np.array_equal(valid, nz)
            f = {"+": np.add, "-": np.subtract, "*": np.multiply, "//": np.floor_divide, "%": np.mod}[op]
            want = f(a[nz], b[nz]) if op in ("//", "%") else f(a, b)
            got = vals[nz] if op in ("//", "%") else vals
            assert np.array_equal(got.astype(NP[dt]), want.astype(NP[dt]))
