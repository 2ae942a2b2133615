"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front end of oracle/polars_oracle.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
this module, as the checker.  See polars_oracle.c for the reference
file:line each function restates.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

BOOL, I32, I64, F64, U32 = 1, 2, 3, 4, 5
I8, I16, U8, U16, U64, F32 = 7, 8, 9, 10, 11, 12
_NP_OF = {I8: np.int8, I16: np.int16, I32: np.int32, I64: np.int64, U8: np.uint8, U16: np.uint16,
          U32: np.uint32, U64: np.uint64, F32: np.float32, F64: np.float64}
SUM_KAHAN, SUM_NAIVE, SUM_EXACT = 0, 1, 2
AGG = dict(sum=1, mean=2, min=3, max=4, count=5, len=6, first=7, last=8)


class _Col(C.Structure):  # layout of plgpu_column (include/polaroid_gpu.h)
    _fields_ = [
        ("dtype", C.c_int32), ("device_id", C.c_int32), ("length", C.c_int64), ("offset", C.c_int64),
        ("null_count", C.c_int64), ("values", C.c_void_p), ("validity", C.c_void_p),
        ("release", C.c_void_p), ("private_data", C.c_void_p), ("data", C.c_void_p),
    ]


class _Imm(C.Union):
    _fields_ = [("f64", C.c_double), ("i64", C.c_int64)]


class _Instr(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32), ("imm", _Imm)]


class _Agg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("col", C.c_int32)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.or_eval.restype = C.c_int
        L.or_filter.restype = C.c_int64
        L.or_group_by_agg.restype = C.c_int64
        L.or_join_inner.restype = C.c_int64
        L.or_join_inner.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p]
        L.or_join.restype = C.c_int64
        L.or_join.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p]
        L.or_arg_sort.restype = None
        L.or_arg_sort.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.or_rolling.restype = None
        L.or_rolling.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
        L.or_fsum.restype = C.c_double
        L.or_fsum.argtypes = [C.c_void_p, C.c_int64]
        L.or_baseline_filter_groupby_sum.restype = C.c_int64
        L.or_baseline_filter_groupby_sum.argtypes = [
            C.c_void_p, C.c_void_p, C.c_double, C.c_void_p, C.c_int32, C.c_int64, C.c_int32,
            C.POINTER(C.c_double)]
        L.or_baseline_sort_rolling.restype = C.c_double
        L.or_baseline_sort_rolling.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int64,
                                               C.c_int32, C.c_void_p, C.c_void_p]
        L.or_baseline_join_inner.restype = C.c_int64
        L.or_baseline_join_inner.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                             C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.or_baseline_filter.restype = C.c_int64
        L.or_baseline_filter.argtypes = [C.c_void_p, C.c_double, C.c_void_p, C.c_int32, C.c_int64, C.c_int32,
                                         C.c_void_p]
        L.or_rolling_var.restype = None
        L.or_rolling_var.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_void_p, C.c_void_p]
        L.or_float_sum.restype = C.c_double
        L.or_float_sum.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        L.or_var_welford.restype = C.c_double
        L.or_var_welford.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32]
        L.or_var_chunked.restype = C.c_double
        L.or_var_chunked.argtypes = [C.c_void_p, C.c_int64, C.c_int32]
        _lib = L
    return _lib


def _np_dtype(code: int):
    return _NP_OF[code]


def _code_of(a: np.ndarray) -> int:
    if a.dtype == np.bool_:
        return BOOL
    return {np.dtype(t): c for c, t in _NP_OF.items()}[a.dtype]


class HostCol:
    """(values, validity) numpy pair exposed as a plgpu_column over host memory."""

    def __init__(self, values: np.ndarray, valid: np.ndarray | None = None):
        self.code = _code_of(values)
        n = values.shape[0]
        if self.code == BOOL:
            self.buf = np.packbits(values.astype(np.uint8), bitorder="little")
            if self.buf.size == 0:
                self.buf = np.zeros(1, np.uint8)
        else:
            self.buf = np.ascontiguousarray(values)
        self.vbuf = None if valid is None else np.packbits(valid.astype(np.uint8), bitorder="little")
        self.c = _Col()
        self.c.dtype = self.code
        self.c.length = n
        self.c.offset = 0
        self.c.values = self.buf.ctypes.data if self.buf.size else None
        self.c.validity = self.vbuf.ctypes.data if self.vbuf is not None and self.vbuf.size else None
        if valid is not None and self.c.validity is None:
            self.vbuf = np.zeros(1, np.uint8)
            self.c.validity = self.vbuf.ctypes.data


def _cols(cols: list[HostCol]):
    arr = (_Col * max(1, len(cols)))()
    for i, c in enumerate(cols):
        arr[i] = c.c
    return arr


def _prog(program):
    if not program:
        return None, 0
    arr = (_Instr * len(program))()
    for i, (op, arg, imm) in enumerate(program):
        arr[i].op, arr[i].arg = op, arg
        if op == 2:
            arr[i].imm.f64 = float(imm)
        else:
            arr[i].imm.i64 = int(imm)
    return arr, len(program)


def eval_program(cols: list[HostCol], program, nrows: int):
    """Returns (dtype_code, values ndarray, validity bool ndarray)."""
    words = (nrows + 63) // 64 + 1
    vals = np.zeros(max(nrows, 1) * 8 + 8, dtype=np.uint8)
    valid = np.zeros(words * 8, dtype=np.uint8)
    p, n = _prog(program)
    dt = lib().or_eval(_cols(cols), len(cols), p, n, C.c_int64(nrows), vals.ctypes.data_as(C.c_void_p),
                       valid.ctypes.data_as(C.c_void_p))
    if dt < 0:
        raise ValueError("oracle: ill-typed program")
    validity = np.unpackbits(valid, bitorder="little")[:nrows].astype(bool)
    if dt == BOOL:
        v = np.unpackbits(vals, bitorder="little")[:nrows].astype(bool)
    else:
        t = np.dtype(_NP_OF[dt])
        v = vals[: nrows * t.itemsize].view(t).copy()
    return dt, v, validity


def filter_column(cols: list[HostCol], program, nrows: int, which: int):
    c = cols[which]
    eb = np.dtype(_NP_OF[c.code]).itemsize
    out = np.zeros(max(nrows, 1) * eb, dtype=np.uint8)
    outv = np.zeros((nrows + 7) // 8 + 8, dtype=np.uint8)
    p, n = _prog(program)
    m = lib().or_filter(_cols(cols), len(cols), p, n, C.c_int64(nrows), which,
                        out.ctypes.data_as(C.c_void_p), outv.ctypes.data_as(C.c_void_p))
    vals = out[: m * eb].view(_np_dtype(c.code)).copy()
    valid = np.unpackbits(outv, bitorder="little")[:m].astype(bool)
    return vals, valid


def group_by_agg(key: HostCol, cols: list[HostCol], program, aggs: list[tuple[str, int]], nrows: int,
                 sum_mode: int = SUM_EXACT):
    """Groups in first-occurrence order.  Returns (keys, key_valid, [(values, valid)])."""
    maxg = max(nrows, 1)
    keys = np.zeros(maxg, np.int64)
    kvalid = np.zeros(maxg, np.uint8)
    outs, outv = [], []
    for kind, ci in aggs:
        code = cols[ci].code
        if kind in ("count", "len"):
            dt = np.uint32
        elif kind == "mean" or code in (F64, F32):
            dt = np.float64  # Float32 results are exact / rounded in f64; the caller rounds to f32
        else:
            dt = np.int64    # integer results as int64 bits; the caller narrows to the output dtype
        outs.append(np.zeros(maxg, dt))
        outv.append(np.zeros(maxg, np.uint8))
    agg_arr = (_Agg * max(1, len(aggs)))()
    for i, (kind, ci) in enumerate(aggs):
        agg_arr[i].kind, agg_arr[i].col = AGG[kind], ci
    vp = (C.c_void_p * max(1, len(aggs)))(*[o.ctypes.data for o in outs])
    vv = (C.c_void_p * max(1, len(aggs)))(*[o.ctypes.data for o in outv])
    p, n = _prog(program)
    g = lib().or_group_by_agg(C.byref(key.c), _cols(cols), len(cols), p, n, agg_arr, len(aggs),
                              C.c_int64(nrows), sum_mode, C.c_int64(maxg), keys.ctypes.data_as(C.c_void_p),
                              kvalid.ctypes.data_as(C.c_void_p), vp, vv)
    if g < 0:
        raise ValueError("oracle: group_by failed")
    return keys[:g].copy(), kvalid[:g].astype(bool), [(o[:g].copy(), v[:g].astype(bool))
                                                       for o, v in zip(outs, outv)]


def _input_col(cols: list[HostCol], program, nrows: int, kinds: set) -> HostCol:
    """One computed aggregation input: the program evaluated by or_eval (the
    elementwise restatement).  A Boolean input sums as IdxSize counts
    (polars-expr/src/reduce/sum.rs:147-180 BoolSumReducer) and averages as
    0 / 1 Float64 (reduce/mean.rs)."""
    if nrows == 0:
        # no row: the program's dtype from one all-zero row of the same columns
        probe = [HostCol(np.zeros(1, np.bool_ if c.code == BOOL else _NP_OF[c.code])) for c in cols]
        dt, _, _ = eval_program(probe, program, 1)
        v, valid = np.zeros(0, np.bool_ if dt == BOOL else _NP_OF[dt]), np.zeros(0, bool)
    else:
        dt, v, valid = eval_program(cols, program, nrows)
    if dt == BOOL:
        v = v.astype(np.float64 if "mean" in kinds else np.uint32)
    return HostCol(np.ascontiguousarray(v), valid)


def group_by_agg_inputs(key: HostCol | None, cols: list[HostCol], program, inputs: list, aggs: list[tuple[str, int]],
                        nrows: int, sum_mode: int = SUM_EXACT):
    """Aggregations over computed inputs, the partitionable group-by's
    pre-aggregated expressions (polars-plan/src/plans/aexpr/properties/
    general.rs:303-356 can_pre_agg: Agg over BinaryExpr / Ternary / Cast /
    elementwise Function): each input program is evaluated over every row by
    or_eval and aggregated as a column (agg column index len(cols) + j names
    inputs[j]).  key None: a global reduction (select(aggs); reduce/sum.rs:112
    reduce_ca and siblings), one group -- and one output row even when no row
    is selected: sum / len / count 0, mean / min / max / first / last null
    (the reducers' init values, reduce/sum.rs:94, len.rs, count.rs; mean and
    min / max finish an empty state as null).  Returns (keys, key_valid,
    [(values, valid)]) like group_by_agg."""
    nc = len(cols)
    extra = []
    for j, prog in enumerate(inputs):
        kinds = {k for k, c in aggs if c == nc + j}
        extra.append(_input_col(cols, prog, nrows, kinds))
    allc = list(cols) + extra
    k = key if key is not None else HostCol(np.zeros(nrows, np.int64))
    keys, kvalid, outs = group_by_agg(k, allc, program, aggs, nrows, sum_mode)
    if key is None and keys.shape[0] == 0:
        keys, kvalid = np.zeros(1, np.int64), np.ones(1, bool)
        empty = []
        for (kind, ci), (o, _) in zip(aggs, outs):
            ok = kind in ("sum", "len", "count")
            empty.append((np.zeros(1, o.dtype), np.array([ok])))
        outs = empty
    return keys, kvalid, outs


def _row_words(values: np.ndarray, valid: np.ndarray | None) -> np.ndarray:
    """One key column as 2 uint64 words per row (validity, canonical value):
    the unordered row encoding of polars-core/src/chunked_array/ops/
    row_encode.rs:11 up to a bijection (a null encodes as (0, 0); f64 by
    TotalOrd: -0.0 == 0.0, every NaN equal)."""
    n = values.shape[0]
    v = np.ones(n, bool) if valid is None else valid.astype(bool)
    if values.dtype == np.float64:
        w = values.view(np.uint64).copy()
        w[values == 0] = 0
        w[np.isnan(values)] = 0x7FF8000000000000
    elif values.dtype == np.bool_:
        w = values.astype(np.uint64)
    else:
        w = values.astype(np.int64).view(np.uint64)
    w = np.where(v, w, np.uint64(0))
    return np.stack([v.astype(np.uint64), w], axis=1)


def group_by_agg_multi(keys: list[tuple[np.ndarray, np.ndarray | None]], cols: list[HostCol], program,
                       aggs: list[tuple[str, int]], nrows: int, sum_mode: int = SUM_EXACT):
    """Group-by on several key columns, restating DataFrame::group_by_with_series
    (polars-core/src/frame/group_by/mod.rs:91): rows are encoded
    (row_encode.rs:11) and grouped by the encoded tuple.  The tuples get dense
    ids here and or_group_by_agg aggregates by id.  Groups in first-occurrence
    order of the selected rows; each group's key tuple is its first selected
    row's.  Returns ([(key values, key valid)], [(agg values, agg valid)])."""
    enc = np.concatenate([_row_words(v, m) for v, m in keys], axis=1) if nrows else np.zeros((0, 2), np.uint64)
    if nrows:
        _, inv = np.unique(enc, axis=0, return_inverse=True)
        ids = inv.reshape(-1).astype(np.int64)
    else:
        ids = np.zeros(0, np.int64)
    gids, _, outs = group_by_agg(HostCol(ids), cols, program, aggs, nrows, sum_mode)
    if program:
        _, sel, selv = eval_program(cols, program, nrows)
        sel = sel & selv
    else:
        sel = np.ones(nrows, bool)
    first = np.full(ids.max() + 1 if nrows else 1, np.iinfo(np.int64).max, np.int64)
    rows = np.nonzero(sel)[0]
    np.minimum.at(first, ids[rows], rows)  # first selected row per tuple id
    rep = first[gids]
    out_keys = []
    for v, m in keys:
        out_keys.append((v[rep], np.ones(rep.size, bool) if m is None else m[rep].astype(bool)))
    return out_keys, outs


def join_inner(left: HostCol, right: HostCol, nulls_equal: bool = False):
    """Inner-join row pairs in (left, right) order: (left_idx, right_idx)."""
    cap = 1 << 16
    while True:
        ol = np.zeros(cap, np.int64)
        orr = np.zeros(cap, np.int64)
        n = lib().or_join_inner(C.byref(left.c), C.byref(right.c), int(nulls_equal), cap,
                                ol.ctypes.data, orr.ctypes.data)
        if n >= 0:
            return ol[:n].copy(), orr[:n].copy()
        cap *= 4


_HOW = {"left": 1, "full": 3, "semi": 4, "anti": 5}
_FLIP = {None: "none", "none": "none", "left": "right", "right": "left", "left_right": "right_left",
         "right_left": "left_right"}
_IDX_NULL = np.int64(2**32 - 1)  # IdxSize::MAX, the reference's null index


def _raw_join(left: HostCol, right: HostCol, how: str, nulls_equal: bool):
    if how == "inner":
        return join_inner(left, right, nulls_equal)
    cap = 1 << 16
    while True:
        ol = np.zeros(cap, np.int64)
        orr = np.zeros(cap, np.int64)
        n = lib().or_join(C.byref(left.c), C.byref(right.c), _HOW[how], int(nulls_equal), cap,
                          ol.ctypes.data, orr.ctypes.data)
        if n >= 0:
            return ol[:n].copy(), orr[:n].copy()
        cap *= 4


def _sort_pairs(ol: np.ndarray, orr: np.ndarray, by: list[str]):
    """Stable sort of the pairs by the listed index columns, a null (-1)
    index last (SortMultipleOptions maintain_order + nulls_last)."""
    if not by or ol.size == 0:
        return ol, orr
    cols = {"a": np.where(ol < 0, _IDX_NULL, ol), "b": np.where(orr < 0, _IDX_NULL, orr)}
    perm = np.lexsort(tuple(cols[c] for c in reversed(by)))  # lexsort is stable
    return ol[perm], orr[perm]


def join(left: HostCol, right: HostCol, how: str = "inner", nulls_equal: bool = False,
         maintain_order: str | None = "none"):
    """Row pairs of a join of any type in the reference's order for
    `maintain_order`: (left_idx, right_idx) with -1 as the null index;
    semi / anti: (left rows, None).
      inner   pairs in (left, right) order; "right" / "right_left" sort them
              by the right index (hash_join/mod.rs _inner_join orders);
      left    left order (the reference's left join is always ordered);
              "right" / "right_left" stably sort by the raw right index,
              whose null is IdxSize::MAX (dispatch_left_right.rs:143
              maintain_order_idx);
      right   the left join with the sides swapped and the order flipped
              (dispatch_left_right.rs:19);
      full    stable sort by the listed columns, nulls last
              (hash_join/mod.rs:164); "none" leaves the order unspecified.
    """
    order = maintain_order or "none"
    if how == "right":
        r, l = join(right, left, "left", nulls_equal, _FLIP[order])
        return l, r
    ol, orr = _raw_join(left, right, how, nulls_equal)
    if how in ("semi", "anti"):
        return ol, None
    if how in ("inner", "left"):
        if order in ("right", "right_left"):
            return _sort_pairs(ol, orr, ["b", "a"] if how == "inner" else ["b"])
        return ol, orr
    by = {"none": [], "left": ["a"], "left_right": ["a", "b"], "right": ["b"], "right_left": ["b", "a"]}[order]
    return _sort_pairs(ol, orr, by)


def join_multi(left_keys: list[tuple[np.ndarray, np.ndarray | None]],
               right_keys: list[tuple[np.ndarray, np.ndarray | None]], how: str = "inner",
               nulls_equal: bool = False, maintain_order: str | None = "none"):
    """`join` on several key columns: tuples encoded to dense ids as in
    join_inner_multi, then joined as one key."""
    lc, rc = _multi_ids(left_keys, right_keys, nulls_equal)
    return join(lc, rc, how, nulls_equal, maintain_order)


def _multi_ids(left_keys, right_keys, nulls_equal: bool):
    nl, nr = left_keys[0][0].shape[0], right_keys[0][0].shape[0]
    enc_l = np.concatenate([_row_words(v, m) for v, m in left_keys], axis=1)
    enc_r = np.concatenate([_row_words(v, m) for v, m in right_keys], axis=1)
    enc = np.concatenate([enc_l, enc_r], axis=0)
    if nl + nr:
        _, inv = np.unique(enc, axis=0, return_inverse=True)
        ids = inv.reshape(-1).astype(np.int64)
    else:
        ids = np.zeros(0, np.int64)

    def valid(keys, n):
        v = np.ones(n, bool)
        if not nulls_equal:
            for _, m in keys:
                if m is not None:
                    v &= m.astype(bool)
        return None if v.all() else v

    return HostCol(ids[:nl].copy(), valid(left_keys, nl)), HostCol(ids[nl:].copy(), valid(right_keys, nr))


def join_inner_multi(left_keys: list[tuple[np.ndarray, np.ndarray | None]],
                     right_keys: list[tuple[np.ndarray, np.ndarray | None]], nulls_equal: bool = False):
    """Inner join on several key columns, restating the reference's multi-key
    join (polars-ops/src/frame/join/mod.rs:625 prepare_keys_multiple): both
    sides' key tuples are row-encoded (row_encode.rs:11) and joined as one
    key; without nulls_equal a tuple holding a null is a null key
    (encode_rows_vertical_par_unordered_broadcast_nulls).  Here equal tuples
    get one dense id and or_join_inner joins the ids.  Pairs in (left, right)
    order."""
    nl, nr = left_keys[0][0].shape[0], right_keys[0][0].shape[0]
    enc_l = np.concatenate([_row_words(v, m) for v, m in left_keys], axis=1)
    enc_r = np.concatenate([_row_words(v, m) for v, m in right_keys], axis=1)
    enc = np.concatenate([enc_l, enc_r], axis=0)
    if nl + nr:
        _, inv = np.unique(enc, axis=0, return_inverse=True)
        ids = inv.reshape(-1).astype(np.int64)
    else:
        ids = np.zeros(0, np.int64)

    def valid(keys, n):
        v = np.ones(n, bool)
        if not nulls_equal:
            for _, m in keys:
                if m is not None:
                    v &= m.astype(bool)
        return None if v.all() else v

    return join_inner(HostCol(ids[:nl].copy(), valid(left_keys, nl)), HostCol(ids[nl:].copy(), valid(right_keys, nr)),
                      nulls_equal)


def arg_sort(col: HostCol, descending: bool = False, nulls_last: bool = False) -> np.ndarray:
    out = np.zeros(max(col.c.length, 1), np.int64)
    lib().or_arg_sort(C.byref(col.c), int(descending), int(nulls_last), out.ctypes.data)
    return out[: col.c.length].copy()


ROLLING_REFERENCE, ROLLING_EXACT = 0, 1


def arg_sort_multi(cols: list[tuple[np.ndarray, np.ndarray | None]], descending: list[bool],
                   nulls_last: list[bool]) -> np.ndarray:
    """Stable multi-column arg-sort restating arg_sort_multiple_impl
    (polars-core/src/chunked_array/ops/sort/arg_sort_multiple.rs:24):
    lexicographic over the columns; per column TotalOrd on the values
    (NaN greatest, -0.0 == 0.0), reversed when descending, and nulls first or
    last by that column's nulls_last alone; ties keep row order
    (maintain_order)."""
    n = cols[0][0].shape[0]
    lex = []
    for (v, m), desc, nl in reversed(list(zip(cols, descending, nulls_last))):
        valid = np.ones(n, bool) if m is None else m.astype(bool)
        w = v.astype(np.float64) + 0.0 if v.dtype == np.float64 else v.astype(np.int64)
        w = np.where(valid, w, w[valid][0] if valid.any() else 0)
        _, rank = np.unique(w, return_inverse=True)   # NaNs equal and last
        rank = rank.reshape(-1).astype(np.int64)
        if desc:
            rank = rank.max(initial=0) - rank
        rank = np.where(valid, rank, 0)
        flag = np.where(valid, 0, 1) if nl else np.where(valid, 1, 0)
        lex += [rank, flag]
    return np.lexsort(lex) if n else np.zeros(0, np.int64)


def rolling(col: HostCol, kind: str, window_size: int, min_periods: int | None = None, center: bool = False,
            mode: int = ROLLING_REFERENCE):
    """rolling_sum / rolling_mean -> (values, valid).  mode 0 restates the
    reference's Kahan sliding window; mode 1 is the exact window sum."""
    n = col.c.length
    mp = window_size if min_periods is None else min_periods
    k = {"sum": 1, "mean": 2, "min": 3, "max": 4}[kind]
    of = np.zeros(max(n, 1), np.float64)
    oi = np.zeros(max(n, 1), np.int64)
    ov = np.zeros(max(n, 1), np.uint8)
    lib().or_rolling(C.byref(col.c), k, window_size, mp, int(center), mode, of.ctypes.data, oi.ctypes.data,
                     ov.ctypes.data)
    isint = k in (1, 3, 4) and col.code != F64
    vals = (oi if isint else of)[:n].copy()
    return vals, ov[:n].astype(bool)


def rolling_var(col: HostCol, window_size: int, min_periods: int | None = None, center: bool = False,
                ddof: int = 1, std: bool = False, mode: int = ROLLING_REFERENCE):
    """rolling_var / rolling_std -> (values, valid).  mode 0 restates the
    reference's MomentWindow<VarianceMoment> (a sliding Welford VarState);
    mode 1 is the exact form the GPU computes (or_rolling_var)."""
    n = col.c.length
    mp = window_size if min_periods is None else min_periods
    of = np.zeros(max(n, 1), np.float64)
    ov = np.zeros(max(n, 1), np.uint8)
    lib().or_rolling_var(C.byref(col.c), window_size, mp, int(center), ddof, int(std), mode, of.ctypes.data,
                         ov.ctypes.data)
    return of[:n].copy(), ov[:n].astype(bool)


def fsum(x: np.ndarray) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().or_fsum(x.ctypes.data, x.shape[0])


def baseline_filter_groupby_sum(key: np.ndarray, pred: np.ndarray, k: float, sums: list[np.ndarray],
                                threads: int) -> tuple[int, float]:
    ptrs = (C.c_void_p * len(sums))(*[s.ctypes.data for s in sums])
    chk = C.c_double(0.0)
    g = lib().or_baseline_filter_groupby_sum(key.ctypes.data, pred.ctypes.data, k, ptrs, len(sums),
                                             key.shape[0], threads, C.byref(chk))
    return int(g), chk.value


def baseline_filter(pred: np.ndarray, k: float, cols: list[np.ndarray], threads: int) -> list[np.ndarray]:
    """CPU baseline of filter(pred > k).collect() (or_baseline_filter): every
    8-byte column compacted by the mask, row order kept."""
    n = pred.shape[0]
    cols = [np.ascontiguousarray(c).view(np.uint64) for c in cols]
    outs = [np.empty(n, dtype=np.uint64) for _ in cols]
    ip = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    op = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    m = lib().or_baseline_filter(np.ascontiguousarray(pred, dtype=np.float64).ctypes.data, k, ip, len(cols), n,
                                 threads, op)
    return [o[:m] for o in outs]


def baseline_sort_rolling(key: np.ndarray, cols: list[np.ndarray], roll: int, window: int,
                          threads: int) -> tuple[list[np.ndarray], np.ndarray, float]:
    """CPU baseline of configs[2] (or_baseline_sort_rolling): sort the frame
    by `key` (stable), gather every column, rolling_mean(window) of
    cols[roll].  Returns (sorted columns, rolling output, checksum)."""
    n = key.shape[0]
    key = np.ascontiguousarray(key, dtype=np.int64)
    cols = [np.ascontiguousarray(c).view(np.uint64) for c in cols]
    outs = [np.empty(n, dtype=np.uint64) for _ in cols]
    roll_out = np.empty(n, dtype=np.float64)
    ip = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    op = (C.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
    chk = lib().or_baseline_sort_rolling(key.ctypes.data, ip, len(cols), roll, n, window, threads, op,
                                         roll_out.ctypes.data)
    return outs, roll_out, chk


def baseline_join_inner(pk: np.ndarray, pv: np.ndarray, bk: np.ndarray, bv: np.ndarray,
                        threads: int) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """CPU baseline of configs[3] (or_baseline_join_inner): inner join on one
    Int64 key, probe rows in order within each thread's chunk, materialised
    (probe key, probe payload, build payload)."""
    np_, nb = pk.shape[0], bk.shape[0]
    cap = np_ * 2 + 16
    ok = np.empty(cap, dtype=np.int64)
    opv = np.empty(cap, dtype=np.float64)
    obv = np.empty(cap, dtype=np.float64)
    n = lib().or_baseline_join_inner(pk.ctypes.data, pv.ctypes.data, np_, bk.ctypes.data, bv.ctypes.data, nb,
                                     threads, ok.ctypes.data, opv.ctypes.data, obv.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("baseline join: more output rows than the buffer holds")
    return ok[:n], opv[:n], obv[:n]


def float_sum(x: np.ndarray, valid: np.ndarray | None = None) -> float:
    """The reference's keyless f64 sum of one chunk (polars-compute/src/
    float_sum.rs sum_arr_as_f64: 16-lane stripes, 128-value pairwise
    blocks); null values add +0.0."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    v = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    return lib().or_float_sum(x.ctypes.data, None if v is None else v.ctypes.data, x.shape[0])


def var_welford(x: np.ndarray, part: np.ndarray | None = None, ddof: int = 1) -> float:
    """The streaming group-by's variance of one group's values in row order
    (VarState.insert_one per row; one state per `part` id, combined in
    order); NaN for None."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    p = np.zeros(x.shape[0], np.int64) if part is None else np.ascontiguousarray(part, dtype=np.int64)
    return lib().or_var_welford(x.ctypes.data, p.ctypes.data, x.shape[0], ddof)


def var_chunked(x: np.ndarray, ddof: int = 1) -> float:
    """The in-memory keyless variance (moment.rs var: VarState::new per
    128-value chunk, combined in order); NaN for None."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    return lib().or_var_chunked(x.ctypes.data, x.shape[0], ddof)
