"""Expression DSL mirroring py-polars' `pl.col` / `pl.lit` / Expr API for the
filter -> arithmetic/comparison -> group_by-agg path.

An Expr is lowered to the postfix program of include/polaroid_gpu.h
(`plgpu_instr`), which the native library type-checks and runs per row on
the GPU (reference: polars-expr/src/expressions/{column,literal,binary}.rs).
"""

from __future__ import annotations

import builtins
from typing import Any, Sequence

from . import _native as N

_AGG_KINDS = ("sum", "mean", "min", "max", "count", "len")


class Expr:
    """A node of the expression tree."""

    __slots__ = ("kind", "args", "op", "value", "_name")

    def __init__(self, kind: str, args: Sequence["Expr"] = (), op: str | None = None,
                 value: Any = None, name: str | None = None):
        self.kind = kind          # col | lit | bin | un | agg | alias | len
        self.args = tuple(args)
        self.op = op
        self.value = value
        self._name = name

    # ---------------------------------------------------------- naming
    def output_name(self) -> str:
        if self.kind == "alias":
            return self.value
        if self.kind == "col":
            return self.value
        if self.kind == "len":
            return "len"
        if self.kind == "lit":
            return "literal"
        if self.kind == "ternary":  # when/then/otherwise is named after its first then()
            return self.args[1].output_name()
        return self.args[0].output_name()

    def meta_root_names(self) -> list[str]:
        if self.kind == "col":
            return [self.value]
        out: list[str] = []
        for a in self.args:
            for n in a.meta_root_names():
                if n not in out:
                    out.append(n)
        return out

    def __repr__(self) -> str:
        if self.kind == "col":
            return f'col("{self.value}")'
        if self.kind == "lit":
            return f"lit({self.value!r})"
        if self.kind == "bin":
            return f"[({self.args[0]!r}) {self.op} ({self.args[1]!r})]"
        if self.kind == "alias":
            return f'{self.args[0]!r}.alias("{self.value}")'
        if self.kind == "len":
            return "len()"
        if self.kind == "rolling":
            return f"{self.args[0]!r}.rolling_{self.op}{self.value}"
        if self.kind == "ternary":
            return f"when({self.args[0]!r}).then({self.args[1]!r}).otherwise({self.args[2]!r})"
        if self.kind == "cast":
            return f"{self.args[0]!r}.cast({self.value!r}, {self.op})"
        if self.kind == "fill_null":
            return f"{self.args[0]!r}.fill_null({self.args[1]!r})"
        return f"{self.args[0]!r}.{self.op}()"

    def __bool__(self):
        raise TypeError("the truth value of an Expr is ambiguous")

    # -------------------------------------------------------- operators
    def _bin(self, op: str, other: Any, swap: bool = False) -> "Expr":
        o = _to_expr(other)
        return Expr("bin", (o, self) if swap else (self, o), op=op)

    def __add__(self, o): return self._bin("+", o)
    def __radd__(self, o): return self._bin("+", o, True)
    def __sub__(self, o): return self._bin("-", o)
    def __rsub__(self, o): return self._bin("-", o, True)
    def __mul__(self, o): return self._bin("*", o)
    def __rmul__(self, o): return self._bin("*", o, True)
    def __truediv__(self, o): return self._bin("/", o)
    def __rtruediv__(self, o): return self._bin("/", o, True)
    def __floordiv__(self, o): return self._bin("//", o)
    def __rfloordiv__(self, o): return self._bin("//", o, True)
    def __mod__(self, o): return self._bin("%", o)
    def __rmod__(self, o): return self._bin("%", o, True)
    def __xor__(self, o): return self._bin("^", o)
    def __rxor__(self, o): return self._bin("^", o, True)
    def __gt__(self, o): return self._bin(">", o)
    def __ge__(self, o): return self._bin(">=", o)
    def __lt__(self, o): return self._bin("<", o)
    def __le__(self, o): return self._bin("<=", o)
    def __eq__(self, o): return self._bin("==", o)  # type: ignore[override]
    def __ne__(self, o): return self._bin("!=", o)  # type: ignore[override]
    def __and__(self, o): return self._bin("&", o)
    def __rand__(self, o): return self._bin("&", o, True)
    def __or__(self, o): return self._bin("|", o)
    def __ror__(self, o): return self._bin("|", o, True)
    def __neg__(self): return Expr("un", (self,), op="neg")
    def __abs__(self): return Expr("un", (self,), op="abs")
    def __invert__(self): return Expr("un", (self,), op="not")
    __hash__ = object.__hash__

    def gt(self, o): return self._bin(">", o)
    def ge(self, o): return self._bin(">=", o)
    def lt(self, o): return self._bin("<", o)
    def le(self, o): return self._bin("<=", o)
    def eq(self, o): return self._bin("==", o)
    def ne(self, o): return self._bin("!=", o)
    def eq_missing(self, o): return self._bin("eq_missing", o)
    def ne_missing(self, o): return self._bin("ne_missing", o)
    def add(self, o): return self._bin("+", o)
    def sub(self, o): return self._bin("-", o)
    def mul(self, o): return self._bin("*", o)
    def truediv(self, o): return self._bin("/", o)
    def floordiv(self, o): return self._bin("//", o)
    def mod(self, o): return self._bin("%", o)
    def xor(self, o): return self._bin("^", o)
    def and_(self, o): return self._bin("&", o)
    def or_(self, o): return self._bin("|", o)
    def not_(self): return Expr("un", (self,), op="not")
    def abs(self): return Expr("un", (self,), op="abs")
    def is_null(self): return Expr("un", (self,), op="is_null")
    def is_not_null(self): return Expr("un", (self,), op="is_not_null")
    def is_nan(self): return Expr("un", (self,), op="is_nan")
    def is_finite(self): return Expr("un", (self,), op="is_finite")

    @property
    def str(self) -> "_StrNamespace":
        """String functions (Expr.str): literal pattern tests."""
        return _StrNamespace(self)

    def cast(self, dtype, *, strict: bool = True, wrap_numerical: bool = False) -> "Expr":
        """Expr.cast.  Non-strict: a value that does not fit becomes null;
        wrap_numerical: integers wrap.  A strict cast is taken when it cannot
        fail (widening casts); otherwise it raises (see frame._check_strict)."""
        from .frame import Float64, DataType
        if dtype == "f64":
            dtype = Float64
        if not isinstance(dtype, DataType):
            raise N.InvalidOperationError(f"cast to {dtype!r} is not supported on the GPU executor")
        mode = "wrap" if wrap_numerical else ("strict" if strict else "non-strict")
        return Expr("cast", (self,), op=mode, value=dtype)

    def fill_null(self, value: Any = None) -> "Expr":
        """Expr.fill_null(value) (FunctionExpr::FillNull)."""
        if value is None:
            raise N.InvalidOperationError("fill_null needs a value (strategies are not supported on the GPU executor)")
        return Expr("fill_null", (self, _to_expr(value)), op="fill_null")

    def is_in(self, other: Sequence[Any], *, nulls_equal: bool = False) -> "Expr":
        """Expr.is_in over a literal collection: x == v0 | x == v1 | ...
        (BooleanFunction::IsIn); a null x gives null unless nulls_equal."""
        vals = list(other)
        if builtins.len(vals) > 15:
            raise N.InvalidOperationError("is_in takes at most 15 literal values on the GPU executor")
        has_null = any(v is None for v in vals)
        vals = [v for v in vals if v is not None]
        if nulls_equal:
            out = self.is_null() if has_null else None
            for v in vals:
                t = self.eq_missing(v)
                out = t if out is None else (out | t)
            return out if out is not None else self.is_null() & lit(False)
        out = None
        for v in vals:
            t = self == v
            out = t if out is None else (out | t)
        return out if out is not None else self.ne(self)  # empty: null for null x, else false

    def is_between(self, lower_bound: Any, upper_bound: Any, closed: str = "both") -> "Expr":
        """Expr.is_between (BooleanFunction::IsBetween): both / left / right / none."""
        if closed not in ("both", "left", "right", "none"):
            raise N.InvalidOperationError(f"invalid closed={closed!r}")
        lo = self >= lower_bound if closed in ("both", "left") else self > lower_bound
        hi = self <= upper_bound if closed in ("both", "right") else self < upper_bound
        return lo & hi

    def alias(self, name: str) -> "Expr":
        return Expr("alias", (self,), value=name)

    # ----------------------------------------------------- aggregations
    def sum(self): return Expr("agg", (self,), op="sum")
    def mean(self): return Expr("agg", (self,), op="mean")
    def min(self): return Expr("agg", (self,), op="min")
    def max(self): return Expr("agg", (self,), op="max")
    def count(self): return Expr("agg", (self,), op="count")
    def len(self): return Expr("agg", (self,), op="len")
    def std(self, ddof: int = 1): return Expr("agg", (self,), op="std", value=int(ddof))
    def var(self, ddof: int = 1): return Expr("agg", (self,), op="var", value=int(ddof))
    def first(self): return Expr("agg", (self,), op="first")
    def last(self): return Expr("agg", (self,), op="last")

    # ------------------------------------------------- window / ordering
    def rolling_sum(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Expr":
        """Fixed-window sum (Expr.rolling_sum)."""
        return _rolling(self, "sum", window_size, weights, min_samples, center)

    def rolling_mean(self, window_size: int, weights=None, *, min_samples: int | None = None,
                     center: bool = False) -> "Expr":
        """Fixed-window mean (Expr.rolling_mean)."""
        return _rolling(self, "mean", window_size, weights, min_samples, center)

    def rolling_min(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Expr":
        """Fixed-window minimum (Expr.rolling_min; a NaN in the window propagates)."""
        return _rolling(self, "min", window_size, weights, min_samples, center)

    def rolling_max(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Expr":
        """Fixed-window maximum (Expr.rolling_max; a NaN in the window propagates)."""
        return _rolling(self, "max", window_size, weights, min_samples, center)

    def rolling_var(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False, ddof: int = 1) -> "Expr":
        """Fixed-window variance (Expr.rolling_var; a non-finite value gives NaN)."""
        return _rolling(self, "var", window_size, weights, min_samples, center, ddof)

    def rolling_std(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False, ddof: int = 1) -> "Expr":
        """Fixed-window standard deviation (Expr.rolling_std)."""
        return _rolling(self, "std", window_size, weights, min_samples, center, ddof)

    def sort(self, *, descending: bool = False, nulls_last: bool = False) -> "Expr":
        return Expr("sort", (self,), op="sort", value=(bool(descending), bool(nulls_last)))

    def arg_sort(self, *, descending: bool = False, nulls_last: bool = False) -> "Expr":
        return Expr("sort", (self,), op="arg_sort", value=(bool(descending), bool(nulls_last)))


def _rolling(e: Expr, kind: str, window_size: int, weights, min_samples, center, ddof: int = 0) -> Expr:
    if weights is not None:
        raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
    if not isinstance(window_size, int) or window_size < 1:
        raise N.InvalidOperationError("`window_size` must be a positive integer")
    ms = window_size if min_samples is None else int(min_samples)
    if ms > window_size:
        raise N.InvalidOperationError("`min_samples` should be <= `window_size`")
    if not 0 <= int(ddof) <= 255:
        raise N.InvalidOperationError("`ddof` must be in 0..255")
    return Expr("rolling", (e,), op=kind, value=(window_size, ms, bool(center), int(ddof)))


def _to_expr(v: Any) -> Expr:
    return v if isinstance(v, Expr) else lit(v)


class _Then:
    def __init__(self, branches: list):
        self._branches = branches

    def when(self, cond: Any) -> "_When":
        return _When(self._branches, _to_expr(cond))

    def otherwise(self, value: Any) -> Expr:
        out = _to_expr(value)
        for cond, val in reversed(self._branches):
            out = Expr("ternary", (cond, val, out), op="if_else")
        return out

    # a chain used without otherwise() ends in null, as in polars
    def _finish(self) -> Expr:
        return self.otherwise(None)

    def __getattr__(self, name: str):
        # pl.when(c).then(x).sum() / .alias(...): the chain as an expression
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._finish(), name)


class _When:
    def __init__(self, branches: list, cond: Expr):
        self._branches, self._cond = branches, cond

    def then(self, value: Any) -> _Then:
        return _Then(self._branches + [(self._cond, _to_expr(value))])


def when(condition: Any) -> _When:
    """pl.when(cond).then(a)[.when(c2).then(b)].otherwise(c) -> a ternary
    expression (if_then_else; a null condition takes the otherwise branch)."""
    return _When([], _to_expr(condition))


def col(name: str) -> Expr:
    return Expr("col", value=name)


def lit(value: Any) -> Expr:
    if isinstance(value, Expr):
        return value
    return Expr("lit", value=value)


def len() -> Expr:  # noqa: A001 - mirrors pl.len()
    return Expr("len")


def sum(name: str) -> Expr:  # noqa: A001
    return col(name).sum()


def mean(name: str) -> Expr:
    return col(name).mean()


def min(name: str) -> Expr:  # noqa: A001
    return col(name).min()


def max(name: str) -> Expr:  # noqa: A001
    return col(name).max()


def count(name: str) -> Expr:
    return col(name).count()


def first(name: str) -> Expr:
    return col(name).first()


def last(name: str) -> Expr:
    return col(name).last()


class _StrNamespace:
    """Expr.str: starts_with / ends_with / contains(literal=True), evaluated
    on the GPU as Boolean columns (frame._lower_strings)."""

    def __init__(self, e: Expr):
        self._e = e

    def _fn(self, op: str, pattern) -> Expr:
        if not isinstance(pattern, str):
            raise N.InvalidOperationError(f"str.{op} takes a string literal on the GPU executor")
        return Expr("strfn", (self._e,), op=op, value=pattern)

    def starts_with(self, prefix: str) -> Expr:
        return self._fn("starts_with", prefix)

    def ends_with(self, suffix: str) -> Expr:
        return self._fn("ends_with", suffix)

    def contains(self, pattern: str, *, literal: bool = False, strict: bool = True) -> Expr:
        if not literal and any(ch in pattern for ch in ".^$*+?()[]{}|\\"):
            raise N.InvalidOperationError("regex patterns are not supported on the GPU executor (use literal=True)")
        return self._fn("contains", pattern)


_BIN_OPS = {
    "+": "ADD", "-": "SUB", "*": "MUL", "/": "TRUEDIV", "//": "FLOORDIV", "%": "MOD", "div": "DIVIDE",
    "^": "XOR", "fill_null": "FILL_NULL",
    ">": "GT", ">=": "GE", "<": "LT", "<=": "LE", "==": "EQ", "!=": "NE",
    "eq_missing": "EQ_MISSING", "ne_missing": "NE_MISSING", "&": "AND", "|": "OR",
}
_UN_OPS = {
    "neg": "NEG", "abs": "ABS", "not": "NOT", "is_null": "IS_NULL",
    "is_not_null": "IS_NOT_NULL", "is_nan": "IS_NAN", "is_finite": "IS_FINITE",
    "cast_f64": "CAST_F64",
}


def lower(expr: Expr, col_index: dict[str, int], schema: dict[str, int]) -> list[tuple[int, int, Any]]:
    """Lower an (aggregation-free) Expr to a postfix program.

    Returns a list of (opcode, arg, imm) triples; `imm` is a float for
    LIT_F64 and an int otherwise.
    """
    out: list[tuple[int, int, Any]] = []

    def emit(e: Expr) -> None:
        k = e.kind
        if k == "alias":
            emit(e.args[0])
        elif k == "col":
            if e.value not in col_index:
                raise N.ComputeError(f'unable to find column "{e.value}"')
            out.append((N.OP["COL"], col_index[e.value], 0))
        elif k == "lit":
            v = e.value
            if v is None:
                out.append((N.OP["LIT_NULL"], 0, 0))  # untyped: takes the other operand's type
            elif isinstance(v, bool):
                out.append((N.OP["LIT_BOOL"], 0, int(v)))
            elif isinstance(v, int):
                if not -(2 ** 63) <= v < 2 ** 63:
                    raise N.InvalidOperationError(f"integer literal {v} does not fit Int64")
                out.append((N.OP["LIT_I64"], 0, v))
            elif isinstance(v, float):
                out.append((N.OP["LIT_F64"], 0, float(v)))
            else:
                raise N.InvalidOperationError(f"literal of type {type(v).__name__} is not supported")
        elif k in ("bin", "fill_null"):
            emit(e.args[0])
            emit(e.args[1])
            out.append((N.OP[_BIN_OPS[e.op]], 0, 0))
        elif k == "ternary":
            for a in e.args:
                emit(a)
            out.append((N.OP["IF_ELSE"], 0, 0))
        elif k == "cast":
            emit(e.args[0])
            out.append((N.OP["CAST"], e.value.code, 1 if e.op == "wrap" else 0))
        elif k == "un":
            emit(e.args[0])
            out.append((N.OP[_UN_OPS[e.op]], 0, 0))
        elif k in ("agg", "len"):
            raise N.InvalidOperationError(f"aggregation {e!r} is not allowed in this context")
        else:
            raise N.InvalidOperationError(f"unsupported expression {e!r}")

    emit(expr)
    if not out:
        raise N.InvalidOperationError("empty expression")
    return out


def to_instr_array(prog: list[tuple[int, int, Any]]):
    arr = (N.Instr * builtins.len(prog))()
    for i, (op, arg, imm) in enumerate(prog):
        arr[i].op = op
        arr[i].arg = arg
        if op == N.OP["LIT_F64"]:
            arr[i].imm.f64 = float(imm)
        else:
            arr[i].imm.i64 = int(imm)
    return arr
