"""ctypes binding of the C-ABI in include/polaroid_gpu.h.

The product path always goes through libpolaroid_gpu.so; there is no CPU
fallback.  If the library is missing the import fails loudly.
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PLGPU_LIB: another build of the library (the checked build of
# `make CHECKS=1`, libpolaroid_gpu_checked.so), for debugging runs only
LIB_PATH = os.environ.get("PLGPU_LIB") or os.path.join(_HERE, "libpolaroid_gpu.so")

# dtypes (enum plgpu_dtype)
BOOL, I32, I64, F64, U32, STR = 1, 2, 3, 4, 5, 6
I8, I16, U8, U16, U64, F32 = 7, 8, 9, 10, 11, 12
DTYPE_BYTES = {I32: 4, I64: 8, F64: 8, U32: 4, I8: 1, I16: 2, U8: 1, U16: 2, U64: 8, F32: 4}

# status codes
OK = 0
ERR_INVALID, ERR_SCHEMA, ERR_SHAPE, ERR_OOM, ERR_HIP, ERR_NO_DEVICE, ERR_CAPACITY = (
    -1, -2, -3, -4, -5, -6, -7)

# opcodes (enum plgpu_opcode)
OP = dict(
    COL=1, LIT_F64=2, LIT_I64=3, LIT_BOOL=4, LIT_NULL=5,
    ADD=10, SUB=11, MUL=12, TRUEDIV=13, NEG=14, ABS=15, CAST_F64=16, FLOORDIV=17, MOD=18, DIVIDE=19,
    CAST=50, XOR=51, FILL_NULL=52, IF_ELSE=53,
    EQ=20, NE=21, LT=22, LE=23, GT=24, GE=25, EQ_MISSING=26, NE_MISSING=27,
    AND=30, OR=31, NOT=32, IS_NULL=33, IS_NOT_NULL=34, IS_NAN=35, IS_FINITE=36,
    STR_STARTS_WITH=40, STR_ENDS_WITH=41, STR_CONTAINS=42,
)
AGG = dict(sum=1, mean=2, min=3, max=4, count=5, len=6, first=7, last=8, var=9, std=10)  # var / std: ddof << 8
MAX_COLS = 8
MAX_KEYS = 8


class Column(C.Structure):
    pass


RELEASE_FN = C.CFUNCTYPE(None, C.POINTER(Column))
Column._fields_ = [
    ("dtype", C.c_int32),
    ("device_id", C.c_int32),
    ("length", C.c_int64),
    ("offset", C.c_int64),
    ("null_count", C.c_int64),
    ("values", C.c_void_p),
    ("validity", C.c_void_p),
    ("release", C.c_void_p),
    ("private_data", C.c_void_p),
    ("data", C.c_void_p),  # PLGPU_STR bytes (Arrow buffers[2])
]


class _Imm(C.Union):
    _fields_ = [("f64", C.c_double), ("i64", C.c_int64)]


class Instr(C.Structure):
    _fields_ = [("op", C.c_int32), ("arg", C.c_int32), ("imm", _Imm)]


class Agg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("col", C.c_int32)]


class AggInput(C.Structure):
    """plgpu_agg_input: an aggregation input given as a program over the columns."""
    _fields_ = [("program", C.POINTER(Instr)), ("n_instr", C.c_int32), ("_pad", C.c_int32)]


class GroupByInfo(C.Structure):
    _fields_ = [
        ("rows_in", C.c_int64),
        ("rows_selected", C.c_int64),
        ("groups", C.c_int64),
        ("global_path_rows", C.c_int64),
        ("reruns", C.c_int32),
        ("lds_slots", C.c_int32),
        ("grid", C.c_int32),
        ("sum_inexact", C.c_int32),
        ("table_capacity", C.c_int64),
        ("main_kernel_ms", C.c_double),
        ("path", C.c_int32),
        ("sum_limbs", C.c_int32),
        ("local_range", C.c_int32),
        ("register_runs", C.c_int32),
        ("key_pack", C.c_int32),
        ("part_layout", C.c_int32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


# Every symbol declared in include/polaroid_gpu.h, with its signature.
_P = C.c_void_p
_COLP = C.POINTER(Column)
SIGNATURES = {
    "plgpu_abi_version": (C.c_int, []),
    "plgpu_last_error": (C.c_char_p, []),
    "plgpu_set_option": (C.c_int, [C.c_char_p, C.c_int64]),
    "plgpu_get_option": (C.c_int, [C.c_char_p, C.POINTER(C.c_int64)]),
    "plgpu_ktime_read": (C.c_int, [C.c_char_p, C.c_int64, C.c_int32]),
    "plgpu_release_cached": (C.c_int, []),
    "plgpu_debug_checks": (C.c_int, [C.POINTER(C.c_uint32)]),
    "plgpu_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "plgpu_set_device": (C.c_int, [C.c_int]),
    "plgpu_synchronize": (C.c_int, [_P]),
    "plgpu_alloc": (C.c_int, [C.POINTER(C.c_void_p), C.c_size_t, _P]),
    "plgpu_free": (C.c_int, [_P, _P]),
    "plgpu_memcpy_h2d": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "plgpu_memcpy_d2h": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "plgpu_memcpy_d2h_many": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_size_t), _P]),
    "plgpu_memcpy_d2d": (C.c_int, [_P, _P, C.c_size_t, _P]),
    "plgpu_column_release": (None, [_COLP]),
    "plgpu_expr_dtype": (C.c_int, [_COLP, C.c_int32, C.POINTER(Instr), C.c_int32, C.POINTER(C.c_int32)]),
    "plgpu_column_alloc": (C.c_int, [C.c_int32, C.c_int64, C.c_int32, C.c_int64, _COLP, _P]),
    "plgpu_ingest_chunk": (C.c_int, [_COLP, C.c_int64, C.c_int64, _P, _P, _P, C.c_int64, C.c_int64, _P]),
    "plgpu_eval": (C.c_int, [_COLP, C.c_int32, C.POINTER(Instr), C.c_int32, _COLP, _P]),
    "plgpu_filter": (C.c_int, [_COLP, C.c_int32, _COLP, _COLP, C.POINTER(C.c_int64), _P]),
    "plgpu_filter_expr": (C.c_int, [_COLP, C.c_int32, C.POINTER(Instr), C.c_int32, _COLP,
                                    C.POINTER(C.c_int64), _P]),
    "plgpu_group_by_agg": (C.c_int, [_COLP, _COLP, C.c_int32, C.POINTER(Instr), C.c_int32,
                                     C.POINTER(Agg), C.c_int32, C.c_int32, _COLP, _COLP,
                                     C.POINTER(GroupByInfo), _P]),
    "plgpu_group_by_agg_multi": (C.c_int, [_COLP, C.c_int32, _COLP, C.c_int32, C.POINTER(Instr), C.c_int32,
                                           C.POINTER(Agg), C.c_int32, C.c_int32, _COLP, _COLP,
                                           C.POINTER(GroupByInfo), _P]),
    "plgpu_group_by_agg_ex": (C.c_int, [_COLP, C.c_int32, _COLP, C.c_int32, C.POINTER(AggInput), C.c_int32,
                                        C.POINTER(Instr), C.c_int32, C.POINTER(Agg), C.c_int32, C.c_int32, _COLP,
                                        _COLP, C.POINTER(GroupByInfo), _P]),
    "plgpu_gb_record_words": (C.c_int, [_COLP, C.c_int32, C.POINTER(Agg), C.c_int32,
                                        C.POINTER(C.c_int32)]),
    "plgpu_gb_plan_bottoms": (C.c_int, [_COLP, _COLP, C.c_int32, C.POINTER(Agg), C.c_int32,
                                        C.POINTER(C.c_int32), _P]),
    "plgpu_gb_partial_begin": (C.c_int, [_COLP, _COLP, C.c_int32, C.POINTER(Instr), C.c_int32,
                                         C.POINTER(Agg), C.c_int32, C.POINTER(C.c_int32), C.c_int32,
                                         C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                         C.POINTER(GroupByInfo), _P]),
    "plgpu_gb_partial_export": (C.c_int, [_P, _P, C.POINTER(C.c_int64), _P]),
    "plgpu_gb_partial_free": (None, [_P]),
    "plgpu_gb_partial_wide": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "plgpu_gb_partial_set_wide": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                            C.POINTER(C.c_int32)]),
    "plgpu_gb_partial_record_words": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "plgpu_gb_route": (C.c_int, [_COLP, C.c_int32, _COLP, C.POINTER(C.c_int64), _P]),
    "plgpu_key_ranges": (C.c_int, [_COLP, C.c_int32, C.POINTER(C.c_int64), _P]),
    "plgpu_float_key_encode": (C.c_int, [_COLP, _COLP, _P]),
    "plgpu_key_pack": (C.c_int, [_COLP, C.c_int32, C.POINTER(C.c_int64), _COLP, C.POINTER(C.c_int32), _P]),
    "plgpu_key_unpack": (C.c_int, [_COLP, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_int64), _COLP, _P]),
    "plgpu_gb_merge": (C.c_int, [_P, C.c_int64, _COLP, C.c_int32, C.POINTER(Agg), C.c_int32,
                                 C.POINTER(C.c_int32), C.c_int32, _COLP, _COLP,
                                 C.POINTER(GroupByInfo), _P]),
    "plgpu_gb_merge_sources": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int32), _COLP,
                                         C.c_int32, C.POINTER(Agg), C.c_int32, C.c_int32, _COLP, _COLP,
                                         C.POINTER(GroupByInfo), _P]),
    "plgpu_gb_merge_sources_wide": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                              C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                              _COLP, C.c_int32, C.POINTER(Agg), C.c_int32, C.c_int32, _COLP, _COLP,
                                              C.POINTER(GroupByInfo), _P]),
    "plgpu_join_inner_multi": (C.c_int, [_COLP, _COLP, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _COLP, _COLP,
                                         _P]),
    "plgpu_join_inner": (C.c_int, [_COLP, _COLP, C.c_int32, C.c_int32, C.c_int32, _COLP, _COLP, _P]),
    "plgpu_join_inner_take": (C.c_int, [_COLP, _COLP, _COLP, C.c_int32, _COLP, C.c_int32, C.c_int32, C.c_int32,
                                        C.c_int32, _COLP, _COLP, C.POINTER(C.c_int64), _P]),
    "plgpu_join_inner_take_multi": (C.c_int, [_COLP, _COLP, C.c_int32, _COLP, C.c_int32, _COLP, C.c_int32, C.c_int32,
                                              C.c_int32, C.c_int32, _COLP, _COLP, C.POINTER(C.c_int64), _P]),
    "plgpu_join": (C.c_int, [_COLP, _COLP, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _COLP, _COLP, _P]),
    "plgpu_join_multi": (C.c_int, [_COLP, _COLP, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _COLP,
                                   _COLP, _P]),
    "plgpu_coalesce": (C.c_int, [_COLP, _COLP, _COLP, _P]),
    "plgpu_str_compare": (C.c_int, [_COLP, _COLP, C.c_char_p, C.c_int64, C.c_int32, _COLP, _P]),
    "plgpu_str_encode_short": (C.c_int, [_COLP, _COLP, C.POINTER(C.c_int32), _P]),
    "plgpu_str_decode_short": (C.c_int, [_COLP, _COLP, _P]),
    "plgpu_group_sq_dev": (C.c_int, [_COLP, _COLP, _COLP, _COLP, _COLP, _P]),
    "plgpu_var_finalize": (C.c_int, [_COLP, _COLP, C.c_int32, C.c_int32, _COLP, _P]),
    "plgpu_gather": (C.c_int, [_COLP, C.c_int32, _COLP, _COLP, _P]),
    "plgpu_hash_partition": (C.c_int, [_COLP, C.c_int32, C.c_int32, C.c_int32, _COLP, C.POINTER(C.c_int64), _P]),
    "plgpu_gather_rows": (C.c_int, [_COLP, C.c_int32, _COLP, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _P]),
    "plgpu_pack_bits": (C.c_int, [_P, C.c_int64, _P, C.POINTER(C.c_int64), _P]),
    "plgpu_arg_sort_multi": (C.c_int, [_COLP, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), _COLP, _P]),
    "plgpu_arg_sort": (C.c_int, [_COLP, C.c_int32, C.c_int32, _COLP, _P]),
    "plgpu_rolling": (C.c_int, [_COLP, C.c_int32, C.c_int64, C.c_int64, C.c_int32, _COLP, _P]),
}

GB_MAX_ACC = 6
JOIN_ORDER = {None: 0, "none": 0, "left": 1, "right": 2, "left_right": 3, "right_left": 4}
JOIN_VALIDATE = {"m:m": 0, "1:m": 1, "m:1": 2, "1:1": 3}
JOIN_HOW = {"inner": 0, "left": 1, "right": 2, "full": 3, "semi": 4, "anti": 5}
ROLLING = {"sum": 1, "mean": 2, "min": 3, "max": 4, "var": 5, "std": 6}

_lib = None


def _share_hip_runtime_with_torch() -> None:
    """PyTorch-ROCm wheels bundle their own libamdhip64.so.7.  If this
    library were loaded first, the process would end up with two HIP
    runtimes (ours from /opt/rocm and torch's), which breaks whichever
    initialises second.  Importing torch first makes the dynamic loader
    resolve our DT_NEEDED libamdhip64.so.7 to torch's copy (same SONAME), so
    device pointers, streams and RCCL buffers are shared by one runtime."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libpolaroid_gpu.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"polaroid_amd native library missing: {LIB_PATH}. Build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C polaroid_amd/csrc)."
            )
        _share_hip_runtime_with_torch()
        handle = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


class PolaroidError(Exception):
    """Base error of the GPU executor."""


class ComputeError(PolaroidError):
    pass


class InvalidOperationError(PolaroidError):
    pass


class ShapeError(PolaroidError):
    pass


class DuplicateError(PolaroidError):
    pass


class OutOfMemoryError(PolaroidError):
    pass


class DeviceError(PolaroidError):
    pass


_ERRMAP = {
    ERR_INVALID: InvalidOperationError,
    ERR_SCHEMA: ComputeError,
    ERR_SHAPE: ShapeError,
    ERR_OOM: OutOfMemoryError,
    ERR_HIP: DeviceError,
    ERR_NO_DEVICE: DeviceError,
    ERR_CAPACITY: ComputeError,
}


def check(rc: int) -> None:
    if rc != OK:
        msg = lib().plgpu_last_error().decode(errors="replace")
        raise _ERRMAP.get(rc, PolaroidError)(msg)


def download_many(ranges: list) -> list:
    """[(device address, nbytes)] -> one host uint8 array per range, in one
    round trip (plgpu_memcpy_d2h_many)."""
    import numpy as np

    outs = [np.empty(nb, dtype=np.uint8) for _, nb in ranges]
    n = len(ranges)
    if n:
        dst = (C.c_void_p * n)(*[o.ctypes.data if o.nbytes else None for o in outs])
        src = (C.c_void_p * n)(*[p if nb else None for p, nb in ranges])
        sz = (C.c_size_t * n)(*[nb for _, nb in ranges])
        check(lib().plgpu_memcpy_d2h_many(n, dst, src, sz, None))
    return outs


def set_option(name: str, value: int) -> int:
    """Set a library option (test hooks / diagnostics, include/polaroid_gpu.h
    plgpu_set_option); returns the previous value."""
    prev = C.c_int64(0)
    check(lib().plgpu_get_option(name.encode(), C.byref(prev)))
    check(lib().plgpu_set_option(name.encode(), int(value)))
    return int(prev.value)


def release_cached() -> None:
    """Hand the library allocator's cached free blocks back to HIP."""
    check(lib().plgpu_release_cached())


def ktime_read(reset: bool = True) -> dict:
    """Per-kernel HIP-event times recorded while option "ktime" was 1
    (plgpu_ktime_read): {kernel name: (total ms, launches)}."""
    cap = 1 << 16
    buf = C.create_string_buffer(cap)
    check(lib().plgpu_ktime_read(buf, cap, int(bool(reset))))
    out = {}
    for line in buf.value.decode().splitlines():
        name, ms, cnt = line.split("\t")
        out[name] = (float(ms), int(cnt))
    return out


class option:
    """Context manager: `with option("no_pack", 1): ...` restores the value."""

    def __init__(self, name: str, value: int):
        self.name, self.value, self.prev = name, int(value), None

    def __enter__(self):
        self.prev = set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.name, self.prev)
        return False


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().plgpu_device_count(C.byref(n))
    return n.value if rc == OK else 0


class DeviceBuffer:
    """Raw device allocation from the library's stream-ordered pool."""

    __slots__ = ("ptr", "nbytes")

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(lib().plgpu_alloc(C.byref(p), C.c_size_t(max(int(nbytes), 1)), None))
        self.ptr = p.value
        self.nbytes = int(nbytes)

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.plgpu_free(C.c_void_p(self.ptr), None)
            self.ptr = None
