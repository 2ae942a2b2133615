"""Series / DataFrame / LazyFrame mirroring py-polars' API over device columns.

Columns live in HBM as Arrow arrays (values buffer + LSB-first validity
bitmap).  `LazyFrame.collect()` plans the query the way polars-mem-engine
builds executors (polars-mem-engine/src/planner/lp.rs) and runs every node
through the C-ABI of libpolaroid_gpu.so; a Filter directly below a GroupBy
is pushed into the aggregation kernel (one pass over the data).
"""

from __future__ import annotations

import builtins
import ctypes as C
from typing import Any, Iterable, Sequence

import numpy as np

from . import _native as N
from .expr import Expr, col, lit, lower, to_instr_array


# ------------------------------------------------------------------ dtypes
class DataType:
    """A column dtype.  `code` is the physical device dtype (enum
    plgpu_dtype); the temporal types (Date, Datetime, Duration) are logical
    types over a physical integer, as in polars."""

    code = 0
    name = "?"
    np_dtype: Any = None
    logical = False

    def __repr__(self):
        return self.name

    def physical(self) -> "DataType":
        return _BY_CODE[self.code]


def _phys(code, name, np_dtype):
    t = type(name, (DataType,), {})
    t.code, t.name, t.np_dtype = code, name, np_dtype
    return t()


Int8, Int16, Int32, Int64 = (_phys(N.I8, "Int8", np.int8), _phys(N.I16, "Int16", np.int16),
                             _phys(N.I32, "Int32", np.int32), _phys(N.I64, "Int64", np.int64))
UInt8, UInt16, UInt32, UInt64 = (_phys(N.U8, "UInt8", np.uint8), _phys(N.U16, "UInt16", np.uint16),
                                 _phys(N.U32, "UInt32", np.uint32), _phys(N.U64, "UInt64", np.uint64))
Float32, Float64 = _phys(N.F32, "Float32", np.float32), _phys(N.F64, "Float64", np.float64)
Boolean = _phys(N.BOOL, "Boolean", np.bool_)
String = _phys(N.STR, "String", np.object_)  # UTF-8 as Arrow large_string (int64 offsets + bytes)
_BY_CODE = {d.code: d for d in (Int8, Int16, Int32, Int64, UInt8, UInt16, UInt32, UInt64, Float32, Float64,
                                Boolean, String)}
INTEGER_DTYPES = (Int8, Int16, Int32, Int64, UInt8, UInt16, UInt32, UInt64)
FLOAT_DTYPES = (Float32, Float64)
_TIME_UNITS = ("ns", "us", "ms")


class _Temporal(DataType):
    logical = True

    def __eq__(self, other):
        return type(other) is type(self) and repr(other) == repr(self)

    def __hash__(self):
        return hash(repr(self))


class Datetime(_Temporal):
    """Datetime(time_unit, time_zone): Int64 ticks since the Unix epoch (UTC)."""

    code, np_dtype = N.I64, np.int64

    def __init__(self, time_unit: str = "us", time_zone: str | None = None):
        if time_unit not in _TIME_UNITS:
            raise N.InvalidOperationError(f"invalid time_unit {time_unit!r}")
        self.time_unit, self.time_zone = time_unit, time_zone

    @property
    def name(self):
        return f"Datetime(time_unit={self.time_unit!r}, time_zone={self.time_zone!r})"


class Duration(_Temporal):
    """Duration(time_unit): Int64 ticks."""

    code, np_dtype = N.I64, np.int64

    def __init__(self, time_unit: str = "us"):
        if time_unit not in _TIME_UNITS:
            raise N.InvalidOperationError(f"invalid time_unit {time_unit!r}")
        self.time_unit = time_unit

    @property
    def name(self):
        return f"Duration(time_unit={self.time_unit!r})"


class _Date(_Temporal):
    """Date: Int32 days since the Unix epoch."""

    code, name, np_dtype = N.I32, "Date", np.int32


Date = _Date()


def _dtype_from_numpy(a: np.ndarray) -> DataType:
    k = a.dtype
    if k == np.bool_:
        return Boolean
    if k.kind in ("U", "S", "O"):
        return String
    if k.kind == "M":
        unit = np.datetime_data(k)[0]
        if unit not in _TIME_UNITS:
            raise N.InvalidOperationError(f"datetime64[{unit}] is not supported (ns / us / ms)")
        return Datetime(unit)
    if k.kind == "m":
        unit = np.datetime_data(k)[0]
        if unit not in _TIME_UNITS:
            raise N.InvalidOperationError(f"timedelta64[{unit}] is not supported (ns / us / ms)")
        return Duration(unit)
    for d in INTEGER_DTYPES + FLOAT_DTYPES:
        if k == d.np_dtype:
            return d
    if np.issubdtype(k, np.integer):
        return Int64
    if np.issubdtype(k, np.floating):
        return Float64
    raise N.InvalidOperationError(f"unsupported numpy dtype {k}")


def _pack_bits(mask: np.ndarray) -> np.ndarray:
    """bool array -> Arrow LSB-first bitmap padded to 8-byte words."""
    n = mask.shape[0]
    words = (n + 63) // 64
    packed = np.packbits(mask.astype(np.uint8), bitorder="little")
    out = np.zeros(words * 8, dtype=np.uint8)
    out[: packed.shape[0]] = packed
    return out


def _unpack_bits(buf: np.ndarray, offset: int, n: int) -> np.ndarray:
    bits = np.unpackbits(buf, bitorder="little")
    return bits[offset: offset + n].astype(bool)


class _Owned:
    """Keeps a library-produced column alive; releases it once."""

    __slots__ = ("col",)

    def __init__(self, col: N.Column):
        self.col = col

    def __del__(self):
        if self.col is not None and self.col.release and N._lib is not None:
            N._lib.plgpu_column_release(C.byref(self.col))
            self.col = None


# ------------------------------------------------------------------ Series
class Series:
    """A named Arrow array in device memory.

    A Categorical / Enum column arrives as an Arrow dictionary array and is
    kept as its codes (`_cat`: the unique dictionary strings and the UInt32
    indices into them, both on the device).  Its value is the strings: the
    first use that needs them gathers them on the device (`_col`), while
    the group-by keys on the codes directly (polars-core/src/frame/group_by/
    into_groups.rs:132-139 groups a Categorical by its physical codes)."""

    __slots__ = ("name", "_c", "_keep", "_logical", "_cat")

    @property
    def _col(self) -> N.Column:
        c = self._c
        if c is None:
            c = self._materialize_cat()
        return c

    @_col.setter
    def _col(self, col_: N.Column) -> None:
        self._c = col_
        self._cat = None

    def _materialize_cat(self) -> N.Column:
        """The strings of a Categorical column, gathered once from its
        dictionary by its codes (a null code gathers a null)."""
        dictionary, codes = self._cat
        strs = dictionary.gather(codes)
        self._c = strs._col
        self._keep = list(self._keep) + [strs]
        return self._c

    @classmethod
    def _categorical(cls, name: str, dictionary: "Series", codes: "Series") -> "Series":
        s = cls.__new__(cls)
        s.name = name
        s._c = None
        s._keep = [dictionary, codes]
        s._logical = None
        s._cat = (dictionary, codes)
        return s

    def _cat_codes(self) -> "tuple[Series, Series] | None":
        """(dictionary, UInt32 codes) of a Categorical column, else None."""
        return getattr(self, "_cat", None)

    def __init__(self, name: str = "", values: Any = None, dtype: DataType | None = None):
        self.name = name
        self._keep: list = []
        self._logical = dtype if dtype is not None and dtype.logical else None
        if values is None:
            values = []
        if isinstance(values, Series):
            self._c, self._keep, self._cat = values._c, values._keep, values._cat_codes()
            self._logical = values._logical_dtype()
            return
        validity = None
        if isinstance(values, np.ndarray):
            arr = values
        else:
            vals = list(values)
            validity = np.array([v is not None for v in vals], dtype=bool)
            if dtype is None:
                nonnull = [v for v in vals if v is not None]
                if nonnull and builtins.all(isinstance(v, str) for v in nonnull):
                    dtype = String
                elif any(isinstance(v, float) for v in nonnull):
                    dtype = Float64
                elif nonnull and builtins.all(isinstance(v, bool) for v in nonnull):
                    dtype = Boolean
                else:
                    dtype = Int64
            fill = False if dtype is Boolean else ("" if dtype is String else 0)
            arr = np.array([fill if v is None else v for v in vals], dtype=dtype.np_dtype)
            if validity.all():
                validity = None
        if isinstance(arr, np.ndarray) and arr.dtype.kind in ("M", "m") and dtype is None:
            dtype = _dtype_from_numpy(arr)
            self._logical = dtype
        if dtype is not None and arr.dtype != dtype.np_dtype:
            arr = arr.astype(dtype.np_dtype)
        dt = (dtype or _dtype_from_numpy(arr)).physical()
        self._upload(np.ascontiguousarray(arr), dt, validity)

    # construction helpers -------------------------------------------------
    def _upload_strings(self, arr, validity: np.ndarray | None) -> None:
        """Strings -> large_string buffers (int64 offsets, UTF-8 bytes) in HBM."""
        n = builtins.len(arr)
        enc = [(x if isinstance(x, (bytes, bytearray)) else str(x).encode()) if (validity is None or validity[i])
               else b"" for i, x in enumerate(arr)]
        offsets = np.zeros(n + 1, np.int64)
        if n:
            np.cumsum([builtins.len(b) for b in enc], out=offsets[1:])
        self._upload_string_buffers(offsets, np.frombuffer(b"".join(enc), np.uint8), validity)

    def _upload_string_buffers(self, offsets: np.ndarray, data: np.ndarray, validity: np.ndarray | None) -> None:
        n = int(offsets.shape[0]) - 1
        col_ = N.Column()
        col_.dtype, col_.length, col_.offset = N.STR, n, 0
        col_.null_count = 0 if validity is None else int((~validity).sum())
        self._keep = []
        for field, payload in (("values", np.ascontiguousarray(offsets, np.int64)),
                               ("data", np.ascontiguousarray(data, np.uint8))):
            buf = N.DeviceBuffer(payload.nbytes)
            if payload.nbytes:
                N.check(N.lib().plgpu_memcpy_h2d(C.c_void_p(buf.ptr), payload.ctypes.data_as(C.c_void_p),
                                                 payload.nbytes, None))
            setattr(col_, field, buf.ptr)
            self._keep.append(buf)
        if validity is not None:
            bits = _pack_bits(validity)
            mbuf = N.DeviceBuffer(bits.nbytes)
            N.check(N.lib().plgpu_memcpy_h2d(C.c_void_p(mbuf.ptr), bits.ctypes.data_as(C.c_void_p),
                                             bits.nbytes, None))
            col_.validity = mbuf.ptr
            self._keep.append(mbuf)
        self._col = col_

    def _upload(self, arr: np.ndarray, dt: DataType, validity: np.ndarray | None) -> None:
        if dt is String:
            return self._upload_strings(arr, validity)
        n = int(arr.shape[0])
        col_ = N.Column()
        col_.dtype = dt.code
        col_.length = n
        col_.offset = 0
        col_.null_count = 0 if validity is None else int((~validity).sum())
        if dt is Boolean:
            payload = _pack_bits(arr.astype(bool))
        else:
            payload = arr
        vbuf = N.DeviceBuffer(payload.nbytes)
        if payload.nbytes:
            N.check(N.lib().plgpu_memcpy_h2d(C.c_void_p(vbuf.ptr), payload.ctypes.data_as(C.c_void_p),
                                             payload.nbytes, None))
        col_.values = vbuf.ptr
        self._keep = [vbuf]
        if validity is not None:
            bits = _pack_bits(validity)
            mbuf = N.DeviceBuffer(bits.nbytes)
            N.check(N.lib().plgpu_memcpy_h2d(C.c_void_p(mbuf.ptr), bits.ctypes.data_as(C.c_void_p),
                                             bits.nbytes, None))
            col_.validity = mbuf.ptr
            self._keep.append(mbuf)
        self._col = col_

    @classmethod
    def from_numpy(cls, name: str, values: np.ndarray, valid: np.ndarray | None = None,
                   dtype: DataType | None = None) -> "Series":
        """Upload a numpy array (plus optional boolean validity) to the device."""
        s = cls.__new__(cls)
        s.name = name
        arr = np.ascontiguousarray(values)
        dt = dtype or _dtype_from_numpy(arr)
        s._logical = dt if dt.logical else None
        if dt is String:
            s._upload_strings(list(arr), None if valid is None else np.asarray(valid, dtype=bool))
            return s
        if arr.dtype.kind in ("M", "m"):
            arr = arr.view(np.int64)
        if arr.dtype != dt.np_dtype:
            arr = arr.astype(dt.np_dtype)
        s._upload(arr, dt.physical(), None if valid is None else np.asarray(valid, dtype=bool))
        return s

    def slice(self, offset: int, length: int | None = None) -> "Series":
        """Zero-copy slice (Arrow offset semantics), like Series.slice."""
        n = self.len()
        offset = max(0, min(int(offset), n))
        length = n - offset if length is None else max(0, min(int(length), n - offset))
        s = Series.__new__(Series)
        s.name = self.name
        s._logical = self._logical_dtype()
        c = N.Column.from_buffer_copy(self._col)
        c.offset = self._col.offset + offset
        c.length = length
        c.release = None
        c.private_data = None
        c.null_count = -1 if self._col.validity else 0
        s._col = c
        s._keep = [self]
        return s

    @classmethod
    def _from_native(cls, name: str, col_: N.Column, logical: DataType | None = None) -> "Series":
        s = cls.__new__(cls)
        s.name = name
        s._col = col_
        s._keep = [_Owned(col_)] if col_.release else []
        s._logical = logical
        return s

    def _logical_dtype(self) -> DataType | None:
        return getattr(self, "_logical", None)

    def _with_logical(self, logical: DataType | None) -> "Series":
        self._logical = logical
        return self

    @classmethod
    def from_device(cls, name: str, dtype: DataType, values_ptr: int, length: int,
                    validity_ptr: int | None = None, offset: int = 0, keepalive: Any = None,
                    null_count: int = -1, data_ptr: int | None = None) -> "Series":
        """Borrow existing device buffers (e.g. torch tensors) without copying.
        String: `values_ptr` holds the int64 offsets, `data_ptr` the bytes."""
        s = cls.__new__(cls)
        s.name = name
        s._logical = dtype if dtype.logical else None
        c = N.Column()
        c.dtype = dtype.code
        c.length = int(length)
        c.offset = int(offset)
        c.null_count = 0 if validity_ptr is None else int(null_count)
        c.values = int(values_ptr)
        c.validity = int(validity_ptr) if validity_ptr else None
        if data_ptr:
            c.data = int(data_ptr)
        s._col = c
        s._keep = [keepalive] if keepalive is not None else []
        return s

    @classmethod
    def from_torch(cls, name: str, tensor, validity=None) -> "Series":
        import torch

        m = {torch.int64: Int64, torch.int32: Int32, torch.float64: Float64, torch.float32: Float32,
             torch.int16: Int16, torch.int8: Int8, torch.uint8: UInt8}
        if tensor.dtype not in m or not tensor.is_cuda or not tensor.is_contiguous():
            raise N.InvalidOperationError("from_torch needs a contiguous int / float GPU tensor")
        vptr = validity.data_ptr() if validity is not None else None
        return cls.from_device(name, m[tensor.dtype], tensor.data_ptr(), tensor.numel(), vptr,
                               keepalive=(tensor, validity))

    def to_torch(self):
        """The values as a new torch tensor on the device (a device-to-device
        copy; nulls keep whatever their slots hold).  Fixed-width dtypes only."""
        import torch

        m = {"Int64": torch.int64, "Int32": torch.int32, "Float64": torch.float64, "Float32": torch.float32,
             "Int16": torch.int16, "Int8": torch.int8, "UInt8": torch.uint8, "UInt32": torch.int32,
             "UInt64": torch.int64, "UInt16": torch.int16}
        phys = _BY_CODE[self._col.dtype]
        if phys.name not in m:
            raise N.InvalidOperationError(f"to_torch: {phys} has no torch tensor form")
        t = torch.empty(self.len(), dtype=m[phys.name], device="cuda")
        nb = t.element_size() * self.len()
        if nb:
            src = int(self._col.values) + int(self._col.offset) * t.element_size()
            N.check(N.lib().plgpu_memcpy_d2d(C.c_void_p(t.data_ptr()), C.c_void_p(src), nb, None))
            N.check(N.lib().plgpu_synchronize(None))
        return t

    # properties -----------------------------------------------------------
    @property
    def dtype(self) -> DataType:
        if self._c is None:  # Categorical: its values are strings
            return String
        return self._logical_dtype() or _BY_CODE[self._c.dtype]

    def len(self) -> int:
        return int((self._c if self._c is not None else self._cat[1]._col).length)

    def __len__(self) -> int:
        return self.len()

    def alias(self, name: str) -> "Series":
        s = Series.__new__(Series)
        s.name, s._c, s._keep, s._logical, s._cat = name, self._c, self._keep, self._logical_dtype(), self._cat_codes()
        return s

    # host materialisation (tests / display only) --------------------------
    def _download(self, ptr, nbytes) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            N.check(N.lib().plgpu_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), nbytes, None))
        return out

    def validity_numpy(self) -> np.ndarray:
        n, off = self.len(), int(self._col.offset)
        if not self._col.validity:
            return np.ones(n, dtype=bool)
        nb = (off + n + 7) // 8
        return _unpack_bits(self._download(self._col.validity, nb), off, n)

    def _string_buffers(self) -> tuple[np.ndarray, np.ndarray]:
        """(offsets of this slice rebased to 0, its bytes) on the host."""
        n, off = self.len(), int(self._col.offset)
        offs = self._download(self._col.values + off * 8, (n + 1) * 8).view(np.int64).copy()
        base = int(offs[0]) if n + 1 else 0
        data = self._download(self._col.data + base if self._col.data else 0, int(offs[-1]) - base)
        return offs - base, data

    def to_numpy(self) -> np.ndarray:
        """Values as numpy (null slots hold whatever the buffer holds)."""
        n, off = self.len(), int(self._col.offset)
        dt = self.dtype
        if dt is String:
            offs, data = self._string_buffers()
            raw = data.tobytes()
            return np.array([raw[offs[i]:offs[i + 1]].decode() for i in range(n)], dtype=object)
        if dt is Boolean:
            nb = (off + n + 7) // 8
            return _unpack_bits(self._download(self._col.values, nb), off, n)
        eb = np.dtype(dt.np_dtype).itemsize
        raw = self._download(self._col.values + off * eb if self._col.values else 0, n * eb)
        return raw.view(dt.np_dtype).copy()

    # Arrow interchange (polars DataFrames cross the plugin boundary as Arrow)
    @classmethod
    def from_arrow(cls, name: str, arr) -> "Series":
        """Upload a pyarrow Array / ChunkedArray chunk by chunk (the buffers
        as they are: no host concatenation, no bitmap unpacking)."""
        import pyarrow as pa

        chunks = list(arr.chunks) if isinstance(arr, pa.ChunkedArray) else [arr]
        return _ingest_chunks(name, chunks, arr.type)

    def to_arrow(self):
        import pyarrow as pa

        if self._cat_codes() is not None:
            # Categorical (gathered strings or not): its codes and dictionary
            # as an Arrow dictionary array (what polars exports it as)
            dictionary, codes = self._cat
            return pa.DictionaryArray.from_arrays(codes.to_arrow(), dictionary.to_arrow())
        if self.dtype is String:
            offs, data = self._string_buffers()
            valid = self.validity_numpy()
            vb = None if valid.all() else pa.py_buffer(np.packbits(valid, bitorder="little").tobytes())
            return pa.Array.from_buffers(pa.large_string(), self.len(),
                                         [vb, pa.py_buffer(offs.tobytes()), pa.py_buffer(data.tobytes())],
                                         null_count=int((~valid).sum()))
        phys = _BY_CODE[self._col.dtype]
        vals = self.to_numpy()
        valid = self.validity_numpy()
        arr = pa.array(vals, type=_ARROW_OF[phys.name], mask=None if valid.all() else ~valid)
        lg = self._logical_dtype()
        return arr.view(_arrow_logical(lg)) if lg is not None else arr

    def to_list(self) -> list:
        if self._logical_dtype() is not None:
            return self.to_arrow().to_pylist()
        vals = self.to_numpy().tolist()
        valid = self.validity_numpy()
        return [v if ok else None for v, ok in zip(vals, valid)]

    def null_count(self) -> int:
        return int((~self.validity_numpy()).sum())

    def __repr__(self) -> str:
        return f"shape: ({self.len()},)\nSeries: '{self.name}' [{self.dtype}]\n{self.to_list()[:20]}"

    # sort / rolling (Series.arg_sort, Series.sort, Series.rolling_*) ---------
    def arg_sort(self, *, descending: bool = False, nulls_last: bool = False) -> "Series":
        out = N.Column()
        if self.dtype in (Boolean, String):  # the multi-column sort handles these key types
            N.check(N.lib().plgpu_arg_sort_multi((N.Column * 1)(self._col), 1, (C.c_int32 * 1)(int(descending)),
                                                 (C.c_int32 * 1)(int(nulls_last)), C.byref(out), None))
        else:
            N.check(N.lib().plgpu_arg_sort(C.byref(self._col), int(descending), int(nulls_last), C.byref(out),
                                           None))
        return Series._from_native(self.name, out)

    def gather(self, idx: "Series") -> "Series":
        out = (N.Column * 1)()
        N.check(N.lib().plgpu_gather((N.Column * 1)(self._col), 1, C.byref(idx._col), out, None))
        return Series._from_native(self.name, out[0], self._logical_dtype())

    def sort(self, *, descending: bool = False, nulls_last: bool = False) -> "Series":
        return self.gather(self.arg_sort(descending=descending, nulls_last=nulls_last))

    def _cast_to(self, dtype: DataType) -> "Series":
        """Non-strict cast on the device (plgpu_eval of one CAST)."""
        return _eval(Expr("cast", (col(self.name),), op="non-strict", value=dtype),
                     DataFrame([self])).alias(self.name)._with_logical(None)

    def _rolling(self, kind: int, window_size: int, min_samples: int | None, center: bool,
                 ddof: int = 0) -> "Series":
        """Fixed windows over Int32 / Int64 / Float64 on the device; the other
        dtypes the way polars-time's rolling dispatch takes them
        (rolling_window/dispatch.rs:228): rolling_sum of Int8 / Int16 / UInt8 /
        UInt16 sums as Int64, means of integers are Float64; Float32 runs as
        Float64 and is rounded back; min / max keep the dtype.  var / std
        (dispatch.rs:478,526) run on the values as floats (`to_float`:
        integers as Float64; Float32 stays Float32, the variance rounded to
        Float32 before std's square root, as the reference's f32 sqrt)."""
        lg = self._logical_dtype()
        is_var = kind in (N.ROLLING["var"], N.ROLLING["std"])
        if is_var:
            if lg is not None:
                raise N.InvalidOperationError(f"rolling var / std of a {lg} column is not supported")
            if not 0 <= int(ddof) <= 255:  # the reference's ddof is a u8; packed into bits 8..15 below
                raise N.InvalidOperationError("`ddof` must be in 0..255")
            phys = _BY_CODE[self._col.dtype]
            src, f32 = self, phys is Float32
            if phys in (Int8, Int16, UInt8, UInt16, UInt32, UInt64, Float32):
                src = self._cast_to(Float64)
            out = N.Column()
            ms = window_size if min_samples is None else min_samples
            code = kind | (int(ddof) << 8) | ((1 << 16) if f32 and kind == N.ROLLING["std"] else 0)
            N.check(N.lib().plgpu_rolling(C.byref(src._col), code, int(window_size), int(ms), int(center),
                                          C.byref(out), None))
            res = Series._from_native(self.name, out)
            return res._cast_to(Float32) if f32 else res
        is_sum_mean = kind in (N.ROLLING["sum"], N.ROLLING["mean"])
        if lg is not None and is_sum_mean and not (kind == N.ROLLING["sum"] and isinstance(lg, Duration)):
            raise N.InvalidOperationError(f"rolling sum / mean of a {lg} column is not supported")
        phys = _BY_CODE[self._col.dtype]
        src, back = self, None
        if phys is UInt32 and kind == N.ROLLING["sum"]:
            raise N.InvalidOperationError("rolling_sum over UInt32 (wrapping at 32 bits) is not supported")
        if phys in (Int8, Int16, UInt8, UInt16, UInt32):
            src = self._cast_to(Int64)
            back = None if is_sum_mean else phys
        elif phys is Float32:
            src, back = self._cast_to(Float64), Float32
        elif phys is UInt64:
            raise N.InvalidOperationError("rolling windows over UInt64 are not supported on the GPU executor")
        out = N.Column()
        ms = window_size if min_samples is None else min_samples
        N.check(N.lib().plgpu_rolling(C.byref(src._col), kind, int(window_size), int(ms), int(center),
                                      C.byref(out), None))
        res = Series._from_native(self.name, out)
        if back is not None:
            res = res._cast_to(back)
        return res._with_logical(lg if not is_sum_mean or isinstance(lg, Duration) else None)

    def rolling_sum(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        return self._rolling(N.ROLLING["sum"], window_size, min_samples, center)

    def rolling_mean(self, window_size: int, weights=None, *, min_samples: int | None = None,
                     center: bool = False) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        return self._rolling(N.ROLLING["mean"], window_size, min_samples, center)

    def rolling_min(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        return self._rolling(N.ROLLING["min"], window_size, min_samples, center)

    def rolling_max(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        return self._rolling(N.ROLLING["max"], window_size, min_samples, center)

    def rolling_var(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False, ddof: int = 1) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        if min_samples is not None and min_samples > window_size:
            raise N.InvalidOperationError("`min_samples` should be <= `window_size`")
        return self._rolling(N.ROLLING["var"], window_size, min_samples, center, ddof)

    def rolling_std(self, window_size: int, weights=None, *, min_samples: int | None = None,
                    center: bool = False, ddof: int = 1) -> "Series":
        if weights is not None:
            raise N.InvalidOperationError("weighted rolling windows are not supported on the GPU executor")
        if min_samples is not None and min_samples > window_size:
            raise N.InvalidOperationError("`min_samples` should be <= `window_size`")
        return self._rolling(N.ROLLING["std"], window_size, min_samples, center, ddof)

    # eager conveniences mirroring Series.filter ------------------------------
    def filter(self, mask: "Series") -> "Series":
        out = (N.Column * 1)()
        n = C.c_int64(0)
        cols = (N.Column * 1)(self._col)
        m = mask._col
        N.check(N.lib().plgpu_filter(cols, 1, C.byref(m), out, C.byref(n), None))
        return Series._from_native(self.name, out[0], self._logical_dtype())


# ------------------------------------------------------------- ingestion
def _arrow_physical(t) -> DataType | None:
    """Arrow type -> device dtype of the path, logical for the temporal types
    (None: unsupported)."""
    import pyarrow as pa

    if t in (pa.string(), pa.large_string()):
        return String
    if pa.types.is_timestamp(t):
        return Datetime(t.unit, t.tz) if t.unit in _TIME_UNITS else None
    if pa.types.is_duration(t):
        return Duration(t.unit) if t.unit in _TIME_UNITS else None
    if t == pa.date32():
        return Date
    for d in INTEGER_DTYPES + FLOAT_DTYPES + (Boolean,):
        if t == _ARROW_OF[d.name]:
            return d
    return None


def _arrow_logical(dt: DataType):
    import pyarrow as pa

    if isinstance(dt, Datetime):
        return pa.timestamp(dt.time_unit, dt.time_zone)
    if isinstance(dt, Duration):
        return pa.duration(dt.time_unit)
    if dt is Date:
        return pa.date32()
    return _ARROW_OF[dt.name]


class _ArrowOf(dict):
    def __missing__(self, name):
        import pyarrow as pa

        self.update({"Int8": pa.int8(), "Int16": pa.int16(), "Int32": pa.int32(), "Int64": pa.int64(),
                     "UInt8": pa.uint8(), "UInt16": pa.uint16(), "UInt32": pa.uint32(), "UInt64": pa.uint64(),
                     "Float32": pa.float32(), "Float64": pa.float64(), "Boolean": pa.bool_(),
                     "String": pa.large_string()})
        return dict.__getitem__(self, name)


_ARROW_OF = _ArrowOf()


def _ingest_chunks(name: str, chunks: list, atype, sync: bool = True) -> Series:
    """Arrow chunks (host) -> one device column through plgpu_column_alloc /
    plgpu_ingest_chunk: every chunk's value, validity and string buffers are
    copied as they lie (Arrow offsets honoured), with one synchronisation at
    the end (none with sync=False: the caller synchronises once after all
    its columns, as the plugin's scan does)."""
    import pyarrow as pa

    if pa.types.is_dictionary(atype):
        # polars Categorical / Enum: the dictionary and the indices go to the
        # device as they are, and the strings are gathered there (a null
        # index gathers a null).  Chunks may carry different dictionaries.
        if builtins.len(chunks) > 1:
            chunks = list(pa.chunked_array(chunks, type=atype).unify_dictionaries().chunks)
        dict_arr = chunks[0].dictionary if chunks else pa.array([], atype.value_type)
        dictionary = _ingest_chunks(name, [dict_arr], dict_arr.type)
        if dictionary.dtype is not String:
            raise N.InvalidOperationError(f"column {name!r}: dictionary of {dict_arr.type} is not supported")
        idx = _ingest_chunks("__idx", [c.indices.cast(pa.uint32()) for c in chunks], pa.uint32())
        import pyarrow.compute as pc

        if dict_arr.null_count == 0 and pc.count_distinct(dict_arr).as_py() == builtins.len(dict_arr):
            # unique categories (polars' dictionaries are): equal strings <=>
            # equal codes, so the codes stand for the values; the strings are
            # gathered only where they are needed
            return Series._categorical(name, dictionary, idx)
        return dictionary.gather(idx).alias(name)
    if atype in (pa.string(), pa.utf8()):
        chunks = [c.cast(pa.large_string()) for c in chunks]
        atype = pa.large_string()
        sync = True  # the cast buffers die with this call: wait for their copies
    dt = _arrow_physical(atype)
    if dt is None:
        raise N.InvalidOperationError(f"column {name!r}: arrow type {atype} is not supported on the GPU")
    logical = dt if dt.logical else None
    dt = dt.physical()
    n = builtins.sum(builtins.len(c) for c in chunks)
    nulls = builtins.sum(c.null_count for c in chunks)
    spans = []
    str_bytes = 0
    for c in chunks:
        bufs = c.buffers()
        if dt is String:
            offs = np.frombuffer(bufs[1], np.int64, builtins.len(c) + 1, c.offset * 8) if builtins.len(c) else None
            b0, b1 = (int(offs[0]), int(offs[-1])) if offs is not None else (0, 0)
            spans.append((c, bufs, str_bytes))
            str_bytes += b1 - b0
        else:
            spans.append((c, bufs, 0))
    col_ = N.Column()
    N.check(N.lib().plgpu_column_alloc(dt.code, n, int(nulls > 0), str_bytes, C.byref(col_), None))
    out = Series._from_native(name, col_, logical)
    row = 0
    for c, bufs, byte in spans:
        m = builtins.len(c)
        if m:
            vb = bufs[0].address if (c.null_count and bufs[0] is not None) else None
            data = bufs[2].address if dt is String and bufs[2] is not None else None
            N.check(N.lib().plgpu_ingest_chunk(C.byref(out._col), row, byte, bufs[1].address, vb, data,
                                               c.offset, m, None))
        row += m
    if sync:
        N.check(N.lib().plgpu_synchronize(None))
    out._col.null_count = nulls
    return out


# --------------------------------------------------------------- DataFrame
class DataFrame:
    def __init__(self, data: Any = None, schema: Any = None):
        self._cols: dict[str, Series] = {}
        if data is None:
            data = {}
        if isinstance(data, dict):
            for name, v in data.items():
                dt = None
                if isinstance(schema, dict) and name in schema:
                    dt = schema[name]
                s = v.alias(name) if isinstance(v, Series) else Series(name, v, dt)
                self._cols[name] = s
        elif isinstance(data, (list, tuple)) and builtins.all(isinstance(s, Series) for s in data):
            for s in data:
                self._cols[s.name] = s
        else:
            raise N.InvalidOperationError("DataFrame expects a dict of columns or a list of Series")
        h = {s.len() for s in self._cols.values()}
        if builtins.len(h) > 1:
            raise N.ShapeError("could not create a new DataFrame: lengths don't match")

    @property
    def columns(self) -> list[str]:
        return list(self._cols)

    @property
    def height(self) -> int:
        return next(iter(self._cols.values())).len() if self._cols else 0

    @property
    def width(self) -> int:
        return builtins.len(self._cols)

    @property
    def schema(self) -> dict[str, DataType]:
        return {k: s.dtype for k, s in self._cols.items()}

    @property
    def shape(self) -> tuple[int, int]:
        return (self.height, self.width)

    def __getitem__(self, name: str) -> Series:
        return self._cols[name]

    def get_column(self, name: str) -> Series:
        return self._cols[name]

    def is_empty(self) -> bool:
        return self.height == 0

    def to_dict(self, as_series: bool = True) -> dict:
        if as_series:
            return dict(self._cols)
        return {k: s.to_list() for k, s in self._cols.items()}

    def rows(self) -> list[tuple]:
        cols = [s.to_list() for s in self._cols.values()]
        return list(zip(*cols)) if cols else []

    @classmethod
    def from_arrow(cls, table) -> "DataFrame":
        return cls([Series.from_arrow(nm, table.column(nm)) for nm in table.column_names])

    @classmethod
    def from_batches(cls, batches: Sequence[Any], columns: Sequence[str] | None = None) -> "DataFrame":
        """Device frame from a list of Arrow RecordBatches, the form in which
        the reference exports a DataFrame (PyDataFrame.to_arrow,
        crates/polars-python/src/dataframe/export.rs:80): each column is
        ingested chunk by chunk, without concatenating on the host."""
        batches = list(batches)
        if not batches:
            raise N.InvalidOperationError("from_batches needs at least one RecordBatch (schema unknown)")
        names = list(columns) if columns is not None else list(batches[0].schema.names)
        out = []
        for nm in names:
            i = batches[0].schema.get_field_index(nm)
            if i < 0:
                raise N.ComputeError(f"column {nm!r} not found in the scanned batches")
            out.append(_ingest_chunks(nm, [b.column(i) for b in batches], batches[0].schema.field(i).type))
        return cls(out)

    def to_arrow(self):
        """The frame as an Arrow table.  The buffers of its fixed-width
        columns come back in one device -> host round trip
        (plgpu_memcpy_d2h_many); String / Categorical columns take their
        own path."""
        import pyarrow as pa

        plain = [nm for nm, s in self._cols.items()
                 if s._cat_codes() is None and s.dtype not in (String, Boolean) and s.len() > 0]
        ranges = []
        for nm in plain:
            s = self._cols[nm]
            n, off = s.len(), int(s._col.offset)
            eb = np.dtype(s.dtype.np_dtype).itemsize
            ranges.append((s._col.values + off * eb, n * eb))
            ranges.append((s._col.validity, (off + n + 7) // 8) if s._col.validity else (0, 0))
        host = N.download_many(ranges)
        got = {}
        for i, nm in enumerate(plain):
            s = self._cols[nm]
            n, off = s.len(), int(s._col.offset)
            vals = host[2 * i].view(s.dtype.np_dtype)
            valid = _unpack_bits(host[2 * i + 1], off, n) if s._col.validity else None
            phys = _BY_CODE[s._col.dtype]
            arr = pa.array(vals, type=_ARROW_OF[phys.name],
                           mask=None if valid is None or valid.all() else ~valid)
            lg = s._logical_dtype()
            got[nm] = arr.view(_arrow_logical(lg)) if lg is not None else arr
        return pa.table({nm: got[nm] if nm in got else s.to_arrow() for nm, s in self._cols.items()})

    def lazy(self) -> "LazyFrame":
        return LazyFrame(("scan", self))

    def filter(self, *predicates: Expr, **constraints: Any) -> "DataFrame":
        return self.lazy().filter(*predicates, **constraints).collect()

    def sort(self, by: Any, *more_by: Any, descending: bool | Sequence[bool] = False,
             nulls_last: bool | Sequence[bool] = False, multithreaded: bool = True,
             maintain_order: bool = False) -> "DataFrame":
        """DataFrame.sort by 1..8 columns (always stable, so maintain_order holds)."""
        return self.lazy().sort(by, *more_by, descending=descending, nulls_last=nulls_last,
                                maintain_order=maintain_order).collect()

    def join(self, other: "DataFrame", on: str | None = None, how: str = "inner", *,
             left_on: str | None = None, right_on: str | None = None, suffix: str = "_right",
             validate: str = "m:m", nulls_equal: bool = False, coalesce: bool | None = None,
             maintain_order: str | None = None) -> "DataFrame":
        """Eager join (py-polars DataFrame.join): runs the lazy plan."""
        return self.lazy().join(other.lazy(), on, how, left_on=left_on, right_on=right_on, suffix=suffix,
                                validate=validate, nulls_equal=nulls_equal, coalesce=coalesce,
                                maintain_order=maintain_order).collect()

    def group_by(self, *by: Any, maintain_order: bool = False) -> "GroupBy":
        return GroupBy(self.lazy(), by, maintain_order)

    def select(self, *exprs: Any) -> "DataFrame":
        return self.lazy().select(*exprs).collect()

    def with_columns(self, *exprs: Any) -> "DataFrame":
        return self.lazy().with_columns(*exprs).collect()

    def __repr__(self) -> str:
        return f"DataFrame(shape={self.shape}, schema={self.schema})"


# --------------------------------------------------------------- LazyFrame
def _parse_exprs(items: Sequence[Any]) -> list[Expr]:
    out: list[Expr] = []
    for it in items:
        if isinstance(it, (list, tuple)):
            out.extend(_parse_exprs(it))
        elif isinstance(it, str):
            out.append(col(it))
        elif isinstance(it, Expr):
            out.append(it)
        else:
            raise N.InvalidOperationError(f"cannot interpret {it!r} as an expression")
    return out


def _combine_predicates(preds: Sequence[Expr], constraints: dict) -> Expr:
    ps = list(_parse_exprs(preds)) + [col(k) == v for k, v in constraints.items()]
    if not ps:
        raise N.InvalidOperationError("filter needs at least one predicate")
    p = ps[0]
    for q in ps[1:]:
        p = p & q
    return p


class LazyFrame:
    """A logical plan: ('scan', df) | ('filter', input, pred) | ('group_by', input,
    keys, aggs, maintain_order) | ('select' / 'with_columns', input, exprs)."""

    def __init__(self, node: tuple):
        self._node = node

    def filter(self, *predicates: Expr, **constraints: Any) -> "LazyFrame":
        return LazyFrame(("filter", self._node, _combine_predicates(predicates, constraints)))

    def group_by(self, *by: Any, maintain_order: bool = False) -> "LazyGroupBy":
        return LazyGroupBy(self, by, maintain_order)

    def sort(self, by: Any, *more_by: Any, descending: bool | Sequence[bool] = False,
             nulls_last: bool | Sequence[bool] = False, multithreaded: bool = True,
             maintain_order: bool = False) -> "LazyFrame":
        """Sort by 1..8 plain columns (py-polars LazyFrame.sort); per-column
        `descending` / `nulls_last` as bools or sequences of bools."""
        keys = _parse_exprs([by, *more_by])
        if not keys or any(k.kind != "col" for k in keys) or builtins.len(keys) > N.MAX_KEYS:
            raise N.InvalidOperationError("the GPU executor sorts by 1..8 plain columns")
        names = [k.value for k in keys]

        def per_col(v, what):
            vals = [bool(v)] * builtins.len(names) if isinstance(v, bool) else [bool(x) for x in v]
            if builtins.len(vals) != builtins.len(names):
                raise ValueError(f"the length of `{what}` ({builtins.len(vals)}) does not match the length of "
                                 f"`by` ({builtins.len(names)})")
            return vals

        desc, nl = per_col(descending, "descending"), per_col(nulls_last, "nulls_last")
        if builtins.len(names) == 1:
            return LazyFrame(("sort", self._node, names[0], desc[0], nl[0]))
        return LazyFrame(("sort", self._node, tuple(names), tuple(desc), tuple(nl)))

    def join(self, other: "LazyFrame", on: str | None = None, how: str = "inner", *,
             left_on: str | None = None, right_on: str | None = None, suffix: str = "_right",
             validate: str = "m:m", nulls_equal: bool = False, coalesce: bool | None = None,
             maintain_order: str | None = None) -> "LazyFrame":
        """Equi-join on 1..8 key columns (py-polars LazyFrame.join;
        polars-ops/src/frame/join/args.rs:25 JoinArgs): how = inner / left /
        right / full / semi / anti; `coalesce=None` is the join-specific
        default (JoinCoalesce::JoinSpecific: every type but full coalesces
        its key columns)."""
        if on is not None:
            if left_on is not None or right_on is not None:
                raise ValueError("cannot use 'on' together with 'left_on' / 'right_on'")
            left_on = right_on = on
        if left_on is None or right_on is None:
            raise ValueError("must specify `on` OR `left_on` and `right_on`")
        left_on, right_on = _join_keys(left_on), _join_keys(right_on)
        nl = 1 if isinstance(left_on, str) else builtins.len(left_on)
        nr = 1 if isinstance(right_on, str) else builtins.len(right_on)
        if nl != nr:
            raise N.InvalidOperationError("the number of columns given as join key (left: %d, right: %d) "
                                          "should be equal" % (nl, nr))
        if how not in N.JOIN_HOW:
            raise N.InvalidOperationError(f"join how={how!r} is not supported on the GPU executor")
        if validate not in N.JOIN_VALIDATE:
            raise ValueError(f"invalid `validate` argument {validate!r}")
        if maintain_order not in N.JOIN_ORDER:
            raise ValueError(f"invalid `maintain_order` argument {maintain_order!r}")
        return LazyFrame(("join", self._node, other._node, left_on, right_on, suffix, validate, bool(nulls_equal),
                          maintain_order, how, coalesce))

    def select(self, *exprs: Any) -> "LazyFrame":
        return LazyFrame(("select", self._node, _parse_exprs(exprs)))

    def with_columns(self, *exprs: Any) -> "LazyFrame":
        return LazyFrame(("with_columns", self._node, _parse_exprs(exprs)))

    def collect(self, engine: str = "gpu", info: dict | None = None) -> DataFrame:
        """Execute on the GPU.  `engine` is accepted for API parity with
        polars' `collect(engine=...)`; every node runs on the HIP executor."""
        return _execute(self._node, info)

    def explain(self) -> str:
        return _explain(self._node)


def _join_keys(on: Any) -> str | tuple:
    """Join key spec -> one name, or a tuple of 2..8 plain column names."""
    keys = _parse_exprs([on])
    if not keys or any(k.kind != "col" for k in keys):
        raise N.InvalidOperationError("the GPU executor joins on plain key columns")
    if builtins.len(keys) > N.MAX_KEYS:
        raise N.InvalidOperationError("the GPU executor joins on at most 8 key columns")
    names = [k.value for k in keys]
    return names[0] if builtins.len(names) == 1 else tuple(names)


class LazyGroupBy:
    def __init__(self, lf: LazyFrame, by: Sequence[Any], maintain_order: bool):
        keys = _parse_exprs(by)
        if not keys or any(k.kind != "col" for k in keys) or builtins.len(keys) > N.MAX_KEYS:
            raise N.InvalidOperationError("the GPU executor groups by 1..8 plain key columns")
        names = [k.value for k in keys]
        if builtins.len(set(names)) != builtins.len(names):
            raise N.DuplicateError("group-by keys must be distinct columns")
        # one key: its name; several: a tuple of names (plan node field 2)
        self._lf, self._maintain = lf, maintain_order
        self._key = names[0] if builtins.len(names) == 1 else tuple(names)

    def agg(self, *aggs: Any, **named: Any) -> LazyFrame:
        exprs = _parse_exprs(aggs) + [e.alias(k) for k, e in named.items()]
        return LazyFrame(("group_by", self._lf._node, self._key, exprs, self._maintain))

    def len(self, name: str = "len") -> LazyFrame:
        from .expr import len as len_expr
        return self.agg(len_expr().alias(name))


class GroupBy:
    """Eager DataFrame.group_by: runs the lazy plan (as py-polars does)."""

    def __init__(self, lf: LazyFrame, by: Sequence[Any], maintain_order: bool):
        self._g = LazyGroupBy(lf, by, maintain_order)

    def agg(self, *aggs: Any, **named: Any) -> DataFrame:
        return self._g.agg(*aggs, **named).collect()

    def len(self, name: str = "len") -> DataFrame:
        return self._g.len(name).collect()


# ----------------------------------------------------------------- planner
def _explain(node: tuple, depth: int = 0) -> str:
    pad = "  " * depth
    kind = node[0]
    if kind == "scan":
        return f"{pad}DF {node[1].columns}"
    if kind == "filter":
        return f"{pad}FILTER {node[2]!r}\n" + _explain(node[1], depth + 1)
    if kind == "group_by":
        return f"{pad}AGGREGATE {node[3]!r} BY {node[2]}\n" + _explain(node[1], depth + 1)
    if kind == "join":
        return (f"{pad}INNER JOIN ON {node[3]} = {node[4]}\n" + _explain(node[1], depth + 1) + "\n"
                + _explain(node[2], depth + 1))
    return f"{pad}{kind.upper()} {node[2]!r}\n" + _explain(node[1], depth + 1)


_CMP_OPS = {"==": "EQ", "!=": "NE", "<": "LT", "<=": "LE", ">": "GT", ">=": "GE",
            "eq_missing": "EQ_MISSING", "ne_missing": "NE_MISSING"}
_CMP_MIRROR = {"<": ">", "<=": ">=", ">": "<", ">=": "<="}


def _lower_strings(expr: Expr, df: DataFrame) -> tuple[Expr, DataFrame]:
    """Replace every comparison that involves a String column (with a string
    literal or another String column) and every is_null / is_not_null of a
    String column by a Boolean column computed on the GPU
    (plgpu_str_compare; polars-compute/src/comparisons/view.rs), so the rest
    of the expression lowers to the numeric program as usual.  Returns the
    rewritten expression and the frame extended by those columns."""
    extra: list[Series] = []

    def is_str(e: Expr) -> bool:
        return (e.kind == "col" and e.value in df._cols and df._cols[e.value].dtype is String) or \
            (e.kind == "lit" and isinstance(e.value, str))

    def new_col(c_: N.Column) -> Expr:
        name = f"__strcmp{builtins.len(extra)}"
        extra.append(Series._from_native(name, c_))
        return col(name)

    def walk(e: Expr) -> Expr:
        if e.kind == "bin" and e.op in _CMP_OPS and (is_str(e.args[0]) or is_str(e.args[1])):
            a, b = e.args
            op = e.op
            if a.kind == "lit":  # literal on the left: mirror the comparison
                a, b = b, a
                op = _CMP_MIRROR.get(op, op)
            if not (is_str(a) and is_str(b)) or a.kind != "col":
                raise N.InvalidOperationError(f"comparison {e!r} of a String with a non-string operand")
            out = N.Column()
            ac = df._cols[a.value]._col
            if b.kind == "col":
                N.check(N.lib().plgpu_str_compare(C.byref(ac), C.byref(df._cols[b.value]._col), None, 0,
                                                  N.OP[_CMP_OPS[op]], C.byref(out), None))
            else:
                lit_b = b.value.encode()
                N.check(N.lib().plgpu_str_compare(C.byref(ac), None, lit_b, builtins.len(lit_b),
                                                  N.OP[_CMP_OPS[op]], C.byref(out), None))
            return new_col(out)
        if e.kind == "strfn":
            if e.args[0].kind != "col" or not is_str(e.args[0]):
                raise N.InvalidOperationError(f"{e!r}: str functions take a String column")
            out = N.Column()
            pat = e.value.encode()
            N.check(N.lib().plgpu_str_compare(C.byref(df._cols[e.args[0].value]._col), None, pat, builtins.len(pat),
                                              N.OP["STR_" + e.op.upper()], C.byref(out), None))
            return new_col(out)
        if e.kind == "un" and e.op in ("is_null", "is_not_null") and is_str(e.args[0]) and e.args[0].kind == "col":
            out = N.Column()
            N.check(N.lib().plgpu_str_compare(C.byref(df._cols[e.args[0].value]._col), None, None, 0,
                                              N.OP["IS_NULL" if e.op == "is_null" else "IS_NOT_NULL"],
                                              C.byref(out), None))
            return new_col(out)
        if not e.args:
            return e
        args = tuple(walk(a) for a in e.args)
        if all(x is y for x, y in zip(args, e.args)):
            return e
        return Expr(e.kind, args, op=e.op, value=e.value, name=e._name)

    new = walk(expr)
    if not extra:
        return expr, df
    return new, DataFrame(list(df._cols.values()) + extra)


# ------------------------------------------------ typing before lowering
_EPOCH_DT = None


def _temporal_literal(v: Any, dt: DataType) -> int:
    """A Python datetime / date / timedelta literal as the physical integer of
    the temporal dtype `dt` it is compared with or added to."""
    import datetime as _dt

    per = {"ns": 1_000_000_000, "us": 1_000_000, "ms": 1_000}
    if isinstance(v, np.datetime64) or isinstance(v, np.timedelta64):
        unit = getattr(dt, "time_unit", "us")
        return int(v.astype(f"{'M8' if isinstance(v, np.datetime64) else 'm8'}[{unit}]").view(np.int64))
    if isinstance(v, _dt.datetime):
        if not isinstance(dt, Datetime):
            raise N.InvalidOperationError(f"cannot compare a datetime literal with {dt}")
        if (v.tzinfo is None) != (dt.time_zone is None):
            raise N.InvalidOperationError("datetime literal and column differ in time-zone awareness")
        epoch = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc if v.tzinfo else None)
        d = v - epoch
        return (d.days * 86400 + d.seconds) * per[dt.time_unit] + d.microseconds * per[dt.time_unit] // 1_000_000
    if isinstance(v, _dt.date):
        if dt is not Date:
            raise N.InvalidOperationError(f"cannot compare a date literal with {dt}")
        return (v - _dt.date(1970, 1, 1)).days
    if isinstance(v, _dt.timedelta):
        if not isinstance(dt, Duration):
            raise N.InvalidOperationError(f"cannot combine a timedelta literal with {dt}")
        return (v.days * 86400 + v.seconds) * per[dt.time_unit] + v.microseconds * per[dt.time_unit] // 1_000_000
    raise N.InvalidOperationError(f"literal {v!r} is not a temporal value")


def _is_temporal_lit(e: Expr) -> bool:
    import datetime as _dt

    return e.kind == "lit" and isinstance(e.value, (_dt.date, _dt.timedelta, np.datetime64, np.timedelta64))


_CMP = ("==", "!=", "<", "<=", ">", ">=", "eq_missing", "ne_missing")


def _can_fail(src: DataType, dst: DataType) -> bool:
    """Whether a strict cast src -> dst can meet a value that does not fit
    (only those fail in polars: int -> float and float -> float round)."""
    s, d = src.physical(), dst.physical()
    if s is d or d is Boolean or d in FLOAT_DTYPES or s is Boolean:
        return False
    if s in FLOAT_DTYPES:
        return True
    bits = {Int8: 8, Int16: 16, Int32: 32, Int64: 64, UInt8: 8, UInt16: 16, UInt32: 32, UInt64: 64}
    su, du = s.name.startswith("U"), d.name.startswith("U")
    if su == du:
        return bits[d] < bits[s]
    if su and not du:  # unsigned -> signed: needs one more bit
        return bits[d] <= bits[s]
    return True  # signed -> unsigned: negatives


def _prepare(expr: Expr, df: DataFrame) -> tuple[Expr, DataType | None, list]:
    """Resolve what the device program cannot see: temporal logical types
    (literals become physical integers in the column's unit, results get
    their logical dtype: Datetime - Datetime = Duration, Datetime +-
    Duration = Datetime, Duration +- Duration = Duration; polars-core/src/
    series/arithmetic), and strict casts that can fail (collected, checked
    by _check_strict).  Returns (expr, logical dtype of the result, strict
    casts)."""
    strict: list = []

    def dtype_of(e: Expr) -> DataType | None:
        return df._cols[e.value].dtype if e.kind == "col" and e.value in df._cols else None

    def go(e: Expr) -> tuple[Expr, DataType | None]:
        k = e.kind
        if k == "col":
            d = dtype_of(e)
            return e, d if d is not None and d.logical else None
        if k == "lit":
            if _is_temporal_lit(e):
                return e, "lit"
            return e, None
        if k == "alias":
            a, la = go(e.args[0])
            return Expr("alias", (a,), value=e.value), la
        if k == "bin":
            (a, la), (b, lb) = go(e.args[0]), go(e.args[1])
            if la is None and lb is None:
                return Expr("bin", (a, b), op=e.op), None
            # settle temporal literals against the other side's logical dtype
            if la == "lit":
                if lb in (None, "lit"):
                    raise N.InvalidOperationError(f"temporal literal in {e!r} has no temporal operand")
                a, la = Expr("lit", value=_temporal_literal(a.value, lb)), lb
            if lb == "lit":
                lit_dt = la
                if e.op in ("+", "-") and isinstance(la, Datetime):
                    lit_dt = Duration(la.time_unit)
                b, lb = Expr("lit", value=_temporal_literal(b.value, lit_dt)), lit_dt
            out = Expr("bin", (a, b), op=e.op)
            if e.op in _CMP:
                if la is not None and lb is not None and la != lb:
                    raise N.InvalidOperationError(f"cannot compare {la} with {lb}")
                return out, None
            dur = lambda t: isinstance(t, Duration)  # noqa: E731
            dtm = lambda t: isinstance(t, Datetime)  # noqa: E731
            if e.op == "-" and dtm(la) and dtm(lb) and la == lb:
                return out, Duration(la.time_unit)
            if e.op in ("+", "-") and dtm(la) and dur(lb) and la.time_unit == lb.time_unit:
                return out, la
            if e.op == "+" and dur(la) and dtm(lb) and la.time_unit == lb.time_unit:
                return out, lb
            if e.op in ("+", "-") and dur(la) and dur(lb) and la == lb:
                return out, la
            raise N.InvalidOperationError(f"operation {e.op!r} on {la} and {lb} is not supported on the GPU executor")
        if k == "un":
            a, la = go(e.args[0])
            if la is not None and e.op not in ("is_null", "is_not_null") and not (
                    isinstance(la, Duration) and e.op in ("neg", "abs")):
                raise N.InvalidOperationError(f"{e.op} of {la} is not supported on the GPU executor")
            return Expr("un", (a,), op=e.op), (la if e.op in ("neg", "abs") else None)
        if k == "cast":
            a, la = go(e.args[0])
            src = la if la is not None else _static_dtype(a, df)
            dst = e.value
            if src is not None and e.op == "strict" and _can_fail(src, dst):
                strict.append((a, dst))
            return Expr("cast", (a,), op=e.op, value=dst.physical()), (dst if dst.logical else None)
        if k in ("fill_null", "ternary"):
            parts = [go(x) for x in e.args]
            vals = parts[1:] if k == "ternary" else parts
            lgs = [lg for _, lg in vals]
            base = next((lg for lg in lgs if lg not in (None, "lit")), None)
            args = []
            for (x, lg) in parts:
                if lg == "lit":
                    if base is None:
                        raise N.InvalidOperationError(f"temporal literal in {e!r} has no temporal operand")
                    x = Expr("lit", value=_temporal_literal(x.value, base))
                args.append(x)
            if base is not None and any(lg not in (base, "lit") and not (x.kind == "lit" and x.value is None)
                                        for (x, lg) in vals):
                raise N.InvalidOperationError(f"{e!r} mixes {base} with another dtype")
            return Expr(k, tuple(args), op=e.op, value=e.value), base
        return e, None

    out, lg = go(expr)
    if lg == "lit":
        raise N.InvalidOperationError("a temporal literal alone is not supported on the GPU executor")
    return out, lg, strict


def _static_dtype(e: Expr, df: DataFrame) -> DataType | None:
    """Dtype of a plain column expression (strict-cast checks)."""
    if e.kind == "col" and e.value in df._cols:
        return df._cols[e.value].dtype
    if e.kind == "alias":
        return _static_dtype(e.args[0], df)
    return None


def _check_strict(strict: list, df: DataFrame) -> None:
    """A strict cast that met a value that does not fit raises, as polars'
    strict cast does (InvalidOperationError 'conversion ... failed')."""
    for inner, dst in strict:
        probe = inner.is_not_null() & Expr("cast", (inner,), op="non-strict", value=dst.physical()).is_null()
        used, prog, n = _program(probe, df)
        out = (N.Column * builtins.len(used))()
        cnt = C.c_int64(0)
        N.check(N.lib().plgpu_filter_expr(_col_array(used), builtins.len(used), prog, n, out, C.byref(cnt), None))
        for i in range(builtins.len(used)):
            N.lib().plgpu_column_release(C.byref(out[i]))
        if cnt.value:
            raise N.InvalidOperationError(
                f"conversion from `{_static_dtype(inner, df) or '?'}` to `{dst}` failed for {cnt.value} value(s); "
                "set `strict=False` to allow null")


def _program(expr: Expr, df: DataFrame) -> tuple[list[Series], Any, int]:
    names = expr.meta_root_names()
    if builtins.len(names) > N.MAX_COLS:
        raise N.InvalidOperationError("expression references more than 8 columns")
    for nm in names:
        if nm not in df._cols:
            raise N.ComputeError(f'unable to find column "{nm}"; valid columns: {df.columns}')
    idx = {nm: i for i, nm in enumerate(names)}
    schema = {nm: df._cols[nm].dtype.code for nm in names}
    prog = lower(expr, idx, schema)
    return [df._cols[nm] for nm in names], to_instr_array(prog), builtins.len(prog)


def _col_array(series: Sequence[Series]):
    arr = (N.Column * max(1, builtins.len(series)))()
    for i, s in enumerate(series):
        arr[i] = s._col
    return arr


def _eval(expr: Expr, df: DataFrame) -> Series:
    if expr.kind in ("col",) or (expr.kind == "alias" and expr.args[0].kind == "col"):
        return df._cols[expr.meta_root_names()[0]].alias(expr.output_name())
    base = expr.args[0] if expr.kind == "alias" else expr
    if base.kind in ("rolling", "sort"):
        inner = _eval(base.args[0], df)
        if base.kind == "rolling":
            w, ms, center, ddof = base.value
            res = inner._rolling(N.ROLLING[base.op], w, ms, center, ddof)
        elif base.op == "arg_sort":
            res = inner.arg_sort(descending=base.value[0], nulls_last=base.value[1])
        else:
            res = inner.sort(descending=base.value[0], nulls_last=base.value[1])
        return res.alias(expr.output_name())
    expr, df = _lower_strings(expr, df)
    name = expr.output_name()
    expr, logical, strict = _prepare(expr, df)
    _check_strict(strict, df)
    used, prog, n = _program(expr, df)
    if not used:
        raise N.InvalidOperationError("literal-only expressions are not supported on the GPU executor")
    out = N.Column()
    N.check(N.lib().plgpu_eval(_col_array(used), builtins.len(used), prog, n, C.byref(out), None))
    return Series._from_native(name, out, logical)


def _filter(df: DataFrame, pred: Expr) -> DataFrame:
    names = df.columns
    pred, df = _lower_strings(pred, df)
    pred, _, strict = _prepare(pred, df)
    _check_strict(strict, df)
    if not pred.meta_root_names():
        # Constant predicate (plan-time simplification, as polars'
        # simplify_expression does): keep every row or none.
        keep = _const_bool(pred)
        return DataFrame([s if keep else s.slice(0, 0) for s in df._cols.values()])
    used, prog, n = _program(pred, df)
    # The fused path evaluates the predicate inside the compaction kernels; the
    # predicate's columns must be in the same call, so compact in chunks of up
    # to 8 columns that always carry the predicate columns first.
    pred_names = [s.name for s in used]
    others = [nm for nm in names if nm not in pred_names]
    room = N.MAX_COLS - builtins.len(pred_names)
    chunks = [others[i: i + room] for i in range(0, builtins.len(others), room)] or [[]]
    result: dict[str, Series] = {}
    for chunk in chunks:
        series = used + [df._cols[nm] for nm in chunk]
        out = (N.Column * builtins.len(series))()
        cnt = C.c_int64(0)
        N.check(N.lib().plgpu_filter_expr(_col_array(series), builtins.len(series), prog, n, out,
                                          C.byref(cnt), None))
        for i, s in enumerate(series):
            result.setdefault(s.name, Series._from_native(s.name, out[i], s._logical_dtype()))
    return DataFrame([result[nm] for nm in names])


_AGG_CODE = N.AGG


def _const_bool(e: Expr):
    """Kleene evaluation of a column-free boolean predicate (null -> drop)."""
    def ev(x: Expr):
        if x.kind == "alias":
            return ev(x.args[0])
        if x.kind == "lit":
            if x.value is None or isinstance(x.value, bool):
                return x.value
            raise N.ComputeError("filter predicate must be of type `Boolean`")
        if x.kind == "un" and x.op == "not":
            v = ev(x.args[0])
            return None if v is None else not v
        if x.kind == "bin" and x.op in ("&", "|"):
            a, b = ev(x.args[0]), ev(x.args[1])
            if x.op == "&":
                return False if (a is False or b is False) else (None if (a is None or b is None) else True)
            return True if (a is True or b is True) else (None if (a is None or b is None) else False)
        raise N.InvalidOperationError(f"unsupported constant predicate {x!r}")
    return ev(e) is True


class _GbCall:
    """Lowered arguments of one group-by call through the C-ABI (shared by
    the single-GPU path and polaroid_amd.distributed)."""

    __slots__ = ("key", "keys", "keycol", "keycols", "names", "cols", "ncols", "prog", "n_instr", "aggs", "naggs",
                 "inputs", "ninputs", "out_names", "key_logical", "out_logical", "_keep")


def _gb_keys(key: str | tuple | None) -> list[str]:
    if key is None:
        return []
    return [key] if isinstance(key, str) else list(key)


_BOOL_AGG_CAST = {"sum": "UInt32", "mean": "Float64"}  # reduce/sum.rs: Boolean sums count (IdxSize)


def _gb_lower(df: DataFrame, key: str | tuple | None, aggs: list[Expr], pred: Expr | None) -> _GbCall:
    """The group-by's C-ABI arguments.  An aggregation over a plain column
    reads the column; over any other elementwise expression (`(close *
    volume).sum()`, polars' can_pre_agg inputs, plans/aexpr/properties/
    general.rs:335) it reads a computed input (plgpu_agg_input), which the
    fused kernel evaluates in registers when it is `x op y` of Float64 columns
    / literals.  `key` None: a global reduction (select(aggs))."""
    keys = _gb_keys(key)
    for k in keys:
        if k not in df._cols:
            raise N.ComputeError(f'unable to find column "{k}"')
    # len() needs some aggregatable column for its accumulator slot (it only
    # reads the group's row count): a column another aggregation already reads
    # (one accumulator, no extra column pass), else an 8-byte key column (the
    # fused kernel's loads), else the first non-Boolean key, else any column
    plain = [b.args[0].value for b in (e.args[0] if e.kind == "alias" else e for e in aggs)
             if b.kind == "agg" and b.args and b.args[0].kind == "col" and b.args[0].value in df._cols
             and df._cols[b.args[0].value].dtype not in (Boolean, String)]
    len_col = plain[0] if plain else next((k for k in keys if df._cols[k].dtype in (Int64, UInt64, Float64)), None)
    if len_col is None:
        len_col = next((k for k in keys if df._cols[k].dtype not in (Boolean, String)), None)
    if len_col is None:
        len_col = next((c for c in df.columns if df._cols[c].dtype not in (Boolean, String)), None)
    if len_col is None:
        # no numeric column at all: a zero column of the frame's height
        len_col = "__len"
        df = DataFrame(list(df._cols.values()) + [Series.from_numpy("__len", np.zeros(df.height, np.int64))])
    specs: list[tuple[str, Any]] = []  # (kind, column name | ("input", j))
    exprs: list[Expr] = []             # computed inputs
    out_names: list[str] = []
    out_logical: list = []
    for e in aggs:
        name = e.output_name()
        base = e.args[0] if e.kind == "alias" else e
        if base.kind == "len":
            specs.append(("len", len_col))
            out_logical.append(None)
        elif (base.kind == "agg" and base.op in ("var", "std") and base.args[0].kind == "col"
              and base.args[0].value in df._cols and df._cols[base.args[0].value].dtype is Float64):
            # one fused pass (plgpu_group_by_agg_ex: exact sums of x and of
            # x * x's two parts, ddof in bits 8..15 of the kind)
            specs.append(((base.op, int(base.value)), base.args[0].value))
            out_logical.append(None)
        elif (base.kind == "agg" and base.args[0].kind == "col" and base.args[0].value in df._cols
              and df._cols[base.args[0].value].dtype is not Boolean):
            c_ = base.args[0].value
            specs.append((base.op, c_))
            lg = df._cols[c_]._logical_dtype()
            if lg is not None and base.op not in ("min", "max", "first", "last", "count", "len") and not (
                    base.op == "sum" and isinstance(lg, Duration)):
                raise N.InvalidOperationError(f"`{base.op}` of a {lg} column is not supported on the GPU executor")
            out_logical.append(lg if base.op in ("min", "max", "first", "last", "sum") else None)
        elif base.kind == "agg" and base.op in ("sum", "mean", "min", "max", "count", "len", "first", "last"):
            x, df = _lower_strings(base.args[0], df)
            x, lg, strict = _prepare(x, df)
            _check_strict(strict, df)
            if not x.meta_root_names():
                raise N.InvalidOperationError(f"aggregation {e!r} of a literal is not supported on the GPU executor")
            if lg is not None and base.op not in ("min", "max", "first", "last", "count", "len") and not (
                    base.op == "sum" and isinstance(lg, Duration)):
                raise N.InvalidOperationError(f"`{base.op}` of a {lg} expression is not supported on the GPU executor")
            exprs.append(x)
            specs.append((base.op, ("input", builtins.len(exprs) - 1)))
            out_logical.append(lg if base.op in ("min", "max", "first", "last", "sum") else None)
        else:
            raise N.InvalidOperationError(
                f"aggregation {e!r} is not supported on the GPU executor "
                "(need <expr>.sum/mean/min/max/count/len/first/last)")
        out_names.append(name)
    # columns passed to the kernel: predicate columns, aggregated columns,
    # then the columns the computed inputs read
    names: list[str] = []
    g = _GbCall()
    g.prog, g.n_instr = None, 0
    if pred is not None:
        names = pred.meta_root_names()
    for _, c_ in specs:
        if isinstance(c_, str) and c_ not in names:
            names.append(c_)
    for x in exprs:
        for c_ in x.meta_root_names():
            if c_ not in names:
                names.append(c_)
    if builtins.len(names) > N.MAX_COLS:
        raise N.InvalidOperationError("group-by references more than 8 columns")
    for nm in names:
        if nm not in df._cols:
            raise N.ComputeError(f'unable to find column "{nm}"')
    idx = {nm: i for i, nm in enumerate(names)}
    schema = {nm: df._cols[nm].dtype.code for nm in names}
    if pred is not None:
        p = lower(pred, idx, schema)
        g.prog, g.n_instr = to_instr_array(p), builtins.len(p)
    ncols = builtins.len(names)
    cols = _col_array([df._cols[nm] for nm in names])
    inputs = (N.AggInput * max(1, builtins.len(exprs)))()
    keep_progs = []
    for j, x in enumerate(exprs):
        prog = to_instr_array(lower(x, idx, schema))
        dt = C.c_int32(0)
        N.check(N.lib().plgpu_expr_dtype(cols, ncols, prog, builtins.len(prog), C.byref(dt)))
        if dt.value == N.BOOL:
            # Boolean inputs: sums count (IdxSize), means average 0 / 1
            kinds = {k for k, c_ in specs if c_ == ("input", j)}
            if kinds - set(_BOOL_AGG_CAST) - {"count", "len"}:
                raise N.InvalidOperationError("min / max / first / last of a Boolean expression are not supported "
                                              "on the GPU executor")
            if builtins.len({_BOOL_AGG_CAST[k] for k in kinds if k in _BOOL_AGG_CAST}) > 1:
                raise N.InvalidOperationError("sum and mean of one Boolean expression in one group-by")
            to = next((_BOOL_AGG_CAST[k] for k in kinds if k in _BOOL_AGG_CAST), "UInt32")
            prog = to_instr_array(lower(x.cast(UInt32 if to == "UInt32" else Float64), idx, schema))
        keep_progs.append(prog)
        inputs[j].program = C.cast(prog, C.POINTER(N.Instr))
        inputs[j].n_instr = builtins.len(prog)
    agg_arr = (N.Agg * max(1, builtins.len(specs)))()
    for i, (k, c_) in enumerate(specs):
        agg_arr[i].kind = _AGG_CODE[k[0]] | (k[1] << 8) if isinstance(k, tuple) else _AGG_CODE[k]
        agg_arr[i].col = idx[c_] if isinstance(c_, str) else ncols + c_[1]
    g.key = keys[0] if keys else None
    g.keys = keys
    g.keycol = df._cols[keys[0]]._col if keys else None
    g.keycols = _col_array([df._cols[k] for k in keys])
    g.names = names
    g.cols = cols
    g.ncols = ncols
    g.inputs = inputs
    g.ninputs = builtins.len(exprs)
    g.aggs = agg_arr
    g.naggs = builtins.len(specs)
    g.out_names = out_names
    # logical dtypes of the outputs: keys keep theirs; min / max / first /
    # last / Duration sums keep the input's, counts and lengths have none
    g.key_logical = [df._cols[k]._logical_dtype() for k in keys]
    g.out_logical = out_logical
    g._keep = [df._cols[nm] for nm in names] + [df._cols[k] for k in keys] + keep_progs
    return g


def _gb_frame(g: _GbCall, out_key, out_aggs) -> DataFrame:
    """`out_key`: one Column, or an array of len(g.keys) Columns (none for a
    global reduction)."""
    if isinstance(out_key, N.Column):
        series = [Series._from_native(g.key, out_key, g.key_logical[0])]
    else:
        series = [Series._from_native(k, out_key[i], g.key_logical[i]) for i, k in enumerate(g.keys)]
    for i, nm in enumerate(g.out_names):
        series.append(Series._from_native(nm, out_aggs[i], g.out_logical[i]))
    return DataFrame(series)


def _agg_base(e: Expr) -> Expr:
    return e.args[0] if e.kind == "alias" else e


def _group_by_fused_var(df: DataFrame, key: str | tuple, aggs: list[Expr], maintain_order: bool,
                        pred: Expr | None, info: dict | None) -> DataFrame:
    """var / std of Float64 columns in fused passes.  A var column takes
    three of the kernel's six accumulators (x, and x * x's two parts), so
    more than two var columns, or two next to other aggregated columns, run
    as several passes over the same selected rows with first-occurrence
    group order (identical groups and order in every pass), put side by
    side."""
    vcols = list(dict.fromkeys(_agg_base(e).args[0].value for e in aggs
                               if _agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var")))
    plain = [e for e in aggs if not (_agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var"))]
    pcols = {c for e in plain for c in e.meta_root_names()}
    # len() rides on _gb_lower's len_col: the first aggregation over a plain
    # numeric column (var / std included) when there is one, which already
    # holds an accumulator; otherwise a key column, an accumulator of its own
    has_col = builtins.any(
        b.kind == "agg" and b.args and b.args[0].kind == "col" and b.args[0].value in df._cols
        and df._cols[b.args[0].value].dtype not in (Boolean, String) for b in map(_agg_base, aggs))
    nlen = 1 if not has_col and builtins.any(_agg_base(e).kind == "len" for e in plain) else 0
    if 3 * builtins.len(vcols) + builtins.len(pcols) + nlen <= N.GB_MAX_ACC:
        return _group_by_plain(df, key, aggs, maintain_order, pred, info)
    names = [e.output_name() for e in aggs]
    parts = []
    batches = [vcols[i:i + 2] for i in range(0, builtins.len(vcols), 2)]
    for bi, vb in enumerate(batches):
        sel = [e for e in aggs if _agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var")
               and _agg_base(e).args[0].value in vb]
        parts.append(_group_by_plain(df, key, sel, True, pred, info if bi == 0 else None))
    if plain:
        parts.append(_group_by_plain(df, key, plain, True, pred, None))
    keys = _gb_keys(key)
    cols = {}
    for part in parts:
        for nm in part.columns:
            if nm not in keys:
                cols[nm] = part[nm]
    return DataFrame([parts[0][k] for k in keys] + [cols[nm] for nm in names])


def _group_by_var(df: DataFrame, key: str | tuple, aggs: list[Expr], maintain_order: bool,
                  pred: Expr | None, info: dict | None) -> DataFrame:
    """group_by().agg() with var / std (polars-expr/src/reduce/var_std.rs),
    composed of GPU passes:
      1. the exact group-by with sum(x) and count(x) of every var / std
         column next to the other aggregations (first-occurrence order);
      2. every row's group mean: for one integer key plgpu_group_sq_dev
         looks it up in a table of the group keys and writes d directly;
         otherwise a left join of the rows with the groups' means (null keys
         match: they form a group);
      3. d = (x - mean)^2 per row (one rounding), exactly summed per group
         by a second group-by with the same predicate (same group order);
      4. plgpu_var_finalize: null when count <= ddof, else sum / (count - ddof),
         square root for std.
    The reference's Welford state (moment.rs VarState) rounds differently;
    the results agree to ~1e-13 relative (tests/test_gpu_first_last.py)."""
    keys = list(_gb_keys(key))
    var_cols: list[str] = []
    plain: list[tuple[int, Expr]] = []
    aggs = list(aggs)
    for i, e in enumerate(aggs):
        b = _agg_base(e)
        if b.kind == "agg" and b.op in ("std", "var"):
            if b.args[0].kind != "col":
                # var / std of an expression: the expression evaluated once
                # into a column (plgpu_eval), then as for a column
                nm = f"__vx{i}"
                df = DataFrame(list(df._cols.values()) + [_eval(b.args[0].alias(nm), df)])
                b = Expr("agg", (col(nm),), op=b.op, value=b.value)
                aggs[i] = b.alias(e.output_name())
            if b.args[0].value not in var_cols:
                var_cols.append(b.args[0].value)
        else:
            plain.append((i, e))
    # one pass: exact sums of x and of x * x (split into its rounded product
    # and that product's exact error), combined exactly per group (DESIGN.md
    # "var / std in one pass"); an integer column as its f64 values (the
    # reference casts before its Welford update); inputs whose exact state
    # would leave its range, and Float32 columns, take the passes below
    fdf, faggs, casts = df, list(aggs), {}
    for i, e in enumerate(faggs):
        b = _agg_base(e)
        if b.kind == "agg" and b.op in ("std", "var") and fdf._cols[b.args[0].value].dtype in INTEGER_DTYPES:
            c = b.args[0].value
            if c not in casts:
                casts[c] = f"__vf_{c}"
                fdf = DataFrame(list(fdf._cols.values()) + [_eval(col(c).cast("f64").alias(casts[c]), fdf)])
            faggs[i] = Expr("agg", (col(casts[c]),), op=b.op, value=b.value).alias(e.output_name())
    vbases = [_agg_base(e) for e in faggs if _agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var")]
    if builtins.all(fdf._cols[b.args[0].value].dtype is Float64 and 0 <= int(b.value) <= 255 for b in vbases):
        try:
            out = _group_by_fused_var(fdf, key, faggs, maintain_order, pred, info)
            if info is not None:
                info["var_path"] = "fused"
            return out
        except (N.ComputeError, N.InvalidOperationError):
            pass  # out of the exact range, or too many columns: the passes below
    if info is not None:
        info["var_path"] = "two_pass"
    helpers = []
    for c in var_cols:
        # mean(): f64 from the exact sum of the values widened to f64, so an
        # integer group whose sum overflows the input width does not wrap
        # (the reference casts to f64 before its Welford update, var_std.rs)
        helpers += [col(c).mean().alias(f"__vm_{c}"), col(c).count().alias(f"__vn_{c}")]
    first = _group_by(df, key, [e for _, e in plain] + helpers, True, pred, info)
    means = [first[k] for k in keys] + [first[f"__vm_{c}"] for c in var_cols]
    if not keys:
        # a global var / std: the one mean as a literal (host scalar)
        sq = []
        for c, m in zip(var_cols, means):
            mv = m.to_list()[0]
            mv = float("nan") if mv is None else float(mv)
            sq.append(_eval(((col(c).cast("f64") - lit(mv)) * (col(c).cast("f64") - lit(mv))).alias(f"__vd_{c}"),
                            df))
        rows = DataFrame(list(df._cols.values()) + sq)
    elif builtins.len(keys) == 1 and df[keys[0]]._col.dtype in (N.I64, N.I32, N.U32, N.BOOL):
        # one integer key: squared deviations straight from a group-key table
        sq = []
        for c, m in zip(var_cols, means[1:]):
            o = N.Column()
            N.check(N.lib().plgpu_group_sq_dev(C.byref(df[keys[0]]._col), C.byref(df[c]._col),
                                               C.byref(means[0]._col), C.byref(m._col), C.byref(o), None))
            sq.append(Series._from_native(f"__vd_{c}", o))
        rows = DataFrame(list(df._cols.values()) + sq)
    else:
        rows = _join(df, DataFrame(means), key, key, "_right", "m:m", True, "left", "left")
        sq = [_eval(((col(c).cast("f64") - col(f"__vm_{c}")) * (col(c).cast("f64") - col(f"__vm_{c}")))
                    .alias(f"__vd_{c}"), rows) for c in var_cols]
        rows = DataFrame(list(rows._cols.values()) + sq)
    second = _group_by(rows, key, [col(f"__vd_{c}").sum().alias(f"__vd_{c}") for c in var_cols], True, pred, None)
    out: list[Series] = [first[k] for k in keys]
    res: dict[int, Series] = {}
    for i, e in plain:
        res[i] = first[e.output_name()]
    for i, e in enumerate(aggs):
        b = _agg_base(e)
        if i in res:
            continue
        c = b.args[0].value
        o = N.Column()
        N.check(N.lib().plgpu_var_finalize(C.byref(second[f"__vd_{c}"]._col), C.byref(first[f"__vn_{c}"]._col),
                                           int(b.value), int(b.op == "std"), C.byref(o), None))
        res[i] = Series._from_native(e.output_name(), o)
    return DataFrame(out + [res[i] for i in range(builtins.len(aggs))])


def _group_by(df: DataFrame, key: str | tuple, aggs: list[Expr], maintain_order: bool,
              pred: Expr | None, info: dict | None) -> DataFrame:
    if any(_agg_base(e).kind == "agg" and _agg_base(e).op in ("std", "var") for e in aggs):
        return _group_by_var(df, key, aggs, maintain_order, pred, info)
    return _group_by_plain(df, key, aggs, maintain_order, pred, info)


def _cat_keys(df: DataFrame, key: str | tuple, aggs: list[Expr], pred: Expr | None):
    """Categorical key columns -> their UInt32 codes (polars-core/src/frame/
    group_by/into_groups.rs:132-139 groups a Categorical by its physical
    codes): the frame with those key columns replaced, and their
    dictionaries, which decode the output keys.  A key column an aggregation
    or the predicate also reads keeps its strings."""
    keys = _gb_keys(key)
    used = {c for e in aggs for c in e.meta_root_names()}
    if pred is not None:
        used |= set(pred.meta_root_names())
    dicts: dict = {}
    cols = []
    for nm, s in df._cols.items():
        cc = s._cat_codes() if nm in keys and nm not in used else None
        if cc is not None:
            dicts[nm] = cc[0]
            cols.append(cc[1].alias(nm))
        else:
            cols.append(s)
    return (DataFrame(cols) if dicts else df), dicts


def _group_by_plain(df: DataFrame, key: str | tuple, aggs: list[Expr], maintain_order: bool,
                    pred: Expr | None, info: dict | None) -> DataFrame:
    if pred is not None:
        pred, df = _lower_strings(pred, df)
        pred, _, strict = _prepare(pred, df)
        _check_strict(strict, df)
    df, cat_dicts = _cat_keys(df, key, aggs, pred)
    g = _gb_lower(df, key, aggs, pred)
    out_aggs = (N.Column * max(1, g.naggs))()
    gi = N.GroupByInfo()
    # one integer key: the single-key kernels; several keys (or a Float /
    # Boolean / String key): packed or hashed tuples; none: a global reduction
    out_key = (N.Column * max(1, builtins.len(g.keys)))()
    N.check(N.lib().plgpu_group_by_agg_ex(g.keycols, builtins.len(g.keys), g.cols, g.ncols, g.inputs, g.ninputs,
                                          g.prog, g.n_instr, g.aggs, g.naggs, int(bool(maintain_order)), out_key,
                                          out_aggs, C.byref(gi), None))
    if info is not None:
        info.update(gi.as_dict())
        info["categorical_codes"] = builtins.len(cat_dicts)
    out = _gb_frame(g, out_key, out_aggs)
    if cat_dicts:
        # output keys: the group codes over the column's dictionary
        out = DataFrame([Series._categorical(nm, cat_dicts[nm], s) if nm in cat_dicts else s
                         for nm, s in out._cols.items()])
    return out


def _join(left: DataFrame, right: DataFrame, left_on: str | tuple, right_on: str | tuple, suffix: str,
          validate: str, nulls_equal: bool, maintain_order: str | None, how: str = "inner",
          coalesce: bool | None = None) -> DataFrame:
    """Join two frames on the GPU and materialise the result as the reference
    does: semi / anti keep the left rows (_finish_anti_semi_join); otherwise
    left columns then right columns, a right name that clashes gets `suffix`
    (general.rs:17 _finish_join).  Coalescing drops the right key columns
    (the left ones for a right join, dispatch_left_right.rs:19); a coalesced
    full join keeps coalesce(left key, right key) in the left key's place
    (general.rs:52 _coalesce_full_join)."""
    lkeys, rkeys = _gb_keys(left_on), _gb_keys(right_on)
    for df, ks in ((left, lkeys), (right, rkeys)):
        for k in ks:
            if k not in df._cols:
                raise N.ComputeError(f'unable to find column "{k}"; valid columns: {df.columns}')
    lks, rks = [left._cols[k] for k in lkeys], [right._cols[k] for k in rkeys]
    for lk, rk in zip(lks, rks):
        if lk.dtype != rk.dtype:
            raise N.InvalidOperationError(
                f"join keys must have the same dtype on the GPU executor (got {lk.dtype} and {rk.dtype})")
    li, ri = N.Column(), N.Column()
    order, val, hw = N.JOIN_ORDER[maintain_order], N.JOIN_VALIDATE[validate], N.JOIN_HOW[how]
    rpay = [n for n in right.columns if n not in rkeys]
    take_single = builtins.len(lks) == 1 and lks[0].dtype.physical() in INTEGER_DTYPES
    take_multi = builtins.len(lks) > 1 and builtins.all(k.dtype.physical() in INTEGER_DTYPES + (Boolean,) for k in lks)
    if (how == "inner" and coalesce is not False and (take_single or take_multi)
            and builtins.len(left.columns) <= N.MAX_COLS and builtins.len(rpay) <= N.MAX_COLS):
        # join + the takes in one call (plgpu_join_inner_take): a row-format
        # table when one unique-keyed right column rides along
        lc = [left._cols[n] for n in left.columns]
        rc_ = [right._cols[n] for n in rpay]
        ol = (N.Column * max(1, builtins.len(lc)))()
        orr = (N.Column * max(1, builtins.len(rc_)))()
        nout = C.c_int64(0)
        if take_single:
            N.check(N.lib().plgpu_join_inner_take(C.byref(lks[0]._col), C.byref(rks[0]._col), _col_array(lc),
                                                  builtins.len(lc), _col_array(rc_), builtins.len(rc_),
                                                  int(nulls_equal), order, val, ol, orr, C.byref(nout), None))
        else:
            N.check(N.lib().plgpu_join_inner_take_multi(_col_array(lks), _col_array(rks), builtins.len(lks),
                                                        _col_array(lc), builtins.len(lc), _col_array(rc_),
                                                        builtins.len(rc_), int(nulls_equal), order, val, ol, orr,
                                                        C.byref(nout), None))
        out = [Series._from_native(n, ol[i], left._cols[n]._logical_dtype()) for i, n in enumerate(left.columns)]
        for i, n in enumerate(rpay):
            out.append(Series._from_native(n + suffix if n in left.columns else n, orr[i],
                                           right._cols[n]._logical_dtype()))
        return DataFrame(out)
    if builtins.len(lks) == 1 and lks[0].dtype.physical() in INTEGER_DTYPES:
        N.check(N.lib().plgpu_join(C.byref(lks[0]._col), C.byref(rks[0]._col), hw, int(nulls_equal), order, val,
                                   C.byref(li), C.byref(ri), None))
    else:
        # several keys (or a Float64 / Boolean key): packed or hashed tuples
        N.check(N.lib().plgpu_join_multi(_col_array(lks), _col_array(rks), builtins.len(lks), hw,
                                         int(nulls_equal), order, val, C.byref(li), C.byref(ri), None))
    lidx, ridx = Series._from_native("__left_idx", li), Series._from_native("__right_idx", ri)

    def take(df: DataFrame, names: list[str], idx: Series) -> list[Series]:
        if not names:
            return []
        out = (N.Column * builtins.len(names))()
        N.check(N.lib().plgpu_gather(_col_array([df._cols[n] for n in names]), builtins.len(names),
                                     C.byref(idx._col), out, None))
        return [Series._from_native(n, out[i], df._cols[n]._logical_dtype()) for i, n in enumerate(names)]

    if how in ("semi", "anti"):
        return DataFrame(take(left, left.columns, lidx))
    if coalesce is None:
        coalesce = how != "full"
    if coalesce and how == "right":
        lnames = [n for n in left.columns if n not in lkeys]
        rnames = right.columns
    else:
        lnames = left.columns
        rnames = [n for n in right.columns if not (coalesce and n in rkeys)]
    # A left join in left order that produced one row per left row has the
    # identity as its left index: the left columns are shared, not gathered
    # (the reference's _create_left_df_from_slice shortcut for a sorted index
    # of full length); likewise the right side of a right join.
    same_left = (how == "left" and maintain_order not in ("right", "right_left") and lidx.len() == left.height)
    same_right = (how == "right" and maintain_order not in ("left", "left_right") and ridx.len() == right.height)
    if same_right:
        take_right = [right._cols[n].alias(n) for n in rnames]
    out = [left._cols[n].alias(n) for n in lnames] if same_left else take(left, lnames, lidx)
    if coalesce and how == "full":
        rk_cols = take(right, rkeys, ridx)
        for lk, rk in zip(lkeys, rk_cols):
            i = lnames.index(lk)
            c = N.Column()
            N.check(N.lib().plgpu_coalesce(C.byref(out[i]._col), C.byref(rk._col), C.byref(c), None))
            out[i] = Series._from_native(lk, c, out[i]._logical_dtype())
    for s in (take_right if same_right else take(right, rnames, ridx)):
        if s.name in lnames:
            s.name = s.name + suffix
        out.append(s)
    return DataFrame(out)


def _sort(df: DataFrame, by: str | tuple, descending: bool | tuple, nulls_last: bool | tuple) -> DataFrame:
    names = _gb_keys(by)
    for nm in names:
        if nm not in df._cols:
            raise N.ComputeError(f'unable to find column "{nm}"; valid columns: {df.columns}')
    if builtins.len(names) == 1 and df._cols[names[0]].dtype.physical() not in (Boolean, String):
        idx = df._cols[names[0]].arg_sort(descending=bool(descending), nulls_last=bool(nulls_last))
    else:
        k = builtins.len(names)
        desc = descending if isinstance(descending, tuple) else (descending,)
        nl = nulls_last if isinstance(nulls_last, tuple) else (nulls_last,)
        out_idx = N.Column()
        N.check(N.lib().plgpu_arg_sort_multi(_col_array([df._cols[nm] for nm in names]), k,
                                             (C.c_int32 * k)(*map(int, desc)), (C.c_int32 * k)(*map(int, nl)),
                                             C.byref(out_idx), None))
        idx = Series._from_native("__idx", out_idx)
    names = df.columns
    out = (N.Column * builtins.len(names))()
    N.check(N.lib().plgpu_gather(_col_array([df._cols[n] for n in names]), builtins.len(names),
                                 C.byref(idx._col), out, None))
    return DataFrame([Series._from_native(n, out[i], df._cols[n]._logical_dtype()) for i, n in enumerate(names)])


def _execute(node: tuple, info: dict | None = None) -> DataFrame:
    kind = node[0]
    if kind == "scan":
        return node[1]
    if kind == "join":
        return _join(_execute(node[1], info), _execute(node[2], info), *node[3:])
    if kind == "sort":
        return _sort(_execute(node[1], info), node[2], node[3], node[4])
    if kind == "filter":
        df = _execute(node[1], info)
        return _filter(df, node[2])
    if kind == "group_by":
        child = node[1]
        pred = None
        if child[0] == "filter":  # predicate pushed into the aggregation kernel
            pred = child[2]
            child = child[1]
        df = _execute(child, info)
        return _group_by(df, node[2], node[3], node[4], pred, info)
    if kind == "select" and node[2] and builtins.all(_agg_base(e).kind in ("agg", "len") for e in node[2]):
        # select(aggregations): a global reduction (polars-expr/src/reduce/
        # sum.rs:112 reduce_ca and siblings), the fused group-by kernel with
        # one group; a filter below it runs inside the same pass
        child, pred = node[1], None
        if child[0] == "filter":
            pred, child = child[2], child[1]
        return _group_by(_execute(child, info), None, node[2], False, pred, info)
    if kind in ("select", "with_columns"):
        df = _execute(node[1], info)
        if builtins.any(_agg_base(e).kind in ("agg", "len") for e in node[2]):
            raise N.InvalidOperationError("mixing aggregations and elementwise expressions in one select is not "
                                          "supported on the GPU executor")
        new = [_eval(e, df) for e in node[2]]
        if kind == "select":
            return DataFrame(new)
        cols = dict(df._cols)
        for s in new:
            cols[s.name] = s
        return DataFrame(list(cols.values()))
    raise N.InvalidOperationError(f"unknown plan node {kind}")


def from_dict(data: dict, schema: Any = None) -> DataFrame:
    return DataFrame(data, schema)
