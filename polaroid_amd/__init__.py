"""polaroid_amd — MI355X-native executor backend for the Polars filter /
arithmetic / comparison / hash-group-by-aggregation hot path.

    import polaroid_amd as pl
    out = (pl.DataFrame({...}).lazy()
             .filter(pl.col("close") > 100.0)
             .group_by("symbol")
             .agg(pl.col("volume").sum(), pl.col("close").mean())
             .collect())

All compute runs in libpolaroid_gpu.so (hand-written HIP kernels for
gfx950) behind the C-ABI of include/polaroid_gpu.h.
"""

from . import _native
from ._native import (
    ComputeError,
    DeviceError,
    DuplicateError,
    InvalidOperationError,
    OutOfMemoryError,
    PolaroidError,
    ShapeError,
    device_count,
)
from .expr import Expr, col, count, first, last, len, lit, max, mean, min, sum, when
from .frame import (
    Boolean,
    DataFrame,
    DataType,
    Date,
    Datetime,
    Duration,
    Float32,
    Float64,
    GroupBy,
    Int8,
    Int16,
    Int32,
    Int64,
    LazyFrame,
    LazyGroupBy,
    Series,
    String,
    UInt8,
    UInt16,
    UInt32,
    UInt64,
    from_dict,
)

__all__ = [
    "Boolean", "ComputeError", "DataFrame", "DataType", "Date", "Datetime", "DeviceError", "DuplicateError",
    "Duration", "Expr", "Float32", "Float64", "GroupBy", "Int8", "Int16", "Int32", "Int64",
    "InvalidOperationError", "LazyFrame", "LazyGroupBy", "OutOfMemoryError", "PolaroidError", "Series",
    "ShapeError", "String", "UInt8", "UInt16", "UInt32", "UInt64", "col", "count", "device_count", "from_dict",
    "first", "last", "len", "lit", "max", "mean", "min", "sum", "when",
]


def native_library_path() -> str:
    return _native.LIB_PATH
