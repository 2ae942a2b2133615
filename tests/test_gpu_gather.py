"""GPU parity of the multi-column gather (plgpu_gather), the materialisation
step of sort_by and of joins (reference: polars-core/src/chunked_array/ops/
gather.rs, take by index; DataFrame::sort = arg_sort then take).

Four or more null-free 8-byte columns of >= 2^20 rows take the packed-row
route (aos_pack_kernel + aos_gather_kernel: rows transposed through LDS on
both sides); fewer columns, other widths and nullable columns go column by
column.  Bar: bit-exact against numpy's take of the same index, for every
column count 1..9 (an odd count pads the packed row), a tail block of fewer
than 256 rows, repeated indices and index columns shorter / longer than the
frame.
"""

import ctypes as C

import numpy as np
import pytest

import polaroid_amd as pl
from polaroid_amd import _native as N
from polaroid_amd.frame import _col_array

pytestmark = pytest.mark.gpu


def _gather(series, idx):
    out = (N.Column * len(series))()
    s_idx = pl.Series.from_numpy("idx", idx.astype(np.uint32))
    N.check(N.lib().plgpu_gather(_col_array(series), len(series), C.byref(s_idx._col), out, None))
    return [pl.Series._from_native(s.name, out[i], s._logical_dtype()) for i, s in enumerate(series)]


@pytest.mark.parametrize("ncols", [1, 3, 4, 5, 7, 8, 9])
@pytest.mark.parametrize("rows,nidx", [((1 << 20) + 77, (1 << 20) + 77), ((1 << 20) + 3, 1_500_001),
                                       (2_000_000, (1 << 20) + 255)])
def test_packed_gather_vs_numpy(gpu, ncols, rows, nidx):
    rng = np.random.default_rng(ncols * 7 + rows % 97 + nidx % 13)
    cols = []
    for k in range(ncols):
        if k % 2:
            cols.append(rng.standard_normal(rows))
        else:
            cols.append(rng.integers(-2**62, 2**62, rows).astype(np.int64))
    idx = rng.integers(0, rows, nidx).astype(np.int64)
    idx[: nidx // 4] = idx[0]  # repeated rows
    series = [pl.Series.from_numpy(f"c{k}", c) for k, c in enumerate(cols)]
    df = pl.DataFrame(series)
    got = _gather([df[f"c{k}"] for k in range(ncols)], idx)
    for k in range(ncols):
        assert got[k].len() == nidx
        assert np.array_equal(got[k].to_numpy().view(np.uint64), cols[k][idx].view(np.uint64)), k


def test_sort_frame_8_columns_packed_route(gpu):
    """DataFrame.sort of an 8-column frame above the packed-route threshold,
    with a tail block and ties (stable), against numpy's stable argsort."""
    rng = np.random.default_rng(3)
    n = (1 << 20) + 1234
    ts = rng.integers(0, 1 << 40, n).astype(np.int64)
    ts[rng.random(n) < 0.2] = 123456
    data = {"ts": ts}
    for k in range(3):
        data[f"i{k}"] = rng.integers(0, 1 << 20, n).astype(np.int64)
    for k in range(4):
        data[f"f{k}"] = 100 + rng.random(n) * 50
    df = pl.DataFrame({k: pl.Series.from_numpy(k, v) for k, v in data.items()})
    out = df.sort("ts")
    order = np.argsort(ts, kind="stable")
    for k, v in data.items():
        assert np.array_equal(out[k].to_numpy().view(np.uint64), v[order].view(np.uint64)), k
