"""GPU parity of the radix arg-sort and the fixed-window rolling sum / mean
through the C-ABI, against the oracle (oracle/polars_oracle.c: or_arg_sort,
or_rolling) and the golden cases of operations/test_sort.py and
operations/rolling/test_rolling.py.

Bars:
  sort    - bit-exact permutation (stable; TotalOrd; nulls first / last);
  rolling - bit-exact against the exact window sum (oracle mode 1); against
            the reference's Kahan sliding window (mode 0) within the drift
            measured in tests/test_oracle.py (<= 2 ULP for w >= 20 on
            null-free data; otherwise relative 1e-10 of the window's sum of
            |x|, measured up to 4.6e-12); integer sums identical (wrapping).
"""

import math

import numpy as np
import pytest

import polaroid_amd as pl
from conftest import check_rolling_case, load_golden, unhex
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _vals(case_vals):
    return [unhex(v) if isinstance(v, str) else v for v in case_vals]


def _series(vals):
    isf = any(isinstance(v, float) for v in vals if v is not None)
    return pl.Series("x", vals, pl.Float64 if isf else pl.Int64)


def _same(a, b):
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b


# ------------------------------------------------------------------ sort
def test_sort_golden(gpu):
    for case in load_golden("sort_cases.json")["cases"]:
        vals = _vals(case["values"])
        s = _series(vals)
        a = case["args"]
        kw = dict(descending=a.get("descending", False), nulls_last=a.get("nulls_last", False))
        if "expected_arg_sort" in case:
            assert s.arg_sort(**kw).to_list() == case["expected_arg_sort"], case["name"]
        else:
            got = s.sort(**kw).to_list()
            assert all(_same(g, e) for g, e in zip(got, _vals(case["expected_sorted"]))), case["name"]
        # DataFrame.sort agrees
        df = pl.DataFrame([s, pl.Series("i", list(range(len(vals))), pl.Int64)])
        out = df.sort("x", **kw)
        assert out["i"].to_list() == O.arg_sort(_host(vals), **kw).tolist()


def _host(vals):
    isf = any(isinstance(v, float) for v in vals if v is not None)
    arr = np.array([0 if v is None else v for v in vals], np.float64 if isf else np.int64)
    valid = np.array([v is not None for v in vals], bool)
    return O.HostCol(arr, None if valid.all() else valid)


def _rand_col(rng, n, dtype, nulls, specials):
    if dtype == "f64":
        v = rng.standard_normal(n) * 1000
        v[rng.random(n) < 0.3] = 42.0  # ties
        if specials and n:
            v[rng.random(n) < 0.02] = np.nan
            v[rng.random(n) < 0.02] = -0.0
            v[rng.random(n) < 0.02] = 0.0
            v[rng.random(n) < 0.01] = np.inf
            v[rng.random(n) < 0.01] = -np.inf
    elif dtype == "i64":
        v = rng.integers(-2**62, 2**62, n).astype(np.int64)
        v[rng.random(n) < 0.3] = 7  # ties
        if specials and n:
            v[rng.random(n) < 0.01] = np.iinfo(np.int64).min
            v[rng.random(n) < 0.01] = np.iinfo(np.int64).max
    elif dtype == "i32":
        v = rng.integers(-2**31, 2**31 - 1, n).astype(np.int32)
        v[rng.random(n) < 0.3] = -5
    else:
        v = rng.integers(0, 1000, n).astype(np.uint32)
    valid = (rng.random(n) > 0.1) if nulls else None
    return v, valid


@pytest.mark.parametrize("n", [0, 1, 2, 100, 4095, 4096, 4097, 100003, 1_000_000])
@pytest.mark.parametrize("dtype", ["f64", "i64", "i32", "u32"])
@pytest.mark.parametrize("nulls", [False, True])
def test_arg_sort_vs_oracle(gpu, n, dtype, nulls):
    rng = np.random.default_rng(n + len(dtype) * 7 + nulls)
    v, valid = _rand_col(rng, n, dtype, nulls, True)
    s = pl.Series.from_numpy("x", v, valid)
    for descending in (False, True):
        for nulls_last in (False, True):
            got = s.arg_sort(descending=descending, nulls_last=nulls_last).to_numpy()
            exp = O.arg_sort(O.HostCol(v, valid), descending, nulls_last)
            assert np.array_equal(got.astype(np.int64), exp), (descending, nulls_last)


def test_sort_frame_and_slices(gpu):
    rng = np.random.default_rng(4)
    n = 50_000
    k = rng.integers(0, 100, n).astype(np.int64)
    a = rng.standard_normal(n)
    va = rng.random(n) > 0.2
    df = pl.DataFrame({"k": pl.Series.from_numpy("k", k), "a": pl.Series.from_numpy("a", a, va)})
    out = df.sort("k", descending=True)
    idx = O.arg_sort(O.HostCol(k), True, False)
    assert np.array_equal(out["k"].to_numpy(), k[idx])
    assert np.array_equal(out["a"].validity_numpy(), va[idx])
    assert np.array_equal(out["a"].to_numpy()[va[idx]], a[idx][va[idx]])
    # a sliced (offset) column sorts like the same values in a fresh column
    s = pl.Series.from_numpy("k", k).slice(1234, 10_000)
    assert np.array_equal(s.arg_sort().to_numpy().astype(np.int64), O.arg_sort(O.HostCol(k[1234:11234])))


@pytest.mark.slow
def test_sort_large_properties(gpu):
    import torch

    n = 100_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    k = torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g, dtype=torch.int64)
    s = pl.Series.from_torch("k", k)
    idx = torch.from_numpy(s.arg_sort().to_numpy().astype(np.int64)).cuda()
    sk = k[idx]
    assert bool((sk[1:] >= sk[:-1]).all())
    assert torch.equal(torch.sort(idx).values, torch.arange(n, device="cuda"))
    ref = torch.sort(k, stable=True)
    assert torch.equal(ref.indices, idx)


# --------------------------------------------------------------- rolling
def test_rolling_golden(gpu):
    for case in load_golden("rolling_cases.json")["cases"]:
        s = _series(_vals(case["values"]))
        fn = getattr(s, "rolling_" + case["kind"])
        kw = {"ddof": case["ddof"]} if "ddof" in case else {}
        got = fn(case["window"], min_samples=case["min"], center=case["center"], **kw).to_list()
        check_rolling_case(got, case, "gpu")


def _rolling_check(v, valid, kind, w, ms, center, ref_bound=True):
    s = pl.Series.from_numpy("x", v, valid)
    fn = s.rolling_mean if kind == "mean" else s.rolling_sum
    out = fn(w, min_samples=ms, center=center)
    gv, gok = out.to_numpy(), out.validity_numpy()
    hc = O.HostCol(v, valid)
    ev, eok = O.rolling(hc, kind, w, ms, center, O.ROLLING_EXACT)
    assert np.array_equal(gok, eok)
    if gv.dtype.kind in "iu":
        assert np.array_equal(gv[gok].astype(np.int64), ev[eok].astype(np.int64))
        rv, rok = O.rolling(hc, kind, w, ms, center, O.ROLLING_REFERENCE)
        assert np.array_equal(gok, rok) and np.array_equal(gv[gok].astype(np.int64), rv[rok])
        return
    g, e = gv[gok], ev[eok]
    assert np.array_equal(np.isnan(g), np.isnan(e))
    m = ~np.isnan(e)
    assert np.array_equal(g[m].view(np.int64), e[m].view(np.int64)), (kind, w, ms, center)
    if ref_bound:
        rv, rok = O.rolling(hc, kind, w, ms, center, O.ROLLING_REFERENCE)
        assert np.array_equal(gok, rok)
        r = rv[rok]
        fin = np.isfinite(r) & np.isfinite(g)
        assert np.array_equal(np.isfinite(r), np.isfinite(g))
        if w >= 20 and valid is None:
            d = np.abs(g[fin].view(np.int64) - r[fin].view(np.int64))
            assert d.max(initial=0) <= 2
        else:
            # relative to the window's sum of |x| (finite, non-null values)
            n = v.shape[0]
            i = np.arange(n)
            if center:
                right = (w + 1) // 2
                st, en = np.maximum(0, i - (w - right)), np.minimum(n, i + right)
            else:
                st, en = np.maximum(0, i + 1 - w), i + 1
            a = np.where(np.isfinite(v) & (valid if valid is not None else True), np.abs(v.astype(np.float64)), 0.0)
            cs = np.concatenate([[0.0], np.cumsum(a)])
            mag = (cs[en] - cs[st])[gok]
            if kind == "mean":
                cnt = np.concatenate([[0], np.cumsum(valid if valid is not None else np.ones(n, bool))])
                mag = mag / np.maximum(1, (cnt[en] - cnt[st])[gok])
            rel = np.abs(g[fin] - r[fin]) / np.maximum(mag[fin], 1e-300)
            # the reference's sliding Kahan state drifts: measured 2.1e-13
            # (w=3, positive data) and 4.6e-12 (w=3, mixed signs, nulls, inf)
            assert rel.max(initial=0) <= 1e-10


@pytest.mark.parametrize("n", [1, 7, 1023, 1024, 1025, 5000, 300_001])
@pytest.mark.parametrize("w", [1, 2, 3, 20, 257, 1500, 5000])
@pytest.mark.parametrize("kind", ["sum", "mean"])
def test_rolling_vs_oracle(gpu, n, w, kind):
    if n > 50_000 and w == 5000:
        pytest.skip("direct path, covered at smaller n")
    rng = np.random.default_rng(n * 31 + w)
    v = rng.uniform(10, 500, n) * np.exp(0.02 * rng.standard_normal(n))
    for ms, center in ((None, False), (1, False), (max(1, w // 2), True)):
        _rolling_check(v, None, kind, w, w if ms is None else ms, center)


@pytest.mark.parametrize("kind", ["sum", "mean"])
def test_rolling_nulls_and_specials(gpu, kind):
    rng = np.random.default_rng(12)
    n = 50_000
    v = rng.standard_normal(n) * 10
    v[rng.random(n) < 0.01] = np.nan
    v[rng.random(n) < 0.01] = np.inf
    v[rng.random(n) < 0.01] = -np.inf
    valid = rng.random(n) > 0.2
    for w, ms, center in ((3, 1, False), (20, 5, True), (300, 300, False), (4000, 100, False)):
        _rolling_check(v, valid, kind, w, ms, center)


def _span_data(kind, n, rng):
    if kind == "narrow":      # one int64 fixed-point word per value
        return rng.uniform(100, 150, n)
    if kind == "mixed":       # ~40 binades, mixed signs: 128-bit words
        return rng.standard_normal(n) * np.exp2(rng.integers(-20, 20, n))
    if kind == "tiny":        # subnormal values and results
        v = rng.standard_normal(n) * 5e-324 * 2 ** 40
        v[::7] = rng.integers(-3, 4, v[::7].shape[0]) * 5e-324
        return v
    if kind == "cancel":      # exact cancellations around large values
        v = rng.uniform(-1, 1, n)
        v[::5] = 2.0 ** 60
        v[2::5] = -(2.0 ** 60)
        return v
    v = rng.uniform(-1, 1, n)  # "huge": beyond 128 bits, per-output exact
    v[::31] = 1e200
    v[1::31] = -1e200
    v[3::31] = -0.0          # all -0.0 windows sum to +0.0 (SumWindow starts at +0.0)
    return v


@pytest.mark.parametrize("span", ["narrow", "mixed", "tiny", "cancel", "huge"])
@pytest.mark.parametrize("w", [1, 2, 5, 63, 64])
def test_rolling_wave_kernel_modes(gpu, span, w):
    """The w <= 64 wave-scan kernel in each number format it picks per wave
    (int64 / 128-bit fixed point, per-output exact), across wave and
    workgroup boundaries (1024 / 4096 outputs), centred and clipped."""
    rng = np.random.default_rng(w * 7 + len(span))
    n = 4096 * 3 + 1024 + 17
    v = _span_data(span, n, rng)
    valid = rng.random(n) > 0.1
    for ms, center in ((w, False), (1, True), (max(1, w // 3), False)):
        for kind in ("sum", "mean"):
            _rolling_check(v, None, kind, w, ms, center, ref_bound=False)
            _rolling_check(v, valid, kind, w, ms, center, ref_bound=False)


@pytest.mark.parametrize("data", ["narrow", "zeros", "low", "high", "overflow"])
@pytest.mark.parametrize("full", [1, 0])
def test_rolling_full_waves_specialised_scan(gpu, plgpu_option, data, full):
    """Interior int64-form waves take rw_scan_full (option rl_full): its
    window indexing, the zeroed prefix -1 and the one-correction mean with
    no per-lane range test when the wave's exponents allow it ("low" /
    "high": just outside that range, divided; "overflow": sums that round
    to inf).  Bit-exact against the oracle with the option on and off."""
    plgpu_option("rl_full", full)
    rng = np.random.default_rng(len(data) * 5 + full)
    n = 4096 * 2 + 777
    v = {"narrow": lambda: rng.uniform(100, 150, n),
         "zeros": lambda: np.where(rng.random(n) < 0.5, 0.0, -0.0),
         "low": lambda: rng.uniform(1, 2, n) * 2.0 ** -851,
         "high": lambda: rng.uniform(1, 2, n) * 2.0 ** 990,
         "overflow": lambda: rng.uniform(0.5, 1, n) * 1.7e308}[data]()
    for w in (1, 2, 20, 64):
        for center in (False, True):
            for kind in ("sum", "mean"):
                _rolling_check(v, None, kind, w, w, center, ref_bound=False)


def test_rolling_wide_exponent_span_is_exact(gpu):
    """A tile whose values span far more than one fixed-point window takes
    the exact per-output path (1e300 next to 1e-300 and cancellations)."""
    rng = np.random.default_rng(3)
    n = 20_000
    v = rng.uniform(-1, 1, n)
    v[::97] = 1e300
    v[1::97] = -1e300
    v[5::113] = 1e-300
    for kind in ("sum", "mean"):
        _rolling_check(v, None, kind, 5, 1, False, ref_bound=False)


@pytest.mark.parametrize("dt", [np.int64, np.int32])
def test_rolling_integers(gpu, dt):
    rng = np.random.default_rng(8)
    n = 100_000
    v = rng.integers(np.iinfo(dt).min // 2, np.iinfo(dt).max // 2, n).astype(dt)
    valid = rng.random(n) > 0.05
    for kind in ("sum", "mean"):
        for w in (2, 50, 3000):
            _rolling_check(v, valid, kind, w, 1, False, ref_bound=False)
            _rolling_check(v, None, kind, w, w, False, ref_bound=False)


def test_rolling_select_expression(gpu):
    df = pl.DataFrame({"a": [1.0, 2.0, 3.0, 4.0, 5.0]})
    out = df.select(pl.col("a").rolling_mean(3, min_samples=1).alias("m"), (pl.col("a") * 2).rolling_sum(2))
    assert out["m"].to_list() == [1.0, 1.5, 2.0, 3.0, 4.0]
    assert out["a"].to_list() == [None, 6.0, 10.0, 14.0, 18.0]
    with pytest.raises(pl.InvalidOperationError):
        pl.col("a").rolling_mean(2, min_samples=3)


@pytest.mark.parametrize("kind", ["min", "max"])
@pytest.mark.parametrize("w,n", [(1, 300_001), (3, 300_001), (20, 300_001), (64, 300_001), (65, 300_001),
                                 (1000, 100_001), (5000, 60_000)])
@pytest.mark.parametrize("nulls", [False, True])
@pytest.mark.parametrize("center", [False, True])
def test_rolling_minmax_vs_oracle(gpu, kind, w, n, nulls, center):
    """rolling_min / rolling_max: direct windows (w <= 64) and van Herk blocks
    (w > 64) against the oracle's window scan; NaN / inf / -0.0 / nulls;
    Float64, Int64 and Int32.  Bar: bit-exact values (signed zeros compare
    equal: the reference's choice between -0.0 and 0.0 follows its scan
    order) and validity."""
    rng = np.random.default_rng(w + 2 * nulls + center + len(kind))
    x = rng.standard_normal(n) * 100
    x[rng.random(n) < 0.001] = np.nan
    x[rng.random(n) < 0.001] = np.inf
    x[rng.random(n) < 0.001] = -0.0
    valid = rng.random(n) > 0.05 if nulls else None
    for v in (x, rng.integers(-2**40, 2**40, n).astype(np.int64), rng.integers(-2**31, 2**31, n).astype(np.int32)):
        ms = None if not nulls else max(1, w // 2)
        s = pl.Series.from_numpy("x", v, valid)
        out = getattr(s, "rolling_" + kind)(w, min_samples=ms, center=center)
        ev, eok = O.rolling(O.HostCol(v, valid), kind, w, ms, center)
        gv, gok = out.to_numpy(), out.validity_numpy()
        assert np.array_equal(gok, eok)
        if v.dtype == np.float64:
            g, e = gv[gok], ev[eok]
            assert np.array_equal(np.isnan(g), np.isnan(e))
            m = ~np.isnan(e)
            assert np.array_equal(g[m], e[m])
        else:
            assert out.dtype is s.dtype
            assert np.array_equal(gv[gok].astype(np.int64), ev[eok].astype(np.int64))


# ------------------------------------------------------ rolling var / std
def _var_check(v, valid, w, ms, center, ddof, std, ref_bound=False):
    """Bit-exact against the oracle's exact mode ((RN(c sum x^2 - (sum x)^2)
    / c) / (c - ddof)); validity identical to the reference's MomentWindow
    restatement (mode 0), and its values within the Welford fold's drift."""
    s = pl.Series.from_numpy("x", v, valid)
    out = (s.rolling_std if std else s.rolling_var)(w, min_samples=ms, center=center, ddof=ddof)
    assert out.dtype == (pl.Float32 if v.dtype == np.float32 else pl.Float64)
    gv, gok = out.to_numpy().astype(np.float64), out.validity_numpy()
    hc = O.HostCol(v.astype(np.float64) if v.dtype == np.float32 else v, valid)
    ev, eok = O.rolling_var(hc, w, ms, center, ddof, std, O.ROLLING_EXACT)
    rv, rok = O.rolling_var(hc, w, ms, center, ddof, std, O.ROLLING_REFERENCE)
    assert np.array_equal(gok, eok) and np.array_equal(gok, rok), (w, ms, center, ddof, std)
    g, e = gv[gok], ev[eok]
    if v.dtype == np.float32:
        # the variance rounded to Float32 (std: its f32 square root)
        e = (np.sqrt(O.rolling_var(hc, w, ms, center, ddof, False, O.ROLLING_EXACT)[0][eok].astype(np.float32))
             if std else e.astype(np.float32)).astype(np.float64)
    assert np.array_equal(np.isnan(g), np.isnan(e))
    m = ~np.isnan(e)
    assert np.array_equal(g[m].view(np.int64), e[m].view(np.int64)), (w, ms, center, ddof, std, g[m][:4], e[m][:4])
    if ref_bound:
        r = rv[rok]
        fin = np.isfinite(r) & np.isfinite(g)
        rel = np.abs(g[fin] - r[fin]) / np.maximum(np.abs(r[fin]), 1e-300)
        # the reference's sliding Welford state drifts with the column
        # (measured on 1e5 prices: 2.0e-11 at w = 5, 2.7e-13 at w = 20; at
        # w = 2 it reaches 3.4e-4, so no bound is asserted below w = 5)
        assert rel.max(initial=0) <= 1e-9


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1025, 100_003])
@pytest.mark.parametrize("w", [1, 2, 5, 20, 63, 64, 65, 200])
def test_rolling_var_std_vs_oracle(gpu, n, w):
    """Prices (the wave kernel's fast form), every window length form
    (w <= 64: wave kernel; larger: the direct kernel), ddof 0 / 1 / 2,
    centred and clipped windows, var and std."""
    rng = np.random.default_rng(n * 13 + w)
    v = rng.uniform(10, 500, n) * np.exp(0.02 * rng.standard_normal(n))
    for ms, center, ddof in ((w, False, 1), (1, True, 0), (max(1, w // 2), False, 2)):
        for std in (False, True):
            _var_check(v, None, w, ms, center, ddof, std, ref_bound=ms > ddof and w >= 5)


@pytest.mark.parametrize("span", ["narrow", "mixed", "tiny", "cancel", "huge"])
@pytest.mark.parametrize("w", [2, 5, 20, 64])
def test_rolling_var_wave_forms(gpu, span, w):
    """The fast form (prefix sums of t and t^2) and the exact per-output big
    integers, chosen per wave: narrow prices, 40-binade mixed signs, subnormal
    values, exact cancellations around 2^60, 1e200 spans; nulls and
    centred windows."""
    rng = np.random.default_rng(w * 11 + len(span))
    n = 4096 * 2 + 1024 + 17
    v = _span_data(span, n, rng)
    valid = rng.random(n) > 0.1
    for ms, center, ddof in ((w, False, 1), (1, True, 0)):
        for std in (False, True):
            _var_check(v, None, w, ms, center, ddof, std)
            _var_check(v, valid, w, ms, center, ddof, std)


@pytest.mark.parametrize("data", ["narrow", "constant", "low", "high"])
@pytest.mark.parametrize("full", [1, 0])
def test_rolling_var_full_waves_specialised_scan(gpu, plgpu_option, data, full):
    """Interior fast-form waves take rw_var_scan_full (option rl_full): its
    32-bit ring indexing, the zeroed prefix -1 slots and the one-correction
    quotients num / w / (w - ddof) ("low" / "high": exponents just outside
    their range, divided; "constant": zero numerators).  Bit-exact against
    the oracle with the option on and off; ddof up to w (all null)."""
    plgpu_option("rl_full", full)
    rng = np.random.default_rng(len(data) * 7 + full)
    n = 4096 * 2 + 777
    v = {"narrow": lambda: rng.uniform(100, 150, n),
         "constant": lambda: np.full(n, 3.25),
         "low": lambda: rng.uniform(1, 2, n) * 2.0 ** -420,
         "high": lambda: rng.uniform(1, 2, n) * 2.0 ** 494}[data]()
    for w in (2, 20, 64):
        for center in (False, True):
            for ddof in (0, 1, w):
                _var_check(v, None, w, w, center, ddof, std=(ddof == 1))


def test_rolling_var_specials_nulls_and_dtypes(gpu):
    """NaN / inf in the window give NaN (MomentWindow's non-finite count),
    nulls are skipped, Int32 / Int64 enter as Float64 and Float32 stays
    Float32 (its variance rounded to Float32, std its f32 square root)."""
    rng = np.random.default_rng(21)
    n = 30_011
    v = rng.standard_normal(n) * 10
    v[rng.random(n) < 0.005] = np.nan
    v[rng.random(n) < 0.005] = np.inf
    v[rng.random(n) < 0.005] = -np.inf
    valid = rng.random(n) > 0.2
    for w, ms, center in ((3, 1, False), (20, 5, True), (100, 50, False)):
        for std in (False, True):
            _var_check(v, valid, w, ms, center, 1, std)
    for dt in (np.int32, np.int64):
        iv = rng.integers(-10**6, 10**6, n).astype(dt)
        for std in (False, True):
            _var_check(iv, valid, 10, 3, False, 1, std)
    fv = (rng.uniform(10, 500, n)).astype(np.float32)
    for std in (False, True):
        _var_check(fv, None, 20, 20, False, 1, std)


def test_rolling_var_expression(gpu):
    df = pl.DataFrame({"a": [1.0, 5.0, 3.0, 4.0]})
    out = df.select(pl.col("a").rolling_var(2).alias("v"), pl.col("a").rolling_std(2, ddof=0).alias("s"))
    assert out["v"].to_list() == [None, 8.0, 2.0, 0.5]
    assert out["s"].to_list() == [None, 2.0, 1.0, 0.5]


def test_rolling_var_ddof_range(gpu):
    """ddof is the reference's u8 (rolling/no_nulls/moment.rs RollingVarParams):
    the Series and Expr paths both refuse values outside 0..255 instead of
    wrapping them into the packed kind code."""
    s = pl.Series("a", [1.0, 5.0, 3.0, 4.0])
    for ddof in (-1, 256):
        with pytest.raises(pl.InvalidOperationError):
            s.rolling_var(2, ddof=ddof)
        with pytest.raises(pl.InvalidOperationError):
            s.rolling_std(2, ddof=ddof)
        with pytest.raises(pl.InvalidOperationError):
            pl.DataFrame({"a": [1.0, 2.0]}).select(pl.col("a").rolling_std(2, ddof=ddof))
    assert s.rolling_var(2, ddof=255).to_list() == [None, None, None, None]


@pytest.mark.parametrize("var128", [1, 0])
@pytest.mark.parametrize("span", [0, 1, 3, 4, 6])
def test_rolling_var_numerator_modulo_2_128(gpu, plgpu_option, var128, span):
    """rw_var_scan_full forms w S2 - S1^2 modulo 2^128 (option rl_var128)
    when the wave's exponent span bounds it below 2^128 (2 (54 + span) +
    2 lw <= 129; w = 64 allows span <= 3, w = 20 span <= 4, w = 2 span <=
    8), else in 192 bits.  Mixed signs with alternating extremes put the
    numerators at their largest; spans on both sides of each window's limit.
    Bit-exact against the oracle's exact variance with the option on and off."""
    plgpu_option("rl_var128", var128)
    rng = np.random.default_rng(span * 3 + var128)
    n = 4096 * 2 + 555
    mag = np.ldexp(rng.uniform(1.0, 2.0, n), rng.integers(0, span + 1, n))
    v = np.where(rng.random(n) < 0.5, -mag, mag)
    v[::2] = np.ldexp(1.999999, span)  # alternating near-extremes
    v[1::4] = -np.ldexp(1.999999, span)
    for w in (2, 20, 64):
        for ddof in (0, 1):
            _var_check(v, None, w, w, False, ddof, std=(ddof == 1))


@pytest.mark.parametrize("hot", [1, 0])
def test_rolling_var_common_block_kernel(gpu, plgpu_option, hot):
    """Option rl_var_hot: interior finite blocks whose numerators fit 128 bits
    run in rl_var_hot_kernel (std by the scaling-free square root), every
    other block is listed for rl_var_rest_kernel.  Prices with one NaN block,
    one 40-binade block and one block of values near 2^-380 (variances under
    the square root's unscaled range) between common blocks; bit-exact
    against the oracle with the option on and off."""
    plgpu_option("rl_var_hot", hot)
    rng = np.random.default_rng(70 + hot)
    n = 512 * 24 + 333
    v = rng.uniform(100, 150, n)
    v[512 * 5 + 100] = np.nan
    v[512 * 9:512 * 10] = rng.standard_normal(512) * np.exp2(rng.integers(-20, 20, 512))
    v[512 * 14:512 * 15] = rng.uniform(1, 2, 512) * 2.0 ** -380
    for w in (5, 20, 64):
        for ddof in (0, 1):
            for std in (False, True):
                _var_check(v, None, w, w, False, ddof, std)
                _var_check(v, None, w, 1, True, ddof, std)


@pytest.mark.parametrize("hot", [1, 0])
@pytest.mark.parametrize("kind", ["sum", "mean"])
def test_rolling_common_block_kernel(gpu, plgpu_option, kind, hot):
    """Option rl_mean_hot: interior finite blocks in the 64-bit form run in
    rl_mean_hot_kernel, every other block is listed for the general kernel.
    Prices with one NaN block, one 40-binade block (beyond 64 bits), one of
    values near 2^-930 (below the 64-bit form) and one near 2^970 (sums near
    the top of the one-correction quotient's range) between common blocks; Int64 and Int32 means enter as Float64.  Bit-exact against
    the oracle's exact mode with the option on and off."""
    plgpu_option("rl_mean_hot", hot)
    rng = np.random.default_rng(90 + hot)
    n = 512 * 24 + 333
    v = rng.uniform(100, 150, n)
    v[512 * 5 + 100] = np.nan
    v[512 * 9:512 * 10] = rng.standard_normal(512) * np.exp2(rng.integers(-20, 20, 512))
    v[512 * 14:512 * 15] = rng.uniform(1, 2, 512) * 2.0 ** -930
    v[512 * 18:512 * 19] = rng.uniform(1, 2, 512) * 2.0 ** 970
    for w in (1, 5, 20, 64):
        _rolling_check(v, None, kind, w, w, False, ref_bound=False)
        _rolling_check(v, None, kind, w, 1, True, ref_bound=False)
    if kind == "mean":
        for dt in (np.int64, np.int32):
            iv = rng.integers(-10**6, 10**6, n).astype(dt)
            s = pl.Series.from_numpy("x", iv, None)
            out = s.rolling_mean(20, min_samples=20)
            ev, eok = O.rolling(O.HostCol(iv.astype(np.float64), None), "mean", 20, 20, False, O.ROLLING_EXACT)
            assert np.array_equal(out.validity_numpy(), eok)
            assert np.array_equal(out.to_numpy()[eok].view(np.int64), ev[eok].view(np.int64))
