"""GPU parity of the partitioned (radix) inner join + take (join.hip
jn_radix_take): the order-free join of BASELINE configs[3] with L2-resident
per-partition sub-tables.  Reference: polars-ops/src/frame/join/hash_join/
single_keys.rs:16 build_tables (per-partition tables), single_keys_inner.rs:40
probe_inner; the pairs are the oracle's (oracle/polars_oracle.c:or_join_inner)
compared as a multiset, since maintain_order="none" leaves the order
unspecified (as in the reference).

Bar: bit-exact, every (left row, right row) pair once, payloads travelling with
their rows.  The path is checked to have run (its kernels in the kernel
timer), and forced onto one and two partition levels, carried-column counts
0 .. 4, both probe batch widths, and its fallbacks (duplicate / INT64_MIN
build keys).
"""
import ctypes as C

import numpy as np
import pytest

import polaroid_amd as pl
from polaroid_amd import _native as N
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _kt():
    return N.ktime_read(reset=True)


def _join(left, right, **kw):
    N.set_option("ktime", 1)
    _kt()
    try:
        out = left.join(right, on="k", **kw)
        names = _kt()
    finally:
        N.set_option("ktime", 0)
    return out, names


def _unique_keys(rng, n, span):
    return (rng.permutation(span)[:n].astype(np.int64) - span // 2) * 1_000_003


def _check(out, lk, rk, ncarry, lcols, pay):
    """Multiset equality of (left row, right row) pairs against the oracle,
    with the key and every carried column taken at the left row."""
    ol, orr = O.join_inner(O.HostCol(lk), O.HostCol(rk))
    assert out.height == ol.shape[0]
    li = out["li"].to_numpy().astype(np.int64)
    p = out["p"].to_numpy()
    a = np.argsort(li, kind="stable")
    b = np.argsort(ol, kind="stable")
    assert np.array_equal(li[a], ol[b])
    assert np.array_equal(p[a], pay[orr[b]])
    assert np.array_equal(out["k"].to_numpy()[a], lk[ol[b]])
    for j in range(ncarry - 1):
        assert np.array_equal(out[f"c{j}"].to_numpy()[a], lcols[j][ol[b]]), j


@pytest.mark.parametrize("nl,nr,keys_per,ncarry", [
    (1, 1, 0, 1), (1000, 100, 16, 1), (50_000, 20_000, 64, 1), (300_001, 60_000, 1024, 2),
    (300_001, 60_000, 32, 3),      # 2^11 partitions: two scatter levels
    (200_000, 100_000, 512, 4), (120_000, 7, 1, 5), (4099, 3000, 100, 2)])
@pytest.mark.parametrize("batch", [8, 4])
def test_radix_join_forced_vs_oracle(gpu, plgpu_option, nl, nr, keys_per, ncarry, batch):
    """Forced onto the partitioned path (join_radix = 2) with small
    partitions; carried left columns besides the key: li plus ncarry - 1;
    the match pass with 8 or 4 probe steps in flight."""
    plgpu_option("join_radix", 2)
    plgpu_option("join_radix_keys", keys_per)
    plgpu_option("join_radix_batch", batch)
    rng = np.random.default_rng(nl + nr + keys_per)
    rk = _unique_keys(rng, nr, 4 * max(nr, 1))
    rk[0] = np.iinfo(np.int64).max
    lk = rk[rng.integers(0, nr, nl)].copy()
    miss = rng.random(nl) < 0.5
    lk[miss] = (rng.integers(0, 1 << 40, int(miss.sum())) * 2 + 1)  # odd: never a build key
    if nl > 3:
        lk[3] = np.iinfo(np.int64).min  # the empty marker as a probe key: no match
    pay = np.arange(nr, dtype=np.int64) * 5 - 7
    lcols = [rng.standard_normal(nl), rng.integers(-9, 9, nl).astype(np.int64), rng.random(nl)][:max(ncarry - 2, 0)]
    left = pl.DataFrame([pl.Series.from_numpy("k", lk), pl.Series.from_numpy("li", np.arange(nl, dtype=np.int64))] +
                        [pl.Series.from_numpy(f"c{j}", c) for j, c in enumerate(lcols)])
    right = pl.DataFrame([pl.Series.from_numpy("k", rk), pl.Series.from_numpy("p", pay)])
    out, names = _join(left, right)
    assert "rj_match_kernel" in names, names
    _check(out, lk, rk, len(lcols) + 1, lcols, pay)


def test_radix_join_fallbacks(gpu, plgpu_option):
    """Duplicate or INT64_MIN build keys leave the partitioned path for the
    row-format / pairs join, with the same result; ordered modes never take
    it."""
    plgpu_option("join_radix", 2)
    plgpu_option("join_radix_keys", 64)
    rng = np.random.default_rng(9)
    nl, nr = 100_000, 20_000
    base = _unique_keys(rng, nr, 100_000)
    pay = np.arange(nr, dtype=np.int64)
    lk = base[rng.integers(0, nr, nl)]
    left = pl.DataFrame([pl.Series.from_numpy("k", lk), pl.Series.from_numpy("li", np.arange(nl, dtype=np.int64))])
    for case in ("dup", "min"):
        rk = base.copy()
        if case == "dup":
            rk[10] = rk[11]
        else:
            rk[10] = np.iinfo(np.int64).min
        right = pl.DataFrame([pl.Series.from_numpy("k", rk), pl.Series.from_numpy("p", pay)])
        out, names = _join(left, right)
        assert "rj_match_kernel" not in names, case
        ol, orr = O.join_inner(O.HostCol(lk), O.HostCol(rk))
        a, b = np.lexsort((out["p"].to_numpy(), out["li"].to_numpy())), np.lexsort((orr, ol))
        assert np.array_equal(out["li"].to_numpy()[a], ol[b]) and np.array_equal(out["p"].to_numpy()[a], pay[orr[b]])
    right = pl.DataFrame([pl.Series.from_numpy("k", base), pl.Series.from_numpy("p", pay)])
    out, names = _join(left, right, maintain_order="left")
    assert "rj_match_kernel" not in names
    ol, orr = O.join_inner(O.HostCol(lk), O.HostCol(base))
    perm = np.argsort(ol, kind="stable")
    assert np.array_equal(out["li"].to_numpy(), ol[perm]) and np.array_equal(out["p"].to_numpy(), pay[orr[perm]])


def test_radix_join_key_listed_twice_and_absent(gpu, plgpu_option):
    """Through the C-ABI: the key column listed twice among the left columns
    (the second is a copy of the first) and not at all."""
    from polaroid_amd.frame import _col_array

    plgpu_option("join_radix", 2)
    plgpu_option("join_radix_keys", 128)
    rng = np.random.default_rng(4)
    nl, nr = 70_000, 9_000
    rk = _unique_keys(rng, nr, 40_000)
    lk = rk[rng.integers(0, nr, nl)]
    lk[rng.random(nl) < 0.3] = 3  # 3 * odd: not a build key (keys are multiples of 1_000_003)
    sk, sl = pl.Series.from_numpy("k", lk), pl.Series.from_numpy("li", np.arange(nl, dtype=np.int64))
    sr, sp = pl.Series.from_numpy("k", rk), pl.Series.from_numpy("p", np.arange(nr, dtype=np.int64) * 3)
    ol, orr = O.join_inner(O.HostCol(lk), O.HostCol(rk))
    for lcols in ([sk, sl, sk], [sl]):
        ol_ = (N.Column * len(lcols))()
        or_ = (N.Column * 1)()
        nout = C.c_int64(0)
        N.check(N.lib().plgpu_join_inner_take(C.byref(sk._col), C.byref(sr._col), _col_array(lcols), len(lcols),
                                              _col_array([sp]), 1, 0, N.JOIN_ORDER["none"], N.JOIN_VALIDATE["m:m"],
                                              ol_, or_, C.byref(nout), None))
        outs = [pl.Series._from_native(f"o{i}", ol_[i]) for i in range(len(lcols))]
        pay = pl.Series._from_native("p", or_[0])
        assert nout.value == ol.shape[0]
        li = outs[next(i for i, s in enumerate(lcols) if s is sl)].to_numpy().astype(np.int64)
        a, b = np.argsort(li, kind="stable"), np.argsort(ol, kind="stable")
        assert np.array_equal(li[a], ol[b])
        assert np.array_equal(pay.to_numpy()[a], (np.arange(nr, dtype=np.int64) * 3)[orr[b]])
        for i, s in enumerate(lcols):
            if s is sk:
                assert np.array_equal(outs[i].to_numpy()[a], lk[ol[b]])


@pytest.mark.slow
def test_radix_join_default_path_sampled_estimate(gpu):
    """Default thresholds (probe >= 2^22 rows, build >= 2^17 keys): the
    partitioned path runs by itself, with the sampled (not exact) estimate
    of the output regions; 9e6 x 3e5, 40 % hits, checked on the device."""
    import torch

    n, m = 9_000_000, 300_000
    g = torch.Generator(device="cuda")
    g.manual_seed(12)
    bk = torch.randperm(4 * m, device="cuda", generator=g)[:m].to(torch.int64) * 3
    pk = torch.randint(0, 4 * m, (n,), device="cuda", generator=g, dtype=torch.int64)
    pk = torch.where(torch.rand(n, device="cuda", generator=g) < 0.45, bk[pk % m], pk * 3 + 1)
    left = pl.DataFrame([pl.Series.from_torch("k", pk),
                         pl.Series.from_torch("a", torch.arange(n, device="cuda", dtype=torch.int64))])
    right = pl.DataFrame([pl.Series.from_torch("k", bk), pl.Series.from_torch("b", torch.arange(m, device="cuda",
                                                                                                   dtype=torch.int64))])
    out, names = _join(left, right)
    assert "rj_match_kernel" in names and names["rj_match_kernel"][1] == 1
    member = torch.zeros(12 * m + 2, dtype=torch.bool, device="cuda")
    member[bk] = True
    hit = member[pk]
    assert out.height == int(hit.sum().item())
    a, b, k = out["a"].to_torch(), out["b"].to_torch(), out["k"].to_torch()
    assert torch.equal(pk[a], k) and torch.equal(bk[b], k)
    assert torch.equal(torch.sort(a).values, torch.nonzero(hit).flatten())
