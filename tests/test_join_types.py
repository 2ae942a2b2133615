"""Left / right / full / semi / anti joins.

CPU (no marker): the oracle's restatement (oracle/polars_oracle.c:or_join +
oracle.join's order handling) reproduces every fixture transcribed from
operations/test_join.py (tests/golden/join_types_cases.json).

GPU (`-m gpu`): plgpu_join / plgpu_join_multi through the C-ABI against the
same fixtures and against the oracle on seeded random keys.  Bar:
bit-exact index sequences for every ordered mode; multisets where the
reference leaves the order unspecified (full join, maintain_order="none").
"""

import numpy as np
import pytest

from conftest import load_golden
from oracle import oracle as O

HOWS = ["left", "right", "full", "semi", "anti"]
ORDERS = ["none", "left", "right", "left_right", "right_left"]


def _keys(case):
    on = case["on"]
    return [on] if isinstance(on, str) else list(on)


def _host(vals):
    return (np.array([0 if v is None else v for v in vals], np.int64), np.array([v is not None for v in vals]))


def _oracle_pairs(case):
    ks = _keys(case)
    args = case["args"]
    lk = [_host(case["left"][k]) for k in ks]
    rk = [_host(case["right"][k]) for k in ks]
    neq, order = args.get("nulls_equal", False), args.get("maintain_order", "none")
    if len(ks) == 1:
        return O.join(O.HostCol(*lk[0]), O.HostCol(*rk[0]), case["how"], neq, order)
    return O.join_multi(lk, rk, case["how"], neq, order)


def _materialise(case, li, ri):
    """Output columns of a fixture join from its index pairs, laid out as the
    reference materialises them (semi / anti: the left rows; otherwise left
    columns, then right columns with `_right` on a clash; coalesced key
    columns dropped, a coalesced full join keeping coalesce(left, right))."""
    left, right, how = case["left"], case["right"], case["how"]
    ks = _keys(case)
    if how in ("semi", "anti"):
        return {c: [left[c][i] for i in li] for c in left}
    coalesce = case["args"].get("coalesce", how != "full")

    def get(col, idx):
        return [None if i < 0 else col[i] for i in idx]

    if coalesce and how == "right":
        lnames, rnames = [c for c in left if c not in ks], list(right)
    else:
        lnames, rnames = list(left), [c for c in right if not (coalesce and c in ks)]
    out = {c: get(left[c], li) for c in lnames}
    if coalesce and how == "full":
        for k in ks:
            out[k] = [a if a is not None else b for a, b in zip(out[k], get(right[k], ri))]
    for c in rnames:
        out[c + "_right" if c in lnames else c] = get(right[c], ri)
    return out


def _check(case, out):
    """`out`: column name -> list of values."""
    if "columns" in case:
        assert list(out) == case["columns"], case["name"]
    exp = case["expected"]
    cols = list(exp)
    if case["ordered"]:
        for c in cols:
            got = list(out[c])
            if "prefix" in case:
                got = got[: case["prefix"]]
            assert got == exp[c], (case["name"], c, got)
    else:
        key = lambda t: tuple((x is None, x if x is not None else 0) for x in t)  # noqa: E731
        got = sorted(zip(*[out[c] for c in cols]), key=key)
        want = sorted(zip(*[exp[c] for c in cols]), key=key)
        assert got == want, case["name"]


def test_oracle_join_types_golden():
    for case in load_golden("join_types_cases.json")["cases"]:
        li, ri = _oracle_pairs(case)
        _check(case, _materialise(case, list(li), None if ri is None else list(ri)))


def test_oracle_join_types_vs_nested_loop():
    """or_join against a nested loop over all pairs, for every type."""
    rng = np.random.default_rng(5)
    nl, nr = 300, 200
    lk, rk = rng.integers(0, 40, nl), rng.integers(0, 40, nr)
    lv, rv = rng.random(nl) > 0.1, rng.random(nr) > 0.1
    for neq in (False, True):
        def eq(i, j):
            if lv[i] and rv[j]:
                return lk[i] == rk[j]
            return neq and not lv[i] and not rv[j]

        m = [[j for j in range(nr) if eq(i, j)] for i in range(nl)]
        li, ri = O.join(O.HostCol(lk, lv), O.HostCol(rk, rv), "left", neq)
        exp = [(i, j) for i in range(nl) for j in (m[i] or [-1])]
        assert list(zip(li, ri)) == exp
        li, ri = O.join(O.HostCol(lk, lv), O.HostCol(rk, rv), "full", neq, "left_right")
        matched = {j for row in m for j in row}
        assert list(zip(li, ri)) == exp + [(-1, j) for j in range(nr) if j not in matched]
        semi, _ = O.join(O.HostCol(lk, lv), O.HostCol(rk, rv), "semi", neq)
        anti, _ = O.join(O.HostCol(lk, lv), O.HostCol(rk, rv), "anti", neq)
        assert list(semi) == [i for i in range(nl) if m[i]]
        assert list(anti) == [i for i in range(nl) if not m[i]]


# ----------------------------------------------------------------- GPU
def _frame(pl, d):
    return pl.DataFrame([pl.Series(k, v, pl.Int64) for k, v in d.items()])


@pytest.mark.gpu
def test_join_types_golden(gpu):
    import polaroid_amd as pl

    for case in load_golden("join_types_cases.json")["cases"]:
        left, right = _frame(pl, case["left"]), _frame(pl, case["right"])
        on = case["on"]
        out = left.join(right, on=on, how=case["how"], **case["args"])
        _check(case, {c: out[c].to_list() for c in out.columns})


def _rand(rng, n, card, null_frac):
    k = rng.integers(-card // 2, card - card // 2, n).astype(np.int64) * 7919
    if n:
        k[rng.random(n) < 0.01] = np.iinfo(np.int64).min
    return k, rng.random(n) >= null_frac


def _pairs_equal(how, order, gl, gr, ol, orr):
    if how in ("semi", "anti"):
        assert np.array_equal(gl, ol)
        return
    assert gl.shape == ol.shape
    if how == "full" and order == "none":
        a, b = np.lexsort((gr, gl)), np.lexsort((orr, ol))
        gl, gr, ol, orr = gl[a], gr[a], ol[b], orr[b]
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)


def _gpu_pairs(out, how):
    """Index columns of the output: the "li" / "ri" payloads, -1 where null."""
    def idx(name):
        s = out[name]
        v = s.to_numpy().astype(np.int64)
        return np.where(s.validity_numpy(), v, -1)

    return idx("li"), (None if how in ("semi", "anti") else idx("ri"))


@pytest.mark.gpu
@pytest.mark.parametrize("nl,nr,card", [(0, 10, 5), (10, 0, 5), (1, 1, 1), (1000, 100, 50), (100, 1000, 50),
                                        (20000, 5000, 3000), (300001, 40000, 100000), (5000, 4000, 7)])
@pytest.mark.parametrize("nulls_equal", [False, True])
@pytest.mark.parametrize("how", HOWS)
def test_join_types_vs_oracle(gpu, nl, nr, card, nulls_equal, how):
    import polaroid_amd as pl

    rng = np.random.default_rng(nl * 7 + nr + card + len(how))
    lk, lv = _rand(rng, nl, card, 0.05)
    rk, rv = _rand(rng, nr, card, 0.05)
    left = pl.DataFrame({"k": pl.Series.from_numpy("k", lk, lv), "li": pl.Series.from_numpy("li", np.arange(nl))})
    right = pl.DataFrame({"k": pl.Series.from_numpy("k", rk, rv), "ri": pl.Series.from_numpy("ri", np.arange(nr))})
    for order in ORDERS:
        ol, orr = O.join(O.HostCol(lk, lv), O.HostCol(rk, rv), how, nulls_equal, order)
        out = left.join(right, on="k", how=how, nulls_equal=nulls_equal, maintain_order=order)
        gl, gr = _gpu_pairs(out, how)
        _pairs_equal(how, order, gl, gr, ol, orr)
        if how in ("left", "right"):
            # the coalesced key is the kept side's key
            kept, keep_idx, kk, kv = (gl, gl, lk, lv) if how == "left" else (gr, gr, rk, rv)
            assert np.array_equal(out["k"].validity_numpy(), kv[keep_idx])


def _mkeys(rng, n, card):
    a = rng.integers(0, card, n).astype(np.int64)
    b = rng.integers(-2, 2, n).astype(np.int32)
    bv = rng.random(n) > 0.1
    f = np.array([0.0, -0.0, np.nan, 2.5])[rng.integers(0, 4, n)]
    return [(a, None), (b, bv), (f, None)]


@pytest.mark.gpu
@pytest.mark.parametrize("nl,nr,card", [(0, 10, 5), (2000, 300, 40), (300, 2000, 40), (100003, 30000, 5000)])
@pytest.mark.parametrize("nkeys", [2, 3])
@pytest.mark.parametrize("nulls_equal", [False, True])
@pytest.mark.parametrize("how", HOWS)
@pytest.mark.parametrize("pack", [True, False])
def test_join_types_multi_vs_oracle(gpu, nl, nr, card, nkeys, nulls_equal, how, pack, plgpu_option):
    """Integer tuples pack into one Int64 key; Float64 keys (nkeys=3) or
    PLGPU_NO_PACK take the hashed path with pair verification (semi / anti
    through a verified left join)."""
    import polaroid_amd as pl

    if not pack:
        plgpu_option("no_pack", 1)
    rng = np.random.default_rng(nl + 3 * nr + card + nkeys + len(how))
    lk, rk = _mkeys(rng, nl, card)[:nkeys], _mkeys(rng, nr, card)[:nkeys]
    names = ["a", "b", "f"][:nkeys]

    def df(keys, idxname):
        n = keys[0][0].shape[0]
        s = [pl.Series.from_numpy(nm, v, m) for nm, (v, m) in zip(names, keys)]
        s.append(pl.Series.from_numpy(idxname, np.arange(n, dtype=np.int64)))
        return pl.DataFrame(s)

    for order in ("none", "left_right", "right_left"):
        ol, orr = O.join_multi(lk, rk, how, nulls_equal, order)
        out = df(lk, "li").join(df(rk, "ri"), on=names, how=how, nulls_equal=nulls_equal, maintain_order=order)
        gl, gr = _gpu_pairs(out, how)
        _pairs_equal(how, order, gl, gr, ol, orr)


@pytest.mark.gpu
@pytest.mark.parametrize("how", HOWS)
def test_join_types_hash_collisions(gpu, how, plgpu_option):
    """A forced 3-bit first tuple hash: every type must detect the false
    matches through pair verification and re-run."""
    import polaroid_amd as pl

    plgpu_option("mk_collide", 1)
    plgpu_option("no_pack", 1)
    rng = np.random.default_rng(9)
    lk, rk = _mkeys(rng, 4000, 30), _mkeys(rng, 600, 30)
    names = ["a", "b", "f"]

    def df(keys, idxname):
        s = [pl.Series.from_numpy(nm, v, m) for nm, (v, m) in zip(names, keys)]
        s.append(pl.Series.from_numpy(idxname, np.arange(keys[0][0].shape[0], dtype=np.int64)))
        return pl.DataFrame(s)

    ol, orr = O.join_multi(lk, rk, how, False, "left_right")
    out = df(lk, "li").join(df(rk, "ri"), on=names, how=how, maintain_order="left_right")
    gl, gr = _gpu_pairs(out, how)
    _pairs_equal(how, "left_right", gl, gr, ol, orr)


@pytest.mark.gpu
def test_join_types_columns_and_coalesce(gpu):
    """Output layout per type: suffixes, dropped / coalesced keys, nullable
    partner columns (validity from the null indices) of every dtype."""
    import polaroid_amd as pl

    rng = np.random.default_rng(4)
    n, m = 3000, 800
    lk = rng.integers(0, 1000, n).astype(np.int32)
    rk = rng.integers(500, 1500, m).astype(np.int32)
    v = rng.standard_normal(n)
    f = rng.random(m) > 0.5
    fv = rng.random(m) > 0.2
    w = rng.standard_normal(m)
    left = pl.DataFrame({"k": pl.Series.from_numpy("k", lk), "v": pl.Series.from_numpy("v", v)})
    right = pl.DataFrame({"k": pl.Series.from_numpy("k", rk), "v": pl.Series.from_numpy("v", w),
                          "f": pl.Series.from_numpy("f", f, fv)})
    out = left.join(right, on="k", how="left", maintain_order="left_right")
    assert out.columns == ["k", "v", "v_right", "f"]
    ol, orr = O.join(O.HostCol(lk.astype(np.int64)), O.HostCol(rk.astype(np.int64)), "left", False, "left_right")
    hit = orr >= 0
    assert np.array_equal(out["v_right"].validity_numpy(), hit)
    assert np.array_equal(out["v_right"].to_numpy()[hit], w[orr[hit]])
    assert np.array_equal(out["f"].validity_numpy(), hit & fv[np.where(hit, orr, 0)])
    fm = out["f"].validity_numpy()
    assert np.array_equal(out["f"].to_numpy()[fm], f[orr[fm]])
    full = left.join(right, on="k", how="full", maintain_order="left_right")
    assert full.columns == ["k", "v", "k_right", "v_right", "f"]
    co = left.join(right, on="k", how="full", coalesce=True, maintain_order="left_right")
    assert co.columns == ["k", "v", "v_right", "f"]
    fl, fr = O.join(O.HostCol(lk.astype(np.int64)), O.HostCol(rk.astype(np.int64)), "full", False, "left_right")
    assert co["k"].to_list() == [int(lk[a]) if a >= 0 else int(rk[b]) for a, b in zip(fl, fr)]
    assert co["k"].dtype == pl.Int32
    right_j = left.join(right, on="k", how="right", maintain_order="right")
    assert right_j.columns == ["v", "k", "v_right", "f"]
    semi = left.join(right, on="k", how="semi")
    assert semi.columns == ["k", "v"]
    with pytest.raises(pl.InvalidOperationError):
        left.join(right, on="k", how="cross")
