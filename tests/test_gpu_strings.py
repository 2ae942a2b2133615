"""String columns (Arrow large_string in HBM): upload / download and Arrow
interchange, filter and gather of string payloads, and string keys in
group-by and every join type.  Checked against the oracle with the strings
replaced by dense ids (equality is all the reference's hash paths look at:
polars-core/src/chunked_array/ops/row_encode.rs encodes the bytes), and the
output strings against the original strings of the rows the oracle names.
Bar: exact strings, exact index sequences / aggregates."""

import numpy as np
import pytest

import polaroid_amd as pl
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _words(rng, n, card, null_frac=0.05, long_frac=0.0, short=False):
    """`short`: every string <= 7 bytes (the exact integer-code path);
    otherwise some keys are longer (the hashed path with byte checks)."""
    if short:
        pool = ["", "a", "AAPL", "MSFT", "BRK.B", "é", "日本", "\x00"] + [f"s{i:05d}" for i in range(card)]
    else:
        pool = ["", "a", "AAPL", "MSFT", "BRK.B", "é", "日本", "x" * 9, "y" * 17] + [f"sym{i:05d}" for i in range(card)]
    pool = pool[: max(card, 1)] if not short else pool[: max(card, 8)]
    idx = rng.integers(0, len(pool), n)
    vals = np.array([pool[i] for i in idx], dtype=object)
    if long_frac:
        for i in np.nonzero(rng.random(n) < long_frac)[0]:
            vals[i] = ("long-" + pool[idx[i]]) * 40  # > 256 bytes: the wave copy path
    valid = rng.random(n) >= null_frac
    return vals, valid


def _ids(*arrays_valid):
    """Dense ids of the strings over all arrays (shared dictionary)."""
    allv = np.concatenate([v for v, _ in arrays_valid]) if arrays_valid else np.zeros(0, object)
    uniq = {s: i for i, s in enumerate(sorted(set(allv.tolist())))}
    return [np.array([uniq[s] for s in v], dtype=np.int64) for v, _ in arrays_valid]


def test_string_roundtrip_and_arrow(gpu):
    import pyarrow as pa

    vals = ["AAPL", None, "", "日本語", "x" * 300, "a\x00b"]
    s = pl.Series("s", vals)
    assert s.dtype == pl.String and s.len() == 6
    assert s.to_list() == vals
    assert s.slice(1, 4).to_list() == vals[1:5]
    arr = pa.array(vals, type=pa.string())
    for a in (arr, arr.cast(pa.large_string()), arr.slice(2, 3)):
        t = pl.Series.from_arrow("t", a)
        assert t.to_list() == a.to_pylist()
        back = t.to_arrow()
        assert back.type == pa.large_string() and back.to_pylist() == a.to_pylist()
    df = pl.DataFrame.from_arrow(pa.table({"k": arr, "v": pa.array(np.arange(6, dtype=np.int64))}))
    assert df["k"].to_list() == vals


@pytest.mark.parametrize("n", [0, 1, 5000, 300_001])
def test_filter_and_gather_strings(gpu, n):
    rng = np.random.default_rng(n)
    w, wv = _words(rng, n, 50, long_frac=0.01)
    x = rng.standard_normal(n)
    df = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "x": pl.Series.from_numpy("x", x)})
    out = df.filter(pl.col("x") > 0.3)
    sel = x > 0.3
    assert out["w"].to_list() == [s if ok else None for s, ok in zip(w[sel], wv[sel])]
    # sort materialises every column by a gather
    srt = df.sort("x")
    order = np.argsort(x, kind="stable")
    assert srt["w"].to_list() == [s if ok else None for s, ok in zip(w[order], wv[order])]


@pytest.mark.parametrize("n,card", [(1, 1), (1000, 7), (200_003, 60), (300_001, 5000)])
@pytest.mark.parametrize("maintain_order", [False, True])
@pytest.mark.parametrize("short", [False, True])
def test_group_by_string_key(gpu, n, card, maintain_order, short):
    rng = np.random.default_rng(n + card)
    w, wv = _words(rng, n, card, short=short)
    v = rng.standard_normal(n)
    df = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "v": pl.Series.from_numpy("v", v)})
    out = df.group_by("w", maintain_order=maintain_order).agg(pl.col("v").sum(), pl.col("v").first().alias("f"),
                                                              pl.len())
    (ids,) = _ids((w, wv))
    okeys, outs = O.group_by_agg_multi([(ids, wv)], [O.HostCol(v)], None, [("sum", 0), ("first", 0), ("len", 0)], n)
    kid, kval = okeys[0]
    names = {}
    for i, ok in zip(kid.tolist(), kval.tolist()):
        names[len(names)] = None if not ok else w[np.nonzero(ids == i)[0][0]]
    exp_keys = [names[g] for g in range(len(names))]
    got_keys = out["w"].to_list()
    assert out["w"].dtype == pl.String
    if maintain_order:
        assert got_keys == exp_keys
        order = list(range(len(exp_keys)))
    else:
        assert sorted(got_keys, key=lambda s: (s is None, s or "")) == sorted(exp_keys, key=lambda s: (s is None, s or ""))
        pos = {k: i for i, k in enumerate(got_keys)}
        order = [pos[k] for k in exp_keys]
    for nm, (vals, valid) in zip(["v", "f", "len"], outs):
        g = out[nm].to_numpy()[order]
        assert np.array_equal(out[nm].validity_numpy()[order], valid), nm
        if vals.dtype == np.float64:
            assert np.array_equal(g[valid].view(np.uint64), vals[valid].view(np.uint64)), nm
        else:
            assert np.array_equal(g[valid].astype(np.int64), vals[valid].astype(np.int64)), nm


@pytest.mark.parametrize("how", ["inner", "left", "right", "full", "semi", "anti"])
@pytest.mark.parametrize("nl,nr,card", [(0, 10, 5), (2000, 300, 40), (100_003, 20_000, 3000)])
@pytest.mark.parametrize("nulls_equal", [False, True])
@pytest.mark.parametrize("short", [False, True])
def test_join_string_key(gpu, how, nl, nr, card, nulls_equal, short):
    rng = np.random.default_rng(nl + nr + card + len(how))
    lw, lv = _words(rng, nl, card, short=short)
    rw, rv = _words(rng, nr, card, long_frac=0.0 if short else 0.02, short=short)
    lid, rid = _ids((lw, lv), (rw, rv))
    left = pl.DataFrame({"k": pl.Series.from_numpy("k", lw, lv), "li": pl.Series.from_numpy("li", np.arange(nl))})
    right = pl.DataFrame({"k": pl.Series.from_numpy("k", rw, rv), "ri": pl.Series.from_numpy("ri", np.arange(nr)),
                          "p": pl.Series.from_numpy("p", rw, rv)})
    for order in ("none", "left_right", "right_left"):
        ol, orr = O.join(O.HostCol(lid, lv), O.HostCol(rid, rv), how, nulls_equal, order)
        out = left.join(right, on="k", how=how, nulls_equal=nulls_equal, maintain_order=order)

        def idx(name):
            s = out[name]
            return np.where(s.validity_numpy(), s.to_numpy().astype(np.int64), -1)

        gl = idx("li")
        if how in ("semi", "anti"):
            assert np.array_equal(gl, ol)
            assert out["k"].to_list() == [lw[i] if lv[i] else None for i in ol]
            continue
        gr = idx("ri")
        if order == "none" and how in ("inner", "full"):  # unspecified order: multisets
            a, b = np.lexsort((gr, gl)), np.lexsort((orr, ol))
            gl, gr, ol, orr, perm = gl[a], gr[a], ol[b], orr[b], a
        else:
            perm = np.arange(gl.size)
        assert np.array_equal(gl, ol) and np.array_equal(gr, orr)
        # the right payload strings follow the right index (null where none)
        p = np.array(out["p"].to_list(), dtype=object)[perm]
        assert p.tolist() == [rw[j] if j >= 0 and rv[j] else None for j in orr]


def test_multi_key_with_string(gpu, plgpu_option):
    rng = np.random.default_rng(5)
    n, m = 50_000, 8000
    lw, lv = _words(rng, n, 30)
    rw, rv = _words(rng, m, 30)
    sw, sv = _words(rng, n, 30, short=True)  # a short-string key next to an integer key
    sa = rng.integers(0, 5, n)
    (sid,) = _ids((sw, sv))
    sdf = pl.DataFrame({"w": pl.Series.from_numpy("w", sw, sv), "a": pl.Series.from_numpy("a", sa)})
    sg = sdf.group_by("w", "a", maintain_order=True).agg(pl.len())
    okeys, outs = O.group_by_agg_multi([(sid, sv), (sa, None)], [O.HostCol(sa)], None, [("len", 0)], n)
    first = {}
    for r, (i, ok) in enumerate(zip(sid.tolist(), sv.tolist())):
        first.setdefault((i if ok else None), sw[r] if ok else None)
    assert sg["w"].to_list() == [first[i if ok else None] for i, ok in zip(okeys[0][0].tolist(), okeys[0][1].tolist())]
    assert np.array_equal(sg["len"].to_numpy(), outs[0][0])
    la, ra = rng.integers(0, 5, n), rng.integers(0, 5, m)
    lid, rid = _ids((lw, lv), (rw, rv))
    left = pl.DataFrame({"w": pl.Series.from_numpy("w", lw, lv), "a": pl.Series.from_numpy("a", la),
                         "li": pl.Series.from_numpy("li", np.arange(n))})
    right = pl.DataFrame({"w": pl.Series.from_numpy("w", rw, rv), "a": pl.Series.from_numpy("a", ra),
                          "ri": pl.Series.from_numpy("ri", np.arange(m))})
    out = left.join(right, on=["w", "a"], how="left", maintain_order="left_right")
    ol, orr = O.join_multi([(lid, lv), (la, None)], [(rid, rv), (ra, None)], "left", False, "left_right")
    ri = out["ri"]
    assert np.array_equal(out["li"].to_numpy(), ol)
    assert np.array_equal(np.where(ri.validity_numpy(), ri.to_numpy(), -1), orr)
    g = left.group_by("w", "a", maintain_order=True).agg(pl.len())
    okeys, outs = O.group_by_agg_multi([(lid, lv), (la, None)], [O.HostCol(la)], None, [("len", 0)], n)
    assert np.array_equal(g["a"].to_numpy(), okeys[1][0])
    assert np.array_equal(g["len"].to_numpy(), outs[0][0])
    # collisions forced: byte-exact verification must catch them
    plgpu_option("mk_collide", 1)
    g2 = left.group_by("w", "a", maintain_order=True).agg(pl.len())
    assert g2["w"].to_list() == g["w"].to_list() and np.array_equal(g2["len"].to_numpy(), g["len"].to_numpy())
    out2 = left.join(right, on=["w", "a"], how="left", maintain_order="left_right")
    assert np.array_equal(out2["li"].to_numpy(), ol)


def test_string_errors(gpu):
    df = pl.DataFrame({"w": pl.Series("w", ["a", "b"]), "v": pl.Series("v", [1.0, 2.0])})
    with pytest.raises(pl.PolaroidError):
        df.group_by("v").agg(pl.col("w").sum())
    with pytest.raises(pl.PolaroidError):
        df.filter(pl.col("w") > 1)


@pytest.mark.parametrize("n", [0, 1, 3000, 200_003])
@pytest.mark.parametrize("descending", [False, True])
@pytest.mark.parametrize("nulls_last", [False, True])
def test_sort_by_string(gpu, n, descending, nulls_last):
    """Byte-wise (UTF-8) order as the reference's string sort; a proper
    prefix first; ties and nulls keep row order (stable)."""
    rng = np.random.default_rng(n + 2 * descending + nulls_last)
    w, wv = _words(rng, n, 300, long_frac=0.01)
    extra = np.array(["ab", "ab\x00", "abc", "a", "", "b" * 20, "b" * 19 + "a", "日", "z"], dtype=object)
    w[: min(n, extra.size)] = extra[: min(n, extra.size)]
    df = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "i": pl.Series.from_numpy("i", np.arange(n))})
    out = df.sort("w", descending=descending, nulls_last=nulls_last)
    valid_rows = [i for i in range(n) if wv[i]]
    null_rows = [i for i in range(n) if not wv[i]]
    ordered = sorted(valid_rows, key=lambda i: w[i].encode(), reverse=descending)
    exp = ordered + null_rows if nulls_last else null_rows + ordered
    assert out["i"].to_list() == exp
    # two keys: string then integer
    a = rng.integers(0, 3, n)
    df2 = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "a": pl.Series.from_numpy("a", a),
                        "i": pl.Series.from_numpy("i", np.arange(n))})
    out2 = df2.sort("w", "a")
    # nulls of `w` compare equal to each other, so `a` orders them too
    key = lambda i: (0, b"", int(a[i])) if not wv[i] else (1, w[i].encode(), int(a[i]))  # noqa: E731
    assert out2["i"].to_list() == sorted(range(n), key=key)


def _cmp(x, y, op):
    if x is None or y is None:
        return None
    a, b = x.encode(), y.encode()
    return {"==": a == b, "!=": a != b, "<": a < b, "<=": a <= b, ">": a > b, ">=": a >= b}[op]


@pytest.mark.parametrize("n", [0, 1, 4000, 100_003])
def test_string_predicates(gpu, n):
    """String comparisons (view.rs TotalEqKernel / TotalOrdKernel semantics:
    byte order, null in -> null out, *_missing never null) in filter,
    select and the group-by's fused predicate."""
    rng = np.random.default_rng(n)
    w, wv = _words(rng, n, 40, long_frac=0.01)
    u, uv = _words(rng, n, 40, short=True)
    x = rng.standard_normal(n)
    wl = [s if ok else None for s, ok in zip(w, wv)]
    ul = [s if ok else None for s, ok in zip(u, uv)]
    df = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "u": pl.Series.from_numpy("u", u, uv),
                       "x": pl.Series.from_numpy("x", x), "i": pl.Series.from_numpy("i", np.arange(n))})
    for op in ("==", "!=", "<", "<=", ">", ">="):
        for litv in ("AAPL", "", "sym00017", "z"):
            e = {"==": pl.col("w") == litv, "!=": pl.col("w") != litv, "<": pl.col("w") < litv,
                 "<=": pl.col("w") <= litv, ">": pl.col("w") > litv, ">=": pl.col("w") >= litv}[op]
            got = df.select(e.alias("m"))["m"].to_list()
            assert got == [_cmp(s, litv, op) for s in wl], (op, litv)
        # column vs column, and the literal on the left (mirrored)
        e2 = {"==": pl.col("w") == pl.col("u"), "!=": pl.col("w") != pl.col("u"), "<": pl.col("w") < pl.col("u"),
              "<=": pl.col("w") <= pl.col("u"), ">": pl.col("w") > pl.col("u"),
              ">=": pl.col("w") >= pl.col("u")}[op]
        assert df.select(e2.alias("m"))["m"].to_list() == [_cmp(a, b, op) for a, b in zip(wl, ul)], op
    left = df.select((pl.lit("MSFT") < pl.col("w")).alias("m"))["m"].to_list()
    assert left == [_cmp(s, "MSFT", ">") for s in wl]
    em = df.select(pl.col("w").eq_missing(pl.col("u")).alias("m"))["m"].to_list()
    assert em == [(a == b) if (a is not None and b is not None) else (a is None and b is None) for a, b in zip(wl, ul)]
    assert df.select(pl.col("w").is_null().alias("m"))["m"].to_list() == [s is None for s in wl]
    # filter: string predicate combined with a numeric one (Kleene and)
    out = df.filter((pl.col("w") == "AAPL") & (pl.col("x") > 0.0))
    keep = [i for i in range(n) if wl[i] == "AAPL" and x[i] > 0.0]
    assert out["i"].to_list() == keep and out["w"].to_list() == [wl[i] for i in keep]
    assert out.columns == ["w", "u", "x", "i"]
    # group-by with the string predicate fused into the aggregation
    g = df.lazy().filter(pl.col("u") != "AAPL").group_by("w", maintain_order=True).agg(pl.col("x").sum()).collect()
    sel = [i for i in range(n) if ul[i] is not None and ul[i] != "AAPL"]
    keys = []
    for i in sel:
        if wl[i] not in keys:
            keys.append(wl[i])
    assert g["w"].to_list() == keys
    for k, v in zip(keys, g["x"].to_list()):
        assert v == O.fsum(np.array([x[i] for i in sel if wl[i] == k]))


def test_dictionary_columns_from_arrow(gpu):
    """polars Categorical / Enum columns arrive as Arrow dictionary arrays:
    the dictionary and indices are uploaded and the strings gathered on the
    GPU (a null index gives a null); they then group / join / filter as
    String columns."""
    import pyarrow as pa

    vals = ["AAPL", "MSFT", None, "AAPL", "BRK.B", "MSFT", "AAPL", None]
    darr = pa.array(vals).dictionary_encode()
    for a in (darr, darr.slice(1, 6), pa.chunked_array([darr.slice(0, 3), darr.slice(3)])):
        s = pl.Series.from_arrow("sym", a)
        assert s.dtype == pl.String and s.to_list() == a.to_pylist()
    t = pa.table({"sym": darr, "v": pa.array(np.arange(8, dtype=np.float64))})
    df = pl.DataFrame.from_arrow(t)
    g = df.group_by("sym", maintain_order=True).agg(pl.col("v").sum())
    assert g["sym"].to_list() == ["AAPL", "MSFT", None, "BRK.B"]
    assert g["v"].to_list() == [0.0 + 3 + 6, 1.0 + 5, 2.0 + 7, 4.0]
    f = df.filter(pl.col("sym") == "MSFT")
    assert f["v"].to_list() == [1.0, 5.0]


def test_string_pattern_predicates(gpu):
    """str.starts_with / ends_with / contains(literal): byte-wise tests, a
    null string gives null (binary/namespace.rs starts_with / ends_with,
    strings/namespace.rs contains_literal)."""
    rng = np.random.default_rng(12)
    n = 50_000
    w, wv = _words(rng, n, 60, long_frac=0.01)
    wl = [s if ok else None for s, ok in zip(w, wv)]
    df = pl.DataFrame({"w": pl.Series.from_numpy("w", w, wv), "i": pl.Series.from_numpy("i", np.arange(n))})
    for pat in ("", "s", "sym0001", "AAPL", "日", "long-", "9", "x" * 9, "zz"):
        for fn, ref in (("starts_with", str.startswith), ("ends_with", str.endswith),
                        ("contains", lambda s, p: p in s)):
            e = getattr(pl.col("w").str, fn)(pat) if fn != "contains" else pl.col("w").str.contains(pat, literal=True)
            got = df.select(e.alias("m"))["m"].to_list()
            assert got == [None if s is None else ref(s, pat) for s in wl], (fn, pat)
    out = df.filter(pl.col("w").str.starts_with("sym000") & (pl.col("i") > 1000))
    assert out["i"].to_list() == [i for i in range(n) if wl[i] is not None and wl[i].startswith("sym000") and i > 1000]
    with pytest.raises(pl.InvalidOperationError, match="regex"):
        df.filter(pl.col("w").str.contains("a.*b"))
