"""BASELINE configs[2] and configs[3] at their stated size (1e9 rows), with
size-independent properties checked on the device (torch):

  configs[3]  1e9-row probe x 1e7-row build hash inner join, i64 key:
              the matched probe rows are exactly the rows whose key is a
              build key (each once, build keys unique), every pair joins equal
              keys, payloads travel with their rows;
  configs[2]  1e9 rows x 8 columns (4 i64 + 4 f64) sorted by a 40-bit
              timestamp: keys non-decreasing, the row permutation is a
              permutation, stable (equal keys keep row order), and every column
              moved with its row;
              rolling_mean(20) / rolling_sum(20) over the sorted f64 column: every one of the 1e9
              outputs bit-exact against an exact fixed-point window sum computed
              with torch integer prefix sums (prices in [100, 150) are exact
              multiples of 2^-46, so 20-value window sums fit int64).
"""
import pytest

import polaroid_amd as pl

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N_ROWS = 1_000_000_000


def _gen():
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(20261016)
    return torch, g


def test_configs3_join_1e9_x_1e7(gpu):
    torch, g = _gen()
    n, m = N_ROWS, 10_000_000
    pk = torch.randint(0, 2 * m, (n,), device="cuda", generator=g, dtype=torch.int64)
    bk = torch.randperm(2 * m, device="cuda", generator=g)[:m].to(torch.int64)
    left = pl.DataFrame([pl.Series.from_torch("k", pk),
                         pl.Series.from_torch("a", torch.arange(n, device="cuda", dtype=torch.int64))])
    right = pl.DataFrame([pl.Series.from_torch("k", bk),
                          pl.Series.from_torch("b", torch.arange(m, device="cuda", dtype=torch.int64))])
    out = left.join(right, on="k")
    member = torch.zeros(2 * m, dtype=torch.bool, device="cuda")
    member[bk] = True
    hit = member[pk]
    assert out.height == int(hit.sum().item())
    a, b, k = out["a"].to_torch(), out["b"].to_torch(), out["k"].to_torch()
    assert torch.equal(pk[a], k) and torch.equal(bk[b], k)
    # each matching probe row exactly once
    assert torch.equal(torch.sort(a).values, torch.nonzero(hit).flatten())
    del a, b, k, out, left, right, member, hit, pk, bk
    torch.cuda.empty_cache()


def test_configs2_sort_8_columns_and_rolling_mean_1e9(gpu):
    torch, g = _gen()
    n = N_ROWS
    ts = torch.randint(0, 1 << 40, (n,), device="cuda", generator=g, dtype=torch.int64)
    ts[::1000] = 12345  # a run of equal keys: stability is observable
    r = torch.arange(n, device="cuda", dtype=torch.int64)
    cols = {"ts": ts, "r": r, "i2": r * 7 + 3, "i3": r ^ 0x5555, "price": None, "f1": None, "f2": None, "f3": None}
    price = 100 + torch.rand(n, device="cuda", generator=g, dtype=torch.float64) * 50
    cols["price"] = price
    cols["f1"] = r.to(torch.float64) * 0.5
    cols["f2"] = -r.to(torch.float64)
    cols["f3"] = price * 2
    df = pl.DataFrame([pl.Series.from_torch(k, v) for k, v in cols.items()])
    srt = df.sort("ts")
    sts, sr = srt["ts"].to_torch(), srt["r"].to_torch()
    assert bool((sts[1:] >= sts[:-1]).all())
    assert torch.equal(ts[sr], sts)
    same = sts[1:] == sts[:-1]
    assert bool((sr[1:][same] > sr[:-1][same]).all())  # stable
    assert torch.equal(torch.sort(sr).values, r)  # a permutation
    del sts, same
    assert torch.equal(srt["i2"].to_torch(), sr * 7 + 3)
    assert torch.equal(srt["i3"].to_torch(), sr ^ 0x5555)
    assert torch.equal(srt["f1"].to_torch(), sr.to(torch.float64) * 0.5)
    assert torch.equal(srt["f2"].to_torch(), -sr.to(torch.float64))
    sp = srt["price"].to_torch()
    assert torch.equal(sp, price[sr])
    assert torch.equal(srt["f3"].to_torch(), sp * 2)
    del sr, srt, df, cols, r, ts, price
    torch.cuda.empty_cache()

    w = 20
    got = pl.Series.from_torch("p", sp).rolling_mean(w)
    gv = got.to_torch()
    assert int(got.null_count()) == w - 1
    # exact window sums: every price in [100, 150) is a multiple of 2^-46
    q = (sp * 2.0 ** 46).to(torch.int64)
    assert torch.equal(q.to(torch.float64) * 2.0 ** -46, sp)
    cs = torch.cumsum(q, 0)
    ws = cs[w - 1:].clone()
    ws[1:] -= cs[:-w]
    exact_sum = ws.to(torch.float64) * 2.0 ** -46  # int64 -> f64 rounds once; the scaling is exact
    # (tensor / tensor: torch turns division by a Python scalar into a
    # multiplication by its reciprocal, which is not the IEEE quotient)
    exact = exact_sum / torch.full_like(exact_sum, float(w))
    assert torch.equal(gv[w - 1:], exact)
    del gv, got, exact
    gs = pl.Series.from_torch("p", sp).rolling_sum(w).to_torch()
    assert torch.equal(gs[w - 1:], exact_sum)
