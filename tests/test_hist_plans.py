"""Histogram launch plans of the scan engine (HipTreeBuilder._plan / _choose),
evaluated on the CPU: the headline 11M-row plans stay one full round of
1024-thread workgroups, strong-scaled shards (11M / 2, 4, 8 rows) spread over
every CU, and grids that overflow a round of resident workgroups are widened
to fill it (profiles/r3/small_shard_ab.txt, fill_rounds_ab.txt)."""
import pytest

from h2omx.models.tree.engine import HipTreeBuilder


def _builder(n, F, small=True, fill=True):
    b = HipTreeBuilder.__new__(HipTreeBuilder)
    b.F, b.nbt, b.max_rows_per_wg = F, 256, None

    class BM:
        npad = -(-n // 64) * 64

    b.bm = BM
    b.SMALL_SHARD, b.FILL_ROUNDS = small, fill
    return b


def _wgs(p):
    return p["n_groups"] * p["wgpg"]


def test_headline_plans_unchanged():
    b = _builder(11_000_000, 28)
    l0 = b._plan(1, b.DEEP_LDS_BUDGET, b.THREADS, mult=8)
    assert (l0["n_groups"], l0["fg"], l0["wgpg"], l0["threads"]) == (4, 7, 64, 1024)
    got = {s: (lambda p: (p["n_groups"], p["wgpg"], p["threads"]))(b._choose(s)) for s in (1, 2, 4, 8)}
    assert got == {1: (1, 256, 1024), 2: (2, 128, 1024), 4: (2, 128, 1024), 8: (4, 64, 1024)}
    ref = _builder(11_000_000, 28, small=False, fill=False)
    for s in (1, 2, 4, 8):
        assert b._choose(s) == ref._choose(s)


@pytest.mark.parametrize("n", [1_375_000, 2_750_000, 5_500_000])
def test_small_shards_fill_every_cu(n):
    b = _builder(n, 28)
    old = _builder(n, 28, small=False)
    for s in (1, 2, 4, 8):
        p = b._choose(s)
        assert _wgs(p) >= HipTreeBuilder.N_CUS or _wgs(p) >= _wgs(old._choose(s))
        assert p["threads"] == 1024 and p["wgpg"] % 8 == 0 and p["fg"] * p["n_groups"] >= 28
    if n == 1_375_000:   # 11M / 8: level 1 went from 40 to 256 workgroups
        assert _wgs(old._choose(1)) == 40 and _wgs(b._choose(1)) == 256


def test_fill_rounds_widens_capped_grids():
    # Airlines-shape 18.75M x 31: the 256K-row chunk cap forces 72 workgroups per group
    b = _builder(18_750_000, 31)
    nofill = _builder(18_750_000, 31, fill=False)
    p0 = nofill._plan(1, b.DEEP_LDS_BUDGET, b.THREADS, mult=8)
    p1 = b._plan(1, b.DEEP_LDS_BUDGET, b.THREADS, mult=8)
    assert _wgs(p0) == 288 and _wgs(p1) == 512
    units = b.bm.npad // b.ROWS_PER_LANE
    # chunks only shrink (the fixed-point scale bound max_rows_per_wg still holds)
    assert -(-units // p1["wgpg"]) <= -(-units // p0["wgpg"])
