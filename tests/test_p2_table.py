"""The pair-tiled pass's compile-time thread table (csrc/include/wave3d/leapfrog_p2_kernel.hpp make_tab), checked on the
CPU against an independent Python statement of what the kernel needs: an out-of-range or missing position would
fault or silently corrupt the GPU pass, so its geometry is pinned here where a mistake costs nothing.

Per thread the table gives a pair (a, b) of the tile's region — rows a ∈ [0, HY), pair columns b ∈ [0, PZ), nodes
z = 2b, 2b+1 — and its wave's role: kind 1 computes stages 1..lv, kind 2 only loads the u^n ring, kind 0 nothing."""
import collections

import pytest

C = pytest.importorskip("mpi_cuda_amd._C")

KT, NT = 32, 1024


def _decode(d):
    return (d & 0xFF) - 2, ((d >> 8) & 0xFF) - 2, (d >> 16) & 0xF, (d >> 20) & 0x3


def _level(S, E, HY, a, b):
    """Deepest stage whose region holds the pair: stage k needs y rows [k−1, HY−k+1) and nodes z within S−k of the
    tile's 32 columns (region column origin E)."""
    lv = 0
    for k in range(1, S + 1):
        row = k - 1 <= a < HY - (k - 1)
        zlo, zhi = E - (S - k), E + KT + (S - k)
        if row and 2 * b + 1 >= zlo and 2 * b < zhi:
            lv = k
    return lv


@pytest.mark.parametrize("S", [2, 3, 4, 5])
def test_p2_table_covers_every_position_once(S):
    tab, geo = C.leapfrog_p2_table(S)
    E, HY, HZ, PZ, tile = geo[:5]
    assert tile == KT and len(tab) == NT
    assert E == (S // 2) * 2 and HY == KT + 2 * (S - 1) and HZ == KT + 2 * E and PZ == HZ // 2
    waves = [[_decode(tab[w * 64 + l]) for l in range(64)] for w in range(16)]
    # waves 0-7: the tile's own 32 x 32 nodes = 512 pairs, every stage, one row per ds_read_b128 lane group
    own = {(S - 1 + r, E // 2 + c) for r in range(KT) for c in range(KT // 2)}
    got = [(a, b) for w in range(8) for a, b, lv, kind in waves[w]]
    assert sorted(got) == sorted(own)
    assert all(lv == S and kind == 1 for w in range(8) for _, _, lv, kind in waves[w])
    # every other region pair exactly once in a kind-1 wave whose stage count covers it (idle lanes repeat the wave's
    # first pair), and nothing outside the region
    region = {(a, b): _level(S, E, HY, a, b) for a in range(HY) for b in range(PZ)}
    need = {p for p, lv in region.items() if 1 <= lv < S}
    seen = collections.Counter()
    for w in range(8, 16):
        kinds = {kind for *_, kind in waves[w]}
        assert len(kinds) == 1  # (a wave's role is uniform)
        if kinds == {1}:
            first = waves[w][0][:2]
            wlv = waves[w][0][2]
            for a, b, lv, _ in waves[w]:
                assert lv == wlv and region.get((a, b), 0) <= wlv
                if (a, b) != first or seen[(a, b)] == 0:
                    seen[(a, b)] += 1
    assert set(seen) == need and all(n == 1 for n in seen.values())
    # the u^n ring (one pair beyond the region on every side, corners excluded) in kind-2 waves, each pair once
    ring = {(-1, b) for b in range(PZ)} | {(HY, b) for b in range(PZ)} | {(a, -1) for a in range(HY)} | \
        {(a, PZ) for a in range(HY)}
    rseen = {(a, b) for w in range(8, 16) for a, b, _, kind in waves[w] if kind == 2}
    assert rseen == ring
    # the stage work per SIMD (wave w on SIMD w mod 4) is balanced to within one wave's stages
    load = [0] * 4
    for w in range(16):
        if waves[w][0][3] == 1:
            load[w % 4] += waves[w][0][2]
    assert max(load) - min(load) <= S


@pytest.mark.parametrize("S", [2, 3, 4, 5])
def test_p2_lds_budget(S):
    """The pass (and for S <= 4 the analytic start) fits gfx950's 160 KiB of LDS with a 512-plane x march, and the
    x chunking never needs to go below 512 planes."""
    _, geo = C.leapfrog_p2_table(S)
    lds, lds_init, maxlen, maxlen_init = geo[5:9]
    assert 0 < lds <= 160 * 1024 and maxlen >= 512
    if S <= 4:
        assert 0 < lds_init <= 160 * 1024 and maxlen_init >= 512


def test_round5_solver_options_exposed():
    """The round-5 options reach Python with their C++ defaults: 5-step passes, the pair-tiled kernel on, no CUs kept
    off the passes, no fake-rank self-traffic."""
    o = C.SolverOptions()
    assert o.temporal == 5 and o.tiling_tb.p2 is True
    assert o.reserve_cus == 0 and o.fake_traffic is False
    o.reserve_cus = 16
    assert o.reserve_cus == 16


@pytest.mark.parametrize("S", [4, 5])
def test_p2_split_store_partners(S):
    """Split stores (leapfrog_p2_kernel.hpp kSplitSt): thread 512 + t of waves 8-15 stores level S-1 of the pair that
    thread t of the own waves 0-7 holds (the kernel reads p2_desc(tid & 511)), so the 8 non-owning waves cover the
    tile's 512 own pairs exactly once, one lane each, and every wave issues one store per plane. The zero-size u^{n-1}
    descriptor goes to the kind-2 (u^n ring) waves, which compute no stage and so never read u^{n-1}."""
    tab, geo = C.leapfrog_p2_table(S)
    E = geo[0]
    own = {(S - 1 + r, E // 2 + c) for r in range(KT) for c in range(KT // 2)}
    partners = [_decode(tab[t & 511])[:2] for t in range(512, 1024)]
    assert sorted(partners) == sorted(own)
    for w in range(16):
        a, b, lv, kind = _decode(tab[w * 64])
        if kind == 2:
            assert lv == 0
