"""CPU validation of the 3-D block schedule of the LDS multi-step passes (S-deep ghosts on every split axis).

Each rank's pass runs in tools/tb_emulate.py (the host mirror of k_leapfrog_tb, every global access bounds-checked,
positions outside the stage-real / allocated ranges reading the layout's zero slot), with the stage-real ranges the
GPU solver passes; between passes the ghosts move exactly as the native plan (make_deep_plan: faces, edges and corners
straight to each of up to 26 neighbours, u^{n+S} then u^{n+S-1} per message) says. The decomposed result must equal the
single-rank CPU leapfrog bit for bit — the property the GPU tests check on hardware.
"""
import math
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import tb_emulate  # noqa: E402

from mpi_cuda_amd.ops import stencil as ops  # noqa: E402


def _global_to_local(C, lay, g):
    """Flat padded local field from a global (N+1)^3 grid: owned nodes and every ghost inside the domain."""
    out = np.zeros(int(lay.total))
    N = g.shape[0] - 1
    xg, yg, zg = int(lay.xg), int(lay.yg), int(lay.zg)
    nx, ny, nz = int(lay.nx), int(lay.ny), int(lay.nz)
    gx0, gy0, gz0 = int(lay.gx0), int(lay.gy0), int(lay.gz0)
    P, R, zs = int(lay.plane), int(lay.pitch), int(lay.zs)
    for x in range(-xg, nx + xg):
        for y in range(-yg, ny + yg):
            gx, gy = gx0 + x, gy0 + y
            if not (0 <= gx <= N and 0 <= gy <= N):
                continue
            z0, z1 = max(-zg, -gz0), min(nz + zg, N + 1 - gz0)
            base = (x + xg) * P + (y + yg) * R + zg + zs
            out[base + z0: base + z1] = g[gx, gy, gz0 + z0: gz0 + z1]
    return out


def _local_owned(lay, f):
    nx, ny, nz = int(lay.nx), int(lay.ny), int(lay.nz)
    xg, yg, zg, P, R, zs = int(lay.xg), int(lay.yg), int(lay.zg), int(lay.plane), int(lay.pitch), int(lay.zs)
    rows = f.reshape(nx + 2 * xg, ny + 2 * yg, R)
    return rows[xg:xg + nx, yg:yg + ny, zg + zs: zg + zs + nz]


def _box(f, lay, b):
    xg, yg, zg, R, zs = int(lay.xg), int(lay.yg), int(lay.zg), int(lay.pitch), int(lay.zs)
    rows = f.reshape(-1, int(lay.ny) + 2 * yg, R)
    x0, x1, y0, y1, z0, z1 = b.as_tuple()
    return rows[x0 + xg:x1 + xg, y0 + yg:y1 + yg, z0 + zg + zs:z1 + zg + zs]


@pytest.mark.parametrize("dims,S,s2,xlen", [((2, 2, 1), 3, 2, None), ((2, 2, 2), 4, 3, None), ((1, 2, 2), 3, 3, 7),
                                            ((3, 2, 1), 2, 2, 5), ((2, 1, 2), 4, 4, None)])
def test_block_passes_match_single_rank(C, dims, S, s2, xlen):
    N = 36
    prob = C.Problem(N, 1e-3 * 40 / N, 20, 1.0)
    co = C.Coeffs.from_problem(prob)
    # global reference: random interior fields, S + s2 single CPU steps
    gl = C.make_layout(prob, C.rank_box(prob, C.Dims(1, 1, 1), 0))
    rng = np.random.default_rng(sum(dims) * 10 + S)
    g_prev = np.zeros((N + 1,) * 3)
    g_cur = np.zeros((N + 1,) * 3)
    g_prev[1:-1, 1:-1, 1:-1] = rng.standard_normal((N - 1,) * 3)
    g_cur[1:-1, 1:-1, 1:-1] = rng.standard_normal((N - 1,) * 3)
    s = ops.sin_table_ext(prob)
    box = C.compute_box(gl)
    a = ops.from_grid(gl, torch.from_numpy(np.pad(g_prev, 1)))
    b = ops.from_grid(gl, torch.from_numpy(np.pad(g_cur, 1)))
    levels = []
    for _ in range(S + s2):
        ops.leapfrog(gl, co, b, a, [box], s)
        a, b = b, a
        levels.append(ops.to_grid(gl, b).numpy()[1:-1, 1:-1, 1:-1].copy())

    D = C.Dims(*dims)
    world = D.size()
    ranks = []
    for r in range(world):
        rb = C.rank_box(prob, D, r)
        g = [S if dims[a_] > 1 else 1 for a_ in range(3)]
        lay = C.make_layout(prob, rb, 16, *g)
        full = C.compute_box(lay)
        nb = [[C.neighbor_rank(D, r, a_, side) >= 0 for side in (0, 1)] for a_ in range(3)]
        lo = [full.x0, full.y0, full.z0]
        hi = [full.x1, full.y1, full.z1]
        real = []
        for a_ in range(3):
            real += [lo[a_] - (S - 1 if nb[a_][0] else 0), hi[a_] + (S - 1 if nb[a_][1] else 0)]
        ranks.append(dict(lay=lay, box=rb, full=full, real=tuple(real),
                          prev=_global_to_local(C, lay, g_prev), cur=_global_to_local(C, lay, g_cur)))

    def run_pass(rk, steps, prev, cur):
        o1, o2 = np.zeros(int(rk["lay"].total)), np.zeros(int(rk["lay"].total))
        tb_emulate.run_pass(rk["lay"], co, prev, cur, o1, o2, rk["full"], s.numpy(), steps, rk["real"], xlen=xlen)
        return o1, o2

    outs = [run_pass(rk, S, rk["prev"], rk["cur"]) for rk in ranks]
    for r, rk in enumerate(ranks):  # first pass: owned nodes of u^{n+S-1}, u^{n+S}
        x0, y0, z0 = int(rk["lay"].gx0), int(rk["lay"].gy0), int(rk["lay"].gz0)
        nx, ny, nz = int(rk["lay"].nx), int(rk["lay"].ny), int(rk["lay"].nz)
        for lev, f in ((S - 2, outs[r][0]), (S - 1, outs[r][1])):
            assert np.array_equal(_local_owned(rk["lay"], f), levels[lev][x0:x0 + nx, y0:y0 + ny, z0:z0 + nz])
    # exchange for a pass of s2 steps, following the native plan on both ends of every message
    plans = [C.make_deep_plan(rk["lay"], D, r, s2) for r, rk in enumerate(ranks)]
    recv = [(outs[r][0].copy(), outs[r][1].copy()) for r in range(world)]
    for r, rk in enumerate(ranks):
        for msg in plans[r].peers:
            q = msg.peer
            back = [m for m in plans[q].peers if m.peer == r]
            assert len(back) == 1 and back[0].count == msg.count
            assert tuple(back[0].dir) == tuple(-d for d in msg.dir)
            for mine, theirs in zip(msg.parts, back[0].parts):
                assert mine.field == theirs.field and mine.off == theirs.off
                src = outs[q][1] if theirs.field == 0 else outs[q][0]
                dst = recv[r][1] if mine.field == 0 else recv[r][0]
                _box(dst, rk["lay"], mine.recv)[...] = _box(src, ranks[q]["lay"], theirs.send)
    for r, rk in enumerate(ranks):
        o1, o2 = run_pass(rk, s2, recv[r][0], recv[r][1])
        x0, y0, z0 = int(rk["lay"].gx0), int(rk["lay"].gy0), int(rk["lay"].gz0)
        nx, ny, nz = int(rk["lay"].nx), int(rk["lay"].ny), int(rk["lay"].nz)
        for lev, f in ((S + s2 - 2, o1), (S + s2 - 1, o2)):
            assert np.array_equal(_local_owned(rk["lay"], f), levels[lev][x0:x0 + nx, y0:y0 + ny, z0:z0 + nz]), r


def test_deep_plan_covers_every_ghost(C):
    """Per rank, the receive regions of the plan tile the whole s-deep ghost shell towards existing neighbours (no
    double writes, no holes), and every send region lies inside the owned box."""
    prob = C.Problem(40, 1e-3, 20, 1.0)
    D = C.Dims(3, 2, 2)
    for s in (2, 4):
        for r in range(D.size()):
            lay = C.make_layout(prob, C.rank_box(prob, D, r), 16, 4, 4, 4)
            n = (int(lay.nx), int(lay.ny), int(lay.nz))
            mark = {0: np.zeros(tuple(v + 2 * s for v in n), dtype=int), 1: np.zeros(tuple(v + 2 * s for v in n), dtype=int)}
            for msg in C.make_deep_plan(lay, D, r, s).peers:
                for part in msg.parts:
                    x0, x1, y0, y1, z0, z1 = part.recv.as_tuple()
                    mark[part.field][x0 + s:x1 + s, y0 + s:y1 + s, z0 + s:z1 + s] += 1
                    sx0, sx1, sy0, sy1, sz0, sz1 = part.send.as_tuple()
                    assert 0 <= sx0 < sx1 <= n[0] and 0 <= sy0 < sy1 <= n[1] and 0 <= sz0 < sz1 <= n[2]
            for f, w in ((0, s), (1, s - 1)):
                m = mark[f]
                assert m.max() <= 1
                # expected: every node within w of the box along each axis that has a neighbour on that side
                c = C.rank_coords(D, r)
                lim = (D.px, D.py, D.pz)
                exp = np.zeros_like(m)
                rng = []
                for a in range(3):
                    lo = -w if c[a] > 0 else 0
                    hi = n[a] + w if c[a] < lim[a] - 1 else n[a]
                    rng.append(slice(lo + s, hi + s))
                exp[tuple(rng)] = 1
                exp[s:s + n[0], s:s + n[1], s:s + n[2]] = 0
                assert np.array_equal(m, exp), (s, r, f)
