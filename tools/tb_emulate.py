"""Host emulation of k_leapfrog_tb (csrc/src/kernels_leapfrog_tb.hip): same tiling, rings, stage schedule, masks and
global offsets, executed workgroup by workgroup with numpy, with every global and LDS index bounds-checked.

Used by tests/test_tb_emulate.py (CPU) to validate the algorithm and its address arithmetic bit-exactly against the
native CPU leapfrog before the kernel runs on a GPU, where an out-of-range access faults the device.
"""
from __future__ import annotations

import numpy as np

T = 32  # tile edge (kTile)


class Geom:
    def __init__(self, S: int):
        self.S = S

    def halo(self, j):
        return self.S - 1 if j < 0 else self.S - j

    def W(self, j):
        return T + 2 * self.halo(j)


def fma(a, b, c):
    """IEEE a·b + c rounded once (stencil.hpp's fused leapfrog / first step), through the native binding."""
    from mpi_cuda_amd._native import load

    a, b, c = np.broadcast_arrays(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64),
                                  np.asarray(c, dtype=np.float64))
    r = load().fma_array(a.ravel(), b.ravel(), c.ravel())
    return np.asarray(r).reshape(a.shape)


def lap7(c, xm, xp, ym, yp, zm, zp, ihx2, ihy2, ihz2):
    c2 = 2.0 * c  # stencil.hpp::d2sum (h²·Δ_h; the update coefficients carry 1/h²)
    return (xp - c2 + xm) + (yp - c2 + ym) + (zp - c2 + zm)


def run_pass(lay, co, prev: np.ndarray, cur: np.ndarray, out1: np.ndarray, out2: np.ndarray, box, s_ext: np.ndarray,
             S: int, sx, ct=None, check_mask: int = 0, analytic_start: bool = False, xlen: int | None = None):
    """Emulate one launch. Arrays are the flat padded fields (layout.total doubles); s_ext is the extended sin table
    (element g+1 ↔ global g). Returns {k: (max, sumsq)} for checked stages (per-tile partials combined in order).
    analytic_start: u^{n-1} = φ and u^n = u¹ come from the kernel's LDS sin tables (same index math and clamping)
    instead of prev/cur. sx: the stage-real range, (sx0, sx1) or (sx0, sx1, sy0, sy1, sz0, sz1) (y/z default: the whole
    allocation). xlen: x chunk length (the kernel's chunking of small boxes; default: one chunk)."""
    G = Geom(S)
    N = int(lay.N)
    P, R, zs, xg = int(lay.plane), int(lay.pitch), int(lay.zs), int(lay.xg)
    yg, zg = int(getattr(lay, "yg", 1)), int(getattr(lay, "zg", 1))
    nyl, nzl = int(lay.ny), int(lay.nz)
    gx0, gy0, gz0 = int(lay.gx0), int(lay.gy0), int(lay.gz0)
    total = int(lay.total)
    kb = (xg - 1) * P + (yg - 1) * R + (zg - 1)
    zero_off = P - 1  # Layout::zero_off: the plane's last double (row padding), only ever 0
    bx0, bx1, y0, y1, z0, z1 = int(box.x0), int(box.x1), int(box.y0), int(box.y1), int(box.z0), int(box.z1)
    sx = tuple(sx)
    sx0, sx1 = sx[0], sx[1]  # the kernel's default is the rank's compute-box x range
    sy0, sy1, sz0, sz1 = sx[2:6] if len(sx) == 6 else (-yg, nyl + yg, -zg, nzl + zg)
    ax0, ax1 = -xg, int(lay.nx) + xg
    ay0, ay1, az0, az1 = -yg, nyl + yg, -zg, nzl + zg
    ihx2, ihy2, ihz2, tau2 = co.ihx2, co.ihy2, co.ihz2, co.lam  # tau2 here: τ²/h², the coefficient of d2sum
    ct = list(ct) if ct is not None else [0.0] * S

    def inside(g):
        return (g >= 1) & (g <= N - 1)

    def goff(x, y, z):
        # the kernel's split: plane base (x + xg)·P plus a plane-relative offset that must fit its 28 flag-free bits
        inp = (y + yg) * R + (z + zg + zs)
        if np.any(inp < 0) or np.any(inp >= min(P, 1 << 28)):
            raise IndexError(f"in-plane offset out of range at x={x}")
        o = (x + xg) * P + inp
        assert np.all(o == kb + (x + 1) * P + (y + 1) * R + (z + 1 + zs))
        if np.any(o < 0) or np.any(o >= total):
            raise IndexError(f"global offset out of range at x={x}")
        return o

    def zoff(x):  # the zero slot of plane x
        o = (x + xg) * P + zero_off
        if o < 0 or o >= total:
            raise IndexError(f"zero slot out of range at x={x}")
        return o

    def sget(g):
        g = np.asarray(g)
        if np.any(g < -1) or np.any(g > N + 1):
            raise IndexError(f"sin table index out of range: {g.min()}..{g.max()}")
        return s_ext[g + 1]

    nty, ntz = -(-(y1 - y0) // T), -(-(z1 - z0) // T)
    xlen = xlen or max(1, bx1 - bx0)
    chunks = [(c, min(bx1, c + xlen)) for c in range(bx0, bx1, xlen)]
    errs = {k: [0.0, 0.0] for k in range(1, S + 1) if check_mask >> (k - 1) & 1}
    for (x0, x1), tyi, tzi in ((c, a, b) for c in chunks for a in range(nty) for b in range(ntz)):
        i0, i1 = x0 - S + 1, x1 + S - 2
        if True:
            ty0, tz0 = y0 + tyi * T, z0 + tzi * T
            ring = {j: [np.zeros((G.W(j), G.W(j))) for _ in range(1 if j < 0 else 3)] for j in range(-1, S)}
            emax = [0.0] * S
            esum = [0.0] * S

            # the kernel's sin tables: syw[j] ↔ y = ty0 - S - 1 + j, sxw[i] ↔ x = x0 - S - 1 + i, clamped to -1..N+1
            W0 = T + 2 * S
            nyw = T + 2 * S + 2

            def sc(g):
                return s_ext[np.clip(g, -1, N + 1) + 1]

            syw = sc(gy0 + ty0 - S - 1 + np.arange(nyw))
            szw = sc(gz0 + tz0 - S - 1 + np.arange(nyw))
            sxw = sc(gx0 + x0 - S - 1 + np.arange(x1 - x0 + 2 * S + 4))
            xtab0 = S + 1 - x0

            def tables(h, w, x):
                # LDS position (level-0 coordinates) of the level's region → table indices (ytab, ztab)
                a = np.arange(w)
                li_a = a + (S - h)  # level-0 row of region row a
                ya = np.minimum(li_a + 1, W0)[:, None] + 0 * a[None, :]
                zb = (li_a + 1)[None, :] + 0 * a[:, None]
                xi = x + xtab0
                if xi - 1 < 0 or xi + 1 >= len(sxw) or ya.max() + 1 >= nyw or zb.max() + 1 >= nyw:
                    raise IndexError(f"sin table index out of range: x={x} xi={xi} n={len(sxw)} ya={ya.max()} zb={zb.max()} nyw={nyw}")
                return ya, zb, xi

            def fetch(j, src, x):
                h, w = G.halo(j), G.W(j)
                a = np.arange(w)
                y = ty0 - h + a[:, None] + 0 * a[None, :]
                z = tz0 - h + a[None, :] + 0 * a[:, None]
                v = np.zeros((w, w))
                if analytic_start:
                    ya, zb, xi = tables(h, w, x)
                    sxc, sy, sz = sxw[xi], syw[ya], szw[zb]
                    cy = sxc * sy
                    c = cy * sz
                    if j < 0:  # u0 = φ
                        return c
                    lap = lap7(c, (sxw[xi - 1] * sy) * sz, (sxw[xi + 1] * sy) * sz, (sxc * syw[ya - 1]) * sz,
                               (sxc * syw[ya + 1]) * sz, cy * szw[zb - 1], cy * szw[zb + 1], co.ihx2, co.ihy2, co.ihz2)
                    in_a = (y >= ay0) & (y < ay1) & (z >= az0) & (z < az1)
                    real = inside(gy0 + y) & inside(gz0 + z) & (1 <= gx0 + x <= N - 1) & in_a
                    return np.where(real, fma(co.half_lam, lap, c), 0.0)
                if ax0 <= x < ax1 and 1 <= gx0 + x <= N - 1:
                    # loaded wherever the rank holds the node (interior ∩ allocation); elsewhere the zero slot
                    in_a = (y >= ay0) & (y < ay1) & (z >= az0) & (z < az1)
                    m = inside(gy0 + y) & inside(gz0 + z) & in_a
                    v[m] = src[goff(x, y[m], z[m])]
                    if (~m).any():
                        v[~m] = src[zoff(x)]
                return v

            def commit(x):
                ring[0][x % 3] = fetch(0, cur, x)
                if x - 1 >= i0:  # like the kernel, u^{n-1} is only fetched from plane i0 on
                    ring[-1][0] = fetch(-1, prev, x - 1)

            def stage(k, xp):
                hk, wk = G.halo(k), G.W(k)
                di = G.halo(k - 1) - hk
                dd = G.halo(k - 2) - hk
                im, ic, ip = (ring[k - 1][(xp - 1) % 3], ring[k - 1][xp % 3], ring[k - 1][(xp + 1) % 3])
                od = ring[-1][0] if k == 1 else ring[k - 2][xp % 3]
                wi = G.W(k - 1)
                assert wi == wk + 2 * di and di == 1
                sl = slice(di, di + wk)
                c = ic[sl, sl]
                lap = lap7(c, im[sl, sl], ip[sl, sl], ic[di - 1: di - 1 + wk, sl], ic[di + 1: di + 1 + wk, sl],
                           ic[sl, di - 1: di - 1 + wk], ic[sl, di + 1: di + 1 + wk], ihx2, ihy2, ihz2)
                o = od[dd: dd + wk, dd: dd + wk]
                a = np.arange(wk)
                y = ty0 - hk + a[:, None] + 0 * a[None, :]
                z = tz0 - hk + a[None, :] + 0 * a[:, None]
                xreal = sx0 <= xp < sx1 and 1 <= gx0 + xp <= N - 1
                real = xreal & inside(gy0 + y) & inside(gz0 + z) & (y >= sy0) & (y < sy1) & (z >= sz0) & (z < sz1)
                v = np.where(real, fma(tau2, lap, 2.0 * c - o), 0.0)
                if k < S:
                    ring[k][xp % 3] = v
                xown = x0 <= xp < x1
                aa, bb = a[:, None] + 0 * a[None, :], a[None, :] + 0 * a[:, None]
                own = real & xown & (aa >= hk) & (aa < hk + T) & (bb >= hk) & (bb < hk + T) & (y < y1) & (z < z1)
                if k >= S - 1 and own.any():
                    (out2 if k == S else out1)[goff(xp, y[own], z[own])] = v[own]
                if k in errs and own.any():
                    e = np.abs(v[own] - ((sget(gx0 + xp) * sget(gy0 + y[own])) * ct[k - 1]) * sget(gz0 + z[own]))
                    emax[k - 1] = max(emax[k - 1], float(e.max()))
                    esum[k - 1] += float((e * e).sum())

            commit(i0 - 1)
            commit(i0)
            for i in range(i0, i1 + 1):
                commit(i + 1)
                for k in range(1, S + 1):
                    xp = i - (k - 1)
                    if x0 - (S - k) <= xp < x1 + (S - k):
                        stage(k, xp)
            for k in errs:
                errs[k][0] = max(errs[k][0], emax[k - 1])
                errs[k][1] += esum[k - 1]
    return {k: tuple(v) for k, v in errs.items()}
