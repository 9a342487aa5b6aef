"""Kernel-level ops on torch tensors: the CDNA4 HIP kernels (GPU) and the native OpenMP kernels (CPU).

Fields are flat float64 tensors in the padded local layout of ``mpi_cuda_amd._C.Layout`` (ghost layer of width 1,
row pitch a multiple of 16 doubles, rows shifted so updated nodes sit in aligned 16-byte pairs). ``to_grid`` /
``from_grid`` convert between that layout and a dense (nx+2, ny+2, nz+2) array including the ghosts.

GPU ops never fall back to PyTorch: if the extension is missing the import fails loudly.
"""
from __future__ import annotations

import torch

from .._native import load


def _C():
    return load()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def alloc_field(layout, device="cpu") -> torch.Tensor:
    return torch.zeros(int(layout.total), dtype=torch.float64, device=device)


def sin_table_ext(problem, device="cpu") -> torch.Tensor:
    return torch.as_tensor(_C().sin_table_ext(problem), dtype=torch.float64, device=device)


def grid_view(layout, u: torch.Tensor) -> torch.Tensor:
    """Dense (nx+2, ny+2, nz+2) view (one ghost layer on every side) of a padded flat field."""
    nx, ny, nz, p, zs = int(layout.nx), int(layout.ny), int(layout.nz), int(layout.pitch), int(layout.zs)
    xg = int(getattr(layout, "xg", 1))
    yg = int(getattr(layout, "yg", 1))
    zg = int(getattr(layout, "zg", 1))
    rows = u.view(nx + 2 * xg, ny + 2 * yg, p)
    return rows[xg - 1: xg + nx + 1, yg - 1: yg + ny + 1, zs + zg - 1: zs + zg + nz + 1]


def to_grid(layout, u: torch.Tensor) -> torch.Tensor:
    return grid_view(layout, u).contiguous()


def from_grid(layout, g: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    if out is None:
        out = alloc_field(layout, device=g.device)
    grid_view(layout, out).copy_(g)
    return out


# ---------------------------------------------------------------------------------------------------------------
# dispatch: CPU tensors -> native OpenMP kernels, CUDA tensors -> HIP kernels
# ---------------------------------------------------------------------------------------------------------------
def init_first(layout, coeffs, s_ext: torch.Tensor, u0: torch.Tensor, u1: torch.Tensor) -> None:
    """u0 = φ, u1 = first step, over the whole local allocation (ghosts included)."""
    C = _C()
    if u0.is_cuda:
        C.gpu_init_first(layout, coeffs, s_ext.data_ptr(), u0.data_ptr(), u1.data_ptr(), _stream())
    else:
        C.cpu_init_first(layout, coeffs, s_ext.numpy(), u0.numpy(), u1.numpy())


def leapfrog(layout, coeffs, cur: torch.Tensor, old: torch.Tensor, boxes, s_ext: torch.Tensor, ct: float = 0.0,
             check: bool = False, tiling=None):
    """One leapfrog step over ``boxes`` (list of LBox), in place over ``old``.

    Returns None, or the (L∞, Σe²) error of the new values vs φ·ct over the boxes if ``check``.
    """
    C = _C()
    if cur.is_cuda:
        t = tiling if tiling is not None else C.LeapfrogTiling()
        nb = C.gpu_leapfrog_blocks(layout, list(boxes), t)
        part = torch.empty((max(nb, 1), 2), dtype=torch.float64, device=cur.device) if check else None
        C.gpu_leapfrog(layout, coeffs, cur.data_ptr(), old.data_ptr(), list(boxes), s_ext.data_ptr(), ct,
                       part.data_ptr() if check else 0, t, _stream())
        if not check:
            return None
        out = torch.empty(2, dtype=torch.float64, device=cur.device)
        C.gpu_reduce(part.data_ptr(), nb, out.data_ptr(), _stream())
        o = out.cpu()
        return float(o[0]), float(o[1])
    acc = None
    for b in boxes:
        r = C.cpu_leapfrog(layout, coeffs, cur.numpy(), old.numpy(), b, s_ext.numpy(), ct, check)
        if check:
            acc = r if acc is None else (max(acc[0], r[0]), acc[1] + r[1])
    return acc


def leapfrog2(layout, coeffs, prev: torch.Tensor, cur: torch.Tensor, out1: torch.Tensor, out2: torch.Tensor, box,
              s_ext: torch.Tensor, ct2: float = 0.0, check: bool = False, tiling=None):
    """Two fused leapfrog steps (HIP only): out1 = u^{n+1}, out2 = u^{n+2} from prev = u^{n-1}, cur = u^n.

    ``box`` must be the whole single-rank interior. Returns the (L∞, Σe²) error of u^{n+2} if ``check``."""
    C = _C()
    if not cur.is_cuda:
        raise ValueError("leapfrog2 is a GPU kernel; on the CPU take two leapfrog() steps")
    t = tiling if tiling is not None else C.Leapfrog2Tiling()
    nb = C.gpu_leapfrog2_partials(layout, box, t)
    part = torch.empty((max(nb, 1), 2), dtype=torch.float64, device=cur.device) if check else None
    C.gpu_leapfrog2(layout, coeffs, prev.data_ptr(), cur.data_ptr(), out1.data_ptr(), out2.data_ptr(), box,
                    s_ext.data_ptr(), ct2, part.data_ptr() if check else 0, t, _stream())
    if not check:
        return None
    out = torch.empty(2, dtype=torch.float64, device=cur.device)
    C.gpu_reduce(part.data_ptr(), nb, out.data_ptr(), _stream())
    o = out.cpu()
    return float(o[0]), float(o[1])


def leapfrog_tb(layout, coeffs, prev: torch.Tensor, cur: torch.Tensor, out1: torch.Tensor, out2: torch.Tensor, box,
                s_ext: torch.Tensor, stages: int = 4, ct=None, check_mask: int = 0, threads: int = 1024,
                analytic_start: bool = False, p2: bool = True, target_blocks: int | None = None):
    """``stages`` fused leapfrog steps held in LDS (HIP only): out1 = u^{n+S-1}, out2 = u^{n+S}.

    ``p2`` selects the pair-tiled kernel (S <= 5) wherever it applies, else k_leapfrog_tb (S <= 4).

    ``ct[k-1]`` is the time factor of u^{n+k}; for every bit k-1 set in ``check_mask`` the (L∞, Σe²) error of u^{n+k}
    is returned in a dict {k: (max, sumsq)}. ``analytic_start``: n = 1, u⁰ and u¹ are computed in the kernel
    (``prev``/``cur`` are not read)."""
    C = _C()
    if not out1.is_cuda:
        raise ValueError("leapfrog_tb is a GPU kernel; on the CPU take single leapfrog() steps")
    t = C.LeapfrogTbTiling()
    t.stages = stages
    t.threads = threads
    t.p2 = p2  # the pair-tiled kernel (k_leapfrog_p2) where it applies; False: k_leapfrog_tb
    if target_blocks is not None:
        t.target_blocks = target_blocks
    nb = C.gpu_leapfrog_tb_partials(layout, box, t)
    ct = list(ct) if ct is not None else [0.0] * stages
    part = torch.empty((stages * max(nb, 1), 2), dtype=torch.float64, device=out1.device) if check_mask else None
    C.gpu_leapfrog_tb(layout, coeffs, prev.data_ptr() if prev is not None else 0,
                      cur.data_ptr() if cur is not None else 0, out1.data_ptr(), out2.data_ptr(), box,
                      s_ext.data_ptr(), ct, check_mask, part.data_ptr() if check_mask else 0, t, _stream(),
                      analytic_start=analytic_start)
    res = {}
    for k in range(1, stages + 1):
        if check_mask >> (k - 1) & 1:
            out = torch.empty(2, dtype=torch.float64, device=out1.device)
            C.gpu_reduce(part[(k - 1) * nb:].data_ptr(), nb, out.data_ptr(), _stream())
            o = out.cpu()
            res[k] = (float(o[0]), float(o[1]))
    return res


def error(layout, u: torch.Tensor, box, s_ext: torch.Tensor, ct: float):
    C = _C()
    if u.is_cuda:
        nb = C.gpu_error_blocks(layout, box)
        if nb == 0:
            return 0.0, 0.0
        part = torch.empty((nb, 2), dtype=torch.float64, device=u.device)
        C.gpu_error(layout, u.data_ptr(), box, s_ext.data_ptr(), ct, part.data_ptr(), _stream())
        out = torch.empty(2, dtype=torch.float64, device=u.device)
        C.gpu_reduce(part.data_ptr(), nb, out.data_ptr(), _stream())
        o = out.cpu()
        return float(o[0]), float(o[1])
    return tuple(C.cpu_error(layout, u.numpy(), box, s_ext.numpy(), ct))


def pack(layout, plan, u: torch.Tensor, buf: torch.Tensor) -> None:
    """Gather every strided (y/z) face of ``plan`` into ``buf`` at the faces' pack offsets."""
    C = _C()
    if u.is_cuda:
        C.gpu_pack(layout, plan, u.data_ptr(), buf.data_ptr(), _stream())
        return
    for f in plan.faces:
        if not f.contiguous:
            C.cpu_pack_face(layout, f, u.numpy(), buf[f.pack_off: f.pack_off + f.count].numpy())


def unpack(layout, plan, buf: torch.Tensor, u: torch.Tensor) -> None:
    C = _C()
    if u.is_cuda:
        C.gpu_unpack(layout, plan, buf.data_ptr(), u.data_ptr(), _stream())
        return
    for f in plan.faces:
        if not f.contiguous:
            C.cpu_unpack_face(layout, f, buf[f.pack_off: f.pack_off + f.count].numpy(), u.numpy())


# ---------------------------------------------------------------------------------------------------------------
# plain PyTorch fp64 reference ops (the numerics baseline the kernel tests compare against)
# ---------------------------------------------------------------------------------------------------------------
def ref_leapfrog_grid(cur: torch.Tensor, old: torch.Tensor, ihx2: float, ihy2: float, ihz2: float, tau2: float,
                      box) -> torch.Tensor:
    """Reference leapfrog on dense ghost-padded grids (index i ↔ local node i-1); returns the updated copy of old."""
    out = old.clone()
    x0, x1, y0, y1, z0, z1 = (box.x0 + 1, box.x1 + 1, box.y0 + 1, box.y1 + 1, box.z0 + 1, box.z1 + 1)
    c = cur[x0:x1, y0:y1, z0:z1]
    c2 = 2.0 * c
    assert ihx2 == ihy2 == ihz2, "uniform grid: one 1/h² factor (stencil.hpp::d2sum)"
    s = ((cur[x0 + 1:x1 + 1, y0:y1, z0:z1] - c2 + cur[x0 - 1:x1 - 1, y0:y1, z0:z1])
         + (cur[x0:x1, y0 + 1:y1 + 1, z0:z1] - c2 + cur[x0:x1, y0 - 1:y1 - 1, z0:z1])
         + (cur[x0:x1, y0:y1, z0 + 1:z1 + 1] - c2 + cur[x0:x1, y0:y1, z0 - 1:z1 - 1]))
    # (unfused τ²-term: a plain-PyTorch reference, within one rounding of the kernels' fused leapfrog)
    out[x0:x1, y0:y1, z0:z1] = (2.0 * c - old[x0:x1, y0:y1, z0:z1]) + (tau2 * ihx2) * s
    return out
