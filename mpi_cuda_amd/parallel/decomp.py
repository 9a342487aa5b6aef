"""Domain decomposition helpers (Python view of the native planner in csrc/include/wave3d/decomp.hpp).

The reference decomposes the (N+1)³ node grid into blocks, one per MPI rank, for P ∈ {1,2,4,8,10,16,20,32}
(report.pdf p.4 §1, p.9-10 §3.1.4). Supported here: ``slab`` (P×1×1, contiguous x faces),
``block`` (surface-minimising px·py·pz) and an explicit ``PxQxR``.
"""
from __future__ import annotations

from dataclasses import dataclass

from .._native import load


@dataclass(frozen=True)
class RankPlan:
    rank: int
    world: int
    dims: tuple[int, int, int]
    box: tuple[int, int, int, int, int, int]  # global node ranges [x0,x1) [y0,y1) [z0,z1)
    neighbors: dict  # (axis, side) -> rank
    layout: object
    halo: object


def plan(N: int, world: int, rank: int, decomp: str = "slab", tau: float = 1e-3, K: int = 20, L: float = 1.0):
    C = load()
    prob = C.Problem(N, tau, K, L)
    dims = C.parse_dims(decomp, world, N)
    b = C.rank_box(prob, dims, rank)
    lay = C.make_layout(prob, b)
    halo = C.make_halo_plan(lay, dims, rank)
    nbrs = {}
    for axis in range(3):
        for side in range(2):
            r = C.neighbor_rank(dims, rank, axis, side)
            if r >= 0:
                nbrs[(axis, side)] = r
    return RankPlan(rank, world, dims.as_tuple(), (b.x0, b.x1, b.y0, b.y1, b.z0, b.z1), nbrs, lay, halo)


def all_boxes(N: int, world: int, decomp: str = "slab"):
    return [plan(N, world, r, decomp).box for r in range(world)]


def split_boxes(layout, neighbors: dict):
    """(shell boxes, interior box) of a rank: the shell is every updated node within one layer of a face that has a
    neighbour (computed first so its faces can be sent while the interior is updated). The native runtime's own split
    (``shell_split`` in csrc/include/wave3d/cpu.hpp, the one GpuSolver uses), not a re-implementation."""
    C = load()
    full = C.compute_box(layout)
    nb = [[(a, s) in neighbors for s in range(2)] for a in range(3)]
    shell, interior = C.shell_split(full, nb)
    return list(shell), interior
