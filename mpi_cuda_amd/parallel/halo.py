"""Halo (ghost-layer) exchange over torch.distributed.

This is the portable transport: gloo for CPU tensors (the reference's MPI / MPI+OpenMP CPU programs, report.pdf
p.9-11 §3.1.4-3.1.5) and RCCL ("nccl" backend) for GPU tensors. Production multi-GPU runs use the native C++ RCCL
path instead (csrc/src/solver_gpu.cpp: ncclSend/ncclRecv on a side stream, overlapped, graph-captured); this module is
the A/B baseline and what the multi-process CPU tests exercise.

x faces are contiguous planes sent straight from the field; y/z faces are packed into a staging buffer first.
With ``stage_via_host`` (GPU tensors over gloo, e.g. several ranks sharing one GPU in a test) faces are copied
through host memory.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import stencil as ops


class TorchHaloExchange:
    def __init__(self, layout, plan, device, group=None, stage_via_host: bool = False):
        self.layout = layout
        self.plan = plan
        self.group = group
        self.device = torch.device(device)
        self.stage = stage_via_host and self.device.type == "cuda"
        n = int(plan.packed_doubles)
        self.send_buf = torch.zeros(max(n, 1), dtype=torch.float64, device=self.device)
        self.recv_buf = torch.zeros(max(n, 1), dtype=torch.float64, device=self.device)
        self.faces = list(plan.faces)
        if self.stage:
            self.h_send = [torch.empty(int(f.count), dtype=torch.float64) for f in self.faces]
            self.h_recv = [torch.empty(int(f.count), dtype=torch.float64) for f in self.faces]

    def _views(self, u: torch.Tensor):
        out = []
        for f in self.faces:
            c = int(f.count)
            if f.contiguous:
                s = u[int(f.send_off): int(f.send_off) + c]
                r = u[int(f.recv_off): int(f.recv_off) + c]
            else:
                s = self.send_buf[int(f.pack_off): int(f.pack_off) + c]
                r = self.recv_buf[int(f.pack_off): int(f.pack_off) + c]
            out.append((f, s, r))
        return out

    def exchange(self, u: torch.Tensor) -> None:
        if not self.faces:
            return
        if self.plan.packed_doubles > 0:
            ops.pack(self.layout, self.plan, u, self.send_buf)
        views = self._views(u)
        if self.stage:
            for i, (_, s, _) in enumerate(views):
                self.h_send[i].copy_(s)
            torch.cuda.synchronize(self.device)
            send = [self.h_send[i] for i in range(len(views))]
            recv = [self.h_recv[i] for i in range(len(views))]
        else:
            send = [s for _, s, _ in views]
            recv = [r for _, _, r in views]
        p2p = []
        for i, (f, _, _) in enumerate(views):
            p2p.append(dist.P2POp(dist.isend, send[i], int(f.peer), group=self.group))
            p2p.append(dist.P2POp(dist.irecv, recv[i], int(f.peer), group=self.group))
        for req in dist.batch_isend_irecv(p2p):
            req.wait()
        if self.stage:
            for i, (_, _, r) in enumerate(views):
                r.copy_(self.h_recv[i])
        if self.plan.packed_doubles > 0:
            ops.unpack(self.layout, self.plan, self.recv_buf, u)
