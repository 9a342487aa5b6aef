"""High-level entry point: ``Solver`` (persistent, for repeated timed solves) and ``solve()`` (one shot).

Backends / transports:

=========  ==========  =============================================================================================
backend    transport   what runs
=========  ==========  =============================================================================================
hip        rccl        native C++ GpuSolver: HIP kernels, C++ step loop, RCCL P2P halos on a side stream overlapped
                       with the interior update, whole solve captured in one hipGraph (production path, any world)
hip        torch       Python step loop, HIP kernels, halos over torch.distributed (RCCL, or gloo staged via host)
hip        loopback    native GpuGroup: all ranks of a decomposition in THIS process on one GPU, device-copy halos
                       (exercises the production multi-rank C++ path on a single GPU; tests)
hip        rccl-self   native GpuGroup as above, halos moved by the production RCCL ncclSend/ncclRecv calls, each rank
                       over its own one-rank communicator (RCCL refuses 2 ranks of one communicator on one GPU)
hip        push        world > 1 in ONE process: native GpuGroup as above on the slab LDS passes, halos pushed by the
                       passes themselves into the neighbours' fine-grained staging + flag signalling
hip        push-ipc    one process per rank (torchrun): native GpuSolver on the slab LDS passes with the push transport
                       between processes (IPC handles all-gathered over torch.distributed; RCCL for the error log)
hip        sdma        world > 1 in ONE process: native GpuGroup on the LDS passes (slab or block), halos copied by the
                       SDMA copy engines into the peers' buffers, ordered by command-processor flag waits
hip        multi-dev.  world ≤ visible GPUs in ONE process: rank r on device r, one RCCL communicator from
                       ncclCommInitAll, one host thread per rank running the production GpuSolver (transport
                       "multi-device"; sdma=True: copy engines between the devices instead of RCCL)
hip        sdma-ipc    one process per rank (torchrun): native GpuSolver with the copy-engine transport between
                       processes (IPC handles all-gathered over torch.distributed; RCCL for the error log)
cpu        native      C++ CpuSolver, OpenMP (the reference's sequential / OpenMP programs), world == 1
cpu        torch       Python step loop, native OpenMP kernels, halos over torch.distributed gloo (MPI analogue)
torch      -           plain PyTorch fp64 reference solver (oracle), world == 1
=========  ==========  =============================================================================================

``runtime="process"`` (hip with rccl / sdma / push, one process per rank): the rank's production GpuSolver runs in a
``bin/wave3d --serve`` child that stays up between ``run()`` calls and graph-captures the multi-rank schedule, which a
torch process's HIP 7.0 runtime cannot (``parallel/native_proc.py``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from ._native import load
from .models.wave3d import ProblemSpec, torch_reference_solve


@dataclass
class SolveResult:
    spec: ProblemSpec
    backend: str
    transport: str
    world: int
    dims: tuple
    steps: list
    max_err: list
    rms_err: list
    solve_s: float
    finite: bool = True
    extra: dict = field(default_factory=dict)

    def lines(self) -> list[str]:
        from .utils.report import error_line

        return [error_line(n, n * self.spec.tau, m, r) for n, m, r in zip(self.steps, self.max_err, self.rms_err)]

    @property
    def gcell_per_s(self) -> float:
        return self.spec.cell_updates / self.solve_s / 1e9 if self.solve_s > 0 else float("nan")


def _resolve(backend: str, transport: str, world: int) -> tuple[str, str]:
    if backend == "auto":
        backend = "hip" if torch.cuda.is_available() else "cpu"
    if transport == "auto":
        transport = {"hip": "rccl", "cpu": "native" if world == 1 else "torch", "torch": "none"}[backend]
    ok = {("hip", "rccl"), ("hip", "torch"), ("hip", "loopback"), ("hip", "rccl-self"), ("hip", "push"),
          ("hip", "push-ipc"), ("hip", "sdma"), ("hip", "sdma-ipc"), ("hip", "multi-device"),
          ("cpu", "native"),
          ("cpu", "torch"),
          ("torch", "none")}
    if (backend, transport) not in ok:
        raise ValueError(f"unsupported backend/transport combination {backend}/{transport}")
    if backend == "cpu" and transport == "native" and world > 1:
        raise ValueError("the native CPU solver is single-rank; use transport='torch' for world > 1")
    if backend == "torch" and world > 1:
        raise ValueError("the torch reference solver is single-rank")
    return backend, transport


class Solver:
    """Construct once (allocation, communicator, graph capture on the first run), then ``run()`` repeatedly."""

    def __init__(self, spec: ProblemSpec, backend: str = "auto", transport: str = "auto", decomp: str = "slab",
                 rank: int | None = None, world: int | None = None, device: int | None = None,
                 overlap: bool = True, graph: bool = True, threads: int = 0, tiling: dict | None = None,
                 comm=None, group=None, stage_via_host: bool = False, force: bool = False, temporal: int = 5,
                 tiling2: dict | None = None, init2: bool = True, timers: bool = False, tb: bool = True,
                 tiling_tb: dict | None = None,
                 debug_sync: bool = False, poison_ghosts: bool = False, deep_min_planes: int | None = None,
                 tb_min_planes: int | None = None, rccl: bool = True, autotune: bool = False,
                 autotune_rounds: int = 5, copy_engines: bool = False, fused_pack: bool = True,
                 ghost_store: bool = True,
                 runtime: str = "inproc"):
        import torch.distributed as dist

        if not spec.cfl_ok and not force:
            raise ValueError(f"CFL violated: courant = {spec.courant:.4f} > 1 (tau_max = {spec.tau_max:.3e}); "
                             "pass force=True to run anyway")
        if rank is None or world is None:
            if dist.is_initialized():
                rank, world = dist.get_rank(), dist.get_world_size()
            else:
                rank, world = 0, 1
        self.spec, self.rank, self.world = spec, rank, world
        self.backend, self.transport = _resolve(backend, transport, world)
        self.decomp = decomp
        self._impl = None
        if runtime not in ("inproc", "process"):
            raise ValueError("runtime is 'inproc' (this process) or 'process' (a native bin/wave3d rank process)")
        self.runtime = runtime
        if runtime == "process":
            # every option the rank process honours becomes its CLI flag; the others raise (none is
            # dropped silently)
            flags = []
            if tiling is not None or tiling2 is not None:
                raise ValueError("runtime='process' takes no tiling / tiling2 overrides (the rank process uses its "
                                 "defaults; run in-process to sweep tilings)")
            tt = dict(tiling_tb or {})
            for k, flag in (("threads", "--tb-threads"), ("init_threads", "--tb-init-threads")):
                if k in tt:
                    flags += [flag, str(int(tt.pop(k)))]
            if tt:
                raise ValueError(f"runtime='process' cannot honour tiling_tb keys {sorted(tt)}")
            if copy_engines and self.transport not in ("sdma", "sdma-ipc"):
                raise ValueError("runtime='process': copy engines are the 'sdma' transport (transport='sdma')")
            for on, flag in ((timers, "--timers"), (debug_sync, "--debug-sync"), (poison_ghosts, "--poison-ghosts"),
                             (not tb, "--no-tb"), (not init2, "--no-init2"), (not fused_pack, "--no-fused-pack"),
                             (not ghost_store, "--no-ghost-store")):
                if on:
                    flags.append(flag)
            for val, flag in ((tb_min_planes, "--tb-min-planes"), (deep_min_planes, "--deep-min-planes")):
                if val is not None:
                    flags += [flag, str(int(val))]
            if autotune_rounds != 5:
                flags += ["--autotune-rounds", str(int(autotune_rounds))]
            self._init_process(device, decomp, temporal, overlap, graph, rccl, autotune, group, tuple(flags))
            return
        C = load()
        if self.backend == "hip":
            if not torch.cuda.is_available():
                raise RuntimeError("backend 'hip' needs a GPU")
            dev = device if device is not None else (rank % torch.cuda.device_count())
            torch.cuda.set_device(dev)
            C.gpu_set_device(dev)
            self.device = torch.device("cuda", dev)
        else:
            self.device = torch.device("cpu")
        if self.backend == "hip" and self.transport in ("loopback", "rccl-self", "push", "sdma", "multi-device"):
            opts = self._options(C, decomp, spec, overlap, graph, tiling, temporal, tiling2, init2, tb, tiling_tb)
            opts.timers, opts.debug_sync, opts.poison_ghosts = timers, debug_sync, poison_ghosts
            opts.fused_pack, opts.ghost_store = fused_pack, ghost_store
            if deep_min_planes is not None:
                opts.deep_min_planes = deep_min_planes
            if tb_min_planes is not None:
                opts.tb_min_planes = tb_min_planes
            opts.sdma = copy_engines and self.transport == "multi-device"
            self._impl = C.GpuGroup(spec.native(), opts, world, self.transport)
            self.dims = self._impl.dims().as_tuple()
        elif self.backend == "hip" and self.transport in ("rccl", "push-ipc", "sdma-ipc"):
            from .parallel.rccl import make_comm

            opts = self._options(C, decomp, spec, overlap, graph, tiling, temporal, tiling2, init2, tb, tiling_tb)
            opts.timers, opts.debug_sync, opts.poison_ghosts = timers, debug_sync, poison_ghosts
            opts.fused_pack, opts.ghost_store = fused_pack, ghost_store
            if deep_min_planes is not None:
                opts.deep_min_planes = deep_min_planes
            if tb_min_planes is not None:
                opts.tb_min_planes = tb_min_planes
            opts.push = self.transport == "push-ipc"
            opts.sdma = self.transport == "sdma-ipc"
            # (push-ipc / sdma-ipc without RCCL — ranks sharing one GPU, which RCCL refuses: no communicator, so no
            # end-of-solve collective; each rank's error log is its own)
            opts.push_no_collective = (opts.push or opts.sdma) and not rccl
            if comm is None and world > 1 and (rccl or not (opts.push or opts.sdma)):
                comm = make_comm(rank, world, group)
            self.comm = comm
            self.schedule, self.autotune_times, self.autotune_rejected = None, {}, {}
            if autotune:
                # the CLI's autotune (csrc/src/runtime_autotune.cpp): every candidate built, checked against the first
                # accepted one's error log, timed in interleaved rounds; the slowest rank decides
                if self.transport != "rccl":
                    raise ValueError("autotune picks the transport itself: use transport='rccl' (the default)")
                self._impl, self.schedule, self.autotune_times, self.autotune_rejected = C.autotune(
                    spec.native(), opts, rank, world, comm, rounds=autotune_rounds)
            else:
                self._impl = C.GpuSolver(spec.native(), opts, rank, world, comm)
            if self._impl.push and world > 1:  # every rank's IPC handles, over torch.distributed (gloo)
                import torch.distributed as tdist

                handles = [None] * world
                tdist.all_gather_object(handles, self._impl.push_handles(), group=group)
                self._impl.connect_push(handles)
            if self._impl.sdma and world > 1:
                import torch.distributed as tdist

                handles = [None] * world
                tdist.all_gather_object(handles, self._impl.sdma_handles(), group=group)
                self._impl.connect_sdma(handles)
            self.dims = self._impl.dims.as_tuple()
        elif self.transport in ("torch",):
            from .parallel.dist_solver import TorchDistSolver

            self._impl = TorchDistSolver(spec, rank, world, decomp, self.device, group, stage_via_host, threads)
            self.dims = self._impl.plan.dims
        elif self.backend == "cpu":
            self._impl = C.CpuSolver(spec.native(), spec.check_every, threads)
            self.dims = (1, 1, 1)
        else:
            self.dims = (1, 1, 1)

    def _init_process(self, device, decomp, temporal, overlap, graph, rccl, autotune, group, flags=()) -> None:
        """runtime="process": this rank's production solver in a ``bin/wave3d --serve`` child (graph-captured under
        the system ROCm runtime, which a torch process cannot do for multi-rank schedules; parallel/native_proc.py).
        Transports: rccl, sdma / sdma-ipc (copy engines), push / push-ipc; one process per rank (torchrun)."""
        import torch.distributed as dist

        from .parallel.native_proc import NativeRankProcess

        if self.backend != "hip":
            raise ValueError("runtime='process' runs the native HIP backend")
        if device is None:
            device = self.rank % max(1, torch.cuda.device_count())  # (device_count does not initialise the GPU)
        self.device = torch.device("cuda", device)
        self.comm = None
        # one Python process driving all ranks (no torch.distributed job): the whole in-process group lives in ONE
        # rank process (bin/wave3d --group P --group-transport T --serve), graph-captured under its ROCm 7.2 runtime
        self._group_proc = self.world > 1 and not dist.is_initialized() and self.transport in (
            "loopback", "rccl-self", "push", "sdma", "multi-device")
        if self._group_proc:
            if autotune:
                raise ValueError("runtime='process' with an in-process group has no autotune")
            self._impl = NativeRankProcess(self.spec, 0, 1, device, "rccl", decomp, temporal, overlap, graph, True,
                                           False, None, extra_args=("--group", str(self.world), "--group-transport",
                                                                    self.transport, *flags))
        else:
            self.transport = {"sdma": "sdma-ipc", "push": "push-ipc"}.get(self.transport, self.transport)
            self._impl = NativeRankProcess(self.spec, self.rank, self.world, device, self.transport, decomp,
                                           temporal, overlap, graph, rccl, autotune, group, extra_args=flags)
        self.dims = tuple(self._impl.info["dims"])
        self.schedule = self._impl.info["schedule"]
        self.autotune_times, self.autotune_rejected = {}, {}

    def _process_fields(self, which: int, assemble: bool) -> torch.Tensor:
        """runtime="process": u^K through the rank process's wave3d-dump-v1 files — this rank's owned nodes, or (assemble)
        the global (N+1)³ field from every rank of an in-process group / of a single rank."""
        import json
        import tempfile

        import numpy as np

        if which != 0:
            raise ValueError("runtime='process' downloads u^K (which=0) only")
        if assemble and self.world > 1 and not self._group_proc:
            raise RuntimeError("global_field of a process-per-rank job: gather the ranks' owned_field instead")
        with tempfile.TemporaryDirectory() as d:
            prefix = os.path.join(d, "f")
            self._impl.dump(prefix)
            ranks = range(self.world) if (assemble or self._group_proc) else [self.rank]
            n = self.spec.N + 1
            out = np.zeros((n, n, n)) if assemble else None
            for r in ranks:
                tag = f".rank{r}" if self.world > 1 else ""
                meta = json.loads(open(prefix + tag + ".json").read())
                a = np.fromfile(prefix + tag + ".bin", dtype=np.float64).reshape(meta["shape"])
                if not assemble:
                    return torch.from_numpy(a)
                x0, y0, z0 = meta["offset"]
                out[x0:x0 + a.shape[0], y0:y0 + a.shape[1], z0:z0 + a.shape[2]] = a
        return torch.from_numpy(out)

    def close(self) -> None:
        """Stop the native rank process (runtime="process"); a no-op otherwise."""
        if self.runtime == "process" and self._impl is not None:
            self._impl.close()

    @staticmethod
    def _options(C, decomp, spec, overlap, graph, tiling, temporal=5, tiling2=None, init2=True, tb=True,
                 tiling_tb=None):
        opts = C.SolverOptions()
        opts.temporal = temporal
        opts.init2 = init2
        opts.tb = tb
        if tiling2:
            for k, v in tiling2.items():
                setattr(opts.tiling2, k, v)
        if tiling_tb:
            for k, v in tiling_tb.items():
                setattr(opts.tiling_tb, k, v)
        opts.decomp = decomp
        opts.check_every = spec.check_every
        opts.overlap = overlap
        opts.graph = graph
        if tiling:
            for k, v in tiling.items():
                setattr(opts.tiling, k, v)
        return opts

    def run(self) -> SolveResult:
        if self.backend == "torch":
            import time

            t0 = time.perf_counter()
            errs = torch_reference_solve(self.spec)
            dt = time.perf_counter() - t0
            steps = sorted(errs)
            return SolveResult(self.spec, "torch", "none", 1, (1, 1, 1), steps, [errs[n][0] for n in steps],
                               [errs[n][1] for n in steps], dt,
                               all(math.isfinite(v) for n in steps for v in errs[n]))
        r = self._impl.run()
        return SolveResult(self.spec, self.backend, self.transport, self.world, tuple(self.dims), list(r["steps"]),
                           list(r["max_err"]), list(r["rms_err"]), float(r["solve_s"]), bool(r["finite"]),
                           {k: v for k, v in r.items() if k not in ("steps", "max_err", "rms_err", "solve_s",
                                                                    "finite")})

    def run_batch(self, n: int) -> list:
        """n solves back to back, each with its own error log. A one-rank in-process HIP solver enqueues the n graph
        replays and synchronises once (``GpuSolver::run_batch``, the bench's timed block; solve_s = batch time / n);
        every other backend runs run() n times."""
        if self.backend == "hip" and self.runtime == "inproc" and hasattr(self._impl, "run_batch"):
            return [SolveResult(self.spec, self.backend, self.transport, self.world, tuple(self.dims), list(r["steps"]),
                                list(r["max_err"]), list(r["rms_err"]), float(r["solve_s"]), bool(r["finite"]),
                                {k: v for k, v in r.items() if k not in ("steps", "max_err", "rms_err", "solve_s",
                                                                         "finite")})
                    for r in self._impl.run_batch(int(n))]
        return [self.run() for _ in range(int(n))]

    def set_state(self, prev, cur, step: int) -> None:
        """Loaded-field start (resume): every following run() starts at ``step`` from u^{step-1} = prev and
        u^{step} = cur (GLOBAL (N+1)³ float64 arrays or tensors, e.g. utils.dump.load of a checkpoint) and continues to
        K, checking the steps after ``step``. Native backends take each rank's box and ghost layers from the global
        fields (no exchange before the first pass); the result is bit-identical to an uninterrupted run."""
        import numpy as np

        if self.backend == "torch":
            raise ValueError("the torch reference solver has no resume")
        if self.runtime == "process":
            raise ValueError("runtime='process' has no resume from Python (use bin/wave3d --resume)")
        if self.transport == "torch":
            to_t = (lambda a: a if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a)))
            self._impl.set_state(to_t(prev), to_t(cur), int(step))
            return
        to_np = (lambda a: np.ascontiguousarray(a.cpu().numpy() if isinstance(a, torch.Tensor) else a,
                                                dtype=np.float64).reshape(-1))
        self._impl.set_state(to_np(prev), to_np(cur), int(step))

    @property
    def native(self):
        return self._impl

    def traffic(self) -> dict:
        """Bytes one solve of the last run()'s schedule moves on this rank (native HIP backend, one rank or a
        process-per-rank job): ``field_bytes`` = compulsory field reads + writes of the pass schedule (SURVEY.md §5.5:
        divide by the solve time for the effective GB/s), ``halo_bytes`` = what this rank sends its neighbours."""
        if self.backend != "hip" or self.transport == "torch" or not hasattr(self._impl, "traffic"):
            raise ValueError("traffic needs the native HIP backend with one solver per process")
        return dict(self._impl.traffic())

    def field_hash(self, which: int = 0) -> int:
        """Order-independent 64-bit hash of u^K (which=0) / u^{K-1} (which=1) over the nodes this process owns (an
        in-process group: over all its ranks), mod 2**64. Summed over the ranks of a job it does not depend on the
        decomposition or schedule of a bit-identical solve (the autotune's field check, GpuSolver::field_hash)."""
        if self.backend != "hip" or self.transport == "torch":
            raise ValueError("field_hash needs the native HIP backend")
        if self.runtime == "process":
            return self._impl.field_hash(which)
        if isinstance(self._impl, load().GpuGroup):
            return sum(self._impl.field_hash(r, which) for r in range(self._impl.world)) % (1 << 64)
        return int(self._impl.field_hash(which))

    def global_field(self, which: int = 0) -> torch.Tensor:
        """The whole (N+1)³ field u^K (which=0) / u^{K-1} (which=1) on the CPU (single rank or loopback group)."""
        from .ops.stencil import grid_view

        if self.runtime == "process":  # the rank process dumps u^K (all its ranks for a group): assemble the dumps
            return self._process_fields(which, assemble=True)
        if self.transport not in ("loopback", "rccl-self", "push", "sdma", "multi-device"):
            if self.world != 1:
                raise RuntimeError("global_field needs world == 1 or the loopback transport")
            return self.owned_field(which)
        n = self.spec.N + 1
        out = torch.empty((n, n, n), dtype=torch.float64)
        for r in range(self.world):
            lay = self._impl.layout(r)
            g = grid_view(lay, torch.from_numpy(self._impl.download(r, which)))
            out[lay.gx0:lay.gx0 + lay.nx, lay.gy0:lay.gy0 + lay.ny, lay.gz0:lay.gz0 + lay.nz] = \
                g[1:1 + int(lay.nx), 1:1 + int(lay.ny), 1:1 + int(lay.nz)]
        return out

    def owned_field(self, which: int = 0) -> torch.Tensor:
        """This rank's owned nodes of u^K (which=0) or u^{K-1} (which=1) as a CPU (nx, ny, nz) float64 tensor."""
        from .ops.stencil import grid_view

        if self.runtime == "process":  # through a wave3d-dump-v1 file of the rank process (u^K only)
            return self._process_fields(which, assemble=False)
        if self.transport == "torch":
            return self._impl.owned_field(which)
        if self.backend == "hip":
            flat = torch.from_numpy(self._impl.download(which))
            lay = self._impl.layout
        else:
            flat = torch.from_numpy(self._impl.field(which).copy())
            lay = self._impl.layout
        g = grid_view(lay, flat)
        return g[1:1 + int(lay.nx), 1:1 + int(lay.ny), 1:1 + int(lay.nz)].clone()


def solve(spec: ProblemSpec, **kw) -> SolveResult:
    return Solver(spec, **kw).run()
