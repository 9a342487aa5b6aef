"""Native rank process: the Python ``Solver(runtime="process")`` backend.

A torch process cannot graph-capture the multi-rank schedules: the HIP 7.0 runtime PyTorch-ROCm bundles crashes in
``hipStreamEndCapture`` on their repeated cross-stream event joins (``csrc/src/solver_gpu.cpp``
``multistream_capture_safe``), so an in-process ``GpuSolver`` with world > 1 launches eagerly. The native CLI links the
system ROCm 7.2 runtime and captures them (one graph per solve, or per parity for the copy-engine transport). This
module therefore runs each rank's solver in a ``bin/wave3d --serve`` child — the same runtime ``bench.py`` starts per
rank — and talks to it one JSON line per command (``run``, ``hash W``, ``traffic``, ``dump P``, ``quit``; protocol in
``csrc/app/cli.hpp`` ``serve_loop``, handlers in ``wave3d_main.cpp`` ``serve`` and ``cli_cpu.cpp``). The solver, its buffers, communicator and captured graphs stay up between
``run()`` calls, so repeated solves time the replayed graph exactly as the CLI does.

Rendezvous: rank 0 draws a nonce, broadcast over the torch.distributed group (gloo or RCCL), which names the file the
children exchange the RCCL unique id / IPC handles through (``W3D_RDZV_FILE``). Every rank must issue the same command
sequence (``run`` and ``quit`` are collective inside the children).
"""
from __future__ import annotations

import json
import os
import select
import subprocess
import tempfile
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CLI = os.path.join(ROOT, "bin", "wave3d")

# Solver transport -> bin/wave3d transport flags
_TRANSPORT_FLAGS = {"rccl": [], "sdma-ipc": ["--transport", "sdma"], "push-ipc": ["--transport", "push"]}


class NativeRankProcess:
    """One ``bin/wave3d --serve`` child holding this rank's production GpuSolver."""

    def __init__(self, spec, rank: int, world: int, device: int, transport: str = "rccl", decomp: str = "slab",
                 temporal: int = 4, overlap: bool = True, graph: bool = True, rccl: bool = True,
                 autotune: bool = False, group=None, timeout_s: float | None = None, nonce: str | None = None,
                 extra_args: tuple = ()):
        if transport not in _TRANSPORT_FLAGS:
            raise ValueError(f"runtime='process' runs transports {sorted(_TRANSPORT_FLAGS)}, not {transport!r}")
        if not os.path.exists(CLI):
            raise RuntimeError(f"native runtime {CLI} is missing (python tools/build.py)")
        # bound of every reply (the greeting includes the solver's setup): W3D_PROC_TIMEOUT_S, default 300 s
        if timeout_s is None:
            timeout_s = float(os.environ.get("W3D_PROC_TIMEOUT_S", "300"))
        self.rank, self.world, self.timeout_s = rank, world, timeout_s
        if nonce is None:
            nonce = uuid.uuid4().hex
            if world > 1:
                from .rccl import broadcast_bytes

                nonce = broadcast_bytes(nonce.encode() if rank == 0 else None, 0, group).decode()
        tmp = tempfile.gettempdir()
        cmd = [CLI, str(spec.N), repr(spec.tau), str(spec.K), repr(spec.L), "--serve", "--quiet",
               "--decomp", decomp, "--temporal", str(temporal), "--check-every", str(spec.check_every),
               *_TRANSPORT_FLAGS[transport]]
        if not overlap:
            cmd.append("--no-overlap")
        if not graph:
            cmd.append("--no-graph")
        if not rccl:
            cmd.append("--no-rccl")
        if autotune:
            cmd.append("--autotune")
        cmd += list(extra_args)
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(device),
                   W3D_RDZV_FILE=os.path.join(tmp, f"wave3d-proc-{nonce}.uid"), W3D_JOB_ID=f"proc{nonce}")
        if not rccl and world > 1:
            env["W3D_SHARE_GPUS"] = "1"  # (ranks without a communicator may share one GPU)
        self._log = tempfile.NamedTemporaryFile("w+", prefix=f"wave3d-proc-{nonce}-r{rank}-", suffix=".log",
                                                delete=False)
        self._p = subprocess.Popen(cmd, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=self._log,
                                   text=True, bufsize=1)
        # replies are split into lines here, from raw reads: a buffered readline() after select() could leave the
        # greeting in Python's buffer behind a library's banner lines and then wait on an empty pipe
        self._buf = b""
        self.info = self._read()
        if not self.info.get("ready"):
            raise RuntimeError(f"native rank process {rank}: unexpected greeting {self.info}")

    def _stderr_tail(self) -> str:
        self._log.flush()
        with open(self._log.name) as f:
            return f.read()[-2000:]

    def _line(self, deadline: float) -> bytes | None:
        """Next complete stdout line (without its newline), or None when none has arrived by ``deadline``."""
        fd = self._p.stdout.fileno()
        while b"\n" not in self._buf:
            left = deadline - time.monotonic()
            if left <= 0:
                return None
            ready, _, _ = select.select([fd], [], [], min(left, 1.0))
            if ready:
                chunk = os.read(fd, 1 << 16)
                if not chunk:
                    rc = self._p.wait()
                    raise RuntimeError(f"native rank process {self.rank} exited (rc={rc}):\n{self._stderr_tail()}")
                self._buf += chunk
            elif self._p.poll() is not None:
                raise RuntimeError(f"native rank process {self.rank} exited (rc={self._p.returncode}):\n"
                                   f"{self._stderr_tail()}")
        line, self._buf = self._buf.split(b"\n", 1)
        return line

    def _read(self) -> dict:
        deadline = time.monotonic() + self.timeout_s
        while True:
            line = self._line(deadline)
            if line is None:
                self._p.kill()
                raise TimeoutError(f"native rank process {self.rank}: no reply in {self.timeout_s:.0f} s\n"
                                   f"{self._stderr_tail()}")
            if not line.lstrip().startswith(b"{"):
                continue  # (a library's own stdout line, e.g. RCCL's banner: not a reply)
            msg = json.loads(line)
            if "error" in msg:
                raise RuntimeError(f"native rank process {self.rank}: {msg['error']}")
            return msg

    def command(self, line: str) -> dict:
        try:
            self._p.stdin.write(line + "\n")
            self._p.stdin.flush()
        except (BrokenPipeError, OSError):
            rc = self._p.wait()
            raise RuntimeError(f"native rank process {self.rank} exited (rc={rc}):\n{self._stderr_tail()}") from None
        return self._read()

    def run(self) -> dict:
        """One solve; the same keys as the in-process GpuSolver.run() dict (steps, max_err, rms_err, solve_s = max over
        ranks, finite) plus graph / overlap / local_s."""
        r = self.command("run")
        steps = r.pop("steps")
        r["steps"] = [int(s[0]) for s in steps]
        r["max_err"] = [float(s[1]) for s in steps]
        r["rms_err"] = [float(s[2]) for s in steps]
        return r

    def field_hash(self, which: int = 0) -> int:
        return int(self.command(f"hash {int(which)}")["hash"])

    def traffic(self) -> dict:
        return self.command("traffic")

    def dump(self, prefix: str) -> None:
        self.command(f"dump {prefix}")

    def close(self) -> None:
        if self._p.poll() is None:
            try:
                self.command("quit")
                self._p.wait(timeout=30)
            except Exception:
                self._p.kill()
                self._p.wait()
        for f in (self._p.stdin, self._p.stdout):
            try:
                f.close()
            except Exception:
                pass
        self._log.close()
        if os.path.exists(self._log.name):
            os.remove(self._log.name)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
