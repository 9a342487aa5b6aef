#!/usr/bin/env python3
"""Headline benchmark: 512³ (N=512), τ=1e-3, K=20, L=1, fp64 — the reference's MPI+CUDA config (BASELINE.md,
readme.md:99-100, report.pdf p.16 §4.4).

One bench "step" = one COMPLETE solve exactly as the reference times it: field init (u⁰, u¹) → 19 leapfrog steps →
error check vs the analytic solution every 2nd step → global error log on the host. Nothing is cached between solves:
every solve re-initialises the fields and recomputes all K steps.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

What runs: every rank starts the native runtime (``bin/wave3d``, C++ + HIP kernels + RCCL, built in-tree) as a child
process on its GPU and hands it the launch (RANK / LOCAL_RANK / WORLD_SIZE from torchrun, a per-launch rendezvous
nonce for the RCCL unique id). The child runs W untimed solves (plus, on several ranks, the schedule autotune, whose
candidate solves are untimed too), then EXACTLY K solves between a device sync + RCCL barrier on both sides, and reports
the interval as the max over ranks. This process only orchestrates (torch.distributed over gloo: nonce broadcast and
the agreement on success); it never touches the GPU. The child runs on the system ROCm (HIP 7.2 + RCCL 2.27), whose
stream capture of the multi-rank schedules is verified; the HIP 7.0 runtime bundled with PyTorch crashes in
hipStreamEndCapture on those graphs (tools/probes/capture_probe*.hip, csrc/src/solver_gpu.cpp multistream_capture_safe).

Rank 0 prints ONE JSON line. ``value`` = whole-job GCell-updates/s = N³·K / t_solve (reference convention) with
t_solve = (max over ranks of the K-solve interval) / K; ``ms_per_step`` = ``ms_per_solve`` = t_solve in ms (one bench
step is one solve); ``vs_baseline`` = value ÷ the reference's published total-time GCell/s at the same GPU count (1 GPU:
3.570 = 512³·20/0.752 s; 2 GPUs: 5.316 = 512³·20/0.505 s; for 4 and 8 GPUs, where the reference publishes nothing, its
best number, the 2-GPU 5.316 — ``vs_baseline_basis`` says which). The problem size is fixed as GPUs are added:
``scaling`` is "strong". ``rccl_nranks`` is the communicator size RCCL itself reports (ncclCommCount).

On several ranks the copy-engine (SDMA) schedules join the autotune only after a cross-device qualification child (a
64³ solve whose log must equal a one-rank solve's) passes. If the main native run fails on any rank, every rank starts
ONE fresh child with the conservative schedule (RCCL slabs, 4-step passes, no overlap, no autotune) and the line says
so (``fallback_schedule``, ``first_failure``); if that fails too, every rank stops with a non-zero exit and no JSON
line. ``--allow-fallback`` then re-runs the solve in-process over the torch.distributed transport (the Python
single-step loop) and marks the line ``"degraded": true`` with the error text. ``--python`` runs the in-process Python ``Solver`` path directly.
``--cpu`` drives the same orchestration with the native CPU ranks (the contract test without a GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
import uuid

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_GCELL = {1: 512**3 * 20 / 0.752 / 1e9, 2: 512**3 * 20 / 0.505 / 1e9}
REF_FINAL_LINF = 3.960129e-09  # report.pdf p.16 §4.3.1, step 20
CLI = os.path.join(ROOT, "bin", "wave3d")


def _args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed full solves")
    ap.add_argument("--warmup", type=int, default=3, help="untimed full solves (at least 1; 2 on several ranks)")
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--tau", type=float, default=1e-3)
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--L", type=float, default=1.0)
    ap.add_argument("--decomp", default="slab", help="slab | block | PxQxR (with --no-autotune)")
    ap.add_argument("--temporal", type=int, default=5,
                    help="at most this many leapfrog steps per HBM pass (1..5; the push transport uses at most 4)")
    ap.add_argument("--no-temporal", action="store_true", help="one leapfrog step per HBM pass")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-autotune", action="store_true",
                    help="several ranks: use --decomp/--temporal as given instead of timing the candidate schedules")
    ap.add_argument("--autotune", action="store_true", help="time the candidate schedules even on one rank")
    ap.add_argument("--no-phases", action="store_true", help="skip the traced per-phase breakdown solve")
    ap.add_argument("--cpu", action="store_true", help="native CPU ranks (contract test without a GPU)")
    ap.add_argument("--python", action="store_true", help="in-process Python Solver instead of the native runtime")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "torch"], help="--python: halo transport")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="if the native runtime fails, re-run over the torch transport (marked degraded)")
    ap.add_argument("--share-gpus", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (ranks share GPUs; RCCL refuses this, so use it "
                         "with --no-rccl --native-transport push; each rank then gets its own share of the CUs)")
    ap.add_argument("--native-transport", default="rccl", choices=["rccl", "push", "sdma"],
                    help="halo transport of the native runtime with --no-autotune (push: slab passes forward their "
                         "faces; sdma: copy engines move the halos into the peers' memory)")
    ap.add_argument("--no-rccl", action="store_true",
                    help="native ranks without an RCCL communicator (push / sdma only; host collectives through files)")
    ap.add_argument("--autotune-sdma", action="store_true",
                    help="several ranks: include the copy-engine candidates in the autotune (opt-in across GPUs)")
    ap.add_argument("--no-qualify", action="store_true",
                    help="several ranks: skip the cross-device copy-engine qualification before the autotune")
    ap.add_argument("--timeout", type=float, default=420.0,
                    help="seconds before a native rank is killed (below the driver's 600 s bench limit)")
    ap.add_argument("--out", default="", help="also append the JSON line to this file")
    return ap.parse_args(argv)


def _line(a, world, value, ms, cfg, extra) -> dict:
    base = REF_GCELL.get(world, REF_GCELL[2])
    line = {
        "metric": f"gcell_updates_per_s_{a.N}cube_K{a.K}",
        "value": round(value, 3),
        "unit": "GCell-updates/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "ms_per_solve": round(ms, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(value / base, 3),
        "vs_baseline_basis": {1: "1x P100, 0.752 s", 2: "2x P100, 0.505 s"}.get(
            world, "2x P100, 0.505 s (the reference publishes no 4/8-GPU number; its best)"),
        "dtype": "fp64",
        "data": "analytic initial condition sin(pi x)sin(pi y)sin(pi z) (synthetic, as the reference)",
        "config": {"model": "wave3d leapfrog 7-point fp64 (AICCer1/MPI-CUDA mpigpu-1 config)", "global_batch": 1,
                   "seq_len": a.N + 1, "grid": f"{a.N}^3", "N": a.N, "tau": a.tau, "K": a.K, "L": a.L, **cfg},
    }
    line.update(extra)
    return line


def _emit(a, line) -> None:
    s = json.dumps(line)
    print(s, flush=True)
    if a.out:
        with open(a.out, "a") as f:
            f.write(s + "\n")


def _correct(a, finite, steps) -> tuple[bool, str]:
    """Every config is checked against the closed-form oracle of the discrete scheme (SURVEY.md §1.6,
    models/wave3d.py oracle_errors): each checked step's L∞ and RMS within 1e-5 relative plus a rounding allowance of
    4e-16 per step (≈ 2 ulp of the O(1) field per step: at 2048³, τ = 2.5e-4 the error itself is 1.6e-13 at step 2 and
    the measured log sits 3e-16 from the oracle there, 1e-15 at step 20). The reference config must also reproduce
    the reference's printed step-20 L∞ (report.pdf p.16 §4.3.1)."""
    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.models.wave3d import oracle_errors

    if not finite or not steps:
        return False, "non-finite or empty error log"
    spec = ProblemSpec(N=a.N, tau=a.tau, K=a.K, L=a.L, check_every=2)
    ref = oracle_errors(spec, steps=[int(n) for n, _, _ in steps])
    for n, m, e in steps:
        om, oe = ref[int(n)]
        tol = 4e-16 * int(n)
        if abs(m - om) > 1e-5 * om + tol or abs(e - oe) > 1e-5 * oe + tol:
            return False, f"step {n}: L-inf {m:.6e} / RMS {e:.6e} vs oracle {om:.6e} / {oe:.6e}"
    ref_cfg = a.N == 512 and a.K == 20 and a.tau == 1e-3 and a.L == 1.0
    if ref_cfg and abs(steps[-1][1] / REF_FINAL_LINF - 1) >= 1e-5:
        return False, f"final L-inf {steps[-1][1]:.6e} is not the reference's {REF_FINAL_LINF:.6e}"
    return True, f"{len(steps)} checked steps match the closed-form oracle"


# ------------------------------------------------------------------------------------------------------------------
# native runtime (default)
# ------------------------------------------------------------------------------------------------------------------
def _agree(ok: int, world: int) -> int:
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist

    t = torch.tensor([ok], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def _child(a, rank: int, world: int, local: int, args: list[str], tag: str, ranks: int | None = None) -> dict:
    """One native child per rank (``bin/wave3d`` with ``args``) in a fresh rendezvous; every rank learns whether all
    succeeded. ``ranks`` = 1: rank 0 runs a one-rank job alone (the others wait). Returns {ok, res (rank 0), tail,
    rc, why}."""
    import torch.distributed as dist

    from mpi_cuda_amd.parallel.rccl import broadcast_bytes

    nonce = uuid.uuid4().hex.encode() if rank == 0 else None
    if world > 1:
        nonce = broadcast_bytes(nonce, 0)
    nonce = nonce.decode()
    jw = world if ranks is None else ranks
    runs = rank < jw
    tmp = tempfile.gettempdir()
    rdzv = os.path.join(tmp, f"wave3d-bench-{nonce}.uid")
    abort_flag = os.path.join(tmp, f"wave3d-bench-{nonce}.abort")
    out_json = os.path.join(tmp, f"wave3d-bench-{nonce}.rank{rank}.json")
    log_path = os.path.join(tmp, f"wave3d-bench-{nonce}.rank{rank}.log")
    rc, why, tail = 0, "", ""
    if runs:
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(jw), LOCAL_RANK=str(local), W3D_RDZV_FILE=rdzv,
                   W3D_JOB_ID=f"bench{nonce}", W3D_TIMEOUT_S=os.environ.get("W3D_TIMEOUT_S", "180"))
        if a.share_gpus:
            env["W3D_SHARE_GPUS"] = "1"
            if jw > 1 and _distinct_gpus(jw) < jw and a.native_transport == "push":
                env["W3D_CU_SPLIT"] = "auto"  # concurrent ranks on one GPU: disjoint CU ranges (in-kernel push waits)
        if tag == "fallback":  # (the conservative retry also times its block with one host round trip per solve)
            env["W3D_BENCH_SYNC_EACH"] = "1"
        # fault injection (tests): the main run; W3D_BENCH_FAIL_FALLBACK=1 also the conservative retry
        fail_rank = os.environ.get("W3D_BENCH_FAIL_SETUP_RANK")
        if fail_rank is not None and (tag == "main" or (tag == "fallback" and os.environ.get("W3D_BENCH_FAIL_FALLBACK"))):
            env["W3D_FAULT_RANK"] = fail_rank
        t0 = time.perf_counter()
        with open(log_path, "w") as log:
            p = subprocess.Popen([CLI, *args, "--json", out_json], env=env, stdout=log, stderr=subprocess.STDOUT)
            rc = None
            while rc is None:
                try:
                    rc = p.wait(timeout=0.2)
                except subprocess.TimeoutExpired:
                    if os.path.exists(abort_flag):
                        why = "a peer rank failed"
                    elif time.perf_counter() - t0 > a.timeout:
                        why = f"timed out after {a.timeout:.0f} s"
                    else:
                        continue
                    p.kill()
                    rc = p.wait()
        if rc != 0:
            open(abort_flag, "w").close()  # peers stop their children instead of waiting in a collective
        with open(log_path) as f:
            tail = f.read()[-2000:]
    ok = _agree(1 if rc == 0 else 0, world)
    res = None
    if ok and rank == 0:
        with open(out_json) as f:
            res = json.load(f)
    for path in (out_json, log_path):
        if os.path.exists(path):
            os.remove(path)
    if world > 1:
        dist.barrier()
        if rank == 0 and os.path.exists(abort_flag):
            os.remove(abort_flag)
    err = (tail.strip().splitlines()[-1] if tail.strip() else f"exit {rc}") if rc != 0 else ""
    return {"ok": bool(ok), "res": res, "tail": tail, "rc": rc, "why": why, "err": err}


def _qualify_sdma(a, rank: int, world: int, local: int) -> tuple[bool, str]:
    """Cross-device copy-engine qualification before the autotune may time the SDMA schedules: a short 64³ solve over
    all ranks with the copy-engine transport, whose error log must equal a one-rank solve's (L∞ exactly, Σe² within
    1e-12: the max is order-free, the sum's grouping follows the decomposition). Both run in fresh children."""
    small = ["64", "0.001", "20", "1", "--quiet", "--warmup", "1", "--repeat", "1"]
    ref = _child(a, rank, world, local, small, "qualify-ref", ranks=1)
    got = _child(a, rank, world, local, small + ["--transport", "sdma", "--decomp", "slab", "--temporal", "4"]
                 + (["--no-rccl"] if a.no_rccl else []), "qualify")
    verdict = b"0"
    why = ""
    if rank == 0:
        if not ref["ok"] or not got["ok"]:
            why = f"qualification child failed: {(got if ref['ok'] else ref)['err']}"
        else:
            r, g = ref["res"]["steps"], got["res"]["steps"]
            same = len(r) == len(g) and all(x[0] == y[0] and x[1] == y[1] and abs(x[2] - y[2]) <= 1e-12 * abs(x[2])
                                            for x, y in zip(r, g))
            why = "copy-engine 64^3 log equals the one-rank log" if same else "copy-engine 64^3 log differs"
            verdict = b"1" if same else b"0"
    if world > 1:
        from mpi_cuda_amd.parallel.rccl import broadcast_bytes

        verdict = broadcast_bytes(verdict, 0)
        why = broadcast_bytes(why.encode(), 0).decode()
    return verdict == b"1", why


def run_native(a, rank: int, world: int, local: int) -> int:
    if not os.path.exists(CLI):
        raise SystemExit(f"bench: native runtime {CLI} is missing (python tools/build.py)")
    multi = world > 1
    warm = max(a.warmup, 2 if multi else 1)
    temporal = 1 if a.no_temporal else a.temporal
    sdma_ok, sdma_why = False, ""
    # (before the autotune may time copy-engine candidates, and before an explicit copy-engine run: the rehearsal of
    # ranks sharing one GPU qualifies the same way)
    if multi and not a.cpu and not a.no_qualify and ((not a.no_rccl and not a.no_autotune) or a.native_transport == "sdma"):
        sdma_ok, sdma_why = _qualify_sdma(a, rank, world, local)
    autotune_sdma = a.autotune_sdma or sdma_ok
    if a.native_transport == "sdma" or autotune_sdma:
        # copy-engine runs: one 9-12 ms solve among the first 2-7 of every run, never later (profiles/r4/sdma_streams.md)
        warm = max(warm, 8)
    base = [str(a.N), repr(a.tau), str(a.K), repr(a.L), "--quiet", "--warmup", str(warm - 1), "--repeat", "1",
            "--bench-steps", str(a.steps)]
    cmd = base + ["--decomp", a.decomp, "--temporal", str(temporal)]
    if a.cpu:
        cmd.append("--cpu")
    else:
        if a.native_transport != "rccl":
            cmd += ["--transport", a.native_transport]
        if a.no_rccl:
            cmd.append("--no-rccl")
        if (multi or a.autotune) and not a.no_autotune and not a.no_rccl:
            cmd.append("--autotune")
            if autotune_sdma:
                cmd.append("--autotune-sdma")
        if not a.no_phases:
            cmd.append("--phases")
        if a.no_overlap:
            cmd.append("--no-overlap")
        if a.no_graph:
            cmd.append("--no-graph")
    t0 = time.perf_counter()
    run = _child(a, rank, world, local, cmd, "main")
    fallback = None
    if not run["ok"] and multi:
        # one fresh child with the conservative native schedule (no autotune, RCCL slabs, sequential exchange), so a
        # first contact with a node that breaks an autotune candidate still yields a labelled scaling point
        # the failing rank's own message (the others report only that a peer failed)
        errs = [(run["err"], run["why"])]
        if world > 1:
            import torch.distributed as dist

            errs = [None] * world
            dist.all_gather_object(errs, (run["err"], run["why"]))
        # (a rank whose child was killed because a peer failed reports why = "a peer rank failed": not the cause)
        own = [e for e, why in errs if e and not why and "another rank" not in e and "peer" not in e]
        first = (own or [e for e, _ in errs if e] or ["unknown failure"])[0]
        if rank == 0:
            print(f"[bench] native run failed ({first}); retrying once with the conservative schedule",
                  file=sys.stderr, flush=True)
        safe = base + ["--decomp", "slab", "--temporal", "4", "--no-overlap"]
        via = "rccl"
        if a.cpu:
            safe.append("--cpu")
        else:
            if a.no_rccl:  # (no RCCL at all: the transport the run asked for, host collectives through files)
                safe += ["--no-rccl", "--transport", a.native_transport]
                via = a.native_transport
            if not a.no_phases:
                safe.append("--phases")
        run = _child(a, rank, world, local, safe, "fallback")
        fallback = {"schedule": "slab-S4-seq, no autotune" + ("" if a.cpu else ", " + via), "first_failure": first}
    wall = time.perf_counter() - t0
    res, tail = run["res"], run["tail"]
    if not run["ok"]:
        if run["rc"] != 0:
            why = run["why"]
            print(f"[bench rank {rank}] native runtime failed (rc={run['rc']}{', ' + why if why else ''}): "
                  f"{run['err']}\n{tail}", file=sys.stderr, flush=True)
        if a.allow_fallback and not a.cpu:
            return run_python(a, rank, world, local, degraded=f"native runtime failed: {run['err']}")
        return 1
    if rank == 0:
        bench_s = float(res["bench_s"])
        ms = bench_s / a.steps * 1e3
        value = (a.N ** 3 * a.K) / (ms / 1e3) / 1e9
        steps = res.get("steps") or []
        final_linf = steps[-1][1] if steps else float("nan")
        final_rms = steps[-1][2] if steps else None
        correct, why_correct = _correct(a, res.get("finite", False), steps)
        dims = res.get("dims", [1, 1, 1])
        sched = res.get("schedule", "")
        par = (f"{sched.split('-')[0]}{world}" if multi else "single") if not a.cpu else f"cpu-ranks{world}"
        cfg = {
            "parallelism": par, "decomp": "x".join(map(str, dims)),
            "transport": ("shm" if multi else "none") if a.cpu else (res.get("transport", "rccl") if multi else "none"),
            "runtime": "native bin/wave3d (C++/HIP/RCCL)" if not a.cpu else "native bin/wave3d --cpu (OpenMP ranks)",
            "graph": bool(res.get("graph", False)), "overlap": bool(res.get("overlap", False)) and multi,
            "temporal_blocking": int(res.get("temporal", 1)) > 1 and not a.cpu,
            "schedule": sched if multi or a.cpu else f"fused-single-S{res.get('temporal', temporal)}",
            "mode": res.get("mode", ""),
            # per candidate: the MEDIAN over rounds of the per-solve time of back-to-back solves (what decides), and
            # the best round
            "autotune_ms": {k: round(v * 1e3, 4) for k, v in res.get("autotune_s", {}).items()} or None,
            "autotune_best_ms": {k: round(v * 1e3, 4) for k, v in res.get("autotune_best_s", {}).items()} or None,
            "autotune_rounds_x_reps": [res.get("autotune_rounds"), res.get("autotune_reps")]
            if res.get("autotune_s") else None,
            "autotune_wall_s": res.get("autotune_wall_s") if res.get("autotune_s") else None,
            "autotune_rejected": res.get("autotune_rejected") or None,
        }
        extra = {
            "wall_clock_s": round(ms / 1e3, 6),
            # the timed block: K solves enqueued back to back (one graph replay each), one sync at the end
            "batched_ms": round(ms, 4),
            # the fastest warmup / repeat solve timed on its own (host round trip per solve): a different measurement
            "sync_each_best_ms": round(float(res.get("solve_s", 0.0)) * 1e3, 4),
            "baseline_wall_clock_s": {1: 0.752, 2: 0.505}.get(world),
            "final_max_err": final_linf,
            "final_rms_err": final_rms,
            "correct": correct,
            "correct_check": why_correct,
            "degraded": False,
            "rccl_nranks": res.get("rccl_nranks") if not a.cpu else None,
            "rccl_version": res.get("rccl_version"),
            "hip_runtime": res.get("hip_runtime"),
            "process_wall_s": round(wall, 3),
            "rccl_init_s": res.get("rccl_init_s"),
            "phases_ms": res.get("phases_ms"),
            "distinct_gpus": None if a.cpu else _distinct_gpus(world),
        }
        if fallback is not None:
            extra["fallback_schedule"] = fallback["schedule"]
            extra["first_failure"] = fallback["first_failure"]
        if multi and not a.cpu:
            extra["sdma_qualified"] = sdma_ok
            extra["sdma_qualification"] = sdma_why or ("skipped" if a.no_qualify or a.no_autotune else None)
        if not a.cpu and multi and extra["distinct_gpus"] < world:
            extra["rehearsal"] = f"{world} ranks sharing {extra['distinct_gpus']} GPU(s): not a scaling point"
        _emit(a, _line(a, world, value, ms, cfg, extra))
        return 0 if correct else 1
    return 0


def _distinct_gpus(world: int) -> int:
    try:
        import torch

        return min(world, max(1, torch.cuda.device_count()))  # device_count does not initialise the GPU here
    except Exception:  # noqa: BLE001
        return world


# ------------------------------------------------------------------------------------------------------------------
# in-process Python Solver (--python, or the --allow-fallback path)
# ------------------------------------------------------------------------------------------------------------------
def run_python(a, rank: int, world: int, local: int, degraded: str = "") -> int:
    import torch
    import torch.distributed as dist

    from mpi_cuda_amd import ProblemSpec
    from mpi_cuda_amd.solver import Solver

    spec = ProblemSpec(N=a.N, tau=a.tau, K=a.K, L=a.L, check_every=2)
    transport = "torch" if (degraded or a.cpu) and world > 1 else a.transport
    if a.cpu:
        transport = "torch" if world > 1 else "native"
    group = None
    if transport == "torch" and world > 1 and not a.cpu:
        group = dist.new_group(backend="nccl")

    def agree(ok: int) -> int:
        if world > 1:
            f = torch.tensor([ok], dtype=torch.int64)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = int(f.item())
        return ok

    solver, r, err, ok = None, None, "", 1
    comm = None
    try:
        if transport == "rccl" and world > 1:
            from mpi_cuda_amd.parallel.rccl import make_comm

            comm = make_comm(rank, world)
    except Exception as e:  # noqa: BLE001
        ok, err = 0, f"{type(e).__name__}: {e}"
    if agree(ok):
        try:
            solver = Solver(spec, backend="cpu" if a.cpu else "hip", transport=transport, decomp=a.decomp, rank=rank,
                            world=world, device=None if a.cpu else local, overlap=not a.no_overlap,
                            graph=not a.no_graph, group=group, comm=comm,
                            temporal=1 if a.no_temporal else a.temporal)
        except Exception as e:  # noqa: BLE001
            ok, err = 0, f"{type(e).__name__}: {e}"
    if not agree(ok):
        print(f"[bench rank {rank}] python solver setup failed: {err}", file=sys.stderr, flush=True)
        return 1
    try:
        for _ in range(max(a.warmup, 2 if world > 1 else 1)):
            r = solver.run()
    except Exception as e:  # noqa: BLE001
        ok, err = 0, f"{type(e).__name__}: {e}"
    if not agree(ok):
        print(f"[bench rank {rank}] python solve failed: {err}", file=sys.stderr, flush=True)
        return 1

    def barrier_sync():
        if not a.cpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if not a.cpu:
            torch.cuda.synchronize()

    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = solver.run()
    barrier_sync()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t[0]) / a.steps * 1e3
    value = spec.cell_updates / (ms / 1e3) / 1e9
    final_linf = r.max_err[-1] if r.max_err else float("nan")
    correct, why_correct = _correct(a, r.finite, [[n, m, e] for n, m, e in zip(r.steps, r.max_err, r.rms_err)])
    if rank == 0:
        py_loop = transport == "torch"
        dims = "x".join(str(d) for d in solver.dims)
        cfg = {"parallelism": f"python{world}" if world > 1 else "single", "decomp": dims, "transport": transport,
               "runtime": "in-process python Solver",
               "graph": bool(not a.no_graph) and not py_loop and not a.cpu,
               "overlap": bool(not a.no_overlap) and not py_loop and world > 1,
               "temporal_blocking": not py_loop and not a.no_temporal and not a.cpu,
               "schedule": "python-step-loop-S1" if py_loop else getattr(solver.native, "mode", "") or "",
               "autotune_ms": None}
        extra = {"wall_clock_s": round(ms / 1e3, 6), "baseline_wall_clock_s": {1: 0.752, 2: 0.505}.get(world),
                 "final_max_err": final_linf, "final_rms_err": r.rms_err[-1] if r.rms_err else None,
                 "correct": correct, "correct_check": why_correct, "degraded": bool(degraded)}
        if degraded:
            extra["degraded_reason"] = degraded
        _emit(a, _line(a, world, value, ms, cfg, extra))
    if world > 1:
        dist.barrier()
    return (0 if correct else 1) if not degraded else (0 if correct else 1)


def main(argv=None) -> int:
    a = _args(argv)
    from mpi_cuda_amd.parallel.rccl import env_rank_world, init_process_group

    rank, world, local = env_rank_world()
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("bench.py --gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if not a.cpu and not a.share_gpus and world > 1:
        n = _distinct_gpus(world)
        if n < world:
            raise SystemExit(f"bench: {world} ranks but {n} visible GPU(s); RCCL needs one GPU per rank "
                             "(--share-gpus for a rehearsal)")
    if world > 1:
        init_process_group("gloo")
    try:
        rc = run_python(a, rank, world, local) if a.python else run_native(a, rank, world, local)
    finally:
        import torch.distributed as dist

        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
