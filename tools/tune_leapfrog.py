#!/usr/bin/env python3
"""Kernel-level tuning sweep for the leapfrog kernel on one GPU (HIP events, no profiler needed).

Times one leapfrog launch over the 512³ compute box for every tiling in the sweep, plus streaming baselines
measured in the same process (torch copy = 1 read + 1 write stream, torch add = 2 reads + 1 write — the stencil's
compulsory pattern) so achieved TB/s can be read against what this HBM actually delivers.

    python tools/tune_leapfrog.py [--N 512] [--iters 20] [--json out.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters: int, warm: int = 3) -> float:
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2] * 1e3  # median µs


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--minimal", action="store_true", help="only the default single-step and two-step kernels "
                    "(for counter collection under rocprofv3)")
    ap.add_argument("--tb", action="store_true", help="only the deep temporal-blocking kernel (k_leapfrog_tb) sweep "
                    "plus the default two-step kernel")
    a = ap.parse_args()
    import torch

    from mpi_cuda_amd._native import load
    from mpi_cuda_amd.ops import stencil as ops

    C = load()
    torch.cuda.set_device(0)
    prob = C.Problem(a.N, 1e-3, 20, 1.0)
    co = C.Coeffs.from_problem(prob)
    lay = C.make_layout(prob, C.rank_box(prob, C.Dims(1, 1, 1), 0))
    box = C.compute_box(lay)
    nodes = box.count()
    s = ops.sin_table_ext(prob, "cuda")
    u0, u1 = ops.alloc_field(lay, "cuda"), ops.alloc_field(lay, "cuda")
    ops.init_first(lay, co, s, u0, u1)
    torch.cuda.synchronize()
    out = []

    nbytes = int(lay.total) * 8
    x = torch.empty(int(lay.total), dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    t = timeit(lambda: y.copy_(x), a.iters)
    out.append({"kernel": "torch copy (1R+1W)", "us": t, "TBps": 2 * nbytes / t / 1e6})
    t = timeit(lambda: torch.add(x, y, out=z), a.iters)
    out.append({"kernel": "torch add (2R+1W)", "us": t, "TBps": 3 * nbytes / t / 1e6})
    t = timeit(lambda: ops.init_first(lay, co, s, u0, u1), a.iters)
    out.append({"kernel": "k_init_first (2W)", "us": t, "TBps": 2 * nbytes / t / 1e6})
    del x, y, z

    configs = []
    for ty, tb, nt in itertools.product([8, 16], [0, 1024], [False, True]):
        configs.append(dict(variant=0, ty=ty, target_blocks=tb, xcd_remap=True, nt_store=nt))
    for rows, tb, rm, nt in itertools.product([1, 2, 4, 8], [0, 2048, 8192], [True, False], [False, True]):
        configs.append(dict(variant=1, rows=rows, target_blocks=tb, xcd_remap=rm, nt_store=nt))
    if a.quick:
        configs = [c for c in configs if c["target_blocks"] == 0 and c["xcd_remap"]]
    if a.minimal:
        configs = [dict(variant=1, rows=2, target_blocks=0, xcd_remap=True, nt_store=True)]
    if a.tb:
        configs = []
    for cfg, chk in itertools.product(configs, [False, True] if not (a.quick or a.minimal) else [False]):
        tl = C.LeapfrogTiling()
        for k, v in cfg.items():
            setattr(tl, k, v)
        nb = C.gpu_leapfrog_blocks(lay, [box], tl)
        part = torch.empty((nb, 2), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def step():
            C.gpu_leapfrog(lay, co, u1.data_ptr(), u0.data_ptr(), [box], s.data_ptr(), 0.5,
                           part.data_ptr() if chk else 0, tl, st)

        t = timeit(step, a.iters)
        out.append({"kernel": "k_leapfrog", **cfg, "partials": nb, "check": chk, "us": t,
                    "TBps": 24 * nodes / t / 1e6})
    # temporally blocked two-step kernel: 32 B per node per pass = 16 B per node-step
    bufs = [ops.alloc_field(lay, "cuda") for _ in range(2)]
    sweep2 = list(itertools.product([1, 2, 4], [0, 4096, 8192, 16384], [True, False],
                                    [False, True] if not a.quick else [False]))
    if a.minimal or a.tb:
        sweep2 = [(2, 0, True, False)]
    for rows, tw, nt, chk in sweep2:
        t2 = C.Leapfrog2Tiling()
        t2.rows, t2.target_waves, t2.nt_store = rows, tw, nt
        nb = C.gpu_leapfrog2_partials(lay, box, t2)
        part = torch.empty((nb, 2), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def pass2():
            C.gpu_leapfrog2(lay, co, u0.data_ptr(), u1.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(), box,
                            s.data_ptr(), 0.5, part.data_ptr() if chk else 0, t2, st)

        t = timeit(pass2, a.iters)
        out.append({"kernel": "k_leapfrog2", "rows": rows, "target_waves": tw, "nt_store": nt, "partials": nb,
                    "check": chk, "us": t, "us_per_step": t / 2, "TBps": 32 * nodes / t / 1e6})
    # deep temporal blocking: S steps per pass, 32 B per node per pass
    sweep_tb = list(itertools.product([2, 3, 4], [512, 1024], [True, False], [False, True]))
    if a.minimal:
        sweep_tb = [(4, 1024, True, False)]
    if a.quick:
        sweep_tb = [c for c in sweep_tb if c[2] and not c[3]]
    for stages, threads, nt, chk in sweep_tb:
        tt = C.LeapfrogTbTiling()
        tt.stages, tt.threads, tt.xcd_blocks = stages, threads, nt
        nb = C.gpu_leapfrog_tb_partials(lay, box, tt)
        part = torch.empty((stages * nb, 2), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        mask = (0b1010 & ((1 << stages) - 1)) if chk else 0  # production pattern: every 2nd level checked

        def pass_tb():
            C.gpu_leapfrog_tb(lay, co, u0.data_ptr(), u1.data_ptr(), bufs[0].data_ptr(), bufs[1].data_ptr(), box,
                              s.data_ptr(), [0.5] * stages, mask, part.data_ptr() if chk else 0, tt, st)

        t = timeit(pass_tb, a.iters)
        out.append({"kernel": "k_leapfrog_tb", "stages": stages, "threads": threads, "xcd_blocks": nt, "partials": nb,
                    "check": chk, "us": t, "us_per_step": t / stages, "TBps": 32 * nodes / t / 1e6})
    # analytic-start pass (no HBM reads): u⁰, u¹ computed in the kernel; production check pattern (odd levels)
    for stages in ([4] if a.minimal else [2, 3, 4]):
        tt = C.LeapfrogTbTiling()
        tt.stages, tt.threads = stages, 1024
        nb = C.gpu_leapfrog_tb_partials(lay, box, tt)
        part = torch.empty((stages * nb, 2), dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        mask = 0b0101 & ((1 << stages) - 1)

        def pass_an():
            C.gpu_leapfrog_tb(lay, co, 0, 0, bufs[0].data_ptr(), bufs[1].data_ptr(), box, s.data_ptr(),
                              [0.5] * stages, mask, part.data_ptr(), tt, st, analytic_start=True)

        t = timeit(pass_an, a.iters)
        out.append({"kernel": "k_leapfrog_tb analytic", "stages": stages, "threads": 1024, "check": True, "us": t,
                    "us_per_step": t / stages, "TBps": 16 * nodes / t / 1e6})
    for r in out:
        print(json.dumps(r), flush=True)
    if any(r["kernel"] == "k_leapfrog" for r in out):
        best = min((r for r in out if r["kernel"] == "k_leapfrog"), key=lambda r: r["us"])
        print("BEST", json.dumps(best))
    best2 = min((r for r in out if r["kernel"] == "k_leapfrog2"), key=lambda r: r["us"])
    print("BEST2", json.dumps(best2))
    best_tb = min((r for r in out if r["kernel"] == "k_leapfrog_tb"), key=lambda r: r["us_per_step"])
    print("BEST_TB", json.dumps(best_tb))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
