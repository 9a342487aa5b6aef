#!/usr/bin/env python3
"""RCCL smoke probe: one all-reduce over ``torch.distributed`` (backend "nccl" = RCCL on ROCm).

    python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 tools/rccl_probe.py [--same-device]

``--same-device`` puts every rank on cuda:0 (checks whether this RCCL build accepts several ranks per GPU, which
would let one-GPU boxes rehearse the multi-rank RCCL halo path).
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true")
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = 0 if a.same_device else local
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    r = dist.get_rank()
    x = torch.ones(4, device="cuda") * (r + 1)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {r} device {dev} allreduce {x.tolist()}", flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
