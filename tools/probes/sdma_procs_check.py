"""Runtime check of the copy-engine transport across PROCESSES sharing one GPU: runs bin/wave3d --np P --no-rccl
--transport sdma in a few variants and compares each dumped field with the single-GPU solve (max |diff|, first plane).
Usage: python tools/probes/sdma_procs_check.py [variant ...]   (variants: graph, nograph, debugsync, poison)"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
CLI = os.path.join(ROOT, "bin", "wave3d")
N, K = 96, 20


def read(prefix, world):
    f = np.zeros((N + 1,) * 3)
    for r in range(world):
        m = json.loads(open(f"{prefix}.rank{r}.json").read())
        nx, ny, nz = m["shape"]
        x0, y0, z0 = m["offset"]
        f[x0:x0 + nx, y0:y0 + ny, z0:z0 + nz] = np.fromfile(f"{prefix}.rank{r}.bin").reshape(nx, ny, nz)
    return f


def main():
    variants = sys.argv[1:] or ["nograph", "graph"]
    tmp = tempfile.mkdtemp()
    subprocess.run([CLI, str(N), "0.001", str(K), "1", "--dump", f"{tmp}/ref", "--quiet"], check=True, timeout=60)
    m = json.loads(open(f"{tmp}/ref.json").read())
    ref = np.fromfile(f"{tmp}/ref.bin").reshape(m["shape"])
    extra = {"graph": [], "nograph": ["--no-graph"], "debugsync": ["--debug-sync"], "poison": ["--poison-ghosts"],
             "seq": ["--no-overlap"], "seqnograph": ["--no-overlap", "--no-graph"], "one": ["--repeat", "1"]}
    env = dict(os.environ, W3D_SHARE_GPUS="1", W3D_TIMEOUT_S="20")
    env.pop("W3D_RDZV_FILE", None)
    for v in variants:
        for np_ in (2,):
            pre = f"{tmp}/{v}{np_}"
            cmd = [CLI, str(N), "0.001", str(K), "1", "--np", str(np_), "--transport", "sdma", "--no-rccl",
                   "--repeat", "3", "--dump", pre, "--json", pre + ".json", *extra[v]]
            p = subprocess.run(cmd, timeout=120, env=env, capture_output=True, text=True)
            if p.returncode != 0:
                print(v, np_, "rc", p.returncode, p.stderr[-800:], flush=True)
                continue
            f = read(pre, np_)
            d = np.abs(f - ref)
            bad = np.argwhere(d > 0)
            print(f"{v} P={np_}: max|diff| {d.max():.3e}, {len(bad)} nodes differ" +
                  (f", x planes {sorted(set(bad[:, 0].tolist()))[:12]}" if len(bad) else ""), flush=True)
            print("   log:", [s for s in p.stdout.splitlines() if s.startswith("Step 20") or "Total" in s], flush=True)


if __name__ == "__main__":
    main()
