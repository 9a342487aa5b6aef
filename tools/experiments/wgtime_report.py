#!/usr/bin/env python3
"""Per-workgroup timeline of the pair-tiled passes from a W3D_EXPERIMENT_WGTIME build (W3D_WGTIME_OUT file): for each
launch (the last replay of a captured one) the dispatch skew, prologue, march and finish spread in µs."""
import sys


def load(path):
    out, cur = [], None
    for line in open(path):
        f = line.split()
        if f[0] == "launch":
            cur = {"S": int(f[2]), "init": int(f[3]), "wg": []}
            out.append(cur)
        else:
            cur["wg"].append([int(x) for x in f])
    return out


def main():
    for path in sys.argv[1:]:
        print(path)
        print("launch S init  wgs  total  entry-skew  prologue(avg/max)  march(min/avg/max)  exit-spread  tail(last exit - "
              "median exit)")
        for i, L in enumerate(load(path)):
            w = [r for r in L["wg"] if all(r)]
            if not w:
                continue
            us = 0.01  # 100 MHz clock
            t0 = min(r[0] for r in w)
            ent = sorted(r[0] for r in w)
            pro = [r[1] - r[0] for r in w]
            mar = [r[2] - r[1] for r in w]
            ex = sorted(r[3] for r in w)
            print(f"{i:5d} {L['S']} {L['init']:4d} {len(w):5d} {(ex[-1] - t0) * us:7.1f} {(ent[-1] - ent[0]) * us:10.1f}"
                  f"   {sum(pro) / len(pro) * us:6.1f}/{max(pro) * us:6.1f}"
                  f"   {min(mar) * us:6.1f}/{sum(mar) / len(mar) * us:6.1f}/{max(mar) * us:6.1f}"
                  f"   {(ex[-1] - ex[0]) * us:8.1f}   {(ex[-1] - ex[len(ex) // 2]) * us:8.1f}")


if __name__ == "__main__":
    main()
