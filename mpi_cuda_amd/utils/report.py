"""Reference-compatible output: per-step error lines, timing summary, JSON records.

The reference GPU program prints one line per even step (report.pdf p.15-16 §4.3.1):
``Step 2, t = 0.002000, Max Error = 3.967859e-11, L2 Error = 1.406978e-11`` — i.e. C printf
``"Step %d, t = %f, Max Error = %e, L2 Error = %e"``. The phase columns of the timing summary follow report.pdf p.16
§4.4 (compute / copy / exchange); the speedup/efficiency conventions follow readme.md:84-114 (S = T_seq/T_p,
E = S/p, p = number of ranks).
"""
from __future__ import annotations

import json
import math


def error_line(step: int, t: float, max_err: float, rms_err: float) -> str:
    return "Step %d, t = %f, Max Error = %e, L2 Error = %e" % (step, t, max_err, rms_err)


def parse_error_line(line: str):
    """Inverse of error_line: (step, t, max, rms) or None."""
    import re

    m = re.match(r"Step (\d+), t = ([-+0-9.eE]+), Max Error = ([-+0-9.eEnaif]+), L2 Error = ([-+0-9.eEnaif]+)",
                 line.strip())
    if not m:
        return None
    return int(m.group(1)), float(m.group(2)), float(m.group(3)), float(m.group(4))


def gcell_per_s(N: int, K: int, seconds: float) -> float:
    return float(N) ** 3 * K / seconds / 1e9 if seconds > 0 else math.nan


def speedup_table(t_seq: float, times: dict[int, float]) -> list[dict]:
    """Speedup S = T_seq / T_p and efficiency E = S / p per worker count (readme.md:84-100 conventions)."""
    rows = []
    for p, t in sorted(times.items()):
        s = t_seq / t
        rows.append({"p": p, "time_s": t, "speedup": s, "efficiency": s / p})
    return rows


def dumps(obj) -> str:
    return json.dumps(obj, sort_keys=False)
