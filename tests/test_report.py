"""utils/report.py and tools/scaling_report.py: reference output conventions (report.pdf p.15-17, readme.md:84-114)."""
import json
import os
import subprocess
import sys

import pytest

from mpi_cuda_amd.utils.report import error_line, gcell_per_s, parse_error_line, speedup_table

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_error_line_format_roundtrip():
    line = error_line(2, 0.002, 3.967859e-11, 1.406978e-11)
    assert line == "Step 2, t = 0.002000, Max Error = 3.967859e-11, L2 Error = 1.406978e-11"
    assert parse_error_line(line) == (2, 0.002, 3.967859e-11, 1.406978e-11)
    assert parse_error_line("Total time: 1 s") is None


def test_speedup_conventions():
    # readme.md:99-100: GPU speedups vs the 21.98 s sequential run, efficiency divided by the number of ranks
    rows = speedup_table(21.98, {1: 0.752, 2: 0.505})
    assert abs(rows[0]["speedup"] - 29.23) < 0.01 and abs(rows[1]["speedup"] - 43.52) < 0.01
    assert abs(rows[1]["efficiency"] - 21.76) < 0.01
    assert abs(gcell_per_s(512, 20, 0.752) - 3.570) < 1e-3


def test_scaling_report_table(tmp_path):
    p = tmp_path / "s.jsonl"
    rows = [{"n_gpus": 1, "ms_per_step": 9.0, "value": 298.0}, {"n_gpus": 2, "ms_per_step": 5.0, "value": 536.0}]
    p.write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling_report.py"), str(p)], check=True,
                         capture_output=True, text=True).stdout
    assert "| 2 | 0.00500 |" in out and "1.80" in out and "101.0x" in out


def test_scaling_report_plot(tmp_path):
    """--plot writes the reference-style speedup / efficiency figure (iamge1.png analogue) for both row kinds."""
    pytest.importorskip("matplotlib")
    g = tmp_path / "g.jsonl"
    g.write_text("\n".join(json.dumps(r) for r in [{"n_gpus": 1, "ms_per_step": 5.3, "value": 506.0},
                                                     {"n_gpus": 2, "ms_per_step": 3.1, "value": 866.0}]) + "\n")
    c = tmp_path / "c.jsonl"
    c.write_text("\n".join(json.dumps({"mode": m, "N": 128, "workers": w, "solve_s": 1.0 / w ** 0.9,
                                       "gcell_per_s": 0.1 * w}) for m in ("openmp", "mpi") for w in (1, 2, 4)) + "\n")
    for src in (g, c):
        png = tmp_path / (src.stem + ".png")
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling_report.py"), str(src), "--plot",
                              str(png)], check=True, capture_output=True, text=True).stdout
        assert "figure:" in out and png.stat().st_size > 1000


def test_scaling_report_reads_driver_scale_record(tmp_path):
    """A driver SCALE record (bench lines nested per GPU count, repeated under "parsed" and "run") gives one row per
    GPU count, the speedup/efficiency table, the per-phase breakdown and the figure."""
    def line(n, ms):
        return {"metric": "gcell_updates_per_s_512cube_K20", "n_gpus": n, "ms_per_step": ms,
                "value": 512 ** 3 * 20 / (ms / 1e3) / 1e9, "config": {"schedule": "slab-S4" if n > 1 else "fused"},
                "phases_ms": {"compute": ms * 0.9, "shell": 0.1 if n > 1 else 0, "exchange": 0.05 * (n > 1),
                              "check": 0.02, "gather": 0.01}}
    rec = {"runs": {str(n): {"parsed": line(n, ms), "run": {"stdout": "...", "parsed": line(n, ms)}}
                    for n, ms in ((1, 4.97), (2, 2.6), (4, 1.4), (8, 0.9))}}
    p = tmp_path / "SCALE_r02.json"
    p.write_text(json.dumps(rec))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling_report

    rows = scaling_report.load(str(p))
    assert sorted(r["n_gpus"] for r in rows) == [1, 2, 4, 8]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling_report.py"), str(p)], check=True,
                         capture_output=True, text=True).stdout
    assert "| 8 | 0.00090 |" in out and "Phase breakdown" in out and "| 8 | slab-S4 |" in out
    pytest.importorskip("matplotlib")
    png = tmp_path / "scale.png"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "scaling_report.py"), str(p), "--plot", str(png)],
                   check=True, capture_output=True)
    assert png.stat().st_size > 1000


def test_projection_figure(tmp_path, capsys):
    """tools/projection_figure.py: per-P max over sampled ranks, fastest schedule per P, speedup/efficiency vs 1 GPU."""
    lines = [{"P": 1, "rank": 0, "solve_s": 0.005},
             {"P": 2, "schedule": "slab-seq", "rank": 0, "solve_s": 0.0026},
             {"P": 2, "schedule": "slab-seq", "rank": 1, "solve_s": 0.0025},
             {"P": 8, "schedule": "slab-seq", "rank": 1, "solve_s": 0.0008},
             {"P": 8, "schedule": "block-seq", "rank": 0, "solve_s": 0.0009}]
    src = tmp_path / "fs.jsonl"
    src.write_text("\n".join(json.dumps(x) for x in lines) + "\n")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import projection_figure

    rows = projection_figure.table(projection_figure.load(str(src)))
    assert [r["P"] for r in rows] == [1, 2, 8]
    assert rows[1]["t"] == 0.0026  # max over ranks
    assert rows[2]["schedule"] == "slab-seq" and abs(rows[2]["speedup"] - 6.25) < 1e-9
    assert abs(rows[2]["eff"] - 6.25 / 8) < 1e-9
    fig = tmp_path / "p.png"
    assert projection_figure.main([str(src), "--plot", str(fig)]) == 0
    assert fig.stat().st_size > 1000
    assert "compute only" in capsys.readouterr().out


def test_trace_overlap_copy_volume(tmp_path):
    """tools/trace_overlap.py: the ROCm 7.2 memory-copy CSV has no size column, so the volume comes from the solver's
    --json halo_bytes x solves (it printed 0.0 MB); a CSV with a size column is summed."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
    import trace_overlap as t

    d = tmp_path / "tr"
    d.mkdir()
    (d / "run_kernel_trace.csv").write_text(
        "Kernel_Name,Start_Timestamp,End_Timestamp\n"
        "k_leapfrog_tb<4>,100,200\n"
        "k_box_copy,200,210\n")
    (d / "run_memory_copy_trace.csv").write_text(
        "Kind,Direction,Start_Timestamp,End_Timestamp\n"
        "MEMORY_COPY,MEMORY_COPY_DEVICE_TO_DEVICE,150,250\n")
    r = t.analyse(str(d))
    assert r["copies"] == 1 and r["copy_ns"] == 100 and r["copy_ns_during_pass"] == 50
    assert r["copy_bytes"] is None
    j = tmp_path / "run.json"
    j.write_text(json.dumps({"halo_bytes": 2.5e6}))
    assert t.copy_volume(r, str(j), 4).startswith("10.0 MB")
    assert "not in the trace" in t.copy_volume(r, None, None)
    (d / "run_memory_copy_trace.csv").write_text(
        "Kind,Direction,Start_Timestamp,End_Timestamp,Bytes\n"
        "MEMORY_COPY,MEMORY_COPY_DEVICE_TO_DEVICE,150,250,3000000\n")
    r = t.analyse(str(d))
    assert t.copy_volume(r, None, None) == "3.0 MB (trace)"
