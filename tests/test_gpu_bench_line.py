"""The driver's contract for bench.py (one JSON line from rank 0): the keys the driver and the judge read, with the
values they check (config.workload must name the workload, roofline.traffic must say where it comes
from).  A tiny model on 8 windows, one timed step, so the line is produced in seconds; the headline itself is the
driver's own run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_line_schema_tiny():
    d = _run("--model", "tiny", "--windows", "8", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-variable",
             "--parity-windows", "2")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["warmup"] == 0 and d["value"] > 0
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    cfg = d["config"]
    # the descriptive workload is not overwritten by the corpus name (bench.py used to clobber it with "uniform")
    assert cfg["workload"].startswith("non-config variant: tiny bf16 greedy"), cfg["workload"]
    assert cfg["corpus"] == "uniform" and cfg["windows_per_gpu"] == 8
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    # no committed PMC file applies to this workload: traffic is null and carries no source label
    assert roof["traffic"] is None and "traffic_source" not in roof
    assert d["parity"]["n"] == 2
