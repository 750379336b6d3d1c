"""bench.py's one-GPU line (the driver's contract) on the benchmarked workload, short: one warmup and one
timed move of 4096 games x 25 sims, a tiny CPU-baseline sample.  The JSON line carries every field the
contract names, the roofline of the dominant kernel with its PMC traffic, the CPU baseline, the tree and
transform rooflines, and values in their physical ranges."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--generation", "off",
           "--learn-iteration", "off", "--cpu-moves", "3", "--cpu-proc-moves", "2", "--cpu-procs", "2"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=150, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 1 and out["warmup"] == 1 and out["higher_is_better"]
    assert out["scaling"] == "weak" and out["vs_baseline"] is None
    assert out["config"]["games_per_gpu"] == 4096 and out["config"]["sims_per_move"] == 25
    assert "workload" in out["config"]
    # ~4096 x 25 expansions in one timed move
    assert 0.95 * 4096 * 25 <= out["expansions"] <= 4096 * 25
    assert 1.0e6 < out["value"] < 5.0e6
    rf = out["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 2500.0
    assert 0.2 < rf["frac"] < 1.0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert rf["traffic"] is not None and 0.8e9 < rf["traffic"] < 1.2e9  # PMC bytes per GEMM launch
    for k in ("roofline_tree", "roofline_transforms"):
        assert out[k]["bound"] == "hbm" and 0 < out[k]["frac"] < 1 and out[k]["traffic"] is not None
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["sample"]
