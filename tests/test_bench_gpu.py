"""bench.py end to end on the GPU (a short run): one JSON line with the driver's contract fields,
the roofline block of the batched K matvec (frac below 1, PMC traffic from the committed summary)
and the per-pass HIP-event times -- so a change that breaks the driver's bench line fails here
first."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--pcg-reps", "1", "--settle-s", "0", "--no-cpu-baseline", "--no-legs"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "pcg_wall_clock_ms"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] < 1 and r["peak"] == 8000.0
    assert abs(r["achieved"] - r["bytes_per_launch"] / (d["ms_per_step"] * 1e-3) / 1e9) < 1e-6 * r["achieved"]
    assert r["traffic"] is not None and r["traffic"] > r["bytes_per_launch"]
    assert len(r["passes"]) == 3 and all(ps["ms"] > 0 for ps in r["passes"])
    assert d["config"]["workload"].startswith("C2")
