"""bench.py's rank launch contract (no GPU needed): `--gpus N` without a torch.distributed
environment starts N ranks itself, a rank process runs, and WORLD_SIZE != --gpus is refused
before anything touches the GPU."""
import os
import subprocess
import sys
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_plan_single_gpu_runs_in_process():
    assert bench.launch_plan(SimpleNamespace(gpus=1), {}) == ("run", None)


def test_launch_plan_starts_n_ranks():
    what, cmd = bench.launch_plan(SimpleNamespace(gpus=4), {})
    assert what == "launch"
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert os.path.basename(cmd[cmd.index("--master-port") + 2]) == "bench.py"


def test_launch_plan_rank_process_runs():
    assert bench.launch_plan(SimpleNamespace(gpus=8), {"WORLD_SIZE": "8"}) == ("run", None)


@pytest.mark.parametrize("gpus, ws", [(2, "3"), (1, "2"), (8, "1")])
def test_launch_plan_refuses_mismatch(gpus, ws):
    what, why = bench.launch_plan(SimpleNamespace(gpus=gpus), {"WORLD_SIZE": ws})
    assert what == "refuse" and f"WORLD_SIZE={ws}" in why


def test_bench_refuses_world_size_mismatch_exit_code():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr
    assert "refusing" in p.stderr and "WORLD_SIZE=3" in p.stderr


def test_empty_shard_reports_every_phase():
    """The bench's config-4 leg barriers inside sharded_compute_kn's phase hook: a rank with no
    right-hand sides must report the same phases as the others, or the barriers would not pair."""
    import torch
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    from hipgp_amd.dist import sharded_compute_kn
    grids = [torch.linspace(-1, 1, 6), torch.linspace(-1, 1, 5)]
    mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=1.5, dtype=torch.float32), grids, num_obs=10, learn_kernel=False,
                                 dtype=torch.float32)
    seen = []
    kn = sharded_compute_kn(mod, torch.zeros(0, mod.M), exact_break=False, on_phase=seen.append)
    assert kn.shape == (0, mod.Mprime)
    assert seen == ["setup", "pcg", "rt"]
