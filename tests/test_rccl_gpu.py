"""The RCCL ("nccl") branches of the distributed layers on real hardware, world size 1 (one
GPU per rank: the box has one).  The gloo tests cover the partition logic over 2-3 ranks;
these run the code that only the nccl backend takes:
  * ToeplitzPlan.pcg_allranks -- the break flag stays on the device (hgp_pcg_local_flag, an
    RCCL all-reduce on the stream, hgp_pcg_set_done), no host synchronisation per iteration;
  * hdist.sharded_elbo_and_grad -- stats all-reduced in place on the device (G5 fixture);
  * the slab (grid-block) layer -- RCCL all-to-all transposes and all-reduced CG dots.
Each case runs in a spawned process (init/destroy of the process group stays out of pytest)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_cases import load, rel_err
from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu


def _model(fx, dtype=torch.float64):
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    k = zk.Matern(nu=1.5, dtype=dtype)
    grids = [torch.tensor(fx["grid0"], dtype=dtype), torch.tensor(fx["grid1"], dtype=dtype)]
    mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=64, sig2_init=1., ell_init=.1, noise2_init=.01,
                                 learn_kernel=False, dtype=dtype)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["theta1"], dtype=dtype))
        mod.global_theta2.copy_(torch.tensor(fx["theta2"], dtype=dtype))
    return mod.cuda_params(0)


def _column(dims):
    grids = [np.linspace(-1, 1, m) for m in dims]
    return zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.05)


def _worker(rank, port, what, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        from hipgp_amd import _lib
        if what == "pcg":
            from hipgp_amd.plan import ToeplitzPlan
            dims = (96, 80)
            P = ToeplitzPlan(dims, torch.float64, "cuda")
            P.set_column(torch.tensor(_column(dims), device="cuda"))
            g = torch.Generator(device="cuda").manual_seed(3)
            b = torch.randn(5, int(np.prod(dims)), device="cuda", generator=g, dtype=torch.float64)
            x, it = P.pcg_allranks(b, 200, 1e-7, precond=True)
            x0, it0 = P.pcg(b, 200, 1e-7, precond=True, return_iters=True)
            torch.cuda.synchronize()
            out["pcg"] = (x.cpu().numpy(), it, x0.cpu().numpy(), it0)
        elif what == "elbo":
            from hipgp_amd import dist as hdist
            fx = load("G5", "f64")
            mod = _model(fx)
            x = torch.tensor(fx["xobs"], device="cuda")
            y = torch.tensor(fx["yobs"], device="cuda")
            elbo = hdist.sharded_elbo_and_grad(mod, x, y, maxiter_cg=20, exact_break=True)
            torch.cuda.synchronize()
            out["elbo"] = (float(elbo), mod.global_theta1.grad.cpu().numpy(), mod.global_theta2.grad.cpu().numpy())
        else:
            from hipgp_amd.plan import ToeplitzPlan
            from hipgp_amd.slab import slab_toeplitz
            dims, dt = ((64, 48), torch.float64) if what == "slab2" else ((16, 12, 10), torch.float64)
            col = torch.tensor(_column(dims), device="cuda", dtype=dt)
            S = slab_toeplitz(dims, col, dtype=dt, device="cuda")
            P = ToeplitzPlan(dims, dt, "cuda")
            P.set_column(col)
            M = int(np.prod(dims))
            g = torch.Generator(device="cuda").manual_seed(9)
            v = torch.randn(3, M, device="cuda", generator=g, dtype=dt)
            errs = {}
            for name, op in (("K", _lib.OP_K), ("Cinv", _lib.OP_CINV), ("RT", _lib.OP_RT)):
                got = S.apply(op, S.scatter_rows(v, "m")).double().cpu().numpy()
                ref = P.apply(op, v).double().cpu().numpy()
                errs[name] = float(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))
            xs, _ = S.pcg(S.scatter_rows(v), maxiter=10, tol=1e-30)
            xr = P.pcg(v, 10, 1e-30, precond=True)
            errs["pcg"] = float(np.linalg.norm(xs.double().cpu().numpy() - xr.cpu().numpy()) /
                                np.linalg.norm(xr.cpu().numpy()))
            torch.cuda.synchronize()
            out[what] = errs
    finally:
        dist.destroy_process_group()


def _run(what):
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29400 + os.getpid() % 300 + len(what)
    mp.spawn(_worker, args=(port, what, out), nprocs=1, join=True)
    return out[what]


def test_rccl_pcg_allranks_device_flag():
    """Device-side break flag through an RCCL all-reduce == the single-plan PCG: same iterate,
    same iteration count (cg.py:69-71 break rule)."""
    x, it, x0, it0 = _run("pcg")
    assert it == it0 and 1 < it < 200, (it, it0)
    assert np.max(np.abs(x - x0)) <= 1e-12 * np.max(np.abs(x0))


def test_rccl_sharded_elbo_G5():
    """RHS-sharded ELBO / natural gradients with RCCL reductions against the reference's G5."""
    fx = load("G5", "f64")
    elbo, g1, g2 = _run("elbo")
    assert abs(elbo - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
    assert rel_err(g1, fx["theta1_grad"]) < 1e-7
    assert rel_err(g2, fx["theta2_grad"]) < 1e-7


@pytest.mark.parametrize("what", ["slab2", "slab3"])
def test_rccl_slab_ops_and_pcg(what):
    """Grid-block layer with RCCL transposes / dot all-reduces == the plan (fp64 rounding)."""
    errs = _run(what)
    for k, e in errs.items():
        assert e < (1e-9 if k == "pcg" else 1e-11), (k, e)
