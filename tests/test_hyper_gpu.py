"""Kernel / noise hyper-parameter learning through `elbo_and_grad` on the GPU (learn_kernel and
learn_noise set): the ELBO carries the autograd graph to log_sig2 / log_ell / log_noise2 through
Knm, Knn, the PCG solve (InvMatmul.backward -> hgp_plan_dqf) and the R^T whitening
(hgp_plan_column_grad), as the reference's fit loop needs (`svi_gp.py:317-326`).  Checked
against G16 (mean-field) / G17 (block) made by running the reference's own
`elbo_and_grad(...).backward()` (tests/golden/make_golden_elbo_grad.py); and the RHS-sharded
version over 2 processes on one GPU (gloo), whose summed shares equal the single process."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_cases import load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
HYPER = ("log_sig2_grad", "log_ell_grad", "log_noise2_grad")


def _model(fx, family, dtype):
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    k = zk.Matern(nu=1.5, dtype=dtype)
    grids = [torch.tensor(fx["grid0"], dtype=dtype), torch.tensor(fx["grid1"], dtype=dtype)]
    kw = dict(sig2_init=1.2, ell_init=.3, noise2_init=.05, learn_kernel=True, learn_noise=True, dtype=dtype)
    if family == "G16":
        mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=400, **kw)
    else:
        mod = hg.BlockToeplitzGP(k, grids, num_obs=400, block_sizes=[2, 3], **kw)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["theta1"], dtype=dtype))
        mod.global_theta2.copy_(torch.tensor(fx["theta2"], dtype=dtype))
    return mod.cuda_params(0)


def _hyper(mod):
    return np.array([float(mod.log_sig2.grad), float(mod.log_ell.grad), float(mod.log_noise2.grad)])


@pytest.mark.parametrize("name", ["G16", "G17"], ids=["mean_field", "block"])
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_elbo_hyper_grads_vs_reference(name, tag):
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx = load(name, tag)
    f64 = load(name, "f64")
    mod = _model(fx, name, dtype)
    x = torch.tensor(fx["xobs"], device=DEV)
    y = torch.tensor(fx["yobs"], device=DEV)
    elbo = mod.elbo_and_grad(x, y, maxiter_cg=20)
    assert elbo.requires_grad
    elbo.backward()
    g = _hyper(mod)
    ref64 = np.array([float(f64[k]) for k in HYPER])
    if tag == "f64":
        assert abs(float(elbo) - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
        assert rel_err(mod.global_theta1.grad.cpu().numpy(), fx["theta1_grad"]) < 1e-7
        assert rel_err(mod.global_theta2.grad.cpu().numpy(), fx["theta2_grad"]) < 1e-7
        assert np.all(np.abs(g - ref64) <= 1e-6 * np.abs(ref64) + 1e-9), (g, ref64)
    else:
        ref32 = np.array([float(fx[k]) for k in HYPER])
        # fp32: no worse than 4x the reference's own fp32 error vs fp64 per
        # hyper-parameter, with a 1e-5 relative floor
        e_me, e_ref = np.abs(g - ref64), np.abs(ref32 - ref64)
        assert np.all(e_me <= 4 * e_ref + 1e-5 * np.abs(ref64)), (g, ref32, ref64)
        assert abs(float(elbo) - float(f64["elbo"])) < 1e-4 * abs(float(f64["elbo"]))


def test_no_graph_without_hyper_learning():
    """learn_kernel = learn_noise = False: the natural-gradient-only ELBO (no graph, no solve
    backward), exactly the round-1 value path."""
    fx = load("G16", "f64")
    mod = _model(fx, "G16", torch.float64)
    mod.learn_kernel = False
    mod.log_noise2.requires_grad_(False)
    assert not mod.hyper_grad_needed()
    elbo = mod.elbo_and_grad(torch.tensor(fx["xobs"], device=DEV), torch.tensor(fx["yobs"], device=DEV),
                             maxiter_cg=20)
    assert not elbo.requires_grad


def _worker(rank, world_size, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        torch.cuda.set_device(0)
        fx = load("G16", "f64")
        mod = _model(fx, "G16", torch.float64)
        x = torch.tensor(fx["xobs"], device=DEV)
        y = torch.tensor(fx["yobs"], device=DEV)
        elbo = hdist.sharded_elbo_and_grad(mod, x, y, maxiter_cg=20, exact_break=False)
        elbo.backward()
        hdist.allreduce_hyper_grads(mod)
        out[rank] = (float(elbo), mod.global_theta1.grad.cpu().numpy(), _hyper(mod))
    finally:
        dist.destroy_process_group()


def test_sharded_hyper_grads_two_ranks():
    fx = load("G16", "f64")
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29900 + os.getpid() % 90
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    ref = np.array([float(fx[k]) for k in HYPER])
    for r in range(2):
        elbo, g1, gh = out[r]
        assert abs(elbo - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
        assert rel_err(g1, fx["theta1_grad"]) < 1e-7
        assert np.all(np.abs(gh - ref) <= 1e-6 * np.abs(ref) + 1e-9), (gh, ref)


def _worker_exact(rank, world_size, port, out, nobs):
    """The default exact_break (on for fp64): the all-ranks break rule in the forward AND the
    backward solve (AllRanksInvMatmul), with the kernel hyper-parameters learned."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        torch.cuda.set_device(0)
        fx = load("G16", "f64")
        mod = _model(fx, "G16", torch.float64)
        x = torch.tensor(fx["xobs"], device=DEV)[:nobs]
        y = torch.tensor(fx["yobs"], device=DEV)[:nobs]
        elbo = hdist.sharded_elbo_and_grad(mod, x, y, maxiter_cg=20)
        assert elbo.requires_grad, "the exact-break kn must carry the autograd graph (ADVICE r2)"
        elbo.backward()
        hdist.allreduce_hyper_grads(mod)
        out[rank] = (float(elbo), mod.global_theta1.grad.cpu().numpy(), _hyper(mod))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size,nobs", [(2, 40), (3, 2)])
def test_sharded_hyper_grads_exact_break(world_size, nobs):
    """fp64 with the default exact_break: every rank's ELBO, natural gradient and summed
    hyper-parameter gradients equal the single-process values (G16 itself for the full batch;
    for a 2-row minibatch on 3 ranks -- one empty shard -- the single-process GPU run)."""
    fx = load("G16", "f64")
    if nobs == 40:
        ref_elbo, ref_g1 = float(fx["elbo"]), fx["theta1_grad"]
        ref_h = np.array([float(fx[k]) for k in HYPER])
    else:
        mod = _model(fx, "G16", torch.float64)
        x = torch.tensor(fx["xobs"], device=DEV)[:nobs]
        y = torch.tensor(fx["yobs"], device=DEV)[:nobs]
        e = mod.elbo_and_grad(x, y, maxiter_cg=20)
        e.backward()
        ref_elbo, ref_g1, ref_h = float(e), mod.global_theta1.grad.cpu().numpy(), _hyper(mod)
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29800 + os.getpid() % 90 + world_size
    mp.spawn(_worker_exact, args=(world_size, port, out, nobs), nprocs=world_size, join=True)
    for r in range(world_size):
        elbo, g1, gh = out[r]
        assert abs(elbo - ref_elbo) < 1e-8 * abs(ref_elbo)
        assert rel_err(g1, ref_g1) < 1e-7
        assert np.all(np.abs(gh - ref_h) <= 1e-6 * np.abs(ref_h) + 1e-9), (gh, ref_h)
