"""Model-level parity on the GPU: MeanFieldToeplitzGP.elbo_and_grad / predict with kn from the
HIP path (hgp_pcg_solve + R^T) against the reference's own outputs (G5, made by running
/root/reference), and the RHS-sharded solve over 2 processes sharing the GPU."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_cases import load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(fx, dtype=torch.float64, device=DEV):
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    k = zk.Matern(nu=1.5, dtype=dtype)
    grids = [torch.tensor(fx["grid0"], dtype=dtype), torch.tensor(fx["grid1"], dtype=dtype)]
    mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=64, sig2_init=1., ell_init=.1, noise2_init=.01,
                                 learn_kernel=False, dtype=dtype)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["theta1"], dtype=dtype))
        mod.global_theta2.copy_(torch.tensor(fx["theta2"], dtype=dtype))
    return mod.cuda_params(0) if device != "cpu" else mod


def test_compute_kn_elbo_grad_predict_G5():
    """hipgp.py:117-146 (compute_kn), 194-276 (elbo_and_grad), 416-446 (predict), fp64."""
    fx = load("G5", "f64")
    mod = _model(fx)
    x = torch.tensor(fx["xobs"], device=DEV)
    y = torch.tensor(fx["yobs"], device=DEV)
    Knm, _ = mod._make_grams(x)
    kn = mod.compute_kn(Knm, maxiter_cg=20)
    assert rel_err(kn.cpu().numpy(), fx["kn"]) < 1e-8
    elbo = mod.elbo_and_grad(x, y, maxiter_cg=20)
    assert abs(float(elbo) - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
    assert rel_err(mod.global_theta1.grad.cpu().numpy(), fx["theta1_grad"]) < 1e-7
    assert rel_err(mod.global_theta2.grad.cpu().numpy(), fx["theta2_grad"]) < 1e-7
    mu, sig = mod.predict(x[:50], maxiter_cg=50)
    assert rel_err(mu.numpy(), fx["pred_mu"]) < 1e-7
    assert rel_err(sig.numpy(), fx["pred_sig"]) < 1e-7


def test_compute_kn_fp32_G5():
    """fp32 model (the reference default dtype, hipgp.py:23) against the reference's fp32 run:
    no worse than 4x the reference's own fp32 error vs fp64."""
    fx32 = load("G5", "f32")
    fx64 = load("G5", "f64")
    mod = _model(fx32, dtype=torch.float32)
    Knm, _ = mod._make_grams(torch.tensor(fx32["xobs"], device=DEV))
    kn = mod.compute_kn(Knm, maxiter_cg=20).double().cpu().numpy()
    e_me = np.linalg.norm(kn - fx64["kn"])
    e_ref = np.linalg.norm(fx32["kn"].astype(np.float64) - fx64["kn"])
    assert e_me <= 4 * e_ref + 1e-6 * np.linalg.norm(fx64["kn"]), (e_me, e_ref)


def _worker(rank, world_size, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        torch.cuda.set_device(0)
        fx = load("G5", "f64")
        mod = _model(fx)
        x = torch.tensor(fx["xobs"], device=DEV)
        y = torch.tensor(fx["yobs"], device=DEV)
        elbo = hdist.sharded_elbo_and_grad(mod, x, y, maxiter_cg=20, exact_break=True)
        # the all-RHS break rule across ranks: a tolerance every RHS meets only late
        Knm, _ = mod._make_grams(x[hdist.rhs_shard(64, world_size, rank)])
        T = mod.toeplitz()
        _, iters = T._plan.pcg_allranks(Knm, 200, 1e-6, precond=True)
        torch.cuda.synchronize()
        out[rank] = (float(elbo), mod.global_theta1.grad.cpu().numpy(), iters)
    finally:
        dist.destroy_process_group()


def test_sharded_two_ranks_one_gpu():
    """2 processes on the GPU (gloo for the host-side reductions): identical ELBO/grads to
    the reference, and both ranks stop PCG at the same (global) iteration."""
    fx = load("G5", "f64")
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29700 + os.getpid() % 200
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    assert len(out) == 2
    for r in range(2):
        elbo, g1, _ = out[r]
        assert abs(elbo - float(fx["elbo"])) < 1e-8 * abs(float(fx["elbo"]))
        assert rel_err(g1, fx["theta1_grad"]) < 1e-7
    assert out[0][2] == out[1][2] and out[0][2] < 200


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("per_obs_noise", [False, True], ids=["noise2", "noise_std"])
def test_meanfield_stats_kernel(dtype, per_obs_noise):
    """hgp_meanfield_stats (two passes over kn) against the torch expression of the same batch
    sums (hipgp.py:234-250, 370-414) on random kn of a C2-sized expanded grid slice."""
    fx = load("G5", "f64")
    mod = _model(fx, dtype=dtype)
    g = torch.Generator().manual_seed(7)
    B, Mp = 37, mod.Mprime
    kn = (torch.randn(B, Mp, generator=g, dtype=torch.float64) * .05).to(DEV, dtype)
    y = torch.randn(B, 1, generator=g, dtype=torch.float64).to(DEV, dtype)
    knn = (torch.rand(B, generator=g, dtype=torch.float64) + 1).to(DEV, dtype)
    nsd = (torch.rand(B, 1, generator=g, dtype=torch.float64) * .5 + .1).to(DEV, dtype) if per_obs_noise else None
    st = mod.batch_stats(kn, y, knn, nsd)
    # torch expression on the device (the reference's formulas)
    torch.set_grad_enabled(False)
    qm, qS = mod.standard_variational_params()
    ivar, log_sd = mod.noise_terms(nsd)
    iv = ivar.reshape(-1) if ivar.dim() > 0 else ivar
    knm = kn.matmul(qm).reshape(-1)
    an = -0.5 * iv * ((knm - y.reshape(-1)) ** 2 + knn - (kn * kn).sum(-1) + (kn * kn).matmul(qS).reshape(-1)) \
        - (log_sd.reshape(-1) if log_sd.dim() > 0 else log_sd) - 0.5 * np.log(2 * np.pi)
    lam = torch.sum((iv[:, None] if iv.dim() > 0 else iv) * kn * kn, dim=0)
    dm = -((iv * (knm - y.reshape(-1)))[None, :].matmul(kn)).reshape(-1)
    torch.set_grad_enabled(True)
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    assert abs(float(st["an_sum"] - an.sum())) <= tol * float(an.abs().sum())
    assert rel_err(st["lam_sum"].cpu().numpy(), lam.cpu().numpy()) < tol
    assert rel_err(st["dm_sum"].cpu().numpy(), dm.cpu().numpy()) < tol


def test_meanfield_stats_large_batch():
    """hgp_meanfield_stats with more than 65535 observations (a full-batch elbo_and_grad): the
    row statistics run in RHS chunks of the grid's y-dimension limit; against torch."""
    from hipgp_amd import _lib
    import ctypes
    B, Mp = 70000, 37
    g = torch.Generator(device=DEV).manual_seed(3)
    kn = torch.randn(B, Mp, device=DEV, generator=g, dtype=torch.float64) * .1
    qm = torch.randn(Mp, device=DEV, generator=g, dtype=torch.float64)
    qS = torch.rand(Mp, device=DEV, generator=g, dtype=torch.float64)
    y = torch.randn(B, device=DEV, generator=g, dtype=torch.float64)
    iv = torch.rand(B, device=DEV, generator=g, dtype=torch.float64) + .5
    knn = torch.rand(B, device=DEV, generator=g, dtype=torch.float64) + 1
    lsd = torch.randn(B, device=DEV, generator=g, dtype=torch.float64) * .1
    an = torch.empty(B, device=DEV, dtype=torch.float64)
    lam = torch.empty(Mp, device=DEV, dtype=torch.float64)
    dm = torch.empty(Mp, device=DEV, dtype=torch.float64)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    _lib.check(_lib.lib().hgp_meanfield_stats(_lib.HGP_F64, p(kn), B, Mp, p(qm), p(qS), p(y), p(iv), p(knn), p(lsd),
                                              p(an), p(lam), p(dm), _lib.stream_ptr(kn.device)))
    knm = kn @ qm
    an_ref = -0.5 * iv * ((knm - y) ** 2 + knn - (kn * kn).sum(1) + (kn * kn) @ qS) - lsd - 0.5 * np.log(2 * np.pi)
    assert float((an - an_ref).abs().max()) < 1e-10
    assert float((lam - (iv[:, None] * kn * kn).sum(0)).abs().max()) < 1e-9
    assert float((dm + ((iv * (knm - y))[:, None] * kn).sum(0)).abs().max()) < 1e-9


def test_plan_pool_trim_and_release():
    """Idle pooled plans trim their scratch beyond the pool budget and release_pool() frees them;
    a trimmed plan re-allocates on demand and computes the same result."""
    import gc
    from hipgp_amd import plan as hp
    from hipgp_amd import _lib
    hp.release_pool()
    dims = (300, 200)
    col = torch.tensor(zo_column(dims), device=DEV)
    v = torch.randn(3, 300 * 200, device=DEV, dtype=torch.float64)
    P = hp.ToeplitzPlan(dims, torch.float64, DEV)
    P.set_column(col)
    x1 = P.pcg(v, 10, 1e-30).clone()
    assert P.mem()["scratch"] > 0 and P.mem()["tables"] > 0
    old = hp._POOL_ENV
    hp._POOL_ENV = "0"                      # force trimming on the way into the pool
    try:
        del P
        gc.collect()
        assert hp.pool_scratch_bytes() == 0
        Q = hp.ToeplitzPlan(dims, torch.float64, DEV)   # the trimmed idle plan, re-used
        Q.set_column(col)
        assert torch.equal(Q.pcg(v, 10, 1e-30), x1)
        del Q
        gc.collect()
    finally:
        hp._POOL_ENV = old
    hp.release_pool()
    assert hp.pool_scratch_bytes() == 0 and not hp._POOL


def zo_column(dims):
    from oracle import ziggy_oracle as zo
    grids = [np.linspace(-1, 1, m) for m in dims]
    return zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 1e-2)
