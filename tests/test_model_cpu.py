"""Host-side model logic (no GPU): the mean-field ELBO / natural gradient assembled from kn,
against the reference's own outputs (G5 fixture, made by running /root/reference), and the
RHS-sharded version over world_size 2 with the gloo backend (one all-reduce of the stats)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from golden_cases import load, rel_err


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
    return mod


def test_grams_and_sizes_match_reference():
    fx = load("G5", "f64")
    mod = _model(fx)
    assert mod.Mprime == fx["kn"].shape[1] == 38 * 38
    Knm, Knn = mod._make_grams(torch.tensor(fx["xobs"]))
    assert rel_err(Knm.numpy(), fx["Knm"]) < 1e-12
    assert rel_err(Knn.numpy(), fx["Knn_diag"]) < 1e-12


def test_mean_field_elbo_and_natgrad_from_kn():
    """hipgp.py:194-276 given kn: ELBO, theta1.grad, theta2.grad equal the reference's."""
    fx = load("G5", "f64")
    mod = _model(fx)
    kn = torch.tensor(fx["kn"])
    stats = mod.batch_stats(kn, torch.tensor(fx["yobs"]), torch.tensor(fx["Knn_diag"]))
    elbo = mod.apply_stats(stats, kn.shape[0])
    assert abs(float(elbo) - float(fx["elbo"])) < 1e-9 * abs(float(fx["elbo"]))
    assert rel_err(mod.global_theta1.grad.numpy(), fx["theta1_grad"]) < 1e-10
    assert rel_err(mod.global_theta2.grad.numpy(), fx["theta2_grad"]) < 1e-10


def test_batch_an_matches_elbo_definition():
    fx = load("G5", "f64")
    mod = _model(fx)
    kn = torch.tensor(fx["kn"])
    qm, qS = mod.standard_variational_params()
    an = mod.compute_batch_an(torch.tensor(fx["xobs"]), torch.tensor(fx["yobs"]), qm=qm, qS=qS,
                              Knm=torch.tensor(fx["Knm"]), Knn_diag=torch.tensor(fx["Knn_diag"]), kn=kn)
    elbo = an.mean() - mod.get_kl_to_prior(qm, qS) / mod.N
    assert abs(float(elbo) - float(fx["elbo"])) < 1e-9 * abs(float(fx["elbo"]))


def test_rhs_shard_partition():
    from hipgp_amd.dist import rhs_shard
    for n in (1, 5, 32, 200, 201):
        for ws in (1, 2, 3, 8):
            idx = []
            for r in range(ws):
                sl = rhs_shard(n, ws, r)
                idx.extend(range(n)[sl])
                assert abs((sl.stop - sl.start) - n / ws) < 1
            assert idx == list(range(n))


def _dist_worker(rank, world_size, port, out, nobs=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        fx = load("G5", "f64")
        mod = _model(fx)
        kn_full = torch.tensor(fx["kn"])
        x = torch.tensor(fx["xobs"])
        y = torch.tensor(fx["yobs"])
        if nobs is not None:     # a short minibatch: fewer rows than ranks, some shards empty
            kn_full, x, y = kn_full[:nobs], x[:nobs], y[:nobs]
        # inject kn for this rank's rows (the device solve is exercised by the GPU tests)
        sl = hdist.rhs_shard(x.shape[0], world_size, rank)
        fake_kn = lambda model, Knm_local: kn_full[sl]
        elbo = hdist.sharded_elbo_and_grad(mod, x, y, compute_kn=fake_kn)
        out[rank] = (float(elbo), mod.global_theta1.grad.numpy().copy(), mod.global_theta2.grad.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world_size", [2, 3])
def test_sharded_natgrad_gloo(world_size):
    """RHS-sharded ELBO/natgrad over `world_size` gloo ranks == the single-process reference
    values (fp64 reduction-order tolerance)."""
    fx = load("G5", "f64")
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + os.getpid() % 1000 + world_size
    mp.spawn(_dist_worker, args=(world_size, port, out), nprocs=world_size, join=True)
    assert len(out) == world_size
    for r in range(world_size):
        elbo, g1, g2 = out[r]
        assert abs(elbo - float(fx["elbo"])) < 1e-9 * abs(float(fx["elbo"]))
        assert rel_err(g1, fx["theta1_grad"]) < 1e-10
        assert rel_err(g2, fx["theta2_grad"]) < 1e-10
    # every rank holds bit-identical gradients
    for r in range(1, world_size):
        assert np.array_equal(out[0][1], out[r][1]) and np.array_equal(out[0][2], out[r][2])


def _dist_worker_short(rank, world_size, port, out):
    _dist_worker(rank, world_size, port, out, nobs=2)


def test_sharded_natgrad_empty_shard_gloo():
    """3 ranks, a minibatch of 2 observations: one rank's shard is empty; it contributes zero
    statistics and joins the all-reduces (no hang), and every rank gets the single-process
    ELBO / natural gradient of those 2 observations."""
    fx = load("G5", "f64")
    mod = _model(fx)
    kn = torch.tensor(fx["kn"])[:2]
    stats = mod.batch_stats(kn, torch.tensor(fx["yobs"])[:2], torch.tensor(fx["Knn_diag"])[:2])
    elbo_ref = float(mod.apply_stats(stats, 2))
    g1_ref = mod.global_theta1.grad.numpy().copy()
    empty = mod.batch_stats(kn[:0], torch.tensor(fx["yobs"])[:0], torch.tensor(fx["Knn_diag"])[:0])
    assert empty["n"] == 0 and float(empty["lam_sum"].abs().sum()) == 0.0
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + os.getpid() % 1000 + 7
    mp.spawn(_dist_worker_short, args=(3, port, out), nprocs=3, join=True)
    assert len(out) == 3
    for r in range(3):
        elbo, g1, _ = out[r]
        assert abs(elbo - elbo_ref) < 1e-12 * abs(elbo_ref)
        assert rel_err(g1, g1_ref) < 1e-12


def test_hyper_grad_needed_flags():
    fx = load("G5", "f64")
    mod = _model(fx)                       # learn_kernel=False, learn_noise default False
    assert not mod.hyper_grad_needed()
    mod.log_noise2.requires_grad_(True)
    assert mod.hyper_grad_needed()         # noise2 drives ivar when no per-observation noise
    assert not mod.hyper_grad_needed(torch.ones(3, 1, dtype=torch.float64))
    with torch.no_grad():
        assert not mod.hyper_grad_needed()


def _dist_worker_hyper_short(rank, world_size, port, out):
    """learn_noise with a 2-row minibatch on 3 ranks: one empty shard still runs backward()."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        fx = load("G5", "f64")
        mod = _model(fx)
        mod.log_noise2.requires_grad_(True)
        kn_full = torch.tensor(fx["kn"])[:2]
        x, y = torch.tensor(fx["xobs"])[:2], torch.tensor(fx["yobs"])[:2]
        sl = hdist.rhs_shard(2, world_size, rank)
        elbo = hdist.sharded_elbo_and_grad(mod, x, y, compute_kn=lambda model, Knm_local: kn_full[sl])
        elbo.backward()
        hdist.allreduce_hyper_grads(mod)
        out[rank] = (float(elbo), float(mod.log_noise2.grad))
    finally:
        dist.destroy_process_group()


def test_sharded_hyper_grad_empty_shard_gloo():
    """an empty shard with hyper-parameter learning must run backward() and reach
    allreduce_hyper_grads (no exception on that rank, no hang on the others); every rank gets
    the single-process log_noise2 gradient (`hipgp.py:214-227` with the noise learned)."""
    fx = load("G5", "f64")
    mod = _model(fx)
    mod.log_noise2.requires_grad_(True)
    x, y = torch.tensor(fx["xobs"])[:2], torch.tensor(fx["yobs"])[:2]
    _, Knn = mod._make_grams(x)
    ref = mod.autograd_elbo(x, y, None, None, Knn, torch.tensor(fx["kn"])[:2])
    ref.backward()
    g_ref = float(mod.log_noise2.grad)
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + os.getpid() % 1000 + 11
    mp.spawn(_dist_worker_hyper_short, args=(3, port, out), nprocs=3, join=True)
    assert len(out) == 3
    for r in range(3):
        elbo, g = out[r]
        assert abs(elbo - float(ref)) < 1e-12 * abs(float(ref))
        assert abs(g - g_ref) < 1e-12 * abs(g_ref), (g, g_ref)
