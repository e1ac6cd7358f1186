"""Block-diagonal variational family, host logic (no GPU): BlockToeplitzGP's block maps, ELBO and
natural gradient assembled from kn (CPU tensors) against the reference's own outputs (G11, G12),
and the RHS-sharded version over gloo world size 2 (one all-reduce of the packed stats)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from block_cases import block_model, noise_of
from golden_cases import rel_err


@pytest.mark.parametrize("name", ["G11", "G12"])
def test_block_layout_matches_reference(name):
    mod, fx = block_model(name)
    assert np.array_equal(mod.block_idx.numpy(), fx["block_idx"])
    assert (mod.num_blocks, mod.block_size) == fx["block_idx"].shape
    assert tuple(mod.global_theta2.shape) == fx["theta2"].shape
    qm, qS = mod.standard_variational_params()
    assert rel_err(qm.detach().numpy(), fx["qm"]) < 1e-12
    assert abs(float(mod.get_kl_to_prior(qm, qS)) - float(fx["kl"])) < 1e-10 * abs(float(fx["kl"]))


@pytest.mark.parametrize("name", ["G11", "G12"])
def test_block_elbo_natgrad_from_kn(name):
    """hipgp.py:194-276 ('block' branch) given kn: ELBO, theta1.grad, theta2.grad, batch a_n."""
    mod, fx = block_model(name)
    kn = torch.tensor(fx["kn"])
    nstd = noise_of(fx)
    stats = mod.batch_stats(kn, torch.tensor(fx["yobs"]), torch.tensor(fx["Knn_diag"]), nstd)
    elbo = mod.apply_stats(stats, kn.shape[0])
    assert abs(float(elbo) - float(fx["elbo"])) < 1e-10 * abs(float(fx["elbo"]))
    assert rel_err(mod.global_theta1.grad.numpy(), fx["theta1_grad"]) < 1e-10
    assert rel_err(mod.global_theta2.grad.numpy(), fx["theta2_grad"]) < 1e-10
    qm, qS = mod.standard_variational_params()
    an = mod.compute_batch_an(None, torch.tensor(fx["yobs"]), nstd, qm=qm, qS=qS, Knm=torch.tensor(fx["Knm"]),
                              Knn_diag=torch.tensor(fx["Knn_diag"]), kn=kn)
    assert an.shape == fx["batch_an"].shape        # incl. the (bsz, bsz) broadcast quirk
    assert rel_err(an.detach().numpy(), fx["batch_an"]) < 1e-10
    assert rel_err(mod.compute_knSkn(kn, qS).detach().numpy(), fx["knSkn"]) < 1e-10


def test_block_get_lam_definition():
    mod, fx = block_model("G11")
    kn = torch.tensor(fx["kn"])
    iv = torch.rand(kn.shape[0], 1, dtype=torch.float64)
    lam = mod.get_lam(iv, kn, bscale=3., add_identity=True)
    kb = kn[:, mod.block_idx]
    ref = 3. * torch.einsum("b,bki,bkj->kij", iv[:, 0], kb, kb) + torch.eye(mod.block_size)[None]
    assert rel_err(lam.numpy(), ref.numpy()) < 1e-12


def _dist_worker(rank, world_size, port, name, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from hipgp_amd import dist as hdist
        mod, fx = block_model(name)
        kn_full = torch.tensor(fx["kn"])
        x = torch.tensor(fx["xobs"])
        sl = hdist.rhs_shard(x.shape[0], world_size, rank)
        fake_kn = lambda model, Knm_local: kn_full[sl]
        elbo = hdist.sharded_elbo_and_grad(mod, x, torch.tensor(fx["yobs"]), noise_std_batch=noise_of(fx),
                                           compute_kn=fake_kn)
        out[rank] = (float(elbo), mod.global_theta1.grad.numpy().copy(), mod.global_theta2.grad.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["G11", "G12"])
def test_block_sharded_natgrad_gloo(name):
    """RHS-sharded block ELBO/natgrad over 2 gloo ranks == the single-process reference values."""
    from golden_cases import load
    fx = load(name, "f64")
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29700 + os.getpid() % 1000 + (0 if name == "G11" else 1)
    mp.spawn(_dist_worker, args=(2, port, name, out), nprocs=2, join=True)
    for r in range(2):
        elbo, g1, g2 = out[r]
        assert abs(elbo - float(fx["elbo"])) < 1e-10 * abs(float(fx["elbo"]))
        assert rel_err(g1, fx["theta1_grad"]) < 1e-10
        assert rel_err(g2, fx["theta2_grad"]) < 1e-10
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])
