"""Grid-block sharded fits and line-integral observations under `svigp_fit` on the CPU (gloo,
world size 2) -- the host logic of round 6's multi-GPU config-5 path:

* shard="grid" with kn kept in slabs (`hipgp_amd.slab.SlabFit`: each rank's Knm columns, the
  slab PCG / R^T, statistics from all-reduced B-length dots) on config 3's settings (G19 "box")
  equals the single-process fit;
* integrated (line-integral) observations with the MC estimator in both shardings, with the
  ranks' torch RNGs seeded DIFFERENTLY: the estimator's offset is drawn once and broadcast
  from rank 0 (`hipgp_amd.dist.shared_mc_offset`), so every rank holds bit-identical parameters
  equal to the single-process fit's.

Operators: the slab stages run the reference's own operator definition on NumPy
(tests/slab_cpu_engine.py) and the RHS-sharded solve is the injected NumPy oracle (TEST
INFRASTRUCTURE); the device versions are tests/test_fit_sharded_gpu.py."""
import os

import numpy as np
import torch
import torch.multiprocessing as mp

from golden_cases import load


def _model_oracle(model):
    """The oracle of the model's Kmm: the first row from the model's own kernel, nugget on c0
    (`toeplitz_tensor.py:127-133`)."""
    from oracle import ziggy_oracle as zo
    params = model.get_kernel_params()
    with torch.no_grad():
        row = model.kernel(model.xinduce[:1], model.xinduce, params)[0].numpy().copy()
    row[0] += model.jitter_val
    return zo.ToeplitzOracle(row, [len(g) for g in model.xgrids])


def _oracle_kn(model, Knm, maxiter=20, tol=1e-8):
    """kn of this rank's rows by the oracle with the all-RHS break over every rank (as
    test_fit_sharded_cpu._oracle_kn, for any kernel)."""
    import torch.distributed as dist
    from oracle import ziggy_oracle as zo
    from test_fit_sharded_cpu import _converged_at
    T = _model_oracle(model)
    b = Knm.detach().numpy()
    pred = torch.tensor(_converged_at(T, b, maxiter, tol) if b.shape[0] else [True] * maxiter, dtype=torch.int32)
    dist.all_reduce(pred, op=dist.ReduceOp.MIN)
    stop = next((n + 1 for n in range(maxiter) if int(pred[n])), maxiter)
    if b.shape[0] == 0:
        return Knm.new_zeros((0, model.Mprime))
    return torch.tensor(zo.compute_kn(T, b, maxiter_cg=stop, tol=-1.0))


def _cpu_slab(model):
    from slab_cpu_engine import CpuSlabEngine
    from hipgp_amd.slab import SlabToeplitz
    T = _model_oracle(model)
    return SlabToeplitz(T.dims, CpuSlabEngine(T))


def _g19(shard, nbatch=3):
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    fx = load("G19", "f64")
    dt = torch.float64
    grids = [torch.tensor(fx["box_grid0"], dtype=dt), torch.tensor(fx["box_grid1"], dtype=dt)]
    mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=1.5, dtype=dt), grids, num_obs=100_000,
                                 sig2_init=float(fx["box_sig2_init"]), ell_init=.1, init_Svar=.1,
                                 learn_kernel=False, jitter_val=1e-3, dtype=dt)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["box_theta1_init"], dtype=dt))
        mod.global_theta2.copy_(torch.tensor(fx["box_theta2_init"], dtype=dt))
    x, y, s = (fx[f"box_{k}"][:200 * nbatch] for k in "xys")
    return mod, (x, y, s), dict(lr=1e-2, schedule_lr=False, batch_size=200, epochs=1, maxiter_cg=20)


def _semi(shard):
    """A 3-D grid (8 x 7 x 6) with line-integral observations (the interstellar-dust setting of
    config 5, `run_domain_experiment.py:276`: integrated_obs, a Matern kernel -> the MC estimator)."""
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    from oracle import ziggy_oracle as zo
    dt = torch.float64
    grids = [torch.linspace(-1, 1, 8, dtype=dt), torch.linspace(-1, 1, 7, dtype=dt), torch.linspace(-.5, .5, 6, dtype=dt)]
    kern = zk.Matern(nu=2.5, dtype=dt)
    # a well-conditioned Kmm (ell = 0.25 at a 0.2-0.29 spacing, nugget 1e-2): 20 PCG iterations of
    # two exact implementations then agree to rounding (ell = 0.6 / nugget 1e-3 is the chaotic
    # regime where they end 3e-3 apart, as the clamped goldens do)
    mod = hg.MeanFieldToeplitzGP(kern, grids, num_obs=48, sig2_init=1., ell_init=.25, init_Svar=.5,
                                 learn_kernel=False, jitter_val=1e-2, dtype=dt)
    # Knn_diag: the doubly-integrated table of the oracle (the library's table kernel is device
    # only); the same function on every rank and in the single process
    table = zo.doubly_diag_table("matern", nu=2.5)
    kern.k_doubly_diag = lambda x, params: torch.tensor(
        zo.doubly_diag(x.detach().numpy(), [float(p) for p in params], table), dtype=dt)
    rs = np.random.RandomState(3)
    x = rs.uniform(-.9, .9, (48, 3)) * np.array([1, 1, .5])
    y = np.sin(2 * x[:, :1]) * np.cos(x[:, 1:2]) + .05 * rs.randn(48, 1)
    s = np.full((48, 1), .1)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(rs.randn(mod.Mprime, 1) * .1))
    return mod, (x, y, s), dict(lr=1e-2, schedule_lr=True, batch_size=16, epochs=1, maxiter_cg=20,
                                integrated_obs=True, semi_integrated_estimator="mc-biased", num_semi_mc_samples=10)


def _fit(case, shard, seed):
    torch.manual_seed(seed)
    mod, (x, y, s), kw = (_g19 if case == "g19" else _semi)(shard)
    snaps = []
    cb = lambda m, xb, yb, sb: snaps.append(np.concatenate([m.global_theta1.detach().numpy().ravel(),
                                                            m.global_theta2.detach().numpy().ravel()]))
    extra = dict(compute_kn=_oracle_kn) if shard == "rhs" else dict(slab=_cpu_slab(mod))
    mod.fit(None, x, y, s, None, None, None, None, None, None, batch_callback=cb, epoch_callback=None,
            do_cuda=False, batch_log_interval=1, learn_kernel=False, distributed=True, shard=shard, **kw, **extra)
    cb(mod, None, None, None)
    return np.stack(snaps), list(mod.fit_trace)


def _worker(rank, ws, port, case, shard, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        torch.set_num_threads(2)
        out[rank] = _fit(case, shard, 1000 + rank)     # ranks seeded differently on purpose
    finally:
        dist.destroy_process_group()


def _spawn(ws, case, shard):
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + os.getpid() % 97 + 5 * ws + (17 if shard == "grid" else 0) + (40 if case == "semi" else 0)
    mp.spawn(_worker, args=(ws, port, case, shard, out), nprocs=ws, join=True)
    assert len(out) == ws
    return [out[r] for r in range(ws)]


def _check(case, shard, ws=2):
    (ref, ref_tr), = _spawn(1, case, "rhs")           # the single-process fit (world size 1, seed 1000)
    res = _spawn(ws, case, shard)
    for r, (snaps, tr) in enumerate(res):
        assert snaps.shape == ref.shape
        assert np.array_equal(snaps, res[0][0]), r     # bit-identical parameters on every rank
        rel = np.linalg.norm(snaps - ref, axis=1) / np.linalg.norm(ref, axis=1)
        assert float(rel.max()) < 1e-10, (case, shard, rel)
        assert np.allclose(tr, ref_tr, rtol=1e-10, atol=0), (tr, ref_tr)
    return ref


def test_grid_fit_kn_in_slabs_matches_single_process_gloo():
    _check("g19", "grid")


def test_grid_fit_three_ranks_uneven_slabs_gloo():
    """World size 3: uneven axis-0 slabs (8 rows as 3 + 3 + 2, 14 expanded rows as 5 + 5 + 4) on the
    line-integral 3-D fit, so the Knm sub-grids, kn column ranges and statistic slices are ragged."""
    _check("semi", "grid", ws=3)


def test_integrated_obs_rhs_shard_shared_mc_offset_gloo():
    ref = _check("semi", "rhs")
    assert np.all(np.isfinite(ref)) and np.linalg.norm(ref[-1] - ref[0]) > 0


def test_integrated_obs_grid_shard_gloo():
    _check("semi", "grid")
