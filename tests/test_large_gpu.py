"""The BASELINE configs C3 (2048^2) and C4 (4096^2) on the GPU: PCG (`_solve`, `compute_kn`)
and the mean-field ELBO / natural gradient at full grid size in fp32, against the fp64 plan
of the same problem, plus residual checks.  At these sizes the rows are longer than one wave's
line (16-pair row blocks, the fused PCG epilogues k_row_inv_t<float, 2048 | 4096, EPI_XR | EPI_P>
with the alpha / beta mid-pass), the 4096^2 fp32 twiddles are two-level LDS tables, and the RHS
run in several workspace chunks over the two streams (the 2 GiB budget: 8 RHS per chunk at
4096^2 fp32, 4 in fp64).  Nugget 0.1 keeps the problems well conditioned, so fp32 and fp64
agree to ~1e-4 (a difference of the implementations, not of the chaos of a clamped solve)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tt(m, dtype, jitter=0.1):
    """Matern-3/2 with a length scale of 10 grid spacings (ell = 20/m on [-1, 1]) and nugget 0.1:
    cond(K) ~ 1e3-1e4, so 20 preconditioned iterations converge well at every grid size."""
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    k = zk.Matern(nu=1.5, dtype=dtype)
    grids = [torch.linspace(-1, 1, m, device=DEV, dtype=dtype) for _ in range(2)]
    return ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=(1., 20. / m)), jitter_val=jitter)


@pytest.mark.parametrize("m,B", [(2048, 16), (4096, 10), (4096, 25)],
                         ids=["C3_2048x2048_B16", "C4_4096x4096_B10", "C4_4096x4096_B25"])
def test_pcg_compute_kn_fp32_vs_fp64(m, B):
    g = torch.Generator(device=DEV).manual_seed(21)
    b64 = torch.randn(B, m * m, device=DEV, generator=g, dtype=torch.float64)
    out = {}
    for dt in (torch.float64, torch.float32):
        T = _tt(m, dt)
        b = b64.to(dt)
        x = T._solve(b, do_precond=True, maxiter=20, tol=1e-8)
        res = (T._matmul_by_K(x).double() - b64).norm(dim=1) / b64.norm(dim=1)
        kn = None
        if m == 2048 or dt == torch.float32:      # fp64 R^T rows of H = 8192 exceed one CU's LDS
            kn = T._matmul_by_RT(T.inv_matmul(b, do_precond=True, maxiter=20, tol=1e-8))
            assert kn.shape == (B, (2 * m - 2) ** 2)
            # the whitening identity R (R^T d) = K d on the same solve
            d = T.inv_matmul(b[:2], do_precond=True, maxiter=20, tol=1e-8)
            Kd = T._matmul_by_K(d)
            rr = T._matmul_by_R(T._matmul_by_RT(d))
            # fp32: the rounding of R and R^T scales with |R^T d| ~ sqrt(D_max) |d| while |K d| ~ |b|, so
            # it is amplified by ~cond(K) eps relative to max|K d| (measured 2.4e-4 at 2048^2)
            assert float((rr - Kd).abs().max() / Kd.abs().max()) < (1e-10 if dt == torch.float64 else 2e-3)
        out[dt] = (x.double(), float(res.max()), kn)
        del T
        torch.cuda.empty_cache()
    x64, r64, kn64 = out[torch.float64]
    x32, r32, kn32 = out[torch.float32]
    assert r64 < 0.05, r64                      # 20 preconditioned iterations have converged well
    assert abs(r32 - r64) < 1e-3, (r32, r64)
    rel = float(((x32 - x64).norm(dim=1) / x64.norm(dim=1)).max())
    assert rel < 1e-3, rel
    if kn64 is not None:
        rel_kn = float(((kn32.double() - kn64).norm(dim=1) / kn64.norm(dim=1)).max())
        assert rel_kn < 1e-3, rel_kn


def test_pcg_break_rule_C3():
    """The all-RHS break rule at 2048^2 (fp64, a tolerance met after a few iterations): the
    fused 2-D iteration stops at the same iteration as a stepwise run with a callback."""
    T = _tt(2048, torch.float64)
    g = torch.Generator(device=DEV).manual_seed(22)
    b = torch.randn(3, 2048 * 2048, device=DEV, generator=g, dtype=torch.float64)
    tol = 1e-4 * float(b.norm(dim=1).min())
    x, iters = T._plan.pcg(b, 50, tol, precond=True, return_iters=True)
    calls = []
    x2 = T._plan.pcg_steps(b, 50, tol, precond=True, callback=lambda n, xx: calls.append(n))
    assert 1 < iters < 50 and len(calls) == iters - 1
    assert torch.equal(x, x2)
    T.set_batch_shape((3,))
    r = (T._matmul_by_K(x) - b).norm(dim=1)
    assert float(r.max()) < tol * 1.01


def test_meanfield_elbo_C3():
    """Mean-field `elbo_and_grad` at the C3 grid (2048^2, M' = 4094^2) with 16 observations:
    the fp32 model's ELBO and natural gradient against the fp64 model's."""
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    res = {}
    rs = np.random.RandomState(5)
    x = rs.rand(16, 2) * 1.8 - .9
    y = rs.randn(16, 1)
    for dt in (torch.float64, torch.float32):
        k = zk.Matern(nu=1.5, dtype=dt)
        grids = [torch.linspace(-1, 1, 2048, dtype=dt) for _ in range(2)]
        mod = hg.MeanFieldToeplitzGP(k, grids, num_obs=100000, sig2_init=1., ell_init=20. / 2048, noise2_init=.05,
                                     dtype=dt, jitter_val=0.1)
        torch.manual_seed(3)
        with torch.no_grad():
            mod.global_theta1.copy_(torch.randn(mod.Mprime, 1, dtype=torch.float64).to(dt) * .01)
        mod = mod.cuda_params(0)
        elbo = mod.elbo_and_grad(torch.tensor(x, dtype=dt, device=DEV), torch.tensor(y, dtype=dt, device=DEV),
                                 maxiter_cg=20)
        res[dt] = (float(elbo), mod.global_theta1.grad.double(), mod.global_theta2.grad.double())
        del mod
        torch.cuda.empty_cache()
    e64, g1_64, g2_64 = res[torch.float64]
    e32, g1_32, g2_32 = res[torch.float32]
    assert abs(e32 - e64) < 1e-4 * abs(e64), (e32, e64)
    for a, b in ((g1_32, g1_64), (g2_32, g2_64)):
        assert float((a - b).norm() / b.norm()) < 1e-4, float((a - b).norm() / b.norm())


# fp32 vs the fp64 plan at B = 200 (solve, kn): 10x the largest gap measured on the GPU, instead
# of round 5's flat 1e-3 (profiles/r6_B200_gaps.txt: C3 1.13e-5 / 5.80e-6, C4 1.14e-5 / 5.88e-6)
B200_BOUND = {2048: (1.2e-4, 6e-5), 4096: (1.2e-4, 6e-5)}


@pytest.mark.parametrize("m", [2048, 4096], ids=["C3_2048x2048_B200", "C4_4096x4096_B200"])
def test_configs_own_batch_B200(m):
    """The configs' own minibatch (C3 / C4: 200 RHS, `run_ukhousing_experiment.py:31`,
    `run_3droad_experiment.py:48`) through the full chunk / two-stream schedule in fp32:
    `_solve` and `compute_kn` of all 200 RHS in one call.  A seeded subset of 5 rows (first,
    last, chunk-boundary neighbours and a middle row) is checked (a) against the fp64 plan of
    the same problem -- SURVEY §8(c)'s PCG rule in the form the other full-size tests use here
    (nugget 0.1: fp32 and fp64 differ by the implementation's rounding, ~1e-5) -- and
    (b) against the same rows solved in a batch of 2 (other chunks, other streams, other batch
    positions): every RHS runs its own FFTs and fixed-order reductions, so a row's result does
    not depend on the batch around it -- bitwise in practice, held to 1e-6.  The fp64 bound is
    10x the measured gap (B200_BOUND)."""
    B = 200
    g = torch.Generator(device=DEV).manual_seed(31)
    b = torch.randn(B, m * m, device=DEV, generator=g, dtype=torch.float32)
    rows = [0, 1, 7, 101, B - 1]
    T = _tt(m, torch.float32)
    x = T._solve(b, do_precond=True, maxiter=20, tol=1e-8)
    xs = x[rows].double()
    del x
    kn = T._matmul_by_RT(T.inv_matmul(b, do_precond=True, maxiter=20, tol=1e-8))
    assert kn.shape == (B, (2 * m - 2) ** 2)
    kns = kn[rows].double()
    del kn
    # (b) the same rows in batches of 2: batch-position independence
    for j in range(0, len(rows) - 1, 2):
        sub = b[rows[j:j + 2]]
        x2 = T._solve(sub, do_precond=True, maxiter=20, tol=1e-8).double()
        rel = float(((x2 - xs[j:j + 2]).norm(dim=1) / xs[j:j + 2].norm(dim=1)).max())
        assert rel < 1e-6, (rows[j:j + 2], rel)
        kn2 = T._matmul_by_RT(T.inv_matmul(sub, do_precond=True, maxiter=20, tol=1e-8)).double()
        rel = float(((kn2 - kns[j:j + 2]).norm(dim=1) / kns[j:j + 2].norm(dim=1)).max())
        assert rel < 1e-6, (rows[j:j + 2], rel)
    del T
    torch.cuda.empty_cache()
    # (a) against the fp64 plan on the subset
    T64 = _tt(m, torch.float64)
    b64 = b[rows].double()
    x64 = T64._solve(b64, do_precond=True, maxiter=20, tol=1e-8)
    rel = float(((xs - x64).norm(dim=1) / x64.norm(dim=1)).max())
    res = (T64._matmul_by_K(xs) - b64).norm(dim=1) / b64.norm(dim=1)
    kn64 = T64._matmul_by_RT(T64.inv_matmul(b64, do_precond=True, maxiter=20, tol=1e-8))
    rel_kn = float(((kns - kn64).norm(dim=1) / kn64.norm(dim=1)).max())
    print(f"B200 m={m}: solve fp32 vs fp64 {rel:.3e}, kn {rel_kn:.3e}, residual {float(res.max()):.3e}")
    assert rel < B200_BOUND[m][0], rel
    assert float(res.max()) < 0.05, res
    assert rel_kn < B200_BOUND[m][1], rel_kn
