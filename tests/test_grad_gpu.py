"""GPU parity of the backward through the ziggy drop-in and the C ABI
(hgp_sym_toeplitz_dqf, hgp_plan_column_grad) against the reference's own gradients
(G13 1-D m=40, G14 2-D 9x7, G15 3-D 5x4x3; tests/golden/make_golden_grad.py) and the oracle.
Tolerances: fp64 1e-9 relative to max, for gradients that go through a PCG solve no more than
10x the forward solve's own distance from the reference (G14, SqExp on 9x7: the two fp64 PCGs
differ by 4.7e-6 after 30 iterations because the FFT lengths round differently); fp32 no worse
than 4x the reference's own fp32 error against its fp64 result (+1e-5 relative)."""
import numpy as np
import pytest
import torch

from golden_cases import load, grids_of, rel_err
from grad_cases import GRAD_CASES, GRAD_MAXITER, GRAD_TOL
from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = {"f64": torch.float64, "f32": torch.float32}


def _np(t):
    return t.detach().cpu().numpy()


def _setup(name, tag, params=None):
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    kind, nu, p = GRAD_CASES[name]
    dtype = DT[tag]
    fx = load(name, tag)
    k = zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)
    grids = [torch.tensor(g, dtype=dtype, device=DEV) for g in grids_of(fx)]
    params = params if params is not None else p
    kfun = lambda x, y: k.forward(x, y, params=params)   # noqa: E731
    return fx, grids, kfun, ToeplitzTensor


def _ok(name, tag, got, key, base_tol=1e-9, fwd_err=0.0):
    ref64 = load(name, "f64")[key]
    if tag == "f64":
        return rel_err(got, ref64) < max(base_tol, 10 * fwd_err)
    ref32 = load(name, "f32")[key]
    return rel_err(got, ref64) <= 4 * rel_err(ref32, ref64) + 1e-5


@pytest.mark.parametrize("name", sorted(GRAD_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_inv_matmul_backward(name, tag):
    from ziggy.misc._inv_matmul import InvMatmul
    fx, grids, kfun, TT = _setup(name, tag)
    T = TT(grids, kfun, batch_shape=None, jitter_val=1e-3)
    col = T.column.detach().clone().requires_grad_(True)
    R = torch.tensor(fx["R"], device=DEV).requires_grad_(True)
    sol = InvMatmul.apply(T, col, R, True, GRAD_MAXITER, GRAD_TOL)
    sol.backward(torch.tensor(fx["grad_out"], device=DEV))
    fwd = rel_err(_np(sol), load(name, "f64")["solves"])
    assert _ok(name, tag, _np(col.grad), "inv_column_grad", fwd_err=fwd)
    assert _ok(name, tag, _np(R.grad), "inv_right_grad", fwd_err=fwd)


@pytest.mark.parametrize("name", sorted(GRAD_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_operator_column_grads(name, tag):
    dtype = DT[tag]
    sig2 = torch.tensor(GRAD_CASES[name][2][0], dtype=dtype, device=DEV, requires_grad=True)
    ell = torch.tensor(GRAD_CASES[name][2][1], dtype=dtype, device=DEV, requires_grad=True)
    fx, grids, kfun, TT = _setup(name, tag, params=(sig2, ell))
    T = TT(grids, kfun, batch_shape=None, jitter_val=1e-3)
    B = fx["rt_v"].shape[0]
    T.set_batch_shape((B,))
    fns = {"rt": T._matmul_by_RT, "K": T._matmul_by_K, "Cinv": T._matmul_by_Cinv, "R": T._matmul_by_R}
    for key, fn in fns.items():
        x = torch.tensor(fx[f"{key}_x" if key != "rt" else "rt_v"], device=DEV)
        g = torch.tensor(fx[f"{key}_g" if key != "rt" else "rt_g"], device=DEV)
        (gc,) = torch.autograd.grad((fn(x) * g).sum(), T.column, retain_graph=True)
        assert _ok(name, tag, _np(gc), f"{key}_column_grad"), key
    # vector gradient = the adjoint operator
    v = torch.tensor(fx["rt_v"], device=DEV).requires_grad_(True)
    g = torch.tensor(fx["rt_g"], device=DEV)
    (T._matmul_by_RT(v) * g).sum().backward()
    want = T._matmul_by_R(g).detach()
    assert rel_err(_np(v.grad), _np(want)) == 0.0


@pytest.mark.parametrize("name", sorted(GRAD_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_compute_kn_hyperparameter_grads(name, tag):
    """End to end: d/d(sig2, ell) of sum(W * R^T K^{-1} Knm^T) with the Toeplitz column and Knm
    from the same kernel parameters (ziggy whitening with learn_kernel, `hipgp.py:117-146`)."""
    dtype = DT[tag]
    p = GRAD_CASES[name][2]
    sig2 = torch.tensor(p[0], dtype=dtype, device=DEV, requires_grad=True)
    ell = torch.tensor(p[1], dtype=dtype, device=DEV, requires_grad=True)
    fx, grids, kfun, TT = _setup(name, tag, params=(sig2, ell))
    x = torch.tensor(fx["x"], device=DEV)
    mesh = torch.meshgrid(*grids, indexing="ij")
    xinduce = torch.stack([m.reshape(-1) for m in mesh], dim=-1)
    Knm = kfun(x, xinduce)
    T = TT(grids, kfun, batch_shape=None, jitter_val=1e-3)
    d0 = T.inv_matmul(Knm, do_precond=True, maxiter=GRAD_MAXITER, tol=GRAD_TOL)
    kn = T._matmul_by_RT(d0)
    loss = (kn * torch.tensor(fx["W"], device=DEV)).sum()
    gs, ge = torch.autograd.grad(loss, (sig2, ell))
    f64 = load(name, "f64")
    fwd = rel_err(_np(kn), f64["kn"])
    if tag == "f64":
        assert fwd < (1e-4 if name == "G14" else 1e-8), fwd
    else:
        assert _ok(name, tag, _np(kn), "kn")
    for got, key in ((gs, "dsig2"), (ge, "dell")):
        ref64 = float(f64[key])
        err = abs(float(got) - ref64) / max(abs(ref64), 1e-30)
        if tag == "f64":
            # G14 is ill-conditioned for 30 PCG iterations: two fp64 PCGs differ by ~1e-5 in kn
            # and the backward's extra solve amplifies that ~17x (measured 2.1e-4 on dsig2, the
            # reference's own fp32 error there is 9.4e-4): a sanity bound, as for the clamped
            # cases of test_parity_gpu; G13 / G15 are pinned at 1e-8
            assert err < (1e-3 if name == "G14" else 1e-8), (key, err, fwd)
        else:
            ref32 = float(load(name, "f32")[key])
            assert err <= 4 * abs(ref32 - ref64) / max(abs(ref64), 1e-30) + 1e-4, (key, err)


@pytest.mark.parametrize("n,s", [(1, 2), (255, 3), (256, 1), (700, 4), (2049, 2)])
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_dqf_vs_oracle(n, s, tag):
    """hgp_sym_toeplitz_dqf over ragged lengths and several 256-lag tiles."""
    from hipgp_amd.plan import sym_toeplitz_dqf
    rs = np.random.RandomState(n + s)
    l, r = rs.randn(n, s), rs.randn(n, s)
    got = sym_toeplitz_dqf(torch.tensor(l, dtype=DT[tag], device=DEV),
                           torch.tensor(r, dtype=DT[tag], device=DEV))
    want = zo.sym_toeplitz_dqf(l, r)
    assert rel_err(_np(got), want) < (1e-12 if tag == "f64" else 2e-6)


@pytest.mark.parametrize("dims", [(33,), (12, 10), (6, 5, 4), (2, 7), (9000,), (8300, 2)],
                         ids=lambda d: "x".join(map(str, d)))
def test_column_grad_vs_oracle(dims):
    """hgp_plan_column_grad for every operator on grids beyond the golden shapes (incl. an axis
    of 2 points, whose embedding has no interior copy, and axes beyond 8192 points: the full-grid
    route's radix-2 levels and long-axis DCT), fp64, against the oracle."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    rs = np.random.RandomState(sum(dims))
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda a, b: zo.kernel_eval("matern", a, b, (1., .3), nu=1.5), 1e-3)
    T = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, dtype=torch.float64, device=DEV)
    P.set_column(torch.tensor(col, device=DEV))
    M, Mp = T.M, T.Mp
    for op, name, nin, nout in ((_lib.OP_K, "K", M, M), (_lib.OP_CINV, "Cinv", M, M),
                                (_lib.OP_RT, "RT", M, Mp), (_lib.OP_R, "R", Mp, M)):
        x, g = rs.randn(3, nin), rs.randn(3, nout)
        got = P.column_grad(op, torch.tensor(x, device=DEV), torch.tensor(g, device=DEV))
        assert rel_err(_np(got), T.column_grad(name, x, g)) < 1e-9, name


@pytest.mark.parametrize("scale", [1e6, 1e-6], ids=["x_big", "x_small"])
def test_column_grad_mismatched_scales(scale):
    """The column gradient correlates x with the upstream gradient g through one packed complex
    transform (x + i g): with |x| / |g| = 1e6 (a solve at the 1e-6 clamp against an O(1) loss
    gradient) or 1e-6, the smaller one must not carry the larger one's rounding -- g is packed at
    x's magnitude by a power of two (hgp_grad.hip k_absmax2 / pack_scale).  fp64 vs the oracle."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims = (24, 20)
    rs = np.random.RandomState(7)
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda a, b: zo.kernel_eval("matern", a, b, (1., .3), nu=1.5), 1e-3)
    T = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, dtype=torch.float64, device=DEV)
    P.set_column(torch.tensor(col, device=DEV))
    for op, name, nin, nout in ((_lib.OP_K, "K", T.M, T.M), (_lib.OP_CINV, "Cinv", T.M, T.M),
                                (_lib.OP_RT, "RT", T.M, T.Mp), (_lib.OP_R, "R", T.Mp, T.M)):
        x, g = rs.randn(2, nin) * scale, rs.randn(2, nout)
        got = P.column_grad(op, torch.tensor(x, device=DEV), torch.tensor(g, device=DEV))
        err = rel_err(_np(got), T.column_grad(name, x, g))
        print(name, scale, err)
        assert err < 1e-12, (name, err)


@pytest.mark.parametrize("dims", [(300,), (12, 10), (2, 9), (6, 5, 4), (3, 2, 7), (9000,)],
                         ids=lambda d: "x".join(map(str, d)))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_plan_dqf_vs_oracle(dims, tag):
    """hgp_plan_dqf (the flattened-index quadratic form through the grid's factorisation) against
    the oracle's 1-D restatement and the direct-sum kernel, incl. axes of 2 points."""
    from hipgp_amd.plan import ToeplitzPlan, sym_toeplitz_dqf
    rs = np.random.RandomState(len(dims) * 7 + dims[-1])
    M = int(np.prod(dims))
    l, r = rs.randn(4, M), rs.randn(4, M)
    P = ToeplitzPlan(dims, dtype=DT[tag], device=DEV)
    P.set_column(torch.tensor(np.exp(-np.arange(M) / 5.0), dtype=DT[tag], device=DEV))
    got = P.dqf(torch.tensor(l, dtype=DT[tag], device=DEV), torch.tensor(r, dtype=DT[tag], device=DEV))
    want = zo.sym_toeplitz_dqf(l.T, r.T)
    tol = 1e-12 if tag == "f64" else 2e-6
    assert rel_err(_np(got), want) < tol
    direct = sym_toeplitz_dqf(torch.tensor(l.T, dtype=DT[tag], device=DEV),
                              torch.tensor(r.T, dtype=DT[tag], device=DEV))
    assert rel_err(_np(direct), want) < tol
