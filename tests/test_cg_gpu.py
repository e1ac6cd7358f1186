"""Row a11 and the generic CG paths on the GPU:
  * `conj_grad` (column layout, `cg.py:5-41`) with the ColumnOp operators `gram_solve` builds
    -> one fused hgp_pcg_solve(LAYOUT_COLS), against the reference's G1 goldens (config-1 shape);
  * `conj_grad` / `conj_grad2` (`cg.py:44-80`) with arbitrary callables (the `_generic`
    recurrence with hgp_rowdot dots) against the G1 / G2 goldens;
  * hgp_pcg_solve(LAYOUT_COLS) == LAYOUT_ROWS bit for bit (same kernels after a device
    transpose), with and without iters_done, 1-D / 2-D / 3-D;
  * hgp_rowdot against torch, alternating streams and growing sizes (pooled scratch)."""
import numpy as np
import pytest
import torch

from golden_cases import GRID_CASES, load, grids_of, pcg_ok, rel_err
from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _np(t):
    return t.detach().cpu().numpy()


def _g1_matmul(fx, dtype):
    import ziggy.kernels as zk
    from ziggy.misc import toeplitz_expanded as te
    k = zk.Matern(nu=2.5, dtype=dtype)
    kf = lambda x, y: k.forward(x, y, params=(1., .1))
    g = torch.tensor(fx["grid0"], device=DEV)
    vec = torch.tensor(fx["vec"], device=DEV)
    return te.ToeplitzMatmul([g], kf, batch_shape=vec.shape[:-1]), vec


def _check_g1(res, its, fx, f64, key, tag):
    assert res.shape == fx[key].shape, key
    if tag == "f64":
        tol = 1e-5 if "p1" in key else 1e-3   # no nugget: cond ~3e5 (see test_parity_gpu)
        assert rel_err(res, fx[key]) < tol, (key, rel_err(res, fx[key]))
        assert len(its) == int(fx[key + "_ncb"]), (key, len(its))
    else:
        ok, (e, eref) = pcg_ok(res, fx[key], f64[key])
        assert ok, (key, e, eref)


@pytest.mark.parametrize("tag", ["f64", "f32"])
@pytest.mark.parametrize("fused", [True, False], ids=["ColumnOp_fused", "lambdas_generic"])
def test_conj_grad_columns_G1(tag, fused):
    """`gram_solve`'s own call (`toeplitz_expanded.py:46-53`): conj_grad on vec^T (M, bsz)."""
    from hipgp_amd import _lib
    from ziggy.misc.cg import ColumnOp, conj_grad
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx, f64 = load("G1", tag), load("G1", "f64")
    K, vec = _g1_matmul(fx, dtype)
    for pre in (0, 1):
        if fused:
            Kmul = ColumnOp(K._plan, _lib.OP_K)
            P = ColumnOp(K._plan, _lib.OP_CINV) if pre else None
        else:
            Kmul = lambda x: K(x.t(), multiply_type="gram").t()
            P = (lambda x: K(x.t(), multiply_type="circ_inv").t()) if pre else None
        for mi in (1, 5, 20):
            its = []
            shapes = set()

            def cb(n, x):
                its.append(n)
                shapes.add(tuple(x.shape))
            d = conj_grad(Kmul, vec.t(), precond=P, maxiter=mi, tol=1e-10, callback=cb)
            assert tuple(d.shape) == (vec.shape[1], vec.shape[0])
            assert shapes <= {(vec.shape[1], vec.shape[0])}   # the callback sees (M, bsz)
            _check_g1(_np(d.t()), its, fx, f64, f"gram_p{pre}_rt0_it{mi}", tag)
            # and without a callback (no per-iteration host stepping)
            d2 = conj_grad(Kmul, vec.t(), precond=P, maxiter=mi, tol=1e-10)
            if fused:
                assert torch.equal(d2, d)
            else:
                _check_g1(_np(d2.t()), its, fx, f64, f"gram_p{pre}_rt0_it{mi}", tag)


@pytest.mark.parametrize("name", ["G2", "G3", "G7"])
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_conj_grad2_generic_callables(name, tag):
    """conj_grad2 with callables that are not a ToeplitzTensor's bound methods: the generic
    recurrence (torch axpys + hgp_rowdot dots), against the reference's _solve goldens."""
    import ziggy.kernels as zk
    from ziggy.misc.cg import conj_grad2
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx, f64, f32 = load(name, tag), load(name, "f64"), load(name, "f32")
    kind, nu, params, jit = GRID_CASES[name]
    k = zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)
    grids = [torch.tensor(g, dtype=dtype, device=DEV) for g in grids_of(fx)]
    T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=params), jitter_val=jit)
    v = torch.tensor(fx["v"], device=DEV)
    T.set_batch_shape(v.shape[:-1])
    A = lambda x: T._matmul_by_K(x)
    P = lambda x: T._matmul_by_Cinv(x)
    for mi in (1, 2, 5):
        key = f"solve_p1_it{mi}"
        x = _np(conj_grad2(A, v, precond=P, maxiter=mi, tol=1e-8))
        if tag == "f64":
            assert rel_err(x, f64[key]) < 1e-8, (key, rel_err(x, f64[key]))
        else:
            assert pcg_ok(x, f32[key], f64[key])[0], key
    x = _np(conj_grad2(A, v, precond=None, maxiter=5, tol=1e-8))
    if tag == "f64":
        assert rel_err(x, f64["solve_p0_it5"]) < 1e-8
    else:
        assert pcg_ok(x, f32["solve_p0_it5"], f64["solve_p0_it5"])[0]


@pytest.mark.parametrize("dims,dtype", [((300,), torch.float64), ((64, 48), torch.float32), ((65, 64), torch.float32),
                                        ((33, 40), torch.float64), ((16, 12, 10), torch.float64),
                                        ((1024, 1024), torch.float32)],
                         ids=["1d_f64", "2d_f32", "2d_odd_f32", "2d_f64", "3d_f64", "C2_f32"])
def test_pcg_cols_layout_equals_rows(dims, dtype):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 1e-2)
    P = ToeplitzPlan(dims, dtype, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=dtype))
    g = torch.Generator(device=DEV).manual_seed(11)
    B = 5
    b = torch.randn(B, int(np.prod(dims)), device=DEV, generator=g, dtype=torch.float64).to(dtype)
    for pre in (True, False):
        xr, ir = P.pcg(b, 12, 1e-30, precond=pre, return_iters=True)
        xc, ic = P.pcg(b.t().contiguous(), 12, 1e-30, precond=pre, return_iters=True, layout=_lib.LAYOUT_COLS)
        xc2 = P.pcg(b.t().contiguous(), 12, 1e-30, precond=pre, layout=_lib.LAYOUT_COLS)
        assert tuple(xc.shape) == (b.shape[1], B)
        assert torch.equal(xc.t(), xr) and torch.equal(xc2, xc)
        assert ir == ic
    # early break in column layout: the iteration count matches the row layout's
    rtol = 1e-3 if dtype == torch.float64 else 3e-2     # fp32 stalls near its rounding floor
    xr, ir = P.pcg(b, 200, rtol * float(b.norm(dim=1).min()), precond=True, return_iters=True)
    xc, ic = P.pcg(b.t().contiguous(), 200, rtol * float(b.norm(dim=1).min()), precond=True, return_iters=True,
                   layout=_lib.LAYOUT_COLS)
    assert ir == ic < 200 and torch.equal(xc.t(), xr)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_rowdot_pooled(dtype):
    from hipgp_amd.plan import rowdot
    g = torch.Generator(device=DEV).manual_seed(3)
    side = torch.cuda.Stream()
    for i, (B, M) in enumerate([(3, 17), (32, 1 << 20), (7, 5000), (64, 300001), (1, 1)]):
        a = torch.randn(B, M, device=DEV, generator=g, dtype=dtype)
        c = torch.randn(B, M, device=DEV, generator=g, dtype=dtype)
        st = side if i % 2 else torch.cuda.current_stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            out = rowdot(a, c)
            ref = (a.double() * c.double()).sum(1)
        torch.cuda.current_stream().wait_stream(st)
        tol = 1e-12 if dtype == torch.float64 else 1e-5
        err = float(((out.double() - ref).abs() / (a.double().norm(dim=1) * c.double().norm(dim=1))).max())
        assert err < tol, (B, M, err)
