"""Grid axes longer than 4097 points (the reference has no length limit, `toeplitz_tensor.py:85-97`).

An axis of m in 4098..8192 points needs L_R >= 3m - 3 > 12288-point transforms for R / R^T:
fp32 plans run them as one-line-per-block passes (H up to 16384), and the fp64 set-up of every
plan transforms the L_R grid with fft_lines_f64's radix-2 step (two half-length transforms +
k_r2_combine).  fp64 plans run K / C^-1 lines of up to 8192 points per half (one line per block)
and R / R^T either as passes (L_R / 2 <= 8192: axes up to 5462 points with the 3 * 2^k or
power-of-two L_R <= 16384) or, beyond that, on the full fp64 L_R grid (run_op_grid).  Here the
operators and PCG of 1-D / 2-D / 3-D grids with such an axis (any position) are checked against
the fp64 oracle of the same column, in both dtypes.

Round 4: axes of MORE than 8192 points (the passes hold lines of at most 16384 fp32 / 8192 fp64
points) run every operator on the full fp64 grid (run_op_grid): the set-up's DCT-I (Bluestein),
the L_K / L_R grid transforms and the operators go through fft_lines_f64's radix-2 levels as
deep as the length needs (9000 points: L_K = L_R = 32768, one level; 12000: L_R = 49152, two
levels to a 12288-point base; 20000: L_K = L_R = 65536, two levels), fp32 plans with fp32 in /
out.  The PCG runs the unfused iteration (dots by row-chunk partials).  `LONG_CASES` pin them
against the fp64 oracle like the cases above."""
import numpy as np
import pytest
import torch

from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = {"1d_5000": (5000,), "2d_4200x12": (4200, 12), "2d_10x4500": (10, 4500),
         "3d_4100x5x4": (4100, 5, 4), "3d_4x4100x3": (4, 4100, 3), "3d_3x5x4300": (3, 5, 4300)}
# axes beyond 8192 points: the full-grid route for every operator
LONG_CASES = {"1d_9000": (9000,), "1d_20000": (20000,), "2d_10000x6": (10000, 6), "2d_5x12000": (5, 12000),
              "3d_3x9000x4": (3, 9000, 4)}


def _column(dims):
    # Matern-3/2 with ell = 20 grid spacings, nugget 0.1: a well-conditioned K
    grids = [np.linspace(-1, 1, m) for m in dims]
    ell = 40.0 / max(dims)
    return zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1.0, ell), nu=1.5), 0.1)


@pytest.mark.parametrize("case", sorted(CASES))
def test_long_axis_ops_and_pcg_fp32(case):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims = CASES[case]
    col = _column(dims)
    O = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, torch.float32, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=torch.float32))
    M, Mp = O.M, O.Mp
    rs = np.random.RandomState(3)
    v = rs.randn(3, M)
    w = rs.randn(3, Mp)
    for name, op, x, ref in (("K", _lib.OP_K, v, O.matmul_K(v)), ("Cinv", _lib.OP_CINV, v, O.matmul_Cinv(v)),
                             ("RT", _lib.OP_RT, v, O.matmul_RT(v)), ("R", _lib.OP_R, w, O.matmul_R(w))):
        got = P.apply(op, torch.tensor(x, device=DEV, dtype=torch.float32)).double().cpu().numpy()
        assert got.shape == ref.shape, name
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        # fp32 transforms of up to 32768 points: a few ulp of log2(L) ~ 15 stages
        assert err < 2e-5, (name, err)
    b = rs.randn(2, M)
    x_ref = O.solve(b, do_precond=True, maxiter=10, tol=1e-30)
    x_ref32 = zo.ToeplitzOracle(col.astype(np.float32), dims).solve(b.astype(np.float32), do_precond=True,
                                                                     maxiter=10, tol=1e-30)
    x = P.pcg(torch.tensor(b, device=DEV, dtype=torch.float32), 10, 1e-30, precond=True).double().cpu().numpy()
    e = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    e_ref = np.linalg.norm(x_ref32.astype(np.float64) - x_ref) / np.linalg.norm(x_ref)
    assert e <= 4 * e_ref + 1e-6, (e, e_ref)        # SURVEY §8(c) fp32 PCG bound
    # the whitening identity on the same grid: R (R^T v) = K v
    vt = torch.tensor(v, device=DEV, dtype=torch.float32)
    rr = P.apply(_lib.OP_R, P.apply(_lib.OP_RT, vt)).double().cpu().numpy()
    kv = O.matmul_K(v)
    assert float(np.abs(rr - kv).max() / np.abs(kv).max()) < 3e-5


# fp64: pass route (L_R / 2 <= 8192) and full-grid R / R^T route (6000-point axes)
CASES64 = {"1d_5000": (5000,), "2d_4200x12": (4200, 12), "2d_10x4500": (10, 4500), "3d_3x5x4300": (3, 5, 4300),
           "2d_6000x10": (6000, 10), "3d_4x6000x3": (4, 6000, 3), "2d_8x8192": (8, 8192)}


@pytest.mark.parametrize("case", sorted(CASES64))
def test_long_axis_ops_and_pcg_fp64(case):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims = CASES64[case]
    col = _column(dims)
    O = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, torch.float64, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=torch.float64))
    M, Mp = O.M, O.Mp
    rs = np.random.RandomState(5)
    v = rs.randn(2, M)
    w = rs.randn(2, Mp)
    for name, op, x, ref in (("K", _lib.OP_K, v, O.matmul_K(v)), ("Cinv", _lib.OP_CINV, v, O.matmul_Cinv(v)),
                             ("RT", _lib.OP_RT, v, O.matmul_RT(v)), ("R", _lib.OP_R, w, O.matmul_R(w))):
        got = P.apply(op, torch.tensor(x, device=DEV, dtype=torch.float64)).cpu().numpy()
        assert got.shape == ref.shape, name
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        assert err < 1e-10, (name, err)
    b = rs.randn(2, M)
    x_ref = O.solve(b, do_precond=True, maxiter=10, tol=1e-30)
    x = P.pcg(torch.tensor(b, device=DEV), 10, 1e-30, precond=True).cpu().numpy()
    assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) < 1e-9
    vt = torch.tensor(v, device=DEV)
    rr = P.apply(_lib.OP_R, P.apply(_lib.OP_RT, vt)).cpu().numpy()
    kv = O.matmul_K(v)
    assert float(np.abs(rr - kv).max() / np.abs(kv).max()) < 1e-10
    if max(dims) > 5462:
        # the full-grid R / R^T route: its two L_R-grid buffers are scratch and its stored-order
        # spectrum a table in hgp_plan_mem (so the plan pool sees them)
        nLR = int(np.prod(P.L_R[:len(dims)]))
        mem = P.mem()
        assert mem["scratch"] >= 2 * nLR * 16 and mem["tables"] >= nLR * 16, (mem, nLR)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("case", sorted(LONG_CASES))
def test_beyond_8192_points(case, dt):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims = LONG_CASES[case]
    col = _column(dims)
    O = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, dt, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=dt))
    rs = np.random.RandomState(6)
    v = rs.randn(2, O.M)
    w = rs.randn(2, O.Mp)
    # measured (profiles/r4_w_long_axis_op_errors.txt): fp64 2e-15 .. 2.4e-14 (C^-1), fp32 6e-8 ..
    # 1.3e-6 (C^-1) -- an exact implementation's rounding; the bounds keep >= 8x margin
    tol_op = 1e-5 if dt == torch.float32 else 1e-12
    for name, op, x, ref in (("K", _lib.OP_K, v, O.matmul_K(v)), ("Cinv", _lib.OP_CINV, v, O.matmul_Cinv(v)),
                             ("RT", _lib.OP_RT, v, O.matmul_RT(v)), ("R", _lib.OP_R, w, O.matmul_R(w))):
        got = P.apply(op, torch.tensor(x, device=DEV, dtype=dt)).double().cpu().numpy()
        assert got.shape == ref.shape, name
        err = float(np.abs(got - ref).max() / np.abs(ref).max())
        print(case, dt, name, "op err vs oracle", err)
        assert err < tol_op, (name, err)
    # the spectrum served to ToeplitzTensor.D (n-grid) from the long-axis DCT set-up
    D = P.spectrum(_lib.SPEC_D).double().cpu().numpy().reshape(-1)
    assert float(np.abs(D - O.D.reshape(-1)).max() / np.abs(O.D).max()) < (1e-6 if dt == torch.float32 else 1e-12)
    b = rs.randn(2, O.M)
    x_ref = O.solve(b, do_precond=True, maxiter=10, tol=1e-30)
    x, it = P.pcg(torch.tensor(b, device=DEV, dtype=dt), 10, 1e-30, precond=True, return_iters=True)
    err = float(np.linalg.norm(x.double().cpu().numpy() - x_ref) / np.linalg.norm(x_ref))
    calls = []
    O.solve(b, do_precond=True, maxiter=10, tol=1e-30, callback=lambda n, xx: calls.append(n))
    rr = [float(np.linalg.norm(O.matmul_K(x.double().cpu().numpy())[j] - b[j])) for j in range(2)]
    print(case, dt, "iterations", it, "oracle callbacks", len(calls), "err", err, "true residual", rr)
    assert err < (1e-4 if dt == torch.float32 else 1e-9), err
    if dt == torch.float64:
        # the recursive r.r falls below tol^2 = 1e-60 after 8 iterations here, in the oracle too
        # (fp32's cannot underflow that far: 10 iterations)
        assert it == min(10, len(calls) + 1)
    # the break rule on this route (unfused iteration): the iterate of a maxiter stop
    xb, itb = P.pcg(torch.tensor(b, device=DEV, dtype=dt), 200, float(np.linalg.norm(b[0])) * 1e-3, precond=True,
                    return_iters=True)
    xs = P.pcg(torch.tensor(b, device=DEV, dtype=dt), itb, 1e-30, precond=True)
    assert itb < 200 and torch.equal(xb, xs)


def test_long_axis_refusals():
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    # axes of more than 8192 points are accepted (full-grid route); grid-block sharding of them is not
    P = ToeplitzPlan((8193, 3), torch.float32, DEV)
    col = _column((8193, 3))
    P.set_column(torch.tensor(col, device=DEV, dtype=torch.float32))
    import ctypes
    with pytest.raises(_lib.HipgpError, match="full-grid route"):
        E = torch.empty(1024 * 1024, dtype=torch.complex64, device=DEV)
        x = torch.zeros(1, 8193 * 3, device=DEV)
        _lib.check(_lib.lib().hgp_slab_pass(P._h, _lib.OP_K, _lib.SLAB_FWD, ctypes.c_void_p(x.data_ptr()),
                                            ctypes.c_void_p(E.data_ptr()), 1, 1, 0, 0))
    ToeplitzPlan((8192, 3), torch.float64, DEV)        # the pass limit itself


def test_beyond_8192_drop_in_compute_kn():
    """The drop-in ToeplitzTensor (`toeplitz_tensor.py:9-52`) and `compute_kn` (`hipgp.py:117-146`)
    on a 9000 x 3 grid (full-grid route), fp64, against the oracle's compute_kn of the same column."""
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    dims = (9000, 3)
    ell = 40.0 / max(dims)
    k = zk.Matern(nu=1.5, dtype=torch.float64)
    grids = [torch.linspace(-1, 1, m, dtype=torch.float64, device=DEV) for m in dims]
    T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=(1.0, ell)), jitter_val=0.1)
    col = T.column.detach().cpu().numpy()
    O = zo.ToeplitzOracle(col, dims)
    assert np.abs(col - _column(dims)).max() < 1e-12        # the same first row as the oracle's
    Knm = np.random.RandomState(8).rand(3, O.M)
    d0 = T.inv_matmul(torch.tensor(Knm, device=DEV), do_precond=True, maxiter=20, tol=1e-8)
    kn = T._matmul_by_RT(d0).cpu().numpy()
    ref = zo.compute_kn(O, Knm, maxiter_cg=20, tol=1e-8)
    assert kn.shape == ref.shape == (3, O.Mp)
    assert np.linalg.norm(kn - ref) / np.linalg.norm(ref) < 1e-9
