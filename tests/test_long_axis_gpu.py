"""Grid axes longer than 4097 points (the reference has no length limit, `toeplitz_tensor.py:85-97`).

An axis of m in 4098..8192 points needs L_R >= 3m - 3 > 12288-point transforms for R / R^T:
fp32 plans run them as one-line-per-block passes (H up to 16384), and the fp64 set-up of every
plan transforms the L_R grid with fft_lines_f64's radix-2 step (two half-length transforms +
k_r2_combine).  fp64 plans run K / C^-1 lines of up to 8192 points per half (one line per block)
and R / R^T either as passes (L_R / 2 <= 8192: axes up to 5462 points with the 3 * 2^k or
power-of-two L_R <= 16384) or, beyond that, on the full fp64 L_R grid (run_op_grid).  Here the
operators and PCG of 1-D / 2-D / 3-D grids with such an axis (any position) are checked against
the fp64 oracle of the same column, in both dtypes; axes beyond 8192 points are refused."""
import numpy as np
import pytest
import torch

from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = {"1d_5000": (5000,), "2d_4200x12": (4200, 12), "2d_10x4500": (10, 4500),
         "3d_4100x5x4": (4100, 5, 4), "3d_4x4100x3": (4, 4100, 3), "3d_3x5x4300": (3, 5, 4300)}


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


def test_long_axis_refusals():
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    for dt in (torch.float32, torch.float64):
        with pytest.raises(_lib.HipgpError, match="longer than 8192"):
            ToeplitzPlan((8193,), dt, DEV)
        with pytest.raises(_lib.HipgpError, match="longer than 8192"):
            ToeplitzPlan((3, 8193), dt, DEV)
    ToeplitzPlan((8192, 3), torch.float64, DEV)        # the limit itself is accepted in fp64 too
