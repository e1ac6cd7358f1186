"""GPU parity: the HIP path (through the C ABI, via the ziggy drop-in) against the
reference's golden vectors (tests/golden, made by running /root/reference) and against the
CPU oracle.  Tolerances:
  fp32 ops  : max|y - y_ref| <= 1e-5 max|y_ref| + 1e-7, or no worse than 4x the reference's
              own fp32 error vs fp64 (ops near the clamp, see golden_cases.op_ok)
  fp32 PCG  : ||x - x64|| <= 4 ||x_ref32 - x64|| + 1e-6 ||x64||
  fp64      : ops within 50x the NumPy oracle's own error vs the reference; PCG 1e-8
  clamped 20-iteration solves (G4a-c, G7: chaotic at the 1e-6 clamp): within 10x the reference's
              own spread over nine self-perturbed re-runs (tests/golden/make_golden_clamp_alt.py),
              plus the true-residual check
"""
import os

import numpy as np
import pytest
import torch

from golden_cases import GRID_CASES, CLAMPED, load, grids_of, rel_err, op_ok, pcg_ok, alt_spread, chaotic_bound
from oracle import ziggy_oracle as zo

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _kernel(kind, nu, dtype):
    import ziggy.kernels as zk
    return zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)


def _tt(fx, name, dtype):
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    kind, nu, params, jit = GRID_CASES[name]
    k = _kernel(kind, nu, dtype)
    grids = [torch.tensor(g, dtype=dtype, device=DEV) for g in grids_of(fx)]
    return ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=params), jitter_val=jit)


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", sorted(GRID_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_ops_vs_golden(name, tag):
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx = load(name, tag)
    f64 = load(name, "f64")
    T = _tt(fx, name, dtype)
    assert rel_err(_np(T.column), fx["column"]) < (1e-12 if tag == "f64" else 2e-6)
    # C is an exact rearrangement of our column; the column itself is a GPU kernel evaluation
    np.testing.assert_array_equal(_np(T.C), zo.circulant_embed(_np(T.column).reshape(T.dims)))
    assert rel_err(_np(T.C), fx["C"]) < (1e-12 if tag == "f64" else 2e-6)
    # spectrum (computed in fp64 on the device for both plan dtypes)
    dtol = 1e-12 if tag == "f64" else 1e-6
    assert rel_err(_np(T.D[..., 0]), f64["D"]) < dtol
    assert rel_err(_np(T.D_sqrt[..., 0]).astype(np.float64) ** 2, f64["D_sqrt"] ** 2) < dtol
    assert rel_err(1 / _np(T.Di[..., 0]).astype(np.float64), 1 / f64["Di"]) < dtol
    if tag == "f64":
        assert np.array_equal(_np(T.D[..., 0]) <= 1e-6, fx["D"] <= 1e-6)
        # the set-up's clamp counter (hgp_plan_set_column n_clamped) against the raw spectrum
        from hipgp_amd.plan import ToeplitzPlan
        P = ToeplitzPlan(T.dims, dtype=torch.float64, device=DEV)
        # (the golden column already holds the jitter on c0, as the reference's T.column)
        n = P.set_column(torch.tensor(fx["column"], device=DEV), count_clamped=True)
        raw = np.fft.fftn(zo.circulant_embed(fx["column"].reshape(T.dims))).real
        assert n == int(np.sum(raw < 1e-6)), (n, int(np.sum(raw < 1e-6)))
    v = torch.tensor(fx["v"], device=DEV)
    w = torch.tensor(fx["w"], device=DEV)
    T.set_batch_shape(v.shape[:-1])
    O = zo.ToeplitzOracle(f64["column"].astype(np.float64), T.dims)
    oracle = {"Kv": O.matmul_K, "Cinv_v": O.matmul_Cinv, "RTv": O.matmul_RT, "Rw": O.matmul_R}
    for key, fn, x in (("Kv", T._matmul_by_K, v), ("Cinv_v", T._matmul_by_Cinv, v),
                       ("RTv", T._matmul_by_RT, v), ("Rw", T._matmul_by_R, w)):
        y = _np(fn(x))
        assert y.shape == fx[key].shape, key
        if tag == "f64":
            # as accurate as an exact fp64 FFT implementation: within 50x the NumPy oracle's own
            # distance from the reference (1e-9 before round 4 -- loose enough to hide a 400x K
            # error at the clamp)
            e_or = rel_err(oracle[key](f64["v" if key != "Rw" else "w"].astype(np.float64)), fx[key])
            print(name, key, "gpu", rel_err(y, fx[key]), "oracle", e_or)
            assert rel_err(y, fx[key]) <= 50 * e_or + 1e-14, (key, rel_err(y, fx[key]), e_or)
        else:
            assert op_ok(y, fx[key], f64[key]), (key, rel_err(y, f64[key]), rel_err(fx[key], f64[key]))


@pytest.mark.parametrize("name", sorted(GRID_CASES))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_solves_vs_golden(name, tag):
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx = load(name, tag)
    f64 = load(name, "f64")
    f32 = load(name, "f32")
    T = _tt(fx, name, dtype)
    v = torch.tensor(fx["v"], device=DEV)
    for mi in (1, 2, 5, 20):
        key = f"solve_p1_it{mi}"
        x = _np(T._solve(v, do_precond=True, maxiter=mi, tol=1e-8))
        chaotic = name in CLAMPED and mi == 20
        if tag == "f64":
            assert rel_err(x, f64[key]) < (0.25 if chaotic else 1e-8), (key, rel_err(x, f64[key]))
        else:
            ok, (e, eref) = pcg_ok(x, f32[key], f64[key])
            assert ok or chaotic, (key, e, eref)
        if chaotic:
            # eigenvalues at the 1e-6 clamp: 20 iterations amplify rounding chaotically, so two
            # implementations' iterates differ.  (1) Against the reference's own spread: its nine
            # self-perturbed re-runs (tests/golden/make_golden_clamp_alt.py) land up to `spread`
            # from its golden (fp64 1.4e-5 .. 0.14, fp32 4.8e-4 .. 0.26); ours is within 10x that
            # (capped at 0.25 / 0.5; golden_cases.chaotic_bound).  (2) How far it got: the true
            # residual |K x - b| (fp64 oracle K) of ours is within 3x of the reference's own
            # (0.3-12 |b| after 20 iterations: neither has converged).
            print(name, tag, key, "err vs reference", rel_err(x, fx[key]), "reference spread", alt_spread(name, tag, key))
            assert rel_err(x, fx[key]) <= chaotic_bound(name, tag, key), (key, rel_err(x, fx[key]))
            O = zo.ToeplitzOracle(_np(T.column).astype(np.float64), T.dims)
            b64 = fx["v"].astype(np.float64)
            res = lambda y: float(np.linalg.norm(O.matmul_K(y.astype(np.float64)) - b64) / np.linalg.norm(b64))
            ref = max(res(f64[key]), res(f32[key])) if tag == "f32" else res(f64[key])
            assert res(x) <= 3 * ref + 1e-12, (key, res(x), ref)
    x = _np(T._solve(v, do_precond=False, maxiter=5, tol=1e-8))
    if tag == "f64":
        assert rel_err(x, f64["solve_p0_it5"]) < 1e-8
    else:
        assert pcg_ok(x, f32["solve_p0_it5"], f64["solve_p0_it5"])[0]
    kn = _np(T._matmul_by_RT(T.inv_matmul(v, do_precond=True, maxiter=20, tol=1e-8)))
    if name in CLAMPED:
        print(name, tag, "kn_it20 err vs reference", rel_err(kn, fx["kn_it20"]), "reference spread",
              alt_spread(name, tag, "kn_it20"))
        assert rel_err(kn, fx["kn_it20"]) <= chaotic_bound(name, tag, "kn_it20"), rel_err(kn, fx["kn_it20"])
    elif tag == "f64":
        assert rel_err(kn, f64["kn_it20"]) < 1e-8
    else:
        assert pcg_ok(kn, f32["kn_it20"], f64["kn_it20"])[0]


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_gram_solve_config1(tag):
    import ziggy.kernels as zk
    from ziggy.misc import toeplitz_expanded as te
    dtype = torch.float64 if tag == "f64" else torch.float32
    fx = load("G1", tag)
    f64 = load("G1", "f64")
    k = zk.Matern(nu=2.5, dtype=dtype)
    kf = lambda x, y: k.forward(x, y, params=(1., .1))
    g = torch.tensor(fx["grid0"], device=DEV)
    vec = torch.tensor(fx["vec"], device=DEV)
    g64 = np.asarray(fx["grid0"], np.float64)
    O = zo.ToeplitzOracle(zo.toeplitz_column([g64], lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=2.5), 0.0),
                          (len(g64),))
    b64 = np.asarray(fx["vec"], np.float64)

    def Kres(x):      # gram_solve works on vec.t(): rows of x / b are the RHS
        x = np.asarray(x, np.float64)
        xr, br = (x, b64) if x.shape == b64.shape else (x.T, b64.T)
        return float(np.linalg.norm(O.matmul_K(np.ascontiguousarray(xr)) - br) / np.linalg.norm(br))

    for pre in (0, 1):
        for rt in (0, 1):
            for mi in (1, 5, 20):
                key = f"gram_p{pre}_rt{rt}_it{mi}"
                its = []
                res = _np(te.gram_solve([g], kf, vec, maxiter=mi, do_precond=bool(pre), tol=1e-10,
                                        callback=lambda n, x: its.append(n), mult_RT=bool(rt)))
                assert res.shape == fx[key].shape
                if tag == "f64":
                    # no nugget (toeplitz_expanded.py:248): cond(K) ~ 3e5, so CG amplifies
                    # the rounding difference of the FFT lengths (ours L=512, ref n=510)
                    tol = 1e-5 if pre else 1e-3
                    assert rel_err(res, fx[key]) < tol, (key, rel_err(res, fx[key]))
                    assert len(its) == int(fx[key + "_ncb"]), (key, len(its))
                    if not rt:
                        # and the true residual |K x - b| (oracle K of the same column) agrees
                        # with the reference's own to 1 % (or 1e-8 of |b| once converged)
                        r_ours, r_ref = Kres(res), Kres(fx[key])
                        assert abs(r_ours - r_ref) <= 1e-2 * r_ref + 1e-8, (key, r_ours, r_ref)
                else:
                    ok, (e, eref) = pcg_ok(res, fx[key], f64[key])
                    assert ok, (key, e, eref)


def test_compute_kn_model_G5():
    """kn = R^T K^{-1} Knm^T as `hipgp.compute_kn` (hipgp.py:139-146), model-level fixture."""
    fx = load("G5", "f64")
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    k = zk.Matern(nu=1.5, dtype=torch.float64)
    kf = lambda x, y: k.forward(x, y, params=(1., .1))
    grids = [torch.tensor(fx["grid0"], device=DEV), torch.tensor(fx["grid1"], device=DEV)]
    T = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=1e-3)
    Knm = torch.tensor(fx["Knm"], device=DEV)
    kn = T._matmul_by_RT(T.inv_matmul(Knm, do_precond=True, maxiter=20, tol=1e-8))
    assert rel_err(_np(kn), fx["kn"]) < 1e-8


# ---- oracle comparisons at sizes the golden set does not cover -----------------------------
ORACLE_CASES = [
    ((300,), "matern", 2.5, (1., .05)),
    ((64, 48), "sqexp", None, (1., .08)),
    ((33, 17), "matern", 1.5, (1., .2)),
    ((16, 12, 10), "matern", .5, (1., .3)),
    ((9, 1, 7), "sqexp", None, (1., .3)),
]


@pytest.mark.parametrize("case", ORACLE_CASES, ids=lambda c: "x".join(map(str, c[0])))
def test_ops_and_solve_vs_oracle_f64(case):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims, kind, nu, params = case
    grids = [np.linspace(-1, 1, m) for m in dims]
    kf = lambda x, y: zo.kernel_eval(kind, x, y, params, nu=nu)
    col = zo.toeplitz_column(grids, kf, 1e-3)
    T = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, torch.float64, DEV)
    P.set_column(torch.tensor(col, device=DEV))
    rs = np.random.RandomState(3)
    B = 5
    v = rs.randn(B, T.M)
    w = rs.randn(B, T.Mp)
    vt = torch.tensor(v, device=DEV)
    for op, ref in ((_lib.OP_K, T.matmul_K(v)), (_lib.OP_CINV, T.matmul_Cinv(v)), (_lib.OP_RT, T.matmul_RT(v))):
        assert rel_err(_np(P.apply(op, vt)), ref) < 1e-10, op
    assert rel_err(_np(P.apply(_lib.OP_R, torch.tensor(w, device=DEV))), T.matmul_R(w)) < 1e-10
    x = _np(P.pcg(vt, 10, 1e-8, precond=True))
    assert rel_err(x, T.solve(v, True, 10, 1e-8)) < 1e-7


# ---- size-independent properties at BASELINE sizes ------------------------------------------
@pytest.mark.parametrize("dims", [(1024, 1024), (256, 256, 128)], ids=["C2_1024x1024", "C5_256x256x128"])
def test_properties_full_size(dims):
    """R (R^T v) = K v (same clamped spectrum), symmetry <u,Kv> = <Ku,v>, linearity, and PCG
    residual decrease — at the headline grid sizes, fp32."""
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    k = zk.SqExp(dtype=torch.float32) if len(dims) == 2 else zk.Matern(nu=2.5, dtype=torch.float32)
    params = (1., .01) if len(dims) == 2 else (.1, .1)
    grids = [torch.linspace(-1, 1, m, device=DEV) for m in dims]
    T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=params), jitter_val=1e-3)
    g = torch.Generator(device=DEV).manual_seed(0)
    B = 4
    u = torch.randn(B, T.M, device=DEV, generator=g)
    v = torch.randn(B, T.M, device=DEV, generator=g)
    T.set_batch_shape((B,))
    Kv = T._matmul_by_K(v)
    RRv = T._matmul_by_R(T._matmul_by_RT(v))
    assert float((RRv - Kv).abs().max() / Kv.abs().max()) < 1e-4
    Ku = T._matmul_by_K(u)
    lhs = (u.double() * Kv.double()).sum(1)
    rhs = (Ku.double() * v.double()).sum(1)
    assert float(((lhs - rhs).abs() / (u.norm(dim=1) * Kv.norm(dim=1)).double()).max()) < 1e-5
    K2 = T._matmul_by_K(2.0 * u - 3.0 * v)
    assert float((K2 - (2.0 * Ku - 3.0 * Kv)).abs().max() / K2.abs().max()) < 1e-5


@pytest.mark.parametrize("dims", [(1024, 1024), (128, 128, 64)], ids=["C2_1024x1024", "3D_128x128x64"])
def test_pcg_fp32_vs_fp64_full_size(dims):
    """The fp32 PCG (20 iterations) agrees with the fp64 PCG of the same problem, and the
    fp64 residual has dropped: a well-conditioned problem (nugget 0.1) at full size."""
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    out = {}
    for dt in (torch.float64, torch.float32):
        k = zk.Matern(nu=1.5, dtype=dt)
        grids = [torch.linspace(-1, 1, m, device=DEV, dtype=dt) for m in dims]
        T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=(1., .05)), jitter_val=0.1)
        g = torch.Generator(device=DEV).manual_seed(1)
        b = torch.randn(3, T.M, device=DEV, generator=g, dtype=torch.float64).to(dt)
        x = T._solve(b, do_precond=True, maxiter=20, tol=1e-12)
        res = (T._matmul_by_K(x) - b).norm(dim=1) / b.norm(dim=1)
        out[dt] = (x.double(), float(res.max()))
    x64, r64 = out[torch.float64]
    x32, r32 = out[torch.float32]
    # 20 PCG iterations cut the relative residual at least 5x (measured 0.066 at 1024^2:
    # the fp64 solution's own residual, independent of the fp32 path under test)
    assert r64 < 0.2, r64
    rel = float(((x32 - x64).norm(dim=1) / x64.norm(dim=1)).max())
    assert rel < 1e-3, (rel, r64, r32)


@pytest.mark.parametrize("m", [2048, 4096], ids=["C3_2048x2048", "C4_4096x4096"])
def test_large_grid_fp32_vs_fp64(m):
    """C3 / C4 grid sizes (rows longer than one wave's line: 16-pair row blocks, and at 4096 the
    fp32 two-level LDS twiddle table): the fp32 K, C^-1 and R^T agree with the fp64 plan of the
    same well-conditioned problem (nugget 0.1; fp64 ops are pinned to the oracle elsewhere).
    At 4096 the fp64 R^T rows (H = 8192) exceed the row-pair kernels' LDS and run the generic
    2-D sequence (row-major intermediate, strided axis-0 pass): R(R^T v) = K v in fp64 there."""
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    outs = {}
    g = torch.Generator(device=DEV).manual_seed(2)
    v64 = torch.randn(2, m * m, device=DEV, generator=g, dtype=torch.float64)
    for dt in (torch.float64, torch.float32):
        k = zk.Matern(nu=1.5, dtype=dt)
        grids = [torch.linspace(-1, 1, m, device=DEV, dtype=dt) for _ in range(2)]
        T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=(1., 20. / m)), jitter_val=0.1)
        T.set_batch_shape((2,))
        v = v64.to(dt)
        res = [T._matmul_by_K(v), T._matmul_by_Cinv(v), T._matmul_by_RT(v)]
        rr = T._matmul_by_R(res[2])
        assert float((rr - res[0]).abs().max() / res[0].abs().max()) < (1e-11 if dt == torch.float64 else 1e-4)
        outs[dt] = [o.double() for o in res]
        del T, res, rr
        torch.cuda.empty_cache()
    for name, a, b, tol in zip(("K", "Cinv", "RT"), outs[torch.float32], outs[torch.float64], (2e-5, 2e-4, 1e-4)):
        err = float((a - b).abs().max() / b.abs().max())
        assert err < tol, (name, err)


@pytest.mark.parametrize("dims,dtype", [((1025, 8), torch.float64), ((2048, 8), torch.float64), ((4096, 8), torch.float64),
                                        ((8, 2048), torch.float64), ((600, 600), torch.float64),
                                        ((2048, 2048), torch.float32), ((1024, 1024), torch.float32),
                                        ((4096, 8), torch.float32), ((4096, 4096), torch.float32)],
                         ids=["1025x8_f64", "2048x8_f64", "4096x8_f64", "8x2048_f64", "600x600_f64", "C3_f32", "C2_f32",
                              "4096x8_f32", "C4_f32"])
def test_long_lines_accuracy_and_repeatability(dims, dtype):
    """Contiguous-line passes with lines of several waves (axis-0 columns of 2048 / 4096 points,
    fp64 setup DCTs along long rows): fp64 ops at fp64 accuracy against the oracle, and every op
    bitwise identical from run to run (a race once showed as 1e-8 run-to-run noise in fp64: the
    VMEM store-data hazard of 128-bit stores).  fp32 lines of 4 waves (4096 points,
    C4) against the fp64 oracle / the fp64 plan of the same grid."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.1)
    P = ToeplitzPlan(dims, dtype, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=dtype))
    v = np.random.RandomState(0).randn(4, int(np.prod(dims)))
    vt = torch.tensor(v, device=DEV, dtype=dtype)
    for op in (_lib.OP_K, _lib.OP_CINV, _lib.OP_RT):
        ys = [P.apply(op, vt) for _ in range(4)]
        for y in ys[1:]:
            assert torch.equal(y, ys[0]), op
    if dtype == torch.float32:
        if np.prod(dims) < 5e6:
            T = zo.ToeplitzOracle(col, dims)
            refs = {_lib.OP_K: T.matmul_K(v), _lib.OP_RT: T.matmul_RT(v)}
        else:       # C4: the fp64 plan of the same grid (itself pinned by the fp64 cases)
            P64 = ToeplitzPlan(dims, torch.float64, DEV)
            P64.set_column(torch.tensor(col, device=DEV))
            v64 = torch.tensor(v, device=DEV)
            refs = {op: _np(P64.apply(op, v64)) for op in (_lib.OP_K, _lib.OP_RT)}
            del P64, v64
        # R^T: fp32 FFT rounding over the L_R grid (8192^2 at C4) grows with its size: 1e-6 at
        # 4096 x 8, 7e-6 at 2048^2, 1.3e-5 at 4096^2 (measured); K stays within 5e-6
        for op, ref in refs.items():
            assert rel_err(_np(P.apply(op, vt)), ref) < (5e-6 if op == _lib.OP_K else 3e-5), op
    if dtype == torch.float64 and np.prod(dims) < 5e6:
        T = zo.ToeplitzOracle(col, dims)
        assert rel_err(P.spectrum(_lib.SPEC_D).cpu().numpy(), T.D) < 1e-12
        for op, ref in ((_lib.OP_K, T.matmul_K(v)), (_lib.OP_RT, T.matmul_RT(v))):
            assert rel_err(_np(P.apply(op, vt)), ref) < 1e-11, op


@pytest.mark.parametrize("lr", ["pow2", "short"])
@pytest.mark.parametrize("dims", [(700, 2100), (40, 4096)], ids=["700x2100", "40x4096"])
def test_generic_2d_sequence_fp64(dims, lr, monkeypatch):
    """fp64 rows whose row-pair kernels do not fit one CU's LDS (R / R^T with L_R >= 16384 along
    axis 1: the power-of-two L_R, HGP_LR=pow2) run the generic 2-D sequence; against the oracle,
    and the fp64 PCG through it.  "short": the plan's own choice (3 * 2^k or 2^k >= 3m - 3)."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .05), nu=1.5), 0.1)
    T = zo.ToeplitzOracle(col, dims)
    if lr == "pow2":
        monkeypatch.setenv("HGP_LR", "pow2")
    P = ToeplitzPlan(dims, torch.float64, DEV)
    P.set_column(torch.tensor(col, device=DEV))
    if lr == "pow2":
        assert P.L_R[1] >= 16384
    rs = np.random.RandomState(1)
    v = rs.randn(2, T.M)
    w = rs.randn(2, T.Mp)
    vt = torch.tensor(v, device=DEV)
    assert rel_err(_np(P.apply(_lib.OP_RT, vt)), T.matmul_RT(v)) < 1e-11
    assert rel_err(_np(P.apply(_lib.OP_R, torch.tensor(w, device=DEV))), T.matmul_R(w)) < 1e-11
    assert rel_err(_np(P.apply(_lib.OP_K, vt)), T.matmul_K(v)) < 1e-11


# ---- seeded shape sweep: edge shapes of every pass sequence ---------------------------------
# tiny axes (H = 2: one-point half spectra), odd sizes, size-1 axes in every position, 3-D
# planes whose row pairs / line tiles are ragged (hgp_lines.hpp), long-and-thin grids; fp64 to
# 1e-10 and fp32 within the SURVEY §8(c) rules, ops and the fused PCG (2-D / 3-D epilogues).
SWEEP = [(2,), (3,), (2, 2), (3, 2), (2, 5), (2, 2, 2), (3, 2, 5), (2, 17, 3), (5, 40, 2), (7, 3, 130),
         (65, 9, 33), (129, 3, 2), (1, 6, 1), (31, 1, 9), (4, 4, 1), (200, 3), (3, 200), (17, 18, 19)]


@pytest.mark.parametrize("dims", SWEEP, ids=lambda d: "x".join(map(str, d)))
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_shape_sweep_vs_oracle(dims, tag):
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dt = torch.float64 if tag == "f64" else torch.float32
    grids = [np.linspace(-1, 1, m) for m in dims]
    ell = 4.0 / max(dims)
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., ell), nu=1.5), 0.05)
    O = zo.ToeplitzOracle(col, dims)
    P = ToeplitzPlan(dims, dt, DEV)
    P.set_column(torch.tensor(col, device=DEV, dtype=dt))
    rs = np.random.RandomState(sum(dims))
    v = rs.randn(3, O.M)
    w = rs.randn(3, O.Mp)
    tol = 1e-10 if tag == "f64" else 2e-5
    for name, op, x, ref in (("K", _lib.OP_K, v, O.matmul_K(v)), ("Cinv", _lib.OP_CINV, v, O.matmul_Cinv(v)),
                             ("RT", _lib.OP_RT, v, O.matmul_RT(v)), ("R", _lib.OP_R, w, O.matmul_R(w))):
        got = _np(P.apply(op, torch.tensor(x, device=DEV, dtype=dt))).astype(np.float64)
        assert got.shape == ref.shape, name
        assert float(np.abs(got - ref).max() / np.abs(ref).max()) < tol, name
    b = rs.randn(2, O.M)
    it = min(8, max(1, O.M - 1))    # short of an exhausted Krylov space (r = 0 -> 0/0 in cg.py:66 too)
    xr = O.solve(b, True, it, 1e-30)
    x = _np(P.pcg(torch.tensor(b, device=DEV, dtype=dt), it, 1e-30, precond=True)).astype(np.float64)
    e = np.linalg.norm(x - xr) / np.linalg.norm(xr)
    if tag == "f64":
        assert e < 1e-8, e
    else:
        x32 = zo.ToeplitzOracle(col.astype(np.float32), dims).solve(b.astype(np.float32), True, it, 1e-30)
        e32 = np.linalg.norm(x32.astype(np.float64) - xr) / np.linalg.norm(xr)
        if not np.isfinite(e32):    # the fp32 reference itself hit 0/0 on a nearly exhausted Krylov space
            e32 = 2.5e-5
        assert e <= 4 * e32 + 1e-6, (e, e32)


@pytest.mark.parametrize("dims,dt,tol", [((400, 300), torch.float64, 1e-10), ((1024, 1000), torch.float32, 2e-6),
                                         ((300, 900), torch.float32, 2e-6)],
                         ids=["f64_400x300", "f32_1024x1000", "f32_300x900"])
def test_dcny_packed_columns(dims, dt, tol):
    """Round 5: the 2-D K / C^-1 intermediate packs its real DC and Nyquist compact columns as one
    complex column (PassDesc::dcny: one axis-0 line fewer per RHS, split again by Hermitian
    symmetry inside the axis-0 pass).  The same operator: against a plan without the packing
    (HGP_DCNY=0) to rounding, K against the oracle, and the fused PCG (spectral dots of the
    packed line) against the unpacked plan's."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    grids = [np.linspace(-1, 1, m) for m in dims]
    col_np = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .05), nu=1.5), 1e-2)
    col = torch.tensor(col_np, device=DEV, dtype=dt)
    plans = {}
    for pk in ("1", "0"):
        os.environ["HGP_DCNY"] = pk
        try:
            P = ToeplitzPlan(dims, dt, DEV)
        finally:
            del os.environ["HGP_DCNY"]
        P.set_column(col)
        plans[pk] = P
    M = int(np.prod(dims))
    g = torch.Generator(device=DEV).manual_seed(13)
    v = torch.randn(5, M, device=DEV, generator=g, dtype=torch.float64).to(dt)
    for op in (_lib.OP_K, _lib.OP_CINV):
        a, b = plans["1"].apply(op, v).double(), plans["0"].apply(op, v).double()
        err = float((a - b).abs().max() / b.abs().max())
        assert err < tol, (op, err)
    ref = zo.ToeplitzOracle(col_np, dims).matmul_K(v.double().cpu().numpy())
    got = plans["1"].apply(_lib.OP_K, v).double().cpu().numpy()
    assert float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))) < (1e-9 if dt == torch.float64 else 1e-5)
    xa = plans["1"].pcg(v, 10, 1e-30, precond=True).double()
    xb = plans["0"].pcg(v, 10, 1e-30, precond=True).double()
    assert float((xa - xb).norm() / xb.norm()) < (1e-9 if dt == torch.float64 else 1e-4)


@pytest.mark.parametrize("nrhs", [1, 8, 13], ids=["q1", "q8", "q13"])
def test_conv_two_lines_per_wave_opt_in(nrhs):
    """Round 6: the opt-in fp32 1024-point column conv with two lines per wave and radix-32 stages
    (HGP_CONV_P32=1, LAY_CONTIG2: one wave-shared buffer resource for two lines; measured slower
    and kept off by default, profiles/r6r_conv_p32_ab.txt).  C2's grid (in_len = out_len = H):
    K and C^-1 against the default layout to rounding and K against the oracle, over odd RHS counts
    (a wave's two lines then straddle RHS and column boundaries, and the last block holds invalid
    lines); the fused PCG (spectral dots, packed DC / Nyquist line) against the default plan."""
    from hipgp_amd import _lib
    from hipgp_amd.plan import ToeplitzPlan
    dims, dt = (1024, 1024), torch.float32
    grids = [np.linspace(-1, 1, m) for m in dims]
    col_np = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .05), nu=1.5), 1e-2)
    col = torch.tensor(col_np, device=DEV, dtype=dt)
    plans = {}
    for knob in ("1", "0"):
        os.environ["HGP_CONV_P32"] = knob
        try:
            P = ToeplitzPlan(dims, dt, DEV)
        finally:
            del os.environ["HGP_CONV_P32"]
        P.set_column(col)
        plans[knob] = P
    g = torch.Generator(device=DEV).manual_seed(17 + nrhs)
    v = torch.randn(nrhs, int(np.prod(dims)), device=DEV, generator=g, dtype=torch.float64).to(dt)
    for op in (_lib.OP_K, _lib.OP_CINV):
        a, b = plans["1"].apply(op, v).double(), plans["0"].apply(op, v).double()
        err = float((a - b).abs().max() / b.abs().max())
        assert err < 2e-6, (op, err)
    ref = zo.ToeplitzOracle(col_np, dims).matmul_K(v[:2].double().cpu().numpy())
    got = plans["1"].apply(_lib.OP_K, v[:2]).double().cpu().numpy()
    assert float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))) < 1e-5
    xa = plans["1"].pcg(v, 10, 1e-30, precond=True).double()
    xb = plans["0"].pcg(v, 10, 1e-30, precond=True).double()
    assert float((xa - xb).norm() / xb.norm()) < 1e-4
