"""Generate golden input/output vectors for the Toeplitz/PCG hot path by running the
*reference* `ziggy` package (read-only at /root/reference) in THIS container.

Test infrastructure only: the fixtures it writes (`tests/golden/*.npz`) are data
(inputs + expected outputs); no reference source is copied.  The GPU box never runs
this script (it has no /root/reference); it only reads the committed .npz files.

The reference is pinned to torch 1.4 (`requirements.txt:9`) and calls the removed
callable `torch.fft(x, signal_ndim)` / `torch.ifft` API
(`ziggy/misc/toeplitz_tensor.py:25,79,82`, `ziggy/misc/toeplitz_expanded.py:96,170,184`).
The shim below replaces the module-global name `torch` inside the reference modules by a
proxy that forwards everything to real torch except `fft`/`ifft` (re-expressed with
`torch.fft.fftn/ifftn`, same unnormalised/1/N C2C definition) and `solve`.
No reference file is modified.  `pyprind` (imported at `ziggy/kernels.py:247`) is stubbed.

Usage:  python tests/golden/make_golden.py          (writes tests/golden/*.npz)
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


class _TorchProxy(types.ModuleType):
    """Forward to real torch, except the torch-1.4 callables the reference uses."""

    def __init__(self):
        super().__init__("torch_proxy")

    def __getattr__(self, name):
        return getattr(torch, name)

    @staticmethod
    def fft(x, signal_ndim, normalized=False):
        dims = tuple(range(-signal_ndim, 0))
        c = torch.view_as_complex(x.contiguous())
        return torch.view_as_real(torch.fft.fftn(c, dim=dims))

    @staticmethod
    def ifft(x, signal_ndim, normalized=False):
        dims = tuple(range(-signal_ndim, 0))
        c = torch.view_as_complex(x.contiguous())
        return torch.view_as_real(torch.fft.ifftn(c, dim=dims))

    @staticmethod
    def solve(B, A):
        return torch.linalg.solve(A, B), None


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    sys.modules["pyprind"] = types.SimpleNamespace(prog_bar=lambda x: x)
    import ziggy.kernels as zk
    import ziggy.misc.toeplitz_tensor as tt
    import ziggy.misc.toeplitz_expanded as te
    import ziggy.misc.cg as cg
    import ziggy.hipgp as hg
    import ziggy.misc.stats as st
    proxy = _TorchProxy()
    for mod in (tt, te, hg, st):
        mod.torch = proxy
    assert os.path.realpath(tt.__file__).startswith(REF)
    return zk, tt, te, cg, hg


def _np(t):
    return t.detach().cpu().numpy()


def gen_G1(zk, te, dtype, tag):
    """config-1 shape: 1-D m=256 on [0,4], Matern-5/2 (1, .1), ToeplitzMatmul (no jitter)
    (`run_solve_kn_experiment.py:30,53`; `toeplitz_expanded.py:17-58`)."""
    out = {}
    kern = zk.Matern(nu=2.5, length_scale=.5, dtype=dtype)
    kfun = lambda x, y: kern.forward(x, y, params=(1., .1))
    xg = torch.linspace(0, 4, 256, dtype=dtype)
    rs = np.random.RandomState(42)
    xobs = torch.tensor(rs.rand(32, 1) * 4, dtype=dtype)
    vec = kfun(xobs, xg[:, None])                       # (32, 256) = Kun^T rows
    out["grid0"] = _np(xg)
    out["vec"] = _np(vec)
    for pre in (0, 1):
        for rt in (0, 1):
            for mi in (1, 5, 20):
                its = []
                res = te.gram_solve([xg], kfun, vec, do_precond=bool(pre), tol=1e-10,
                                    maxiter=mi, callback=lambda n, x: its.append(n),
                                    mult_RT=bool(rt))
                key = f"gram_p{pre}_rt{rt}_it{mi}"
                out[key] = _np(res)
                out[key + "_ncb"] = np.array(len(its))
    # (the tol=1e-10 runs above pin the break rule: PCG converges at iteration 4 < maxiter)
    np.savez_compressed(os.path.join(OUT, f"G1_{tag}.npz"), **out)


def _grid_case(zk, tt, dtype, tag, name, dims, lo, hi, kern, params, jitter, seed=0, B=3):
    out = {}
    kfun = lambda x, y: kern.forward(x, y, params=params)
    xgrids = [torch.linspace(lo[d], hi[d], dims[d], dtype=dtype) for d in range(len(dims))]
    T = tt.ToeplitzTensor(xgrids, kfun, batch_shape=None, jitter_val=jitter)
    for d, xg in enumerate(xgrids):
        out[f"grid{d}"] = _np(xg)
    out["column"] = _np(T.column)
    out["C"] = _np(T.C)
    out["D"] = _np(T.D[..., 0])
    out["D_sqrt"] = _np(T.D_sqrt[..., 0])
    out["Di"] = _np(T.Di[..., 0])
    M = int(np.prod(dims))
    Mp = int(np.prod(T.C.shape))
    g = torch.Generator().manual_seed(seed)
    # same RHS values in both precisions (drawn in fp64, rounded for the fp32 run)
    v = torch.randn(B, M, generator=g, dtype=torch.float64).to(dtype)
    w = torch.randn(B, Mp, generator=g, dtype=torch.float64).to(dtype)
    out["v"] = _np(v)
    out["w"] = _np(w)
    T.set_batch_shape((B,))
    out["Kv"] = _np(T._matmul_by_K(v))
    out["Cinv_v"] = _np(T._matmul_by_Cinv(v))
    out["RTv"] = _np(T._matmul_by_RT(v))
    out["Rw"] = _np(T._matmul_by_R(w))
    for mi in (1, 2, 5, 20):
        out[f"solve_p1_it{mi}"] = _np(T._solve(v, do_precond=True, maxiter=mi, tol=1e-8))
    out["solve_p0_it5"] = _np(T._solve(v, do_precond=False, maxiter=5, tol=1e-8))
    # compute_kn-equivalent: R^T K^{-1} v (`hipgp.py:143-145`) with maxiter 20
    out["kn_it20"] = _np(T._matmul_by_RT(T.inv_matmul(v, do_precond=True, maxiter=20, tol=1e-8)))
    np.savez_compressed(os.path.join(OUT, f"{name}_{tag}.npz"), **out)


def gen_G5(zk, hg, dtype, tag):
    """model-level compute_kn: MeanFieldToeplitzGP 20x20, Matern-3/2 (1, .1), 64 obs
    (`hipgp.py:117-146`, `svi_gp.py:72`)."""
    torch.manual_seed(0)
    rs = np.random.RandomState(42)
    kern = zk.Matern(nu=1.5, length_scale=.1, dtype=dtype)
    xgrids = [torch.linspace(-1, 1, 20, dtype=dtype), torch.linspace(-1, 1, 20, dtype=dtype)]
    mod = hg.MeanFieldToeplitzGP(kern, xgrids, num_obs=64, sig2_init=1., ell_init=.1,
                                 noise2_init=.01, learn_kernel=False, dtype=dtype)
    xobs = torch.tensor(rs.rand(64, 2) * 2 - 1, dtype=dtype)
    yobs = torch.tensor(rs.randn(64, 1), dtype=dtype)
    Knm, Knn = mod._make_grams(xobs)
    kn = mod.compute_kn(Knm, maxiter_cg=20)
    out = {"grid0": _np(xgrids[0]), "grid1": _np(xgrids[1]), "xobs": _np(xobs),
           "yobs": _np(yobs), "Knm": _np(Knm), "Knn_diag": _np(Knn), "kn": _np(kn),
           "theta1": _np(mod.global_theta1), "theta2": _np(mod.global_theta2)}
    elbo = mod.elbo_and_grad(xobs, yobs, maxiter_cg=20)
    out["elbo"] = np.array(float(elbo))
    out["theta1_grad"] = _np(mod.global_theta1.grad)
    out["theta2_grad"] = _np(mod.global_theta2.grad)
    mu, sig = mod.predict(xobs[:50], maxiter_cg=50)
    out["pred_mu"] = _np(mu)
    out["pred_sig"] = _np(sig)
    np.savez_compressed(os.path.join(OUT, f"G5_{tag}.npz"), **out)


def main():
    zk, tt, te, cg, hg = import_reference()
    torch.set_num_threads(8)
    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        gen_G1(zk, te, dtype, tag)
        # G2: 2-D 32x24 SqExp (1, .1), jitter 1e-3
        _grid_case(zk, tt, dtype, tag, "G2", (32, 24), (-1, -1), (1, 1),
                   zk.SqExp(dtype=dtype), (1., .1), 1e-3)
        # G3: 3-D 8x6x5 Matern-3/2 (1, .3): pins d=3 ordering and the expanded layout
        _grid_case(zk, tt, dtype, tag, "G3", (8, 6, 5), (-1, -1, -1), (1, 1, 1),
                   zk.Matern(nu=1.5, dtype=dtype), (1., .3), 1e-3)
        # G4: clamp cases (negative embedding eigenvalues -> clamp(min=1e-6) active)
        _grid_case(zk, tt, dtype, tag, "G4a", (32, 24), (-1, -1), (1, 1),
                   zk.SqExp(dtype=dtype), (1., .5), 1e-3)
        _grid_case(zk, tt, dtype, tag, "G4b", (32, 24), (-1, -1), (1, 1),
                   zk.Matern(nu=.5, dtype=dtype), (1., 5.), 1e-3)
        _grid_case(zk, tt, dtype, tag, "G4c", (32, 24), (-1, -1), (1, 1),
                   zk.Matern(nu=2.5, dtype=dtype), (1., 1.), 1e-3)
        # G6: 1-D ToeplitzTensor (exact_gp_1d_derivatives path), m=64
        _grid_case(zk, tt, dtype, tag, "G6", (64,), (0,), (2,),
                   zk.Matern(nu=2.5, dtype=dtype), (1., .2), 1e-3)
        # G7: ragged 2-D (non-power-of-two, odd sizes, one tiny axis) + odd batch
        _grid_case(zk, tt, dtype, tag, "G7", (37, 3), (-1, 0), (1, .5),
                   zk.Matern(nu=1.5, dtype=dtype), (1., .4), 1e-3, B=5)
        gen_G5(zk, hg, dtype, tag)
        print("wrote", tag)


if __name__ == "__main__":
    main()
