"""Where do the GPU's clamped-case PCG iterates leave the reference's?  (GPU box diagnostic.)

For a golden case (default G4b, fp64): the GPU ops against the goldens and the NumPy oracle;
then the GPU PCG iterate x_k (maxiter = k, k = 1..20) against the oracle's conj_grad2 iterate
(the oracle tracks the reference to ~1e-5 on these cases), and the same with the GPU's C^-1 or K
swapped for the oracle's inside an otherwise GPU recurrence -- which operator's accuracy the
20-iteration divergence comes from.

    python tools/clamp_diag.py [G4b] [f64]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from golden_cases import GRID_CASES, load, grids_of, rel_err  # noqa: E402
from oracle import ziggy_oracle as zo  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "G4b"
    tag = sys.argv[2] if len(sys.argv) > 2 else "f64"
    dtype = torch.float64 if tag == "f64" else torch.float32
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    fx = load(name, tag)
    kind, nu, params, jit = GRID_CASES[name]
    k = zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)
    grids = [torch.tensor(g, dtype=dtype, device="cuda") for g in grids_of(fx)]
    T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=params), jitter_val=jit)
    v = torch.tensor(fx["v"], device="cuda")
    T.set_batch_shape((v.shape[0],))
    O = zo.ToeplitzOracle(fx["column"].astype(np.float64), T.dims)
    vn = fx["v"].astype(np.float64)
    for key, fn, ofn in (("Kv", T._matmul_by_K, O.matmul_K), ("Cinv_v", T._matmul_by_Cinv, O.matmul_Cinv)):
        y = fn(v).double().cpu().numpy()
        yo = ofn(vn)
        print(f"{key}: gpu vs golden {rel_err(y, fx[key]):.2e}  oracle vs golden {rel_err(yo, fx[key]):.2e}  "
              f"gpu vs oracle 2-norm {np.linalg.norm(y - yo) / np.linalg.norm(yo):.2e}")
    # iterate-by-iterate divergence from the oracle's recurrence
    xs_o = []
    zo.conj_grad2(O.matmul_K, vn, precond=O.matmul_Cinv, maxiter=20, tol=1e-8,
                  callback=lambda n, x: xs_o.append(x.copy()))
    for kk in range(1, 21):
        x = T._solve(v, do_precond=True, maxiter=kk, tol=1e-8).double().cpu().numpy()
        ref = xs_o[kk - 1] if kk - 1 < len(xs_o) else zo.conj_grad2(O.matmul_K, vn, precond=O.matmul_Cinv,
                                                                   maxiter=kk, tol=1e-8)
        print(f"it {kk:2d}: gpu vs oracle {rel_err(x, ref):.2e}", flush=True)
    # mixed recurrences: oracle conj_grad2 with one GPU operator swapped in
    Kg = lambda y: T._matmul_by_K(torch.tensor(y, device="cuda", dtype=dtype)).double().cpu().numpy()
    Cg = lambda y: T._matmul_by_Cinv(torch.tensor(y, device="cuda", dtype=dtype)).double().cpu().numpy()
    x_ref = zo.conj_grad2(O.matmul_K, vn, precond=O.matmul_Cinv, maxiter=20, tol=1e-8)
    for lab, A, P in (("oracle K + GPU C^-1", O.matmul_K, Cg), ("GPU K + oracle C^-1", Kg, O.matmul_Cinv),
                      ("GPU K + GPU C^-1 (host recurrence)", Kg, Cg)):
        x = zo.conj_grad2(A, vn, precond=P, maxiter=20, tol=1e-8)
        print(f"{lab}: it 20 vs oracle {rel_err(x, x_ref):.2e}  vs golden {rel_err(x, fx['solve_p1_it20']):.2e}")
    print("oracle vs golden it 20:", f"{rel_err(x_ref, fx['solve_p1_it20']):.2e}")


if __name__ == "__main__":
    main()
