"""Diagnostic: K / R^T of thin 2-D grids (the axis-0 column pass dominates) in fp32 and fp64
against the fp64 oracle; compare library builds with HGP_LIB."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ziggy_oracle as zo
from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan

for s in sys.argv[1:]:
    dims = tuple(int(v) for v in s.split("x"))
    grids = [np.linspace(-1, 1, m) for m in dims]
    col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.1)
    T = zo.ToeplitzOracle(col, dims)
    v = np.random.RandomState(0).randn(4, T.M)
    refs = {"K": T.matmul_K(v), "RT": T.matmul_RT(v)}
    for dt in (torch.float32, torch.float64):
        P = ToeplitzPlan(dims, dt, "cuda")
        P.set_column(torch.tensor(col, device="cuda", dtype=dt))
        out = {}
        for name, op in (("K", _lib.OP_K), ("RT", _lib.OP_RT)):
            y = P.apply(op, torch.tensor(v, device="cuda", dtype=dt)).double().cpu().numpy()
            out[name] = float(np.max(np.abs(y - refs[name])) / np.max(np.abs(refs[name])))
        print(dims, str(dt)[6:], "H_K0", P.L_K[0] // 2, "H_R0", P.L_R[0] // 2, {k: f"{e:.2e}" for k, e in out.items()}, flush=True)

# repeatability: the same op five times on the same input, bitwise
if os.environ.get("REPEAT"):
    for s in sys.argv[1:]:
        dims = tuple(int(v) for v in s.split("x"))
        grids = [np.linspace(-1, 1, m) for m in dims]
        col = zo.toeplitz_column(grids, lambda x, y: zo.kernel_eval("matern", x, y, (1., .1), nu=1.5), 0.1)
        P = ToeplitzPlan(dims, torch.float64, "cuda")
        P.set_column(torch.tensor(col, device="cuda"))
        v = torch.tensor(np.random.RandomState(0).randn(4, int(np.prod(dims))), device="cuda")
        ys = [P.apply(_lib.OP_K, v) for _ in range(5)]
        print(dims, "repeat max|y_i - y_0| / max|y_0|:",
              [f"{float((y - ys[0]).abs().max() / ys[0].abs().max()):.1e}" for y in ys[1:]], flush=True)
