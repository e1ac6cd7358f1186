"""Diagnostic: relative errors of the backward against the G13-G15 goldens (GPU box)."""
import sys
sys.path[:0] = ["tests", "."]
import numpy as np
import torch
from golden_cases import load, grids_of, rel_err
from grad_cases import GRAD_CASES
import ziggy.kernels as zk
from ziggy.misc.toeplitz_tensor import ToeplitzTensor
from ziggy.misc._inv_matmul import InvMatmul

for name in sorted(GRAD_CASES):
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        kind, nu, p = GRAD_CASES[name]
        fx = load(name, tag); f64 = load(name, "f64")
        k = zk.SqExp(dtype=dt) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dt)
        grids = [torch.tensor(g, dtype=dt, device="cuda") for g in grids_of(fx)]
        T = ToeplitzTensor(grids, lambda x, y: k.forward(x, y, params=p), jitter_val=1e-3)
        col = T.column.detach().clone().requires_grad_(True)
        R = torch.tensor(fx["R"], device="cuda").requires_grad_(True)
        sol = InvMatmul.apply(T, col, R, True, 30, 1e-10)
        sol.backward(torch.tensor(fx["grad_out"], device="cuda"))
        print(name, tag, "sol %.2e col %.2e right %.2e | ref32 col %.2e right %.2e" % (
            rel_err(sol.detach().cpu().numpy(), f64["solves"]),
            rel_err(col.grad.cpu().numpy(), f64["inv_column_grad"]),
            rel_err(R.grad.cpu().numpy(), f64["inv_right_grad"]),
            rel_err(load(name, "f32")["inv_column_grad"], f64["inv_column_grad"]),
            rel_err(load(name, "f32")["inv_right_grad"], f64["inv_right_grad"])), flush=True)
