"""Timing of the backward kernels on the GPU box: hgp_sym_toeplitz_dqf
(InvMatmul's column gradient) and hgp_plan_column_grad (R^T through D_sqrt).  One JSON line each."""
import json
import sys

sys.path.insert(0, ".")
import torch

from hipgp_amd import _lib
from hipgp_amd.plan import ToeplitzPlan, sym_toeplitz_dqf


def t_ms(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for n, nvec in ((4096, 8), (65536, 8)):
    l = torch.randn(n, nvec, device="cuda")
    r = torch.randn(n, nvec, device="cuda")
    ms = t_ms(lambda: sym_toeplitz_dqf(l, r), reps=2 if n > 100000 else 5)
    fl = 4.0 * nvec * n * n     # 2 FMAs per (lag, k, vector)
    print(json.dumps({"kernel": "k_dqf", "n": n, "nvec": nvec, "ms": ms, "tflops": fl / ms / 1e9}), flush=True)

for dims, B in (((64, 64), 4), ((1024, 1024), 32), ((256, 256, 128), 8)):
    P = ToeplitzPlan(dims, dtype=torch.float32, device="cuda")
    M, Mp = P.M, P.Mprime
    col = torch.exp(-torch.linspace(0, 3, M, device="cuda"))
    P.set_column(col)
    v = torch.randn(B, M, device="cuda")
    g = torch.randn(B, Mp, device="cuda")
    ms = t_ms(lambda: P.column_grad(_lib.OP_RT, v, g), reps=2)
    print(json.dumps({"kernel": "column_grad RT (fp64 cross spectrum on L_R)", "dims": dims, "B": B,
                      "L_R": P.L_R, "ms": ms}), flush=True)
    u = torch.randn(2 * B, M, device="cuda")
    w = torch.randn(2 * B, M, device="cuda")
    ms = t_ms(lambda: P.dqf(u, w), reps=2)
    print(json.dumps({"kernel": "plan dqf (InvMatmul column grad, fp64 FFT on L_K)", "dims": dims, "nvec": 2 * B,
                      "L_K": P.L_K, "ms": ms}), flush=True)
    del v, g, u, w, P
    torch.cuda.empty_cache()
