"""Per-pass HIP-event timings of one batched operator at arbitrary grid dims (GPU box).

    python tools/passtime.py --dims 256,256,128 --rhs 25 [--op K]
Prints op time, per-pass times and the op's algorithmic HBM rate (SURVEY §8(d) B_K)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="256,256,128")
    ap.add_argument("--rhs", type=int, default=25)
    ap.add_argument("--op", default="K", choices=["K", "CINV", "RT", "R"])
    ap.add_argument("--ell", type=float, default=0.1, help="Matern-5/2 lengthscale of the grid kernel")
    ap.add_argument("--op-only", type=int, default=0, help="only run the op this many times (PMC passes)")
    ap.add_argument("--pcg-only", type=int, default=0,
                    help="only run this many batched PCG(20) solves (the fused iteration's kernels, PMC passes)")
    a = ap.parse_args()
    from hipgp_amd import _lib
    import ziggy.kernels as zk
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    dev = torch.device("cuda", 0)
    dims = [int(v) for v in a.dims.split(",")]
    k = zk.Matern(nu=2.5, dtype=torch.float32)
    kf = lambda x, y: k.forward(x, y, params=(a.ell, 0.1))
    grids = [torch.linspace(-.25, .25, m, device=dev) for m in dims]
    T = ToeplitzTensor(grids, kf, batch_shape=(a.rhs,), jitter_val=1e-3)
    plan = T._plan
    M = int(np.prod(dims))
    Mp = int(np.prod([2 * m - 2 for m in dims]))
    op = getattr(_lib, "OP_" + a.op)
    nin = Mp if a.op == "R" else M
    nout = Mp if a.op == "RT" else M
    x = torch.randn(a.rhs, nin, device=dev)
    y = torch.empty(a.rhs, nout, device=dev)
    st = torch.cuda.current_stream(dev)

    def tm(fn, reps=10):
        for _ in range(3):   # warm (the op's graph is captured on its second identical call)
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(reps):
            fn()
        e.record(st)
        e.synchronize()
        return s.elapsed_time(e) / reps

    if a.pcg_only:
        for _ in range(a.pcg_only):
            plan.pcg(x if a.op != "R" else torch.randn(a.rhs, M, device=dev), 20, 1e-8, precond=True)
        torch.cuda.synchronize()
        print(json.dumps({"dims": dims, "rhs": a.rhs, "pcg": a.pcg_only}))
        return
    if a.op_only:
        for _ in range(a.op_only):
            plan.apply(op, x, out=y)
        torch.cuda.synchronize()
        print(json.dumps({"dims": dims, "rhs": a.rhs, "op": a.op, "ops": a.op_only}))
        return
    op_ms = tm(lambda: plan.apply(op, x, out=y))
    npass = _lib.lib().hgp_op_pass_count(plan._h)
    passes = []
    for p in range(npass):
        passes.append(round(tm(lambda: _lib.check(_lib.lib().hgp_toeplitz_apply_pass(
            plan._h, op, x.data_ptr(), y.data_ptr(), a.rhs, p))), 4))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import byte_model
    bk = byte_model.op_bytes(a.op, dims)
    out = {"dims": dims, "rhs": a.rhs, "op": a.op, "op_ms": round(op_ms, 4), "passes_ms": passes,
           "L_K": list(plan.L_K), "L_R": list(plan.L_R)}
    out["algo_gbs"] = round(a.rhs * bk / (op_ms * 1e-3) / 1e9, 1)
    out["model"] = "B_RT" if a.op in ("RT", "R") else "B_K"
    out["frac"] = round(out["algo_gbs"] / 8000, 3)
    if a.op in ("RT", "R"):
        n = byte_model.ngrid(dims)
        LR = list(plan.L_R)[:len(dims)]
        real = all(L >= 2 * v - 1 for L, v in zip(LR, n))
        per, spec = byte_model.floor_rt(dims, LR, real_spec=real)
        out["L_R_floor_gbs"] = round((a.rhs * per + spec) / (op_ms * 1e-3) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
