"""Coverage benchmark over the five BASELINE.json configs (GPU box; not the driver's bench line).

For each config: batched K matvec throughput and compute_kn wall-clock (set-up + PCG + R^T,
`hipgp.py:117-146`) on synthetic data of the config's shape.  The reference CPU timings quoted
next to them are BASELINE.md §2 (reference ziggy itself, survey container, 8 threads); the
same-box CPU baseline of the headline config is bench.py's cpu_baseline.

    python tools/bench_configs.py [--only C2,C5] > gpurun_out/configs.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name: (dims, kernel, params, jitter, B, maxiter, tol, reference CPU)
CONFIGS = {
    "C1": ((256,), ("matern", 2.5), (1.0, 0.1), 0.0, 1000, 2000, 1e-10,
           {"gram_solve_s": 0.065, "note": "1000 RHS, PCG to tol 1e-10 + R^T"}),
    "C2": ((1024, 1024), ("sqexp", None), (1.0, 0.01), 1e-3, 32, 20, 1e-8,
           {"kmatvec_rhs_per_s": 16.0, "compute_kn_s": 83.8, "note": "B=32"}),
    "C3": ((2048, 2048), ("matern", 1.5), (1.0, 0.1), 1e-3, 200, 20, 1e-8,
           {"kmatvec_rhs_per_s": 3.64, "compute_kn_s_per_rhs": 12.4, "note": "extrapolated per RHS"}),
    "C4": ((4096, 4096), ("matern", 1.5), (0.1, 0.1), 1e-3, 25, 20, 1e-8,
           {"kmatvec_rhs_per_s": 1.06, "compute_kn_s_per_rhs": 38.7, "note": "B=25 = one GPU's share of 200 over 8"}),
    "C5": ((256, 256, 128), ("matern", 2.5), (0.1, 0.1), 1e-3, 25, 20, 1e-8,
           {"kmatvec_rhs_per_s": 1.07, "compute_kn_s_per_rhs": 41.8, "note": "B=25 = one GPU's share of 200 over 8"}),
}
BOX = {1: [(0.0, 4.0)], 2: [(-1.0, 1.0)] * 2, 3: [(-0.25, 0.25), (-0.25, 0.25), (-0.05, 0.05)]}


def kernel(kind, nu, dtype):
    import ziggy.kernels as zk
    return zk.SqExp(dtype=dtype) if kind == "sqexp" else zk.Matern(nu=nu, dtype=dtype)


HBM_PEAK = 8.0e12


def byte_model(dims, maxiter):
    """SURVEY §8(d) pruned-pass algorithmic bytes per RHS (fp32): B_K, B_RT, compute_kn."""
    d = len(dims)
    M = int(np.prod(dims))
    n = [2 * m - 2 for m in dims]
    Mp = int(np.prod(n))
    h = dims[-1]                          # n_last / 2 + 1 = m_last
    if d == 1:
        bk, brt = 8 * M, 4 * M + 4 * Mp
    elif d == 2:
        bk = 8 * M + 32 * dims[0] * h
        brt = 4 * M + 16 * dims[0] * h + 16 * n[0] * h + 4 * Mp
    else:
        bk = 8 * M + 32 * dims[0] * dims[1] * h + 32 * dims[0] * n[1] * h
        brt = 4 * M + 16 * dims[0] * dims[1] * h + 16 * dims[0] * n[1] * h + 32 * n[0] * n[1] * h + 4 * Mp
    kn = maxiter * (2 * bk + 44 * M) + bk + brt
    return bk, brt, kn


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def run(name, dev):
    from hipgp_amd import _lib
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    from ziggy.misc import toeplitz_expanded as te
    dims, (kind, nu), params, jitter, B, maxiter, tol, ref = CONFIGS[name]
    d = len(dims)
    k = kernel(kind, nu, torch.float32)
    kf = lambda x, y: k.forward(x, y, params=params)
    grids = [torch.linspace(lo, hi, m, device=dev) for (lo, hi), m in zip(BOX[d], dims)]
    g = torch.Generator(device="cpu").manual_seed(42)
    lo = torch.tensor([b[0] for b in BOX[d]])
    hi = torch.tensor([b[1] for b in BOX[d]])
    xobs = (lo + (hi - lo) * torch.rand(B, d, generator=g)).to(dev)
    mesh = torch.meshgrid(*grids, indexing="ij")
    xs = torch.stack([x.reshape(-1) for x in mesh], dim=-1)
    from hipgp_amd.kuf import kuf_grid
    out = {"config": name, "dims": dims, "M": int(np.prod(dims)), "B": B, "maxiter": maxiter, "tol": tol}
    Knm = kuf_grid(k, grids, xobs, params)
    out["kuf_fused_ms"] = timed(lambda: kuf_grid(k, grids, xobs, params), reps=5) * 1e3
    try:    # the reference's broadcast evaluation (kernels.py:78,149), for comparison
        out["kuf_broadcast_ms"] = timed(lambda: kf(xobs, xs), reps=3) * 1e3
    except torch.cuda.OutOfMemoryError:
        out["kuf_broadcast_ms"] = None
    torch.cuda.empty_cache()
    if d == 3:   # config 5's line-integral observations, npts 10 (svi_gp.py:212)
        from hipgp_amd.kuf import kuf_semi_mc, kuf_semi_sqexp
        xi = xobs * 1.0
        t_mc = timed(lambda: kuf_semi_mc(k, grids, xi, params, 10), reps=3)
        out["kuf_semi_mc10_ms"] = t_mc * 1e3
        out["kuf_semi_mc10_evals_per_s"] = B * out["M"] * 10 / t_mc
        ks = kernel("sqexp", None, torch.float32)
        out["kuf_semi_sqexp_ms"] = timed(lambda: kuf_semi_sqexp(ks, grids, xi, params), reps=3) * 1e3
        out["kuf_semi_write_gbs"] = B * out["M"] * 4 / (out["kuf_semi_sqexp_ms"] * 1e-3) / 1e9
    if d == 1:
        t = timed(lambda: te.gram_solve(grids, kf, Knm, maxiter=maxiter, do_precond=True, tol=tol, mult_RT=True))
        out.update({"gram_solve_s": t, "reference_cpu": ref, "speedup_vs_reference_cpu": ref["gram_solve_s"] / t})
        return out
    T = ToeplitzTensor(grids, kf, batch_shape=(B,), jitter_val=jitter)
    y = torch.empty_like(Knm)
    t_op = timed(lambda: T._plan.apply(_lib.OP_K, Knm, out=y), reps=5)
    out["kmatvec_batched_ms"] = t_op * 1e3
    out["kmatvec_rhs_per_s"] = B / t_op

    def compute_kn():
        Tk = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=jitter)
        return Tk._matmul_by_RT(Tk.inv_matmul(Knm, do_precond=True, maxiter=maxiter, tol=tol))

    t_kn = timed(compute_kn, reps=2)
    out["compute_kn_s"] = t_kn
    out["compute_kn_s_per_rhs"] = t_kn / B
    out["reference_cpu"] = ref
    out["speedup_kmatvec_vs_reference_cpu"] = out["kmatvec_rhs_per_s"] / ref["kmatvec_rhs_per_s"]
    if "compute_kn_s_per_rhs" in ref:
        out["speedup_compute_kn_vs_reference_cpu"] = ref["compute_kn_s_per_rhs"] / out["compute_kn_s_per_rhs"]
    else:
        out["speedup_compute_kn_vs_reference_cpu"] = ref["compute_kn_s"] / t_kn
    bk, brt, bkn = byte_model(dims, maxiter)
    out["kmatvec_hbm_frac"] = B * bk / t_op / HBM_PEAK
    out["compute_kn_model_s"] = B * bkn / HBM_PEAK
    out["compute_kn_hbm_frac"] = B * bkn / t_kn / HBM_PEAK
    out["ws_mb"] = os.environ.get("HGP_WS_MB", "default")
    out["peak_mem_gb"] = torch.cuda.max_memory_allocated(dev) / 1e9
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C2,C3,C4,C5")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = []
    for name in a.only.split(","):
        r = run(name, dev)
        res.append(r)
        print(json.dumps(r), flush=True)
        # each config is its own workload: drop the previous grid's pooled plans (their
        # workspaces sit outside torch's allocator) before the next one
        import gc
        from hipgp_amd.plan import release_pool
        gc.collect()
        release_pool()
        torch.cuda.empty_cache()
    return res


if __name__ == "__main__":
    main()
