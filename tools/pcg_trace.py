"""Kernel timeline of one C2 compute_kn (GPU box, under rocprofv3 --kernel-trace): run it 3 times
with 50 ms host gaps; tools/pcg_trace.py --analyze <kernel_trace.csv> then splits the trace at
the gaps and reports, for the last run, wall time, GPU-busy time (union of kernel intervals over
all streams), idle gaps and the time per kernel.

    rocprofv3 --kernel-trace -d out -o run --output-format csv -- python3 tools/pcg_trace.py [C4]
    python3 tools/pcg_trace.py --analyze out/.../run_kernel_trace.csv"""
import csv
import os
import sys
import time
from collections import defaultdict


def run(cfg="C2"):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    dev = torch.device("cuda", 0)
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    if cfg == "C2":
        import bench
        grids, kf, Knm = bench.make_problem(1024, 32, dev, seed=1234)
        jitter, maxiter, tol = 1e-3, 20, 1e-8
    else:                                   # a BASELINE config of tools/bench_configs.py
        from tools.bench_configs import BOX, CONFIGS, kernel
        from hipgp_amd.kuf import kuf_grid
        dims, (kind, nu), params, jitter, B, maxiter, tol, _ = CONFIGS[cfg]
        d = len(dims)
        k = kernel(kind, nu, torch.float32)
        kf = lambda x, y: k.forward(x, y, params=params)
        grids = [torch.linspace(lo, hi, m, device=dev) for (lo, hi), m in zip(BOX[d], dims)]
        g = torch.Generator(device="cpu").manual_seed(42)
        lo = torch.tensor([b[0] for b in BOX[d]])
        hi = torch.tensor([b[1] for b in BOX[d]])
        xobs = (lo + (hi - lo) * torch.rand(B, d, generator=g)).to(dev)
        Knm = kuf_grid(k, grids, xobs, params)
    for _ in range(3):
        Tk = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=jitter)
        d0 = Tk.inv_matmul(Knm, do_precond=True, maxiter=maxiter, tol=tol)
        Tk._matmul_by_RT(d0)
        torch.cuda.synchronize()
        time.sleep(0.05)


def analyze(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    runs, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - max(e for _, e, _ in cur) > 20_000_000:   # > 20 ms host gap
            runs.append(cur)
            cur = []
        cur.append(r)
    runs.append(cur)
    last = runs[-1]
    t0, t1 = last[0][0], max(e for _, e, _ in last)
    busy, ce = 0, t0
    gaps = []
    for s, e, _ in last:
        if s > ce:
            gaps.append(s - ce)
        busy += max(0, e - max(s, ce))
        ce = max(ce, e)
    per = defaultdict(lambda: [0, 0])
    for s, e, n in last:
        per[n.split("(")[0][:70]][0] += 1
        per[n.split("(")[0][:70]][1] += e - s
    print(f"runs {len(runs)}  last run: wall {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  "
          f"kernels {len(last)}  idle gaps {len(gaps)} = {sum(gaps) / 1e6:.3f} ms (max {max(gaps, default=0) / 1e3:.1f} us)")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {n:72s} n={c:4d} sum={t / 1e6:8.3f} ms avg={t / c / 1e3:8.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run(sys.argv[1] if len(sys.argv) > 1 else "C2")
