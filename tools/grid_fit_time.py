"""One config-5 natural-gradient minibatch (256 x 256 x 128 inducing grid, Matern-5/2, fp32,
line-integral observations with the MC estimator, `run_domain_experiment.py:61,112,276`: batch
200, PCG(20)) timed three ways on the GPU box, median of 3 after a warm-up:

  single   MeanFieldToeplitzGP.elbo_and_grad (fused device PCG, one process)
  rhs      hipgp_amd.dist.sharded_elbo_and_grad at world size 1 over RCCL
  grid     hipgp_amd.slab.SlabFit.elbo_and_grad at world size 1 over RCCL (the slab PCG: unfused
           conj_grad2 with all-reduced dots, all-to-all transposes -- at one rank, the cost of
           the grid-block machinery itself)

    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/grid_fit_time.py [--batch 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    from hipgp_amd import dist as hdist
    from hipgp_amd.slab import SlabFit
    dt = torch.float32
    grids = [torch.linspace(-1, 1, 256, dtype=dt), torch.linspace(-1, 1, 256, dtype=dt),
             torch.linspace(-.5, .5, 128, dtype=dt)]
    mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=2.5, dtype=dt), grids, num_obs=100_000, sig2_init=1.,
                                 ell_init=.1, learn_kernel=False, jitter_val=1e-3, dtype=dt).cuda_params(local)
    g = torch.Generator().manual_seed(7)
    B = a.batch
    x = ((torch.rand(B, 3, generator=g) * 2 - 1) * torch.tensor([.9, .9, .45])).to(dev)
    y = torch.randn(B, 1, generator=g).to(dev)
    s = torch.full((B, 1), .1, device=dev)
    kw = dict(integrated_obs=True, semi_integrated_estimator="mc-biased", semi_integrated_samps=10)
    fit = SlabFit(mod)
    runs = {
        "single": lambda: mod.elbo_and_grad(x, y, s, maxiter_cg=20, **kw),
        "rhs": lambda: hdist.sharded_elbo_and_grad(mod, x, y, s, maxiter_cg=20, **kw),
        "grid": lambda: fit.elbo_and_grad(x, y, s, maxiter_cg=20, **kw),
    }
    out = {"grid": [256, 256, 128], "batch": B, "dtype": "f32", "world_size": dist.get_world_size()}
    for name, fn in runs.items():
        torch.manual_seed(11)
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            torch.manual_seed(11)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_ms"] = round(float(np.median(ts)) * 1e3, 1)
        out[name + "_elbo"] = float(e)
        print(json.dumps({"mode": name, "ms": out[name + "_ms"], "elbo": float(e)}), flush=True)
    out["peak_torch_bytes"] = int(torch.cuda.max_memory_allocated(dev))
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
