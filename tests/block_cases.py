"""Shared builders for the block-diagonal family fixtures G11 / G12 (tests/golden/make_golden_block.py)."""
import torch

from golden_cases import load


def block_model(name, tag="f64", dtype=torch.float64, device=None):
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    fx = load(name, tag)
    nd = len(fx["dims"])
    k = zk.Matern(nu=1.5, dtype=dtype) if name == "G11" else zk.SqExp(dtype=dtype)
    grids = [torch.tensor(fx[f"grid{i}"], dtype=dtype) for i in range(nd)]
    mod = hg.BlockToeplitzGP(k, grids, num_obs=int(fx["num_obs"]), block_sizes=[int(b) for b in fx["blocks"]],
                             sig2_init=float(fx["params"][0]), ell_init=float(fx["params"][1]),
                             noise2_init=float(fx["noise2"]), learn_kernel=False, dtype=dtype)
    with torch.no_grad():
        mod.global_theta1.copy_(torch.tensor(fx["theta1"], dtype=dtype))
        mod.global_theta2.copy_(torch.tensor(fx["theta2"], dtype=dtype))
    if device is not None:
        mod = mod.cuda_params(0)
    return mod, fx


def noise_of(fx, dtype=torch.float64, device="cpu"):
    return torch.tensor(fx["noise_std"], dtype=dtype, device=device) if "noise_std" in fx else None
