"""Block-diagonal family statistics on the GPU box: hgp_block_stats (per-block grams + kn^T S kn,
one read of kn) against the reference's torch expression of the same sums on the same GPU
(`hipgp.py:252-256` to_blocks / matmul / sum, `:661-664` block_diag_multiply), fp32.

Algorithmic bytes of the natural-gradient statistics call (grams + <S, G>): kn read once
(B M' s) + S read (nblk bs^2 s) + gram written (nblk bs^2 s).  HBM roofline 8 TB/s.  The
per-row kn^T S kn (predict) is timed beside it.

    python tools/bench_block.py > gpurun_out/block.json
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [   # (grid m per axis, block sides, B)
    ((1024, 1024), (2, 2), 32),        # C2 grid, expanded 2046^2, 4-point blocks
    ((501, 501), (10, 10), 32),        # the experiments' 10x10 blocks (expanded 1000^2)
    ((1024, 1024), (2, 2), 200),       # C3-sized minibatch on the C2 grid
    ((129, 129, 65), (2, 2, 2), 25),   # 3-D (expanded 256x256x128), 2x2x2 blocks (domain script)
]


def ev_time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    dev = torch.device("cuda:0")
    for m, blocks, B in CASES:
        grids = [torch.linspace(-1, 1, k) for k in m]
        mod = hg.BlockToeplitzGP(zk.SqExp(), grids, num_obs=10 * B, block_sizes=list(blocks),
                                 dtype=torch.float32).cuda_params(0)
        nblk, bs = mod.num_blocks, mod.block_size
        g = torch.Generator(device=dev).manual_seed(0)
        kn = torch.randn(B, mod.Mprime, generator=g, device=dev)
        iv = torch.rand(B, generator=g, device=dev) + .5
        S = torch.randn(nblk, bs, bs, generator=g, device=dev) * .1
        # elbo_and_grad's statistics: grams + sum_n iv_n knSkn_n (= <S, G>), one read of kn
        ms = ev_time(lambda: mod._block_kernel(kn, ivar=iv, S=S, knSkn=False, trace=True))
        # predict / compute_batch_an: per-row kn^T S kn
        ms_q = ev_time(lambda: mod._block_kernel(kn, S=S, gram=False))

        def ref():
            # the reference expression, in RHS chunks of 8 so no broadcast temporary reaches
            # 2^31 elements (torch's batched matmul indexes them with 32-bit integers)
            G = torch.zeros(nblk, bs, bs, device=dev)
            q = []
            for c in range(0, B, 8):
                k = kn[c:c + 8]
                blk = mod.to_blocks(k).transpose(0, 1)
                G += torch.matmul(blk.transpose(1, 2), iv[None, c:c + 8, None] * blk)
                q.append(torch.sum(k * mod.block_diag_multiply(S, k), dim=-1))
            return G, torch.cat(q)
        try:
            ms_ref = ev_time(ref, reps=3)
        except torch.OutOfMemoryError:
            ms_ref = None
        nbytes = 4 * (B * mod.Mprime + 2 * nblk * bs * bs)
        print(json.dumps({"grid": list(m), "expanded": mod.block_dims, "blocks": list(blocks), "bs": bs,
                          "nblk": nblk, "B": B, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                          "hbm_frac": round(nbytes / ms / 1e6 / 8000, 3), "bytes": nbytes,
                          "knSkn_ms": round(ms_q, 4),
                          "torch_ref_ms": None if ms_ref is None else round(ms_ref, 3)}), flush=True)
        del kn, S


if __name__ == "__main__":
    main()
