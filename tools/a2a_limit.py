"""Where does one RCCL all_to_all_single stop moving the right bytes?  (GPU box, world size 1.)

Round 5 saw a 2.4 GB exchange (config 5's fp64 R^T, two RHS; complex128 viewed as float64)
come back wrong from one `all_to_all_single` at world size 1, and hipgp_amd/slab.py split
larger exchanges into 1 GiB pieces.  This probes the cause: for several dtypes and byte sizes
around 2^31 and 2^32, one all_to_all_single (with and without explicit split sizes) is checked
element for element against its input.  If the failures follow the BYTE count whatever the
dtype, a 32-bit byte count is the culprit; if they follow the ELEMENT count, an element count.

    torchrun --nproc-per-node 1 tools/a2a_limit.py
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    G, Mi = 1 << 30, 1 << 20
    # round 6, first probe (profiles/r6_a2a_limit.jsonl): every size from 2 GiB - 1 MiB up came back
    # with exactly its second half wrong; this sweep brackets the threshold below that
    sizes = [256 * Mi, 512 * Mi, G - Mi, G, G + Mi, G + 256 * Mi, G + 512 * Mi, 2 * G - 256 * Mi, 2 * G - Mi]
    if os.environ.get("A2A_SIZES"):
        sizes = [int(float(v)) for v in os.environ["A2A_SIZES"].split(",")]
    for dtype in (torch.float32, torch.float64):
        esz = torch.empty((), dtype=dtype).element_size()
        for nbytes in sizes:
            n = nbytes // esz
            for splits in (False, True):
                res = {"dtype": str(dtype), "bytes": n * esz, "elements": n, "explicit_splits": splits}
                try:
                    src = torch.arange(n, device=dev, dtype=torch.int64)
                    src = (src % 251).to(dtype) if dtype == torch.uint8 else src.to(dtype)
                    out = torch.full_like(src, 7 if dtype == torch.uint8 else -1)
                    if splits:
                        dist.all_to_all_single(out, src, [n], [n])
                    else:
                        dist.all_to_all_single(out, src)
                    torch.cuda.synchronize()
                    bad = (out != src)
                    nbad = int(bad.sum())
                    res["ok"] = nbad == 0
                    res["mismatches"] = nbad
                    if nbad:
                        blk = 1 << 12                 # locate the bad range by 4096-element blocks
                        nb = n // blk
                        anyb = bad[:nb * blk].view(nb, blk).any(dim=1)
                        idx = torch.nonzero(anyb)[:, 0]
                        if idx.numel():
                            res["first_bad_byte"] = int(idx[0]) * blk * esz
                            res["last_bad_block_end_byte"] = (int(idx[-1]) + 1) * blk * esz
                    del src, out, bad
                except RuntimeError as e:
                    res["ok"] = False
                    res["error"] = str(e).splitlines()[0][:200]
                torch.cuda.empty_cache()
                print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
