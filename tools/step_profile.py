"""Per-step durations of the bench's timed loop (C2 K matvec, graph replay): an event after
every step on the plan's stream, plus the host clock of the whole region (GPU box)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from hipgp_amd import _lib
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor
    dev = torch.device("cuda", 0)
    grids, kf, Knm = bench.make_problem(1024, 32, dev, seed=1234)
    T = ToeplitzTensor(grids, kf, batch_shape=(32,), jitter_val=1e-3)
    y = torch.empty_like(Knm)
    step = lambda: T._plan.apply(_lib.OP_K, Knm, out=y)
    st = torch.cuda.current_stream(dev)
    for _ in range(60):
        step()
    for rep in range(3):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
        t0 = time.perf_counter()
        ev[0].record(st)
        for i in range(20):
            step()
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        per = [ev[i].elapsed_time(ev[i + 1]) for i in range(20)]
        print(f"rep {rep}: host {dt:.3f} ms  events total {ev[0].elapsed_time(ev[20]):.3f} ms  "
              f"steps {' '.join(f'{p:.3f}' for p in per)}", flush=True)


if __name__ == "__main__":
    main()
