import time, torch, sys, os
sys.path.insert(0, os.getcwd())
import bench
from hipgp_amd import _lib
from ziggy.misc.toeplitz_tensor import ToeplitzTensor
dev = torch.device("cuda", 0)
grids, kf, Knm = bench.make_problem(1024, 32, dev, seed=1)
T = ToeplitzTensor(grids, kf, batch_shape=(32,), jitter_val=1e-3)
y = torch.empty_like(Knm)
for i in range(6):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    T._plan.apply(_lib.OP_K, Knm, out=y)
    t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"call {i}: host {1e3*(t1-t0):.3f} ms  total {1e3*(t2-t0):.3f} ms")
