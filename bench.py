"""Benchmark: Toeplitz-FFT Kuu matvecs/sec + PCG wall-clock at M = 1M inducing points.

Workload (BASELINE.json configs[1]): 2-D 1024x1024 grid on [-1,1]^2,
SqExp(sig2=1, ell=0.01), jitter 1e-3, fp32, B = 32 right-hand sides per GPU = rows of Knm for
32 synthetic observations x ~ U(-1,1)^2 (seeded per rank).

  step          = one batched Kuu matvec over the rank's 32 RHS (hgp_toeplitz_apply, op K)
  value         = RHS-matvecs/s over all ranks (weak scaling: each rank owns 32 RHS)
  pcg_*         = compute_kn wall-clock (hipgp.py:117-146): spectrum setup + PCG(maxiter 20,
                  tol 1e-8, C^-1 preconditioner) + R^T, for the same 32 RHS
  roofline      = HBM roofline of the batched K matvec (3 pass kernels back to back) with
                  SURVEY §8(d)'s algorithmic bytes B_K = 8M + 32*m1*h2 per RHS; `achieved`
                  divides them by ms_per_step (the timed steps), HIP-event figures beside it
  cpu_baseline  = the NumPy/SciPy oracle (scipy.fft; the faster of the process's CPU share and
                  every host CPU as workers): K matvecs on a bounded sample, and compute_kn on
                  all 32 RHS (~30 s of CPU work), rank 0 at N=1 only

The compute_kn timing and the per-pass event timing run BEFORE the timed steps (untimed for
the metric), so the timed steps see the GPU at its steady clock.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) WORLD_SIZE must equal --gpus;
`python bench.py --gpus N` with no torch.distributed environment starts the N ranks itself (a
torchrun child launched before this process touches the GPU; it exits with the child's code).
n_gpus is the world size of the initialised process group.  RHS are sharded (each rank its own 32), no
collective inside the timed region apart from the barriers; max-over-ranks timing.  Beside the
weak K-matvec line, two legs measured at every N (untimed for the metric, max over ranks) that
CAN fail to scale:
  strong        = compute_kn for a FIXED global batch (C2's 32 RHS split 32/N per rank,
                  hipgp_amd.dist.sharded_compute_kn with the reference's all-RHS break rule:
                  one all-reduce(MIN) of a device flag per PCG iteration, RCCL on GPUs)
  elbo_step     = one mean-field `elbo_and_grad` minibatch of 32 observations sharded 32/N
                  (hipgp_amd.dist.sharded_elbo_and_grad: fused Kuf + compute_kn + statistics and
                  the all-reduce of the 2 M' natural-gradient sums, hipgp.py:234-266), and that
                  all-reduce (33.5 MB at C2) timed alone
  strong_c4     = config 4's own multi-GPU workload (BASELINE configs[3]):
                  compute_kn for its fixed global batch of 200 RHS on the 4096^2 grid
                  (Matern-3/2, sig2 0.1, ell 0.1, jitter 1e-3), split 200/N per rank -- 25 per GPU
                  at N = 8 -- with the same all-RHS break; one warm-up call, then the median and
                  min of --c4-reps timed calls (~1.7 s each at N = 1) with the set-up / PCG / R^T
                  split of every call; an error is recorded in the line instead of failing it
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--m", type=int, default=1024, help="grid points per axis (2-D)")
    ap.add_argument("--rhs", type=int, default=32)
    ap.add_argument("--pcg-reps", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=0.4,
                    help="seconds of untimed back-to-back steps before the warmup (steady clock)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle worker threads (0: the faster of the CPU share and all host CPUs)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (with --backend gloo)")
    ap.add_argument("--kop-only", action="store_true",
                    help="only the timed K matvec steps (for rocprofv3 --pmc passes)")
    ap.add_argument("--no-legs", action="store_true", help="skip the strong-scaling / ELBO-step legs")
    ap.add_argument("--legs-reps", type=int, default=3)
    ap.add_argument("--no-c4-leg", action="store_true", help="skip the config-4 (200 RHS at 4096^2) strong leg")
    ap.add_argument("--c4-reps", type=int, default=3, help="timed repetitions of the config-4 leg")
    return ap.parse_args()


# tools/pmc_kop.sh summaries, newest round first (the kernels of the op change between rounds)
PMC_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r6_pmc_kop_C2.json", "r5_pmc_kop_C2.json",
                                                          "r4_pmc_kop_C2.json", "r3_pmc_kop_C2.json",
                                                          "r2_pmc_kop_C2.json")]


def pmc_traffic(M, B):
    """HBM bytes per batched K matvec from the committed rocprofv3 PMC summary
    (tools/pmc_kop.sh): (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB summed over the op's kernels —
    FETCH_SIZE counts half the bytes of wide streaming reads on gfx950 (MI355X_MICROARCH.md
    §HBM).  None when no summary for this workload is committed."""
    for f in PMC_FILES:
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("M") == M and d.get("rhs") == B:
            return d.get("traffic_bytes_per_op"), os.path.relpath(f, ROOT)
    return None, None


def make_problem(m, B, device, seed):
    import ziggy.kernels as zk
    k = zk.SqExp(dtype=torch.float32)
    params = (1.0, 0.01)
    kf = lambda x, y: k.forward(x, y, params=params)
    grids = [torch.linspace(-1, 1, m, device=device, dtype=torch.float32) for _ in range(2)]
    g = torch.Generator(device="cpu").manual_seed(seed)
    xobs = (torch.rand(B, 2, generator=g, dtype=torch.float32) * 2 - 1).to(device)
    xx = torch.meshgrid(*grids, indexing="ij")
    xs = torch.stack([x.reshape(-1) for x in xx], dim=-1)
    Knm = torch.cat([kf(xobs[i:i + 1], xs) for i in range(B)], dim=0).contiguous()   # (B, M)
    return grids, kf, Knm


def time_events(fn, reps, stream):
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / reps


def host_cpu_info():
    """(host logical CPUs, CPUs this process may use, CPU model string)."""
    host = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = host
    try:   # cgroup v2 quota ("max 100000" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            usable = max(1, min(usable, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return host, usable, model


def cpu_baseline(m, B, grids_np, seed, threads=None):
    """Oracle (scipy.fft) on the host cores: K matvecs on a bounded sample (4 RHS, repeated
    until 4 s or 20 repetitions, whichever comes first), then the full compute_kn (PCG(20) +
    R^T) on all B right-hand sides of the workload (C2 timed in full).  The
    worker count is the faster of the process's CPU share and every host CPU (both reported)."""
    from oracle import ziggy_oracle as zo
    host, usable, model = host_cpu_info()
    cands = [threads] if threads else sorted({usable, host})
    kf = lambda x, y: zo.kernel_eval("sqexp", x, y, (1.0, 0.01))
    col = zo.toeplitz_column(grids_np, kf, 1e-3).astype(np.float32)
    T = zo.ToeplitzOracle(col, (m, m))
    rs = np.random.RandomState(seed)
    nb = 4
    v = rs.randn(B, m * m).astype(np.float32)
    rates, runs = {}, {}
    for th in cands:
        zo.set_workers(th)
        T.matmul_K(v[:nb])                  # warm the FFT plans / thread pool
        t0 = time.perf_counter()
        reps = 0
        while True:
            T.matmul_K(v[:nb])
            reps += 1
            if time.perf_counter() - t0 > 4.0 or reps >= 20:
                break
        el = time.perf_counter() - t0
        rates[th] = nb * reps / el
        runs[th] = (reps, el)
    best = max(rates, key=rates.get)
    zo.set_workers(best)
    t0 = time.perf_counter()
    xs = T.solve(v, do_precond=True, maxiter=20, tol=1e-8)
    T.matmul_RT(xs)
    pcg_s = time.perf_counter() - t0
    reps, el = runs[best]
    return {"value": rates[best], "unit": "RHS-matvecs/s", "cores": best, "kind": "port",
            "host_cpus": host, "usable_cpus": usable, "cpu_model": model,
            "matvec_rate_by_threads": {str(k): v for k, v in rates.items()},
            "sample": f"oracle (scipy.fft, {best} workers; best of {sorted(rates)}): K matvec on {nb} RHS x "
                      f"{reps} repetitions = {el:.2f} s; compute_kn (PCG(20, tol 1e-8, precond) + R^T) on all "
                      f"{B} RHS = {pcg_s:.2f} s",
            "pcg_s": pcg_s, "pcg_rhs": B}


def _timed_max(fn, reps, dist, device, backend):
    """warm-up + median of `reps` barrier-bracketed, synchronised wall-clocks; max over ranks (ms)"""
    import torch.distributed as tdist
    out = []
    fn()
    for _ in range(reps):
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        out.append(time.perf_counter() - t0)
    v = float(np.median(out))
    if dist:
        tt = torch.tensor([v], device=device if backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        v = float(tt.item())
    return v * 1e3


def _all_ok(ok, dist, device, backend):
    """True on every rank iff `ok` on every rank (one MIN all-reduce; no-op at N = 1)."""
    if not dist:
        return ok
    import torch.distributed as tdist
    t = torch.tensor([1 if ok else 0], device=device if backend == "nccl" else "cpu", dtype=torch.int32)
    tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
    return bool(int(t.item()))


def c4_strong_leg(args, device, dist, world, rank, reps=3):
    """Config 4 (4096^2, Matern-3/2, 200 RHS global) compute_kn split over the ranks: the
    workload the 8-GPU configuration is quoted on (25 RHS per GPU at N = 8).

    One untimed warm-up call (plan creation, workspace and CG-vector allocation, twiddle tables),
    then `reps` timed calls, each barrier + synchronise bracketed, max over ranks: the median and
    the min, every repetition, and the phase split of each -- set-up (ToeplitzTensor: pooled plan
    + spectrum), PCG(20), R^T -- with a synchronise (and a barrier) after every phase, so the
    phases sum to the call.  The plan's device scratch and the peak torch allocation are reported
    beside it (a plan trimmed from the idle pool re-allocates its scratch inside the next call).

    The set-up (model, Knm) holds no collective: a failure there (e.g. out of device memory on
    a smaller card) is agreed on by every rank (one all-reduce of an ok flag) and the leg is
    skipped on all of them together, so no rank waits in a collective another one left.  The
    timed solve all-reduces every PCG iteration; an error there is recorded only at N = 1 and
    re-raised otherwise (torchrun then stops every rank instead of leaving them blocked)."""
    import torch.distributed as tdist
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    from hipgp_amd import dist as hdist
    from hipgp_amd import plan as hplan
    G, m4 = 200, 4096
    sl = hdist.rhs_shard(G, world, rank)
    grids4 = [torch.linspace(-1, 1, m4, device=device) for _ in range(2)]
    g = torch.Generator(device="cpu").manual_seed(2024)       # the same batch on every rank
    x = (torch.rand(G, 2, generator=g, dtype=torch.float32) * 2 - 1).to(device)
    out = {"what": "config 4: compute_kn (set-up + PCG(20, tol 1e-8, precond, all-RHS break over ranks) + R^T) "
                   "for its fixed global batch of 200 RHS on the 4096^2 grid, split over the ranks",
           "global_rhs": G, "rhs_per_rank": sl.stop - sl.start, "grid": [m4, m4], "scaling": "strong"}
    mod = Knm_local = None
    err = None
    try:
        mod = hg.MeanFieldToeplitzGP(zk.Matern(nu=1.5, dtype=torch.float32), grids4, num_obs=100_000,
                                     sig2_init=0.1, ell_init=0.1, learn_kernel=False, jitter_val=1e-3,
                                     dtype=torch.float32).cuda_params(device.index)
        Knm_local, _ = mod._make_grams(x[sl])
        torch.cuda.synchronize()
    except RuntimeError as e:      # e.g. out of device memory on a smaller card
        err = str(e).splitlines()[0][:200]
    if not _all_ok(err is None, dist, device, args.backend):
        out["error"] = err if err is not None else "set-up failed on another rank"
        del mod, Knm_local
        torch.cuda.empty_cache()
        return out

    def sync():
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()

    def one_call(phases):
        t = [time.perf_counter()]

        def tick(name):
            sync()
            now = time.perf_counter()
            phases[name] = (now - t[0]) * 1e3
            t[0] = now
        kn = hdist.sharded_compute_kn(mod, Knm_local, maxiter_cg=20, tol=1e-8, exact_break=dist, on_phase=tick)
        del kn

    def reduce_max(v):
        if not dist:
            return v
        tt = torch.tensor(v, device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        return tt.tolist()

    try:
        torch.cuda.reset_peak_memory_stats(device)
        sync()
        t0 = time.perf_counter()
        warm = {}
        one_call(warm)
        sync()
        warm_ms = (time.perf_counter() - t0) * 1e3
        runs = []
        for _ in range(reps):
            ph = {}
            sync()
            t0 = time.perf_counter()
            one_call(ph)
            sync()
            total = (time.perf_counter() - t0) * 1e3
            runs.append(reduce_max([total, ph.get("setup", 0.0), ph.get("pcg", 0.0), ph.get("rt", 0.0)]))
        warm = reduce_max([warm_ms, warm.get("setup", 0.0), warm.get("pcg", 0.0), warm.get("rt", 0.0)])
        tot = [r[0] for r in runs]
        med = float(np.median(tot))
        idle = hplan._POOL.get(((m4, m4), torch.float32, device.index), [])
        scratch = [hplan._scratch_bytes(h) for h in idle]
        out.update({"ms": med, "ms_min": float(min(tot)), "reps": reps, "rhs_per_s": G / (med * 1e-3),
                    "runs_ms": [dict(zip(("total", "setup", "pcg", "rt"), [round(v, 2) for v in r])) for r in runs],
                    "warmup_ms": dict(zip(("total", "setup", "pcg", "rt"), [round(v, 2) for v in warm])),
                    "phase_median_ms": {k: float(np.median([r[i] for r in runs]))
                                        for i, k in enumerate(("total", "setup", "pcg", "rt"))},
                    "plan_scratch_bytes": max(scratch) if scratch else None,
                    "torch_peak_bytes": int(torch.cuda.max_memory_allocated(device)),
                    "note": "phases max over ranks each, synchronised (and barriered) after every phase"})
    except RuntimeError as e:
        if dist:
            raise
        out["error"] = str(e).splitlines()[0][:200]
    del mod, Knm_local
    torch.cuda.empty_cache()
    return out


def multi_gpu_legs(args, m, grids, kf, device, dist, world, rank, reps):
    """The fixed-global-batch legs (see the module docstring); every timing is a barrier +
    synchronise on both sides, max over ranks, median of `reps`."""
    import torch.distributed as tdist
    import ziggy.hipgp as hg
    import ziggy.kernels as zk
    from hipgp_amd import dist as hdist
    G = args.rhs                                              # C2's global batch
    sl = hdist.rhs_shard(G, world, rank)
    g = torch.Generator(device="cpu").manual_seed(4321)       # the SAME minibatch on every rank
    x = (torch.rand(G, 2, generator=g, dtype=torch.float32) * 2 - 1).to(device)
    y = (torch.sin(3 * x[:, :1]) * torch.cos(2 * x[:, 1:]) + 0.1 * torch.randn(G, 1, generator=g).to(device))
    s = torch.full((G, 1), 0.1, device=device)
    mod = hg.MeanFieldToeplitzGP(zk.SqExp(dtype=torch.float32), grids, num_obs=100_000, sig2_init=1.,
                                 ell_init=.01, learn_kernel=False, jitter_val=1e-3, dtype=torch.float32)
    mod = mod.cuda_params(device.index)
    Knm_local, _ = mod._make_grams(x[sl])

    def timed(fn):
        out = []
        fn()
        for _ in range(reps):
            torch.cuda.synchronize()
            if dist:
                tdist.barrier()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if dist:
                tdist.barrier()
            out.append(time.perf_counter() - t0)
        v = float(np.median(out))
        if dist:
            tt = torch.tensor([v], device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
            tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
            v = float(tt.item())
        return v * 1e3

    grp = None
    # N = 1: the plan's own break test is the all-RHS rule (no process group to reduce over)
    kn_ms = timed(lambda: hdist.sharded_compute_kn(mod, Knm_local, maxiter_cg=20, tol=1e-8, exact_break=dist))
    elbo_ms = timed(lambda: hdist.sharded_elbo_and_grad(mod, x, y, s, maxiter_cg=20, tol=1e-8, exact_break=dist))
    Mp = mod.Mprime
    stats = [torch.zeros(Mp, device=device), torch.zeros(Mp, device=device)]
    ar_ms = timed(lambda: [hdist._allreduce_(t, grp) for t in stats]) if dist else 0.0
    return {"strong": {"what": "compute_kn (set-up + PCG(20, tol 1e-8, precond, all-RHS break over ranks) + R^T) "
                                "for a fixed global batch split over the ranks",
                       "global_rhs": G, "rhs_per_rank": sl.stop - sl.start, "ms": kn_ms,
                       "rhs_per_s": G / (kn_ms * 1e-3), "scaling": "strong"},
            "elbo_step": {"what": "mean-field elbo_and_grad minibatch (Kuf + compute_kn + statistics + "
                                  "all-reduce of the 2 M' natural-gradient sums), batch split over the ranks",
                          "global_batch": G, "ms": elbo_ms, "stats_allreduce_ms": ar_ms,
                          "stats_allreduce_bytes": 2 * Mp * 4, "backend": args.backend if dist else None}}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(argv, gpus, port):
    """The torchrun command that starts `gpus` rank processes of this script (same arguments),
    one per GPU, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_plan(args, env):
    """What main() does with --gpus N in environment `env`: ("run", None) in a rank process
    (WORLD_SIZE == N, or N = 1 with no torch.distributed environment), ("launch", cmd) for N > 1
    without one (this process starts the N ranks as a torchrun child BEFORE touching the GPU,
    and exits with its code), ("refuse", why) when WORLD_SIZE and --gpus disagree."""
    ws = env.get("WORLD_SIZE")
    if args.gpus < 1:
        return "refuse", f"--gpus must be >= 1, got {args.gpus}"
    if ws is None:
        if args.gpus == 1:
            return "run", None
        return "launch", rank_launch_cmd(sys.argv[1:], args.gpus, _free_port())
    if int(ws) != args.gpus:
        return "refuse", (f"WORLD_SIZE={ws} but --gpus {args.gpus}: launch {args.gpus} ranks "
                          f"(torchrun --nproc-per-node {args.gpus}) or pass --gpus {ws}")
    return "run", None


def main():
    args = parse()
    what, detail = launch_plan(args, os.environ)
    if what == "refuse":
        print(f"bench.py: refusing to run: {detail}", file=sys.stderr)
        sys.exit(2)
    if what == "launch":
        # no GPU call has happened in this process: the ranks are children, never an exec
        import subprocess
        sys.exit(subprocess.call(detail))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    dev_index = 0 if (args.same_device or not dist) else local
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(dev_index)
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            tdist.init_process_group(args.backend)
        world = tdist.get_world_size()           # as the initialised process group sees it
        rank = tdist.get_rank()
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)

    from hipgp_amd import _lib
    from ziggy.misc.toeplitz_tensor import ToeplitzTensor

    m, B = args.m, args.rhs
    M = m * m
    grids, kf, Knm = make_problem(m, B, device, seed=1234 + rank)
    stream = torch.cuda.current_stream(device)

    def reduce_max(v):
        if not dist:
            return v
        tt = torch.tensor([v], device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        return float(tt.item())

    T = ToeplitzTensor(grids, kf, batch_shape=(B,), jitter_val=1e-3)
    plan = T._plan
    y = torch.empty_like(Knm)
    step = lambda: plan.apply(_lib.OP_K, Knm, out=y)

    def settle():
        # sustained untimed load: the clock keeps rising over the first few hundred ms of
        # back-to-back work (tools/step_profile.py: 0.300 -> 0.286 ms per K step over three
        # 20-step rounds after 60 warm steps), so timed work runs at the steady clock
        t_end = time.perf_counter() + args.settle_s
        while time.perf_counter() < t_end:
            for _ in range(20):
                step()
            torch.cuda.synchronize()

    # ---- PCG wall-clock: compute_kn = setup + PCG(20) + R^T (untimed for the metric) ---------
    def compute_kn():
        Tk = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=1e-3)
        d0 = Tk.inv_matmul(Knm, do_precond=True, maxiter=20, tol=1e-8)
        return Tk._matmul_by_RT(d0)

    pcg_times = []
    if not args.kop_only:
        compute_kn()
        torch.cuda.synchronize()
        settle()
        for _ in range(args.pcg_reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            kn = compute_kn()
            torch.cuda.synchronize()
            pcg_times.append(time.perf_counter() - t1)
        del kn
        # split: setup alone, and the PCG+R^T alone with a prebuilt plan
        t1 = time.perf_counter()
        Tk = ToeplitzTensor(grids, kf, batch_shape=None, jitter_val=1e-3)
        torch.cuda.synchronize()
        setup_s = time.perf_counter() - t1
        t1 = time.perf_counter()
        d0 = Tk.inv_matmul(Knm, do_precond=True, maxiter=20, tol=1e-8)
        Tk._matmul_by_RT(d0)
        torch.cuda.synchronize()
        solve_s = time.perf_counter() - t1
        del Tk, d0

        # ---- per-kernel HIP-event timing of the K matvec (on the plan's stream) ------------
        for _ in range(3):
            step()                                           # workspaces allocated, clocks up
        op_ms = time_events(step, 20, stream)
        npass = _lib.lib().hgp_op_pass_count(plan._h)
        pass_ms = []
        for pidx in range(npass):
            fn = lambda: _lib.check(_lib.lib().hgp_toeplitz_apply_pass(
                plan._h, _lib.OP_K, Knm.data_ptr(), y.data_ptr(), B, pidx))
            fn()
            pass_ms.append(time_events(fn, 20, stream))

    legs = None
    if not args.kop_only and not args.no_legs:
        legs = multi_gpu_legs(args, m, grids, kf, device, dist, world, rank, args.legs_reps)
        torch.cuda.empty_cache()
        if not args.no_c4_leg:
            legs["strong_c4"] = c4_strong_leg(args, device, dist, world, rank, reps=args.c4_reps)

    # ---- the metric: W warmup + K timed batched K matvec steps --------------------------------
    settle()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    dt = reduce_max(time.perf_counter() - t0)
    ms_per_step = dt / args.steps * 1e3
    value = world * B * args.steps / dt
    if args.kop_only:
        if rank == 0:
            print(json.dumps({"kop_only": True, "value": value, "ms_per_step": ms_per_step}))
        if dist:
            tdist.destroy_process_group()
        return

    h2 = m                                                   # n2/2 + 1 = m2
    bytes_K_rhs = 8 * M + 32 * m * h2                        # SURVEY §8(d) B_K (d=2), fp32
    bytes_launch = B * bytes_K_rhs
    achieved = bytes_launch / (ms_per_step * 1e-3) / 1e9     # driver-clock: the timed steps
    achieved_ev = bytes_launch / (op_ms * 1e-3) / 1e9         # HIP events on the plan's stream
    L = plan.L_K
    pair_int = m * L[1] * 8                                  # complex intermediate per RHS pair
    Q = (B + 1) // 2
    pass_bytes = [Q * (2 * M * 4 + pair_int), Q * 2 * pair_int + L[0] * L[1] * 4, Q * (pair_int + 2 * M * 4)]
    kernels = [{"pass": i, "kernel": ("rows fwd", "column conv", "rows inv")[i] if npass == 3 else str(i),
                "ms": round(pass_ms[i], 4), "bytes": pass_bytes[i],
                "gbs": round(pass_bytes[i] / (pass_ms[i] * 1e-3) / 1e9, 1),
                "frac": round(pass_bytes[i] / (pass_ms[i] * 1e-3) / 1e9 / HBM_PEAK_GBS, 3)} for i in range(npass)]
    pcg_ms = reduce_max(float(np.median(pcg_times) * 1e3))
    traffic, traffic_src = pmc_traffic(M, B)

    out = {
        "metric": "Toeplitz-FFT Kuu matvecs/sec + PCG wall-clock at M=1M inducing",
        "value": value,
        "unit": "RHS-matvecs/s",
        "n_gpus": world,
        "process_group": ({"world_size": world, "backend": tdist.get_backend(), "same_device": bool(args.same_device)}
                          if dist else None),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Knm rows of seeded uniform observations; random-free kernel grid)",
        "config": {"workload": f"C2: 2-D {m}x{m} SqExp(1,0.01) jitter 1e-3, batched K matvec, "
                               f"{B} RHS per GPU", "M": M, "rhs_per_gpu": B, "global_rhs": B * world,
                   "parallelism": f"rhs-shard x{world}"},
        "pcg_wall_clock_ms": pcg_ms,
        "pcg": {"what": "compute_kn: setup + PCG(maxiter=20, tol=1e-8, precond) + R^T, B RHS",
                "median_ms": pcg_ms, "setup_ms": setup_s * 1e3, "pcg_plus_rt_ms": solve_s * 1e3},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "achieved_note": "bytes_per_launch / ms_per_step (the timed steps' own clock)",
                     "traffic_note": f"HBM bytes per batched K matvec from {traffic_src} "
                                     "(rocprofv3 --pmc, 2*FETCH_SIZE + WRITE_SIZE); algorithmic "
                                     "bytes per launch = bytes_per_launch",
                     "kernel": "batched K matvec = 3 pass kernels (FWD rows, CONV cols, INV rows)",
                     "bytes_per_launch": bytes_launch,
                     "event_op_ms": op_ms, "event_achieved": achieved_ev,
                     "event_frac": achieved_ev / HBM_PEAK_GBS, "passes": kernels,
                     # the op's slowest pass-isolated kernel (the column conv at C2) with its own
                     # algorithmic bytes and roofline fraction
                     "dominant_pass": max(kernels, key=lambda k: k["ms"])},
    }
    if legs is not None:
        out.update(legs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        grids_np = [np.linspace(-1, 1, m, dtype=np.float32) for _ in range(2)]
        out["cpu_baseline"] = cpu_baseline(m, B, grids_np, seed=7, threads=args.cpu_threads)
        out["cpu_baseline"]["speedup_matvec"] = value / out["cpu_baseline"]["value"]
        out["cpu_baseline"]["speedup_pcg"] = out["cpu_baseline"]["pcg_s"] * 1e3 / pcg_ms
    if rank == 0:
        print(json.dumps(out))
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
