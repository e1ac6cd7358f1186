"""Right-hand-side sharding of the HIP-GP hot path over GPUs (one process per GPU).

SURVEY §8(e): every CG scalar is per right-hand side (`cg.py:64,66,69,74`), so a minibatch's
observations split into contiguous shards, one per rank, and each rank runs set-up + PCG + R^T
for its own rows with NO collective inside the solve.  Two places couple ranks:

* the all-RHS break rule of `cg.py:70` — `ToeplitzPlan.pcg_allranks` applies it exactly with one
  all-reduce(MIN) of an int flag per iteration, on the device with RCCL (only when
  `exact_break` is on: the default for fp64; with fp32 / tol 1e-8 it never fires and ranks run
  `maxiter` steps on their own);
* the natural-gradient statistics (`hipgp.py:234-266`): sum_n a_n, -sum_n ivar (kn.m - y) kn and
  sum_n ivar kn^2 (mean-field) or the per-block grams sum_n ivar kn_blk kn_blk^T (block family)
  — all-reduced (SUM, in place) once per minibatch, after which every rank holds identical
  theta gradients.

Backend: "nccl" (= RCCL over xGMI on ROCm) on GPUs, "gloo" for the CPU tests.
"""
import torch
import torch.distributed as dist


def world():
    """(world_size, rank) of the default group, (1, 0) when torch.distributed is not up."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def rhs_shard(n, world_size, rank):
    """Contiguous, balanced slice of n right-hand sides owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world_size)
    start = rank * base + min(rank, extra)
    return slice(start, start + base + (1 if rank < extra else 0))


def _allreduce_(t, group):
    """In-place SUM all-reduce; gloo reduces CUDA tensors through a host copy."""
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        host = t.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_stats(stats, group=None):
    """Sum the batch statistics of all ranks: lam_sum ((M',) mean-field or (nblk, bs, bs) block
    grams) and dm_sum (M',) are reduced in place (no packed copy of the M'-sized vectors), the
    two scalars (sum a_n, n) in one small buffer."""
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    if ws == 1:
        return stats
    lam, dm = stats["lam_sum"].contiguous(), stats["dm_sum"].contiguous()
    _allreduce_(lam, group)
    _allreduce_(dm, group)
    small = torch.stack([torch.as_tensor(stats["an_sum"], dtype=lam.dtype, device=lam.device).reshape(()),
                         torch.as_tensor(float(stats["n"]), dtype=lam.dtype, device=lam.device)])
    _allreduce_(small, group)
    return {"lam_sum": lam, "dm_sum": dm, "an_sum": small[0], "n": int(round(float(small[1])))}


def sharded_compute_kn(model, Knm_local, maxiter_cg=10, tol=1e-8, exact_break=None, group=None, Kmm=None):
    """kn = R^T K^{-1} Knm^T for this rank's rows (`hipgp.py:117-146`).  exact_break applies
    the all-RHS break rule across ranks (see module docstring); default: on for fp64 (where
    tol = 1e-8 can be met) and off for fp32 (where it never is at these sizes).  A rank whose
    shard is empty returns a (0, M') kn and still joins the break rule's all-reduces."""
    if exact_break is None:
        exact_break = Knm_local.dtype == torch.float64
    if Knm_local.shape[0] == 0:
        if exact_break:
            from hipgp_amd.plan import pcg_idle_rank
            pcg_idle_rank(maxiter_cg, Knm_local.device, group)
        return Knm_local.new_zeros((0, model.Mprime))
    if Kmm is None:
        Kmm = model.toeplitz()
    if exact_break:
        Kmm.set_batch_shape(Knm_local.shape[:-1])   # as _solve does (toeplitz_tensor.py:61)
        d0, _ = Kmm._plan.pcg_allranks(Knm_local, maxiter_cg, tol, precond=True, group=group)
    else:
        d0 = Kmm.inv_matmul(Knm_local, do_precond=True, maxiter=maxiter_cg, tol=tol)
    return Kmm._matmul_by_RT(d0)


def sharded_elbo_and_grad(model, xbatch, ybatch, noise_std_batch=None, maxiter_cg=10, tol=1e-8,
                          exact_break=None, group=None, compute_kn=None, integrated_obs=False,
                          semi_integrated_estimator="analytic", semi_integrated_samps=10):
    """`elbo_and_grad` (mean-field or block family) with the minibatch sharded by rows over the
    ranks of `group`; every rank passes the SAME full minibatch and gets the same ELBO and theta
    grads.  `compute_kn(model, Knm_local)` may be injected (tests run the host logic on CPU).
    Line-integral observations ("mc-biased") draw the reference's one torch.rand(1) offset per
    rank: ranks seeded alike draw the same offset, as the single-process reference does.

    Hyper-parameter learning (learn_kernel / learn_noise): the returned ELBO's value is the
    global one and its graph holds this rank's share of sum_n a_n / bsz; after backward(),
    `allreduce_hyper_grads(model)` sums the shares (as the single process would get them)."""
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    rk = dist.get_rank(group) if dist.is_initialized() else 0
    sl = rhs_shard(xbatch.shape[0], ws, rk)
    Knm, Knn_diag = model._make_grams(xbatch[sl], integrated_obs=integrated_obs,
                                      semi_integrated_estimator=semi_integrated_estimator,
                                      semi_integrated_samps=semi_integrated_samps)
    if compute_kn is None:
        kn = sharded_compute_kn(model, Knm, maxiter_cg=maxiter_cg, tol=tol, exact_break=exact_break, group=group)
    else:
        kn = compute_kn(model, Knm)
    nsd = None if noise_std_batch is None else noise_std_batch[sl]
    stats = allreduce_stats(model.batch_stats(kn, ybatch[sl], Knn_diag, nsd), group=group)
    elbo = model.apply_stats(stats, xbatch.shape[0])
    if model.hyper_grad_needed(nsd):
        n_local = sl.stop - sl.start
        if n_local > 0:
            share = model.autograd_elbo(xbatch[sl], ybatch[sl], nsd, Knm, Knn_diag, kn, nsum=n_local,
                                        bsz=xbatch.shape[0])
            elbo = elbo.detach() + (share - share.detach())
    return elbo


def allreduce_hyper_grads(model, group=None):
    """Sum the kernel / noise hyper-parameter gradients over the ranks after backward() of
    `sharded_elbo_and_grad`'s ELBO (a rank with no observations contributes zeros)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    for p in (model.log_sig2, model.log_ell, model.log_noise2):
        if not p.requires_grad:
            continue
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        p.grad = _allreduce_(g.detach().clone(), group)
