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


class AllRanksInvMatmul(torch.autograd.Function):
    """`InvMatmul` (`_inv_matmul.py:9-64`) for one rank's share of the RHS, with the reference's
    all-RHS break rule (`cg.py:69-71`) applied over every rank of `group`
    (`ToeplitzPlan.pcg_allranks`) in BOTH solves: the forward K^-1 b and the backward's left
    solves K^-1 grad (`_inv_matmul.py:34-36`), whose break the single process also decides over
    all B gradient rows.  The column gradient is the rank's share of the quadratic form
    (`_inv_matmul.py:52-60`, hgp_plan_dqf); `allreduce_hyper_grads` sums the shares.  A rank with
    no RHS joins both solves' all-reduces (`pcg_idle_rank`) and contributes zero gradients, so
    every rank must run backward (sharded_elbo_and_grad keeps a graph on empty ranks)."""

    @staticmethod
    def forward(ctx, tt, column, rhs, maxiter, tol, group):
        ctx.tt, ctx.maxiter, ctx.tol, ctx.group = tt, int(maxiter), float(tol), group
        x = _allranks_solve(tt, rhs.detach(), ctx.maxiter, ctx.tol, group)
        ctx.save_for_backward(x)
        return x

    @staticmethod
    def backward(ctx, grad):
        (right,) = ctx.saved_tensors
        left = _allranks_solve(ctx.tt, grad.detach().contiguous(), ctx.maxiter, ctx.tol, ctx.group)
        gcol = None
        if ctx.needs_input_grad[1]:
            column = ctx.tt.column
            if right.shape[0] == 0:
                gcol = torch.zeros_like(column)
            else:
                with torch.no_grad():
                    lv = torch.cat([left, right], 0)
                    rv = torch.cat([right, left], 0).mul(-0.5)
                    gcol = ctx.tt._plan.dqf(lv, rv).view(column.shape)
        return None, gcol, (left if ctx.needs_input_grad[2] else None), None, None, None


def _allranks_solve(tt, b, maxiter, tol, group):
    """K^-1 b (PCG, preconditioned) with the break rule over all ranks; b may have 0 rows."""
    with torch.no_grad():
        if b.shape[0] == 0:
            from hipgp_amd.plan import pcg_idle_rank
            pcg_idle_rank(maxiter, b.device, group)
            return b.new_zeros(b.shape)
        tt.set_batch_shape(b.shape[:-1])       # as _solve does (toeplitz_tensor.py:61)
        x, _ = tt._plan.pcg_allranks(b, maxiter, tol, precond=True, group=group)
        return x


def sharded_compute_kn(model, Knm_local, maxiter_cg=10, tol=1e-8, exact_break=None, group=None, Kmm=None,
                       on_phase=None):
    """kn = R^T K^{-1} Knm^T for this rank's rows (`hipgp.py:117-146`).  exact_break applies
    the all-RHS break rule across ranks (see module docstring); default: on for fp64 (where
    tol = 1e-8 can be met) and off for fp32 (where it never is at these sizes).  The exact-break
    solve is differentiable (AllRanksInvMatmul), like the reference's InvMatmul.  A rank whose
    shard is empty returns a (0, M') kn and still joins the break rule's all-reduces (and, when
    kn carries a graph, the backward solve's).  on_phase(name) is called after the set-up
    ("setup"), the solve ("pcg") and R^T ("rt") -- the bench's phase split."""
    tick = on_phase if on_phase is not None else (lambda name: None)
    if exact_break is None:
        exact_break = Knm_local.dtype == torch.float64
    # the solve carries a graph iff the kernel parameters are learned (column and Knm need grad);
    # the same on every rank, so an empty rank then keeps it too
    kernel_grad = (torch.is_grad_enabled() and bool(model.learn_kernel)
                   and bool(model.log_sig2.requires_grad or model.log_ell.requires_grad))
    if Knm_local.shape[0] == 0 and not (exact_break and kernel_grad):
        tick("setup")                 # every rank reports the same phases (a caller may barrier in them)
        if exact_break:
            from hipgp_amd.plan import pcg_idle_rank
            pcg_idle_rank(maxiter_cg, Knm_local.device, group)
        tick("pcg")
        tick("rt")
        return Knm_local.new_zeros((0, model.Mprime))
    if Kmm is None:
        Kmm = model.toeplitz()
    tick("setup")
    if exact_break:
        d0 = AllRanksInvMatmul.apply(Kmm, Kmm.column, Knm_local, maxiter_cg, tol, group)
    else:
        d0 = Kmm.inv_matmul(Knm_local, do_precond=True, maxiter=maxiter_cg, tol=tol)
    tick("pcg")
    if Knm_local.shape[0] == 0:
        # keep the solve in the graph (its backward joins the other ranks' all-reduces)
        tick("rt")
        return Knm_local.new_zeros((0, model.Mprime)) + 0 * d0.sum()
    Kmm.set_batch_shape(d0.shape[:-1])
    kn = Kmm._matmul_by_RT(d0)
    tick("rt")
    return kn


def shared_mc_offset(dtype, device, group=None):
    """The MC line-integral estimator's one offset draw per minibatch (`kernels.py:28-29`,
    `torch.rand(1)` in the kernel dtype on the observations' device), the same on every rank:
    each rank draws it exactly as the single process does (so every rank's RNG stream advances
    alike) and then takes rank 0's value by a broadcast -- ranks agree without relying on being
    seeded alike (the reference's domain script seeds only NumPy)."""
    u = torch.rand(1, dtype=dtype, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if dist.get_backend(group) == "gloo" and u.is_cuda:
            h = u.cpu()
            dist.broadcast(h, src, group=group)
            u.copy_(h)
        else:
            dist.broadcast(u, src, group=group)
    return u


def sharded_elbo_and_grad(model, xbatch, ybatch, noise_std_batch=None, maxiter_cg=10, tol=1e-8,
                          exact_break=None, group=None, compute_kn=None, integrated_obs=False,
                          semi_integrated_estimator="analytic", semi_integrated_samps=10):
    """`elbo_and_grad` (mean-field or block family) with the minibatch sharded by rows over the
    ranks of `group`; every rank passes the SAME full minibatch and gets the same ELBO and theta
    grads.  `compute_kn(model, Knm_local)` may be injected (tests run the host logic on CPU).
    Line-integral observations ("mc-biased"): the reference's one torch.rand(1) offset per
    minibatch is drawn once and broadcast from rank 0 (shared_mc_offset), so every rank's rows
    use the offset the single process would use for the whole minibatch.

    Hyper-parameter learning (learn_kernel / learn_noise): the returned ELBO's value is the
    global one and its graph holds this rank's share of sum_n a_n / bsz; after backward(),
    `allreduce_hyper_grads(model)` sums the shares (as the single process would get them)."""
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    rk = dist.get_rank(group) if dist.is_initialized() else 0
    sl = rhs_shard(xbatch.shape[0], ws, rk)
    u = None
    if integrated_obs and semi_integrated_estimator == "mc-biased":
        u = shared_mc_offset(model.kernel.dtype, xbatch.device, group)
    Knm, Knn_diag = model._make_grams(xbatch[sl], integrated_obs=integrated_obs,
                                      semi_integrated_estimator=semi_integrated_estimator,
                                      semi_integrated_samps=semi_integrated_samps, mc_offset=u)
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
        else:
            # an empty shard: a zero share that still holds a graph, so backward() runs here too
            # (it joins the exact-break backward solve's all-reduces) and allreduce_hyper_grads
            # is reached on every rank
            params = [p for p in (model.log_sig2, model.log_ell, model.log_noise2) if p.requires_grad]
            share = 0 * (kn.sum() + sum(p.sum() for p in params))
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
