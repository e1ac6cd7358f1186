"""The SVI base class and its minibatch natural-gradient driver (`ziggy/svi_gp.py:14-442`),
on the MI355X operators.

The driver is host-side Python (a DataLoader loop); every step's work is the model's
`elbo_and_grad` — the fused Kuf kernel, one PCG solve through libhipgp and the statistics
kernels — followed by torch's SGD / Adam updates on the device.

Reference map:
  SviGP.torch / _make_grams / batch_predict       `svi_gp.py:24-97`
  SviGP.fit -> svigp_fit                          `svi_gp.py:99-114, 172-442`
  SviGP.ell_fit -> ell_fit                        `svi_gp.py:116-169`
  estimate_predictive_variance_correction         `svi_gp.py:119-128`

Behaviour kept from the reference loop: sequential (unshuffled) minibatches, SGD on
(theta1, theta2) with a per-BATCH StepLR decay, Adam on the log kernel / noise parameters
when they are learned (`(-elbo).backward()` before the natural-gradient step), the ELBO trace
of logged batches, the best epoch ELBO, the per-epoch callback and `time_report.csv`.
Where the reference cannot run, this one does and says so:
  * learn_noise=True: the reference moves `noise_std_batch=None` to the device
    (`svi_gp.py:302`) and logs an undefined `log_noise_std` (`:348`); here the noise
    variance is read from `log_noise2`.
"""
import os
import time

import numpy as np
import torch
from torch import nn
from torch.utils.data import DataLoader, TensorDataset


class SviGP(nn.Module):
    """Abstract GP fitted by stochastic variational inference (`svi_gp.py:14-128`)."""

    def __init__(self):
        super().__init__()
        self.pred_scale_factor = 1.

    def torch(self, arr):
        """numpy -> tensor of the model dtype; tensors must already have it (`svi_gp.py:24-32`).

        Quirk kept: the reference builds `torch.Tensor(arr)` first -- the DEFAULT dtype (fp32)
        -- and only then casts to the model dtype, so an fp64 model sees its numpy data
        (observation coordinates, values, noise) rounded to fp32.  With UK-box coordinates
        (~50-55, G19) the difference is 2e-5 of the first natural-gradient step."""
        if isinstance(arr, np.ndarray):
            return torch.tensor(arr, dtype=torch.get_default_dtype()).to(self.dtype)
        if isinstance(arr, torch.Tensor):
            assert arr.dtype == self.dtype, f"model dtype = {self.dtype}, data dtype = {arr.dtype}"
            return arr
        raise ValueError(f"Only accepts np.ndarray or torch.Tensor, got {type(arr)}")

    def cuda_params(self, cuda_num=0):
        raise NotImplementedError

    def elbo_and_grad(self, xbatch, ybatch, noise_std_batch, **kwargs):
        raise NotImplementedError

    def predict(self, x, **kwargs):
        raise NotImplementedError

    def batch_solve(self, xbatch, ybatch, noise_std_batch, **kwargs):
        raise NotImplementedError

    def _make_grams(self, xbatch, integrated_obs=False, semi_integrated_estimator="analytic",
                    semi_integrated_samps=10, mc_offset=None, grid_rows=None):
        """(Knm, Knn_diag) for a minibatch (`svi_gp.py:48-76`): on a grid model the fused HIP
        kernels of `hipgp_amd.kuf` write Knm directly in the PCG layout.

        Not in the reference (sharded fits): mc_offset -- the MC line-integral estimator's offset
        draw to use instead of drawing one here (`hipgp_amd.dist.shared_mc_offset`); grid_rows =
        (a, b) -- only the Knm columns of the grid's axis-0 rows [a, b) (a grid-block slab,
        `hipgp_amd.slab.SlabFit`: columns [a * M / m0, b * M / m0) of the full Knm)."""
        params = self.get_kernel_params()
        grids, xinduce = getattr(self, "xgrids", None), self.xinduce
        if grid_rows is not None:
            a, b = grid_rows
            rest = self.xinduce.shape[0] // len(grids[0])
            grids = [grids[0][a:b]] + list(grids[1:])
            xinduce = xinduce[a * rest:b * rest]
        if integrated_obs:
            return self._make_integrated_grams(xbatch, params, semi_integrated_estimator, semi_integrated_samps,
                                               grids, xinduce, mc_offset)
        Knm = None
        if grids is not None:
            from hipgp_amd.kuf import kuf_grid
            Knm = kuf_grid(self.kernel, grids, xbatch, params)          # fused HIP kernel
        if Knm is None:
            Knm = self.kernel(xbatch, xinduce, params)
        return Knm, self.kernel.diag(xbatch, params)

    def _make_integrated_grams(self, xbatch, params, estimator, samps, grids=None, xinduce=None, mc_offset=None):
        """Line-integral observations, `svi_gp.py:55-69`: Knm by the analytic SqExp integral or
        the biased MC estimator (fused HIP kernels on the grid, `hipgp_amd.kuf`), Knn_diag by the
        doubly-integrated table (`hgp_knn_doubly_diag`)."""
        from hipgp_amd import kuf
        if xinduce is None:
            grids, xinduce = getattr(self, "xgrids", None), self.xinduce
        if estimator == "analytic":
            Knm = kuf.kuf_semi_sqexp(self.kernel, grids, xbatch, params) if grids is not None else None
            if Knm is None:
                Knm = self.kernel.k_semi(xinduce, xbatch, params).transpose(0, 1)
        elif estimator == "mc-biased":
            Knm = kuf.kuf_semi_mc(self.kernel, grids, xbatch, params, samps, u=mc_offset) if grids is not None else None
            if Knm is None:
                Knm = self.kernel.k_semi_mc(xinduce, xbatch, params, npts=samps, u=mc_offset).transpose(0, 1)
        elif estimator == "numerical":
            Knm = self.kernel.k_semi_num(xinduce, xbatch, params).transpose(0, 1)
        else:
            raise NotImplementedError
        return Knm, self.kernel.k_doubly_diag(xbatch, params)

    def batch_predict(self, x, batch_size, verbose=True, **kwargs):
        """predict() over consecutive chunks of x, concatenated (`svi_gp.py:78-97`)."""
        nb = int(np.ceil(len(x) / batch_size))
        mus, sigs = [], []
        for b in range(nb):
            mu, sig = self.predict(x[b * batch_size:(b + 1) * batch_size], **kwargs)
            mus.append(mu)
            sigs.append(sig)
            if verbose and b % 100 == 0:
                print(" ... batch_predict %d / %d batches" % (b, nb))
        return torch.cat(mus, dim=0), torch.cat(sigs, dim=0)

    def fit(self, odir, xtrain, ytrain, noise_std_train, xtest, ftest, etest, xgrid, fgrid, egrid,
            xvalid=None, fvalid=None, evalid=None, batch_callback=None, epoch_callback=None, **kwargs):
        """Natural-gradient SVI over minibatches (`svi_gp.py:99-114`); see `svigp_fit`."""
        return svigp_fit(self, odir, xtrain, ytrain, noise_std_train, xtest, ftest, etest, xgrid, fgrid, egrid,
                         xvalid, fvalid, evalid, batch_callback, epoch_callback, **kwargs)

    def ell_fit(self, mod, odir, xobs, yobs, sobs, **fit_kwargs):
        return ell_fit(mod, odir, xobs, yobs, sobs, **fit_kwargs)

    def estimate_predictive_variance_correction(self, xobs, aobs, sobs, **kwargs):
        """Scale predictive sds so the residual variance matches (`svi_gp.py:119-128`)."""
        self.pred_scale_factor = 1.
        fmu, fsig = self.batch_predict(xobs, batch_size=100, **kwargs)
        resid = (aobs - fmu).squeeze()
        self.pred_scale_factor = torch.sqrt((torch.sum(resid ** 2) - torch.sum(sobs ** 2))
                                            / torch.sum(fsig ** 2)).item()
        print("changing pred_scale_factor to {}".format(self.pred_scale_factor))


def ell_fit(mod, odir, xobs, yobs, sobs, **fit_kwargs):
    """Grid search of the length scale by full-batch solves (`svi_gp.py:131-169`): for each ell
    in arange(ell_min, ell_max + step, step) set the kernel, batch_solve with the ELBO, keep the
    best; the model ends solved at the best ell.  Returns (ells, best_ell, elbos, best_elbo)."""
    lo, hi, step = fit_kwargs["ell_min"], fit_kwargs["ell_max"], fit_kwargs["ell_step_size"]
    ells = np.arange(lo, hi + step, step)
    print("Annealing ell among", list(ells))

    def solve():
        return mod.batch_solve(mod.torch(xobs), mod.torch(yobs), mod.torch(sobs),
                               batch_size=fit_kwargs["batch_solve_bsz"],
                               integrated_obs=fit_kwargs["integrated_obs"],
                               semi_integrated_estimator=fit_kwargs["ksemi_method"],
                               semi_integrated_samps=fit_kwargs["ksemi_samps"],
                               maxiter_cg=fit_kwargs["maxiter_cg"], compute_elbo=True)

    best_ell, best_elbo, elbos = -1, -1e10, []
    for ell in ells:
        mod.update_kernel_params(ell=ell)
        elbo = solve()
        elbos.append(elbo.detach().cpu().numpy())
        if elbo > best_elbo:
            best_ell, best_elbo = ell, elbo
        print("ell={} elbo={:.5f} Best ell={} Best elbo={:.5f} \n".format(ell, elbo, best_ell, best_elbo))
    mod.update_kernel_params(ell=best_ell)
    elbo = solve()
    assert best_elbo == elbo, "best elbo = {}, elbo = {}".format(best_elbo, elbo)
    return list(ells), best_ell, elbos, best_elbo


def _fit_options(kw):
    """The reference's fit_kwargs and their defaults (`svi_gp.py:182-221`)."""
    o = dict(do_cuda=kw.get("do_cuda", torch.cuda.is_available()), cuda_num=kw.get("cuda_num", 0),
             fit_method=kw.get("fit_method", "natgrad"), lr=kw.get("lr", 1e-2),
             schedule_lr=kw.get("schedule_lr", True), step_decay=kw.get("step_decay", .99),
             batch_size=kw.get("batch_size", 256), epochs=kw.get("epochs", 50),
             learn_kernel=kw.get("learn_kernel", False), kernel_lr=kw.get("kernel_lr", 1e-3),
             learn_noise=kw.get("learn_noise", False), print_debug_info=kw.get("print_debug_info", False),
             epoch_log_interval=kw.get("epoch_log_interval", 1), batch_log_interval=kw.get("batch_log_interval", 1),
             maxiter_cg=kw.get("maxiter_cg", 5), integrated_obs=kw.get("integrated_obs", False),
             do_integrated_predictions=kw.get("do_integrated_predictions", False),
             semi_integrated_estimator=kw.get("semi_integrated_estimator", "analytic"),
             num_semi_mc_samples=kw.get("num_semi_mc_samples", 10),
             predict_ksemi_method=kw.get("predict_ksemi_method", "analytic"),
             predict_ksemi_samps=kw.get("predict_ksemi_samps", 200),
             predict_maxiter_cg=kw.get("predict_maxiter_cg", 50), eval_train=kw.get("eval_train", False),
             only_eval_last_epoch=kw.get("only_eval_last_epoch", False))
    assert o["fit_method"] in ("natgrad", "gd"), \
        "got fit_method = {}, must choose from natgrad and gd".format(o["fit_method"])
    # multi-GPU (not in the reference, which is single-device): one process per GPU under
    # torchrun, every rank running the same script on the same data.  "distributed": "auto"
    # (sharded when torch.distributed is initialised with world size > 1), True, False;
    # "shard": "rhs" (each rank solves its rows of every minibatch, hipgp_amd.dist) or "grid"
    # (each rank owns an axis-0 slab of the inducing grid, hipgp_amd.slab.SlabKmm)
    # "slab": a prebuilt hipgp_amd.slab.SlabToeplitz for shard="grid" (tests inject a CPU engine);
    # "dist_timeout_s": the process-group timeout when the fit initialises the group itself --
    # only rank 0 runs the epoch callback (predictions), the other ranks wait at a barrier
    o.update(distributed=kw.get("distributed", "auto"), shard=kw.get("shard", "rhs"),
             process_group=kw.get("process_group", None), compute_kn=kw.get("compute_kn", None),
             slab=kw.get("slab", None), dist_timeout_s=kw.get("dist_timeout_s", 4 * 3600))
    assert o["shard"] in ("rhs", "grid"), "shard must be 'rhs' or 'grid', got {}".format(o["shard"])
    return o


def _fit_world(o, mod=None):
    """(sharded?, world size, rank) of a fit under torch.distributed (see _fit_options).  An
    unchanged experiment script launched by torchrun (WORLD_SIZE > 1 in the environment) has
    not initialised a process group: it is initialised here -- RCCL ("nccl") on cuda:LOCAL_RANK,
    gloo when the fit runs on the CPU.

    Only the Toeplitz ("ziggy") whitening shards: a cholesky-whitened model (`hipgp.py:120-128`,
    a dense M x M factor, M' = M) has no RHS / grid-block split here, so with distributed="auto"
    every rank runs the whole single-process fit (as before sharding existed; a warning says
    so), and distributed=True refuses it."""
    import torch.distributed as dist
    if mod is not None and getattr(mod, "whitened_type", "ziggy") != "ziggy":
        if o["distributed"] is True:
            raise NotImplementedError("sharded fits need whitened_type='ziggy' (the Toeplitz operators); "
                                      f"this model is whitened_type={mod.whitened_type!r}")
        if o["distributed"] == "auto" and ((dist.is_available() and dist.is_initialized())
                                           or int(os.environ.get("WORLD_SIZE", "1")) > 1):
            import warnings
            warnings.warn(f"whitened_type={mod.whitened_type!r} does not shard: every rank runs the whole fit",
                          RuntimeWarning, stacklevel=3)
        return False, 1, 0
    up = dist.is_available() and dist.is_initialized()
    if (not up and o["distributed"] is not False and dist.is_available()
            and int(os.environ.get("WORLD_SIZE", "1")) > 1):
        import datetime
        timeout = datetime.timedelta(seconds=float(o["dist_timeout_s"]))
        if o["do_cuda"]:
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
        up = True
    if o["distributed"] is False or (o["distributed"] == "auto" and not (up and dist.get_world_size(o["process_group"]) > 1)):
        return False, 1, 0
    if not up:
        raise RuntimeError("distributed=True needs an initialised torch.distributed process group (torchrun)")
    return True, dist.get_world_size(o["process_group"]), dist.get_rank(o["process_group"])


def svigp_fit(mod, odir, xtrain, ytrain, noise_std_train, xtest, ftest, etest, xgrid, fgrid, egrid,
              xvalid, fvalid, evalid, batch_callback, epoch_callback, **fit_kwargs):
    """Minibatch natural-gradient SVI (`svi_gp.py:172-442`).

    Per minibatch (in order, no shuffling): batch_callback(mod, x, y, s); zero the grads;
    elbo = mod.elbo_and_grad(...) (fills theta1/theta2 .grad with minus the natural gradient);
    with learned kernel / noise parameters (-elbo).backward() and an Adam step on them; the SGD
    step on (theta1, theta2); the per-batch StepLR decay.  Per epoch: the mean logged ELBO, the
    epoch callback, and finally `odir/time_report.csv`.  Returns None (the model is fitted in
    place); the ELBO trace of logged batches is kept on `mod.fit_trace`.

    Sharded (an unchanged experiment script under `torchrun --nproc-per-node N`, see
    INTEGRATION.md §4): every rank iterates the same minibatches; with shard="rhs" each rank
    solves its contiguous share of each minibatch's rows and the natural-gradient sums (and the
    learned hyper-parameters' gradients) are all-reduced, with shard="grid" each rank owns an
    axis-0 slab of the inducing grid for the solve.  Either way every rank takes the same
    optimiser steps on identical gradients, so the variational and kernel parameters stay
    identical on every rank.  Each rank runs on cuda:LOCAL_RANK; rank 0 alone prints, runs the
    epoch callback and writes `time_report.csv`."""
    import pandas as pd
    o = _fit_options(fit_kwargs)
    sharded, world_size, rank = _fit_world(o, mod)
    if sharded and "LOCAL_RANK" in os.environ:
        o["cuda_num"] = int(os.environ["LOCAL_RANK"])
    if sharded and o["shard"] == "grid" and (o["learn_kernel"] or o["learn_noise"]):
        raise NotImplementedError("shard='grid' runs the natural-gradient fit with fixed kernel / noise "
                                  "hyper-parameters; use shard='rhs' to learn them")
    device = torch.device("cuda:{}".format(o["cuda_num"]))
    print0 = print if rank == 0 else (lambda *a, **k: None)
    print0("\n-------------- Start training ---------------")
    if sharded:
        print0("sharded fit: {} ranks, {} sharding".format(world_size, o["shard"]))
    estimator = o["semi_integrated_estimator"]
    if o["integrated_obs"] and estimator == "analytic" and not mod.kernel.has_k_semi:
        print0("kernel_fun %s does not have k_semi --- doing MC estimate" % str(mod.kernel))
        estimator = "mc-biased"

    assert len(xtrain.shape) == len(ytrain.shape) == 2
    xtrain, ytrain = mod.torch(xtrain), mod.torch(ytrain)
    learn_noise, learn_kernel = o["learn_noise"], o["learn_kernel"]
    if learn_noise:
        data = TensorDataset(xtrain, ytrain)
    else:
        assert len(noise_std_train.shape) == 2
        data = TensorDataset(xtrain, ytrain, mod.torch(noise_std_train))
    loader = DataLoader(dataset=data, batch_size=o["batch_size"], shuffle=False)

    natgrad_opt = torch.optim.SGD([mod.global_theta1, mod.global_theta2], lr=o["lr"])
    hyper = ([mod.log_ell, mod.log_sig2] if learn_kernel else []) + ([mod.log_noise2] if learn_noise else [])
    hyper_opt = torch.optim.Adam(hyper, lr=o["kernel_lr"]) if hyper else None
    sig2_list = [] if learn_kernel else None
    ell_list = [] if learn_kernel else None
    noisesq_list = [] if learn_noise else None
    scheduler = (torch.optim.lr_scheduler.StepLR(natgrad_opt, step_size=1, gamma=o["step_decay"])
                 if o["schedule_lr"] else None)
    if o["do_cuda"]:
        print0("Fitting SVI GP with CUDA!")
        print0("device: cuda:{}".format(o["cuda_num"]))
        mod = mod.cuda_params(o["cuda_num"])

    # grid-block sharding: the slab operators are built once (the kernel is fixed in this mode);
    # the mean-field family keeps kn in slabs (SlabFit), the block family gathers it (SlabKmm)
    slabfit = kmm = None
    if sharded and o["shard"] == "grid":
        from hipgp_amd.slab import SlabFit, SlabKmm
        if getattr(mod, "name", None) == "mean-field":
            slabfit = SlabFit(mod, group=o["process_group"], slab=o["slab"])
        else:
            kmm = SlabKmm.from_model(mod, group=o["process_group"]) if o["slab"] is None else SlabKmm(o["slab"])

    trace = []
    mod.fit_trace = trace
    best_elbo = -np.inf
    times = {k: [] for k in ("fitting", "ftest_eval", "etest_eval", "fgrid_eval", "egrid_eval",
                             "fvalid_eval", "evalid_eval")}
    ntotal = len(loader.dataset)
    log_every = o["batch_log_interval"]
    for epoch in range(o["epochs"]):
        print0("\n------- epoch {} -----------".format(epoch))
        t_epoch = time.time()
        epoch_loss, nbatch, ndata, ntracked = 0., 0, 0, 0
        for batch in loader:
            xb, yb = batch[0], batch[1]
            sb = None if learn_noise else batch[2]
            t_batch = time.time()
            nbatch += 1
            ndata += xb.shape[0]
            if o["do_cuda"]:
                xb, yb = xb.to(device), yb.to(device)
                sb = None if sb is None else sb.to(device)
            if batch_callback is not None:
                batch_callback(mod, xb, yb, sb)
            logged = (log_every is not False) and (nbatch % log_every == 0)
            natgrad_opt.zero_grad()
            if hyper_opt is not None:
                hyper_opt.zero_grad()
            if sharded and o["shard"] == "rhs":
                from hipgp_amd import dist as hdist
                lval = hdist.sharded_elbo_and_grad(mod, xb, yb, sb, maxiter_cg=o["maxiter_cg"],
                                                   group=o["process_group"], compute_kn=o["compute_kn"],
                                                   integrated_obs=o["integrated_obs"],
                                                   semi_integrated_estimator=estimator,
                                                   semi_integrated_samps=o["num_semi_mc_samples"])
            elif slabfit is not None:           # shard == "grid", mean-field: kn stays in slabs
                lval = slabfit.elbo_and_grad(xb, yb, sb, maxiter_cg=o["maxiter_cg"], integrated_obs=o["integrated_obs"],
                                             semi_integrated_estimator=estimator,
                                             semi_integrated_samps=o["num_semi_mc_samples"])
            else:
                u = None
                if kmm is not None and o["integrated_obs"] and estimator == "mc-biased":
                    from hipgp_amd.dist import shared_mc_offset
                    u = shared_mc_offset(mod.kernel.dtype, xb.device, o["process_group"])
                lval = mod.elbo_and_grad(xbatch=xb, ybatch=yb, noise_std_batch=sb, maxiter_cg=o["maxiter_cg"],
                                         integrated_obs=o["integrated_obs"], semi_integrated_estimator=estimator,
                                         semi_integrated_samps=o["num_semi_mc_samples"],
                                         print_debug_info=o["print_debug_info"], Kmm=kmm, mc_offset=u)
            if hyper_opt is not None:
                (-lval).backward()
                if sharded:
                    from hipgp_amd import dist as hdist
                    hdist.allreduce_hyper_grads(mod, group=o["process_group"])
                hyper_opt.step()
            natgrad_opt.step()
            if scheduler is not None:
                scheduler.step()
            if logged:
                dt = time.time() - t_batch
                val = float(lval.item())
                trace.append(val)
                epoch_loss += val
                ntracked += 1
                msg = ' ... [{}/{} ({:.0f}%)] ELBO: {:.4f}'.format(ndata, ntotal, 100 * ndata / ntotal,
                                                                    epoch_loss / ntracked)
                if hyper_opt is not None:
                    sig2, ell = (float(v.detach().cpu()) for v in mod.get_kernel_params())
                    if learn_kernel:
                        sig2_list.append(np.array(sig2))
                        ell_list.append(np.array(ell))
                        msg += ' sig2={:.4f} ell={:.4f}'.format(sig2, ell)
                    if learn_noise:
                        noisesq = float(torch.exp(mod.log_noise2).detach().cpu())
                        noisesq_list.append(np.array(noisesq))
                        msg += ' noisesq={:.4f}'.format(noisesq)
                print0(msg + ' takes {:.4f}'.format(dt))

        epoch_elbo = epoch_loss / ntracked if ntracked else float("nan")
        elapsed = time.time() - t_epoch
        times["fitting"].append(elapsed)
        if o["epoch_log_interval"] is not False and epoch % o["epoch_log_interval"] == 0:
            print0("Epoch {:5}: {:>10} ({:4} batches) takes {:.4f}".format(epoch, "%2.3f" % epoch_elbo,
                                                                         "%d" % nbatch, elapsed))
        if epoch_elbo > best_elbo:
            best_elbo = epoch_elbo
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        evals = (None,) * 6
        if epoch_callback is not None and rank == 0 and (not o["only_eval_last_epoch"] or epoch == o["epochs"] - 1):
            print0("------- epoch {} -----------\n".format(epoch))
            evals = epoch_callback(os.path.join(odir, "epoch{}".format(epoch)), mod, o["eval_train"], xtrain, ytrain,
                                   noise_std_train, xtest, ftest, etest, xgrid, fgrid, egrid, o["cuda_num"],
                                   o["predict_maxiter_cg"], o["do_integrated_predictions"], o["predict_ksemi_method"],
                                   o["predict_ksemi_samps"], trace, True, True, trace[-1] if trace else None,
                                   sig2_list=sig2_list, ell_list=ell_list, noisesq_list=noisesq_list,
                                   xvalid=xvalid, fvalid=fvalid, evalid=evalid)
        for k, v in zip(("ftest_eval", "etest_eval", "fgrid_eval", "egrid_eval", "fvalid_eval", "evalid_eval"), evals):
            times[k].append(v)
        if sharded:
            # the other ranks wait here while rank 0 runs the epoch callback (its own timeout:
            # dist_timeout_s when this fit initialised the group)
            import torch.distributed as dist
            dist.barrier(group=o["process_group"])

    report = pd.DataFrame(times, index=["epoch{}".format(i) for i in range(o["epochs"])])
    report.loc["Total"] = report.sum()
    print0("\n##############################\n")
    print0("Finish training and evaluating")
    print0("Time report")
    print0(report)
    if odir is not None and rank == 0:
        os.makedirs(odir, exist_ok=True)
        report.to_csv(os.path.join(odir, "time_report.csv"))
    return None
