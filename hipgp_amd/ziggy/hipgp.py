"""Toeplitz-whitened SVGP ("HIP-GP") models on the MI355X operators.

Mirrors the reference model API of `ziggy/hipgp.py` for the parts that sit on the hot path:
`ToeplitzInducingGP.compute_kn` (`hipgp.py:117-146`) and the mean-field
family's ELBO, natural gradient and prediction (`hipgp.py:160-276, 370-446, 449-524`,
SURVEY §8(f) row 3).  `Knm` comes from the fused grid kernel hgp_kuf_grid (SURVEY §8(f)
row 1, `hipgp_amd/kuf.py`).  `kn = R^T K^{-1} Knm^T` runs as one plan set-up + hgp_pcg_solve +
hgp_toeplitz_apply(R^T) on the device; the batch reductions are device tensor ops.

The natural-gradient statistics are split into per-RHS sums (`batch_stats`) and the update
built from them (`apply_stats`), so a caller that shards the minibatch over GPUs
(`hipgp_amd.dist`) all-reduces exactly those sums.

Line-integral observations come from the fused kernels of `hipgp_amd.kuf`.
The block-diagonal family's statistics (per-block grams, kn^T S kn) are the fused kernel
hgp_block_stats.

Kernel / noise hyper-parameter learning: with learn_kernel / learn_noise the
ELBO returned by `elbo_and_grad` carries the autograd graph through Knm, Knn and kn (InvMatmul's
backward PCG + hgp_plan_dqf, the R^T column gradient hgp_plan_column_grad), as the reference's
fit loop needs it (`svi_gp.py:317-326`).

`batch_solve` (`hipgp.py:278-368`, the full-batch solve of the mean-field family) is built:
one compute_kn per batch and the device statistics kernel, with the reference's
UnboundLocalError at `hipgp.py:314` fixed (parity pinned by the oracle restatement only).
Not built (OUT of the hot path): the full-rank variational family
(`FullRankToeplitzGP`, `hipgp.py:693-797`: a dense M' x M' covariance, 70 TB at C2).
"""
import numpy as np
import torch
from torch import nn

from hipgp_amd.ziggy.misc.toeplitz_tensor import ToeplitzTensor
from hipgp_amd.ziggy.svi_gp import SviGP

LN_2PI = float(np.log(2 * np.pi))


def diag_kl_to_standard(m, S):
    """KL(N(m, diag S) || N(0, I))  (`ziggy/misc/stats.py:4-8`)."""
    return 0.5 * (torch.sum(S) + torch.sum(m * m) - torch.sum(torch.log(S)) - m.shape[0])


def expanded_size(xgrids):
    """M' = prod(2 m_i - 2) (m_i > 1) else m_i  (`hipgp.py:72`)."""
    return int(np.prod([2 * len(g) - 2 if len(g) > 1 else len(g) for g in xgrids]))


class ToeplitzInducingGP(SviGP):
    """`hipgp.py:15-446` (hot-path subset)."""

    def __init__(self, kernel, xgrids, num_obs, sig2_init=1., ell_init=.05, noise2_init=1.,
                 learn_kernel=True, learn_noise=True, dtype=torch.float, whitened_type='ziggy',
                 parameterization='expectation-family', jitter_val=1e-3):
        super().__init__()
        assert len(xgrids) > 1, len(xgrids)
        self.learn_kernel = learn_kernel
        self.learn_noise = learn_noise
        self.jitter_val = jitter_val
        self.dtype = dtype
        self.kernel = kernel
        self.N = num_obs
        self.ell = torch.tensor(ell_init, dtype=dtype)
        self.sig2 = torch.tensor(sig2_init, dtype=dtype)
        self.noise2 = torch.tensor(noise2_init, dtype=dtype)
        self.log_ell = nn.Parameter(torch.log(self.ell.clone()), requires_grad=learn_kernel)
        self.log_sig2 = nn.Parameter(torch.log(self.sig2.clone()), requires_grad=learn_kernel)
        self.log_noise2 = nn.Parameter(torch.log(self.noise2.clone()), requires_grad=learn_noise)
        print(f"Model initialization: sig2 = {sig2_init:.2f}, ell_init = {ell_init:.2f}, noise2 = {noise2_init:.2f}")
        self.xgrids = xgrids
        mesh = torch.meshgrid(*xgrids, indexing="ij")
        self.xinduce = torch.stack([g.reshape(-1) for g in mesh], dim=-1)
        self.M = self.xinduce.shape[0]
        self.whitened_type = whitened_type
        if whitened_type == 'cholesky':
            self.Mprime = self.M
        else:
            assert whitened_type == 'ziggy', whitened_type
            self.Mprime = expanded_size(xgrids)
        self.parameterization = parameterization

    @property
    def name(self):
        raise NotImplementedError

    def cuda_params(self, cuda_num=0):
        """Move the model and its grids to `cuda:{cuda_num}` (`hipgp.py:80-90`)."""
        device = torch.device(f"cuda:{cuda_num}")
        self.to(device)
        self.xinduce = self.xinduce.to(device)
        self.kernel = self.kernel.to(device)
        self.xgrids = [g.to(device) for g in self.xgrids]
        return self

    def get_kernel_params(self):
        if not self.learn_kernel:
            return self.sig2, self.ell
        return torch.exp(self.log_sig2), torch.exp(self.log_ell)

    def update_kernel_params(self, sig2=None, ell=None):
        assert not self.learn_kernel
        if sig2 is not None:
            self.sig2 = torch.tensor(sig2, dtype=self.dtype, device=self.sig2.device)
        if ell is not None:
            self.ell = torch.tensor(ell, dtype=self.dtype, device=self.ell.device)

    def noise_terms(self, noise_std_batch):
        """(1/sigma_n^2, log sigma_n): per observation or from log_noise2 (`hipgp.py:227-230,394-399`)."""
        if noise_std_batch is not None:
            return (1 / noise_std_batch ** 2), torch.log(noise_std_batch)
        return torch.exp(-self.log_noise2), 0.5 * self.log_noise2

    # ---- the hot path ----------------------------------------------------------------------
    def toeplitz(self):
        """A fresh ToeplitzTensor for the current kernel parameters (`hipgp.py:142-143`)."""
        params = self.get_kernel_params()
        return ToeplitzTensor(xgrids=self.xgrids, kernel=lambda x, y: self.kernel(x, y, params=params),
                              batch_shape=None, jitter_val=self.jitter_val)

    def compute_kn(self, Knm, maxiter_cg=10, tol=1e-8, Kmm=None):
        """kn = R^T Kmm^{-1} Knm^T (ziggy whitening) or L^{-1} Knm^T (cholesky), (bsz, M')."""
        if self.whitened_type == 'cholesky':
            params = self.get_kernel_params()
            if Kmm is None:
                Kmm = self.kernel(self.xinduce, self.xinduce, params)
            eye = torch.eye(Kmm.shape[0], dtype=Knm.dtype, device=Knm.device)
            L = torch.linalg.cholesky(Kmm + self.jitter_val * eye)
            return torch.linalg.solve_triangular(L, Knm.t(), upper=False).t()
        if Kmm is None:
            Kmm = self.toeplitz()
        d0 = Kmm.inv_matmul(Knm, do_precond=True, maxiter=maxiter_cg, tol=tol)
        return Kmm._matmul_by_RT(d0)

    # ---- variational family hooks ------------------------------------------------------------
    def standard_variational_params(self):
        raise NotImplementedError

    def compute_knSkn(self, kn, qS):
        raise NotImplementedError

    def get_kl_to_prior(self, qm, qS):
        raise NotImplementedError

    # ---- ELBO --------------------------------------------------------------------------------
    def compute_batch_an(self, xbatch, ybatch, noise_std_batch=None, qm=None, qS=None, Knm=None,
                         Knn_diag=None, kn=None, maxiter_cg=10, integrated_obs=False,
                         semi_integrated_estimator=None, semi_integrated_samps=None,
                         cache_K_matmul=None, print_debug_info=False, Kmm=None):
        """a_n = -1/2 ln 2 pi s^2 - (mse + Knn - kn.kn + kn S kn) / 2 s^2  (`hipgp.py:370-414`)."""
        if qm is None or qS is None:
            qm, qS = self.standard_variational_params()
        if Knm is None or Knn_diag is None:
            Knm, Knn_diag = self._make_grams(xbatch, integrated_obs=integrated_obs,
                                             semi_integrated_estimator=semi_integrated_estimator or "analytic",
                                             semi_integrated_samps=semi_integrated_samps or 10)
        if kn is None:
            kn = self.compute_kn(Knm, maxiter_cg=maxiter_cg, Kmm=Kmm)
        ivar, log_sd = self.noise_terms(noise_std_batch)
        if noise_std_batch is not None:
            # reference shapes (hipgp.py:396-398): ivar squeezed, log(noise_std) kept (bsz, 1), so
            # with per-observation noise a_n broadcasts to (bsz, bsz); its mean is the ELBO term
            ivar = ivar.squeeze()
        mse = (kn.matmul(qm).squeeze() - ybatch.squeeze()) ** 2
        variance = Knn_diag.squeeze() - torch.sum(kn * kn, dim=-1).squeeze() + self.compute_knSkn(kn, qS)
        if print_debug_info:
            print("mse = {:.4f}".format(torch.mean(mse)))
            print("variance = {:.4f}".format(torch.mean(variance)))
        return -0.5 * ivar * (mse + variance) - log_sd - 0.5 * LN_2PI

    def elbo(self, xbatch, ybatch, noise_std_batch=None, maxiter_cg=10, integrated_obs=False,
             semi_integrated_estimator="analytic", semi_integrated_samps=10, Kmm=None,
             print_debug_info=False):
        """mean_n a_n - KL/N  (`hipgp.py:160-192`)."""
        Knm, Knn_diag = self._make_grams(xbatch, integrated_obs=integrated_obs,
                                         semi_integrated_estimator=semi_integrated_estimator,
                                         semi_integrated_samps=semi_integrated_samps)
        kn = self.compute_kn(Knm, maxiter_cg=maxiter_cg, Kmm=Kmm)
        qm, qS = self.standard_variational_params()
        an = self.compute_batch_an(xbatch, ybatch, noise_std_batch, qm=qm, qS=qS, Knm=Knm,
                                   Knn_diag=Knn_diag, kn=kn)
        return torch.mean(an) - self.get_kl_to_prior(qm, qS) / self.N

    def elbo_and_grad(self, xbatch, ybatch, noise_std_batch=None, maxiter_cg=10, integrated_obs=False,
                      semi_integrated_estimator="analytic", semi_integrated_samps=10,
                      print_debug_info=False, Kmm=None, mc_offset=None):
        """ELBO estimate; sets theta1.grad / theta2.grad to minus the natural gradient
        (`hipgp.py:194-276`).  mc_offset: see `SviGP._make_grams` (sharded fits)."""
        assert self.parameterization == 'expectation-family', \
            "need parameterization=expectation-family when performing natural gradient descent"
        Knm, Knn_diag = self._make_grams(xbatch, integrated_obs=integrated_obs,
                                         semi_integrated_estimator=semi_integrated_estimator,
                                         semi_integrated_samps=semi_integrated_samps, mc_offset=mc_offset)
        kn = self.compute_kn(Knm, maxiter_cg=maxiter_cg, Kmm=Kmm)
        stats = self.batch_stats(kn, ybatch, Knn_diag, noise_std_batch)
        elbo = self.apply_stats(stats, xbatch.shape[0])
        if self.hyper_grad_needed(noise_std_batch):
            # learn_kernel / learn_noise: the fit loop back-propagates the returned ELBO
            # (`svi_gp.py:317-326`), so it carries the graph to log_sig2 / log_ell / log_noise2
            # through Knm, Knn and kn (InvMatmul.backward + the R^T column gradient) as in
            # `hipgp.py:214-227`, with the variational parameters held fixed (`:216-217`)
            elbo = self.autograd_elbo(xbatch, ybatch, noise_std_batch, Knm, Knn_diag, kn)
        return elbo

    def batch_solve(self, xobs, yobs, noise_std=None, batch_size=-1, maxiter_cg=10, integrated_obs=False,
                    semi_integrated_estimator="analytic", semi_integrated_samps=10, compute_elbo=False,
                    Kmm=None, print_debug_info=False):
        """Closed-form variational parameters from all observations (`hipgp.py:278-368`):
           lam  = I_lam + sum_n ivar_n kn_n kn_n^T restricted to the family (diag / blocks),
           b    = sum_n ivar_n y_n kn_n,
           m    = (I + sum_n ivar_n kn_n kn_n^T)^{-1} b   (dense M' x M' solve),
           theta2 = -lam / 2, theta1 = lam m (mean-field) / blockdiag(lam) m (block);
        with compute_elbo the ELBO of the solved model over the same batches.

        kn per batch is the device compute_kn (one plan reused for every batch: the reference
        builds an identical ToeplitzTensor per call, `:294`).  The dense M' x M' system limits this
        to small grids (M' = 1444 on 20 x 20), as in the reference.  The reference reads
        `noise_std_batch` before assigning it (`:314`, UnboundLocalError on every call); here the
        intended rule holds: per-observation noise_std[bi] when given, else exp(-log_noise2)."""
        if xobs.shape[0] != self.N:
            print("x obs shape = {}, total_num_obs = {}".format(xobs.shape[0], self.N))
        if batch_size == -1:
            batch_size = xobs.shape[0]
        nb = int(np.ceil(len(xobs) / batch_size))
        batches = [slice(i * batch_size, min((i + 1) * batch_size, len(xobs))) for i in range(nb)]
        dev = self.xgrids[0].device
        if self.whitened_type == 'cholesky':
            Kmm = self.kernel(self.xinduce, self.xinduce, self.get_kernel_params())
        elif Kmm is None:
            Kmm = self.toeplitz()
        gram_kw = dict(integrated_obs=integrated_obs, semi_integrated_estimator=semi_integrated_estimator,
                       semi_integrated_samps=semi_integrated_samps)

        def noise_of(bi):
            return None if noise_std is None else noise_std[bi].to(dev)

        lam = self.get_identity_for_lam()
        b = 0
        big_lam = torch.eye(self.Mprime, dtype=self.dtype, device=dev)
        with torch.no_grad():
            for bi in batches:
                xb, yb = xobs[bi].to(dev), yobs[bi].to(dev)
                Knm, _ = self._make_grams(xb, **gram_kw)
                kn = self.compute_kn(Knm, maxiter_cg=maxiter_cg, Kmm=Kmm)
                sb = noise_of(bi)
                ivar = 1 / sb ** 2 if sb is not None else torch.exp(-self.log_noise2)
                lam = lam + self.get_lam(ivar_noise=ivar, kn=kn, bscale=1.0, add_identity=False)
                b = b + torch.sum(ivar * yb * kn, dim=0)
                big_lam += (ivar * kn).t().matmul(kn)
            mhat = torch.linalg.solve(big_lam, b[:, None])
            if self.parameterization == 'standard':
                self.global_S.data[:] = self.get_S_from_lam(lam)
                self.global_m.data[:] = mhat
            else:
                self.global_theta2.data[:] = -.5 * lam
                if self.name == 'mean-field':
                    self.global_theta1.data[:] = (mhat.squeeze() * lam.squeeze())[:, None]
                else:
                    self.global_theta1.data[:] = self.block_diag_multiply(lam, mhat.t()).t()
        if not compute_elbo:
            return None
        qm, qS = self.standard_variational_params()
        elbo = 0
        for bi in batches:
            an = self.compute_batch_an(xobs[bi].to(dev), yobs[bi].to(dev), noise_of(bi), qm=qm, qS=qS,
                                       maxiter_cg=maxiter_cg, Kmm=Kmm, print_debug_info=print_debug_info,
                                       **gram_kw)
            elbo += torch.sum(an)
        return elbo / xobs.shape[0] - self.get_kl_to_prior(qm, qS) / self.N

    def hyper_grad_needed(self, noise_std_batch=None):
        """True when the ELBO must carry an autograd graph to the kernel / noise parameters."""
        if not torch.is_grad_enabled():
            return False
        kern = self.learn_kernel and (self.log_sig2.requires_grad or self.log_ell.requires_grad)
        noise = noise_std_batch is None and self.log_noise2.requires_grad
        return bool(kern or noise)

    def autograd_elbo(self, xbatch, ybatch, noise_std_batch, Knm, Knn_diag, kn, nsum=None, bsz=None):
        """mean_n a_n - KL/N with autograd through Knm, Knn_diag, kn and the noise terms
        (`hipgp.py:214-227`); qm, qS fixed.  With nsum/bsz (a shard of a minibatch of bsz rows)
        the shard's share sum_n a_n / bsz is returned instead (no KL term)."""
        with torch.no_grad():
            qm, qS = self.standard_variational_params()
            qm, qS = qm.detach(), qS.detach()
        an = self.compute_batch_an(xbatch, ybatch, noise_std_batch, qm=qm, qS=qS, Knm=Knm,
                                   Knn_diag=Knn_diag, kn=kn)
        if bsz is not None:
            # a_n may be the reference's (n, n) broadcast (per-observation noise): its mean
            # equals the mean of the per-row values, so mean * n is the shard's sum
            return torch.mean(an) * nsum / bsz
        return torch.mean(an) - self.get_kl_to_prior(qm, qS) / self.N

    def predict(self, x, integrated_obs=False, semi_integrated_estimator="analytic",
                semi_integrated_samps=10, maxiter_cg=50, Kmm=None):
        """E[f(x)] and sd[f(x)] (`hipgp.py:416-446`), returned on the CPU."""
        x = x.to(self.xgrids[0].device)
        Knm, Knn_diag = self._make_grams(x, integrated_obs=integrated_obs,
                                         semi_integrated_estimator=semi_integrated_estimator,
                                         semi_integrated_samps=semi_integrated_samps)
        kn = self.compute_kn(Knm, maxiter_cg=maxiter_cg, Kmm=Kmm)
        qm, qS = self.standard_variational_params()
        mu = kn.matmul(qm)
        ktilde = (Knn_diag - torch.sum(kn * kn, dim=-1)).clamp_min(1e-5)
        sig = torch.sqrt(ktilde + self.compute_knSkn(kn, qS))[:, None]
        return mu.cpu().detach(), sig.cpu().detach()


class MeanFieldToeplitzGP(ToeplitzInducingGP):
    """Diagonal variational covariance in the expanded space (`hipgp.py:449-524`)."""

    def __init__(self, kernel, xgrids, num_obs, sig2_init=1., ell_init=.05, noise2_init=1.,
                 init_Svar=.1, learn_kernel=False, learn_noise=False, dtype=torch.float,
                 whitened_type='ziggy', parameterization='expectation-family', jitter_val=1e-3):
        super().__init__(kernel, xgrids, num_obs, sig2_init=sig2_init, ell_init=ell_init,
                         noise2_init=noise2_init, learn_kernel=learn_kernel, learn_noise=learn_noise,
                         dtype=dtype, whitened_type=whitened_type, parameterization=parameterization,
                         jitter_val=jitter_val)
        col = lambda: torch.zeros(self.Mprime, 1, dtype=dtype)
        if parameterization == 'standard':
            self.global_m = nn.Parameter(nn.init.xavier_normal_(col()), requires_grad=True)
            self.global_S = nn.Parameter(init_Svar * torch.ones(self.Mprime, 1, dtype=dtype), requires_grad=True)
        else:
            self.global_theta1 = nn.Parameter(nn.init.xavier_normal_(col()), requires_grad=True)
            self.global_theta2 = nn.Parameter((-.5 / init_Svar) * torch.ones(self.Mprime, 1, dtype=dtype),
                                              requires_grad=True)

    @property
    def name(self):
        return 'mean-field'

    def standard_variational_params(self):
        if self.parameterization == 'standard':
            return self.global_m, self.global_S
        S = -0.5 / self.global_theta2
        return S * self.global_theta1, S

    def get_kl_to_prior(self, qm=None, qS=None):
        if qm is None or qS is None:
            qm, qS = self.standard_variational_params()
        return diag_kl_to_standard(qm, qS)

    def get_identity_for_lam(self):
        return 1

    def get_lam(self, ivar_noise, kn, bscale=1, add_identity=True):
        return (bscale * torch.sum(ivar_noise * kn * kn, dim=0) + (1 if add_identity else 0))[:, None]

    def get_S_from_lam(self, lam):
        return 1. / lam

    def compute_knSkn(self, kn, qS):
        return torch.sum(kn * kn * qS.t(), dim=-1).squeeze()

    # ---- natural gradient as batch sums + update (sharding-friendly) ------------------------
    def batch_stats(self, kn, ybatch, Knn_diag, noise_std_batch=None):
        """Sums over this minibatch (or this rank's shard of it):
           an_sum  = sum_n a_n
           lam_sum = sum_n ivar_n kn_n^2            (M',)   `hipgp.py:241`
           dm_sum  = -sum_n ivar_n (kn_n.m - y_n) kn_n   (M',)   `hipgp.py:234-236`"""
        if kn.shape[0] == 0:    # an empty shard of a minibatch (hipgp_amd.dist)
            z = kn.new_zeros(kn.shape[1])
            return {"an_sum": kn.new_zeros(()), "lam_sum": z, "dm_sum": z.clone(), "n": 0}
        with torch.no_grad():
            qm, qS = self.standard_variational_params()
            ivar, log_sd = self.noise_terms(noise_std_batch)
            if kn.is_cuda:      # the device path: two streaming passes of hgp_meanfield_stats
                return self._batch_stats_device(kn, ybatch, Knn_diag, qm, qS, ivar, log_sd)
            # CPU tensors only reach here in the gloo host-logic tests (tests/test_model_cpu.py)
            y = ybatch.reshape(-1)
            knm = kn.matmul(qm).reshape(-1)
            kk = kn * kn
            knkn = kk.sum(dim=-1)
            knSkn = kk.matmul(qS).reshape(-1)
            iv = ivar.reshape(-1) if torch.is_tensor(ivar) and ivar.dim() > 0 else ivar
            lsd = log_sd.reshape(-1) if torch.is_tensor(log_sd) and log_sd.dim() > 0 else log_sd
            an = -0.5 * iv * ((knm - y) ** 2 + Knn_diag.reshape(-1) - knkn + knSkn) - lsd - 0.5 * LN_2PI
            ivcol = iv[:, None] if torch.is_tensor(iv) and iv.dim() > 0 else iv
            lam_sum = torch.sum(ivcol * kk, dim=0)
            bdiff = iv * (knm - y)
            dm_sum = -(bdiff[None, :].matmul(kn)).reshape(-1)
            an_sum = an.sum()
        return {"an_sum": an_sum, "lam_sum": lam_sum, "dm_sum": dm_sum, "n": kn.shape[0]}

    def _batch_stats_device(self, kn, ybatch, Knn_diag, qm, qS, ivar, log_sd):
        import ctypes
        from hipgp_amd import _lib
        B, Mp = kn.shape
        dev, dt = kn.device, kn.dtype
        col = lambda v: torch.as_tensor(v, dtype=dt, device=dev).reshape(-1).expand(B).contiguous()
        knc = kn.detach().contiguous()
        qmv = qm.detach().reshape(-1).to(dt).contiguous()
        qSv = qS.detach().reshape(-1).to(dt).contiguous()
        y, iv, kd, lsd = col(ybatch), col(ivar), col(Knn_diag), col(log_sd)
        an = torch.empty(B, dtype=dt, device=dev)
        lam = torch.empty(Mp, dtype=dt, device=dev)
        dm = torch.empty(Mp, dtype=dt, device=dev)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        _lib.check(_lib.lib().hgp_meanfield_stats(_lib.dtype_code(dt), p(knc), B, Mp, p(qmv), p(qSv), p(y), p(iv),
                                                  p(kd), p(lsd), p(an), p(lam), p(dm), _lib.stream_ptr(dev)))
        return {"an_sum": an.sum(), "lam_sum": lam, "dm_sum": dm, "n": B}

    def batch_stats_slab(self, kn, j0, ybatch, Knn_diag, noise_std_batch=None, reduce=None, lead=True):
        """`batch_stats` of a minibatch whose kn is held in column slabs over ranks (grid-block
        sharding, `hipgp_amd.slab.SlabFit`): kn (B, w) are this rank's expanded-grid columns
        [j0, j0 + w).  The per-observation dots kn.qm, |kn|^2 and kn^2.qS are sums over the
        slabs: this rank's partials (hgp_meanfield_rowdots) go through `reduce` (an in-place SUM
        all-reduce of the (B, 3) tensor, B values per dot), then a_n and the slab's columns of
        lam_sum / dm_sum follow as in `batch_stats` (hgp_meanfield_cols), written into zero
        M'-vectors: summed over the ranks (allreduce_stats) they give the single-process sums.
        an_sum and n are counted on the `lead` rank only, so that sum is not multiplied."""
        B, w = kn.shape
        Mp = self.Mprime
        with torch.no_grad():
            qm, qS = self.standard_variational_params()
            ivar, log_sd = self.noise_terms(noise_std_batch)
            dev, dt = kn.device, kn.dtype
            col = lambda v: torch.as_tensor(v, dtype=dt, device=dev).reshape(-1).expand(B).contiguous()
            qmv = qm.detach().reshape(-1)[j0:j0 + w].to(dt).contiguous()
            qSv = qS.detach().reshape(-1)[j0:j0 + w].to(dt).contiguous()
            knc = kn.detach().contiguous()
            y, iv, kd, lsd = col(ybatch), col(ivar), col(Knn_diag), col(log_sd)
            if kn.is_cuda:
                import ctypes
                from hipgp_amd import _lib
                p = lambda t: ctypes.c_void_p(t.data_ptr())
                dots = torch.zeros((B, 3), dtype=dt, device=dev)
                _lib.check(_lib.lib().hgp_meanfield_rowdots(_lib.dtype_code(dt), p(knc), B, w, p(qmv), p(qSv), p(dots),
                                                            _lib.stream_ptr(dev)))
            else:       # CPU tensors only in the gloo host-logic tests
                kk = knc * knc
                dots = torch.stack([knc.matmul(qmv), kk.sum(-1), kk.matmul(qSv)], dim=1).contiguous()
            if reduce is not None:
                reduce(dots)
            knm, knkn, knSkn = dots[:, 0], dots[:, 1], dots[:, 2]
            an = -0.5 * iv * ((knm - y) ** 2 + kd - knkn + knSkn) - lsd - 0.5 * LN_2PI
            bdiff = (iv * (knm - y)).contiguous()
            lam = torch.zeros(Mp, dtype=dt, device=dev)
            dm = torch.zeros(Mp, dtype=dt, device=dev)
            if kn.is_cuda:
                ls, ds = lam[j0:j0 + w], dm[j0:j0 + w]
                _lib.check(_lib.lib().hgp_meanfield_cols(_lib.dtype_code(dt), p(knc), B, w, p(iv), p(bdiff), p(ls), p(ds),
                                                         _lib.stream_ptr(dev)))
            else:
                lam[j0:j0 + w] = torch.sum(iv[:, None] * knc * knc, dim=0)
                dm[j0:j0 + w] = -(bdiff[None, :].matmul(knc)).reshape(-1)
            an_sum = an.sum() if lead else an.new_zeros(())
        return {"an_sum": an_sum, "lam_sum": lam, "dm_sum": dm, "n": B if lead else 0}

    def apply_stats(self, stats, bsz):
        """ELBO estimate and theta grads from (all-reduced) batch sums of `bsz` observations."""
        qm, qS = self.standard_variational_params()
        with torch.no_grad():
            qm, qS = qm.detach(), qS.detach()
            bscale = self.N / bsz
            elbo = stats["an_sum"] / bsz - self.get_kl_to_prior(qm, qS) / self.N
            dm = bscale * stats["dm_sum"][:, None] - qm
            lam_diag = bscale * stats["lam_sum"] + 1
            dS = -.5 * lam_diag[:, None] - self.global_theta2.data
            deta1 = dm + dS * (-2 * qm)
        self.global_theta1.grad = -deta1
        self.global_theta2.grad = -dS
        return elbo


# ---- block-diagonal variational family -------------------------------------------------------
def block_chunks(dims, chunk_sizes):
    """Block ordering of a 2-D / 3-D grid (`ziggy/misc/util.py:79-130`, define_block_chunks):
    blocks C-order over the block grid, points C-order inside a block.  Returns
    (block_idx (num_blocks, block_size) int64 on the CPU, to_blocks, from_blocks); the two maps are
    reshape/permute views (no gather table on the device)."""
    dims, chunks = [int(d) for d in dims], [int(c) for c in chunk_sizes]
    assert len(dims) == len(chunks), "xgrids ndim = {}, chunk_sizes ndim = {}".format(len(dims), len(chunks))
    assert len(dims) in (2, 3), "only 2d or 3d inputs"
    for d, (n, c) in enumerate(zip(dims, chunks)):
        assert n % c == 0, "xgrid-{}={} not divis by chunk_size={}".format(d, n, c)
    nd = len(dims)
    split = []
    for n, c in zip(dims, chunks):
        split += [n // c, c]
    perm = [2 * a for a in range(nd)] + [2 * a + 1 for a in range(nd)]
    inv = [perm.index(a) for a in range(2 * nd)]
    nblk, bs = int(np.prod([n // c for n, c in zip(dims, chunks)])), int(np.prod(chunks))

    def to_blocks(m):
        lead = m.shape[:-1]
        t = m.reshape(*lead, *split).permute(*range(len(lead)), *[len(lead) + p for p in perm])
        return t.reshape(*lead, nblk, bs)

    def from_blocks(block_m):
        b = block_m.shape[0]
        t = block_m.reshape(b, *[split[p] for p in perm]).permute(0, *[1 + p for p in inv])
        return t.reshape(b, -1)

    block_idx = to_blocks(torch.arange(int(np.prod(dims))))
    return block_idx, to_blocks, from_blocks


def block_kl_to_standard(blk_m, blk_S):
    """KL(N(m, blockdiag S) || N(0, I)) with a 1e-4 nugget in the log det (`ziggy/misc/stats.py:15-29`)."""
    eye = torch.eye(blk_S.shape[1], dtype=blk_S.dtype, device=blk_S.device)
    L = torch.linalg.cholesky(blk_S + 1e-4 * eye)
    lndet = 2.0 * torch.sum(torch.log(torch.diagonal(L, dim1=-2, dim2=-1)))
    n_blk, blk_size, _ = blk_S.shape
    Strace = torch.sum(torch.diagonal(blk_S, dim1=-2, dim2=-1))
    return .5 * (Strace + torch.sum(blk_m * blk_m) - lndet - n_blk * blk_size)


class BlockToeplitzGP(ToeplitzInducingGP):
    """Block-diagonal variational covariance over neighbouring points of the (expanded) grid
    (`hipgp.py:527-691`).  qm lives in grid order, qS / theta2 in block order
    (num_blocks, block_size, block_size).  On the device the per-block statistics are one fused
    kernel (hgp_block_stats): sum_n ivar_n kn_blk kn_blk^T and kn^T S kn in a single read of kn."""

    def __init__(self, kernel, xgrids, num_obs, xblock_size=10, block_sizes=None, sig2_init=1., ell_init=.05,
                 noise2_init=1., init_Svar=.1, learn_kernel=False, learn_noise=False, dtype=torch.float,
                 whitened_type='ziggy', parameterization='expectation-family', jitter_val=1e-3):
        super().__init__(kernel, xgrids, num_obs, sig2_init=sig2_init, ell_init=ell_init,
                         noise2_init=noise2_init, learn_kernel=learn_kernel, learn_noise=learn_noise,
                         dtype=dtype, whitened_type=whitened_type, parameterization=parameterization,
                         jitter_val=jitter_val)
        input_dim = len(xgrids)
        if block_sizes is not None:
            assert input_dim == len(block_sizes), "xgrids ndim = {}, block ndim = {}".format(input_dim, len(block_sizes))
        else:
            block_sizes = [xblock_size for _ in range(input_dim)]
        if self.whitened_type == 'cholesky':
            self.block_dims = [len(x) for x in xgrids]
        else:      # blocks of the expanded grid arange(2m - 2)  (hipgp.py:599-601, 629-634)
            self.block_dims = [2 * len(x) - 2 for x in xgrids]
        self.block_sides = [int(b) for b in block_sizes]
        self.block_idx, self.to_blocks, self.from_blocks = block_chunks(self.block_dims, self.block_sides)
        self.num_blocks, self.block_size = self.block_idx.shape
        eye = torch.eye(self.block_size, dtype=dtype)
        col = lambda: torch.zeros(self.Mprime, 1, dtype=dtype)
        if parameterization == 'standard':
            self.global_m = nn.Parameter(nn.init.xavier_normal_(col()), requires_grad=True)
            self.global_S = nn.Parameter((init_Svar * eye)[None].repeat(self.num_blocks, 1, 1), requires_grad=True)
        else:
            self.global_theta1 = nn.Parameter(nn.init.xavier_normal_(col()), requires_grad=True)
            self.global_theta2 = nn.Parameter(((-.5 / init_Svar) * eye)[None].repeat(self.num_blocks, 1, 1),
                                              requires_grad=True)

    @property
    def name(self):
        return 'block'

    def get_expanded_xgrids(self, xgrids):
        return [torch.arange(2 * len(x) - 2) for x in xgrids]

    def standard_variational_params(self):
        if self.parameterization == 'standard':
            return self.global_m, self.global_S
        S = torch.inverse(-2 * self.global_theta2)                      # block inverse
        m = self.block_diag_multiply(S, self.global_theta1.t()).t()
        return m, S

    def block_diag_multiply(self, S_block, v):
        """rows of v (bsz, M') times the block-diagonal S (num_blocks, bs, bs)  (`hipgp.py:645-656`)."""
        Sv_block = S_block.matmul(self.to_blocks(v)[..., None])
        return self.from_blocks(Sv_block)

    def get_S_from_lam(self, lam):
        return torch.inverse(lam)

    def _block_kernel(self, kn, ivar=None, S=None, gram=True, knSkn=True, trace=False):
        import ctypes
        from hipgp_amd import _lib
        B, Mp = kn.shape
        dev, dt = kn.device, kn.dtype
        nd = len(self.block_dims)
        dims = (ctypes.c_int64 * nd)(*self.block_dims)
        blks = (ctypes.c_int64 * nd)(*self.block_sides)
        knc = kn.detach().contiguous()
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        ivv = None if ivar is None else torch.as_tensor(ivar, dtype=dt, device=dev).reshape(-1).expand(B).contiguous()
        Sc = None if S is None else S.detach().to(dt).contiguous()
        G = torch.empty(self.num_blocks, self.block_size, self.block_size, dtype=dt, device=dev) if gram else None
        q = torch.empty(B, dtype=dt, device=dev) if knSkn else None
        tr = torch.empty((), dtype=dt, device=dev) if trace else None
        _lib.check(_lib.lib().hgp_block_stats(_lib.dtype_code(dt), nd, dims, blks, p(knc), B, p(ivv), p(Sc),
                                              p(G), p(q), p(tr), _lib.stream_ptr(dev)))
        return (G, q, tr) if trace else (G, q)

    def compute_knSkn(self, kn, qS):
        """kn_n^T S kn_n per row (`hipgp.py:661-664`)."""
        if kn.is_cuda and not (torch.is_grad_enabled() and (kn.requires_grad or qS.requires_grad)):
            return self._block_kernel(kn, S=qS, gram=False)[1].squeeze()
        Skn = self.block_diag_multiply(qS, kn)
        return torch.sum(kn * Skn, dim=-1).squeeze()

    def get_identity_for_lam(self):
        return torch.eye(self.block_size, device=self.xgrids[0].device, dtype=self.dtype)

    def get_lam(self, ivar_noise, kn, bscale=1, add_identity=True):
        """bscale sum_n ivar_n kn_blk kn_blk^T (+ I), (num_blocks, bs, bs)  (`hipgp.py:669-685`)."""
        if kn.is_cuda:
            G = self._block_kernel(kn, ivar=ivar_noise, knSkn=False)[0]
        else:
            blk_kn = self.to_blocks(kn).transpose(0, 1)
            G = torch.matmul(blk_kn.transpose(1, 2), ivar_noise * blk_kn)
        return bscale * G + (self.get_identity_for_lam() if add_identity else 0)

    def get_kl_to_prior(self, qm=None, qS=None):
        if qm is None or qS is None:
            qm, qS = self.standard_variational_params()
        return block_kl_to_standard(qm, qS)

    # ---- natural gradient as batch sums + update (sharding-friendly) ------------------------
    def batch_stats(self, kn, ybatch, Knn_diag, noise_std_batch=None):
        """Sums over this minibatch (or this rank's shard of it):
           an_sum  = sum_n a_n                                         `hipgp.py:370-414`
           lam_sum = sum_n ivar_n kn_blk kn_blk^T   (num_blocks, bs, bs)  `hipgp.py:252-256`
           dm_sum  = -sum_n ivar_n (kn_n.m - y_n) kn_n   (M',)          `hipgp.py:234-236`"""
        if kn.shape[0] == 0:    # an empty shard of a minibatch (hipgp_amd.dist)
            G = kn.new_zeros((self.num_blocks, self.block_size, self.block_size))
            return {"an_sum": kn.new_zeros(()), "lam_sum": G, "dm_sum": kn.new_zeros(kn.shape[1]), "n": 0}
        with torch.no_grad():
            qm, qS = self.standard_variational_params()
            qm, qS = qm.detach(), qS.detach()
            ivar, log_sd = self.noise_terms(noise_std_batch)
            B = kn.shape[0]
            if kn.is_cuda:
                import ctypes
                from hipgp_amd import _lib
                dev, dt = kn.device, kn.dtype
                colv = lambda v: torch.as_tensor(v, dtype=dt, device=dev).reshape(-1).expand(B).contiguous()
                # per-block grams and sum_n ivar_n kn_n^T S kn_n = sum_blk <S, G>_F in one read of kn
                G, _, trSG = self._block_kernel(kn, ivar=ivar, S=qS, knSkn=False, trace=True)
                # a_n without the kn S kn term and dm from the streaming row/column passes
                knc = kn.detach().contiguous()
                zero = torch.zeros(kn.shape[1], dtype=dt, device=dev)
                qmv = qm.reshape(-1).to(dt).contiguous()
                y, iv, kd, lsd = colv(ybatch), colv(ivar), colv(Knn_diag), colv(log_sd)
                an = torch.empty(B, dtype=dt, device=dev)
                lam_diag = torch.empty(kn.shape[1], dtype=dt, device=dev)
                dm = torch.empty(kn.shape[1], dtype=dt, device=dev)
                p = lambda t: ctypes.c_void_p(t.data_ptr())
                _lib.check(_lib.lib().hgp_meanfield_stats(_lib.dtype_code(dt), p(knc), B, kn.shape[1], p(qmv),
                                                          p(zero), p(y), p(iv), p(kd), p(lsd), p(an), p(lam_diag),
                                                          p(dm), _lib.stream_ptr(dev)))
                return {"an_sum": an.sum() - 0.5 * trSG, "lam_sum": G, "dm_sum": dm, "n": B}
            # CPU tensors only reach here in the gloo host-logic tests
            y = ybatch.reshape(-1)
            knm = kn.matmul(qm).reshape(-1)
            knSkn = torch.sum(kn * self.block_diag_multiply(qS, kn), dim=-1)
            iv = torch.as_tensor(ivar, dtype=kn.dtype).reshape(-1).expand(B)
            lsd = torch.as_tensor(log_sd, dtype=kn.dtype).reshape(-1).expand(B)
            an = -0.5 * iv * ((knm - y) ** 2 + Knn_diag.reshape(-1) - (kn * kn).sum(-1) + knSkn) - lsd - 0.5 * LN_2PI
            blk_kn = self.to_blocks(kn).transpose(0, 1)                     # (nblk, B, bs)
            G = torch.matmul(blk_kn.transpose(1, 2), iv[None, :, None] * blk_kn)
            dm_sum = -((iv * (knm - y))[None, :].matmul(kn)).reshape(-1)
        return {"an_sum": an.sum(), "lam_sum": G, "dm_sum": dm_sum, "n": B}

    def apply_stats(self, stats, bsz):
        """ELBO estimate and theta grads from (all-reduced) batch sums of `bsz` observations
        (`hipgp.py:222-276`, 'block' branch)."""
        qm, qS = self.standard_variational_params()
        with torch.no_grad():
            qm, qS = qm.detach(), qS.detach()
            bscale = self.N / bsz
            elbo = stats["an_sum"] / bsz - self.get_kl_to_prior(qm, qS) / self.N
            dm = bscale * stats["dm_sum"][:, None] - qm
            lam_block = bscale * stats["lam_sum"] + self.get_identity_for_lam().to(qm.device)
            dS = -.5 * lam_block - self.global_theta2.data
            dSdeta1 = self.block_diag_multiply(dS, -2 * qm[None, :, 0])
            deta1 = dm + dSdeta1.squeeze().unsqueeze(-1)
        self.global_theta1.grad = -deta1
        self.global_theta2.grad = -dS
        return elbo
