"""CPU ORACLE for the HIP-GP structured-kernel PCG hot path — TEST INFRASTRUCTURE ONLY.

This module restates, in NumPy/SciPy, the reference algorithm of `suyashk12/hipgp`
(package `ziggy`, snapshot mounted at /root/reference).  It is the checker that the HIP
path is compared against; it is imported only by `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg.  The product path (`hipgp_amd`, `ziggy`) never imports it.

Parity pinning: every function below is checked against golden vectors produced by running
the reference itself (tests/golden/make_golden.py -> tests/golden/*.npz) in
tests/test_oracle.py.  FFT boundary: the reference calls torch-1.4 `torch.fft/ifft`
(unnormalised forward / 1/N inverse C2C); here `scipy.fft.fftn/ifftn` with the same
definition, computed in the input precision (complex64 for fp32, complex128 for fp64).
"""
import numpy as np
import scipy.fft as sfft

_WORKERS = -1   # all host cores for scipy.fft (bench cpu_baseline states the core count)


def set_workers(n):
    global _WORKERS
    _WORKERS = n


# --------------------------------------------------------------------------------------
# kernels (ziggy/kernels.py)
# --------------------------------------------------------------------------------------
def kernel_eval(kind, x, y, params, nu=None):
    """Stationary kernel k(x, y) for x:(N,D), y:(M,D) -> (N,M).
    SqExp: `kernels.py:73-79`; Matern nu in {.5,1.5,2.5}: `kernels.py:145-158`."""
    sig2, ell = params
    x = np.asarray(x)
    y = np.asarray(y)
    if kind == "sqexp":
        sq = np.sum(((x[:, None, :] - y[None, :, :]) / ell) ** 2, axis=-1)
        return sig2 * np.exp(-sq / 2)
    if kind == "matern":
        sq = np.sum((x[:, None, :] - y[None, :, :]) ** 2, axis=-1)
        if nu == .5:
            k = np.exp(-np.sqrt(sq) / ell)
        elif nu == 1.5:
            dp = np.sqrt(3) * np.sqrt(sq) / ell
            k = (1 + dp) * np.exp(-dp)
        elif nu == 2.5:
            dp = np.sqrt(5) * np.sqrt(sq) / ell
            k = (1 + dp + (5. / 3.) * sq / (ell ** 2)) * np.exp(-dp)
        else:
            raise ValueError(nu)
        return (sig2 * k).astype(x.dtype)
    if kind == "gneiting":          # `kernels.py:108-117` (alpha = nu argument)
        alpha = 1. if nu is None else nu
        t = np.sqrt(np.sum(((x[:, None, :] - y[None, :, :]) / ell) ** 2, axis=-1))
        c = (1 - t) * np.cos(np.pi * t) + (1 / np.pi) * np.sin(np.pi * t)
        c = (1 + t ** alpha) ** (-3) * c
        c[t > 1.] = 0.
        return (sig2 * c).astype(x.dtype)
    raise ValueError(kind)


# --------------------------------------------------------------------------------------
# line-integral (semi-integrated) cross covariance, SURVEY §8(f) row 2
# --------------------------------------------------------------------------------------
def k_semi_mc(kind, xinduce, xint, params, npts, u, nu=None):
    """`Kernel.k_semi_mc` `kernels.py:19-39`, transposed as `svi_gp._make_grams` uses it
    (`svi_gp.py:61-64`): Knm[n, m] = |x_n| * mean_j k(u_m, alpha_j x_n),
    alpha_j = j/npts + u/npts with u the single torch.rand(1) draw (passed explicitly)."""
    dt = xint.dtype
    alphas = np.arange(npts, dtype=dt) / dt.type(npts) + dt.type(u) * dt.type(1. / npts)
    xg = (xint[:, None, :] * alphas[None, :, None]).reshape(-1, xint.shape[1])
    K = kernel_eval(kind, xinduce, xg, params, nu=nu).reshape(xinduce.shape[0], xint.shape[0], npts)
    dists = np.sqrt(np.sum(xint ** 2, axis=-1))
    return (np.mean(K, axis=-1) * dists[None, :]).T.astype(dt)


def _normal_cdf(x, loc, scale):      # `ziggy/misc/stats.py:74-76`
    from scipy.special import erf
    return .5 * (1. + erf((x - loc) / (scale * np.sqrt(2))))


def k_semi_sqexp(xinduce, xint, params):
    """`SqExp.k_semi` `kernels.py:80-85` -> `semi_integrated_sqe` `kernels.py:223-237`
    (integral of k(u, a x) over a in [0, 1] times |x|), returned as (nobs, M)."""
    sig2, ell = params
    dt = xint.dtype
    D = xint.shape[1]
    Sinv = (1. / (ell ** 2)) * np.eye(D, dtype=dt)
    xdists = np.sqrt(np.sum(xint * xint, axis=-1))
    xi_S = xint @ Sinv
    a = np.sum(xi_S * xint, axis=-1)
    b = xi_S @ xinduce.T
    c = np.sum((xinduce @ Sinv) * xinduce, axis=-1)
    scale = np.sqrt(1 / a[:, None])
    loc = b / a[:, None]
    coef = sig2 * np.exp((b ** 2) / (2 * a[:, None]) - c[None, :] / 2) * np.sqrt(2 * np.pi) * scale
    return (coef * (_normal_cdf(1, loc, scale) - _normal_cdf(0, loc, scale)) * xdists[:, None]).astype(dt)


def doubly_diag_table(kind, N=50, dmax=5., nu=None):
    """`KernelDoublyDiagInterpolator.__init__` `kernels.py:172-198`: knn(d) = |x|^2 *
    int_0^1 int_0^1 k(a x, a' x) da da' at x = (d, 0), kernel params (1, 1), by the same
    scipy dblquad tolerances as `doubly_integrated_diag` `kernels.py:266-289`; stored as
    float32 (`torch.Tensor(...)`) before the cast to the model dtype, as the reference."""
    from scipy import integrate
    dgrid = np.linspace(0, dmax, N)
    knn = np.zeros(N)
    for n, d in enumerate(dgrid):
        xn = np.array([d, 0.])
        f = lambda a, ap: float(kernel_eval(kind, (a * xn)[None, :], (ap * xn)[None, :], (1., 1.), nu=nu)[0, 0])
        res = integrate.dblquad(f, a=0, b=1, gfun=lambda a: 0, hfun=lambda b: 1, epsrel=1.49e-5, epsabs=1.49e-1)
        knn[n] = res[0] * d * d
    slopes = (knn[1:] - knn[:-1]) / (dgrid[1:] - dgrid[:-1])
    slopes = np.concatenate([slopes, [slopes[-1]]])
    f32 = lambda v: np.asarray(v, dtype=np.float32)
    return f32(dgrid), f32(knn), f32(slopes)


def doubly_diag(x, params, table):
    """`KernelDoublyDiagInterpolator.forward` `kernels.py:200-220` (linear interpolation in
    |x/ell|; an index of -1 (|x| = 0) wraps to the last entry, as torch indexing does)."""
    sig2, ell = params
    grid, knn, slopes = (np.asarray(t, dtype=x.dtype) for t in table)
    d = np.sqrt(np.sum((x / ell) ** 2, axis=-1))
    lo = np.sum(d[:, None] > grid[None, :], axis=-1) - 1
    iv = knn[lo] + slopes[lo] * (d - grid[lo])
    return (ell * ell * sig2 * iv).astype(x.dtype)


def grid_points(grids):
    """C-order meshgrid(indexing='ij') points, last axis fastest (`hipgp.py:63-64`)."""
    mesh = np.meshgrid(*grids, indexing="ij")
    return np.stack([g.reshape(-1) for g in mesh], axis=-1)


# --------------------------------------------------------------------------------------
# ToeplitzTensor (ziggy/misc/toeplitz_tensor.py)
# --------------------------------------------------------------------------------------
def toeplitz_column(grids, kfun, jitter):
    """`toeplitz_tensor.py:127-133`: first row k(x0, x_j), nugget on c0 (absent in
    `toeplitz_expanded.py:242-250`, i.e. jitter=0)."""
    xs = grid_points(grids)
    row = np.array(kfun(xs[0][None, :], xs))[0].copy()
    row[0] += jitter
    return row


def expanded_dims(dims):
    """n_i = 2 m_i - 2 (m_i > 1) else m_i  (`hipgp.py:72`)."""
    return tuple(2 * m - 2 if m > 1 else m for m in dims)


def circulant_embed(K):
    """`toeplitz_tensor.py:135-143`: per dim cat([K, flip(K)[1:-1]])."""
    for d in range(K.ndim):
        rev = np.flip(K, axis=d)
        idx = [slice(None)] * d + [slice(1, -1)]
        K = np.concatenate([K, rev[tuple(idx)]], axis=d)
    return K


def _cdtype(dt):
    return np.complex64 if np.dtype(dt) == np.float32 else np.complex128


class ToeplitzOracle:
    """Restatement of `ToeplitzTensor.__init__` (`toeplitz_tensor.py:9-45`) and its ops."""

    def __init__(self, column, dims, clamp_min=1e-6):
        self.dims = tuple(int(m) for m in dims)
        self.ndim = len(self.dims)
        self.M = int(np.prod(self.dims))
        self.dtype = np.asarray(column).dtype
        self.column = np.asarray(column)
        self.C = circulant_embed(self.column.reshape(self.dims))
        self.ndims = self.C.shape
        self.Mp = int(np.prod(self.ndims))
        F = sfft.fftn(self.C.astype(_cdtype(self.dtype)), workers=_WORKERS)
        # D = clamp(Re FFT(C), 1e-6); imag discarded (`toeplitz_tensor.py:25-31`)
        self.D = np.maximum(F.real, self.dtype.type(clamp_min)).astype(self.dtype)
        self.D_sqrt = np.sqrt(self.D)
        self.Di = (1. / self.D).astype(self.dtype)

    def _apply(self, spec, x_full):
        ax = tuple(range(1, self.ndim + 1))
        Fv = sfft.fftn(x_full, axes=ax, workers=_WORKERS)
        return sfft.ifftn(Fv * spec[None], axes=ax, workers=_WORKERS)

    def _pad(self, v):
        B = v.shape[0]
        c = np.zeros((B,) + self.ndims, dtype=_cdtype(self.dtype))
        c[(slice(None),) + tuple(slice(0, m) for m in self.dims)] = v.reshape((B,) + self.dims)
        return c

    def _crop(self, c):
        B = c.shape[0]
        return np.ascontiguousarray(
            c[(slice(None),) + tuple(slice(0, m) for m in self.dims)].real).reshape(B, -1)

    def matmul_K(self, v):           # `toeplitz_tensor.py:70-83`
        return self._crop(self._apply(self.D, self._pad(v))).astype(self.dtype)

    def matmul_Cinv(self, v):        # `toeplitz_tensor.py:114-125`
        return self._crop(self._apply(self.Di, self._pad(v))).astype(self.dtype)

    def matmul_RT(self, v):          # `toeplitz_tensor.py:85-97` (full expanded grid, no crop)
        B = v.shape[0]
        return self._apply(self.D_sqrt, self._pad(v)).real.reshape(B, -1).astype(self.dtype)

    def matmul_R(self, w):           # `toeplitz_tensor.py:99-112`
        B = w.shape[0]
        c = w.reshape((B,) + self.ndims).astype(_cdtype(self.dtype))
        return self._crop(self._apply(self.D_sqrt, c)).astype(self.dtype)

    def solve(self, b, do_precond=True, maxiter=100, tol=1e-8, callback=None):
        """`ToeplitzTensor._solve` (`toeplitz_tensor.py:54-68`)."""
        P = self.matmul_Cinv if do_precond else None
        return conj_grad2(self.matmul_K, b, precond=P, maxiter=maxiter, tol=tol,
                          callback=callback)


    # ---- backward w.r.t. the column ------------------------------------
    def column_grad(self, op, x, g):
        """d/dcolumn of sum(g * op(x)) as torch autograd differentiates the reference:
        op = crop?(Re IFFT(S . FFT(pad? x))) with S in {D, 1/D, sqrt D} (`toeplitz_tensor.py:70-125`),
        D = clamp(Re FFT(C), 1e-6) (`:25-31`), C = circulant_embed(column) (`:20, 135-143`).
        dL/dS = sum_b Re(FFT(x_b) conj(FFT(g_b))) / N; dL/dD = dL/dS S'(D) [Draw >= 1e-6];
        dL/dC = Re FFT(dL/dD); dL/dcolumn = adjoint of the embedding (sum of the copies)."""
        ax = tuple(range(1, self.ndim + 1))
        N = float(self.Mp)
        x = np.asarray(x, np.float64)
        g = np.asarray(g, np.float64)
        B = x.shape[0]
        if op == "R":       # input on the n-grid, output cropped to the m-grid
            X = sfft.fftn(x.reshape((B,) + self.ndims), axes=ax)
            G = sfft.fftn(self._pad(g).astype(np.complex128), axes=ax)
        elif op == "RT":    # input padded, output the full n-grid
            X = sfft.fftn(self._pad(x).astype(np.complex128), axes=ax)
            G = sfft.fftn(g.reshape((B,) + self.ndims), axes=ax)
        else:               # K / Cinv: padded input, cropped output
            X = sfft.fftn(self._pad(x).astype(np.complex128), axes=ax)
            G = sfft.fftn(self._pad(g).astype(np.complex128), axes=ax)
        dS = np.sum((X * np.conj(G)).real, axis=0) / N
        D = self.D.astype(np.float64)
        mask = sfft.fftn(self.C.astype(np.complex128)).real >= 1e-6
        fac = {"K": np.ones_like(D), "Cinv": -1.0 / D ** 2}.get(op, 0.5 / np.sqrt(D))
        dD = np.where(mask, dS * fac, 0.0)
        dC = sfft.fftn(dD.astype(np.complex128)).real
        for a, m in enumerate(self.dims):        # adjoint of cat([K, flip(K)[1:-1]]) per axis
            if m < 2:
                continue
            head = np.take(dC, np.arange(m), axis=a)
            tail = np.flip(np.take(dC, np.arange(m, dC.shape[a]), axis=a), axis=a)
            idx = [slice(None)] * dC.ndim
            idx[a] = slice(1, m - 1)
            head[tuple(idx)] += tail
            dC = head
        return dC.reshape(-1)


def sym_toeplitz_dqf(left_vectors, right_vectors):
    """gpytorch's sym_toeplitz_derivative_quadratic_form (`ziggy/misc/gpt_toeplitz.py:169-209`):
    left/right (n, s); out[i] = sum_j sum_k l_j[k] (r_j[k+i] + r_j[k-i]) for i >= 1 (terms outside
    [0, n) vanish), out[0] = sum_j l_j . r_j.  Linear correlations by FFT of length >= 2n."""
    l = np.asarray(left_vectors, np.float64)
    r = np.asarray(right_vectors, np.float64)
    if l.ndim == 1:
        l, r = l[:, None], r[:, None]
    n = l.shape[0]
    L = 1 << int(np.ceil(np.log2(2 * n)))
    corr = np.fft.irfft(np.sum(np.conj(np.fft.rfft(l, L, axis=0)) * np.fft.rfft(r, L, axis=0), axis=1), L)
    out = corr[:n].copy()                          # sum_k l[k] r[k+i]
    out[1:] += corr[L - 1:L - n:-1]                # sum_k l[k] r[k-i]
    return out


def inv_matmul_column_grad(T, solves, grad_output, maxiter, tol):
    """`InvMatmul.backward` (`ziggy/misc/_inv_matmul.py:27-64`): left solves (preconditioned) and
    the column gradient over the flattened column; returns (column_grad, right_grad)."""
    left = T.solve(grad_output, do_precond=True, maxiter=maxiter, tol=tol)
    lv = np.concatenate([left, solves], 0).T
    rv = np.concatenate([solves, left], 0).T * -0.5
    return sym_toeplitz_dqf(lv, rv), left


# --------------------------------------------------------------------------------------
# CG (ziggy/misc/cg.py)
# --------------------------------------------------------------------------------------
def conj_grad2(A_mul, b, precond=None, maxiter=20, tol=1e-10, callback=None, info=None):
    """Row layout (bsz, M), per-RHS alpha/beta (`cg.py:44-80`): x0=0, r=b-A0, break when
    ALL sqrt(r.r) < tol (after the x/r update), callback after the p update."""
    if precond is None:
        precond = lambda x: x
    x = np.zeros_like(b)
    r = b - A_mul(x)
    z = precond(r)
    p = z
    n_done = 0
    with np.errstate(invalid="ignore", divide="ignore"):
        for n in range(maxiter):
            rs = np.sum(r * z, axis=1)
            Ap = A_mul(p)
            alpha = rs / np.sum(p * Ap, axis=1)
            x = x + alpha[:, None] * p
            r = r - alpha[:, None] * Ap
            rnew = np.sum(r * r, axis=1)
            n_done = n + 1
            if np.all(np.sqrt(rnew) < tol):
                break
            z = precond(r)
            beta = np.sum(z * r, axis=1) / rs
            p = z + beta[:, None] * p
            if callback is not None:
                callback(n, x)
    if info is not None:
        info["iters"] = n_done
    return x


def conj_grad(A_mul, b, precond=None, maxiter=20, tol=1e-10, callback=None, info=None):
    """Column layout (M, L), dim=0 dots (`cg.py:5-41`)."""
    At = lambda y: A_mul(y.T).T
    Pt = None if precond is None else (lambda y: precond(y.T).T)
    cb = None if callback is None else (lambda n, x: callback(n, x.T))
    return conj_grad2(At, b.T, precond=Pt, maxiter=maxiter, tol=tol, callback=cb,
                      info=info).T


# --------------------------------------------------------------------------------------
# gram_solve (ziggy/misc/toeplitz_expanded.py) and compute_kn (ziggy/hipgp.py)
# --------------------------------------------------------------------------------------
def gram_solve(grids, kfun, vec, maxiter=20, do_precond=True, tol=1e-10, callback=None,
               mult_RT=True, info=None):
    """`toeplitz_expanded.py:17-58`: ToeplitzMatmul has NO jitter (`:248`)."""
    dims = tuple(len(g) for g in grids)
    T = ToeplitzOracle(toeplitz_column(grids, kfun, 0.0).astype(vec.dtype), dims)
    Kmul = lambda x: T.matmul_K(x.T).T
    P = (lambda x: T.matmul_Cinv(x.T).T) if do_precond else None
    d = conj_grad(Kmul, vec.T, precond=P, maxiter=maxiter, tol=tol, callback=callback,
                  info=info)
    if mult_RT:
        return T.matmul_RT(d.T)
    return d.T


def compute_kn(T, Knm, maxiter_cg=10, tol=1e-8):
    """`hipgp.py:117-146` (ziggy whitening): kn = R^T K^{-1} Knm^T."""
    d0 = T.solve(Knm, do_precond=True, maxiter=maxiter_cg, tol=tol)
    return T.matmul_RT(d0)


# --------------------------------------------------------------------------------------
# block-diagonal variational family (ziggy/hipgp.py:527-691, ziggy/misc/util.py:79-130)
# --------------------------------------------------------------------------------------
def block_index(dims, blocks):
    """(num_blocks, block_size) table of flat indices into the (expanded) grid `dims`:
    blocks enumerated C-order over the block grid, points C-order inside a block
    (`util.py:79-119`, `define_block_chunks`; the ziggy family blocks the expanded grid
    `arange(2m-2)`, `hipgp.py:599-601,629-634`)."""
    dims, blocks = tuple(int(d) for d in dims), tuple(int(b) for b in blocks)
    assert len(dims) in (2, 3) and len(dims) == len(blocks)
    assert all(d % b == 0 for d, b in zip(dims, blocks)), (dims, blocks)
    flat = np.arange(int(np.prod(dims))).reshape(dims)
    nb = [d // b for d, b in zip(dims, blocks)]
    shp = []
    for n, b in zip(nb, blocks):
        shp += [n, b]
    t = flat.reshape(shp)                         # (n0, b0, n1, b1[, n2, b2])
    d = len(dims)
    t = t.transpose([2 * i for i in range(d)] + [2 * i + 1 for i in range(d)])
    return t.reshape(int(np.prod(nb)), int(np.prod(blocks)))


def block_diag_multiply(S, v, idx):
    """`hipgp.py:645-656`: rows of v (bsz, M') times the block-diagonal S (nb, bs, bs)."""
    vb = v[:, idx]                                  # (bsz, nb, bs)
    out = np.empty_like(v)
    out[:, idx] = np.einsum("kij,bkj->bki", S, vb)
    return out


def block_kl_to_standard(m, S):
    """`stats.py:15-29`: KL(N(m, blockdiag S) || N(0, I)) with the 1e-4 nugget in the log det."""
    bs = S.shape[1]
    L = np.linalg.cholesky(S + 1e-4 * np.eye(bs)[None])
    lndet = 2.0 * np.sum(np.log(np.diagonal(L, axis1=-2, axis2=-1)))
    return 0.5 * (np.trace(S, axis1=-2, axis2=-1).sum() + np.sum(m * m) - lndet - S.shape[0] * bs)


def block_elbo_and_grad(kn, y, Knn_diag, theta1, theta2, idx, N, ivar, log_sd):
    """BlockToeplitzGP ELBO estimate and natural-gradient theta grads given kn (bsz, M')
    (`hipgp.py:194-276` 'block' branch, `compute_batch_an` :370-414, `standard_variational_params`
    :636-643, `compute_knSkn` :661-664, `get_kl_to_prior` :687-691).  ivar/log_sd are scalars
    (shared noise) or (bsz,) arrays (per-observation noise).
    Returns (elbo, theta1_grad (M',1), theta2_grad (nb,bs,bs), batch_an, knSkn)."""
    bsz = kn.shape[0]
    S = np.linalg.inv(-2 * theta2)
    qm = block_diag_multiply(S, theta1.T, idx).T                    # (M', 1)
    knm = (kn @ qm).reshape(-1)
    knSkn = np.sum(kn * block_diag_multiply(S, kn, idx), axis=-1)
    iv = np.broadcast_to(np.asarray(ivar, dtype=kn.dtype).reshape(-1), (bsz,))
    lsd = np.broadcast_to(np.asarray(log_sd, dtype=kn.dtype).reshape(-1), (bsz,))
    y = y.reshape(-1)
    an = (-0.5 * iv * ((knm - y) ** 2 + Knn_diag.reshape(-1) - np.sum(kn * kn, axis=-1) + knSkn)
          - lsd - 0.5 * np.log(2 * np.pi))
    elbo = np.mean(an) - block_kl_to_standard(qm, S) / N
    bscale = N / bsz
    bdiff = iv * (knm - y)
    dm = bscale * (-(bdiff[None, :] @ kn).T) - qm
    kb = kn[:, idx]                                                  # (bsz, nb, bs)
    G = np.einsum("b,bki,bkj->kij", iv, kb, kb)
    lam = bscale * G + np.eye(idx.shape[1])[None]
    dS = -0.5 * lam - theta2
    deta1 = dm + block_diag_multiply(dS, -2 * qm.T, idx).T
    return elbo, -deta1, -dS, an, knSkn


# --------------------------------------------------------------------------------------
# full-batch solve of the mean-field family (ziggy/hipgp.py:278-368)
# --------------------------------------------------------------------------------------
def meanfield_batch_solve(kn, y, Knn_diag, ivar, log_sd, N):
    """`hipgp.py:296-345` ('mean-field', expectation family) given every observation's kn
    (n, M'): lam = 1 + sum_n ivar_n kn_n^2, b = sum_n ivar_n y_n kn_n, m = (I + sum_n ivar_n
    kn_n kn_n^T)^{-1} b, theta2 = -lam/2, theta1 = m lam; and the ELBO of `:347-368`
    (mean_n a_n - KL/N, shared or per-observation noise).  The reference's own batch_solve
    raises UnboundLocalError at `:314` before any of this runs (see hipgp_amd batch_solve).
    Returns (theta1 (M',1), theta2 (M',1), elbo)."""
    n, Mp = kn.shape
    iv = np.broadcast_to(np.asarray(ivar, dtype=kn.dtype).reshape(-1), (n,))
    lsd = np.broadcast_to(np.asarray(log_sd, dtype=kn.dtype).reshape(-1), (n,))
    y = y.reshape(-1)
    lam = 1 + np.einsum("n,nm->m", iv, kn * kn)
    b = kn.T @ (iv * y)
    big = np.eye(Mp) + (kn * iv[:, None]).T @ kn
    m = np.linalg.solve(big, b)
    theta1, theta2 = (m * lam)[:, None], (-0.5 * lam)[:, None]
    S = 1 / lam
    knm = kn @ m
    an = (-0.5 * iv * ((knm - y) ** 2 + Knn_diag.reshape(-1) - np.sum(kn * kn, -1) + (kn * kn) @ S)
          - lsd - 0.5 * np.log(2 * np.pi))
    kl = 0.5 * (S.sum() + m @ m - np.log(S).sum() - Mp)
    return theta1, theta2, an.mean() - kl / N
