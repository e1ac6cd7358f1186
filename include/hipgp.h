/*
 * hipgp.h — C ABI of libhipgp.so, the MI355X (gfx950) native structured-kernel PCG path of
 * HIP-GP (`suyashk12/hipgp`, package `ziggy`).
 *
 * The reference has no FFI: its operator boundary is duck-typed Python.
 * Each entry point below replaces the reference interface named next to it; the Python
 * drop-in (`hipgp_amd/ziggy/...`, re-exported as `ziggy`) binds them through ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - All data pointers are DEVICE pointers on the plan's device, C-contiguous, in the plan's
 *    dtype (HGP_F32 = float, HGP_F64 = double).  Caller owns them; nothing is freed across
 *    the ABI.  Vectors are row layout (nrhs, M) unless a `layout` argument says otherwise.
 *  - M = prod(m_i); M' = prod(n_i) with n_i = 2 m_i - 2 (m_i > 1) else 1  (`hipgp.py:72`).
 *  - Calls are asynchronous w.r.t. the host and ordered on the plan's stream, except where a
 *    host output pointer is passed (that call synchronises the stream).
 *  - Every function returns 0 on success or a negative HGP_E* code, and sets a thread-local
 *    message readable with hgp_last_error().  No C++ exception crosses the ABI.
 */
#ifndef HIPGP_H
#define HIPGP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hgp_plan hgp_plan;

enum { HGP_F32 = 0, HGP_F64 = 1 };
enum { HGP_OP_K = 0, HGP_OP_CINV = 1, HGP_OP_RT = 2, HGP_OP_R = 3 };
enum { HGP_SPEC_D = 0, HGP_SPEC_DSQRT = 1, HGP_SPEC_DI = 2 };
enum { HGP_LAYOUT_ROWS = 0, HGP_LAYOUT_COLS = 1 };
enum { HGP_KERN_SQEXP = 0, HGP_KERN_MATERN12 = 1, HGP_KERN_MATERN32 = 2, HGP_KERN_MATERN52 = 3,
       HGP_KERN_GNEITING = 4 };
enum {
  HGP_OK = 0, HGP_E_ARG = -1, HGP_E_HIP = -2, HGP_E_STATE = -3, HGP_E_UNSUPPORTED = -4,
  HGP_E_OOM = -5
};

/* Plan for one gridded inducing mesh m[0..ndim-1] (ndim 1..3, C order, last axis fastest).
 * Replaces the shape/state part of `ToeplitzTensor.__init__` (toeplitz_tensor.py:9-45) and
 * `ToeplitzMatmul.__init__` (toeplitz_expanded.py:82-127).  `hip_stream` may be NULL (null
 * stream).  max_rhs is a capacity hint; workspaces grow on demand.  Any axis length (fp32 and
 * fp64 plans): axes of up to 8192 points run the pruned per-axis passes; fp64 plans whose R / R^T
 * lines exceed 16384 points (axes of 5463..8192) run those two ops on the full fp64 L_R grid, and
 * a plan with an axis beyond 8192 points runs all four operators on the full fp64 L_K / L_R grid
 * (recursive radix-2 levels down to an 8192-point base pass; unfused PCG, no slab split).  One
 * right-hand side's intermediate must stay below 2^31 values, else HGP_E_UNSUPPORTED. */
int hgp_plan_create(int device, int ndim, const int64_t* m, int dtype, int64_t max_rhs,
                    void* hip_stream, hgp_plan** out);

/* Change the stream later calls are ordered on (synchronises the previous stream first, so a
 * plan can be handed between streams, e.g. from a pool of idle plans). */
int hgp_plan_set_stream(hgp_plan* plan, void* hip_stream);

/* Spectrum setup from the kernel-evaluated Toeplitz first column (device, M values):
 * column[0] += jitter (toeplitz_tensor.py:132; pass 0 when already included), circulant
 * embedding (toeplitz_tensor.py:135-143), D = clamp(Re FFT(C), clamp_min) (:25-31), and the
 * operator spectra for K, C^-1 and R/R^T.  Replaces toeplitz_tensor.py:12-33.
 * If n_clamped != NULL it receives the number of clamped eigenvalues of the full expanded
 * (n-grid) spectrum, each mirror image counted, as (D_raw < clamp_min).sum() over the
 * reference's D (synchronises). */
int hgp_plan_set_column(hgp_plan* plan, const void* column, double jitter, double clamp_min,
                        int64_t* n_clamped);

/* y = op(x) for nrhs right-hand sides, row layout.
 *   HGP_OP_K    : K v            x:(nrhs,M)  -> y:(nrhs,M)    toeplitz_tensor.py:70-83
 *   HGP_OP_CINV : C^-1 block v   x:(nrhs,M)  -> y:(nrhs,M)    toeplitz_tensor.py:114-125
 *   HGP_OP_RT   : R^T v          x:(nrhs,M)  -> y:(nrhs,M')   toeplitz_tensor.py:85-97
 *   HGP_OP_R    : R w            x:(nrhs,M') -> y:(nrhs,M)    toeplitz_tensor.py:99-112
 * (same four ops as ToeplitzMatmul.forward "gram"/"circ_inv"/"RTv"/"Rv",
 *  toeplitz_expanded.py:139-189).  x and y must not alias. */
int hgp_toeplitz_apply(hgp_plan* plan, int op, const void* x, void* y, int64_t nrhs);

/* Batched PCG, exactly the recurrence of conj_grad2 (cg.py:44-80) for layout ROWS
 * (b,x:(nrhs,M)) and conj_grad (cg.py:5-41) for layout COLS (b,x:(M,nrhs)): A = K,
 * preconditioner C^-1 if use_precond, x0 = 0, per-RHS alpha/beta, stop when ALL
 * sqrt(r.r) < tol after the x/r update.  The early-exit test runs on the device (a flag read
 * by every later kernel), so the host is not synchronised per iteration (solves with
 * maxiter > 32 read the flag every 16 iterations to stop queueing no-op iterations).
 * iters_done (host, may be NULL): number of iterations executed (synchronises).
 * Replaces ToeplitzTensor._solve (toeplitz_tensor.py:54-68) / InvMatmul.forward. */
int hgp_pcg_solve(hgp_plan* plan, const void* b, void* x, int64_t nrhs, int maxiter,
                  double tol, int use_precond, int layout, int* iters_done);

/* Profiling: run only pass `pass` (0-based; -1 = all) of the op's pass sequence (the
 * intermediate workspace is whatever the previous call left).  hgp_op_pass_count returns the
 * number of passes (1 for 1-D, 3 for 2-D, 5 for 3-D).  Used by bench.py to time each kernel
 * with HIP events. */
int hgp_toeplitz_apply_pass(hgp_plan* plan, int op, const void* x, void* y, int64_t nrhs, int pass);
int hgp_op_pass_count(const hgp_plan* plan);

/* Stepwise PCG for the callback form of conj_grad/conj_grad2 (cg.py:77-78): begin() sets
 * x0 = 0, r = b, z = P r, p = z; step() runs one iteration and, if `converged` != NULL,
 * reports (synchronising) whether the break test fired on it.  x is updated in place in the
 * caller's buffer given to begin(). */
int hgp_pcg_begin(hgp_plan* plan, const void* b, void* x, int64_t nrhs, int use_precond,
                  int layout);
int hgp_pcg_step(hgp_plan* plan, double tol, int* converged);

/* Per-RHS r.r after the last hgp_pcg_step (device, nrhs values in the plan dtype).  With
 * tol < 0 a step never sets the convergence flag, so a caller that shards the right-hand
 * sides over processes can apply the reference's ALL-RHS break rule (cg.py:69-71) globally:
 * step(tol = -1), read r.r, all-reduce "every sqrt(r.r) < tol", stop.  x is final after the
 * step that met the test (the break precedes only the z/p update). */
int hgp_pcg_rnorm2(hgp_plan* plan, void* out);

/* Device-side form of the same all-rank break rule (no host round trip per iteration):
 * hgp_pcg_local_flag writes *flag (device int) = 1 when every sqrt(r.r) of the plan's RHS is
 * below tol after the last step(tol = -1); the caller all-reduces it (MIN, e.g. RCCL on the
 * same stream order) and hgp_pcg_set_done(flag) raises the plan's done flag when the reduced
 * value is 1, so every later step of the solve is a no-op on the device. */
int hgp_pcg_local_flag(hgp_plan* plan, double tol, int* flag);
int hgp_pcg_set_done(hgp_plan* plan, const int* flag);
/* Iterations the current solve has executed whose break test did not stop it, plus the one
 * that did (host int; synchronises the plan's stream). */
int hgp_pcg_iters(hgp_plan* plan, int* iters);

/* Grid-block (slab) sharding along axis 0 (row e2: a 2-D / 3-D grid's axis-0 rows split over
 * ranks; hipgp_amd/slab.py drives it).  Each op is its pass sequence split at the axis-0
 * convolution, which needs whole axis-0 lines and so runs between two all-to-all transposes.
 * Exchange layout E (plan dtype, interleaved complex): E[g][q][i][c]
 *   d = 2: g < NG = L1/2 + 1 compact axis-1 columns, inner = 1;
 *   d = 3: g < NG = L1 axis-1 frequencies, c < inner = the compact half-spectrum pitch of axis 2;
 *   q < nrhs; i = axis-0 row (a rank's rows in FWD / INV, whole lines in CONV).
 * stage HGP_SLAB_FWD : x (nrhs, nrows, rest of the input row) real -> E over this rank's nrows
 *                      input rows (all NG groups)                 toeplitz_tensor.py:79,94,109,122
 * stage HGP_SLAB_CONV: E lines [ng][nrhs][P0][inner], P0 = max(in0, out0) rows per line, groups
 *                      [g0, g0 + ng) of the op's spectrum; in place allowed  (:80-82 etc.)
 * stage HGP_SLAB_INV : E over this rank's nrows output rows -> y (nrhs, nrows, rest) real, crop
 * stage HGP_SLAB_CONV_A2A: the axis-0 convolution of groups [g0, g0 + ng) straight from the
 *                      receive buffer of the first all-to-all to the send buffer of the second
 *                      (no line buffer, no gather / scatter copies): `nrows` = the world size W,
 *                      in  = [r][g][q][i - a_r][c] for the balanced split of the in0 input rows
 *                            over the W ranks (rank r: rows [a_r, a_r + cnt_r)),
 *                      out = [r][g][q][o - b_r][c] for the split of the out0 output rows,
 *                      g < ng, q < nrhs, c < inner; in != out.
 * Partial dot products / PCG scalars are the caller's (all-reduced over ranks). */
enum { HGP_SLAB_FWD = 0, HGP_SLAB_CONV = 1, HGP_SLAB_INV = 2, HGP_SLAB_CONV_A2A = 3 };
int hgp_slab_info(const hgp_plan* plan, int op, int64_t* ngroups, int64_t* inner);
int hgp_slab_pass(hgp_plan* plan, int op, int stage, const void* in, void* out, int64_t nrhs,
                  int64_t nrows, int64_t g0, int64_t ng);
/* hgp_slab_pass with two options for the slab PCG (hipgp_amd/slab.py SlabToeplitz.pcg):
 *   done (device int or NULL): every kernel of the stage is a no-op once *done != 0, so the
 *        iterations after the all-rank break cost (almost) nothing without a host round trip;
 *   dotv, dot_out (HGP_SLAB_INV only, device, or NULL): the stage also leaves this rank's
 *        per-RHS dot dot_out[q] = sum_j y[q, j] dotv[q, j] of its output y (dotv laid out
 *        like y), from per-row-pair partials summed in a fixed order -- p.Ap / z.r of
 *        cg.py:66,74 without a second read of the vectors.  dot_out: nrhs values. */
int hgp_slab_pass_ex(hgp_plan* plan, int op, int stage, const void* in, void* out, int64_t nrhs,
                     int64_t nrows, int64_t g0, int64_t ng, const void* dotv, void* dot_out,
                     const int* done);

/* The slab PCG's vector / scalar updates (cg.py:63-78) on this rank's slab (nrhs rows of M
 * values, plan dtype; M may be 0 on a rank without rows), with every per-RHS dot ALREADY
 * all-reduced by the caller between the calls.  done / iters: device ints (0 at the start);
 * every call is a no-op once *done != 0 (done = the iteration the break fired in).
 *   hgp_slab_cg_xr   : alpha = rs / pAp; x += alpha p; r -= alpha Ap; rr = local sum r.r
 *   hgp_slab_cg_check: iters += 1; done = iters when every sqrt(rr) < tol (rr reduced; NaN =
 *                      not converged, cg.py:70)
 *   hgp_slab_cg_p    : beta = zr / rs; rs = zr; p = z + beta p
 * All per-RHS scalars are device arrays of nrhs values; ordered on the plan's stream. */
int hgp_slab_cg_xr(hgp_plan* plan, void* x, void* r, const void* p, const void* Ap, const void* rs,
                   const void* pAp, void* rr, int64_t nrhs, int64_t M, const int* done);
int hgp_slab_cg_check(hgp_plan* plan, const void* rr, int64_t nrhs, double tol, int* done, int* iters);
int hgp_slab_cg_p(hgp_plan* plan, void* p, const void* z, void* rs, const void* zr, int64_t nrhs,
                  int64_t M, const int* done);

/* The clamped spectrum D (which=HGP_SPEC_D), sqrt(D) or 1/D on the full expanded grid
 * (device, M' reals) — the real parts of ToeplitzTensor.D / D_sqrt / Di
 * (toeplitz_tensor.py:28-31). */
int hgp_get_spectrum(hgp_plan* plan, int which, void* out);

/* Per-row dot products out[b] = sum_j a[b,j] c[b,j] (device), used by the generic
 * conj_grad2 path with caller-supplied A_mul callables (cg.py:64,66,69,74). */
int hgp_rowdot(int dtype, const void* a, const void* c, void* out, int64_t nrhs, int64_t M,
               void* hip_stream);

/* Point-observation cross covariance on a gridded mesh, the PCG right-hand sides:
 *   out[n, j] = k(x_n, u_j),  x: (nobs, ndim) device, u_j the C-order mesh of grids[0..ndim-1]
 *   (device arrays of m[a] points), out: (nobs, M) device, dtype HGP_F32 / HGP_F64.
 * kind: HGP_KERN_SQEXP  sig2 exp(-|(x-u)/ell|^2 / 2)            (kernels.py:73-79)
 *       HGP_KERN_MATERN{12,32,52}  Matern nu = 1/2, 3/2, 5/2    (kernels.py:145-158)
 * Same per-element arithmetic as the reference, without its (nobs, M, ndim) broadcast
 * (replaces svi_gp.py:72 `self.kernel(xbatch, self.xinduce, kern_params)`). */
int hgp_kuf_grid(int dtype, int kind, int ndim, const int64_t* m, const void* const* grids,
                 const void* x, int64_t nobs, double sig2, double ell, void* out,
                 void* hip_stream);

/* Line-integral ("semi-integrated") cross covariance on a gridded mesh, SURVEY §8(f) row 2
 * (the inter-domain observations of config 5: observation n is the segment 0 -> x_n):
 *   out[n, j] = |x_n| * mean_{a < npts} k(u_j, alpha_a x_n),  alpha_a = a/npts + u[0]/npts
 * = Kernel.k_semi_mc (kernels.py:19-39) as svi_gp._make_grams uses it (svi_gp.py:61-64,
 * transposed).  u: device scalar holding the reference's single torch.rand(1) draw, so the
 * caller consumes the RNG exactly as the reference does.  kind: any HGP_KERN_*; kparam is
 * Gneiting's alpha (ignored otherwise).  1 <= npts <= 1024.  Layout as hgp_kuf_grid. */
int hgp_kuf_semi_mc(int dtype, int kind, double kparam, int ndim, const int64_t* m,
                    const void* const* grids, const void* x, int64_t nobs, double sig2,
                    double ell, int npts, const void* u, void* out, void* hip_stream);

/* Analytic SqExp line integral, SqExp.k_semi -> semi_integrated_sqe (kernels.py:80-85,
 * 223-237), replacing svi_gp.py:58-59:  out[n, j] = |x_n| int_0^1 k(u_j, a x_n) da
 * (NaN for |x_n| = 0, as the reference).  Layout as hgp_kuf_grid. */
int hgp_kuf_semi_sqexp(int dtype, int ndim, const int64_t* m, const void* const* grids,
                       const void* x, int64_t nobs, double sig2, double ell, void* out,
                       void* hip_stream);

/* Doubly-integrated diagonal Knn_diag by table interpolation,
 * KernelDoublyDiagInterpolator.forward (kernels.py:200-220): table = device array of 3*N
 * values in dtype (distance grid, knn, slopes: the reference's float32 table), x: (nobs,
 * ndim), out: (nobs,). */
int hgp_knn_doubly_diag(int dtype, int ndim, const void* x, int64_t nobs, double sig2, double ell,
                        const void* table, int N, void* out, void* hip_stream);

/* Mean-field natural-gradient statistics of a minibatch (the batch sums
 * of MeanFieldToeplitzGP.elbo_and_grad, hipgp.py:234-250, and a_n of compute_batch_an,
 * hipgp.py:370-414), from kn = R^T K^-1 Knm^T (nrhs, Mp) and the variational mean qm / diagonal
 * covariance qS (Mp,), with per-observation y, ivar = 1/noise^2, Knn_diag, log_sd (nrhs,):
 *   an[n]  = -1/2 ivar_n ((kn_n.qm - y_n)^2 + Knn_n - |kn_n|^2 + kn_n^2.qS) - log_sd_n - ln(2 pi)/2
 *   lam[j] = sum_n ivar_n kn_nj^2,   dm[j] = -sum_n ivar_n (kn_n.qm - y_n) kn_nj
 * All device arrays of dtype; deterministic (fixed reduction order), two reads of kn.
 * Per rank these are the partial sums RCCL all-reduces across the RHS shards. */
int hgp_meanfield_stats(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm,
                        const void* qS, const void* y, const void* ivar, const void* Knn_diag,
                        const void* log_sd, void* an, void* lam, void* dm, void* hip_stream);

/* The two passes of hgp_meanfield_stats apart, for kn held in column slabs over ranks (grid-block
 * sharding, hipgp_amd/slab.py; same reference lines).  hgp_meanfield_rowdots: for the Mp columns
 * of kn given (qm, qS: the matching slices), out3[n*3 + c] = (kn_n.qm, |kn_n|^2, kn_n^2.qS),
 * fixed reduction order.  A caller all-reduces out3 over the slabs and forms
 * bdiff_n = ivar_n (kn_n.qm - y_n) and a_n from the totals; hgp_meanfield_cols then writes the
 * slab's lam[j] = sum_n ivar_n kn_nj^2 and dm[j] = -sum_n bdiff_n kn_nj (Mp = 0: nothing). */
int hgp_meanfield_rowdots(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm,
                          const void* qS, void* out3, void* hip_stream);
int hgp_meanfield_cols(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* ivar,
                       const void* bdiff, void* lam, void* dm, void* hip_stream);

/* Block-diagonal variational family (BlockToeplitzGP, ziggy/hipgp.py:527-691), SURVEY §8(f) row 3.
 * The expanded grid dims[ndim] (ndim 2 or 3, n_a = 2 m_a - 2) is tiled by blocks[ndim] (each n_a
 * divisible by blocks[a]; points per block bs = prod blocks <= 128), blocks enumerated C-order
 * over the block grid and points C-order inside a block (ziggy/misc/util.py:79-119).
 *   gram[nblk][bs][bs] = sum_n ivar_n kn_{n,blk} kn_{n,blk}^T     (hipgp.py:252-256, get_lam :669-685)
 *   knSkn[nrhs]        = sum_blk kn_{n,blk}^T S_blk kn_{n,blk}    (compute_knSkn :661-664; S [nblk][bs][bs])
 *   trSG[1]            = sum_blk <S_blk, gram_blk>_F = sum_n ivar_n knSkn_n   (the ELBO's a_n sum needs only this)
 * kn (nrhs, M') row layout; gram, knSkn, trSG may each be NULL to skip that output (trSG needs
 * gram; ivar may be NULL without gram, S without knSkn/trSG).  gram is the per-shard sum RCCL
 * all-reduces across RHS shards.  Deterministic. */
int hgp_block_stats(int dtype, int ndim, const int64_t* dims, const int64_t* blocks, const void* kn,
                    int64_t nrhs, const void* ivar, const void* S, void* gram, void* knSkn,
                    void* trSG, void* hip_stream);

/* Backward of the solve w.r.t. the Toeplitz column, SURVEY §8(f) row 4.  Replaces gpytorch's
 * sym_toeplitz_derivative_quadratic_form (reference ziggy/misc/gpt_toeplitz.py:169-209) as
 * InvMatmul.backward calls it (ziggy/misc/_inv_matmul.py:52-60, left_vecs = [L; R],
 * right_vecs = -0.5 [R; L] over the FLATTENED column):
 *   out[i] = sum_j sum_k left_j[k] (right_j[k+i] + right_j[k-i])  (i >= 1, out-of-range terms 0)
 *   out[0] = sum_j left_j . right_j
 * left, right: (nvec, n) row layout (the reference's (n, s) input transposed), out: (n,), all
 * device arrays of dtype.  Direct lagged sums (O(nvec n^2)), deterministic. */
int hgp_sym_toeplitz_dqf(int dtype, const void* left, const void* right, int64_t nvec, int64_t n,
                         void* out, void* hip_stream);

/* hgp_sym_toeplitz_dqf for n = the plan's M, through the grid's factorisation: the flattened-index
 * correlation sum_k u[k] v[k+i] is the fold of the d-D correlation over its signed-digit lags,
 * computed as one fp64 FFT per vector pair on the L_K grid (O(nvec prod L_K log)).  left, right
 * (nvec, M) row layout, out (M,), plan dtype.  Synchronises the plan stream. */
int hgp_plan_dqf(hgp_plan* plan, const void* left, const void* right, int64_t nvec, void* out);

/* Gradient of sum(g * op(x)) w.r.t. the plan's column through the operator's spectrum
 * (K: D, CINV: 1/D, RT and R: D_sqrt; D = clamp(Re FFT_n(circulant_embed(column)), clamp_min),
 * reference toeplitz_tensor.py:20-31, ops :70-125).  The x-gradient is the adjoint operator
 * (K, CINV self-adjoint; R <-> RT) through hgp_toeplitz_apply.  x (nrhs, M) or (nrhs, M') for R,
 * g shaped like op(x); column_grad (M,); device arrays of the plan dtype; fp64 chain (DCT-I pair
 * on the m-grid); the filter correlation is one fp64 cross spectrum per RHS on the L_K / L_R grid.
 * Synchronises the plan stream. */
int hgp_plan_column_grad(hgp_plan* plan, int op, const void* x, const void* g, int64_t nrhs,
                         void* column_grad);

/* Sizes of a plan: M, M' and the padded FFT lengths per axis (K-type and R-type ops). */
int hgp_plan_info(const hgp_plan* plan, int64_t* M, int64_t* Mprime, int64_t* L_K,
                  int64_t* L_R);

/* Device memory a plan holds: scratch (operator workspaces, CG vectors, set-up scratch; all
 * re-allocated on demand) and tables (twiddles, Bluestein DCT tables, spectra).
 * hgp_plan_trim frees the scratch (after synchronising the plan's streams) and keeps the tables,
 * so an idle plan kept for re-use holds only what its next set-up needs. */
int hgp_plan_mem(const hgp_plan* plan, int64_t* scratch_bytes, int64_t* table_bytes);
int hgp_plan_trim(hgp_plan* plan);
int hgp_plan_destroy(hgp_plan* plan);

const char* hgp_last_error(void);

/* Library/ABI version string. */
const char* hgp_version(void);

#ifdef __cplusplus
}
#endif

#endif /* HIPGP_H */
