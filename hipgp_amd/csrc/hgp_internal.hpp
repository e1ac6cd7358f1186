// hgp_internal.hpp — declarations shared by the kernel and API translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hgp_pass.hpp"

namespace hgp {

struct GridDims { int d; int64_t m[3]; int64_t n[3]; int64_t L[3]; };

struct PassGeom { int C; int threads; int lds; };
template <typename T>
hipError_t launch_pass(int H, int mode, int lay, const PassDesc& d, int64_t nblocks, hipStream_t s);
template <typename T> PassGeom pass_geom(int H, int lay);
// 2-D row-pair passes with the column-major intermediate (hgp_rows.hpp); inv = 0 FWD, 1 INV;
// grouped = 1: the grouped-column layout of the 2-D operators (G = rowt_group(H) columns
// interleaved; the axis-0 pass then reads it as LAY_CONTIG_G), 0: plain (3-D planes, slabs)
template <typename T>
hipError_t launch_rowt(int H, int inv, int epi, const PassDesc& d, hipStream_t s, int grouped);
// row pairs per block of the row passes (partials of the fused PCG epilogue are per block)
template <typename T> int rowt_pairs(int H, int grouped);
// threads per block of the row-pair kernels
template <typename T> int rowt_threads(int H, int grouped);
// whether the row-pair kernels of H points fit one CU's LDS (else run_op takes the generic path)
template <typename T> int rowt_fits(int H, int grouped);
// columns per group of the 2-D operators' intermediate at row half-length H (1: plain layout)
template <typename T> int rowt_group(int H);
// 3-D middle-axis transposing line passes (hgp_lines.hpp): inv = 0 k_line_fwd_t, 1 k_line_inv_t
template <typename T>
hipError_t launch_linet(int H, int inv, const PassDesc& d, hipStream_t s);
template <typename T> int linet_fits(int H);

// setup (fp64)
// Bluestein partial DFT pieces of the DCT-I (hgp_kernels.hip)
void chirp_tables(double2* pre, double2* post, int64_t m, int64_t n, hipStream_t s);
void chirp_filter(double2* h, int64_t m, int64_t n, int64_t L, double scale, hipStream_t s);
void chirp_pre(const double* x, const double2* pre, double2* c, int64_t total, int64_t m, int64_t I, hipStream_t s);
void chirp_post(const double2* c, const double2* post, double* y, int64_t total, int64_t m, int64_t I, double scale,
                hipStream_t s);
template <typename T> void to_f64(const void* src, double* dst, int64_t n, double add0, hipStream_t s);
// nclamp[0] counts the clamped entries; nclamp[1] / nclamp[2] receive max D / max 1/D (finite
// values, as the bits of positive doubles) for pack_scale
void clamp_spectrum(const double* Draw, double* out3, int64_t M, double clamp_min, unsigned long long* nclamp,
                    const GridDims& g, hipStream_t s);
// The set-up transforms the K and C^-1 generators as ONE complex grid (K real, C^-1 imaginary).
// A transform's rounding is relative to its largest value, and at the clamp 1/D reaches 1e6 where
// D stays ~1e3: packed as they are, the K spectrum would carry C^-1-sized rounding (K matvec 400x
// less accurate in its small modes -- what 20 clamped PCG iterations amplify).  The C^-1
// generator is therefore packed scaled by pack_scale = 2^(ilogb max D - ilogb max 1/D) (exact)
// and unscaled on extraction.  `mx` = nclamp + 1 (nullptr: no scaling).
__device__ __forceinline__ double pack_scale(const unsigned long long* mx) {
  if (mx == nullptr) return 1.0;
  const double a = __longlong_as_double((long long)mx[0]), b = __longlong_as_double((long long)mx[1]);
  if (!(a > 0.0) || !(b > 0.0) || !isfinite(a) || !isfinite(b)) return 1.0;
  return ldexp(1.0, ilogb(a) - ilogb(b));
}
void embed_K(const double* cK, const double* cI, double2* out, const GridDims& g, const unsigned long long* mx,
             hipStream_t s);
void embed_R(const double* sv, double2* out, const GridDims& g, hipStream_t s);
// sym: mirror the filter over (-n, n) on every axis (needs L >= 2n - 1): the embedded filter is
// then even and its spectrum real (set_column_t, hgp_plan::r_real)
void embed_R_real(const double* sv, double* out, const GridDims& g, int sym, hipStream_t s);
void r2_combine(const double2* in, double2* out, int64_t L, int64_t Rn, int64_t r_stride, int64_t In, int64_t ps,
                const double2* tw, hipStream_t s, const int* done = nullptr);
// d >= 2: tiled transposing extraction into [c][k1][k0] (hgp_kernels.hip k_extract_t); b == nullptr:
// complex spectrum into a, else the pair (Re -> a, Im -> b)
template <typename T>
void extract_t(const double2* F, void* a, void* b, int64_t L0, int64_t L1, int64_t H, int64_t Ssrc, int compact_src,
               double scale, hipStream_t s, const unsigned long long* mx = nullptr);
// the same extraction keeping the real part only (a real spectrum: Re -> a)
template <typename T>
void extract_t_re(const double2* F, void* a, int64_t L0, int64_t L1, int64_t H, int64_t Ssrc, int compact_src,
                  double scale, hipStream_t s);
template <typename T> void extract_pair(const double2* F, void* a, void* b, int64_t n, int64_t L, int64_t S, int compact,
                                        double scale, hipStream_t s, int64_t L0t = 0, int64_t L1t = 0,
                                        const unsigned long long* mx = nullptr);
template <typename T> void extract_cplx(const double2* F, void* o, int64_t n, int64_t L, int64_t S, int compact, double scale,
                                        hipStream_t s, int64_t L0t = 0, int64_t L1t = 0);
template <typename T> void expand_spec(const double* src, void* out, const GridDims& g, hipStream_t s);

// dense grid cross covariance (hgp_kuf.hip)
hipError_t kuf_grid(int dtype, int kind, int ndim, const int64_t* m, const void* const* grids, const void* x,
                    int64_t nobs, double sig2, double ell, void* out, hipStream_t s);
hipError_t kuf_semi(int dtype, int kind, double kp, int ndim, const int64_t* m, const void* const* grids,
                    const void* x, int64_t nobs, double sig2, double ell, int npts, const void* u, void* out,
                    hipStream_t s);
hipError_t doubly_diag(int dtype, int ndim, const void* x, int64_t nobs, double sig2, double ell, const void* tab,
                       int N, void* out, hipStream_t s);
hipError_t meanfield_stats(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                           const void* y, const void* iv, const void* knn, const void* lsd, void* an, void* lam,
                           void* dm, hipStream_t s);
hipError_t meanfield_rowdots(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                             void* out3, hipStream_t s);
hipError_t meanfield_cols(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* iv, const void* bdiff,
                          void* lam, void* dm, hipStream_t s);
// expanded grid n[a] tiled by blocks of side b[a] (nb[a] per axis); bs points per block, nbw
// blocks per workgroup
struct BlockGeom {
  int d, bs, nbw;
  int64_t nblk, Mp;
  int64_t n[3], b[3], nb[3];
};
int block_geom(int ndim, const int64_t* dims, const int64_t* blocks, BlockGeom* g, const char** why);
hipError_t block_stats(int dtype, const BlockGeom& g, const void* kn, int64_t nrhs, const void* iv, const void* S,
                       void* gram, void* knSkn, void* trSG, hipStream_t s);
hipError_t kuf_semi_grid(int dtype, int kind, int method, int ndim, const int64_t* m, const void* const* grids,
                         const void* x, int64_t nobs, double sig2, double ell, const void* nodes,
                         const void* weights, int npts, void* out, hipStream_t s);

// backward w.r.t. the Toeplitz column (hgp_grad.hip)
hipError_t sym_toeplitz_dqf(int dtype, const void* u, const void* v, int64_t nvec, int64_t n, void* out,
                            hipStream_t s);
void fold_div_mu(const double* X, int64_t M, const GridDims& gd, double* y, hipStream_t s);
void spec_bwd(double* y, const double* D3, int64_t M, int kind, double cmin, hipStream_t s);
void mul_mu_out(int dtype, const double* r, int64_t M, const GridDims& gd, void* out, hipStream_t s);
// v + i h on the L-grid, h scaled to v's magnitude by pack_scale (mx: 2 device words, reduced
// here over the nv / nh values of v / h); xspec_acc undoes the scale
void pack_pair(int dtype, const void* v, const void* h, int h_periodic, const GridDims& gd, int64_t prodL, double2* z,
               unsigned long long* mx, int64_t nv, int64_t nh, hipStream_t s);
void xspec_acc(const double2* Z, double2* S, const GridDims& gd, int64_t prodL, int first, const unsigned long long* mx,
               hipStream_t s);
void conj_inplace(double2* S, int64_t n, hipStream_t s);
// fp64 full-grid route of R / R^T (hgp_grad.hip): gd.m = the input / output extents, gd.L = L_R;
// done (optional device flag): every kernel is a no-op once *done != 0 (the PCG's break)
void grid_embed(int dtype, const void* x, const GridDims& gd, int64_t prodL, double2* z, hipStream_t s,
                const int* done = nullptr);
void grid_mul_unperm(const double2* F, const double2* S, const GridDims& gd, int64_t prodL, int conj_spec,
                     double2* out, hipStream_t s, const int* done = nullptr);
void grid_crop(int dtype, const double2* Z, const GridDims& gd, int64_t outM, void* y, hipStream_t s,
               const int* done = nullptr);
void scale_copy(const double2* a, double2* b, int64_t n, double sc, hipStream_t s,
                const unsigned long long* mx = nullptr);   // mx: the imaginary part also / pack_scale
// long-axis DCT line batches (hgp_grad.hip)
void line_embed(const double2* c, double2* E, int64_t O, int64_t m, int64_t I, int64_t L, hipStream_t s);
void line_mul_unperm_conj(const double2* X, const double2* f, double2* Z, int64_t O, int64_t L, int64_t I,
                          hipStream_t s);
void line_unperm_conj(const double2* Y, double2* c, int64_t O, int64_t L, int64_t I, int64_t m, hipStream_t s);
void gather_n(const double2* F, const GridDims& gd, int h_periodic, int64_t Mp, double invL, double* X, hipStream_t s);
void gather_flat(int dtype, const double2* F, const GridDims& gd, int64_t M, double invL, void* out, hipStream_t s);
// CG
int update_np(int64_t M);
template <typename T> void cg_init(const void* b, void* x, void* r, int64_t n, hipStream_t s);
template <typename T> void vcopy(const void* src, void* dst, int64_t n, const int* done, hipStream_t s);
template <typename T> void transpose(const void* in, void* out, int64_t rows, int64_t cols, hipStream_t s);
template <typename T> void rowdot_part(const void* a, const void* c, void* part, int64_t nrhs, int64_t M, int np, hipStream_t s);
template <typename T> void reduce_rows(const void* part, int np, int nrhs, void* out, hipStream_t s);
// rows of np > fold_groups threshold partials -> fold_groups(np) partials per RHS (0: no fold needed)
int fold_groups(int np);
template <typename T> void fold_rows(const void* part, int np, int nrhs, void* out, const int* done, hipStream_t s);
template <typename T> void cg_alpha(const void* part, int np, int nrhs, const void* rs, void* alpha, const int* done, hipStream_t s);
template <typename T> void cg_update_xr(void* x, void* r, const void* p, const void* Ap, const void* alpha, void* part,
                                        int64_t nrhs, int64_t M, const int* done, hipStream_t s);
template <typename T> void cg_check(const void* part, int np, int nrhs, double tol, void* rnew, int* done, int* iters,
                                    hipStream_t s);
template <typename T> void cg_beta(const void* part, int np, int nrhs, void* rs, void* beta, const int* done, hipStream_t s);
template <typename T> void cg_update_p(void* p, const void* z, const void* beta, int64_t nrhs, int64_t M, const int* done,
                                       hipStream_t s);
template <typename T> void cg_local_flag(const void* rnew, int nrhs, double tol, int* flag, hipStream_t s);
void cg_set_done(int* done, const int* flag, hipStream_t s);

}  // namespace hgp
