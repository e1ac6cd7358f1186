// hgp_kuf.hip — dense point-observation cross covariance Knm = k(x_n, u_m) on a gridded mesh
// (the PCG right-hand sides, `svi_gp.py:72` -> `kernels.py:73-79, 145-158`), written straight
// into the (B, M) row layout the solve reads.
//
// The reference forms the (B, M, D) broadcast x[:, None, :] - y[None, :, :] and reduces it
// (1.6 GB at C2's 32 x 1M, 13 GB per 200-observation minibatch at 4096^2).  Here one thread
// produces outputs directly: the mesh is (outer, inner) with inner = the last axis; a block
// owns one observation n and one outer index o (uniform per block, so the outer axes'
// squared differences are one scalar), threads stride the last axis.  Same per-element
// arithmetic and axis summation order as the reference, in the tensor dtype.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hipgp.h"

namespace hgp {

constexpr int KUF_THREADS = 256;
constexpr int KUF_PER_THREAD = 4;
constexpr int KUF_CHUNK = KUF_THREADS * KUF_PER_THREAD;

struct KufGrid {
  int d;
  int64_t m[3];
  const void* g[3];
};

// s: SqExp / Gneiting -> sum ((x - y) / ell)^2 ; Matern -> sum (x - y)^2   (as the reference)
__host__ __device__ inline bool scaled_dist(int kind) { return kind == HGP_KERN_SQEXP || kind == HGP_KERN_GNEITING; }

template <typename T>
__device__ __forceinline__ T kern_eval(int kind, T s, T sig2, T ell, T kp = (T)1) {
  if (kind == HGP_KERN_SQEXP) return sig2 * exp(-s / (T)2);
  const T r = sqrt(s);
  if (kind == HGP_KERN_MATERN12) return sig2 * exp(-r / ell);
  if (kind == HGP_KERN_MATERN32) {
    const T dp = (T)1.7320508075688772935 * r / ell;
    return sig2 * (((T)1 + dp) * exp(-dp));
  }
  if (kind == HGP_KERN_GNEITING) {   // kernels.py:108-117: r = t, kp = alpha, zero beyond t = 1
    const T pit = (T)3.14159265358979323846 * r;
    T c = ((T)1 - r) * cos(pit) + ((T)1 / (T)3.14159265358979323846) * sin(pit);
    c = pow((T)1 + pow(r, kp), (T)-3) * c;
    return r > (T)1 ? (T)0 * sig2 : sig2 * c;
  }
  const T dp = (T)2.2360679774997896964 * r / ell;       // Matern 5/2
  return sig2 * (((T)1 + dp + ((T)5 / (T)3) * s / (ell * ell)) * exp(-dp));
}

template <typename T>
__global__ __launch_bounds__(KUF_THREADS) void k_kuf_grid(KufGrid g, const T* __restrict__ x, int64_t B, int kind,
                                                         T sig2, T ell, T* __restrict__ out) {
  const int d = g.d;
  const int64_t inner = g.m[d - 1];
  const int64_t nchunk = (inner + KUF_CHUNK - 1) / KUF_CHUNK;
  int64_t outer = 1;
  for (int a = 0; a < d - 1; ++a) outer *= g.m[a];
  const int64_t bid = blockIdx.x;
  const int64_t chunk = bid % nchunk;
  const int64_t rest = bid / nchunk;
  const int64_t o = rest % outer;
  const int64_t n = rest / outer;
  if (n >= B) return;
  const bool sq = scaled_dist(kind);
  // outer axes: one scalar per block, summed in axis order (as the reference's sum over D)
  auto sqd = [&](int a, int64_t ia) -> T {
    T dv = x[n * d + a] - reinterpret_cast<const T*>(g.g[a])[ia];
    if (sq) dv = dv / ell;
    return dv * dv;
  };
  T so = 0;
  if (d == 2) so = sqd(0, o);
  if (d == 3) so = sqd(0, o / g.m[1]) + sqd(1, o % g.m[1]);
  const T xl = x[n * d + d - 1];
  const T* gl = reinterpret_cast<const T*>(g.g[d - 1]);
  T* orow = out + (n * outer + o) * inner;
#pragma unroll
  for (int k = 0; k < KUF_PER_THREAD; ++k) {
    const int64_t i = chunk * KUF_CHUNK + k * KUF_THREADS + threadIdx.x;
    if (i < inner) {
      T dv = xl - gl[i];
      if (sq) dv = dv / ell;
      const T s = (d == 1) ? dv * dv : so + dv * dv;
      orow[i] = kern_eval<T>(kind, s, sig2, ell);
    }
  }
}


// ---- line-integral (semi-integrated) cross covariance, SURVEY §8(f) row 2 -----------------
// Observation n is the segment from the origin to x_n; Knm[n, j] = |x_n| * int_0^1 k(u_j, a x_n) da.

// Monte-Carlo estimate of `Kernel.k_semi_mc` (kernels.py:19-39, transposed as svi_gp.py:61-64
// uses it): Knm[n, j] = |x_n| * (1/npts) sum_a k(u_j, alpha_a x_n), alpha_a = a/npts + u/npts.
// The reference builds the (M, nobs*npts, D) broadcast; here a block owns (n, outer index o):
// the sample points alpha_a x_n and their outer-axis squared distances are block constants in
// LDS, threads stride the last axis and sum the npts kernel values in registers.
constexpr int SEMI_MAX_NPTS = 1024;

template <typename T>
__global__ __launch_bounds__(KUF_THREADS) void k_kuf_semi_mc(KufGrid g, const T* __restrict__ x, int64_t B, int kind,
                                                            T sig2, T ell, T kp, int npts,
                                                            const T* __restrict__ u, T* __restrict__ out) {
  __shared__ T so_s[SEMI_MAX_NPTS];   // outer-axis sum of squared distances of sample a
  __shared__ T xl_s[SEMI_MAX_NPTS];   // last coordinate of sample a
  const int d = g.d;
  const int64_t inner = g.m[d - 1];
  const int64_t nchunk = (inner + KUF_CHUNK - 1) / KUF_CHUNK;
  int64_t outer = 1;
  for (int a = 0; a < d - 1; ++a) outer *= g.m[a];
  const int64_t bid = blockIdx.x;
  const int64_t chunk = bid % nchunk;
  const int64_t rest = bid / nchunk;
  const int64_t o = rest % outer;
  const int64_t n = rest / outer;
  if (n >= B) return;
  const bool sq = scaled_dist(kind);
  const T uoff = u[0] * (T)(1.0 / (double)npts);           // torch.rand(1) * delta
  for (int a = threadIdx.x; a < npts; a += KUF_THREADS) {
    const T al = (T)a / (T)npts + uoff;                      // arange(npts) / npts + rand * delta
    auto sqd = [&](int ax, int64_t ia) -> T {
      T dv = reinterpret_cast<const T*>(g.g[ax])[ia] - x[n * d + ax] * al;   // u - alpha x
      if (sq) dv = dv / ell;
      return dv * dv;
    };
    T so = 0;
    if (d == 2) so = sqd(0, o);
    if (d == 3) so = sqd(0, o / g.m[1]) + sqd(1, o % g.m[1]);
    so_s[a] = so;
    xl_s[a] = x[n * d + d - 1] * al;
  }
  __syncthreads();
  T xn2 = 0;
  for (int ax = 0; ax < d; ++ax) xn2 += x[n * d + ax] * x[n * d + ax];
  const T dist = sqrt(xn2);
  const T* gl = reinterpret_cast<const T*>(g.g[d - 1]);
  T* orow = out + (n * outer + o) * inner;
#pragma unroll
  for (int k = 0; k < KUF_PER_THREAD; ++k) {
    const int64_t i = chunk * KUF_CHUNK + k * KUF_THREADS + threadIdx.x;
    if (i < inner) {
      const T ui = gl[i];
      T acc = 0;
      for (int a = 0; a < npts; ++a) {
        T dv = ui - xl_s[a];
        if (sq) dv = dv / ell;
        const T s = (d == 1) ? dv * dv : so_s[a] + dv * dv;
        acc += kern_eval<T>(kind, s, sig2, ell, kp);
      }
      orow[i] = acc / (T)npts * dist;                        // mean(dim=-1) * dists
    }
  }
}

// Analytic SqExp line integral, `SqExp.k_semi` -> `semi_integrated_sqe` (kernels.py:80-85,
// 223-237) with Sinv = I / ell^2:  a = x S x, b = x S u, c = u S u, scale = sqrt(1/a),
// loc = b/a, Knm = sig2 exp(b^2/(2a) - c/2) sqrt(2 pi) scale (Phi(1) - Phi(0)) |x|, with the
// normal CDFs of ziggy/misc/stats.py:74-76.  Same formula and rounding steps; |x| = 0 gives
// NaN exactly where the reference does.
template <typename T>
__global__ __launch_bounds__(KUF_THREADS) void k_kuf_semi_sqexp(KufGrid g, const T* __restrict__ x, int64_t B,
                                                               T sig2, T ell, T* __restrict__ out) {
  const int d = g.d;
  const int64_t inner = g.m[d - 1];
  const int64_t nchunk = (inner + KUF_CHUNK - 1) / KUF_CHUNK;
  int64_t outer = 1;
  for (int a = 0; a < d - 1; ++a) outer *= g.m[a];
  const int64_t bid = blockIdx.x;
  const int64_t chunk = bid % nchunk;
  const int64_t rest = bid / nchunk;
  const int64_t o = rest % outer;
  const int64_t n = rest / outer;
  if (n >= B) return;
  const T sinv = (T)1 / (ell * ell);
  T xs[3], ua[3];
  T av = 0, xn2 = 0;
  int64_t oi[2] = {0, 0};
  if (d == 2) oi[0] = o;
  if (d == 3) { oi[0] = o / g.m[1]; oi[1] = o % g.m[1]; }
  for (int ax = 0; ax < d; ++ax) {
    const T xv = x[n * d + ax];
    xs[ax] = xv * sinv;                    // xintegrated @ Sinv
    av += xs[ax] * xv;
    xn2 += xv * xv;
    if (ax < d - 1) ua[ax] = reinterpret_cast<const T*>(g.g[ax])[oi[ax]];
  }
  T bo = 0, co = 0;                        // outer-axis terms of b and c, in axis order
  for (int ax = 0; ax < d - 1; ++ax) {
    bo += xs[ax] * ua[ax];
    co += (ua[ax] * sinv) * ua[ax];
  }
  const T xdist = sqrt(xn2);
  const T scale = sqrt((T)1 / av);
  const T sqrt2 = (T)1.4142135623730950488, sqrt2pi = (T)2.5066282746310005024;
  const T* gl = reinterpret_cast<const T*>(g.g[d - 1]);
  T* orow = out + (n * outer + o) * inner;
#pragma unroll
  for (int k = 0; k < KUF_PER_THREAD; ++k) {
    const int64_t i = chunk * KUF_CHUNK + k * KUF_THREADS + threadIdx.x;
    if (i < inner) {
      const T ui = gl[i];
      const T b = (d == 1) ? xs[0] * ui : bo + xs[d - 1] * ui;
      const T c = (d == 1) ? (ui * sinv) * ui : co + (ui * sinv) * ui;
      const T loc = b / av;
      const T coef = sig2 * exp((b * b) / ((T)2 * av) - c / (T)2) * sqrt2pi * scale;
      const T ca = (T)0.5 * ((T)1 + erf(((T)1 - loc) / (scale * sqrt2)));
      const T cb = (T)0.5 * ((T)1 + erf(((T)0 - loc) / (scale * sqrt2)));
      orow[i] = coef * (ca - cb) * xdist;
    }
  }
}

// Doubly-integrated diagonal by table interpolation, `KernelDoublyDiagInterpolator.forward`
// (kernels.py:200-220): r = |x / ell|, lo = #(r > grid) - 1 (-1 wraps to the last entry, as
// torch indexing does), knn[lo] + slopes[lo] (r - grid[lo]), times ell^2 sig2.
template <typename T>
__global__ __launch_bounds__(256) void k_doubly_diag(const T* __restrict__ x, int64_t B, int d, T sig2, T ell,
                                                    const T* __restrict__ tab, int N, T* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= B) return;
  T s = 0;
  for (int ax = 0; ax < d; ++ax) {
    const T v = x[n * d + ax] / ell;
    s += v * v;
  }
  const T r = sqrt(s);
  const T* grid = tab;
  const T* knn = tab + N;
  const T* slopes = tab + 2 * N;
  int lo = -1;
  for (int j = 0; j < N; ++j) lo += (r > grid[j]) ? 1 : 0;
  if (lo < 0) lo += N;
  const T iv = knn[lo] + slopes[lo] * (r - grid[lo]);
  out[n] = ell * ell * sig2 * iv;
}

hipError_t kuf_semi(int dtype, int kind, double kp, int ndim, const int64_t* m, const void* const* grids,
                    const void* x, int64_t nobs, double sig2, double ell, int npts, const void* u, void* out,
                    hipStream_t s) {
  KufGrid g{};
  g.d = ndim;
  int64_t outer = 1;
  for (int a = 0; a < ndim; ++a) {
    g.m[a] = m[a];
    g.g[a] = grids[a];
    if (a < ndim - 1) outer *= m[a];
  }
  const int64_t nchunk = (m[ndim - 1] + KUF_CHUNK - 1) / KUF_CHUNK;
  const int64_t nb = nobs * outer * nchunk;
  if (nb > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const bool mc = npts > 0;
  if (dtype == HGP_F32) {
    const float* xf = reinterpret_cast<const float*>(x);
    float* of = reinterpret_cast<float*>(out);
    if (mc)
      hipLaunchKernelGGL((k_kuf_semi_mc<float>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g, xf, nobs, kind,
                         (float)sig2, (float)ell, (float)kp, npts, reinterpret_cast<const float*>(u), of);
    else
      hipLaunchKernelGGL((k_kuf_semi_sqexp<float>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g, xf, nobs,
                         (float)sig2, (float)ell, of);
  } else {
    const double* xd = reinterpret_cast<const double*>(x);
    double* od = reinterpret_cast<double*>(out);
    if (mc)
      hipLaunchKernelGGL((k_kuf_semi_mc<double>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g, xd, nobs, kind,
                         sig2, ell, kp, npts, reinterpret_cast<const double*>(u), od);
    else
      hipLaunchKernelGGL((k_kuf_semi_sqexp<double>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g, xd, nobs, sig2,
                         ell, od);
  }
  return hipGetLastError();
}

hipError_t doubly_diag(int dtype, int ndim, const void* x, int64_t nobs, double sig2, double ell, const void* tab,
                       int N, void* out, hipStream_t s) {
  const unsigned nb = (unsigned)((nobs + 255) / 256);
  if (dtype == HGP_F32)
    hipLaunchKernelGGL((k_doubly_diag<float>), dim3(nb), dim3(256), 0, s, reinterpret_cast<const float*>(x), nobs,
                       ndim, (float)sig2, (float)ell, reinterpret_cast<const float*>(tab), N,
                       reinterpret_cast<float*>(out));
  else
    hipLaunchKernelGGL((k_doubly_diag<double>), dim3(nb), dim3(256), 0, s, reinterpret_cast<const double*>(x), nobs,
                       ndim, sig2, ell, reinterpret_cast<const double*>(tab), N, reinterpret_cast<double*>(out));
  return hipGetLastError();
}

// launcher behind hgp_kuf_grid (argument checks in hgp_api.hip)
hipError_t kuf_grid(int dtype, int kind, int ndim, const int64_t* m, const void* const* grids, const void* x,
                    int64_t nobs, double sig2, double ell, void* out, hipStream_t s) {
  KufGrid g{};
  g.d = ndim;
  int64_t outer = 1;
  for (int a = 0; a < ndim; ++a) {
    g.m[a] = m[a];
    g.g[a] = grids[a];
    if (a < ndim - 1) outer *= m[a];
  }
  const int64_t nchunk = (m[ndim - 1] + KUF_CHUNK - 1) / KUF_CHUNK;
  const int64_t nb = nobs * outer * nchunk;
  if (nb > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  if (dtype == HGP_F32)
    hipLaunchKernelGGL((k_kuf_grid<float>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g,
                       reinterpret_cast<const float*>(x), nobs, kind, (float)sig2, (float)ell,
                       reinterpret_cast<float*>(out));
  else
    hipLaunchKernelGGL((k_kuf_grid<double>), dim3((unsigned)nb), dim3(KUF_THREADS), 0, s, g,
                       reinterpret_cast<const double*>(x), nobs, kind, sig2, ell, reinterpret_cast<double*>(out));
  return hipGetLastError();
}

}  // namespace hgp
