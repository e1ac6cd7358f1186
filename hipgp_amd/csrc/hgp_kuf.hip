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

template <typename T>
__device__ __forceinline__ T kern_eval(int kind, T s, T sig2, T ell) {
  // s: SqExp -> sum ((x - y) / ell)^2 ; Matern -> sum (x - y)^2   (as the reference)
  if (kind == HGP_KERN_SQEXP) return sig2 * exp(-s / (T)2);
  const T r = sqrt(s);
  if (kind == HGP_KERN_MATERN12) return sig2 * exp(-r / ell);
  if (kind == HGP_KERN_MATERN32) {
    const T dp = (T)1.7320508075688772935 * r / ell;
    return sig2 * (((T)1 + dp) * exp(-dp));
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
  const bool sq = kind == HGP_KERN_SQEXP;
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
