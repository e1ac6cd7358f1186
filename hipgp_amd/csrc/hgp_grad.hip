// hgp_grad.hip — backward of the solve and of the whitening w.r.t. the Toeplitz column
// (SURVEY §8(f) row 4).
//
// * k_dqf: gpytorch's sym_toeplitz_derivative_quadratic_form (reference
//   ziggy/misc/gpt_toeplitz.py:169-209, called by InvMatmul.backward _inv_matmul.py:52-60):
//     out[i] = sum_j sum_k u_j[k] (v_j[k+i] + v_j[k-i])  (i >= 1),   out[0] = sum_j u_j . v_j
//   over the FLATTENED column (the reference applies the 1-D rule to the multi-D column).
//   Direct lagged sums, O(nvec * n^2): a block owns 256 lags, u and the two v windows of a
//   256-wide k tile are staged in LDS (u read as a broadcast, the windows conflict-free), partial
//   sums per tile in T, tiles accumulated in fp64.  Deterministic (fixed order).
// * k_circ_xcorr + fold/mask/scale helpers: gradient of <g, op v> w.r.t. the column through the
//   operator's spectrum (D, 1/D or D_sqrt = sqrt(clamp(Re FFT_n(embed(column)), cmin)),
//   toeplitz_tensor.py:20-31; ops :70-125), e.g. for R^T:
//     X[w]   = sum_b sum_{j in m-grid} v_b[j] g_b[(j + w) mod n]         (n-grid, = dL/ds[w])
//   then folded to the unique m-grid values and chained through the DCT-I pair in hgp_api.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hgp_internal.hpp"

namespace hgp {
namespace {

constexpr int GT = 256;   // lags per block / k tile width

template <typename T>
__global__ __launch_bounds__(GT) void k_dqf(const T* __restrict__ u, const T* __restrict__ v, int64_t nvec,
                                            int64_t n, T* __restrict__ out) {
  __shared__ T su[GT];
  __shared__ T sa[2 * GT];   // sa[q] = v[k0 + i0 + q]
  __shared__ T sb[2 * GT];   // sb[q] = v[k0 - i0 - (GT - 1) + q]
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * GT;
  double acc = 0.0;
  for (int64_t j = 0; j < nvec; ++j) {
    const T* uj = u + j * n;
    const T* vj = v + j * n;
    for (int64_t k0 = 0; k0 < n; k0 += GT) {
      // tiles contributing to neither term are skipped (uniform over the block)
      if (k0 + i0 >= n && k0 + GT <= i0) continue;
      __syncthreads();
      su[t] = (k0 + t < n) ? uj[k0 + t] : T(0);
      for (int q = t; q < 2 * GT; q += GT) {
        const int64_t a = k0 + i0 + q;
        const int64_t b = k0 - i0 - (GT - 1) + q;
        sa[q] = (a < n) ? vj[a] : T(0);
        sb[q] = (b >= 0 && b < n) ? vj[b] : T(0);
      }
      __syncthreads();
      T s = 0;
#pragma unroll 8
      for (int kk = 0; kk < GT; ++kk) s += su[kk] * (sa[kk + t] + sb[kk - t + GT - 1]);
      acc += (double)s;
    }
  }
  const int64_t i = i0 + t;
  // lag 0: both terms are u.v, the reference subtracts one copy (gpt_toeplitz.py:207)
  if (i < n) out[i] = (T)(i == 0 ? 0.5 * acc : acc);
}

struct Geo {
  int d;
  int m[3], n[3];
};

__device__ __forceinline__ void decode(int64_t f, const int* ext, int d, int* c) {
  for (int a = d - 1; a >= 0; --a) {
    c[a] = (int)(f % ext[a]);
    f /= ext[a];
  }
}

// X[w] = sum_b sum_j v_b[j] g_b[(j + w) mod n], w over the n-grid; thread per w, j tiles in LDS.
// g rows live on the n-grid, or (g_on_m) on the m-grid, zero outside it (the K / C^-1 crop).
template <typename T>
__global__ __launch_bounds__(GT) void k_circ_xcorr(const T* __restrict__ v, const T* __restrict__ g, int64_t nrhs,
                                                   int64_t M, int64_t Mp, Geo G, int g_on_m,
                                                   double* __restrict__ X) {
  __shared__ T sv[GT];
  __shared__ int sj[3][GT];
  const int t = threadIdx.x;
  const int64_t w = (int64_t)blockIdx.x * GT + t;
  int wc[3] = {0, 0, 0};
  decode(w < Mp ? w : 0, G.n, G.d, wc);
  double acc = 0.0;
  for (int64_t b = 0; b < nrhs; ++b) {
    const T* vb = v + b * M;
    const T* gb = g + b * (g_on_m ? M : Mp);
    for (int64_t j0 = 0; j0 < M; j0 += GT) {
      __syncthreads();
      const int64_t j = j0 + t;
      int jc[3] = {0, 0, 0};
      if (j < M) decode(j, G.m, G.d, jc);
      sv[t] = (j < M) ? vb[j] : T(0);
      sj[0][t] = jc[0]; sj[1][t] = jc[1]; sj[2][t] = jc[2];
      __syncthreads();
      const int cnt = (int)((M - j0) < GT ? (M - j0) : GT);
      T s = 0;
      for (int q = 0; q < cnt; ++q) {
        int64_t idx = 0;
        bool in = true;
        for (int a = 0; a < G.d; ++a) {
          int e = sj[a][q] + wc[a];
          if (e >= G.n[a]) e -= G.n[a];
          const int ext = g_on_m ? G.m[a] : G.n[a];
          in = in && e < ext;
          idx = idx * ext + e;
        }
        if (in) s += sv[q] * gb[idx];
      }
      acc += (double)s;
    }
  }
  if (w < Mp) X[w] = acc;
}

__device__ __forceinline__ double mu_of(const int* c, const Geo& G) {
  double mu = 1.0;
  for (int a = 0; a < G.d; ++a)
    if (c[a] != 0 && c[a] != G.m[a] - 1) mu *= 2.0;
  return mu;
}

// y[x] = (sum over the n-grid images of x of X) / mu(x), x over the m-grid
__global__ void k_fold_div(const double* __restrict__ X, int64_t M, Geo G, double* __restrict__ y) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= M) return;
  int c[3] = {0, 0, 0};
  decode(x, G.m, G.d, c);
  const int nimg = 1 << G.d;
  double s = 0.0;
  for (int mask = 0; mask < nimg; ++mask) {
    bool dup = false;
    int64_t idx = 0;
    for (int a = 0; a < G.d; ++a) {
      int e = c[a];
      if (mask & (1 << a)) {
        if (c[a] == 0 || c[a] == G.m[a] - 1) dup = true;   // its own mirror image
        e = G.n[a] - c[a];
      }
      idx = idx * G.n[a] + e;
    }
    if (!dup) s += X[idx];
  }
  y[x] = s / mu_of(c, G);
}

// y[x] *= dS/dD at x for the operator's spectrum S (K: D, C^-1: 1/D, R/R^T: sqrt D) where D
// passed the clamp (torch.clamp's gradient mask), else 0.  D3 = [D | 1/D | sqrt D].
__global__ void k_spec_bwd(double* __restrict__ y, const double* __restrict__ D3, int64_t M, int kind,
                           double cmin) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= M) return;
  const double D = D3[x];
  double f = 1.0;
  if (kind == 1) f = -D3[M + x] * D3[M + x];
  else if (kind == 2) f = 0.5 / D3[2 * M + x];
  y[x] = D > cmin ? y[x] * f : 0.0;
}

template <typename T>
__global__ void k_mul_mu_out(const double* __restrict__ r, int64_t M, Geo G, T* __restrict__ out) {
  const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= M) return;
  int c[3] = {0, 0, 0};
  decode(x, G.m, G.d, c);
  out[x] = (T)(r[x] * mu_of(c, G));
}

Geo make_geo(const GridDims& g) {
  Geo G;
  G.d = g.d;
  for (int a = 0; a < 3; ++a) { G.m[a] = (int)g.m[a]; G.n[a] = (int)g.n[a]; }
  return G;
}

inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t sym_toeplitz_dqf(int dtype, const void* u, const void* v, int64_t nvec, int64_t n, void* out,
                            hipStream_t s) {
  if (dtype == 1)
    k_dqf<double><<<nblk(n, GT), GT, 0, s>>>((const double*)u, (const double*)v, nvec, n, (double*)out);
  else
    k_dqf<float><<<nblk(n, GT), GT, 0, s>>>((const float*)u, (const float*)v, nvec, n, (float*)out);
  return hipGetLastError();
}

hipError_t circ_xcorr(int dtype, const void* v, const void* g, int g_on_m, int64_t nrhs, const GridDims& gd,
                      int64_t M, int64_t Mp, double* X, hipStream_t s) {
  const Geo G = make_geo(gd);
  if (dtype == 1)
    k_circ_xcorr<double><<<nblk(Mp, GT), GT, 0, s>>>((const double*)v, (const double*)g, nrhs, M, Mp, G, g_on_m, X);
  else
    k_circ_xcorr<float><<<nblk(Mp, GT), GT, 0, s>>>((const float*)v, (const float*)g, nrhs, M, Mp, G, g_on_m, X);
  return hipGetLastError();
}

void fold_div_mu(const double* X, int64_t M, const GridDims& gd, double* y, hipStream_t s) {
  k_fold_div<<<nblk(M, 256), 256, 0, s>>>(X, M, make_geo(gd), y);
}

void spec_bwd(double* y, const double* D3, int64_t M, int kind, double cmin, hipStream_t s) {
  k_spec_bwd<<<nblk(M, 256), 256, 0, s>>>(y, D3, M, kind, cmin);
}

void mul_mu_out(int dtype, const double* r, int64_t M, const GridDims& gd, void* out, hipStream_t s) {
  if (dtype == 1) k_mul_mu_out<double><<<nblk(M, 256), 256, 0, s>>>(r, M, make_geo(gd), (double*)out);
  else k_mul_mu_out<float><<<nblk(M, 256), 256, 0, s>>>(r, M, make_geo(gd), (float*)out);
}

}  // namespace hgp
