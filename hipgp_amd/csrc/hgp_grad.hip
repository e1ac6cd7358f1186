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
// * gradient of <g, op v> w.r.t. the column through the operator's spectrum (D, 1/D or
//   D_sqrt = sqrt(clamp(Re FFT_n(embed(column)), cmin)), toeplitz_tensor.py:20-31; ops :70-125),
//   e.g. for R^T:  X[w] = sum_b sum_{j in m-grid} v_b[j] g_b[(j + w) mod n]   (n-grid, = dL/ds[w])
//   by one fp64 cross spectrum per RHS on the power-of-two grid (k_pack_pair, k_xspec_acc,
//   k_gather_n), then folded to the unique m-grid values (k_fold_div) and chained through the
//   DCT-I pair in hgp_api.hip.  The plan-based dqf (k_gather_flat) folds the d-D correlation
//   onto the flattened lags, so InvMatmul's column gradient is O(M log M) as well.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

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

// ---- FFT route: cross-correlations on the power-of-two grids --------------------------------
// corr[t] = sum_b sum_j v_b[j] h_b[j + t] is computed as IFFT_L(sum_b conj(V_b) H_b) on an L-grid
// large enough that the lags needed do not alias (L_K >= 2m - 1 for lags in (-m, m) with h on the
// m-grid; L_R >= n + m - 1 for lags [0, n) with h the n-periodic extension).  One complex fp64
// FFT per RHS: z = pad(v) + i h_ext, split by Hermitian symmetry.
struct LGeo {
  int d;
  int m[3], n[3], L[3];
};

// The FWD passes store frequency k of a length-L line at position pos_of(k): even k = 2s at s,
// odd k = 2s + 1 at L/2 + s (hgp_pass.hpp: the even / odd frequency halves).
__device__ __forceinline__ int pos_of(int k, int L) { return (k & 1) ? (L >> 1) + (k >> 1) : (k >> 1); }
__device__ __forceinline__ int freq_of(int s, int L) { return s < (L >> 1) ? 2 * s : 2 * (s - (L >> 1)) + 1; }

// L is 2^k or 3 * 2^k (the mixed-radix R lengths): index arithmetic by division, not masks
__device__ __forceinline__ void decodeL(int64_t f, const LGeo& G, int* c) {
  for (int a = G.d - 1; a >= 0; --a) {
    const int64_t q = f / G.L[a];
    c[a] = (int)(f - q * G.L[a]);
    f = q;
  }
}
// t mod L for t in (-L, 2L)
__device__ __forceinline__ int wrapL(int t, int L) { return t < 0 ? t + L : (t >= L ? t - L : t); }

// max |v| and max |h| of one RHS (finite values, as the bits of positive doubles) -> mx[0], mx[1]
// for pack_scale: h is packed with v at v's magnitude, so neither transform carries the other's
// rounding (the same reason as the set-up's K + i C^-1 grid, hgp_internal.hpp)
template <typename T>
__global__ void k_absmax2(const T* __restrict__ v, int64_t nv, const T* __restrict__ h, int64_t nh,
                          unsigned long long* mx) {
  double a = 0.0, b = 0.0;
  const int64_t n = nv > nh ? nv : nh;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < nv) { const double x = fabs((double)v[i]); if (isfinite(x)) a = fmax(a, x); }
    if (i < nh) { const double x = fabs((double)h[i]); if (isfinite(x)) b = fmax(b, x); }
  }
  __shared__ double sm[2][256 / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a = fmax(a, __shfl_xor(a, off, 64));
    b = fmax(b, __shfl_xor(b, off, 64));
  }
  if ((threadIdx.x & 63) == 0) { sm[0][threadIdx.x >> 6] = a; sm[1][threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { a = fmax(a, sm[0][w]); b = fmax(b, sm[1][w]); }
    atomicMax(mx, (unsigned long long)__double_as_longlong(a));
    atomicMax(mx + 1, (unsigned long long)__double_as_longlong(b));
  }
}

template <typename T>
__global__ void k_pack_pair(const T* __restrict__ v, const T* __restrict__ h, int h_periodic, LGeo G,
                            int64_t prodL, double2* __restrict__ z, const unsigned long long* mx) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= prodL) return;
  const double sc = pack_scale(mx);
  int c[3];
  decodeL(f, G, c);
  bool inm = true, inh = true;
  int64_t im = 0, ih = 0;
  for (int a = 0; a < G.d; ++a) {
    inm = inm && c[a] < G.m[a];
    im = im * G.m[a] + c[a];
    if (h_periodic) {
      inh = inh && c[a] < G.n[a] + G.m[a] - 1;
      ih = ih * G.n[a] + (c[a] >= G.n[a] ? c[a] - G.n[a] : c[a]);
    }
  }
  double2 r;
  r.x = inm ? (double)v[im] : 0.0;
  r.y = (h_periodic ? (inh ? (double)h[ih] : 0.0) : (inm ? (double)h[im] : 0.0)) * sc;
  z[f] = r;
}

// S (+)= conj(V) H with V = (Z + conj Z(-f)) / 2, H = (Z - conj Z(-f)) / 2i; Z in the FWD
// passes' stored order, S written in natural frequency order (the input of the inverse FFT)
__global__ void k_xspec_acc(const double2* __restrict__ Z, double2* __restrict__ S, LGeo G, int64_t prodL,
                            int first, const unsigned long long* mx) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= prodL) return;
  const double isc = 0.5 / pack_scale(mx);     // H was packed x pack_scale (exact power of two)
  int c[3];
  decodeL(f, G, c);
  int64_t nf = 0, fn = 0;
  for (int a = 0; a < G.d; ++a) {
    const int k = freq_of(c[a], G.L[a]);
    nf = nf * G.L[a] + pos_of(wrapL(G.L[a] - k, G.L[a]), G.L[a]);
    fn = fn * G.L[a] + k;
  }
  const double2 zf = Z[f], zn = Z[nf];
  const double vr = 0.5 * (zf.x + zn.x), vi = 0.5 * (zf.y - zn.y);      // V
  const double hr = isc * (zf.y + zn.y), hi = -isc * (zf.x - zn.x);     // H
  double2 p;
  p.x = vr * hr + vi * hi;                                              // conj(V) H
  p.y = vr * hi - vi * hr;
  if (!first) { const double2 o = S[fn]; p.x += o.x; p.y += o.y; }
  S[fn] = p;
}

__global__ void k_conj(double2* __restrict__ S, int64_t n) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f < n) S[f].y = -S[f].y;
}

// X[w] (n-grid) = sum of corr[t] over the lags t == w (mod n) of the window; F = FFT(conj S) in
// stored order, so corr[t] = Re F[pos_of(t mod L)] / prodL.  Window: [0, n) (periodic h) or (-m, m) (h on the m-grid).
__global__ void k_gather_n(const double2* __restrict__ F, LGeo G, int h_periodic, int64_t Mp, double invL,
                           double* __restrict__ X) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= Mp) return;
  int c[3] = {0, 0, 0};
  int64_t r = w;
  for (int a = G.d - 1; a >= 0; --a) { c[a] = (int)(r % G.n[a]); r /= G.n[a]; }
  int t[3][2], nt[3];
  for (int a = 0; a < G.d; ++a) {
    nt[a] = 0;
    if (h_periodic || c[a] < G.m[a]) t[a][nt[a]++] = c[a];
    if (!h_periodic && c[a] >= G.m[a] - 1) t[a][nt[a]++] = c[a] - G.n[a];
  }
  double s = 0.0;
  const int combos = 1 << G.d;
  for (int k = 0; k < combos; ++k) {
    int64_t idx = 0;
    bool ok = true;
    for (int a = 0; a < G.d; ++a) {
      const int sel = (k >> a) & 1;
      if (sel >= nt[a]) { ok = false; break; }
      idx = idx * G.L[a] + pos_of(wrapL(t[a][sel], G.L[a]), G.L[a]);
    }
    if (ok) s += F[idx].x;
  }
  X[w] = s * invL;
}

// dqf over the flattened m-grid from the d-D correlation C (lags (-m, m), corr = Re F / prodL):
// out[i] = sum over the signed-digit preimages a of i (flat(a) = i) of C[a] + C[-a]; out[0] = C[0]
template <typename T>
__global__ void k_gather_flat(const double2* __restrict__ F, LGeo G, int64_t M, double invL, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  double s = 0.0;
  const int combos = 1 << (G.d - 1);
  for (int k = 0; k < combos; ++k) {
    int64_t rem = i;
    int dig[3];
    bool ok = true;
    for (int a = G.d - 1; a >= 1; --a) {
      const int r = (int)(rem % G.m[a]);
      int64_t q = rem / G.m[a];
      if ((k >> (a - 1)) & 1) {            // borrow: digit r - m (needs r > 0)
        if (r == 0) { ok = false; break; }
        dig[a] = r - G.m[a];
        q += 1;
      } else {
        dig[a] = r;
      }
      rem = q;
    }
    if (!ok || rem >= G.m[0]) continue;
    dig[0] = (int)rem;
    int64_t ip = 0, in = 0;
    for (int a = 0; a < G.d; ++a) {
      ip = ip * G.L[a] + pos_of(wrapL(dig[a], G.L[a]), G.L[a]);
      in = in * G.L[a] + pos_of(wrapL(G.L[a] - dig[a], G.L[a]), G.L[a]);
    }
    s += i == 0 ? F[ip].x : F[ip].x + F[in].x;
  }
  out[i] = (T)(s * invL);
}


// ---- fp64 full-grid route of R / R^T (plans whose L_R lines exceed one CU's LDS in fp64) ------
// y = crop(IFFT(S' . FFT(pad x))) with the forward transforms of fwd_grid_f64 (stored order,
// pos_of per axis) and the inverse as conj(FFT(conj Y)) / N (the 1/N is in the stored S).
// z[f] = x at natural grid point f when inside the input extents (G.m), else 0
template <typename T>
__global__ void k_grid_embed(const T* __restrict__ x, LGeo G, int64_t prodL, double2* __restrict__ z,
                             const int* done) {
  if (done != nullptr && *done) return;
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= prodL) return;
  int c[3];
  decodeL(f, G, c);
  bool in = true;
  int64_t ix = 0;
  for (int a = 0; a < G.d; ++a) {
    in = in && c[a] < G.m[a];
    ix = ix * G.m[a] + c[a];
  }
  z[f] = make_double2(in ? (double)x[ix] : 0.0, 0.0);
}

// out[f] (natural order) = conj(F[pos(f)] S'[pos(f)]), S' = S (mode 0), conj(S) (1), Re S (2: the
// K spectrum of a packed K + i C^-1 transform) or Im S (3: the C^-1 spectrum)
__global__ void k_grid_mul_unperm(const double2* __restrict__ F, const double2* __restrict__ S, LGeo G,
                                  int64_t prodL, int mode, double2* __restrict__ out, const int* done) {
  if (done != nullptr && *done) return;
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= prodL) return;
  int c[3];
  decodeL(f, G, c);
  int64_t p = 0;
  for (int a = 0; a < G.d; ++a) p = p * G.L[a] + pos_of(c[a], G.L[a]);
  const double2 a = F[p];
  double2 w = S[p];
  if (mode == 1) w.y = -w.y;
  else if (mode == 2) w.y = 0.0;
  else if (mode == 3) w = make_double2(w.y, 0.0);
  out[f] = make_double2(a.x * w.x - a.y * w.y, -(a.x * w.y + a.y * w.x));
}

// y[j] (j over the output extents G.m) = Re Z[pos(j)]
template <typename T>
__global__ void k_grid_crop(const double2* __restrict__ Z, LGeo G, int64_t outM, T* __restrict__ y,
                            const int* done) {
  if (done != nullptr && *done) return;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= outM) return;
  int c[3] = {0, 0, 0};
  int64_t r = j;
  for (int a = G.d - 1; a >= 0; --a) { c[a] = (int)(r % G.m[a]); r /= G.m[a]; }
  int64_t p = 0;
  for (int a = 0; a < G.d; ++a) p = p * G.L[a] + pos_of(c[a], G.L[a]);
  y[j] = (T)Z[p].x;
}

__global__ void k_scale_copy(const double2* __restrict__ a, double2* __restrict__ b, int64_t n, double sc,
                             const unsigned long long* mx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = make_double2(a[i].x * sc, a[i].y * (sc / pack_scale(mx)));
}

// Line-batch helpers of the long-axis DCT (hgp_api.hip dct_axis: lines of L/2 > 8192 fp64 points
// go through fft_lines_f64's radix-2 levels instead of one CONVC pass).  Lines [O][.][I]: the
// position index at stride I, the I inner lines adjacent.
// E[o][j][i] = c[o][j][i] for j < m, 0 for m <= j < L
__global__ void k_line_embed(const double2* __restrict__ c, double2* __restrict__ E, int64_t O, int64_t m, int64_t I,
                             int64_t L) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * L * I) return;
  const int64_t i = t % I, rest = t / I;
  const int64_t j = rest % L, o = rest / L;
  E[t] = j < m ? c[(o * m + j) * I + i] : make_double2(0.0, 0.0);
}
// Z[o][f][i] (natural order f) = conj(X[o][pos(f)][i] f[pos(f)]): the filter product of the pass-order
// transform X, un-permuted and conjugated for the inverse as conj(FFT(conj .))
__global__ void k_line_mul_unperm_conj(const double2* __restrict__ X, const double2* __restrict__ flt,
                                       double2* __restrict__ Z, int64_t O, int64_t L, int64_t I) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * L * I) return;
  const int64_t i = t % I, rest = t / I;
  const int64_t f = rest % L, o = rest / L;
  const int64_t p = pos_of((int)f, (int)L);
  const double2 x = X[(o * L + p) * I + i], w = flt[p];
  Z[t] = make_double2(x.x * w.x - x.y * w.y, -(x.x * w.y + x.y * w.x));
}
// c[o][j][i] = conj(Y[o][pos(j)][i]) for j < m: IFFT(Z) = conj(FFT(conj Z)) (the 1/L is in the filter)
__global__ void k_line_unperm_conj(const double2* __restrict__ Y, double2* __restrict__ c, int64_t O, int64_t L,
                                   int64_t I, int64_t m) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * m * I) return;
  const int64_t i = t % I, rest = t / I;
  const int64_t j = rest % m, o = rest / m;
  const double2 y = Y[(o * L + pos_of((int)j, (int)L)) * I + i];
  c[t] = make_double2(y.x, -y.y);
}

LGeo make_lgeo(const GridDims& g) {
  LGeo G;
  G.d = g.d;
  for (int a = 0; a < 3; ++a) { G.m[a] = (int)g.m[a]; G.n[a] = (int)g.n[a]; G.L[a] = (int)g.L[a]; }
  return G;
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

void pack_pair(int dtype, const void* v, const void* h, int h_periodic, const GridDims& gd, int64_t prodL, double2* z,
               unsigned long long* mx, int64_t nv, int64_t nh, hipStream_t s) {
  const LGeo G = make_lgeo(gd);
  const int64_t n = nv > nh ? nv : nh;
  const unsigned nb = (unsigned)std::min<int64_t>(1024, (n + 255) / 256);
  (void)hipMemsetAsync(mx, 0, 2 * sizeof(unsigned long long), s);
  if (dtype == 1) {
    k_absmax2<double><<<nb, 256, 0, s>>>((const double*)v, nv, (const double*)h, nh, mx);
    k_pack_pair<double><<<nblk(prodL, 256), 256, 0, s>>>((const double*)v, (const double*)h, h_periodic, G, prodL, z, mx);
  } else {
    k_absmax2<float><<<nb, 256, 0, s>>>((const float*)v, nv, (const float*)h, nh, mx);
    k_pack_pair<float><<<nblk(prodL, 256), 256, 0, s>>>((const float*)v, (const float*)h, h_periodic, G, prodL, z, mx);
  }
}

void xspec_acc(const double2* Z, double2* S, const GridDims& gd, int64_t prodL, int first, const unsigned long long* mx,
               hipStream_t s) {
  k_xspec_acc<<<nblk(prodL, 256), 256, 0, s>>>(Z, S, make_lgeo(gd), prodL, first, mx);
}

void conj_inplace(double2* S, int64_t n, hipStream_t s) { k_conj<<<nblk(n, 256), 256, 0, s>>>(S, n); }

void gather_n(const double2* F, const GridDims& gd, int h_periodic, int64_t Mp, double invL, double* X, hipStream_t s) {
  k_gather_n<<<nblk(Mp, 256), 256, 0, s>>>(F, make_lgeo(gd), h_periodic, Mp, invL, X);
}

void gather_flat(int dtype, const double2* F, const GridDims& gd, int64_t M, double invL, void* out, hipStream_t s) {
  const LGeo G = make_lgeo(gd);
  if (dtype == 1) k_gather_flat<double><<<nblk(M, 256), 256, 0, s>>>(F, G, M, invL, (double*)out);
  else k_gather_flat<float><<<nblk(M, 256), 256, 0, s>>>(F, G, M, invL, (float*)out);
}

void grid_embed(int dtype, const void* x, const GridDims& gd, int64_t prodL, double2* z, hipStream_t s,
                const int* done) {
  const LGeo G = make_lgeo(gd);
  if (dtype == 1) k_grid_embed<double><<<nblk(prodL, 256), 256, 0, s>>>((const double*)x, G, prodL, z, done);
  else k_grid_embed<float><<<nblk(prodL, 256), 256, 0, s>>>((const float*)x, G, prodL, z, done);
}

void grid_mul_unperm(const double2* F, const double2* S, const GridDims& gd, int64_t prodL, int mode,
                     double2* out, hipStream_t s, const int* done) {
  k_grid_mul_unperm<<<nblk(prodL, 256), 256, 0, s>>>(F, S, make_lgeo(gd), prodL, mode, out, done);
}

void grid_crop(int dtype, const double2* Z, const GridDims& gd, int64_t outM, void* y, hipStream_t s,
               const int* done) {
  const LGeo G = make_lgeo(gd);
  if (dtype == 1) k_grid_crop<double><<<nblk(outM, 256), 256, 0, s>>>(Z, G, outM, (double*)y, done);
  else k_grid_crop<float><<<nblk(outM, 256), 256, 0, s>>>(Z, G, outM, (float*)y, done);
}

void line_embed(const double2* c, double2* E, int64_t O, int64_t m, int64_t I, int64_t L, hipStream_t s) {
  k_line_embed<<<nblk(O * L * I, 256), 256, 0, s>>>(c, E, O, m, I, L);
}
void line_mul_unperm_conj(const double2* X, const double2* f, double2* Z, int64_t O, int64_t L, int64_t I,
                          hipStream_t s) {
  k_line_mul_unperm_conj<<<nblk(O * L * I, 256), 256, 0, s>>>(X, f, Z, O, L, I);
}
void line_unperm_conj(const double2* Y, double2* c, int64_t O, int64_t L, int64_t I, int64_t m, hipStream_t s) {
  k_line_unperm_conj<<<nblk(O * m * I, 256), 256, 0, s>>>(Y, c, O, L, I, m);
}

void scale_copy(const double2* a, double2* b, int64_t n, double sc, hipStream_t s, const unsigned long long* mx) {
  k_scale_copy<<<nblk(n, 256), 256, 0, s>>>(a, b, n, sc, mx);
}

}  // namespace hgp
