// hgp_kernels.hip — pass dispatch, spectrum-setup kernels and batched-CG kernels.
#include <algorithm>

#include "hgp_internal.hpp"

namespace hgp {

// ------------------------------------------------------------------------------------------
// spectrum setup (fp64)
// ------------------------------------------------------------------------------------------

// Partial DFT of the length-n even extension by Bluestein's chirp-z identity
//   X[k] = sum_{t<m} a_t W^{tk} = W^{k^2/2} sum_t (a_t W^{t^2/2}) W^{-(k-t)^2/2},  W = e^{-2 pi i/n},
// so the DCT-I D[k] = Re sum_t w_t c_t W^{tk} (w = 1 at t = 0, m-1, else 2) is a chirp
// pre-multiply, a linear convolution with the chirp filter (taps k-t in (-m, m): any FFT length
// L >= 2m-1, the operator length L_K, hgp_pass CONVC) and a chirp post-multiply.  fp64.
// pre[t] = w_t e^{-i pi t^2/n}, post[k] = e^{-i pi k^2/n}; angles reduced exactly (t^2 mod 2n).
__global__ void k_chirp_tables(double2* __restrict__ pre, double2* __restrict__ post, int64_t m, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m) return;
  const double ang = (double)((t * t) % (2 * n)) / (double)n;    // in units of pi
  double sv, cv;
  sincospi(ang, &sv, &cv);
  const double w = (t == 0 || t == m - 1) ? 1.0 : 2.0;
  pre[t] = make_double2(w * cv, -w * sv);
  post[t] = make_double2(cv, -sv);
}

// filter h[u] = scale * e^{+i pi u^2/n} on the L-grid: u in [0, m) and L - u for u in [1, m)
__global__ void k_chirp_filter(double2* __restrict__ h, int64_t m, int64_t n, int64_t L, double scale) {
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= L) return;
  int64_t v = -1;
  if (u < m) v = u;
  else if (u > L - m) v = L - u;
  double2 r = make_double2(0.0, 0.0);
  if (v >= 0) {
    double sv, cv;
    sincospi((double)((v * v) % (2 * n)) / (double)n, &sv, &cv);
    r = make_double2(scale * cv, scale * sv);
  }
  h[u] = r;
}

// c[j] = x[j] * pre[t(j)], t = (j / I) mod m  (real in, complex out)
__global__ void k_chirp_pre(const double* __restrict__ x, const double2* __restrict__ pre, double2* __restrict__ c,
                            int64_t total, int64_t m, int64_t I) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const double2 w = pre[(j / I) % m];
  const double v = x[j];
  c[j] = make_double2(v * w.x, v * w.y);
}

// y[j] = scale * Re(c[j] * post[k(j)])
__global__ void k_chirp_post(const double2* __restrict__ c, const double2* __restrict__ post, double* __restrict__ y,
                             int64_t total, int64_t m, int64_t I, double scale) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const double2 w = post[(j / I) % m];
  const double2 v = c[j];
  y[j] = scale * (v.x * w.x - v.y * w.y);
}

void chirp_tables(double2* pre, double2* post, int64_t m, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_chirp_tables, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, pre, post, m, n);
}
void chirp_filter(double2* h, int64_t m, int64_t n, int64_t L, double scale, hipStream_t s) {
  hipLaunchKernelGGL(k_chirp_filter, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, s, h, m, n, L, scale);
}
void chirp_pre(const double* x, const double2* pre, double2* c, int64_t total, int64_t m, int64_t I, hipStream_t s) {
  hipLaunchKernelGGL(k_chirp_pre, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, x, pre, c, total, m, I);
}
void chirp_post(const double2* c, const double2* post, double* y, int64_t total, int64_t m, int64_t I, double scale,
                hipStream_t s) {
  hipLaunchKernelGGL(k_chirp_post, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, c, post, y, total, m, I,
                     scale);
}

template <typename T>
__global__ void k_to_f64(const T* __restrict__ src, double* __restrict__ dst, int64_t n, double add0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (double)src[i] + (i == 0 ? add0 : 0.0);
}

template <typename T>
void to_f64(const void* src, double* dst, int64_t n, double add0, hipStream_t s) {
  hipLaunchKernelGGL((k_to_f64<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const T*)src, dst, n, add0);
}
template void to_f64<float>(const void*, double*, int64_t, double, hipStream_t);
template void to_f64<double>(const void*, double*, int64_t, double, hipStream_t);

// D = max(Draw, clamp); write [D | 1/D | sqrt(D)] (3 x M) and count clamped entries; the
// maxima of D and 1/D (pack_scale) by a grid-stride sweep of <= 1024 blocks, one atomic each per
// block (one per 256 elements serialised on two words: 97 us at 1M elements)
// The m-grid holds the DCT-I half spectrum: entry (k_0, .., k_{d-1}) stands for prod_a w(k_a)
// eigenvalues of the circulant (w = 1 at k = 0 and k = m - 1, else 2: the mirror n - k), so the
// count is the number of clamped eigenvalues of the full expanded spectrum the reference clamps.
__global__ void k_clamp(const double* __restrict__ Draw, double* __restrict__ out3, int64_t M, double clamp_min,
                        unsigned long long* nclamp, GridDims g) {
  double a = 0.0, b = 0.0;
  unsigned long long nc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    double d = Draw[i];
    if (!(d >= clamp_min)) {    // torch.clamp(min=) semantics: values below min (NaN stays NaN)
      if (d < clamp_min) {
        d = clamp_min;
        unsigned long long w = 1;
        int64_t r = i;
        for (int ax = g.d - 1; ax >= 0; --ax) {
          const int64_t k = r % g.m[ax];
          r /= g.m[ax];
          if (k != 0 && k != g.m[ax] - 1) w *= 2;
        }
        nc += w;
      }
    }
    out3[i] = d;
    out3[M + i] = 1.0 / d;
    out3[2 * M + i] = sqrt(d);
    if (d > 0.0 && isfinite(d)) a = fmax(a, d);
    if (d > 0.0 && isfinite(1.0 / d)) b = fmax(b, 1.0 / d);
  }
  __shared__ double smx[2][256 / 64];
  __shared__ unsigned long long snc[256 / 64];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a = fmax(a, __shfl_xor(a, off, 64));
    b = fmax(b, __shfl_xor(b, off, 64));
    nc += __shfl_xor(nc, off, 64);
  }
  if ((threadIdx.x & 63) == 0) { smx[0][threadIdx.x >> 6] = a; smx[1][threadIdx.x >> 6] = b; snc[threadIdx.x >> 6] = nc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { a = fmax(a, smx[0][w]); b = fmax(b, smx[1][w]); nc += snc[w]; }
    if (nc) atomicAdd(nclamp, nc);
    atomicMax(nclamp + 1, (unsigned long long)__double_as_longlong(a));
    atomicMax(nclamp + 2, (unsigned long long)__double_as_longlong(b));
  }
}

void clamp_spectrum(const double* Draw, double* out3, int64_t M, double clamp_min, unsigned long long* nclamp,
                    const GridDims& g, hipStream_t s) {
  const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(1024, (M + 255) / 256));
  hipLaunchKernelGGL(k_clamp, dim3((unsigned)nb), dim3(256), 0, s, Draw, out3, M, clamp_min, nclamp, g);
}

// K-type embedding (L >= 2m-1): G[u] = c[|t|], t = u (u < m) or u - L (u > L - m); complex
// pair (re = cK, im = cInv).
__global__ void k_embed_K(const double* __restrict__ cK, const double* __restrict__ cI, double2* __restrict__ out,
                          GridDims g, int64_t total, const unsigned long long* mx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const double sc = pack_scale(mx);
  int64_t rem = idx, src = 0, mstride = 1;
  bool ok = true;
  for (int a = g.d - 1; a >= 0; --a) {
    const int64_t u = rem % g.L[a];
    rem /= g.L[a];
    int64_t t;
    if (u < g.m[a]) t = u;
    else if (u > g.L[a] - g.m[a]) t = g.L[a] - u;
    else { ok = false; t = 0; }
    src += t * mstride;
    mstride *= g.m[a];
  }
  double2 v;
  v.x = ok ? cK[src] : 0.0;
  v.y = ok ? cI[src] * sc : 0.0;
  out[idx] = v;
}

// R-type embedding (L >= n + m - 1): filter s_per(t) on t in [-(m-1), n-1], s_per even and
// n-periodic, unique values s[0..m-1].
__global__ void k_embed_R(const double* __restrict__ s, double2* __restrict__ out, GridDims g, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int64_t rem = idx, src = 0, mstride = 1;
  bool ok = true;
  for (int a = g.d - 1; a >= 0; --a) {
    const int64_t u = rem % g.L[a];
    rem /= g.L[a];
    const int64_t m = g.m[a], n = g.n[a], L = g.L[a];
    int64_t t;
    if (u < n) t = (u <= m - 1) ? u : n - u;
    else if (u >= L - m + 1) t = L - u;
    else { ok = false; t = 0; }
    src += t * mstride;
    mstride *= m;
  }
  double2 v;
  v.x = ok ? s[src] : 0.0;
  v.y = 0.0;
  out[idx] = v;
}

// Radix-2 step of fft_lines_f64: the two interleaved half-length subsequences of every line
// (e = 0, 1 at offsets e * ps, positions at 2 ps) hold their length-L/2 spectra in pass order;
// X[f] = E[f'] +- W_L^f' O[f'] (f' = f mod L/2), written in the pass order of length L.
__global__ void k_r2_combine(const double2* __restrict__ in, double2* __restrict__ out, int64_t L, int64_t Rn,
                             int64_t r_stride, int64_t In, int64_t ps, const double2* __restrict__ tw,
                             const int* done) {
  if (done != nullptr && *done) return;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t half_len = L / 2, Hp = L / 4;
  if (t >= Rn * In * half_len) return;
  const int64_t i = t % In, rest = t / In;
  const int64_t idx = rest % half_len, r = rest / half_len;
  const int64_t base = r * r_stride + i;
  const int64_t hp = idx / Hp, kp = idx - hp * Hp;
  const int64_t f = 2 * kp + hp;
  const double2 E = in[base + (2 * idx) * ps];
  const double2 O = in[base + (2 * idx + 1) * ps];
  const double2 w = tw[f];
  const double2 wo = make_double2(w.x * O.x - w.y * O.y, w.x * O.y + w.y * O.x);
  const int64_t oa = hp * half_len + kp;
  out[base + oa * ps] = make_double2(E.x + wo.x, E.y + wo.y);
  out[base + (oa + half_len / 2) * ps] = make_double2(E.x - wo.x, E.y - wo.y);
}
void r2_combine(const double2* in, double2* out, int64_t L, int64_t Rn, int64_t r_stride, int64_t In, int64_t ps,
                const double2* tw, hipStream_t s, const int* done) {
  const int64_t total = Rn * In * (L / 2);
  hipLaunchKernelGGL(k_r2_combine, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, out, L, Rn, r_stride, In,
                     ps, tw, done);
}

// the same R filter as a REAL grid (the set-up transforms it with the real row-pair pass)
__global__ void k_embed_R_real(const double* __restrict__ s, double* __restrict__ out, GridDims g, int64_t total,
                               int sym) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int64_t rem = idx, src = 0, mstride = 1;
  bool ok = true;
  for (int a = g.d - 1; a >= 0; --a) {
    const int64_t u = rem % g.L[a];
    rem /= g.L[a];
    const int64_t m = g.m[a], n = g.n[a], L = g.L[a];
    int64_t t;
    // the n-periodic even filter r[j] (r[j] = s[j], j < m; s[n - j] above) at offsets (-m, n), or
    // with `sym` at (-n, n): the extra offsets (-n, -m] are never read by outputs j < n
    if (u < n) t = (u <= m - 1) ? u : n - u;
    else if (u >= L - (sym ? n : m) + 1) { const int64_t j = L - u; t = (j <= m - 1) ? j : n - j; }
    else { ok = false; t = 0; }
    src += t * mstride;
    mstride *= m;
  }
  out[idx] = ok ? s[src] : 0.0;
}
void embed_R_real(const double* sv, double* out, const GridDims& g, int sym, hipStream_t s) {
  int64_t total = 1;
  for (int a = 0; a < g.d; ++a) total *= g.L[a];
  hipLaunchKernelGGL(k_embed_R_real, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sv, out, g, total, sym);
}

void embed_K(const double* cK, const double* cI, double2* out, const GridDims& g, const unsigned long long* mx,
             hipStream_t s) {
  int64_t total = 1;
  for (int a = 0; a < g.d; ++a) total *= g.L[a];
  hipLaunchKernelGGL(k_embed_K, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, cK, cI, out, g, total, mx);
}
void embed_R(const double* sv, double2* out, const GridDims& g, hipStream_t s) {
  int64_t total = 1;
  for (int a = 0; a < g.d; ++a) total *= g.L[a];
  hipLaunchKernelGGL(k_embed_R, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, sv, out, g, total);
}

// Spectrum extraction from the full permuted-order FFT grid F (outer x L_last complex) into
// the layout the passes read: when `compact`, the last axis keeps only the S >= H+1 "compact"
// half-spectrum columns c (even frequency 2c for c <= H/2, odd 2(c-H/2-1)+1 after; zero pad
// beyond H) — the real-data passes store exactly these columns.
__device__ __forceinline__ int64_t spec_src(int64_t idx, int64_t L, int64_t S, int compact, int64_t L0t,
                                            int64_t L1t) {
  if (!compact) return idx;
  int64_t o, c;
  const int64_t H = L / 2;
  if (L0t > 0 && L1t > 0) {                               // 3-D transposed: [c][k1][k0]
    const int64_t k0 = idx % L0t, rest = idx / L0t;
    const int64_t k1 = rest % L1t;
    c = rest / L1t;
    o = k0 * L1t + k1;
  } else if (L0t > 0) { c = idx / L0t; o = idx - c * L0t; }   // 2-D transposed: [c][k0], k0 < L0t
  else { o = idx / S; c = idx - o * S; }
  if (c > H) return -1;
  const int64_t kp = (c <= H / 2) ? c : H + (c - H / 2 - 1);
  return o * L + kp;
}

template <typename T>
__global__ void k_extract_pair(const double2* __restrict__ F, T* __restrict__ a, T* __restrict__ b, int64_t n,
                               int64_t L, int64_t S, int compact, double scale, int64_t L0t, int64_t L1t,
                               const unsigned long long* mx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t src = spec_src(i, L, S, compact, L0t, L1t);
  const double2 f = src >= 0 ? F[src] : make_double2(0.0, 0.0);
  a[i] = (T)(f.x * scale);
  b[i] = (T)(f.y * (scale / pack_scale(mx)));
}
template <typename T>
__global__ void k_extract_cplx(const double2* __restrict__ F, C2<T>* __restrict__ o, int64_t n, int64_t L, int64_t S,
                               int compact, double scale, int64_t L0t, int64_t L1t) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t src = spec_src(i, L, S, compact, L0t, L1t);
  const double2 f = src >= 0 ? F[src] : make_double2(0.0, 0.0);
  o[i] = mk<T>((T)(f.x * scale), (T)(f.y * scale));
}
// L0t > 0: 2-D transposed layout [compact column c][axis-0 frequency k0 < L0t] read by the
// column pass of the column-major intermediate (hgp_rows.hpp); L0t, L1t > 0: 3-D
// [c][k1 < L1t][k0 < L0t], read by the contiguous axis-0 pass of the 3-D sequence
// (hgp_lines.hpp); else [outer][c] with pitch S.
template <typename T>
void extract_pair(const double2* F, void* a, void* b, int64_t n, int64_t L, int64_t S, int compact, double scale,
                  hipStream_t s, int64_t L0t, int64_t L1t, const unsigned long long* mx) {
  hipLaunchKernelGGL((k_extract_pair<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, (T*)a, (T*)b, n, L, S,
                     compact, scale, L0t, L1t, mx);
}
template <typename T>
void extract_cplx(const double2* F, void* o, int64_t n, int64_t L, int64_t S, int compact, double scale, hipStream_t s,
                  int64_t L0t, int64_t L1t) {
  hipLaunchKernelGGL((k_extract_cplx<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, (C2<T>*)o, n, L, S,
                     compact, scale, L0t, L1t);
}
// Transposing spectrum extraction for d >= 2 through 32 x 32 LDS tiles (both the grid reads
// and the spectrum writes are contiguous): source F[(k0 * L1 + k1) * Ssrc + col] (col = c for
// a compact source from the real row-pair transform, else the permuted-order position of
// compact column c), destination [c][k1][k0] (2-D: L1 = 1, [c][k0]), c < NC = H + 1.
template <typename T, bool PAIR>
__global__ __launch_bounds__(256) void k_extract_t(const double2* __restrict__ F, T* __restrict__ a,
                                                   T* __restrict__ b, int64_t L0, int64_t L1, int64_t NC,
                                                   int64_t Ssrc, int compact_src, int64_t H, double scale,
                                                   const unsigned long long* mx) {
  __shared__ double2 tile[32][33];
  const double scale_b = scale / pack_scale(mx);
  const int64_t k1 = blockIdx.z;
  const int64_t c0 = (int64_t)blockIdx.x * 32, k00 = (int64_t)blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int j = ty; j < 32; j += 8) {
    const int64_t k0 = k00 + j, c = c0 + tx;
    double2 v = make_double2(0.0, 0.0);
    if (k0 < L0 && c < NC) {
      const int64_t col = compact_src ? c : (c <= H / 2 ? c : H + (c - H / 2 - 1));
      v = F[(k0 * L1 + k1) * Ssrc + col];
    }
    tile[j][tx] = v;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int64_t c = c0 + j, k0 = k00 + tx;
    if (c < NC && k0 < L0) {
      const double2 v = tile[tx][j];
      const int64_t oi = (c * L1 + k1) * L0 + k0;
      if constexpr (PAIR) {
        a[oi] = (T)(v.x * scale);
        if (b != nullptr) b[oi] = (T)(v.y * scale_b);
      } else {
        reinterpret_cast<C2<T>*>(a)[oi] = mk<T>((T)(v.x * scale), (T)(v.y * scale));
      }
    }
  }
}
template <typename T>
void extract_t(const double2* F, void* a, void* b, int64_t L0, int64_t L1, int64_t H, int64_t Ssrc, int compact_src,
               double scale, hipStream_t s, const unsigned long long* mx) {
  const dim3 grid((unsigned)((H + 1 + 31) / 32), (unsigned)((L0 + 31) / 32), (unsigned)L1);
  if (b != nullptr)
    hipLaunchKernelGGL((k_extract_t<T, true>), grid, dim3(256), 0, s, F, (T*)a, (T*)b, L0, L1, H + 1, Ssrc,
                       compact_src, H, scale, mx);
  else
    hipLaunchKernelGGL((k_extract_t<T, false>), grid, dim3(256), 0, s, F, (T*)a, (T*)nullptr, L0, L1, H + 1, Ssrc,
                       compact_src, H, scale, mx);
}
template <typename T>
void extract_t_re(const double2* F, void* a, int64_t L0, int64_t L1, int64_t H, int64_t Ssrc, int compact_src,
                  double scale, hipStream_t s) {
  const dim3 grid((unsigned)((H + 1 + 31) / 32), (unsigned)((L0 + 31) / 32), (unsigned)L1);
  hipLaunchKernelGGL((k_extract_t<T, true>), grid, dim3(256), 0, s, F, (T*)a, (T*)nullptr, L0, L1, H + 1, Ssrc,
                     compact_src, H, scale, (const unsigned long long*)nullptr);
}
template void extract_t_re<float>(const double2*, void*, int64_t, int64_t, int64_t, int64_t, int, double, hipStream_t);
template void extract_t_re<double>(const double2*, void*, int64_t, int64_t, int64_t, int64_t, int, double, hipStream_t);
template void extract_t<float>(const double2*, void*, void*, int64_t, int64_t, int64_t, int64_t, int, double, hipStream_t,
                               const unsigned long long*);
template void extract_t<double>(const double2*, void*, void*, int64_t, int64_t, int64_t, int64_t, int, double, hipStream_t,
                                const unsigned long long*);

template void extract_pair<float>(const double2*, void*, void*, int64_t, int64_t, int64_t, int, double, hipStream_t, int64_t,
                                  int64_t, const unsigned long long*);
template void extract_pair<double>(const double2*, void*, void*, int64_t, int64_t, int64_t, int, double, hipStream_t, int64_t,
                                   int64_t, const unsigned long long*);
template void extract_cplx<float>(const double2*, void*, int64_t, int64_t, int64_t, int, double, hipStream_t, int64_t, int64_t);
template void extract_cplx<double>(const double2*, void*, int64_t, int64_t, int64_t, int, double, hipStream_t, int64_t, int64_t);

// full expanded-grid spectrum from the unique m-grid values: u -> min(u, n-u) per axis
template <typename T>
__global__ void k_expand_spec(const double* __restrict__ src, T* __restrict__ out, GridDims g, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int64_t rem = idx, s = 0, mstride = 1;
  for (int a = g.d - 1; a >= 0; --a) {
    const int64_t u = rem % g.n[a];
    rem /= g.n[a];
    const int64_t t = (u < g.n[a] - u) ? u : g.n[a] - u;
    s += t * mstride;
    mstride *= g.m[a];
  }
  out[idx] = (T)src[s];
}
template <typename T>
void expand_spec(const double* src, void* out, const GridDims& g, hipStream_t s) {
  int64_t total = 1;
  for (int a = 0; a < g.d; ++a) total *= g.n[a];
  hipLaunchKernelGGL((k_expand_spec<T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, (T*)out, g,
                     total);
}
template void expand_spec<float>(const double*, void*, const GridDims&, hipStream_t);
template void expand_spec<double>(const double*, void*, const GridDims&, hipStream_t);

// ------------------------------------------------------------------------------------------
// batched CG kernels (cg.py:44-80 / 5-41).  Per-RHS scalars live on the device; every
// kernel returns early once the device flag `done` is set by the convergence test.
// Reductions are fixed-order (deterministic across runs and across RHS sharding).
// ------------------------------------------------------------------------------------------
constexpr int UPD_THREADS = 256;
constexpr int UPD_PER_THREAD = 8;
constexpr int UPD_CHUNK = UPD_THREADS * UPD_PER_THREAD;

int update_np(int64_t M) { return (int)((M + UPD_CHUNK - 1) / UPD_CHUNK); }

template <typename T>
__device__ __forceinline__ T block_sum_det(T v, T* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  T s = 0;
  if (threadIdx.x == 0)
    for (int k = 0; k < nw; ++k) s += red[k];
  return s;
}

// x <- 0, r <- b (row layout)
template <typename T>
__global__ void k_cg_init(const T* __restrict__ b, T* __restrict__ x, T* __restrict__ r, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { x[i] = (T)0; r[i] = b[i]; }
}

template <typename T>
__global__ void k_copy(const T* __restrict__ s, T* __restrict__ d, int64_t n, const int* done) {
  if (done && *done) return;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = s[i];
}

// out[c][r] = in[r][c]  (in: rows x cols)
template <typename T>
__global__ void k_transpose(const T* __restrict__ in, T* __restrict__ out, int64_t rows, int64_t cols) {
  __shared__ T tile[32][33];
  const int64_t c0 = (int64_t)blockIdx.x * 32, r0 = (int64_t)blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = r0 + k, c = c0 + tx;
    if (r < rows && c < cols) tile[k][tx] = in[r * cols + c];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = c0 + k, r = r0 + tx;
    if (r < rows && c < cols) out[c * rows + r] = tile[tx][k];
  }
}

// per-row dot partials: part[b*np + chunk]
template <typename T>
__global__ __launch_bounds__(UPD_THREADS) void k_rowdot_part(const T* __restrict__ a, const T* __restrict__ c,
                                                             T* __restrict__ part, int64_t M, int np) {
  __shared__ T red[UPD_THREADS / 64];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int64_t base = (int64_t)b * M;
  T s = 0;
#pragma unroll
  for (int k = 0; k < UPD_PER_THREAD; ++k) {
    const int64_t j = (int64_t)chunk * UPD_CHUNK + k * UPD_THREADS + threadIdx.x;
    if (j < M) s += a[base + j] * c[base + j];
  }
  s = block_sum_det<T>(s, red);
  if (threadIdx.x == 0) part[(int64_t)b * np + chunk] = s;
}

// out[b] = sum_g part[b*np + g]   (one wave per RHS, fixed tree)
// One block of RED_THREADS per RHS sums that RHS's row of partials: every lane issues its
// loads up front (np <= ~1k: one or two rounds), then a wave shuffle and a 4-entry LDS
// combine.  A wave per RHS walking the row serially left these scalar kernels at ~15 us,
// on the critical path between the column pass and the row-inverse pass of each chunk.
constexpr int RED_THREADS = 256;
template <typename T>
__device__ __forceinline__ T block_row_sum(const T* __restrict__ row, int np) {
  __shared__ T red[RED_THREADS / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T s = 0;
#pragma unroll 4
  for (int g = threadIdx.x; g < np; g += RED_THREADS) s += row[g];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) red[w] = s;
  __syncthreads();
  T t = 0;
#pragma unroll
  for (int i = 0; i < RED_THREADS / 64; ++i) t += red[i];
  return t;
}

template <typename T>
__global__ __launch_bounds__(RED_THREADS) void k_reduce_rows(const T* __restrict__ part, int np, int nrhs,
                                                             T* __restrict__ out) {
  const int b = blockIdx.x;
  const T s = block_row_sum(part + (int64_t)b * np, np);
  if (threadIdx.x == 0) out[b] = s;
}

// Long partial rows (the 3-D spectral dots: (L_2/2 + 1) L_1 per RHS) are folded first: block
// (g, b) sums FOLD_PER consecutive partials of RHS b (all loads issued up front) into
// out[b][g], so the one-block-per-RHS kernels below see ceil(np / FOLD_PER) values.  Fixed
// summation order: deterministic.
constexpr int FOLD_PER = 16 * RED_THREADS;
template <typename T>
__global__ __launch_bounds__(RED_THREADS) void k_fold_rows(const T* __restrict__ part, int np, int G,
                                                           T* __restrict__ out, const int* done) {
  if (done != nullptr && *done) return;
  __shared__ T red[RED_THREADS / 64];
  const int g = blockIdx.x, b = blockIdx.y;
  const T* row = part + (int64_t)b * np + (int64_t)g * FOLD_PER;
  const int n = np - g * FOLD_PER < FOLD_PER ? np - g * FOLD_PER : FOLD_PER;
  T v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int idx = threadIdx.x + k * RED_THREADS;
    v[k] = idx < n ? row[idx] : (T)0;
  }
  T s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += v[k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    T t = 0;
#pragma unroll
    for (int i = 0; i < RED_THREADS / 64; ++i) t += red[i];
    out[(int64_t)b * G + g] = t;
  }
}

// per RHS: alpha = rs / sum(part)   (cg.py:66)
template <typename T>
__global__ __launch_bounds__(RED_THREADS) void k_cg_alpha(const T* __restrict__ part, int np, int nrhs,
                                                          const T* __restrict__ rs, T* __restrict__ alpha,
                                                          const int* done) {
  if (*done) return;   // block-uniform
  const int b = blockIdx.x;
  const T s = block_row_sum(part + (int64_t)b * np, np);
  if (threadIdx.x == 0) alpha[b] = rs[b] / s;
}

// x += alpha p ; r -= alpha Ap ; partial r.r    (cg.py:67-69)
template <typename T>
__global__ __launch_bounds__(UPD_THREADS) void k_cg_update_xr(T* __restrict__ x, T* __restrict__ r,
                                                              const T* __restrict__ p, const T* __restrict__ Ap,
                                                              const T* __restrict__ alpha, T* __restrict__ part,
                                                              int64_t M, int np, const int* done) {
  if (*done) return;
  __shared__ T red[UPD_THREADS / 64];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int64_t base = (int64_t)b * M;
  const T al = alpha[b];
  T s = 0;
#pragma unroll
  for (int k = 0; k < UPD_PER_THREAD; ++k) {
    const int64_t j = (int64_t)chunk * UPD_CHUNK + k * UPD_THREADS + threadIdx.x;
    if (j < M) {
      const int64_t o = base + j;
      x[o] = x[o] + al * p[o];
      const T rn = r[o] - al * Ap[o];
      r[o] = rn;
      s += rn * rn;
    }
  }
  s = block_sum_det<T>(s, red);
  if (threadIdx.x == 0) part[(int64_t)b * np + chunk] = s;
}

// rnew = sum(part); done |= all(sqrt(rnew) < tol); iters++ (cg.py:69-71)
template <typename T>
__global__ __launch_bounds__(1024) void k_cg_check(const T* __restrict__ part, int np, int nrhs, double tol,
                                                   T* __restrict__ rnew, int* done, int* iters) {
  if (*done) return;
  __shared__ int any_not;
  if (threadIdx.x == 0) any_not = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int local_not = 0;
  for (int b = w; b < nrhs; b += nw) {
    T s = 0;
    for (int g = lane; g < np; g += 64) s += part[(int64_t)b * np + g];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) {
      rnew[b] = s;
      // torch.all(torch.sqrt(rnew) < tol): NaN compares false -> not converged
      if (!(sqrt(s) < (T)tol)) local_not = 1;
    }
  }
  if (lane == 0 && local_not) atomicOr(&any_not, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    *iters += 1;
    if (!any_not) *done = *iters;   // nonzero; = the iteration it fired in (PassDesc::cg_fix)
  }
}

// zr = sum(part); beta = zr / rs; rs = zr   (cg.py:74 and next iteration's rs, cg.py:64)
template <typename T>
__global__ __launch_bounds__(RED_THREADS) void k_cg_beta(const T* __restrict__ part, int np, int nrhs,
                                                         T* __restrict__ rs, T* __restrict__ beta, const int* done) {
  if (*done) return;   // block-uniform
  const int b = blockIdx.x;
  const T s = block_row_sum(part + (int64_t)b * np, np);
  if (threadIdx.x == 0) {
    beta[b] = s / rs[b];
    rs[b] = s;
  }
}

// p = z + beta p   (cg.py:75)
template <typename T>
__global__ __launch_bounds__(UPD_THREADS) void k_cg_update_p(T* __restrict__ p, const T* __restrict__ z,
                                                             const T* __restrict__ beta, int64_t M, const int* done) {
  if (*done) return;
  const int chunk = blockIdx.x, b = blockIdx.y;
  const int64_t base = (int64_t)b * M;
  const T be = beta[b];
#pragma unroll
  for (int k = 0; k < UPD_PER_THREAD; ++k) {
    const int64_t j = (int64_t)chunk * UPD_CHUNK + k * UPD_THREADS + threadIdx.x;
    if (j < M) {
      const int64_t o = base + j;
      p[o] = z[o] + be * p[o];
    }
  }
}

// ---- host launchers ------------------------------------------------------------------------
template <typename T>
void cg_init(const void* b, void* x, void* r, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL((k_cg_init<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const T*)b, (T*)x, (T*)r, n);
}
template <typename T>
void vcopy(const void* src, void* dst, int64_t n, const int* done, hipStream_t s) {
  hipLaunchKernelGGL((k_copy<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const T*)src, (T*)dst, n, done);
}
template <typename T>
void transpose(const void* in, void* out, int64_t rows, int64_t cols, hipStream_t s) {
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  hipLaunchKernelGGL((k_transpose<T>), grid, dim3(256), 0, s, (const T*)in, (T*)out, rows, cols);
}
template <typename T>
void rowdot_part(const void* a, const void* c, void* part, int64_t nrhs, int64_t M, int np, hipStream_t s) {
  dim3 grid((unsigned)np, (unsigned)nrhs);
  hipLaunchKernelGGL((k_rowdot_part<T>), grid, dim3(UPD_THREADS), 0, s, (const T*)a, (const T*)c, (T*)part, M, np);
}
template <typename T>
void reduce_rows(const void* part, int np, int nrhs, void* out, hipStream_t s) {
  hipLaunchKernelGGL((k_reduce_rows<T>), dim3((unsigned)nrhs), dim3(RED_THREADS), 0, s, (const T*)part, np, nrhs,
                     (T*)out);
}
int fold_groups(int np) { return np > FOLD_PER ? (np + FOLD_PER - 1) / FOLD_PER : 0; }
template <typename T>
void fold_rows(const void* part, int np, int nrhs, void* out, const int* done, hipStream_t s) {
  const int G = fold_groups(np);
  hipLaunchKernelGGL((k_fold_rows<T>), dim3((unsigned)G, (unsigned)nrhs), dim3(RED_THREADS), 0, s, (const T*)part, np, G,
                     (T*)out, done);
}
template <typename T>
void cg_alpha(const void* part, int np, int nrhs, const void* rs, void* alpha, const int* done, hipStream_t s) {
  hipLaunchKernelGGL((k_cg_alpha<T>), dim3((unsigned)nrhs), dim3(RED_THREADS), 0, s, (const T*)part, np, nrhs,
                     (const T*)rs, (T*)alpha, done);
}
template <typename T>
void cg_update_xr(void* x, void* r, const void* p, const void* Ap, const void* alpha, void* part, int64_t nrhs,
                  int64_t M, const int* done, hipStream_t s) {
  const int np = update_np(M);
  dim3 grid((unsigned)np, (unsigned)nrhs);
  hipLaunchKernelGGL((k_cg_update_xr<T>), grid, dim3(UPD_THREADS), 0, s, (T*)x, (T*)r, (const T*)p, (const T*)Ap,
                     (const T*)alpha, (T*)part, M, np, done);
}
template <typename T>
void cg_check(const void* part, int np, int nrhs, double tol, void* rnew, int* done, int* iters, hipStream_t s) {
  hipLaunchKernelGGL((k_cg_check<T>), dim3(1), dim3(1024), 0, s, (const T*)part, np, nrhs, tol, (T*)rnew, done, iters);
}
template <typename T>
void cg_beta(const void* part, int np, int nrhs, void* rs, void* beta, const int* done, hipStream_t s) {
  hipLaunchKernelGGL((k_cg_beta<T>), dim3((unsigned)nrhs), dim3(RED_THREADS), 0, s, (const T*)part, np, nrhs,
                     (T*)rs, (T*)beta, done);
}
template <typename T>
void cg_update_p(void* p, const void* z, const void* beta, int64_t nrhs, int64_t M, const int* done, hipStream_t s) {
  dim3 grid((unsigned)update_np(M), (unsigned)nrhs);
  hipLaunchKernelGGL((k_cg_update_p<T>), grid, dim3(UPD_THREADS), 0, s, (T*)p, (const T*)z, (const T*)beta, M, done);
}

// All-rank break rule without a host round trip (hgp_pcg_local_flag / hgp_pcg_set_done):
// flag = 1 when every sqrt(r.r) of this rank's RHS is below tol (cg.py:70, NaN = not converged)
template <typename T>
__global__ __launch_bounds__(256) void k_cg_local_flag(const T* __restrict__ rnew, int nrhs, double tol, int* flag) {
  __shared__ int any_not;
  if (threadIdx.x == 0) any_not = 0;
  __syncthreads();
  int mine = 0;
  for (int b = threadIdx.x; b < nrhs; b += blockDim.x)
    if (!(sqrt(rnew[b]) < (T)tol)) mine = 1;
  if (mine) atomicOr(&any_not, 1);
  __syncthreads();
  if (threadIdx.x == 0) *flag = any_not ? 0 : 1;
}
template <typename T>
void cg_local_flag(const void* rnew, int nrhs, double tol, int* flag, hipStream_t s) {
  hipLaunchKernelGGL((k_cg_local_flag<T>), dim3(1), dim3(256), 0, s, (const T*)rnew, nrhs, tol, flag);
}
// the plan's done flag := the (all-reduced) flag; later kernels of the solve are no-ops
__global__ void k_cg_set_done(int* done, const int* flag) {
  if (threadIdx.x == 0 && *flag != 0) *done = 1;
}
void cg_set_done(int* done, const int* flag, hipStream_t s) {
  hipLaunchKernelGGL(k_cg_set_done, dim3(1), dim3(64), 0, s, done, flag);
}

#define HGP_INST(T)                                                                                            \
  template void cg_init<T>(const void*, void*, void*, int64_t, hipStream_t);                                 \
  template void vcopy<T>(const void*, void*, int64_t, const int*, hipStream_t);                              \
  template void transpose<T>(const void*, void*, int64_t, int64_t, hipStream_t);                             \
  template void rowdot_part<T>(const void*, const void*, void*, int64_t, int64_t, int, hipStream_t);         \
  template void reduce_rows<T>(const void*, int, int, void*, hipStream_t);                                   \
  template void fold_rows<T>(const void*, int, int, void*, const int*, hipStream_t);                         \
  template void cg_alpha<T>(const void*, int, int, const void*, void*, const int*, hipStream_t);             \
  template void cg_update_xr<T>(void*, void*, const void*, const void*, const void*, void*, int64_t, int64_t, \
                                const int*, hipStream_t);                                                    \
  template void cg_check<T>(const void*, int, int, double, void*, int*, int*, hipStream_t);                  \
  template void cg_beta<T>(const void*, int, int, void*, void*, const int*, hipStream_t);                    \
  template void cg_update_p<T>(void*, const void*, const void*, int64_t, int64_t, const int*, hipStream_t); \
  template void cg_local_flag<T>(const void*, int, double, int*, hipStream_t);
HGP_INST(float)
HGP_INST(double)
#undef HGP_INST

}  // namespace hgp
