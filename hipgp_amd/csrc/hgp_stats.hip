// hgp_stats.hip — mean-field natural-gradient statistics of one minibatch:
// the batch sums `MeanFieldToeplitzGP.elbo_and_grad` needs from kn = R^T K^-1 Knm^T
// (hipgp.py:234-250, a_n of compute_batch_an hipgp.py:370-414), in two streaming passes over kn
// instead of the ~8 full-size temporaries the torch expression materialises (kn*kn, ivar*kk, ...).
//
//   pass 1 (rows):    knm_n = kn_n . qm,  knkn_n = |kn_n|^2,  knSkn_n = kn_n^2 . qS   (partials per
//                     (row, chunk), then a fixed-order reduce per row that also forms
//                     a_n = -1/2 iv_n ((knm_n - y_n)^2 + Knn_n - knkn_n + knSkn_n) - log_sd_n - ln(2 pi)/2
//                     and bdiff_n = iv_n (knm_n - y_n))
//   pass 2 (columns): lam_j = sum_n iv_n kn_nj^2,  dm_j = -sum_n bdiff_n kn_nj   (one thread per
//                     column, RHS loop in order: coalesced, deterministic)
// Bytes: 2 reads of kn (B M' s) + qm, qS + 2 M' s written.  HBM-bound.
#include "hgp_internal.hpp"
#include "../../include/hipgp.h"

namespace hgp {

constexpr int ST_THREADS = 256;
constexpr int ST_PER_THREAD = 8;
constexpr int ST_CHUNK = ST_THREADS * ST_PER_THREAD;

template <typename T>
__global__ __launch_bounds__(ST_THREADS) void k_stats_rows(const T* __restrict__ kn, const T* __restrict__ qm,
                                                          const T* __restrict__ qS, int64_t Mp, int np,
                                                          T* __restrict__ part) {
  __shared__ T red[3][ST_THREADS / 64];
  const int chunk = blockIdx.x, b = blockIdx.y;
  const T* row = kn + (int64_t)b * Mp;
  T s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
  for (int k = 0; k < ST_PER_THREAD; ++k) {
    const int64_t j = (int64_t)chunk * ST_CHUNK + k * ST_THREADS + threadIdx.x;
    if (j < Mp) {
      const T v = row[j];
      const T v2 = v * v;
      s0 += v * qm[j];
      s1 += v2;
      s2 += v2 * qS[j];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s0 += __shfl_xor(s0, off, 64);
    s1 += __shfl_xor(s1, off, 64);
    s2 += __shfl_xor(s2, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = s0; red[1][w] = s1; red[2][w] = s2; }
  __syncthreads();
  if (threadIdx.x < 3) {
    T s = 0;
    for (int k = 0; k < ST_THREADS / 64; ++k) s += red[threadIdx.x][k];
    part[((int64_t)b * np + chunk) * 3 + threadIdx.x] = s;
  }
}

template <typename T>
__global__ void k_stats_finish(const T* __restrict__ part, int np, int nrhs, const T* __restrict__ y,
                               const T* __restrict__ iv, const T* __restrict__ knn, const T* __restrict__ lsd,
                               T* __restrict__ an, T* __restrict__ bdiff) {
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= nrhs) return;
  T s[3] = {0, 0, 0};
  for (int g = lane; g < np; g += 64)
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] += part[((int64_t)b * np + g) * 3 + c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int c = 0; c < 3; ++c) s[c] += __shfl_xor(s[c], off, 64);
  if (lane == 0) {
    const T e = s[0] - y[b];
    an[b] = (T)-0.5 * iv[b] * (e * e + knn[b] - s[1] + s[2]) - lsd[b] - (T)0.91893853320467274178;
    bdiff[b] = iv[b] * e;
  }
}

template <typename T>
__global__ __launch_bounds__(ST_THREADS) void k_stats_cols(const T* __restrict__ kn, int64_t Mp, int nrhs,
                                                          const T* __restrict__ iv, const T* __restrict__ bdiff,
                                                          T* __restrict__ lam, T* __restrict__ dm) {
  constexpr int CPT = 4;                      // columns per thread (independent loads in flight)
  const int64_t j0 = (int64_t)blockIdx.x * ST_THREADS * CPT + threadIdx.x;
  T l[CPT], m[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) { l[c] = 0; m[c] = 0; }
  for (int b = 0; b < nrhs; ++b) {
    const T ivb = iv[b], bd = bdiff[b];
    const T* row = kn + (int64_t)b * Mp;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int64_t j = j0 + c * ST_THREADS;
      if (j < Mp) {
        const T v = row[j];
        l[c] += ivb * (v * v);
        m[c] += bd * v;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int64_t j = j0 + c * ST_THREADS;
    if (j < Mp) { lam[j] = l[c]; dm[j] = -m[c]; }
  }
}

template <typename T>
hipError_t meanfield_stats_t(const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                             const void* y, const void* iv, const void* knn, const void* lsd, void* an, void* lam,
                             void* dm, hipStream_t s) {
  const int np = (int)((Mp + ST_CHUNK - 1) / ST_CHUNK);
  T* scratch = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&scratch), (size_t)(nrhs * np * 3 + nrhs) * sizeof(T), s);
  if (e != hipSuccess) return e;
  T* part = scratch;
  T* bdiff = scratch + nrhs * np * 3;
  hipLaunchKernelGGL((k_stats_rows<T>), dim3((unsigned)np, (unsigned)nrhs), dim3(ST_THREADS), 0, s,
                     (const T*)kn, (const T*)qm, (const T*)qS, Mp, np, part);
  hipLaunchKernelGGL((k_stats_finish<T>), dim3((unsigned)((nrhs + 3) / 4)), dim3(256), 0, s, (const T*)part, np,
                     (int)nrhs, (const T*)y, (const T*)iv, (const T*)knn, (const T*)lsd, (T*)an, bdiff);
  const int64_t nb = (Mp + ST_THREADS * 4 - 1) / (ST_THREADS * 4);
  hipLaunchKernelGGL((k_stats_cols<T>), dim3((unsigned)nb), dim3(ST_THREADS), 0, s, (const T*)kn, Mp, (int)nrhs,
                     (const T*)iv, (const T*)bdiff, (T*)lam, (T*)dm);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipFreeAsync(scratch, s);
}

hipError_t meanfield_stats(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                           const void* y, const void* iv, const void* knn, const void* lsd, void* an, void* lam,
                           void* dm, hipStream_t s) {
  if (dtype == HGP_F64) return meanfield_stats_t<double>(kn, nrhs, Mp, qm, qS, y, iv, knn, lsd, an, lam, dm, s);
  return meanfield_stats_t<float>(kn, nrhs, Mp, qm, qS, y, iv, knn, lsd, an, lam, dm, s);
}

}  // namespace hgp
