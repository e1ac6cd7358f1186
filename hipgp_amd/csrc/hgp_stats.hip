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

#include <algorithm>

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
  // grid.y is the RHS: chunks of at most 65535 (the y-dimension limit), any batch size
  for (int64_t b0 = 0; b0 < nrhs; b0 += 65535) {
    const int64_t nb0 = std::min<int64_t>(65535, nrhs - b0);
    hipLaunchKernelGGL((k_stats_rows<T>), dim3((unsigned)np, (unsigned)nb0), dim3(ST_THREADS), 0, s,
                       (const T*)kn + b0 * Mp, (const T*)qm, (const T*)qS, Mp, np, part + b0 * np * 3);
  }
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

// ---- the two passes apart, for kn held in column slabs (grid-block sharding, hipgp_amd/slab.py):
// each rank runs pass 1 on its columns (qm, qS its slices), the (nrhs, 3) row dots are all-reduced
// (B values per dot instead of the B x M' kn), a_n and bdiff_n come from the reduced dots, and
// pass 2 gives the rank's slice of lam / dm.
template <typename T>
__global__ void k_rowdots_finish(const T* __restrict__ part, int np, int nrhs, T* __restrict__ out3) {
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
  if (lane < 3) out3[(int64_t)b * 3 + lane] = lane == 0 ? s[0] : lane == 1 ? s[1] : s[2];
}

template <typename T>
hipError_t meanfield_rowdots_t(const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS, void* out3,
                               hipStream_t s) {
  if (nrhs == 0) return hipSuccess;
  if (Mp == 0) return hipMemsetAsync(out3, 0, (size_t)(3 * nrhs) * sizeof(T), s);
  const int np = (int)((Mp + ST_CHUNK - 1) / ST_CHUNK);
  T* part = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&part), (size_t)(nrhs * np * 3) * sizeof(T), s);
  if (e != hipSuccess) return e;
  for (int64_t b0 = 0; b0 < nrhs; b0 += 65535) {
    const int64_t nb0 = std::min<int64_t>(65535, nrhs - b0);
    hipLaunchKernelGGL((k_stats_rows<T>), dim3((unsigned)np, (unsigned)nb0), dim3(ST_THREADS), 0, s,
                       (const T*)kn + b0 * Mp, (const T*)qm, (const T*)qS, Mp, np, part + b0 * np * 3);
  }
  hipLaunchKernelGGL((k_rowdots_finish<T>), dim3((unsigned)((nrhs + 3) / 4)), dim3(256), 0, s, (const T*)part, np,
                     (int)nrhs, (T*)out3);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipFreeAsync(part, s);
}

template <typename T>
hipError_t meanfield_cols_t(const void* kn, int64_t nrhs, int64_t Mp, const void* iv, const void* bdiff, void* lam,
                            void* dm, hipStream_t s) {
  if (Mp == 0) return hipSuccess;
  const int64_t nb = (Mp + ST_THREADS * 4 - 1) / (ST_THREADS * 4);
  hipLaunchKernelGGL((k_stats_cols<T>), dim3((unsigned)nb), dim3(ST_THREADS), 0, s, (const T*)kn, Mp, (int)nrhs,
                     (const T*)iv, (const T*)bdiff, (T*)lam, (T*)dm);
  return hipGetLastError();
}

hipError_t meanfield_rowdots(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                             void* out3, hipStream_t s) {
  if (dtype == HGP_F64) return meanfield_rowdots_t<double>(kn, nrhs, Mp, qm, qS, out3, s);
  return meanfield_rowdots_t<float>(kn, nrhs, Mp, qm, qS, out3, s);
}

hipError_t meanfield_cols(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* iv, const void* bdiff,
                          void* lam, void* dm, hipStream_t s) {
  if (dtype == HGP_F64) return meanfield_cols_t<double>(kn, nrhs, Mp, iv, bdiff, lam, dm, s);
  return meanfield_cols_t<float>(kn, nrhs, Mp, iv, bdiff, lam, dm, s);
}


// ---- block-diagonal family (BlockToeplitzGP, hipgp.py:527-691) ---------------------------------
// Blocks tile the expanded grid (dims n_a, block sides b_a, util.py:79-119): block beta enumerates
// the block grid C-order, point i the block C-order, flat index sum_a (c_a b_a + i_a) stride_a.
//   gram[beta]  = sum_n iv_n k_{n,beta} k_{n,beta}^T        (bs x bs; hipgp.py:252-256, get_lam :669-685)
//   knSkn[n]    = sum_beta k_{n,beta}^T S_beta k_{n,beta}    (compute_knSkn :661-664)
// One workgroup owns NBW = min(16, max(1, 1024 / bs^2)) consecutive blocks.  The flat kn column of
// each of its NBW * bs points is computed once (32-bit, LDS); S of its blocks is staged in LDS once
// (SL, when it fits); the RHS stream through an LDS tile K[n][col] in chunks of 64 rows, one row
// per wave and pass, lanes along the columns.
// gram (TA = 0, bs <= 16): thread t owns entries t + 256 r (r < 4) of the workgroup's contiguous
// gram slab;
// (TA >= 1) a 16 x 16 thread grid, thread (ti, tj) owning the TA x TA register tile
// i = ti + 16 a, j = tj + 16 b (per RHS: 2 TA LDS reads, TA^2 FMAs).
// knSkn: lane = RHS of the chunk, wave = row (local block, i): u = sum_j S[i][j] K[n][j] (S
// wave-uniform), v = K[n][i] u accumulated per (wave, n) in LDS by its only writer, then summed over
// the 4 waves in order -> part[n][workgroup]; rows reduced by k_reduce_rows.
// trSG = sum_beta <S_beta, gram_beta>_F = sum_n iv_n knSkn_n (the ELBO needs only this sum): formed
// from the gram registers as they are stored, S read along the same coalesced slab.
// Every sum has a fixed order (deterministic).
constexpr int BK_THREADS = 256;
constexpr int BK_NB = 64;          // RHS per chunk
constexpr int BK_MAXBS = 128;
constexpr int BK_UNR = 8;          // rows per load batch of the K-tile fill
constexpr int BK_ER = 4;           // gram entries per thread for small blocks (TA = 0)
constexpr size_t BK_LDS_MAX = 160 * 1024;

// LDS row pitch of the K tile: covers the 16 * TA gram tile columns (zero beyond ncol), odd
__host__ __device__ inline int bk_pitch(int ncol, int TA) { return (ncol > 16 * TA ? ncol : 16 * TA) + 1; }

template <typename T>
__host__ __device__ inline size_t bk_lds(int nbw, int bs, int TA, bool SL) {
  const int ncol = nbw * bs;
  return (size_t)(BK_NB * bk_pitch(ncol, TA) + BK_NB + 4 * BK_NB + (SL ? nbw * bs * bs : 0)) * sizeof(T) +
         (size_t)ncol * sizeof(int);
}

template <typename T, int TA, bool SL>
__global__ __launch_bounds__(BK_THREADS) void k_block_stats(BlockGeom g, const T* __restrict__ kn, int nrhs,
                                                           const T* __restrict__ iv, const T* __restrict__ S,
                                                           T* __restrict__ gram, T* __restrict__ part,
                                                           T* __restrict__ tpart) {
  extern __shared__ unsigned char smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const int bs = g.bs, nbw = g.nbw, bs2 = bs * bs;
  const int ncol = nbw * bs, pitch = bk_pitch(ncol, TA);
  T* Kt = smem;                                   // [BK_NB][pitch]
  T* ivs = Kt + BK_NB * pitch;                    // [BK_NB]
  T* Q = ivs + BK_NB;                             // [4][BK_NB]
  T* Ss = Q + 4 * BK_NB;                          // [nbw][bs][bs] (SL)
  int* colofs = reinterpret_cast<int*>(Ss + (SL ? nbw * bs2 : 0));   // [ncol], -1 = no block
  const int64_t beta0 = (int64_t)blockIdx.x * nbw;
  const int nvalid = (int)min<int64_t>(nbw, g.nblk - beta0);
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  for (int col = t; col < ncol; col += BK_THREADS) {
    const int bl = col / bs, i = col - bl * bs;
    int64_t rem = beta0 + bl, irem = i, flat = 0, stride = 1;
    for (int a = g.d - 1; a >= 0; --a) {
      const int64_t c = rem % g.nb[a], ii = irem % g.b[a];
      rem /= g.nb[a];
      irem /= g.b[a];
      flat += (c * g.b[a] + ii) * stride;
      stride *= g.n[a];
    }
    colofs[col] = bl < nvalid ? (int)flat : -1;
  }
  if (SL && part != nullptr) {
    const T* Sg = S + beta0 * bs2;
    for (int q = t; q < nbw * bs2; q += BK_THREADS) Ss[q] = (q < nvalid * bs2) ? Sg[q] : (T)0;
  }
  constexpr int NA = TA > 0 ? TA : 1;
  T acc[NA][NA];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NA; ++b) acc[a][b] = 0;
  // TA = 0: entries e = t + 256 r (r < BK_ER) of the workgroup's contiguous gram slab
  T acc0[BK_ER];
  int oi[BK_ER], oj[BK_ER];
  const int nent = nvalid * bs2;
#pragma unroll
  for (int r = 0; r < BK_ER; ++r) {
    acc0[r] = 0;
    const int e = min(t + BK_THREADS * r, nbw * bs2 - 1);
    const int bl = e / bs2, ij = e - bl * bs2, i = ij / bs;
    oi[r] = bl * bs + i;
    oj[r] = bl * bs + (ij - i * bs);
  }
  const int gi = t >> 4, gj = t & 15;
  const bool gram_thread = gram != nullptr && (TA > 0 || t < nent);
  const int nwg = gridDim.x;
  __syncthreads();
  for (int n0 = 0; n0 < nrhs; n0 += BK_NB) {
    const int nn = min(BK_NB, nrhs - n0);
    // BK_UNR independent row loads in flight.  Columns >= ncol (tile padding) stay unset: they only
    // feed gram entries i or j >= bs, which are never stored.
    for (int col = lane; col < ncol; col += 64) {
      const int o = col < ncol ? colofs[col] : -1;
      for (int rn0 = w; rn0 < nn; rn0 += 4 * BK_UNR) {
        T v[BK_UNR];
#pragma unroll
        for (int u = 0; u < BK_UNR; ++u) {
          const int rn = rn0 + 4 * u;
          v[u] = 0;
          if (o >= 0 && rn < nn) v[u] = kn[(int64_t)(n0 + rn) * g.Mp + o];
        }
#pragma unroll
        for (int u = 0; u < BK_UNR; ++u)
          if (rn0 + 4 * u < nn) Kt[(rn0 + 4 * u) * pitch + col] = v[u];
      }
    }
    if (t < BK_NB) ivs[t] = (t < nn && iv != nullptr) ? iv[n0 + t] : (T)0;   // iv may be NULL without gram
    __syncthreads();
    if (TA == 0 && gram_thread) {
      for (int k = 0; k < nn; ++k) {
        const T ivk = ivs[k];
        const T* kr = Kt + k * pitch;
#pragma unroll
        for (int r = 0; r < BK_ER; ++r)
          if (t + BK_THREADS * r < nent) acc0[r] += ivk * kr[oi[r]] * kr[oj[r]];
      }
    } else if (gram_thread) {
      const T* ki = Kt + gi;
      const T* kj = Kt + gj;
      for (int k = 0; k < nn; ++k) {
        const T ivk = ivs[k];
        T vi[NA], vj[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          vi[a] = ivk * ki[k * pitch + 16 * a];
          vj[a] = kj[k * pitch + 16 * a];
        }
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int b = 0; b < NA; ++b) acc[a][b] += vi[a] * vj[b];
      }
    }
    if (part != nullptr) {
      T qv = 0;
      if (lane < nn) {
        const T* kr = Kt + lane * pitch;
        for (int row = w; row < nvalid * bs; row += 4) {
          const int bl = row / bs, i = row - bl * bs;
          const T* srow = SL ? Ss + (bl * bs + i) * bs : S + ((beta0 + bl) * bs + i) * bs;
          const T* kb = kr + bl * bs;
          T u = 0;
          for (int j = 0; j < bs; ++j) u += srow[j] * kb[j];
          qv += kb[i] * u;
        }
      }
      Q[w * BK_NB + lane] = qv;
    }
    __syncthreads();
    if (part != nullptr && t < nn)
      part[(int64_t)(n0 + t) * nwg + blockIdx.x] = (Q[t] + Q[BK_NB + t]) + (Q[2 * BK_NB + t] + Q[3 * BK_NB + t]);
    __syncthreads();
  }
  T tr = 0;
  if (TA == 0 && gram_thread) {
    T* gb = gram + beta0 * bs2;
    const T* sb = S + beta0 * bs2;
#pragma unroll
    for (int r = 0; r < BK_ER; ++r) {
      const int e = t + BK_THREADS * r;
      if (e < nent) {
        gb[e] = acc0[r];
        if (tpart != nullptr) tr += sb[e] * acc0[r];
      }
    }
  } else if (gram_thread) {        // TA > 0: one block per workgroup
    T* gb = gram + beta0 * bs2;
    const T* sb = S + beta0 * bs2;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NA; ++b) {
        const int i = gi + 16 * a, j = gj + 16 * b;
        if (i < bs && j < bs) {
          gb[i * bs + j] = acc[a][b];
          if (tpart != nullptr) tr += sb[i * bs + j] * acc[a][b];
        }
      }
  }
  if (tpart != nullptr) {          // <S, G>_F of the workgroup's blocks, fixed-order reduction
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tr += __shfl_xor(tr, off, 64);
    if (lane == 0) Q[w] = tr;
    __syncthreads();
    if (t == 0) tpart[blockIdx.x] = (Q[0] + Q[1]) + (Q[2] + Q[3]);
  }
}

template <typename T, int TA>
void launch_block_stats(const BlockGeom& g, int64_t grid, const void* kn, int nrhs, const void* iv, const void* S,
                        void* gram, void* part, void* tpart, hipStream_t s) {
  const bool sl = part != nullptr && bk_lds<T>(g.nbw, g.bs, TA, true) <= BK_LDS_MAX;
  const size_t lds = bk_lds<T>(g.nbw, g.bs, TA, sl);
  auto launch = [&](auto kern) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BK_THREADS), lds, s, g, (const T*)kn, nrhs, (const T*)iv,
                       (const T*)S, (T*)gram, (T*)part, (T*)tpart);
  };
  if (sl) launch(k_block_stats<T, TA, true>);
  else launch(k_block_stats<T, TA, false>);
}

template <typename T>
hipError_t block_stats_t(const BlockGeom& g, const void* kn, int64_t nrhs, const void* iv, const void* S, void* gram,
                         void* knSkn, void* trSG, hipStream_t s) {
  const int64_t grid = (g.nblk + g.nbw - 1) / g.nbw;
  T* part = nullptr;
  T* tpart = nullptr;
  if (knSkn != nullptr && nrhs > 0) {
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&part), (size_t)(nrhs * grid) * sizeof(T), s);
    if (e != hipSuccess) return e;
  }
  if (trSG != nullptr && nrhs > 0) {
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&tpart), (size_t)grid * sizeof(T), s);
    if (e != hipSuccess) return e;
  }
  void* gp = gram;
  if (nrhs == 0) {     // empty batch: sums over no observations
    if (gram != nullptr) {
      hipError_t e = hipMemsetAsync(gram, 0, (size_t)(g.nblk * g.bs * g.bs) * sizeof(T), s);
      if (e != hipSuccess) return e;
    }
    if (trSG != nullptr) {
      hipError_t e = hipMemsetAsync(trSG, 0, sizeof(T), s);
      if (e != hipSuccess) return e;
    }
    gp = nullptr;
  }
  if (nrhs > 0) {
    const int TA = g.bs <= 16 ? 0 : (g.bs + 15) / 16;
    switch (TA) {
      case 0: launch_block_stats<T, 0>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 2: launch_block_stats<T, 2>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 3: launch_block_stats<T, 3>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 4: launch_block_stats<T, 4>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 5: launch_block_stats<T, 5>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 6: launch_block_stats<T, 6>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      case 7: launch_block_stats<T, 7>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
      default: launch_block_stats<T, 8>(g, grid, kn, (int)nrhs, iv, S, gp, part, tpart, s); break;
    }
    if (knSkn != nullptr) reduce_rows<T>(part, (int)grid, (int)nrhs, knSkn, s);
    if (trSG != nullptr) reduce_rows<T>(tpart, (int)grid, 1, trSG, s);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (part != nullptr && (e = hipFreeAsync(part, s)) != hipSuccess) return e;
  if (tpart != nullptr) return hipFreeAsync(tpart, s);
  return hipSuccess;
}

int block_geom(int ndim, const int64_t* dims, const int64_t* blocks, BlockGeom* g, const char** why) {
  if (ndim < 2 || ndim > 3) { *why = "block family supports 2-D and 3-D grids only (util.py:88)"; return -1; }
  g->d = ndim;
  g->Mp = 1;
  g->nblk = 1;
  int64_t bs = 1;
  for (int a = 0; a < ndim; ++a) {
    if (dims[a] <= 0 || blocks[a] <= 0) { *why = "dims and blocks must be positive"; return -1; }
    if (dims[a] % blocks[a] != 0) { *why = "each expanded-grid size must be divisible by its block side"; return -1; }
    g->n[a] = dims[a];
    g->b[a] = blocks[a];
    g->nb[a] = dims[a] / blocks[a];
    g->Mp *= dims[a];
    g->nblk *= g->nb[a];
    bs *= blocks[a];
  }
  if (bs > BK_MAXBS) { *why = "block size (points per block) must be <= 128"; return -1; }
  if (g->Mp >= ((int64_t)1 << 31)) { *why = "expanded grid must have < 2^31 points"; return -1; }
  g->bs = (int)bs;
  // blocks per workgroup: up to 4 gram entries per thread, at most 16 (longer contiguous kn runs)
  g->nbw = bs > 16 ? 1 : (int)std::min<int64_t>(16, std::max<int64_t>(1, BK_THREADS * BK_ER / (bs * bs)));
  return 0;
}

hipError_t block_stats(int dtype, const BlockGeom& g, const void* kn, int64_t nrhs, const void* iv, const void* S,
                       void* gram, void* knSkn, void* trSG, hipStream_t s) {
  if (dtype == HGP_F64) return block_stats_t<double>(g, kn, nrhs, iv, S, gram, knSkn, trSG, s);
  return block_stats_t<float>(g, kn, nrhs, iv, S, gram, knSkn, trSG, s);
}

}  // namespace hgp
