// hgp_lines.hpp — transposing middle-axis passes of the 3-D operators.
//
// The 3-D operator runs as five passes (hgp_api.hip run_op):
//   k_row_fwd_t  (hgp_rows.hpp) per (RHS, i0) plane: real rows along axis 2 -> W1 [q][i0][c2][i1]
//   k_line_fwd_t : complex lines along axis 1 (contiguous i1, one line per (i0, c2)), FFT, and a
//                  transposing store through an LDS tile: W2 [q][c2][k1][i0] (i0 contiguous)
//   k_pass<CONTIG, CONV> : axis-0 lines (q, c2, k1) = the barrier-free contiguous column kernel
//                  of the 2-D operator (spectrum [c2][k1][k0], spectral dots for the PCG)
//   k_line_inv_t : the tiles back, inverse FFT along axis 1, crop -> W1 [q][o0][c2][o1]
//   k_row_inv_t  (hgp_rows.hpp) per plane: real rows out, fused dot / PCG epilogue
// so that every pass reads and writes whole contiguous segments (C lines x sizeof(complex) per
// frequency column, C = 16: 128 B in fp32), and the heavy axis-0 pass (four FFTs per line) is
// the wave-local contiguous kernel instead of a strided one with block barriers.
//
// Geometry of both kernels (PassDesc):
//   a block = (q, group r, C consecutive lines i .. i+C-1), grid = Q * Rn * ceil(In / C)
//   line side:   View{ptr, q_stride, r_stride (per group), p_stride (per line), len}
//   column side: View{ptr, q_stride, r_stride (per group), p_stride (per frequency column), len}
//   (FWD: in = line side with len = valid input length <= H, out = column side, all L columns;
//    INV: in = column side (L columns), out = line side with len = output length, the crop)
#pragma once
#include "hgp_pass.hpp"

#ifndef HGP_LINET_C
#define HGP_LINET_C 16            // lines per block (= the contiguous segment per column)
#endif

namespace hgp {

// occupancy of the line-inverse pass with 4-wave blocks (0: from the LDS footprint).  3 waves per
// SIMD: the 256-point kernel (C5 axis 1) no longer spills 15 VGPRs, 1.12 -> 1.07 ms
// (profiles/r3_l_passtime.txt)
#ifndef HGP_MINW_LINE_INV
#define HGP_MINW_LINE_INV 3
#endif
template <typename T, int H> struct LineTCfg {
  static constexpr int P = PFor<T, H>::v;
  static constexpr int TT = H / P;
  static constexpr int ex_elems(int c) { return c * H + (c * H) / 16; }
  static constexpr int tile_elems(int c) { return H * (c + 1); }   // one frequency half, pitch c+1
  static constexpr int area(int c) { return ex_elems(c) > tile_elems(c) ? ex_elems(c) : tile_elems(c); }
  static constexpr int lds_bytes_for(int c) { return area(c) * (int)sizeof(C2<T>) + TwTab<T, H>::BYTES; }
  static constexpr int c_lines() {
    int c = HGP_LINET_C;
    while (c > 1 && (c * TT > 1024 || lds_bytes_for(c) > LDS_CAP)) c >>= 1;
    return c;
  }
  static constexpr int C = c_lines();
  static constexpr int THREADS = C * TT;
  static constexpr int AREA = area(C);
  static constexpr int LDS = lds_bytes_for(C);
  static constexpr int PITCH = C + 1;
  static constexpr bool WAVE = TT <= 64;
  static constexpr int BLOCKS_BY_LDS = LDS_CAP / LDS;
  static constexpr int MINW_LDS = (BLOCKS_BY_LDS * ((THREADS + 63) / 64)) / 4;
  static constexpr int MINW = MINW_LDS < 1 ? 1 : (MINW_LDS > 4 ? 4 : MINW_LDS);
  static constexpr int MINW_INV = (HGP_MINW_LINE_INV > 0 && THREADS == 256) ? HGP_MINW_LINE_INV : MINW;
};

// block -> (q, r, first line i0); l = line of this thread group, t = position index
struct LineTBlock { int q, r, i0; };
__device__ __forceinline__ LineTBlock line_block(const PassDesc& d, int C) {
  const int nib = (d.In + C - 1) / C;
  const int b = blockIdx.x;
  const int per_q = d.Rn * nib;
  LineTBlock o;
  o.q = b / per_q;
  const int rem = b - o.q * per_q;
  o.r = rem / nib;
  o.i0 = (rem - o.r * nib) * C;
  return o;
}

template <typename T, int H>
__global__ __launch_bounds__((LineTCfg<T, H>::THREADS), (LineTCfg<T, H>::MINW)) void k_line_fwd_t(const PassDesc d) {
  using Cfg = LineTCfg<T, H>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C, PITCH = Cfg::PITCH;
  if (d.done != nullptr && *d.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  C2<T>* tab = lds + Cfg::AREA;
  const C2<T>* __restrict__ twg = reinterpret_cast<const C2<T>*>(d.tw);
  stage_tw<T, H>(tab, twg, threadIdx.x, Cfg::THREADS);
  const LineTBlock B = line_block(d, C);
  const int l = (TT % 64 == 0) ? __builtin_amdgcn_readfirstlane(threadIdx.x / TT) : threadIdx.x / TT;
  const int t = threadIdx.x & (TT - 1);
  const bool valid = B.i0 + l < d.In;
  // one buffer resource from the block's first line (uniform; its C lines lie within 2 GiB of it,
  // checked on the host), per-lane 32-bit offsets; positions past the line and invalid lines read
  // at an offset past the range, which returns 0 (no clamped 64-bit addresses, no zeroing selects)
  const C2<T>* inb0 = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)B.q * d.in.q_stride +
                      (int64_t)B.r * d.in.r_stride + (int64_t)B.i0 * d.in.p_stride;
  const BufRsrc rin = buf_rsrc(inb0, 0x7fffffffu);
  constexpr uint32_t DROP = 0x80000000u;
  const uint32_t li = (uint32_t)l * (uint32_t)d.in.p_stride;
  const int in_len = d.in.len;     // <= 2H; > H (folded halves) for the R operator's n-grid input
  C2<T> va[P], vb[P];
  // fold (when L_R = 3 * 2^k < 2n) as a compile-time branch of its own straight-line loads
  auto load_lines = [&](auto fold_c) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = t + TT * k;
      const C2<T> a = buf_ld_c2<T>(rin, (valid && p < in_len) ? (li + (uint32_t)p) * (uint32_t)sizeof(C2<T>) : DROP);
      va[k] = a;
      vb[k] = a;
      if constexpr (decltype(fold_c)::value) {
        const C2<T> hi = buf_ld_c2<T>(rin, (valid && p + H < in_len) ? (li + (uint32_t)(p + H)) * (uint32_t)sizeof(C2<T>) : DROP);
        va[k] = cadd<T>(a, hi);
        vb[k] = csub<T>(a, hi);
      }
    }
  };
  if (in_len > H) load_lines(std::true_type{});
  else load_lines(std::false_type{});
  __syncthreads();   // twiddle table staged
#pragma unroll
  for (int k = 0; k < P; ++k) vb[k] = cmul<T>(vb[k], tw_at<T, H>(tab, t + TT * k));
  fft_line2<T, H, P, -1, 1, Cfg::WAVE>(va, vb, lds, l * H, t, tab);
  // frequencies half*H + p of line l -> tile [p][l] -> column segments of C lines
  C2<T>* outb = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)B.q * d.out.q_stride + (int64_t)B.r * d.out.r_stride;
  const BufRsrc ro = buf_rsrc(outb, 0x7fffffffu);   // one group's columns: < 2 GiB (host check)
  const uint32_t ps = (uint32_t)d.out.p_stride;
  const int nl = d.In - B.i0 < C ? d.In - B.i0 : C;
  auto put_half = [&](int half, C2<T>(&v)[P]) {
    __syncthreads();   // every group is done with its exchange image / the previous tile
#pragma unroll
    for (int k = 0; k < P; ++k) lds[(t + TT * k) * PITCH + l] = v[k];
    __syncthreads();
    constexpr int NE = H * C;
#pragma unroll
    for (int j = 0; j < (NE + Cfg::THREADS - 1) / Cfg::THREADS; ++j) {
      const int e = threadIdx.x + j * Cfg::THREADS;
      const int col = e / C;
      const int row = e - col * C;
      if (e < NE && row < nl)
        buf_st_c2<T>(lds[col * PITCH + row], ro,
                     ((uint32_t)(half * H + col) * ps + (uint32_t)(B.i0 + row)) * (uint32_t)sizeof(C2<T>));
    }
  };
  put_half(0, va);
  put_half(1, vb);
}

template <typename T, int H>
__global__ __launch_bounds__((LineTCfg<T, H>::THREADS), (LineTCfg<T, H>::MINW_INV)) void k_line_inv_t(const PassDesc d) {
  using Cfg = LineTCfg<T, H>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C, PITCH = Cfg::PITCH;
  if (d.done != nullptr && *d.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  C2<T>* tab = lds + Cfg::AREA;
  const C2<T>* __restrict__ twg = reinterpret_cast<const C2<T>*>(d.tw);
  stage_tw<T, H>(tab, twg, threadIdx.x, Cfg::THREADS);
  const LineTBlock B = line_block(d, C);
  const int l = (TT % 64 == 0) ? __builtin_amdgcn_readfirstlane(threadIdx.x / TT) : threadIdx.x / TT;
  const int t = threadIdx.x & (TT - 1);
  const bool valid = B.i0 + l < d.In;
  const C2<T>* inb = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)B.q * d.in.q_stride + (int64_t)B.r * d.in.r_stride;
  const BufRsrc ri = buf_rsrc(inb, 0x7fffffffu);
  const uint32_t ps = (uint32_t)d.in.p_stride;
  const int nl = d.In - B.i0 < C ? d.In - B.i0 : C;
  constexpr int NE = H * C;
  constexpr int ITER = (NE + Cfg::THREADS - 1) / Cfg::THREADS;
  C2<T> buf[ITER];
  auto load_half = [&](int half) {
#pragma unroll
    for (int j = 0; j < ITER; ++j) {         // all of the half's loads in flight at once
      const int e = threadIdx.x + j * Cfg::THREADS;
      const int ee = e < NE ? e : NE - 1;
      const int col = ee / C;
      const int row = ee - col * C;
      const int rr = row < nl ? row : 0;
      C2<T> v = buf_ld_c2<T>(ri, ((uint32_t)(half * H + col) * ps + (uint32_t)(B.i0 + rr)) * (uint32_t)sizeof(C2<T>));
      if (row >= nl) v = mk<T>(0, 0);
      buf[j] = v;
    }
  };
  auto park = [&]() {
#pragma unroll
    for (int j = 0; j < ITER; ++j) {
      const int e = threadIdx.x + j * Cfg::THREADS;
      const int col = e / C;
      const int row = e - col * C;
      if (e < NE) lds[col * PITCH + row] = buf[j];
    }
  };
  auto take = [&](C2<T>(&v)[P]) {
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = lds[(t + TT * k) * PITCH + l];
  };
  C2<T> va[P], vb[P];
  load_half(0);
  __syncthreads();   // twiddles staged (the tile area is free)
  park();
  __syncthreads();
  load_half(1);      // in flight while the even half is read out of the tile
  take(va);
  __syncthreads();
  park();
  __syncthreads();
  take(vb);
  __syncthreads();   // tile consumed: the exchange images overlay it
  fft_line2<T, H, P, +1, 1, Cfg::WAVE>(va, vb, lds, l * H, t, tab);
  // y[p] = ye + conj(W_L^p) yo, y[p + H] = ye - conj(W_L^p) yo; crop to out.len
  // one buffer resource from the block's first line (uniform; its C lines lie within 2 GiB of it,
  // checked on the host), per-lane 32-bit offsets, masked positions sent past the range (dropped)
  // instead of per-position exec branches with 64-bit addresses
  C2<T>* outb0 = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)B.q * d.out.q_stride + (int64_t)B.r * d.out.r_stride +
                 (int64_t)B.i0 * d.out.p_stride;
  const BufRsrc ro = buf_rsrc(outb0, 0x7fffffffu);
  constexpr uint32_t DROP = 0x80000000u;
  const uint32_t lo = (uint32_t)l * (uint32_t)d.out.p_stride;
  const int out_len = d.out.len;
  int tt = t;
  asm volatile("" : "+v"(tt));
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int p = tt + TT * k;
    const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
    const uint32_t o = (lo + (uint32_t)p) * (uint32_t)sizeof(C2<T>);
    buf_st_c2<T>(cadd<T>(va[k], wo), ro, (valid && p < out_len) ? o : DROP);
    if (H < out_len)   // uniform: the second half reaches the output (R^T's n-grid lines)
      buf_st_c2<T>(csub<T>(va[k], wo), ro, (valid && p + H < out_len) ? o + (uint32_t)(H * (int)sizeof(C2<T>)) : DROP);
  }
}

}  // namespace hgp
