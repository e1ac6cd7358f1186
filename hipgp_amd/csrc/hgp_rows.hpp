// hgp_rows.hpp — row-pair passes of the 2-D operators with a COLUMN-MAJOR intermediate.
//
// The 2-D Toeplitz operator y = crop(IFFT2(S . FFT2(pad x))) runs as three passes:
//   k_row_fwd_t : real rows (2j, 2j+1) of one RHS -> one complex FFT (pair packed as Re/Im),
//                 Hermitian split into the two rows' half spectra, stored TRANSPOSED:
//                 W[q][c][i0] (compact column c = 0..H, row i0), through an LDS tile so that
//                 each column gets one contiguous 2C-row segment (C pairs per block).
//   k_pass<CONTIG, CONV> (hgp_pass.hpp) : per column c, a contiguous complex line of m0
//                 values: pad -> FFT -> x spectrum -> IFFT -> crop, wave-local exchanges.
//   k_row_inv_t : the column-major tiles back through LDS, Hermitian rebuild of the pair,
//                 inverse FFT, crop, real rows out (+ fused per-pair dot with a second vector).
// Compared with a row-major intermediate this turns the heavy pass (4 FFTs per line) into a
// barrier-free contiguous-line kernel; the transposition costs one LDS tile round trip in
// each row pass.  Compact columns: c <= H/2 holds even frequency 2c, c > H/2 odd frequency
// 2(c - H/2 - 1) + 1 (the order the frequency halves leave the FFT in, hgp_fft.hpp).
#pragma once
#include "hgp_pass.hpp"

#ifndef HGP_ROWT_PAIRS
#define HGP_ROWT_PAIRS 8          // row pairs per block (16 rows = 128-B column segments)
#endif
// Block order of the row-inverse pass.  A block's column segments are 2C rows long; below one
// 128-B line (fp32 rows of 4096: C = 4 pairs, 64 B) the two blocks reading each line are dealt
// to the same XCD (xcd_remap), so the second one finds the line in that L2 (C4 row inverse
// 2.11 -> 1.67 ms).  The same order in the forward pass (whose partial lines are writes)
// measured slower (1.42 -> 1.55 ms), so it keeps the plain order.
//   0: never remap, 1: row inverse below 128-B segments, 2: row inverse always, 3: both passes
#ifndef HGP_ROW_XCD
#define HGP_ROW_XCD 1
#endif
// the forward transform in the EPI_RF tail: the two halves one after the other (fits the
// row-inverse kernel's register budget: interleaved, the C2 kernel spilled 28 VGPRs)
#ifndef HGP_RF_SEQ
#define HGP_RF_SEQ 1
#endif
#ifndef HGP_ROWT_PAIRS_BIG
#define HGP_ROWT_PAIRS_BIG 16     // the same knob for rows longer than one wave's line (TT > 64)
#endif

namespace hgp {

// Phase stagger of the long-row passes (knob, default off).  A 4096-point row block fills a CU
// alone (16 waves at ~117 VGPRs), and every CU starts its first block at the launch: all CUs then
// load, transform and store in step, so HBM idles during the transforms.  With HGP_ROW_STAGGER = n
// the first-round blocks of every other CU (hardware order: workgroup i -> XCD i % 8, its
// (i / 8)-th block) sleep n x 127 x 64 clocks first, so half the CUs run half a block out of phase.
#ifndef HGP_ROW_STAGGER
#define HGP_ROW_STAGGER 0
#endif
template <int THREADS>
__device__ __forceinline__ void row_stagger() {
  if constexpr (HGP_ROW_STAGGER > 0 && THREADS >= 1024) {
    if (blockIdx.x < 256u && ((blockIdx.x >> 3) & 1u)) {
#pragma unroll 1
      for (int i = 0; i < HGP_ROW_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
    }
  }
}

// Grouped columns (long fp32 rows).  A block's tile is 2C rows of every compact column; with the
// plain column-major intermediate W[c][i0] its stores / loads are 2C x sizeof(complex) segments,
// and at H = 4096 the LDS (four 4096-point exchange images, 139 KB) holds one 4-pair block per
// CU: 64-B segments, no second block to overlap load, transform and store with (row passes
// 0.37 of HBM at C4, PMC traffic 1.64x).  The grouped layout interleaves G consecutive compact
// columns, element (c, i0) at ((c / G) S0 + i0) G + c % G, so 2C rows x G columns are one
// contiguous 128-B segment with C = 8 / G pairs per block; the tile of each frequency half is
// moved in NCH column chunks, and two such blocks fit a CU.  The axis-0 pass reads the layout
// as LAY_CONTIG_G (hgp_pass.hpp).  G = 1 is the plain layout (the 3-D planes, the slab passes,
// fp64 and rows of one wave or less).
#ifndef HGP_ROWG_2048
#define HGP_ROWG_2048 2           // G at H = 2048 (fp32): 4 pairs x 2 columns = 128 B
#endif
// H >= 4096: G = 4 (2 pairs x 4 columns = 128 B).  Round 3 (before the spill fixes) measured the
// axis-0 pass reading one column of every 32 B losing more than the rows gained (C4 K matvec 5.64
// plain vs 5.78 ms).  Round 4, on the spill-free kernels (profiles/r4_e_grouped4096_K_Cinv.txt):
// rows 1.44 -> 1.12 and 1.52 -> 1.16 ms, the axis-0 pass 2.03 -> 2.41 ms, K matvec 4.98 -> 4.83 ms,
// C^-1 4.96 -> 4.82 ms (G = 2: 4.91 / 4.99) -- so G = 4.
#ifndef HGP_ROWG_4096
#define HGP_ROWG_4096 4
#endif
// pairs per block of the grouped 4096-point rows (0: 8 / G, i.e. 128-B segments).  2 with G = 2:
// 64-B segments but a 70 KB block, two per CU.
#ifndef HGP_ROWG_PAIRS_LONG
#define HGP_ROWG_PAIRS_LONG 0
#endif
// pairs per ROW-INVERSE block of the grouped 2048-point rows (0: as the forward pass, 8 / G).
// 2: 35 KB blocks, four per CU (C3 row inverse 2.08 -> 1.92 ms, K op 8.04 -> 8.00 ms, PCG(20)
// equal; profiles/r5_w_rowinv_small.txt)
#ifndef HGP_ROWG_PAIRS_2048_INV
#define HGP_ROWG_PAIRS_2048_INV 2
#endif
// pairs per ROW-INVERSE block of the ungrouped power-of-two rows of one wave (TT = 64, the C2
// 1024-point rows; 0: as the forward pass, HGP_ROWT_PAIRS).  4 measured slower (three 45 KB
// blocks per CU, 12 waves instead of 16: C2 bench op 0.281 -> 0.285-0.287 ms, PCG(20) 14.8 ->
// 15.8 ms; profiles/r5_w_rowinv_small.txt)
#ifndef HGP_ROWT_PAIRS_INV
#define HGP_ROWT_PAIRS_INV 0
#endif
// the same for the ROW-INVERSE pass alone (0: as the forward pass).  1: 35 KB blocks, four per
// CU instead of two (C4 row inverse 1.09 -> 1.01 ms, K op 4.48 -> 4.46 ms, PCG(20) 210.6 ->
// 208 ms on one box; profiles/r5_t_rowinv4096.txt); the forward pass keeps 128-B segments
#ifndef HGP_ROWG_PAIRS_LONG_INV
#define HGP_ROWG_PAIRS_LONG_INV 1
#endif
// G for the fp32 3 * 2^k rows of >= 6144 points (the 2-D R / R^T of 4096-point axes, L_R = 12288):
// their row-pair blocks hold 2 pairs (123 KB of LDS), i.e. 32-B column segments with G = 1; G = 4
// makes them 128 B (C4 R^T 21.0 -> 17.8 ms, R 21.6 -> 18.1 ms: row forward 5.3 -> 2.7 ms, row
// inverse 7.2 -> 6.1 ms, the column pass 9.1 -> 9.8 ms; profiles/r3_p_tri_rows.txt)
#ifndef HGP_ROWG_TRI
#define HGP_ROWG_TRI 4
#endif
// pairs per block of the ROW-INVERSE pass over those grouped 3 * 2^k rows (0: 8 / G).  Two
// 6144-point pairs (106 KB of LDS) leave one 16-wave block per CU, whose load / transform / store
// phases then run in step; one pair is a 53 KB block, three per CU, at 64-B column segments (the
// two blocks of a 128-B unit land in the same XCD, XCD_INV).  C4 (profiles/r5_l_tri_pairs.txt):
// R^T row inverse 5.96 -> 3.70 ms, R row inverse 2.77 -> 1.83 ms.  The forward pass keeps two
// pairs: its partial-unit WRITES do not merge (R^T row forward 2.63 -> 3.96 ms, R 5.81 -> 9.13).
#ifndef HGP_ROWG_PAIRS_TRI_INV
#define HGP_ROWG_PAIRS_TRI_INV 1
#endif
// threads per ROW-INVERSE block of the ungrouped 3 * 2^k rows longer than a wave (0: as the
// forward pass, HGP_ROWT_PAIRS_BIG pairs of 64 threads' worth = 1024 threads, ~104 KB of LDS,
// one block per CU).  512: ~52 KB, three blocks per CU (C3 R^T row inverse 11.9 -> 9.0 ms, op
// 30.3 -> 27.8 ms; C2 R^T 1.23 -> 1.17 ms; profiles/r5_n_tri_inv_threads.txt).  HGP_ROWT_THREADS_
// TRI_FWD: the same for the forward pass (0: 1024), only where the block's column segments stay
// >= 64 B: its partial-segment WRITES do not merge (C3, 3072-point rows at 2 pairs = 32 B: R^T row
// forward 4.82 -> 11.9 ms; C2, 1536-point rows at 4 pairs = 64 B: 0.203 -> 0.151 ms, R 0.455 ->
// 0.324 ms; profiles/r5_o_tri_fwd_threads.txt)
#ifndef HGP_ROWT_THREADS_TRI_INV
#define HGP_ROWT_THREADS_TRI_INV 512
#endif
#ifndef HGP_ROWT_THREADS_TRI_FWD
#define HGP_ROWT_THREADS_TRI_FWD 512
#endif
template <typename T, int H> struct RowGroup {
  static constexpr int G = !std::is_same<T, float>::value ? 1
                         : !is_pow2(H) ? (H >= 6144 ? HGP_ROWG_TRI : 1)
                         : H == 2048 ? HGP_ROWG_2048 : H >= 4096 ? HGP_ROWG_4096 : 1;
};

// points per thread of the fp32 row passes at H >= 4096 (0: PFor's 16).  32: a pair's line is two
// waves instead of four, a 4-pair block 8 waves, 2 waves per SIMD with up to 256 VGPRs (no spills;
// the P = 16 row inverse spilled 13 VGPRs to HBM scratch at C4).
#ifndef HGP_ROW_P_LONG
#define HGP_ROW_P_LONG 0
#endif
// points per thread of the grouped fp32 3 * 2^k rows (>= 6144 points; 0: PFor's 12).  24: radix-8
// stages, as the column pass (HGP_TRI_P_CONV): C4 R^T row forward 2.63 -> 2.34 ms, row inverse
// 3.71 -> 3.60, op 14.65 -> 14.21 ms; R 15.04 -> 14.07 ms (profiles/r5_aa_rows_p24.txt)
#ifndef HGP_ROW_P_TRI
#define HGP_ROW_P_TRI 24
#endif
template <typename T, int H, int G = 1, bool INV = false> struct RowTCfg {
  static constexpr bool F32 = std::is_same<T, float>::value;
  static constexpr int P = (F32 && is_pow2(H) && H >= 4096 && HGP_ROW_P_LONG > 0) ? HGP_ROW_P_LONG
                         : (F32 && !is_pow2(H) && G > 1 && HGP_ROW_P_TRI > 0) ? HGP_ROW_P_TRI
                                                                            : PFor<T, H>::v;
  static constexpr int TT = H / P;
  // tile chunks per frequency half (the grouped blocks keep a chunk of columns in LDS at a time)
  static constexpr int NCH = G > 1 ? 2 : 1;
  static constexpr int CHC = H / 2 / NCH;                        // nominal columns per chunk
  // exchange images: pair l owns logical elements [l*H, (l+1)*H), padded by lds_phys
  static constexpr int ex_elems(int c) { return c * H + (c * H) / 16; }
  static constexpr int TS(int c) { return 2 * c + 1; }           // tile row pitch (pad: banks)
  static constexpr int tile_elems(int c) { return (CHC + 1) * TS(c); }
  static constexpr int area(int c) { return ex_elems(c) > tile_elems(c) ? ex_elems(c) : tile_elems(c); }
  static constexpr int lds_bytes_for(int c) { return area(c) * (int)sizeof(C2<T>) + TwTab<T, H>::BYTES; }
  static constexpr int c_pairs() {
    if (G > 1) return (INV && !is_pow2(H) && HGP_ROWG_PAIRS_TRI_INV > 0) ? HGP_ROWG_PAIRS_TRI_INV
                      : (INV && is_pow2(H) && H >= 4096 && HGP_ROWG_PAIRS_LONG_INV > 0) ? HGP_ROWG_PAIRS_LONG_INV
                      : (INV && H == 2048 && HGP_ROWG_PAIRS_2048_INV > 0) ? HGP_ROWG_PAIRS_2048_INV
                      : (H >= 4096 && HGP_ROWG_PAIRS_LONG > 0) ? HGP_ROWG_PAIRS_LONG
                                                              : 8 / G;   // 2C rows x G columns = 128 B (fp32)
    int c = (TT > 64 ? HGP_ROWT_PAIRS_BIG : HGP_ROWT_PAIRS) * 64 / TT;   // 512 threads at the default
    if (INV && is_pow2(H) && H >= 1024 && TT == 64 && HGP_ROWT_PAIRS_INV > 0) c = HGP_ROWT_PAIRS_INV;
    if (INV && !is_pow2(H) && TT > 64 && HGP_ROWT_THREADS_TRI_INV > 0) c = HGP_ROWT_THREADS_TRI_INV / TT;
    if (!INV && !is_pow2(H) && TT > 64 && HGP_ROWT_THREADS_TRI_FWD > 0 &&
        (HGP_ROWT_THREADS_TRI_FWD / TT) * 2 * (int)sizeof(C2<T>) >= 64)
      c = HGP_ROWT_THREADS_TRI_FWD / TT;
    if (c < 1) c = 1;
    if (c > 64) c = 64;                            // tiny rows: cap the tile height
    while (c > 1 && (c * TT > 1024 || lds_bytes_for(c) > LDS_CAP)) c >>= 1;
    return c;
  }
  static constexpr int C = c_pairs();
  static constexpr int THREADS = C * TT;
  static constexpr int AREA = area(C);
  static constexpr int LDS = lds_bytes_for(C);
  static constexpr int PITCH = TS(C);
  static constexpr bool WAVE = TT <= 64;
  static constexpr int BLOCKS_BY_LDS = LDS_CAP / LDS;
  static constexpr int MINW_LDS = (BLOCKS_BY_LDS * ((THREADS + 63) / 64)) / 4;
  static constexpr int MINW = MINW_LDS < 1 ? 1 : (MINW_LDS > 4 ? 4 : MINW_LDS);
  static constexpr bool SHORT_SEG = 2 * C * G * (int)sizeof(C2<T>) < 128;
  static constexpr bool XCD_INV = HGP_ROW_XCD >= 2 || (HGP_ROW_XCD == 1 && SHORT_SEG);
  static constexpr bool XCD_FWD = HGP_ROW_XCD == 3;
  // one tile chunk as 128-B units: (column group, row, column in group), column fastest
  static constexpr int SEG = 2 * C * G;                           // elements per group segment
  static constexpr int MAXGRP = (CHC + 1 + G - 1) / G + 1;        // groups a chunk can touch
  static constexpr int ITER = (MAXGRP * SEG + THREADS - 1) / THREADS;
};

// element offset of compact column c, row i0 of one RHS's intermediate (column pitch S0).
// G = 4 is the "quad" order (hgp_pass.hpp LAY_CONTIG_Q): a group's 128-B unit of 4 rows x 4
// columns holds two 64-B halves of 2 columns x 4 rows, (row, column) column-fastest in each, so
// that the axis-0 pass's 2-line blocks write whole halves; the row passes move whole units either
// way (S0 is a multiple of 16, a block's first row a multiple of 4)
template <int G>
__device__ __forceinline__ uint32_t wg_off(int c, int i0, int64_t S0) {
  if constexpr (G == 1) return (uint32_t)c * (uint32_t)S0 + (uint32_t)i0;
  if constexpr (G == 4 && HGP_QUAD)
    return (uint32_t)(c >> 2) * (uint32_t)S0 * 4u + (uint32_t)quad_pos(i0) + (uint32_t)((c >> 1) & 1) * 8u + (uint32_t)(c & 1);
  return ((uint32_t)(c / G) * (uint32_t)S0 + (uint32_t)i0) * (uint32_t)G + (uint32_t)(c % G);
}

// columns [a, b) of tile chunk j of frequency half `half`, relative to the half's first column
template <int H, int NCH, int CHC>
__device__ __forceinline__ void chunk_cols(int half, int j, int& a, int& b) {
  const int ncol = half == 0 ? H / 2 + 1 : H / 2;
  a = j * CHC;
  b = (j == NCH - 1) ? ncol : (j + 1) * CHC;
}

template <bool REMAP>
__device__ __forceinline__ int row_block_id() {
  return REMAP ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
}

// The forward row transform of a block's row pairs after their even-half inputs are in va and
// their odd-half inputs (before the twiddle) in vb (Re = row 2l, Im = row 2l+1, positions
// t + TT k < H: va = x[p] + x[p+H], vb = x[p] - x[p+H], = x[p] both for rows of <= H values):
// twiddled odd half, both halves' FFTs,
// Hermitian split, and the transposed half spectra out to the intermediate (column pitch S0,
// grouped by G).  Needs the twiddle table staged in `tab`; uses the LDS area from `lds`.
template <typename T, int H, int P, int G, bool SEQ = false, typename Cfg = RowTCfg<T, H, G>>
__device__ __forceinline__ void row_fwd_tail(C2<T> (&va)[P], C2<T> (&vb)[P],
                                             C2<T>* lds, const C2<T>* tab, const C2<T>* __restrict__ twg, int t,
                                             int l, int lbase, C2<T>* W, int64_t S0, int row0, int nrow_blk,
                                             bool dcny = false) {
  constexpr int TT = Cfg::TT, C = Cfg::C, PITCH = Cfg::PITCH, NCH = Cfg::NCH, CHC = Cfg::CHC, SEG = Cfg::SEG;
  static_assert(P == Cfg::P, "row_fwd_tail: P");
#pragma unroll
  for (int k = 0; k < P; ++k) vb[k] = cmul<T>(vb[k], tw_at<T, H>(tab, t + TT * k));
  const BufRsrc rW = buf_rsrc(W, 0x7fffffffu);     // one RHS's slab: < 2 GiB (checked on the host)
  // both frequency halves' transforms, interleaved over the group's exchange image (SEQ: one
  // after the other, 32 fewer live VGPRs -- the row-inverse kernel's EPI_RF tail)
  fft_line2<T, H, P, -1, 1, Cfg::WAVE, SEQ>(va, vb, lds, lbase, t, tab);
  auto do_half = [&](auto half_c, C2<T>(&v)[P]) {
    constexpr int half = decltype(half_c)::value;
    constexpr int C0 = (half == 0) ? 0 : H / 2 + 1;
    // Hermitian split through this group's exchange image
    xsync<Cfg::WAVE>();
#pragma unroll
    for (int k = 0; k < P; ++k) lds[lds_phys(lbase + t + TT * k)] = v[k];
    xsync<Cfg::WAVE>();
    C2<T> A[P], B[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = t + TT * k;
      const int pp = (half == 0) ? herm_partner0<H>(p) : (H - 1 - p);
      const C2<T> zp = lds[lds_phys(lbase + pp)];
      herm_split<T>(v[k], zp, A[k], B[k]);
    }
    if constexpr (half == 0) {
      // packed DC / Nyquist (PassDesc::dcny): both real, both held by thread 0 (positions 0 and
      // H / 2 = TT P / 2): column 0 carries DC + i Nyquist (column H / 2 is stored but unread)
      if (dcny && t == 0) {
        A[0] = mk<T>(A[0].x, A[P / 2].x);
        B[0] = mk<T>(B[0].x, B[P / 2].x);
      }
    }
    __syncthreads();   // every group done with its exchange image: the tile overlays them
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      int ca, cb;
      chunk_cols<H, NCH, CHC>(half, j, ca, cb);
      // tile[col - ca][row]: col = compact column relative to the half, row = 2l + {0,1}
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        if (p >= ca && p < cb && l < C) {
          lds[(p - ca) * PITCH + 2 * l] = A[k];
          lds[(p - ca) * PITCH + 2 * l + 1] = B[k];
        }
      }
      __syncthreads();
      // 128-B units: column group, row, column in the group (columns of other chunks / halves
      // in a straddled group are left to them)
      const int g0 = (C0 + ca) / G;
#pragma unroll
      for (int it = 0; it < Cfg::ITER; ++it) {
        const int e = threadIdx.x + it * Cfg::THREADS;
        const int gr = e / SEG;
        const int rem = e - gr * SEG;
        const int row = rem / G;
        const int c = (g0 + gr) * G + (rem - row * G);     // absolute compact column
        if (c >= C0 + ca && c < C0 + cb && row < nrow_blk)
          buf_st_c2<T>(lds[(c - C0 - ca) * PITCH + row], rW, wg_off<G>(c, row0 + row, S0) * (uint32_t)sizeof(C2<T>));
      }
      __syncthreads();   // tile read before the next chunk / half reuses the area
    }
  };
  do_half(std::integral_constant<int, 0>{}, va);
  do_half(std::integral_constant<int, 1>{}, vb);
}

// Real row pairs -> column-major compact half spectra.
//   in : View{x, q_stride (elements per RHS), r_stride (row pitch), 1, len = row length}
//   out: View{W, q_stride (complex per RHS), r_stride = column pitch S0, 1, 0}  (grouped by G)
//   Q RHS, Rn pairs per RHS (= ceil(nrows / 2)), grid = Q * ceil(Rn / C).
template <typename T, int H, int G>
__global__ __launch_bounds__((RowTCfg<T, H, G>::THREADS), (RowTCfg<T, H, G>::MINW)) void k_row_fwd_t(const PassDesc d) {
  using Cfg = RowTCfg<T, H, G>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C;
  if (d.done != nullptr && *d.done) return;
  row_stagger<Cfg::THREADS>();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  C2<T>* tab = lds + Cfg::AREA;
  const C2<T>* __restrict__ twg = reinterpret_cast<const C2<T>*>(d.tw);
  stage_tw<T, H>(tab, twg, threadIdx.x, Cfg::THREADS);
  const int nrb = (d.Rn + C - 1) / C;
  const int lb = row_block_id<Cfg::XCD_FWD>();
  const int q = lb / nrb;
  const int rb = lb - q * nrb;
  // a pair's line spans whole waves at every H used here (TT >= 64): l is wave-uniform (scalar
  // register, scalar row bases), t's known range folds the half-table sign tests
  const int l = (TT % 64 == 0) ? __builtin_amdgcn_readfirstlane(threadIdx.x / TT) : threadIdx.x / TT;
  const int t = threadIdx.x & (TT - 1);
  const int lbase = l * H;
  const int rp = rb * C + l;                       // this group's pair
  const bool pvalid = (l < C) && (rp < d.Rn);
  const int row_a = pvalid ? 2 * rp : 0;
  const bool has2 = pvalid && (2 * rp + 1 < d.nrows);
  const T* in_a = reinterpret_cast<const T*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)row_a * d.in.r_stride;
  const T* in_b = has2 ? in_a + d.in.r_stride : in_a;
  const int in_len = d.in.len;

  C2<T> va[P], vb[P];
  // rows longer than H (the R operator's n-grid input when L_R = 3 * 2^k < 2n): folded halves.
  // The (uniform) fold test selects one of two straight-line load sequences: a branch inside the
  // unrolled loop splits its batch of loads (C2 row forward 0.082 -> 0.10 ms).
  auto load_rows = [&](auto fold_c) {
    constexpr bool FOLD = decltype(fold_c)::value;
    if constexpr (TT % 64 == 0) {
      // raw buffer loads (the pair is wave-uniform): past the row length (zero padding) and for
      // absent rows they return 0
      const BufRsrc ra = buf_rsrc(in_a, pvalid ? (uint32_t)in_len * (uint32_t)sizeof(T) : 0u);
      const BufRsrc rb_ = buf_rsrc(in_b, has2 ? (uint32_t)in_len * (uint32_t)sizeof(T) : 0u);
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const uint32_t lo = (uint32_t)t * (uint32_t)sizeof(T), so = (uint32_t)(TT * k * (int)sizeof(T));
        va[k] = mk<T>(buf_ld<T>(ra, lo, so), buf_ld<T>(rb_, lo, so));
        vb[k] = va[k];
        if constexpr (FOLD) {
          const uint32_t sh = so + (uint32_t)(H * (int)sizeof(T));
          const C2<T> hi = mk<T>(buf_ld<T>(ra, lo, sh), buf_ld<T>(rb_, lo, sh));
          vb[k] = csub<T>(va[k], hi);
          va[k] = cadd<T>(va[k], hi);
        }
      }
    } else {
      // several pairs per wave: the row bases differ between lanes, and a buffer resource must be
      // wave-uniform (a per-lane base costs a readfirstlane loop per load: 2x the VALU of the
      // whole kernel at H = 128).  One resource from the block's first row instead (its 2C rows
      // lie within 2 GiB of it, checked on the host), per-lane 32-bit offsets; positions past the
      // row, absent pairs and absent second rows read at an offset past the range (returns 0)
      const T* blk = reinterpret_cast<const T*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)(2 * rb * C) * d.in.r_stride;
      const BufRsrc rbk = buf_rsrc(blk, 0x7fffffffu);
      constexpr uint32_t DROP = 0x80000000u;
      const uint32_t oa = (uint32_t)(2 * l) * (uint32_t)d.in.r_stride, ob = oa + (uint32_t)d.in.r_stride;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        const bool ok = p < in_len;
        const T a = buf_ld<T>(rbk, (ok && pvalid) ? (oa + (uint32_t)p) * (uint32_t)sizeof(T) : DROP);
        const T b = buf_ld<T>(rbk, (ok && has2) ? (ob + (uint32_t)p) * (uint32_t)sizeof(T) : DROP);
        va[k] = mk<T>(a, b);
        vb[k] = va[k];
        if constexpr (FOLD) {
          const bool ok2 = p + H < in_len;
          const T a2 = buf_ld<T>(rbk, (ok2 && pvalid) ? (oa + (uint32_t)(p + H)) * (uint32_t)sizeof(T) : DROP);
          const T b2 = buf_ld<T>(rbk, (ok2 && has2) ? (ob + (uint32_t)(p + H)) * (uint32_t)sizeof(T) : DROP);
          const C2<T> hi = mk<T>(a2, b2);
          vb[k] = csub<T>(va[k], hi);
          va[k] = cadd<T>(va[k], hi);
        }
      }
    }
  };
  if (in_len > H) load_rows(std::true_type{});
  else load_rows(std::false_type{});
  __syncthreads();   // twiddle table staged
  C2<T>* W = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride;
  const int row0 = 2 * rb * C;                     // first row of this block's tile
  const int nrow_blk = d.nrows - row0 < 2 * C ? d.nrows - row0 : 2 * C;
  row_fwd_tail<T, H, P, G>(va, vb, lds, tab, twg, t, l, lbase, W, d.out.r_stride, row0, nrow_blk, d.dcny > 0);
}

// Column-major compact half spectra -> real row pairs (crop), optional fused dot.
//   in : View{W, q_stride, r_stride = column pitch S0, 1, 0}
//   out: View{y, q_stride (elements per RHS), r_stride (row pitch), 1, len = out row length}
//   nrows = output rows per RHS, Rn = ceil(nrows / 2); dot/partial as in k_pass.
// Fused PCG update of one block's output rows y (staged in LDS, `ys` [row][col], pitch
// out_len), streamed with the row layout of the (nrhs, M) vectors:
//   EPI_XR (y = A p):     x += a p;  r -= a y;  returns this thread's share of r.r  (cg.py:67-69)
//   EPI_R  (y = A p):     r -= a y;  returns this thread's share of r.r           (cg.py:68-69)
//   EPI_XP (y = C^-1 r):  x += a p;  p = y + b p  (the iteration's x update, deferred) (cg.py:67, 75)
//   EPI_RF (y = A p):     as EPI_R, and the new r values overwrite y in `ys` (the caller then
//                         transforms them for the C^-1 pass)
// x is never read by the recurrence, so moving its update from the A p pass to the C^-1 r pass
// (where p is read anyway) saves one read of p per iteration with the same arithmetic; a
// break after the r update is finished by the EPI_XP pass alone (PassDesc::cg_fix).
// Four elements per thread are loaded before any is stored (the vectors never alias).
// (Measured and not kept, round 4: a software-pipelined sweep -- 8 elements per batch, the next
// batch's loads issued before the current one is stored, shift-based indices -- C2 compute_kn
// 17.3 -> 19.1 ms.  The epilogue's cost is structural: an 8-RHS C2 dispatch is ONE round of
// blocks per CU, so the r / p / x loads start only after the FFT and nothing overlaps them.)
template <typename T, int EPI, int THREADS>
__device__ __forceinline__ T cg_epilogue(const T* __restrict__ ys, int nrow, int out_len, T* __restrict__ xg,
                                         T* __restrict__ rg, T* __restrict__ pg, int64_t rpitch, T coef,
                                         T coef2 = 0) {
  const int nel = nrow * out_len;
  // the block's rows are one < 2 GiB window of each vector: raw buffers, 32-bit lane offsets
  const BufRsrc rp = buf_rsrc(pg, 0x7fffffffu), rx = buf_rsrc(xg, 0x7fffffffu), rr = buf_rsrc(rg, 0x7fffffffu);
  T s = 0;
  for (int e0 = threadIdx.x; e0 < nel; e0 += 4 * THREADS) {
    uint32_t g[4];
    T yv[4], pv[4], xv[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * THREADS;
      const int ee = e < nel ? e : nel - 1;
      const int row = ee / out_len;
      const int c = ee - row * out_len;
      g[u] = ((uint32_t)row * (uint32_t)rpitch + (uint32_t)c) * (uint32_t)sizeof(T);
      yv[u] = ys[ee];
      if constexpr (!epi_r(EPI)) pv[u] = buf_ld<T>(rp, g[u]);
      if constexpr (EPI == EPI_XR || EPI == EPI_XP) xv[u] = buf_ld<T>(rx, g[u]);
      if constexpr (EPI == EPI_XR || epi_r(EPI)) rv[u] = buf_ld<T>(rr, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + u * THREADS < nel) {
        if constexpr (EPI == EPI_XR || epi_r(EPI)) {
          if constexpr (EPI == EPI_XR) buf_st<T>(xv[u] + coef * pv[u], rx, g[u]);
          const T rn = rv[u] - coef * yv[u];
          buf_st<T>(rn, rr, g[u]);
          if constexpr (EPI == EPI_RF) const_cast<T*>(ys)[e0 + u * THREADS] = rn;   // this thread's own slot
          s += rn * rn;
        } else {
          buf_st<T>(xv[u] + coef2 * pv[u], rx, g[u]);
          buf_st<T>(yv[u] + coef * pv[u], rp, g[u]);
        }
      }
    }
  }
  return s;
}

// The x update of an iteration whose break test fired after its r update (EPI_XP pass of that
// iteration, nothing else of it runs): x += a p over the block's rows.
template <typename T, int THREADS>
__device__ __forceinline__ void cg_fix_x(int nrow, int out_len, T* __restrict__ xg, const T* __restrict__ pg,
                                         int64_t rpitch, T a) {
  const int nel = nrow * out_len;
  for (int e = threadIdx.x; e < nel; e += THREADS) {
    const int row = e / out_len;
    const int64_t o = (int64_t)row * rpitch + (e - row * out_len);
    xg[o] = xg[o] + a * pg[o];
  }
}

template <typename T, int H, int EPI = EPI_OUT, int G = 1>
__global__ __launch_bounds__((RowTCfg<T, H, G, true>::THREADS), (RowTCfg<T, H, G, true>::MINW)) void k_row_inv_t(const PassDesc d) {
  using Cfg = RowTCfg<T, H, G, true>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C, PITCH = Cfg::PITCH, NCH = Cfg::NCH, CHC = Cfg::CHC;
  constexpr int SEG = Cfg::SEG;
  // staged rows (2C x out_len <= 2C x H values) + two wave-sum areas fit the LDS area
  static_assert((2 * C * H + 2 * (Cfg::THREADS / 64)) * (int)sizeof(T) <= Cfg::AREA * (int)sizeof(C2<T>), "epilogue LDS");
  const int nrb = (d.Rn + C - 1) / C;
  const int lb = row_block_id<Cfg::XCD_INV>();
  const int q = lb / nrb;
  const int rb = lb - q * nrb;
  if (d.done != nullptr) {
    const int dv = *d.done;                      // uniform
    if (dv != 0) {
      if constexpr (EPI == EPI_XP) {
        if (dv == d.cg_fix) {                    // the break fired in this iteration
          const int row0 = 2 * rb * C;
          const int nrow_blk = d.nrows - row0 < 2 * C ? d.nrows - row0 : 2 * C;
          const int64_t g0 = (int64_t)q * d.out.q_stride + (int64_t)row0 * d.out.r_stride;
          const T a = reinterpret_cast<const T*>(d.cg_coef2)[d.cg_div > 1 ? q / d.cg_div : q];
          cg_fix_x<T, Cfg::THREADS>(nrow_blk, d.out.len, reinterpret_cast<T*>(d.cg_x) + g0,
                                    reinterpret_cast<const T*>(d.cg_p) + g0, d.out.r_stride, a);
        }
      }
      return;
    }
  }
  row_stagger<Cfg::THREADS>();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  C2<T>* tab = lds + Cfg::AREA;
  const C2<T>* __restrict__ twg = reinterpret_cast<const C2<T>*>(d.tw);
  stage_tw<T, H>(tab, twg, threadIdx.x, Cfg::THREADS);
  // a pair's line spans whole waves at every H used here (TT >= 64): l is wave-uniform (scalar
  // register, scalar row bases), t's known range folds the half-table sign tests
  const int l = (TT % 64 == 0) ? __builtin_amdgcn_readfirstlane(threadIdx.x / TT) : threadIdx.x / TT;
  const int t = threadIdx.x & (TT - 1);
  const int lbase = l * H;
  const int rp = rb * C + l;
  const bool pvalid = (l < C) && (rp < d.Rn);
  const bool has2 = pvalid && (2 * rp + 1 < d.nrows);
  const C2<T>* W = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride;
  const int64_t S0 = d.in.r_stride;
  const BufRsrc rW = buf_rsrc(W, 0x7fffffffu);     // one RHS's slab: < 2 GiB (checked on the host)
  const int row0 = 2 * rb * C;
  const int nrow_blk = d.nrows - row0 < 2 * C ? d.nrows - row0 : 2 * C;

  C2<T> va[P], vb[P];
  // The tile chunks (frequency half, column chunk) go through the same LDS area one after the
  // other; each chunk's global loads are issued before the previous chunk is rebuilt from LDS,
  // so their memory latency overlaps that work.  Chunk u = half * NCH + j.
  constexpr int NU = 2 * NCH;
  constexpr int ITER = Cfg::ITER;
  C2<T> buf[ITER];
  auto load_tile = [&](int u) {
    const int half = u / NCH;
    int ca, cb;
    chunk_cols<H, NCH, CHC>(half, u - half * NCH, ca, cb);
    const int C0 = half == 0 ? 0 : H / 2 + 1;
    const int g0 = (C0 + ca) / G;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {         // all global loads in flight at once
      const int e = threadIdx.x + it * Cfg::THREADS;
      const int gr = e / SEG;
      const int rem = e - gr * SEG;
      const int row = rem / G;
      int c = (g0 + gr) * G + (rem - row * G);
      const bool ok = c >= C0 + ca && c < C0 + cb && row < nrow_blk;
      if (!ok) c = C0 + ca;                      // clamped in-bounds address, zeroed below
      C2<T> val = buf_ld_c2<T>(rW, wg_off<G>(c, row0 + (ok ? row : 0), S0) * (uint32_t)sizeof(C2<T>));
      if (!ok) val = mk<T>(0, 0);
      buf[it] = val;
    }
  };
  auto park_tile = [&](int u) {
    const int half = u / NCH;
    int ca, cb;
    chunk_cols<H, NCH, CHC>(half, u - half * NCH, ca, cb);
    const int C0 = half == 0 ? 0 : H / 2 + 1;
    const int g0 = (C0 + ca) / G;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int e = threadIdx.x + it * Cfg::THREADS;
      const int gr = e / SEG;
      const int rem = e - gr * SEG;
      const int row = rem / G;
      const int c = (g0 + gr) * G + (rem - row * G);
      if (c >= C0 + ca && c < C0 + cb && row < 2 * C) lds[(c - C0 - ca) * PITCH + row] = buf[it];
    }
  };
  // Hermitian rebuild Z = A + iB of the pair at frequency half `half`, position p, for the
  // positions whose compact column lies in the chunk [ca, cb) (relative to the half)
  auto rebuild = [&](int u, C2<T>(&v)[P]) {
    const int half = u / NCH;
    int ca, cb;
    chunk_cols<H, NCH, CHC>(half, u - half * NCH, ca, cb);
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = t + TT * k;
      bool cj;
      int c;
      if (half == 0) { cj = p > H / 2; c = cj ? H - p : p; }
      else { cj = p >= H / 2; c = cj ? H - 1 - p : p; }
      if (NCH == 1 || (c >= ca && c < cb)) {
        const int li = l < C ? l : 0;
        // packed DC / Nyquist (PassDesc::dcny, NCH = 1): positions 0 and H / 2 of the even half
        // both read column 0, the DC as its real and the Nyquist as its imaginary part
        const bool pk = NCH == 1 && d.dcny > 0 && half == 0 && (p == 0 || p == H / 2);
        const int cc = pk ? 0 : c;
        C2<T> A = lds[(cc - ca) * PITCH + 2 * li];
        C2<T> B = lds[(cc - ca) * PITCH + 2 * li + 1];
        if (pk) {
          A = p == 0 ? mk<T>(A.x, (T)0) : mk<T>(A.y, (T)0);
          B = p == 0 ? mk<T>(B.x, (T)0) : mk<T>(B.y, (T)0);
        }
        if (!has2) B = mk<T>(0, 0);
        if (cj) { A.y = -A.y; B.y = -B.y; }
        v[k] = herm_join<T>(A, B);
      }
    }
  };
  load_tile(0);
  // in-kernel CG scalar: the RHS's spectral partials are loaded behind the first tile (their
  // latency hides under the tile's) and summed per thread and per wave right after it lands;
  // the wave sums are combined in the epilogue (cg_scalar)
  T csum = 0;
  if constexpr (EPI != EPI_OUT) {
    if (d.cg_sp != nullptr) {   // uniform
      const int qc = d.cg_div > 1 ? q / d.cg_div : q;
      const T* sp = reinterpret_cast<const T*>(d.cg_sp) + (int64_t)qc * d.cg_np;
      const int lim = d.cg_np - 1;
      T cv[CG_LOADS];
#pragma unroll
      for (int u = 0; u < CG_LOADS; ++u) {
        const int i = threadIdx.x + u * Cfg::THREADS;
        cv[u] = 0;
        if (u * Cfg::THREADS < d.cg_np)     // uniform: only the rounds that hold partials
          cv[u] = sp[i < lim ? i : lim];    // (clamped) loads, the tail zeroed below
      }
#pragma unroll
      for (int u = 0; u < CG_LOADS; ++u)
        if (threadIdx.x + u * Cfg::THREADS < d.cg_np) csum += cv[u];
    }
  }
  __syncthreads();   // twiddles staged (the tile area is free)
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    park_tile(u);
    __syncthreads();
    if (u + 1 < NU) load_tile(u + 1);            // in flight during this chunk's rebuild
    if (u < NCH) rebuild(u, va);
    else rebuild(u, vb);
    __syncthreads();   // chunk consumed (the last: the FFT exchange images overlay the tile)
  }
  fft_line2<T, H, P, +1, 1, Cfg::WAVE>(va, vb, lds, lbase, t, tab);

  // combine: y[p] = ye + conj(W_L^p) yo, y[p+H] = ye - conj(W_L^p) yo; real rows out
  const int out_len = d.out.len;
  if constexpr (EPI != EPI_OUT) {
    // PCG epilogue: stage the block's 2C output rows in LDS, then update the CG vectors in
    // one coalesced sweep (y itself never goes to HBM)
    T* ys = reinterpret_cast<T*>(smem_raw);
    __syncthreads();   // every group is done with its exchange image
    int tt = t;
    asm volatile("" : "+v"(tt));
    if (out_len == H) {
      // rows of exactly H outputs (every power-of-two grid): the even half's positions are all
      // outputs and the odd half's none, so the only tests left are uniform (pair / second row
      // present) -- no per-position exec branches (the 4096-point kernels spilled 9-17 VGPRs with
      // them, to HBM scratch)
      T* ya = ys + (2 * l) * H;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = tt + TT * k;
        const C2<T> y = cadd<T>(va[k], cmulc<T>(vb[k], tw_at<T, H>(tab, p)));
        if (pvalid) {
          ya[p] = y.x;
          if (has2) ya[H + p] = y.y;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = tt + TT * k;
        const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const C2<T> y = hh == 0 ? cadd<T>(va[k], wo) : csub<T>(va[k], wo);
          const int pp = p + hh * H;
          if (pvalid && pp < out_len) {
            ys[(2 * l) * out_len + pp] = y.x;
            if (has2) ys[(2 * l + 1) * out_len + pp] = y.y;
          }
        }
      }
    }
    // wave sums of the CG scalar's partials, behind the staged rows and the r.r partials
    T* red2 = ys + 2 * C * out_len + Cfg::THREADS / 64;
    if (d.cg_sp != nullptr) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) csum += __shfl_xor(csum, off, 64);
      if ((threadIdx.x & 63) == 0) red2[threadIdx.x >> 6] = csum;
    }
    __syncthreads();
    const int64_t g0 = (int64_t)q * d.out.q_stride + (int64_t)row0 * d.out.r_stride;
    const int qc = d.cg_div > 1 ? q / d.cg_div : q;
    T coef;
    if (d.cg_sp != nullptr) {
      T tot = 0;
#pragma unroll
      for (int w = 0; w < Cfg::THREADS / 64; ++w) tot += red2[w];   // wave order: deterministic
      const T rs = reinterpret_cast<const T*>(d.cg_rs)[qc];
      if constexpr (EPI == EPI_XR || epi_r(EPI)) {
        coef = rs / tot;
        if (epi_r(EPI) && d.cg_alpha_out != nullptr && rb == 0 && threadIdx.x == 0 &&
            (d.cg_div <= 1 || q % d.cg_div == 0))
          reinterpret_cast<T*>(d.cg_alpha_out)[qc] = coef;   // for this iteration's EPI_XP
      } else {
        coef = tot / rs;
        if (rb == 0 && threadIdx.x == 0 && (d.cg_div <= 1 || q % d.cg_div == 0))
          reinterpret_cast<T*>(d.cg_rs_out)[qc] = tot;
      }
    } else {
      coef = reinterpret_cast<const T*>(d.cg_coef)[qc];
    }
    T* pg = reinterpret_cast<T*>(d.cg_p) + g0;
    T* xg = !epi_r(EPI) ? reinterpret_cast<T*>(d.cg_x) + g0 : pg;
    T* rg = EPI != EPI_XP ? reinterpret_cast<T*>(d.cg_r) + g0 : pg;
    const T coef2 = EPI == EPI_XP ? reinterpret_cast<const T*>(d.cg_coef2)[qc] : (T)0;
    T s = cg_epilogue<T, EPI, Cfg::THREADS>(ys, nrow_blk, out_len, xg, rg, pg, d.out.r_stride, coef, coef2);
    if constexpr (EPI == EPI_XR || epi_r(EPI)) {   // deterministic block sum of r.r -> partial [q][rb]
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      T* red = ys + 2 * C * out_len;   // past the staged rows (2C x out_len <= C x H values)
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
      __syncthreads();
      if (threadIdx.x == 0) {
        T tot = 0;
        for (int w = 0; w < Cfg::THREADS / 64; ++w) tot += red[w];
        reinterpret_cast<T*>(d.cg_part)[(int64_t)q * nrb + rb] = tot;
      }
    }
    if constexpr (EPI == EPI_RF) {
      // C^-1 r of the same iteration starts with the forward row transform of r: run it here on
      // the block's rows of the updated r (staged in ys by cg_epilogue), writing them into the
      // same rows of this RHS's intermediate -- this block read those rows' tiles above and no
      // other block touches them, so in place is safe.  The C^-1 op then starts at its axis-0
      // pass, and r is not read back from HBM.  (out_len = the row length: K's output rows are
      // C^-1's input rows, both on the m-grid, at most H values, no fold.)
      C2<T> fa[P], fb[P];
      const T* ra = ys + (2 * l) * out_len;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        const bool in = pvalid && p < out_len;
        const T a = in ? ra[p] : (T)0;
        const T b = (in && has2) ? ra[out_len + p] : (T)0;
        fa[k] = mk<T>(a, b);
        fb[k] = fa[k];
      }
      __syncthreads();   // ys consumed: the exchange images overlay it
      row_fwd_tail<T, H, P, G, HGP_RF_SEQ, Cfg>(fa, fb, lds, tab, twg, t, l, lbase, const_cast<C2<T>*>(W), S0, row0, nrow_blk,
                                           d.dcny > 0);
    }
    return;
  }
  T* out_a = reinterpret_cast<T*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)(pvalid ? 2 * rp : 0) * d.out.r_stride;
  T* out_b = out_a + d.out.r_stride;
  const T* dot_a = nullptr;
  const T* dot_b = nullptr;
  if (d.partial != nullptr) {
    dot_a = reinterpret_cast<const T*>(d.dot) + (out_a - reinterpret_cast<T*>(d.out.ptr));
    dot_b = dot_a + d.out.r_stride;
  }
  T dsum = 0;
  int tt = t;
  asm volatile("" : "+v"(tt));
  if constexpr (TT % 64 == 0) {
    // the pair is wave-uniform: raw buffer stores from the rows' scalar bases with 32-bit lane
    // offsets; the resource ranges crop (pp >= out_len) and drop an absent pair / second row, so
    // no per-position branch or 64-bit address is formed.  (Plain stores here held a 64-bit
    // address per position under per-position exec branches: the 4096-point kernel spilled 13
    // VGPRs, and its scratch traffic went to HBM.)
    const uint32_t rowb = (uint32_t)out_len * (uint32_t)sizeof(T);
    const BufRsrc ra = buf_rsrc(out_a, pvalid ? rowb : 0u);
    const BufRsrc rb2 = buf_rsrc(out_b, has2 ? rowb : 0u);
    const uint32_t lo = (uint32_t)tt * (uint32_t)sizeof(T);
    auto put = [&](auto dot_c) {
      constexpr bool DOT = decltype(dot_c)::value;
      BufRsrc da, db;
      if constexpr (DOT) {
        da = buf_rsrc(dot_a, pvalid ? rowb : 0u);
        db = buf_rsrc(dot_b, has2 ? rowb : 0u);
      }
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = tt + TT * k;
        const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if (hh * H < out_len) {               // uniform: does this half reach the output at all
            const C2<T> y = hh == 0 ? cadd<T>(va[k], wo) : csub<T>(va[k], wo);
            const uint32_t so = (uint32_t)(TT * k + hh * H) * (uint32_t)sizeof(T);
            buf_st<T>(y.x, ra, lo, so);
            buf_st<T>(y.y, rb2, lo, so);
            if constexpr (DOT) {                // loads past the range return 0; the select keeps
              const bool in = p + hh * H < out_len;   // a cropped (never stored) value out of the sum
              const T xa = buf_ld<T>(da, lo, so), xb = buf_ld<T>(db, lo, so);
              dsum += in ? y.x * xa : (T)0;      // the plain path's order: row a, then row b
              dsum += in ? y.y * xb : (T)0;
            }
          }
        }
      }
    };
    if (dot_a != nullptr) put(std::true_type{});
    else put(std::false_type{});
  } else if (dot_a == nullptr) {
    // several pairs per wave (TT < 64): one buffer resource from the block's first row (uniform;
    // the block's 2C rows lie within 2 GiB of it, checked on the host), per-lane 32-bit offsets,
    // and masked positions sent past the range (dropped) instead of per-position exec branches
    T* blk = reinterpret_cast<T*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)(2 * rb * C) * d.out.r_stride;
    const BufRsrc ro = buf_rsrc(blk, 0x7fffffffu);
    const uint32_t rowa = (uint32_t)(2 * l) * (uint32_t)d.out.r_stride, rowp = (uint32_t)d.out.r_stride;
    constexpr uint32_t DROP = 0x80000000u;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = tt + TT * k;
      const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (hh * H < out_len) {
          const C2<T> y = hh == 0 ? cadd<T>(va[k], wo) : csub<T>(va[k], wo);
          const int pp = p + hh * H;
          const bool in = pvalid && pp < out_len;
          const uint32_t oa = (rowa + (uint32_t)pp) * (uint32_t)sizeof(T);
          buf_st<T>(y.x, ro, in ? oa : DROP);
          buf_st<T>(y.y, ro, (in && has2) ? oa + rowp * (uint32_t)sizeof(T) : DROP);
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = tt + TT * k;
      const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const C2<T> y = hh == 0 ? cadd<T>(va[k], wo) : csub<T>(va[k], wo);
        const int pp = p + hh * H;
        if (pvalid && pp < out_len) {
          out_a[pp] = y.x;
          if (dot_a != nullptr) dsum += y.x * dot_a[pp];
          if (has2) {
            out_b[pp] = y.y;
            if (dot_a != nullptr) dsum += y.y * dot_b[pp];
          }
        }
      }
    }
  }
  if (d.partial != nullptr) {   // uniform over the block
    const T s = line_sum<T, TT>(dsum, reinterpret_cast<T*>(smem_raw));
    if (t == 0 && pvalid) reinterpret_cast<T*>(d.partial)[(int64_t)q * d.Rn + rp] = s;
  }
}

}  // namespace hgp
