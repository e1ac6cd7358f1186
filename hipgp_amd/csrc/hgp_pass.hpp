// hgp_pass.hpp — one axis pass of a batched multi-dimensional Toeplitz convolution.
//
// A "pass" runs length-L = 2H transforms along one axis for a batch of lines:
//   FWD  : load (pad/fold) -> forward FFT -> store the frequencies                (first axes)
//   INV  : load frequencies -> inverse FFT -> combine halves, crop -> store         (last axes)
//   CONV : load -> forward -> x spectrum -> inverse -> crop -> store                (axis 0)
//          (PASS_CONV: real spectrum, prefetched with the data so the pass makes a single
//          memory round trip; PASS_CONVC: complex spectrum of the R / R^T ops, loaded per half)
//
// One thread group of TT = H/P threads owns a line and runs its even-frequency half and then
// its odd-frequency half (hgp_fft.hpp) one after the other, re-using one LDS exchange image:
// the input stays in registers between the two halves, and the inverse halves are combined in
// registers (both halves leave position p in the same thread).  The twiddle half-table W_L^q
// (q < H) is staged in LDS once per block, so the FFT issues no global loads at all.
//
// Real data never shares a complex FFT with another right-hand side: the last (real) axis
// packs two ROWS OF THE SAME RHS as Re/Im (rows 2j, 2j+1), splits them after the forward
// transform by Hermitian symmetry and stores each row's half spectrum ("compact" columns
// c = 0..H: even frequencies 2c for c <= H/2, odd 2(c-H/2-1)+1 after).  The inverse rebuilds
// the pair from the two half spectra.  Rounding therefore only couples values of one RHS
// (error ~ eps*||v_b||, like a plain 2-D FFT), never two RHS.
//
// Layouts (compile time):
//   LAY_STRIDED : complex lines along a non-last axis; C adjacent lines per block, threads
//                 line-fast so each position is one coalesced C*sizeof(complex) row segment
//                 (C = 16 fp32 lines = one 128-B line at H <= 1024).
//   LAY_CONTIG  : complex lines along the last axis; threads position-fast (setup grids).
//   LAY_RP      : last axis of (nrhs, M) real vectors, row pair (2j, 2j+1) of RHS q
//                 <-> two compact half-spectrum rows (FWD input / INV output).
//   LAY_R1      : 1-D: one real line per RHS (z = x + 0i), CONV only.
//   LAY_CONTIG_G: LAY_CONTIG over the grouped-column intermediate of the long-row 2-D operators
//                 (hgp_rows.hpp): G = d.grp columns interleaved, element (c, p) of one RHS at
//                 ((c / G) * S0 + p) * G + c % G; a block's C lines are the G columns of one group
//                 (x C / G right-hand sides), so the 128-B segments a line touches are used whole
//                 by the block.
//   LAY_SEG_C / LAY_SEG_S: the axis-0 conv of the grid-block (slab) sharding reading the receive
//                 buffer of the all-to-all and writing the send buffer of the return all-to-all
//                 directly (hipgp_amd/slab.py): a line's rows are split over seg_ws ranks in
//                 balanced blocks (rows [a_r, a_r + cnt_r) of rank r), stored per rank block
//                 [r][line][row - a_r][c] (line = g * Q + q over the Rn groups and Q RHS, c < inner):
//                 element (line, row p, c) at NL inner a_r + (line cnt_r + p - a_r) inner + c,
//                 NL = Rn Q.  _C: position-fast lines (d = 2, inner = 1); _S: C adjacent c lines
//                 per block as LAY_STRIDED (d = 3, In lines, inner = in.p_stride).  Input split
//                 over in.len rows, output split over out.len rows.
//   LAY_CONTIG_Q: the grouped intermediate of G = 4 columns in the "quad" order (hgp_rows.hpp
//                 wg_off<4>): within a group's 128-B unit of 4 positions x 4 columns the columns
//                 go in two 64-B halves of 2 columns, each half 4 positions x 2 columns, element
//                 (c, p) at (c / 4) 4 S0 + (p / 4) 16 + ((c / 2) % 2) 8 + (p % 4) 2 + c % 2.  A block
//                 holds the 2 columns of one half (C = 2 lines, position-fast), so its two lines'
//                 stores of the same position fill whole 16-B pairs and every 64-B half of a line
//                 comes from one block at one time (no partially written 32-B sectors, which the
//                 plain G = 4 order with one column per block left to four blocks, C4 K op conv
//                 writes 1.54x their bytes, profiles/r4_C4K_kernel_bytes_final.txt).
//   LAY_CONTIG2 : LAY_CONTIG for the fp32 1024-point K / C^-1 column conv (PASS_CONV) with 32 points
//                 per thread: two lines per wave (TT = 32), radix-32 stages, so one LDS exchange per
//                 transform instead of two.  The wave's two lines share one raw-buffer resource based
//                 at the smaller of their offsets (32-bit lane offsets: the host picks this layout only
//                 when the chunk's intermediate is < 2 GiB, and only for in_len = out_len = H -- no zero
//                 padding and no crop, which the per-line resource ranges of LAY_CONTIG provide).
//   LAY_GRP2 / LAY_GRP4: the grouped-column intermediate as LAY_CONTIG_G, but a block holds the
//                 G = 2 / 4 columns of one group of one RHS with threads column-fast (the strided
//                 mapping, C = G): every load / store instruction of a wave covers one contiguous
//                 64 / G-position run of the group (512 B), instead of G blocks each taking one
//                 column out of every 8 G bytes.
#pragma once
#include <type_traits>

#include "hgp_fft.hpp"

// Block-shape tunables (measured on MI355X):
#ifndef HGP_ROW_THREADS
#define HGP_ROW_THREADS 256      // target block size of the contiguous-line (row) passes
#endif
#ifndef HGP_CMAX_STRIDED
#define HGP_CMAX_STRIDED 16      // max adjacent lines (columns) per strided-pass block
#endif
#ifndef HGP_MINW_STRIDED
#define HGP_MINW_STRIDED 0       // waves/SIMD occupancy hint; 0 = from the LDS footprint
#endif
#ifndef HGP_MINW_STRIDED_SMALL
#define HGP_MINW_STRIDED_SMALL 0 // short lines (< 16 threads per line): from the LDS footprint
#endif
#ifndef HGP_MINW_ROW
#define HGP_MINW_ROW 0
#endif
#ifndef HGP_CONTIG_THREADS
#define HGP_CONTIG_THREADS 512   // complex contiguous lines (2-D column CONV, setup grids)
#endif
// the same for lines of several waves (TT >= 128): one 4096-point line (or two 2048-point lines)
// per block, so that a CU's blocks are small enough for the occupancy chosen below
// (profiles/r3_h_variants_passtime.txt: C4 column pass 2.47 -> 2.00 ms with MINW 3, C3 0.745 -> 0.69 ms)
#ifndef HGP_CONTIG_THREADS_LONG
#define HGP_CONTIG_THREADS_LONG 256
#endif
// the column passes' two half-length transforms one after the other on lines of several waves
// (instead of interleaved over one exchange image, hgp_fft.hpp fft_line2)
#ifndef HGP_SEQ_PASS
#define HGP_SEQ_PASS 0
#endif
// the same for the 2048-point lines (2 waves) only
#ifndef HGP_SEQ_PASS_2048
#define HGP_SEQ_PASS_2048 0
#endif
#ifndef HGP_MINW_CONTIG
#define HGP_MINW_CONTIG 4
#endif
// lines of H <= 512 (several lines per wave: the 3-D axis-0 passes): 256-thread blocks at 3 waves
// per SIMD (the 256-point column kernel spilled 16 VGPRs at 4; C5 K op column pass 2.13 -> 1.74 ms,
// R^T's 384-point one 8.41 -> 7.56 ms, profiles/r3_k_c5_passtime.txt)
#ifndef HGP_MINW_CONTIG_SHORT
#define HGP_MINW_CONTIG_SHORT 3
#endif
#ifndef HGP_CONTIG_THREADS_SHORT
#define HGP_CONTIG_THREADS_SHORT 256
#endif
#ifndef HGP_MINW_CONTIG_LONG
#define HGP_MINW_CONTIG_LONG HGP_MINW_CONTIG   // lines of H = 2048 (multi-wave, two-level twiddles)
#endif
// lines of H = 4096 (4 waves): 3 waves per SIMD (up to 168 VGPRs).  At 4 the 4096-point column kernel
// spilled 23 VGPRs, and every spill went to HBM (PMC: 5.8 of the C4 K op's 24 GB were scratch),
// column pass 2.47 ms; at 3 (1-line blocks, 3 per CU) it spills none: 2.00 ms, traffic 1.15x.
#ifndef HGP_MINW_CONTIG_4096
#define HGP_MINW_CONTIG_4096 3
#endif
// mixed-radix lines of >= 4 waves (the R / R^T 6144- and 12288-point axis-0 convolutions)
#ifndef HGP_MINW_CONTIG_TRI
#define HGP_MINW_CONTIG_TRI HGP_MINW_CONTIG_LONG
#endif
#ifndef HGP_DCNY_CONV
#define HGP_DCNY_CONV 1
#endif
// the G = 4 grouped intermediate in the quad order (LAY_CONTIG_Q; 0: the plain G = 4 order,
// one column per axis-0 block, LAY_CONTIG_G)
#ifndef HGP_QUAD
#define HGP_QUAD 1
#endif
// the quad-order (LAY_CONTIG_Q) column pass of 4096-point lines: lines per block and waves per
// SIMD.  One line per block at 4 waves/SIMD (four 4-wave blocks per CU): C4 K op 4.63 -> 4.54 ms
// (column pass 2.13 -> 2.01 ms against the plain G = 4 order); two lines per block (8-wave blocks,
// whole 64-B halves per block) cut the pass's HBM writes 5.16 -> 3.64 GB per op but ran 2.27 ms,
// and one line at 3 waves/SIMD 2.03 ms (profiles/r5_e_quad_variants.txt)
#ifndef HGP_QUAD_LINES_4096
#define HGP_QUAD_LINES_4096 1
#endif
#ifndef HGP_MINW_CONTIG_Q4096
#define HGP_MINW_CONTIG_Q4096 4
#endif

namespace hgp {

enum { PASS_FWD = 0, PASS_INV = 1, PASS_CONV = 2, PASS_CONVC = 3 };   // CONV: real spectrum, CONVC: complex
enum { LAY_STRIDED = 0, LAY_CONTIG = 1, LAY_RP = 2, LAY_R1 = 3, LAY_CONTIG_G = 4, LAY_SEG_C = 5, LAY_SEG_S = 6,
       LAY_GRP2 = 7, LAY_GRP4 = 8, LAY_CONTIG_Q = 9, LAY_CONTIG2 = 10 };
// element offset of position p within its line in the quad order (LAY_CONTIG_Q, wg_off<4>)
__host__ __device__ constexpr int quad_pos(int p) { return ((p >> 2) << 4) + ((p & 3) << 1); }
// columns per block of the interleaved grouped layouts (0: not one)
constexpr int lay_grp(int lay) { return lay == LAY_GRP2 ? 2 : lay == LAY_GRP4 ? 4 : 0; }
// strided thread mapping (C adjacent lines, threads line-fast) vs position-fast lines
constexpr bool lay_smap(int lay) { return lay == LAY_STRIDED || lay == LAY_SEG_S || lay_grp(lay) > 0; }
enum { SPEC_REAL = 0, SPEC_CPLX = 1, SPEC_CPLX_CONJ = 2 };
// row-inverse epilogue (hgp_rows.hpp): EPI_XR x/r update (unpreconditioned PCG); with the
// preconditioner the x update is deferred to the C^-1 pass: EPI_R r update, EPI_XP x and p
// EPI_RF: EPI_R, then the forward row transform of the updated r rows (the first pass of the
// C^-1 r that follows in the same PCG iteration) into the block's rows of the intermediate
enum { EPI_OUT = 0, EPI_XR = 1, EPI_R = 2, EPI_XP = 3, EPI_RF = 4 };
constexpr bool epi_r(int e) { return e == EPI_R || e == EPI_RF; }

struct View {
  void* ptr;
  int64_t q_stride;           // per RHS (LAY_RP/R1 real side: M; complex side: rows*S)
  int64_t r_stride;           // per outer line index r (LAY_RP: per ROW, not per pair)
  int64_t p_stride;           // per position (strided complex views; 1 otherwise)
  int len;                    // valid length along the axis (input: in_len, output: out_len)
};

struct PassDesc {
  View in, out;
  const void* dot;            // optional: second operand (same layout as the real `out`)
  void* partial;              // fused dot partials [q][Rn]
  const void* spec;           // CONV: spectrum at i*spec_i + r*spec_r + kperm*spec_p
  int64_t spec_i, spec_p, spec_r;
  int spec_kind;
  const void* tw;             // W_L^q, q < L (forward sign); the kernel stages q < H in LDS
  int Q;                      // right-hand sides (setup grids: 1)
  int Rn, In;                 // lines per RHS: r in [0,Rn) (outer), i in [0,In) (inner, strided)
  int nrows;                  // LAY_RP: real rows per RHS (the pair (2r, 2r+1) needs 2r+1 < nrows)
  int grp;                    // LAY_CONTIG_G: columns per group G (r_stride = S0, the group's pitch / G)
  int seg_ws;                 // LAY_SEG_*: ranks the rows are split over
  // 2-D K / C^-1 with the plain column-major intermediate (G = 1): the real DC (c = 0) and
  // Nyquist (c = dcny = H1 / 2) compact columns packed as one complex column at c = 0 (row passes
  // k_row_fwd_t / k_row_inv_t), so the axis-0 pass runs H1 lines per RHS instead of H1 + 1 (a
  // C2 chunk of 8 RHS: 8192 lines = exactly two rounds of resident blocks).  0: not packed.
  int dcny;
  const int* done;            // optional device flag: skip the pass when *done != 0
  // CONV passes: spectral dot of the transformed line with itself weighted by the real
  // spectrum, sum_k S_k |X_k|^2 = <x, op x> by Parseval (the crop is exact: x is zero outside
  // it), stored as spart[q * Rn + r] (strided: spart[(q * Rn + r) * In + i]) x the weight of
  // the compact column r (1 for columns 0 and spart_mid, else 2 = the column and its
  // Hermitian mirror; spart_mid < 0: weight 1).
  void* spart;
  int spart_mid;
  int spart_div;              // > 1: the compact column of line r is r / spart_div (3-D: r = c2 * L1 + k1)
  // fused PCG epilogue of the row-inverse pass (hgp_rows.hpp, EPI_XR / EPI_R / EPI_XP)
  void* cg_r;
  void* cg_x;
  void* cg_p;
  const void* cg_coef;        // per-RHS alpha (EPI_XR, EPI_R) or beta (EPI_XP)
  const void* cg_coef2;       // EPI_XP: per-RHS alpha of the same iteration (x += alpha p)
  void* cg_alpha_out;         // EPI_R with the in-kernel alpha: alpha per RHS for EPI_XP
  int cg_fix;                 // EPI_XP: *done == cg_fix (the break fired in this iteration):
                              // the pass only applies the pending x += alpha p
  void* cg_part;              // EPI_XR: per-block partial sums of r.r  [q][row block]
  int cg_div;                 // > 1: cg_div consecutive q (3-D: the i0 planes of one RHS) share a coefficient
  // in-kernel CG scalar (cg_sp != nullptr; else cg_coef is read): the block sums the RHS's
  // cg_np spectral-dot partials itself (fixed order, so every block of the RHS gets the same
  // bits) -- EPI_XR/R: alpha = cg_rs / sum (cg.py:66); EPI_XP: beta = sum / cg_rs (cg.py:74), and
  // the sum is the next iteration's rs, written to cg_rs_out (cg.py:64).
  const void* cg_sp;
  int cg_np;
  const void* cg_rs;
  void* cg_rs_out;
};

constexpr int LDS_CAP = 160 * 1024;
// at most CG_LOADS partials per thread for the in-kernel CG scalar (the host checks
// cg_np <= CG_LOADS x THREADS, else it passes cg_coef from a k_cg_alpha / k_cg_beta launch)
constexpr int CG_LOADS = 8;

// points per thread of the fp32 contiguous-line passes at tri lengths of >= HGP_TRI_P_CONV_MIN
// points (HGP_TRI_P_CONV; 12 = PFor's): 24 runs radix-8 stages (three exchanges for a 6144-point
// half transform instead of five radix-4 ones) with lines of TT = H / 24 threads.  Measured per
// length (profiles/r5_r_tri_p.txt, R^T conv pass): 6144 (C4) 9.29 -> 7.97 ms; 3072 (C3) 12.37 ->
// 13.80 ms, i.e. slower; 1536 (C2) 0.554 -> 0.547 ms.  So from 6144 points up.
#ifndef HGP_TRI_P_CONV
#define HGP_TRI_P_CONV 24
#endif
#ifndef HGP_TRI_P_CONV_MIN
#define HGP_TRI_P_CONV_MIN 6144
#endif
// points per thread of the fp32 1024-point contiguous-line passes (0: PFor's 16).  8: lines of
// two waves at ~71 VGPRs, HGP_MINW_CONTIG_P8 waves per SIMD -- measured slower (C2 column pass
// 0.17 -> 0.19-0.20 ms, bench op 0.278 -> 0.319 ms: block barriers and a fourth exchange, and
// no DC / Nyquist packing on lines of more than one wave; profiles/r5_y_conv1024_p8.txt)
#ifndef HGP_P_CONV_1024
#define HGP_P_CONV_1024 0
#endif
#ifndef HGP_MINW_CONTIG_P8
#define HGP_MINW_CONTIG_P8 6
#endif
// 32 points per thread: two lines per wave (TT = 32), radix-32 stages; 16 lines per CU as at P = 16
// (the LDS images bound it), in 2 waves per SIMD of up to 256 VGPRs
#ifndef HGP_MINW_CONTIG_P32
#define HGP_MINW_CONTIG_P32 2
#endif
template <typename T, int H, int LAY> struct PassP {
  static constexpr bool CONTIG_LINE = LAY == LAY_CONTIG || LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q || LAY == LAY_CONTIG2;
  static constexpr bool F32 = std::is_same<T, float>::value;
  static constexpr int v = LAY == LAY_CONTIG2 ? 32
                         : (F32 && is_tri(H) && H >= HGP_TRI_P_CONV_MIN && CONTIG_LINE) ? HGP_TRI_P_CONV
                         : (F32 && H == 1024 && CONTIG_LINE && HGP_P_CONV_1024 > 0) ? HGP_P_CONV_1024
                                                                                    : PFor<T, H>::v;
};

template <typename T, int H, int LAY> struct PassCfg {
  static constexpr int P = PassP<T, H, LAY>::v;
  static constexpr int TT = H / P;
  // LDS: exchange image of C lines (H complex each, 1 pad slot per 16) + twiddle half table
  static constexpr int ex_elems(int c) { return c * H + ((c * H) >> 4); }
  static constexpr int TW_BYTES = TwTab<T, H>::BYTES;
  static constexpr int lds_bytes_for(int c) { return ex_elems(c) * (int)sizeof(C2<T>) + TW_BYTES; }
  static constexpr int c_strided() {
    int c = TT >= 16 ? HGP_CMAX_STRIDED : 64;
    while (c > 1 && (c * TT > 1024 || lds_bytes_for(c) > LDS_CAP)) c >>= 1;
    return c;
  }
  static constexpr int ROWT = (LAY == LAY_CONTIG || LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q || LAY == LAY_SEG_C ||
                               LAY == LAY_CONTIG2)
                                  ? (TT >= 128 ? HGP_CONTIG_THREADS_LONG : H <= 512 ? HGP_CONTIG_THREADS_SHORT : HGP_CONTIG_THREADS)
                                  : HGP_ROW_THREADS;
  static constexpr int c_contig() {
    int c = (TT >= ROWT) ? 1 : ROWT / TT;
    while (c > 1 && (c * TT > 1024 || lds_bytes_for(c) > LDS_CAP / 2)) c >>= 1;
    return c;
  }
  // quad order: the 2 lines of a 64-B half per block for the 4-wave (4096-point) lines
  // (HGP_QUAD_LINES_4096); longer lines (the 6144-point R / R^T conv: 8 waves each) keep one
  // line per block -- two made 16-wave blocks, one per CU (C4 R^T conv 8.5 -> 12.7 ms)
  static constexpr int c_quad() {
    const int c = c_contig();
    if (c >= 2) return c;
    return (TT == 256 && HGP_QUAD_LINES_4096 == 2 && lds_bytes_for(2) <= LDS_CAP) ? 2 : 1;
  }
  static constexpr int C = lay_grp(LAY) ? lay_grp(LAY) : lay_smap(LAY) ? c_strided()
                           : LAY == LAY_CONTIG_Q ? c_quad() : c_contig();
  // position-fast layouts keep each line inside one wavefront when TT <= 64: exchanges then
  // need no block barrier (hgp_fft.hpp xsync)
  static constexpr bool WAVE = !lay_smap(LAY) && TT <= 64;
  static constexpr int THREADS = C * TT;
  static constexpr int EX_ELEMS = ex_elems(C);
  static constexpr int LDS = lds_bytes_for(C);
  // occupancy hint (waves per SIMD) from the blocks the LDS footprint lets share a CU
  static constexpr int WAVES_PER_BLOCK = (THREADS + 63) / 64;
  static constexpr int BLOCKS_BY_LDS = LDS_CAP / LDS;
  static constexpr int MINW_LDS = (BLOCKS_BY_LDS * WAVES_PER_BLOCK) / 4;
  static constexpr int MINW_AUTO = MINW_LDS < 1 ? 1 : (MINW_LDS > 4 ? 4 : MINW_LDS);
  // (3 waves per SIMD only for lines of 4 waves: 3 whole blocks per CU)
  static constexpr int MINW_CL = (P == 24) ? 3 : (H == 1024 && P == 8) ? HGP_MINW_CONTIG_P8
                                 : (H == 1024 && P == 32) ? HGP_MINW_CONTIG_P32
                                 : (!is_pow2(H) && TT >= 256) ? HGP_MINW_CONTIG_TRI
                                 : (H >= 4096 && TT == 256) ? HGP_MINW_CONTIG_4096
                                 : H >= 2048 ? HGP_MINW_CONTIG_LONG : H <= 512 ? HGP_MINW_CONTIG_SHORT : HGP_MINW_CONTIG;
  // a block's waves must fit the SIMDs' share at once: >= WAVES_PER_BLOCK / 4 waves per SIMD
  static constexpr int MINW_BLK = (WAVES_PER_BLOCK + 3) / 4;
  // quad-order blocks of 4096-point lines (4 waves each): HGP_MINW_CONTIG_Q4096 waves per SIMD
  static constexpr int MINW_Q = P == 24 ? 3 : TT == 256 ? HGP_MINW_CONTIG_Q4096 : MINW_CL;
  static constexpr int MINW_SET = lay_grp(LAY) ? (MINW_CL > MINW_BLK ? MINW_CL : MINW_BLK)
                                 : lay_smap(LAY) ? (TT >= 16 ? HGP_MINW_STRIDED : HGP_MINW_STRIDED_SMALL)
                                 : LAY == LAY_CONTIG_Q ? (MINW_Q > MINW_BLK ? MINW_Q : MINW_BLK)
                                 : (LAY == LAY_CONTIG || LAY == LAY_CONTIG_G || LAY == LAY_SEG_C || LAY == LAY_CONTIG2) ? MINW_CL
                                                                                                  : HGP_MINW_ROW;
  static constexpr int MINW = MINW_SET > 0 ? MINW_SET : MINW_AUTO;
};

template <typename T>
__device__ __forceinline__ C2<T> spec_mul(int kind, const void* spec, int64_t soff, C2<T> x) {
  if (kind == SPEC_REAL) {
    const T s = reinterpret_cast<const T*>(spec)[soff];
    return mk<T>(x.x * s, x.y * s);
  }
  const C2<T> s = reinterpret_cast<const C2<T>*>(spec)[soff];
  return kind == SPEC_CPLX ? cmul<T>(x, s) : cmulc<T>(x, s);
}

// Bijective XCD-aware remap: blocks dealt to the same XCD (b mod 8) get consecutive logical
// ids, so the RHS q of one strided line group (same spectrum slab) run on one XCD and share
// its L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int x = b & 7, qq = nb >> 3, rr = nb & 7;
  const int start = (x < rr) ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;
  return start + (b >> 3);
}

// compact half-spectrum column of frequency half h, position p (valid for the stored range)
template <int H>
__device__ __forceinline__ int compact_col(int h, int p) { return h == 0 ? p : H / 2 + 1 + p; }

// Deterministic sum over the TT consecutive threads of one line (fixed shuffle tree; lines of
// more than one wave add their wave sums in wave order through `red`).  Valid in the line's
// first thread.  Every thread of the block must call it (barriers when TT > 64).
template <typename T, int TT>
__device__ __forceinline__ T line_sum(T v, T* red) {
  constexpr int W = TT < 64 ? TT : 64;
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if constexpr (TT > 64) {
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x % TT == 0) {
      T s = 0;
      const int w0 = threadIdx.x >> 6;
      for (int w = 0; w < TT / 64; ++w) s += red[w0 + w];
      v = s;
    }
  }
  return v;
}

template <typename T, int H, int MODE, int LAY>
__global__ __launch_bounds__((PassCfg<T, H, LAY>::THREADS), (PassCfg<T, H, LAY>::MINW)) void k_pass(const PassDesc d) {
  using Cfg = PassCfg<T, H, LAY>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C;
  constexpr bool RP_IN = (LAY == LAY_RP) && (MODE == PASS_FWD);     // real row pair in
  constexpr bool RP_OUT = (LAY == LAY_RP) && (MODE == PASS_INV);    // real row pair out
  constexpr bool HERM_IN = RP_OUT;                                   // compact half spectra in
  constexpr bool HERM_OUT = RP_IN;                                   // compact half spectra out
  constexpr bool R1 = (LAY == LAY_R1);
  constexpr bool REAL_OUT = RP_OUT || R1;
  // inputs longer than H (folded x[p] +- x[p+H]): the fp64 set-up grids' forward transforms,
  // and the R operator's passes when L_R = 3 * 2^k < 2n (its input lives on the n-grid); the
  // K / C^-1 column pass (PASS_CONV) never folds (in_len <= H, checked on the host)
  constexpr bool CAN_FOLD = MODE == PASS_FWD || MODE == PASS_CONVC;
  if (d.done != nullptr && *d.done) return;                          // uniform: before any barrier
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  C2<T>* tab = lds + Cfg::EX_ELEMS;
  const C2<T>* __restrict__ twg = reinterpret_cast<const C2<T>*>(d.tw);
  stage_tw<T, H>(tab, twg, threadIdx.x, Cfg::THREADS);

  const int tid = threadIdx.x;
  int l, t, lbase;
  constexpr bool SMAP = lay_smap(LAY);
  constexpr bool SEG = (LAY == LAY_SEG_C || LAY == LAY_SEG_S);
  constexpr int LSTRIDE = SMAP ? C : 1;
  if constexpr (SMAP) { t = tid / C; l = tid - t * C; lbase = l; }
  else {
    // lines of whole waves: the line index is wave-uniform, kept in a scalar register so the
    // line's base pointers are scalar and every load/store is base + 32-bit lane offset
    l = (TT % 64 == 0) ? __builtin_amdgcn_readfirstlane(tid / TT) : tid / TT;
    t = tid & (TT - 1);           // TT is a power of two: the known range of t folds the
                                  // half-table sign tests of positions t + TT k < H
    lbase = l * H;
  }

  // ---- line coordinates (q = RHS, r = outer line, i = inner line) ----
  // Strided: q, r and the block's first column i0 are block-uniform (scalar registers); a lane
  // adds a 32-bit element offset lc + p*stride to uniform base pointers, so no 64-bit address
  // is held per position across the FFT.
  int q, r, i, i0 = 0, lc = 0;
  int64_t gbase = 0;          // LAY_CONTIG_G / GRP: element offset of the line's group in its RHS's slab
  bool valid;
  constexpr bool GRP = lay_grp(LAY) > 0;
  if constexpr (GRP) {
    // logical block = (column group, RHS) with the RHS fastest: the XCD remap keeps every RHS of
    // a group (one set of spectrum lines) on one XCD
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int cg = lb / d.Q;
    q = lb - cg * d.Q;
    i0 = cg * C;                    // the group's first column
    r = i0 + l;
    i = 0;
    valid = r < d.Rn;               // the last group's padding columns: computed, never stored
    lc = l;
    gbase = (int64_t)i0 * d.in.r_stride;
  } else if constexpr (SMAP) {
    // logical block = (q, g) with g fastest; the XCD remap keeps consecutive g (adjacent
    // column groups) of one RHS on one XCD.
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int GI = (d.In + C - 1) / C;
    const int G = d.Rn * GI;
    q = lb / G;
    const int g = lb - q * G;
    r = g / GI;
    i0 = (g - r * GI) * C;
    i = i0 + l;
    valid = i < d.In;               // (q, r, i0) of a launched block are always in range
    lc = valid ? l : 0;             // keep every (unconditional) load in bounds
  } else if constexpr (LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q) {
    // lines (cg, q, cl), cl fastest: a block's C lines are the G columns of one group (x C / G
    // RHS), or (quad, C = 2) one 64-B half of them; the XCD remap keeps consecutive groups on one
    // XCD (the two halves of a quad group: consecutive logical blocks)
    const int G = LAY == LAY_CONTIG_Q ? 4 : d.grp;
    const int64_t line = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * C + l;
    const int64_t rest = line / G;
    const int cl = (int)(line - rest * G);
    const int cg = (int)(rest / d.Q);
    q = (int)(rest - (int64_t)cg * d.Q);
    r = cg * G + cl;
    i = 0;
    valid = r < d.Rn;
    if (!valid) { q = 0; r = 0; }
    if constexpr (LAY == LAY_CONTIG_Q) gbase = (int64_t)(r >> 2) * d.in.r_stride * 4 + ((r >> 1) & 1) * 8 + (r & 1);
    else gbase = (int64_t)(r / G) * d.in.r_stride * G + (r % G);
  } else if constexpr (LAY == LAY_CONTIG || LAY == LAY_SEG_C || LAY == LAY_CONTIG2) {
    // RHS-fastest: the C lines of a block are the same column r of C right-hand sides, so
    // they share one spectrum line; the XCD remap keeps the blocks of one column (all its
    // RHS) on one XCD, so the line is fetched into that L2 once.  Packed DC / Nyquist
    // (d.dcny > 0): Rn - 1 lines per RHS, line r >= dcny is column r + 1
    const int64_t line = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * C + l;
    r = (int)(line / d.Q);
    q = (int)(line - (int64_t)r * d.Q);
    i = 0;
    valid = r < (d.dcny > 0 ? d.Rn - 1 : d.Rn);
    if (!valid) { q = 0; r = 0; }
    if (d.dcny > 0 && r >= d.dcny) ++r;
  } else {
    const int64_t line = (int64_t)blockIdx.x * C + l;
    q = (int)(line / d.Rn);
    r = (int)(line - (int64_t)q * d.Rn);
    i = 0;
    valid = q < d.Q;
    if (!valid) { q = 0; r = 0; }
  }
  const bool has2 = (LAY == LAY_RP) ? (2 * r + 1 < d.nrows) : false;   // second row of the pair

  // ---- base pointers ----
  const T* in_re = nullptr; const T* in_im = nullptr;       // real inputs
  const C2<T>* in_c = nullptr; const C2<T>* in_c2 = nullptr; // complex inputs (row b: in_c2)
  if constexpr (RP_IN) {
    in_re = reinterpret_cast<const T*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)(2 * r) * d.in.r_stride;
    in_im = has2 ? in_re + d.in.r_stride : in_re;
  } else if constexpr (R1) {
    in_re = reinterpret_cast<const T*>(d.in.ptr) + (int64_t)q * d.in.q_stride;
  } else if constexpr (HERM_IN) {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)(2 * r) * d.in.r_stride;
    in_c2 = has2 ? in_c + d.in.r_stride : in_c;
  } else if constexpr (SEG) {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr);   // positions by seg_off (the rank blocks)
  } else if constexpr (LAY == LAY_STRIDED) {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)r * d.in.r_stride + i0;
  } else if constexpr (LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q || GRP) {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + gbase;
  } else {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)r * d.in.r_stride;
  }
  T* out_re = nullptr; T* out_im = nullptr;
  C2<T>* out_c = nullptr; C2<T>* out_c2 = nullptr;
  if constexpr (RP_OUT) {
    out_re = reinterpret_cast<T*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)(2 * r) * d.out.r_stride;
    out_im = out_re + d.out.r_stride;
  } else if constexpr (R1) {
    out_re = reinterpret_cast<T*>(d.out.ptr) + (int64_t)q * d.out.q_stride;
  } else if constexpr (HERM_OUT) {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)(2 * r) * d.out.r_stride;
    out_c2 = out_c + d.out.r_stride;
  } else if constexpr (SEG) {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr);
  } else if constexpr (LAY == LAY_STRIDED) {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)r * d.out.r_stride + i0;
  } else if constexpr (LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q || GRP) {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + gbase;
  } else {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)r * d.out.r_stride;
  }
  // element offset of position p in this lane's line (32-bit: one RHS slab < 2^31 elements)
  const int ips = (LAY == LAY_STRIDED) ? (int)d.in.p_stride : (LAY == LAY_CONTIG_G) ? d.grp : GRP ? C : 1;
  const int ops = (LAY == LAY_STRIDED) ? (int)d.out.p_stride : (LAY == LAY_CONTIG_G) ? d.grp : GRP ? C : 1;
  // rank-block layouts: element offset of row p of this lane's line (balanced split of n rows)
  const int s_inner = (LAY == LAY_SEG_S) ? (int)d.in.p_stride : 1;   // element pitch of c
  const int64_t s_line = SEG ? (int64_t)r * d.Q + q : 0;
  const int64_t s_nl = SEG ? (int64_t)d.Rn * d.Q : 0;
  const int s_c = (LAY == LAY_SEG_S) ? i0 + lc : 0;
  auto seg_off = [&](int p, int n) -> int64_t {
    const int ws = d.seg_ws, base = n / ws, extra = n - base * ws;
    const int big = extra * (base + 1);
    const int rk = p < big ? p / (base + 1) : extra + (p - big) / (base > 0 ? base : 1);
    const int a = rk * base + (rk < extra ? rk : extra);
    const int cnt = base + (rk < extra ? 1 : 0);
    return (s_nl * a + s_line * cnt + (p - a)) * s_inner + s_c;
  };
  using Off = std::conditional_t<SEG, int64_t, int>;   // 32-bit lane offsets on the fast layouts
  auto in_at = [&](int p) -> Off {
    if constexpr (SEG) return seg_off(p, d.in.len);
    else if constexpr (LAY == LAY_CONTIG_Q) return quad_pos(p);
    else return (LAY == LAY_STRIDED || GRP) ? lc + p * ips : (LAY == LAY_CONTIG_G) ? p * ips : p;
  };
  auto out_at = [&](int p) -> Off {
    if constexpr (SEG) return seg_off(p, d.out.len);
    else if constexpr (LAY == LAY_CONTIG_Q) return quad_pos(p);
    else return (LAY == LAY_STRIDED || GRP) ? lc + p * ops : (LAY == LAY_CONTIG_G) ? p * ops : p;
  };

  // Loads are unconditional on clamped (always in-bounds) addresses and zeroed afterwards:
  // a per-element branch around a load makes hipcc wait vmcnt(0) per element.
  auto load_in = [&](int p) -> C2<T> {
    if constexpr (RP_IN) {
      const T re = in_re[p];
      const T im = in_im[p];
      return mk<T>(re, has2 ? im : (T)0);
    } else if constexpr (R1) {
      return mk<T>(in_re[p], (T)0);
    } else {
      return in_c[in_at(p)];
    }
  };
  // Hermitian rebuild of Z = A + iB at frequency half h, position p from the two compact rows
  auto load_herm = [&](int h, int p) -> C2<T> {
    bool cj;
    int c;
    if (h == 0) { cj = p > H / 2; c = cj ? H - p : p; }
    else { cj = p >= H / 2; c = H / 2 + 1 + (cj ? H - 1 - p : p); }
    C2<T> A = in_c[c];
    C2<T> B = in_c2[c];
    if (!has2) B = mk<T>(0, 0);
    if (cj) { A.y = -A.y; B.y = -B.y; }
    return herm_join<T>(A, B);
  };
  // second half of an input longer than H (only the fp64 setup grids): x[p + H], or 0
  auto load_hi = [&](int p) -> C2<T> {
    const int in_len = d.in.len;
    const int p2 = p + H;
    C2<T> c = load_in(p2 < in_len ? p2 : in_len - 1);
    if (p2 >= in_len) c = mk<T>(0, 0);
    return c;
  };

  __syncthreads();   // twiddle table staged

  // FWD/CONV: both halves' inputs are formed up front (x dies at once): even x[p] + x[p+H],
  // odd (x[p] - x[p+H]) W_L^p.  Peak live data is two P-arrays in every mode.
  C2<T> va[P], vb[P];
  constexpr bool CONV = MODE == PASS_CONV || MODE == PASS_CONVC;
  // real spectrum: the even half's values are issued together with the data loads, the odd
  // half's right after the even product (in flight during the even IFFT + odd FFT), so at
  // most one half's spectrum is live in registers
  T sre[P];
  T sdot = 0;
  const T* sb = nullptr;
  int so = 0, sp = 0;
  if constexpr (MODE == PASS_CONV) {
    sp = (int)d.spec_p;
    if constexpr (GRP) {            // columns i0 + lc (the padding columns read column i0's)
      sb = reinterpret_cast<const T*>(d.spec) + (int64_t)i0 * d.spec_r;
      so = (valid ? lc : 0) * (int)d.spec_r + t * sp;
    } else {
      sb = reinterpret_cast<const T*>(d.spec) + (int64_t)i0 * d.spec_i + (int64_t)r * d.spec_r;
      so = (SMAP ? lc * (int)d.spec_i : 0) + t * sp;
    }
  }
  // contiguous lines of whole waves: wave-uniform line bases -> raw buffer accesses (32-bit
  // lane offsets; the zero padding beyond in_len and the crop beyond out_len come from the
  // resource's range, invalid lines get an empty range).  fp64 too: its 128-bit stores once
  // raced (round 2, run-to-run different results on lines of >= 4 waves) through the store-data
  // hazard of an SGPR soffset; buf_st_c2<double> no longer uses one (profiles/r3_buf64_race.txt)
#ifndef HGP_BUF_F64
#define HGP_BUF_F64 1
#endif
  constexpr bool QUAD = LAY == LAY_CONTIG_Q;
  constexpr bool CONTIG = (LAY == LAY_CONTIG || LAY == LAY_CONTIG_G || QUAD);
  constexpr bool TWO = LAY == LAY_CONTIG2;   // two lines per wave on one shared resource
  constexpr bool BUF = (std::is_same<T, float>::value || HGP_BUF_F64) && ((CONTIG && (TT % 64 == 0)) || TWO);
  // element stride of a line's positions: 1, or G in the grouped layout; the range then ends
  // one element past the line's last valid position ((len - 1) G + 1 elements).  Quad order:
  // the offset of p = t + x (x a multiple of 4: TT k, H) splits into the lane's quad_pos(t) and
  // 4 x elements; it grows with p, so the range still crops at quad_pos(len - 1) + 1
  const uint32_t es = (uint32_t)(QUAD ? 4 : ips) * (uint32_t)sizeof(C2<T>);
  const uint32_t lane_b = QUAD ? (uint32_t)quad_pos(t) * (uint32_t)sizeof(C2<T>) : (uint32_t)t * es;
  auto range_b = [&](int len, int st) -> uint32_t {
    if (QUAD) return ((uint32_t)quad_pos(len - 1) + 1u) * (uint32_t)sizeof(C2<T>);
    return ((uint32_t)(len - 1) * (uint32_t)st + 1u) * (uint32_t)sizeof(C2<T>);
  };
  // LAY_CONTIG2: the resources start at the smaller of the wave's two line offsets (lanes 0 and
  // 32), each lane adds its line's byte distance from there; invalid lines get an offset past the
  // 2^31 - 1 byte range (their loads return 0, their stores are dropped; the host keeps the chunk's
  // views below 2 GiB, so a valid offset plus the per-position step never reaches it)
  int64_t two_ib = 0, two_ob = 0;
  uint32_t lane_bi = lane_b, lane_bo = lane_b;
  if constexpr (TWO) {
    const int64_t io = (int64_t)q * d.in.q_stride + (int64_t)r * d.in.r_stride;
    const int64_t oo = (int64_t)q * d.out.q_stride + (int64_t)r * d.out.r_stride;
    auto rl = [](int64_t v, int lane) -> int64_t {
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
      return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    two_ib = rl(io, 0) < rl(io, 32) ? rl(io, 0) : rl(io, 32);
    two_ob = rl(oo, 0) < rl(oo, 32) ? rl(oo, 0) : rl(oo, 32);
    lane_bi = valid ? (uint32_t)((io - two_ib) * (int64_t)sizeof(C2<T>)) + lane_b : 0x80000000u;
    lane_bo = valid ? (uint32_t)((oo - two_ob) * (int64_t)sizeof(C2<T>)) + lane_b : 0x80000000u;
  }
  const BufRsrc rin = TWO ? buf_rsrc(reinterpret_cast<const C2<T>*>(d.in.ptr) + two_ib, 0x7fffffffu)
                          : buf_rsrc(BUF ? (const void*)in_c : nullptr, (BUF && valid && d.in.len > 0) ? range_b(d.in.len, ips) : 0u);
  const BufRsrc rout = TWO ? buf_rsrc(reinterpret_cast<const C2<T>*>(d.out.ptr) + two_ob, 0x7fffffffu)
                           : buf_rsrc(BUF ? (const void*)out_c : nullptr, (BUF && valid && d.out.len > 0) ? range_b(d.out.len, ops) : 0u);
  if constexpr (MODE == PASS_FWD || CONV) {
    const int in_len = d.in.len;
    const int lim = in_len - 1;
    // the (uniform) fold test picks one of two straight-line load sequences
    auto load_line = [&](auto fold_c) {
      constexpr bool FOLD = decltype(fold_c)::value;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        C2<T> a;
        if constexpr (BUF) {
          a = buf_ld_c2<T>(rin, lane_bi, (uint32_t)(TT * k) * es);
        } else {
          a = load_in(p < in_len ? p : lim);
          if (p >= in_len) a = mk<T>(0, 0);
        }
        if constexpr (FOLD) {       // beyond in_len the buffer range returns 0
          C2<T> c;
          if constexpr (BUF) c = buf_ld_c2<T>(rin, lane_bi, (uint32_t)(TT * k + H) * es);
          else c = load_hi(p);
          va[k] = cadd<T>(a, c);
          vb[k] = cmul<T>(csub<T>(a, c), tw_at<T, H>(tab, p));
        } else {
          // no second half: x[p] itself (an explicit "+ 0" is not folded -- it maps -0 to +0 --
          // and cost one packed add per point)
          va[k] = a;
          vb[k] = cmul<T>(a, tw_at<T, H>(tab, p));
        }
      }
    };
    if constexpr (CAN_FOLD) {
      if (in_len > H) load_line(std::true_type{});
      else load_line(std::false_type{});
    } else {
      load_line(std::false_type{});
    }
  }

  if constexpr (MODE == PASS_FWD) {
    // both halves' transforms interleaved over one exchange image (hgp_fft.hpp fft_line2)
    fft_line2<T, H, P, -1, LSTRIDE, Cfg::WAVE, (HGP_SEQ_PASS == 2 || ((HGP_SEQ_PASS || HGP_SEQ_MULTIWAVE || (HGP_SEQ_PASS_2048 && TT == 128)) && !Cfg::WAVE))>(va, vb, lds, lbase, t, tab);
    auto fwd_half = [&](auto half_c, C2<T>(&v)[P]) {
      constexpr int half = decltype(half_c)::value;
      if constexpr (HERM_OUT) {
        // split Z = X_a + i X_b by Hermitian symmetry: partner of position p is
        // (H - p) mod H in the even half and H - 1 - p in the odd half.
        xsync<Cfg::WAVE>();
#pragma unroll
        for (int k = 0; k < P; ++k) lds[lds_phys(lbase + t + TT * k)] = v[k];
        xsync<Cfg::WAVE>();
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int p = t + TT * k;
          const int pp = (half == 0) ? herm_partner0<H>(p) : (H - 1 - p);
          const C2<T> zp = lds[lds_phys(lbase + pp)];
          const bool store = (half == 0) ? (p <= H / 2) : (p < H / 2);
          if (valid && store) {
            const int c = compact_col<H>(half, p);
            C2<T> A, B;
            herm_split<T>(v[k], zp, A, B);
            out_c[c] = A;
            if (has2) out_c2[c] = B;
          }
        }
      } else if (valid) {
#pragma unroll
        for (int k = 0; k < P; ++k) out_c[out_at(half * H + t + TT * k)] = v[k];
      }
    };
    fwd_half(std::integral_constant<int, 0>{}, va);
    fwd_half(std::integral_constant<int, 1>{}, vb);
  } else {
    // va ends as the even half's inverse (ye), vb as the odd half's (yo); the two halves'
    // transforms run interleaved over one exchange image (hgp_fft.hpp fft_line2)
    if constexpr (MODE == PASS_CONV) {
      fft_line2<T, H, P, -1, LSTRIDE, Cfg::WAVE, (HGP_SEQ_PASS == 2 || ((HGP_SEQ_PASS || HGP_SEQ_MULTIWAVE || (HGP_SEQ_PASS_2048 && TT == 128)) && !Cfg::WAVE))>(va, vb, lds, lbase, t, tab);
      // the packed DC + i Nyquist line (wave-uniform: one line per wave where the host packs):
      // z = a + i b with a, b the two real columns, each with its own real spectrum S0 / S1:
      // A = (Z + conj Z(-f)) / 2, B = (Z - conj Z(-f)) / 2i (herm_split through this line's LDS
      // image, one frequency half at a time), Y = S0 A + i S1 B, the spectral dot
      // sum S0 |A|^2 + S1 |B|^2 (both columns have Hermitian weight 1).  The spectra are read per
      // position here, so this rarely taken branch (one line in H1) holds no more registers than
      // the common one.
      constexpr bool PLAIN = LAY == LAY_CONTIG || LAY == LAY_CONTIG2;
      const bool packed = HGP_DCNY_CONV && PLAIN && Cfg::WAVE && d.dcny > 0 && r == 0 && valid;
      if constexpr (HGP_DCNY_CONV && PLAIN && Cfg::WAVE) {
        if (packed) {
          const T* sn = sb + (int64_t)d.dcny * d.spec_r;      // the Nyquist column's spectrum
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            xsync<true>();
#pragma unroll
            for (int k = 0; k < P; ++k) lds[lds_phys(lbase + t + TT * k)] = half ? vb[k] : va[k];
            xsync<true>();
#pragma unroll
            for (int k = 0; k < P; ++k) {
              const int p = t + TT * k;
              const int pp = (half == 0) ? herm_partner0<H>(p) : (H - 1 - p);
              const T s0 = sb[so + (half * H + TT * k) * sp];
              const T s1 = sn[so + (half * H + TT * k) * sp];
              C2<T> A, B;
              herm_split<T>(half ? vb[k] : va[k], lds[lds_phys(lbase + pp)], A, B);
              sdot += s0 * (A.x * A.x + A.y * A.y) + s1 * (B.x * B.x + B.y * B.y);
              const C2<T> y = herm_join<T>(cscale<T>(A, s0), cscale<T>(B, s1));
              if (half) vb[k] = y; else va[k] = y;
            }
          }
          xsync<true>();   // partners read before the inverse transform reuses the image
          if (d.spart == nullptr) sdot = 0;
        }
      }
      if (!packed) {
        // the line's real spectrum, loaded after the forward transforms (no registers held across
        // them); L2-resident: every line of a block shares it (RHS-fastest map, XCD-grouped)
        T sre1[P];
        if constexpr (BUF) {
          // (LAY_CONTIG2: the two lines' spectrum columns differ; base at the spectrum, lane offset r)
          const BufRsrc rspec = buf_rsrc(TWO ? reinterpret_cast<const T*>(d.spec) : sb, 0x7fffffffu);
          const uint32_t sso = TWO ? (uint32_t)((int64_t)r * d.spec_r + so) : (uint32_t)so;
#pragma unroll
          for (int k = 0; k < P; ++k) {
            sre[k] = buf_ld<T>(rspec, sso * (uint32_t)sizeof(T), (uint32_t)(TT * k * sp) * (uint32_t)sizeof(T));
            sre1[k] = buf_ld<T>(rspec, sso * (uint32_t)sizeof(T), (uint32_t)((H + TT * k) * sp) * (uint32_t)sizeof(T));
          }
        } else {
#pragma unroll
          for (int k = 0; k < P; ++k) {
            sre[k] = sb[so + TT * k * sp];
            sre1[k] = sb[so + (H + TT * k) * sp];
          }
        }
        if (d.spart != nullptr) {   // uniform: spectral dot sum_k S_k |X_k|^2 of this line
#pragma unroll
          for (int k = 0; k < P; ++k) {
            sdot += sre[k] * (va[k].x * va[k].x + va[k].y * va[k].y);
            sdot += sre1[k] * (vb[k].x * vb[k].x + vb[k].y * vb[k].y);
          }
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
          va[k] = mk<T>(va[k].x * sre[k], va[k].y * sre[k]);
          vb[k] = mk<T>(vb[k].x * sre1[k], vb[k].y * sre1[k]);
        }
      }
    } else if constexpr (MODE == PASS_CONVC) {
      fft_line2<T, H, P, -1, LSTRIDE, Cfg::WAVE, (HGP_SEQ_PASS == 2 || ((HGP_SEQ_PASS || HGP_SEQ_MULTIWAVE || (HGP_SEQ_PASS_2048 && TT == 128)) && !Cfg::WAVE))>(va, vb, lds, lbase, t, tab);
      // complex spectrum at (i, r, kperm): block-uniform base + 32-bit lane offset
      const C2<T>* sbase = reinterpret_cast<const C2<T>*>(d.spec) +
                           (GRP ? (int64_t)i0 * d.spec_r : (int64_t)i0 * d.spec_i + (int64_t)r * d.spec_r);
      const int sp = (int)d.spec_p;
      const int so0 = (GRP ? (valid ? lc : 0) * (int)d.spec_r : SMAP ? lc * (int)d.spec_i : 0) + t * sp;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const C2<T> s0 = sbase[so0 + TT * k * sp];
        const C2<T> s1 = sbase[so0 + (H + TT * k) * sp];
        va[k] = d.spec_kind == SPEC_CPLX ? cmul<T>(va[k], s0) : cmulc<T>(va[k], s0);
        vb[k] = d.spec_kind == SPEC_CPLX ? cmul<T>(vb[k], s1) : cmulc<T>(vb[k], s1);
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        if constexpr (HERM_IN) {
          va[k] = load_herm(0, t + TT * k);
          vb[k] = load_herm(1, t + TT * k);
        } else {
          va[k] = load_in(t + TT * k);
          vb[k] = load_in(H + t + TT * k);
        }
      }
    }
    fft_line2<T, H, P, +1, LSTRIDE, Cfg::WAVE, (HGP_SEQ_PASS == 2 || ((HGP_SEQ_PASS || HGP_SEQ_MULTIWAVE || (HGP_SEQ_PASS_2048 && TT == 128)) && !Cfg::WAVE))>(va, vb, lds, lbase, t, tab);
    // combine in registers: y[p] = ye + conj(W_L^p) yo, y[p+H] = ye - conj(W_L^p) yo; crop.
    const int out_len = d.out.len;
    const T* dot_re = nullptr; const T* dot_im = nullptr;
    if constexpr (REAL_OUT) {
      if (d.partial != nullptr) {
        dot_re = reinterpret_cast<const T*>(d.dot) + (out_re - reinterpret_cast<T*>(d.out.ptr));
        dot_im = dot_re + d.out.r_stride;
      }
    }
    T dsum = 0;
    // opaque copies: positions/offsets are recomputed here instead of being kept live (in
    // registers or scratch) from the loads at the top of the kernel
    asm volatile("" : "+v"(t));
    if constexpr (SMAP) asm volatile("" : "+v"(lc));
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = t + TT * k;
      const C2<T> wo = cmulc<T>(vb[k], tw_at<T, H>(tab, p));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const C2<T> y = hh == 0 ? cadd<T>(va[k], wo) : csub<T>(va[k], wo);
        const int pp = p + hh * H;
        // buffer stores: the resource range crops (and drops invalid lines); only the
        // uniform test whether the half hh reaches the output at all remains
        if (BUF ? (hh * H < out_len) : (valid && pp < out_len)) {
          if constexpr (REAL_OUT) {
            out_re[pp] = y.x;
            if (dot_re != nullptr) dsum += y.x * dot_re[pp];
            if constexpr (RP_OUT) {
              if (has2) {
                out_im[pp] = y.y;
                if (dot_re != nullptr) dsum += y.y * dot_im[pp];
              }
            }
          } else if constexpr (BUF) {
            buf_st_c2<T>(y, rout, lane_bo, (uint32_t)(pp - t) * es);
          } else {
            out_c[out_at(pp)] = y;
          }
        }
      }
    }
    if constexpr (REAL_OUT) {
      if (d.partial != nullptr) {   // uniform over the block
        const T s = line_sum<T, TT>(dsum, reinterpret_cast<T*>(smem_raw));
        if (t == 0 && valid) reinterpret_cast<T*>(d.partial)[(int64_t)q * d.Rn + r] = s;
      }
    }
    if constexpr (MODE == PASS_CONV && !SMAP) {   // CONTIG / CONTIG_G / SEG_C / R1
      if (d.spart != nullptr) {     // uniform over the block
        const T s = line_sum<T, TT>(sdot, reinterpret_cast<T*>(smem_raw));
        if (t == 0 && valid) {
          const int col = d.spart_div > 1 ? r / d.spart_div : r;
          const T w = (d.spart_mid < 0 || col == 0 || col == d.spart_mid) ? (T)1 : (T)2;
          reinterpret_cast<T*>(d.spart)[(int64_t)q * d.Rn + r] = w * s;
          // packed: the Nyquist column's dot is in column 0's; its own slot reads 0
          if (d.dcny > 0 && r == 0) reinterpret_cast<T*>(d.spart)[(int64_t)q * d.Rn + d.dcny] = (T)0;
        }
      }
    } else if constexpr (MODE == PASS_CONV) {
      if (d.spart != nullptr) {     // uniform: a line's TT threads are C apart (t-major ids)
        T* red = reinterpret_cast<T*>(smem_raw);
        __syncthreads();            // the last exchange image is consumed
        red[tid] = sdot;
        __syncthreads();
        if (tid < C && valid) {     // fixed summation order: deterministic
          T s = 0;
          for (int tt2 = 0; tt2 < TT; ++tt2) s += red[tt2 * C + tid];
          const T w = (d.spart_mid < 0 || r == 0 || r == d.spart_mid) ? (T)1 : (T)2;
          reinterpret_cast<T*>(d.spart)[((int64_t)q * d.Rn + r) * d.In + i] = w * s;
        }
      }
    }
  }
}

}  // namespace hgp
