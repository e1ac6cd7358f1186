// hgp_pass.hpp — one axis pass of a batched multi-dimensional Toeplitz convolution.
//
// A "pass" runs length-L = 2H transforms along one axis for a batch of lines:
//   FWD  : load (pad/fold) -> forward FFT -> store the frequencies                (first axes)
//   INV  : load frequencies -> inverse FFT -> combine halves, crop -> store         (last axes)
//   CONV : load -> forward -> x spectrum -> inverse -> crop -> store                (axis 0)
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
//                 line-fast so each position is one coalesced C*8-byte row segment.
//   LAY_CONTIG  : complex lines along the last axis; threads position-fast (setup grids).
//   LAY_RP      : last axis of (nrhs, M) real vectors, row pair (2j, 2j+1) of RHS q
//                 <-> two compact half-spectrum rows (FWD input / INV output).
//   LAY_R1      : 1-D: one real line per RHS (z = x + 0i), CONV only.
#pragma once
#include "hgp_fft.hpp"

namespace hgp {

enum { PASS_FWD = 0, PASS_INV = 1, PASS_CONV = 2 };
enum { LAY_STRIDED = 0, LAY_CONTIG = 1, LAY_RP = 2, LAY_R1 = 3 };
enum { SPEC_REAL = 0, SPEC_CPLX = 1, SPEC_CPLX_CONJ = 2 };

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
  const void* tw;             // W_L^q, q < L (forward sign)
  int Q;                      // right-hand sides (setup grids: 1)
  int Rn, In;                 // lines per RHS: r in [0,Rn) (outer), i in [0,In) (inner, strided)
  int nrows;                  // LAY_RP: real rows per RHS (the pair (2r, 2r+1) needs 2r+1 < nrows)
  const int* done;            // optional device flag: skip the pass when *done != 0
};

template <typename T, int H, int LAY> struct PassCfg {
  static constexpr int P = (H < PMax<T>::v) ? H : PMax<T>::v;
  static constexpr int TT = H / P;
  // LDS image of C lines of one frequency half (H complex each, 1 pad slot per 16)
  static constexpr int half_elems(int c) { return c * H + ((c * H) >> 4); }
  static constexpr int lds_bytes_for(int c) { return 2 * half_elems(c) * (int)sizeof(C2<T>); }
  static constexpr int c_strided() {
    int c = 64;
    while (c > 1 && (2 * c * TT > 1024 || lds_bytes_for(c) > 140 * 1024)) c >>= 1;
    return c;
  }
  static constexpr int c_contig() {
    int c = (2 * TT >= 512) ? 1 : 512 / (2 * TT);
    while (c > 1 && lds_bytes_for(c) > 72 * 1024) c >>= 1;
    return c;
  }
  static constexpr int C = (LAY == LAY_STRIDED) ? c_strided() : c_contig();
  static constexpr int GROUP = C * TT;           // threads of one frequency half
  static constexpr int THREADS = 2 * GROUP;      // even-half group + odd-half group
  static constexpr int HALF_ELEMS = half_elems(C);
  static constexpr int LDS_FFT = lds_bytes_for(C);
  static constexpr int LDS_RED = THREADS * (int)sizeof(T);
  static constexpr int LDS = LDS_FFT > LDS_RED ? LDS_FFT : LDS_RED;
  // occupancy hint (waves per SIMD) -> register budget 512/MINW per lane: aim at 128 VGPRs
  // (4 waves/SIMD) where the LDS footprint lets that many blocks share a CU.
  static constexpr int WAVES_PER_BLOCK = (THREADS + 63) / 64;
  static constexpr int BLOCKS_BY_LDS = LDS > 0 ? (160 * 1024) / LDS : 16;
  static constexpr int MINW_LDS = (BLOCKS_BY_LDS * WAVES_PER_BLOCK) / 4;
  static constexpr int MINW = MINW_LDS < 1 ? 1 : (MINW_LDS > 4 ? 4 : MINW_LDS);
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
  if (d.done != nullptr && *d.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const C2<T>* __restrict__ twL = reinterpret_cast<const C2<T>*>(d.tw);

  // Each block = two thread groups of C lines: group `half` runs the length-H FFT of the
  // even (half=0) or odd (half=1) frequencies of the same lines, in its own LDS image.
  const int half = threadIdx.x / Cfg::GROUP;
  const int tid = threadIdx.x - half * Cfg::GROUP;
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw) + half * Cfg::HALF_ELEMS;
  C2<T>* lds_other = reinterpret_cast<C2<T>*>(smem_raw) + (1 - half) * Cfg::HALF_ELEMS;
  int l, t, lbase;
  constexpr int LSTRIDE = (LAY == LAY_STRIDED) ? C : 1;
  if constexpr (LAY == LAY_STRIDED) { t = tid / C; l = tid - t * C; lbase = l; }
  else { l = tid / TT; t = tid - l * TT; lbase = l * H; }

  // ---- line coordinates (q = RHS, r = outer line, i = inner line) ----
  int q, r, i;
  bool valid;
  if constexpr (LAY == LAY_STRIDED) {
    // logical block = (q, g) with g fastest; the XCD remap keeps consecutive g (adjacent
    // column groups: the two halves of each 128-B line) on one XCD.
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int GI = (d.In + C - 1) / C;
    const int G = d.Rn * GI;
    q = lb / G;
    const int g = lb - q * G;
    r = g / GI;
    i = (g - r * GI) * C + l;
    valid = (r < d.Rn) && (i < d.In);
    if (!valid) { r = 0; i = 0; }     // keep every (unconditional) load in bounds
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
  } else {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)r * d.in.r_stride + i;
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
  } else {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)r * d.out.r_stride + i;
  }
  const int64_t ips = (LAY == LAY_STRIDED) ? d.in.p_stride : 1;
  const int64_t ops = (LAY == LAY_STRIDED) ? d.out.p_stride : 1;

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
      return in_c[(int64_t)p * ips];
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
    return mk<T>(A.x - B.y, A.y + B.x);
  };

  C2<T> v[P];
  T dsum = 0;

  // ---- load this group's half: even x[p]+x[p+H], odd (x[p]-x[p+H]) W_L^p; or frequencies
  if constexpr (MODE == PASS_FWD || MODE == PASS_CONV) {
    const int in_len = d.in.len;
    const int lim = in_len - 1;
    if (in_len > H) {                 // uniform: input longer than H -> fold x[p] and x[p+H]
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        const int p2 = p + H;
        C2<T> a = load_in(p);
        C2<T> c = load_in(p2 < in_len ? p2 : lim);
        if (p2 >= in_len) c = mk<T>(0, 0);
        v[k] = half == 0 ? cadd<T>(a, c) : cmul<T>(csub<T>(a, c), twL[p]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        C2<T> a = load_in(p < in_len ? p : lim);
        if (p >= in_len) a = mk<T>(0, 0);
        v[k] = half == 0 ? a : cmul<T>(a, twL[p]);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if constexpr (HERM_IN) v[k] = load_herm(half, t + TT * k);
      else v[k] = load_in(half * H + t + TT * k);
    }
  }

  if constexpr (MODE == PASS_FWD) {
    fft_line<T, H, P, -1, LSTRIDE>(v, lds, lbase, t, twL);
    if constexpr (HERM_OUT) {
      // split Z = X_a + i X_b by Hermitian symmetry: partner of position p is
      // (H - p) mod H in the even half and H - 1 - p in the odd half (same group).
      __syncthreads();
#pragma unroll
      for (int k = 0; k < P; ++k) lds[lds_phys(lbase + t + TT * k)] = v[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        const int pp = (half == 0) ? ((H - p) & (H - 1)) : (H - 1 - p);
        const C2<T> zp = lds[lds_phys(lbase + pp)];
        const bool store = (half == 0) ? (p <= H / 2) : (p < H / 2);
        if (valid && store) {
          const int c = compact_col<H>(half, p);
          const T hf = (T)0.5;
          out_c[c] = mk<T>(hf * (v[k].x + zp.x), hf * (v[k].y - zp.y));               // (Z + conj Zp)/2
          if (has2) out_c2[c] = mk<T>(hf * (v[k].y + zp.y), -hf * (v[k].x - zp.x));  // (Z - conj Zp)/2i
        }
      }
    } else if (valid) {
#pragma unroll
      for (int k = 0; k < P; ++k) out_c[(int64_t)(half * H + t + TT * k) * ops] = v[k];
    }
  } else {
    if constexpr (MODE == PASS_CONV) {
      fft_line<T, H, P, -1, LSTRIDE>(v, lds, lbase, t, twL);
      const int64_t sb = (int64_t)i * d.spec_i + (int64_t)r * d.spec_r + (int64_t)(half * H + t) * d.spec_p;
#pragma unroll
      for (int k = 0; k < P; ++k) v[k] = spec_mul<T>(d.spec_kind, d.spec, sb + (int64_t)(TT * k) * d.spec_p, v[k]);
    }
    fft_line<T, H, P, +1, LSTRIDE>(v, lds, lbase, t, twL);
    // combine halves through LDS: y[p] = ye + conj(W_L^p) yo (even group stores),
    // y[p+H] = ye - conj(W_L^p) yo (odd group stores); crop to out_len.
    if (half == 1) {
#pragma unroll
      for (int k = 0; k < P; ++k) v[k] = cmulc<T>(v[k], twL[t + TT * k]);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) lds[lds_phys(lbase + (t + TT * k) * LSTRIDE)] = v[k];
    __syncthreads();
    const int out_len = d.out.len;
    const T* dot_re = nullptr; const T* dot_im = nullptr;
    if constexpr (REAL_OUT) {
      if (d.partial != nullptr) {
        dot_re = reinterpret_cast<const T*>(d.dot) + (out_re - reinterpret_cast<T*>(d.out.ptr));
        dot_im = dot_re + d.out.r_stride;
      }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int p = t + TT * k;
      const C2<T> o = lds_other[lds_phys(lbase + p * LSTRIDE)];
      const C2<T> y = half == 0 ? cadd<T>(v[k], o) : csub<T>(o, v[k]);
      const int pp = p + half * H;
      if (valid && pp < out_len) {
        if constexpr (REAL_OUT) {
          out_re[pp] = y.x;
          if (dot_re != nullptr) dsum += y.x * dot_re[pp];
          if constexpr (RP_OUT) {
            if (has2) {
              out_im[pp] = y.y;
              if (dot_re != nullptr) dsum += y.y * dot_im[pp];
            }
          }
        } else {
          out_c[(int64_t)pp * ops] = y;
        }
      }
    }
  }

  if constexpr (REAL_OUT) {
    if (d.partial != nullptr) {
      // per-line fused dot: every thread parks its partial sum; the line's first thread of
      // the even group adds both groups' sums in fixed order (deterministic) -> partial[q][r].
      T* red = reinterpret_cast<T*>(smem_raw);
      __syncthreads();
      red[threadIdx.x] = dsum;
      __syncthreads();
      if (half == 0 && t == 0 && valid) {
        T s = 0;
        for (int k = 0; k < TT; ++k) s += red[tid + k];
        for (int k = 0; k < TT; ++k) s += red[Cfg::GROUP + tid + k];
        reinterpret_cast<T*>(d.partial)[(int64_t)q * d.Rn + r] = s;
      }
    }
  }
}

}  // namespace hgp
