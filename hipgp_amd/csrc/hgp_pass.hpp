// hgp_pass.hpp — one axis pass of a batched multi-dimensional Toeplitz convolution.
//
// A "pass" runs length-L = 2H transforms along one axis for a batch of lines:
//   FWD  : load (pad/fold) -> forward FFT -> store both frequency halves      (first axes)
//   INV  : load both halves -> inverse FFT -> combine, crop -> store           (last axes)
//   CONV : load -> forward -> x spectrum -> inverse -> crop -> store           (axis 0)
// Two right-hand sides b = 2q, 2q+1 travel together as the real and imaginary parts of one
// complex line ("real pair"): every operator here is a convolution with a REAL filter, so
// the two never mix (Re -> op(v_2q), Im -> op(v_2q+1)).
//
// Layouts (compile time):
//   LAY_STRIDED : complex lines along a non-last axis; C adjacent lines per block, threads
//                 line-fast so each position is one coalesced C*8-byte row segment.
//   LAY_CONTIG  : complex lines along the last axis; threads position-fast.
//   LAY_RP      : last axis of the (nrhs, M) real vectors: the pair (2q, 2q+1) is loaded
//                 /stored as two real rows (input of FWD/CONV, output of INV/CONV).
#pragma once
#include "hgp_fft.hpp"

namespace hgp {

enum { PASS_FWD = 0, PASS_INV = 1, PASS_CONV = 2 };
enum { LAY_STRIDED = 0, LAY_CONTIG = 1, LAY_RP = 2 };
enum { SPEC_REAL = 0, SPEC_CPLX = 1, SPEC_CPLX_CONJ = 2 };

struct View {
  void* ptr;
  int64_t q_stride;           // per pair (complex elems) / per RHS row (reals, LAY_RP: row b)
  int64_t r_stride;           // per outer line index r
  int64_t p_stride;           // per position (complex views; 1 for contiguous)
  int len;                    // valid length along the axis (input: in_len, output: out_len)
};

struct PassDesc {
  View in, out;
  const void* dot;            // optional: second operand (same layout as `out`, LAY_RP only)
  void* partial;              // fused dot partials [b][Rn]
  const void* spec;           // CONV: spectrum at i*spec_i + r*spec_r + kperm*spec_p
  int64_t spec_i, spec_p, spec_r;
  int spec_kind;
  const void* tw;             // W_L^q, q < L (forward sign)
  int nrhs;                   // valid RHS count (pairs: b = 2q, 2q+1)
  int Q;                      // pairs
  int Rn, In;                 // lines per pair: r in [0,Rn) (outer), i in [0,In) (inner, strided)
  const int* done;            // optional device flag: skip the pass when *done != 0
};

template <typename T, int H, int LAY> struct PassCfg {
  static constexpr int P = (H < PMax<T>::v) ? H : PMax<T>::v;
  static constexpr int TT = H / P;
  static constexpr int lds_bytes_for(int c) { return (c * H + ((c * H) >> 4)) * (int)sizeof(C2<T>); }
  static constexpr int c_strided() {
    int c = 64;
    while (c > 1 && (c * TT > 512 || lds_bytes_for(c) > 140 * 1024)) c >>= 1;
    return c;
  }
  static constexpr int c_contig() {
    int c = (TT >= 256) ? 1 : 256 / TT;
    while (c > 1 && lds_bytes_for(c) > 64 * 1024) c >>= 1;
    return c;
  }
  static constexpr int C = (LAY == LAY_STRIDED) ? c_strided() : c_contig();
  static constexpr int THREADS = C * TT;
  static constexpr int LDS_FFT = (TT > 1) ? lds_bytes_for(C) : 0;
  static constexpr int LDS_RED = THREADS * 2 * (int)sizeof(T);
  static constexpr int LDS = LDS_FFT > LDS_RED ? LDS_FFT : LDS_RED;
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
// ids, so the pairs q of one strided line group (same spectrum slab) run on one XCD and share
// its L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int x = b & 7, qq = nb >> 3, rr = nb & 7;
  const int start = (x < rr) ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq;
  return start + (b >> 3);
}

template <typename T, int H, int MODE, int LAY>
__global__ __launch_bounds__((PassCfg<T, H, LAY>::THREADS)) void k_pass(const PassDesc d) {
  using Cfg = PassCfg<T, H, LAY>;
  constexpr int P = Cfg::P, TT = Cfg::TT, C = Cfg::C;
  constexpr bool RP_IN = (LAY == LAY_RP) && (MODE != PASS_INV);
  constexpr bool RP_OUT = (LAY == LAY_RP) && (MODE != PASS_FWD);
  if (d.done != nullptr && *d.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  C2<T>* lds = reinterpret_cast<C2<T>*>(smem_raw);
  const C2<T>* __restrict__ twL = reinterpret_cast<const C2<T>*>(d.tw);

  const int tid = threadIdx.x;
  int l, t, lbase;
  constexpr int LSTRIDE = (LAY == LAY_STRIDED) ? C : 1;
  if constexpr (LAY == LAY_STRIDED) { t = tid / C; l = tid - t * C; lbase = l; }
  else { l = tid / TT; t = tid - l * TT; lbase = l * H; }

  // ---- line coordinates (q, r, i) ----
  int q, r, i;
  bool valid;
  if constexpr (LAY == LAY_STRIDED) {
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int g = lb / d.Q;
    q = lb - g * d.Q;
    const int GI = (d.In + C - 1) / C;
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
  const bool has_b = (2 * q + 1 < d.nrhs);   // second member of the pair exists

  // ---- base pointers (64-bit, per line) ----
  const T* in_re = nullptr; const T* in_im = nullptr; const C2<T>* in_c = nullptr;
  if constexpr (RP_IN) {
    in_re = reinterpret_cast<const T*>(d.in.ptr) + (int64_t)(2 * q) * d.in.q_stride + (int64_t)r * d.in.r_stride;
    in_im = in_re + d.in.q_stride;
  } else {
    in_c = reinterpret_cast<const C2<T>*>(d.in.ptr) + (int64_t)q * d.in.q_stride + (int64_t)r * d.in.r_stride + i;
  }
  T* out_re = nullptr; T* out_im = nullptr; C2<T>* out_c = nullptr;
  if constexpr (RP_OUT) {
    out_re = reinterpret_cast<T*>(d.out.ptr) + (int64_t)(2 * q) * d.out.q_stride + (int64_t)r * d.out.r_stride;
    out_im = out_re + d.out.q_stride;
  } else {
    out_c = reinterpret_cast<C2<T>*>(d.out.ptr) + (int64_t)q * d.out.q_stride + (int64_t)r * d.out.r_stride + i;
  }
  const int64_t ips = (LAY == LAY_STRIDED) ? d.in.p_stride : 1;
  const int64_t ops = (LAY == LAY_STRIDED) ? d.out.p_stride : 1;

  // Loads are unconditional on clamped (always in-bounds) addresses and zeroed afterwards:
  // a per-element branch around a load makes hipcc wait vmcnt(0) per element.
  const T* in_im_safe = nullptr;
  if constexpr (RP_IN) in_im_safe = has_b ? in_im : in_re;
  auto load_in = [&](int p) -> C2<T> {
    if constexpr (RP_IN) {
      const T re = in_re[p];
      const T im = in_im_safe[p];
      return mk<T>(re, has_b ? im : (T)0);
    } else {
      return in_c[(int64_t)p * ips];
    }
  };

  C2<T> v[P];
  C2<T> keep[P];   // FWD/CONV: odd-half input; INV/CONV: even-half output
  T dsum_a = 0, dsum_b = 0;

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
        v[k] = cadd<T>(a, c);
        keep[k] = cmul<T>(csub<T>(a, c), twL[p]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int p = t + TT * k;
        C2<T> a = load_in(p < in_len ? p : lim);
        if (p >= in_len) a = mk<T>(0, 0);
        v[k] = a;
        keep[k] = cmul<T>(a, twL[p]);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = load_in(t + TT * k);
  }

#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    if constexpr (MODE == PASS_FWD) {
      if (half == 1) {
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = keep[k];
      }
      fft_line<T, H, P, -1, LSTRIDE>(v, lds, lbase, t, twL);
      if (valid) {
#pragma unroll
        for (int k = 0; k < P; ++k) out_c[(int64_t)(half * H + t + TT * k) * ops] = v[k];
      }
    } else {
      if constexpr (MODE == PASS_CONV) {
        fft_line<T, H, P, -1, LSTRIDE>(v, lds, lbase, t, twL);
        const int64_t sb = (int64_t)i * d.spec_i + (int64_t)r * d.spec_r + (int64_t)(half * H + t) * d.spec_p;
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = spec_mul<T>(d.spec_kind, d.spec, sb + (int64_t)(TT * k) * d.spec_p, v[k]);
      } else {  // INV: half 0 input loaded above; half 1 loads the odd frequencies
        if (half == 1) {
#pragma unroll
          for (int k = 0; k < P; ++k) {
            keep[k] = v[k];
            v[k] = load_in(H + t + TT * k);
          }
        }
      }
      fft_line<T, H, P, +1, LSTRIDE>(v, lds, lbase, t, twL);
      if (half == 0) {
        if constexpr (MODE == PASS_CONV) {
#pragma unroll
          for (int k = 0; k < P; ++k) { C2<T> tmp = v[k]; v[k] = keep[k]; keep[k] = tmp; }
        }
      } else {
        // y[p] = ye + conj(W_L^p) yo ;  y[p+H] = ye - conj(W_L^p) yo ; crop to out_len
        const int out_len = d.out.len;
        const T* dot_re = nullptr; const T* dot_im = nullptr;
        if constexpr (RP_OUT) {
          if (d.partial != nullptr) {
            dot_re = reinterpret_cast<const T*>(d.dot) + (int64_t)(2 * q) * d.out.q_stride + (int64_t)r * d.out.r_stride;
            dot_im = dot_re + d.out.q_stride;
          }
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int p = t + TT * k;
          const C2<T> yo = cmulc<T>(v[k], twL[p]);
          const C2<T> y0 = cadd<T>(keep[k], yo);
          const C2<T> y1 = csub<T>(keep[k], yo);
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int pp = p + s2 * H;
            const C2<T> y = s2 ? y1 : y0;
            if (valid && pp < out_len) {
              if constexpr (RP_OUT) {
                out_re[pp] = y.x;
                if (has_b) out_im[pp] = y.y;
                if (dot_re != nullptr) {
                  dsum_a += y.x * dot_re[pp];
                  if (has_b) dsum_b += y.y * dot_im[pp];
                }
              } else {
                out_c[(int64_t)pp * ops] = y;
              }
            }
          }
        }
      }
    }
  }

  if constexpr (RP_OUT) {
    if (d.partial != nullptr) {
      // per-line fused dot: every thread parks its two partial sums, the line's first
      // thread adds them in fixed order (deterministic) and writes partial[b][r].
      T* red = reinterpret_cast<T*>(smem_raw);
      __syncthreads();
      red[2 * tid] = dsum_a;
      red[2 * tid + 1] = dsum_b;
      __syncthreads();
      if (t == 0 && valid) {
        T sa = 0, sb = 0;
        for (int k = 0; k < TT; ++k) { sa += red[2 * (tid + k)]; sb += red[2 * (tid + k) + 1]; }
        T* part = reinterpret_cast<T*>(d.partial);
        part[(int64_t)(2 * q) * d.Rn + r] = sa;
        if (has_b) part[(int64_t)(2 * q + 1) * d.Rn + r] = sb;
      }
    }
  }
}

}  // namespace hgp
