// hgp_fft.hpp — device FFT engine for the Toeplitz/BTTB operators (gfx950, wave64).
//
// What it computes.  Every Toeplitz-type operator of the reference (toeplitz_tensor.py:70-125)
// is a per-axis-separable convolution  y = crop( IFFT_L( S ⊙ FFT_L( pad x ) ) )  with a
// power-of-two length L per axis (see DESIGN.md §2 for why L replaces the reference's
// circulant size n = 2m-2 exactly).  A length-L transform of a line is split into its even
// and odd frequency halves, each an H = L/2 point FFT:
//     X[2k]   = FFT_H( x[p] + x[p+H] )[k]
//     X[2k+1] = FFT_H( (x[p] - x[p+H]) * W_L^p )[k]
// which (a) prunes the zero padding for free (x[p+H] = 0 when the input fits in H) and
// (b) halves the LDS footprint per line.  Frequencies are stored "half-major"
// (index = half*H + k), and every pass/spectrum uses that same order.
//
// One H-point FFT = Stockham autosort stages of radix <= P, where each thread owns the P
// positions {t + T*k, k < P} (T = H/P threads per line).  The first stage reads from
// registers, intermediate stages exchange through LDS, and the last stage leaves the result
// in registers in natural order at the SAME positions — so load, spectrum multiply and
// store all happen in registers with coalesced global accesses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace hgp {

template <typename T> struct cx;
template <> struct cx<float> { using t = float2; };
template <> struct cx<double> { using t = double2; };
template <typename T> using C2 = typename cx<T>::t;

template <typename T> __device__ __forceinline__ C2<T> mk(T a, T b) { C2<T> r; r.x = a; r.y = b; return r; }
template <typename T> __device__ __forceinline__ C2<T> cadd(C2<T> a, C2<T> b) { return mk<T>(a.x + b.x, a.y + b.y); }
template <typename T> __device__ __forceinline__ C2<T> csub(C2<T> a, C2<T> b) { return mk<T>(a.x - b.x, a.y - b.y); }
template <typename T> __device__ __forceinline__ C2<T> cmul(C2<T> a, C2<T> b) {
  return mk<T>(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// a * conj(b)
template <typename T> __device__ __forceinline__ C2<T> cmulc(C2<T> a, C2<T> b) {
  return mk<T>(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
template <typename T> __device__ __forceinline__ C2<T> cscale(C2<T> a, T s) { return mk<T>(a.x * s, a.y * s); }
// a + i b, a - i b
template <typename T> __device__ __forceinline__ C2<T> caddi(C2<T> a, C2<T> b) { return mk<T>(a.x - b.y, a.y + b.x); }
template <typename T> __device__ __forceinline__ C2<T> csubi(C2<T> a, C2<T> b) { return mk<T>(a.x + b.y, a.y - b.x); }
// a * (cr + i ci) for compile-time constants
template <typename T> __device__ __forceinline__ C2<T> cmulk(C2<T> a, T cr, T ci) { return cmul<T>(a, mk<T>(cr, ci)); }

// fp32 complex arithmetic on the packed-f32 VALU (v_pk_add/mul/fma_f32: both components in one
// 64-bit register pair, one instruction where the scalar forms take two; the f32 VALU peak is
// the packed rate).  The backend folds lane selects into op_sel but not a one-lane negation, so
// the forms that need one (complex products, +-i b) are written out.  Each component is computed
// as fma(+-u, v, rn(w z)) -- one rounding per product, like the contracted scalar forms.
#ifndef HGP_PK32
#define HGP_PK32 1
#endif
#if HGP_PK32
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pv(C2<float> a) { return __builtin_bit_cast(f32x2, a); }
__device__ __forceinline__ C2<float> pc(f32x2 v) { return __builtin_bit_cast(C2<float>, v); }
template <> __device__ __forceinline__ C2<float> cadd<float>(C2<float> a, C2<float> b) { return pc(pv(a) + pv(b)); }
template <> __device__ __forceinline__ C2<float> csub<float>(C2<float> a, C2<float> b) { return pc(pv(a) - pv(b)); }
template <> __device__ __forceinline__ C2<float> cscale<float>(C2<float> a, float s) {
  return pc(pv(a) * f32x2{s, s});
}
// One asm block per product: the hazard recognizer pads every VALU read of an inline-asm result
// that follows it directly with an s_nop (it cannot see the asm writes no dst_sel), so a split
// mul / fma pair cost one s_nop per product (140 in the C2 column kernel).
#ifndef HGP_PK_SPLIT
#define HGP_PK_SPLIT 0    // 1: the product as two asm statements (A/B knob)
#endif
#if HGP_PK_SPLIT
template <> __device__ __forceinline__ C2<float> cmul<float>(C2<float> a, C2<float> b) {
  f32x2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(pv(a)), "v"(pv(b)));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(pv(a)), "v"(pv(b)), "v"(t));
  return pc(r);
}
template <> __device__ __forceinline__ C2<float> cmulc<float>(C2<float> a, C2<float> b) {
  f32x2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(pv(a)), "v"(pv(b)));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(r) : "v"(pv(a)), "v"(pv(b)), "v"(t));
  return pc(r);
}
#else
// (ax bx - ay by, ax by + ay bx)
template <> __device__ __forceinline__ C2<float> cmul<float>(C2<float> a, C2<float> b) {
  f32x2 t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r), "=&v"(t) : "v"(pv(a)), "v"(pv(b)));
  return pc(r);
}
// (ax bx + ay by, ay bx - ax by)
template <> __device__ __forceinline__ C2<float> cmulc<float>(C2<float> a, C2<float> b) {
  f32x2 t, r;
  asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
      : "=v"(r), "=&v"(t) : "v"(pv(a)), "v"(pv(b)));
  return pc(r);
}
#endif
template <> __device__ __forceinline__ C2<float> caddi<float>(C2<float> a, C2<float> b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(a)), "v"(pv(b)));
  return pc(r);
}
template <> __device__ __forceinline__ C2<float> csubi<float>(C2<float> a, C2<float> b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(a)), "v"(pv(b)));
  return pc(r);
}
// constant factor: the negated lane lives in the constant, so plain vector code folds to
// v_pk_mul (op_sel) + v_pk_fma (op_sel) with the constants in scalar registers
template <> __device__ __forceinline__ C2<float> cmulk<float>(C2<float> a, float cr, float ci) {
  const f32x2 x = pv(a);
  const f32x2 t = __builtin_shufflevector(x, x, 0, 0) * f32x2{cr, ci};
  return pc(__builtin_elementwise_fma(__builtin_shufflevector(x, x, 1, 1), f32x2{-ci, cr}, t));
}
#endif


// Two real rows packed as Z = a + i b, transformed: their spectra from Z at k and Zp = Z at -k,
// A = (Z + conj Zp) / 2, B = (Z - conj Zp) / 2i (exact halvings, same rounding either form).
template <typename T>
__device__ __forceinline__ void herm_split(C2<T> z, C2<T> zp, C2<T>& A, C2<T>& B) {
  const T hf = (T)0.5;
#if HGP_PK32
  if constexpr (std::is_same<T, float>::value) {
    f32x2 s, d;   // s = z + conj(zp); d = (z.y + zp.y, zp.x - z.x)
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(s) : "v"(pv(z)), "v"(pv(zp)));
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(d) : "v"(pv(z)), "v"(pv(zp)));
    A = pc(s * f32x2{hf, hf});
    B = pc(d * f32x2{hf, hf});
    return;
  }
#endif
  A = mk<T>(hf * (z.x + zp.x), hf * (z.y - zp.y));
  B = mk<T>(hf * (z.y + zp.y), -hf * (z.x - zp.x));
}
// the inverse: Z = A + i B
template <typename T>
__device__ __forceinline__ C2<T> herm_join(C2<T> A, C2<T> B) {
  return caddi<T>(A, B);
}

// Raw buffer access (gfx9 resource word 3 = 0x00020000, stride 0): a wave-uniform base in
// scalar registers plus a 32-bit lane byte offset, so no 64-bit address is formed per access;
// loads at offsets >= `bytes` return 0 and stores there are dropped (used for zero padding,
// cropping and invalid lines without per-element selects).  The lane offset `off` is shared by
// a thread's points; the per-point stride goes in the scalar offset `soff`.
using BufRsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ BufRsrc buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <typename T> __device__ __forceinline__ C2<T> buf_ld_c2(BufRsrc r, uint32_t off, uint32_t soff = 0);
template <> __device__ __forceinline__ C2<float> buf_ld_c2<float>(BufRsrc r, uint32_t off, uint32_t soff) {
  return __builtin_bit_cast(C2<float>, __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0));
}
template <> __device__ __forceinline__ C2<double> buf_ld_c2<double>(BufRsrc r, uint32_t off, uint32_t soff) {
  return __builtin_bit_cast(C2<double>, __builtin_amdgcn_raw_buffer_load_b128(r, off, soff, 0));
}
template <typename T> __device__ __forceinline__ void buf_st_c2(C2<T> v, BufRsrc r, uint32_t off, uint32_t soff = 0);
template <> __device__ __forceinline__ void buf_st_c2<float>(C2<float> v, BufRsrc r, uint32_t off, uint32_t soff) {
  using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V, v), r, off, soff, 0);
}
// 128-bit stores never take an SGPR soffset: a store of more than 8 bytes reads its data VGPRs
// after issue, and a VALU write of them in the next cycle changes the stored data of the last
// lanes (run-to-run different fp64 results on contiguous lines, profiles/r3_buf64_race.txt).
// LLVM's hazard recognizer inserts that wait state only when soffset is NOT a register
// (GCNHazardRecognizer::createsVALUHazard), so the scalar offset is folded into the lane offset
// here; the wait state then follows every such store (tools/hazard_lint.py checks the build).
template <> __device__ __forceinline__ void buf_st_c2<double>(C2<double> v, BufRsrc r, uint32_t off, uint32_t soff) {
  using V = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(V, v), r, off + soff, 0, 0);
}
template <typename T> __device__ __forceinline__ T buf_ld(BufRsrc r, uint32_t off, uint32_t soff = 0);
template <> __device__ __forceinline__ float buf_ld<float>(BufRsrc r, uint32_t off, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0));
}
template <> __device__ __forceinline__ double buf_ld<double>(BufRsrc r, uint32_t off, uint32_t soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0));
}

template <typename T> __device__ __forceinline__ void buf_st(T v, BufRsrc r, uint32_t off, uint32_t soff = 0);
template <> __device__ __forceinline__ void buf_st<float>(float v, BufRsrc r, uint32_t off, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, soff, 0);
}
template <> __device__ __forceinline__ void buf_st<double>(double v, BufRsrc r, uint32_t off, uint32_t soff) {
  using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V, v), r, off, soff, 0);
}

// points per thread: 16 complex in fp32 (32 VGPRs), 8 in fp64 (32 VGPRs)
template <typename T> struct PMax;
template <> struct PMax<float> { static constexpr int v = 16; };
template <> struct PMax<double> { static constexpr int v = 8; };

// Transform half-lengths: powers of two, and H = 3 * 2^j (j >= 2, "tri": the R / R^T lengths
// L_R = 3 * 2^k that replace the next power of two where they are shorter, hgp_plan_create).
constexpr bool is_pow2(int h) { return h > 0 && (h & (h - 1)) == 0; }
constexpr int ilog2c(int h) { return h <= 1 ? 0 : 1 + ilog2c(h >> 1); }
constexpr bool is_tri(int h) { return h >= 12 && h % 3 == 0 && is_pow2(h / 3); }
// points per thread: P = min(H, PMax) for powers of two, 12 for tri lengths (TT = H / 12 then
// stays a power of two, and 12 holds the radix-3 stage)
template <typename T, int H> struct PFor {
  static_assert(is_pow2(H) || is_tri(H), "transform half-length: 2^k or 3 * 2^k (k >= 2)");
  static constexpr int v = is_pow2(H) ? (H < PMax<T>::v ? H : PMax<T>::v) : 12;
};

// Stockham stage radices.  Powers of two: radix P stages (the last one smaller).  Tri lengths:
// radix-4 / -2 stages first and the factor 3 in the LAST stage (radix 3 * min(4, H / 3), which
// divides P = 12): every non-last stage's span NS is then a power of two dividing TT, as the
// exchange index math of fft_xchg needs.
// P = 32 (the 1024-point column lines of two lines per wave, hgp_pass.hpp HGP_P_CONV_1024): radix-32
// stages (1024 = 32 x 32, one LDS exchange per transform instead of two); 0: two radix-16 DFTs per
// stage
#ifndef HGP_RADIX32
#define HGP_RADIX32 1
#endif
template <int H, int P> struct Stages {
  static constexpr bool TRI = !is_pow2(H);
  static constexpr int RMAX = (P >= 32 && HGP_RADIX32) ? 32 : P < 16 ? P : 16;   // in-register DFT size
  // tri lengths: radix-4 stages with P = 12 (three butterflies a thread), radix-8 with P = 24
  static constexpr int RTRI = P % 8 == 0 ? 8 : 4;
  static constexpr int last_tri() { return 3 * (H / 3 >= 4 ? 4 : H / 3); }
  static constexpr int count() {
    if (!TRI) { int n = 0, rem = H; while (rem > 1) { int r = rem >= RMAX ? RMAX : rem; rem /= r; ++n; } return n; }
    int n = 1, rem = H / last_tri();
    while (rem > 1) { rem /= (rem >= RTRI ? RTRI : rem); ++n; }
    return n;
  }
  static constexpr int radix(int s) {
    if (!TRI) { int rem = H; for (int i = 0; i < s; ++i) rem /= (rem >= RMAX ? RMAX : rem); return rem >= RMAX ? RMAX : rem; }
    int rem = H / last_tri(), i = 0;
    while (rem > 1) { const int r = rem >= RTRI ? RTRI : rem; if (i == s) return r; rem /= r; ++i; }
    return last_tri();
  }
  static constexpr int ns(int s) { int v = 1; for (int i = 0; i < s; ++i) v *= radix(i); return v; }
};

// multiply by exp(DIR * 2*pi*i*Q/16), DIR = -1 forward / +1 inverse; Q a compile-time
// constant after unrolling (the switch folds).
template <typename T, int DIR>
__device__ __forceinline__ C2<T> rot16(C2<T> v, int Q) {
  const T c8 = (T)0.70710678118654752440, c1 = (T)0.92387953251128675613, s1 = (T)0.38268343236508977173;
  Q &= 15;
  if (DIR > 0) Q = (16 - Q) & 15;           // inverse: exp(+i th) = forward rotation by -Q
  switch (Q) {                              // forward: multiply by (cos th, -sin th), th=2pi Q/16
    case 0: return v;
    case 4: return mk<T>(v.y, -v.x);
    case 8: return mk<T>(-v.x, -v.y);
    case 12: return mk<T>(-v.y, v.x);
    case 2: return cscale<T>(csubi<T>(v, v), c8);      // (c8 (x + y), c8 (y - x))
    case 6: return cscale<T>(caddi<T>(v, v), -c8);     // (c8 (y - x), -c8 (x + y))
    case 10: return cscale<T>(csubi<T>(v, v), -c8);    // (-c8 (x + y), c8 (x - y))
    case 14: return cscale<T>(caddi<T>(v, v), c8);     // (c8 (x - y), c8 (x + y))
    case 1: return cmulk<T>(v, c1, -s1);
    case 3: return cmulk<T>(v, s1, -c1);
    case 5: return cmulk<T>(v, -s1, -c1);
    case 7: return cmulk<T>(v, -c1, -s1);
    case 9: return cmulk<T>(v, -c1, s1);
    case 11: return cmulk<T>(v, -s1, c1);
    case 13: return cmulk<T>(v, s1, c1);
    default: return cmulk<T>(v, c1, s1);   // 15
  }
}

// multiply by exp(DIR * 2*pi*i*Q/12) (the radix-12 / -6 / -3 stages); Q a compile-time constant.
template <typename T, int DIR>
__device__ __forceinline__ C2<T> rot12(C2<T> v, int Q) {
  const T c = (T)0.86602540378443864676, h = (T)0.5;
  Q %= 12;
  if (DIR > 0) Q = (12 - Q) % 12;           // inverse: exp(+i th) = forward rotation by -Q
  switch (Q) {                              // forward: multiply by (cos th, -sin th), th = 2pi Q/12
    case 0: return v;
    case 3: return mk<T>(v.y, -v.x);
    case 6: return mk<T>(-v.x, -v.y);
    case 9: return mk<T>(-v.y, v.x);
    case 1: return cmulk<T>(v, c, -h);
    case 2: return cmulk<T>(v, h, -c);
    case 4: return cmulk<T>(v, -h, -c);
    case 5: return cmulk<T>(v, -c, -h);
    case 7: return cmulk<T>(v, -c, h);
    case 8: return cmulk<T>(v, -h, c);
    case 10: return cmulk<T>(v, h, c);
    default: return cmulk<T>(v, c, h);    // 11
  }
}

// multiply by exp(DIR * 2*pi*i*Q/32) (the radix-32 DFT's inner twiddles); Q a compile-time
// constant.  Even Q: rot16.
template <typename T, int DIR>
__device__ __forceinline__ C2<T> rot32(C2<T> v, int Q) {
  Q &= 31;
  if ((Q & 1) == 0) return rot16<T, DIR>(v, Q >> 1);
  // cos / sin of 2 pi j / 32, j = 1, 3, 5, 7
  const T c1 = (T)0.98078528040323044913, s1 = (T)0.19509032201612826785;
  const T c3 = (T)0.83146961230254523708, s3 = (T)0.55557023301960222474;
  if (DIR > 0) Q = (32 - Q) & 31;           // inverse: exp(+i th) = forward rotation by -Q
  // forward: multiply by (cos th, -sin th), th = 2 pi Q / 32; Q = 8 m + j with j odd
  switch (Q) {
    case 1: return cmulk<T>(v, c1, -s1);
    case 3: return cmulk<T>(v, c3, -s3);
    case 5: return cmulk<T>(v, s3, -c3);
    case 7: return cmulk<T>(v, s1, -c1);
    case 9: return cmulk<T>(v, -s1, -c1);
    case 11: return cmulk<T>(v, -s3, -c3);
    case 13: return cmulk<T>(v, -c3, -s3);
    case 15: return cmulk<T>(v, -c1, -s1);
    case 17: return cmulk<T>(v, -c1, s1);
    case 19: return cmulk<T>(v, -c3, s3);
    case 21: return cmulk<T>(v, -s3, c3);
    case 23: return cmulk<T>(v, -s1, c1);
    case 25: return cmulk<T>(v, s1, c1);
    case 27: return cmulk<T>(v, s3, c3);
    case 29: return cmulk<T>(v, c3, s3);
    default: return cmulk<T>(v, c1, s1);    // 31
  }
}

// In-register DFT of size R (natural order in and out), R in {1,2,3,4,6,8,12,16,32}.
template <typename T, int R, int DIR>
__device__ __forceinline__ void dft(C2<T>* v) {
  if constexpr (R == 1) {
    return;
  } else if constexpr (R == 3) {
    // y0 = a + s, y1,2 = a - s/2 -+ i DIR' (sqrt(3)/2) d with s = b + c, d = b - c
    const T c = (T)0.86602540378443864676;
    const C2<T> a = v[0], s = cadd<T>(v[1], v[2]), d = csub<T>(v[1], v[2]);
    const C2<T> m = csub<T>(a, cscale<T>(s, (T)0.5));
    // forward: m -+ i c d; inverse: m +- i c d
    const C2<T> cd = cscale<T>(d, c);
    v[0] = cadd<T>(a, s);
    v[1] = (DIR < 0) ? csubi<T>(m, cd) : caddi<T>(m, cd);
    v[2] = (DIR < 0) ? caddi<T>(m, cd) : csubi<T>(m, cd);
  } else if constexpr (R % 3 == 0) {
    // R = R1 x 3 (R1 = 4 or 2): R1-point DFTs of stride 3, twiddles exp(-+2 pi i n2 k1 / R), 3-point DFTs
    constexpr int R1 = R / 3, R2 = 3;
    C2<T> y[R];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) {
      C2<T> a[R1];
#pragma unroll
      for (int n1 = 0; n1 < R1; ++n1) a[n1] = v[R2 * n1 + n2];
      dft<T, R1, DIR>(a);
#pragma unroll
      for (int k1 = 0; k1 < R1; ++k1) y[n2 * R1 + k1] = rot12<T, DIR>(a[k1], (n2 * k1 * (12 / R)) % 12);
    }
#pragma unroll
    for (int k1 = 0; k1 < R1; ++k1) {
      C2<T> b[R2];
#pragma unroll
      for (int n2 = 0; n2 < R2; ++n2) b[n2] = y[n2 * R1 + k1];
      dft<T, R2, DIR>(b);
#pragma unroll
      for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = b[k2];
    }
  } else if constexpr (R == 2) {
    C2<T> a = v[0], b = v[1];
    v[0] = cadd<T>(a, b);
    v[1] = csub<T>(a, b);
  } else if constexpr (R == 4) {
    C2<T> s02 = cadd<T>(v[0], v[2]), d02 = csub<T>(v[0], v[2]);
    C2<T> s13 = cadd<T>(v[1], v[3]), d13 = csub<T>(v[1], v[3]);
    // forward: d02 -+ i d13; inverse: d02 +- i d13
    v[0] = cadd<T>(s02, s13);
    v[2] = csub<T>(s02, s13);
    v[1] = (DIR < 0) ? csubi<T>(d02, d13) : caddi<T>(d02, d13);
    v[3] = (DIR < 0) ? caddi<T>(d02, d13) : csubi<T>(d02, d13);
  } else {
    constexpr int R1 = 4, R2 = R / 4;
    C2<T> y[R];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) {
      C2<T> a[R1];
#pragma unroll
      for (int n1 = 0; n1 < R1; ++n1) a[n1] = v[R2 * n1 + n2];
      dft<T, R1, DIR>(a);
#pragma unroll
      for (int k1 = 0; k1 < R1; ++k1) {
        if constexpr (R == 32) y[n2 * R1 + k1] = rot32<T, DIR>(a[k1], n2 * k1);
        else y[n2 * R1 + k1] = rot16<T, DIR>(a[k1], (n2 * k1 * (16 / R)) & 15);
      }
    }
#pragma unroll
    for (int k1 = 0; k1 < R1; ++k1) {
      C2<T> b[R2];
#pragma unroll
      for (int n2 = 0; n2 < R2; ++n2) b[n2] = y[n2 * R1 + k1];
      dft<T, R2, DIR>(b);
#pragma unroll
      for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = b[k2];
    }
  }
}

// Exchange synchronisation.  WAVE = true when every line of the block lives inside one
// wavefront (position-fast layouts with H/P <= 64 threads per line): a wave's LDS
// instructions execute in order, so only the compiler must be kept from moving LDS accesses
// across the exchange -- no s_barrier.  Otherwise a block barrier.
#ifndef HGP_DIAG_NO_BARRIER
#define HGP_DIAG_NO_BARRIER 0   // 1: DIAGNOSTIC BUILD ONLY (racy, wrong results): no block barrier at
                                // the multi-wave exchanges, to time what those barriers cost
#endif
template <bool WAVE>
__device__ __forceinline__ void xsync() {
  if constexpr (WAVE || HGP_DIAG_NO_BARRIER) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// Twiddles W_L^q (forward sign), q in [0, L = 2H), live in LDS, staged once per block:
//  * half table (H * sizeof(complex) <= HGP_TW_FULL_MAX = 16 KB): tab[q] = W_L^q for q < H, W_L^{q+H} = -W_L^q;
//  * two-level table beyond that (fp64 at H >= 2048, fp32 at H >= 4096: a whole table there
//    halves the blocks a CU holds; 4096^2 K matvec 10.3 -> 6.2 ms): tab = [A | B], A[j] = W_L^j (j < S),
//    B[i] = W_L^{iS} (i < H/S), W_L^q = A[q mod S] B[q div S] (one extra product, ~1 ulp).
#ifndef HGP_TW_FULL_MAX
#define HGP_TW_FULL_MAX (8 * 1024)    // largest half table (bytes) kept whole in LDS (8 KB: the
                                      // grouped 2048-point row blocks then fit two per CU)
#endif
template <typename T, int H> struct TwTab {
  static constexpr bool TWO = H * (int)sizeof(C2<T>) > HGP_TW_FULL_MAX;
  // ceil(log2 H); S = 2^ceil(LG / 2) divides H for every supported H (2^k, 3 * 2^k, k >= 2)
  static constexpr int LG = [] { int l = 0; while ((1 << l) < H) ++l; return l; }();
  static constexpr int S = TWO ? (1 << ((LG + 1) / 2)) : H;
  static constexpr int ENTRIES = TWO ? S + H / S : H;
  static constexpr int BYTES = ENTRIES * (int)sizeof(C2<T>);
};

// copy the table layout above from the global W_L^q array (all threads of the block)
template <typename T, int H>
__device__ __forceinline__ void stage_tw(C2<T>* tab, const C2<T>* __restrict__ twg, int tid, int nthreads) {
  using TW = TwTab<T, H>;
  for (int q = tid; q < TW::ENTRIES; q += nthreads) {
    if constexpr (TW::TWO) tab[q] = q < TW::S ? twg[q] : twg[(q - TW::S) * TW::S];
    else tab[q] = twg[q];
  }
}

// W_L^q for q in [0, 2H) (L = 2H), W_L^{q+H} = -W_L^q
template <typename T, int H>
__device__ __forceinline__ C2<T> tw_at(const C2<T>* __restrict__ tab, int q) {
  using TW = TwTab<T, H>;
  C2<T> w;
  int qq;
  bool neg;
  if constexpr (is_pow2(H)) { qq = q & (H - 1); neg = (q & H) != 0; }
  else { neg = q >= H; qq = neg ? q - H : q; }
  if constexpr (TW::TWO) w = cmul<T>(tab[qq & (TW::S - 1)], tab[TW::S + (qq >> (TW::LG + 1) / 2)]);
  else w = tab[qq];
  if (neg) { w.x = -w.x; w.y = -w.y; }
  return w;
}

// Stage twiddles: a[r] *= w^r (forward) / conj(w)^r (inverse), r = 1..R-1, w = W_H^{kk H/(NS R)}.
// Default: powers by binary powering (at most 4 products deep, ~4 ulp), all R-1 live at once.
// HGP_TW_CHAIN: a running product (one live power: fewer VGPRs, up to R-2 products deep).
#ifndef HGP_TW_CHAIN
#define HGP_TW_CHAIN 0
#endif
template <typename T, int H, int R, int DIR, int NS>
__device__ __forceinline__ void stage_twiddle(C2<T>* a, int kk, const C2<T>* __restrict__ tab) {
#ifdef HGP_DIAG_NO_STAGE_TW
  return;   // DIAGNOSTIC BUILD ONLY (wrong results): tools/isa_mix.py counts what the stage twiddles cost
#endif
  const int q1 = (2 * (H / (NS * R))) * kk;   // w = W_L^q1; w^r = W_L^{q1 r}, q1 r < L
  const C2<T> w = tw_at<T, H>(tab, q1);
  if constexpr (R > 16) {
    // radix 32: w^1..w^7 by binary powering, w^{8m} from the table, w^{8m + j} = w^{8m} w^j (at
    // most 4 products deep, ~20 live VGPRs instead of 62 for all 31 powers)
    C2<T> wp[8];
    wp[1] = w;
#pragma unroll
    for (int r = 2; r < 8; ++r) {
      const int hi = (r & (r - 1)) == 0 ? r / 2 : (1 << (31 - __builtin_clz(r)));
      wp[r] = cmul<T>(wp[hi], wp[r - hi]);
    }
#pragma unroll
    for (int r = 1; r < 8; ++r) a[r] = (DIR < 0) ? cmul<T>(a[r], wp[r]) : cmulc<T>(a[r], wp[r]);
#pragma unroll
    for (int m = 1; m < R / 8; ++m) {
      const C2<T> w8 = tw_at<T, H>(tab, q1 * 8 * m);
      a[8 * m] = (DIR < 0) ? cmul<T>(a[8 * m], w8) : cmulc<T>(a[8 * m], w8);
#pragma unroll
      for (int j = 1; j < 8; ++j) {
        const C2<T> wr = cmul<T>(w8, wp[j]);
        a[8 * m + j] = (DIR < 0) ? cmul<T>(a[8 * m + j], wr) : cmulc<T>(a[8 * m + j], wr);
      }
    }
  } else if constexpr (HGP_TW_CHAIN) {
    C2<T> wr = w;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      if (r > 1) wr = cmul<T>(wr, w);
      a[r] = (DIR < 0) ? cmul<T>(a[r], wr) : cmulc<T>(a[r], wr);
    }
  } else {
    C2<T> wp[R];
    wp[1] = w;
#pragma unroll
    for (int r = 2; r < R; ++r) {
      const int hi = (r & (r - 1)) == 0 ? r / 2 : (1 << (31 - __builtin_clz(r)));   // r = hi + lo
      const int lo = r - hi;
      wp[r] = cmul<T>(wp[hi], wp[lo]);
    }
#pragma unroll
    for (int r = 1; r < R; ++r) a[r] = (DIR < 0) ? cmul<T>(a[r], wp[r]) : cmulc<T>(a[r], wp[r]);
  }
}

// Hermitian partner of position p in the even frequency half: (H - p) mod H
template <int H>
__device__ __forceinline__ int herm_partner0(int p) {
  if constexpr (is_pow2(H)) return (H - p) & (H - 1);
  return p == 0 ? 0 : H - p;
}

// LDS address of logical element e (padding breaks the power-of-two strides of the
// Stockham write pattern: one complex slot per 16).
__device__ __forceinline__ int lds_phys(int e) { return e + (e >> 4); }

// phys(base + x) for a compile-time x: exact split into phys(base) + x*17/16 whenever x is a
// multiple of 16, or when base is 16-aligned and x < 16 (then the pad term is unchanged).
// (x is a constant after loop unrolling, so the branches fold.)
__device__ __forceinline__ int lds_at(int pbase, int base, int x, bool base16) {
  if (x % 16 == 0) return pbase + x + x / 16;
  if (base16 && x < 16) return pbase + x;
  return lds_phys(base + x);
}

// One H-point FFT of the line whose P values this thread holds in v (positions t + T*k,
// k = register index).  Result in v, natural order, same positions.  Line element e of the
// block's LDS image lives at lds_phys(base + e*STRIDE) (STRIDE = 1: line-contiguous image;
// STRIDE = C: lines interleaved).  tab: LDS half table of W_L^q (L = 2H, see tw_at), so
// W_H^e = W_L^{2e}.  All threads of the block must call it when T > 1 (block barriers).
template <typename T, int H, int P, int DIR, int STRIDE, bool WAVE, int S>
__device__ __forceinline__ void fft_stage(C2<T> (&v)[P], C2<T>* lds, int base, int t,
                                          const C2<T>* __restrict__ tab) {
  using St = Stages<H, P>;
  constexpr int NST = St::count();
  if constexpr (S < NST) {
    constexpr int R = St::radix(S), NS = St::ns(S), TT = H / P, NB = P / R;
    C2<T> a[NB][R];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int r = 0; r < R; ++r) a[b][r] = v[b + r * NB];
      if constexpr (NS > 1) {
        const int j = t + b * TT;
        // w = W_H^{kk*H/(NS*R)}: one LDS lookup, its powers in registers (stage_twiddle)
        stage_twiddle<T, H, R, DIR, NS>(a[b], j & (NS - 1), tab);
      }
      dft<T, R, DIR>(a[b]);
    }
    if constexpr (S + 1 < NST) {
      // TT is a multiple of NS at every non-last stage, so butterfly b of this thread
      // writes at idxD(t) + b*TT*R + r*NS.
      const int idxD = (t / NS) * NS * R + (t & (NS - 1));
      const int wb = base + idxD * STRIDE;
      const int pwb = lds_phys(wb);
      constexpr bool WB16 = (STRIDE == 1) && (NS == 1) && (R == 16);   // base 16-aligned
      xsync<WAVE>();   // previous readers of this LDS region are done
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < R; ++r)
          lds[lds_at(pwb, wb, (b * TT * R + r * NS) * STRIDE, WB16)] = a[b][r];
      xsync<WAVE>();
      const int rb = base + t * STRIDE;
      const int prb = lds_phys(rb);
#pragma unroll
      for (int k = 0; k < P; ++k) v[k] = lds[lds_at(prb, rb, TT * k * STRIDE, false)];
      fft_stage<T, H, P, DIR, STRIDE, WAVE, S + 1>(v, lds, base, t, tab);
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < R; ++r) v[b + r * NB] = a[b][r];
    }
  }
}

template <typename T, int H, int P, int DIR, int STRIDE, bool WAVE = false>
__device__ __forceinline__ void fft_line(C2<T> (&v)[P], C2<T>* lds, int base, int t,
                                         const C2<T>* __restrict__ tab) {
  // Opaque copy of t: every twiddle index below is recomputed and re-read from LDS, instead of
  // the compiler keeping the previous transform's twiddles live in VGPRs (that CSE across the
  // two FFTs of a line costs ~50 VGPRs and halves occupancy).
  int tt = t;
  asm volatile("" : "+v"(tt));
  fft_stage<T, H, P, DIR, STRIDE, WAVE, 0>(v, lds, base, tt, tab);
}

// ---- two independent transforms of one thread group, software-pipelined over ONE exchange
// image.  Stage S of transform a exchanges through LDS while the butterflies of transform b
// run (and vice versa), so the LDS write -> read latency of one transform is covered by the
// other's arithmetic instead of stalling the wave.  Same arithmetic, per transform, as
// fft_line (bitwise identical results).

// stage-S butterflies of the P values in v -> a, in exchange-write order a[b*R + r]
template <typename T, int H, int P, int DIR, int S>
__device__ __forceinline__ void fft_bfly(const C2<T> (&v)[P], C2<T> (&a)[P], int t,
                                         const C2<T>* __restrict__ tab) {
  using St = Stages<H, P>;
  constexpr int R = St::radix(S), NS = St::ns(S), TT = H / P, NB = P / R;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
#pragma unroll
    for (int r = 0; r < R; ++r) a[b * R + r] = v[b + r * NB];
    if constexpr (NS > 1) {
      const int j = t + b * TT;
      stage_twiddle<T, H, R, DIR, NS>(&a[b * R], j & (NS - 1), tab);
    }
    dft<T, R, DIR>(&a[b * R]);
  }
}

// exchange after stage S: write a (stage-S outputs), read this thread's stage-(S+1) inputs
template <typename T, int H, int P, int STRIDE, bool WAVE, int S>
__device__ __forceinline__ void fft_xchg(C2<T> (&a)[P], C2<T> (&v)[P], C2<T>* lds, int base, int t) {
  using St = Stages<H, P>;
  constexpr int R = St::radix(S), NS = St::ns(S), TT = H / P, NB = P / R;
  const int idxD = (t / NS) * NS * R + (t & (NS - 1));
  const int wb = base + idxD * STRIDE;
  const int pwb = lds_phys(wb);
  constexpr bool WB16 = (STRIDE == 1) && (NS == 1) && (R == 16);
  xsync<WAVE>();   // earlier readers of the image are done
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lds_at(pwb, wb, (b * TT * R + r * NS) * STRIDE, WB16)] = a[b * R + r];
  xsync<WAVE>();
  const int rb = base + t * STRIDE;
  const int prb = lds_phys(rb);
#pragma unroll
  for (int k = 0; k < P; ++k) v[k] = lds[lds_at(prb, rb, TT * k * STRIDE, false)];
}

// last stage's outputs back to natural register order
template <typename T, int H, int P, int S>
__device__ __forceinline__ void fft_final(const C2<T> (&a)[P], C2<T> (&v)[P]) {
  using St = Stages<H, P>;
  constexpr int R = St::radix(S), NB = P / R;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < R; ++r) v[b + r * NB] = a[b * R + r];
}

template <typename T, int H, int P, int DIR, int STRIDE, bool WAVE, int S>
__device__ __forceinline__ void fft_stage2(C2<T> (&va)[P], C2<T> (&vb)[P], C2<T> (&a)[P], C2<T>* lds, int base, int t,
                                           const C2<T>* __restrict__ tab) {
  // entry: a = stage-S butterflies of va (already computed); vb holds stage-S inputs
  constexpr int NST = Stages<H, P>::count();
  if constexpr (S + 1 < NST) {
    fft_xchg<T, H, P, STRIDE, WAVE, S>(a, va, lds, base, t);       // va: stage S+1 inputs in flight
    fft_bfly<T, H, P, DIR, S>(vb, a, t, tab);                       // ... while vb's butterflies run
    fft_xchg<T, H, P, STRIDE, WAVE, S>(a, vb, lds, base, t);
    fft_bfly<T, H, P, DIR, S + 1>(va, a, t, tab);                   // ... while vb's reads land
    fft_stage2<T, H, P, DIR, STRIDE, WAVE, S + 1>(va, vb, a, lds, base, t, tab);
  } else {
    fft_final<T, H, P, S>(a, va);
    fft_bfly<T, H, P, DIR, S>(vb, a, t, tab);
    fft_final<T, H, P, S>(a, vb);
  }
}

// Two H-point FFTs (same direction) of the lines whose values this thread holds in va and vb,
// through one exchange image at `base` (fft_line semantics for each).
// HGP_SEQ_MULTIWAVE: lines of several waves (block barriers at every exchange) run the two
// transforms one after the other instead (32 fewer live VGPRs: no `a` array in flight).
#ifndef HGP_SEQ_MULTIWAVE
#define HGP_SEQ_MULTIWAVE 0
#endif
template <typename T, int H, int P, int DIR, int STRIDE, bool WAVE = false, bool SEQ = (HGP_SEQ_MULTIWAVE && !WAVE)>
__device__ __forceinline__ void fft_line2(C2<T> (&va)[P], C2<T> (&vb)[P], C2<T>* lds, int base, int t,
                                          const C2<T>* __restrict__ tab) {
  if constexpr (SEQ) {
    fft_line<T, H, P, DIR, STRIDE, WAVE>(va, lds, base, t, tab);
    fft_line<T, H, P, DIR, STRIDE, WAVE>(vb, lds, base, t, tab);
    return;
  }
  int tt = t;
  asm volatile("" : "+v"(tt));
  C2<T> a[P];
  fft_bfly<T, H, P, DIR, 0>(va, a, tt, tab);
  fft_stage2<T, H, P, DIR, STRIDE, WAVE, 0>(va, vb, a, lds, base, tt, tab);
}

}  // namespace hgp
