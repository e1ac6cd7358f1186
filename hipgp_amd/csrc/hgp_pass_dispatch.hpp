// hgp_pass_dispatch.hpp — instantiation + launch of k_pass for one dtype (included by
// hgp_pass_f32.hip / hgp_pass_f64.hip so the two compile in parallel).
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "hgp_internal.hpp"
#include "hgp_rows.hpp"
#include "hgp_lines.hpp"

namespace hgp {

// Co-residency experiments (round 6): a minimum dynamic-LDS request per block for the
// 2-D column conv (HGP_CONV_LDS_MIN), row-forward (HGP_ROWF_LDS_MIN) and row-inverse
// (HGP_ROWI_LDS_MIN) kernels, in bytes, caps how many blocks of one kind a CU takes, so the other
// stream's pass can share the CU.  Unset (0): the kernel's own LDS size.  Read once per process.
inline int lds_min_env(const char* name) {
  const char* e = std::getenv(name);
  const int v = e ? std::atoi(e) : 0;
  return v < 0 ? 0 : (v > LDS_CAP ? LDS_CAP : v);
}
inline int lds_conv_min() { static const int v = lds_min_env("HGP_CONV_LDS_MIN"); return v; }
inline int lds_rowf_min() { static const int v = lds_min_env("HGP_ROWF_LDS_MIN"); return v; }
inline int lds_rowi_min() { static const int v = lds_min_env("HGP_ROWI_LDS_MIN"); return v; }

template <typename T, int H, int MODE, int LAY>
static hipError_t launch_one(const PassDesc& d, int64_t nblocks, hipStream_t s) {
  using Cfg = PassCfg<T, H, LAY>;
  constexpr bool col2d = (MODE == PASS_CONV || MODE == PASS_CONVC) &&
                         (LAY == LAY_CONTIG || LAY == LAY_CONTIG_G || LAY == LAY_CONTIG_Q);
  const int lds = col2d ? std::max<int>(Cfg::LDS, lds_conv_min()) : Cfg::LDS;
  static bool attr_set = false;   // opt in to > 64 KB dynamic LDS once per instance
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_pass<T, H, MODE, LAY>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_pass<T, H, MODE, LAY>), dim3((unsigned)nblocks), dim3(Cfg::THREADS), lds, s, d);
  return hipGetLastError();
}

// the interleaved grouped layouts exist where one group's G lines fit a block
template <typename T, int H, int LAY>
constexpr bool grp_ok() {
  return std::is_same<T, float>::value && PassCfg<T, H, LAY>::THREADS <= 1024 && PassCfg<T, H, LAY>::LDS <= LDS_CAP;
}

template <typename T, int H, int MODE>
static hipError_t launch_grp(int lay, const PassDesc& d, int64_t nblocks, hipStream_t s) {
  if constexpr (grp_ok<T, H, LAY_GRP2>())
    if (lay == LAY_GRP2) return launch_one<T, H, MODE, LAY_GRP2>(d, nblocks, s);
  if constexpr (grp_ok<T, H, LAY_GRP4>())
    if (lay == LAY_GRP4) return launch_one<T, H, MODE, LAY_GRP4>(d, nblocks, s);
  return hipErrorInvalidValue;
}

template <typename T, int H>
static hipError_t launch_h(int mode, int lay, const PassDesc& d, int64_t nblocks, hipStream_t s) {
  if (mode == PASS_FWD) {
    if (lay == LAY_STRIDED) return launch_one<T, H, PASS_FWD, LAY_STRIDED>(d, nblocks, s);
    if (lay == LAY_CONTIG) return launch_one<T, H, PASS_FWD, LAY_CONTIG>(d, nblocks, s);
    if (lay == LAY_RP) return launch_one<T, H, PASS_FWD, LAY_RP>(d, nblocks, s);
  } else if (mode == PASS_INV) {
    if (lay == LAY_STRIDED) return launch_one<T, H, PASS_INV, LAY_STRIDED>(d, nblocks, s);
    if (lay == LAY_RP) return launch_one<T, H, PASS_INV, LAY_RP>(d, nblocks, s);
  } else if (mode == PASS_CONV) {
    if (lay == LAY_STRIDED) return launch_one<T, H, PASS_CONV, LAY_STRIDED>(d, nblocks, s);
    if (lay == LAY_CONTIG) return launch_one<T, H, PASS_CONV, LAY_CONTIG>(d, nblocks, s);
    if (lay == LAY_R1) return launch_one<T, H, PASS_CONV, LAY_R1>(d, nblocks, s);
    if constexpr (std::is_same<T, float>::value && H == 1024)   // two lines per wave (hgp_pass.hpp)
      if (lay == LAY_CONTIG2) return launch_one<T, H, PASS_CONV, LAY_CONTIG2>(d, nblocks, s);
    // the grouped-column intermediate of long fp32 rows (hgp_rows.hpp RowTCfg::G); any axis-0 H
    if constexpr (std::is_same<T, float>::value) {
      if (lay == LAY_CONTIG_G) return launch_one<T, H, PASS_CONV, LAY_CONTIG_G>(d, nblocks, s);
      if (lay == LAY_CONTIG_Q) return launch_one<T, H, PASS_CONV, LAY_CONTIG_Q>(d, nblocks, s);
    }
    if (lay == LAY_SEG_C) return launch_one<T, H, PASS_CONV, LAY_SEG_C>(d, nblocks, s);
    if (lay == LAY_SEG_S) return launch_one<T, H, PASS_CONV, LAY_SEG_S>(d, nblocks, s);
    if (lay_grp(lay)) return launch_grp<T, H, PASS_CONV>(lay, d, nblocks, s);
  } else if (mode == PASS_CONVC) {
    if (lay == LAY_STRIDED) return launch_one<T, H, PASS_CONVC, LAY_STRIDED>(d, nblocks, s);
    if (lay == LAY_CONTIG) return launch_one<T, H, PASS_CONVC, LAY_CONTIG>(d, nblocks, s);
    if (lay == LAY_R1) return launch_one<T, H, PASS_CONVC, LAY_R1>(d, nblocks, s);
    if constexpr (std::is_same<T, float>::value) {
      if (lay == LAY_CONTIG_G) return launch_one<T, H, PASS_CONVC, LAY_CONTIG_G>(d, nblocks, s);
      if (lay == LAY_CONTIG_Q) return launch_one<T, H, PASS_CONVC, LAY_CONTIG_Q>(d, nblocks, s);
    }
    if (lay == LAY_SEG_C) return launch_one<T, H, PASS_CONVC, LAY_SEG_C>(d, nblocks, s);
    if (lay == LAY_SEG_S) return launch_one<T, H, PASS_CONVC, LAY_SEG_S>(d, nblocks, s);
    if (lay_grp(lay)) return launch_grp<T, H, PASS_CONVC>(lay, d, nblocks, s);
  }
  return hipErrorInvalidValue;
}

template <typename T, int H, int LAY>
static PassGeom geom_one() {
  return PassGeom{PassCfg<T, H, LAY>::C, PassCfg<T, H, LAY>::THREADS, PassCfg<T, H, LAY>::LDS};
}

template <typename T, int H>
static PassGeom geom_h(int lay) {
  // the geometry of the very instantiation launch_h runs (block shape and lines per block)
  if (lay == LAY_STRIDED) return geom_one<T, H, LAY_STRIDED>();
  if (lay == LAY_SEG_S) return geom_one<T, H, LAY_SEG_S>();
  if (lay == LAY_CONTIG) return geom_one<T, H, LAY_CONTIG>();
  if (lay == LAY_CONTIG2) {
    if constexpr (std::is_same<T, float>::value && H == 1024) return geom_one<T, H, LAY_CONTIG2>();
    return PassGeom{0, 0, 0};
  }
  if (lay == LAY_CONTIG_G) return geom_one<T, H, LAY_CONTIG_G>();
  if (lay == LAY_CONTIG_Q) return geom_one<T, H, LAY_CONTIG_Q>();
  if (lay == LAY_SEG_C) return geom_one<T, H, LAY_SEG_C>();
  if (lay == LAY_RP) return geom_one<T, H, LAY_RP>();
  if (lay == LAY_GRP2) return grp_ok<T, H, LAY_GRP2>() ? geom_one<T, H, LAY_GRP2>() : PassGeom{0, 0, 0};
  if (lay == LAY_GRP4) return grp_ok<T, H, LAY_GRP4>() ? geom_one<T, H, LAY_GRP4>() : PassGeom{0, 0, 0};
  return geom_one<T, H, LAY_R1>();
}

#define HGP_H_SWITCH(FN, ...)                                                                        \
  switch (H) {                                                                                       \
    case 2: return FN<T, 2>(__VA_ARGS__);       case 4: return FN<T, 4>(__VA_ARGS__);               \
    case 8: return FN<T, 8>(__VA_ARGS__);       case 16: return FN<T, 16>(__VA_ARGS__);             \
    case 32: return FN<T, 32>(__VA_ARGS__);     case 64: return FN<T, 64>(__VA_ARGS__);             \
    case 128: return FN<T, 128>(__VA_ARGS__);   case 256: return FN<T, 256>(__VA_ARGS__);           \
    case 512: return FN<T, 512>(__VA_ARGS__);   case 1024: return FN<T, 1024>(__VA_ARGS__);         \
    case 2048: return FN<T, 2048>(__VA_ARGS__); case 4096: return FN<T, 4096>(__VA_ARGS__);         \
    case 8192: return FN<T, 8192>(__VA_ARGS__);                                                      \
    case 16384:   /* fp32 only: one 16384-point fp64 line exceeds one CU's LDS */                     \
      if constexpr (std::is_same<T, float>::value) return FN<T, 16384>(__VA_ARGS__);                 \
      break;                                                                                         \
    /* 3 * 2^k (hgp_fft.hpp is_tri): the mixed-radix R / R^T lengths */                              \
    case 12: return FN<T, 12>(__VA_ARGS__);     case 24: return FN<T, 24>(__VA_ARGS__);             \
    case 48: return FN<T, 48>(__VA_ARGS__);     case 96: return FN<T, 96>(__VA_ARGS__);             \
    case 192: return FN<T, 192>(__VA_ARGS__);   case 384: return FN<T, 384>(__VA_ARGS__);           \
    case 768: return FN<T, 768>(__VA_ARGS__);   case 1536: return FN<T, 1536>(__VA_ARGS__);         \
    case 3072: return FN<T, 3072>(__VA_ARGS__); case 6144: return FN<T, 6144>(__VA_ARGS__);         \
    case 12288:   /* fp32 only, as 16384 */                                                          \
      if constexpr (std::is_same<T, float>::value) return FN<T, 12288>(__VA_ARGS__);                 \
      break;                                                                                         \
    default: break;                                                                                  \
  }

template <typename T, int H, int EPI, int G>
static hipError_t launch_rowt_inv(const PassDesc& d, hipStream_t s) {
  using Cfg = RowTCfg<T, H, G, true>;
  const int64_t nb = (int64_t)d.Q * ((d.Rn + Cfg::C - 1) / Cfg::C);
  if (nb <= 0) return hipSuccess;
  const int lds = std::max<int>(Cfg::LDS, lds_rowi_min());
  static bool attr_set = false;   // opt in to > 64 KB dynamic LDS once per instance
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_row_inv_t<T, H, EPI, G>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_row_inv_t<T, H, EPI, G>), dim3((unsigned)nb), dim3(Cfg::THREADS), lds, s, d);
  return hipGetLastError();
}

template <typename T, int H, int G>
static hipError_t launch_rowt_g(int inv, int epi, const PassDesc& d, hipStream_t s) {
  using Cfg = RowTCfg<T, H, G>;
  if constexpr (Cfg::LDS > LDS_CAP || RowTCfg<T, H, G, true>::LDS > LDS_CAP)
    return hipErrorNotSupported;   // e.g. fp64 rows of H = 8192
  if (inv) {
    if (epi == EPI_XR) return launch_rowt_inv<T, H, EPI_XR, G>(d, s);
    if (epi == EPI_R) return launch_rowt_inv<T, H, EPI_R, G>(d, s);
    if (epi == EPI_XP) return launch_rowt_inv<T, H, EPI_XP, G>(d, s);
    if (epi == EPI_RF) return launch_rowt_inv<T, H, EPI_RF, G>(d, s);
    return launch_rowt_inv<T, H, EPI_OUT, G>(d, s);
  }
  const int64_t nb = (int64_t)d.Q * ((d.Rn + Cfg::C - 1) / Cfg::C);
  if (nb <= 0) return hipSuccess;
  const int lds = std::max<int>(Cfg::LDS, lds_rowf_min());
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)k_row_fwd_t<T, H, G>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_row_fwd_t<T, H, G>), dim3((unsigned)nb), dim3(Cfg::THREADS), lds, s, d);
  return hipGetLastError();
}

// grouped: the 2-D operators' intermediate in the grouped-column layout (RowGroup<T, H>::G)
template <typename T, int H>
static hipError_t launch_rowt_h(int inv, int epi, const PassDesc& d, hipStream_t s, int grouped) {
  constexpr int G = RowGroup<T, H>::G;
  if constexpr (G > 1)
    if (grouped) return launch_rowt_g<T, H, G>(inv, epi, d, s);
  return launch_rowt_g<T, H, 1>(inv, epi, d, s);
}

template <typename T, int H>
static hipError_t launch_linet_h(int inv, const PassDesc& d, hipStream_t s) {
  using Cfg = LineTCfg<T, H>;
  if constexpr (Cfg::LDS > LDS_CAP) return hipErrorNotSupported;
  const int64_t nb = (int64_t)d.Q * d.Rn * ((d.In + Cfg::C - 1) / Cfg::C);
  if (nb <= 0) return hipSuccess;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  static bool attr_f = false, attr_i = false;
  bool& attr = inv ? attr_i : attr_f;
  const void* fn = inv ? (const void*)k_line_inv_t<T, H> : (const void*)k_line_fwd_t<T, H>;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (inv) hipLaunchKernelGGL((k_line_inv_t<T, H>), dim3((unsigned)nb), dim3(Cfg::THREADS), Cfg::LDS, s, d);
  else hipLaunchKernelGGL((k_line_fwd_t<T, H>), dim3((unsigned)nb), dim3(Cfg::THREADS), Cfg::LDS, s, d);
  return hipGetLastError();
}

template <typename T, int H>
static int linet_fits_h() { return LineTCfg<T, H>::LDS <= LDS_CAP ? 1 : 0; }

template <typename T>
int linet_fits(int H) {
  HGP_H_SWITCH(linet_fits_h)
  return 0;
}

template <typename T>
hipError_t launch_linet(int H, int inv, const PassDesc& d, hipStream_t s) {
  HGP_H_SWITCH(launch_linet_h, inv, d, s)
  return hipErrorInvalidValue;
}

// pairs / threads per block of the ROW-INVERSE pass (its per-block partials and epilogue loads)
template <typename T, int H>
static int rowt_pairs_h(int grouped) {
  return grouped ? RowTCfg<T, H, RowGroup<T, H>::G, true>::C : RowTCfg<T, H, 1, true>::C;
}

template <typename T, int H>
static int rowt_threads_h(int grouped) {
  return grouped ? RowTCfg<T, H, RowGroup<T, H>::G, true>::THREADS : RowTCfg<T, H, 1, true>::THREADS;
}

template <typename T, int H>
static int rowt_fits_h(int grouped) {
  constexpr int G = RowGroup<T, H>::G;
  const int lf = grouped ? RowTCfg<T, H, G>::LDS : RowTCfg<T, H>::LDS;
  const int li = grouped ? RowTCfg<T, H, G, true>::LDS : RowTCfg<T, H, 1, true>::LDS;
  return (lf <= LDS_CAP && li <= LDS_CAP) ? 1 : 0;
}

template <typename T, int H>
static int rowt_group_h() { return RowGroup<T, H>::G; }

template <typename T>
int rowt_fits(int H, int grouped) {
  HGP_H_SWITCH(rowt_fits_h, grouped)
  return 0;
}

template <typename T>
hipError_t launch_rowt(int H, int inv, int epi, const PassDesc& d, hipStream_t s, int grouped) {
  HGP_H_SWITCH(launch_rowt_h, inv, epi, d, s, grouped)
  return hipErrorInvalidValue;
}

template <typename T>
int rowt_pairs(int H, int grouped) {
  HGP_H_SWITCH(rowt_pairs_h, grouped)
  return 0;
}

template <typename T>
int rowt_threads(int H, int grouped) {
  HGP_H_SWITCH(rowt_threads_h, grouped)
  return 0;
}

template <typename T>
int rowt_group(int H) {
  HGP_H_SWITCH(rowt_group_h)
  return 1;
}

template <typename T>
hipError_t launch_pass(int H, int mode, int lay, const PassDesc& d, int64_t nblocks, hipStream_t s) {
  HGP_H_SWITCH(launch_h, mode, lay, d, nblocks, s)
  return hipErrorInvalidValue;
}

template <typename T>
PassGeom pass_geom(int H, int lay) {
  HGP_H_SWITCH(geom_h, lay)
  return PassGeom{0, 0, 0};
}

}  // namespace hgp
