// passbench — time single k_pass configurations of the C2 K-op geometry (m = 1024, L = 2048,
// 32 RHS) with HIP events, without torch.  Tuning tool, not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I hipgp_amd/csrc tools/passbench.hip -o build/passbench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hgp_pass.hpp"

using namespace hgp;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } \
  } while (0)

template <int H, int MODE, int LAY>
float run(const PassDesc& d, int64_t nb, int reps) {
  using Cfg = PassCfg<float, H, LAY>;
  CK(hipFuncSetAttribute((const void*)k_pass<float, H, MODE, LAY>, hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_pass<float, H, MODE, LAY>), dim3(nb), dim3(Cfg::THREADS), Cfg::LDS, 0, d);
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_pass<float, H, MODE, LAY>), dim3(nb), dim3(Cfg::THREADS), Cfg::LDS, 0, d);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int Q = argc > 1 ? atoi(argv[1]) : 32;
  const int m = 1024, L = 2048, H = 1024, Sl = 1032;
  const int64_t M = (int64_t)m * m, B1 = (int64_t)m * Sl;
  float *x, *y, *spec;
  float2 *w, *tw;
  CK(hipMalloc(&x, Q * M * 4));
  CK(hipMalloc(&y, Q * M * 4));
  CK(hipMalloc(&w, Q * B1 * 8));
  CK(hipMalloc(&spec, (int64_t)L * Sl * 4));
  CK(hipMalloc(&tw, L * 8));
  std::vector<float2> htw(L);
  for (int q = 0; q < L; ++q) htw[q] = make_float2(cos(-2 * M_PI * q / L), sin(-2 * M_PI * q / L));
  CK(hipMemcpy(tw, htw.data(), L * 8, hipMemcpyHostToDevice));
  CK(hipMemset(x, 0, Q * M * 4));
  CK(hipMemset(w, 0, Q * B1 * 8));
  CK(hipMemset(spec, 0, (int64_t)L * Sl * 4));
  const int reps = 20;
  const double pair_bytes = (double)m * Sl * 8;     // complex intermediate per RHS

  // A: FWD rows (RP)
  {
    PassDesc A{};
    A.in = View{x, M, m, 1, m};
    A.out = View{w, B1, Sl, 1, 0};
    A.tw = tw; A.Q = Q; A.Rn = m / 2; A.nrows = m;
    using Cfg = PassCfg<float, H, LAY_RP>;
    const int64_t nb = ((int64_t)Q * A.Rn + Cfg::C - 1) / Cfg::C;
    float ms = run<H, PASS_FWD, LAY_RP>(A, nb, reps);
    printf("rowFWD  C=%d thr=%d lds=%d : %.4f ms  %.0f GB/s\n", Cfg::C, Cfg::THREADS, Cfg::LDS, ms, Q * (M * 4 + pair_bytes) / ms / 1e6);
  }
  // B: CONV cols (strided), in place
  {
    PassDesc Bd{};
    Bd.in = View{w, B1, 0, Sl, m};
    Bd.out = View{w, B1, 0, Sl, m};
    Bd.spec = spec; Bd.spec_kind = SPEC_REAL; Bd.spec_i = 1; Bd.spec_p = Sl; Bd.spec_r = 0;
    Bd.tw = tw; Bd.Q = Q; Bd.Rn = 1; Bd.In = H + 1;
    using Cfg = PassCfg<float, H, LAY_STRIDED>;
    const int64_t nb = (int64_t)Q * ((Bd.In + Cfg::C - 1) / Cfg::C);
    float ms = run<H, PASS_CONV, LAY_STRIDED>(Bd, nb, reps);
    printf("colCONV C=%d thr=%d lds=%d : %.4f ms  %.0f GB/s\n", Cfg::C, Cfg::THREADS, Cfg::LDS, ms, Q * 2 * pair_bytes / ms / 1e6);
    // same geometry, forward only (no spectrum), out of place into y-sized scratch: FWD writes L rows
    float2* w2;
    CK(hipMalloc(&w2, (int64_t)Q * L * Sl * 8));
    PassDesc F = Bd;
    F.out = View{w2, (int64_t)L * Sl, 0, Sl, 0};
    ms = run<H, PASS_FWD, LAY_STRIDED>(F, nb, reps);
    printf("colFWD  C=%d : %.4f ms  %.0f GB/s (reads m rows, writes L rows)\n", Cfg::C, ms, Q * (pair_bytes + 2 * pair_bytes) / ms / 1e6);
    PassDesc I = Bd;
    I.in = View{w2, (int64_t)L * Sl, 0, Sl, L};
    ms = run<H, PASS_INV, LAY_STRIDED>(I, nb, reps);
    printf("colINV  C=%d : %.4f ms  %.0f GB/s (reads L rows, writes m rows)\n", Cfg::C, ms, Q * (pair_bytes + 2 * pair_bytes) / ms / 1e6);
    CK(hipFree(w2));
  }
  // B': CONV along contiguous (transposed) column lines: w as [q][c][i0], spectrum [c][kperm]
  {
    PassDesc Bt{};
    Bt.in = View{w, B1, m, 1, m};
    Bt.out = View{w, B1, m, 1, m};
    Bt.spec = spec; Bt.spec_kind = SPEC_REAL; Bt.spec_i = 0; Bt.spec_p = 1; Bt.spec_r = L;
    Bt.tw = tw; Bt.Q = Q; Bt.Rn = H + 1; Bt.In = 1;
    using Cfg = PassCfg<float, H, LAY_CONTIG>;
    const int64_t nb = ((int64_t)Q * Bt.Rn + Cfg::C - 1) / Cfg::C;
    float ms = run<H, PASS_CONV, LAY_CONTIG>(Bt, nb, reps);
    printf("colCONVt C=%d thr=%d lds=%d wave=%d : %.4f ms  %.0f GB/s\n", Cfg::C, Cfg::THREADS, Cfg::LDS, (int)Cfg::WAVE, ms, Q * 2 * pair_bytes / ms / 1e6);
  }
  // B'': wave-split CONV on the same transposed lines
  {
    PassDesc Bt{};
    Bt.in = View{w, B1, m, 1, m};
    Bt.out = View{w, B1, m, 1, m};
    Bt.spec = spec; Bt.spec_kind = SPEC_REAL; Bt.spec_i = 0; Bt.spec_p = 1; Bt.spec_r = L;
    Bt.tw = tw; Bt.Q = Q; Bt.Rn = H + 1; Bt.In = 1;
    using Cfg = ConvCfg<float, H>;
    CK(hipFuncSetAttribute((const void*)k_conv_ws<float, H, false>, hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS));
    const int64_t nb = ((int64_t)Q * Bt.Rn + Cfg::C - 1) / Cfg::C;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_conv_ws<float, H, false>), dim3(nb), dim3(Cfg::THREADS), Cfg::LDS, 0, Bt);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_conv_ws<float, H, false>), dim3(nb), dim3(Cfg::THREADS), Cfg::LDS, 0, Bt);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("colCONVws C=%d thr=%d lds=%d : %.4f ms  %.0f GB/s\n", Cfg::C, Cfg::THREADS, Cfg::LDS, ms, Q * 2 * pair_bytes / ms / 1e6);
  }
  // C: INV rows (RP)
  {
    PassDesc Cd{};
    Cd.in = View{w, B1, Sl, 1, L};
    Cd.out = View{y, M, m, 1, m};
    Cd.tw = tw; Cd.Q = Q; Cd.Rn = m / 2; Cd.nrows = m;
    using Cfg = PassCfg<float, H, LAY_RP>;
    const int64_t nb = ((int64_t)Q * Cd.Rn + Cfg::C - 1) / Cfg::C;
    float ms = run<H, PASS_INV, LAY_RP>(Cd, nb, reps);
    printf("rowINV  C=%d thr=%d lds=%d : %.4f ms  %.0f GB/s\n", Cfg::C, Cfg::THREADS, Cfg::LDS, ms, Q * (M * 4 + pair_bytes) / ms / 1e6);
  }
  // reference: plain copy of the intermediate (achievable HBM rate for this footprint)
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float2* w3;
    CK(hipMalloc(&w3, Q * B1 * 8));
    CK(hipMemcpy(w3, w, Q * B1 * 8, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) CK(hipMemcpyAsync(w3, w, Q * B1 * 8, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("memcpy  %.0f MB : %.4f ms  %.0f GB/s\n", Q * B1 * 8 / 1e6, ms, 2.0 * Q * B1 * 8 / ms / 1e6);
  }
  return 0;
}
