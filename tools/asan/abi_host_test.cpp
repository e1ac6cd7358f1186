// abi_host_test.cpp — host-side sanitizer run of libhipgp's C ABI (SURVEY §5 "race detection /
// sanitizers": -fsanitize=address,undefined on the host code only; GPU sanitizers are not
// available on this pool).  No GPU is needed: every call below is refused by the library's
// own argument / state checks or is pure host logic (block geometry, empty inputs, thread-local
// error messages), so ASan/UBSan see the whole host path of those calls.  Built and run by
// tools/asan/Makefile (`make -C tools/asan run`); tests/test_abi_asan.py runs it on the CPU.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hipgp.h"

static int g_fail = 0;
#define EXPECT(cond)                                                                  \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      std::fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, #cond, \
                   hgp_last_error());                                                 \
      ++g_fail;                                                                       \
    }                                                                                 \
  } while (0)

int main() {
  EXPECT(hgp_version() != nullptr && std::strlen(hgp_version()) > 0);
  EXPECT(hgp_last_error() != nullptr);

  // ---- plan lifecycle: refused before any device work -----------------------------------
  int64_t m2[2] = {8, 6};
  hgp_plan* P = reinterpret_cast<hgp_plan*>(0x1);
  EXPECT(hgp_plan_create(0, 2, m2, HGP_F32, 0, nullptr, nullptr) == HGP_E_ARG);
  EXPECT(hgp_plan_create(0, 2, nullptr, HGP_F32, 0, nullptr, &P) == HGP_E_ARG);
  EXPECT(hgp_plan_create(0, 0, m2, HGP_F32, 0, nullptr, &P) == HGP_E_ARG && P == nullptr);
  EXPECT(hgp_plan_create(0, 4, m2, HGP_F32, 0, nullptr, &P) == HGP_E_ARG);
  EXPECT(hgp_plan_create(0, 2, m2, 7, 0, nullptr, &P) == HGP_E_ARG);
  EXPECT(std::string(hgp_last_error()).find("dtype") != std::string::npos);

  // ---- every plan entry point refuses a null plan --------------------------------------
  float buf[16] = {0};
  int iv = 0;
  int64_t i64[3] = {0, 0, 0};
  EXPECT(hgp_plan_set_stream(nullptr, nullptr) == HGP_E_ARG);
  EXPECT(hgp_plan_set_column(nullptr, buf, 0., 1e-6, nullptr) == HGP_E_ARG);
  EXPECT(hgp_toeplitz_apply(nullptr, HGP_OP_K, buf, buf + 8, 1) == HGP_E_ARG);
  EXPECT(hgp_toeplitz_apply_pass(nullptr, HGP_OP_K, buf, buf + 8, 1, 0) == HGP_E_ARG);
  EXPECT(hgp_op_pass_count(nullptr) == HGP_E_ARG);
  EXPECT(hgp_pcg_begin(nullptr, buf, buf + 8, 1, 1, HGP_LAYOUT_ROWS) == HGP_E_ARG);
  EXPECT(hgp_pcg_step(nullptr, 1e-8, &iv) == HGP_E_ARG);
  EXPECT(hgp_pcg_solve(nullptr, buf, buf + 8, 1, 10, 1e-8, 1, HGP_LAYOUT_ROWS, &iv) == HGP_E_ARG);
  EXPECT(hgp_pcg_rnorm2(nullptr, buf) == HGP_E_ARG);
  EXPECT(hgp_pcg_local_flag(nullptr, 1e-8, &iv) == HGP_E_ARG);
  EXPECT(hgp_pcg_set_done(nullptr, &iv) == HGP_E_ARG);
  EXPECT(hgp_pcg_iters(nullptr, &iv) == HGP_E_ARG);
  EXPECT(hgp_get_spectrum(nullptr, HGP_SPEC_D, buf) == HGP_E_ARG);
  EXPECT(hgp_plan_column_grad(nullptr, HGP_OP_K, buf, buf, 1, buf) == HGP_E_ARG);
  EXPECT(hgp_plan_dqf(nullptr, buf, buf, 1, buf) == HGP_E_ARG);
  EXPECT(hgp_plan_info(nullptr, i64, i64, i64, i64) == HGP_E_ARG);
  EXPECT(hgp_plan_destroy(nullptr) == 0);
  EXPECT(hgp_plan_trim(nullptr) == HGP_E_ARG);
  EXPECT(hgp_plan_mem(nullptr, i64, i64) == HGP_E_ARG);
  EXPECT(hgp_slab_info(nullptr, HGP_OP_K, i64, i64) == HGP_E_ARG);
  EXPECT(hgp_slab_pass(nullptr, HGP_OP_K, HGP_SLAB_FWD, buf, buf + 8, 1, 1, 0, 0) == HGP_E_ARG);
  EXPECT(hgp_slab_pass_ex(nullptr, HGP_OP_K, HGP_SLAB_INV, buf, buf + 8, 1, 1, 0, 0, buf, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_slab_cg_xr(nullptr, buf, buf, buf, buf, buf, buf, buf, 1, 4, nullptr) == HGP_E_ARG);
  EXPECT(hgp_slab_cg_check(nullptr, buf, 1, 1e-8, nullptr, nullptr) == HGP_E_ARG);
  EXPECT(hgp_slab_cg_p(nullptr, buf, buf, buf, buf, 1, 4, nullptr) == HGP_E_ARG);

  // ---- stand-alone kernels: argument checks and empty inputs ---------------------------
  EXPECT(hgp_rowdot(HGP_F32, buf, buf, buf, 0, 16, nullptr) == 0);            // nothing to do
  EXPECT(hgp_rowdot(HGP_F32, nullptr, buf, buf, 2, 16, nullptr) == HGP_E_ARG);
  EXPECT(hgp_rowdot(5, buf, buf, buf, 2, 16, nullptr) == HGP_E_ARG);
  const void* grids[3] = {buf, buf, buf};
  int64_t m3[3] = {4, 5, 6};
  EXPECT(hgp_kuf_grid(HGP_F32, HGP_KERN_SQEXP, 0, m3, grids, buf, 1, 1., 1., buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_kuf_grid(HGP_F32, 99, 2, m3, grids, buf, 1, 1., 1., buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_kuf_grid(HGP_F32, HGP_KERN_SQEXP, 2, m3, grids, buf, 0, 1., 1., buf, nullptr) == 0);
  int64_t mbad[2] = {4, 0};
  EXPECT(hgp_kuf_grid(HGP_F32, HGP_KERN_SQEXP, 2, mbad, grids, buf, 3, 1., 1., buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_kuf_semi_mc(HGP_F32, HGP_KERN_SQEXP, 1., 2, m3, grids, buf, 3, 1., 1., 0, buf, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_kuf_semi_mc(HGP_F32, HGP_KERN_SQEXP, 1., 2, m3, grids, buf, 3, 1., 1., 10, nullptr, buf, nullptr) ==
         HGP_E_ARG);
  EXPECT(hgp_kuf_semi_mc(HGP_F32, HGP_KERN_SQEXP, 1., 2, m3, grids, buf, 0, 1., 1., 10, buf, buf, nullptr) == 0);
  EXPECT(hgp_kuf_semi_sqexp(HGP_F64, 2, m3, grids, buf, 0, 1., 1., buf, nullptr) == 0);
  EXPECT(hgp_knn_doubly_diag(HGP_F32, 2, buf, 3, 1., 1., buf, 1, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_knn_doubly_diag(HGP_F32, 2, buf, 0, 1., 1., buf, 50, buf, nullptr) == 0);
  EXPECT(hgp_meanfield_stats(HGP_F32, buf, -1, 16, buf, buf, buf, buf, buf, buf, buf, buf, buf, nullptr) ==
         HGP_E_ARG);
  EXPECT(hgp_meanfield_stats(HGP_F32, buf, 2, 16, buf, nullptr, buf, buf, buf, buf, buf, buf, buf, nullptr) ==
         HGP_E_ARG);
  EXPECT(hgp_meanfield_rowdots(HGP_F32, buf, -1, 16, buf, buf, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_meanfield_rowdots(HGP_F32, buf, 2, 16, buf, nullptr, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_meanfield_rowdots(HGP_F64, nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr) == 0);
  EXPECT(hgp_meanfield_cols(7, buf, 2, 16, buf, buf, buf, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_meanfield_cols(HGP_F32, buf, 2, 16, buf, nullptr, buf, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_meanfield_cols(HGP_F32, nullptr, 2, 0, nullptr, nullptr, nullptr, nullptr, nullptr) == 0);
  EXPECT(hgp_sym_toeplitz_dqf(HGP_F32, buf, buf, 1, 0, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_sym_toeplitz_dqf(HGP_F32, nullptr, buf, 1, 4, buf, nullptr) == HGP_E_ARG);

  // ---- block-family geometry (pure host logic) ----------------------------------------
  int64_t d2[2] = {22, 18}, b2[2] = {2, 3};
  EXPECT(hgp_block_stats(HGP_F32, 2, d2, b2, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == 0);
  int64_t b2bad[2] = {4, 3};
  EXPECT(hgp_block_stats(HGP_F32, 2, d2, b2bad, buf, 1, buf, buf, buf, nullptr, nullptr, nullptr) ==
         HGP_E_UNSUPPORTED);
  int64_t d1[1] = {10}, b1[1] = {2};
  EXPECT(hgp_block_stats(HGP_F32, 1, d1, b1, buf, 1, buf, buf, buf, nullptr, nullptr, nullptr) == HGP_E_UNSUPPORTED);
  int64_t dbig[2] = {256, 256}, bbig[2] = {16, 16};    // 256 points per block > 128
  EXPECT(hgp_block_stats(HGP_F32, 2, dbig, bbig, buf, 1, buf, buf, buf, nullptr, nullptr, nullptr) ==
         HGP_E_UNSUPPORTED);
  int64_t dhuge[3] = {1 << 12, 1 << 12, 1 << 8}, bh[3] = {2, 2, 2};   // M' = 2^32
  EXPECT(hgp_block_stats(HGP_F32, 3, dhuge, bh, buf, 1, buf, buf, buf, nullptr, nullptr, nullptr) ==
         HGP_E_UNSUPPORTED);
  EXPECT(hgp_block_stats(HGP_F32, 2, d2, b2, buf, 1, buf, buf, nullptr, nullptr, buf, nullptr) == HGP_E_ARG);
  EXPECT(hgp_block_stats(HGP_F32, 2, d2, b2, buf, -1, buf, buf, buf, nullptr, nullptr, nullptr) == HGP_E_ARG);

  // ---- thread-local error messages (concurrent callers never see each other's) ---------
  std::atomic<int> bad{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) {
    th.emplace_back([t, &bad] {
      for (int i = 0; i < 2000; ++i) {
        int64_t mm[2] = {8, 8};
        hgp_plan* q = nullptr;
        if (t % 2 == 0) {
          (void)hgp_plan_create(0, 9, mm, HGP_F32, 0, nullptr, &q);        // "ndim must be 1..3"
          if (std::string(hgp_last_error()).find("ndim") == std::string::npos) ++bad;
        } else {
          (void)hgp_plan_create(0, 2, mm, 9, 0, nullptr, &q);              // "dtype must be ..."
          if (std::string(hgp_last_error()).find("dtype") == std::string::npos) ++bad;
        }
      }
    });
  }
  for (auto& x : th) x.join();
  EXPECT(bad.load() == 0);

  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("abi_host_test: all host-side checks passed under the sanitizers\n");
  return 0;
}
