// valu_rate.hip — calibration: wave64 fp32 VALU throughput per SIMD on gfx950 vs waves/SIMD
// for scalar and packed forms (independent chains), incl. packed ops with op_sel swizzles.
// Decides how the FFT passes' fp32 arithmetic should be written.
// hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_rate.hip -o tools/valu_rate.bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;
constexpr int CH = 8;   // independent chains per lane
typedef float f2 __attribute__((ext_vector_type(2)));

#define KSCALAR(NAME, EXPR)                                                             \
  __global__ void NAME(float* out, float a, float b) {                                  \
    float v[CH];                                                                        \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 0.001f + c;    \
    for (int i = 0; i < ITERS; ++i) {                                                   \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) v[c] = EXPR;                       \
    }                                                                                   \
    float s = 0;                                                                        \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s += v[c];                           \
    if (s == 12345.f) out[threadIdx.x] = s;                                             \
  }
#define KPACKED(NAME, EXPR)                                                             \
  __global__ void NAME(float* out, float a, float b) {                                  \
    f2 v[CH / 2];                                                                       \
    _Pragma("unroll") for (int c = 0; c < CH / 2; ++c) v[c] = f2{threadIdx.x * 0.001f + c, c + 0.5f}; \
    const f2 A = f2{a, -a}, B = f2{b, b};                                               \
    for (int i = 0; i < ITERS; ++i) {                                                   \
      _Pragma("unroll") for (int c = 0; c < CH / 2; ++c) v[c] = EXPR;                   \
    }                                                                                   \
    float s = 0;                                                                        \
    _Pragma("unroll") for (int c = 0; c < CH / 2; ++c) s += v[c].x + v[c].y;            \
    if (s == 12345.f) out[threadIdx.x] = s;                                             \
  }

KSCALAR(k_fma, __builtin_fmaf(v[c], a, b))
KSCALAR(k_add, v[c] + b)
KSCALAR(k_mul, v[c] * a)
KPACKED(k_pkfma, __builtin_elementwise_fma(v[c], A, B))
KPACKED(k_pkadd, v[c] + B)
KPACKED(k_pkmul, v[c] * A)
// swapped operand (op_sel): v * swap(v) + B
KPACKED(k_pkfma_swap, __builtin_elementwise_fma(__builtin_shufflevector(v[c], v[c], 1, 0), A, B))
// broadcast operand (op_sel_hi): lo(v) * A + B
KPACKED(k_pkfma_bcast, __builtin_elementwise_fma(__builtin_shufflevector(v[c], v[c], 0, 0), A, B))

using KFn = void (*)(float*, float, float);
struct KDesc { const char* name; KFn fn; int flops_per_lane_chain; };

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  float* out;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // "ops" = lane results per instruction: scalar 1, packed 2 (fma counted as 1 op here)
  KDesc ks[] = {{"v_fma_f32", k_fma, 1},        {"v_add_f32", k_add, 1},        {"v_mul_f32", k_mul, 1},
                {"v_pk_fma_f32", k_pkfma, 2},   {"v_pk_add_f32", k_pkadd, 2},   {"v_pk_mul_f32", k_pkmul, 2},
                {"pk_fma op_sel swap", k_pkfma_swap, 2}, {"pk_fma op_sel bcast", k_pkfma_bcast, 2}};
  for (const KDesc& k : ks) {
    for (int wps = 1; wps <= 4; wps *= 2) {
      const int threads = 64 * 4 * wps;   // one block per CU: wps waves on each of the 4 SIMDs
      float ms = 0;
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k.fn, dim3(cus), dim3(threads), 0, 0, out, 0.999f, 0.001f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
      }
      // wave-instructions per SIMD: ITERS * CH / (lanes-results per instr) * wps
      const double instr = (double)ITERS * CH / k.flops_per_lane_chain * wps;
      const double ns = ms * 1e6;
      printf("%-22s waves/SIMD=%d: %.3f ms  %.2f ns per wave-instruction per SIMD  (%.1f G lane-results/s)\n",
             k.name, wps, ms, ns / instr, (double)ITERS * CH * threads * cus / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
