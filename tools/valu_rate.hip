// valu_rate.hip — calibration: wave64 fp32 VALU throughput per SIMD on gfx950 vs waves/SIMD,
// scalar v_fma_f32 and packed v_pk_fma_f32, independent chains.  Decides whether the FFT
// passes (mostly scalar fp32 VALU) are issue-bound at their 4 waves/SIMD.
// hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;
constexpr int CH = 8;   // independent chains per lane

__global__ void k_fma(float* out, float a, float b) {
  float v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 0.001f + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = __builtin_fmaf(v[c], a, b);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += v[c];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k_pkfma(float* out, float a, float b) {
  f2 v[CH / 2];
#pragma unroll
  for (int c = 0; c < CH / 2; ++c) v[c] = f2{threadIdx.x * 0.001f + c, c + 0.5f};
  const f2 A = f2{a, a}, B = f2{b, b};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH / 2; ++c) v[c] = __builtin_elementwise_fma(v[c], A, B);
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH / 2; ++c) s += v[c].x + v[c].y;
  if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  float* out;
  hipMalloc(&out, 4096 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pk = 0; pk < 2; ++pk) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      const int threads = 64 * 4 * wps;   // one block per CU: wps waves on each of the 4 SIMDs
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (pk) hipLaunchKernelGGL(k_pkfma, dim3(cus), dim3(threads), 0, 0, out, 0.999f, 0.001f);
        else hipLaunchKernelGGL(k_fma, dim3(cus), dim3(threads), 0, 0, out, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * ITERS * CH * threads * (double)cus;
        if (rep) printf("%s waves/SIMD=%d: %.3f ms  %.1f TFLOP/s\n", pk ? "v_pk_fma_f32" : "v_fma_f32   ", wps, ms,
                        flops / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
