// Checks the lane mapping of v_permlane16_swap / v_permlane32_swap on gfx950 (tuning aid):
// prints, per lane, the source value (= 100*reg + lane) that ends up in each operand.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  const int l = threadIdx.x;
  unsigned a = l, b = 100 + l;
  auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  o[l] = r[0]; o[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  o[128 + l] = s[0]; o[192 + l] = s[1];
}
int main() {
  int* d; int h[256];
  hipMalloc(&d, 1024);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int w = 0; w < 4; ++w) {
    printf("%s: ", w == 0 ? "p16 vdst" : w == 1 ? "p16 src " : w == 2 ? "p32 vdst" : "p32 src ");
    for (int l = 0; l < 64; l += 8) printf("%d:%d ", l, h[w * 64 + l]);
    printf("| 20:%d 40:%d 56:%d\n", h[w * 64 + 20], h[w * 64 + 40], h[w * 64 + 56]);
  }
  return 0;
}
