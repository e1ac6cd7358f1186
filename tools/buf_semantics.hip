// Diagnostic: which offset operands of a raw buffer access does gfx950's range check cover?
// A raw resource of `bytes` = 64 B over a 4 KiB buffer filled with 1.0; loads / stores of
// 8 B (b64) and 16 B (b128) at (voffset, soffset) pairs whose sum lies beyond the range.
// Printed: the loaded value (0 = clipped by the range check, 1 = memory read) and whether a
// store beyond the range reached memory.  hipcc --offload-arch=gfx950 -O2 buf_semantics.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

using R = __amdgpu_buffer_rsrc_t;
__device__ R mk(void* p, int bytes) { return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, 0x00020000); }

// case c: (voff, soff) in bytes; soff is a compile-time constant in the instruction stream
template <int SOFF>
__device__ void ld_case(double* buf, double* out, int voff, int slot) {
  R r = mk(buf, 64);
  auto v4 = __builtin_amdgcn_raw_buffer_load_b128(r, voff, SOFF, 0);
  auto v2 = __builtin_amdgcn_raw_buffer_load_b64(r, voff, SOFF, 0);
  { double2 w = __builtin_bit_cast(double2, v4); out[2 * slot] = w.x + w.y; }
  out[2 * slot + 1] = __builtin_bit_cast(double, v2);
}

__global__ void k_load(double* buf, double* out, int vsmall, int vlarge) {
  if (threadIdx.x != 0) return;
  ld_case<0>(buf, out, vsmall, 0);        // in range
  ld_case<0>(buf, out, vlarge, 1);        // voffset beyond
  ld_case<1024>(buf, out, vsmall, 2);     // constant soffset beyond (fits the 12-bit imm)
  ld_case<8192>(buf, out, vsmall, 3);     // constant soffset beyond (does not fit the imm)
  R r = mk(buf, 64);
  // runtime (SGPR) soffset beyond
  int s = __builtin_amdgcn_readfirstlane(vlarge);
  auto v4 = __builtin_amdgcn_raw_buffer_load_b128(r, vsmall, s, 0);
  { double2 w = __builtin_bit_cast(double2, v4); out[8] = w.x + w.y; }
}

__global__ void k_store(double* buf, int vsmall, int vlarge) {
  if (threadIdx.x != 0) return;
  R r = mk(buf, 64);
  using V4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
  using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
  double2 d = {7.0, 7.0};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(V4, d), r, vlarge, 0, 0);      // buf[128]
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(V4, d), r, vsmall, 2048, 0);   // buf[256]
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, 7.0), r, vsmall, 3072, 0); // buf[384]
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(V4, d), r, vsmall, 512, 0);    // buf[64]
}

int main() {
  double *buf, *out;
  hipMalloc(&buf, 4096 * sizeof(double));
  hipMalloc(&out, 16 * sizeof(double));
  double h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = 1.0;
  hipMemcpy(buf, h, sizeof h, hipMemcpyHostToDevice);
  hipMemset(out, 0xff, 16 * sizeof(double));
  // vsmall = 0, vlarge = 1024 B (beyond the 64-B range)
  k_load<<<1, 64>>>(buf, out, 0, 1024);
  double o[16];
  hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
  const char* names[] = {"in range", "voffset 1024", "soffset 1024 (const)", "soffset 8192 (const)"};
  for (int c = 0; c < 4; ++c) printf("load %-22s b128 %.1f  b64 %.1f\n", names[c], o[2 * c], o[2 * c + 1]);
  printf("load %-22s b128 %.1f\n", "soffset 1024 (SGPR)", o[8]);
  k_store<<<1, 64>>>(buf, 0, 1024);
  hipMemcpy(h, buf, sizeof h, hipMemcpyDeviceToHost);
  printf("store b128 voffset 1024        -> memory %s\n", h[128] == 7.0 ? "WRITTEN" : "untouched");
  printf("store b128 soffset 2048 (const) -> memory %s\n", h[256] == 7.0 ? "WRITTEN" : "untouched");
  printf("store b64  soffset 3072 (const) -> memory %s\n", h[384] == 7.0 ? "WRITTEN" : "untouched");
  printf("store b128 soffset 512 (const)  -> memory %s\n", h[64] == 7.0 ? "WRITTEN" : "untouched");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
