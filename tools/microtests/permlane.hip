// v_permlane32_swap / v_permlane16_swap semantics check (sum over the 4 rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../sevennet_finetuning_amd/csrc/common.h"
__global__ void k(const float* in, float* out, float* raw) {
  const int l = threadIdx.x;
  const float v = in[l];
  out[l] = e3gnn::sum_rows4(v);
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const unsigned w = __builtin_bit_cast(unsigned, v + 1000.f);
  float x = v, y = v + 1000.f;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  raw[l] = x;
  raw[64 + l] = y;
  x = v, y = v + 1000.f;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  raw[128 + l] = x;
  raw[192 + l] = y;
  (void)u;
  (void)w;
}
int main() {
  float h[64], o[64], r[256];
  for (int i = 0; i < 64; ++i) h[i] = (float)i;
  float *din, *dout, *draw;
  (void)hipMalloc(&din, 256);
  (void)hipMalloc(&dout, 256);
  (void)hipMalloc(&draw, 1024);
  (void)hipMemcpy(din, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, draw);
  (void)hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost);
  (void)hipMemcpy(r, draw, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    const int c = i & 15;
    const float want = 4 * c + 96;  // c + (c+16) + (c+32) + (c+48)
    if (o[i] != want) ++bad;
  }
  printf("sum_rows4 mismatches: %d\n", bad);
  for (int q = 0; q < 4; ++q) {
    printf("raw%d:", q);
    for (int i = 0; i < 64; i += 8) printf(" %g", r[64 * q + i]);
    printf("\n");
  }
  return 0;
}
