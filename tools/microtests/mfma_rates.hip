// Cycles per MFMA, one wave per SIMD, back-to-back on one accumulator chain and
// on 4 independent chains: v_mfma_f32_16x16x4_f32, _16x16x16_bf16, _16x16x32_bf16.
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int N = 256;

template <int KIND, int CH>
__global__ void k(const float* in, float* out, long long* cyc) {
  const int l = threadIdx.x;
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0, 0, 0, 0};
  float a = in[l], b = in[64 + l];
  bf16x4 a4, b4;
  bf16x8 a8, b8;
  for (int t = 0; t < 4; ++t) a4[t] = (__bf16)in[l + t], b4[t] = (__bf16)in[64 + l + t];
  for (int t = 0; t < 8; ++t) a8[t] = (__bf16)in[l + t], b8[t] = (__bf16)in[64 + l + t];
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0);
  long long t0 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N / CH; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (KIND == 0) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
      if constexpr (KIND == 1) acc[c] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[c], 0, 0, 0);
      if constexpr (KIND == 2) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[c], 0, 0, 0);
    }
  for (int c = 0; c < CH; ++c) asm volatile("s_nop 0" ::"v"(acc[c]));
  __builtin_amdgcn_sched_barrier(0);
  long long t1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * 64 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int CH>
void run(const char* name, float* in, float* out, long long* cyc) {
  hipLaunchKernelGGL((k<KIND, CH>), dim3(1), dim3(64), 0, 0, in, out, cyc);
  hipLaunchKernelGGL((k<KIND, CH>), dim3(1), dim3(64), 0, 0, in, out, cyc);
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-22s chains=%d  %.1f clock64 ticks per MFMA\n", name, CH, (double)c / N);
}

int main() {
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 4096);
  hipMemset(in, 0, 4096);
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 64);
  run<0, 1>("16x16x4_f32", in, out, cyc);
  run<0, 4>("16x16x4_f32", in, out, cyc);
  run<1, 1>("16x16x16_bf16", in, out, cyc);
  run<1, 4>("16x16x16_bf16", in, out, cyc);
  run<2, 1>("16x16x32_bf16", in, out, cyc);
  run<2, 4>("16x16x32_bf16", in, out, cyc);
  return 0;
}
