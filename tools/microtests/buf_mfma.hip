// Microtests: raw buffer loads (voffset/soffset) and f32 MFMA accumulator chaining.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ constexpr int ROW(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__global__ void k_buf(const float* w, int n, float* out) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, n * 4, 0x00020000);
  int lane = threadIdx.x;
  for (int s = 0; s < 4; ++s)
    out[s * 64 + lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, s * 256, 0));
  // out of range voffset
  out[256 + lane] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (n + lane) * 4, 0, 0));
}

// D = A(32x2) B(2x32) chained: compute C = A1 * B1 (K=64) then E = C^T-as-operand test:
// H^T = W^T X^T ; then Z = H W2 with H^T's accumulator used as A operand (permuted k)
__global__ void k_chain(const float* X /*32x64*/, const float* W2 /*64x32*/, float* Z /*32x32*/) {
  int lane = threadIdx.x, half = lane >> 5, col = lane & 31;
  // build H^T = X^T directly: H^T[h][i] = X[i][h]: compute via identity MFMA: H^T = I * X^T
  f32x16 hT[2];
  for (int b = 0; b < 2; ++b) {
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int s = 0; s < 32; ++s) {
      // A = I(64x64) rows 32b..: A[i=h][k] = (h == k); k = 2s + half
      float a = (32 * b + col == 2 * s + half) ? 1.f : 0.f;
      float bb = X[col * 64 + 2 * s + half];  // B[k][j=i] = X^T[k][i] = X[i][k]
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
    }
    hT[b] = acc;
  }
  // Z = H W2: A[i][k=h] = H^T[h][i] from accumulators, permuted k
  f32x16 z;
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  for (int s = 0; s < 32; ++s) {
    int h = 32 * (s >> 4) + ROW(s & 15, half);
    z = __builtin_amdgcn_mfma_f32_32x32x2f32(hT[s >> 4][s & 15], W2[h * 32 + col], z, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) Z[ROW(r, half) * 32 + col] = z[r];
}

int main() {
  const int n = 300;
  std::vector<float> w(n);
  for (int i = 0; i < n; ++i) w[i] = i + 0.5f;
  float *dw, *dout;
  hipMalloc(&dw, n * 4); hipMalloc(&dout, 512 * 4);
  hipMemcpy(dw, w.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_buf, 1, 64, 0, 0, dw, n, dout);
  std::vector<float> o(512);
  hipMemcpy(o.data(), dout, 512 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int s = 0; s < 4; ++s)
    for (int l = 0; l < 64; ++l) {
      int idx = s * 64 + l;
      float exp = idx < n ? w[idx] : 0.f;
      if (o[s * 64 + l] != exp) { if (bad < 5) printf("buf s=%d l=%d got %g exp %g\n", s, l, o[s*64+l], exp); ++bad; }
    }
  for (int l = 0; l < 64; ++l) if (o[256 + l] != 0.f) { if (bad < 10) printf("oob l=%d got %g\n", l, o[256+l]); ++bad; }
  printf("buffer test: %d bad\n", bad);

  std::vector<float> X(32 * 64), W2(64 * 32), Zr(32 * 32, 0.f), Z(32 * 32);
  for (int i = 0; i < 32 * 64; ++i) X[i] = std::sin(0.37f * i);
  for (int i = 0; i < 64 * 32; ++i) W2[i] = std::cos(0.11f * i + 0.3f);
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { double s = 0; for (int k = 0; k < 64; ++k) s += X[i*64+k] * W2[k*32+j]; Zr[i*32+j] = s; }
  float *dX, *dW2, *dZ;
  hipMalloc(&dX, X.size()*4); hipMalloc(&dW2, W2.size()*4); hipMalloc(&dZ, Z.size()*4);
  hipMemcpy(dX, X.data(), X.size()*4, hipMemcpyHostToDevice);
  hipMemcpy(dW2, W2.data(), W2.size()*4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_chain, 1, 64, 0, 0, dX, dW2, dZ);
  hipMemcpy(Z.data(), dZ, Z.size()*4, hipMemcpyDeviceToHost);
  double md = 0; for (int i = 0; i < 32*32; ++i) md = fmax(md, fabs(Z[i] - Zr[i]));
  printf("chain test: max diff %g (Zr[0]=%g Z[0]=%g)\n", md, Zr[0], Z[0]);
  return 0;
}
