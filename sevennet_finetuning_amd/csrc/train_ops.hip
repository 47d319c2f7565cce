// Element-wise kernels of the fine-tune step's autograd graph
// (sevennet_finetuning_amd/nn.py): the scaled SiLU of the radial MLP and the
// gates (e3nn normalize2mom(silu) = 1.6792 * silu) and
// its first and second derivatives, one launch each instead of the 2 / 2-3 /
// ~6 PyTorch kernels the composite op expands to under double backward.
#include "train_ops.h"

namespace e3gnn {
namespace {

__device__ __forceinline__ float sig(float x) { return 1.0f / (1.0f + __expf(-x)); }

// y = c silu(x)
__global__ void k_act_fwd(int64_t n, const float* __restrict__ x, float* __restrict__ y, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  y[i] = c * v * sig(v);
}

// dx = g c silu'(x),  silu'(x) = s (1 + x (1 - s))
__global__ void k_act_bwd(int64_t n, const float* __restrict__ x, const float* __restrict__ g,
                          float* __restrict__ dx, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sig(v);
  dx[i] = g[i] * c * s * (1.0f + v * (1.0f - s));
}

// cotangent gg of dx:  d/dx = gg g c silu''(x),  d/dg = gg c silu'(x),
// silu''(x) = s (1 - s) (2 + x (1 - 2 s))
__global__ void k_act_bwd2(int64_t n, const float* __restrict__ x, const float* __restrict__ g,
                           const float* __restrict__ gg, float* __restrict__ dx,
                           float* __restrict__ dg, float c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i], s = sig(v), a = gg[i] * c;
  if (dx) dx[i] = a * g[i] * s * (1.0f - s) * (2.0f + v * (1.0f - 2.0f * s));
  if (dg) dg[i] = a * s * (1.0f + v * (1.0f - s));
}

}  // namespace

hipError_t launch_act(int op, int64_t n, const float* x, const float* g, const float* gg,
                      float* out0, float* out1, float c, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  switch (op) {
    case 0: hipLaunchKernelGGL(k_act_fwd, grid, block, 0, s, n, x, out0, c); break;
    case 1: hipLaunchKernelGGL(k_act_bwd, grid, block, 0, s, n, x, g, out0, c); break;
    default: hipLaunchKernelGGL(k_act_bwd2, grid, block, 0, s, n, x, g, gg, out0, out1, c); break;
  }
  return hipGetLastError();
}

}  // namespace e3gnn
