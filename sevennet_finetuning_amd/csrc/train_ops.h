// Element-wise kernels of the fine-tune step (train_ops.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {
// op 0: out0 = c silu(x); 1: out0 = g c silu'(x); 2: out0 = gg g c silu''(x),
// out1 = gg c silu'(x) (either nullable)
hipError_t launch_act(int op, int64_t n, const float* x, const float* g, const float* gg,
                      float* out0, float* out1, float c, hipStream_t s);
}  // namespace e3gnn
