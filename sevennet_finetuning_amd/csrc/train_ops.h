// Element-wise kernels of the fine-tune step (train_ops.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {
// op 0: out0 = c silu(x); 1: out0 = g c silu'(x); 2: out0 = gg g c silu''(x),
// out1 = gg c silu'(x) (either nullable)
hipError_t launch_act(int op, int64_t n, const float* x, const float* g, const float* gg,
                      float* out0, float* out1, float c, hipStream_t s);
// e3nn Gate rows (nn.py gate): op 0 out0 = o(y); 1 out0 = dy(y, go);
// 2 (cotangent q of dy) out0 = d/dgo, out1 = d/dy (either nullable).
// dims: ns, ng, din, dout, ngroups, then per group (<= 2): off_in, off_out, mul, 2l+1
hipError_t launch_gate(int op, int64_t n, const int* dims, const float* y, const float* go,
                       const float* q, float* out0, float* out1, float c, hipStream_t s);
// reverse of (phi(x), phi'(x) x'): og = g phi' + gd phi'' x', ogd = gd phi'
hipError_t launch_act_dual(int64_t n, const float* x, const float* xd, const float* g,
                           const float* gd, float* og, float* ogd, float c, hipStream_t s);
// gate tangent (op 0: out0 = J y') and the reverse of (G(y), J y') (op 1:
// out0 = J^T xb + d/dy <xdb, J y'>, out1 = J^T xdb)
hipError_t launch_gate_dual(int op, int64_t n, const int* dims, const float* y, const float* yd,
                            const float* xb, const float* xdb, float* out0, float* out1, float c,
                            hipStream_t s);
// the fine-tune step's radial-MLP chains (mlp_train.hip): forward / tangent
// (A1p, A2p: primal pre-activations) and reverse / dual (A1d, A2d: tangent
// pre-activations; 2E rows) of e -> W0 -> phi -> W1 -> phi -> W2
hipError_t launch_mlp_fwd(int E, int W, const float* emb, const float* W0, const float* W1,
                          const float* W2, const float* A1p, const float* A2p, float* A1, float* H1,
                          float* A2, float* H2, float* WT, float c, hipStream_t s,
                          const void* W2p = nullptr);   // W2p: W2's piece image (layer 2 on bf16x6)
int64_t mlp_w2_piece_bytes(int W);
hipError_t launch_mlp_w2_pieces(int n, const float* const* W2, const int* W, void* const* img, hipStream_t s);
hipError_t launch_mlp_bwd(int E, int W, const float* WB, const float* W0, const float* W1,
                          const float* W2, const float* A1, const float* A2, const float* A1d,
                          const float* A2d, float* A2B, float* A1B, float* EB, float c,
                          hipStream_t s, const void* W2p = nullptr);
// the explicit step's loss (MSE / Huber, mean over labelled entries) and its
// cotangents: terms[0..2] = weighted energy-per-atom / force / stress terms
struct LossArgs {
  int criterion;  // 0 MSELoss, 1 HuberLoss(delta)
  float delta;
  int64_t nb, n;
  const float *e_pred, *e_ref;
  const int64_t* natoms;
  const float *f_pred, *f_ref, *s_pred, *s_ref;  // s_* null: no stress term
  float w_e, w_f, w_s, s_scale;
  float *terms, *ce, *cf, *cs;
};
hipError_t launch_loss_efs(const LossArgs& a, hipStream_t s);
hipError_t launch_ewc_flat(int64_t n, const float* th, const float* f, const float* o, const float* ft,
                           float lam, float* grad, float* part, hipStream_t s);
}  // namespace e3gnn
