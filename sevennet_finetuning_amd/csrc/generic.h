// The generic nequip-family engine behind the C ABI (generic.cpp + generic.hip):
// every deployment of the reference's E3_equivariant_model that is not
// SevenNet-0's architecture (pair_e3gnn.cpp:294-386 loads any deployed model;
// model_build.py:186-445 builds them).  api.cpp routes e3gnn_load, the serial
// evaluation and the segment API here when the manifest is not SevenNet-0's.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace minijson {
struct Value;
}

namespace e3gnn {

// ---------------------------------------------------------------- kernel args
struct GenEdgeArgs {
  int cut;             // 0 XPLOR (r_on), 1 polynomial (p)
  float rc, ron, p;
  int nb;              // radial basis size
  const float* coeffs; // [nb] Bessel frequencies (device)
  int lmax;            // spherical harmonics lmax (<= 2)
  int normalize;       // 1: SH of the unit vector, 0: of the raw vector (sevenn < 0.9)
};
// output column of the gate: act(y[src]) (gate < 0) or act(y[gate]) * y[src]
struct GenGateCol {
  int src, gate, act;  // act 0: silu * silu_norm, 1: tanh * tanh_norm
};
struct GenGateArgs {
  int din, dout;
  float tanh_norm;
  const GenGateCol* cols;  // [dout] (device)
};

hipError_t launch_gen_embed(int n, int d, const int* type, int nsp, const float* W, float* x,
                            int* err, hipStream_t s);
hipError_t launch_gen_edge_embed(const GenEdgeArgs& a, int64_t E, const float* vec, float* Y,
                                 float* emb, hipStream_t s);
int gen_edge_force_blocks(int64_t E);
hipError_t launch_gen_edge_force(const GenEdgeArgs& a, int64_t E, const float* vec, const float* dY,
                                 const float* demb, float* fe, float* vir_part, hipStream_t s);
hipError_t launch_gen_gate_fwd(int n, const GenGateArgs& g, const float* y, float* x, hipStream_t s);
hipError_t launch_gen_gate_bwd(int n, const GenGateArgs& g, const float* y, const float* dx,
                               float* dy, hipStream_t s);
hipError_t launch_gen_species_linear(int n, int din, int dout, const int* type, const float* x,
                                     const float* W, float* y, int beta, hipStream_t s);
hipError_t launch_gen_readout(int n, int d, const float* x, const float* v, const int* type,
                              const float* scale, const float* shift, int per_species, float* eat,
                              float* dx, hipStream_t s);
hipError_t launch_gen_add(int64_t n, const float* a, float* acc, hipStream_t s);
hipError_t launch_gen_bias(int64_t n, int d, const float* b, float* y, hipStream_t s);
hipError_t launch_gen_fcn_act(int64_t n, int kind, float c, int mode, const float* z, const float* gin,
                              float* out, hipStream_t s);

// ---------------------------------------------------------------- host engine
struct GenModel;
struct GenCtx;

// the rank graph the caller (api.cpp e3gnn_graph_set) has uploaded and indexed
struct GenGraph {
  int64_t n, nl, E;  // nodes (owned + ghost), owned centres, edges
  const int* type;
  const int* nbr;
  const float* vec;
  const int* row_ptr;   // [nl + 1] CSR over edges by centre
  const int* src_ptr;   // [n + 1] transposed CSR
  const int* src_perm;  // [E]
  int* err;
};

// Build from the manifest and the flat weights (throws std::runtime_error with
// the reason on any unsupported or inconsistent deployment).
GenModel* gen_load(const minijson::Value& man, const std::vector<float>& flat);
void gen_free(GenModel* m);
int gen_num_layers(const GenModel* m);
int gen_num_species(const GenModel* m);
float gen_cutoff(const GenModel* m);
int gen_feature_dim(const GenModel* m, int layer);  // dim of x[layer], 0..L

GenCtx* gen_ctx_create(const GenModel* m);
void gen_ctx_free(GenCtx* c);
float* gen_x(GenCtx* c, int layer);
float* gen_grad(GenCtx* c, int layer);

// every call returns hipSuccess or the first failing HIP status
hipError_t gen_graph_set(GenCtx* c, const GenModel* m, const GenGraph& g, hipStream_t s);
hipError_t gen_layer_forward(GenCtx* c, const GenModel* m, const GenGraph& g, int t, hipStream_t s);
hipError_t gen_readout(GenCtx* c, const GenModel* m, const GenGraph& g, float* energy,
                       float* atomic_energy, hipStream_t s);
hipError_t gen_layer_backward(GenCtx* c, const GenModel* m, const GenGraph& g, int t, hipStream_t s);
hipError_t gen_forces(GenCtx* c, const GenModel* m, const GenGraph& g, float* forces, float* virial6,
                      float* edge_grad, hipStream_t s);

}  // namespace e3gnn
