// Launchers of node.hip (edge geometry, graph indices, node ops, reductions).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace e3gnn {
hipError_t launch_edge_embed(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                             int raw_sh, float* Y, float* emb, hipStream_t s);
// the fine-tune step's edge-geometry tangent / coefficient gradient (node.hip)
hipError_t launch_edge_geom_jvp(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                                int raw_sh, const int* center, const int* nbr, const int64_t* batch,
                                const float* cF, const float* cS, const float* vol, float* Yd,
                                float* embd, float* rd, hipStream_t s);
hipError_t launch_edge_geom_coeff(int64_t E, const float* vec, const float* coeffs, float rc,
                                  float ron, const float* embb, const float* embdb, const float* rd,
                                  float* out, hipStream_t s);
int edge_force_blocks(int64_t E);
hipError_t launch_edge_force(int64_t E, const float* vec, const float* coeffs, float rc, float ron,
                             int raw_sh, const float* dY, const float* dgu, const float* demb, float* fe,
                             float* vir_part, hipStream_t s);  // vir_part nullable
hipError_t launch_atom_force(int n_nodes, int n_centers, const int* row_ptr, const int* src_ptr,
                             const int* src_perm, const float* fe, float* F, hipStream_t s);
hipError_t launch_build_graph(int64_t E, int n_centers, int n_nodes, const int* center,
                              const int* nbr, int* row_ptr, int* src_ptr, int* src_perm, int* cnt,
                              int* err, hipStream_t s, int n_interior = 0);
// the whole build in one workgroup (n <= graph_small_max_nodes(), E <=
// graph_small_max_edges()); int64
// indices (c64 / j64, converted into cout / jout) or int32 ones (c32 / j32);
// writes *err (no memset needed)
hipError_t launch_build_graph_small(int64_t E, int n, const int* c32, const int* j32, const int64_t* c64,
                                    const int64_t* j64, int* cout, int* jout, int* row_ptr, int* src_ptr,
                                    int* src_perm, int* err, hipStream_t s);
int graph_small_max_nodes();
int graph_small_max_edges();
hipError_t launch_embed(int n, int D, const int* type, int nsp, const float* W, float* x, int* err,
                        hipStream_t s);
// e3nn Gate of the SevenNet-0-shaped family: y = [ns scalars | g1 + g2 gates |
// g1 x 1e | g2 x 2e] -> x = [ns x 0e | g1 x 1e | g2 x 2e]; the last block
// (scalars only) uses ns alone
struct GateDims {
  int ns, g1, g2;
  __host__ __device__ int dx() const { return ns + 3 * g1 + 5 * g2; }
  __host__ __device__ int dy() const { return ns + 4 * g1 + 6 * g2; }
};
hipError_t launch_gate_fwd(int n, bool last, GateDims d, const float* y, float* x, hipStream_t s);
hipError_t launch_gate_bwd(int n, bool last, GateDims d, const float* y, const float* dx, float* dy,
                           hipStream_t s);
hipError_t launch_readout(int n, int D, const float* x, const float* v, const int* type,
                          const float* scale, const float* shift, float* eat, hipStream_t s);
hipError_t launch_readout_bwd(int n, int D, const float* v, const int* type, const float* scale,
                              float* dx, hipStream_t s);
int sum_blocks(int64_t n);
hipError_t launch_sum(int64_t n, const float* a, float* part, float* out, hipStream_t s);
hipError_t launch_final_sum(int nb, int k, const float* part, float* out, hipStream_t s);
hipError_t launch_zero(float* p, int64_t n, hipStream_t s);
// acc: dst += the sums instead of dst = (the explicit fine-tune derivatives)
// two gathers over the same transposed CSR in one launch (src -> dst, src2 -> dst2)
hipError_t launch_gather_rows2(int n, int D, const int* ptr, const int* perm, const float* src,
                               float* dst, const float* src2, float* dst2, hipStream_t s);
hipError_t launch_gather_rows(int n, int D, const int* ptr, const int* perm, const float* src,
                              float* dst, hipStream_t s, int acc = 0);
// the same over neighbour nodes [j_begin, j_end) only
hipError_t launch_gather_rows_range(int j_begin, int j_end, int D, const int* ptr, const int* perm,
                                    const float* src, float* dst, hipStream_t s, int acc = 0);
hipError_t launch_pack(int64_t n, int dim, const int* idx, const float* src, int64_t ss, float* dst,
                       hipStream_t s);
hipError_t launch_unpack(int64_t n, int dim, const int* idx, const float* src, float* dst,
                         int64_t ds, int acc, hipStream_t s);
}  // namespace e3gnn
