/*
 * e3gnn.h -- C ABI of the MI355X-native SevenNet-0 energy/force library
 * (libe3gnn_hip.so, built from sevennet_finetuning_amd/csrc/ for gfx950).
 *
 * This is the drop-in boundary for the reference's message-passing hot path.
 * Every entry point names the reference interface it replaces:
 *
 *   reference (kskjs1203/SevenNet_finetuning)                      here
 *   -----------------------------------------------------------   -------------------------
 *   torch::jit::load(model.pt, _extra_files)                        e3gnn_load
 *     pair_e3gnn.cpp:294-386 (coeff), deploy.py:15-51
 *   model.forward(dict) + autograd forces/stress                    e3gnn_energy_forces
 *     pair_e3gnn.cpp:205-256, force_output.py:74-130,
 *     sevennet_calculator.py:119-157
 *   segment forward model_list[i].forward(dict)                    e3gnn_graph_set +
 *     pair_e3gnn_parallel.cpp:347-403                                e3gnn_layer_forward
 *   inferred_total_energy / atomic_energy of the last segment        e3gnn_readout
 *   torch::autograd::grad per segment                               e3gnn_layer_backward
 *     pair_e3gnn_parallel.cpp:417-454
 *   force/virial scatter of dE_dr                                   e3gnn_forces
 *     pair_e3gnn_parallel.cpp:474-519
 *   pack/unpack_{forward,reverse}_comm_gnn                          e3gnn_halo_pack/_unpack
 *     pair_e3gnn_parallel.cpp:803-933
 *   ASE primitive_neighbor_list / pair_e3gnn.cpp:144-182            e3gnn_nlist_*
 *   e3nn TensorProduct + message_gather under double backward       e3gnn_conv_graph /
 *     (training: convolution.py:104-123, trainer.py:155-222)         _forward / _backward
 *   e3nn normalize2mom(silu) and its derivatives (training)          e3gnn_act
 *   EquivariantGate / e3nn Gate and its derivatives (training)       e3gnn_gate
 *   second-order fine-tune derivatives, hand-scheduled (training)   e3gnn_act_dual, e3gnn_gate_dual
 *   LAMMPS pair_style d3 settings/coeff, compute/update             e3gnn_d3_create /
 *     (pair_d3.cu:265-767, :2003-2056)                               e3gnn_d3_compute
 *   error->all(FLERR, msg)                                           return code +
 *                                                                    e3gnn_last_error()
 *
 * Conventions (bit-for-bit those of the reference):
 *   edge_center = edge_index[0] (aggregation target), sorted non-decreasing;
 *   edge_nbr    = edge_index[1] (gathered source);
 *   edge_vec    = x_j - x_i (+ periodic image), E x 3 fp32;
 *   F_i += dE/dr_ij, F_j -= dE/dr_ij;
 *   virial6 = -dE/dstrain = inferred_stress * volume, order (xx, yy, zz, xy, yz, zx);
 *     LAMMPS order (xx,yy,zz,xy,xz,yz) is virial6[0,1,2,3,5,4] (pair_e3gnn.cpp:250-255).
 *
 * Memory: every array argument is caller-owned DEVICE memory of the model's
 * device unless stated; the library owns its workspaces (grow-only).  Calls
 * are asynchronous on `stream` (a hipStream_t; NULL = default stream) except
 * where noted.  A context is not thread-safe; use one per host thread.
 * Return value: 0 on success, else a nonzero E3GNN_ERR_* code with a message
 * in e3gnn_last_error() (thread-local).
 */
#ifndef E3GNN_H_
#define E3GNN_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define E3GNN_OK 0
#define E3GNN_ERR_ARG 1   /* bad argument / shape */
#define E3GNN_ERR_HIP 2   /* HIP runtime error */
#define E3GNN_ERR_IO 3    /* model files */
#define E3GNN_ERR_GRAPH 4 /* unsorted edge_center, index or species out of range */

typedef struct e3gnn_model e3gnn_model;
typedef struct e3gnn_ctx e3gnn_ctx;
typedef struct e3gnn_nlist e3gnn_nlist;

const char* e3gnn_last_error(void);
int e3gnn_abi_version(void);

/* Load weights.bin + manifest.json (this build's deploy format; replaces the
 * TorchScript archive + _extra_files, deploy.py:34-51) onto HIP device
 * `device`.  Any E3_equivariant_model deployment (pair_e3gnn.cpp:294-386
 * loads any deployed model): SevenNet-0's architecture runs on its
 * specialised fused kernels, every other member of the nequip family (irreps
 * with parity, lmax <= 2, XPLOR or polynomial cutoff, raw-vector SH, linear or
 * `nequip` self-connection, any radial MLP) on the generic engine; both serve
 * e3gnn_energy_forces and the segment API below.  Returns NULL on failure. */
e3gnn_model* e3gnn_load(const char* weights_path, const char* manifest_path, int device);
void e3gnn_free(e3gnn_model* m);
/* _extra_files metadata: num_species, cutoff, number of interaction layers,
 * comm_size (features exchanged per ghost atom between layers). */
int e3gnn_model_info(const e3gnn_model* m, int* num_species, float* cutoff, int* num_layers,
                     int* comm_size);
/* Grouped f32 GEMM on the library's matrix-core kernel (tgemm.hip), the dense
 * products of the fine-tune step (train_explicit.py) instead of a vendor BLAS:
 *   C = beta C + alpha (op(A) op(B) + op(A2) op(B2))      beta 0 or 1
 * op(X) = X^T when trans_* is set; row-major storage with leading dimensions
 * ld*; k2 = 0: no second operand pair (A2/B2 ignored).  Up to 12 independent
 * problems per call (their outputs must not overlap); long-K problems are split
 * over K into `workspace` (e3gnn_gemm_workspace_floats floats) and reduced in a
 * fixed order: deterministic, no atomics. */
/* General operand layout of a grouped-GEMM problem (e3gnn_gemm_desc::layout):
 * element (i, k) of op(A) (i = row m) or of op(B)^T (i = column n) at
 *   X[(i / rep) * ld + (i % rep) * rs + (k % ks) * kst + (k / ks) * sst]
 * (X, K from the descriptor; K a whole number of ks-row segments) -- e.g. an
 * e3nn irreps block [node][mul][2l+1] as rows (node, m) (rep = 2l + 1), or a
 * linear's weight gradient summed over K = (m, node) segments.  C(m, n) at
 * c[(m / crep) * ldc + (m % crep) * crs + n * cns]. */
typedef struct e3gnn_gemm_layout {
  int64_t ld, kst, sst;
  int32_t rep, rs, ks;
} e3gnn_gemm_layout;
typedef struct e3gnn_gemm_layouts {
  e3gnn_gemm_layout a, b, a2, b2;
  int64_t ldc;
  int32_t crep, crs, cns;
} e3gnn_gemm_layouts;
typedef struct e3gnn_gemm_desc {
  const float* a;
  const float* b;
  const float* a2;
  const float* b2;
  float* c;
  int64_t lda, ldb, lda2, ldb2, ldc;
  int32_t m, n, k, k2;
  int32_t trans_a, trans_b, trans_a2, trans_b2;
  float alpha;
  int32_t beta;
  /* optional block sparsity (nullable): per output tile (64 x 64; tile
   * (tm, tn) reads entry tm * krange_stride_m + tn) four int32 -- the k
   * ranges [lo1, hi1) of the first operand pair and [lo2, hi2) of the second
   * that can be nonzero; the product skips the rest (a linear's dense matrix
   * is block-diagonal by l).  krange_stride_m = 0: one entry per column tile. */
  const int32_t* krange;
  int32_t krange_stride_m;
  /* nullable: the general layouts (then lda.. / trans_* / ldc are unused) */
  const e3gnn_gemm_layouts* layout;
} e3gnn_gemm_desc;
int64_t e3gnn_gemm_workspace_floats(int n, const e3gnn_gemm_desc* d);
int e3gnn_gemm_grouped(int n, const e3gnn_gemm_desc* d, float* workspace, int64_t workspace_floats,
                       void* stream);
/* flags E3GNN_GEMM_DEFER_REDUCE: the split problems' partial slabs stay in
 * `workspace` (not reused until reduced) and their outputs are written later
 * by e3gnn_gemm_reduce -- the fine-tune step reduces all its weight
 * gradients in one launch at the end of the reverse sweep. */
#define E3GNN_GEMM_DEFER_REDUCE 1
int e3gnn_gemm_grouped_ex(int n, const e3gnn_gemm_desc* d, float* workspace, int64_t workspace_floats,
                          int flags, void* stream);
/* The deferred reductions of problems d[0..n) (the descriptors of their
 * launches, in order; workspaces[i] = the workspace pointer their launch got
 * plus the floats of the split problems before it in that launch); problems
 * that were not split are skipped.  Same sums, same order as undeferred. */
int e3gnn_gemm_reduce(int n, const e3gnn_gemm_desc* d, float* const* workspaces, void* stream);

/* The fine-tune loss of the hand-scheduled step in one launch (train.py
 * LossDefinition, loss.py:8-206): criterion 0 MSELoss, 1 HuberLoss(delta), mean
 * over the labelled (non-NaN) entries of each term -- energy per atom
 * (e_pred / natoms, nb graphs), forces (n x 3), stress (nb x 6, times s_scale =
 * eV/A^3 -> kbar; s_pred null: no stress term) -- weighted by w_*.  Writes the
 * weighted term values terms[3] and the cotangents dL/dE[nb], dL/dF[n*3],
 * dL/dS[nb*6].  Deterministic fixed-order sums. */
int e3gnn_loss_efs(int criterion, float delta, int64_t nb, int64_t n, const float* e_pred,
                   const float* e_ref, const int64_t* natoms, const float* f_pred, const float* f_ref,
                   const float* s_pred, const float* s_ref, float w_e, float w_f, float w_s,
                   float s_scale, float* terms, float* ce, float* cf, float* cs, void* stream);
/* EWC over the flat parameter buffer (loss.py:209-252): value[0] = sum f (theta
 * - o)^2 (fixed-order sum; `part`: n + n / 256 + 1 floats of scratch), grad += lam f_train
 * (theta - o) (grad nullable). */
int e3gnn_ewc_flat(int64_t n, const float* theta, const float* f, const float* o, const float* f_train,
                   float lam, float* grad, float* part, float* value, void* stream);

/* Which engine serves the deployment: the channel family of the fused
 * radial-MLP + tensor-product kernels (>= 0: 0 SevenNet-0's 128x0e+64x1e+32x2e,
 * 1 uniform 64, 2 uniform 32 channels; lmax 2, even parity, XPLOR, linear
 * self-connection, 8 Bessel, 64-64 radial MLP, any number of blocks >= 2), or
 * -1: the generic runtime-path-table engine (every other nequip-family model). */
int e3gnn_model_family(const e3gnn_model* m);

e3gnn_ctx* e3gnn_ctx_create(e3gnn_model* m);
void e3gnn_ctx_free(e3gnn_ctx* c);

/* Whole energy+force(+virial) evaluation of one graph (serial pair_e3gnn /
 * deployed_serial.pt).  type[n_atoms] (species index), edge_center/edge_nbr[E]
 * int32, edge_vec[E*3].  Outputs (each nullable except energy): energy[1],
 * atomic_energy[n_atoms], forces[n_atoms*3], virial6[6], edge_grad[E*3] =
 * dE/dedge_vec.  Synchronises `stream` before returning unless the context is
 * in stream-ordered mode (e3gnn_set_stream_ordered). */
int e3gnn_energy_forces(e3gnn_ctx* c, int64_t n_atoms, int64_t n_edges, const int32_t* type,
                        const int32_t* edge_center, const int32_t* edge_nbr,
                        const float* edge_vec, float* energy, float* atomic_energy,
                        float* forces, float* virial6, float* edge_grad, void* stream);

/* ---- segment API (pair_e3gnn_parallel): one rank's local + ghost graph ---- */
/* Nodes [0, n_local) are owned (edge centres), [n_local, n_local+n_ghost) are
 * ghosts.  Copies the inputs (device or host pointers), builds the CSR
 * indices, edge embedding and layer-0 features.  Synchronises `stream` to
 * validate the graph. */
int e3gnn_graph_set(e3gnn_ctx* c, int64_t n_local, int64_t n_ghost, int64_t n_edges,
                    const int32_t* type, const int32_t* edge_center, const int32_t* edge_nbr,
                    const float* edge_vec, void* stream);
/* Interaction block `layer` (0..num_layers-1): reads features of layer
 * `layer` on all n_local+n_ghost rows, writes features of layer+1 on the
 * n_local owned rows (ghost rows are the caller's halo exchange). */
int e3gnn_layer_forward(e3gnn_ctx* c, int layer, void* stream);
/* Device pointer / row width of the features entering layer `layer`
 * (0..num_layers); rows are n_local+n_ghost, contiguous, fp32. */
float* e3gnn_feature_ptr(e3gnn_ctx* c, int layer);
int e3gnn_feature_dim(const e3gnn_ctx* c, int layer);
/* Readout of the owned atoms; energy[1] and atomic_energy[n_local] (nullable)
 * receive the rank-local totals.  Also seeds the backward pass. */
int e3gnn_readout(e3gnn_ctx* c, float* energy, float* atomic_energy, void* stream);
/* Backward of block `layer` (num_layers-1 down to 0): reads dE/dfeatures of
 * layer+1 on owned rows, writes dE/dfeatures of `layer` on all rows (ghost
 * rows are the caller's reverse halo exchange, to be accumulated into the
 * owners' rows before the next call). */
int e3gnn_layer_backward(e3gnn_ctx* c, int layer, void* stream);
float* e3gnn_grad_ptr(e3gnn_ctx* c, int layer);
/* Forces on all n_local+n_ghost rows (ghost rows: reverse-communicate),
 * rank-local virial6 and optional edge_grad[E*3]. */
int e3gnn_forces(e3gnn_ctx* c, float* forces, float* virial6, float* edge_grad, void* stream);

/* ---- halo overlap (the forward_comm / reverse_comm loop of
 * pair_e3gnn_parallel.cpp:371-454, overlapped instead of serialised) ----
 * Owned centres [0, n_interior) have no ghost neighbour (the rank-graph
 * builder orders them first; checked at the next e3gnn_graph_set, which it
 * must precede).  e3gnn_layer_forward = part 0 then part 1, where part 0
 * reads only the OWNED rows of the block's input features (self_interaction_1
 * of the owned rows, the interior centres' convolution) -- run it while the
 * ghost rows are exchanged -- and part 1 the rest.  e3gnn_layer_backward =
 * part 0 then part 1, where part 0 produces everything the GHOST rows of
 * dE/dfeatures need (boundary centres' edges, the ghost rows' gather and
 * self_interaction_1 backward) -- start the reverse exchange after it -- and
 * part 1 the interior centres and the owned rows (accumulate the received
 * ghost contributions after part 1).  n_interior = 0 (default): part 0 of
 * the forward is the owned rows' self_interaction_1 only. */
int e3gnn_set_interior(e3gnn_ctx* c, int64_t n_interior);
int e3gnn_layer_forward_part(e3gnn_ctx* c, int layer, int part, void* stream);
int e3gnn_layer_backward_part(e3gnn_ctx* c, int layer, int part, void* stream);

/* ---- halo kernels ---- */
/* dst[r*dim + k] = src[idx[r]*src_stride + k], r < n */
int e3gnn_halo_pack(const int32_t* idx, int64_t n, int dim, const float* src, int64_t src_stride,
                    float* dst, void* stream);
/* dst[idx[r]*dst_stride + k] (+)= src[r*dim + k]; idx entries must be unique */
int e3gnn_halo_unpack(const int32_t* idx, int64_t n, int dim, const float* src, float* dst,
                      int64_t dst_stride, int accumulate, void* stream);

/* ---- training ops (fine-tune step) ----
 * Stateless convolution primitives on caller-owned device tensors, for the
 * differentiable model of sevennet_finetuning_amd/nn.py, which replaces the
 * reference's e3nn TensorProduct + message_gather inside
 * IrrepsConvolution.forward (sevenn/nn/convolution.py:104-123) when the
 * trainer takes parameter gradients of a force loss (create_graph=True,
 * force_output.py:158-215; trainer.py:155-222).  The product
 *   agg[i] = sum_{e: edge_center[e] = i} TP(h[edge_nbr[e]], Y[e], w[e])
 * is trilinear in (h, Y, w), so every derivative of every order is one of the
 * two launches below with permuted operands.  `kind` selects the SevenNet-0
 * path table: 0 = first block (h 128, w 384, agg 1152), 1 = middle blocks
 * (480, 960, 3136), 2 = last block (480, 224, 224); e3gnn_conv_dims reports
 * them.  Sums are raw (no 1/denominator; the caller divides). */
int e3gnn_conv_dims(int kind, int* h_dim, int* w_dim, int* agg_dim);
/* CSR of the edges (edge_center sorted non-decreasing): row_ptr[n+1],
 * transposed CSR src_ptr[n+1] / src_perm[E] (edges per neighbour, ascending
 * edge id), scratch[n+1] int32.  Validates the graph (synchronises `stream`;
 * E3GNN_ERR_GRAPH if unsorted or out of range). */
int e3gnn_conv_graph(int64_t n_nodes, int64_t n_edges, const int32_t* edge_center,
                     const int32_t* edge_nbr, int32_t* row_ptr, int32_t* src_ptr,
                     int32_t* src_perm, int32_t* scratch, void* stream);
/* The same build from int64 edge indices (a batch's edge_index rows), also
 * writing their int32 copies center_out / nbr_out [E]; graphs of at most
 * e3gnn_conv_graph_small_max_nodes() nodes and e3gnn_conv_graph_small_max_edges()
 * edges (one workgroup, one launch -- the per-step rebuild of a captured
 * fine-tune step). */
int e3gnn_conv_graph_i64(int64_t n_nodes, int64_t n_edges, const int64_t* edge_center,
                         const int64_t* edge_nbr, int32_t* center_out, int32_t* nbr_out,
                         int32_t* row_ptr, int32_t* src_ptr, int32_t* src_perm, int32_t* scratch,
                         void* stream);
int e3gnn_conv_graph_small_max_nodes(void);
int e3gnn_conv_graph_small_max_edges(void);
/* agg[n_nodes x agg_dim] = segmented sum of TP(h[nbr], Y, w); Y [E x 9],
 * w [E x w_dim], h [n_nodes x h_dim]. */
int e3gnn_conv_forward(int kind, int64_t n_nodes, const int32_t* row_ptr, const int32_t* edge_nbr,
                       const float* h, const float* Y, const float* w, float* agg, void* stream);
/* Gradients of <gagg, agg(h, Y, w)>: dY [E x 9] and dw [E x w_dim]
 * (overwritten), dh [n_nodes x h_dim] (nullable; needs dxc [E x h_dim] scratch
 * and the transposed CSR; summed per neighbour in ascending edge order). */
int e3gnn_conv_backward(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                        const int32_t* edge_nbr, const int32_t* src_ptr, const int32_t* src_perm,
                        const float* h, const float* Y, const float* w, const float* gagg,
                        float* dh, float* dY, float* dw, float* dxc, void* stream);
/* The same with accumulation (the hand-scheduled fine-tune derivatives sum
 * several trilinear products into one buffer): forward accumulate & 1: agg +=;
 * backward accumulate bits 1 / 2 / 4: dh / dY / dw += instead of =. */
int e3gnn_conv_forward_acc(int kind, int64_t n_nodes, const int32_t* row_ptr,
                           const int32_t* edge_nbr, const float* h, const float* Y, const float* w,
                           float* agg, int accumulate, void* stream);
int e3gnn_conv_backward_acc(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                            const int32_t* edge_nbr, const int32_t* src_ptr,
                            const int32_t* src_perm, const float* h, const float* Y, const float* w,
                            const float* gagg, float* dh, float* dY, float* dw, float* dxc,
                            int accumulate, void* stream);

/* Radial MLP of the fine-tune step (convolution.py:97-106's weight_nn, e ->
 * W0 -> phi -> W1 -> phi -> W2, phi = 1.6792 silu = act_scale * silu; W0
 * [8, 64], W1 [64, 64], W2 [64, width] row-major, already scaled by
 * 1/sqrt(fan-in)), whole chains per 16-row tile (mlp_train.hip):
 *   e3gnn_radial_mlp_forward   a1 = e W0, h1 = phi(a1), a2 = h1 W1,
 *                              h2 = phi(a2), w = h2 W2 (rows of 8 / 64 / width);
 *                              with a1_primal / a2_primal: the tangent chain
 *                              (h1 = phi'(a1_primal) a1, h2 = phi'(a2_primal) a2)
 *   e3gnn_radial_mlp_backward  h2b = wb W2^T, a2b = phi'(a2) h2b,
 *                              h1b = a2b W1^T, a1b = phi'(a1) h1b, embb += a1b W0^T;
 *                              with a1_tangent / a2_tangent: the reverse of the
 *                              (primal, tangent) pairs over 2 n_rows rows of wb /
 *                              a2b / a1b / embb (primal rows first);
 *                              a2b / a1b nullable.  width % 16 == 0 (both). */
int e3gnn_radial_mlp_forward(int64_t n_rows, int width, const float* emb, const float* W0,
                             const float* W1, const float* W2, const float* a1_primal,
                             const float* a2_primal, float* a1, float* h1, float* a2, float* h2,
                             float* w, float act_scale, void* stream);
/* The forward / tangent chain with layer 2 on bf16 matrix cores at f32-grade
 * accuracy (bf16x6: three bf16 pieces per operand, the six products above
 * 2^-24): w2_pieces = W2's piece image from e3gnn_radial_mlp_w2_pieces
 * (e3gnn_radial_mlp_w2_piece_bytes(width) bytes, 16-byte aligned; rebuilt
 * whenever W2 changes); null: the f32 form above. */
int e3gnn_radial_mlp_forward_p(int64_t n_rows, int width, const float* emb, const float* W0,
                               const float* W1, const float* W2, const void* w2_pieces,
                               const float* a1_primal, const float* a2_primal, float* a1, float* h1,
                               float* a2, float* h2, float* w, float act_scale, void* stream);
/* The reverse / dual chain with h2b = wb W2^T on bf16x6 (w2_pieces as above;
 * width % 32 == 0, else the f32 form runs). */
int e3gnn_radial_mlp_backward_p(int64_t n_rows, int width, const float* wb, const float* W0,
                                const float* W1, const float* W2, const void* w2_pieces, const float* a1,
                                const float* a2, const float* a1_tangent, const float* a2_tangent,
                                float* a2b, float* a1b, float* embb, float act_scale, void* stream);
int64_t e3gnn_radial_mlp_w2_piece_bytes(int width);
/* piece images of n (<= 8) W2 matrices [64, widths[i]] in one launch */
int e3gnn_radial_mlp_w2_pieces(int n, const float* const* W2, const int32_t* widths, void* const* images,
                               void* stream);
int e3gnn_radial_mlp_backward(int64_t n_rows, int width, const float* wb, const float* W0,
                              const float* W1, const float* W2, const float* a1, const float* a2,
                              const float* a1_tangent, const float* a2_tangent, float* a2b,
                              float* a1b, float* embb, float act_scale, void* stream);

/* Edge geometry of the fine-tune step (train_explicit.py), float32, one thread
 * per edge; raw_sh as the model's sh_normalize == false:
 *   e3gnn_edge_geometry      Y [E, 9], emb [E, 8] (EdgeEmbedding.forward,
 *                            edge_embedding.py:220-230; as e3gnn_energy_forces)
 *   e3gnn_edge_geometry_vjp  fij [E, 3] = dE/dr_e from dE/dY, dE/demb
 *                            (force_output.py:158-215's autograd.grad)
 *   e3gnn_edge_geometry_jvp  the tangent along v_e = cF[center] - cF[nbr]
 *                            - (c0 r0 + c5 r2, c1 r1 + c3 r0, c2 r2 + c4 r1),
 *                            c = cS[batch[nbr]] / vol[batch[nbr]] (cS, batch,
 *                            vol NULL: no stress term): Yd [E, 9], embd [E, 8],
 *                            rd [E] = r_hat . v
 *   e3gnn_edge_geometry_coeff_grad  out [E, 8]: per-edge d/dc_n of
 *                            <embb, emb> + <embdb, emb'> (Bessel coefficients)
 *   e3gnn_edge_forces_to_atoms  F_i = sum_{centre i} fij - sum_{nbr i} fij
 *                            over the CSR of e3gnn_conv_graph (fixed order) */
int e3gnn_edge_geometry(int64_t n_edges, const float* vec, const float* coeffs, float rc, float ron,
                        int raw_sh, float* Y, float* emb, void* stream);
int e3gnn_edge_geometry_jvp(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                            float ron, int raw_sh, const int32_t* center, const int32_t* nbr,
                            const int64_t* batch, const float* cF, const float* cS,
                            const float* vol, float* Yd, float* embd, float* rd, void* stream);
int e3gnn_edge_geometry_vjp(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                            float ron, int raw_sh, const float* Yb, const float* embb, float* fij,
                            void* stream);
int e3gnn_edge_geometry_coeff_grad(int64_t n_edges, const float* vec, const float* coeffs, float rc,
                                   float ron, const float* embb, const float* embdb, const float* rd,
                                   float* out, void* stream);
int e3gnn_edge_forces_to_atoms(int64_t n_nodes, const int32_t* row_ptr, const int32_t* src_ptr,
                               const int32_t* src_perm, const float* fij, float* F, void* stream);

/* The fine-tune step's derivatives of the trilinear agg = C(h, Y, w) along a
 * tangent (h', Y', w') (train_explicit.py), one launch each:
 *   tangent forward  agg' (= or += with accumulate & 1)
 *                    = C(h, Y', w) + C(h, Y, w') + C(h', Y, w);
 *   dual backward, cotangents (g, g') of (agg, agg'):
 *     dh  = B_h(Y, w; g) + B_h(Y', w; g') + B_h(Y, w'; g')   dh' = B_h(Y, w; g')
 *     dw  = B_w(h, Y; g) + B_w(h, Y'; g') + B_w(h', Y; g')   dw' = B_w(h, Y; g')
 * (B_h / B_w: e3gnn_conv_backward's dh / dw).  hd may be NULL (no h'; then
 * dhd must be NULL too).  dxc: scratch of [2 n_edges, DX] floats ([n_edges,
 * DX] without h').  Outputs are overwritten.  Replaces the reference's
 * autograd double backward of convolution.py:104-123 under
 * force_output.py:158-215 (create_graph=True, trainer.py:155-222). */
int e3gnn_conv_tangent_forward(int kind, int64_t n_nodes, const int32_t* row_ptr,
                               const int32_t* edge_nbr, const float* h, const float* hd,
                               const float* Y, const float* Yd, const float* w, const float* wd,
                               float* agg, int accumulate, void* stream);
int e3gnn_conv_dual_backward(int kind, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                             const int32_t* edge_nbr, const int32_t* src_ptr,
                             const int32_t* src_perm, const float* h, const float* hd,
                             const float* Y, const float* Yd, const float* w, const float* wd,
                             const float* g, const float* gd, float* dh, float* dhd, float* dw,
                             float* dwd, float* dxc, void* stream);

/* ---- generic path tables: the convolution of any nequip-family model ----
 * Same contract as e3gnn_conv_forward / _backward (IrrepsConvolution,
 * sevenn/nn/convolution.py:36-123), with the instruction list given at run
 * time instead of the SevenNet-0 kinds: paths[8 * n_paths] = per instruction
 * (l1, l2, l3, mul, x offset, Y offset, w column offset, agg offset), l <= 2,
 * uvu coupling wigner_3j * sqrt(2 l3 + 1); h [n x dx], Y [E x dy], w [E x dw],
 * agg [n x dm].  Serves e.g. the reference's HfO2 example deployment
 * (odd parity, lmax 1; example_inputs/md_serial_example).  The handle lives on
 * the device current at creation. */
typedef struct e3gnn_gtp e3gnn_gtp;
e3gnn_gtp* e3gnn_gtp_create(int n_paths, const int32_t* paths, int dx, int dy, int dw, int dm);
void e3gnn_gtp_free(e3gnn_gtp* g);
int e3gnn_gtp_dims(const e3gnn_gtp* g, int* dx, int* dy, int* dw, int* dm);
int e3gnn_gtp_forward(const e3gnn_gtp* g, int64_t n_nodes, const int32_t* row_ptr,
                      const int32_t* edge_nbr, const float* h, const float* Y, const float* w,
                      float* agg, void* stream);
int e3gnn_gtp_backward(const e3gnn_gtp* g, int64_t n_nodes, int64_t n_edges, const int32_t* row_ptr,
                       const int32_t* edge_nbr, const int32_t* src_ptr, const int32_t* src_perm,
                       const float* h, const float* Y, const float* w, const float* gagg,
                       float* dh, float* dY, float* dw, float* dxc, void* stream);

/* Scaled SiLU of the trainable model (y = scale * silu(x); e3nn normalize2mom,
 * SevenNet's act_radial / act_scalar / act_gate, silu_norm 1.6792), element-
 * wise over n floats: op 0 out0 = y(x); op 1 out0 = g * y'(x); op 2 (the
 * derivative of op 1 against the cotangent gg) out0 = gg * g * y''(x),
 * out1 = gg * y'(x) (either nullable). */
int e3gnn_act(int op, int64_t n, const float* x, const float* g, const float* gg, float* out0,
              float* out1, float scale, void* stream);

/* e3nn Gate of the trainable model (EquivariantGate, equivariant_gate.py:13-61)
 * on n rows: y = [scalars | gates | gated blocks], o = [act(scalars) |
 * act(gate_k) * block_k] with act = scale * silu.  op 0: out0 = o; op 1: out0 =
 * dy for the output cotangent go; op 2 (cotangent q of that dy): out0 = d/dgo,
 * out1 = d/dy (either nullable).  dims[13]: n_scalars, n_gates, row_in, row_out,
 * n_groups (<= 2), then per group: offset_in, offset_out, mul, 2l+1. */
int e3gnn_gate(int op, int64_t n, const int32_t* dims, const float* y, const float* go,
               const float* q, float* out0, float* out1, float scale, void* stream);

/* The hand-scheduled fine-tune derivatives (train_explicit.py: a tangent
 * forward along dL/dforces and one reverse sweep replace the double backward
 * of ForceStressOutputFromEdge, force_output.py:158-215, under the trainer's
 * loss.backward(), trainer.py:155-222).  e3gnn_act_dual: the reverse of
 * (y(x), y'(x) xd): og = g y'(x) + gd y''(x) xd, ogd = gd y'(x). */
int e3gnn_act_dual(int64_t n, const float* x, const float* xd, const float* g, const float* gd,
                   float* og, float* ogd, float scale, void* stream);

/* Gate of e3gnn_gate, tangent and dual reverse: op 0 out0 = J(y) yd; op 1
 * out0 = J(y)^T xb + d/dy <xdb, J(y) yd>, out1 = J(y)^T xdb. */
int e3gnn_gate_dual(int op, int64_t n, const int32_t* dims, const float* y, const float* yd,
                    const float* xb, const float* xdb, float* out0, float* out1, float scale,
                    void* stream);

/* ---- device neighbour list (the graph build in front of the hot path) ----
 * Replaces ASE primitive_neighbor_list('ijDS', pbc, cell, pos, cutoff,
 * self_interaction=True) minus the (i, i, S = 0) pair (sevenn/train/
 * dataload.py:31-68, :113-125) and the host loops of pair_e3gnn.cpp:155-182.
 * Edges (i, j, S): r_ij = pos[j] + S cell - pos[i], |r_ij| < cutoff, sorted by
 * (i, j, S) -- the CSR order e3gnn_energy_forces takes.  pos: device f64
 * [n][3]; cell: HOST f64 [3][3] (rows a, b, c; unused when pbc is all 0);
 * pbc: HOST int[3], all 1 (periodic) or all 0 (isolated cluster).
 * e3gnn_nlist_build counts the edges (synchronises `stream`) and keeps the
 * binning; e3gnn_nlist_fetch then writes edge_center/edge_nbr int32 [E],
 * shift int32 [E][3] and edge_vec f32 [E][3] (both nullable) -- device memory
 * the caller sized from *n_edges.  At most 512 neighbours per centre. */
e3gnn_nlist* e3gnn_nlist_create(int device);
void e3gnn_nlist_free(e3gnn_nlist* h);
int e3gnn_nlist_build(e3gnn_nlist* h, int64_t n, const double* pos, const double* cell,
                      const int* pbc, double cutoff, int64_t* n_edges, void* stream);
int e3gnn_nlist_fetch(e3gnn_nlist* h, int32_t* edge_center, int32_t* edge_nbr, int32_t* shift,
                      float* edge_vec, void* stream);

/* ---- DFT-D3 dispersion ----
 * Replaces the reference's LAMMPS pair style d3 (sevenn/pair_e3gnn/pair_d3.cu):
 * e3gnn_d3_create = PairD3::settings + coeff (:265-307, :656-767),
 * e3gnn_d3_compute = PairD3::compute + update (:2030-2056, :2003-2024).
 * damping: 1 zero ("damp_zero"), 2 Becke-Johnson ("damp_bj"), 4 "damp_bjm"
 * (the BJ kernel, as in the reference); 3 "damp_zerom" is refused (the
 * reference leaves it unimplemented, :1550-1553).  func = {s6, s8, a1, a2,
 * alp6, alp8} (setfuncpar :422-653: a1 = rs6, a2 = rs18, s8 = s18, alp8 =
 * alp6 + 2); rthr / cn_thr: squared cutoffs in bohr^2 (pair_style d3 args).
 * Per-type tables (host, copied): rcov [nt] (bohr), r2r4 [nt], r0ab [nt][nt]
 * (bohr), mxc [nt], c6ab [nt][nt][5][5][3] = (C6, CN_ref_i, CN_ref_j).
 * e3gnn_d3_compute takes HOST arrays as LAMMPS holds them: pos f64 [n][3] (A),
 * cell f64 [3][3] (rows a, b, c, A), pbc int[3], type int32 [n] in
 * [0, ntypes); returns energy (eV), forces f64 [n][3] (eV/A) and virial6 (eV,
 * LAMMPS order xx, yy, zz, xy, xz, yz) on the host; synchronises `stream`.
 * Deterministic (no atomics). */
typedef struct e3gnn_d3 e3gnn_d3;
e3gnn_d3* e3gnn_d3_create(int device, int damping, const float* func, float rthr, float cn_thr,
                          int ntypes, const float* rcov, const float* r2r4, const float* r0ab,
                          const int32_t* mxc, const float* c6ab);
void e3gnn_d3_free(e3gnn_d3* h);
int e3gnn_d3_compute(e3gnn_d3* h, int64_t n, const double* pos, const double* cell,
                     const int32_t* pbc, const int32_t* type, double* energy, double* forces,
                     double* virial6, void* stream);

/* ---- diagnostics ---- */
/* Kernel implementation of the convolution: 0 = fused radial-MLP + tensor
 * product (default), 1 = unfused v1 kernels (per-edge weights materialised in
 * HBM; kept as an independent cross-check).  Env E3GNN_IMPL=v1 sets 1.
 * Takes effect at the next e3gnn_graph_set / e3gnn_energy_forces. */
int e3gnn_set_impl(e3gnn_ctx* c, int impl);
/* enable per-kernel-class HIP-event timing on the context */
int e3gnn_set_timing(e3gnn_ctx* c, int enable);
/* Stream-ordered mode (default off): e3gnn_energy_forces returns once its
 * work is enqueued on `stream` (the inputs already copied and the graph
 * validated) instead of synchronising it -- the outputs are ready in stream
 * order, as a PyTorch module's outputs are (the reference's deployed model
 * called from Python, deploy.py:20-32).  Hosts that read the outputs from
 * other streams or the CPU synchronise the stream themselves.  The context's
 * workspaces are shared between calls: a call on a different stream than the
 * previous stream-ordered evaluation first makes its stream wait (device-side
 * event) for that evaluation's end. */
int e3gnn_set_stream_ordered(e3gnn_ctx* c, int enable);
/* Number of kernel classes recorded; fills up to `max` entries: name (static
 * string), total ms, launches, algorithmic FLOP and algorithmic HBM bytes. */
int e3gnn_kernel_stats(e3gnn_ctx* c, const char** names, double* ms, int64_t* launches,
                       double* flops, double* bytes, int max);
int e3gnn_reset_stats(e3gnn_ctx* c);
/* Dense coupling table C_{l1 l2 l3}[m1][m2][m3] * sqrt(2 l3 + 1) used by the
 * kernels (host memory, (2l1+1)(2l2+1)(2l3+1) floats). */
int e3gnn_cg_table(int l1, int l2, int l3, float* out);
/* Device pointer + element count of an internal workspace buffer (debug /
 * layer-wise parity tests): "x","grad" (layer 0..L), "h","y","agg" (0..L-1;
 * "agg" holds the last layer computed), "Y","emb","dY","dgu","demb","dxc","fe". */
float* e3gnn_debug_ptr(e3gnn_ctx* c, const char* name, int layer, int64_t* numel);
/* Bytes of device workspace currently held by the context. */
int64_t e3gnn_workspace_bytes(const e3gnn_ctx* c);

#ifdef __cplusplus
}
#endif
#endif /* E3GNN_H_ */
