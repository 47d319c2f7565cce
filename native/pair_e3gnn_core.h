// pair_e3gnn_core -- the LAMMPS-independent per-step core of the LAMMPS pair
// styles e3gnn/hip and e3gnn/parallel/hip (native/lammps/), over the C ABI of
// libe3gnn_hip.so.  The LAMMPS adaptors only map Atom / NeighList / Comm onto
// the views below; everything the reference does per step between LAMMPS and
// the model lives here, so it is compiled and tested without LAMMPS
// (native/e3gnn_pair_check.cpp).
//
// Reference: sevenn/pair_e3gnn/pair_e3gnn.cpp (PairE3GNN::compute :72-275,
// ::coeff :294-386) and pair_e3gnn_parallel.cpp (PairE3GNNParallel::compute
// :207-541, comm_preprocess / pack_/unpack_{forward,reverse}_comm_gnn
// :693-933).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "e3gnn.h"

namespace e3gnn_pair {

// What LAMMPS hands a full-neighbour-list pair style each step (Atom + NeighList)
struct NeighborView {
  int inum = 0;                      // list->inum (== atom->nlocal)
  const int* ilist = nullptr;        // list->ilist
  const int* numneigh = nullptr;     // list->numneigh
  int* const* firstneigh = nullptr;  // list->firstneigh (j may carry special bits)
  double* const* x = nullptr;        // atom->x, local then ghost rows
  const int* type = nullptr;         // atom->type (1-based LAMMPS types)
  const int64_t* tag = nullptr;      // atom->tag (1..natoms; ghosts carry their owner's tag)
  int nlocal = 0, nghost = 0;
  int neighmask = 0x1FFFFFFF;        // NEIGHMASK
};

// LAMMPS' per-step accumulators of a pair style (Pair::eng_vdwl, virial[6],
// eatom[], f[][3]); virial in LAMMPS order (xx, yy, zz, xy, xz, yz)
struct PairOut {
  double energy = 0.0;
  double virial[6] = {0, 0, 0, 0, 0, 0};
};

// The deployment and its species map: pair_coeff * * <model dir> <element per type>
class Model {
 public:
  // weights.bin + manifest.json of `model_dir`; throws std::runtime_error
  Model(const std::string& model_dir, int device);
  ~Model();
  Model(const Model&) = delete;
  Model& operator=(const Model&) = delete;
  // PairE3GNN::coeff (pair_e3gnn.cpp:330-378): elements[k] is the chemical
  // symbol of LAMMPS type k + 1; returns map[type] = species index (map[0]
  // unused); throws on an element the model does not know
  std::vector<int> type_map(const std::vector<std::string>& elements) const;
  double cutoff() const { return cutoff_; }
  int comm_size() const { return comm_size_; }
  int num_layers() const { return nlayers_; }
  e3gnn_model* handle() const { return m_; }
  const std::vector<std::string>& symbols() const { return symbols_; }

 private:
  e3gnn_model* m_ = nullptr;
  double cutoff_ = 0.0;
  int comm_size_ = 0, nlayers_ = 0, nspecies_ = 0;
  std::vector<std::string> symbols_;
};

// Device buffers that grow with the graph (the reference's nedges_bound)
struct DeviceGraph {
  int32_t *type = nullptr, *center = nullptr, *nbr = nullptr;
  float *vec = nullptr, *forces = nullptr, *atomic = nullptr, *scalars = nullptr;
  int64_t cap_n = 0, cap_e = 0;
  void reserve(int64_t n, int64_t e);
  void release();
};

// pair_style e3gnn/hip: one rank holds every atom (local rows), ghosts are
// periodic images identified by tag (PairE3GNN::compute, pair_e3gnn.cpp:72-275):
// graph nodes are tag - 1, edges i -> j for every full-list neighbour within
// the cutoff, edge_vec = x_j - x_i.  Forces and eatom are ADDED to what the
// host holds in f / eatom (the reference assigns; adding keeps pair_style
// hybrid/overlay correct), the energy and virial (LAMMPS order) added to `out`.
class SerialStep {
 public:
  explicit SerialStep(const Model& model);
  ~SerialStep();
  // returns 0, or an E3GNN_ERR_* code with the message in error()
  int compute(const NeighborView& nv, const std::vector<int>& map, double** f, double* eatom,
              PairOut& out);
  const std::string& error() const { return err_; }
  int64_t last_edges() const { return nedges_; }

 private:
  const Model& model_;
  e3gnn_ctx* ctx_ = nullptr;
  void* stream_ = nullptr;
  DeviceGraph g_;
  std::vector<int32_t> type_, center_, nbr_;
  std::vector<float> vec_, forces_, atomic_;
  std::vector<int> tag2i_;
  int64_t nedges_ = 0;
  std::string err_;
};

// pair_style e3gnn/parallel/hip (PairE3GNNParallel::compute,
// pair_e3gnn_parallel.cpp:207-541): graph rows = the rank's local atoms (list
// order), then every ghost within the cutoff of a local atom, first seen,
// deduplicated by tag; per layer the ghost rows' features arrive through the
// halo exchange, after the readout the ghost rows' dE/dx go back.  Forces of
// local AND ghost rows are added to f (a ghost row's force to the first-seen
// LAMMPS image of its atom); the host's own newton-on reverse communication
// then sums the ghost forces onto their owners -- compute() does not.  The
// exchange itself belongs to the host (LAMMPS CommBrick through
// pack/unpack_*_comm_gnn, row maps in CommMaps below): the step exposes the row
// buffer `comm_rows()` = [graph rows | extra rows | zero row | trash rows].
class ParallelStep {
 public:
  // the host's exchange: called once per layer boundary (forward) and once
  // per backward layer boundary (reverse)
  struct Exchange {
    virtual ~Exchange() = default;
    // ghost rows <- owners' rows of step.comm_rows() (row width step.comm_dim())
    virtual int forward(ParallelStep& step) = 0;
    // owners' rows += ghost rows' values of step.comm_rows()
    virtual int reverse(ParallelStep& step) = 0;
  };
  explicit ParallelStep(const Model& model);
  ~ParallelStep();
  // builds the rank graph (tag -> graph row map of the reference); call before compute
  int build(const NeighborView& nv, const std::vector<int>& map, int64_t natoms);
  // graph row of a LAMMPS atom index (local or ghost), or -1 when it is not in
  // this rank's graph (the host then gives it an extra row: extra_row())
  int graph_row(int lammps_index) const;
  // the extra row (>= graph_size) of an atom this rank relays but does not
  // use.  Keyed by TAG, O(1): every LAMMPS image of one atom shares one extra
  // row (the reference keys by LAMMPS index, pair_e3gnn_parallel.cpp:764-777,
  // which gives a relayed periodic self-image of a relayed ghost a fresh zero row)
  int extra_row(int lammps_index);
  // graph row, else extra row
  int row_of(int lammps_index) { const int r = graph_row(lammps_index); return r >= 0 ? r : extra_row(lammps_index); }
  int graph_size() const { return (int)row_to_i_.size(); }
  int extra_rows() const { return nextra_; }
  int64_t nlocal() const { return nlocal_; }
  int64_t nedges() const { return (int64_t)center_.size(); }
  // row buffer of the current exchange on the device, width comm_dim() floats
  float* comm_rows() const { return comm_; }
  int comm_dim() const { return comm_dim_; }
  // a row that stays zero (source of the reverse copies that must add nothing)
  int zero_row() const { return graph_size() + nextra_; }
  // sink rows for duplicate entries of one unpack (each used once per call)
  int trash_row(int k) const { return zero_row() + 1 + k; }
  void set_trash_rows(int n) { ntrash_ = n; }
  int comm_row_count() const { return zero_row() + 1 + ntrash_; }
  // device row pack / unpack for the host's message buffers (e3gnn_halo_pack
  // / _unpack on comm_rows(); idx: device int32 rows)
  int pack(const int32_t* idx, int64_t n, float* buf);
  int unpack(const int32_t* idx, int64_t n, const float* buf, bool accumulate);
  // one evaluation: forward with `ex.forward` between the blocks, backward
  // with `ex.reverse` after each block and for the ghost forces
  int compute(Exchange& ex, double** f, double* eatom, PairOut& out);
  const std::string& error() const { return err_; }
  void* stream() const { return stream_; }

 private:
  int grow_comm(int rows, int dim);
  int load_rows(float* src, int dim, int rows);    // graph rows of src -> comm
  int store_rows(float* dst, int dim, int rows);   // comm -> src (rows)
  const Model& model_;
  e3gnn_ctx* ctx_ = nullptr;
  void* stream_ = nullptr;
  DeviceGraph g_;
  int64_t nlocal_ = 0, nghost_graph_ = 0;
  std::vector<int32_t> type_, center_, nbr_;
  std::vector<float> vec_, forces_, atomic_;
  std::vector<int> row_to_i_;          // graph row -> LAMMPS atom index
  std::vector<int> i_to_row_;          // LAMMPS atom index -> graph row (-1)
  std::vector<int> tag_to_row_;        // tag -> graph row (-1)
  std::vector<int> tag_to_extra_;      // tag -> extra row (-1)
  int nextra_ = 0, ntrash_ = 0;
  const int64_t* tag_ = nullptr;
  int64_t ntotal_ = 0;                 // nlocal + nghost of the last build
  float* comm_ = nullptr;
  int64_t comm_cap_ = 0;
  int comm_dim_ = 0, comm_nrows_ = 0;
  std::string err_;
};

// The per-swap row maps of CommBrick's GNN exchange, LAMMPS-free: what
// PairE3GNNParallel builds in its "false" preprocessing forward_comm
// (pack_forward_init / unpack_forward_init, pair_e3gnn_parallel.cpp:750-801)
// and comm_preprocess (:703-748), and the four row copies of
// pack/unpack_{forward,reverse}_comm_gnn (:803-933) on device buffers.
//
// CommBrick (comm_brick.cpp:1057-1120) runs up to 6 swaps (-/+ per dimension,
// self swaps skipped); a swap also forwards ghosts received in earlier swaps
// (corner atoms relayed through extra rows).  Rows are per TAG on every rank,
// so one rank may receive an atom several times (both swaps of a dimension
// with two ranks; several images relayed in one swap) into one row.  The
// reverse must return each row's value to its sender exactly once:
//  * receiver side: a received entry packs its row's value only at the row's
//    first occurrence over (swap, position); later copies pack the zero row;
//  * sender side: within one swap the first occurrence of a row accumulates,
//    later ones (zeros by the rule above) go to distinct trash rows, so every
//    e3gnn_halo_unpack call has unique destination rows (its contract);
//  * a forward-received duplicate is written to a trash row likewise.
// This differs from the reference's sender-only dedup (one `already_met` set
// over all swaps, :712-733), which drops a corner atom's gradient returned by a
// SECOND rank (e.g. the y neighbour after the x neighbour in a 2x2x1 grid) and
// adds duplicate extra-row copies more than once.
class CommMaps {
 public:
  static constexpr int kPhases = 6;
  explicit CommMaps(ParallelStep& step) : s_(step) {}
  ~CommMaps();
  CommMaps(const CommMaps&) = delete;
  CommMaps& operator=(const CommMaps&) = delete;
  // before the preprocessing forward_comm (comm_preprocess_done = false)
  void begin();
  // the CommBrick hooks; return 0 or E3GNN_ERR_ARG (phase >= 6: "Cell size is too small")
  int pack_forward_init(int n, const int* list_send, int phase);
  int unpack_forward_init(int n, int first, int phase);
  // builds the dedup lists, sizes the trash rows, uploads the index lists
  int finish();
  bool ready() const { return ready_; }
  int64_t nsend(int phase) const { return (int64_t)send_[phase].size(); }
  int64_t nrecv(int phase) const { return (int64_t)recv_[phase].size(); }
  // device buffers of nsend/nrecv x comm_dim floats; return the float count or -1
  int64_t pack_forward(int phase, float* buf);
  int64_t unpack_forward(int phase, const float* buf);
  int64_t pack_reverse(int phase, float* buf);
  int64_t unpack_reverse(int phase, const float* buf);
  struct Stats {
    int64_t swaps = 0;          // non-self swaps with traffic
    int64_t sent = 0;           // forward entries sent
    int64_t relayed = 0;        // ... of them ghosts received in an earlier swap
    int64_t extra_rows = 0;     // rows of atoms outside this rank's graph
    int64_t zero_sends = 0;     // reverse copies that add nothing (repeat receptions)
    int64_t trash_forward = 0;  // forward duplicates written to trash rows
    int64_t trash_reverse = 0;  // reverse duplicates accumulated into trash rows
  };
  const Stats& stats() const { return st_; }
  const std::string& error() const { return err_; }

 private:
  ParallelStep& s_;
  // per swap: send rows (forward pack), recv rows (raw), forward unpack rows,
  // reverse pack rows, reverse unpack rows
  std::vector<int32_t> send_[kPhases], recv_[kPhases], fwd_dst_[kPhases], rev_src_[kPhases],
      rev_dst_[kPhases];
  std::vector<char> send_is_ghost_[kPhases];
  int32_t* d_[kPhases][4] = {};
  int64_t cap_[kPhases][4] = {};
  bool ready_ = false;
  Stats st_;
  std::string err_;
};

}  // namespace e3gnn_pair
