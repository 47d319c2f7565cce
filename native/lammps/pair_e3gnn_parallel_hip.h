/* -*- c++ -*- ----------------------------------------------------------
   pair_style e3gnn/parallel on MI355X: a drop-in for the reference's
   PairE3GNNParallel (sevenn/pair_e3gnn/pair_e3gnn_parallel.{h,cpp}) -- same
   class name and the same hooks, so the reference's patched CommBrick
   (sevenn/pair_e3gnn/comm_brick.cpp:1057-1120, installed by patch_lammps.sh)
   drives it unchanged -- with the per-segment TorchScript models replaced by the
   segment API of libe3gnn_hip.so through native/pair_e3gnn_core.  One deployment
   directory serves every segment:

     pair_style e3gnn/parallel
     pair_coeff * * <n segments (ignored)> <deployment dir> <element per type>

   Build: this header as src/pair_e3gnn_parallel.h (the name the CommBrick patch
   includes) with pair_e3gnn_parallel_hip.cpp, pair_e3gnn_core.{h,cpp},
   include/e3gnn.h; link libe3gnn_hip.so.
------------------------------------------------------------------------- */

#ifdef PAIR_CLASS
// clang-format off
PairStyle(e3gnn/parallel, PairE3GNNParallel)
// clang-format on
#else

#ifndef LMP_PAIR_E3GNN_PARALLEL
#define LMP_PAIR_E3GNN_PARALLEL

#include "pair.h"

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace e3gnn_pair {
class Model;
class ParallelStep;
class CommMaps;
}  // namespace e3gnn_pair

namespace LAMMPS_NS {

class PairE3GNNParallel : public Pair {
 public:
  PairE3GNNParallel(class LAMMPS *);
  ~PairE3GNNParallel() override;
  void compute(int, int) override;
  void settings(int, char **) override;
  void coeff(int, char **) override;
  void init_style() override;
  double init_one(int, int) override;
  void allocate();

  // the CommBrick hooks (comm_brick.cpp:1057-1120, pair_e3gnn_parallel.cpp:693-933)
  void pack_forward_init(int n, int *list, int comm_phase);
  void unpack_forward_init(int n, int first, int comm_phase);
  int pack_forward_comm_gnn(float *buf, int comm_phase);
  void unpack_forward_comm_gnn(float *buf, int comm_phase);
  int pack_reverse_comm_gnn(float *buf, int comm_phase);
  void unpack_reverse_comm_gnn(float *buf, int comm_phase);
  int get_x_dim();
  bool use_cuda_mpi_();
  bool is_comm_preprocess_done();

  // the per-swap row maps of the last compute (counters for tests and logs)
  const e3gnn_pair::CommMaps *comm_maps() const { return maps.get(); }
  bool print_info = false;
  int world_rank = 0;

 private:
  struct Exchange;
  void comm_preprocess();
  int host_stage(int64_t floats);
  double cutoff = 0.0;
  int device = 0;
  bool use_cuda_mpi = false;   // device buffers straight to MPI (GPU-aware MPI)
  bool comm_preprocess_done = false;
  std::unique_ptr<e3gnn_pair::Model> model;
  std::unique_ptr<e3gnn_pair::ParallelStep> step;
  std::vector<int> species;
  std::vector<int64_t> tag64;
  std::unique_ptr<e3gnn_pair::CommMaps> maps;   // per-swap row maps (comm_preprocess)
  int gnn_copy(int which, float *buf, int comm_phase);
  float *d_stage = nullptr;    // device staging when MPI takes host buffers
  int64_t stage_cap = 0;
};

// device send / receive buffers for GPU-aware MPI (comm_brick.cpp:1066, :1101)
class DeviceBuffManager {
 public:
  static DeviceBuffManager &getInstance();
  void get_buffer(int send_size, int recv_size, float *&send, float *&recv);
  ~DeviceBuffManager();

 private:
  DeviceBuffManager() {}
  DeviceBuffManager(const DeviceBuffManager &) = delete;
  DeviceBuffManager &operator=(const DeviceBuffManager &) = delete;
  float *send_dev = nullptr, *recv_dev = nullptr;
  int send_cap = 0, recv_cap = 0;
};

}  // namespace LAMMPS_NS

#endif
#endif
