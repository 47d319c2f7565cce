/* ----------------------------------------------------------------------
   pair_style e3gnn/parallel on MI355X (see pair_e3gnn_parallel_hip.h).

   Reference: sevenn/pair_e3gnn/pair_e3gnn_parallel.cpp -- compute (:207-541),
   coeff (:560-690), init_style (:693-699), comm_preprocess (:703-748),
   pack_/unpack_forward_init (:750-801), pack_/unpack_{forward,reverse}_comm_gnn
   (:803-933).  The graph build, the per-layer segment calls and the force /
   virial / eatom scatter are e3gnn_pair::ParallelStep (native/pair_e3gnn_core.cpp);
   this file keeps the CommBrick side: the per-swap row index maps the
   reference builds in its "false" preprocessing forward_comm, and the packing
   of the rows into / out of the MPI buffers with the library's halo kernels
   (device buffers with GPU-aware MPI, host-staged otherwise).
------------------------------------------------------------------------- */

#include "pair_e3gnn_parallel.h"

#include "atom.h"
#include "comm.h"
#include "comm_brick.h"
#include "domain.h"
#include "error.h"
#include "force.h"
#include "memory.h"
#include "neigh_list.h"
#include "neighbor.h"

#include "e3gnn.h"
#include "pair_e3gnn_core.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <set>
#include <stdexcept>

using namespace LAMMPS_NS;

// the core's exchange = LAMMPS' patched brick communication
struct PairE3GNNParallel::Exchange : e3gnn_pair::ParallelStep::Exchange {
  PairE3GNNParallel *pair;
  CommBrick *brick;
  int forward(e3gnn_pair::ParallelStep &) override
  {
    brick->forward_comm(pair);
    return 0;
  }
  int reverse(e3gnn_pair::ParallelStep &) override
  {
    brick->reverse_comm(pair);
    return 0;
  }
};

PairE3GNNParallel::PairE3GNNParallel(LAMMPS *lmp) : Pair(lmp)
{
  single_enable = 0;
  restartinfo = 0;
  one_coeff = 1;
  manybody_flag = 1;
  world_rank = comm->me;
  int ngpu = 1;
  if (hipGetDeviceCount(&ngpu) != hipSuccess || ngpu < 1) ngpu = 1;
  device = comm->me % ngpu;   // pair_e3gnn_parallel.cpp:153-189
  const char *env = std::getenv("OFF_E3GNN_PARALLEL_CUDA_MPI");
  use_cuda_mpi = !(env && std::strcmp(env, "1") == 0) && std::getenv("E3GNN_GPU_AWARE_MPI");
  if (hipSetDevice(device) != hipSuccess) error->one(FLERR, "e3gnn/parallel: hipSetDevice failed");
}

PairE3GNNParallel::~PairE3GNNParallel()
{
  for (int p = 0; p < 6; p++)
    for (int32_t *q : {d_pack_fwd[p], d_unpack_fwd[p], d_unpack_rev[p]})
      if (q) (void) hipFree(q);
  if (d_stage) (void) hipFree(d_stage);
  if (allocated) {
    memory->destroy(setflag);
    memory->destroy(cutsq);
  }
}

int PairE3GNNParallel::get_x_dim() { return step && step->comm_dim() ? step->comm_dim() : comm_forward; }
bool PairE3GNNParallel::use_cuda_mpi_() { return use_cuda_mpi; }
bool PairE3GNNParallel::is_comm_preprocess_done() { return comm_preprocess_done; }

void PairE3GNNParallel::compute(int eflag, int vflag)
{
  ev_init(eflag, vflag);
  if (vflag_atom) error->all(FLERR, "atomic stress is not supported");
  if (atom->tag_consecutive() == 0) error->all(FLERR, "Pair e3gnn requires consecutive atom IDs");
  CommBrick *brick = dynamic_cast<CommBrick *>(comm);
  if (!brick)
    error->all(FLERR, "e3gnn/parallel: comm style should be brick & from modified code of comm_brick");

  const int ntotal = atom->nlocal + atom->nghost;
  tag64.resize(ntotal);
  for (int i = 0; i < ntotal; i++) tag64[i] = atom->tag[i];
  e3gnn_pair::NeighborView nv;
  nv.inum = list->inum;
  nv.ilist = list->ilist;
  nv.numneigh = list->numneigh;
  nv.firstneigh = list->firstneigh;
  nv.x = atom->x;
  nv.type = atom->type;
  nv.tag = tag64.data();
  nv.nlocal = atom->nlocal;
  nv.nghost = atom->nghost;
  nv.neighmask = NEIGHMASK;
  // graph: local rows in list order, ghosts within the cutoff deduplicated by tag
  if (step->build(nv, species, atom->natoms)) error->one(FLERR, "e3gnn/parallel: " + step->error());
  comm_preprocess();

  Exchange ex;
  ex.pair = this;
  ex.brick = brick;
  e3gnn_pair::PairOut out;
  if (step->compute(ex, atom->f, eflag_atom ? eatom : nullptr, out))
    error->one(FLERR, "e3gnn/parallel: " + step->error());
  eng_vdwl += out.energy;   // rank-local; LAMMPS sums over ranks
  if (vflag) for (int k = 0; k < 6; k++) virial[k] += out.virial[k];
  // ghost forces go to their owners with LAMMPS' reverse communication (newton on)
  comm_preprocess_done = false;
}

// ---------------------------------------------------------------- comm maps
void PairE3GNNParallel::comm_preprocess()
{
  for (int p = 0; p < 6; p++) {
    idx_pack_fwd[p].clear();
    idx_unpack_fwd[p].clear();
    idx_unpack_rev[p].clear();
  }
  comm_preprocess_done = false;
  // the "false" forward communication: CommBrick calls the *_init hooks per swap
  dynamic_cast<CommBrick *>(comm)->forward_comm(this);
  // reverse accumulation rows: a graph row sent more than once (to several
  // swaps) is accumulated once, the other copies go to the trash row (:712-733)
  std::set<int> already_met;
  const int G = step->graph_size(), trash = step->trash_row();
  for (int p = 0; p < 6; p++) {
    for (int32_t r : idx_pack_fwd[p]) {
      if (r < G) {
        if (already_met.count(r)) idx_unpack_rev[p].push_back(trash);
        else {
          idx_unpack_rev[p].push_back(r);
          already_met.insert(r);
        }
      } else {
        idx_unpack_rev[p].push_back(r);
      }
    }
    std::vector<int32_t> *h[3] = {&idx_pack_fwd[p], &idx_unpack_fwd[p], &idx_unpack_rev[p]};
    int32_t **d[3] = {&d_pack_fwd[p], &d_unpack_fwd[p], &d_unpack_rev[p]};
    for (int k = 0; k < 3; k++) {
      const int64_t n = (int64_t) h[k]->size();
      if (n > cap_idx[p][k]) {
        if (*d[k]) (void) hipFree(*d[k]);
        cap_idx[p][k] = n + n / 4 + 64;
        if (hipMalloc(d[k], cap_idx[p][k] * 4) != hipSuccess) error->one(FLERR, "e3gnn/parallel: hipMalloc");
      }
      if (n && hipMemcpy(*d[k], h[k]->data(), n * 4, hipMemcpyHostToDevice) != hipSuccess)
        error->one(FLERR, "e3gnn/parallel: hipMemcpy");
    }
  }
  comm_preprocess_done = true;
}

// rows of the atoms CommBrick sends in swap `comm_phase`: their graph rows, or
// an extra row for an atom this rank only relays (:750-779; the reference keys
// a new extra row by the loop counter, here by the atom index it stands for)
void PairE3GNNParallel::pack_forward_init(int n, int *list_send, int comm_phase)
{
  auto &idx = idx_pack_fwd[comm_phase];
  idx.reserve(n);
  for (int i = 0; i < n; i++) {
    const int a = list_send[i];
    int r = step->graph_row(a);
    if (r < 0) r = step->extra_row(a);
    idx.push_back(r);
  }
}

// rows of the ghost atoms [first, first + n) received in swap `comm_phase` (:781-801)
void PairE3GNNParallel::unpack_forward_init(int n, int first, int comm_phase)
{
  auto &idx = idx_unpack_fwd[comm_phase];
  idx.reserve(n);
  for (int i = first; i < first + n; i++) {
    int r = step->graph_row(i);
    if (r < 0) r = step->extra_row(i);
    idx.push_back(r);
  }
}

int PairE3GNNParallel::host_stage(int64_t floats)
{
  if (floats > stage_cap) {
    if (d_stage) (void) hipFree(d_stage);
    stage_cap = floats + floats / 4 + 1024;
    if (hipMalloc(&d_stage, stage_cap * 4) != hipSuccess) return 1;
  }
  return 0;
}

// pack rows `idx` of the comm rows into buf (device buffer with GPU-aware MPI,
// else through the device staging buffer to the host buffer)
static int pack_rows(e3gnn_pair::ParallelStep &s, const int32_t *d_idx, int64_t n, float *buf,
                     bool device_buf, float *stage)
{
  float *dst = device_buf ? buf : stage;
  if (s.pack(d_idx, n, dst)) return 1;
  if (!device_buf)
    return hipMemcpyAsync(buf, stage, n * s.comm_dim() * 4, hipMemcpyDeviceToHost,
                          (hipStream_t) s.stream()) != hipSuccess ||
        hipStreamSynchronize((hipStream_t) s.stream()) != hipSuccess;
  return hipStreamSynchronize((hipStream_t) s.stream()) != hipSuccess;
}

static int unpack_rows(e3gnn_pair::ParallelStep &s, const int32_t *d_idx, int64_t n, float *buf,
                       bool device_buf, float *stage, bool accumulate)
{
  const float *src = buf;
  if (!device_buf) {
    if (hipMemcpyAsync(stage, buf, n * s.comm_dim() * 4, hipMemcpyHostToDevice,
                       (hipStream_t) s.stream()) != hipSuccess)
      return 1;
    src = stage;
  }
  if (s.unpack(d_idx, n, src, accumulate)) return 1;
  return hipStreamSynchronize((hipStream_t) s.stream()) != hipSuccess;
}

int PairE3GNNParallel::pack_forward_comm_gnn(float *buf, int comm_phase)
{
  const int64_t n = (int64_t) idx_pack_fwd[comm_phase].size();
  if (!use_cuda_mpi && host_stage(n * step->comm_dim())) error->one(FLERR, "e3gnn/parallel: staging");
  if (n && pack_rows(*step, d_pack_fwd[comm_phase], n, buf, use_cuda_mpi, d_stage))
    error->one(FLERR, "e3gnn/parallel: pack_forward_comm_gnn: " + step->error());
  return (int) (n * step->comm_dim());
}

void PairE3GNNParallel::unpack_forward_comm_gnn(float *buf, int comm_phase)
{
  const int64_t n = (int64_t) idx_unpack_fwd[comm_phase].size();
  if (!use_cuda_mpi && host_stage(n * step->comm_dim())) error->one(FLERR, "e3gnn/parallel: staging");
  if (n && unpack_rows(*step, d_unpack_fwd[comm_phase], n, buf, use_cuda_mpi, d_stage, false))
    error->one(FLERR, "e3gnn/parallel: unpack_forward_comm_gnn: " + step->error());
}

int PairE3GNNParallel::pack_reverse_comm_gnn(float *buf, int comm_phase)
{
  // the rows received in the forward go back to the swap's sender (:873-900)
  const int64_t n = (int64_t) idx_unpack_fwd[comm_phase].size();
  if (!use_cuda_mpi && host_stage(n * step->comm_dim())) error->one(FLERR, "e3gnn/parallel: staging");
  if (n && pack_rows(*step, d_unpack_fwd[comm_phase], n, buf, use_cuda_mpi, d_stage))
    error->one(FLERR, "e3gnn/parallel: pack_reverse_comm_gnn: " + step->error());
  return (int) (n * step->comm_dim());
}

void PairE3GNNParallel::unpack_reverse_comm_gnn(float *buf, int comm_phase)
{
  // accumulated into the rows packed in the forward (duplicates: trash row), :902-933
  const int64_t n = (int64_t) idx_unpack_rev[comm_phase].size();
  if (!use_cuda_mpi && host_stage(n * step->comm_dim())) error->one(FLERR, "e3gnn/parallel: staging");
  if (n && unpack_rows(*step, d_unpack_rev[comm_phase], n, buf, use_cuda_mpi, d_stage, true))
    error->one(FLERR, "e3gnn/parallel: unpack_reverse_comm_gnn: " + step->error());
}

// ---------------------------------------------------------------- setup
void PairE3GNNParallel::allocate()
{
  allocated = 1;
  const int n = atom->ntypes;
  memory->create(setflag, n + 1, n + 1, "pair:setflag");
  memory->create(cutsq, n + 1, n + 1, "pair:cutsq");
}

void PairE3GNNParallel::settings(int narg, char ** /*arg*/)
{
  if (narg != 0) error->all(FLERR, "Illegal pair_style command");
}

// pair_coeff * * <n segments> <deployment dir> <element per type>: the
// reference reads one TorchScript file per segment (:578-608); one deployment
// directory holds every segment here (the segment API cuts at the same layer
// boundaries), so the count is accepted and not needed
void PairE3GNNParallel::coeff(int narg, char **arg)
{
  if (allocated) error->all(FLERR, "pair_e3gnn coeff called twice");
  allocate();
  if (narg < 4 || strcmp(arg[0], "*") != 0 || strcmp(arg[1], "*") != 0)
    error->all(FLERR, "e3gnn: first and second input of pair_coeff should be '*'");
  const int chem0 = 4;
  std::vector<std::string> elements;
  for (int i = chem0; i < narg; i++) elements.emplace_back(arg[i]);
  if (atom->ntypes > (int) elements.size())
    error->all(FLERR, "Not enough chemical specie is given. Check pair_coeff and types in your data/script");
  try {
    model.reset(new e3gnn_pair::Model(arg[3], device));
    species = model->type_map(elements);
    step.reset(new e3gnn_pair::ParallelStep(*model));
  } catch (const std::exception &e) {
    error->all(FLERR, std::string("e3gnn/parallel: ") + e.what());
  }
  cutoff = model->cutoff();
  // per-atom floats exchanged between layers: the buffers CommBrick sizes (:619-624)
  comm_forward = model->comm_size();
  comm_reverse = model->comm_size();
  for (int i = 1; i <= atom->ntypes; i++)
    for (int j = 1; j <= atom->ntypes; j++) {
      setflag[i][j] = 1;
      cutsq[i][j] = cutoff * cutoff;
    }
}

void PairE3GNNParallel::init_style()
{
  // full neighbour list & newton on (:693-699)
  if (force->newton_pair == 0) error->all(FLERR, "Pair style e3gnn/parallel requires newton pair on");
  neighbor->add_request(this, NeighConst::REQ_FULL);
}

double PairE3GNNParallel::init_one(int, int) { return cutoff; }

// ---------------------------------------------------------------- device buffers
DeviceBuffManager &DeviceBuffManager::getInstance()
{
  static DeviceBuffManager instance;
  return instance;
}

void DeviceBuffManager::get_buffer(int send_size, int recv_size, float *&send, float *&recv)
{
  if (send_size > send_cap) {
    if (send_dev) (void) hipFree(send_dev);
    send_cap = send_size;
    if (hipMalloc(&send_dev, (size_t) send_cap * sizeof(float)) != hipSuccess) send_dev = nullptr;
  }
  if (recv_size > recv_cap) {
    if (recv_dev) (void) hipFree(recv_dev);
    recv_cap = recv_size;
    if (hipMalloc(&recv_dev, (size_t) recv_cap * sizeof(float)) != hipSuccess) recv_dev = nullptr;
  }
  send = send_dev;
  recv = recv_dev;
}

DeviceBuffManager::~DeviceBuffManager()
{
  if (send_dev) (void) hipFree(send_dev);
  if (recv_dev) (void) hipFree(recv_dev);
}
