// mini-LAMMPS test scaffold (see lmptype.h): CommBrick's swap tables and
// borders() for one brick sub-domain per emulated rank, plus the reference's
// patch (sevenn/pair_e3gnn/comm_brick.cpp:1057-1120, forward_comm /
// reverse_comm of a PairE3GNNParallel) and LAMMPS' own newton-on reverse
// communication of forces.  Ranks are threads of one process exchanging
// through World (a lock-step MPI_Sendrecv).
#pragma once
#include <condition_variable>
#include <mutex>
#include <vector>

#include "comm.h"

namespace LAMMPS_NS {
class PairE3GNNParallel;

class World {
 public:
  explicit World(int n) : nprocs(n), slots(n) {}
  const int nprocs;
  void barrier();
  void abort();   // wakes every waiting rank with an exception
  // every rank calls it in the same order: `sbytes` of `sbuf` go to `dest`,
  // what `src` sent to this rank lands in `rbuf` (capacity rcap); device
  // buffers are copied with hipMemcpy, host buffers with memcpy
  size_t sendrecv(int me, const void *sbuf, size_t sbytes, int dest, int src, void *rbuf,
                  size_t rcap, bool device);

 private:
  struct Slot {
    const void *ptr = nullptr;
    size_t bytes = 0;
    int dest = -1;
  };
  std::mutex m;
  std::condition_variable cv;
  int count = 0, gen = 0;
  bool aborted = false;
  std::vector<Slot> slots;
};

class CommBrick : public Comm {
 public:
  CommBrick(LAMMPS *lmp, World *world, int me, const int grid[3]);
  // comm_brick.cpp setup(): slabs and periodic shifts of the 2 swaps per
  // dimension for a ghost cutoff (lamda units for any cell)
  void setup(double cutghost_distance);
  // comm_brick.cpp borders(): ghosts of swap k = the slab atoms of the
  // sending rank among its owned atoms and the ghosts of earlier dimensions
  void borders();
  // the reference's patch, comm_brick.cpp:1057-1120
  void forward_comm(PairE3GNNParallel *pair);
  void reverse_comm(PairE3GNNParallel *pair);
  // Comm::reverse_comm(): ghost forces summed onto their owners (newton on)
  void reverse_comm();

  int nswap = 0;
  int maxsend = 0, maxrecv = 0, bufextra = 0;
  int sendproc[6] = {}, recvproc[6] = {}, sendnum[6] = {}, recvnum[6] = {}, firstrecv[6] = {};
  int pbc[6][3] = {};
  double slablo[6] = {}, slabhi[6] = {};
  std::vector<int> sendlist[6];
  double *buf_send = nullptr, *buf_recv = nullptr;

 private:
  void grow_buffers(size_t floats);
  World *world;
  double cutghost[3] = {0, 0, 0};
  std::vector<double> buf_send_s, buf_recv_s;
};
}  // namespace LAMMPS_NS
