// mini-LAMMPS test scaffold (NOT LAMMPS; see lmptype.h): the behaviour behind
// the mock headers -- cell, atoms, full neighbour list, Pair::ev_init and the
// brick communication.  CommBrick::setup / borders follow LAMMPS'
// comm_brick.cpp (single cutoff mode, every dimension periodic, one swap per
// direction and dimension: nswap = 6, what the reference's pair style allows);
// forward_comm / reverse_comm of a PairE3GNNParallel follow the reference's
// patch (sevenn/pair_e3gnn/comm_brick.cpp:1057-1120).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "atom.h"
#include "comm_brick.h"
#include "domain.h"
#include "error.h"
#include "neigh_list.h"
#include "neighbor.h"
#include "pair.h"
#include "pair_e3gnn_parallel.h"

namespace LAMMPS_NS {

// ------------------------------------------------------------------ Domain
void Domain::set_cell(const double cell[9])
{
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) h[r][c] = cell[3 * r + c];
  const double det = h[0][0] * (h[1][1] * h[2][2] - h[1][2] * h[2][1]) -
      h[0][1] * (h[1][0] * h[2][2] - h[1][2] * h[2][0]) + h[0][2] * (h[1][0] * h[2][1] - h[1][1] * h[2][0]);
  if (std::fabs(det) < 1e-12) throw std::runtime_error("singular cell");
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      const int r1 = (c + 1) % 3, r2 = (c + 2) % 3, c1 = (r + 1) % 3, c2 = (r + 2) % 3;
      hinv[r][c] = (h[r1][c1] * h[r2][c2] - h[r1][c2] * h[r2][c1]) / det;
    }
}

void Domain::x2lamda(const double *x, double *s) const
{
  for (int d = 0; d < 3; d++) s[d] = x[0] * hinv[0][d] + x[1] * hinv[1][d] + x[2] * hinv[2][d];
}

void Domain::lamda2x(const double *s, double *x) const
{
  for (int d = 0; d < 3; d++) x[d] = s[0] * h[0][d] + s[1] * h[1][d] + s[2] * h[2][d];
}

// ------------------------------------------------------------------ Atom
void Atom::add(const double *xi, const double *si, tagint t, int ty)
{
  for (int k = 0; k < 3; k++) {
    xs.push_back(xi[k]);
    lamda.push_back(si[k]);
    fs.push_back(0.0);
  }
  tags.push_back(t);
  types.push_back(ty);
}

void Atom::sync()
{
  const size_t n = tags.size();
  xp.resize(n);
  fp.resize(n);
  for (size_t i = 0; i < n; i++) {
    xp[i] = &xs[3 * i];
    fp[i] = &fs[3 * i];
  }
  x = xp.data();
  f = fp.data();
  type = types.data();
  tag = tags.data();
}

// ------------------------------------------------------------------ Neighbor
void Neighbor::build_full(Atom *atom, double cutforce, NeighList *list)
{
  const int nl = atom->nlocal, nt = atom->nlocal + atom->nghost;
  const double c2 = (cutforce + skin) * (cutforce + skin);
  list->inum = nl;
  list->ilist_s.resize(nl);
  list->numneigh_s.assign(nt, 0);
  list->neigh_s.assign(nt, {});
  for (int ii = 0; ii < nl; ii++) list->ilist_s[ii] = nl - 1 - ii;   // list order != index order
  for (int i = 0; i < nl; i++) {
    auto &nb = list->neigh_s[i];
    for (int j = 0; j < nt; j++) {
      if (j == i) continue;
      double r2 = 0;
      for (int k = 0; k < 3; k++) {
        const double d = atom->x[j][k] - atom->x[i][k];
        r2 += d * d;
      }
      if (r2 < c2) nb.push_back(nb.size() & 1 ? (j | (1 << 30)) : j);   // special bits
    }
    list->numneigh_s[i] = (int) nb.size();
  }
  list->first_s.resize(nt);
  for (int i = 0; i < nt; i++) list->first_s[i] = list->neigh_s[i].data();
  list->ilist = list->ilist_s.data();
  list->numneigh = list->numneigh_s.data();
  list->firstneigh = list->first_s.data();
}

// ------------------------------------------------------------------ Pair
void Pair::ev_init(int eflag, int vflag)
{
  eflag_global = eflag & 1;
  eflag_atom = eflag & 2;
  eflag_either = eflag_global || eflag_atom;
  vflag_global = vflag & 3;
  vflag_atom = vflag & 12;
  vflag_either = vflag_global || vflag_atom;
  eng_vdwl = eng_coul = 0.0;
  for (double &v : virial) v = 0.0;
  if (eflag_atom) {
    eatom_s.assign((size_t) atom->nlocal + atom->nghost, 0.0);
    eatom = eatom_s.data();
  }
}

// ------------------------------------------------------------------ World
void World::barrier()
{
  std::unique_lock<std::mutex> lk(m);
  if (aborted) throw std::runtime_error("world aborted");
  const int g = gen;
  if (++count == nprocs) {
    count = 0;
    ++gen;
    cv.notify_all();
  } else {
    cv.wait(lk, [&] { return gen != g || aborted; });
    if (aborted) throw std::runtime_error("world aborted");
  }
}

void World::abort()
{
  std::lock_guard<std::mutex> lk(m);
  aborted = true;
  cv.notify_all();
}

size_t World::sendrecv(int me, const void *sbuf, size_t sbytes, int dest, int src, void *rbuf,
                       size_t rcap, bool device)
{
  slots[me] = {sbuf, sbytes, dest};
  barrier();
  const Slot s = slots[src];
  if (s.dest != me) throw std::runtime_error("sendrecv: rank " + std::to_string(src) + " sends elsewhere");
  if (s.bytes > rcap) throw std::runtime_error("sendrecv: receive buffer too small");
  if (s.bytes) {
    if (device) {
      if (hipMemcpy(rbuf, s.ptr, s.bytes, hipMemcpyDeviceToDevice) != hipSuccess)
        throw std::runtime_error("sendrecv: hipMemcpy");
    } else {
      std::memcpy(rbuf, s.ptr, s.bytes);
    }
  }
  barrier();
  return s.bytes;
}

// ------------------------------------------------------------------ CommBrick
CommBrick::CommBrick(LAMMPS *lmp, World *w, int rank, const int grid[3]) : Comm(lmp), world(w)
{
  me = rank;
  nprocs = w->nprocs;
  for (int d = 0; d < 3; d++) procgrid[d] = grid[d];
  // LAMMPS' default rank order: x fastest
  myloc[0] = me % grid[0];
  myloc[1] = (me / grid[0]) % grid[1];
  myloc[2] = me / (grid[0] * grid[1]);
  for (int d = 0; d < 3; d++)
    for (int s = 0; s < 2; s++) {
      int loc[3] = {myloc[0], myloc[1], myloc[2]};
      loc[d] = (loc[d] + (s ? 1 : grid[d] - 1)) % grid[d];
      procneigh[d][s] = loc[0] + grid[0] * (loc[1] + grid[1] * loc[2]);
    }
}

void CommBrick::setup(double cut)
{
  // cutghost in lamda units = cut x |grad lamda_d| (comm.cpp get_comm_cutoff,
  // triclinic branch); maxneed = cutghost * procgrid / prd + 1 (prd = 1)
  for (int d = 0; d < 3; d++) {
    const double g = std::sqrt(domain->hinv[0][d] * domain->hinv[0][d] + domain->hinv[1][d] * domain->hinv[1][d] +
                               domain->hinv[2][d] * domain->hinv[2][d]);
    cutghost[d] = cut * g;
    const int maxneed = static_cast<int>(cutghost[d] * procgrid[d]) + 1;
    if (maxneed > 1)
      error->all(FLERR, "PairE3GNNParallel: Cell size is too small. Please use a single GPU or replicate the cell.");
  }
  nswap = 0;
  for (int d = 0; d < 3; d++) {
    const double sublo = (double) myloc[d] / procgrid[d], subhi = (double) (myloc[d] + 1) / procgrid[d];
    for (int ineed = 0; ineed < 2; ineed++, nswap++) {
      for (int k = 0; k < 3; k++) pbc[nswap][k] = 0;
      if (ineed % 2 == 0) {
        sendproc[nswap] = procneigh[d][0];
        recvproc[nswap] = procneigh[d][1];
        slablo[nswap] = -1e30;
        slabhi[nswap] = sublo + cutghost[d];
        if (myloc[d] == 0) pbc[nswap][d] = 1;
      } else {
        sendproc[nswap] = procneigh[d][1];
        recvproc[nswap] = procneigh[d][0];
        slablo[nswap] = subhi - cutghost[d];
        slabhi[nswap] = 1e30;
        if (myloc[d] == procgrid[d] - 1) pbc[nswap][d] = -1;
      }
    }
  }
}

namespace {
struct BorderRec {
  double x[3], s[3];
  tagint tag;
  int type;
};
}  // namespace

void CommBrick::borders()
{
  // drop the previous ghosts
  const int nl = atom->nlocal;
  atom->xs.resize(3 * (size_t) nl);
  atom->lamda.resize(3 * (size_t) nl);
  atom->fs.resize(3 * (size_t) nl);
  atom->tags.resize(nl);
  atom->types.resize(nl);
  atom->nghost = 0;
  int iswap = 0, nlast = 0;
  maxsend = maxrecv = 0;
  for (int dim = 0; dim < 3; dim++) {
    for (int ineed = 0; ineed < 2; ineed++, iswap++) {
      if (ineed % 2 == 0) nlast = atom->nlocal + atom->nghost;
      // owned atoms and ghosts of earlier dimensions inside the slab
      auto &sl = sendlist[iswap];
      sl.clear();
      for (int i = 0; i < nlast; i++) {
        const double s = atom->lamda[3 * i + dim];
        if (s >= slablo[iswap] && s <= slabhi[iswap]) sl.push_back(i);
      }
      sendnum[iswap] = (int) sl.size();
      std::vector<BorderRec> out(sl.size());
      for (size_t k = 0; k < sl.size(); k++) {
        const int i = sl[k];
        double sh[3];
        for (int d = 0; d < 3; d++) {
          out[k].s[d] = atom->lamda[3 * i + d] + pbc[iswap][d];
          sh[d] = pbc[iswap][d];
        }
        double dx[3];
        domain->lamda2x(sh, dx);
        for (int d = 0; d < 3; d++) out[k].x[d] = atom->xs[3 * i + d] + dx[d];
        out[k].tag = atom->tags[i];
        out[k].type = atom->types[i];
      }
      std::vector<BorderRec> in;
      if (sendproc[iswap] == me) {
        in = out;
      } else {
        int64_t ns = (int64_t) out.size(), nr = 0;
        world->sendrecv(me, &ns, sizeof(ns), sendproc[iswap], recvproc[iswap], &nr, sizeof(nr), false);
        in.resize(nr);
        world->sendrecv(me, out.data(), out.size() * sizeof(BorderRec), sendproc[iswap], recvproc[iswap],
                        in.data(), in.size() * sizeof(BorderRec), false);
      }
      firstrecv[iswap] = atom->nlocal + atom->nghost;
      recvnum[iswap] = (int) in.size();
      for (const auto &r : in) atom->add(r.x, r.s, r.tag, r.type);
      atom->nghost += (int) in.size();
      maxsend = std::max(maxsend, sendnum[iswap]);
      maxrecv = std::max(maxrecv, recvnum[iswap]);
    }
  }
  atom->sync();
}

void CommBrick::grow_buffers(size_t floats)
{
  const size_t doubles = (floats + 1) / 2 + 1;
  if (buf_send_s.size() < doubles) buf_send_s.resize(doubles);
  if (buf_recv_s.size() < doubles) buf_recv_s.resize(doubles);
  buf_send = buf_send_s.data();
  buf_recv = buf_recv_s.data();
}

// the reference's CommBrick::forward_comm(PairE3GNNParallel *), comm_brick.cpp:1057-1090
void CommBrick::forward_comm(PairE3GNNParallel *pair)
{
  const bool comm_preprocess_done = pair->is_comm_preprocess_done();
  const int nsize = pair->get_x_dim();
  float *buf_send_, *buf_recv_;
  const bool dev = pair->use_cuda_mpi_();
  if (dev) {
    const int m = (std::max(maxsend, maxrecv) + bufextra) * nsize;
    DeviceBuffManager::getInstance().get_buffer(m, m, buf_send_, buf_recv_);
  } else {
    grow_buffers((size_t) std::max(maxsend + bufextra, maxrecv) * nsize);
    buf_send_ = reinterpret_cast<float *>(buf_send);
    buf_recv_ = reinterpret_cast<float *>(buf_recv);
  }
  if (nswap > 6) error->all(FLERR, "PairE3GNNParallel: Cell size is too small. Please use a single GPU or replicate the cell.");
  for (int iswap = 0; iswap < nswap; iswap++) {
    // every rank reaches this test alike: a dimension with one rank is a
    // self swap everywhere, skipped (the ghosts of a self swap share rows by tag)
    if (sendproc[iswap] == me) continue;
    if (!comm_preprocess_done) {
      pair->pack_forward_init(sendnum[iswap], sendlist[iswap].data(), iswap);
      pair->unpack_forward_init(recvnum[iswap], firstrecv[iswap], iswap);
    } else {
      const int n = pair->pack_forward_comm_gnn(buf_send_, iswap);
      world->sendrecv(me, buf_send_, (size_t) n * sizeof(float), sendproc[iswap], recvproc[iswap], buf_recv_,
                      (size_t) nsize * recvnum[iswap] * sizeof(float), dev);
      pair->unpack_forward_comm_gnn(buf_recv_, iswap);
    }
  }
}

// the reference's CommBrick::reverse_comm(PairE3GNNParallel *), comm_brick.cpp:1092-1120
void CommBrick::reverse_comm(PairE3GNNParallel *pair)
{
  const int nsize = pair->get_x_dim();
  float *buf_send_, *buf_recv_;
  const bool dev = pair->use_cuda_mpi_();
  if (dev) {
    // the reverse sends recvnum rows and receives sendnum rows
    const int m = (std::max(maxsend, maxrecv) + bufextra) * nsize;
    DeviceBuffManager::getInstance().get_buffer(m, m, buf_send_, buf_recv_);
  } else {
    grow_buffers((size_t) std::max(maxsend + bufextra, maxrecv) * nsize);
    buf_send_ = reinterpret_cast<float *>(buf_send);
    buf_recv_ = reinterpret_cast<float *>(buf_recv);
  }
  for (int iswap = nswap - 1; iswap >= 0; iswap--) {
    if (sendproc[iswap] == me) continue;
    const int n = pair->pack_reverse_comm_gnn(buf_send_, iswap);
    world->sendrecv(me, buf_send_, (size_t) n * sizeof(float), recvproc[iswap], sendproc[iswap], buf_recv_,
                    (size_t) nsize * sendnum[iswap] * sizeof(float), dev);
    pair->unpack_reverse_comm_gnn(buf_recv_, iswap);
  }
}

// Comm::reverse_comm() for forces, newton on: swaps in reverse order, the
// ghosts received in swap k add their force to the atoms sent in swap k
void CommBrick::reverse_comm()
{
  double **f = atom->f;
  for (int iswap = nswap - 1; iswap >= 0; iswap--) {
    const int nr = recvnum[iswap], ns = sendnum[iswap];
    std::vector<double> out(3 * (size_t) nr), in(3 * (size_t) ns);
    for (int k = 0; k < nr; k++)
      for (int d = 0; d < 3; d++) out[3 * k + d] = f[firstrecv[iswap] + k][d];
    if (sendproc[iswap] == me) {
      in = out;
    } else {
      world->sendrecv(me, out.data(), out.size() * sizeof(double), recvproc[iswap], sendproc[iswap], in.data(),
                      in.size() * sizeof(double), false);
    }
    for (int k = 0; k < ns; k++)
      for (int d = 0; d < 3; d++) f[sendlist[iswap][k]][d] += in[3 * k + d];
  }
}

}  // namespace LAMMPS_NS
