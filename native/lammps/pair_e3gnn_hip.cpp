/* ----------------------------------------------------------------------
   pair_style e3gnn on MI355X (see pair_e3gnn_hip.h).

   Reference: sevenn/pair_e3gnn/pair_e3gnn.cpp -- PairE3GNN::compute
   (:72-275: graph from the full neighbour list keyed by tag, model forward,
   forces / virial / eatom), ::coeff (:294-386: model load, element map),
   ::init_style (:389-398: full neighbour list).  The per-step work is
   e3gnn_pair::SerialStep::compute (native/pair_e3gnn_core.cpp); this file only
   maps LAMMPS' Atom / NeighList / accumulators onto it.
------------------------------------------------------------------------- */

#include "pair_e3gnn_hip.h"

#include "atom.h"
#include "comm.h"
#include "domain.h"
#include "error.h"
#include "force.h"
#include "memory.h"
#include "neigh_list.h"
#include "neighbor.h"

#include "pair_e3gnn_core.h"

#include <cstring>
#include <stdexcept>

using namespace LAMMPS_NS;

PairE3GNN::PairE3GNN(LAMMPS *lmp) : Pair(lmp)
{
  single_enable = 0;
  restartinfo = 0;
  one_coeff = 1;
  manybody_flag = 1;
  // the reference picks the GPU by rank (pair_e3gnn_parallel.cpp:153-189);
  // one rank per GPU here too
  device = comm->me;
}

PairE3GNN::~PairE3GNN()
{
  if (allocated) {
    memory->destroy(setflag);
    memory->destroy(cutsq);
  }
}

void PairE3GNN::compute(int eflag, int vflag)
{
  ev_init(eflag, vflag);
  if (vflag_atom) error->all(FLERR, "atomic stress is not supported");
  if (atom->tag_consecutive() == 0) error->all(FLERR, "Pair e3gnn requires consecutive atom IDs");

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

  e3gnn_pair::PairOut out;
  if (step->compute(nv, species, atom->f, eflag_atom ? eatom : nullptr, out))
    error->all(FLERR, "e3gnn: " + step->error());
  eng_vdwl += out.energy;
  if (vflag) for (int k = 0; k < 6; k++) virial[k] += out.virial[k];
}

void PairE3GNN::allocate()
{
  allocated = 1;
  const int n = atom->ntypes;
  memory->create(setflag, n + 1, n + 1, "pair:setflag");
  memory->create(cutsq, n + 1, n + 1, "pair:cutsq");
}

void PairE3GNN::settings(int narg, char ** /*arg*/)
{
  if (narg != 0) error->all(FLERR, "Illegal pair_style command");
}

// pair_coeff * * <deployment dir> <element of type 1> <element of type 2> ...
void PairE3GNN::coeff(int narg, char **arg)
{
  if (allocated) error->all(FLERR, "pair_e3gnn coeff called twice");
  allocate();
  if (narg < 3 || strcmp(arg[0], "*") != 0 || strcmp(arg[1], "*") != 0)
    error->all(FLERR, "e3gnn: first and second input of pair_coeff should be '*'");
  const int ntypes = atom->ntypes;
  if (ntypes > narg - 3)
    error->all(FLERR, "Not enough chemical specie is given. Check pair_coeff and types in your data/script");
  std::vector<std::string> elements;
  for (int i = 3; i < narg; i++) elements.emplace_back(arg[i]);
  try {
    model.reset(new e3gnn_pair::Model(arg[2], device));
    species = model->type_map(elements);
    step.reset(new e3gnn_pair::SerialStep(*model));
  } catch (const std::exception &e) {
    error->all(FLERR, std::string("e3gnn: ") + e.what());
  }
  cutoff = model->cutoff();
  for (int i = 1; i <= ntypes; i++)
    for (int j = 1; j <= ntypes; j++) {
      setflag[i][j] = 1;
      cutsq[i][j] = cutoff * cutoff;
    }
  if (lmp->logfile)
    for (int i = 3; i < narg; i++)
      fprintf(lmp->logfile, "Chemical specie '%s' is assigned to type %d\n", arg[i], i - 2);
}

void PairE3GNN::init_style()
{
  // full neighbour list (a many-body potential), pair_e3gnn.cpp:389-398
  neighbor->add_request(this, NeighConst::REQ_FULL);
}

double PairE3GNN::init_one(int, int) { return cutoff; }
