// mini-LAMMPS test scaffold (see lmptype.h)
#pragma once
#include "lmptype.h"
#include "lammps.h"

namespace LAMMPS_NS {
class Pointers {
 public:
  explicit Pointers(LAMMPS *ptr)
      : lmp(ptr), memory(ptr->memory), error(ptr->error), atom(ptr->atom), neighbor(ptr->neighbor),
        comm(ptr->comm), domain(ptr->domain), force(ptr->force), screen(ptr->screen),
        logfile(ptr->logfile) {}
  virtual ~Pointers() = default;

 protected:
  LAMMPS *lmp;
  Memory *&memory;
  Error *&error;
  Atom *&atom;
  Neighbor *&neighbor;
  Comm *&comm;
  Domain *&domain;
  Force *&force;
  FILE *&screen;
  FILE *&logfile;
};
}  // namespace LAMMPS_NS
