// mini-LAMMPS test scaffold (see lmptype.h): one instance per emulated MPI rank
#pragma once
#include <cstdio>

namespace LAMMPS_NS {
class Memory;
class Error;
class Atom;
class Neighbor;
class Comm;
class Domain;
class Force;
class LAMMPS {
 public:
  Memory *memory = nullptr;
  Error *error = nullptr;
  Atom *atom = nullptr;
  Neighbor *neighbor = nullptr;
  Comm *comm = nullptr;
  Domain *domain = nullptr;
  Force *force = nullptr;
  FILE *screen = nullptr;
  FILE *logfile = nullptr;
};
}  // namespace LAMMPS_NS
