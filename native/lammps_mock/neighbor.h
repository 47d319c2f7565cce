// mini-LAMMPS test scaffold (see lmptype.h)
#pragma once
#include "lmptype.h"

namespace LAMMPS_NS {
namespace NeighConst {
  enum { REQ_DEFAULT = 0, REQ_FULL = 1 << 0 };
}
class Pair;
class NeighList;
class NeighRequest;
class Neighbor {
 public:
  double skin = 1.0;
  int requested_full = 0;
  NeighRequest *add_request(Pair *, int flags = 0)
  {
    requested_full = flags & NeighConst::REQ_FULL;
    return nullptr;
  }
  // scaffold: full list of the owned atoms over owned + ghost rows within
  // cutforce + skin; ilist reversed, special bits set on every other entry
  void build_full(class Atom *atom, double cutforce, NeighList *list);
};
}  // namespace LAMMPS_NS
