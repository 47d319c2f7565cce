// mini-LAMMPS test scaffold (see lmptype.h)
#pragma once
#include <cstdlib>

namespace LAMMPS_NS {
class Memory {
 public:
  template <typename T> T **create(T **&array, int n1, int n2, const char *)
  {
    T *data = static_cast<T *>(std::calloc((size_t) n1 * n2, sizeof(T)));
    array = static_cast<T **>(std::malloc(sizeof(T *) * n1));
    for (int i = 0; i < n1; i++) array[i] = data + (size_t) i * n2;
    return array;
  }
  template <typename T> void destroy(T **&array)
  {
    if (!array) return;
    std::free(array[0]);
    std::free(array);
    array = nullptr;
  }
};
}  // namespace LAMMPS_NS
