// mini-LAMMPS test scaffold (see lmptype.h): errors throw
#pragma once
#include <stdexcept>
#include <string>

namespace LAMMPS_NS {
class Error {
 public:
  [[noreturn]] void all(const std::string &file, int line, const std::string &msg)
  {
    throw std::runtime_error("ERROR (all) " + msg + " (" + file + ":" + std::to_string(line) + ")");
  }
  [[noreturn]] void one(const std::string &file, int line, const std::string &msg)
  {
    throw std::runtime_error("ERROR (one) " + msg + " (" + file + ":" + std::to_string(line) + ")");
  }
};
}  // namespace LAMMPS_NS
