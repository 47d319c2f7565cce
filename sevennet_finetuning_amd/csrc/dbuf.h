// Grow-only device buffer and host -> device upload, shared by the host
// translation units of libe3gnn_hip.so (api.cpp, generic.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

namespace e3gnn {

struct DBuf {
  void* p = nullptr;
  size_t cap = 0;
  DBuf() = default;
  DBuf(const DBuf&) = delete;  // owns device memory: never copied
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept : p(o.p), cap(o.cap) {
    o.p = nullptr;
    o.cap = 0;
  }
  DBuf& operator=(DBuf&& o) noexcept {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
    return *this;
  }
  ~DBuf() {
    if (p) {
      (void)hipDeviceSynchronize();   // (see ensure)
      (void)hipFree(p);
    }
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      // work still queued may read the old buffer (a stream-ordered
      // e3gnn_energy_forces returns before its kernels finish): drain the
      // device before freeing (growth only, so once per new maximum size)
      (void)hipDeviceSynchronize();
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t b = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&p, b);
    if (e == hipSuccess) cap = b;
    return e;
  }
  float* f() const { return (float*)p; }
  int* i() const { return (int*)p; }
};

inline hipError_t upload(DBuf& b, const std::vector<float>& v) {
  hipError_t e = b.ensure(v.size() * sizeof(float));
  if (e != hipSuccess) return e;
  return hipMemcpy(b.p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice);
}


}  // namespace e3gnn
