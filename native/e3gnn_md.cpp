// e3gnn_md -- a native (C++, no Python) molecular-dynamics host over the C ABI
// of libe3gnn_hip.so: what LAMMPS' pair_style e3gnn does per step
// (pair_e3gnn.cpp:72-275: neighbour list -> model forward -> forces/virial)
// with the TorchScript module replaced by e3gnn_energy_forces and the host
// neighbour loops by the device list (e3gnn_nlist_*), driven by velocity
// Verlet.  It is the compiled, testable stand-in for the LAMMPS shim of
// SURVEY.md §8f row 3 (INTEGRATION.md §2 shows the same calls inside
// PairE3GNN::compute).
//
//   e3gnn_md <weights.bin> <manifest.json> <cells> <steps> <dt_fs> [T_K] [seed]
//
// System: n^3 conventional Si diamond cells (a = 5.43 A), velocities from a
// Maxwell-Boltzmann draw at T_K (default 300 K, zero net momentum, seed 0).
// Prints one JSON line per step: step, potential / kinetic / total energy (eV),
// edges, virial (eV, xx yy zz xy yz zx), and the device time of the step (ms).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "e3gnn.h"

namespace {

constexpr double MASS_SI = 28.0855;             // amu
constexpr double ACC = 9.648533212e-3;          // (eV/A)/amu -> A/fs^2
constexpr double KB = 8.617333262e-5;           // eV/K
constexpr double MV2_TO_EV = 1.0 / ACC;         // amu (A/fs)^2 -> eV

void die(const char* what) {
  std::fprintf(stderr, "e3gnn_md: %s: %s\n", what, e3gnn_last_error());
  std::exit(1);
}

#define HIPOK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "e3gnn_md: %s: %s\n", #x, hipGetErrorString(e_));  \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

// species index of `sym` in the manifest's chemical_symbols (the type map of
// pair_coeff * * model.pt Si ..., pair_e3gnn.cpp:330-360)
int species_index(const std::string& manifest, const std::string& sym) {
  std::ifstream f(manifest);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  const size_t k = s.find("\"chemical_symbols\"");
  if (k == std::string::npos) return -1;
  const size_t a = s.find('[', k), b = s.find(']', a);
  int idx = 0;
  for (size_t p = a; p < b;) {
    const size_t q0 = s.find('"', p);
    if (q0 == std::string::npos || q0 > b) break;
    const size_t q1 = s.find('"', q0 + 1);
    if (s.compare(q0 + 1, q1 - q0 - 1, sym) == 0) return idx;
    ++idx;
    p = q1 + 1;
  }
  return -1;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s weights.bin manifest.json cells steps dt_fs [T_K] [seed]\n",
                 argv[0]);
    return 2;
  }
  const int cells = std::atoi(argv[3]), steps = std::atoi(argv[4]);
  const double dt = std::atof(argv[5]);
  const double T0 = argc > 6 ? std::atof(argv[6]) : 300.0;
  const unsigned seed = argc > 7 ? (unsigned)std::atoi(argv[7]) : 0u;
  const int si = species_index(argv[2], "Si");
  if (si < 0) {
    std::fprintf(stderr, "e3gnn_md: Si not in the manifest\n");
    return 1;
  }

  e3gnn_model* model = e3gnn_load(argv[1], argv[2], 0);
  if (!model) die("e3gnn_load");
  int nspecies = 0, nlayers = 0, comm = 0;
  float cutoff = 0.f;
  if (e3gnn_model_info(model, &nspecies, &cutoff, &nlayers, &comm)) die("e3gnn_model_info");
  e3gnn_ctx* ctx = e3gnn_ctx_create(model);
  if (!ctx) die("e3gnn_ctx_create");
  e3gnn_nlist* nl = e3gnn_nlist_create(0);
  if (!nl) die("e3gnn_nlist_create");

  // Si diamond: fcc sites + (1/4,1/4,1/4) partners, basis innermost
  const double a0 = 5.43;
  const double basis[8][3] = {{0, 0, 0},       {0, .5, .5},     {.5, 0, .5},     {.5, .5, 0},
                              {.25, .25, .25}, {.25, .75, .75}, {.75, .25, .75}, {.75, .75, .25}};
  const int n = 8 * cells * cells * cells;
  std::vector<double> x(3 * n), v(3 * n), f(3 * n);
  int q = 0;
  for (int i = 0; i < cells; ++i)
    for (int j = 0; j < cells; ++j)
      for (int k = 0; k < cells; ++k)
        for (int b = 0; b < 8; ++b, ++q) {
          x[3 * q] = (i + basis[b][0]) * a0;
          x[3 * q + 1] = (j + basis[b][1]) * a0;
          x[3 * q + 2] = (k + basis[b][2]) * a0;
        }
  const double L = cells * a0;
  const double cell[9] = {L, 0, 0, 0, L, 0, 0, 0, L};
  const int pbc[3] = {1, 1, 1};
  std::mt19937 rng(seed);
  std::normal_distribution<double> gauss(0.0, std::sqrt(KB * T0 / MASS_SI * ACC));  // A/fs
  double pm[3] = {0, 0, 0};
  for (int i = 0; i < 3 * n; ++i) {
    v[i] = gauss(rng);
    pm[i % 3] += v[i];
  }
  for (int i = 0; i < 3 * n; ++i) v[i] -= pm[i % 3] / n;

  double* d_pos = nullptr;
  int32_t *d_type = nullptr, *d_c = nullptr, *d_nb = nullptr;
  float *d_vec = nullptr, *d_f = nullptr, *d_e = nullptr, *d_vir = nullptr;
  int64_t cap = 0;
  HIPOK(hipMalloc(&d_pos, 3 * n * sizeof(double)));
  HIPOK(hipMalloc(&d_type, n * sizeof(int32_t)));
  HIPOK(hipMalloc(&d_f, 3 * n * sizeof(float)));
  HIPOK(hipMalloc(&d_e, sizeof(float)));
  HIPOK(hipMalloc(&d_vir, 6 * sizeof(float)));
  std::vector<int32_t> types(n, si);
  HIPOK(hipMemcpy(d_type, types.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  hipStream_t s;
  HIPOK(hipStreamCreate(&s));
  hipEvent_t t0, t1;
  HIPOK(hipEventCreate(&t0));
  HIPOK(hipEventCreate(&t1));
  std::vector<float> hf(3 * n);
  float vir[6];

  auto compute = [&](double& epot, int64_t& E, float& ms) {
    HIPOK(hipMemcpyAsync(d_pos, x.data(), 3 * n * sizeof(double), hipMemcpyHostToDevice, s));
    HIPOK(hipEventRecord(t0, s));
    if (e3gnn_nlist_build(nl, n, d_pos, cell, pbc, cutoff, &E, s)) die("e3gnn_nlist_build");
    if (E > cap) {
      if (cap) {
        HIPOK(hipFree(d_c));
        HIPOK(hipFree(d_nb));
        HIPOK(hipFree(d_vec));
      }
      cap = E + E / 8 + 64;
      HIPOK(hipMalloc(&d_c, cap * sizeof(int32_t)));
      HIPOK(hipMalloc(&d_nb, cap * sizeof(int32_t)));
      HIPOK(hipMalloc(&d_vec, 3 * cap * sizeof(float)));
    }
    if (e3gnn_nlist_fetch(nl, d_c, d_nb, nullptr, d_vec, s)) die("e3gnn_nlist_fetch");
    if (e3gnn_energy_forces(ctx, n, E, d_type, d_c, d_nb, d_vec, d_e, nullptr, d_f, d_vir,
                            nullptr, s))
      die("e3gnn_energy_forces");
    HIPOK(hipEventRecord(t1, s));
    float e;
    HIPOK(hipMemcpyAsync(&e, d_e, sizeof(float), hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(hf.data(), d_f, 3 * n * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(vir, d_vir, 6 * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    HIPOK(hipEventElapsedTime(&ms, t0, t1));
    for (int i = 0; i < 3 * n; ++i) f[i] = hf[i];
    epot = e;
  };
  auto kinetic = [&]() {
    double k = 0;
    for (int i = 0; i < 3 * n; ++i) k += v[i] * v[i];
    return 0.5 * MASS_SI * k * MV2_TO_EV;
  };
  auto report = [&](int step, double epot, int64_t E, float ms) {
    const double ek = kinetic();
    std::printf("{\"step\": %d, \"n_atoms\": %d, \"edges\": %lld, \"epot\": %.8f, \"ekin\": %.8f, "
                "\"etot\": %.8f, \"virial\": [%.6f, %.6f, %.6f, %.6f, %.6f, %.6f], "
                "\"device_ms\": %.4f}\n",
                step, n, (long long)E, epot, ek, epot + ek, vir[0], vir[1], vir[2], vir[3],
                vir[4], vir[5], ms);
    std::fflush(stdout);
  };

  double epot;
  int64_t E;
  float ms;
  compute(epot, E, ms);
  report(0, epot, E, ms);
  const double c = ACC / MASS_SI;
  for (int st = 1; st <= steps; ++st) {
    for (int i = 0; i < 3 * n; ++i) {
      v[i] += 0.5 * dt * c * f[i];
      x[i] += dt * v[i];
    }
    compute(epot, E, ms);
    for (int i = 0; i < 3 * n; ++i) v[i] += 0.5 * dt * c * f[i];
    report(st, epot, E, ms);
  }
  e3gnn_nlist_free(nl);
  e3gnn_ctx_free(ctx);
  e3gnn_free(model);
  return 0;
}
