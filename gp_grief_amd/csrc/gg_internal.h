// Internal helpers shared by the gp_grief_amd HIP translation units.
// Not part of the C ABI (that is include/gp_grief_amd.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/gp_grief_amd.h"

namespace gg {

// Error carried from the implementation to the C ABI boundary, where it is
// turned into a status code and a thread-local message (gg_last_error).
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define GG_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      throw ::gg::Error(GG_ERR_RUNTIME, std::string("HIP error '") +              \
                                           hipGetErrorString(e_) + "' at " +     \
                                           __FILE__ + ":" + std::to_string(__LINE__) + \
                                           " in " #expr);                         \
  } while (0)

#define GG_REQUIRE(cond, code, msg)                 \
  do {                                              \
    if (!(cond)) throw ::gg::Error((code), (msg));  \
  } while (0)

// Run `body` and convert any exception into a GG status code.
template <class F>
int guard(F&& body) {
  try {
    body();
    return GG_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("host allocation failed");
    return GG_ERR_RUNTIME;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return GG_ERR_RUNTIME;
  }
}

inline hipStream_t as_stream(gg_stream s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-error check after a kernel launch (no synchronisation).
#define GG_LAUNCH_CHECK() GG_HIP(hipGetLastError())

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- device scalar block shared by the Krylov drivers (CG / Lanczos) ----
struct CgScalars {
  double rho;       // r.r of the current residual
  double rho_prev;  // r.r of the previous residual
  double pq;        // p.(A p)
  double alpha;
  double beta;
  double tol;       // stop when sqrt(rho) < tol
  double bnorm;
  int iters;        // completed iterations
  int done;         // 1 = converged / stopped: every kernel becomes a no-op
  int first;        // 1 = next p-update is p = r
  int pad;
};

// Fused CG direction update for the first mode product (gg_kron.hip).
struct CgPrologue {
  const double* r;
  const CgScalars* sc;
};

// Output address map of a mode product (see gg_kron.hip epilogue):
//   addr = (j / cg) * gs + (j % cg) + h * hs + a * as + br * cg,
//   a = row / mi, h = (row % mi) / cr, br = (row % mi) % cr.
struct OutMap {
  int identity;
  int64_t cg, gs, mi, cr, hs, as;
  static OutMap ident() { return OutMap{1, 1, 0, 1, 1, 0, 0}; }
};

// Reduction partial-buffer length used by grid-stride vector kernels.
constexpr int kVecBlocks = 2048;
constexpr int kVecThreads = 256;

// ---- vector kernels (gg_vec.hip) used by other translation units ----
void launch_dot_partials(const double* x, const double* y, int64_t n, double* partials,
                         int nblocks, hipStream_t s);
void launch_reduce_to(const double* partials, int64_t count, double* out, hipStream_t s);

}  // namespace gg
