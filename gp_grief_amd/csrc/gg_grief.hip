// GRIEF eigenfunction matrix Phi on MI355X.
//
// Reference (gp_grief/kern/grief_kernel.py:68-111 with tensors/tensors.py:97-128):
//   Kux_f   = k_f(xg_f, x[:, dim_f])                              (m_f x n)
//   X_f     = (Q_f^T)[unique_f, :] . Kux_f                        (u_f x n)
//   sign    = prod_f sign(X_f)[inv_f]        (taken before zeros -> 1)
//   log     = sum_f log|X_f|[inv_f]
//   Phi     = sign^T * exp(log^T - 0.5 log_lam)                    (n x p)
// Two kernels:
//   grief_tables_kernel: a lane quad per data point computes the m_f kernel
//     values on the fly (never storing Kux) and contracts them with the u_f
//     selected eigenvector rows; writes log|X| and sign(X) as an n x U table
//     (U = sum_f u_f), i.e. exactly the reference's x_unique, per point.
//   grief_phi_kernel: HBM-bound writer of Phi (n x p row-major, or p x n):
//     one block owns 64 (32 transposed) data points (their table rows, as
//     signed values S exp(L), in LDS) and a 256-wide range of eigenfunctions
//     j (their table columns c_{j,f} in LDS); every Phi element is d LDS
//     loads and d multiplies, and the transposed tile is stored through LDS.
// Also the dense stationary covariance used for the grid factors K_f.
#include <cmath>
#include <vector>

#include "gg_internal.h"

namespace gg {

enum KernKind { kRBF = 0, kExponential = 1, kMatern32 = 2, kMatern52 = 3 };

// k(r^2) for the reference's 1-D stationary kernels (stationary.py:108-258)
__device__ __forceinline__ double stationary(int kind, double d2, double var, double ls) {
  switch (kind) {
    case kRBF:
      if (ls < 1e-6) return d2 == 0.0 ? var : 0.0;
      return var * exp(-0.5 * d2 / (ls * ls));
    case kExponential: {
      const double r = sqrt(d2) / ls;
      return var * exp(-r);
    }
    case kMatern32: {
      const double r = sqrt(d2) / ls;
      const double s3 = 1.7320508075688772;
      return var * (1.0 + s3 * r) * exp(-s3 * r);
    }
    default: {
      const double r2 = d2 / (ls * ls);
      const double r = sqrt(r2);
      const double s5 = 2.23606797749979;
      return var * (1.0 + s5 * r + (5.0 / 3) * r2) * exp(-s5 * r);
    }
  }
}

// out[i][j] (mode 0 = write, 1 = *=, 2 = +=) for x: N x D, z: M x D row-major
__global__ __launch_bounds__(256) void cov_kernel(int kind, double var, double ls, int D,
                                                  const double* __restrict__ x, int64_t N,
                                                  const double* __restrict__ z, int64_t M,
                                                  int mode, double* __restrict__ out) {
  const int64_t total = N * M;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / M, j = e - i * M;
    double d2 = 0.0;
    for (int k = 0; k < D; ++k) {
      const double t = x[i * D + k] - z[j * D + k];
      d2 = fma(t, t, d2);
    }
    const double v = stationary(kind, d2, var, ls);
    out[e] = mode == 0 ? v : (mode == 1 ? out[e] * v : out[e] + v);
  }
}

constexpr int kUG = 16;  // selected eigenvector rows per thread
constexpr int kTQ = 4;   // lanes per data point: each takes every kTQ-th grid point

// For dim f: X[u][a] = sum_k Qsel[u][k] * k_f(xg[k], x[a]) for u in a group of
// kUG rows; writes table L[a][col0+u] = log|X| (X == 0 -> 0), S = sign(X).
// A lane quad owns a data point: lane q evaluates the kernel at grid points
// k = q, q + 4, ... (m / 4 exps, independent chains), the quad's partial sums
// are combined by two xor-shuffles, and lane q stores the rows t = q mod 4.
// The group's Qsel rows (kUG x m) are staged in LDS once per block.
// kLds = false (m > 512): the rows are read from global memory instead.
template <bool kLds>
__global__ __launch_bounds__(256) void grief_tables_kernel(
    int kind, double var, double ls, const double* __restrict__ x, int64_t x_stride,
    int64_t n, const double* __restrict__ xg, int m, const double* __restrict__ Qsel, int u,
    double* __restrict__ Ltab, double* __restrict__ Stab, int U, int col0) {
  extern __shared__ double qlds[];   // kUG x m
  const int ug = blockIdx.y * kUG;
  const int nu = min(kUG, u - ug);
  if (kLds) {
    for (int e = threadIdx.x; e < kUG * m; e += blockDim.x) {
      const int t = e / m;
      qlds[e] = t < nu ? Qsel[(int64_t)(ug + t) * m + (e - t * m)] : 0.0;
    }
    __syncthreads();
  }
  // rows past u read row ug (any finite value: never stored)
  const double* qs = kLds ? qlds : Qsel + (int64_t)ug * m;
  const int tmax = kLds ? kUG : nu;
  const int64_t a = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kTQ;
  const int q = threadIdx.x % kTQ;
  const bool live = a < n;
  const double xa = live ? x[a * x_stride] : 0.0;
  double acc[kUG];
#pragma unroll
  for (int t = 0; t < kUG; ++t) acc[t] = 0.0;
  for (int k = q; k < m; k += kTQ) {
    const double d = xg[k] - xa;
    const double kv = stationary(kind, d * d, var, ls);
#pragma unroll
    for (int t = 0; t < kUG; ++t) acc[t] = fma(qs[(t < tmax ? t : 0) * m + k], kv, acc[t]);
  }
#pragma unroll
  for (int t = 0; t < kUG; ++t) {
    acc[t] += __shfl_xor(acc[t], 1, 64);
    acc[t] += __shfl_xor(acc[t], 2, 64);
  }
  if (!live) return;
#pragma unroll
  for (int t = 0; t < kUG; ++t) {
    if (t % kTQ == q && t < nu) {
      const double v = acc[t];
      const int64_t o = a * U + col0 + ug + t;
      Stab[o] = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0);
      Ltab[o] = log(fabs(v == 0.0 ? 1.0 : v));
    }
  }
}

constexpr int kPhiRows = 64;    // data points per block (row-major Phi)
constexpr int kPhiRowsT = 32;   // data points per block (transposed Phi)
constexpr int kPhiCols = 256;
constexpr int kMaxDim = 64;

// Phi[a][j] = prod_f S[a][c_jf] * exp(sum_f L[a][c_jf] - 0.5 log_lam[j])
//           = prod_f T[a][c_jf] * exp(-0.5 log_lam[j]),  T = S exp(L) = X
// cidx: p x d column index into the tables (c_jf = col0_f + inverse_f[j]).
// The block forms its kR x U slice of T once in LDS (kR U exps instead of
// kR kPhiCols), so each Phi element is d LDS loads and d multiplies: the
// kernel is bound by the Phi store.  Transposed (p x n): the kR x 256 tile
// goes through LDS so each eigenfunction row is stored as a kR-long run.
// kD > 0: d == kD known at compile time -- each thread keeps its d table
// columns in registers, so an element is d LDS loads + d multiplies (kD == 0:
// any d <= kMaxDim, indices re-read from LDS).  Row-major Phi is written with
// non-temporal stores (8 n p bytes stream past the caches).
template <int kR, bool kT, int kD>
__global__ __launch_bounds__(kPhiCols) void grief_phi_kernel(
    const double* __restrict__ Ltab, const double* __restrict__ Stab, int U, int64_t n,
    const int* __restrict__ cidx, int d, const double* __restrict__ log_lam, int p,
    double* __restrict__ Phi) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sT = sm;                                    // kR x U
  double* sO = sm + kR * U;                           // kT: kPhiCols x (kR + 1)
  int* sC = reinterpret_cast<int*>(sm + kR * U + (kT ? kPhiCols * (kR + 1) : 0));  // d x 256
  const int64_t a0 = (int64_t)blockIdx.x * kR;
  const int j0 = blockIdx.y * kPhiCols;
  const int j = j0 + threadIdx.x;
  const int rows = (int)min<int64_t>(kR, n - a0);
  for (int e = threadIdx.x; e < rows * U; e += blockDim.x)
    sT[e] = Stab[a0 * U + e] * exp(Ltab[a0 * U + e]);
  if (kD == 0 && j < p)
    for (int f = 0; f < d; ++f) sC[f * kPhiCols + threadIdx.x] = cidx[(int64_t)j * d + f];
  int creg[kD > 0 ? kD : 1];
  if (kD > 0) {
#pragma unroll
    for (int f = 0; f < kD; ++f) creg[f] = j < p ? cidx[(int64_t)j * kD + f] : 0;
  }
  __syncthreads();
  if (j < p) {
    const double sc = exp(-0.5 * log_lam[j]);
    for (int r = 0; r < rows; ++r) {
      double v = sc;
      const double* tr = sT + r * U;
      if (kD > 0) {
#pragma unroll
        for (int f = 0; f < kD; ++f) v *= tr[creg[f]];
      } else {
        for (int f = 0; f < d; ++f) v *= tr[sC[f * kPhiCols + threadIdx.x]];
      }
      if (kT)
        sO[threadIdx.x * (kR + 1) + r] = v;
      else
        __builtin_nontemporal_store(v, Phi + (a0 + r) * p + j);
    }
  }
  if (kT) {
    __syncthreads();
    const int cols = min(kPhiCols, p - j0);
    for (int e = threadIdx.x; e < cols * kR; e += blockDim.x) {
      const int jj = e / kR, r = e - jj * kR;
      if (r < rows) Phi[(int64_t)(j0 + jj) * n + a0 + r] = sO[jj * (kR + 1) + r];
    }
  }
}

template <int kR, bool kT, int kD>
static void launch_phi(dim3 grid, size_t lds, hipStream_t s, const double* L, const double* S,
                       int U, int64_t n, const int* cidx, int d, const double* ll, int p,
                       double* phi) {
  static bool attr = false;
  if (!attr) {
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&grief_phi_kernel<kR, kT, kD>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((grief_phi_kernel<kR, kT, kD>), grid, dim3(kPhiCols), lds, s, L, S, U, n,
                     cidx, d, ll, p, phi);
}

template <int kR, bool kT>
static void launch_phi_d(dim3 grid, size_t lds, hipStream_t s, const double* L, const double* S,
                         int U, int64_t n, const int* cidx, int d, const double* ll, int p,
                         double* phi) {
  switch (d) {
    case 1: launch_phi<kR, kT, 1>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 2: launch_phi<kR, kT, 2>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 3: launch_phi<kR, kT, 3>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 4: launch_phi<kR, kT, 4>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 5: launch_phi<kR, kT, 5>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 6: launch_phi<kR, kT, 6>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 7: launch_phi<kR, kT, 7>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    case 8: launch_phi<kR, kT, 8>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
    default: launch_phi<kR, kT, 0>(grid, lds, s, L, S, U, n, cidx, d, ll, p, phi); break;
  }
}

// expand_SKC (tensors.py:97-128) for caller-supplied unique rows: X holds the
// U selected rows x_unique_f = (K_f)[unique_f] . C_f of every factor stacked
// (U x n row-major), cidx the p x d row index c_jf = row0_f + inverse_f[j].
// logged: out = sum_f log|X[c_jf]| (zeros count as log 1), sign = prod_f
// sign(X[c_jf]) (taken before the zeros are replaced); else out = prod_f X.
// Lanes run over data points a: every load and store is a coalesced row run.
__global__ __launch_bounds__(256) void expand_skc_kernel(const double* __restrict__ X,
                                                         int64_t n,
                                                         const int* __restrict__ cidx, int d,
                                                         int p, int logged,
                                                         double* __restrict__ out,
                                                         int* __restrict__ sign) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (a >= n || j >= p) return;
  double acc = logged ? 0.0 : 1.0;
  int sg = 1;
  for (int f = 0; f < d; ++f) {
    const double v = X[(int64_t)cidx[(int64_t)j * d + f] * n + a];
    if (logged) {
      sg *= v > 0.0 ? 1 : (v < 0.0 ? -1 : 0);
      acc += log(fabs(v == 0.0 ? 1.0 : v));
    } else {
      acc *= v;
    }
  }
  out[(int64_t)j * n + a] = acc;
  if (logged) sign[(int64_t)j * n + a] = sg;
}

}  // namespace gg

extern "C" {

int gg_cov(int kind, double variance, double lengthscale, int dims, const double* x_dev,
           int64_t nx, const double* z_dev, int64_t nz, int mode, double* out_dev,
           gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(kind >= 0 && kind <= 3, GG_ERR_VALUE, "unknown kernel kind");
    GG_REQUIRE(mode >= 0 && mode <= 2, GG_ERR_VALUE, "bad mode");
    GG_REQUIRE(dims >= 1 && x_dev && z_dev && out_dev && nx >= 0 && nz >= 0, GG_ERR_VALUE,
               "bad argument");
    const int64_t total = nx * nz;
    if (total == 0) return;
    const int nb = (int)std::min<int64_t>(8192, gg::ceil_div(total, 256));
    hipLaunchKernelGGL(gg::cov_kernel, dim3(nb), dim3(256), 0, gg::as_stream(stream), kind,
                       variance, lengthscale, dims, x_dev, nx, z_dev, nz, mode, out_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_grief_tables(int kind, double variance, double lengthscale, const double* x_dev,
                    int64_t x_stride, int64_t n, const double* xg_dev, int m,
                    const double* qsel_dev, int u, double* ltab_dev, double* stab_dev, int U,
                    int col0, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(kind >= 0 && kind <= 3, GG_ERR_VALUE, "unknown kernel kind");
    GG_REQUIRE(x_dev && xg_dev && qsel_dev && ltab_dev && stab_dev, GG_ERR_VALUE, "NULL");
    GG_REQUIRE(m >= 1 && u >= 1 && col0 >= 0 && col0 + u <= U && n >= 0, GG_ERR_VALUE,
               "bad table geometry");
    if (n == 0) return;
    const bool in_lds = m <= 512;   // the kUG x m rows in at most 64 KiB of LDS
    const size_t lds = in_lds ? (size_t)gg::kUG * m * sizeof(double) : 0;
    dim3 grid((unsigned)gg::ceil_div(n * gg::kTQ, 256), (unsigned)gg::ceil_div(u, gg::kUG));
    hipLaunchKernelGGL(in_lds ? gg::grief_tables_kernel<true> : gg::grief_tables_kernel<false>,
                       grid, dim3(256), lds, gg::as_stream(stream),
                       kind, variance, lengthscale, x_dev, x_stride, n, xg_dev, m, qsel_dev, u,
                       ltab_dev, stab_dev, U, col0);
    GG_LAUNCH_CHECK();
  });
}

int gg_grief_phi(const double* ltab_dev, const double* stab_dev, int U, int64_t n,
                 const int* cidx_dev, int d, const double* log_lam_dev, int p, int transposed,
                 double* phi_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(ltab_dev && stab_dev && cidx_dev && log_lam_dev && phi_dev, GG_ERR_VALUE, "NULL");
    GG_REQUIRE(d >= 1 && d <= gg::kMaxDim && U >= 1 && p >= 1 && n >= 0, GG_ERR_VALUE,
               "bad Phi geometry");
    if (n == 0) return;
    const int kr = transposed ? gg::kPhiRowsT : gg::kPhiRows;
    const size_t lds = (size_t)kr * U * sizeof(double) +
                       (transposed ? (size_t)gg::kPhiCols * (kr + 1) * sizeof(double) : 0) +
                       (size_t)d * gg::kPhiCols * sizeof(int);
    GG_REQUIRE(lds <= 160 * 1024, GG_ERR_VALUE, "too many selected eigenvector rows");
    dim3 grid((unsigned)gg::ceil_div(n, kr), (unsigned)gg::ceil_div(p, gg::kPhiCols));
    if (transposed)
      gg::launch_phi_d<gg::kPhiRowsT, true>(grid, lds, gg::as_stream(stream), ltab_dev,
                                            stab_dev, U, n, cidx_dev, d, log_lam_dev, p, phi_dev);
    else
      gg::launch_phi_d<gg::kPhiRows, false>(grid, lds, gg::as_stream(stream), ltab_dev,
                                            stab_dev, U, n, cidx_dev, d, log_lam_dev, p, phi_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_expand_skc(const double* x_dev, int U, int64_t n, const int* cidx_dev, int d, int p,
                  int logged, double* out_dev, int* sign_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(x_dev && cidx_dev && out_dev && (!logged || sign_dev), GG_ERR_VALUE, "NULL");
    GG_REQUIRE(U >= 1 && d >= 1 && p >= 0 && n >= 0 && p < 65536, GG_ERR_VALUE,
               "bad expand_SKC geometry");
    if (n == 0 || p == 0) return;
    dim3 grid((unsigned)gg::ceil_div(n, 256), (unsigned)p);
    hipLaunchKernelGGL(gg::expand_skc_kernel, grid, dim3(256), 0, gg::as_stream(stream), x_dev,
                       n, cidx_dev, d, p, logged, out_dev, sign_dev);
    GG_LAUNCH_CHECK();
  });
}

}  // extern "C"
