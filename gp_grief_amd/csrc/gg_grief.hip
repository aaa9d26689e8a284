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
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "gg_internal.h"

namespace gg {

typedef double d4 __attribute__((ext_vector_type(4)));

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
      if (Stab == nullptr) {   // value table: X itself
        Ltab[o] = v;
        continue;
      }
      Stab[o] = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0);
      Ltab[o] = log(fabs(v == 0.0 ? 1.0 : v));
    }
  }
}

// MFMA form of the tables (round 3): X[u][a] = sum_k Qsel[u][k] k_f(xg[k], x[a])
// is a (u x m) . (m x n) product on v_mfma_f64_16x16x4_f64.  A wave owns 16
// data points at a time; per k-step its A operand is 16 Qsel rows (LDS, row
// stride m + 1: no bank conflicts) and its B operand the kernel values, each
// lane evaluating the one k(xg[4s + l / 16], x[a_l % 16]) it supplies -- K_ux
// never exists and the contraction costs one MFMA per 4 grid points instead of
// 16 LDS reads + FMAs per grid point per lane (grief_tables_kernel: 72 us per
// C2 factor, profiles/r03/y_c2_phi_trace.txt).  blockIdx.y: a group of 16
// selected rows.
// k(d) for the tables with the per-kernel constants hoisted (one multiply for
// the RBF exponent instead of a divide; r = |d| / l as |d| * (1 / l)): the same
// values as stationary() up to a few ulp of the exponent
template <int kKind>
__device__ __forceinline__ double stationary_fast(double d, double var, double c) {
  if (kKind == kRBF) return var * exp(c * (d * d));                 // c = -1 / (2 l^2)
  const double r = fabs(d) * c;                                      // c = 1 / l
  if (kKind == kExponential) return var * exp(-r);
  if (kKind == kMatern32) {
    const double s3 = 1.7320508075688772;
    return var * fma(s3, r, 1.0) * exp(-s3 * r);
  }
  const double s5 = 2.23606797749979;
  return var * fma(5.0 / 3.0 * r, r, fma(s5, r, 1.0)) * exp(-s5 * r);
}

// One factor's share of the batched tables launch (gg_grief_tables_all).
constexpr int kTabMaxF = 16;
struct TabFactor {
  int kind, m, u, col0, g0;   // g0: first blockIdx.y of this factor's row groups
  double var, c;
  const double* xg;
  const double* qsel;
  int64_t xoff;               // element offset of this dimension in x
};
struct TabBatch {
  int nf;
  TabFactor f[kTabMaxF];
};

template <int kKind>
__device__ __forceinline__ void tables_mfma_body(const TabFactor& F, int grp,
                                                 const double* __restrict__ x, int64_t x_stride,
                                                 int64_t n, double* __restrict__ Ltab,
                                                 double* __restrict__ Stab, int U, double* tl) {
  const int m = F.m, mp = (m + 15) & ~15, ld = mp + 1;
  double* qs = tl;              // 16 x ld
  double* xgs = tl + 16 * ld;   // mp
  const int ug = grp * 16, nu = min(16, F.u - ug);
  for (int e = threadIdx.x; e < 16 * mp; e += blockDim.x) {
    const int t = e / mp, k = e - t * mp;
    qs[t * ld + k] = (t < nu && k < m) ? F.qsel[(int64_t)(ug + t) * m + k] : 0.0;
  }
  // grid points past m: a finite kernel value times a zero Qsel column
  for (int k = threadIdx.x; k < mp; k += blockDim.x) xgs[k] = F.xg[min(k, m - 1)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t tiles = (n + 15) / 16;
  const double var = F.var, c = F.c;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < tiles; t += (int64_t)gridDim.x * 4) {
    const int64_t a = t * 16 + (lane & 15);
    const double xa = x[min(a, n - 1) * x_stride + F.xoff];
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    const double* qrow = qs + (lane & 15) * ld + (lane >> 4);
    const double* xk = xgs + (lane >> 4);
    // four k-steps per iteration: their kernel values are independent
    for (int s = 0; s < mp / 4; s += 4) {
      double kv[4], av[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kv[e] = stationary_fast<kKind>(xk[4 * (s + e)] - xa, var, c);
        av[e] = qrow[4 * (s + e)];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[e], kv[e], acc, 0, 0, 0);
    }
    // D[4 r + l / 16][l % 16]: selected row ug + 4 r + l / 16 of point a
    if (a < n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int uu = 4 * r + (lane >> 4);
        if (uu < nu) {
          const double v = acc[r];
          const int64_t o = a * U + F.col0 + ug + uu;
          if (Stab == nullptr) {   // value table: X itself (half the table bytes)
            Ltab[o] = v;
            continue;
          }
          Stab[o] = v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0);
          Ltab[o] = log(fabs(v == 0.0 ? 1.0 : v));
        }
      }
    }
  }
}

// blockIdx.y runs over every factor's 16-row groups (the factor found by its
// g0); the kernel kind is uniform per block
__global__ __launch_bounds__(256) void grief_tables_mfma_kernel(TabBatch B,
                                                                const double* __restrict__ x,
                                                                int64_t x_stride, int64_t n,
                                                                double* __restrict__ Ltab,
                                                                double* __restrict__ Stab, int U) {
  extern __shared__ double tl[];
  int f = 0;
  while (f + 1 < B.nf && (int)blockIdx.y >= B.f[f + 1].g0) ++f;
  const TabFactor& F = B.f[f];
  const int grp = (int)blockIdx.y - F.g0;
  switch (F.kind) {
    case kRBF: tables_mfma_body<kRBF>(F, grp, x, x_stride, n, Ltab, Stab, U, tl); break;
    case kExponential:
      tables_mfma_body<kExponential>(F, grp, x, x_stride, n, Ltab, Stab, U, tl);
      break;
    case kMatern32: tables_mfma_body<kMatern32>(F, grp, x, x_stride, n, Ltab, Stab, U, tl); break;
    default: tables_mfma_body<kMatern52>(F, grp, x, x_stride, n, Ltab, Stab, U, tl); break;
  }
}

// host: one launch of the batched MFMA tables for factors [0, nf) (nf <=
// kTabMaxF); false when a factor needs the generic kernel (delta RBF, m too
// large for the LDS staging)
static bool launch_tables_mfma(int nf, const int* kinds, const double* variances,
                               const double* lengthscales, const double* x_dev, int64_t x_stride,
                               const int64_t* xoffs, int64_t n, const double* const* xgs,
                               const int* ms, const double* const* qsels, const int* us,
                               double* ltab, double* stab, int U, const int* col0s,
                               hipStream_t s) {
  const char* tv = gg::knob("GG_GRIEF_TABLES");   // 0: the lane-quad kernel (A/B)
  if (tv && atoi(tv) == 0) return false;
  if (nf < 1 || nf > kTabMaxF) return false;
  TabBatch B;
  B.nf = nf;
  int g = 0, mmax = 1;
  for (int f = 0; f < nf; ++f) {
    if (kinds[f] == kRBF && lengthscales[f] < 1e-6) return false;
    const int mp = (ms[f] + 15) & ~15;
    if ((size_t)(16 * (mp + 1) + mp) * sizeof(double) > 64 * 1024) return false;
    mmax = std::max(mmax, mp);
    TabFactor& F = B.f[f];
    F.kind = kinds[f];
    F.m = ms[f];
    F.u = us[f];
    F.col0 = col0s[f];
    F.g0 = g;
    F.var = variances[f];
    F.c = kinds[f] == kRBF ? -0.5 / (lengthscales[f] * lengthscales[f]) : 1.0 / lengthscales[f];
    F.xg = xgs[f];
    F.qsel = qsels[f];
    F.xoff = xoffs[f];
    g += (int)ceil_div(us[f], 16);
  }
  const size_t lds = (size_t)(16 * (mmax + 1) + mmax) * sizeof(double);
  const int64_t tiles = ceil_div(n, (int64_t)16);
  dim3 grid((unsigned)std::min<int64_t>(ceil_div(tiles, (int64_t)4), 1024), (unsigned)g);
  hipLaunchKernelGGL(grief_tables_mfma_kernel, grid, dim3(256), lds, s, B, x_dev, x_stride, n,
                     ltab, stab, U);
  GG_LAUNCH_CHECK();
  return true;
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
    sT[e] = Stab ? Stab[a0 * U + e] * exp(Ltab[a0 * U + e]) : Ltab[a0 * U + e];
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

// Row-major Phi with column pairs (p even, 16-byte aligned Phi): one block
// owns kR data points and every column, so the kR x U slice of T is read and
// exponentiated once (not once per 256-column block), and a thread stores two
// adjacent columns as one 16-byte non-temporal store -- 1 KiB contiguous per
// wave instruction instead of 512 B of 8-byte lanes.  kD = d (1..8).
typedef double gg_d2 __attribute__((ext_vector_type(2)));
template <int kR, int kD>
__global__ __launch_bounds__(kPhiCols) void grief_phi_pair_kernel(
    const double* __restrict__ Ltab, const double* __restrict__ Stab, int U, int64_t n,
    const int* __restrict__ cidx, const double* __restrict__ log_lam, int p,
    double* __restrict__ Phi) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* sT = sm;   // kR x U
  const int64_t a0 = (int64_t)blockIdx.x * kR;
  const int rows = (int)min<int64_t>(kR, n - a0);
  for (int e = threadIdx.x; e < rows * U; e += blockDim.x)
    sT[e] = Stab ? Stab[a0 * U + e] * exp(Ltab[a0 * U + e]) : Ltab[a0 * U + e];
  __syncthreads();
  const int pairs = p >> 1;
  for (int jp = threadIdx.x; jp < pairs; jp += kPhiCols) {
    const int j = 2 * jp;
    int c0[kD], c1[kD];
#pragma unroll
    for (int f = 0; f < kD; ++f) {
      c0[f] = cidx[(int64_t)j * kD + f];
      c1[f] = cidx[(int64_t)(j + 1) * kD + f];
    }
    const double s0 = exp(-0.5 * log_lam[j]), s1 = exp(-0.5 * log_lam[j + 1]);
    double* out = Phi + a0 * p + j;
    for (int r = 0; r < rows; ++r) {
      const double* tr = sT + r * U;
      gg_d2 v = {s0, s1};
#pragma unroll
      for (int f = 0; f < kD; ++f) {
        v.x *= tr[c0[f]];
        v.y *= tr[c1[f]];
      }
      __builtin_nontemporal_store(v, reinterpret_cast<gg_d2*>(out + (int64_t)r * p));
    }
  }
}

template <int kR, int kD>
static void launch_phi_pair(dim3 grid, size_t lds, hipStream_t s, const double* L,
                            const double* S, int U, int64_t n, const int* cidx,
                            const double* ll, int p, double* phi) {
  static bool attr = false;
  if (!attr) {
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&grief_phi_pair_kernel<kR, kD>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((grief_phi_pair_kernel<kR, kD>), grid, dim3(kPhiCols), lds, s, L, S, U, n,
                     cidx, ll, p, phi);
}

// the pair kernel for d <= 8; false: not taken (the caller launches the other)
static bool launch_phi_pair_d(hipStream_t s, const double* L, const double* S, int U, int64_t n,
                              const int* cidx, int d, const double* ll, int p, double* phi) {
  static const bool on = [] {
    const char* e = gg::knob("GG_PHI_PAIR");   // A/B knob: 0 = the 256-column kernel
    return !(e != nullptr && atoi(e) == 0);
  }();
  if (!on || d > 8 || (p & 1) || (reinterpret_cast<uintptr_t>(phi) & 15)) return false;
  constexpr int kR = kPhiRows;
  const size_t lds = (size_t)kR * U * sizeof(double);
  if (lds > 160 * 1024) return false;
  const dim3 grid((unsigned)ceil_div(n, (int64_t)kR));
  switch (d) {
    case 1: launch_phi_pair<kR, 1>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 2: launch_phi_pair<kR, 2>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 3: launch_phi_pair<kR, 3>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 4: launch_phi_pair<kR, 4>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 5: launch_phi_pair<kR, 5>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 6: launch_phi_pair<kR, 6>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    case 7: launch_phi_pair<kR, 7>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
    default: launch_phi_pair<kR, 8>(grid, lds, s, L, S, U, n, cidx, ll, p, phi); break;
  }
  return true;
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
    GG_REQUIRE(x_dev && xg_dev && qsel_dev && ltab_dev, GG_ERR_VALUE, "NULL");
    GG_REQUIRE(m >= 1 && u >= 1 && col0 >= 0 && col0 + u <= U && n >= 0, GG_ERR_VALUE,
               "bad table geometry");
    if (n == 0) return;
    // MFMA contraction (default; GG_GRIEF_TABLES=0 selects the lane-quad kernel)
    // the MFMA contraction (default; GG_GRIEF_TABLES=0 selects the lane-quad kernel)
    const int64_t zero = 0;
    if (gg::launch_tables_mfma(1, &kind, &variance, &lengthscale, x_dev, x_stride, &zero, n,
                               &xg_dev, &m, &qsel_dev, &u, ltab_dev, stab_dev, U, &col0,
                               gg::as_stream(stream)))
      return;
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

int gg_grief_tables_all(int nf, const int* kinds, const double* variances,
                        const double* lengthscales, const double* x_dev, int64_t x_stride,
                        const int64_t* x_offsets, int64_t n, const double* const* xg_devs,
                        const int* ms, const double* const* qsel_devs, const int* us,
                        double* ltab_dev, double* stab_dev, int U, const int* col0s,
                        gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(nf >= 1 && kinds && variances && lengthscales && x_dev && x_offsets && xg_devs &&
                   ms && qsel_devs && us && ltab_dev && col0s && n >= 0,
               GG_ERR_VALUE, "bad argument");
    for (int f = 0; f < nf; ++f) {
      GG_REQUIRE(kinds[f] >= 0 && kinds[f] <= 3, GG_ERR_VALUE, "unknown kernel kind");
      GG_REQUIRE(xg_devs[f] && qsel_devs[f], GG_ERR_VALUE, "NULL");
      GG_REQUIRE(ms[f] >= 1 && us[f] >= 1 && col0s[f] >= 0 && col0s[f] + us[f] <= U &&
                     x_offsets[f] >= 0 && x_offsets[f] < x_stride,
                 GG_ERR_VALUE, "bad table geometry");
    }
    if (n == 0) return;
    hipStream_t s = gg::as_stream(stream);
    // batches of kTabMaxF factors in one launch each
    for (int f0 = 0; f0 < nf; f0 += gg::kTabMaxF) {
      const int c = std::min(gg::kTabMaxF, nf - f0);
      if (gg::launch_tables_mfma(c, kinds + f0, variances + f0, lengthscales + f0, x_dev,
                                 x_stride, x_offsets + f0, n, xg_devs + f0, ms + f0,
                                 qsel_devs + f0, us + f0, ltab_dev, stab_dev, U, col0s + f0, s))
        continue;
      for (int f = f0; f < f0 + c; ++f) {
        const int st = gg_grief_tables(kinds[f], variances[f], lengthscales[f],
                                       x_dev + x_offsets[f], x_stride, n, xg_devs[f], ms[f],
                                       qsel_devs[f], us[f], ltab_dev, stab_dev, U, col0s[f],
                                       stream);
        GG_REQUIRE(st == GG_OK, st, "gg_grief_tables_all: a factor's table failed");
      }
    }
  });
}

int gg_grief_phi(const double* ltab_dev, const double* stab_dev, int U, int64_t n,
                 const int* cidx_dev, int d, const double* log_lam_dev, int p, int transposed,
                 double* phi_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(ltab_dev && cidx_dev && log_lam_dev && phi_dev, GG_ERR_VALUE, "NULL");
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
    else if (!gg::launch_phi_pair_d(gg::as_stream(stream), ltab_dev, stab_dev, U, n, cidx_dev,
                                    d, log_lam_dev, p, phi_dev))
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
