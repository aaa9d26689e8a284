// Row-partitioned Khatri-Rao contraction on the full grid (off-grid P1):
//   out[j] = sum_g c[g] prod_f U_f[j][g_f]
// i.e. K(X*, grid) c with K(X*, grid) = KhatriRaoMatrix(GridKernel.cov_kr(X*, xg))
// (gp_grief/kern/grid_kernel.py:148-179, tensors/khatri_rao_matrix.py:7-50,
// applied row by row by BlockMatrix.__mul__, block_matrix.py:48-66).
//
// The grid vector c is the C-order tensor over factors 0..d-1 (factor 0
// slowest).  View it as C[o][k], o the outer index over factors 0..d-2 and
// k = g_{d-1} the contiguous fastest axis.  Then
//   T[o][j] = sum_k C[o][k] U_{d-1}[j][k]        (a GEMM, 2 N M flop, FP64 MFMA)
//   out[j]  = sum_o T[o][j] prod_{f<d-1} U_f[j][g_f(o)]
// The first step is the MFMA GEMM of gg_dense.hip over chunks of outer rows;
// the second is an HBM-bound weighted column sum over T that walks o with an
// odometer (one table load per row, the slower factors' product cached until
// a carry), with the tables stored transposed (U_f^T: m_f x M) so that each
// row's loads are coalesced over the points j.  Partial sums over row splits
// are combined in a fixed order: results are bitwise reproducible.
#include <algorithm>
#include <climits>

#include "gg_internal.h"

namespace gg {

constexpr int kKrMaxD = 32;
constexpr int kKrThreads = 256;
constexpr int kKrMaxSplits = 256;

struct KrTabs {
  const double* ut[kKrMaxD];  // U_f^T, m_f x M row-major, f < nf
  int64_t m[kKrMaxD];
  int nf;                     // number of outer factors (d - 1)
};

__global__ __launch_bounds__(kKrThreads) void kr_colsum_kernel(
    const double* __restrict__ T, int64_t M, int64_t rows, int64_t row0, int64_t rps,
    KrTabs tabs, double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * kKrThreads + threadIdx.x;
  const int64_t o_beg = (int64_t)blockIdx.y * rps;
  const int64_t o_end = min(rows, o_beg + rps);
  if (j >= M) return;
  double acc = 0.0;
  const int nf = tabs.nf;
  if (nf == 0) {
    for (int64_t o = o_beg; o < o_end; ++o) acc += T[o * M + j];
  } else if (o_beg < o_end) {
    int64_t g[kKrMaxD];
    int64_t rem = row0 + o_beg;
    for (int f = nf - 1; f >= 0; --f) {
      g[f] = rem % tabs.m[f];
      rem /= tabs.m[f];
    }
    auto prefix = [&]() {
      double p = 1.0;
      for (int f = 0; f < nf - 1; ++f) p *= tabs.ut[f][g[f] * M + j];
      return p;
    };
    double pre = prefix();
    const double* __restrict__ ul = tabs.ut[nf - 1];
    const int64_t ml = tabs.m[nf - 1];
    int64_t gl = g[nf - 1];
    for (int64_t o = o_beg; o < o_end; ++o) {
      acc = fma(T[o * M + j], pre * ul[gl * M + j], acc);
      if (++gl == ml) {
        gl = 0;
        for (int f = nf - 2; f >= 0; --f) {
          if (++g[f] < tabs.m[f]) break;
          g[f] = 0;
        }
        pre = prefix();
      }
    }
  }
  part[(int64_t)blockIdx.y * M + j] = acc;
}

__global__ __launch_bounds__(kKrThreads) void kr_finish_kernel(const double* __restrict__ part,
                                                               int splits, int64_t M,
                                                               double* __restrict__ out,
                                                               int accumulate) {
  const int64_t j = (int64_t)blockIdx.x * kKrThreads + threadIdx.x;
  if (j >= M) return;
  double s = accumulate ? out[j] : 0.0;
  for (int k = 0; k < splits; ++k) s += part[(int64_t)k * M + j];
  out[j] = s;
}

// Running product of row-col Khatri-Rao factor blocks (get_rows,
// khatri_rao_matrix.py:117-140).  mode 0: P = X (first) or P *= X.
// mode 1 (logged): S *= sgn(X); L += log|X| with X -> 1 where the running
// sign S is 0 (the reference's rows_1d[sign == 0] = 1 rule).
__global__ __launch_bounds__(kKrThreads) void kr_hadamard_kernel(int64_t n,
                                                                 const double* __restrict__ X,
                                                                 double* __restrict__ P,
                                                                 double* __restrict__ S,
                                                                 int mode, int first) {
  for (int64_t e = (int64_t)blockIdx.x * kKrThreads + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kKrThreads) {
    const double x = X[e];
    if (mode == 0) {
      P[e] = first ? x : P[e] * x;
    } else {
      const double sx = (x > 0.0) ? 1.0 : ((x < 0.0) ? -1.0 : 0.0);
      const double s = (first ? 1.0 : S[e]) * sx;
      S[e] = s;
      const double v = (s == 0.0) ? 1.0 : x;
      P[e] = (first ? 0.0 : P[e]) + log(fabs(v));
    }
  }
}

static int kr_splits(int64_t M) {
  const int64_t bx = ceil_div(M, kKrThreads);
  return (int)std::max<int64_t>(1, std::min<int64_t>(kKrMaxSplits, ceil_div(4096, bx)));
}

}  // namespace gg

extern "C" {

int gg_kr_work_elems(int d, const int64_t* m, int64_t M, int64_t* min_elems) {
  return gg::guard([&] {
    GG_REQUIRE(d >= 1 && d <= gg::kKrMaxD && m && min_elems && M >= 0, GG_ERR_VALUE,
               "bad argument");
    int64_t outer = 1;
    for (int f = 0; f + 1 < d; ++f) outer *= m[f];
    *min_elems = (int64_t)gg::kr_splits(M) * M + std::min<int64_t>(outer, 1024) * M;
  });
}

int gg_kr_hadamard(int64_t n, const double* X_dev, double* P_dev, double* S_dev, int mode,
                   int first, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 0 && (mode == 0 || mode == 1), GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    GG_REQUIRE(X_dev && P_dev && (mode == 0 || S_dev), GG_ERR_VALUE, "NULL pointer");
    const unsigned nb = (unsigned)std::min<int64_t>(8192, gg::ceil_div(n, gg::kKrThreads));
    hipLaunchKernelGGL(gg::kr_hadamard_kernel, dim3(nb), dim3(gg::kKrThreads), 0,
                       gg::as_stream(stream), n, X_dev, P_dev, S_dev, mode, first);
    GG_LAUNCH_CHECK();
  });
}

int gg_kr_contract(int d, const int64_t* m, const double* c_dev, const double* ulast_dev,
                   const double* const* ut_dev, int64_t M, double* out_dev, double* work_dev,
                   int64_t work_elems, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(d >= 1 && d <= gg::kKrMaxD && m, GG_ERR_VALUE, "d must be in [1, 32]");
    GG_REQUIRE(M >= 0 && M <= INT_MAX, GG_ERR_VALUE, "bad number of points");
    if (M == 0) return;
    GG_REQUIRE(c_dev && ulast_dev && out_dev && work_dev, GG_ERR_VALUE, "NULL pointer");
    GG_REQUIRE(d == 1 || ut_dev, GG_ERR_VALUE, "NULL table array");
    gg::KrTabs tabs{};
    tabs.nf = d - 1;
    int64_t outer = 1;
    for (int f = 0; f < d; ++f) GG_REQUIRE(m[f] >= 1, GG_ERR_VALUE, "empty factor");
    for (int f = 0; f + 1 < d; ++f) {
      GG_REQUIRE(ut_dev[f], GG_ERR_VALUE, "NULL table");
      tabs.ut[f] = ut_dev[f];
      tabs.m[f] = m[f];
      outer *= m[f];
    }
    const int64_t mL = m[d - 1];
    GG_REQUIRE(mL <= INT_MAX, GG_ERR_VALUE, "fastest factor too large");
    const int S = gg::kr_splits(M);
    GG_REQUIRE(work_elems > (int64_t)S * M, GG_ERR_VALUE, "work too small (gg_kr_work_elems)");
    int64_t chunk = std::min<int64_t>(outer, (work_elems - (int64_t)S * M) / M);
    chunk = std::min<int64_t>(chunk, INT_MAX);
    GG_REQUIRE(chunk >= 1, GG_ERR_VALUE, "work too small (gg_kr_work_elems)");
    double* part = work_dev;
    double* T = work_dev + (int64_t)S * M;
    const hipStream_t st = gg::as_stream(stream);
    const unsigned bx = (unsigned)gg::ceil_div(M, gg::kKrThreads);
    for (int64_t o0 = 0; o0 < outer; o0 += chunk) {
      const int64_t rows = std::min(chunk, outer - o0);
      // T[rows x M] = C[o0 : o0 + rows][:] * U_{d-1}^T   (FP64 MFMA GEMM)
      const int rc = gg_gemm(0, 1, (int)rows, (int)M, (int)mL, 1.0, c_dev + o0 * mL, mL,
                             ulast_dev, mL, 0.0, T, M, 0, nullptr, 0, stream);
      if (rc != GG_OK) throw gg::Error(rc, "gg_kr_contract: GEMM failed");
      int splits = (int)std::min<int64_t>(S, rows);
      const int64_t rps = gg::ceil_div(rows, splits);
      splits = (int)gg::ceil_div(rows, rps);
      hipLaunchKernelGGL(gg::kr_colsum_kernel, dim3(bx, (unsigned)splits), dim3(gg::kKrThreads),
                         0, st, T, M, rows, o0, rps, tabs, part);
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::kr_finish_kernel, dim3(bx), dim3(gg::kKrThreads), 0, st, part,
                         splits, M, out_dev, (int)(o0 > 0));
      GG_LAUNCH_CHECK();
    }
  });
}

}  // extern "C"
