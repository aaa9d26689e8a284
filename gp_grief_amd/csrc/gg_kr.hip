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
//
// For d <= 8 the two steps are fused (kr_stream_kernel): each wave streams 16
// outer rows of C from HBM against up to 128 points whose U rows are staged in
// LDS, and weights + sums its MFMA tile in the epilogue, so T never reaches
// HBM (C is read once per 128-point column pass).  The outer digits of a row
// are its block's base digits plus the row offset (< 16) carried through the
// (compile-time many) outer factors.
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

typedef double kd4 __attribute__((ext_vector_type(4)));
constexpr int kSK = 16;          // k-chunk depth staged per barrier
constexpr int kSMaxWG = 2048;    // workgroups per launch (partials per column pass)

// Streaming fused contraction.  Each wave owns 16 consecutive outer rows o
// and NT 16-column MFMA tiles (NT*16 <= 128 points of one column pass); C rows are
// streamed straight from HBM -- lane l reads the 4 contiguous doubles
// C[o0 + (l & 15)][k0 + 4 (l >> 4) + t], t = 0..3, so a row's 128-byte chunk
// is one coalesced segment -- and MFMA step t pairs them with the B fragment
// U[col][k0 + 4 (l >> 4) + t] from the LDS-staged U chunk (any assignment of
// k to MFMA steps is valid as long as A and B agree).  U (M x K) is staged 16
// k at a time, double-buffered, one barrier per chunk, shared by the 4 waves.
// The epilogue weights each row by prod_{f<NF} U_f[col][g_f(o)] and adds it
// into per-lane column sums kept across the wave's row blocks; C is read once
// per column pass and T never exists.
template <int NF, int NT>
__global__ __launch_bounds__(kKrThreads, 2) void kr_stream_kernel(
    int64_t O, int M, int K, const double* __restrict__ C, const double* __restrict__ U,
    KrTabs tabs, double* __restrict__ part) {
  constexpr int W = NT * 16;               // columns per pass
  constexpr int LDW = W + 4;               // LDS row stride (doubles)
  constexpr int kStage = (W * kSK + kKrThreads - 1) / kKrThreads;
  __shared__ __attribute__((aligned(16))) double sU[2][kSK * LDW];
  __shared__ double red[4][W];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.x * W;           // first point of this column pass
  const int kq = lane >> 4, li = lane & 15;
  const int64_t nblocks = (O + 15) / 16;   // 16-row blocks
  const int64_t groups = (nblocks + 3) / 4;
  const int nk = (K + kSK - 1) / kSK;

  double colsum[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) colsum[t] = 0.0;
  double ru[kStage];
  auto load_u = [&](int k0) {
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const int e = tid + u * kKrThreads;       // e = col * kSK + kk
      const int col = e / kSK, kk = e % kSK;
      const int gc = c0 + col, gk = k0 + kk;
      ru[u] = (e < W * kSK && gc < M && gk < K) ? U[(int64_t)gc * K + gk] : 0.0;
    }
  };
  auto store_u = [&](int buf) {
#pragma unroll
    for (int u = 0; u < kStage; ++u) {
      const int e = tid + u * kKrThreads;
      if (e < W * kSK) sU[buf][(e % kSK) * LDW + e / kSK] = ru[u];
    }
  };

#pragma unroll 1
  for (int64_t grp = blockIdx.y; grp < groups; grp += gridDim.y) {
    const int64_t blk = grp * 4 + wave;
    const int64_t o0 = blk * 16;
    const int64_t myrow = o0 + li;
    const bool rowok = blk < nblocks && myrow < O;
    const double* __restrict__ crow = C + (rowok ? myrow : 0) * (int64_t)K;
    double ca[4], cn[4];
    auto load_c = [&](int k0, double* dst) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int gk = k0 + 4 * kq + t;
        dst[t] = (rowok && gk < K) ? crow[gk] : 0.0;
      }
    };
    kd4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = kd4{0.0, 0.0, 0.0, 0.0};
    load_u(0);
    store_u(0);
    load_c(0, ca);
    __syncthreads();
#pragma unroll 1
    for (int c = 0; c < nk; ++c) {
      const bool more = c + 1 < nk;
      if (more) {
        load_u((c + 1) * kSK);
        load_c((c + 1) * kSK, cn);
      }
      const double* b_s = sU[c & 1];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double* brow = b_s + (4 * kq + t) * LDW + li;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[t], brow[16 * j], acc[j], 0, 0, 0);
      }
      if (more) {
        store_u((c + 1) & 1);
#pragma unroll
        for (int t = 0; t < 4; ++t) ca[t] = cn[t];
      }
      __syncthreads();
    }

    // epilogue: lane holds T[o0 + kq + 4 r][c0 + 16 j + li]
    if (blk < nblocks) {
      int base[NF > 0 ? NF : 1];
      {
        int64_t rem = o0;
#pragma unroll
        for (int f = NF - 1; f >= 0; --f) {
          base[f] = (int)(rem % tabs.m[f]);
          rem /= tabs.m[f];
        }
      }
#pragma unroll 1
      for (int r = 0; r < 4; ++r) {
        const int dlt = kq + 4 * r;
        if (o0 + dlt >= O) continue;
        int gd[NF > 0 ? NF : 1];
#pragma unroll
        for (int f = 0; f < NF; ++f) gd[f] = base[f];
        if constexpr (NF > 0) {
          gd[NF - 1] += dlt;
#pragma unroll
          for (int f = NF - 1; f >= 1; --f) {
            const int mf = (int)tabs.m[f];
            while (gd[f] >= mf) {
              gd[f] -= mf;
              ++gd[f - 1];
            }
          }
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int col = c0 + 16 * j + li;
          if (col >= M) continue;
          double w = 1.0;
#pragma unroll
          for (int f = 0; f < NF; ++f) w *= tabs.ut[f][(int64_t)gd[f] * M + col];
          const double tv = r == 0 ? acc[j][0] : (r == 1 ? acc[j][1] : (r == 2 ? acc[j][2] : acc[j][3]));
          colsum[j] = fma(tv, w, colsum[j]);
        }
      }
    }
  }

  // reduce over the 4 row groups of each wave, then over the 4 waves
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    colsum[j] += __shfl_xor(colsum[j], 16);
    colsum[j] += __shfl_xor(colsum[j], 32);
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < NT; ++j) red[wave][16 * j + lane] = colsum[j];
  }
  __syncthreads();
  for (int col = tid; col < W; col += kKrThreads) {
    const int gc = c0 + col;
    if (gc < M)
      part[(int64_t)blockIdx.y * M + gc] = ((red[0][col] + red[1][col]) + red[2][col]) + red[3][col];
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
    *min_elems = std::max<int64_t>((int64_t)gg::kr_splits(M) * M + std::min<int64_t>(outer, 1024) * M,
                                   (int64_t)gg::kSMaxWG * M);
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
    const hipStream_t st0 = gg::as_stream(stream);
    if (d - 1 <= 7) {
      // streaming fused contraction: T never reaches HBM
      const int nt = M <= 16 ? 1 : (M <= 64 ? 4 : 8);
      const int64_t groups = gg::ceil_div(gg::ceil_div(outer, (int64_t)16), (int64_t)4);
      const unsigned gx = (unsigned)gg::ceil_div(M, (int64_t)16 * nt);
      const int64_t gy = std::max<int64_t>(
          1, std::min<int64_t>(groups, std::max<int64_t>(1, gg::kSMaxWG / gx)));
      GG_REQUIRE(work_elems >= gy * M, GG_ERR_VALUE, "work too small (gg_kr_work_elems)");
      const dim3 grid(gx, (unsigned)gy);
#define GG_KR_STREAM(NF_, NT_)                                                                \
  hipLaunchKernelGGL((gg::kr_stream_kernel<NF_, NT_>), grid, dim3(gg::kKrThreads), 0, st0,     \
                     outer, (int)M, (int)mL, c_dev, ulast_dev, tabs, work_dev)
#define GG_KR_NF(NT_)                         \
  switch (d - 1) {                            \
    case 0: GG_KR_STREAM(0, NT_); break;      \
    case 1: GG_KR_STREAM(1, NT_); break;      \
    case 2: GG_KR_STREAM(2, NT_); break;      \
    case 3: GG_KR_STREAM(3, NT_); break;      \
    case 4: GG_KR_STREAM(4, NT_); break;      \
    case 5: GG_KR_STREAM(5, NT_); break;      \
    case 6: GG_KR_STREAM(6, NT_); break;      \
    default: GG_KR_STREAM(7, NT_); break;     \
  }
      if (nt == 1) { GG_KR_NF(1) }
      else if (nt == 4) { GG_KR_NF(4) }
      else { GG_KR_NF(8) }
#undef GG_KR_NF
#undef GG_KR_STREAM
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::kr_finish_kernel, dim3((unsigned)gg::ceil_div(M, gg::kKrThreads)),
                         dim3(gg::kKrThreads), 0, st0, work_dev, (int)gy, M, out_dev, 0);
      GG_LAUNCH_CHECK();
      return;
    }
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
