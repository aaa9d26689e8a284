// Dense FP64 building blocks of the GRIEF solve on MI355X: an MFMA GEMM
// (v_mfma_f64_16x16x4_f64, 128x128 block tile, LDS double buffer), GEMV, and a
// blocked Cholesky / triangular-solve suite built on them.
//
// Reference arithmetic replaced (gp_grief/models/gp_grief_model.py):
//   A = Phi^T Phi                       :149   (numpy -> dsyrk)       -> gg_gemm
//   P = A + diag(s / w); cho_factor(P)  :152-153 (LAPACK potrf)       -> gg_potrf
//   cho_solve(P, .)                     :175, 234 (LAPACK potrs)       -> gg_potrs
//   Phi.T.dot(y), Phi.dot(v)            :97, 173, 224, 234            -> gg_gemv
// Layout: every matrix is row-major with an explicit leading dimension.
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "gg_internal.h"

namespace gg {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128, kBN = 128, kBK = 16, kPad = 16;
constexpr int kLdT = kBM + kPad;  // LDS row stride (doubles): 144*8 B = 36*32 -> +32 banks per k-row
constexpr int kGemmThreads = 256;
constexpr int kLoadPerT = kBM * kBK / kGemmThreads;  // 8 doubles of A and of B per thread

// C = alpha op(A) op(B) + beta C.   op(A): M x K, op(B): K x N.
// TA: A stored K x M (lda) ; else M x K.   TB: B stored N x K (ldb) ; else K x N.
// uplo 1: only C[i][j] with i >= j is written (lower), 2: i <= j (upper).
// partial != nullptr: split-K; block z writes its raw sum to partial + z*M*N.
// tri (triangular operands, entries outside the triangle are read as zero and
// never loaded, so the k-loop skips the zero blocks; gg_trtri):
//   tri & 1: op(B) lower triangular (op(B)[k][n] = 0 for k < n): k >= n0;
//   tri & 2: op(A) lower triangular (op(A)[m][k] = 0 for k > m): k < m0 + kBM.
// One 128 x 128 tile (m0, n0) over k in [kbeg, kend); P: the split-K slab
// (raw sums) or nullptr (C = alpha acc + beta C).  Body of gemm_kernel and of
// trtri_level_kernel.
template <bool TA, bool TB>
__device__ __forceinline__ void gemm_tile(int M, int N, double alpha,
                                          const double* __restrict__ A, int64_t lda,
                                          const double* __restrict__ B, int64_t ldb, double beta,
                                          double* C, int64_t ldc, int uplo, int m0, int n0,
                                          int kbeg, int kend, double* __restrict__ P, int tri) {
  __shared__ __attribute__((aligned(16))) double sA[2][kBK * kLdT];
  __shared__ __attribute__((aligned(16))) double sB[2][kBK * kLdT];
  if (tri & 1) kbeg = max(kbeg, n0 - n0 % kBK);
  if (tri & 2) kend = min(kend, m0 + kBM);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  double ra[kLoadPerT], rb[kLoadPerT];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < kLoadPerT; ++u) {
      const int e = tid + u * kGemmThreads;
      int mi, ki;
      if (TA) { ki = e / kBM; mi = e % kBM; } else { mi = e / kBK; ki = e % kBK; }
      const int gm = m0 + mi, gk = k0 + ki;
      double v = 0.0;
      if (gm < M && gk < kend && (!(tri & 2) || gk <= gm))
        v = TA ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk];
      ra[u] = v;
      int ni, kj;
      if (TB) { ni = e / kBK; kj = e % kBK; } else { kj = e / kBN; ni = e % kBN; }
      const int gn = n0 + ni, gk2 = k0 + kj;
      double w = 0.0;
      if (gn < N && gk2 < kend && (!(tri & 1) || gk2 >= gn))
        w = TB ? B[(int64_t)gn * ldb + gk2] : B[(int64_t)gk2 * ldb + gn];
      rb[u] = w;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < kLoadPerT; ++u) {
      const int e = tid + u * kGemmThreads;
      int mi, ki;
      if (TA) { ki = e / kBM; mi = e % kBM; } else { mi = e / kBK; ki = e % kBK; }
      sA[buf][ki * kLdT + mi] = ra[u];
      int ni, kj;
      if (TB) { ni = e / kBK; kj = e % kBK; } else { kj = e / kBN; ni = e % kBN; }
      sB[buf][kj * kLdT + ni] = rb[u];
    }
  };

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  const int nk = (kend - kbeg + kBK - 1) / kBK;
  if (nk > 0) {
    load(kbeg);
    store(0);
    __syncthreads();
    for (int c = 0; c < nk; ++c) {
      const bool more = c + 1 < nk;
      if (more) load(kbeg + (c + 1) * kBK);
      const double* a_s = sA[c & 1];
      const double* b_s = sB[c & 1];
#pragma unroll
      for (int s = 0; s < kBK / 4; ++s) {
        const int kr = (4 * s + (lane >> 4)) * kLdT + (lane & 15);
        double af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = a_s[kr + wm + 16 * i];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = b_s[kr + wn + 16 * j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
      if (more) store((c + 1) & 1);
      __syncthreads();
    }
  }

  // f64 C/D layout: lane holds D[(lane>>4) + 4r][lane & 15]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + (lane >> 4) + 4 * r;
        const int col = n0 + wn + 16 * j + (lane & 15);
        if (row >= M || col >= N) continue;
        if (uplo == 1 && col > row) continue;
        if (uplo == 2 && row > col) continue;
        const double v = acc[i][j][r];
        if (P) {
          P[(int64_t)row * N + col] = v;
        } else {
          double* c = C + (int64_t)row * ldc + col;
          *c = (beta == 0.0) ? alpha * v : fma(alpha, v, beta * *c);
        }
      }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    const double* __restrict__ B, int64_t ldb, double beta, double* C, int64_t ldc, int uplo,
    int kchunk, double* __restrict__ partial, int tri = 0) {
  const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
  if (uplo == 1 && n0 > m0 + kBM - 1) return;
  if (uplo == 2 && m0 > n0 + kBN - 1) return;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  double* P = partial ? partial + (int64_t)blockIdx.z * M * N : nullptr;
  gemm_tile<TA, TB>(M, N, alpha, A, lda, B, ldb, beta, C, ldc, uplo, m0, n0, kbeg, kend, P, tri);
}

// TN GEMM for Gram-type products C = alpha A^T B (+ beta C), A: K x M and
// B: K x N both k-major (row-major, row = k) -- A = Phi^T Phi with Phi n x p.
// Same 128 x 128 workgroup tile and 64 x 64 wave tiles as gemm_kernel, but the
// operand tiles move global -> LDS by LDS-DMA (global_load_lds, 16 B per
// lane: one 1 KB wave instruction per 128-double k-row), kNS stages in flight,
// each retired by a counted s_waitcnt vmcnt + one raw s_barrier: no staging
// registers, no ds_write, and the HBM / L2 stream runs kNS - 1 stages ahead of
// the MFMAs.  Rows are padded to kLdT doubles (the DMA base of each k-row
// instruction), so fragment reads stay conflict-free.  Needs M, N, lda, ldb
// even and 16-byte aligned A, B (the host checks).  Rows k >= kend of the
// last stage are clamped reads, zeroed in the A fragment.
// One 128 x 128 output tile (m0, n0) over k in [kbeg, kbeg + kchunk) -- the
// body of both TN kernels below.
template <int kBKg, int kNSg>
__device__ __forceinline__ void gemm_tn_glds_tile(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    const double* __restrict__ B, int64_t ldb, double beta, double* C, int64_t ldc, int uplo,
    int kchunk, double* __restrict__ partial, int m0, int n0, int kz, double* gl) {
  constexpr int kStageD = 2 * kBKg * kLdT;       // doubles per stage (A then B)
  constexpr int kPerWave = kBKg / 4;             // k-rows of A (and of B) per wave
  static_assert(kBKg % 4 == 0 && kGemmThreads == 256, "four waves share a stage's k-rows");
  constexpr int kInstr = 2 * kPerWave;           // DMA instructions per wave per stage
  const int kbeg = kz * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int nst = (kend - kbeg + kBKg - 1) / kBKg;
  const int acol = min(m0 + 2 * lane, M - 2);
  const int bcol = min(n0 + 2 * lane, N - 2);

  auto issue = [&](int g) {
    double* st = gl + (g % kNSg) * kStageD;
    const int k0 = kbeg + g * kBKg;
#pragma unroll
    for (int j = 0; j < kPerWave; ++j) {
      const int r = wave * kPerWave + j;
      const int k = min(k0 + r, kend - 1);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(A + (int64_t)k * lda + acol),
          (__attribute__((address_space(3))) void*)(st + r * kLdT), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(B + (int64_t)k * ldb + bcol),
          (__attribute__((address_space(3))) void*)(st + kBKg * kLdT + r * kLdT), 16, 0, 0);
    }
  };

  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

#pragma unroll
  for (int g = 0; g < kNSg - 1; ++g)
    if (g < nst) issue(g);
  constexpr int kWait0 = (7 << 4) | (15 << 8);
  for (int g = 0; g < nst; ++g) {
    // retire stage g: the younger stages g+1 .. g+kNS-2 may stay in flight
    const int younger = min(kNSg - 2, nst - 1 - g);
    if (younger >= 2)
      __builtin_amdgcn_s_waitcnt(((2 * kInstr) & 15) | ((((2 * kInstr) >> 4) & 3) << 14) |
                                 (7 << 4) | (15 << 8));
    else if (younger == 1)
      __builtin_amdgcn_s_waitcnt((kInstr & 15) | (((kInstr >> 4) & 3) << 14) | (7 << 4) |
                                 (15 << 8));
    else
      __builtin_amdgcn_s_waitcnt(kWait0);
    __builtin_amdgcn_s_barrier();
    if (g + kNSg - 1 < nst) issue(g + kNSg - 1);
    const double* a_s = gl + (g % kNSg) * kStageD;
    const double* b_s = a_s + kBKg * kLdT;
    const int krem = kend - (kbeg + g * kBKg);   // valid k-rows in this stage
    // fragments of k-step s (the tail mask only in the last, partial stage:
    // a uniform branch, so full stages carry no per-fragment select)
    auto frag = [&](int s_, double (&af)[4], double (&bf)[4], bool masked) {
      const int kk = 4 * s_ + (lane >> 4);
      const int kr = kk * kLdT + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[i] = a_s[kr + wm + 16 * i];
        if (masked && kk >= krem) af[i] = 0.0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = b_s[kr + wn + 16 * j];
    };
    auto mma = [&](const double (&af)[4], const double (&bf)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    };
    const bool full = krem >= kBKg;
#pragma unroll
    for (int s = 0; s < kBKg / 4; ++s) {
      double af[4], bf[4];
      frag(s, af, bf, !full);
      mma(af, bf);
    }
  }
  double* P = partial ? partial + (int64_t)kz * M * N : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + (lane >> 4) + 4 * r;
        const int col = n0 + wn + 16 * j + (lane & 15);
        if (row >= M || col >= N) continue;
        if (uplo == 1 && col > row) continue;
        if (uplo == 2 && row > col) continue;
        const double v = acc[i][j][r];
        if (P) {
          P[(int64_t)row * N + col] = v;
        } else {
          double* c = C + (int64_t)row * ldc + col;
          *c = (beta == 0.0) ? alpha * v : fma(alpha, v, beta * *c);
        }
      }
}

template <int kBKg, int kNSg, int kMinWg>
__global__ __launch_bounds__(kGemmThreads, kMinWg) void gemm_tn_glds_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    const double* __restrict__ B, int64_t ldb, double beta, double* C, int64_t ldc, int uplo,
    int kchunk, double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) double gl[];
  const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
  if (uplo == 1 && n0 > m0 + kBM - 1) return;
  if (uplo == 2 && m0 > n0 + kBN - 1) return;
  gemm_tn_glds_tile<kBKg, kNSg>(M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, uplo, kchunk,
                                partial, m0, n0, blockIdx.z, gl);
}

// Split-K, XCD-grouped by K-slab: a 1-D grid of gn gm S8 workgroups (S8 = S
// rounded up to 8); workgroup b runs on XCD b % 8 (round-robin dispatch) and
// takes slab z = 8 (i / T) + b % 8, tile i % T (i = b / 8, T = gm gn), so all
// tiles of one K-slab run on the same XCD, start together and read the same
// k-rows of A and B at about the same time: each slab crosses the fabric once
// into that XCD's L2 instead of once per XCD.
template <int kBKg, int kNSg, int kMinWg>
__global__ __launch_bounds__(kGemmThreads, kMinWg) void gemm_tn_glds_xcd_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    const double* __restrict__ B, int64_t ldb, double beta, double* C, int64_t ldc, int uplo,
    int kchunk, double* __restrict__ partial, int gn, int gm, int S) {
  extern __shared__ __attribute__((aligned(16))) double gl[];
  const int b = blockIdx.x, i = b >> 3, T = gm * gn;
  const int z = 8 * (i / T) + (b & 7), t = i % T;
  if (z >= S) return;
  const int m0 = (t / gn) * kBM, n0 = (t % gn) * kBN;
  if (uplo == 1 && n0 > m0 + kBM - 1) return;
  if (uplo == 2 && m0 > n0 + kBN - 1) return;
  gemm_tn_glds_tile<kBKg, kNSg>(M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, uplo, kchunk,
                                partial, m0, n0, z, gl);
}

template <int BK, int NS, int MW>
static void launch_tn_xcd(dim3 grid, hipStream_t s, int M, int N, int K, double alpha,
                          const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                          double* C, int64_t ldc, int uplo, int kchunk, double* part) {
  static bool attr = false;
  const void* fn = reinterpret_cast<const void*>(&gemm_tn_glds_xcd_kernel<BK, NS, MW>);
  if (!attr) {
    GG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)((size_t)NS * 2 * BK * kLdT * sizeof(double))));
    attr = true;
  }
  const int gn = (int)grid.x, gm = (int)grid.y, S = (int)grid.z;
  const int64_t S8 = ceil_div(S, 8) * 8;
  const size_t lds = (size_t)NS * 2 * BK * kLdT * sizeof(double);
  hipLaunchKernelGGL((gemm_tn_glds_xcd_kernel<BK, NS, MW>), dim3((unsigned)(gn * gm * S8)),
                     dim3(kGemmThreads), lds, s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc,
                     uplo, kchunk, part, gn, gm, S);
}

template <int kBKg, int kNSg>
constexpr size_t tn_glds_lds() {
  return (size_t)kNSg * 2 * kBKg * kLdT * sizeof(double);
}

__global__ void splitk_reduce_kernel(int M, int N, int S, const double* __restrict__ partial,
                                     double alpha, double beta, double* C, int64_t ldc,
                                     int uplo) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(e / N), col = (int)(e % N);
    if (uplo == 1 && col > row) continue;
    if (uplo == 2 && row > col) continue;
    double s = 0.0;
    for (int z = 0; z < S; ++z) s += partial[(int64_t)z * total + e];
    double* c = C + (int64_t)row * ldc + col;
    *c = (beta == 0.0) ? alpha * s : fma(alpha, s, beta * *c);
  }
}



template <int BK, int NS, int MW>
static void launch_tn(dim3 grid, hipStream_t s, int M, int N, int K, double alpha, const double* A,
                      int64_t lda, const double* B, int64_t ldb, double beta, double* C,
                      int64_t ldc, int uplo, int kchunk, double* part) {
  static bool attr = false;
  const void* fn = reinterpret_cast<const void*>(&gemm_tn_glds_kernel<BK, NS, MW>);
  if (!attr) {
    GG_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)tn_glds_lds<BK, NS>()));
    attr = true;
  }
  const size_t lds = tn_glds_lds<BK, NS>();
  hipLaunchKernelGGL((gemm_tn_glds_kernel<BK, NS, MW>), grid, dim3(kGemmThreads), lds, s, M, N,
                     K, alpha, A, lda, B, ldb, beta, C, ldc, uplo, kchunk, part);
}

// TN-GEMM variant (A/B knob, from the handle-free snapshot): GG_GEMM_TN=0 the
// register-staged gemm_kernel, else the LDS-DMA kernel with the XCD-slab
// split-K grid (BK 8, 2 stages, 3 waves/SIMD, each K-slab's tiles on one
// XCD): n = 1e5, p = 1000 3.37 -> 2.60 ms (29.7 -> 38.5 TF), p = 5000 47.0 ->
// 43.8 ms against the same tile on the launch-order grid
// (profiles/r03/n/gram_xcd_ab.jsonl; 53.0 against 46.9 TF for the
// register-staged kernel on the C5 Gram, profiles/r02_g_gram_tn_variants.jsonl).
// The other stage shapes, the persistent supertile grid and the 128 x 256
// AGPR tile of those A/Bs measured slower and live in the history (round 4).
static int gemm_tn_variant() {
  const char* e = gg::knob("GG_GEMM_TN");
  return e ? atoi(e) : 14;
}

// split-K factor gemm() chooses when the workspace is not the limit
static int splitk_factor(int M, int N, int K) {
  if (K <= 4 * kBK) return 1;
  const int64_t tiles = ceil_div(M, kBM) * ceil_div(N, kBN);
  const int64_t want = std::max<int64_t>(1, 512 / std::max<int64_t>(tiles, 1));
  const int64_t cap_k = std::max<int64_t>(1, K / (4 * kBK));
  const int S = (int)std::min(want, std::min<int64_t>(cap_k, 64));
  const int kchunk = (int)(ceil_div(ceil_div(std::max(K, 1), S), kBK) * kBK);
  return (int)ceil_div(std::max(K, 1), kchunk);
}

static bool tn_dma_shape(bool ta, bool tb, int M, int N) {
  return ta && !tb && gemm_tn_variant() > 0 && M >= 2 && N >= 2 && (M % 2) == 0 && (N % 2) == 0;
}

// Split-K for the TN LDS-DMA kernel (the Gram A = Phi^T Phi, n >> p).  All
// tiles have the same k-length, so with one tile per workgroup they finish in
// rounds of 768 (3 per CU), and the C4 Gram (820 lower-triangle tiles) runs a
// full round plus a round of 52.  Splitting K by S = 8 (units of 1/8 of a
// tile's k-loop, partial sums reduced by splitk_reduce_kernel) measured
// (profiles/r02_zk_gram_splitk.jsonl, n = 1e5):
//   p = 1000  14.95 -> 3.35 ms, p = 5000  53.1 -> 47.3 ms,
//   p = 10^4 192.2 -> 172.6 ms,
// flat from S = 8 to 32 at every shape (S = 2 / 4 gave 188.7 / 179.3 ms at
// p = 10^4).  The partial slabs are capped at 8 GB.
// GG_GEMM_SPLITK=S forces S (A/B).
static int tn_splitk(int M, int N, int K, int uplo) {
  (void)uplo;
  if (K < 4096) return 1;
  const int64_t cap_k = std::max<int64_t>(1, K / (64 * kBK));
  const char* e = gg::knob("GG_GEMM_SPLITK");
  if (e != nullptr) return (int)std::max<int64_t>(1, std::min<int64_t>(atoi(e), cap_k));
  const int64_t cap_mem = std::max<int64_t>(1, (int64_t)1e9 / ((int64_t)M * N));
  // the XCD-slab grid wants whole groups of 8 slabs; small Grams (few tiles)
  // take two groups (p = 1000: 38.5 TF at 16 and 32 slabs, 29.5 at 8)
  const int64_t want = (int64_t)M * N <= (int64_t)2000 * 2000 ? 16 : 8;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, std::min(cap_k, cap_mem)));
}

// the split gemm() will use for this call (given an unlimited workspace)
static int choose_splitk(bool ta, bool tb, int M, int N, int K, int uplo) {
  if (tn_dma_shape(ta, tb, M, N) && K >= 4096) return tn_splitk(M, N, K, uplo);
  return splitk_factor(M, N, K);
}

void gemm(bool ta, bool tb, int M, int N, int K, double alpha, const double* A, int64_t lda,
          const double* B, int64_t ldb, double beta, double* C, int64_t ldc, int uplo,
          hipStream_t s, double* splitk_buf = nullptr, int64_t splitk_elems = 0, int tri = 0) {
  if (M <= 0 || N <= 0) return;
  const int gm = (int)ceil_div(M, kBM), gn = (int)ceil_div(N, kBN);
  int S = 1;
  if (splitk_buf != nullptr && K > 4 * kBK) {
    const int64_t cap_mem = std::max<int64_t>(1, splitk_elems / ((int64_t)M * N));
    S = (int)std::min<int64_t>(choose_splitk(ta, tb, M, N, K, uplo), cap_mem);
  }
  const int kchunk = (int)(ceil_div(ceil_div(std::max(K, 1), S), kBK) * kBK);
  S = (int)ceil_div(std::max(K, 1), kchunk);
  dim3 grid(gn, gm, S);
  double* part = (S > 1) ? splitk_buf : nullptr;
  // TN with even shapes and 16-byte aligned operands: the LDS-DMA kernel
  // (GG_GEMM_TN selects its stage shape for A/B; 0 = the register-staged one)
  if (tri == 0 && tn_dma_shape(ta, tb, M, N) &&
      (lda % 2) == 0 && (ldb % 2) == 0 && ((reinterpret_cast<uintptr_t>(A) & 15) == 0) &&
      ((reinterpret_cast<uintptr_t>(B) & 15) == 0)) {
    // unsplit products keep the launch-order grid (one slab: nothing to group)
    if (grid.z > 1)
      launch_tn_xcd<8, 2, 3>(grid, s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, uplo, kchunk, part);
    else
      launch_tn<8, 2, 3>(grid, s, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, uplo, kchunk, part);
    GG_LAUNCH_CHECK();
    if (part) {
      const int64_t total = (int64_t)M * N;
      const int nb = (int)std::min<int64_t>(4096, ceil_div(total, 256));
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(nb), dim3(256), 0, s, M, N, S, part, alpha,
                         beta, C, ldc, uplo);
      GG_LAUNCH_CHECK();
    }
    return;
  }
#define GG_GEMM_LAUNCH(TA_, TB_)                                                              \
  hipLaunchKernelGGL((gemm_kernel<TA_, TB_>), grid, dim3(kGemmThreads), 0, s, M, N, K, alpha, \
                     A, lda, B, ldb, beta, C, ldc, uplo, kchunk, part, tri)
  if (ta && tb) GG_GEMM_LAUNCH(true, true);
  else if (ta) GG_GEMM_LAUNCH(true, false);
  else if (tb) GG_GEMM_LAUNCH(false, true);
  else GG_GEMM_LAUNCH(false, false);
#undef GG_GEMM_LAUNCH
  GG_LAUNCH_CHECK();
  if (part) {
    const int64_t total = (int64_t)M * N;
    const int nb = (int)std::min<int64_t>(4096, ceil_div(total, 256));
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(nb), dim3(256), 0, s, M, N, S, part, alpha,
                       beta, C, ldc, uplo);
    GG_LAUNCH_CHECK();
  }
}

// ------------------------------------------------------------------ GEMV
// y[j] = alpha * sum_r A[r][j] x[r] + beta y[j]   (A: R x Cn row-major), split over rows
__global__ __launch_bounds__(256) void gemv_t_partial_kernel(int64_t R, int Cn,
                                                             const double* __restrict__ A,
                                                             int64_t lda,
                                                             const double* __restrict__ x,
                                                             int64_t rows_per,
                                                             double* __restrict__ part) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = min(R, r0 + rows_per);
  if (j >= Cn) return;
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) s = fma(A[r * lda + j], x[r], s);
  part[(int64_t)blockIdx.y * Cn + j] = s;
}

__global__ void gemv_t_reduce_kernel(int Cn, int S, const double* __restrict__ part,
                                     double alpha, double beta, double* y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Cn) return;
  double s = 0.0;
  for (int z = 0; z < S; ++z) s += part[(int64_t)z * Cn + j];
  y[j] = (beta == 0.0) ? alpha * s : fma(alpha, s, beta * y[j]);
}

// y[r] = alpha * sum_j A[r][j] x[j] + beta y[r] : one wave per row
__global__ __launch_bounds__(256) void gemv_n_kernel(int64_t R, int Cn,
                                                     const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ x, double alpha,
                                                     double beta, double* y) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const double* row = A + r * lda;
  double s = 0.0;
  for (int j = lane; j < Cn; j += 64) s = fma(row[j], x[j], s);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) y[r] = (beta == 0.0) ? alpha * s : fma(alpha, s, beta * y[r]);
}

void gemv(bool trans, int64_t R, int Cn, double alpha, const double* A, int64_t lda,
          const double* x, double beta, double* y, double* work, int64_t work_elems,
          hipStream_t s) {
  if (R <= 0 || Cn <= 0) return;
  if (!trans) {
    hipLaunchKernelGGL(gemv_n_kernel, dim3((unsigned)ceil_div(R, 4)), dim3(256), 0, s, R, Cn,
                       A, lda, x, alpha, beta, y);
    GG_LAUNCH_CHECK();
    return;
  }
  const int gx = (int)ceil_div(Cn, 256);
  int64_t S = std::max<int64_t>(1, 2048 / gx);
  S = std::min<int64_t>(S, std::max<int64_t>(1, work_elems / Cn));
  S = std::min<int64_t>(S, std::max<int64_t>(1, R / 64));
  const int64_t rows_per = ceil_div(R, S);
  S = ceil_div(R, rows_per);
  GG_REQUIRE(work != nullptr && work_elems >= S * Cn, GG_ERR_VALUE, "gemv work too small");
  hipLaunchKernelGGL(gemv_t_partial_kernel, dim3(gx, (unsigned)S), dim3(256), 0, s, R, Cn, A,
                     lda, x, rows_per, work);
  GG_LAUNCH_CHECK();
  hipLaunchKernelGGL(gemv_t_reduce_kernel, dim3(gx), dim3(256), 0, s, Cn, (int)S, work, alpha,
                     beta, y);
  GG_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ Cholesky
constexpr int kNB = 64;

// Streams of the calling device for gg_potrf's look-ahead (created once per
// device, never destroyed: they live as long as the process).  which 0: the
// factorisation chain (the critical path) at the highest priority; 1: the
// wide trailing updates at the lowest.  (A CU-masked wide stream -- R of
// every 32 CUs left to the chain -- measured slower than the priorities,
// rounds 3-4: removed.)
hipStream_t aux_stream(int which) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> streams;
  int dev = 0;
  GG_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find({dev, which});
  if (it != streams.end()) return it->second;
  int least = 0, greatest = 0;
  GG_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t st;
  GG_HIP(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, which == 1 ? least : greatest));
  streams[{dev, which}] = st;
  return st;
}

// Lane-quad broadcast: the value of lane (lane & ~3) | s (DPP quad_perm).
template <int s>
__device__ __forceinline__ double quad_bcast(double v) {
  constexpr int perm = s | (s << 2) | (s << 4) | (s << 6);
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)bits, perm, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(bits >> 32), perm, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Sum over the four lanes of a quad (DPP quad_perm xor 1, then xor 2).
__device__ __forceinline__ double quad_sum(double v) {
  const long long b1 = __double_as_longlong(v);
  const int lo1 = __builtin_amdgcn_mov_dpp((int)b1, 0xB1, 0xF, 0xF, false);
  const int hi1 = __builtin_amdgcn_mov_dpp((int)(b1 >> 32), 0xB1, 0xF, 0xF, false);
  v += __longlong_as_double(((long long)hi1 << 32) | (unsigned int)lo1);
  const long long b2 = __double_as_longlong(v);
  const int lo2 = __builtin_amdgcn_mov_dpp((int)b2, 0x4E, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_mov_dpp((int)(b2 >> 32), 0x4E, 0xF, 0xF, false);
  return v + __longlong_as_double(((long long)hi2 << 32) | (unsigned int)lo2);
}

// ---- Cholesky block step, round 3 (potrf_fac_kernel + potrf_upd_kernel).
// The round-2 block kernel spent ~27 us of its ~40-75 us factoring the 64 x 64
// diagonal block (two barriers and a correctly rounded sqrt + divide per
// column), ~9 us in a column-at-a-time TRSM and ~12 us per in-panel update
// chunk (GG_POTRF_PROF stamps, profiles/r03/p_potrf_prof.jsonl).  Here the
// factor and the TRSM proceed four columns at a time and the in-panel
// updates are a separate right-looking MFMA launch (potrf_upd_kernel).

// LDS row stride of 64-wide blocks read four doubles at a time: 68 doubles
// keeps rows 16-byte aligned and puts rows 4u + q (q < 4) on disjoint banks.
constexpr int kLdf = 68;
// row stride of the MFMA operand tiles (64 x 64, column reads by 16 lanes)
constexpr int kLdu = kNB + 1;

// 1/sqrt(t): v_rsq_f64 plus one second-order Newton-Raphson correction,
// r = r0 (1 + h/2 + 3h^2/8), h = 1 - t r0^2 (error ~ h^3: full precision).
__device__ __forceinline__ double rsq_refined(double t) {
  const double r0 = __builtin_amdgcn_rsq(t);
  const double h = fma(-(t * r0), r0, 1.0);
  return fma(r0 * h, fma(0.375, h, 0.5), r0);
}

// v[q] for q < 4 as three independent selects (a nested ?: chain on q
// becomes a divergent switch)
__device__ __forceinline__ double pick4(int q, double v0, double v1, double v2, double v3) {
  double r = v0;
  r = q == 1 ? v1 : r;
  r = q == 2 ? v2 : r;
  r = q == 3 ? v3 : r;
  return r;
}

__device__ __forceinline__ double2 lds_ld2(const double* p) {
  return *reinterpret_cast<const double2*>(p);
}

// Fused diagonal-block factor + panel TRSM of one 64-column block (k0, nb):
//   L_bb = chol(A[k0:k0+nb, k0:k0+nb])           (every workgroup, registers)
//   L[rows, k0:k0+nb] = A[rows, k0:k0+nb] L_bb^-T  (workgroup b: 64 rows
//                                                   k0 + nb + 64 b ...)
// Column block k0 is fully updated on entry (potrf_upd_kernel / the narrow
// update did it).  Thread t owns row i = t / 4 and columns 4u + q (q = t & 3,
// u < 16) of the block.  Factor: super-step s handles columns 4s..4s+3 with
// ONE barrier: every thread factors the 4 x 4 pivot block itself (rsq
// pivots), forms the L values of its own row and of row 4(s+1) + q, updates
// its entry of the next column block (written to the pan buffer for step
// s + 1), and applies the previous super-step's rank-4 term to the rest of
// its row (Lp buffer, double-buffered).  TRSM: the four unknowns of a
// super-step are gathered within the lane quad by DPP and solved by every
// quad lane, then the rank-4 term updates the later columns -- no barriers.
// Rows >= pend (below the panel) are also stored transposed into LT
// (LT[c - P0][row - pend]) for the narrow / wide TN updates.  The last
// workgroup to arrive stores L_bb (the block is factored in place).
__global__ __launch_bounds__(256) void potrf_fac_kernel(double* __restrict__ A, int64_t lda,
                                                        int n, int k0, int nb, int P0, int pend,
                                                        int kp,
                                                        double* __restrict__ LT, int64_t ldt,
                                                        int* __restrict__ status,
                                                        int* __restrict__ arrived,
                                                        long long* __restrict__ stamps) {
  auto stamp = [&](int k) {
    if (stamps != nullptr && threadIdx.x < 64)
      stamps[(((int64_t)(k0 / kNB) * 160 + blockIdx.x) * 4 + k) * 64 + threadIdx.x] =
          __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  __shared__ __attribute__((aligned(16))) double Lf[kNB][kLdf];
  __shared__ __attribute__((aligned(16))) double pan[2][kNB][4];
  __shared__ __attribute__((aligned(16))) double Lp[2][kNB][4];
  __shared__ __attribute__((aligned(16))) double invd[kNB];
  __shared__ double term_lds[2 * kNB][kLdu];   // the fused term's operands / products
  __shared__ int last;
  const int tid = threadIdx.x;
  const int i = tid >> 2, q = tid & 3;
  double* Abb = A + (int64_t)k0 * lda + k0;
  const int64_t row = (int64_t)k0 + nb + (int64_t)blockIdx.x * kNB + i;   // TRSM row
  const bool has_row = row < n;
  // the TRSM rows first (their latency hides under the factor), then D; the
  // rows wait in this thread's own slots of Lf (the slots its L entries take
  // after the factor), not in registers
  // (unconditional loads from clamped addresses, then selects: guarded loads
  // become exec-mask branches whose saved masks spill)
  double x[16], d[16];
  {
    const double* xr = A + (has_row ? row : (int64_t)k0) * lda + k0;
    const double* dr = Abb + (int64_t)min(i, nb - 1) * lda;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = 4 * u + q, jc = min(j, nb - 1);
      x[u] = xr[jc];
      d[u] = dr[jc];
    }
  }
  if (kp >= 0) {
    // the newest in-panel term (column block kp = k0 - 64, finished by the
    // previous block step) on MFMA: D -= L_k L_k^T, R -= L_r L_k^T with
    // L_k = L[k0:k0+64, kp:kp+64], L_r = L[rows, kp:kp+64] (potrf_upd_kernel
    // gave the panel's later column blocks the older terms)
    double(*Tk)[kLdu] = reinterpret_cast<double(*)[kLdu]>(&term_lds[0][0]);
    double(*Tr)[kLdu] = reinterpret_cast<double(*)[kLdu]>(&term_lds[kNB][0]);
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t rb0 = (int64_t)k0 + nb + (int64_t)blockIdx.x * kNB;
    for (int e = tid; e < kNB * kNB; e += 256) {
      const int r = e >> 6, c = e & 63;
      Tk[r][c] = A[(int64_t)(k0 + min(r, nb - 1)) * lda + kp + c];
      Tr[r][c] = A[min(rb0 + r, (int64_t)n - 1) * lda + kp + c];
    }
    __syncthreads();
    d4 dacc[4], racc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dacc[t] = d4{0.0, 0.0, 0.0, 0.0};
      racc[t] = d4{0.0, 0.0, 0.0, 0.0};
    }
#pragma unroll
    for (int ks = 0; ks < kNB / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      const double ad = Tk[16 * wave + (lane & 15)][kk];
      const double ar = Tr[16 * wave + (lane & 15)][kk];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double bv = Tk[16 * t + (lane & 15)][kk];
        if (t <= wave) dacc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bv, dacc[t], 0, 0, 0);
        racc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, bv, racc[t], 0, 0, 0);
      }
    }
    __syncthreads();
    // MFMA result layout: row 4 r + (lane >> 4), column lane & 15 of tile t
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Tk[16 * wave + 4 * r + (lane >> 4)][16 * t + (lane & 15)] = dacc[t][r];
        Tr[16 * wave + 4 * r + (lane >> 4)][16 * t + (lane & 15)] = racc[t][r];
      }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      d[u] -= Tk[i][4 * u + q];
      x[u] -= Tr[i][4 * u + q];
    }
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int j = 4 * u + q;
    x[u] = (has_row && j < nb) ? x[u] : 0.0;
    d[u] = (i < nb && j <= i) ? d[u] : (i == j ? 1.0 : 0.0);
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) Lf[i][4 * u + q] = x[u];
  stamp(1);
  pan[0][i][q] = d[0];
  // pivot check kept in two registers (a per-pivot boolean would be a lane
  // mask per column, spilled): the smallest pivot, and NaN if any was not finite
  double pivmin = 1.0, pivnan = 0.0;
  double lo[4] = {0.0, 0.0, 0.0, 0.0};   // own row's L of the previous super-step
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int cb = s & 1, nx = cb ^ 1;
    // ---- the 4 x 4 pivot block (rows 4s..4s+3 of column block s), factored
    // by every thread
    double p[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const double2 v0 = lds_ld2(&pan[cb][4 * s + a][0]), v1 = lds_ld2(&pan[cb][4 * s + a][2]);
      p[a][0] = v0.x;
      p[a][1] = v0.y;
      p[a][2] = v1.x;
      p[a][3] = v1.y;
    }
    double l[4][4], iv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double t = p[c][c];
#pragma unroll
      for (int e = 0; e < c; ++e) t = fma(-l[c][e], l[c][e], t);
      pivmin = t < pivmin ? t : pivmin;
      pivnan += t * 0.0;
      // materialise the running check here: sunk to its use after the loop,
      // it would keep all 64 pivots live across the factor
      asm volatile("" : "+v"(pivmin), "+v"(pivnan));
      const double r = rsq_refined(t);
      iv[c] = r;
      l[c][c] = t * r;
#pragma unroll
      for (int a = c + 1; a < 4; ++a) {
        double v = p[a][c];
#pragma unroll
        for (int e = 0; e < c; ++e) v = fma(-l[a][e], l[c][e], v);
        l[a][c] = v * r;
      }
    }
    if (tid == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) invd[4 * s + c] = iv[c];
    }
    // ---- L of a row from its four column-block-s entries (rows >= 4s + 4)
    auto row_l = [&](const double (&rv)[4], double (&lv)[4]) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        double v = rv[c];
#pragma unroll
        for (int e = 0; e < c; ++e) v = fma(-lv[e], l[c][e], v);
        lv[c] = v * iv[c];
      }
    };
    // own row i: rows inside the pivot block take its factor, rows above it
    // are zero in this column block
    double ro[4], lc[4];
    {
      const double2 v0 = lds_ld2(&pan[cb][i][0]), v1 = lds_ld2(&pan[cb][i][2]);
      ro[0] = v0.x;
      ro[1] = v0.y;
      ro[2] = v1.x;
      ro[3] = v1.y;
    }
    row_l(ro, lc);
    const int rel = i - 4 * s;
#pragma unroll
    for (int c = 0; c < 4; ++c) lc[c] = rel >= c ? lc[c] : 0.0;
    // this thread's entry of column 4s + q is final
    d[s] = pick4(q, lc[0], lc[1], lc[2], lc[3]);
    Lp[cb][i][0] = lc[0];
    Lp[cb][i][1] = lc[1];
    Lp[cb][i][2] = lc[2];
    Lp[cb][i][3] = lc[3];
    if (s < 15) {
      // row j = 4(s+1) + q: the column this thread owns in block s + 1
      const int j = 4 * (s + 1) + q;
      double rj[4], lj[4];
      {
        const double2 v0 = lds_ld2(&pan[cb][j][0]), v1 = lds_ld2(&pan[cb][j][2]);
        rj[0] = v0.x;
        rj[1] = v0.y;
        rj[2] = v1.x;
        rj[3] = v1.y;
      }
      row_l(rj, lj);
      double t = d[s + 1];
      if (s > 0) {   // term s - 1 on column block s + 1 (its bulk was deferred)
        const double2 w0 = lds_ld2(&Lp[nx][j][0]), w1 = lds_ld2(&Lp[nx][j][2]);
        t = fma(-lo[0], w0.x, t);
        t = fma(-lo[1], w0.y, t);
        t = fma(-lo[2], w1.x, t);
        t = fma(-lo[3], w1.y, t);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) t = fma(-lc[c], lj[c], t);
      d[s + 1] = t;
      pan[nx][i][q] = t;
      // term s - 1 on column blocks s + 2.. (rows 4u + q of the Lp buffer)
      if (s > 0) {
#pragma unroll
        for (int u = s + 2; u < 16; ++u) {
          const double2 w0 = lds_ld2(&Lp[nx][4 * u + q][0]), w1 = lds_ld2(&Lp[nx][4 * u + q][2]);
          double v = d[u];
          v = fma(-lo[0], w0.x, v);
          v = fma(-lo[1], w0.y, v);
          v = fma(-lo[2], w1.x, v);
          v = fma(-lo[3], w1.y, v);
          d[u] = v;
          if ((u & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) lo[c] = lc[c];
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int j = 4 * u + q;
    x[u] = Lf[i][j];
    Lf[i][j] = (j <= i) ? d[u] : 0.0;
  }
  stamp(2);
  // The block is factored in place: the LAST workgroup to have read it (every
  // workgroup holds the same L_bb) stores it, so no workgroup can read a
  // half-written block.  No waiting: the counter only picks the writer.
  if (tid == 0) last = atomicAdd(arrived, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (last) {
    if (tid == 0 && !(pivmin > 0.0 && pivnan == 0.0)) *status = 1;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = 4 * u + q;
      if (i < nb && j <= i) Abb[(int64_t)i * lda + j] = d[u];
    }
  }
  if (!has_row) return;
  // ---- TRSM of this workgroup's row: x L_bb^T = r, four columns at a time
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    double lb[4][4];
#pragma unroll
    for (int a = 1; a < 4; ++a) {
      const double2 v0 = lds_ld2(&Lf[4 * s + a][4 * s]), v1 = lds_ld2(&Lf[4 * s + a][4 * s + 2]);
      lb[a][0] = v0.x;
      lb[a][1] = v0.y;
      lb[a][2] = v1.x;
      lb[a][3] = v1.y;
    }
    const double2 i01 = lds_ld2(&invd[4 * s]), i23 = lds_ld2(&invd[4 * s + 2]);
    const double v0 = quad_bcast<0>(x[s]), v1 = quad_bcast<1>(x[s]);
    const double v2 = quad_bcast<2>(x[s]), v3 = quad_bcast<3>(x[s]);
    const double y0 = v0 * i01.x;
    const double y1 = fma(-y0, lb[1][0], v1) * i01.y;
    const double y2 = fma(-y1, lb[2][1], fma(-y0, lb[2][0], v2)) * i23.x;
    const double y3 = fma(-y2, lb[3][2], fma(-y1, lb[3][1], fma(-y0, lb[3][0], v3))) * i23.y;
    x[s] = pick4(q, y0, y1, y2, y3);
#pragma unroll
    for (int u = s + 1; u < 16; ++u) {
      const double2 w0 = lds_ld2(&Lf[4 * u + q][4 * s]), w1 = lds_ld2(&Lf[4 * u + q][4 * s + 2]);
      double v = x[u];
      v = fma(-y0, w0.x, v);
      v = fma(-y1, w0.y, v);
      v = fma(-y2, w1.x, v);
      v = fma(-y3, w1.y, v);
      x[u] = v;
      if ((u & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
    // keep the scheduler from hoisting every super-step's Lf loads (they do
    // not depend on x) to the top: that spills
    __builtin_amdgcn_sched_barrier(0);
  }
  double* Ar = A + row * lda + k0;
  double* Lt = (LT != nullptr && row >= pend) ? LT + (int64_t)(k0 - P0 + q) * ldt + (row - pend)
                                              : nullptr;
  if (nb == kNB) {   // (uniform) full block: unguarded stores
#pragma unroll
    for (int u = 0; u < 16; ++u) Ar[4 * u + q] = x[u];
    if (Lt != nullptr) {
#pragma unroll
      for (int u = 0; u < 16; ++u) Lt[(int64_t)(4 * u) * ldt] = x[u];
    }
  } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = 4 * u + q;
      if (j < nb) Ar[j] = x[u];
      if (Lt != nullptr && j < nb) Lt[(int64_t)(4 * u) * ldt] = x[u];
    }
  }
  stamp(3);
}

// Right-looking update of 64 x 64 blocks by one or more finished 64-column
// blocks: A[r, c] -= L[r, ka:kb] L[c, ka:kb]^T for the column blocks c of
// [c0, c1) and the row blocks r >= c (lower), L read from A itself.  One
// workgroup per (row block, column block): the in-panel update after each
// block step (kb - ka = 64, the panel's later column blocks) and the narrow
// look-ahead update of the next panel (kb - ka = the panel width).  Wave w
// owns rows 16w..16w+15 of the tile (4 MFMA column tiles).
// Diagonal tiles store only their lower triangle.  kPf: the next chunk's
// operands are prefetched into registers while the current one is
// multiplied; without it (the default) they are loaded per chunk and the
// kernel fits three workgroups per CU.
template <bool kPf>
__global__ __launch_bounds__(256, 3) void potrf_upd_kernel(double* __restrict__ A, int64_t lda,
                                                        int n, int ka, int kb, int c0, int c1) {
  // K in chunks of 32: two 64 x 33 operand tiles (33 KB) fit three
  // workgroups per CU
  constexpr int kKc = 32;
  __shared__ double Lr[kNB][kKc + 1];
  __shared__ double Lc[kNB][kKc + 1];
  const int r0 = c0 + (int)blockIdx.x * kNB, cc0 = c0 + (int)blockIdx.y * kNB;
  if (r0 < cc0) return;   // above the diagonal
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  d4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  // staging: thread t loads rows (t >> 3) + 32 m, columns 4 (t & 7) .. +3
  const int sr = tid >> 3, sc = 4 * (tid & 7);
  double2 vr[2][2], vc[2][2];
  auto fetch = [&](int kc) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int rr = sr + 32 * m;
      const int64_t gr = min((int64_t)r0 + rr, (int64_t)n - 1), gc = min(cc0 + rr, n - 1);
      const double* pr = A + gr * lda + kc + sc;
      const double* pc = A + gc * lda + kc + sc;
      vr[m][0] = *reinterpret_cast<const double2*>(pr);
      vr[m][1] = *reinterpret_cast<const double2*>(pr + 2);
      vc[m][0] = *reinterpret_cast<const double2*>(pc);
      vc[m][1] = *reinterpret_cast<const double2*>(pc + 2);
    }
  };
  if (kPf) fetch(ka);
  for (int kc = ka; kc < kb; kc += kKc) {
    if (!kPf) fetch(kc);
    __syncthreads();   // the previous chunk's LDS reads are done
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int rr = sr + 32 * m;
      Lr[rr][sc] = vr[m][0].x;
      Lr[rr][sc + 1] = vr[m][0].y;
      Lr[rr][sc + 2] = vr[m][1].x;
      Lr[rr][sc + 3] = vr[m][1].y;
      Lc[rr][sc] = vc[m][0].x;
      Lc[rr][sc + 1] = vc[m][0].y;
      Lc[rr][sc + 2] = vc[m][1].x;
      Lc[rr][sc + 3] = vc[m][1].y;
    }
    __syncthreads();
    if (kPf && kc + kKc < kb) fetch(kc + kKc);
#pragma unroll
    for (int ks = 0; ks < kKc / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      const double a = Lr[16 * wave + (lane & 15)][kk];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Lc[16 * t + (lane & 15)][kk], acc[t], 0,
                                                      0, 0);
    }
  }
  // MFMA result layout: row 4 r + (lane >> 4), column lane & 15 of tile t
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = 16 * wave + 4 * r + (lane >> 4), cc = 16 * t + (lane & 15);
      const int64_t gr = (int64_t)r0 + rr;
      const int gc = cc0 + cc;
      if (gr < n && gc < c1 && (r0 != cc0 || rr >= cc)) {
        double* pa = A + gr * lda + gc;
        *pa -= acc[t][r];
      }
    }
}

// W_b = L_bb^-1 for every 64-column diagonal block (gg_potrs's diagonal
// solves), one workgroup per block, after the factorisation (off the block
// chain).  Column c = i by the four threads of the quad: the sum over s < r
// splits by s mod 4 (W[s][c] = 0 for s < c), a quad sum reduces it, and the
// owner (s = r mod 4) keeps W[r][c] in w[r >> 2].
__global__ __launch_bounds__(256) void potrf_winv_kernel(const double* __restrict__ A,
                                                         int64_t lda, int n,
                                                         double* __restrict__ Wall) {
  __shared__ double Lf[kNB][kNB + 1];
  __shared__ double invd[kNB];
  const int b = blockIdx.x, k0 = b * kNB, nb = min(kNB, n - k0);
  const int tid = threadIdx.x, i = tid >> 2, q = tid & 3;
  for (int e = tid; e < kNB * kNB; e += 256) {
    const int r = e >> 6, c = e & 63;
    Lf[r][c] = (r < nb && c <= r) ? A[(int64_t)(k0 + r) * lda + k0 + c] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  if (tid < kNB) invd[tid] = 1.0 / Lf[tid][tid];
  __syncthreads();
  const int c = i;
  double w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) w[u] = 0.0;
#pragma unroll
  for (int r = 0; r < kNB; ++r) {
    double sacc = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (4 * u >= r) continue;                 // s >= r for every q
      const double t = fma(Lf[r][q + 4 * u], w[u], sacc);
      sacc = (4 * u + 3 < r) ? t : (q + 4 * u < r ? t : sacc);
    }
    sacc = quad_sum(sacc);
    const double wr = r < c ? 0.0 : ((r == c ? 1.0 : 0.0) - sacc) * invd[r];
    w[r >> 2] = (q == (r & 3)) ? wr : w[r >> 2];
  }
  double* W = Wall + (int64_t)b * kNB * kNB;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int r = q + 4 * u;
    W[(int64_t)r * kNB + c] = (r < nb && c < nb && c <= r) ? w[u] : 0.0;
  }
}

// Triangular solve with ONE right-hand side as a single launch: workgroup j
// owns block row b (forward: b = j; backward, L^T: b = nblk - 1 - j), so the
// dependency order equals the dispatch order and every block it waits on
// belongs to a workgroup dispatched before it (no deadlock: the waits only
// ever point backwards).  It streams its off-diagonal blocks in readiness
// order -- each block's L values are loaded before its flag is polled, so
// the critical step after the flag is one vector load and 16 FMAs -- then
// applies the stored inverse diagonal block W_b, stores its part of the
// solution and releases its flag.  Thread (i, q) = (t / 4, t % 4) owns row i
// of the block and the quarter q of each 64-wide inner product; the quad
// sums by DPP.  Flags: agent-scope release / acquire (the L2 is per XCD), a
// bounded spin (status <- 2 instead of a hang; the host raises).
constexpr int kTrsvSpin = 1 << 24;

template <bool kTrans>
__global__ __launch_bounds__(256) void trsv_chain_kernel(int n, const double* __restrict__ L,
                                                         int64_t lda,
                                                         const double* __restrict__ Winv,
                                                         double* B, int* flags,
                                                         int* __restrict__ status,
                                                         int* __restrict__ ticket) {
  __shared__ double rhs[kNB];
  __shared__ int ok, tk;
  const int nblk = (n + kNB - 1) / kNB;
  // block rows are taken in arrival order from a ticket counter, not from
  // blockIdx: every row this workgroup waits on belongs to a workgroup that
  // is already running, whatever order the hardware dispatches them in
  if (threadIdx.x == 0) tk = atomicAdd(ticket, 1);
  __syncthreads();
  const int b = kTrans ? nblk - 1 - tk : tk;
  const int k0 = b * kNB, nb = min(kNB, n - k0);
  const int tid = threadIdx.x, i = tid >> 2, q = tid & 3;
  const int row = k0 + i;
  if (tid == 0) ok = 1;
  double acc = 0.0;
  const int ndep = kTrans ? nblk - 1 - b : b;
  for (int t = 0; t < ndep; ++t) {
    const int c = kTrans ? nblk - 1 - t : t;       // dependencies in readiness order
    const int c0 = c * kNB;
    double lv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = c0 + 16 * q + u;
      // forward: L[row][j]; backward (L^T): L[j][row]
      lv[u] = (row < n && j < n) ? (kTrans ? L[(int64_t)j * lda + row] : L[(int64_t)row * lda + j])
                                 : 0.0;
    }
    if (tid == 0) {
      int spin = 0;
      while (__hip_atomic_load(&flags[c], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spin > kTrsvSpin) {
          ok = 0;
          break;
        }
      }
    }
    __syncthreads();
    if (!ok) break;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int j = c0 + 16 * q + u;
      if (j < n) acc = fma(lv[u], B[j], acc);
    }
  }
  acc = quad_sum(acc);
  if (q == 0) rhs[i] = (i < nb) ? B[row] - acc : 0.0;
  __syncthreads();
  // x_b = W_b rhs (forward) or W_b^T rhs (backward)
  const double* W = Winv + (int64_t)b * kNB * kNB;
  double y = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int k = 16 * q + u;
    y = fma(kTrans ? W[(int64_t)k * kNB + i] : W[(int64_t)i * kNB + k], rhs[k], y);
  }
  y = quad_sum(y);
  if (q == 0 && i < nb) B[row] = y;
  __threadfence();   // every thread's stores visible device-wide before the flag
  __syncthreads();
  if (tid == 0) {
    if (!ok) *status = 2;
    __hip_atomic_store(&flags[b], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Triangular solve with many right-hand sides as one chained launch per
// direction: workgroup (b, j) computes the 64 x 64 block X[b, j] (block row b
// of the solution, column chunk j of the right-hand sides).  Linear ids run
// b-major in dependency order (forward b = 0.., backward b = nblk-1..), so
// every block a workgroup waits on belongs to an earlier-dispatched one.  Per
// dependency block c: L's 64 x 64 block is staged in LDS first (forward
// L[b, c]; backward L[c, b], read transposed), then the flag of X[c, j] is
// polled (agent-scope acquire, bounded spin) and X[c, j] staged; each wave
// accumulates its 16 rows x 64 columns on MFMA.  Then X[b, j] = W_b (B - acc)
// (forward; W_b^T backward) -- a second MFMA product -- is stored and the
// flag released.  tri (forward only): the right-hand side is lower
// triangular with 64-row blocks (the identity), so X[b, j] = 0 for b < j and
// only c >= j contribute.
__global__ __launch_bounds__(256) void trsm_chain_kernel(int n, int r, const double* __restrict__ L,
                                                         int64_t lda,
                                                         const double* __restrict__ Winv,
                                                         double* Bm, int64_t ldb, int trans,
                                                         int tri, int* flags,
                                                         int* __restrict__ status,
                                                         int* __restrict__ ticket) {
  __shared__ double Ls[kNB][kNB + 1];
  __shared__ double Xs[kNB][kNB + 1];
  __shared__ int ok, tk;
  const int nblk = (n + kNB - 1) / kNB, nch = (r + kNB - 1) / kNB;
  // (block row, column chunk) in arrival order from a ticket counter
  // (trsv_chain_kernel): dispatch order cannot deadlock the chain
  if (threadIdx.x == 0) tk = atomicAdd(ticket, 1);
  __syncthreads();
  const int order = tk / nch, j = tk % nch;
  const int b = trans ? nblk - 1 - order : order;
  const int k0 = b * kNB, nb = min(kNB, n - k0);
  const int j0 = j * kNB, cw = min(kNB, r - j0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) ok = 1;
  int* myflag = flags + (int64_t)b * nch + j;
  if (tri && b < j) {          // X[b, j] = 0 (lower-triangular result)
    for (int e = tid; e < nb * cw; e += 256)
      Bm[(int64_t)(k0 + e / cw) * ldb + j0 + e % cw] = 0.0;
    __threadfence();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(myflag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  d4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  const int cfirst = trans ? nblk - 1 : (tri ? j : 0);
  const int ndep = trans ? nblk - 1 - b : b - cfirst;
  for (int t = 0; t < ndep; ++t) {
    const int c = trans ? nblk - 1 - t : cfirst + t;
    const int c0 = c * kNB, ncb = min(kNB, n - c0);
    __syncthreads();   // the previous block's LDS reads are done
    for (int e = tid; e < kNB * kNB; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      // Ls[i][k]: row i of block b, column k of block c (the A operand)
      double v = 0.0;
      if (!trans) {
        if (rr < nb && cc < ncb) v = L[(int64_t)(k0 + rr) * lda + c0 + cc];
        Ls[rr][cc] = v;
      } else {
        // L^T[b-row i][c-col k] = L[c0 + k][k0 + i]: coalesced over i
        if (rr < ncb && cc < nb) v = L[(int64_t)(c0 + rr) * lda + k0 + cc];
        Ls[cc][rr] = v;
      }
    }
    if (tid == 0) {
      int spin = 0;
      while (__hip_atomic_load(&flags[(int64_t)c * nch + j], __ATOMIC_ACQUIRE,
                               __HIP_MEMORY_SCOPE_AGENT) == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spin > kTrsvSpin) {
          ok = 0;
          break;
        }
      }
    }
    __syncthreads();
    if (!ok) break;
    for (int e = tid; e < kNB * kNB; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      Xs[rr][cc] = (rr < ncb && cc < cw) ? Bm[(int64_t)(c0 + rr) * ldb + j0 + cc] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kNB / 4; ++ks) {
      const int kk = 4 * ks + (lane >> 4);
      const double a = Ls[16 * wave + (lane & 15)][kk];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
        acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Xs[kk][16 * tt + (lane & 15)], acc[tt],
                                                      0, 0, 0);
    }
  }
  // rhs = B[b, j] - acc  (into Xs), W_b (or W_b^T) into Ls
  __syncthreads();
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = 16 * wave + 4 * q + (lane >> 4), cc = 16 * tt + (lane & 15);
      const double bv = (rr < nb && cc < cw) ? Bm[(int64_t)(k0 + rr) * ldb + j0 + cc] : 0.0;
      Xs[rr][cc] = bv - acc[tt][q];
    }
  const double* W = Winv + (int64_t)b * kNB * kNB;
  for (int e = tid; e < kNB * kNB; e += 256) {
    const int rr = e >> 6, cc = e & 63;
    if (!trans) Ls[rr][cc] = W[e];
    else Ls[cc][rr] = W[e];
  }
  __syncthreads();
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) acc[tt] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < kNB / 4; ++ks) {
    const int kk = 4 * ks + (lane >> 4);
    const double a = Ls[16 * wave + (lane & 15)][kk];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
      acc[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Xs[kk][16 * tt + (lane & 15)], acc[tt],
                                                    0, 0, 0);
  }
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = 16 * wave + 4 * q + (lane >> 4), cc = 16 * tt + (lane & 15);
      if (rr < nb && cc < cw) Bm[(int64_t)(k0 + rr) * ldb + j0 + cc] = acc[tt][q];
    }
  __threadfence();
  __syncthreads();
  if (tid == 0) {
    if (!ok) *status = 2;
    __hip_atomic_store(myflag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// X's 64 x 64 diagonal blocks = the W_b = L_bb^-1 gg_potrf formed (lower,
// zero above), one workgroup per block (gg_trtri's leaves).
__global__ __launch_bounds__(256) void trtri_leaves_kernel(int n, const double* __restrict__ Wall,
                                                           double* __restrict__ X, int64_t ldx) {
  const int b = blockIdx.x, k0 = b * kNB, nb = min(kNB, n - k0);
  const double* W = Wall + (int64_t)b * kNB * kNB;
  for (int e = threadIdx.x; e < kNB * kNB; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (r < nb && c < nb) X[(int64_t)(k0 + r) * ldx + k0 + c] = W[e];
  }
}

// X = L^-1 by the recursive split of LAPACK's trtri, for a diagonal block
// [o, o + n) of the factor (n1 = its first half in whole 64-blocks):
//   [L11   0 ]^-1   [ X11            0  ]
//   [L21  L22]    = [ -X22 L21 X11   X22 ],   X11 = L11^-1, X22 = L22^-1
// The leaves (64 x 64) are gg_potrf's W_b.  Every node of one tree level is
// independent, so a level is two launches (grid z = node): phase 0
// T = L21 X11 (X11 lower: tri 1), phase 1 X21 = -X22 T (X22 lower: tri 2),
// each skipping the zero k-blocks of its triangular operand -- ~p^3 / 3 FLOP
// on the MFMA GEMM in 2 log2(p / 64) launches.  nodes: (o, n1, n2, T offset).
template <int PH>
__global__ __launch_bounds__(kGemmThreads, 2) void trtri_level_kernel(
    const double* __restrict__ L, int64_t ldl, double* X, int64_t ldx, double* T,
    const int64_t* __restrict__ nodes) {
  const int64_t* nd = nodes + 4 * blockIdx.z;
  const int o = (int)nd[0], n1 = (int)nd[1], n2 = (int)nd[2];
  double* Tn = T + nd[3];
  const int m0 = blockIdx.y * kBM, n0 = blockIdx.x * kBN;
  if (m0 >= n2 || n0 >= n1) return;
  if (PH == 0)
    gemm_tile<false, false>(n2, n1, 1.0, L + (int64_t)(o + n1) * ldl + o, ldl,
                            X + (int64_t)o * ldx + o, ldx, 0.0, Tn, n1, 0, m0, n0, 0, n1,
                            nullptr, 1);
  else
    gemm_tile<false, false>(n2, n1, -1.0, X + (int64_t)(o + n1) * ldx + o + n1, ldx, Tn, n1,
                            0.0, X + (int64_t)(o + n1) * ldx + o, ldx, 0, m0, n0, 0, n2,
                            nullptr, 2);
}

static void trtri_tree(int o, int n, int depth, std::vector<std::vector<int64_t>>& levels) {
  if (n <= kNB) return;
  const int nblk = (int)ceil_div(n, kNB);
  const int n1 = (nblk / 2) * kNB, n2 = n - n1;
  if ((int)levels.size() <= depth) levels.resize(depth + 1);
  levels[depth].insert(levels[depth].end(), {(int64_t)o, (int64_t)n1, (int64_t)n2, 0});
  trtri_tree(o, n1, depth + 1, levels);
  trtri_tree(o + n1, n2, depth + 1, levels);
}

__global__ void diag_logsum_kernel(const double* A, int64_t lda, int n, double* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += log(A[(int64_t)i * lda + i]);
  __shared__ double red[16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    *out = t;
  }
}

// P = A + diag(s / w)  (w may be null -> s)
__global__ void add_diag_kernel(int n, const double* __restrict__ A, int64_t lda, double s,
                                const double* __restrict__ w, double* P, int64_t ldp) {
  const int64_t total = (int64_t)n * n;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / n), j = (int)(e % n);
    double v = A[(int64_t)i * lda + j];
    if (i == j) v += w ? s / w[i] : s;
    P[(int64_t)i * ldp + j] = v;
  }
}

// out[j] = sum_i M[i][j]^2 (column sums of squares; lower-triangular M uses i >= j)
// 64 columns per workgroup x 16 row phases (1024 threads), fixed-order LDS
// reduction over the phases (deterministic)
__global__ __launch_bounds__(1024) void colsumsq_kernel(int n, const double* __restrict__ Mx,
                                                        int64_t ld, double* out) {
  __shared__ double part[16][65];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  double s = 0.0;
  if (j < n)
    for (int i = j + ph; i < n; i += 16) {
      const double v = Mx[(int64_t)i * ld + j];
      s = fma(v, v, s);
    }
  part[ph][c] = s;
  __syncthreads();
  if (ph == 0 && j < n) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += part[k][c];
    out[j] = t;
  }
}

}  // namespace gg

extern "C" {

int gg_gemm_splitk_elems(int M, int N, int K, int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(elems != nullptr && M >= 0 && N >= 0 && K >= 0, GG_ERR_VALUE, "bad argument");
    const int S = (M > 0 && N > 0) ? gg::splitk_factor(M, N, K) : 1;
    *elems = S > 1 ? (int64_t)S * M * N : 0;
  });
}

int gg_gemm_workspace_elems(int trans_a, int trans_b, int M, int N, int K, int uplo,
                            int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(elems != nullptr && M >= 0 && N >= 0 && K >= 0 && uplo >= 0 && uplo <= 2,
               GG_ERR_VALUE, "bad argument");
    const int S = (M > 0 && N > 0 && K > 4 * gg::kBK)
                      ? gg::choose_splitk(trans_a != 0, trans_b != 0, M, N, K, uplo)
                      : 1;
    *elems = S > 1 ? (int64_t)S * M * N : 0;
  });
}

int gg_gemm(int trans_a, int trans_b, int M, int N, int K, double alpha, const double* A_dev,
            int64_t lda, const double* B_dev, int64_t ldb, double beta, double* C_dev,
            int64_t ldc, int uplo, double* splitk_dev, int64_t splitk_elems, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(M >= 0 && N >= 0 && K >= 0, GG_ERR_VALUE, "negative dimension");
    GG_REQUIRE(C_dev && (K == 0 || (A_dev && B_dev)), GG_ERR_VALUE, "NULL matrix");
    GG_REQUIRE(uplo >= 0 && uplo <= 2, GG_ERR_VALUE, "bad uplo");
    gg::gemm(trans_a != 0, trans_b != 0, M, N, K, alpha, A_dev, lda, B_dev, ldb, beta, C_dev,
             ldc, uplo, gg::as_stream(stream), splitk_dev, splitk_elems);
  });
}

int gg_gemv(int trans, int64_t rows, int cols, double alpha, const double* A_dev, int64_t lda,
            const double* x_dev, double beta, double* y_dev, double* work_dev,
            int64_t work_elems, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(rows >= 0 && cols >= 0 && A_dev && x_dev && y_dev, GG_ERR_VALUE, "bad argument");
    gg::gemv(trans != 0, rows, cols, alpha, A_dev, lda, x_dev, beta, y_dev, work_dev,
             work_elems, gg::as_stream(stream));
  });
}

int gg_add_diag(int n, const double* A_dev, int64_t lda, double s, const double* w_dev,
                double* P_dev, int64_t ldp, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 0 && A_dev && P_dev, GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    const int nb = (int)std::min<int64_t>(4096, gg::ceil_div((int64_t)n * n, 256));
    hipLaunchKernelGGL(gg::add_diag_kernel, dim3(nb), dim3(256), 0, gg::as_stream(stream), n,
                       A_dev, lda, s, w_dev, P_dev, ldp);
    GG_LAUNCH_CHECK();
  });
}

int gg_potrf_work_elems(int n, int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 0 && elems, GG_ERR_VALUE, "bad argument");
    // W blocks, status / log-det slots, one arrival counter per block
    const int64_t nblk = gg::ceil_div(n, gg::kNB);
    *elems = nblk * gg::kNB * gg::kNB + 16 + gg::ceil_div(nblk, 2) + 1;
  });
}

int gg_potrf(int n, double* A_dev, int64_t lda, double* winv_dev, double* logdet_host,
             gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 1 && A_dev && winv_dev, GG_ERR_VALUE, "bad argument");
    hipStream_t s = gg::as_stream(stream);
    const int nblk = (int)gg::ceil_div(n, gg::kNB);
    int* status = reinterpret_cast<int*>(winv_dev + (int64_t)nblk * gg::kNB * gg::kNB);
    double* ld = winv_dev + (int64_t)nblk * gg::kNB * gg::kNB + 8;
    int* arrived = reinterpret_cast<int*>(winv_dev + (int64_t)nblk * gg::kNB * gg::kNB + 16);
    GG_HIP(hipMemsetAsync(status, 0, sizeof(int), s));
    GG_HIP(hipMemsetAsync(arrived, 0, (size_t)nblk * sizeof(int), s));
    // Blocked right-looking factorisation with look-ahead.  Panels of kPanel
    // columns; inside a panel each 64-column block is ONE launch (fused
    // diagonal factor + TRSM, potrf_ftrsm_kernel) plus the in-panel update.
    // After panel P:
    //   narrow (chain stream cs, high priority): the next panel's columns
    //     -= L_P L_P^T
    //   wide (stream ws, low priority): every column right of the next panel
    //     -= L_P L_P^T
    // so the next panel factors on cs while the wide update (the bulk of the
    // flops, one K = kPanel MFMA GEMM) runs beside it and yields CUs to the
    // chain.  Ordering: wide(P) waits for panel P's factor; narrow(P -> P + 1)
    // waits for wide(P - 1), which wrote the same columns; s joins both.
    // Panel width: 512 columns from n = 4096 (the wide update's K = 512 halves
    // its read-modify-write passes over the trailing matrix: p = 10^4 13.4 ->
    // 12.9 ms, p = 5000 4.09 -> 3.95), else 256 (p = 1000: 0.74 vs 0.89 ms;
    // profiles/r03/w_potrf_ab.jsonl).  GG_POTRF_PANEL=<columns> (multiple of
    // 64) for A/B.
    const char* pe = gg::knob("GG_POTRF_PANEL");
    const int kPanel = pe ? std::max(gg::kNB, (atoi(pe) / gg::kNB) * gg::kNB)
                          : (n >= 4096 ? 8 : 4) * gg::kNB;
    // GG_POTRF_LOOKAHEAD=0: everything on s (A/B and debugging)
    const char* la = gg::knob("GG_POTRF_LOOKAHEAD");
    const bool lookahead = !(la != nullptr && atoi(la) == 0);
    hipStream_t cs = lookahead ? gg::aux_stream(0) : s;   // factor chain, high priority
    hipStream_t ws = lookahead ? gg::aux_stream(1) : s;   // wide updates, low priority
    std::vector<hipEvent_t> evs;
    auto new_event = [&]() {
      hipEvent_t e;
      GG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      evs.push_back(e);
      return e;
    };
    hipEvent_t ev_wide = nullptr;   // last wide update issued on ws
    if (lookahead) {
      hipEvent_t e0 = new_event();
      GG_HIP(hipEventRecord(e0, s));
      GG_HIP(hipStreamWaitEvent(cs, e0, 0));
      GG_HIP(hipStreamWaitEvent(ws, e0, 0));
    }
    // two transposed-panel buffers (kPanel x ldt each), stream-ordered
    const int64_t ldt = (n + 1) & ~1;   // even: 16-byte aligned rows for the DMA
    double* lt_buf = nullptr;
    if (n > kPanel) GG_HIP(hipMallocAsync(&lt_buf, 2 * (size_t)kPanel * ldt * sizeof(double), s));
    if (lookahead && lt_buf) {
      hipEvent_t ea = new_event();   // the allocation is ordered on s
      GG_HIP(hipEventRecord(ea, s));
      GG_HIP(hipStreamWaitEvent(cs, ea, 0));
      GG_HIP(hipStreamWaitEvent(ws, ea, 0));
    }
    // GG_POTRF_PROF=<file>: per-block-launch phase stamps of every workgroup
    // (raw int64: nblk, 160, 4, then [nblk][160][4] 100 MHz ticks; 0 = absent)
    const char* prof = gg::knob("GG_POTRF_PROF");
    long long* pstamps = nullptr;
    const size_t nstamp = (size_t)nblk * 160 * 4 * 64;
    if (prof != nullptr && nblk <= 160) {
      GG_HIP(hipMallocAsync(&pstamps, nstamp * sizeof(long long), s));
      GG_HIP(hipMemsetAsync(pstamps, 0, nstamp * sizeof(long long), s));
      if (lookahead) {
        hipEvent_t ep = new_event();
        GG_HIP(hipEventRecord(ep, s));
        GG_HIP(hipStreamWaitEvent(cs, ep, 0));
      }
    }
    // (Measured slower and removed, rounds 2-4: the round-2 left-looking block
    // step; F(k) applying block k - 1's term itself with the in-panel update
    // on a side stream; padding the wide update's workgroups so a block step
    // fits beside them; a CU-masked wide stream.)
    for (int P0 = 0; P0 < n; P0 += kPanel) {
      const int pend = std::min(n, P0 + kPanel);
      double* LT = (lt_buf && pend < n) ? lt_buf + (int64_t)((P0 / kPanel) & 1) * kPanel * ldt
                                        : nullptr;
      // Block step k: F(k) factors column block k and solves the rows below
      // it; U(k) gives the panel's later column blocks the term of block k.
      for (int k0 = P0; k0 < pend; k0 += gg::kNB) {
        const int b = k0 / gg::kNB;
        const int nb = std::min(gg::kNB, n - k0);
        const int grid = std::max(1, (int)gg::ceil_div(n - k0 - nb, gg::kNB));
        hipLaunchKernelGGL(gg::potrf_fac_kernel, dim3(grid), dim3(256), 0, cs, A_dev, lda, n, k0,
                           nb, P0, pend, -1, LT, ldt, status, arrived + b, pstamps);
        GG_LAUNCH_CHECK();
        const int c0 = k0 + gg::kNB;
        if (c0 < pend) {
          dim3 ug((unsigned)gg::ceil_div(n - c0, gg::kNB), (unsigned)gg::ceil_div(pend - c0, gg::kNB));
          hipLaunchKernelGGL(gg::potrf_upd_kernel<false>, ug, dim3(256), 0, cs, A_dev, lda, n, k0,
                             k0 + gg::kNB, c0, pend);
          GG_LAUNCH_CHECK();
        }
      }
      if (pend >= n) break;
      const int nend = std::min(n, pend + kPanel);
      // the wide update may start as soon as LT (written by the block steps) is
      // complete
      hipEvent_t ef = nullptr;
      if (lookahead && nend < n) {
        ef = new_event();
        GG_HIP(hipEventRecord(ef, cs));
      }
      // narrow: A[pend:, pend:nend] -= L[pend:, P] L[pend:nend, P]^T (lower),
      // after the previous wide update (it wrote the same columns)
      if (ev_wide) GG_HIP(hipStreamWaitEvent(cs, ev_wide, 0));
      {
        dim3 ug((unsigned)gg::ceil_div(n - pend, gg::kNB), (unsigned)gg::ceil_div(nend - pend, gg::kNB));
        hipLaunchKernelGGL(gg::potrf_upd_kernel<false>, ug, dim3(256), 0, cs, A_dev, lda, n, P0,
                           pend, pend, nend);
        GG_LAUNCH_CHECK();
      }
      if (nend < n) {
        // wide: A[nend:, nend:] -= L[nend:, P] L[nend:, P]^T (lower), on ws
        if (lookahead) GG_HIP(hipStreamWaitEvent(ws, ef, 0));
        const int pw = pend - P0;
        const double* Lw = LT + (nend - pend);
        gg::gemm(true, false, n - nend, n - nend, pw, -1.0, Lw, ldt, Lw, ldt, 1.0,
                 A_dev + (int64_t)nend * lda + nend, lda, 1, ws);
        if (lookahead) {
          ev_wide = new_event();
          GG_HIP(hipEventRecord(ev_wide, ws));
        }
      } else {
        ev_wide = nullptr;
      }
    }
    if (lookahead) {
      // join: s waits for everything issued on cs and ws
      hipEvent_t ec = new_event(), ew = new_event();
      GG_HIP(hipEventRecord(ec, cs));
      GG_HIP(hipEventRecord(ew, ws));
      GG_HIP(hipStreamWaitEvent(s, ec, 0));
      GG_HIP(hipStreamWaitEvent(s, ew, 0));
    }
    if (lt_buf) GG_HIP(hipFreeAsync(lt_buf, s));
    hipLaunchKernelGGL(gg::potrf_winv_kernel, dim3(nblk), dim3(256), 0, s, A_dev, lda, n,
                       winv_dev);
    GG_LAUNCH_CHECK();
    hipLaunchKernelGGL(gg::diag_logsum_kernel, dim3(1), dim3(1024), 0, s, A_dev, lda, n, ld);
    GG_LAUNCH_CHECK();
    int st = 0;
    double lds = 0.0;
    GG_HIP(hipMemcpyAsync(&st, status, sizeof(int), hipMemcpyDeviceToHost, s));
    GG_HIP(hipMemcpyAsync(&lds, ld, sizeof(double), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    for (hipEvent_t e : evs) GG_HIP(hipEventDestroy(e));
    if (pstamps) {
      std::vector<long long> h64(nstamp), h((size_t)nblk * 160 * 4 + 3);
      GG_HIP(hipMemcpy(h64.data(), pstamps, nstamp * sizeof(long long), hipMemcpyDeviceToHost));
      GG_HIP(hipFree(pstamps));
      h[0] = nblk;
      h[1] = 160;
      h[2] = 4;
      for (size_t q = 0; q + 3 < h.size(); ++q) h[q + 3] = h64[q * 64];
      if (FILE* f = fopen(prof, "wb")) {
        fwrite(h.data(), sizeof(long long), h.size(), f);
        fclose(f);
      }
    }
    GG_REQUIRE(st == 0, GG_ERR_LINALG, "Matrix is not positive definite (device Cholesky)");
    if (logdet_host) *logdet_host = 2.0 * lds;
  });
}

// Solve (L L^T) X = B in place for B: n x r (ldb), using the factor and the
// diagonal-block inverses from gg_potrf.  which: 1 = forward only (L^-1 B),
// 2 = backward only (L^-T B), 3 = both (P^-1 B); | 4 = B is lower triangular
// (e.g. the identity, for L^-1 itself: forward only), so block row k only
// touches columns < k0 + nb.
// Right-looking: after block k is solved, ONE GEMM updates every remaining
// block row (M = rows left, K = nb), so each step is parallel over the rows
// instead of a single row-tile reducing over all previous blocks.
int gg_potrs(int n, int r, const double* L_dev, int64_t lda, const double* winv_dev,
             double* B_dev, int64_t ldb, int which, double* tmp_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 1 && r >= 0 && L_dev && winv_dev && B_dev && tmp_dev, GG_ERR_VALUE,
               "bad argument");
    GG_REQUIRE(!((which & 4) && (which & 2)), GG_ERR_VALUE,
               "triangular right-hand side is forward-only");
    if (r == 0) return;
    hipStream_t s = gg::as_stream(stream);
    const int nblk = (int)gg::ceil_div(n, gg::kNB);
    const bool tri = (which & 4) != 0;
    // one right-hand side: each direction is ONE chained launch
    // (trsv_chain_kernel) instead of a GEMM pair per block row
    const char* ch = gg::knob("GG_TRSV_CHAIN");
    if (r == 1 && !tri && ldb == 1 && !(ch != nullptr && atoi(ch) == 0)) {
      // [forward flags | backward flags | status | two tickets]
      int* flags = nullptr;
      GG_HIP(hipMallocAsync(&flags, (2 * (size_t)nblk + 3) * sizeof(int), s));
      GG_HIP(hipMemsetAsync(flags, 0, (2 * (size_t)nblk + 3) * sizeof(int), s));
      int* st = flags + 2 * nblk;
      if (which & 1)
        hipLaunchKernelGGL(gg::trsv_chain_kernel<false>, dim3(nblk), dim3(256), 0, s, n, L_dev,
                           lda, winv_dev, B_dev, flags, st, st + 1);
      if (which & 2)
        hipLaunchKernelGGL(gg::trsv_chain_kernel<true>, dim3(nblk), dim3(256), 0, s, n, L_dev,
                           lda, winv_dev, B_dev, flags + nblk, st, st + 2);
      GG_LAUNCH_CHECK();
      int hst = 0;
      GG_HIP(hipMemcpyAsync(&hst, st, sizeof(int), hipMemcpyDeviceToHost, s));
      GG_HIP(hipFreeAsync(flags, s));
      GG_HIP(hipStreamSynchronize(s));
      GG_REQUIRE(hst == 0, GG_ERR_RUNTIME, "chained triangular solve timed out");
      return;
    }
    // several right-hand sides: one chained MFMA launch per direction
    // (trsm_chain_kernel) instead of a GEMM pair per block row
    // (a triangular right-hand side -- L^-1 itself -- keeps the blocked path
    // past 100 blocks, where the two measure the same: 26-27 ms at n = 1e4)
    if (r > 1 && !(ch != nullptr && atoi(ch) == 0) && !(tri && nblk > 100)) {
      const int nch = (int)gg::ceil_div(r, gg::kNB);
      const size_t nflags = (size_t)nblk * nch;
      int* flags = nullptr;
      GG_HIP(hipMallocAsync(&flags, (2 * nflags + 3) * sizeof(int), s));
      GG_HIP(hipMemsetAsync(flags, 0, (2 * nflags + 3) * sizeof(int), s));
      int* st = flags + 2 * nflags;
      const unsigned grid = (unsigned)((int64_t)nblk * nch);
      if (which & 1)
        hipLaunchKernelGGL(gg::trsm_chain_kernel, dim3(grid), dim3(256), 0, s, n, r, L_dev, lda,
                           winv_dev, B_dev, ldb, 0, tri ? 1 : 0, flags, st, st + 1);
      if (which & 2)
        hipLaunchKernelGGL(gg::trsm_chain_kernel, dim3(grid), dim3(256), 0, s, n, r, L_dev, lda,
                           winv_dev, B_dev, ldb, 1, 0, flags + nflags, st, st + 2);
      GG_LAUNCH_CHECK();
      int hst = 0;
      GG_HIP(hipMemcpyAsync(&hst, st, sizeof(int), hipMemcpyDeviceToHost, s));
      GG_HIP(hipFreeAsync(flags, s));
      GG_HIP(hipStreamSynchronize(s));
      GG_REQUIRE(hst == 0, GG_ERR_RUNTIME, "chained triangular solve timed out");
      return;
    }
    if (which & 1) {
      for (int b = 0; b < nblk; ++b) {
        const int k0 = b * gg::kNB, nb = std::min(gg::kNB, n - k0);
        const int rc = tri ? std::min(r, k0 + nb) : r;   // live columns
        double* Bk = B_dev + (int64_t)k0 * ldb;
        // Y_k = W_k B_k  (through tmp: W_k reads all nb rows of B_k)
        gg::gemm(false, false, nb, rc, nb, 1.0, winv_dev + (int64_t)b * gg::kNB * gg::kNB,
                 gg::kNB, Bk, ldb, 0.0, tmp_dev, rc, 0, s);
        GG_HIP(hipMemcpy2DAsync(Bk, ldb * sizeof(double), tmp_dev, rc * sizeof(double),
                                rc * sizeof(double), nb, hipMemcpyDeviceToDevice, s));
        const int below = n - k0 - nb;
        if (below > 0)  // B[k0+nb:n] -= L[k0+nb:n, k0:k0+nb] Y_k
          gg::gemm(false, false, below, rc, nb, -1.0, L_dev + (int64_t)(k0 + nb) * lda + k0, lda,
                   Bk, ldb, 1.0, B_dev + (int64_t)(k0 + nb) * ldb, ldb, 0, s);
      }
    }
    if (which & 2) {
      for (int b = nblk - 1; b >= 0; --b) {
        const int k0 = b * gg::kNB, nb = std::min(gg::kNB, n - k0);
        double* Bk = B_dev + (int64_t)k0 * ldb;
        // X_k = W_k^T B_k
        gg::gemm(true, false, nb, r, nb, 1.0, winv_dev + (int64_t)b * gg::kNB * gg::kNB,
                 gg::kNB, Bk, ldb, 0.0, tmp_dev, r, 0, s);
        GG_HIP(hipMemcpy2DAsync(Bk, ldb * sizeof(double), tmp_dev, r * sizeof(double),
                                r * sizeof(double), nb, hipMemcpyDeviceToDevice, s));
        if (k0 > 0)  // B[0:k0] -= L[k0:k0+nb, 0:k0]^T X_k
          gg::gemm(true, false, k0, r, nb, -1.0, L_dev + (int64_t)k0 * lda, lda, Bk, ldb, 1.0,
                   B_dev, ldb, 0, s);
      }
    }
  });
}

int gg_trtri(int n, const double* L_dev, int64_t lda, const double* winv_dev, double* X_dev,
             int64_t ldx, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 1 && L_dev && winv_dev && X_dev && lda >= n && ldx >= n, GG_ERR_VALUE,
               "bad argument");
    hipStream_t s = gg::as_stream(stream);
    const int nblk = (int)gg::ceil_div(n, gg::kNB);
    hipLaunchKernelGGL(gg::trtri_leaves_kernel, dim3(nblk), dim3(256), 0, s, n, winv_dev, X_dev,
                       ldx);
    GG_LAUNCH_CHECK();
    if (nblk == 1) return;
    // the level tables depend only on n: built once per (device, n), kept
    struct Plan {
      std::vector<std::vector<int64_t>> levels;
      int64_t* dtab = nullptr;
      int64_t tmax = 0;
    };
    static std::mutex mu;
    static std::map<std::pair<int, int>, Plan> plans;
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    std::unique_lock<std::mutex> lk(mu);
    Plan& pl = plans[{dev, n}];
    if (pl.dtab == nullptr) {
      gg::trtri_tree(0, n, 0, pl.levels);
      // T offsets per level (the nodes of a level share one scratch)
      std::vector<int64_t> tab;
      for (auto& lv : pl.levels) {
        int64_t off = 0;
        for (size_t i = 0; i < lv.size(); i += 4) {
          lv[i + 3] = off;
          off += lv[i + 1] * lv[i + 2];
        }
        pl.tmax = std::max(pl.tmax, off);
        tab.insert(tab.end(), lv.begin(), lv.end());
      }
      GG_HIP(hipMalloc(reinterpret_cast<void**>(&pl.dtab), tab.size() * sizeof(int64_t)));
      GG_HIP(hipMemcpy(pl.dtab, tab.data(), tab.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    lk.unlock();
    const auto& levels = pl.levels;
    const int64_t* dtab = pl.dtab;
    double* T = nullptr;
    GG_HIP(hipMallocAsync(&T, (size_t)pl.tmax * sizeof(double), s));
    // deepest level first: a node's halves are finished before it runs
    std::vector<int64_t> base(levels.size(), 0);
    for (size_t l = 1; l < levels.size(); ++l) base[l] = base[l - 1] + (int64_t)levels[l - 1].size();
    for (int l = (int)levels.size() - 1; l >= 0; --l) {
      const auto& lv = levels[l];
      const int nodes = (int)(lv.size() / 4);
      int mx1 = 0, mx2 = 0;
      for (int i = 0; i < nodes; ++i) {
        mx1 = std::max(mx1, (int)lv[4 * i + 1]);
        mx2 = std::max(mx2, (int)lv[4 * i + 2]);
      }
      const dim3 grid((unsigned)gg::ceil_div(mx1, gg::kBN), (unsigned)gg::ceil_div(mx2, gg::kBM),
                      (unsigned)nodes);
      hipLaunchKernelGGL(gg::trtri_level_kernel<0>, grid, dim3(gg::kGemmThreads), 0, s, L_dev, lda,
                         X_dev, ldx, T, dtab + base[l]);
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::trtri_level_kernel<1>, grid, dim3(gg::kGemmThreads), 0, s, L_dev, lda,
                         X_dev, ldx, T, dtab + base[l]);
      GG_LAUNCH_CHECK();
    }
    GG_HIP(hipFreeAsync(T, s));
  });
}

int gg_colsumsq_lower(int n, const double* M_dev, int64_t ld, double* out_dev,
                      gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(n >= 0 && M_dev && out_dev, GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    hipLaunchKernelGGL(gg::colsumsq_kernel, dim3((unsigned)gg::ceil_div(n, 64)), dim3(1024), 0,
                       gg::as_stream(stream), n, M_dev, ld, out_dev);
    GG_LAUNCH_CHECK();
  });
}

}  // extern "C"
