// Per-factor symmetric eigendecomposition on device: parallel cyclic Jacobi.
//
// Reference: KronMatrix.schur / svd / eig_vals (gp_grief/tensors/kron_matrix.py:161-200,
// 355-366) call LAPACK (gees / gesdd / syevd) on each 1-D grid-kernel factor.
// Here one workgroup owns one factor and runs two-sided Jacobi with the
// round-robin (tournament) pairing: each round rotates m/2 disjoint index pairs
// at once -- a row pass, then a column pass (+ the eigenvector update), with a
// workgroup barrier between passes.  For m <= 128 the matrix lives in LDS
// (padded rows); larger factors keep it in the caller's HBM scratch
// (L2-resident), so any m fits.  The accumulated rotations are stored
// transposed in the scratch, so their update rides on the coalesced row pass.  Sweeps stop when a whole sweep
// applies no rotation (|a_pq| below eps*sqrt|a_pp a_qq|) or at max_sweeps.
// Output: eigenvalues ascending with matching eigenvector columns (the same
// convention as numpy.linalg.eigh; the reference's gees order is unsorted and
// every consumer is order-invariant).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gg_internal.h"

namespace gg {

constexpr int kEigThreads = 1024;
constexpr int kLdsMaxM = 128;  // A fits in LDS (m x (m+1) f64, 132 KB) up to here

// Dynamic LDS carve-up (both variants): pair tables, rotation table, sort order,
// then (kLds) the padded matrix A.
__host__ __device__ inline int64_t eig_lds_bytes(int m, bool lds_a) {
  const int mm = (m + 1) & ~1, np = mm / 2;
  int64_t b = (int64_t)np * (2 * sizeof(double) + 2 * sizeof(int)) + (int64_t)mm * sizeof(int);
  b = (b + 15) & ~int64_t(15);
  if (lds_a) b += (int64_t)m * (m + 1) * sizeof(double);
  return b;
}

// kLds: A lives in LDS with row stride m + 1 (conflict-free column access);
// else in the HBM scratch (L2-resident).  The eigenvector matrix is kept
// TRANSPOSED (Vt = V^T, row-major) so its update is a row pass -- coalesced --
// fused with A's row pass.
template <bool kLds>
__global__ __launch_bounds__(kEigThreads) void jacobi_kernel(
    const int64_t* __restrict__ dims, const int64_t* __restrict__ offs,
    const double* __restrict__ Ain, double* __restrict__ Qout, double* __restrict__ lam_out,
    const int64_t* __restrict__ lam_offs, double* __restrict__ work,
    const int64_t* __restrict__ work_offs, int max_sweeps, int* __restrict__ status) {
  const int f = blockIdx.x;
  const int m = (int)dims[f];
  const int mm = (m + 1) & ~1;  // padded to even (a dummy index pairs with nobody)
  const int npairs = mm / 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char eig_lds[];
  double* cs = reinterpret_cast<double*>(eig_lds);
  double* sn = cs + npairs;
  int* top = reinterpret_cast<int*>(sn + npairs);
  int* bot = top + npairs;
  int* order = bot + npairs;
  const int64_t head = eig_lds_bytes(m, false);
  const int ld = kLds ? m + 1 : m;
  double* A = kLds ? reinterpret_cast<double*>(eig_lds + head) : work + work_offs[f];
  double* Vt = work + work_offs[f] + (int64_t)m * m;   // m x m, row-major, rows = eigenvectors
  const double* Asrc = Ain + offs[f];
  const int tid = threadIdx.x;
  const int nt = blockDim.x;
  __shared__ int rotated;

  for (int64_t i = tid; i < (int64_t)m * m; i += nt) {
    const int r = (int)(i / m), c = (int)(i % m);
    A[(int64_t)r * ld + c] = 0.5 * (Asrc[i] + Asrc[(int64_t)c * m + r]);
    Vt[i] = (r == c) ? 1.0 : 0.0;
  }
  // tournament (circle method): positions 0..mm-1; pos 0 fixed, the others
  // rotate each round; step 1 derives the round's pairs
  __syncthreads();

  const double eps = 2.220446049250313e-16;
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    if (tid == 0) rotated = 0;
    __syncthreads();
    for (int round = 0; round < mm - 1; ++round) {
      // 1) rotation parameters for the disjoint pairs of this round
      for (int k = tid; k < npairs; k += nt) {
        // index sitting at ring position pos after `round` rotations
        auto at = [&](int pos) -> int {
          return pos == 0 ? 0 : 1 + ((pos - 1 + round) % (mm - 1));
        };
        int p = at(k), q = at(mm - 1 - k);
        if (p > q) {
          const int t = p;
          p = q;
          q = t;
        }
        double c = 1.0, s = 0.0;
        if (q < m) {
          const double apq = A[(int64_t)p * ld + q];
          const double app = A[(int64_t)p * ld + p];
          const double aqq = A[(int64_t)q * ld + q];
          if (fabs(apq) > eps * sqrt(fabs(app * aqq)) && apq != 0.0) {
            const double tau = (aqq - app) / (2.0 * apq);
            const double t = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
            c = 1.0 / sqrt(1.0 + t * t);
            s = t * c;
            rotated = 1;
          }
        }
        cs[k] = c;
        sn[k] = s;
        top[k] = p;  // canonical p < q for the passes below
        bot[k] = q;
      }
      __syncthreads();
      // 2) row pass: rows p, q of A and of Vt  <-  J^T (.)   (adjacent threads:
      //    adjacent columns of one row pair)
      for (int w = tid; w < npairs * m; w += nt) {
        const int k = w / m, col = w - k * m;
        const int p = top[k], q = bot[k];
        const double s = sn[k];
        if (q < m && s != 0.0) {
          const double c = cs[k];
          const double ap = A[p * ld + col], aq = A[q * ld + col];
          A[p * ld + col] = c * ap - s * aq;
          A[q * ld + col] = s * ap + c * aq;
          double* vp_ = Vt + p * m + col;
          double* vq_ = Vt + q * m + col;
          const double vp = *vp_, vq = *vq_;
          *vp_ = c * vp - s * vq;
          *vq_ = s * vp + c * vq;
        }
      }
      __syncthreads();
      // 3) column pass: columns p, q of A  <-  (.) J.  Adjacent threads take
      //    adjacent pairs of the SAME row (one row's cache lines per wave, not
      //    one line per lane)
      for (int w = tid; w < npairs * m; w += nt) {
        const int row = w / npairs, k = w - row * npairs;
        const int p = top[k], q = bot[k];
        const double s = sn[k];
        if (q < m && s != 0.0) {
          const double c = cs[k];
          double* Ar = A + row * ld;
          const double ap = Ar[p], aq = Ar[q];
          Ar[p] = c * ap - s * aq;
          Ar[q] = s * ap + c * aq;
        }
      }
      __syncthreads();
      // 4) annihilated entries are exactly zero; 5) next pairing (circle
      //    method: index 0 fixed, ring positions 1..mm-1 rotate by one per
      //    round, position k meets position mm-1-k) is computed in closed form
      //    by step 1 of the next round, after the barrier below.
      for (int k = tid; k < npairs; k += nt) {
        const int p = top[k], q = bot[k];
        if (q < m && sn[k] != 0.0) {
          A[(int64_t)p * ld + q] = 0.0;
          A[(int64_t)q * ld + p] = 0.0;
        }
      }
      __syncthreads();
    }
    const int any = rotated;
    __syncthreads();
    if (!any) break;
  }
  // eigenvalues = diag(A); sort ascending (stable selection by one thread, m small)
  if (tid == 0) {
    for (int i = 0; i < m; ++i) order[i] = i;
    for (int i = 1; i < m; ++i) {  // insertion sort on the diagonal
      const int oi = order[i];
      const double vi = A[(int64_t)oi * ld + oi];
      int j = i - 1;
      while (j >= 0 && A[(int64_t)order[j] * ld + order[j]] > vi) {
        order[j + 1] = order[j];
        --j;
      }
      order[j + 1] = oi;
    }
    status[f] = (sweep >= max_sweeps) ? 1 : 0;
  }
  __syncthreads();
  double* Q = Qout + offs[f];
  double* lam = lam_out + lam_offs[f];
  for (int i = tid; i < m; i += nt) lam[i] = A[(int64_t)order[i] * ld + order[i]];
  for (int64_t i = tid; i < (int64_t)m * m; i += nt) {
    const int r = (int)(i / m), c = (int)(i % m);
    Q[i] = Vt[(int64_t)order[c] * m + r];
  }
}


// ---------------------------------------------------------------------------
// Householder tridiagonalisation + implicit QL (the LAPACK route: sytd2 /
// orgtr / steqr), one workgroup per matrix.  O(m^3) arithmetic in ~3m
// barrier-separated parallel steps instead of Jacobi's ~10 sweeps x m rounds.
//   1. for i = 0 .. m-3: Householder vector v of A[i+1:, i]; p = tau A22 v;
//      w = p - tau/2 (p.v) v; A22 -= v w^T + w v^T (symmetric rank-2; the
//      full square is kept).  v is stored in A[i+2:, i], tau in LDS.
//   2. Z = H_0 ... H_{m-3}, accumulated backwards in the A storage (the
//      diagonal d and off-diagonal e are in LDS by then).
//   3. implicit QL with Wilkinson shifts on (d, e): wave 0 runs each sweep's
//      scalar rotation chain into LDS (c, s) while the other waves apply the
//      previous sweep's chain to their rows of Z (rotations act on columns).
//   4. eigenvalues ascending by parallel rank; Q columns permuted to match.
// A / Z live in LDS (row stride m + 1) up to kLdsMaxM, else in the HBM
// scratch (L2-resident).
constexpr int kTqThreads = 512;
constexpr int kTqWaves = kTqThreads / 64;

// Bytes of LDS ahead of A in tridiag_ql_kernel: d, e, tau, v, pw, cs, sn
// (m each), red (16), junk (64), the per-wave partial sums of the column
// reductions (kTqWaves x m; in the HBM scratch when A is), rank (m ints).
__host__ __device__ inline int64_t tq_head_bytes(int64_t m, bool lds_a) {
  return ((((int64_t)7 + (lds_a ? kTqWaves : 0)) * m + 80) * (int64_t)sizeof(double) +
          m * (int64_t)sizeof(int) + 15) & ~int64_t(15);
}

__device__ __forceinline__ double tq_block_sum(double v, double* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// Per-wave partial column sums psc[w * ldp + c] = sum over rows r = w, w + nw,
// ... < L of v[r] M[r * ld + c] (lanes over columns: consecutive addresses)
__device__ __forceinline__ void tq_colsum(const double* __restrict__ M, int ld,
                                          const double* __restrict__ v, int L,
                                          double* __restrict__ psc, int ldp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int c0 = 0; c0 < L; c0 += 64) {
    const int c = c0 + lane;
    if (c >= L) break;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int r = wave;
    for (; r + 3 * nw < L; r += 4 * nw) {
      const double* Mr = M + (int64_t)r * ld + c;
      s0 = fma(v[r], Mr[0], s0);
      s1 = fma(v[r + nw], Mr[(int64_t)nw * ld], s1);
      s2 = fma(v[r + 2 * nw], Mr[(int64_t)2 * nw * ld], s2);
      s3 = fma(v[r + 3 * nw], Mr[(int64_t)3 * nw * ld], s3);
    }
    for (; r < L; r += nw) s0 = fma(v[r], M[(int64_t)r * ld + c], s0);
    psc[wave * ldp + c] = (s0 + s1) + (s2 + s3);
  }
}

// Eigenvalues of the symmetric tridiagonal (d, e[0..m-2]) by multisection on
// Sturm counts (ascending: group k finds the k-th smallest).  A group of G
// lanes (G = the largest power of two <= blockDim / m, at most 8; the lanes of
// a group share a wave) evaluates the count at G interior points of the
// bracket at once, so each round shrinks it by G + 1; a ballot over the group
// picks the new bracket.  Stops at an absolute width of 4 eps ||T|| -- the
// accuracy of the QL path (LAPACK dstebz with abstol = 0 uses the same
// absolute ulp * ||T|| tolerance).  The pivots' reciprocal is v_rcp_f64 + one
// Newton step (only the sign of each pivot is counted).  e2 (m doubles of LDS)
// receives e^2; red (>= 16) holds the Gershgorin bounds.
__device__ void tq_bisect(const double* __restrict__ d, const double* __restrict__ e,
                          double* __restrict__ e2, double* __restrict__ red, int m,
                          double* __restrict__ lam) {
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < m; i += nt) e2[i] = (i < m - 1) ? e[i] * e[i] : 0.0;
  if (tid == 0) {
    double lo = d[0], hi = d[0], emax = 0.0;
    for (int i = 0; i < m; ++i) {
      const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < m - 1 ? fabs(e[i]) : 0.0);
      lo = fmin(lo, d[i] - r);
      hi = fmax(hi, d[i] + r);
      if (i < m - 1) emax = fmax(emax, e[i] * e[i]);
    }
    const double nrm = fmax(fabs(lo), fabs(hi));
    // widen the bracket as dstebz does (rounding of the Gershgorin bounds)
    red[0] = lo - 2.1 * 2.220446049250313e-16 * nrm * m - 1e-300;
    red[1] = hi + 2.1 * 2.220446049250313e-16 * nrm * m + 1e-300;
    red[2] = fmax(2.2250738585072014e-308, 2.2250738585072014e-308 * emax);   // pivmin
    red[3] = 4.0 * 2.220446049250313e-16 * fmax(nrm, 1e-300);                 // width
  }
  __syncthreads();
  const double glo = red[0], ghi = red[1], pivmin = red[2], width = red[3];
  int G = 1;
  while (G < 8 && 2 * G * m <= nt) G *= 2;
  const int lane = tid & 63, j = tid % G;
  const int gbase = lane - j;                                  // group's first lane
  const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1)) << gbase;
  const int ngroups = nt / G;
  // every lane of a wave runs the same number of rounds (ballots need the
  // whole group); groups past m idle through them
  const int kmax = ((m + ngroups - 1) / ngroups) * ngroups;
  for (int k = tid / G; k < kmax; k += ngroups) {
    double lo = glo, hi = ghi;
    bool live = k < m;
    for (int it = 0; it < 200; ++it) {
      const bool more = live && (hi - lo > width);
      if (!__ballot(more)) break;
      const double x = lo + (hi - lo) * (double)(j + 1) / (double)(G + 1);
      int cnt = 0;
      double q = d[0] - x;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
      for (int i = 1; i < m; ++i) {
        double rq = __builtin_amdgcn_rcp(q);
        rq = fma(rq, fma(-q, rq, 1.0), rq);
        q = fma(-e2[i - 1], rq, d[i] - x);
        if (fabs(q) < pivmin) q = -pivmin;
        cnt += q < 0.0;
      }
      // first point of the group with more than k eigenvalues below it
      const unsigned long long above = __ballot(cnt > k) & gmask;
      if (more) {
        const int first = above ? __ffsll((long long)above) - 1 - gbase : G;
        const double nlo = first == 0 ? lo : lo + (hi - lo) * (double)first / (double)(G + 1);
        const double nhi = first == G ? hi : lo + (hi - lo) * (double)(first + 1) / (double)(G + 1);
        lo = nlo;
        hi = nhi;
      }
    }
    if (live && j == 0) lam[k] = 0.5 * (lo + hi);
  }
}

// kMode 0: full decomposition (phases 1-4).  kMode 1: eigenvalues only, by
// bisection on the tridiagonal (phase 1, then tq_bisect): the Householder
// reflectors go to Qout (as rows), (d, e, tau) to work + work_offs[f] + m * m,
// the eigenvalues (ascending) to lam_out -- the input of tridiag_invit_kernel
// (selected eigenvectors y of the tridiagonal) and tridiag_backtransform_kernel
// (the eigenvectors of A, Z y = H_0 (H_1 (... H_{m-3} y)), without forming Z).
template <bool kLds, int kMode>
__global__ __launch_bounds__(kTqThreads) void tridiag_ql_kernel(
    const int64_t* __restrict__ dims, const int64_t* __restrict__ offs,
    const double* __restrict__ Ain, double* __restrict__ Qout, double* __restrict__ lam_out,
    const int64_t* __restrict__ lam_offs, double* __restrict__ work,
    const int64_t* __restrict__ work_offs, int max_iter, int* __restrict__ status,
    long long* __restrict__ stamps) {
  const int f = blockIdx.x;
  const int m = (int)dims[f];
  // optional phase timing (GG_EIG_PROF): s_memtime at the phase boundaries
  // (every lane of wave 0 writes its own slot: lane-varying addresses keep
  // these vector stores)
  auto stamp = [&](int k) {
    if (stamps != nullptr && threadIdx.x < 64)
      stamps[((int64_t)f * 8 + k) * 64 + threadIdx.x] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  extern __shared__ __attribute__((aligned(16))) unsigned char tq_lds[];
  // LDS: d, e, tau, v (m each), p/w (m), cs, sn (m each), rank (m ints), red (16)
  double* d = reinterpret_cast<double*>(tq_lds);
  double* e = d + m;
  double* tau = e + m;
  double* v = tau + m;
  double* pw = v + m;
  double* cs = pw + m;
  double* sn = cs + m;
  double* red = sn + m;
  double* junk = red + 16;   // 64 per-lane dummy slots (wave 0's chain stores)
  // per-wave partial column sums (wave w: psc[w * m + c])
  double* psc = kLds ? junk + 64 : work + work_offs[f] + (int64_t)m * m + 2 * m;
  int* rank = reinterpret_cast<int*>(junk + 64 + (kLds ? kTqWaves * m : 0));
  __shared__ int bad;
  const int64_t head = tq_head_bytes(m, kLds);
  const int ld = kLds ? m + 1 : m;
  double* A = kLds ? reinterpret_cast<double*>(tq_lds + head) : work + work_offs[f];
  const double* Asrc = Ain + offs[f];
  const int tid = threadIdx.x, nt = blockDim.x;
  // the L x L loops: wave w takes rows w, w + nw, ..., its lanes the columns
  // (consecutive LDS addresses, no index division)
  const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
  if (tid == 0) bad = 0;
  for (int r = wave; r < m; r += nw)
    for (int c = lane; c < m; c += 64)
      A[(int64_t)r * ld + c] = 0.5 * (Asrc[(int64_t)r * m + c] + Asrc[(int64_t)c * m + r]);
  __syncthreads();

  // ---- 1. tridiagonalisation
  for (int i = 0; i + 2 < m; ++i) {
    const int L = m - i - 1;             // trailing size
    const int r0 = i + 1;
    // Householder of x = A[r0:, i]
    double xs = 0.0;
    for (int t = tid; t < L - 1; t += nt) {
      const double xv = A[(int64_t)(r0 + 1 + t) * ld + i];
      xs = fma(xv, xv, xs);
    }
    const double xnorm2 = tq_block_sum(xs, red);
    const double alpha = A[(int64_t)r0 * ld + i];
    double ti = 0.0, beta = alpha, scal = 0.0;
    if (xnorm2 > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + xnorm2), alpha);
      ti = (beta - alpha) / beta;
      scal = 1.0 / (alpha - beta);
    }
    for (int t = tid; t < L; t += nt)
      v[t] = (t == 0) ? 1.0 : (xnorm2 > 0.0 ? A[(int64_t)(r0 + t) * ld + i] * scal : 0.0);
    if (tid == 0) {
      d[i] = A[(int64_t)i * ld + i];
      e[i] = beta;
      tau[i] = ti;
    }
    __syncthreads();
    if (ti != 0.0) {
      // p = tau A22 v as column sums (A22 is symmetric): per-wave partials
      // over its rows, then one thread per column adds the kTqWaves partials
      tq_colsum(A + (int64_t)r0 * ld + r0, ld, v, L, psc, m);
      __syncthreads();
      double pv = 0.0;
      for (int t = tid; t < L; t += nt) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += psc[w * m + t];
        s *= ti;
        pw[t] = s;
        pv = fma(s, v[t], pv);
      }
      const double ptv = tq_block_sum(pv, red);
      const double k = 0.5 * ti * ptv;
      for (int t = tid; t < L; t += nt) pw[t] -= k * v[t];   // w
      __syncthreads();
      // A22 -= v w^T + w v^T (four rows' loads issued before their stores:
      // the LDS accesses may alias, so the compiler keeps program order)
      for (int c = lane; c < L; c += 64) {
        const double pc = pw[c], vc = v[c];
        double* a = A + (int64_t)r0 * ld + r0 + c;
        int r = wave;
        for (; r + 3 * nw < L; r += 4 * nw) {
          double* a0 = a + (int64_t)r * ld;
          double* a1 = a0 + (int64_t)nw * ld;
          double* a2 = a1 + (int64_t)nw * ld;
          double* a3 = a2 + (int64_t)nw * ld;
          const double x0 = *a0, x1 = *a1, x2 = *a2, x3 = *a3;
          const double v0 = v[r], v1 = v[r + nw], v2 = v[r + 2 * nw], v3 = v[r + 3 * nw];
          const double w0 = pw[r], w1 = pw[r + nw], w2 = pw[r + 2 * nw], w3 = pw[r + 3 * nw];
          *a0 = x0 - (v0 * pc + w0 * vc);
          *a1 = x1 - (v1 * pc + w1 * vc);
          *a2 = x2 - (v2 * pc + w2 * vc);
          *a3 = x3 - (v3 * pc + w3 * vc);
        }
        for (; r < L; r += nw) a[(int64_t)r * ld] -= v[r] * pc + pw[r] * vc;
      }
    }
    // keep v (below its implicit unit head) in A[r0+1:, i] for step 2
    for (int t = tid + 1; t < L; t += nt) A[(int64_t)(r0 + t) * ld + i] = v[t];
    __syncthreads();
  }
  if (tid == 0) {
    if (m >= 2) {
      d[m - 2] = A[(int64_t)(m - 2) * ld + (m - 2)];
      e[m - 2] = A[(int64_t)(m - 1) * ld + (m - 2)];
      tau[m - 2] = 0.0;
    }
    d[m - 1] = A[(int64_t)(m - 1) * ld + (m - 1)];
    e[m - 1] = 0.0;
  }
  __syncthreads();

  stamp(1);
  if (kMode == 1) {
    // the reflectors out as rows (row i = v_i: 1 at column i + 1, A[r][i]
    // for r > i + 1, zeros elsewhere; rows m - 2, m - 1 have none), tau and
    // (d, e) to the work tail, eigenvalues by bisection.  The psc partials
    // (HBM variant) overlap the tau slot: both loops above ended in a barrier.
    double* R = Qout + offs[f];
    for (int r = wave; r < m; r += nw)
      for (int c = lane; c < m; c += 64)
        R[(int64_t)r * m + c] = (r + 2 >= m || c <= r) ? 0.0
                                : (c == r + 1 ? 1.0 : A[(int64_t)c * ld + r]);
    double* de = work + work_offs[f] + (int64_t)m * m;
    for (int i = tid; i < m; i += nt) {
      de[i] = d[i];
      de[m + i] = e[i];
      de[2 * m + i] = i + 2 < m ? tau[i] : 0.0;
    }
    tq_bisect(d, e, v, red, m, lam_out + lam_offs[f]);
    if (tid == 0) status[f] = 0;
    stamp(3);
    return;
  }
  // ---- 2. Z = H_0 H_1 ... H_{m-3}, backwards, into the same storage.  The
  // reflector vectors sit in the strictly-lower columns 0..m-3, below the
  // subdiagonal; Z's block for step i touches rows/cols > i only, and column
  // i's vector is consumed before column i is overwritten.
  // Z starts as the identity in rows/cols >= m-2 (no reflector there).
  for (int64_t q = tid; q < 4; q += nt) {
    const int r = m - 2 + (int)(q / 2), c = m - 2 + (int)(q % 2);
    if (r >= 0 && c >= 0) A[(int64_t)r * ld + c] = (r == c) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int i = m - 3; i >= 0; --i) {
    const int L = m - i - 1, r0 = i + 1;
    for (int t = tid; t < L; t += nt) v[t] = (t == 0) ? 1.0 : A[(int64_t)(r0 + t) * ld + i];
    __syncthreads();
    // the block Z[r0:, r0:] so far is Z[r0+1:, r0+1:] with row/col r0 = e_r0
    for (int t = tid; t < L; t += nt) {
      A[(int64_t)r0 * ld + r0 + t] = (t == 0) ? 1.0 : 0.0;
      if (t > 0) A[(int64_t)(r0 + t) * ld + r0] = 0.0;
    }
    __syncthreads();
    const double ti = tau[i];
    if (ti != 0.0) {
      // u[c] = tau sum_r v[r] Z[r0 + r][r0 + c]: per-wave column partials
      tq_colsum(A + (int64_t)r0 * ld + r0, ld, v, L, psc, m);
      __syncthreads();
      for (int t = tid; t < L; t += nt) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += psc[w * m + t];
        pw[t] = ti * s;
      }
      __syncthreads();
      for (int c = lane; c < L; c += 64) {
        const double pc = pw[c];
        double* z = A + (int64_t)r0 * ld + r0 + c;
        int r = wave;
        for (; r + 3 * nw < L; r += 4 * nw) {
          double* z0 = z + (int64_t)r * ld;
          double* z1 = z0 + (int64_t)nw * ld;
          double* z2 = z1 + (int64_t)nw * ld;
          double* z3 = z2 + (int64_t)nw * ld;
          const double x0 = *z0, x1 = *z1, x2 = *z2, x3 = *z3;
          const double v0 = v[r], v1 = v[r + nw], v2 = v[r + 2 * nw], v3 = v[r + 3 * nw];
          *z0 = x0 - v0 * pc;
          *z1 = x1 - v1 * pc;
          *z2 = x2 - v2 * pc;
          *z3 = x3 - v3 * pc;
        }
        for (; r < L; r += nw) z[(int64_t)r * ld] -= v[r] * pc;
      }
    }
    __syncthreads();
  }
  // row / column 0 of Z: e_0
  for (int t = tid; t < m; t += nt) {
    A[t] = (t == 0) ? 1.0 : 0.0;
    if (t > 0) A[(int64_t)t * ld] = 0.0;
  }
  __syncthreads();

  stamp(2);
  // ---- 3. implicit QL (tql2 / tqli) on (d, e) accumulating into Z's columns.
  // Wave 0 owns (d, e): it finds the next split point (ballot over its
  // lanes) and runs the sweep's scalar rotation chain (every lane computes
  // the same values in lockstep; lane 0 stores), writing (c, s) to buffer
  // k & 1.  Meanwhile waves 1.. apply sweep k-1's chain (buffer (k-1) & 1) to
  // their rows of Z -- the chains pipeline against the Z updates, one
  // barrier per sweep.
  const double eps = 2.220446049250313e-16;
  __shared__ int lo_b[2], hi_b[2], ql_done;
  if (tid == 0) {
    ql_done = 0;
    lo_b[0] = lo_b[1] = 0;
    hi_b[0] = hi_b[1] = 0;
  }
  __syncthreads();
  // the chain buffers: cs / sn hold buffer 0, pw / v hold buffer 1 (selected
  // per sweep, never through a pointer array: the stores must stay ds_write)
  // Wave 0's loop state is wave-uniform (readfirstlane): its branches are
  // scalar, and every lane runs the chain's arithmetic in lockstep.
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  int l = 0, iter = 0;   // wave-0 state
  int kswp = 0;
  for (int k = 0;; ++k) {
    kswp = k;
    if (wv == 0) {
      int mm = l;
      bool have = false;
      while (l < m && !bad) {
        // first split point mm >= l: |e[mm]| <= eps (|d[mm]| + |d[mm+1]|), or m - 1
        mm = m - 1;
        for (int base = l; base < m - 1; base += 64) {
          const int i = base + lane;
          const bool split = i < m - 1 &&
                             fabs(e[i]) <= eps * (fabs(d[i]) + fabs(d[i + 1]));
          const unsigned long long bal = __ballot(split);
          if (bal) {
            mm = base + __ffsll((long long)bal) - 1;
            break;
          }
        }
        mm = __builtin_amdgcn_readfirstlane(mm);
        if (mm == l) {   // d[l] converged
          ++l;
          iter = 0;
          continue;
        }
        have = true;
        break;
      }
      const int b = k & 1;
      if (!have) {
        if (lane == 0) {
          lo_b[b] = hi_b[b] = 0;
          ql_done = 1;
        }
      } else if (iter >= max_iter) {
        if (lane == 0) {
          bad = 1;
          lo_b[b] = hi_b[b] = 0;
          ql_done = 1;
        }
      } else {
        ++iter;
        double* cb = b ? pw : cs;
        double* sb = b ? v : sn;
        const double el = e[l], dl = d[l];
        double g = (d[l + 1] - dl) / (2.0 * el);
        double r = sqrt(fma(g, g, 1.0));
        g = d[mm] - dl + el / (g + copysign(r, g));
        double sv = 1.0, cv = 1.0, pv = 0.0;
        double dip1 = d[mm];            // d[i+1] before this step's update
        // operands e[i], d[i] of the step, of the next step, and two steps
        // ahead: three slots whose roles rotate (the loop is unrolled by
        // hand), so a load is consumed two steps after it is issued and no
        // register move waits on it.  Loads are clamped to l: unconditional.
        double ea = e[mm - 1], da = d[mm - 1];
        const int i2 = mm - 2 > l ? mm - 2 : l;
        double eb = e[i2], db = d[i2];
        double ec = 0.0, dc = 0.0;
        // lane 0 stores the chain's results; the other lanes store the same
        // values to their own dummy slot, so the stores need no exec branch and
        // the LDS counter waits stay exact
        const bool l0 = lane == 0;
        double* jk = junk + lane;
        int i = mm - 1;
        bool early = false;
        // one rotation: cur (ei, di) -> results; loads e/d[i - 2] into (en, dn)
        auto step = [&](double& ei, double& di, double& en, double& dn) -> bool {
          if (i < l) return false;
          const int i3 = i - 2 > l ? i - 2 : l;
          en = e[i3];
          dn = d[i3];
          const double fo = sv * ei, bb = cv * ei;
          const double bb2 = 2.0 * bb;
          const double h2 = fma(fo, fo, g * g);
          if (__builtin_amdgcn_readfirstlane(h2 == 0.0 ? 1 : 0)) {
            if (lane == 0) {
              e[i + 1] = 0.0;
              d[i + 1] = dip1 - pv;
              e[mm] = 0.0;
            }
            early = true;
            return false;
          }
          // 1/r by the hardware reciprocal square root and two Newton steps
          // (the chain's latency: no IEEE sqrt + divide sequences).  h2 is a
          // sum of squares of O(|A|) numbers, far from the f64 range limits.
          double y = __builtin_amdgcn_rsq(h2);
          double hh = h2 * y;
          y = fma(0.5 * y, fma(-hh, y, 1.0), y);
          hh = h2 * y;
          y = fma(0.5 * y, fma(-hh, y, 1.0), y);
          sv = fo * y;
          cv = g * y;
          g = dip1 - pv;
          r = fma(di - g, sv, cv * bb2);
          pv = sv * r;
          *(l0 ? &e[i + 1] : jk) = h2 * y;
          *(l0 ? &d[i + 1] : jk) = g + pv;
          *(l0 ? &cb[i] : jk) = cv;
          *(l0 ? &sb[i] : jk) = sv;
          g = fma(cv, r, -bb);
          dip1 = di;
          --i;
          return true;
        };
        for (;;) {
          if (!step(ea, da, ec, dc)) break;
          if (!step(eb, db, ea, da)) break;
          if (!step(ec, dc, eb, db)) break;
        }
        if (lane == 0) {
          lo_b[b] = early ? i + 1 : l;
          hi_b[b] = mm;
          if (!early) {
            d[l] = dl - pv;
            e[l] = g;
            e[mm] = 0.0;
          }
        }
      }
    } else if (k > 0) {
      // apply sweep k-1: rotations i = hi-1 .. lo on columns (i, i+1) of Z
      const int b = (k - 1) & 1;
      const int lo = lo_b[b], hi = hi_b[b];
      const double* cb = b ? pw : cs;
      const double* sb = b ? v : sn;
      for (int row = tid - 64; row < m && hi > lo; row += nt - 64) {
        double* Zr = A + (int64_t)row * ld;
        double cur = Zr[hi];
        // software pipelined: step i - 1's operands are loaded before step
        // i's store (Zr[i - 1] is not written by step i), so the carried
        // dependency is the two FMAs on cur, not an LDS round trip
        double zi = Zr[hi - 1], ci = cb[hi - 1], si = sb[hi - 1];
        for (int i = hi - 1; i >= lo; --i) {
          const int j = i > lo ? i - 1 : i;
          const double zn = Zr[j], cn = cb[j], sn_ = sb[j];
          Zr[i + 1] = fma(si, zi, ci * cur);
          cur = fma(ci, zi, -si * cur);
          zi = zn;
          ci = cn;
          si = sn_;
        }
        Zr[lo] = cur;
      }
    }
    __syncthreads();
    if (ql_done) break;
  }
  __syncthreads();
  stamp(3);
  if (stamps != nullptr && tid < 64) stamps[((int64_t)f * 8 + 6) * 64 + tid] = kswp;
  // ---- 4. ascending order (parallel rank, ties by index) and output
  for (int i = tid; i < m; i += nt) {
    int r = 0;
    const double di = d[i];
    for (int j = 0; j < m; ++j) r += (d[j] < di || (d[j] == di && j < i)) ? 1 : 0;
    rank[i] = r;
  }
  __syncthreads();
  double* Q = Qout + offs[f];
  double* lam = lam_out + lam_offs[f];
  for (int i = tid; i < m; i += nt) lam[rank[i]] = d[i];
  for (int r = wave; r < m; r += nw)
    for (int c = lane; c < m; c += 64) Q[(int64_t)r * m + rank[c]] = A[(int64_t)r * ld + c];
  if (tid == 0) status[f] = bad;
  stamp(4);
}

// Selected eigenvectors of the tridiagonal T = (d, e) by inverse iteration
// (LAPACK dstein's scheme without its cluster reorthogonalisation: the host
// only takes this path when every selected eigenvalue is separated from its
// neighbours, so the vectors come out orthogonal to ~eps ||T|| / gap).
// One wave per job (a factor and up to kInvB of its selected eigenvalues),
// one lane per eigenvalue lambda: LU of T - lambda I with partial pivoting
// (U with two superdiagonals), three solves from a pseudo-random start (the
// grid factors are centrosymmetric: a symmetric start would miss every odd
// eigenvector), scaled by the max norm each time; output the unit vector y
// (largest component positive) as a row of Y.  The per-lane arrays live in
// LDS, interleaved by lane.
constexpr int kInvThreads = 64;

__global__ __launch_bounds__(kInvThreads) void tridiag_invit_kernel(
    const int* __restrict__ job_f, const int* __restrict__ job_s0, const int* __restrict__ job_n,
    const int64_t* __restrict__ dims, const int64_t* __restrict__ de_offs,
    const double* __restrict__ work, const double* __restrict__ lam,
    const int64_t* __restrict__ lam_offs, const int* __restrict__ sel,
    const int64_t* __restrict__ sel_offs, const int64_t* __restrict__ y_offs,
    double* __restrict__ Y, int B) {
  extern __shared__ __attribute__((aligned(16))) double iv[];
  const int job = blockIdx.x;
  const int f = job_f[job];
  const int m = (int)dims[f];
  const int v = threadIdx.x;
  if (v >= job_n[job]) return;
  const double* d = work + de_offs[f];
  const double* e = d + m;
  const int s = job_s0[job] + v;                       // global selection index
  const int local = s - (int)sel_offs[f];
  const double lmb = lam[lam_offs[f] + sel[s]];
  // lane-interleaved LDS arrays: u0, u1, u2, lm, pv, y
  auto at = [&](int a, int i) -> double& { return iv[((int64_t)a * m + i) * B + v]; };
  double tn = 0.0;   // ||T||_inf
  for (int i = 0; i < m; ++i)
    tn = fmax(tn, fabs(d[i]) + (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < m - 1 ? fabs(e[i]) : 0.0));
  const double tiny = fmax(2.220446049250313e-16 * tn, 1e-300);
  auto guard = [&](double p) { return fabs(p) < tiny ? (p < 0.0 ? -tiny : tiny) : p; };
  // ---- LU with partial pivoting of T - lambda I
  double p = d[0] - lmb, q = m > 1 ? e[0] : 0.0, r = 0.0;
  for (int i = 0; i + 1 < m; ++i) {
    const double c = e[i], an = d[i + 1] - lmb, bn = (i + 2 < m) ? e[i + 1] : 0.0;
    if (fabs(p) >= fabs(c)) {
      const double pg = guard(p);
      const double mult = c / pg;
      at(0, i) = pg;
      at(1, i) = q;
      at(2, i) = r;
      at(3, i) = mult;
      at(4, i) = 0.0;
      p = an - mult * q;
      q = bn - mult * r;
    } else {
      const double mult = p / c;
      at(0, i) = c;
      at(1, i) = an;
      at(2, i) = bn;
      at(3, i) = mult;
      at(4, i) = 1.0;
      p = q - mult * an;
      q = r - mult * bn;
    }
    r = 0.0;
  }
  at(0, m - 1) = guard(p);
  at(1, m - 1) = 0.0;
  at(2, m - 1) = 0.0;
  // ---- start vector: hashed, in (-1, 1)
  for (int i = 0; i < m; ++i) {
    unsigned h = (unsigned)i * 2654435761u ^ ((unsigned)(sel[s] + 1) * 40503u);
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    at(5, i) = (double)(h >> 8) * (1.0 / 8388608.0) - 1.0;
  }
  for (int it = 0; it < 3; ++it) {
    // forward: the row operations of the factorisation on y
    for (int i = 0; i + 1 < m; ++i) {
      double yi = at(5, i), yn = at(5, i + 1);
      if (at(4, i) != 0.0) {
        const double t = yi;
        yi = yn;
        yn = t;
      }
      at(5, i) = yi;
      at(5, i + 1) = yn - at(3, i) * yi;
    }
    // back substitution with U (diag, two superdiagonals)
    double y1 = 0.0, y2 = 0.0, ymax = 0.0;
    for (int i = m - 1; i >= 0; --i) {
      const double yi = (at(5, i) - at(1, i) * y1 - at(2, i) * y2) / at(0, i);
      at(5, i) = yi;
      y2 = y1;
      y1 = yi;
      ymax = fmax(ymax, fabs(yi));
    }
    const double sc = ymax > 0.0 ? 1.0 / ymax : 1.0;
    for (int i = 0; i < m; ++i) at(5, i) *= sc;
  }
  double nrm = 0.0, big = 0.0;
  int ib = 0;
  for (int i = 0; i < m; ++i) {
    const double yi = at(5, i);
    nrm = fma(yi, yi, nrm);
    if (fabs(yi) > big) {
      big = fabs(yi);
      ib = i;
    }
  }
  const double sc = (at(5, ib) < 0.0 ? -1.0 : 1.0) / sqrt(nrm);
  double* yo = Y + y_offs[f] + (int64_t)local * m;
  for (int i = 0; i < m; ++i) yo[i] = at(5, i) * sc;
}

// Eigenvectors of A from those of its tridiagonal: y <- H_i y = y - tau_i
// (v_i . y) v_i for i = m - 3 .. 0, in place on rows of Y.  One workgroup per
// (factor, up to kBtWaves rows), one wave per row (its y in LDS, lanes over
// the row, a shuffle reduction per reflector); the reflector rows are staged
// through LDS in chunks of ch rows shared by the waves.  Work per row: m^2
// FMAs in m - 2 dependent steps, against forming Z (m^3 / 3 behind barriers)
// and the GEMM Y Z^T it replaces.
constexpr int kBtWaves = 8;

__global__ __launch_bounds__(kBtWaves * 64) void tridiag_backtransform_kernel(
    const int* __restrict__ job_f, const int* __restrict__ job_r0, const int* __restrict__ job_n,
    const int64_t* __restrict__ dims, const int64_t* __restrict__ tau_offs,
    const int64_t* __restrict__ r_offs, const int64_t* __restrict__ y_offs,
    const double* __restrict__ work, const double* __restrict__ R, double* Y, int ch) {
  extern __shared__ __attribute__((aligned(16))) double bt[];
  const int job = blockIdx.x;
  const int f = job_f[job];
  const int m = (int)dims[f];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool act = wave < job_n[job];
  const double* tau = work + tau_offs[f];
  const double* Rf = R + r_offs[f];
  double* yrow = Y + y_offs[f] + (int64_t)(job_r0[job] + (act ? wave : 0)) * m;
  double* yw = bt + wave * m;
  double* rc = bt + kBtWaves * m;
  if (act)
    for (int c = lane; c < m; c += 64) yw[c] = yrow[c];
  for (int hi = m - 3; hi >= 0; hi -= ch) {
    const int lo = hi - ch + 1 > 0 ? hi - ch + 1 : 0;
    __syncthreads();   // the previous chunk is consumed
    for (int i = lo + wave; i <= hi; i += kBtWaves)
      for (int c = lane; c < m; c += 64) rc[(int64_t)(i - lo) * m + c] = Rf[(int64_t)i * m + c];
    __syncthreads();
    if (!act) continue;
    for (int i = hi; i >= lo; --i) {
      const double ti = tau[i];
      if (ti == 0.0) continue;
      const double* v = rc + (int64_t)(i - lo) * m;
      double s = 0.0;
      for (int c = i + 1 + lane; c < m; c += 64) s = fma(v[c], yw[c], s);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      s *= ti;
      for (int c = i + 1 + lane; c < m; c += 64) yw[c] = fma(-s, v[c], yw[c]);
    }
  }
  if (act)
    for (int c = lane; c < m; c += 64) yrow[c] = yw[c];
}

// Orthonormalise the rows of V (k x m, row-major) in place by classical
// Gram-Schmidt applied twice ("CGS2"), last row first: row v loses its
// components along rows v+1 .. k-1, twice, then is normalised.  One workgroup
// per matrix; the dot products split over (row, column stripe) and reduce
// through LDS, so each row costs a handful of barriers.  Used on inverse
// iteration's eigenvectors, which are already orthogonal to ~eps ||T|| / gap:
// the second pass takes the result to ~eps.
constexpr int kOrthoThreads = 256;

__global__ __launch_bounds__(kOrthoThreads) void rows_orthonormalize_kernel(
    const int64_t* __restrict__ ks, const int64_t* __restrict__ ms,
    const int64_t* __restrict__ offs, double* __restrict__ Vall) {
  __shared__ double cdot[kOrthoThreads];
  __shared__ double red[kOrthoThreads / 64];
  const int f = blockIdx.x;
  const int k = (int)ks[f], m = (int)ms[f];
  double* V = Vall + offs[f];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int v = k - 1; v >= 0; --v) {
    double* Vv = V + (int64_t)v * m;
    const int nw = k - 1 - v;   // rows already orthonormal: v+1 .. k-1
    for (int pass = 0; pass < 2 && nw > 0; ++pass) {
      // c_w = V_w . V_v: thread group per row w (up to nt rows at a time)
      for (int w0 = 0; w0 < nw; w0 += nt) {
        const int nrow = min(nt, nw - w0);
        const int tpr = max(1, nt / nrow) >= 64 ? 64 : (nt / nrow >= 32 ? 32 :
                        nt / nrow >= 16 ? 16 : nt / nrow >= 8 ? 8 : nt / nrow >= 4 ? 4 :
                        nt / nrow >= 2 ? 2 : 1);
        const int w = w0 + tid / tpr, l = tid % tpr;
        double acc = 0.0;
        if (tid / tpr < nrow) {
          const double* Vw = V + (int64_t)(v + 1 + w) * m;
          for (int i = l; i < m; i += tpr) acc = fma(Vw[i], Vv[i], acc);
        }
        for (int off = tpr >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        __syncthreads();
        if (tid / tpr < nrow && l == 0) cdot[tid / tpr] = acc;
        __syncthreads();
        // V_v -= sum_w c_w V_w over this batch of rows
        for (int i = tid; i < m; i += nt) {
          double s = Vv[i];
          for (int ww = 0; ww < nrow; ++ww)
            s = fma(-cdot[ww], V[(int64_t)(v + 1 + w0 + ww) * m + i], s);
          Vv[i] = s;
        }
        __syncthreads();
      }
    }
    // normalise
    double ss = 0.0;
    for (int i = tid; i < m; i += nt) ss = fma(Vv[i], Vv[i], ss);
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    double tot = 0.0;
    for (int q = 0; q < nt / 64; ++q) tot += red[q];
    const double inv = tot > 0.0 ? 1.0 / sqrt(tot) : 1.0;
    for (int i = tid; i < m; i += nt) Vv[i] *= inv;
    __syncthreads();
  }
}

// work doubles per factor: the HBM copy of A / Z (m x m), then (d, e, tau)
// of the eigenvalue-only mode or the HBM variant's column partials
// (kTqWaves m; the two are never live together), or Jacobi's 2 m^2
inline int64_t eig_work_per(int64_t m) { return std::max(2 * m * m, m * m + (2 + kTqWaves) * m); }

// Full-length eigenvectors of centrosymmetric factors from their half-order
// problems (tensors.centro_halves): factor f's rows r < ke are [y; J y] / sqrt 2
// of the even half's row r, rows ke + r are [y; -J y] / sqrt 2 of the odd
// half's row r.  In: per factor the even block (ke x h) then the odd block
// (ko x h); out: (ke + ko) x 2h per factor.  One launch for up to kCentroMax
// factors (parameters by value), blockIdx.y = factor.
constexpr int kCentroMax = 32;
struct CentroBatch {
  int nf;
  int64_t h[kCentroMax], ke[kCentroMax], ko[kCentroMax], in[kCentroMax], out[kCentroMax];
};

__global__ __launch_bounds__(256) void centro_expand_kernel(CentroBatch B,
                                                            const double* __restrict__ V,
                                                            double* __restrict__ out) {
  const int f = blockIdx.y;
  const int64_t h = B.h[f], m = 2 * h, k = B.ke[f] + B.ko[f];
  const double c = 0.70710678118654752440;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < k * m;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / m, col = e - r * m;
    const bool odd = r >= B.ke[f];
    const int64_t src = B.in[f] + r * h;   // the odd block follows the even one
    const double y = col < h ? V[src + col] : V[src + (m - 1 - col)];
    out[B.out[f] + e] = (col >= h && odd) ? -c * y : c * y;
  }
}

}  // namespace gg

extern "C" {

int gg_sym_eig_work_elems(int count, const int64_t* m, int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(count >= 0 && elems, GG_ERR_VALUE, "bad argument");
    int64_t e = 0;
    for (int i = 0; i < count; ++i) e += gg::eig_work_per(m[i]);
    *elems = e;
  });
}

int gg_sym_eig_batched(int count, const int64_t* m, const double* A_dev, double* Q_dev,
                       double* lam_dev, double* work_dev, int64_t work_elems, int max_sweeps,
                       gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(count >= 1 && m && A_dev && Q_dev && lam_dev && work_dev, GG_ERR_VALUE,
               "bad argument");
    std::vector<int64_t> meta(5 * (size_t)count);
    int64_t off = 0, loff = 0, woff = 0;
    for (int i = 0; i < count; ++i) {
      GG_REQUIRE(m[i] >= 1 && m[i] <= 2048, GG_ERR_VALUE, "factor size must be in [1, 2048]");
      meta[i] = m[i];
      meta[count + i] = off;
      meta[2 * count + i] = loff;
      meta[3 * count + i] = woff;
      off += m[i] * m[i];
      loff += m[i];
      woff += gg::eig_work_per(m[i]);
    }
    GG_REQUIRE(work_elems >= woff, GG_ERR_VALUE, "eigensolver work buffer too small");
    hipStream_t s = gg::as_stream(stream);
    int64_t* dmeta = nullptr;
    GG_HIP(hipMallocAsync(&dmeta, meta.size() * sizeof(int64_t), s));
    GG_HIP(hipMemcpyAsync(dmeta, meta.data(), meta.size() * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    int* dstatus = reinterpret_cast<int*>(dmeta + 4 * count);
    int mmax = 1;
    for (int i = 0; i < count; ++i) mmax = std::max<int>(mmax, (int)m[i]);
    const bool lds_a = mmax <= gg::kLdsMaxM;
    // tridiagonalisation + implicit QL (default), or the round-robin Jacobi
    // (GG_EIG=jacobi: reference implementation kept for A/B)
    const char* ev = gg::knob("GG_EIG");
    const bool jacobi = ev != nullptr && std::string(ev) == "jacobi";
    long long* dstamps = nullptr;
    const bool prof = gg::knob("GG_EIG_PROF") != nullptr;
    if (!jacobi && prof) {
      GG_HIP(hipMallocAsync(&dstamps, 8 * 64 * sizeof(long long) * count, s));
      GG_HIP(hipMemsetAsync(dstamps, 0, 8 * 64 * sizeof(long long) * count, s));
    }
    if (!jacobi) {
      const int64_t head = gg::tq_head_bytes(mmax, lds_a);
      const int64_t lds = head + (lds_a ? (int64_t)mmax * (mmax + 1) * sizeof(double) : 0);
      const int iters = std::max(30, max_sweeps);
      if (lds_a) {
        GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_ql_kernel<true, 0>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((gg::tridiag_ql_kernel<true, 0>), dim3(count), dim3(gg::kTqThreads), lds, s,
                           dmeta, dmeta + count, A_dev, Q_dev, lam_dev, dmeta + 2 * count,
                           work_dev, dmeta + 3 * count, iters, dstatus, dstamps);
      } else {
        GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_ql_kernel<false, 0>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((gg::tridiag_ql_kernel<false, 0>), dim3(count), dim3(gg::kTqThreads), lds,
                           s, dmeta, dmeta + count, A_dev, Q_dev, lam_dev, dmeta + 2 * count,
                           work_dev, dmeta + 3 * count, iters, dstatus, dstamps);
      }
    } else {
      const int64_t lds = gg::eig_lds_bytes(mmax, lds_a);
      if (lds_a) {
        GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::jacobi_kernel<true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(gg::jacobi_kernel<true>, dim3(count), dim3(gg::kEigThreads), lds, s,
                           dmeta, dmeta + count, A_dev, Q_dev, lam_dev, dmeta + 2 * count,
                           work_dev, dmeta + 3 * count, max_sweeps, dstatus);
      } else {
        hipLaunchKernelGGL(gg::jacobi_kernel<false>, dim3(count), dim3(gg::kEigThreads), lds, s,
                           dmeta, dmeta + count, A_dev, Q_dev, lam_dev, dmeta + 2 * count,
                           work_dev, dmeta + 3 * count, max_sweeps, dstatus);
      }
    }
    GG_LAUNCH_CHECK();
    std::vector<int> st(count);
    GG_HIP(hipMemcpyAsync(st.data(), dstatus, count * sizeof(int), hipMemcpyDeviceToHost, s));
    GG_HIP(hipFreeAsync(dmeta, s));
    GG_HIP(hipStreamSynchronize(s));
    if (dstamps) {
      std::vector<long long> h64(8 * 64 * (size_t)count), h(8 * (size_t)count);
      GG_HIP(hipMemcpy(h64.data(), dstamps, h64.size() * sizeof(long long),
                       hipMemcpyDeviceToHost));
      for (size_t q = 0; q < h.size(); ++q) h[q] = h64[q * 64];
      GG_HIP(hipFree(dstamps));
      for (int i = 0; i < count; ++i)
        fprintf(stderr,
                "eig m=%lld phases(us at 100MHz): tridiag %.1f form-Q %.1f QL %.1f sort %.1f "
                "sweeps %lld\n",
                (long long)m[i], (h[8 * i + 1] - h[8 * i]) / 100.0,
                (h[8 * i + 2] - h[8 * i + 1]) / 100.0, (h[8 * i + 3] - h[8 * i + 2]) / 100.0,
                (h[8 * i + 4] - h[8 * i + 3]) / 100.0, h[8 * i + 6]);
    }
    for (int i = 0; i < count; ++i)
      GG_REQUIRE(st[i] == 0, GG_ERR_LINALG,
                 "eigensolver did not converge on factor " + std::to_string(i));
  });
}


int gg_sym_eig_tridiag(int count, const int64_t* m, const double* A_dev, double* Z_dev,
                       double* lam_dev, double* work_dev, int64_t work_elems, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(count >= 1 && m && A_dev && Z_dev && lam_dev && work_dev, GG_ERR_VALUE,
               "bad argument");
    std::vector<int64_t> meta(5 * (size_t)count, 0);
    int64_t off = 0, loff = 0, woff = 0;
    int mmax = 1;
    for (int i = 0; i < count; ++i) {
      GG_REQUIRE(m[i] >= 1 && m[i] <= 2048, GG_ERR_VALUE, "factor size must be in [1, 2048]");
      meta[i] = m[i];
      meta[count + i] = off;
      meta[2 * count + i] = loff;
      meta[3 * count + i] = woff;
      off += m[i] * m[i];
      loff += m[i];
      woff += gg::eig_work_per(m[i]);
      mmax = std::max<int>(mmax, (int)m[i]);
    }
    GG_REQUIRE(work_elems >= woff, GG_ERR_VALUE, "eigensolver work buffer too small");
    hipStream_t s = gg::as_stream(stream);
    int64_t* dmeta = nullptr;
    GG_HIP(hipMallocAsync(&dmeta, meta.size() * sizeof(int64_t), s));
    GG_HIP(hipMemcpyAsync(dmeta, meta.data(), meta.size() * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    int* dstatus = reinterpret_cast<int*>(dmeta + 4 * count);
    const bool lds_a = mmax <= gg::kLdsMaxM;
    const int64_t head = gg::tq_head_bytes(mmax, lds_a);
    const int64_t lds = head + (lds_a ? (int64_t)mmax * (mmax + 1) * sizeof(double) : 0);
    if (lds_a) {
      GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_ql_kernel<true, 1>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL((gg::tridiag_ql_kernel<true, 1>), dim3(count), dim3(gg::kTqThreads), lds,
                         s, dmeta, dmeta + count, A_dev, Z_dev, lam_dev, dmeta + 2 * count,
                         work_dev, dmeta + 3 * count, 0, dstatus, nullptr);
    } else {
      GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_ql_kernel<false, 1>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL((gg::tridiag_ql_kernel<false, 1>), dim3(count), dim3(gg::kTqThreads), lds,
                         s, dmeta, dmeta + count, A_dev, Z_dev, lam_dev, dmeta + 2 * count,
                         work_dev, dmeta + 3 * count, 0, dstatus, nullptr);
    }
    GG_LAUNCH_CHECK();
    GG_HIP(hipFreeAsync(dmeta, s));
  });
}

int gg_sym_eig_tridiag_vectors(int count, const int64_t* m, const double* R_dev,
                               const double* work_dev, int64_t work_elems, const double* lam_dev,
                               const int* nsel, const int* sel, double* Y_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(count >= 1 && m && R_dev && work_dev && lam_dev && nsel && sel && Y_dev,
               GG_ERR_VALUE, "bad argument");
    // per factor: m, (d, e) offset, lambda offset, selection offset, Y offset,
    // tau offset, reflector offset
    std::vector<int64_t> fm(7 * (size_t)count);
    int64_t woff = 0, loff = 0, soff = 0, yoff = 0, roff = 0;
    int mmax = 1;
    for (int i = 0; i < count; ++i) {
      GG_REQUIRE(m[i] >= 1 && m[i] <= 2048 && nsel[i] >= 0 && nsel[i] <= m[i], GG_ERR_VALUE,
                 "bad selection");
      for (int k = 0; k < nsel[i]; ++k)
        GG_REQUIRE(sel[soff + k] >= 0 && sel[soff + k] < m[i], GG_ERR_VALUE,
                   "selected index out of range");
      fm[i] = m[i];
      fm[count + i] = woff + m[i] * m[i];
      fm[2 * count + i] = loff;
      fm[3 * count + i] = soff;
      fm[4 * count + i] = yoff;
      fm[5 * count + i] = woff + m[i] * m[i] + 2 * m[i];
      fm[6 * count + i] = roff;
      roff += m[i] * m[i];
      woff += gg::eig_work_per(m[i]);
      loff += m[i];
      soff += nsel[i];
      yoff += (int64_t)nsel[i] * m[i];
      mmax = std::max<int>(mmax, (int)m[i]);
    }
    GG_REQUIRE(work_elems >= woff, GG_ERR_VALUE, "eigensolver work buffer too small");
    if (soff == 0) return;
    // lanes per wave: the interleaved per-lane arrays (6 m doubles) fit LDS
    const int B = (int)std::max<int64_t>(
        1, std::min<int64_t>(gg::kInvThreads, (150 * 1024) / (6 * (int64_t)mmax * 8)));
    std::vector<int> jf, js, jn;
    for (int i = 0, s0 = 0; i < count; s0 += nsel[i], ++i)
      for (int k = 0; k < nsel[i]; k += B) {
        jf.push_back(i);
        js.push_back(s0 + k);
        jn.push_back(std::min(B, nsel[i] - k));
      }
    const int njobs = (int)jf.size();
    // back-transform jobs: up to kBtWaves rows of one factor
    std::vector<int> bf, br, bn;
    for (int i = 0; i < count; ++i)
      for (int k = 0; k < nsel[i]; k += gg::kBtWaves) {
        bf.push_back(i);
        br.push_back(k);
        bn.push_back(std::min(gg::kBtWaves, nsel[i] - k));
      }
    const int nbt = (int)bf.size();
    // one device block: int64 factor table, then int job tables and selection
    const size_t bytes =
        fm.size() * sizeof(int64_t) + (3 * (size_t)njobs + soff + 3 * (size_t)nbt) * sizeof(int);
    hipStream_t s = gg::as_stream(stream);
    unsigned char* dbuf = nullptr;
    GG_HIP(hipMallocAsync(&dbuf, bytes, s));
    std::vector<unsigned char> hbuf(bytes);
    memcpy(hbuf.data(), fm.data(), fm.size() * sizeof(int64_t));
    int* ip = reinterpret_cast<int*>(hbuf.data() + fm.size() * sizeof(int64_t));
    memcpy(ip, jf.data(), njobs * sizeof(int));
    memcpy(ip + njobs, js.data(), njobs * sizeof(int));
    memcpy(ip + 2 * njobs, jn.data(), njobs * sizeof(int));
    memcpy(ip + 3 * njobs, sel, soff * sizeof(int));
    int* bp = ip + 3 * njobs + soff;
    memcpy(bp, bf.data(), nbt * sizeof(int));
    memcpy(bp + nbt, br.data(), nbt * sizeof(int));
    memcpy(bp + 2 * nbt, bn.data(), nbt * sizeof(int));
    GG_HIP(hipMemcpyAsync(dbuf, hbuf.data(), bytes, hipMemcpyHostToDevice, s));
    const int64_t* dfm = reinterpret_cast<const int64_t*>(dbuf);
    const int* dip = reinterpret_cast<const int*>(dbuf + fm.size() * sizeof(int64_t));
    const size_t lds = (size_t)6 * mmax * B * sizeof(double);
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_invit_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(gg::tridiag_invit_kernel, dim3(njobs), dim3(gg::kInvThreads), lds, s, dip,
                       dip + njobs, dip + 2 * njobs, dfm, dfm + count, work_dev, lam_dev,
                       dfm + 2 * count, dip + 3 * njobs, dfm + 3 * count, dfm + 4 * count, Y_dev,
                       B);
    GG_LAUNCH_CHECK();
    // reflector rows staged per chunk: kBtWaves y rows + ch reflector rows of
    // LDS (at most 144 KB)
    const int ch = std::max(1, std::min(64, 18432 / mmax - gg::kBtWaves));
    const size_t bt_lds = (size_t)(gg::kBtWaves + ch) * mmax * sizeof(double);
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&gg::tridiag_backtransform_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)bt_lds));
    const int* dbp = dip + 3 * njobs + soff;
    hipLaunchKernelGGL(gg::tridiag_backtransform_kernel, dim3(nbt), dim3(gg::kBtWaves * 64),
                       bt_lds, s, dbp, dbp + nbt, dbp + 2 * nbt, dfm, dfm + 5 * count,
                       dfm + 6 * count, dfm + 4 * count, work_dev, R_dev, Y_dev, ch);
    GG_LAUNCH_CHECK();
    GG_HIP(hipFreeAsync(dbuf, s));
  });
}


int gg_centro_expand(int nf, const int64_t* h, const int64_t* ke, const int64_t* ko,
                     const double* V_dev, double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(nf >= 1 && h && ke && ko && V_dev && out_dev, GG_ERR_VALUE, "bad argument");
    hipStream_t s = gg::as_stream(stream);
    int64_t in = 0, out = 0;
    for (int f0 = 0; f0 < nf; f0 += gg::kCentroMax) {
      gg::CentroBatch B;
      B.nf = std::min(gg::kCentroMax, nf - f0);
      int64_t maxel = 1;
      for (int j = 0; j < B.nf; ++j) {
        const int f = f0 + j;
        GG_REQUIRE(h[f] >= 1 && ke[f] >= 0 && ko[f] >= 0 && ke[f] + ko[f] <= 2 * h[f],
                   GG_ERR_VALUE, "bad half block");
        B.h[j] = h[f];
        B.ke[j] = ke[f];
        B.ko[j] = ko[f];
        B.in[j] = in;
        B.out[j] = out;
        in += (ke[f] + ko[f]) * h[f];
        out += (ke[f] + ko[f]) * 2 * h[f];
        maxel = std::max(maxel, (ke[f] + ko[f]) * 2 * h[f]);
      }
      dim3 grid((unsigned)gg::ceil_div(maxel, 256), (unsigned)B.nf);
      hipLaunchKernelGGL(gg::centro_expand_kernel, grid, dim3(256), 0, s, B, V_dev, out_dev);
      GG_LAUNCH_CHECK();
    }
  });
}

int gg_rows_orthonormalize(int count, const int64_t* k, const int64_t* m, double* V_dev,
                           gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(count >= 1 && k && m && V_dev, GG_ERR_VALUE, "bad argument");
    std::vector<int64_t> meta(3 * (size_t)count);
    int64_t off = 0;
    for (int i = 0; i < count; ++i) {
      GG_REQUIRE(k[i] >= 0 && m[i] >= 1 && k[i] <= m[i], GG_ERR_VALUE, "bad row block");
      meta[i] = k[i];
      meta[count + i] = m[i];
      meta[2 * count + i] = off;
      off += k[i] * m[i];
    }
    hipStream_t s = gg::as_stream(stream);
    int64_t* dmeta = nullptr;
    GG_HIP(hipMallocAsync(&dmeta, meta.size() * sizeof(int64_t), s));
    GG_HIP(hipMemcpyAsync(dmeta, meta.data(), meta.size() * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(gg::rows_orthonormalize_kernel, dim3(count), dim3(gg::kOrthoThreads), 0,
                       s, dmeta, dmeta + count, dmeta + 2 * count, V_dev);
    GG_LAUNCH_CHECK();
    GG_HIP(hipFreeAsync(dmeta, s));
  });
}

}  // extern "C"
