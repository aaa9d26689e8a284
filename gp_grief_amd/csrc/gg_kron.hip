// Kronecker operator on MI355X: y = (K_0 (x) ... (x) K_{d-1}) x as a chain of
// FP64 MFMA GEMMs (v_mfma_f64_16x16x4_f64) with LDS-staged factor fragments.
//
// Reference: KronMatrix.kronvec_prod, gp_grief/tensors/kron_matrix.py:52-97.
// The reference reshapes in Fortran order and lets BLAS3 dsymm/dgemm apply one
// factor at a time, transposing the result so the tensor axes rotate.  Here
// every step is the same batched-free GEMM
//
//     Y[b, j] = sum_i X[i, b] * K[j, i]        X: q x M row-major (ld M)
//                                              Y: M x p row-major
//
// i.e. "contract the slowest axis, append the new axis as the fastest".  After
// d steps the axes are back in C order, so no transpose pass ever touches HBM.
//
// Work decomposition (one step):
//   * a wave owns a 16-row strip b0..b0+15 of Y and all p output columns
//     (JT = ceil(p/16) accumulators of 16x16, 4 f64 per lane each);
//   * the A operand (X^T, one f64 per lane per k-step) streams from HBM
//     exactly once: lane l loads X[4ks + (l>>4), b0 + (l&15)] -- four 128-B
//     row segments per wave instruction;
//   * the B operand (K^T) is pre-packed on the host in MFMA fragment order
//     [ks][jt][lane] so a k-chunk is one contiguous block; a workgroup of WAVES
//     waves stages KC k-steps of it in LDS and every wave reads its fragment
//     with one conflict-free ds_read_b64 per MFMA;
//   * epilogue: D[b][j] sits at lane (j & 15), register r = row 4r + (l>>4):
//     four 128-B segments per store.  The last step can fuse y += shift * x
//     and the partial dot x.y (the CG p.q) per workgroup.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gg_mp.h"

namespace gg {

constexpr int kMaxJT = 16;  // accumulator tiles per launch (<= 256 output columns)
constexpr int kEpiBatch = 4;  // epilogue tiles whose x loads are issued together

// Epilogue shared by the mode-product kernels: store D (+ shift * x, CG dot
// partials), per-workgroup partial sums, and the fused-CG side job.  Called
// after the k-loop's last barrier (LDS is free).
// blk: the output block (strip group) index of the partial sums and the side
// job slice.  kRaw: the reduction barrier is a raw s_barrier (LDS DMAs of the
// next strip may be in flight, cdna_hip_programming.md "Pipelining across
// barriers"); red: 4 * kWaves doubles of LDS scratch outside any DMA target.
// value of lane l ^ 1 (DPP quad_perm [1,0,3,2] on both 32-bit halves)
__device__ __forceinline__ double swap_lane_pair(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// kWide: plain stores as 16-byte pairs.  The MFMA result puts one column per
// lane; a 2x2 exchange between lanes l and l ^ 1 gives the even lane rows
// 0 / 2 and the odd lane rows 1 / 3 of two adjacent columns, so each lane
// stores two double2 instead of four doubles per tile (needs p even and Y
// 16-byte aligned, checked at run time).
template <int JT, int kWaves, int kSplit, bool kIdent, int kEpi, int CGP, bool kRaw = false,
          int kBatch = kEpiBatch, bool kWide = false>
__device__ __forceinline__ void mp_finish(const d4 (&acc)[JT], double* __restrict__ Y, int64_t M,
                                          int p, int jt0, const double* __restrict__ xs,
                                          double shift, double* __restrict__ dot_partials,
                                          const OutMap& om, const MpFuse& fz, double rr_acc,
                                          int64_t b0, int hp, double* red, int64_t blk,
                                          double pqo_acc = 0.0) {
  constexpr int kThreads = kWaves * 64;
  const int lane = threadIdx.x & 63;
  // ---- epilogue: D[b][j] at lane (j & 15), register r = row 4r + (lane >> 4).
  // Output address = rowoff(row) + coloff(j): the identity map is row * p + j;
  // the distributed matvec permutes rows / columns into all-to-all order
  // (OutMap, gg_dist.hip).  Offsets are decomposed once per row and column.
  const int col = lane & 15;
  const int64_t rbase = b0 + (lane >> 4);
  int64_t rowoff[4];
  int rowdest[4];
  bool rowok[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = rbase + 4 * r;
    rowok[r] = row < M;
    rowdest[r] = 0;
    if (kIdent) {
      rowoff[r] = row * p;
    } else {
      const int64_t a_ = row / om.mi, bi = row - a_ * om.mi;
      const int64_t h = bi / om.cr, br = bi - h * om.cr;
      rowoff[r] = a_ * om.as + br * om.cg;
      if (om.push == 1) rowdest[r] = (int)h;
      else rowoff[r] += h * om.hs;
    }
  }
  auto colj = [&](int t) -> int64_t { return (int64_t)(jt0 + hp * JT + t) * 16 + col; };
  auto coloff = [&](int t) -> int64_t {
    const int64_t j = colj(t);
    if (kIdent) return j;
    const int64_t jg = j / om.cg;
    return jg * om.gs + (j - jg * om.cg);
  };
  if (!kIdent && om.push != 0) {
    // sharded matvec, push mode (gg_kron_dist_*_push): each element goes
    // straight to its destination rank's buffer (peer memory over xGMI) at
    // this rank's chunk -- the all-to-all is the epilogue's own stores
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const int64_t j = colj(t);
      if (j >= p) continue;
      const int64_t jg = j / om.cg;
      const int64_t co = (j - jg * om.cg) + (om.push == 2 ? 0 : jg * om.gs);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!rowok[r]) continue;
        const int dest = om.push == 1 ? rowdest[r] : (int)jg;
        om.peers[dest][om.self_off + rowoff[r] + co] = acc[t][r];
      }
    }
    // the stores went to other GPUs' HBM over xGMI: release them at system
    // scope before the kernel ends, so the stream-ordered barrier that follows
    // (an RCCL all-reduce) cannot overtake them
    __threadfence_system();
    return;
  }
  double dsum = 0.0, rqsum = 0.0, qqsum = 0.0;
  const double* __restrict__ er = fz.er;
  // er == nullptr with the fused epilogue: r.q from the conjugacy identity
  // (MpFuse::pqo_stride), no pass over r; the recomputing layouts need r
  const bool rq_on = (kEpi >= 2) && (kEpi == 3 || kEpi == 4 || er != nullptr);
  // kEpi 2: fused-CG epilogue (p.q, r.q, q.q) of fusion layout 0; 4: layout 1
  // (p_new recomputed from p_old and r, and stored); 3: layout 2 (also the x
  // update: one more operand per element, so one tile per load batch)
  constexpr bool edots = kEpi >= 2;
  constexpr bool kRecomp = kEpi == 3 || kEpi == 4;
  constexpr bool kXUpd = kEpi == 3;
  constexpr int kEB = kRecomp ? 1 : edots ? (kBatch < 2 ? kBatch : 2) : kBatch;
  if (kWide && kIdent && xs == nullptr && (p & 1) == 0 &&
      (reinterpret_cast<uintptr_t>(Y) & 15) == 0) {
    const bool odd = (col & 1) != 0;
    const int ra = odd ? 1 : 0, rb = odd ? 3 : 2;
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const int64_t j0 = colj(t) & ~(int64_t)1;
      const double a0 = acc[t][0], a1 = acc[t][1], a2 = acc[t][2], a3 = acc[t][3];
      const double g0 = swap_lane_pair(odd ? a0 : a1);
      const double g1 = swap_lane_pair(odd ? a2 : a3);
      const double2 v0 = odd ? double2{g0, a1} : double2{a0, g0};
      const double2 v1 = odd ? double2{g1, a3} : double2{a2, g1};
      if (j0 < p) {
        if (rowok[ra]) *reinterpret_cast<double2*>(Y + rowoff[ra] + j0) = v0;
        if (rowok[rb]) *reinterpret_cast<double2*>(Y + rowoff[rb] + j0) = v1;
      }
    }
  } else if (xs == nullptr) {
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const bool cok = colj(t) < p;
      const int64_t co = coloff(t);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (rowok[r] && cok) Y[rowoff[r] + co] = acc[t][r];
    }
  } else if (!kXUpd) {
    // shift / dots epilogue (textbook p.q, fused-CG p.q, r.q, q.q; layout 1
    // also recomputes p_new = r + beta p_old from xs = p_old and stores it):
    // the loads of tile t + 1 are issued before tile t's stores.  CDNA4
    // retires vmcnt in order and stores count, so a load issued after a store
    // cannot be waited for without also waiting for that store's write
    // acknowledgement; issued first, the wait for tile t + 1 skips the stores
    // of tile t.
    const bool first = kRecomp && fz.sc->first != 0;
    const double beta = kRecomp ? fz.sc->beta : 0.0;
    double xv[2][4], ev[2][4];
    // kIdent: the wave's 16 x p output block is contiguous, so every address
    // is a uniform base (SGPRs) plus a 32-bit lane byte offset (saddr form):
    // one VGPR per address instead of a 64-bit pair
    const int64_t b0u = kIdent ? (int64_t)__builtin_amdgcn_readfirstlane((int)b0) |
                                     ((int64_t)__builtin_amdgcn_readfirstlane((int)(b0 >> 32))
                                      << 32)
                               : 0;
    const char* xbase = reinterpret_cast<const char*>(xs + (kIdent ? b0u * p : 0));
    const char* ebase = reinterpret_cast<const char*>(er + (kIdent ? b0u * p : 0));
    char* ybase = reinterpret_cast<char*>(Y + (kIdent ? b0u * p : 0));
    char* pbase = kRecomp ? reinterpret_cast<char*>(fz.ep_out + (kIdent ? b0u * p : 0)) : nullptr;
    auto boff = [&](int r, int t) -> uint32_t {
      return (uint32_t)(((lane >> 4) + 4 * r) * p + (int)colj(t)) * 8u;
    };
    // rows past M: the block's row count, uniform (kIdent)
    const int rows_left = kIdent ? (int)min<int64_t>(16, M - b0u) : 16;
    auto row_ok = [&](int r) -> bool {
      return kIdent ? ((lane >> 4) + 4 * r) < rows_left : rowok[r];
    };
    auto load_tile = [&](int t, double (&xo)[4], double (&eo)[4]) {
      const bool cok = colj(t) < p;
      const int64_t co = kIdent ? 0 : coloff(t);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = row_ok(r) && cok;
        if (kIdent) {
          const uint32_t o = boff(r, t);
          xo[r] = ok ? *reinterpret_cast<const double*>(xbase + o) : 0.0;
          eo[r] = (ok && rq_on) ? *reinterpret_cast<const double*>(ebase + o) : 0.0;
        } else {
          xo[r] = ok ? xs[rowoff[r] + co] : 0.0;
          eo[r] = (ok && rq_on) ? er[rowoff[r] + co] : 0.0;
        }
      }
    };
    load_tile(0, xv[0], ev[0]);
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const int cb = t & 1;
      // keep the scheduler from hoisting later tiles' loads (register budget)
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < JT) load_tile(t + 1, xv[cb ^ 1], ev[cb ^ 1]);
      const bool cok = colj(t) < p;
      const int64_t co = kIdent ? 0 : coloff(t);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (row_ok(r) && cok) {
          double pv = xv[cb][r];
          if (kRecomp) pv = first ? ev[cb][r] : fma(beta, pv, ev[cb][r]);
          const double v = fma(shift, pv, acc[t][r]);
          dsum = fma(pv, v, dsum);
          if (edots) {
            rqsum = fma(ev[cb][r], v, rqsum);
            qqsum = fma(v, v, qqsum);
          }
          if (kIdent) {
            *reinterpret_cast<double*>(ybase + boff(r, t)) = v;
            if (kRecomp) *reinterpret_cast<double*>(pbase + boff(r, t)) = pv;
          } else {
            Y[rowoff[r] + co] = v;
            if (kRecomp) fz.ep_out[rowoff[r] + co] = pv;
          }
        }
      }
    }
  } else {
    // fusion layouts 1 / 2: p_new recomputed here from p_old (xs) and r
    double* __restrict__ ep_out = kRecomp ? fz.ep_out : nullptr;
    const bool recompute = kRecomp;
    double* __restrict__ ex =
        (kXUpd && recompute && fz.ex != nullptr && fz.sc->pending) ? fz.ex : nullptr;
    const bool first = recompute && fz.sc->first != 0;
    const double beta = recompute ? fz.sc->beta : 0.0;
    const double alpha = ex != nullptr ? fz.sc->alpha : 0.0;
    // batch the x loads so that CDNA4's in-order vmcnt (stores count too)
    // does not serialise one load round trip per output element
#pragma unroll
    for (int t0 = 0; t0 < JT; t0 += kEB) {
      double xv[kEB][4], ev[kEB][4], wv[kXUpd ? kEB : 1][4];
#pragma unroll
      for (int tb = 0; tb < kEB; ++tb) {
        const int t = t0 + tb < JT ? t0 + tb : JT - 1;
        const bool cok = t0 + tb < JT && colj(t) < p;
        const int64_t co = coloff(t);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = rowok[r] && cok;
          xv[tb][r] = ok ? xs[rowoff[r] + co] : 0.0;
          ev[tb][r] = (ok && edots) ? er[rowoff[r] + co] : 0.0;
          if (kXUpd) wv[kXUpd ? tb : 0][r] = (ok && ex != nullptr) ? ex[rowoff[r] + co] : 0.0;
        }
      }
#pragma unroll
      for (int tb = 0; tb < kEB; ++tb) {
        const int t = t0 + tb;
        if (t < JT) {
          const bool cok = colj(t) < p;
          const int64_t co = coloff(t);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (rowok[r] && cok) {
              double pv = xv[tb][r];
              if (recompute) pv = first ? ev[tb][r] : fma(beta, xv[tb][r], ev[tb][r]);
              const double v = fma(shift, pv, acc[t][r]);
              dsum = fma(pv, v, dsum);
              if (edots) {
                rqsum = fma(ev[tb][r], v, rqsum);
                qqsum = fma(v, v, qqsum);
              }
              Y[rowoff[r] + co] = v;
              if (recompute) ep_out[rowoff[r] + co] = pv;
              if (kXUpd && ex != nullptr)
                ex[rowoff[r] + co] = wv[kXUpd ? tb : 0][r] + alpha * xv[tb][r];
            }
          }
        }
      }
    }
  }
  mp_block_sums<kWaves, CGP, edots, kRaw>(dsum, edots ? rqsum : pqo_acc, qqsum, rr_acc,
                                          dot_partials, fz, red, blk);
  if (kEpi >= 1) mp_side_job<kThreads>(fz, blk);
}

// Double-buffered chunk pipeline, one barrier per chunk:
//   issue global loads of chunk c+1 (K^T fragments -> registers, X -> A regs)
//   MFMA over chunk c from LDS buffer c&1
//   write the staged registers into LDS buffer (c+1)&1 ; barrier
// so the L2 latency of the factor fragments and the HBM latency of X hide
// under 8*JT MFMAs (64 cycles each) per wave.
//
// CGP fuses CG's direction update into the first mode product (MpFuse):
//   CGP = 1 (textbook recurrence): the A operand is p_new = beta * p + r
//           (p_new = r on the first iteration, selected, so an uninitialised p
//           never leaks in), written back in place;
//   CGP = 2 (fused recurrence, see gg_vec.hip): when the previous iteration's
//           updates are pending, r -= alpha q_old first (written back, r.r
//           partial per workgroup), then p_new = r + beta p_old goes to a
//           second p buffer.
// Each element is read and written by exactly one lane (kSplit = 1).
//
// kSplit = 2 splits the output columns of a strip over two waves (JT tiles
// each): half the accumulators per wave, so two workgroups fit a CU and one
// workgroup's prologue / epilogue overlaps the other's MFMAs.
//
// kEpi = 1 (fused CG, second mode product): the x-update side job after the
// epilogue.  kEpi = 2 (fused CG, last mode product): the epilogue also reads r
// and accumulates r.q and q.q next to p.q (MpFuse::er), a smaller load batch
// keeping the extra loads within the register budget; side job too (d = 2).
// kT4 (p = 16 (JT - 1) + r, r <= 8: the last output tile is at most half
// real): that tile runs as two v_mfma_f64_4x4x4_4b_f64 (cols 16 (JT-1) + 4h +
// 0..3, h = 0 / 1; 16 cycles each, the same FLOP rate as the 16x16x4 shape,
// tools/mfma_f64_4x4_bench.hip) instead of one 64-cycle 16x16x4 of which
// half is padding.  The 4x4x4_4b A operand is the 16x16x4 one (lane 16 k +
// row, tools/mfma_4x4_layout_probe.hip), its B fragment h holds column
// 4h + (l & 3) of the tail at lane l for every 4-lane group (Factor::frag4
// packs JT + 1 fragments per k-step, the last two these), and D lane
// 16 r + 4 g + c = row 4 g + r, column 4 h + c: one shuffle pass after the
// k-loop rebuilds the 16x16 layout of acc[JT - 1] for the epilogue.
template <int JT, int kWaves, int kKC, int CGP, int kMinW, bool kIdent, int kSplit, int kOpt,
          int kEpi = 0, bool kT4 = false>
__global__ __launch_bounds__(kWaves * 64, kMinW) void mode_product_kernel(
    const double* X, double* __restrict__ Y, const double* __restrict__ Bf,
    int64_t M, int q, int p, int KS, int jt_total, int jt0,
    const double* __restrict__ xs, double shift, double* __restrict__ dot_partials,
    const int* __restrict__ skip, OutMap om, MpFuse fz) {
  static_assert(CGP == 0 || kSplit == 1, "the CG prologue needs one wave per element");
  static_assert(!kT4 || kSplit == 1, "the 4x4 tail needs one wave per strip");
  if (skip != nullptr && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double lds[];  // 2 * kKC * JTL * 64
  constexpr int JTL = JT * kSplit + (kT4 ? 1 : 0);       // fragments staged per k-step
  constexpr int kThreads = kWaves * 64;
  constexpr int kChunk2 = kKC * JTL * 32;                 // double2 per full chunk
  constexpr int kPerT = (kChunk2 + kThreads - 1) / kThreads;
  constexpr int kBuf = kKC * JTL * 64;                    // doubles per LDS buffer

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hp = kSplit == 1 ? 0 : wave % kSplit;         // column part of this wave
  const int strip = kSplit == 1 ? wave : wave / kSplit;
  const int nt = min(JT * kSplit, jt_total - jt0);        // real tiles in this launch
  const int64_t b0 = ((int64_t)blockIdx.x * (kWaves / kSplit) + strip) * 16;
  const int64_t brow = b0 + (lane & 15);
  const bool bvalid = brow < M;
  const int64_t bclamp = bvalid ? brow : M - 1;
  const int krow = lane >> 4;
  const int nchunks = (KS + kKC - 1) / kKC;

  // ---- per-thread addressing, computed once (the k-loop only adds strides)
  // staging: element i of a chunk is double2 o of k-step s, i.e.
  // Bf[((ks0 + s) * jt_total + jt0) * 64 + 2 o].  The packed factor carries 8
  // zero k-steps of padding, so a partial last chunk needs no clamp; tiles
  // past nt (kSplit > 1 only) re-read the last real tile and are never used.
  const double* __restrict__ bbase = Bf + (int64_t)jt0 * 64;
  const int64_t bchunk = (int64_t)kKC * jt_total * 64;          // doubles per chunk
  int boff[kPerT];
  bool bfull[kPerT];
#pragma unroll
  for (int u = 0; u < kPerT; ++u) {
    int i = threadIdx.x + u * kThreads;
    bfull[u] = i < kChunk2;
    i = i < kChunk2 ? i : kChunk2 - 1;
    const int s_ = i / (JTL * 32);
    int o_ = i - s_ * (JTL * 32);
    if (kSplit > 1) o_ = min(o_, nt * 32 - 1);
    boff[u] = s_ * jt_total * 64 + 2 * o_;
  }
  // A operand: lane l reads X[4 ks + (l >> 4)][b0 + (l & 15)]
  const int64_t m4 = 4 * M;
  const int64_t aoff0 = (int64_t)krow * M + bclamp;
  const int64_t alast = (int64_t)(q - 1) * M + bclamp;
  const int64_t achunk = (int64_t)kKC * m4;
  double* __restrict__ Rg = fz.r;
  const double* __restrict__ Qg = fz.q_old;
  // CGP 3 writes its output over q_old's elements (Pout == q_old, each element
  // read then written by the same lane): no restrict on that operand
  const double* Qa = fz.q_old;
  double* Pout = fz.p_out;

  // kOpt & 2: the factor chunk goes global -> LDS directly (global_load_lds,
  // lane-linear 1 KiB per wave instruction), no staging registers
#define GG_STAGE_LOAD(c, st)                                                          \
  do {                                                                                \
    const double* cb_ = bbase + (int64_t)(c) * bchunk;                                \
    if (kOpt & 2) {                                                                   \
      double* dstb_ = lds + ((c) & 1) * kBuf + wave * 128;                            \
      _Pragma("unroll") for (int u = 0; u < kPerT; ++u) {                             \
        if (bfull[u])                                                                 \
          __builtin_amdgcn_global_load_lds(                                           \
              (const __attribute__((address_space(1))) void*)(cb_ + boff[u]),         \
              (__attribute__((address_space(3))) void*)(dstb_ + u * kThreads * 2),    \
              16, 0, 0);                                                              \
      }                                                                               \
    } else {                                                                          \
      _Pragma("unroll") for (int u = 0; u < kPerT; ++u) {                             \
        const double2 v_ = *reinterpret_cast<const double2*>(cb_ + boff[u]);          \
        st##x[u] = v_.x; st##y[u] = v_.y;                                             \
      }                                                                               \
    }                                                                                 \
  } while (0)
#define GG_STAGE_STORE(c, st)                                                         \
  do {                                                                                \
    if (!(kOpt & 2)) {                                                                \
      double2* dst_ = reinterpret_cast<double2*>(lds + ((c) & 1) * kBuf);             \
      _Pragma("unroll") for (int u = 0; u < kPerT; ++u) {                             \
        if (bfull[u]) dst_[threadIdx.x + u * kThreads] = double2{st##x[u], st##y[u]}; \
      }                                                                               \
    }                                                                                 \
  } while (0)
// A fragments: unconditional loads; only the last chunk clamps the row to
// q - 1.  The mask (rows past q, strips past M) is applied when the
// registers are consumed, so no load is followed by a wait.
#define GG_A_LOAD(c, a, rr, qq)                                                       \
  do {                                                                                \
    int64_t o_ = aoff0 + (int64_t)(c) * achunk;                                       \
    if ((c) == nchunks - 1) {                                                         \
      _Pragma("unroll") for (int s_ = 0; s_ < kKC; ++s_) {                            \
        const int64_t oc_ = o_ < alast ? o_ : alast;                                  \
        a[s_] = X[oc_];                                                               \
        if (CGP) rr[s_] = Rg[oc_];                                                    \
        if (CGP >= 2) qq[s_] = CGP == 3 ? Qa[oc_] : Qg[oc_];                          \
        o_ += m4;                                                                     \
      }                                                                               \
    } else {                                                                          \
      _Pragma("unroll") for (int s_ = 0; s_ < kKC; ++s_) {                            \
        a[s_] = X[o_];                                                                \
        if (CGP) rr[s_] = Rg[o_];                                                     \
        if (CGP >= 2) qq[s_] = CGP == 3 ? Qa[o_] : Qg[o_];                            \
        o_ += m4;                                                                     \
      }                                                                               \
    }                                                                                 \
  } while (0)
#define GG_A_MASK(c, a, rr, qq)                                                       \
  do {                                                                                \
    const int ks0_ = (c) * kKC;                                                       \
    _Pragma("unroll") for (int s_ = 0; s_ < kKC; ++s_) {                              \
      const int k_ = (ks0_ + s_) * 4 + krow;                                          \
      const bool ok_ = bvalid && k_ < q;                                              \
      double v_ = a[s_];                                                              \
      if (CGP == 3) {                                                                 \
        const int64_t e_ = (int64_t)k_ * M + brow;                                    \
        v_ = fma(lz_cp, qq[s_], fma(lz_cu, rr[s_], lz_cy * v_));                      \
        if (ok_) {                                                                    \
          Pout[e_] = v_;                                                              \
          rr_acc = fma(v_, v_, rr_acc);                                               \
        }                                                                             \
      } else if (CGP) {                                                               \
        double r_ = rr[s_];                                                           \
        const int64_t e_ = (int64_t)k_ * M + brow;                                    \
        if (CGP == 2 && cg_pending) {                                                 \
          r_ = r_ - cg_alpha * qq[s_];                                                \
          if (ok_) {                                                                  \
            Rg[e_] = r_;                                                              \
            rr_acc = fma(r_, r_, rr_acc);                                             \
          }                                                                           \
        }                                                                             \
        v_ = cg_first ? r_ : fma(cg_beta, v_, r_);                                    \
        if (Pout != nullptr && ok_ && hp == 0) Pout[e_] = v_;                         \
        if (CGP == 2 && pqo_on && ok_ && hp == 0) pqo_acc = fma(v_, qq[s_], pqo_acc); \
      }                                                                               \
      a[s_] = ok_ ? v_ : 0.0;                                                         \
    }                                                                                 \
  } while (0)

  d4 acc[JT];
#pragma unroll
  for (int t = 0; t < JT; ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  double t4[2] = {0.0, 0.0};   // kT4: the tail tile's two 4x4x4_4b accumulators

  double a_cur[kKC], a_nxt[kKC], r_cur[kKC], r_nxt[kKC], q_cur[kKC], q_nxt[kKC];
  double stx[kPerT], sty[kPerT];
  bool cg_first = false, cg_pending = false, pqo_on = false;
  double cg_beta = 0.0, cg_alpha = 0.0, rr_acc = 0.0, pqo_acc = 0.0;
  double lz_cy = 0.0, lz_cu = 0.0, lz_cp = 0.0;
  if (CGP == 3) {
    lz_cy = fz.coef[2];
    lz_cu = fz.coef[3];
    lz_cp = fz.coef[4];
  } else if (CGP) {
    cg_first = fz.sc->first != 0;
    cg_beta = fz.sc->beta;
    if (CGP == 2) {
      cg_pending = fz.sc->pending != 0;
      cg_alpha = fz.sc->alpha;
      // p_new.q_old (conjugacy r.q); q_old is not A p_old on the first step
      pqo_on = fz.pqo_stride > 0 && !cg_first;
    }
  }
  GG_STAGE_LOAD(0, st);
  GG_A_LOAD(0, a_cur, r_cur, q_cur);
  GG_STAGE_STORE(0, st);
  GG_A_MASK(0, a_cur, r_cur, q_cur);
  __syncthreads();

  // Per chunk: the first k-step's MFMAs are placed before the next chunk's
  // global loads in the source (kOpt & 1 pins that order with sched_barrier),
  // so the waves of a SIMD restart their MFMAs right after the barrier.
  for (int c = 0; c < nchunks; ++c) {
    const bool more = c + 1 < nchunks;
    const int kcn = min(kKC, KS - c * kKC);
    const double* buf = lds + (c & 1) * kBuf;
#pragma unroll
    for (int s = 0; s < kKC; ++s) {
      if (s == 1 || (kKC == 1 && s == 0)) {
        if (kOpt & 1) __builtin_amdgcn_sched_barrier(0);
        if (more) {
          GG_STAGE_LOAD(c + 1, st);
          GG_A_LOAD(c + 1, a_nxt, r_nxt, q_nxt);
        }
        if (kOpt & 1) __builtin_amdgcn_sched_barrier(0);
      }
      if (s < kcn) {
        if (kOpt & 8) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int t = 0; t < JT; ++t) {
          if (kT4 && t == JT - 1) {
            const double b0 = buf[(s * JTL + t) * 64 + lane];
            const double b1 = buf[(s * JTL + t + 1) * 64 + lane];
            t4[0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a_cur[s], b0, t4[0], 0, 0, 0);
            t4[1] = __builtin_amdgcn_mfma_f64_4x4x4f64(a_cur[s], b1, t4[1], 0, 0, 0);
          } else if (kSplit == 1 || hp * JT + t < nt) {
            const double b = buf[(s * JTL + hp * JT + t) * 64 + lane];
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a_cur[s], b, acc[t], 0, 0, 0);
          }
        }
        if (kOpt & 8) __builtin_amdgcn_s_setprio(0);
      }
    }
    if (more) {
      GG_STAGE_STORE(c + 1, st);
#pragma unroll
      for (int s = 0; s < kKC; ++s) {
        a_cur[s] = a_nxt[s];
        if (CGP) r_cur[s] = r_nxt[s];
        if (CGP >= 2) q_cur[s] = q_nxt[s];
      }
      GG_A_MASK(c + 1, a_cur, r_cur, q_cur);
    }
    __syncthreads();
  }
#undef GG_STAGE_LOAD
#undef GG_STAGE_STORE
#undef GG_A_LOAD
#undef GG_A_MASK

  if (kT4) {
    // 4x4x4_4b D (lane 16 r + 4 g + c = row 4 g + r, column 4 h + c) -> the
    // 16x16 layout (lane L, register rho = row 4 rho + (L >> 4), column L & 15)
    const int cc = lane & 15;
    const int src0 = 16 * (lane >> 4) + (lane & 3);
#pragma unroll
    for (int rho = 0; rho < 4; ++rho) {
      const double v0 = __shfl(t4[0], src0 + 4 * rho, 64);
      const double v1 = __shfl(t4[1], src0 + 4 * rho, 64);
      acc[JT - 1][rho] = cc < 4 ? v0 : cc < 8 ? v1 : 0.0;
    }
  }
  mp_finish<JT, kWaves, kSplit, kIdent, kEpi, CGP, false, kEpiBatch, (kOpt & 4) != 0>(
      acc, Y, M, p, jt0, xs, shift, dot_partials, om, fz, rr_acc, b0, hp, lds, blockIdx.x,
      pqo_acc);
}

// Launch configuration of one mode product: waves per workgroup, k-steps per
// LDS chunk.  The default -- 4-wave workgroups (one wave per SIMD), 3 k-steps
// per chunk, three independent workgroups per CU, factor chunks staged by
// global_load_lds -- was chosen by A/B on MI355X (profiles/r01_*_mode_variants):
// three workgroups drift apart, so one's barrier or epilogue overlaps the
// others' MFMAs.  The other shapes of that A/B (12 / 8 / 2-wave workgroups,
// 2 / 4 k-steps, register-staged chunks, the all-LDS-DMA and persistent
// kernels, paired stores, s_setprio, and the wider fused-CG prologues) were
// measured slower and live in the history (round 4).
struct ModeConfig {
  mode_kernel_t fn;
  int waves, kc, split, jtl;  // jtl: tiles staged per launch
  size_t lds;                 // dynamic LDS bytes
  bool t4 = false;            // reads Factor::frag4 (JT + 1 fragments per k-step)
};

// JT = output tiles of the launch; a split config gives each wave ceil(JT/2)
template <int JT, int W, int KC, int CGP, int MINW, int SPLIT, int OPT, int EPI = 0>
static ModeConfig cfg() {
  constexpr int JW = (JT + SPLIT - 1) / SPLIT;
  return ModeConfig{mode_product_kernel<JW, W, KC, CGP, MINW, true, SPLIT, OPT, EPI>, W, KC,
                    SPLIT, JW * SPLIT, 2 * (size_t)KC * JW * SPLIT * 64 * sizeof(double)};
}

template <int JT, int W, int KC, int CGP, int MINW, int OPT, int EPI = 0>
static ModeConfig cfg_t4() {
  return ModeConfig{mode_product_kernel<JT, W, KC, CGP, MINW, true, 1, OPT, EPI, true>, W, KC, 1,
                    JT + 1, 2 * (size_t)KC * (JT + 1) * 64 * sizeof(double), true};
}


// cgp: 0 plain, 1 textbook CG prologue, 2 fused CG prologue, 3 fused CG
// epilogue (+ side job when d = 2), 4 fused CG side job, 5 / 6 fusion layouts
// 2 / 1 epilogues, 7 Lanczos prologue
// the default shapes with the 4x4x4 tail (kT4), for factors with frag4
template <int JT>
static ModeConfig config_t4(int cgp) {
  if constexpr (JT == 13) {
    switch (cgp) {
      case 1: return cfg_t4<JT, 4, 3, 1, 3, 2>();
      case 2: return cfg_t4<JT, 4, 3, 2, 3, 2>();
      case 3: return cfg_t4<JT, 4, 3, 0, 3, 2, 2>();
      case 4: return cfg_t4<JT, 4, 3, 0, 3, 2, 1>();
      case 5: return cfg_t4<JT, 4, 3, 0, 3, 2, 3>();
      case 6: return cfg_t4<JT, 4, 3, 0, 3, 2, 4>();
      case 7: return cfg_t4<JT, 4, 3, 3, 3, 2>();
      default: return cfg_t4<JT, 4, 3, 0, 3, 2>();
    }
  }
  throw Error(GG_ERR_VALUE, "no 4x4-tail kernel for this tile count");
}

template <int JT>
static ModeConfig config_for(int cgp) {
  switch (cgp) {
    case 1: return cfg<JT, 4, 3, 1, 3, 1, 2>();
    case 2: return cfg<JT, 4, 3, 2, 3, 1, 2>();
    case 3: return cfg<JT, 4, 3, 0, 3, 1, 2, 2>();
    case 4: return cfg<JT, 4, 3, 0, 3, 1, 2, 1>();
    case 5: return cfg<JT, 4, 3, 0, 3, 1, 2, 3>();
    case 6: return cfg<JT, 4, 3, 0, 3, 1, 2, 4>();
    case 7: return cfg<JT, 4, 3, 3, 3, 1, 2>();   // Lanczos prologue (CGP 3)
    default: return cfg<JT, 4, 3, 0, 3, 1, 2>();
  }
}

static ModeConfig select_kernel(int jt, int cgp) {
  switch (jt) {
    case 1: return config_for<1>(cgp);
    case 2: return config_for<2>(cgp);
    case 3: return config_for<3>(cgp);
    case 4: return config_for<4>(cgp);
    case 5: return config_for<5>(cgp);
    case 6: return config_for<6>(cgp);
    case 7: return config_for<7>(cgp);
    case 8: return config_for<8>(cgp);
    case 9: return config_for<9>(cgp);
    case 10: return config_for<10>(cgp);
    case 11: return config_for<11>(cgp);
    case 12: return config_for<12>(cgp);
    case 13: return config_for<13>(cgp);
    case 14: return config_for<14>(cgp);
    case 15: return config_for<15>(cgp);
    case 16: return config_for<16>(cgp);
    default: throw Error(GG_ERR_VALUE, "bad tile count");
  }
}

static size_t mode_lds_bytes(const ModeConfig& c) { return c.lds; }

// compute units of the current device (persistent launches)
static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    if (n <= 0) n = 256;
  }
  return n;
}

// One factor in fragment order, for the operator and for its transpose.
struct Factor {
  int64_t p = 0, q = 0;   // as applied: p x q
  int KS = 0, JT = 0;     // k-steps of 4, column tiles of 16
  double* frag = nullptr; // [KS][JT][64] device
  // [KS][JT + 1][64]: the last tile as the two 4x4x4_4b B fragments
  // (mode_product_kernel kT4), when that tile is at most half real and the
  // single-launch kernel has a kT4 instance for JT (t4_supported)
  double* frag4 = nullptr;
  // centrosymmetric split (mode_product_fold_kernel): [fKS + 8][2 fFH][64],
  // fJT 16-wide tiles per half, the last as fTT 4x4x4_4b fragments if fTT > 0
  double* ffrag = nullptr;
  int fKS = 0, fJT = 0, fTT = 0;
  // the same fragments at 16 per k-step ([fKS][16][64], zero pads) for the
  // ring kernel (gg_kron_ring.hip), when its shape is instantiated
  double* rfrag = nullptr;
};

static bool t4_supported(int JT) { return JT == 13; }

static void pack_fragments(const double* K, int64_t rows, int64_t cols, bool transpose,
                           Factor& f) {
  // applied factor F = transpose ? K^T : K, F is p x q; B[k][j] = F[j][k]
  f.p = transpose ? cols : rows;
  f.q = transpose ? rows : cols;
  f.KS = (int)ceil_div(f.q, 4);
  f.JT = (int)ceil_div(f.p, 16);
  // 8 zero k-steps of padding: a partial last LDS chunk (kKC <= 8) stays in bounds
  std::vector<double> h(((size_t)f.KS + 8) * f.JT * 64, 0.0);
  for (int ks = 0; ks < f.KS; ++ks)
    for (int jt = 0; jt < f.JT; ++jt)
      for (int l = 0; l < 64; ++l) {
        const int64_t k = (int64_t)ks * 4 + (l >> 4);
        const int64_t j = (int64_t)jt * 16 + (l & 15);
        double v = 0.0;
        if (k < f.q && j < f.p) v = transpose ? K[k * cols + j] : K[j * cols + k];
        h[((size_t)ks * f.JT + jt) * 64 + l] = v;
      }
  GG_HIP(hipMalloc(&f.frag, h.size() * sizeof(double)));
  GG_HIP(hipMemcpy(f.frag, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  if (t4_supported(f.JT) && f.p - 16 * (int64_t)(f.JT - 1) <= 8) {
    const int JF = f.JT + 1;
    std::vector<double> h4(((size_t)f.KS + 8) * JF * 64, 0.0);
    for (int ks = 0; ks < f.KS; ++ks)
      for (int jt = 0; jt < JF; ++jt)
        for (int l = 0; l < 64; ++l) {
          const int64_t k = (int64_t)ks * 4 + (l >> 4);
          // tiles < JT - 1 as before; fragment JT - 1 + h: tail column 4h + (l & 3)
          const int64_t j = jt < f.JT - 1 ? (int64_t)jt * 16 + (l & 15)
                                          : (int64_t)(f.JT - 1) * 16 + 4 * (jt - (f.JT - 1)) + (l & 3);
          double v = 0.0;
          if (k < f.q && j < f.p) v = transpose ? K[k * cols + j] : K[j * cols + k];
          h4[((size_t)ks * JF + jt) * 64 + l] = v;
        }
    GG_HIP(hipMalloc(&f.frag4, h4.size() * sizeof(double)));
    GG_HIP(hipMemcpy(f.frag4, h4.data(), h4.size() * sizeof(double), hipMemcpyHostToDevice));
  }
}

// the centrosymmetric split (mode_product_fold_kernel) for square factors
static int fold_min_size() {
  const char* e = gg::knob("GG_KRON_FOLD_MIN");
  const int v = e ? atoi(e) : 48;
  return v < 8 ? 8 : v;   // h >= 4: the kernel's unclamped row walk stays in bounds
}
static bool fold_enabled() {
  const char* e = gg::knob("GG_KRON_FOLD");
  return !(e && atoi(e) == 0);
}
// tail fragments of a half of hS columns in JT tiles (even m, JT >= 4 only:
// the instantiated shapes)
static int fold_tail(int64_t m, int JT) {
  if (m % 2 != 0 || JT < 4) return 0;
  const int64_t r = (m - m / 2) - 16 * (int64_t)(JT - 1);
  return r <= 4 ? 1 : r <= 8 ? 2 : 0;
}

static void pack_fold(const double* K, int64_t m, bool transpose, Factor& f) {
  if (!fold_enabled() || m < fold_min_size() || m > 256) return;
  auto F = [&](int64_t j, int64_t i) { return transpose ? K[i * m + j] : K[j * m + i]; };
  double amax = 0.0, dmax = 0.0;
  for (int64_t j = 0; j < m; ++j)
    for (int64_t i = 0; i < m; ++i) {
      amax = std::max(amax, std::fabs(F(j, i)));
      dmax = std::max(dmax, std::fabs(F(j, i) - F(m - 1 - j, m - 1 - i)));
    }
  if (!(dmax <= 16.0 * 2.220446049250313e-16 * amax) || !(amax > 0.0)) return;
  // the centrosymmetric part (F + J F J) / 2
  auto Fc = [&](int64_t j, int64_t i) { return 0.5 * (F(j, i) + F(m - 1 - j, m - 1 - i)); };
  const int64_t h = m / 2, hS = m - h;
  const int JT = (int)ceil_div(hS, 16);
  const int TT = fold_tail(m, JT);
  const int FH = JT - (TT > 0 ? 1 : 0) + TT;   // fragments per half and k-step
  const int JF = 2 * FH;
  const int KS = (int)ceil_div(hS, 4);
  std::vector<double> hb(((size_t)KS + 8) * JF * 64, 0.0);
  for (int ks = 0; ks < KS; ++ks)
    for (int fr = 0; fr < JF; ++fr)
      for (int l = 0; l < 64; ++l) {
        const int64_t k = (int64_t)ks * 4 + (l >> 4);   // i'
        const bool odd_half = fr >= FH;
        const int t = odd_half ? fr - FH : fr;
        const int64_t j = (TT > 0 && t >= JT - 1)
                              ? 16 * (int64_t)(JT - 1) + 4 * (t - (JT - 1)) + (l & 3)
                              : 16 * (int64_t)t + (l & 15);   // j'
        double v = 0.0;
        if (!odd_half) {
          if (j < hS && k < hS) v = k < h ? 0.5 * (Fc(j, k) + Fc(j, m - 1 - k)) : Fc(j, k);
        } else if (j < h && k < h) {
          v = 0.5 * (Fc(j, k) - Fc(j, m - 1 - k));
        }
        hb[((size_t)ks * JF + fr) * 64 + l] = v;
      }
  GG_HIP(hipMalloc(&f.ffrag, hb.size() * sizeof(double)));
  GG_HIP(hipMemcpy(f.ffrag, hb.data(), hb.size() * sizeof(double), hipMemcpyHostToDevice));
  f.fKS = KS;
  f.fJT = JT;
  f.fTT = TT;
  if (ring_available(JT, TT, m) && JF <= 16) {
    std::vector<double> rb((size_t)KS * 16 * 64, 0.0);
    for (int ks = 0; ks < KS; ++ks)
      std::copy(hb.begin() + (size_t)ks * JF * 64, hb.begin() + (size_t)(ks + 1) * JF * 64,
                rb.begin() + (size_t)ks * 16 * 64);
    GG_HIP(hipMalloc(&f.rfrag, rb.size() * sizeof(double)));
    GG_HIP(hipMemcpy(f.rfrag, rb.data(), rb.size() * sizeof(double), hipMemcpyHostToDevice));
  }
}

}  // namespace gg

struct gg_kron {
  int d = 0;
  std::vector<gg::Factor> fwd, bwd;  // operator and transposed operator
  gg::BlockOp* blk = nullptr;        // parity-block basis (gg_kronb.hip), when it exists
  int64_t n_rows = 1, n_cols = 1;
  int64_t max_inter_fwd = 0, max_inter_bwd = 0;
  bool square_steps_fwd = true, square_steps_bwd = true;
};

namespace gg {

static void plan_sizes(const std::vector<Factor>& fs, int64_t n_in, int64_t& max_inter,
                       bool& all_square) {
  int64_t s = n_in;
  max_inter = s;
  all_square = true;
  for (const Factor& f : fs) {
    s = s / f.q * f.p;
    max_inter = std::max(max_inter, s);
    if (f.p != f.q) all_square = false;
  }
}

int64_t kron_side_half(const gg_kron* K, int64_t n);

void kron_apply(const gg_kron* K, bool transpose, const double* x, double* y, double shift,
                double* work, double* dot_partials, const int* skip, hipStream_t stream,
                int64_t* n_partials_out, const MpFuse* cg, int cgp, hipEvent_t* ev) {
  // cg / cgp (optional): CG fusions (MpFuse).  cgp = 1: textbook prologue on
  // the first mode product (p updated in place in x); cgp = 2: the fused
  // recurrence -- prologue (p_new -> cg->p_out), side job on the second mode
  // product, r.q / q.q partials on the last.
  // ev (optional, d + 1 events): recorded before the first mode product and
  // after each one, for live per-launch timing (gg_cg_profile)
  const std::vector<Factor>& fs = transpose ? K->bwd : K->fwd;
  const bool square = transpose ? K->square_steps_bwd : K->square_steps_fwd;
  const int64_t n_in = transpose ? K->n_rows : K->n_cols;
  const int64_t max_inter = transpose ? K->max_inter_bwd : K->max_inter_fwd;
  // x == y only for the Lanczos prologue with an even number of square steps:
  // the first step reads x and writes the scratch, y is first written by the
  // second step (gg_lanczos_probe)
  GG_REQUIRE(x != y || (cgp == 3 && cg != nullptr && fs.size() % 2 == 0 &&
                        (transpose ? K->square_steps_bwd : K->square_steps_fwd)),
             GG_ERR_VALUE, "x and y must not alias");
  if (shift != 0.0 || dot_partials != nullptr)
    GG_REQUIRE(K->n_rows == K->n_cols, GG_ERR_VALUE, "shift needs a square operator");
  if (cg == nullptr) cgp = 0;
  const int d = (int)fs.size();
  GG_REQUIRE(cgp != 2 || d >= 2, GG_ERR_VALUE, "the fused CG recurrence needs d >= 2");
  GG_REQUIRE(cgp != 2 || cg->ep_out == nullptr || (cg->p_out == nullptr && fs[0].JT <= kMaxJT),
             GG_ERR_VALUE, "fusion layouts 1 / 2 need one launch for the first factor");
  int64_t size = n_in;
  const double* src = x;
  int64_t np_total = 0;
  if (ev) GG_HIP(hipEventRecord(ev[0], stream));
  for (int k = 0; k < d; ++k) {
    const Factor& f = fs[k];
    const int64_t M = size / f.q;
    const int64_t out_size = M * f.p;
    double* dst;
    if (k == d - 1) {
      dst = y;
    } else if (square) {
      dst = ((d - 1 - k) % 2 == 0) ? y : work;
    } else {
      dst = (k % 2 == 0) ? work : work + max_inter;
    }
    // the fused CG prologue reads q_old == y across workgroups while the
    // first mode product writes its output: never into y (odd d)
    if (k == 0 && k != d - 1 && cgp == 2 && dst == y) {
      GG_REQUIRE(cg->first_dst != nullptr, GG_ERR_VALUE,
                 "the fused CG with an odd number of factors needs a first-step scratch");
      dst = cg->first_dst;
    }
    const bool last = (k == d - 1);
    if (M > 0) {
      const double* step_src = src;
      for (int jt0 = 0; jt0 < f.JT; jt0 += kMaxJT) {
        const int jt = std::min(kMaxJT, f.JT - jt0);
        MpFuse fz;
        // the fused CG direction update runs once, in the first launch of
        // step 0; the later launches of that step read the updated p
        // cgp 3 (Lanczos prologue) is launch kind 7
        const int pro = (cgp != 0 && k == 0 && jt0 == 0) ? (cgp == 3 ? 7 : cgp) : 0;
        const bool epi = cgp == 2 && last && dot_partials != nullptr;
        // the x side job rides on the second mode product; with d >= 4 the
        // third (also a plain, MFMA-bound one) takes the second half of x
        const bool split_side = cgp == 2 && d >= 4 && cg->sx != nullptr;
        const bool side = cgp == 2 && jt0 == 0 && cg->sx != nullptr &&
                          (k == 1 || (split_side && k == 2));
        const int epi_kind = !epi ? 0 : cg->ep_out == nullptr ? 3 : cg->ex != nullptr ? 5 : 6;
        const int kind = epi ? epi_kind : side ? 4 : pro;
        ModeConfig mc = select_kernel(jt, kind);
        // the default shapes take the 4x4x4 tail when the factor has frag4
        if (f.frag4 != nullptr && jt0 == 0 && jt == f.JT && jt == 13) mc = config_t4<13>(kind);
        // centrosymmetric factors: the even/odd split (half the MFMA work)
        const bool fold =
            f.ffrag != nullptr && jt0 == 0 && fold_kind(kind) && !(pro && last);
        if (fold) {
          const double* xs_ = last && (shift != 0.0 || dot_partials != nullptr)
                                  ? (((cgp == 2 && cg->ep_out == nullptr) || cgp == 3) ? cg->p_out
                                                                                      : x)
                                  : nullptr;
          // the persistent LDS-DMA ring kernel (gg_kron_ring.hip) for the plain
          // launch (GG_FOLD_RING=0: the chunked kernel, A/B)
          const bool ring_ok =
              ring_variant_env() != 0 && xs_ == nullptr && f.rfrag != nullptr && M % 2 == 0 && M >= 2 &&
              ((reinterpret_cast<uintptr_t>(step_src) | reinterpret_cast<uintptr_t>(dst)) & 15) ==
                  0;
          if (ring_ok && kind == 0 && skip == nullptr) {
            const RingConfig rc = select_ring(f.fJT, f.fTT);
            const int64_t nb = ceil_div(M, (int64_t)16 * rc.waves);
            const int grid = ring_grid(rc, cu_count(), nb);
            hipLaunchKernelGGL(rc.fn, dim3((unsigned)grid), dim3(64 * rc.waves), rc.lds, stream,
                               step_src, dst, f.rfrag, M, (int)f.q, f.fKS, nb, skip, MpFuse());
            GG_LAUNCH_CHECK();
            continue;
          }
          const bool aligned =
              f.p % 2 == 0 &&
              ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(xs_) |
                reinterpret_cast<uintptr_t>(cg != nullptr ? cg->er : nullptr) |
                reinterpret_cast<uintptr_t>(cg != nullptr ? cg->ep_out : nullptr)) & 15) == 0;
          // the LDS-staged epilogue only where it reads the fused operands;
          // the kLean kernels where every chunk's rows (at most 3 k-steps
          // per chunk) lie inside the factor and the lane offsets fit 32 bits
          const bool lean_ok =
              4 * 3 * ceil_div((int64_t)f.fKS, (int64_t)3) <= (int64_t)f.q &&
              4 * 2 * ceil_div((int64_t)f.fKS, (int64_t)2) <= (int64_t)f.q &&
              32 * M < ((int64_t)1 << 32);
          const FoldConfig fc =
              (aligned && xs_ != nullptr && fold_staged_available(f.fJT, f.fTT, kind))
                  ? select_fold_staged(f.fJT, f.fTT, kind, lean_ok)
                  : select_fold(f.fJT, f.fTT, kind, lean_ok);
          if (fc.lean) {
            const int64_t nch = ceil_div((int64_t)f.fKS, (int64_t)fc.kc);
            GG_REQUIRE(4 * nch * fc.kc <= (int64_t)f.q && 32 * M < ((int64_t)1 << 32),
                       GG_ERR_VALUE, "lean folded kernel outside its row / offset range");
          }
          mc = ModeConfig{fc.fn, fc.waves, fc.kc, 1, fc.jf, fc.lds, false};
        }
        const int64_t nblk = ceil_div(M, (int64_t)(mc.waves / mc.split) * 16);
        GG_REQUIRE(nblk < (int64_t)1 << 31, GG_ERR_VALUE, "vector too long for one launch");
        if (pro) {
          fz.r = cg->r;
          fz.sc = cg->sc;
          fz.p_out = pro == 1 ? const_cast<double*>(x) : cg->p_out;
          if (pro == 2 || pro == 7) {
            fz.q_old = cg->q_old;
            fz.rr_part = cg->rr_part;
            // the partial arrays are sized at handle creation; the launch
            // shape is chosen here (env knobs may change between calls)
            GG_REQUIRE(cg->rr_part == nullptr || nblk <= cg->rr_cap, GG_ERR_VALUE,
                       "prologue launch has more workgroups than its partial array");
            if (cg->pro_blocks != nullptr) *cg->pro_blocks = nblk;
          }
          if (pro == 2) fz.pqo_stride = cg->pqo_stride;
          if (pro == 7) fz.coef = cg->coef;
        }
        if (side && cg->xdefer == 2) {
          // balanced x_defer: this launch's share of half 0 and of half 1 (the
          // device picks by sc->xh); x / p at offset 0
          const int64_t sn = cg->sn;
          int64_t off0, len0, off1, len1;
          if (split_side) {
            const int64_t Q = 2 * ceil_div(sn, (int64_t)8);
            const int L = (k == 2) ? 1 : 0;
            auto quarter = [&](int qd, int64_t& off, int64_t& len) {
              off = std::min<int64_t>((int64_t)qd * Q, sn);
              const int64_t end = qd == 3 ? sn : std::min<int64_t>((int64_t)(qd + 1) * Q, sn);
              len = std::max<int64_t>(end - off, 0);
            };
            quarter(L, off0, len0);
            quarter(2 + L, off1, len1);
          } else {
            const int64_t H = 2 * ceil_div(sn, (int64_t)4);
            off0 = 0;
            len0 = std::min(H, sn);
            off1 = std::min(H, sn);
            len1 = sn - off1;
          }
          fz.sc = cg->sc;
          fz.sx = cg->sx;
          fz.sp = cg->sp;
          fz.xdefer = 2;
          fz.soff = off0;
          fz.sn = len0;
          fz.soff_h1 = off1;
          fz.sn_h1 = len1;
          fz.schunk = 2 * ceil_div(std::max<int64_t>(std::max(len0, len1), 1), 2 * nblk);
        } else if (side) {
          // [off, off + len): all of x, or its half (even split: 16-byte
          // aligned double2 accesses stay aligned)
          const int64_t h = split_side ? 2 * ceil_div(cg->sn, 4) : cg->sn;
          const int64_t off = (split_side && k == 2) ? h : 0;
          const int64_t len = (split_side && k == 2) ? cg->sn - h : h;
          fz.sc = cg->sc;
          fz.sx = cg->sx + off;
          fz.sp = cg->sp + off;
          fz.xdefer = cg->xdefer;
          fz.soff = off;
          fz.sn = len;
          fz.schunk = 2 * ceil_div(std::max<int64_t>(len, 1), 2 * nblk);
        }
        double* parts = nullptr;
        if (last && dot_partials != nullptr) {
          parts = dot_partials + np_total;
          np_total += nblk;
          if (cgp == 2) {
            fz.er = cg->er;
            fz.pstride = cg->pstride;
            fz.ep_out = cg->ep_out;   // fusion layouts 1 / 2
            fz.ex = cg->ex;
            fz.sc = cg->sc;
          }
        }
        int64_t grid = nblk;
        hipLaunchKernelGGL(mc.fn, dim3((unsigned)grid), dim3(mc.waves * 64),
                           mode_lds_bytes(mc), stream, step_src, dst,
                           fold ? f.ffrag : mc.t4 ? f.frag4 : f.frag, M, (int)f.q, (int)f.p,
                           fold ? f.fKS : f.KS, fold ? mc.jtl : mc.t4 ? f.JT + 1 : f.JT, jt0,
                           last && (shift != 0.0 || parts)
                               ? (((cgp == 2 && cg->ep_out == nullptr) || cgp == 3) ? cg->p_out
                                                                                   : x)
                               : nullptr,
                           shift, parts, skip, OutMap::ident(), fz);
        GG_LAUNCH_CHECK();
        if (pro && fz.p_out != nullptr) step_src = fz.p_out;
      }
    }
    (void)out_size;
    if (ev) GG_HIP(hipEventRecord(ev[k + 1], stream));
    size = out_size;
    src = dst;
  }
  if (n_partials_out) *n_partials_out = np_total;
}

int64_t kron_partials_needed(const gg_kron* K, bool transpose) {
  const std::vector<Factor>& fs = transpose ? K->bwd : K->fwd;
  const Factor& f = fs.back();
  const int64_t n_in = transpose ? K->n_rows : K->n_cols;
  int64_t size = n_in;
  for (const Factor& g : fs) size = size / g.q * g.p;
  const int64_t M = size / f.p;
  // upper bound over the launch variants (the smallest workgroup has 2 strips)
  return ceil_div(M, 2 * 16) * ceil_div(f.JT, kMaxJT);
}

// an upper bound on the workgroups of the (forward) first mode product's first
// launch with a fused CG / Lanczos prologue, whatever kernel it selects (every
// workgroup owns at least one 16-row strip): the capacity of its r.r partial
// array.  The launch reports its actual count (MpFuse::pro_blocks).
int64_t kron_prologue_blocks(const gg_kron* K) {
  const Factor& f = K->fwd[0];
  return ceil_div(K->n_cols / f.q, (int64_t)16);
}

int64_t kron_work_elems(const gg_kron* K, bool transpose) {
  const bool square = transpose ? K->square_steps_bwd : K->square_steps_fwd;
  const int64_t mx = transpose ? K->max_inter_bwd : K->max_inter_fwd;
  return square ? mx : 2 * mx;
}

// one launch covers the first (forward) mode product: fusion layouts 1 / 2
bool kron_first_single_launch(const gg_kron* K) { return K->fwd[0].JT <= kMaxJT; }

int64_t kron_n(const gg_kron* K) { return K->n_rows; }
const BlockOp* kron_block(const gg_kron* K) { return K->blk; }
int kron_d(const gg_kron* K) { return K->d; }
// x_defer mode 2: the side jobs' half boundary of an n-vector (d >= 4: two
// launches per half, quarters of 2 ceil(n / 8) elements; else one launch per
// half of 2 ceil(n / 4)); the closing flush uses the same boundary
int64_t kron_side_half(const gg_kron* K, int64_t n) {
  return K->d >= 4 ? 4 * ceil_div(n, (int64_t)8) : 2 * ceil_div(n, (int64_t)4);
}

static void set_lds_limits() {
  static bool done = false;
  if (done) return;
  for (int jt = 1; jt <= kMaxJT; ++jt)
    for (int cgp = 0; cgp < 8; ++cgp) {
      const ModeConfig mc = select_kernel(jt, cgp);
      GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(mc.fn),
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)mode_lds_bytes(mc)));
    }
  for (int cgp = 0; cgp < 8; ++cgp) {
    const ModeConfig mc = config_t4<13>(cgp);
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(mc.fn),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)mode_lds_bytes(mc)));
  }
  set_fold_lds_limits();
  set_ring_lds_limits();
  done = true;
}

}  // namespace gg

extern "C" {

int gg_kron_create(int d, const int64_t* rows, const int64_t* cols,
                   const double* const* factors_host, gg_kron** out) {
  return gg::guard([&] {
    GG_REQUIRE(out != nullptr, GG_ERR_VALUE, "out is NULL");
    GG_REQUIRE(d >= 1, GG_ERR_VALUE, "need at least one factor");
    gg::knobs_reload();   // the handle's switches are the environment's now
    gg::set_lds_limits();
    gg_kron* K = new gg_kron();
    try {
      K->d = d;
      for (int k = 0; k < d; ++k) {
        GG_REQUIRE(rows[k] >= 1 && cols[k] >= 1, GG_ERR_VALUE, "empty factor");
        GG_REQUIRE(rows[k] <= (1 << 20) && cols[k] <= (1 << 20), GG_ERR_VALUE,
                   "factor too large");
        K->n_rows *= rows[k];
        K->n_cols *= cols[k];
      }
      K->fwd.resize(d);
      K->bwd.resize(d);
      for (int k = 0; k < d; ++k) {
        gg::pack_fragments(factors_host[k], rows[k], cols[k], false, K->fwd[k]);
        gg::pack_fragments(factors_host[k], rows[k], cols[k], true, K->bwd[k]);
        if (rows[k] == cols[k]) {
          gg::pack_fold(factors_host[k], rows[k], false, K->fwd[k]);
          gg::pack_fold(factors_host[k], rows[k], true, K->bwd[k]);
        }
      }
      gg::plan_sizes(K->fwd, K->n_cols, K->max_inter_fwd, K->square_steps_fwd);
      gg::plan_sizes(K->bwd, K->n_rows, K->max_inter_bwd, K->square_steps_bwd);
      K->blk = gg::block_create(d, rows, cols, factors_host);
    } catch (...) {
      gg_kron_destroy(K);
      throw;
    }
    *out = K;
  });
}

int gg_kron_destroy(gg_kron* K) {
  return gg::guard([&] {
    if (!K) return;
    for (auto* v : {&K->fwd, &K->bwd})
      for (gg::Factor& f : *v) {
        if (f.frag) (void)hipFree(f.frag);
        if (f.frag4) (void)hipFree(f.frag4);
        if (f.ffrag) (void)hipFree(f.ffrag);
        if (f.rfrag) (void)hipFree(f.rfrag);
      }
    gg::block_destroy(K->blk);
    delete K;
  });
}

int gg_kron_shape(const gg_kron* K, int transpose, int64_t* n_out, int64_t* n_in,
                  int64_t* work_elems) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr, GG_ERR_VALUE, "NULL handle");
    if (n_out) *n_out = transpose ? K->n_cols : K->n_rows;
    if (n_in) *n_in = transpose ? K->n_rows : K->n_cols;
    if (work_elems) *work_elems = gg::kron_work_elems(K, transpose != 0);
  });
}

int gg_kron_fold_mask(const gg_kron* K, int transpose, int64_t* mask) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && mask != nullptr, GG_ERR_VALUE, "NULL argument");
    const std::vector<gg::Factor>& fs = transpose ? K->bwd : K->fwd;
    int64_t v = 0;
    for (size_t k = 0; k < fs.size(); ++k)
      if (fs[k].ffrag != nullptr) v |= (int64_t)1 << k;
    *mask = v;
  });
}

int gg_kron_matvec(const gg_kron* K, int transpose, const double* x_dev, double* y_dev,
                   double shift, double* work_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(work_dev != nullptr || K->d == 1, GG_ERR_VALUE, "work buffer required");
    gg::kron_apply(K, transpose != 0, x_dev, y_dev, shift, work_dev, nullptr, nullptr,
                   gg::as_stream(stream), nullptr, nullptr, 0, nullptr);
  });
}

int gg_kron_matvec_timed(const gg_kron* K, int transpose, const double* x_dev, double* y_dev,
                         double shift, double* work_dev, int reps, double* launch_ms_host,
                         double* total_ms_host, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev && launch_ms_host && total_ms_host && reps >= 1,
               GG_ERR_VALUE, "bad argument");
    GG_REQUIRE(work_dev != nullptr || K->d == 1, GG_ERR_VALUE, "work buffer required");
    hipStream_t s = gg::as_stream(stream);
    const int d = K->d;
    std::vector<hipEvent_t> ev((size_t)reps * (d + 1));
    for (auto& e : ev) e = nullptr;
    auto release = [&] {
      for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    };
    try {
      for (auto& e : ev) GG_HIP(hipEventCreate(&e));
      for (int r = 0; r < reps; ++r)
        gg::kron_apply(K, transpose != 0, x_dev, y_dev, shift, work_dev, nullptr, nullptr, s,
                       nullptr, nullptr, 0, ev.data() + (size_t)r * (d + 1));
      GG_HIP(hipStreamSynchronize(s));
      for (int k = 0; k < d; ++k) launch_ms_host[k] = 0.0;
      for (int r = 0; r < reps; ++r)
        for (int k = 0; k < d; ++k) {
          float ms = 0.f;
          GG_HIP(hipEventElapsedTime(&ms, ev[(size_t)r * (d + 1) + k],
                                     ev[(size_t)r * (d + 1) + k + 1]));
          launch_ms_host[k] += ms;
        }
      float tot = 0.f;
      GG_HIP(hipEventElapsedTime(&tot, ev.front(), ev.back()));
      *total_ms_host = tot;
    } catch (...) {
      release();
      throw;
    }
    release();
  });
}

// ------------------------------------------------ parity-block basis (P1)
int gg_kron_block_info(const gg_kron* K, int* available, int64_t* n, int* launches) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && available != nullptr, GG_ERR_VALUE, "NULL argument");
    *available = K->blk != nullptr ? 1 : 0;
    if (n) *n = K->blk ? gg::block_n(K->blk) : 0;
    if (launches) *launches = K->blk ? gg::block_launches(K->blk) : 0;
  });
}

int gg_kron_block_fold(const gg_kron* K, int inverse, const double* x_dev, double* y_dev,
                       gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(K->blk != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    GG_REQUIRE(x_dev != y_dev, GG_ERR_VALUE, "x and y must not alias");
    gg::block_fold(K->blk, inverse != 0, x_dev, y_dev, nullptr, gg::as_stream(stream));
  });
}

int gg_kron_block_fold_range(const gg_kron* K, int inverse, const double* x_dev, double* y_dev,
                             int64_t blk0, int64_t nblk, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(K->blk != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    GG_REQUIRE(x_dev != y_dev, GG_ERR_VALUE, "x and y must not alias");
    GG_REQUIRE(nblk >= 1, GG_ERR_VALUE, "empty block range");
    gg::block_fold(K->blk, inverse != 0, x_dev, y_dev, nullptr, gg::as_stream(stream), blk0,
                   nblk);
  });
}

int gg_kron_block_matvec_range(const gg_kron* K, const double* x_dev, double* y_dev,
                               double shift, double* work_dev, int64_t blk0, int64_t nblk,
                               gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(K->blk != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    GG_REQUIRE(nblk >= 1, GG_ERR_VALUE, "empty block range");
    gg::block_apply(K->blk, x_dev, y_dev, shift, work_dev, nullptr, nullptr,
                    gg::as_stream(stream), nullptr, nullptr, 0, nullptr, blk0, nblk);
  });
}

int gg_kron_block_matvec(const gg_kron* K, const double* x_dev, double* y_dev, double shift,
                         double* work_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(K->blk != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    gg::block_apply(K->blk, x_dev, y_dev, shift, work_dev, nullptr, nullptr,
                    gg::as_stream(stream), nullptr, nullptr, 0, nullptr);
  });
}

int gg_kron_block_matvec_timed(const gg_kron* K, const double* x_dev, double* y_dev,
                               double shift, double* work_dev, int reps, double* launch_ms_host,
                               double* total_ms_host, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(K != nullptr && x_dev && y_dev && launch_ms_host && total_ms_host && reps >= 1,
               GG_ERR_VALUE, "bad argument");
    GG_REQUIRE(K->blk != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    hipStream_t s = gg::as_stream(stream);
    const int L = gg::block_launches(K->blk);
    std::vector<hipEvent_t> ev((size_t)reps * (L + 1), nullptr);
    auto release = [&] {
      for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    };
    try {
      for (auto& e : ev) GG_HIP(hipEventCreate(&e));
      for (int r = 0; r < reps; ++r)
        gg::block_apply(K->blk, x_dev, y_dev, shift, work_dev, nullptr, nullptr, s, nullptr,
                        nullptr, 0, ev.data() + (size_t)r * (L + 1));
      GG_HIP(hipStreamSynchronize(s));
      for (int k = 0; k < L; ++k) launch_ms_host[k] = 0.0;
      for (int r = 0; r < reps; ++r)
        for (int k = 0; k < L; ++k) {
          float ms = 0.f;
          GG_HIP(hipEventElapsedTime(&ms, ev[(size_t)r * (L + 1) + k],
                                     ev[(size_t)r * (L + 1) + k + 1]));
          launch_ms_host[k] += ms;
        }
      float tot = 0.f;
      GG_HIP(hipEventElapsedTime(&tot, ev.front(), ev.back()));
      *total_ms_host = tot;
    } catch (...) {
      release();
      throw;
    }
    release();
  });
}

}  // extern "C"

// ===================================================================== P1 sharded
// The Kronecker operator sharded over G ranks along factor 0 (the slowest
// axis), one process per GPU; the exchange steps are the caller's RCCL
// all-to-alls (gp_grief_amd/distributed.py).  Local layout of a sharded
// vector: (m_1, ..., m_{d-1}, a) C-order with a = i_0 - rank * s0 fastest,
// s0 = m_0 / G.  A matvec is
//   phase 1  local mode products for factors 1..d-1 (the slab axis rides along
//            in M); the first one may fuse CG's p = r + beta p; the last one
//            writes its rows in all-to-all chunk order;
//   exchange #1 (N/G^2 per peer)  -> recv = (m_0, R/G) row-major, R = N/m_0;
//   phase 2  mode product for factor 0, columns grouped by destination rank;
//   exchange #2                    -> the result in the input layout.
// Every mode product is the same MFMA kernel as the single-GPU path.

struct gg_kron_dist {
  int d = 0, world = 1, rank = 0;
  std::vector<int64_t> m;
  std::vector<gg::Factor> f;
  int64_t n = 1, n_local = 1, s0 = 1;
  // push mode: every rank's exchange buffer [recv | out] (2 n_local doubles),
  // peers' opened through IPC handles or given directly (same process)
  double* own_xbuf = nullptr;
  double** peers_recv = nullptr;   // device array [world]
  double** peers_out = nullptr;    // device array [world]
  std::vector<void*> opened;       // hipIpcOpenMemHandle bases to close
};

namespace gg {

constexpr int kDistWaves = 4, kDistKC = 3;  // the single-GPU default

template <int JT>
static mode_kernel_t dist_kernel(bool cgp, bool ident) {
  if (cgp && ident) return mode_product_kernel<JT, kDistWaves, kDistKC, 1, 3, true, 1, 2>;
  if (cgp) return mode_product_kernel<JT, kDistWaves, kDistKC, 1, 3, false, 1, 2>;  // d == 2: fused + mapped
  if (ident) return mode_product_kernel<JT, kDistWaves, kDistKC, 0, 3, true, 1, 2>;
  return mode_product_kernel<JT, kDistWaves, kDistKC, 0, 3, false, 1, 2>;
}

static mode_kernel_t select_dist(int jt, bool cgp, bool ident) {
  switch (jt) {
    case 1: return dist_kernel<1>(cgp, ident);
    case 2: return dist_kernel<2>(cgp, ident);
    case 3: return dist_kernel<3>(cgp, ident);
    case 4: return dist_kernel<4>(cgp, ident);
    case 5: return dist_kernel<5>(cgp, ident);
    case 6: return dist_kernel<6>(cgp, ident);
    case 7: return dist_kernel<7>(cgp, ident);
    case 8: return dist_kernel<8>(cgp, ident);
    case 9: return dist_kernel<9>(cgp, ident);
    case 10: return dist_kernel<10>(cgp, ident);
    case 11: return dist_kernel<11>(cgp, ident);
    case 12: return dist_kernel<12>(cgp, ident);
    case 13: return dist_kernel<13>(cgp, ident);
    case 14: return dist_kernel<14>(cgp, ident);
    case 15: return dist_kernel<15>(cgp, ident);
    case 16: return dist_kernel<16>(cgp, ident);
    default: throw Error(GG_ERR_VALUE, "bad tile count");
  }
}


static void dist_step(const Factor& f, const double* X, double* Y, int64_t M, OutMap om,
                      const MpFuse* pro, hipStream_t s) {
  if (M <= 0) return;
  GG_REQUIRE(f.JT <= kMaxJT, GG_ERR_VALUE, "sharded operator supports factors up to 256");
  const bool cgp = pro != nullptr;
  if (f.ffrag != nullptr) {
    // centrosymmetric factor: the folded kernel (identity epilogue = launch
    // kinds 0 / 1, mapped = 8 / 9)
    const int kind = om.identity != 0 ? (cgp ? 1 : 0) : (cgp ? 9 : 8);
    const FoldConfig fc = select_fold(f.fJT, f.fTT, kind);
    const int64_t nblk = ceil_div(M, (int64_t)4 * 16);
    hipLaunchKernelGGL(fc.fn, dim3((unsigned)nblk), dim3(256), fc.lds, s, X, Y, f.ffrag, M,
                       (int)f.q, (int)f.p, f.fKS, fc.jf, 0, nullptr, 0.0, nullptr,
                       cgp ? &pro->sc->done : nullptr, om, cgp ? *pro : MpFuse());
    GG_LAUNCH_CHECK();
    return;
  }
  mode_kernel_t fn = select_dist(f.JT, cgp, om.identity != 0);
  static bool attr[2][2][kMaxJT + 1] = {};
  bool& done = attr[cgp][om.identity != 0][f.JT];
  const size_t lds = 2 * (size_t)kDistKC * f.JT * 64 * sizeof(double);
  if (!done) {
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    done = true;
  }
  const int64_t nblk = ceil_div(M, (int64_t)kDistWaves * 16);
  hipLaunchKernelGGL(fn, dim3((unsigned)nblk), dim3(kDistWaves * 64), lds, s, X, Y, f.frag, M,
                     (int)f.q, (int)f.p, f.KS, f.JT, 0, nullptr, 0.0, nullptr,
                     cgp ? &pro->sc->done : nullptr, om, cgp ? *pro : MpFuse());
  GG_LAUNCH_CHECK();
}

}  // namespace gg

extern "C" {

int gg_kron_dist_create(int d, const int64_t* m, const double* const* factors_host, int world,
                        int rank, gg_kron_dist** out) {
  return gg::guard([&] {
    GG_REQUIRE(out && m && factors_host, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(d >= 2, GG_ERR_VALUE, "the sharded operator needs d >= 2 factors");
    GG_REQUIRE(world >= 1 && rank >= 0 && rank < world, GG_ERR_VALUE, "bad rank / world");
    GG_REQUIRE(m[0] % world == 0, GG_ERR_VALUE, "world size must divide the factor-0 size");
    GG_REQUIRE(m[1] % world == 0, GG_ERR_VALUE, "world size must divide the factor-1 size");
    gg::knobs_reload();   // the handle's switches are the environment's now
    gg::set_lds_limits();
    gg_kron_dist* D = new gg_kron_dist();
    try {
      D->d = d;
      D->world = world;
      D->rank = rank;
      D->m.assign(m, m + d);
      D->f.resize(d);
      for (int k = 0; k < d; ++k) {
        GG_REQUIRE(m[k] >= 1 && m[k] <= 256, GG_ERR_VALUE, "factor size must be in [1, 256]");
        gg::pack_fragments(factors_host[k], m[k], m[k], false, D->f[k]);
        gg::pack_fold(factors_host[k], m[k], false, D->f[k]);
        D->n *= m[k];
      }
      D->n_local = D->n / world;
      D->s0 = m[0] / world;
    } catch (...) {
      gg_kron_dist_destroy(D);
      throw;
    }
    *out = D;
  });
}

int gg_kron_dist_destroy(gg_kron_dist* D) {
  return gg::guard([&] {
    if (!D) return;
    for (gg::Factor& f : D->f) {
      if (f.frag) (void)hipFree(f.frag);
      if (f.frag4) (void)hipFree(f.frag4);
      if (f.ffrag) (void)hipFree(f.ffrag);
      if (f.rfrag) (void)hipFree(f.rfrag);
    }
    for (void* b : D->opened) (void)hipIpcCloseMemHandle(b);
    if (D->peers_recv) (void)hipFree(D->peers_recv);
    if (D->peers_out) (void)hipFree(D->peers_out);
    delete D;
  });
}

int gg_ipc_handle(const void* dev_ptr, void* handle_out, int64_t* offset_out) {
  return gg::guard([&] {
    GG_REQUIRE(dev_ptr && handle_out && offset_out, GG_ERR_VALUE, "NULL argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    GG_HIP(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dev_ptr));
    hipIpcMemHandle_t h;
    GG_HIP(hipIpcGetMemHandle(&h, (void*)base));
    std::memcpy(handle_out, &h, sizeof(h));
    *offset_out = (int64_t)((const char*)dev_ptr - (const char*)base);
  });
}

int gg_kron_dist_set_peers(gg_kron_dist* D, double* own_xbuf, int use_ipc, const void* handles,
                           const int64_t* offsets, void* const* ptrs) {
  return gg::guard([&] {
    GG_REQUIRE(D && own_xbuf, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(use_ipc ? (handles && offsets) : (ptrs != nullptr), GG_ERR_VALUE,
               "peer handles / pointers required");
    GG_REQUIRE(D->peers_recv == nullptr, GG_ERR_VALUE, "peers already set");
    const int G = D->world;
    std::vector<double*> recv(G), out(G);
    for (int g = 0; g < G; ++g) {
      double* base = nullptr;
      if (g == D->rank) {
        base = own_xbuf;
      } else if (use_ipc) {
        hipIpcMemHandle_t h;
        std::memcpy(&h, (const char*)handles + (size_t)g * sizeof(h), sizeof(h));
        void* b = nullptr;
        GG_HIP(hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess));
        D->opened.push_back(b);
        base = reinterpret_cast<double*>((char*)b + offsets[g]);
      } else {
        base = reinterpret_cast<double*>(ptrs[g]);
      }
      recv[g] = base;
      out[g] = base + D->n_local;
    }
    D->own_xbuf = own_xbuf;
    GG_HIP(hipMalloc(&D->peers_recv, G * sizeof(double*)));
    GG_HIP(hipMalloc(&D->peers_out, G * sizeof(double*)));
    GG_HIP(hipMemcpy(D->peers_recv, recv.data(), G * sizeof(double*), hipMemcpyHostToDevice));
    GG_HIP(hipMemcpy(D->peers_out, out.data(), G * sizeof(double*), hipMemcpyHostToDevice));
  });
}

int gg_kron_dist_fold_mask(const gg_kron_dist* D, int64_t* mask) {
  return gg::guard([&] {
    GG_REQUIRE(D && mask, GG_ERR_VALUE, "NULL argument");
    int64_t v = 0;
    for (size_t k = 0; k < D->f.size(); ++k)
      if (D->f[k].ffrag != nullptr) v |= (int64_t)1 << k;
    *mask = v;
  });
}

int gg_kron_dist_sizes(const gg_kron_dist* D, int64_t* n_local, int64_t* work_elems) {
  return gg::guard([&] {
    GG_REQUIRE(D, GG_ERR_VALUE, "NULL handle");
    if (n_local) *n_local = D->n_local;
    if (work_elems) *work_elems = D->n_local;
  });
}

static int dist_phase1(const gg_kron_dist* D, double* x_local_dev, double* send_dev,
                       double* work_dev, const double* cg_r_dev, const void* cg_scalars_dev,
                       gg_stream stream, bool push) {
  return gg::guard([&] {
    GG_REQUIRE(D && x_local_dev && send_dev && work_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(!push || D->peers_recv, GG_ERR_VALUE, "push mode needs gg_kron_dist_set_peers");
    GG_REQUIRE((cg_r_dev == nullptr) == (cg_scalars_dev == nullptr), GG_ERR_VALUE,
               "CG fusion needs both r and the scalars");
    hipStream_t s = gg::as_stream(stream);
    const int d = D->d;
    const int G = D->world;
    gg::MpFuse pro;
    pro.r = const_cast<double*>(cg_r_dev);  // read only (textbook prologue)
    pro.sc = reinterpret_cast<const gg::CgScalars*>(cg_scalars_dev);
    pro.p_out = x_local_dev;                // p updated in place
    const int64_t nl = D->n_local;
    const double* src = x_local_dev;
    for (int k = 1; k < d; ++k) {
      const gg::Factor& f = D->f[k];
      const int64_t M = nl / f.q;
      const bool last = (k == d - 1);
      gg::OutMap om = gg::OutMap::ident();
      double* dst;
      if (last) {
        dst = send_dev;
        if (d == 2) {  // rows = slab index, columns j1 grouped by destination
          const int64_t cg = f.p / G;
          om = gg::OutMap{0, cg, D->s0 * cg, 1, 1, 0, cg};
        } else {       // rows = (a, j1..j_{d-2}); chunk by j1
          const int64_t mi = M / D->s0;
          const int64_t cr = mi / G;
          om = gg::OutMap{0, f.p, 0, mi, cr, D->s0 * cr * f.p, cr * f.p};
        }
        if (push) {  // chunk h goes to rank h's receive buffer, at this rank's slot
          om.push = d == 2 ? 2 : 1;
          om.self_off = (int64_t)D->rank * (D->n_local / G);
          om.peers = D->peers_recv;
        }
      } else {
        // alternate work / send so that the last local step lands in send
        dst = ((d - 1 - k) % 2 == 0) ? send_dev : work_dev;
      }
      const bool fuse = (k == 1) && cg_r_dev != nullptr;
      gg::dist_step(f, src, dst, M, om, fuse ? &pro : nullptr, s);
      src = dst;
    }
  });
}

// ---- fused sharded CG, phase 1 (gp_grief_amd/distributed.py, recurrence
// "fused"): the single-GPU fused recurrence's launches on the local slab --
// mode product 1 carries the prologue (r -= alpha q_old when pending, p_new
// = r + beta p_old into its own buffer, r.r and p_new.q_old partials), mode
// product 2 the balanced x side job (half sc->xh of the deferred pair), the
// last one the all-to-all / push epilogue.  Folded (centrosymmetric)
// factors 1..d-1 and d >= 4 only (the caller checks gg_kron_dist_fold_mask).
static int dist_phase1_fused(const gg_kron_dist* D, const double* p_old, double* p_new,
                             double* send_dev, double* work_dev, double* r_dev,
                             const double* q_old, double* x_dev, gg_cgs* cgs, double shift,
                             int push, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(D && p_old && p_new && send_dev && work_dev && r_dev && q_old && x_dev && cgs,
               GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(D->d >= 4, GG_ERR_VALUE, "the fused sharded CG needs d >= 4");
    for (int k = 1; k < D->d; ++k)
      GG_REQUIRE(D->f[k].ffrag != nullptr, GG_ERR_VALUE,
                 "the fused sharded CG needs centrosymmetric (folded) factors 1..d-1");
    GG_REQUIRE(!push || D->peers_recv, GG_ERR_VALUE, "push mode needs gg_kron_dist_set_peers");
    GG_REQUIRE(D->n_local % 2 == 0 &&
                   ((reinterpret_cast<uintptr_t>(x_dev) | reinterpret_cast<uintptr_t>(p_new)) &
                    15) == 0,
               GG_ERR_VALUE, "the fused sharded CG needs 16-byte aligned, even-length vectors");
    hipStream_t s = gg::as_stream(stream);
    const int d = D->d;
    const int G = D->world;
    const int64_t nl = D->n_local;
    gg::CgScalars* sc = gg::cgs_scalars_ptr(cgs);
    const int* skip = &sc->done;
    // balanced x deferral with one side launch per iteration: half h of x
    const int64_t H = 2 * gg::ceil_div(nl, (int64_t)4);
    const double* src = p_old;
    for (int k = 1; k < d; ++k) {
      const gg::Factor& f = D->f[k];
      const int64_t M = nl / f.q;
      const bool last = (k == d - 1);
      gg::OutMap om = gg::OutMap::ident();
      double* dst;
      int kind = 0;
      gg::MpFuse fz;
      if (last) {
        dst = send_dev;
        const int64_t mi = M / D->s0;
        const int64_t cr = mi / G;
        om = gg::OutMap{0, f.p, 0, mi, cr, D->s0 * cr * f.p, cr * f.p};
        if (push) {
          om.push = 1;
          om.self_off = (int64_t)D->rank * (D->n_local / G);
          om.peers = D->peers_recv;
        }
        kind = 8;
      } else {
        dst = ((d - 1 - k) % 2 == 0) ? send_dev : work_dev;
        kind = k == 1 ? 2 : k == 2 ? 4 : 0;
      }
      const bool lean_ok = 4 * 3 * gg::ceil_div((int64_t)f.fKS, (int64_t)3) <= (int64_t)f.q &&
                           4 * 2 * gg::ceil_div((int64_t)f.fKS, (int64_t)2) <= (int64_t)f.q &&
                           32 * M < ((int64_t)1 << 32);
      const gg::FoldConfig fc = gg::select_fold(f.fJT, f.fTT, kind, lean_ok);
      const int64_t nblk = gg::ceil_div(M, (int64_t)fc.waves * 16);
      if (kind == 2) {
        int64_t cap = 0;
        fz.rr_part = gg::cgs_rr_part(cgs, nblk, &cap);
        fz.rr_cap = cap;
        fz.pqo_stride = cap;
        fz.r = r_dev;
        fz.q_old = q_old;
        fz.qshift = shift;   // q_old = K p_old: gg_cgs_fused_post does not shift it
        fz.p_out = p_new;
        fz.sc = sc;
        gg::cgs_set_pro_blocks(cgs, nblk);
      } else if (kind == 4) {
        fz.sc = sc;
        fz.sx = x_dev;
        fz.xdefer = 2;
        fz.soff = 0;
        fz.sn = std::min(H, nl);
        fz.soff_h1 = std::min(H, nl);
        fz.sn_h1 = nl - fz.soff_h1;
        fz.schunk = 2 * gg::ceil_div(std::max<int64_t>(std::max(fz.sn, fz.sn_h1), 1), 2 * nblk);
      }
      if (fc.lean)
        GG_REQUIRE(4 * gg::ceil_div((int64_t)f.fKS, (int64_t)fc.kc) * fc.kc <= (int64_t)f.q &&
                       32 * M < ((int64_t)1 << 32),
                   GG_ERR_VALUE, "lean folded kernel outside its row / offset range");
      hipLaunchKernelGGL(fc.fn, dim3((unsigned)nblk), dim3(64 * fc.waves), fc.lds, s, src, dst,
                         f.ffrag, M, (int)f.q, (int)f.p, f.fKS, fc.jf, 0, nullptr, 0.0, nullptr,
                         skip, om, fz);
      GG_LAUNCH_CHECK();
      // the later steps read the updated direction
      src = dst;
    }
  });
}

int gg_kron_dist_phase1_fused(const gg_kron_dist* D, const double* p_old_dev, double* p_new_dev,
                              double* send_dev, double* work_dev, double* r_dev,
                              const double* q_old_dev, double* x_dev, gg_cgs* cgs,
                              double shift, int push, gg_stream stream) {
  return dist_phase1_fused(D, p_old_dev, p_new_dev, send_dev, work_dev, r_dev, q_old_dev, x_dev,
                           cgs, shift, push, stream);
}

int gg_kron_dist_phase1(const gg_kron_dist* D, double* x_local_dev, double* send_dev,
                        double* work_dev, const double* cg_r_dev, const void* cg_scalars_dev,
                        gg_stream stream) {
  return dist_phase1(D, x_local_dev, send_dev, work_dev, cg_r_dev, cg_scalars_dev, stream, false);
}

int gg_kron_dist_phase1_push(const gg_kron_dist* D, double* x_local_dev, double* scratch_dev,
                             double* work_dev, const double* cg_r_dev,
                             const void* cg_scalars_dev, gg_stream stream) {
  return dist_phase1(D, x_local_dev, scratch_dev, work_dev, cg_r_dev, cg_scalars_dev, stream,
                     true);
}

int gg_kron_dist_phase2_push(const gg_kron_dist* D, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(D && D->peers_out, GG_ERR_VALUE, "push mode needs gg_kron_dist_set_peers");
    const gg::Factor& f = D->f[0];
    const int64_t C = D->n_local / f.q;
    gg::OutMap om{0, D->s0, C * D->s0, C, C, 0, 0};
    om.push = 2;  // destination = output column group j / s0
    om.self_off = (int64_t)D->rank * (D->n_local / D->world);
    om.peers = D->peers_out;
    gg::dist_step(f, D->own_xbuf, nullptr, C, om, nullptr, gg::as_stream(stream));
  });
}

int gg_kron_dist_phase2(const gg_kron_dist* D, const double* recv_dev, double* send_dev,
                        gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(D && recv_dev && send_dev && recv_dev != send_dev, GG_ERR_VALUE, "bad argument");
    const gg::Factor& f = D->f[0];
    const int64_t C = D->n_local / f.q;  // = R / G
    const gg::OutMap om{0, D->s0, C * D->s0, C, C, 0, 0};
    gg::dist_step(f, recv_dev, send_dev, C, om, nullptr, gg::as_stream(stream));
  });
}

}  // extern "C"
