// Device helpers shared by the mode-product kernels (gg_kron.hip,
// gg_kron_fold.hip) and the folded-kernel launch table.  Internal.
#pragma once

#include "gg_internal.h"

namespace gg {

typedef double d4 __attribute__((ext_vector_type(4)));

typedef void (*mode_kernel_t)(const double*, double*, const double*, int64_t, int, int, int,
                              int, int, const double*, double, double*, const int*, OutMap,
                              MpFuse);

// Per-workgroup partial sums of a mode product: p.q (+ r.q, q.q when edots)
// of the epilogue, r.r (or |w|^2) of the fused prologue; a CG prologue passes
// p_new.q_old in the r.q slot (MpFuse::pqo_stride).  Called after the
// k-loop's last barrier (LDS is free); red: 4 * kWaves doubles of LDS.
template <int kWaves, int CGP, bool edots, bool kRaw>
__device__ __forceinline__ void mp_block_sums(double dsum, double rqsum, double qqsum,
                                              double rr_acc, double* __restrict__ dot_partials,
                                              const MpFuse& fz, double* red, int64_t blk) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool want_dot = dot_partials != nullptr;
  const bool want_rr = CGP >= 2 && fz.rr_part != nullptr;
  if (!(want_dot || want_rr)) return;
  double v4[4] = {dsum, rqsum, qqsum, rr_acc};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v4[i] += __shfl_xor(v4[i], off, 64);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[4 * wave + i] = v4[i];
  if (kRaw) {
    __builtin_amdgcn_s_waitcnt((7 << 4) | 0xC00F);  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
  if (threadIdx.x < 4) {
    const int i = threadIdx.x;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += red[4 * w + i];
    if (i == 0 && want_dot) dot_partials[blk] = s;
    if (i == 1 && edots && want_dot) dot_partials[fz.pstride + blk] = s;
    if (i == 2 && want_dot && edots) dot_partials[2 * fz.pstride + blk] = s;
    if (i == 3 && want_rr) fz.rr_part[blk] = s;
    if (i == 1 && CGP == 2 && !edots && want_rr && fz.pqo_stride > 0)
      fz.rr_part[fz.pqo_stride + blk] = s;
  }
}

// Side job (fused CG, second / third mode product): x += alpha p_old over
// this workgroup's slice, 16-byte lanes.  The mode product has HBM headroom;
// the other workgroups of the CU keep the matrix cores busy meanwhile.
// 16-byte loads / stores, non-temporal when kNT (streams read or written once
// per iteration)
typedef double nt_d2 __attribute__((ext_vector_type(2)));
template <bool kNT>
__device__ __forceinline__ double2 ld2(const double* p) {
  if constexpr (kNT) {
    const nt_d2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_d2*>(p));
    return double2{v.x, v.y};
  }
  return *reinterpret_cast<const double2*>(p);
}
template <bool kNT>
__device__ __forceinline__ void st2(double* p, double2 v) {
  if constexpr (kNT) {
    __builtin_nontemporal_store(nt_d2{v.x, v.y}, reinterpret_cast<nt_d2*>(p));
  } else {
    *reinterpret_cast<double2*>(p) = v;
  }
}

template <int kThreads, bool kNT = false>
__device__ __forceinline__ void mp_side_job(const MpFuse& fz, int64_t blk) {
  if (fz.sx == nullptr) return;
  int64_t lo = blk * fz.schunk;
  int64_t hi = min(fz.sn, lo + fz.schunk);
  double* __restrict__ sx = fz.sx;
  constexpr int kB = 4;
  if (fz.xdefer == 2) {
    // balanced: half sc->xh of the pair completed two iterations ago (this
    // launch's quarter of it), so every side launch carries about one pass
    const int h = fz.sc->xh;
    if (h >= 2) return;
    const int64_t off = h ? fz.soff_h1 : fz.soff;
    const int64_t len = h ? fz.sn_h1 : fz.sn;
    hi = min(len, lo + fz.schunk);
    const double c0 = fz.sc->xc[0], c1 = fz.sc->xc[1];
    const double* __restrict__ p0 = fz.sc->xp[0] + off;
    const double* __restrict__ p1 = fz.sc->xp[1] + off;
    double* __restrict__ xo = sx + off;
    constexpr int kB2 = 2;
    int64_t i = lo + 2 * threadIdx.x;
    for (; i + 2 * kThreads * (kB2 - 1) + 1 < hi; i += 2 * kThreads * kB2) {
      double2 xv2[kB2], a2[kB2], b2[kB2];
#pragma unroll
      for (int u = 0; u < kB2; ++u) {
        xv2[u] = ld2<kNT>(xo + i + 2 * kThreads * u);
        a2[u] = ld2<kNT>(p0 + i + 2 * kThreads * u);
        b2[u] = ld2<kNT>(p1 + i + 2 * kThreads * u);
      }
#pragma unroll
      for (int u = 0; u < kB2; ++u) {
        xv2[u].x += c0 * a2[u].x + c1 * b2[u].x;
        xv2[u].y += c0 * a2[u].y + c1 * b2[u].y;
        st2<kNT>(xo + i + 2 * kThreads * u, xv2[u]);
      }
    }
    for (; i < hi; i += 2 * kThreads) {
      xo[i] += c0 * p0[i] + c1 * p1[i];
      if (i + 1 < hi) xo[i + 1] += c0 * p0[i + 1] + c1 * p1[i + 1];
    }
    return;
  }
  if (fz.xdefer) {
    // two deferred steps at once: x += c0 p0 + c1 p1 (4 passes per two CG
    // iterations instead of 6); 2 double2 per operand in flight keeps the
    // fused kernels within their register budget
    constexpr int kB = 2;
    if (fz.sc->xpend != 2) return;
    const double c0 = fz.sc->xc[0], c1 = fz.sc->xc[1];
    const double* __restrict__ p0 = fz.sc->xp[0] + fz.soff;
    const double* __restrict__ p1 = fz.sc->xp[1] + fz.soff;
    int64_t i = lo + 2 * threadIdx.x;
    for (; i + 2 * kThreads * (kB - 1) + 1 < hi; i += 2 * kThreads * kB) {
      double2 xv2[kB], a2[kB], b2[kB];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        xv2[u] = *reinterpret_cast<const double2*>(sx + i + 2 * kThreads * u);
        a2[u] = *reinterpret_cast<const double2*>(p0 + i + 2 * kThreads * u);
        b2[u] = *reinterpret_cast<const double2*>(p1 + i + 2 * kThreads * u);
      }
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        xv2[u].x += c0 * a2[u].x + c1 * b2[u].x;
        xv2[u].y += c0 * a2[u].y + c1 * b2[u].y;
        *reinterpret_cast<double2*>(sx + i + 2 * kThreads * u) = xv2[u];
      }
    }
    for (; i < hi; i += 2 * kThreads) {
      sx[i] += c0 * p0[i] + c1 * p1[i];
      if (i + 1 < hi) sx[i + 1] += c0 * p0[i + 1] + c1 * p1[i + 1];
    }
    return;
  }
  if (!fz.sc->pending) return;
  const double al = fz.sc->alpha;
  const double* __restrict__ sp = fz.sp;
  int64_t i = lo + 2 * threadIdx.x;
  for (; i + 2 * kThreads * (kB - 1) + 1 < hi; i += 2 * kThreads * kB) {
    double2 xv2[kB], pv2[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      xv2[u] = *reinterpret_cast<const double2*>(sx + i + 2 * kThreads * u);
      pv2[u] = *reinterpret_cast<const double2*>(sp + i + 2 * kThreads * u);
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      xv2[u].x += al * pv2[u].x;
      xv2[u].y += al * pv2[u].y;
      *reinterpret_cast<double2*>(sx + i + 2 * kThreads * u) = xv2[u];
    }
  }
  for (; i < hi; i += 2 * kThreads) {
    sx[i] += al * sp[i];
    if (i + 1 < hi) sx[i + 1] += al * sp[i + 1];
  }
}

// The folded (centrosymmetric) mode product, gg_kron_fold.hip: one kernel per
// (tiles per half JT, 4x4 tail fragments TT, kron_apply launch kind; kinds
// 8 / 9 = the sharded operator's OutMap epilogue, plain / textbook prologue)
struct FoldConfig {
  mode_kernel_t fn;
  int kc, jf;     // k-steps per LDS chunk, fragments per k-step (both halves)
  size_t lds;     // dynamic LDS bytes
  bool lean = false;   // kLean A addressing: the launch checks its row / offset range
  int waves = 4;       // waves per workgroup (16 rows b each)
};
bool fold_kind(int kind);
// lean_ok: the launch is in the kLean kernels' range (every chunk's rows
// inside the factor, 4 kc ceil(KS / kc) <= m, and 32 M < 2^32)
FoldConfig select_fold(int JT, int TT, int kind, bool lean_ok = false);
// the LDS-staged identity epilogue for launches with a shift / dot operand
// (kinds 0, 3, 6; m even, 16-byte aligned vectors; GG_FOLD_STAGE=0 disables)
bool fold_staged_available(int JT, int TT, int kind);
FoldConfig select_fold_staged(int JT, int TT, int kind, bool lean_ok = false);
void set_fold_lds_limits();

// The persistent LDS-DMA ring version of the plain folded launch
// (gg_kron_ring.hip): B fragments from Factor::rfrag ([fKS][16][64]).
typedef void (*ring_kernel_t)(const double*, double*, const double*, int64_t, int, int, int64_t,
                              const int*, MpFuse);
struct RingConfig {
  ring_kernel_t fn;
  int waves, ns, kc;   // waves per workgroup, ring stages, k-steps per stage
  size_t lds;          // dynamic LDS bytes
};
int ring_variant_env();   // GG_FOLD_RING: 0 = off (the chunked kernel), else on
bool ring_available(int JT, int TT, int64_t m);
RingConfig select_ring(int JT, int TT);
// persistent grid: resident workgroups per CU x CUs, at most nblk
int ring_grid(const RingConfig& rc, int cus, int64_t nblk);
void set_ring_lds_limits();

}  // namespace gg
