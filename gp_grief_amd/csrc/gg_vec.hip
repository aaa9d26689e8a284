// Vector side of the Krylov solvers on MI355X: HBM-bound, coalesced,
// wave-reduced (shfl over 64 lanes -> LDS across waves -> per-block partial ->
// one deterministic single-block reduction).  No float atomics anywhere, so
// every dot product is bitwise reproducible run to run.
//
// The reference has no CG or Lanczos; the CG recurrence is the
// one of scipy.sparse.linalg.cg (oracle/cg.py restates it), driven here with
// every scalar resident on the device so the host only polls convergence.
#include <cmath>
#include <vector>

#include <map>

#include "gg_internal.h"

namespace gg {

// defined in gg_kron.hip
void kron_apply(const gg_kron* K, bool transpose, const double* x, double* y, double shift,
                double* work, double* dot_partials, const int* skip, hipStream_t stream,
                int64_t* n_partials_out, const MpFuse* cg, int cgp, hipEvent_t* ev);
int64_t kron_partials_needed(const gg_kron* K, bool transpose);
int64_t kron_prologue_blocks(const gg_kron* K);
int64_t kron_work_elems(const gg_kron* K, bool transpose);
int64_t kron_n(const gg_kron* K);
int kron_d(const gg_kron* K);
bool kron_first_single_launch(const gg_kron* K);
int64_t kron_side_half(const gg_kron* K, int64_t n);
const BlockOp* kron_block(const gg_kron* K);

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// block (<= 1024 threads) sum; result valid in thread 0
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double red[16];
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) s += red[i];
  }
  return s;
}

__global__ __launch_bounds__(kVecThreads) void dot_partials_kernel(const double* __restrict__ x,
                                                                   const double* __restrict__ y,
                                                                   int64_t n,
                                                                   double* __restrict__ partials) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n2 = n / 2;
  const double2* x2 = reinterpret_cast<const double2*>(x);
  const double2* y2 = reinterpret_cast<const double2*>(y);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
    const double2 a = x2[i], b = y2[i];
    acc = fma(a.x, b.x, acc);
    acc = fma(a.y, b.y, acc);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) acc = fma(x[n - 1], y[n - 1], acc);
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void reduce_kernel(const double* __restrict__ partials,
                                                      int64_t count, double* __restrict__ out) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += blockDim.x) acc += partials[i];
  const double s = block_sum(acc);
  if (threadIdx.x == 0) *out = s;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void launch_dot_partials(const double* x, const double* y, int64_t n, double* partials,
                         int nblocks, hipStream_t s) {
  GG_REQUIRE(aligned16(x) && aligned16(y), GG_ERR_VALUE, "vectors must be 16-byte aligned");
  hipLaunchKernelGGL(dot_partials_kernel, dim3(nblocks), dim3(kVecThreads), 0, s, x, y, n,
                     partials);
  GG_LAUNCH_CHECK();
}

void launch_reduce_to(const double* partials, int64_t count, double* out, hipStream_t s) {
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(1024), 0, s, partials, count, out);
  GG_LAUNCH_CHECK();
}

static int vec_blocks(int64_t n) {
  const int64_t want = ceil_div(std::max<int64_t>(n / 2, 1), kVecThreads);
  return (int)std::min<int64_t>(kVecBlocks, std::max<int64_t>(want, 1));
}

__global__ __launch_bounds__(kVecThreads) void axpby_kernel(double a, const double* __restrict__ x,
                                                            double b, double* __restrict__ y,
                                                            int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = a * x[i] + b * y[i];
}

// ------------------------------------------------------------------ CG kernels
// (p = beta p + r is fused into the first mode product, gg_kron.hip)

// alpha = rho / (p.q)
__global__ __launch_bounds__(1024) void cg_alpha_kernel(const double* __restrict__ partials,
                                                        int64_t count, CgScalars* sc) {
  if (sc->done) return;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += blockDim.x) acc += partials[i];
  const double s = block_sum(acc);
  if (threadIdx.x == 0) {
    sc->pq = s;
    sc->alpha = sc->rho / s;
  }
}

// x += alpha p ; r -= alpha q ; partial r.r
__global__ __launch_bounds__(kVecThreads) void cg_xr_update_kernel(
    double* __restrict__ x, double* __restrict__ r, const double* __restrict__ p,
    const double* __restrict__ q, int64_t n, const CgScalars* __restrict__ sc,
    double* __restrict__ partials, int need_pending) {
  // need_pending: 0 always, 1 only with a pending fused update, 2 only when
  // the fused recurrence asked for a repair (cancelled beta); x == nullptr:
  // r only (x_defer keeps its own x bookkeeping, cg_x_flush_kernel)
  if (sc->done || (need_pending && !sc->pending)) return;
  if (need_pending == 2 && !sc->repair) return;
  if (x == nullptr) {
    const double a = sc->alpha;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const double rv = r[i] - a * q[i];
      r[i] = rv;
      acc = fma(rv, rv, acc);
    }
    const double s = block_sum(acc);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
    return;
  }
  const double a = sc->alpha;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n2 = n / 2;
  double2* x2 = reinterpret_cast<double2*>(x);
  double2* r2 = reinterpret_cast<double2*>(r);
  const double2* p2 = reinterpret_cast<const double2*>(p);
  const double2* q2 = reinterpret_cast<const double2*>(q);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
    const double2 pv = p2[i], qv = q2[i];
    double2 xv = x2[i], rv = r2[i];
    xv.x += a * pv.x;
    xv.y += a * pv.y;
    rv.x -= a * qv.x;
    rv.y -= a * qv.y;
    x2[i] = xv;
    r2[i] = rv;
    acc = fma(rv.x, rv.x, acc);
    acc = fma(rv.y, rv.y, acc);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {
    x[n - 1] += a * p[n - 1];
    r[n - 1] -= a * q[n - 1];
    acc = fma(r[n - 1], r[n - 1], acc);
  }
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// rho_prev = rho ; rho = r.r ; beta ; iteration count ; convergence
__global__ __launch_bounds__(1024) void cg_rho_kernel(const double* __restrict__ partials,
                                                      int64_t count, CgScalars* sc,
                                                      int need_pending) {
  if (sc->done || (need_pending && !sc->pending)) return;
  if (need_pending == 2 && !sc->repair) return;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += blockDim.x) acc += partials[i];
  const double s = block_sum(acc);
  if (threadIdx.x == 0) {
    sc->rho_prev = sc->rho;
    sc->rho = s;
    sc->beta = s / sc->rho_prev;
    sc->iters += 1;
    sc->first = 0;
    sc->pending = 0;
    sc->repair = 0;
    sc->rstored = 1;   // r is in its buffer (the update just wrote it)
    if (!(sqrt(s) >= sc->tol)) sc->done = 1;  // also stops on NaN
  }
}

// derived r (CgScalars::rstored): write the current r into its buffer --
// r = (rstored ? r : p - beta_p p_prev) (- alpha q when pending) -- with its
// r.r partials.  mode 2: only when the recurrence asked for a repair (before
// the prologue); mode 1: the close (whenever r is not stored or an update is
// pending).  cg_rho_kernel / cg_r_stored_kernel then mark it stored.
// The directions are the ones the scalars recorded (sc->rp_cur, rp_prev).
__global__ __launch_bounds__(kVecThreads) void cg_r_materialize_kernel(
    double* __restrict__ r, const double* __restrict__ q, int64_t n,
    const CgScalars* __restrict__ sc, double* __restrict__ partials, int mode) {
  if (sc->done && sc->rstored) return;
  if (mode == 2 && (sc->done || !sc->repair || !sc->pending)) return;
  if (mode == 1 && sc->rstored && !sc->pending) return;
  const bool st = sc->rstored != 0;
  const double bp = sc->beta_p;
  const double* __restrict__ p = sc->rp_cur;
  const double* __restrict__ pprev = sc->rp_prev;
  const double a = sc->pending ? sc->alpha : 0.0;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double rv = st ? r[i] : fma(-bp, pprev[i], p[i]);
    if (a != 0.0) rv -= a * q[i];
    r[i] = rv;
    acc = fma(rv, rv, acc);
  }
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ void cg_r_stored_kernel(CgScalars* sc) { sc->rstored = 1; }

// x_defer: fold the deferred steps into x, x += sum_{i < xpend} xc[i] xp[i]
// (also after convergence: x lags r by up to two steps)
__global__ __launch_bounds__(kVecThreads) void cg_x_flush_kernel(double* __restrict__ x,
                                                                 int64_t n,
                                                                 const CgScalars* __restrict__ sc) {
  const int k = sc->xpend;
  if (k <= 0) return;
  const double c0 = sc->xc[0], c1 = k >= 2 ? sc->xc[1] : 0.0;
  const double* __restrict__ p0 = sc->xp[0];
  const double* __restrict__ p1 = k >= 2 ? sc->xp[1] : sc->xp[0];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    x[i] += c0 * p0[i] + c1 * p1[i];
}

// x_defer mode 2 on its own stream: half sc->xh of the active pair, x += c0
// p0 + c1 p1 over [0, H) or [H, n) -- no state change (the scalars kernel
// advances xh).  One 256-thread workgroup per CU, few registers, no LDS: it
// fits beside a ring mode product's workgroup (2 waves / SIMD at 226 VGPRs,
// 131 KB of LDS) and streams while that one computes.  Non-temporal: every
// element is touched once per iteration.
__global__ __launch_bounds__(256) void cg_x_half_kernel(double* __restrict__ x, int64_t n,
                                                        int64_t H,
                                                        const CgScalars* __restrict__ sc) {
  if (sc->done) return;
  const int h = sc->xh;
  if (h >= 2) return;
  const int64_t lo = h ? H : 0, hi = h ? n : H;
  const double c0 = sc->xc[0], c1 = sc->xc[1];
  const double* __restrict__ p0 = sc->xp[0];
  const double* __restrict__ p1 = sc->xp[1];
  typedef double v2 __attribute__((ext_vector_type(2)));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 2;
  int64_t i = lo + 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  constexpr int kU = 2;
  for (; i + (kU - 1) * stride + 1 < hi; i += kU * stride) {
    v2 xv[kU], a[kU], b[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      xv[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(x + i + u * stride));
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p0 + i + u * stride));
      b[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p1 + i + u * stride));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      xv[u] += c0 * a[u] + c1 * b[u];
      __builtin_nontemporal_store(xv[u], reinterpret_cast<v2*>(x + i + u * stride));
    }
  }
  for (; i < hi; i += stride) {
    x[i] += c0 * p0[i] + c1 * p1[i];
    if (i + 1 < hi) x[i + 1] += c0 * p0[i + 1] + c1 * p1[i + 1];
  }
}

void launch_x_half(double* x, int64_t n, int64_t H, const CgScalars* sc, hipStream_t s) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  hipLaunchKernelGGL(cg_x_half_kernel, dim3((unsigned)std::max(cus, 1)), dim3(256), 0, s, x, n,
                     H, sc);
  GG_LAUNCH_CHECK();
}

// x_defer mode 2: x += xsc xsp (the waiting single step) + the active pair
// on the halves not yet applied (half 0 = [0, H), half 1 = [H, n))
__global__ __launch_bounds__(kVecThreads) void cg_x_flush2_kernel(double* __restrict__ x,
                                                                  int64_t n, int64_t H,
                                                                  const CgScalars* __restrict__ sc) {
  const int h = sc->xh, xs = sc->xs;
  if (h >= 2 && !xs) return;
  const double cs = xs ? sc->xsc : 0.0;
  const double* __restrict__ ps = xs ? sc->xsp : x;
  const double c0 = h < 2 ? sc->xc[0] : 0.0, c1 = h < 2 ? sc->xc[1] : 0.0;
  const double* __restrict__ p0 = h < 2 ? sc->xp[0] : x;
  const double* __restrict__ p1 = h < 2 ? sc->xp[1] : x;
  const int64_t from = h == 0 ? 0 : H;   // first element the pair still owes
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double v = x[i];
    if (xs) v += cs * ps[i];
    if (h < 2 && i >= from) v += c0 * p0[i] + c1 * p1[i];
    x[i] = v;
  }
}

// The CG prologue's stream pattern alone (gg_cg_calibrate): per element,
// read p_old, r and q, write r, p_new and q -- the six passes of the fused
// prologue launch over the same buffers, with its non-temporal mask (every
// stream but the q write, the launch's output Y); with derived r (RD) the
// five of that prologue: read p_old, p_{j-2} (in r's place) and q, write
// p_new and q.  Values pass through unchanged (r = r, p_new = p_old, q = q;
// the loaded values pass an opaque asm so the compiler cannot drop a store of
// what was just loaded from the same address).  No MFMA work: the launch's
// streams alone on this box.
template <bool RD>
__global__ __launch_bounds__(256) void cg_stream_probe_kernel(double* __restrict__ r,
                                                              const double* __restrict__ p,
                                                              double* __restrict__ p2,
                                                              double* __restrict__ q,
                                                              int64_t n) {
  typedef double v2 __attribute__((ext_vector_type(2)));
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 2;
  constexpr int kU = 2;
  int64_t i = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  for (; i + (kU - 1) * stride + 1 < n; i += kU * stride) {
    v2 a[kU], b[kU], c[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(p + i + u * stride));
      b[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(r + i + u * stride));
      c[u] = __builtin_nontemporal_load(reinterpret_cast<const v2*>(q + i + u * stride));
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) asm volatile("" : "+v"(a[u]), "+v"(b[u]), "+v"(c[u]));
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (RD) {
        // keep the p_{j-2} stream's loads live without changing p_new
        asm volatile("" : : "v"(b[u]));
      } else {
        __builtin_nontemporal_store(b[u], reinterpret_cast<v2*>(r + i + u * stride));
      }
      __builtin_nontemporal_store(a[u], reinterpret_cast<v2*>(p2 + i + u * stride));
      *reinterpret_cast<v2*>(q + i + u * stride) = c[u];
    }
  }
  for (; i < n; i += stride) {
    p2[i] = p[i];
    if (i + 1 < n) p2[i + 1] = p[i + 1];
  }
}

__global__ void cg_x_flushed_kernel(CgScalars* sc) {
  sc->xpend = 0;
  sc->xh = 2;
  sc->xs = 0;
}

// x_defer mode 3: every region gets the steps it has not seen, [wa[r], wn)
// (at most wk of them, all still in the ring) -- the side job's expression
__global__ __launch_bounds__(kVecThreads) void cg_x_flush3_kernel(double* __restrict__ x,
                                                                  int64_t n, int64_t R,
                                                                  const CgScalars* __restrict__ sc) {
  const int K = sc->wk, slots = K + 1, wn = sc->wn;
  if (K <= 0) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int r = (int)(i / R);
    double s = 0.0;
    for (int t = sc->wa[r]; t < wn; ++t) s += sc->wc[t % slots] * sc->wp[t % slots][i];
    x[i] = x[i] + s;
  }
}

__global__ void cg_x_flushed3_kernel(CgScalars* sc) {
  for (int r = 0; r < kXWinMax; ++r) sc->wa[r] = sc->wn;
  sc->warm = 0;
}

// x_defer mode 3 at gg_cg_start: window K, nothing applied or armed
__global__ void cg_xwin_init_kernel(CgScalars* sc, int K) {
  sc->wk = K;
  sc->wn = 0;
  sc->wnext = 0;
  sc->warm = 0;
  sc->sreg = 0;
  sc->scnt = 0;
  for (int r = 0; r < kXWinMax; ++r) sc->wa[r] = 0;
}

// Fused recurrence, end of iteration j (after the last mode product):
//   rho_j = r_j.r_j (partials of the first mode product's prologue, which
//   applied r_j = r_{j-1} - alpha q_{j-1}), stopping test on it;
//   alpha_j = rho_j / (p_j.q_j);
//   beta_j = |r_{j+1}|^2 / rho_j with |r_{j+1}|^2 = rho_j - 2 alpha (r.q) +
//   alpha^2 (q.q), the exact expansion of |r_j - alpha_j q_j|^2.  The true
//   r_{j+1}.r_{j+1} replaces it in the next iteration (stopping test, alpha).
// The x / r updates of iteration j stay pending until the next iteration's
// first two mode products (or gg_cg_iterate's closing update).
//
// x_defer (p_new != nullptr): x is not updated every iteration.  With xpend
// deferred steps at the start of iteration j (the side job folded both into
// x if xpend was 2):  xpend 2 or 0 -> 1 pending, (p_j, alpha_j);  xpend 1 ->
// 2 pending, (p_j, alpha_j) and (p_{j-1}, alpha_{j-1}).  p_new = p_j (this
// iteration's direction buffer); the host keeps three direction buffers so
// p_{j-1} survives the next prologue.
//
// x_defer mode 2 (xmode 2, balanced): the pair of steps (2i, 2i + 1) becomes
// active at the end of iteration 2i + 1 and the side jobs of the next two
// iterations apply it half of x each (sc->xh: 0, 1, then 2 = done), so every
// side launch carries one pass instead of two in every other iteration; four
// direction buffers keep the pair alive.
__global__ __launch_bounds__(1024) void cg_fused_scalars_kernel(
    const double* __restrict__ rr_part, int64_t nrr, int64_t rr_stride,
    const double* __restrict__ mv_part, int64_t nmv, int64_t pstride, CgScalars* sc,
    const double* p_new, int xmode, int rq_ident, int rder) {
  if (sc->done) return;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  for (int64_t i = threadIdx.x; i < nmv; i += blockDim.x) {
    a0 += mv_part[i];
    if (!rq_ident) a1 += mv_part[pstride + i];
    a2 += mv_part[2 * pstride + i];
  }
  // conjugacy r.q: p_j = r_j + beta_j p_{j-1}, so r_j.q_j = p_j.q_j -
  // beta_j p_{j-1}.A p_j = p_j.q_j - beta_j p_j.q_{j-1} (A symmetric); the
  // prologue summed p_j.q_{j-1} (zero on the first step, where beta = 0)
  if (rq_ident)
    for (int64_t i = threadIdx.x; i < nrr; i += blockDim.x) a1 += rr_part[rr_stride + i];
  const bool pend = sc->pending != 0;
  if (pend)
    for (int64_t i = threadIdx.x; i < nrr; i += blockDim.x) a3 += rr_part[i];
  const double pq = block_sum(a0);
  __syncthreads();
  const double rq_raw = block_sum(a1);   // r.q, or p_j.q_{j-1} (rq_ident)
  __syncthreads();
  const double qq = block_sum(a2);
  __syncthreads();
  const double rr = block_sum(a3);
  if (threadIdx.x == 0) {
    // mode 3: this iteration's pair launch applied the armed side job (it ran:
    // done was 0 then, as it is now)
    if (xmode == 3 && sc->warm) {
      sc->wa[sc->sreg] = sc->wn;
      sc->warm = 0;
    }
    // derived r: this iteration's prologue formed p_j with sc->beta; when an
    // update was pending it computed r_j without storing it
    if (rder) {
      sc->beta_p = sc->beta;
      if (pend) sc->rstored = 0;
      sc->rp_prev = sc->rp_cur;
      sc->rp_cur = p_new;
    }
    if (pend) {
      sc->rho_prev = sc->rho;
      sc->rho = rr;
      sc->iters += 1;
      if (!(sqrt(rr) >= sc->tol)) {  // converged (or NaN): x_j, r_j are final
        sc->done = 1;
        sc->pending = 0;
        // x_defer: xpend 2 was folded into x by this iteration's side job;
        // xpend 1 (alpha_{j-1} p_{j-1}) stays for the closing flush.  Mode 2:
        // this iteration's side job took half xh; the flush does the rest
        if (p_new != nullptr && xmode != 2 && sc->xpend == 2) sc->xpend = 0;
        if (p_new != nullptr && xmode == 2 && sc->xh < 2) sc->xh += 1;
        return;
      }
    }
    const double rho = sc->rho;
    const double alpha = rho / pq;
    const double rq = rq_ident ? pq - sc->beta * rq_raw : rq_raw;   // beta_j: not yet replaced
    double rt = rho - 2.0 * alpha * rq + alpha * alpha * qq;
    sc->pq = pq;
    sc->rq = rq;
    sc->qq = qq;
    sc->alpha = alpha;
    // |r_{j+1}|^2 from three terms of size ~rho: when it is below 1e-6 rho
    // the expansion has lost too many digits for beta -- apply the update
    // and take the true r.r instead (repair kernels before the next matvec)
    sc->repair = rt < (sc->cancel_tol > 0.0 ? sc->cancel_tol : 1e-6) * rho ? 1 : 0;
    sc->cancels += sc->repair;
    sc->beta = sc->repair ? 0.0 : rt / rho;
    sc->first = 0;
    sc->pending = 1;
    if (p_new != nullptr && xmode == 3) {
      // step wn = (alpha_j, p_j) into the ring, then arm the next region with
      // every step it has not seen (wk at most: it was armed wk arms ago)
      const int K = sc->wk, slots = K + 1;
      const int j = sc->wn;
      sc->wc[j % slots] = alpha;
      sc->wp[j % slots] = p_new;
      sc->wn = j + 1;
      const int reg = sc->wnext;
      sc->wnext = reg + 1 == K ? 0 : reg + 1;
      const int a = sc->wa[reg];
      const int cnt = sc->wn - a;
      sc->sreg = reg;
      sc->scnt = cnt;
      for (int t = 0; t < kXWinMax; ++t) {
        const int i = a + (t < cnt ? t : 0);
        sc->scoef[t] = t < cnt ? sc->wc[i % slots] : 0.0;
        sc->sdir[t] = sc->wp[i % slots];
      }
      sc->warm = cnt > 0 ? 1 : 0;
    } else if (p_new != nullptr && xmode == 2) {
      if (sc->xh < 2) sc->xh += 1;   // this iteration's side job took a half
      if (!sc->xs) {
        sc->xs = 1;
        sc->xsc = alpha;
        sc->xsp = p_new;
      } else {   // the pair is complete (the previous one finished just now)
        sc->xc[0] = sc->xsc;
        sc->xp[0] = sc->xsp;
        sc->xc[1] = alpha;
        sc->xp[1] = p_new;
        sc->xh = 0;
        sc->xs = 0;
      }
    } else if (p_new != nullptr) {
      if (sc->xpend == 1) {
        sc->xc[1] = sc->xc[0];
        sc->xp[1] = sc->xp[0];
        sc->xpend = 2;
      } else {
        sc->xpend = 1;
      }
      sc->xc[0] = alpha;
      sc->xp[0] = p_new;
    }
  }
}

// a sharded CG rank's local sums of one fused iteration, red = [r.r (of the
// prologue's r update), p.q_old, p.q, r.q, q.q] (gg_cg_iterate_partial); the
// caller all-reduces red and cg_fused_scalars_kernel takes it as one-element
// partial arrays
__global__ __launch_bounds__(1024) void cg_local_red_kernel(
    const double* __restrict__ rr_part, int64_t nrr, int64_t rr_stride,
    const double* __restrict__ mv_part, int64_t nmv, int64_t pstride, int rq_ident,
    double* __restrict__ red) {
  double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < nrr; i += blockDim.x) {
    a[0] += rr_part[i];
    if (rq_ident) a[1] += rr_part[rr_stride + i];
  }
  for (int64_t i = threadIdx.x; i < nmv; i += blockDim.x) {
    a[2] += mv_part[i];
    if (!rq_ident) a[3] += mv_part[pstride + i];
    a[4] += mv_part[2 * pstride + i];
  }
  double t[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    t[k] = block_sum(a[k]);
    __syncthreads();
  }
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 5; ++k) red[k] = t[k];
}

// the closing step of a sharded rank: rho from the all-reduced r.r
__global__ void cg_close_rho_kernel(CgScalars* sc, const double* rr) {
  if (sc->done || !sc->pending) return;
  const double s = *rr;
  sc->rho_prev = sc->rho;
  sc->rho = s;
  sc->beta = s / sc->rho_prev;
  sc->iters += 1;
  sc->first = 0;
  sc->pending = 0;
  sc->repair = 0;
  if (!(sqrt(s) >= sc->tol)) sc->done = 1;
}

__global__ void cg_init_kernel(const double* __restrict__ partials, int64_t count,
                               CgScalars* sc, double rtol, double atol) {
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += blockDim.x) acc += partials[i];
  const double s = block_sum(acc);
  if (threadIdx.x == 0) {
    sc->rho = s;
    sc->rho_prev = 0.0;
    sc->bnorm = sqrt(s);
    sc->tol = fmax(atol, rtol * sc->bnorm);
    sc->iters = 0;
    sc->first = 1;
    sc->pending = 0;
    sc->alpha = sc->beta = sc->pq = sc->rq = sc->qq = 0.0;
    sc->repair = 0;
    sc->cancels = 0;
    sc->xpend = 0;
    sc->xh = 2;
    sc->xs = 0;
    sc->wn = 0;
    sc->wnext = 0;
    sc->warm = 0;
    for (int r = 0; r < kXWinMax; ++r) sc->wa[r] = 0;
    sc->beta_p = 0.0;
    sc->rstored = 1;   // r = b (or P b) is in its buffer
    sc->rp_cur = sc->rp_prev = nullptr;
    sc->done = (s == 0.0 || !(sqrt(s) >= sc->tol)) ? 1 : 0;
  }
}

// ----------------------------------------------------------- Lanczos kernels
// ---- fused Lanczos (gg_lanczos_probe).  The Lanczos vectors are kept
// unnormalised: V holds u with v = sV u, P holds u_prev with v_prev = sP u_prev
// (lzs[0], lzs[1]).  The matvec Y = K u + shift u has alpha's dot u.Y in its
// last epilogue (v.Av = sV^2 u.Y), and ONE streaming pass forms
// w = Av - alpha v - beta v_prev = cy Y + cu u + cp u_prev with |w|^2, in
// place of Y: 13 passes over N per step instead of 18 (no normalisation pass;
// the next step's v is w with sV = 1 / beta).  With an even number of
// factors that pass is the next matvec's prologue instead (CGP 3 in
// gg_kron.hip: w is the MFMA operand, written over u_prev).  alpha = v.Av: the oracle's
// v.(Av - beta v_prev) differs by beta v.v_prev, rounding-level while the
// three-term recurrence keeps local orthogonality.
// lzs: [0] sV, [1] sP, [2] cy, [3] cu, [4] cp
__global__ void lz_coef_kernel(double* __restrict__ lzs, const double* __restrict__ dot,
                               double* __restrict__ alpha_out,
                               const double* __restrict__ beta_prev) {
  const double sV = lzs[0], sP = lzs[1];
  const double a = sV * sV * *dot;
  *alpha_out = a;
  lzs[2] = sV;
  lzs[3] = -a * sV;
  lzs[4] = -(*beta_prev) * sP;
}

// w = cy w + cu v + cp p (in place), partial w.w; 16-byte lanes when all
// three vectors are 16-byte aligned (wide), else 8-byte
__global__ __launch_bounds__(kVecThreads) void lz_update_kernel(
    double* __restrict__ w, const double* __restrict__ v, const double* __restrict__ pv,
    int64_t n, const double* __restrict__ lzs, double* __restrict__ partials, int wide) {
  const double cy = lzs[2], cu = lzs[3], cp = lzs[4];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (!wide) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const double r = fma(cp, pv[i], fma(cu, v[i], cy * w[i]));
      w[i] = r;
      acc = fma(r, r, acc);
    }
    const double s = block_sum(acc);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
    return;
  }
  const int64_t n2 = n / 2;
  double2* __restrict__ w2 = reinterpret_cast<double2*>(w);
  const double2* __restrict__ v2 = reinterpret_cast<const double2*>(v);
  const double2* __restrict__ p2 = reinterpret_cast<const double2*>(pv);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
    const double2 a = w2[i], b = v2[i], c = p2[i];
    double2 r;
    r.x = fma(cp, c.x, fma(cu, b.x, cy * a.x));
    r.y = fma(cp, c.y, fma(cu, b.y, cy * a.y));
    w2[i] = r;
    acc = fma(r.x, r.x, acc);
    acc = fma(r.y, r.y, acc);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    const double r = fma(cp, pv[i], fma(cu, v[i], cy * w[i]));
    w[i] = r;
    acc = fma(r, r, acc);
  }
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// beta = sqrt(|w|^2) ; next step: v_prev = v (sP = sV), v = w (sV = 1 / beta)
__global__ void lz_beta_kernel(double* __restrict__ lzs, double* __restrict__ beta) {
  const double b = sqrt(*beta);
  *beta = b;
  lzs[1] = lzs[0];
  lzs[0] = b > 0.0 ? 1.0 / b : 0.0;
}

// The block-basis Lanczos step's scalars (lanczos_block), after step j's
// three launches: rr = |w_{j-1}|^2 (the prologue's partials; |u_0|^2 = 1 at
// j = 0), dot = u_j.Y_j (the pair launch's p.q partials).  beta_{j-1} =
// sqrt(rr), v_j = u_j / beta_{j-1} (sV), v_{j-1} = sP u_{j-1} (the previous
// sV), alpha_j = sV^2 dot, and the next prologue's w_j = A v_j - alpha_j v_j -
// beta_{j-1} v_{j-1} = cy Y_j + cu u_j + cp u_{j-1}.
// lzs: [0] sV, [1] sP, [2] cy, [3] cu, [4] cp
__global__ __launch_bounds__(1024) void lzb_step_kernel(const double* __restrict__ rr_part,
                                                        int64_t nrr,
                                                        const double* __restrict__ dot_part,
                                                        int64_t ndot, double* __restrict__ lzs,
                                                        double* __restrict__ alpha_out,
                                                        double* __restrict__ beta_out,
                                                        int first) {
  double a0 = 0.0, a1 = 0.0;
  for (int64_t i = threadIdx.x; i < nrr; i += blockDim.x) a0 += rr_part[i];
  for (int64_t i = threadIdx.x; i < ndot; i += blockDim.x) a1 += dot_part[i];
  const double rr = block_sum(a0);
  __syncthreads();
  const double dot = block_sum(a1);
  if (threadIdx.x == 0) {
    const double beta = sqrt(rr);
    if (!first) *beta_out = beta;
    const double sP = lzs[0];
    const double sV = beta > 0.0 ? 1.0 / beta : 0.0;
    const double alpha = sV * sV * dot;
    *alpha_out = alpha;
    lzs[0] = sV;
    lzs[1] = sP;
    lzs[2] = sV;
    lzs[3] = -alpha * sV;
    lzs[4] = first ? 0.0 : -beta * sP;
  }
}

// A[i][j] *= w[i] (mode 0) or /= w[i] (mode 1); square (mode 2): A = A * A
__global__ __launch_bounds__(kVecThreads) void scale_rows_kernel(double* __restrict__ A,
                                                                 int64_t rows, int64_t cols,
                                                                 const double* __restrict__ w,
                                                                 int mode) {
  const int64_t total = rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const double a = A[e];
    if (mode == 2) {
      A[e] = a * a;
    } else {
      const double s = w[e / cols];
      A[e] = mode == 0 ? a * s : a / s;
    }
  }
}

__global__ __launch_bounds__(kVecThreads) void diag_divide_kernel(const double* __restrict__ t,
                                                                  double shift,
                                                                  const double* __restrict__ x,
                                                                  double* __restrict__ y,
                                                                  int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = x[i] / (t[i] + shift);
}

// Rademacher probe, bit-identical to oracle/cg.py probe_signs (splitmix64)
__device__ __forceinline__ uint64_t probe_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kVecThreads) void probe_kernel(uint64_t base, double scale,
                                                            double* __restrict__ z, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = probe_mix(base + (uint64_t)i * 0x9E3779B97F4A7C15ull);
    z[i] = (h >> 63) == 0 ? scale : -scale;
  }
}

static uint64_t probe_base(uint64_t seed, int probe) {
  return (((seed & 0xffffffffull) << 32) ^ (((uint64_t)probe & 0xffffull) << 16) ^
          0x9E3779B97F4A7C15ull);
}

// ----------------------------------------------- Kronecker eigenvalue diagonal
struct KronDiag {
  int d;
  int64_t m[16];
  int64_t off[16];
};

__device__ __forceinline__ double kron_eig_at(const KronDiag& kd, const double* lam, int64_t i) {
  double t = 1.0;
  for (int k = kd.d - 1; k >= 0; --k) {
    const int64_t ik = i % kd.m[k];
    i /= kd.m[k];
    t *= lam[kd.off[k] + ik];
  }
  return t;
}

__global__ __launch_bounds__(kVecThreads) void diag_scale_kernel(KronDiag kd,
                                                                 const double* __restrict__ lam,
                                                                 double shift, int mode,
                                                                 const double* __restrict__ x,
                                                                 double* __restrict__ y,
                                                                 int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double t = kron_eig_at(kd, lam, i);
    double v;
    if (mode == GG_DIAG_DIVIDE)
      v = x[i] / (t + shift);
    else if (mode == GG_DIAG_POSTVAR)
      v = t * shift / (t + shift);
    else
      v = x[i] * (t + shift);
    y[i] = v;
  }
}

__global__ __launch_bounds__(kVecThreads) void logdet_kernel(KronDiag kd,
                                                             const double* __restrict__ lam,
                                                             double shift, int64_t n,
                                                             double* __restrict__ partials) {
  // the last factor varies fastest: decode the head once per run of m_last
  const int64_t ml = kd.m[kd.d - 1];
  const int64_t nhead = n / ml;
  const double* lastl = lam + kd.off[kd.d - 1];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t h = i / ml;
    const int64_t l = i - h * ml;
    double t = lastl[l];
    int64_t hh = h;
    for (int k = kd.d - 2; k >= 0; --k) {
      const int64_t ik = hh % kd.m[k];
      hh /= kd.m[k];
      t *= lam[kd.off[k] + ik];
    }
    acc += log(t + shift);
  }
  (void)nhead;
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

static KronDiag make_diag(int d, const int64_t* m, int64_t* n_out) {
  GG_REQUIRE(d >= 1 && d <= 16, GG_ERR_VALUE, "1 <= d <= 16 factors supported");
  KronDiag kd{};
  kd.d = d;
  int64_t n = 1, off = 0;
  for (int k = 0; k < d; ++k) {
    GG_REQUIRE(m[k] >= 1, GG_ERR_VALUE, "empty factor");
    kd.m[k] = m[k];
    kd.off[k] = off;
    off += m[k];
    n *= m[k];
  }
  *n_out = n;
  return kd;
}

}  // namespace gg

// ------------------------------------------------------------------- CG state
namespace gg {
// RAII set of HIP events (timed Lanczos, calibration)
struct EventSet {
  std::vector<hipEvent_t> ev;
  explicit EventSet(size_t n) {
    ev.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      hipEvent_t e;
      GG_HIP(hipEventCreate(&e));
      ev.push_back(e);
    }
  }
  ~EventSet() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  EventSet(const EventSet&) = delete;
  EventSet& operator=(const EventSet&) = delete;
};

// a handle's scalar block: zeroed, with the cancellation threshold of the
// knob snapshot (GG_CG_CANCEL_TOL, tests: forces the repair / restart paths)
static void scalars_clear(CgScalars* sc) {
  GG_HIP(hipMemset(sc, 0, sizeof(CgScalars)));
  const char* e = knob("GG_CG_CANCEL_TOL");
  if (e) {
    const double t = atof(e);
    GG_HIP(hipMemcpy(&sc->cancel_tol, &t, sizeof(double), hipMemcpyHostToDevice));
  }
}
}  // namespace gg

struct gg_cg {
  const gg_kron* K = nullptr;
  double shift = 0.0;
  int64_t n = 0;
  double *r = nullptr, *p = nullptr, *q = nullptr, *mv_work = nullptr;
  double* p2 = nullptr;        // second direction buffer (fused recurrence)
  double* p3 = nullptr;        // third (x_defer: p_{j-1} outlives the next prologue)
  double* p4 = nullptr;        // fourth (x_defer mode 2: p_{j-2} too)
  double* first_dst = nullptr; // odd d: the first mode product's output (not q)
  bool fused = true;           // recurrence: fused (default) or textbook
  int fusion = 0;              // fused layout (gg_cg_set_fusion): 0, 1 or 2
  int xdefer = 2;              // layouts 0 / 1: x updated in deferred pairs (1: every
                               // other iteration; 2: balanced, half a pair per iteration)
  double* partials = nullptr;  // device, max(kVecBlocks, 3 x matvec partials)
  double* rr_part = nullptr;   // device, prologue r.r (+ p_new.q_old) partials (fused)
  int64_t rr_count = 0;
  int rq = 1;                  // layout 0: r.q from the conjugacy identity (gg_cg_set_rq)
  gg::CgScalars* sc = nullptr; // device
  gg::CgScalars* sc_host = nullptr;  // pinned mirror
  const double* b = nullptr;
  double* x = nullptr;
  int64_t mv_partials = 0;
  // rank of a sharded CG (gg_cg_*_partial / _finish): an iteration's local
  // sums await the caller's all-reduce (the p_new of that iteration)
  bool await_finish = false;
  // live timing of the mode products (gg_cg_profile): d + 1 events per
  // profiled iteration, recorded on the CG stream, read back on demand
  bool profiling = false;
  std::vector<hipEvent_t> events;
  size_t events_used = 0;
  // parity-block basis (gg_kronb.hip): the recurrence runs on P b, P x, ...
  // in the block layout -- xb the iterate, q2 the pair launch's q (swapped
  // with q every iteration); x (the caller's) is written by the unfold of
  // each close.  basis: requested (gg_cg_set_basis); block: in effect for the
  // current solve (fixed at gg_cg_start: fused, layout 0, x_defer 2, rq 1)
  const gg::BlockOp* blk = nullptr;
  int basis = 1;
  bool block = false;
  double* xb = nullptr;
  double* q2 = nullptr;
  // a rank of the block-sharded CG (gg_cg_create_blocks): the handle's
  // vectors are blocks [rblk0, rblk0 + rnblk) of the block layout (rnblk > 0);
  // only the _partial / _finish entry points drive it
  int64_t rblk0 = 0, rnblk = -1;
  // A/B (GG_CG_RESTART=1, latched at create): gg_cg_iterate restarts a
  // cancelled beta (p = r) as a sharded rank does instead of repairing it --
  // the restart penalty measured on one GPU with everything else equal
  bool restart = false;
  // x_defer mode 3 (window; block basis with the LDS pair launch): the window
  // requested at create (GG_CG_XWIN, 0 = the balanced pairs of mode 2), the
  // mode in effect for the current solve (gg_cg_start*), and the ring of
  // xwin + 1 direction buffers (slots 0..3 are p, p2, p3, p4 as created; the
  // rest lie past the scratch region) with the current direction at pcur
  int xwin = 0;
  int xmode = 0;
  double* ring[gg::kXWinMax + 1] = {};
  int pcur = 0;
  double *q_c = nullptr, *q2_c = nullptr;   // q / q2 as created (swapped per iteration)
  // derived r (CgScalars::rstored; with the window in the block basis): the
  // prologue keeps no r -- 5 passes instead of 6.  rder_ok: the knob
  // (GG_CG_RDERIVE, default on) latched at create; rder: in effect this solve
  bool rder_ok = true;
  bool rder = false;
  // the direction before the current one (p_{j-2} for iteration j's prologue)
  double* pprev_buf() const {
    const int ns = nring();
    return ring[(pcur + ns - 1) % ns];
  }
  int launches() const { return block ? gg::block_launches(blk) : gg::kron_d(K); }
  int nring() const { return xmode == 3 ? xwin + 1 : 4; }
  // the length of the recurrence's vectors: the grid's n, or the block
  // layout's (padded pair axes: >= n) for a full handle in the block basis
  // (a block-range handle's n is already its blocks' length)
  int64_t nvec() const { return (block && rnblk < 0) ? gg::block_n(blk) : n; }
  // every solve starts from the buffers as created (a block solve swaps q / q2
  // and rotates the directions)
  void reset_buffers() {
    p = ring[0];
    p2 = ring[1];
    p3 = ring[2];
    p4 = ring[3];
    q = q_c;
    q2 = q2_c;
    pcur = 0;
  }
  // after an iteration's scalars: p_new (p2) becomes the current direction
  void rotate_dirs() {
    if (xmode == 3) {
      const int ns = nring();
      pcur = (pcur + 1) % ns;
      p = ring[pcur];
      p2 = ring[(pcur + 1) % ns];
    } else if (xmode == 2) {
      // (cur, free, p_{j-2}, p_{j-3}) <- (free, p_{j-3}, cur, p_{j-2}): the
      // active pair (at most p_{j-1}, p_{j-2} next iteration) stays alive
      double* cur = p;
      double* o2 = p3;
      p = p2;
      p2 = p4;
      p3 = cur;
      p4 = o2;
    } else if (xmode == 1) {
      // (cur, free, old) <- (free, old, cur): p_j becomes current, p_{j-1}
      // is kept one more iteration for the deferred x update
      double* old_ = p3;
      p3 = p;
      p = p2;
      p2 = old_;
    } else {
      std::swap(p, p2);
    }
  }
};

namespace gg {
// x_defer mode 3's window from the knob snapshot (GG_CG_XWIN; < 2: off)
static int cg_xwin_knob() {
  const char* e = knob("GG_CG_XWIN");
  const int k = e ? atoi(e) : kXWinDefault;
  return k < 2 ? 0 : std::min(k, kXWinMax);
}
// direction buffers beyond the four every handle has
static int64_t cg_extra_dirs(int K) { return K >= 2 ? std::max(0, K + 1 - 4) : 0; }
int64_t xwin_region(int64_t n, int K) { return 2 * ceil_div(n, 2 * (int64_t)K); }
}  // namespace gg

extern "C" {

int gg_dot(const double* x_dev, const double* y_dev, int64_t n, double* out_host,
           gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(x_dev && y_dev && out_host && n >= 0, GG_ERR_VALUE, "bad argument");
    hipStream_t s = gg::as_stream(stream);
    double* buf = nullptr;
    GG_HIP(hipMallocAsync(&buf, (gg::kVecBlocks + 1) * sizeof(double), s));
    const int nb = gg::vec_blocks(n);
    gg::launch_dot_partials(x_dev, y_dev, n, buf, nb, s);
    gg::launch_reduce_to(buf, nb, buf + gg::kVecBlocks, s);
    GG_HIP(hipMemcpyAsync(out_host, buf + gg::kVecBlocks, sizeof(double),
                          hipMemcpyDeviceToHost, s));
    GG_HIP(hipFreeAsync(buf, s));
    GG_HIP(hipStreamSynchronize(s));
  });
}

int gg_axpby(double a, const double* x_dev, double b, double* y_dev, int64_t n,
             gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(x_dev && y_dev && n >= 0, GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    hipLaunchKernelGGL(gg::axpby_kernel, dim3(gg::vec_blocks(2 * n)), dim3(gg::kVecThreads),
                       0, gg::as_stream(stream), a, x_dev, b, y_dev, n);
    GG_LAUNCH_CHECK();
  });
}

int gg_diag_divide(const double* t_dev, double shift, const double* x_dev, double* y_dev,
                   int64_t n, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(t_dev && x_dev && y_dev && n >= 0, GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    hipLaunchKernelGGL(gg::diag_divide_kernel, dim3(gg::vec_blocks(2 * n)),
                       dim3(gg::kVecThreads), 0, gg::as_stream(stream), t_dev, shift, x_dev,
                       y_dev, n);
    GG_LAUNCH_CHECK();
  });
}

int gg_scale_rows(double* A_dev, int64_t rows, int64_t cols, const double* w_dev, int mode,
                  gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(A_dev && rows >= 0 && cols >= 0 && mode >= 0 && mode <= 2, GG_ERR_VALUE,
               "bad argument");
    GG_REQUIRE(mode == 2 || w_dev, GG_ERR_VALUE, "w required");
    if (rows * cols == 0) return;
    hipLaunchKernelGGL(gg::scale_rows_kernel, dim3(gg::vec_blocks(2 * rows * cols)),
                       dim3(gg::kVecThreads), 0, gg::as_stream(stream), A_dev, rows, cols, w_dev,
                       mode);
    GG_LAUNCH_CHECK();
  });
}

int gg_kron_diag_scale(int d, const int64_t* m, const double* lam_dev, double shift, int mode,
                       const double* x_dev, double* y_dev, gg_stream stream) {
  return gg::guard([&] {
    int64_t n = 0;
    gg::KronDiag kd = gg::make_diag(d, m, &n);
    GG_REQUIRE(lam_dev && y_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(mode == GG_DIAG_POSTVAR || x_dev, GG_ERR_VALUE, "x required");
    GG_REQUIRE(mode >= 0 && mode <= 2, GG_ERR_VALUE, "bad mode");
    hipLaunchKernelGGL(gg::diag_scale_kernel, dim3(gg::vec_blocks(2 * n)),
                       dim3(gg::kVecThreads), 0, gg::as_stream(stream), kd, lam_dev, shift,
                       mode, x_dev, y_dev, n);
    GG_LAUNCH_CHECK();
  });
}

int gg_kron_logdet_shifted(int d, const int64_t* m, const double* lam_dev, double shift,
                           double* out_host, gg_stream stream) {
  return gg::guard([&] {
    int64_t n = 0;
    gg::KronDiag kd = gg::make_diag(d, m, &n);
    GG_REQUIRE(lam_dev && out_host, GG_ERR_VALUE, "NULL argument");
    hipStream_t s = gg::as_stream(stream);
    double* buf = nullptr;
    GG_HIP(hipMallocAsync(&buf, (gg::kVecBlocks + 1) * sizeof(double), s));
    const int nb = gg::vec_blocks(2 * n);
    hipLaunchKernelGGL(gg::logdet_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, kd, lam_dev,
                       shift, n, buf);
    GG_LAUNCH_CHECK();
    gg::launch_reduce_to(buf, nb, buf + gg::kVecBlocks, s);
    GG_HIP(hipMemcpyAsync(out_host, buf + gg::kVecBlocks, sizeof(double),
                          hipMemcpyDeviceToHost, s));
    GG_HIP(hipFreeAsync(buf, s));
    GG_HIP(hipStreamSynchronize(s));
  });
}

int gg_probe_fill(uint64_t seed, int probe, double* z_dev, int64_t n, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(z_dev && n >= 0, GG_ERR_VALUE, "bad argument");
    if (n == 0) return;
    hipLaunchKernelGGL(gg::probe_kernel, dim3(gg::vec_blocks(2 * n)), dim3(gg::kVecThreads),
                       0, gg::as_stream(stream), gg::probe_base(seed, probe), 1.0, z_dev, n);
    GG_LAUNCH_CHECK();
  });
}

// The CG vectors start on 256-byte boundaries: the workspace base is rounded
// up and every vector's stride is a multiple of 32 doubles.  A vector off a
// 128-byte line costs the fused prologue (six streams) 13.0 -> 15.4 ms at
// 200^4 -- the "slow level" of rounds 3-4, reproduced by the diagnostic knob
// GG_CG_VEC_PAD (elements, even; added to the stride: pad 2 = every vector
// 16 bytes further off the line than the previous; tools/prologue_levels.py,
// profiles/r04/n_levels.jsonl).  Read from the snapshot gg_cg_work_elems
// takes, which gg_cg_create lays the workspace out by.
static int64_t cg_vec_pad() {
  const char* e = gg::knob("GG_CG_VEC_PAD");
  const int64_t v = e ? atoll(e) : 0;
  return v > 0 ? 2 * (v / 2) : 0;
}
static int64_t cg_vec_stride(int64_t n) { return (n + 31) / 32 * 32 + cg_vec_pad(); }
constexpr int64_t kCgAlignSlack = 32;   // doubles: room to round the base up to 256 B

// gg_cg_create's layout: r, p, q, p2, p3, p4, then the scratch region (the
// matvec scratch, or xb and q2 in the block basis), then the window's extra
// direction buffers; *extra_off = where those start (from the aligned base)
static int64_t cg_layout_elems(const gg_kron* K, int64_t n, int64_t* extra_off = nullptr,
                               int* xwin = nullptr, int64_t* vstride = nullptr) {
  const gg::BlockOp* B = gg::kron_block(K);
  // every vector holds the grid's n or the block layout's (padded) length
  const int64_t vs = cg_vec_stride(B ? std::max(n, gg::block_n(B)) : n);
  if (vstride) *vstride = vs;
  const int64_t scratch = gg::kron_work_elems(K, false) + (gg::kron_d(K) % 2 == 1 ? n : 0);
  const int64_t region = (std::max(scratch, B ? 2 * vs : 0) + 31) / 32 * 32;
  const int w = (B && gg::block_pair_side(B)) ? gg::cg_xwin_knob() : 0;
  if (extra_off) *extra_off = 6 * vs + region;
  if (xwin) *xwin = w;
  return kCgAlignSlack + 6 * vs + region + gg::cg_extra_dirs(w) * vs;
}

// the workspace each thread's last gg_cg_work_elems sized per operator: a
// gg_cg_create whose layout (read from the snapshot current then) needs more
// -- another handle's creation re-took the GG_* snapshot with, say, a wider
// window in between -- is refused instead of overrunning the caller's buffer
static thread_local std::map<const gg_kron*, int64_t> t_cg_sized;

int gg_cg_work_elems(const gg_kron* K, int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(K && elems, GG_ERR_VALUE, "NULL argument");
    gg::knobs_reload();   // the CG handle made next latches this snapshot
    const int64_t n = gg::kron_n(K);
    // r, p, q, p2, p3, p4 (x_defer) + the matvec scratch (+ the first mode
    // product's own output for an odd number of factors, MpFuse::first_dst);
    // the block basis (gg_kronb.hip) takes the scratch region for xb and q2
    // + the window's extra direction buffers (x_defer mode 3, block basis)
    *elems = cg_layout_elems(K, n);
    t_cg_sized[K] = *elems;
  });
}

int gg_cg_work_elems_blocks(const gg_kron* K, int64_t nblk, int64_t* elems) {
  return gg::guard([&] {
    GG_REQUIRE(K && elems, GG_ERR_VALUE, "NULL argument");
    const gg::BlockOp* B = gg::kron_block(K);
    GG_REQUIRE(B != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    GG_REQUIRE(nblk >= 1 && nblk <= ((int64_t)1 << gg::block_d(B)), GG_ERR_VALUE,
               "block count outside 1..2^d");
    gg::knobs_reload();   // the CG handle made next latches this snapshot
    // r, p, q, p2, p3, p4 and q2 (the pair launch's q), then the window's
    // extra direction buffers (x_defer mode 3)
    const int w = gg::block_pair_side(B) ? gg::cg_xwin_knob() : 0;
    *elems = kCgAlignSlack + (7 + gg::cg_extra_dirs(w)) * cg_vec_stride(nblk * gg::block_nb(B));
  });
}

int gg_cg_create_blocks(const gg_kron* K, int64_t blk0, int64_t nblk, double shift,
                        double* work_dev, gg_cg** out) {
  return gg::guard([&] {
    GG_REQUIRE(K && work_dev && out, GG_ERR_VALUE, "NULL argument");
    const gg::BlockOp* B = gg::kron_block(K);
    GG_REQUIRE(B != nullptr, GG_ERR_VALUE, "the operator has no parity-block basis");
    GG_REQUIRE(gg::block_d(B) >= 3, GG_ERR_VALUE, "the block-sharded CG needs d >= 3");
    GG_REQUIRE(blk0 >= 0 && nblk >= 1 && blk0 + nblk <= ((int64_t)1 << gg::block_d(B)),
               GG_ERR_VALUE, "block range outside the 2^d blocks");
    GG_REQUIRE((reinterpret_cast<uintptr_t>(work_dev) & 15) == 0, GG_ERR_VALUE,
               "the CG workspace must be 16-byte aligned");
    const int64_t n = nblk * gg::block_nb(B);
    gg_cg* cg = new gg_cg();
    try {
      cg->K = K;
      cg->shift = shift;
      cg->n = n;
      const int64_t vs = cg_vec_stride(n);
      work_dev = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(work_dev) + 255) &
                                           ~static_cast<uintptr_t>(255));
      cg->r = work_dev;
      cg->p = work_dev + vs;
      cg->q = work_dev + 2 * vs;
      cg->p2 = work_dev + 3 * vs;
      cg->p3 = work_dev + 4 * vs;
      cg->p4 = work_dev + 5 * vs;
      cg->q2 = work_dev + 6 * vs;
      cg->xwin = gg::block_pair_side(B) ? gg::cg_xwin_knob() : 0;
      cg->ring[0] = cg->p;
      cg->ring[1] = cg->p2;
      cg->ring[2] = cg->p3;
      cg->ring[3] = cg->p4;
      for (int i = 0; i < gg::cg_extra_dirs(cg->xwin); ++i) cg->ring[4 + i] = work_dev + (7 + i) * vs;
      cg->q_c = cg->q;
      cg->q2_c = cg->q2;
      cg->blk = B;
      cg->basis = 1;
      cg->rblk0 = blk0;
      cg->rnblk = nblk;
      cg->fused = true;   // layout 0, x_defer 2, rq 1: the block path's only form
      const char* rde = gg::knob("GG_CG_RDERIVE");  // A/B: 0 keeps r in memory
      cg->rder_ok = !(rde && atoi(rde) == 0);
      cg->mv_partials = gg::block_partials_needed(B);
      GG_HIP(hipMalloc(&cg->partials,
                       std::max<int64_t>(gg::kVecBlocks, 3 * cg->mv_partials) * sizeof(double)));
      cg->rr_count = gg::block_prologue_blocks(B);
      GG_HIP(hipMalloc(&cg->rr_part, 2 * cg->rr_count * sizeof(double)));
      GG_HIP(hipMemset(cg->rr_part, 0, 2 * cg->rr_count * sizeof(double)));
      GG_HIP(hipMalloc(&cg->sc, sizeof(gg::CgScalars)));
      GG_HIP(hipHostMalloc(&cg->sc_host, sizeof(gg::CgScalars), hipHostMallocDefault));
      gg::scalars_clear(cg->sc);
    } catch (...) {
      gg_cg_destroy(cg);
      throw;
    }
    *out = cg;
  });
}

int gg_cg_create(const gg_kron* K, double shift, double* work_dev, gg_cg** out) {
  return gg::guard([&] {
    GG_REQUIRE(K && work_dev && out, GG_ERR_VALUE, "NULL argument");
    // the switches (GG_CG_*) come from the snapshot gg_cg_work_elems took, so
    // the vector stride (GG_CG_VEC_PAD) is the one the workspace was sized for
    int64_t nr = 0, nc = 0, we = 0;
    gg_kron_shape(K, 0, &nr, &nc, &we);
    GG_REQUIRE(nr == nc, GG_ERR_VALUE, "CG needs a square operator");
    gg_cg* cg = new gg_cg();
    try {
      cg->K = K;
      cg->shift = shift;
      cg->n = nr;
      int64_t vs = 0;
      const int64_t need = cg_layout_elems(K, nr, nullptr, nullptr, &vs);
      const auto sized = t_cg_sized.find(K);
      GG_REQUIRE(sized == t_cg_sized.end() || need <= sized->second, GG_ERR_VALUE,
                 "the CG workspace was sized (gg_cg_work_elems) under another GG_* snapshot: "
                 "call gg_cg_work_elems again before gg_cg_create");
      if (sized != t_cg_sized.end()) t_cg_sized.erase(sized);   // one check per sizing
      GG_REQUIRE((reinterpret_cast<uintptr_t>(work_dev) & 7) == 0, GG_ERR_VALUE,
                 "the CG workspace must hold doubles (8-byte aligned)");
      work_dev = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(work_dev) + 255) &
                                           ~static_cast<uintptr_t>(255));
      cg->r = work_dev;
      cg->p = work_dev + vs;
      cg->q = work_dev + 2 * vs;
      cg->p2 = work_dev + 3 * vs;
      cg->p3 = work_dev + 4 * vs;
      cg->p4 = work_dev + 5 * vs;
      cg->mv_work = work_dev + 6 * vs;
      if (gg::kron_d(K) % 2 == 1) cg->first_dst = cg->mv_work + gg::kron_work_elems(K, false);
      cg->blk = gg::kron_block(K);
      int64_t extra_off = 0;
      int xwin = 0;
      cg_layout_elems(K, nr, &extra_off, &xwin);
      cg->ring[0] = cg->p;
      cg->ring[1] = cg->p2;
      cg->ring[2] = cg->p3;
      cg->ring[3] = cg->p4;
      cg->q_c = cg->q;
      if (cg->blk != nullptr) {
        cg->xb = work_dev + 6 * vs;
        cg->q2 = work_dev + 7 * vs;
        cg->q2_c = cg->q2;
        const char* be = gg::knob("GG_CG_BASIS");   // read once per handle
        // default: the block basis where its padding costs little
        cg->basis = be ? (atoi(be) != 0 ? 1 : 0) : (gg::block_efficient(cg->blk) ? 1 : 0);
        // the window only where the pair launch carries the side job
        cg->xwin = gg::block_pair_side(cg->blk) ? xwin : 0;
        for (int i = 0; i < gg::cg_extra_dirs(xwin); ++i)
          cg->ring[4 + i] = work_dev + extra_off + i * vs;
      } else {
        cg->basis = 0;
      }
      const char* xd = gg::knob("GG_CG_XDEFER");   // A/B knob: 0, 1 or 2
      if (xd) cg->xdefer = std::min(2, std::max(0, atoi(xd)));
      const char* rqe = gg::knob("GG_CG_RQ");       // A/B knob: 0 (epilogue reads r) or 1
      if (rqe) cg->rq = std::min(2, std::max(0, atoi(rqe)));   // 2: diagnostic
      const char* rse = gg::knob("GG_CG_RESTART");  // A/B: restart instead of repair
      cg->restart = rse && atoi(rse) == 1;
      const char* rde = gg::knob("GG_CG_RDERIVE");  // A/B: 0 keeps r in memory
      cg->rder_ok = !(rde && atoi(rde) == 0);
      cg->mv_partials = gg::kron_partials_needed(K, false);
      if (cg->blk) cg->mv_partials = std::max(cg->mv_partials, gg::block_partials_needed(cg->blk));
      const int64_t np = std::max<int64_t>(gg::kVecBlocks, 3 * cg->mv_partials);
      GG_HIP(hipMalloc(&cg->partials, np * sizeof(double)));
      // the fused recurrence needs d >= 2 and 16-byte aligned vectors (its
      // side job moves double2); otherwise the textbook recurrence runs
      cg->fused = gg::kron_d(K) >= 2 && (nr % 2) == 0 &&
                  (reinterpret_cast<uintptr_t>(work_dev) & 15) == 0;
      if (cg->fused) {
        // capacity for any prologue launch shape; each iteration sums exactly
        // the partials its prologue launch wrote (MpFuse::pro_blocks)
        cg->rr_count = gg::kron_prologue_blocks(K);
        if (cg->blk) cg->rr_count = std::max(cg->rr_count, gg::block_prologue_blocks(cg->blk));
        GG_HIP(hipMalloc(&cg->rr_part, 2 * cg->rr_count * sizeof(double)));
        GG_HIP(hipMemset(cg->rr_part, 0, 2 * cg->rr_count * sizeof(double)));
      }
      GG_HIP(hipMalloc(&cg->sc, sizeof(gg::CgScalars)));
      GG_HIP(hipHostMalloc(&cg->sc_host, sizeof(gg::CgScalars), hipHostMallocDefault));
      gg::scalars_clear(cg->sc);
    } catch (...) {
      gg_cg_destroy(cg);
      throw;
    }
    *out = cg;
  });
}

int gg_cg_destroy(gg_cg* cg) {
  return gg::guard([&] {
    if (!cg) return;
    if (cg->partials) (void)hipFree(cg->partials);
    if (cg->rr_part) (void)hipFree(cg->rr_part);
    if (cg->sc) (void)hipFree(cg->sc);
    if (cg->sc_host) (void)hipHostFree(cg->sc_host);
    for (hipEvent_t e : cg->events) (void)hipEventDestroy(e);
    delete cg;
  });
}

int gg_cg_profile(gg_cg* cg, int enable) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    cg->profiling = enable != 0;
    cg->events_used = 0;
  });
}

int gg_cg_profile_read(gg_cg* cg, int* n_matvecs, double* mode_ms, int mode_ms_len) {
  return gg::guard([&] {
    GG_REQUIRE(cg && n_matvecs, GG_ERR_VALUE, "NULL argument");
    const int d = cg->launches();
    GG_REQUIRE(mode_ms == nullptr || mode_ms_len >= d, GG_ERR_VALUE, "mode_ms too short");
    const size_t per = (size_t)d + 1;
    const int nm = (int)(cg->events_used / per);
    if (mode_ms)
      for (int k = 0; k < d; ++k) mode_ms[k] = 0.0;
    for (int it = 0; it < nm; ++it) {
      hipEvent_t* ev = cg->events.data() + it * per;
      GG_HIP(hipEventSynchronize(ev[d]));
      for (int k = 0; k < d && mode_ms; ++k) {
        float ms = 0.0f;
        GG_HIP(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        mode_ms[k] += ms;
      }
    }
    *n_matvecs = nm;
  });
}

int gg_cg_start(gg_cg* cg, const double* b_dev, double* x_dev, double rtol, double atol,
                gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && b_dev && x_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(rtol >= 0 && atol >= 0, GG_ERR_VALUE,
               "tolerances must be real, non-negative numbers");
    GG_REQUIRE(cg->rnblk < 0, GG_ERR_VALUE,
               "a block-range handle (gg_cg_create_blocks) runs through gg_cg_start_partial");
    hipStream_t s = gg::as_stream(stream);
    cg->b = b_dev;
    cg->x = x_dev;
    const int64_t n = cg->n;
    cg->block = cg->blk != nullptr && cg->basis != 0 && cg->fused && cg->fusion == 0 &&
                cg->xdefer == 2 && cg->rq == 1 && gg::block_d(cg->blk) >= 3;
    cg->xmode = (cg->fused && cg->fusion != 2) ? cg->xdefer : 0;
    if (cg->block && cg->xwin >= 2) cg->xmode = 3;
    cg->rder = cg->xmode == 3 && cg->rder_ok && gg::block_rderive_ok(cg->blk);
    cg->reset_buffers();
    hipLaunchKernelGGL(gg::cg_xwin_init_kernel, dim3(1), dim3(1), 0, s, cg->sc,
                       cg->xmode == 3 ? cg->xwin : 0);
    GG_LAUNCH_CHECK();
    GG_HIP(hipMemsetAsync(x_dev, 0, n * sizeof(double), s));
    if (cg->block) {
      // r = P b (the fold, with its |P b|^2 partials), x_b = 0
      gg::block_fold(cg->blk, false, b_dev, cg->r, cg->partials, s);
      GG_HIP(hipMemsetAsync(cg->xb, 0, cg->nvec() * sizeof(double), s));
      hipLaunchKernelGGL(gg::cg_init_kernel, dim3(1), dim3(1024), 0, s, cg->partials,
                         gg::block_fold_partials(cg->blk), cg->sc, rtol, atol);
      GG_LAUNCH_CHECK();
      return;
    }
    GG_HIP(hipMemcpyAsync(cg->r, b_dev, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    const int nb = gg::vec_blocks(n);
    gg::launch_dot_partials(cg->r, cg->r, n, cg->partials, nb, s);
    hipLaunchKernelGGL(gg::cg_init_kernel, dim3(1), dim3(1024), 0, s, cg->partials,
                       (int64_t)nb, cg->sc, rtol, atol);
    GG_LAUNCH_CHECK();
  });
}

int gg_cg_set_recurrence(gg_cg* cg, int fused) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    GG_REQUIRE(cg->x == nullptr, GG_ERR_VALUE, "set the recurrence before gg_cg_start");
    if (!fused) {
      cg->fused = false;
    } else {
      GG_REQUIRE(cg->rr_part != nullptr, GG_ERR_VALUE,
                 "the fused recurrence needs d >= 2, an even n and 16-byte aligned work");
      cg->fused = true;
    }
  });
}

int gg_cg_set_fusion(gg_cg* cg, int layout) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    GG_REQUIRE(cg->x == nullptr, GG_ERR_VALUE, "set the fusion layout before gg_cg_start");
    GG_REQUIRE(layout >= 0 && layout <= 2, GG_ERR_VALUE, "fusion layout must be 0, 1 or 2");
    GG_REQUIRE(layout == 0 || gg::kron_first_single_launch(cg->K), GG_ERR_VALUE,
               "fusion layouts 1 / 2 need the first factor within one launch (<= 256 rows)");
    cg->fusion = layout;
  });
}

int gg_cg_get_fusion(const gg_cg* cg, int* layout) {
  return gg::guard([&] {
    GG_REQUIRE(cg && layout, GG_ERR_VALUE, "NULL argument");
    *layout = cg->fusion;
  });
}

int gg_cg_set_xdefer(gg_cg* cg, int on) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    GG_REQUIRE(cg->x == nullptr, GG_ERR_VALUE, "set x deferral before gg_cg_start");
    GG_REQUIRE(on >= 0 && on <= 2, GG_ERR_VALUE, "x deferral mode must be 0, 1 or 2");
    cg->xdefer = on;
  });
}

int gg_cg_get_xdefer(const gg_cg* cg, int* on) {
  return gg::guard([&] {
    GG_REQUIRE(cg && on, GG_ERR_VALUE, "NULL argument");
    *on = (cg->fused && cg->fusion != 2) ? cg->xdefer : 0;
  });
}

int gg_cg_get_xwin(const gg_cg* cg, int* K) {
  return gg::guard([&] {
    GG_REQUIRE(cg && K, GG_ERR_VALUE, "NULL argument");
    if (cg->x != nullptr) {
      *K = cg->xmode == 3 ? cg->xwin : 0;
    } else {
      int b = 0;
      gg_cg_get_basis(cg, &b);
      *K = (b && cg->xwin >= 2) ? cg->xwin : 0;
    }
  });
}

int gg_cg_get_rderive(const gg_cg* cg, int* on) {
  return gg::guard([&] {
    GG_REQUIRE(cg && on, GG_ERR_VALUE, "NULL argument");
    if (cg->x != nullptr) {
      *on = cg->rder ? 1 : 0;
    } else {
      int K = 0;
      gg_cg_get_xwin(cg, &K);
      *on = (K >= 2 && cg->rder_ok && gg::block_rderive_ok(cg->blk)) ? 1 : 0;
    }
  });
}

int gg_cg_calibrate(gg_cg* cg, int reps, double* ms_host, int64_t* offsets_host,
                    gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && ms_host && reps >= 1, GG_ERR_VALUE, "bad argument");
    GG_REQUIRE((reinterpret_cast<uintptr_t>(cg->p) & 15) == 0, GG_ERR_VALUE,
               "the CG workspace is not 16-byte aligned");
    hipStream_t s = gg::as_stream(stream);
    int dev = 0, cus = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    gg::EventSet ev(2);
    // the prologue this solve runs: derived r reads p_{j-2} in r's place
    // (a direction slot the first iterations overwrite anyway)
    const bool rd = cg->rder;
    double* second = rd ? cg->ring[(cg->pcur + 2) % cg->nring()] : cg->r;
    // two untimed passes (first touch in this process), then reps timed
    for (int it = 0; it < reps + 2; ++it) {
      if (it == 2) GG_HIP(hipEventRecord(ev.ev[0], s));
      if (rd)
        hipLaunchKernelGGL(gg::cg_stream_probe_kernel<true>,
                           dim3((unsigned)std::max(cus, 1) * 8), dim3(256), 0, s, second, cg->p,
                           cg->p2, cg->q, cg->nvec());
      else
        hipLaunchKernelGGL(gg::cg_stream_probe_kernel<false>,
                           dim3((unsigned)std::max(cus, 1) * 8), dim3(256), 0, s, second, cg->p,
                           cg->p2, cg->q, cg->nvec());
      GG_LAUNCH_CHECK();
    }
    GG_HIP(hipEventRecord(ev.ev[1], s));
    GG_HIP(hipEventSynchronize(ev.ev[1]));
    float ms = 0.f;
    GG_HIP(hipEventElapsedTime(&ms, ev.ev[0], ev.ev[1]));
    *ms_host = ms / reps;
    if (offsets_host) {
      // the buffers' addresses modulo 2 MiB (the allocator's large-page grain)
      const double* b[4] = {second, cg->p, cg->p2, cg->q};
      for (int k = 0; k < 4; ++k)
        offsets_host[k] = (int64_t)(reinterpret_cast<uintptr_t>(b[k]) & ((1u << 21) - 1));
    }
  });
}

int gg_cg_set_rq(gg_cg* cg, int mode) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    GG_REQUIRE(cg->x == nullptr, GG_ERR_VALUE, "set the r.q source before gg_cg_start");
    GG_REQUIRE(mode == 0 || mode == 1, GG_ERR_VALUE, "r.q mode must be 0 or 1");
    cg->rq = mode;
  });
}

int gg_cg_get_rq(const gg_cg* cg, int* mode) {
  return gg::guard([&] {
    GG_REQUIRE(cg && mode, GG_ERR_VALUE, "NULL argument");
    *mode = (cg->fused && cg->fusion == 0 && cg->rq) ? 1 : 0;
  });
}

int gg_cg_set_basis(gg_cg* cg, int block) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    GG_REQUIRE(cg->x == nullptr, GG_ERR_VALUE, "set the basis before gg_cg_start");
    GG_REQUIRE(block == 0 || cg->blk != nullptr, GG_ERR_VALUE,
               "the operator has no parity-block basis");
    cg->basis = block != 0 ? 1 : 0;
  });
}

int gg_cg_get_basis(const gg_cg* cg, int* block) {
  return gg::guard([&] {
    GG_REQUIRE(cg && block, GG_ERR_VALUE, "NULL argument");
    // in effect once started; before, what gg_cg_start will choose
    *block = cg->x != nullptr ? (cg->block ? 1 : 0)
                              : (cg->blk != nullptr && cg->basis != 0 && cg->fused &&
                                 cg->fusion == 0 && cg->xdefer == 2 && cg->rq == 1 &&
                                 gg::block_d(cg->blk) >= 3)
                                    ? 1
                                    : 0;
  });
}

int gg_cg_launches(const gg_cg* cg, int* launches) {
  return gg::guard([&] {
    GG_REQUIRE(cg && launches, GG_ERR_VALUE, "NULL argument");
    int b = 0;
    gg_cg_get_basis(cg, &b);
    *launches = b ? gg::block_launches(cg->blk) : gg::kron_d(cg->K);
  });
}

int gg_cg_get_recurrence(const gg_cg* cg, int* fused) {
  return gg::guard([&] {
    GG_REQUIRE(cg && fused, GG_ERR_VALUE, "NULL argument");
    *fused = cg->fused ? 1 : 0;
  });
}

// Textbook recurrence, one iteration:
//   q = (K + s I) p with p = r + beta p fused into the first mode product
//   and p.q into the last; alpha; x += alpha p, r -= alpha q, r.r; beta.
// Fused recurrence, one iteration j (every vector pass rides on a mode
// product; the matrix cores bound the kernels and HBM has room):
//   mode product 1: r_j = r_{j-1} - alpha q_{j-1} (in place, r.r partials),
//                   p_j = r_j + beta p_{j-1} (into the other p buffer);
//   mode product 2: side job x_j = x_{j-1} + alpha p_{j-1};
//   mode product d: q_j = K p_j + s p_j, partials p.q, r.q, q.q;
//   scalars: rho_j, stopping test, alpha_j, beta_j (cg_fused_scalars_kernel).
// Leaving gg_cg_iterate applies the pending x / r update with the textbook
// kernels, so the state it leaves (x, r, iteration count) is the textbook's.
int gg_cg_iterate(gg_cg* cg, int max_iters, int check_every, gg_stream stream) {
  const int st = gg_cg_iterate_open(cg, max_iters, check_every, stream);
  return st != GG_OK ? st : gg_cg_close(cg, stream);
}

int gg_cg_iterate_open(gg_cg* cg, int max_iters, int check_every, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cg->x, GG_ERR_VALUE, "CG not started");
    GG_REQUIRE(cg->rnblk < 0, GG_ERR_VALUE,
               "a block-range handle (gg_cg_create_blocks) runs through gg_cg_iterate_partial");
    hipStream_t s = gg::as_stream(stream);
    const int64_t n = cg->nvec();
    const int nb = gg::vec_blocks(n);
    if (check_every <= 0) check_every = max_iters;
    for (int it = 0; it < max_iters; ++it) {
      int64_t nparts = 0;
      hipEvent_t* ev = nullptr;
      if (cg->profiling) {
        const size_t need = cg->events_used + (size_t)cg->launches() + 1;
        while (cg->events.size() < need) {
          hipEvent_t e;
          GG_HIP(hipEventCreate(&e));
          cg->events.push_back(e);
        }
        ev = cg->events.data() + cg->events_used;
        cg->events_used = need;
      }
      const int xmode = cg->xmode;   // fixed at gg_cg_start
      const bool xdefer = xmode != 0;
      if (cg->fused) {
        // repair (no-op unless the last beta cancelled): x += alpha p,
        // r -= alpha q, rho = r.r, textbook beta; the prologue then sees no
        // pending update (x_defer: r only, x keeps its deferred steps)
        if (!cg->restart) {
          if (cg->rder)   // r derived from the directions (not stored)
            hipLaunchKernelGGL(gg::cg_r_materialize_kernel, dim3(nb), dim3(gg::kVecThreads), 0,
                               s, cg->r, cg->q, n, cg->sc, cg->partials, 2);
          else
            hipLaunchKernelGGL(gg::cg_xr_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                               xdefer ? nullptr : cg->x, cg->r, cg->p, cg->q, n, cg->sc,
                               cg->partials, 2);
          GG_LAUNCH_CHECK();
          hipLaunchKernelGGL(gg::cg_rho_kernel, dim3(1), dim3(1024), 0, s, cg->partials,
                             (int64_t)nb, cg->sc, 2);
          GG_LAUNCH_CHECK();
        }
        gg::MpFuse fz;
        fz.r = cg->r;
        fz.q_old = cg->q;
        fz.p_out = cg->fusion == 0 ? cg->p2 : nullptr;
        fz.ep_out = cg->fusion == 0 ? nullptr : cg->p2;
        fz.ex = cg->fusion == 2 ? cg->x : nullptr;
        fz.sc = cg->sc;
        fz.rr_part = cg->rr_part;
        fz.rr_cap = cg->rr_count;
        int64_t pro_blocks = 0;   // the prologue launch's workgroups (kron_apply)
        fz.pro_blocks = &pro_blocks;
        fz.sx = cg->fusion == 2 ? nullptr : cg->x;
        fz.sp = cg->p;
        fz.sn = n;
        fz.xdefer = xmode;
        fz.xwin = cg->xwin;
        fz.rderive = cg->rder;
        fz.pprev = cg->rder ? cg->pprev_buf() : nullptr;
        fz.first_dst = cg->first_dst;
        // r.q: conjugacy identity (layout 0: the prologue adds p_new.q_old
        // partials, the epilogue skips its pass over r) or read in the epilogue
        const bool rq_ident = cg->rq != 0 && cg->fusion == 0;
        fz.er = (rq_ident && cg->rq != 2) ? nullptr : cg->r;
        fz.pqo_stride = rq_ident ? cg->rr_count : 0;
        fz.pstride = cg->mv_partials;
        if (cg->block) {
          // the block basis: d - 1 launches, q2 <- (K + s I) p_new
          fz.sx = cg->xb;
          fz.blk_q_out = cg->q2;
          gg::block_apply(cg->blk, cg->p, cg->q, cg->shift, nullptr, cg->partials,
                          &cg->sc->done, s, &nparts, &fz, 2, ev);
        } else {
          gg::kron_apply(cg->K, false, cg->p, cg->q, cg->shift, cg->mv_work, cg->partials,
                         &cg->sc->done, s, &nparts, &fz, 2, ev);
        }
        GG_REQUIRE(pro_blocks > 0 && pro_blocks <= cg->rr_count, GG_ERR_RUNTIME,
                   "fused CG: no prologue launch recorded");
        hipLaunchKernelGGL(gg::cg_fused_scalars_kernel, dim3(1), dim3(1024), 0, s, cg->rr_part,
                           pro_blocks, cg->rr_count, cg->partials, nparts, cg->mv_partials,
                           cg->sc,
                           xdefer ? (const double*)cg->p2 : nullptr, xmode, rq_ident ? 1 : 0,
                           cg->rder ? 1 : 0);
        GG_LAUNCH_CHECK();
        if (cg->block) std::swap(cg->q, cg->q2);
        cg->rotate_dirs();
      } else {
        gg::MpFuse fz;
        fz.r = cg->r;
        fz.sc = cg->sc;
        gg::kron_apply(cg->K, false, cg->p, cg->q, cg->shift, cg->mv_work, cg->partials,
                       &cg->sc->done, s, &nparts, &fz, 1, ev);
        hipLaunchKernelGGL(gg::cg_alpha_kernel, dim3(1), dim3(1024), 0, s, cg->partials, nparts,
                           cg->sc);
        GG_LAUNCH_CHECK();
        hipLaunchKernelGGL(gg::cg_xr_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                           cg->x, cg->r, cg->p, cg->q, n, cg->sc, cg->partials, 0);
        GG_LAUNCH_CHECK();
        hipLaunchKernelGGL(gg::cg_rho_kernel, dim3(1), dim3(1024), 0, s, cg->partials,
                           (int64_t)nb, cg->sc, 0);
        GG_LAUNCH_CHECK();
      }
      if ((it + 1) % check_every == 0 && it + 1 < max_iters) {
        GG_HIP(hipMemcpyAsync(cg->sc_host, cg->sc, sizeof(gg::CgScalars),
                              hipMemcpyDeviceToHost, s));
        GG_HIP(hipStreamSynchronize(s));
        if (cg->sc_host->done) break;
      }
    }
  });
}

// leaving the fused recurrence: the deferred x steps and the pending r update
// (no-op for the textbook recurrence or when nothing is pending)
int gg_cg_close(gg_cg* cg, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cg->x, GG_ERR_VALUE, "CG not started");
    GG_REQUIRE(cg->rnblk < 0, GG_ERR_VALUE,
               "a block-range handle (gg_cg_create_blocks) closes through gg_cg_close_partial");
    hipStream_t s = gg::as_stream(stream);
    const int64_t n = cg->nvec();
    const int nb = gg::vec_blocks(n);
    if (cg->fused) {
      const bool xdefer = cg->xmode != 0;
      // closing update (no-op unless pending): x += alpha p, r -= alpha q,
      // rho = r.r, beta, iteration count -- the textbook state.  x_defer: the
      // deferred steps first (also after convergence), then r only
      if (cg->xmode == 3) {
        hipLaunchKernelGGL(gg::cg_x_flush3_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                           cg->block ? cg->xb : cg->x, n, gg::xwin_region(n, cg->xwin), cg->sc);
        GG_LAUNCH_CHECK();
        hipLaunchKernelGGL(gg::cg_x_flushed3_kernel, dim3(1), dim3(1), 0, s, cg->sc);
        GG_LAUNCH_CHECK();
      } else if (cg->xmode == 2) {
        hipLaunchKernelGGL(gg::cg_x_flush2_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                           cg->block ? cg->xb : cg->x, n,
                           cg->block ? gg::block_side_half(n) : gg::kron_side_half(cg->K, n),
                           cg->sc);
        GG_LAUNCH_CHECK();
        hipLaunchKernelGGL(gg::cg_x_flushed_kernel, dim3(1), dim3(1), 0, s, cg->sc);
        GG_LAUNCH_CHECK();
      } else if (xdefer) {
        hipLaunchKernelGGL(gg::cg_x_flush_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, cg->x,
                           n, cg->sc);
        GG_LAUNCH_CHECK();
        hipLaunchKernelGGL(gg::cg_x_flushed_kernel, dim3(1), dim3(1), 0, s, cg->sc);
        GG_LAUNCH_CHECK();
      }
      if (cg->rder)   // r from the directions (- alpha q when pending) into its buffer
        hipLaunchKernelGGL(gg::cg_r_materialize_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                           cg->r, cg->q, n, cg->sc, cg->partials, 1);
      else
        hipLaunchKernelGGL(gg::cg_xr_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                           xdefer ? nullptr : cg->x, cg->r, cg->p, cg->q, n, cg->sc,
                           cg->partials, 1);
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::cg_rho_kernel, dim3(1), dim3(1024), 0, s, cg->partials,
                         (int64_t)nb, cg->sc, 1);
      GG_LAUNCH_CHECK();
      if (cg->rder) {
        hipLaunchKernelGGL(gg::cg_r_stored_kernel, dim3(1), dim3(1), 0, s, cg->sc);
        GG_LAUNCH_CHECK();
      }
    }
    // the block basis: the caller's x = P^T x_b
    if (cg->block) gg::block_fold(cg->blk, true, cg->xb, cg->x, nullptr, s);
  });
}

// ---- a rank of a sharded CG (include/gp_grief_amd.h, gg_cg_*_partial):
// the fused recurrence on this rank's block of a block-diagonal operator,
// every dot product reduced by the caller between _partial and _finish
int gg_cg_start_partial(gg_cg* cg, const double* b_dev, double* x_dev, double* rr_dev,
                        gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && b_dev && x_dev && rr_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(cg->fused, GG_ERR_VALUE, "the sharded rank runs the fused recurrence");
    hipStream_t s = gg::as_stream(stream);
    cg->b = b_dev;
    cg->x = x_dev;
    // the sharded rank: the handle's own operator layout, or its blocks of
    // the block layout (gg_cg_create_blocks; b and x in that layout)
    cg->block = cg->rnblk > 0;
    cg->await_finish = false;
    cg->xmode = cg->xdefer;
    if (cg->block && cg->xwin >= 2) cg->xmode = 3;
    cg->rder = cg->xmode == 3 && cg->rder_ok && gg::block_rderive_ok(cg->blk);
    cg->reset_buffers();
    hipLaunchKernelGGL(gg::cg_xwin_init_kernel, dim3(1), dim3(1), 0, s, cg->sc,
                       cg->xmode == 3 ? cg->xwin : 0);
    GG_LAUNCH_CHECK();
    const int64_t n = cg->n;
    GG_HIP(hipMemcpyAsync(cg->r, b_dev, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    GG_HIP(hipMemsetAsync(x_dev, 0, n * sizeof(double), s));
    const int nb = gg::vec_blocks(n);
    gg::launch_dot_partials(cg->r, cg->r, n, cg->partials, nb, s);
    gg::launch_reduce_to(cg->partials, nb, rr_dev, s);
  });
}

int gg_cg_start_finish(gg_cg* cg, const double* rr_dev, double rtol, double atol,
                       gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cg->x && rr_dev, GG_ERR_VALUE, "CG not started (gg_cg_start_partial)");
    GG_REQUIRE(rtol >= 0 && atol >= 0, GG_ERR_VALUE,
               "tolerances must be real, non-negative numbers");
    hipLaunchKernelGGL(gg::cg_init_kernel, dim3(1), dim3(1024), 0, gg::as_stream(stream), rr_dev,
                       (int64_t)1, cg->sc, rtol, atol);
    GG_LAUNCH_CHECK();
  });
}

int gg_cg_iterate_partial(gg_cg* cg, double* red_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cg->x && red_dev, GG_ERR_VALUE, "CG not started");
    GG_REQUIRE(cg->fused && cg->fusion == 0, GG_ERR_VALUE,
               "the sharded rank runs the fused recurrence, layout 0");
    GG_REQUIRE(!cg->await_finish, GG_ERR_VALUE, "gg_cg_iterate_finish first");
    hipStream_t s = gg::as_stream(stream);
    const int64_t n = cg->n;
    int64_t nparts = 0;
    hipEvent_t* ev = nullptr;
    if (cg->profiling) {
      const size_t need = cg->events_used + (size_t)cg->launches() + 1;
      while (cg->events.size() < need) {
        hipEvent_t e;
        GG_HIP(hipEventCreate(&e));
        cg->events.push_back(e);
      }
      ev = cg->events.data() + cg->events_used;
      cg->events_used = need;
    }
    // no repair kernels: a cancelled beta (set to 0 by the scalars) restarts
    // the recurrence with p = r instead of a second all-reduce
    const int xmode = cg->xmode;
    gg::MpFuse fz;
    fz.r = cg->r;
    fz.q_old = cg->q;
    fz.p_out = cg->p2;
    fz.sc = cg->sc;
    fz.rr_part = cg->rr_part;
    fz.rr_cap = cg->rr_count;
    int64_t pro_blocks = 0;
    fz.pro_blocks = &pro_blocks;
    fz.sx = cg->x;
    fz.sp = cg->p;
    fz.sn = n;
    fz.xdefer = xmode;
    fz.xwin = cg->xwin;
    fz.rderive = cg->rder;
    fz.pprev = cg->rder ? cg->pprev_buf() : nullptr;
    fz.first_dst = cg->first_dst;
    const bool rq_ident = cg->rq != 0;
    fz.er = rq_ident ? nullptr : cg->r;
    fz.pqo_stride = rq_ident ? cg->rr_count : 0;
    fz.pstride = cg->mv_partials;
    if (cg->block) {
      // the rank's blocks: d - 1 launches, q2 <- (K + s I) p_new
      fz.blk_q_out = cg->q2;
      gg::block_apply(cg->blk, cg->p, cg->q, cg->shift, nullptr, cg->partials, &cg->sc->done, s,
                      &nparts, &fz, 2, ev, cg->rblk0, cg->rnblk);
    } else {
      gg::kron_apply(cg->K, false, cg->p, cg->q, cg->shift, cg->mv_work, cg->partials,
                     &cg->sc->done, s, &nparts, &fz, 2, ev);
    }
    GG_REQUIRE(pro_blocks > 0 && pro_blocks <= cg->rr_count, GG_ERR_RUNTIME,
               "fused CG: no prologue launch recorded");
    if (cg->block) std::swap(cg->q, cg->q2);
    hipLaunchKernelGGL(gg::cg_local_red_kernel, dim3(1), dim3(1024), 0, s, cg->rr_part,
                       pro_blocks, cg->rr_count, cg->partials, nparts, cg->mv_partials,
                       rq_ident ? 1 : 0, red_dev);
    GG_LAUNCH_CHECK();
    cg->await_finish = true;
  });
}

int gg_cg_iterate_finish(gg_cg* cg, const double* red_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && red_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(cg->await_finish, GG_ERR_VALUE, "gg_cg_iterate_partial first");
    hipStream_t s = gg::as_stream(stream);
    const int xmode = cg->xmode;
    const bool rq_ident = cg->rq != 0;
    // red = [rr, p.q_old | p.q, r.q, q.q]: one-element partial arrays
    hipLaunchKernelGGL(gg::cg_fused_scalars_kernel, dim3(1), dim3(1024), 0, s, red_dev,
                       (int64_t)1, (int64_t)1, red_dev + 2, (int64_t)1, (int64_t)1, cg->sc,
                       xmode ? (const double*)cg->p2 : nullptr, xmode, rq_ident ? 1 : 0,
                       cg->rder ? 1 : 0);
    GG_LAUNCH_CHECK();
    cg->rotate_dirs();
    cg->await_finish = false;
  });
}

int gg_cg_close_partial(gg_cg* cg, double* rr_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cg->x && rr_dev, GG_ERR_VALUE, "CG not started");
    GG_REQUIRE(!cg->await_finish, GG_ERR_VALUE, "gg_cg_iterate_finish first");
    hipStream_t s = gg::as_stream(stream);
    const int64_t n = cg->n;
    const int nb = gg::vec_blocks(n);
    if (cg->xmode == 3) {
      hipLaunchKernelGGL(gg::cg_x_flush3_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, cg->x, n,
                         gg::xwin_region(n, cg->xwin), cg->sc);
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::cg_x_flushed3_kernel, dim3(1), dim3(1), 0, s, cg->sc);
      GG_LAUNCH_CHECK();
    } else if (cg->xmode == 2) {
      hipLaunchKernelGGL(gg::cg_x_flush2_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, cg->x, n,
                         cg->block ? gg::block_side_half(n) : gg::kron_side_half(cg->K, n),
                         cg->sc);
      GG_LAUNCH_CHECK();
    } else if (cg->xmode == 1) {
      hipLaunchKernelGGL(gg::cg_x_flush_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, cg->x, n,
                         cg->sc);
      GG_LAUNCH_CHECK();
    }
    if (cg->xmode == 1 || cg->xmode == 2) {
      hipLaunchKernelGGL(gg::cg_x_flushed_kernel, dim3(1), dim3(1), 0, s, cg->sc);
      GG_LAUNCH_CHECK();
    }
    // the pending r update (x: the x_defer bookkeeping above, or here)
    GG_HIP(hipMemsetAsync(cg->partials, 0, nb * sizeof(double), s));
    if (cg->rder) {
      hipLaunchKernelGGL(gg::cg_r_materialize_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                         cg->r, cg->q, n, cg->sc, cg->partials, 1);
      GG_LAUNCH_CHECK();
      hipLaunchKernelGGL(gg::cg_r_stored_kernel, dim3(1), dim3(1), 0, s, cg->sc);
    } else {
      hipLaunchKernelGGL(gg::cg_xr_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                         cg->xmode ? nullptr : cg->x, cg->r, cg->p, cg->q, n, cg->sc,
                         cg->partials, 1);
    }
    GG_LAUNCH_CHECK();
    gg::launch_reduce_to(cg->partials, nb, rr_dev, s);
  });
}

int gg_cg_close_finish(gg_cg* cg, const double* rr_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && rr_dev, GG_ERR_VALUE, "NULL argument");
    hipLaunchKernelGGL(gg::cg_close_rho_kernel, dim3(1), dim3(1), 0, gg::as_stream(stream),
                       cg->sc, rr_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_cg_cancels(gg_cg* cg, int* cancels, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg && cancels, GG_ERR_VALUE, "NULL argument");
    hipStream_t s = gg::as_stream(stream);
    GG_HIP(hipMemcpyAsync(cg->sc_host, cg->sc, sizeof(gg::CgScalars), hipMemcpyDeviceToHost,
                          s));
    GG_HIP(hipStreamSynchronize(s));
    *cancels = cg->sc_host->cancels;
  });
}

int gg_cg_status(gg_cg* cg, int* iters, int* converged, double* resid_norm, double* tol,
                 gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(cg, GG_ERR_VALUE, "NULL handle");
    hipStream_t s = gg::as_stream(stream);
    GG_HIP(hipMemcpyAsync(cg->sc_host, cg->sc, sizeof(gg::CgScalars), hipMemcpyDeviceToHost,
                          s));
    GG_HIP(hipStreamSynchronize(s));
    const gg::CgScalars& h = *cg->sc_host;
    if (iters) *iters = h.iters;
    if (converged) *converged = (h.done && std::sqrt(h.rho) < h.tol) || h.bnorm == 0.0;
    if (resid_norm) *resid_norm = std::sqrt(h.rho);
    if (tol) *tol = h.tol;
  });
}

}  // extern "C"

namespace gg {


// gg_lanczos_probe / gg_lanczos_probe_timed.  step_ms (steps entries, may be
// null): HIP events on the stream at every step boundary -- the first after
// the probe is drawn, so allocation, the u_prev memset and the probe kernel
// are outside -- and the last after the final |w|^2 reduction, before the
// alphas / betas are copied back; launch_ms (d entries, may be null): the
// summed time of each mode-product position over the steps.
static void lanczos_probe(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                          double* work_dev, double* alphas_host, double* betas_host,
                          int* steps_done, double* step_ms, double* launch_ms,
                          gg_stream stream);
static bool lanczos_use_block(const gg_kron* K);

}  // namespace gg

extern "C" {

int gg_lanczos_probe(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                     double* work_dev, double* alphas_host, double* betas_host,
                     int* steps_done, gg_stream stream) {
  return gg::guard([&] {
    gg::lanczos_probe(K, shift, seed, probe, steps, work_dev, alphas_host, betas_host,
                      steps_done, nullptr, nullptr, stream);
  });
}

int gg_lanczos_info(const gg_kron* K, int* block, int* launches) {
  return gg::guard([&] {
    GG_REQUIRE(K && block && launches, GG_ERR_VALUE, "NULL argument");
    const bool b = gg::lanczos_use_block(K);
    *block = b ? 1 : 0;
    *launches = b ? gg::block_launches(gg::kron_block(K)) : gg::kron_d(K);
  });
}

int gg_lanczos_probe_timed(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                           double* work_dev, double* alphas_host, double* betas_host,
                           int* steps_done, double* step_ms_host, double* launch_ms_host,
                           gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(step_ms_host != nullptr, GG_ERR_VALUE, "step_ms_host is NULL");
    gg::lanczos_probe(K, shift, seed, probe, steps, work_dev, alphas_host, betas_host,
                      steps_done, step_ms_host, launch_ms_host, stream);
  });
}

}  // extern "C"

namespace gg {

// the block basis for the probe where the operator has one with d >= 3 (the
// Lanczos tridiagonal is invariant under the orthogonal fold P: the probe z
// becomes P z, the operator P K P^T); GG_LZ_BASIS=0 (snapshot) keeps the grid
static bool lanczos_use_block(const gg_kron* K) {
  const BlockOp* B = kron_block(K);
  // unpadded layouts only: the probe's workspace is 4 n (the grid's n)
  if (B == nullptr || block_d(B) < 3 || block_n(B) != kron_n(K)) return false;
  const char* e = knob("GG_LZ_BASIS");
  if (e) return atoi(e) != 0;
  return block_efficient(B);
}

// The fused Lanczos step in the parity-block basis: d - 1 launches and 10
// passes over N per step -- the first launch's prologue forms w_{j-1} = cy Y +
// cu u + cp u_prev (KIND 4: read Y, u, u_prev, write w over u_prev and the
// launch's output over Y), the plain launches 2 each, the pair launch reads
// its slab and w and writes Y_j = (K + shift) w with the u.Y partials.  One
// fold of the probe before, no unfold (only the tridiagonal leaves).
static void lanczos_block(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                          double* work_dev, double* alphas_host, double* betas_host,
                          int* steps_done, double* step_ms, double* launch_ms,
                          gg_stream stream) {
  hipStream_t s = gg::as_stream(stream);
  const BlockOp* B = kron_block(K);
  const int64_t n = block_n(B);
  const int L = block_launches(B);
  double* P = work_dev;          // u_prev; w is written over it
  double* V = work_dev + n;      // u (v = sV u)
  double* W = work_dev + 2 * n;  // Y of the previous step (the chain runs in place on it)
  double* W2 = work_dev + 3 * n; // the pair launch's output
  const int nb = vec_blocks(n);
  const int64_t npart = std::max<int64_t>(block_partials_needed(B), kVecBlocks);
  const int64_t nrr = std::max<int64_t>(block_prologue_blocks(B), 1);
  // [alphas | betas | partials (3 x npart: p.q, r.q, q.q) | |w|^2 partials | lzs(8)]
  double* scal = nullptr;
  GG_HIP(hipMallocAsync(&scal, (2 * (size_t)steps + 3 * npart + nrr + 8) * sizeof(double), s));
  double* alphas = scal;
  double* betas = scal + steps;
  double* parts = scal + 2 * steps;
  double* rrparts = parts + 3 * npart;
  double* lzs = rrparts + nrr;
  // step 0's prologue copies u_0: w = 0 Y + 1 u + 0 u_prev (Y, u_prev zeroed)
  const double init[5] = {1.0, 0.0, 0.0, 1.0, 0.0};
  GG_HIP(hipMemcpyAsync(lzs, init, sizeof(init), hipMemcpyHostToDevice, s));
  GG_HIP(hipMemsetAsync(P, 0, n * sizeof(double), s));
  GG_HIP(hipMemsetAsync(W, 0, n * sizeof(double), s));
  // the probe (grid layout, |z| = 1) into W2, folded into V
  hipLaunchKernelGGL(probe_kernel, dim3(nb), dim3(kVecThreads), 0, s, probe_base(seed, probe),
                     1.0 / std::sqrt((double)n), W2, n);
  GG_LAUNCH_CHECK();
  block_fold(B, false, W2, V, nullptr, s);
  const bool timed = step_ms != nullptr;
  // step boundaries, then the closing pass's end (ev[steps] -> ev[steps + 1])
  EventSet sev(timed ? (size_t)steps + 2 : 0);
  EventSet mev(timed && launch_ms ? (size_t)steps * (L + 1) : 0);
  auto mp_ev = [&](int j) -> hipEvent_t* {
    return mev.ev.empty() ? nullptr : mev.ev.data() + (size_t)j * (L + 1);
  };
  if (timed) GG_HIP(hipEventRecord(sev.ev[0], s));
  for (int j = 0; j < steps; ++j) {
    MpFuse lf;
    lf.r = V;
    lf.q_old = W;
    lf.p_out = P;
    lf.coef = lzs + 2;
    lf.rr_part = rrparts;
    lf.rr_cap = nrr;
    int64_t pro_blocks = 0;
    lf.pro_blocks = &pro_blocks;
    lf.blk_q_out = W2;
    lf.pstride = npart;
    int64_t np = 0;
    block_apply(B, P, W, shift, nullptr, parts, nullptr, s, &np, &lf, 3, mp_ev(j));
    GG_REQUIRE(pro_blocks > 0 && pro_blocks <= nrr, GG_ERR_RUNTIME,
               "Lanczos: no prologue launch recorded");
    hipLaunchKernelGGL(lzb_step_kernel, dim3(1), dim3(1024), 0, s, rrparts, pro_blocks, parts, np,
                       lzs, alphas + j, j > 0 ? betas + (j - 1) : betas, j == 0 ? 1 : 0);
    GG_LAUNCH_CHECK();
    std::swap(P, V);    // u_prev <- u_j's predecessor ... u <- w (= u_j)
    std::swap(W, W2);   // Y_j becomes the next step's chain
    if (timed && j + 1 < steps) GG_HIP(hipEventRecord(sev.ev[j + 1], s));
  }
  // the closing pass, once per probe: beta_{steps-1} = |w_{steps-1}| (one
  // streaming pass, in place of Y; T_k itself needs beta_0 .. beta_{k-2})
  if (timed) GG_HIP(hipEventRecord(sev.ev[steps], s));
  const int wide = ((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(V) |
                     reinterpret_cast<uintptr_t>(P)) & 15) == 0;
  hipLaunchKernelGGL(lz_update_kernel, dim3(nb), dim3(kVecThreads), 0, s, W, V, P, n, lzs + 0,
                     parts, wide);
  GG_LAUNCH_CHECK();
  launch_reduce_to(parts, nb, betas + (steps - 1), s);
  hipLaunchKernelGGL(lz_beta_kernel, dim3(1), dim3(1), 0, s, lzs, betas + (steps - 1));
  GG_LAUNCH_CHECK();
  if (timed) GG_HIP(hipEventRecord(sev.ev[steps + 1], s));
  GG_HIP(hipMemcpyAsync(alphas_host, alphas, steps * sizeof(double), hipMemcpyDeviceToHost, s));
  GG_HIP(hipMemcpyAsync(betas_host, betas, steps * sizeof(double), hipMemcpyDeviceToHost, s));
  GG_HIP(hipFreeAsync(scal, s));
  GG_HIP(hipStreamSynchronize(s));
  if (timed) {
    for (int j = 0; j < steps; ++j) {
      float ms = 0.f;
      GG_HIP(hipEventElapsedTime(&ms, sev.ev[j], sev.ev[j + 1]));
      step_ms[j] = ms;
    }
    if (launch_ms) {
      const int d = kron_d(K);
      for (int k = 0; k < d; ++k) launch_ms[k] = 0.0;
      for (int j = 0; j < steps; ++j)
        for (int k = 0; k < L; ++k) {
          float ms = 0.f;
          GG_HIP(hipEventElapsedTime(&ms, mp_ev(j)[k], mp_ev(j)[k + 1]));
          launch_ms[k] += ms;
        }
      float ms = 0.f;
      GG_HIP(hipEventElapsedTime(&ms, sev.ev[steps], sev.ev[steps + 1]));
      launch_ms[d] = ms;
    }
  }
  int done = steps;
  for (int j = 0; j < steps; ++j)
    if (!(betas_host[j] > 1e-300)) {
      done = j + 1;
      break;
    }
  if (steps_done) *steps_done = done;
}

static void lanczos_probe(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                          double* work_dev, double* alphas_host, double* betas_host,
                          int* steps_done, double* step_ms, double* launch_ms,
                          gg_stream stream) {
  {
    GG_REQUIRE(K && work_dev && alphas_host && betas_host && steps >= 1, GG_ERR_VALUE,
               "bad argument");
    int64_t nr = 0, nc = 0, we = 0;
    gg_kron_shape(K, 0, &nr, &nc, &we);
    GG_REQUIRE(nr == nc, GG_ERR_VALUE, "Lanczos needs a square operator");
    GG_REQUIRE(we <= nr, GG_ERR_VALUE, "non-square factors are not supported here");
    if (lanczos_use_block(K)) {
      lanczos_block(K, shift, seed, probe, steps, work_dev, alphas_host, betas_host, steps_done,
                    step_ms, launch_ms, stream);
      return;
    }
    hipStream_t s = gg::as_stream(stream);
    const int64_t n = nr;
    double* P = work_dev;        // u_prev (v_prev = sP u_prev)
    double* V = work_dev + n;    // u      (v = sV u)
    double* W = work_dev + 2 * n;
    double* mvw = work_dev + 3 * n;
    const int nb = gg::vec_blocks(n);
    const int64_t npart = std::max<int64_t>(gg::kron_partials_needed(K, false), gg::kVecBlocks);
    const int64_t nrr = std::max<int64_t>(gg::kron_prologue_blocks(K), 1);
    // [alphas | betas | partials | |w|^2 partials | zero | dot | lzs(8)]
    double* scal = nullptr;
    GG_HIP(hipMallocAsync(&scal, (2 * (size_t)steps + npart + nrr + 10 + 8) * sizeof(double), s));
    double* alphas = scal;
    double* betas = scal + steps;
    double* parts = scal + 2 * steps;
    double* rrparts = parts + npart;
    double* zero = rrparts + nrr;
    double* dot = zero + 1;
    double* lzs = dot + 1;
    const double init[2] = {1.0, 0.0};   // sV = 1 (the probe is normalised), sP = 0
    GG_HIP(hipMemsetAsync(zero, 0, sizeof(double), s));
    GG_HIP(hipMemcpyAsync(lzs, init, sizeof(init), hipMemcpyHostToDevice, s));
    GG_HIP(hipMemsetAsync(P, 0, n * sizeof(double), s));
    hipLaunchKernelGGL(gg::probe_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s,
                       gg::probe_base(seed, probe), 1.0 / std::sqrt((double)n), V, n);
    GG_LAUNCH_CHECK();
    const int d = gg::kron_d(K);
    const bool timed = step_ms != nullptr;
    // step boundaries, then the closing pass's end (ev[steps] -> ev[steps + 1];
    // with the update fused, the last step's update pass is the closing one)
    gg::EventSet sev(timed ? (size_t)steps + 2 : 0);
    gg::EventSet mev(timed && launch_ms ? (size_t)steps * (d + 1) : 0);
    auto mp_ev = [&](int j) -> hipEvent_t* {
      return mev.ev.empty() ? nullptr : mev.ev.data() + (size_t)j * (d + 1);
    };
    if (timed) GG_HIP(hipEventRecord(sev.ev[0], s));
    // w = cy W + cu u + cp u_prev in place of W, |w|^2 -> betas[j], scales
    auto update_beta = [&](int j) {
      const int wide = ((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(V) |
                         reinterpret_cast<uintptr_t>(P)) & 15) == 0;
      hipLaunchKernelGGL(gg::lz_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, W, V, P, n,
                         lzs, parts, wide);
      GG_LAUNCH_CHECK();
      gg::launch_reduce_to(parts, nb, betas + j, s);
      hipLaunchKernelGGL(gg::lz_beta_kernel, dim3(1), dim3(1), 0, s, lzs, betas + j);
      GG_LAUNCH_CHECK();
    };
    // The update of step j - 1 rides on step j's first mode product as its
    // prologue (CGP 3: the MFMA operand is w itself, written over u_prev)
    // when the chain's first step writes its scratch, not y (an even number
    // of factors); otherwise it is its own streaming pass.
    const bool fuse = gg::kron_d(K) % 2 == 0;
    for (int j = 0; j < steps; ++j) {
      int64_t np = 0;
      if (j == 0 || !fuse) {
        // W = K u + shift u, and u.W per block of the last mode product
        gg::kron_apply(K, false, V, W, shift, mvw, parts, nullptr, s, &np, nullptr, 0, mp_ev(j));
      } else {
        gg::MpFuse lf;
        lf.r = V;
        lf.q_old = P;
        lf.p_out = P;
        lf.rr_part = rrparts;
        lf.rr_cap = nrr;
        int64_t pro_blocks = 0;
        lf.pro_blocks = &pro_blocks;
        lf.coef = lzs;
        gg::kron_apply(K, false, W, W, shift, mvw, parts, nullptr, s, &np, &lf, 3, mp_ev(j));
        GG_REQUIRE(pro_blocks > 0 && pro_blocks <= nrr, GG_ERR_RUNTIME,
                   "Lanczos: no prologue launch recorded");
        // |w|^2 of the prologue -> beta_{j-1}; w (now in P) is the new u
        gg::launch_reduce_to(rrparts, pro_blocks, betas + (j - 1), s);
        hipLaunchKernelGGL(gg::lz_beta_kernel, dim3(1), dim3(1), 0, s, lzs, betas + (j - 1));
        GG_LAUNCH_CHECK();
        std::swap(P, V);   // u_prev <- u, u <- w
      }
      gg::launch_reduce_to(parts, np, dot, s);
      const double* beta_prev = (j == 0) ? zero : betas + (j - 1);
      hipLaunchKernelGGL(gg::lz_coef_kernel, dim3(1), dim3(1), 0, s, lzs, dot, alphas + j,
                         beta_prev);
      GG_LAUNCH_CHECK();
      const bool closing = fuse && j + 1 == steps;
      if (!fuse || j + 1 == steps) {
        if (timed && closing) GG_HIP(hipEventRecord(sev.ev[steps], s));
        update_beta(j);
        if (j + 1 < steps) {
          // rotate: u_prev <- u, u <- w, the old u_prev buffer takes the next matvec
          double* oldP = P;
          P = V;
          V = W;
          W = oldP;
        }
      }
      if (timed && !closing) GG_HIP(hipEventRecord(sev.ev[j + 1], s));
    }
    if (timed) GG_HIP(hipEventRecord(sev.ev[steps + 1], s));
    GG_HIP(hipMemcpyAsync(alphas_host, alphas, steps * sizeof(double), hipMemcpyDeviceToHost,
                          s));
    GG_HIP(hipMemcpyAsync(betas_host, betas, steps * sizeof(double), hipMemcpyDeviceToHost, s));
    GG_HIP(hipFreeAsync(scal, s));
    GG_HIP(hipStreamSynchronize(s));
    if (timed) {
      for (int j = 0; j < steps; ++j) {
        float ms = 0.f;
        GG_HIP(hipEventElapsedTime(&ms, sev.ev[j], sev.ev[j + 1]));
        step_ms[j] = ms;
      }
      if (launch_ms) {
        for (int k = 0; k < d; ++k) launch_ms[k] = 0.0;
        for (int j = 0; j < steps; ++j)
          for (int k = 0; k < d; ++k) {
            float ms = 0.f;
            GG_HIP(hipEventElapsedTime(&ms, mp_ev(j)[k], mp_ev(j)[k + 1]));
            launch_ms[k] += ms;
          }
        float ms = 0.f;
        GG_HIP(hipEventElapsedTime(&ms, sev.ev[steps], sev.ev[steps + 1]));
        launch_ms[d] = ms;
      }
    }
    int done = steps;
    for (int j = 0; j < steps; ++j)
      if (!(betas_host[j] > 1e-300)) {
        done = j + 1;
        break;
      }
    if (steps_done) *steps_done = done;
  }
}

}  // namespace gg

// ============================================ CG scalars for a host-driven (sharded) CG
// The sharded solve (gp_grief_amd/distributed.py) runs the same recurrence as
// gg_cg_*: local partial dots land in device doubles, the caller all-reduces
// them with RCCL, and these kernels consume the global values.
namespace gg {

// q += shift p ; partial p.q -- 16-byte lanes when q and p are 16-byte
// aligned (wide), else 8-byte
__global__ __launch_bounds__(kVecThreads) void shift_dot_kernel(double* __restrict__ q,
                                                                const double* __restrict__ p,
                                                                int64_t n, double shift,
                                                                const CgScalars* __restrict__ sc,
                                                                double* __restrict__ partials,
                                                                int wide) {
  if (sc->done) return;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (wide) {
    const int64_t n2 = n / 2;
    double2* q2 = reinterpret_cast<double2*>(q);
    const double2* p2 = reinterpret_cast<const double2*>(p);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
      const double2 pv = p2[i];
      double2 v = q2[i];
      v.x = fma(shift, pv.x, v.x);
      v.y = fma(shift, pv.y, v.y);
      q2[i] = v;
      acc = fma(pv.x, v.x, acc);
      acc = fma(pv.y, v.y, acc);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {
      const double v = fma(shift, p[n - 1], q[n - 1]);
      q[n - 1] = v;
      acc = fma(p[n - 1], v, acc);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const double pv = p[i];
      const double v = fma(shift, pv, q[i]);
      q[i] = v;
      acc = fma(pv, v, acc);
    }
  }
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ void cgs_init_kernel(CgScalars* sc, const double* rr, double rtol, double atol) {
  const double s = *rr;
  sc->rho = s;
  sc->rho_prev = 0.0;
  sc->bnorm = sqrt(s);
  sc->tol = fmax(atol, rtol * sc->bnorm);
  sc->iters = 0;
  sc->first = 1;
  sc->pending = 0;
  sc->alpha = sc->beta = sc->pq = 0.0;
  // the fused recurrence's state (unused by the textbook one)
  sc->rq = sc->qq = 0.0;
  sc->repair = 0;
  sc->cancels = 0;
  sc->xpend = 0;
  sc->xh = 2;
  sc->xs = 0;
  sc->done = (s == 0.0 || !(sqrt(s) >= sc->tol)) ? 1 : 0;
}

// ---- fused sharded CG (gg_cgs_fused_*): the single-GPU fused recurrence
// with the dot products reduced across ranks by ONE all-reduce of five
// doubles per iteration, red = [r.r, p.q_old, p.q, 0, q.q] (the caller
// all-reduces it between gg_cgs_fused_post and gg_cgs_fused_scalars)

// block partials of p.q' and q'.q', q' = Y + shift p (Y = K p after the
// exchanges, left unshifted: the next prologue adds shift p_old itself) --
// two read streams, 16-byte lanes (n even, 16-byte aligned vectors)
__global__ __launch_bounds__(kVecThreads) void cgs_post_kernel(
    const double* __restrict__ q, const double* __restrict__ p, int64_t n, double shift,
    const CgScalars* __restrict__ sc, double* __restrict__ part, int64_t pstride) {
  if (sc->done) return;
  double pq = 0.0, qq = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const double2* q2 = reinterpret_cast<const double2*>(q);
  const double2* p2 = reinterpret_cast<const double2*>(p);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += stride) {
    const double2 pv = p2[i];
    double2 v = q2[i];
    v.x = fma(shift, pv.x, v.x);
    v.y = fma(shift, pv.y, v.y);
    pq = fma(pv.x, v.x, pq);
    pq = fma(pv.y, v.y, pq);
    qq = fma(v.x, v.x, qq);
    qq = fma(v.y, v.y, qq);
  }
  const double a = block_sum(pq);
  __syncthreads();
  const double b = block_sum(qq);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = a;
    part[pstride + blockIdx.x] = b;
  }
}

// red = [sum rr_part[0, nrr), sum rr_part[cap, cap + nrr), sum pq, 0, sum qq]
__global__ __launch_bounds__(1024) void cgs_fused_red_kernel(
    const double* __restrict__ rr_part, int64_t nrr, int64_t cap,
    const double* __restrict__ part, int64_t np, int64_t pstride, double* __restrict__ red) {
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t i = threadIdx.x; i < nrr; i += blockDim.x) {
    a[0] += rr_part[i];
    a[1] += rr_part[cap + i];
  }
  for (int64_t i = threadIdx.x; i < np; i += blockDim.x) {
    a[2] += part[i];
    a[3] += part[pstride + i];
  }
  double t[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t[k] = block_sum(a[k]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    red[0] = t[0];
    red[1] = t[1];
    red[2] = t[2];
    red[3] = 0.0;
    red[4] = t[3];
  }
}

// the closing pending update r -= alpha (q + shift p), partial r.r
__global__ __launch_bounds__(kVecThreads) void cgs_close_r_kernel(
    double* __restrict__ r, const double* __restrict__ q, const double* __restrict__ p, int64_t n,
    double shift, const CgScalars* __restrict__ sc, double* __restrict__ partials) {
  if (sc->done || !sc->pending) return;
  const double a = sc->alpha;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double rv = r[i] - a * fma(shift, p[i], q[i]);
    r[i] = rv;
    acc = fma(rv, rv, acc);
  }
  const double s = block_sum(acc);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// the closing textbook step (cg_rho_kernel's need_pending 1) from the global
// r.r (all-reduced by the caller)
__global__ void cgs_close_rho_kernel(CgScalars* sc, const double* rr) {
  if (sc->done || !sc->pending) return;
  const double s = *rr;
  sc->rho_prev = sc->rho;
  sc->rho = s;
  sc->beta = s / sc->rho_prev;
  sc->iters += 1;
  sc->first = 0;
  sc->pending = 0;
  sc->repair = 0;
  if (!(sqrt(s) >= sc->tol)) sc->done = 1;
}

__global__ void cgs_alpha_kernel(CgScalars* sc, const double* pq) {
  if (sc->done) return;
  sc->pq = *pq;
  sc->alpha = sc->rho / *pq;
}

__global__ void cgs_rho_kernel(CgScalars* sc, const double* rr) {
  if (sc->done) return;
  const double s = *rr;
  sc->rho_prev = sc->rho;
  sc->rho = s;
  sc->beta = s / sc->rho_prev;
  sc->iters += 1;
  sc->first = 0;
  if (!(sqrt(s) >= sc->tol)) sc->done = 1;
}

}  // namespace gg

struct gg_cgs {
  gg::CgScalars* sc = nullptr;
  gg::CgScalars* host = nullptr;
  double* partials = nullptr;   // kVecBlocks, or 2 x kVecBlocks (fused post)
  // fused recurrence: the prologue launch's r.r / p.q_old partials
  // (2 x rr_cap) and its actual workgroup count
  double* rr_part = nullptr;
  int64_t rr_cap = 0;
  int64_t pro_blocks = 0;
};

namespace gg {

CgScalars* cgs_scalars_ptr(gg_cgs* c) { return c->sc; }

// the prologue partial arrays for launches of up to `cap` workgroups (grown
// on demand, zero-filled)
double* cgs_rr_part(gg_cgs* c, int64_t cap, int64_t* cap_out) {
  if (c->rr_cap < cap) {
    if (c->rr_part) GG_HIP(hipFree(c->rr_part));
    c->rr_part = nullptr;
    GG_HIP(hipMalloc(&c->rr_part, 2 * (size_t)cap * sizeof(double)));
    GG_HIP(hipMemset(c->rr_part, 0, 2 * (size_t)cap * sizeof(double)));
    c->rr_cap = cap;
  }
  *cap_out = c->rr_cap;
  return c->rr_part;
}

void cgs_set_pro_blocks(gg_cgs* c, int64_t nb) { c->pro_blocks = nb; }

}  // namespace gg

extern "C" {

int gg_cgs_create(gg_cgs** out) {
  return gg::guard([&] {
    gg::knobs_reload();   // the handle's switches are the environment's now
    GG_REQUIRE(out, GG_ERR_VALUE, "NULL argument");
    gg_cgs* c = new gg_cgs();
    try {
      GG_HIP(hipMalloc(&c->sc, sizeof(gg::CgScalars)));
      gg::scalars_clear(c->sc);
      GG_HIP(hipHostMalloc(&c->host, sizeof(gg::CgScalars), hipHostMallocDefault));
      GG_HIP(hipMalloc(&c->partials, 2 * gg::kVecBlocks * sizeof(double)));
    } catch (...) {
      gg_cgs_destroy(c);
      throw;
    }
    *out = c;
  });
}

int gg_cgs_destroy(gg_cgs* c) {
  return gg::guard([&] {
    if (!c) return;
    if (c->sc) (void)hipFree(c->sc);
    if (c->host) (void)hipHostFree(c->host);
    if (c->partials) (void)hipFree(c->partials);
    if (c->rr_part) (void)hipFree(c->rr_part);
    delete c;
  });
}

int gg_cgs_scalars(gg_cgs* c, void** scalars_dev) {
  return gg::guard([&] {
    GG_REQUIRE(c && scalars_dev, GG_ERR_VALUE, "NULL argument");
    *scalars_dev = c->sc;
  });
}

int gg_cgs_local_dot(gg_cgs* c, const double* x_dev, const double* y_dev, int64_t n,
                     double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && x_dev && y_dev && out_dev, GG_ERR_VALUE, "NULL argument");
    hipStream_t s = gg::as_stream(stream);
    const int nb = gg::vec_blocks(n);
    gg::launch_dot_partials(x_dev, y_dev, n, c->partials, nb, s);
    gg::launch_reduce_to(c->partials, nb, out_dev, s);
  });
}

int gg_cgs_init(gg_cgs* c, const double* rr_dev, double rtol, double atol, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && rr_dev && rtol >= 0 && atol >= 0, GG_ERR_VALUE, "bad argument");
    hipLaunchKernelGGL(gg::cgs_init_kernel, dim3(1), dim3(1), 0, gg::as_stream(stream), c->sc,
                       rr_dev, rtol, atol);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_shift_dot(gg_cgs* c, double* q_dev, const double* p_dev, int64_t n, double shift,
                     double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && q_dev && p_dev && out_dev, GG_ERR_VALUE, "NULL argument");
    hipStream_t s = gg::as_stream(stream);
    const int nb = gg::vec_blocks(n);
    const int wide =
        ((reinterpret_cast<uintptr_t>(q_dev) | reinterpret_cast<uintptr_t>(p_dev)) & 15) == 0;
    hipLaunchKernelGGL(gg::shift_dot_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, q_dev,
                       p_dev, n, shift, c->sc, c->partials, wide);
    GG_LAUNCH_CHECK();
    gg::launch_reduce_to(c->partials, nb, out_dev, s);
  });
}

int gg_cgs_alpha(gg_cgs* c, const double* pq_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && pq_dev, GG_ERR_VALUE, "NULL argument");
    hipLaunchKernelGGL(gg::cgs_alpha_kernel, dim3(1), dim3(1), 0, gg::as_stream(stream), c->sc,
                       pq_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_update(gg_cgs* c, double* x_dev, double* r_dev, const double* p_dev,
                  const double* q_dev, int64_t n, double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && x_dev && r_dev && p_dev && q_dev && out_dev, GG_ERR_VALUE, "NULL argument");
    hipStream_t s = gg::as_stream(stream);
    const int nb = gg::vec_blocks(n);
    hipLaunchKernelGGL(gg::cg_xr_update_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, x_dev,
                       r_dev, p_dev, q_dev, n, c->sc, c->partials, 0);
    GG_LAUNCH_CHECK();
    gg::launch_reduce_to(c->partials, nb, out_dev, s);
  });
}

int gg_cgs_rho(gg_cgs* c, const double* rr_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && rr_dev, GG_ERR_VALUE, "NULL argument");
    hipLaunchKernelGGL(gg::cgs_rho_kernel, dim3(1), dim3(1), 0, gg::as_stream(stream), c->sc,
                       rr_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_fused_post(gg_cgs* c, const double* q_dev, const double* p_dev, int64_t n,
                      double shift, double* red_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && q_dev && p_dev && red_dev && n >= 2 && n % 2 == 0, GG_ERR_VALUE,
               "bad argument");
    GG_REQUIRE(((reinterpret_cast<uintptr_t>(q_dev) | reinterpret_cast<uintptr_t>(p_dev)) & 15) ==
                   0,
               GG_ERR_VALUE, "fused post needs 16-byte aligned vectors");
    GG_REQUIRE(c->rr_part && c->pro_blocks > 0, GG_ERR_VALUE,
               "gg_cgs_fused_post needs a fused phase 1 first");
    hipStream_t s = gg::as_stream(stream);
    const int nb = gg::vec_blocks(n);
    hipLaunchKernelGGL(gg::cgs_post_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, q_dev, p_dev,
                       n, shift, c->sc, c->partials, (int64_t)gg::kVecBlocks);
    GG_LAUNCH_CHECK();
    hipLaunchKernelGGL(gg::cgs_fused_red_kernel, dim3(1), dim3(1024), 0, s, c->rr_part,
                       c->pro_blocks, c->rr_cap, c->partials, (int64_t)nb,
                       (int64_t)gg::kVecBlocks, red_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_fused_scalars(gg_cgs* c, const double* red_dev, const double* p_new_dev,
                         gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && red_dev && p_new_dev, GG_ERR_VALUE, "NULL argument");
    // red = [rr, p.q_old | p.q, (r.q), q.q]: the single-GPU scalars kernel
    // with one-element partial arrays (rr stride 1, matvec stride 1)
    hipLaunchKernelGGL(gg::cg_fused_scalars_kernel, dim3(1), dim3(1024), 0, gg::as_stream(stream),
                       red_dev, (int64_t)1, (int64_t)1, red_dev + 2, (int64_t)1, (int64_t)1,
                       c->sc, p_new_dev, 2, 1, 0);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_fused_close(gg_cgs* c, double* x_dev, double* r_dev, const double* q_dev,
                       const double* p_dev, int64_t n, int64_t half, double shift,
                       double* rr_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && x_dev && r_dev && q_dev && p_dev && rr_dev && half >= 0 && half <= n,
               GG_ERR_VALUE, "bad argument");
    hipStream_t s = gg::as_stream(stream);
    const int nb = gg::vec_blocks(n);
    // the deferred x steps, then the pending r update with its r.r partials
    hipLaunchKernelGGL(gg::cg_x_flush2_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, x_dev, n,
                       half, c->sc);
    GG_LAUNCH_CHECK();
    hipLaunchKernelGGL(gg::cg_x_flushed_kernel, dim3(1), dim3(1), 0, s, c->sc);
    GG_LAUNCH_CHECK();
    GG_HIP(hipMemsetAsync(c->partials, 0, nb * sizeof(double), s));
    hipLaunchKernelGGL(gg::cgs_close_r_kernel, dim3(nb), dim3(gg::kVecThreads), 0, s, r_dev,
                       q_dev, p_dev, n, shift, c->sc, c->partials);
    GG_LAUNCH_CHECK();
    gg::launch_reduce_to(c->partials, nb, rr_dev, s);
  });
}

int gg_cgs_fused_close_rho(gg_cgs* c, const double* rr_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c && rr_dev, GG_ERR_VALUE, "NULL argument");
    hipLaunchKernelGGL(gg::cgs_close_rho_kernel, dim3(1), dim3(1), 0, gg::as_stream(stream), c->sc,
                       rr_dev);
    GG_LAUNCH_CHECK();
  });
}

int gg_cgs_status(gg_cgs* c, int* iters, int* done, double* rho, double* tol,
                  gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(c, GG_ERR_VALUE, "NULL handle");
    hipStream_t s = gg::as_stream(stream);
    GG_HIP(hipMemcpyAsync(c->host, c->sc, sizeof(gg::CgScalars), hipMemcpyDeviceToHost, s));
    GG_HIP(hipStreamSynchronize(s));
    if (iters) *iters = c->host->iters;
    if (done) *done = c->host->done;
    if (rho) *rho = c->host->rho;
    if (tol) *tol = c->host->tol;
  });
}

}  // extern "C"
