// The Kronecker operator in its parity-block basis.
//
// Reference: KronMatrix.kronvec_prod, gp_grief/tensors/kron_matrix.py:52-97
// (y = (K_0 (x) ... (x) K_{d-1}) x, one BLAS3 product per factor).  This
// translation unit applies the SAME operator after an orthogonal change of
// basis; the change is an execution detail of that product.
//
// A centrosymmetric factor F (J F J = F, J the index reversal -- every
// stationary kernel on an evenly spaced grid) of even order m = 2h commutes
// with J, so in the basis u_i = (x_i + x_{m-1-i}) / sqrt 2, v_i = (x_i -
// x_{m-1-i}) / sqrt 2 (i < h) it is block diagonal: diag(S, T) with
//     S[j][i] = F[j][i] + F[j][m-1-i],   T[j][i] = F[j][i] - F[j][m-1-i].
// With every factor in that basis the whole operator is block diagonal over
// the 2^d parity patterns beta = (beta_0 .. beta_{d-1}):
//     P K P^T = diag_beta( F_0^{beta_0} (x) ... (x) F_{d-1}^{beta_{d-1}} ),
// F^0 = S, F^1 = T, each block a Kronecker product of h x h matrices.  P is
// orthogonal, so a CG run in this basis takes the same iterates (P x) up to
// rounding; the fold x -> P x and the unfold run once per solve.
//
// Layout in HBM ("block layout"): block beta (index B = sum_k beta_k 2^{d-1-k},
// slowest) of n_b = prod h_k elements, C order over the slab index (i'_0, ...,
// i'_{d-3}); a slab (the two innermost axes, h x h, h = h_{d-2} = h_{d-1} =
// 16 TF + 4) k-step tiled: element (i, a) at (a >> 2) 4 h + 4 i + (a & 3), so
// the h x 4 columns one k-step of the pair kernel's GEMM 1 contracts are one
// contiguous 32 h-byte run (whole 128-B lines; row-major they were 32 bytes
// of every row, each line touched by four k-steps apart in time).  Every other
// kernel treats a slab as a flat run of h^2 columns.
//
// Why: the fold makes each factor's h x h matrix an ordinary dense GEMM (no
// mirrored rows inside the kernels), and it makes the two innermost axes of a
// block one contiguous h x h SLAB (80 KB at h = 100) -- small enough that one
// launch applies BOTH of their factors, Z = F_{d-2} X F_{d-1}^T, with the
// intermediate held in registers.  A matvec is then d - 1 launches over the
// vector instead of d (6 passes instead of 8 at d = 4), every one in place
// (no rotation of axes, no scratch buffer for the chain):
//   * blk_mode_kernel, axes 0 .. d-3: Y[o][j][c] = sum_i F[j][i] X[o][i][c]
//     per block (the axis's rows strided by the inner extent); a wave owns 16
//     columns c and every output row j, the factor's A fragments sit in LDS,
//     the column data streams from HBM straight into the B operand;
//   * blk_pair_kernel, axes d-2, d-1: per slab Z = F_{d-2} X F_{d-1}^T, two
//     waves per slab (each half of the output columns), W = X F^T in
//     registers feeding the second GEMM as its B operand.
// Both run FP64 MFMA (v_mfma_f64_16x16x4_f64, the 4-row / 4-column tails of
// h = 16 TF + 4 on v_mfma_f64_4x4x4_4b_f64) and carry the fused CG's vector
// work like the folded kernels do (prologue on the first launch, the x side
// job on the second, q = K p + s p with the dots on the last).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "gg_internal.h"

namespace gg {

typedef double bd4 __attribute__((ext_vector_type(4)));

constexpr int kBlkMaxD = 6;        // 2^d corner values per fold thread
constexpr int kBlkModeWaves = 12;  // waves per blk_mode_kernel workgroup (3 / SIMD)
constexpr int kBlkPairWaves = 4;   // waves per blk_pair_kernel workgroup (2 slabs)

struct BlockOp {
  int d = 0;
  int64_t m[kBlkMaxD] = {}, h[kBlkMaxD] = {};
  // the layout's extent per axis: h, except the two innermost (the pair
  // axes), padded to hp = 16 TF + 4 >= h (round 6: pair orders that are not
  // 16 TF + 4 -- 64, 96, 128 ... -- run the same pair kernels on slabs whose
  // rows / columns past h are zero in the vectors and in the factors)
  int64_t e[kBlkMaxD] = {};
  int64_t nb = 0, n = 0;          // block size (prod e), vector length (2^d nb)
  // A / B fragments of S (parity 0) and T (1) per axis: [KS][JT][64] doubles,
  // frag(s, t, l) = F[16 t + (l & 15)][4 s + (l >> 4)] for full tiles, the tail
  // tile (T4) F[16 (JT-1) + (l & 3)][4 s + (l >> 4)] (rows replicated over the
  // four 4x4 blocks of v_mfma_f64_4x4x4_4b_f64); zero outside h x h
  double* frag[kBlkMaxD][2] = {};
  int KS[kBlkMaxD] = {}, JT[kBlkMaxD] = {};
  bool T4[kBlkMaxD] = {};
  int pTF = 0;   // pair axes: h = 16 pTF + 4
  int cus = 256;
  // blk_pair_lds_kernel (TF 2..6; GG_BLK_PAIR_LDS=0: blk_pair_kernel) with
  // pair_spw slabs per workgroup (2 when a block holds an even slab count;
  // GG_BLK_PAIR_SPW=1 forces 1)
  bool pair_lds = false;
  int pair_spw = 1;
  bool fast = true;   // blk_mode_fast_kernel where instantiated (GG_BLK_MODE_FAST=0: off)
  // the CG prologue's r / q_old / p_old loads and r / p_new stores non-temporal
  // (default; GG_BLK_PRO_NT=0 off): 200^4 prologue 13.84-14.02 -> 13.52-13.58
  // ms, interleaved processes (profiles/r05/y_pro_nt)
  bool pro_nt = true;
  // the fused CG pair launch's p loads and q stores non-temporal (default;
  // GG_BLK_EPI_NT=0 off): iteration 35.87-36.00 -> 35.41-35.54 ms on one box,
  // interleaved (the pair launch -0.2 ms, the next prologue -0.25;
  // profiles/r05/z_epi_nt)
  bool epi_nt = true;
};

// ------------------------------------------------------------------ fold
// Thread per mirror group (i'_0 .. i'_{d-1}): the 2^d corners x[..., i_k or
// m_k-1-i_k, ...] -> the 2^d blocks at offset i' by a Walsh-Hadamard
// transform over the d parity bits, scaled by 2^{-d/2} (orthogonal; its own
// inverse).  Consecutive threads take consecutive i'_{d-1}: the corner reads
// are ascending or descending runs, the block writes ascending runs.
// A block range [blk0, blk0 + nblk) (a rank of the sharded CG): the forward
// fold writes only those blocks (y holds them contiguously); the inverse reads
// only those (the others count as 0) and writes this range's contribution to
// every grid element (summed over the ranks by the caller).
struct FoldGeom {
  int d;
  int64_t m[kBlkMaxD], h[kBlkMaxD], stride[kBlkMaxD];
  int64_t hp;   // the slab's (padded) extent; positions with i or a >= h are zero
  int64_t nb;
  int64_t blk0, nblk;
};

template <int D>
__global__ __launch_bounds__(256) void blk_fold_kernel(const double* __restrict__ x,
                                                       double* __restrict__ y, FoldGeom g,
                                                       int inverse, double scale,
                                                       double* __restrict__ sq_part) {
  constexpr int C = 1 << D;
  double acc = 0.0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < g.nb;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, span[D];
    // t is the position in the block layout: the slab (outer axes, C order)
    // and, inside it, the k-step tiled (i, a) of the two innermost axes
    const int64_t hs = g.hp;
    const int64_t q = t % (hs * hs);
    int64_t rem = t / (hs * hs);
    {
      const int64_t a4 = q / (4 * hs), r4 = q - a4 * 4 * hs;
      const int64_t i = r4 >> 2, a = 4 * a4 + (r4 & 3);
      if (i >= g.h[D - 2] || a >= g.h[D - 1]) {
        // padding: zero in every block (forward), no grid element (inverse)
        if (!inverse)
          for (int c = 0; c < C; ++c) {
            const int64_t lb = (int64_t)c - g.blk0;
            if (lb >= 0 && lb < g.nblk) y[lb * g.nb + t] = 0.0;
          }
        continue;
      }
      lo = i * g.stride[D - 2] + a * g.stride[D - 1];
      span[D - 2] = (g.m[D - 2] - 1 - 2 * i) * g.stride[D - 2];   // low -> mirrored corner
      span[D - 1] = (g.m[D - 1] - 1 - 2 * a) * g.stride[D - 1];
    }
#pragma unroll
    for (int k = D - 3; k >= 0; --k) {
      const int64_t i = rem % g.h[k];
      rem /= g.h[k];
      lo += i * g.stride[k];
      span[k] = (g.m[k] - 1 - 2 * i) * g.stride[k];
    }
    double v[C];
    if (!inverse) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        int64_t o = lo;
#pragma unroll
        for (int k = 0; k < D; ++k)
          if ((c >> (D - 1 - k)) & 1) o += span[k];
        v[c] = x[o];
      }
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int64_t lb = (int64_t)c - g.blk0;   // wave-uniform
        v[c] = (lb >= 0 && lb < g.nblk) ? x[lb * g.nb + t] : 0.0;
      }
    }
#pragma unroll
    for (int b = 1; b < C; b <<= 1)
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (!(c & b)) {
          const double a0 = v[c], a1 = v[c | b];
          v[c] = a0 + a1;
          v[c | b] = a0 - a1;
        }
    if (!inverse) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int64_t lb = (int64_t)c - g.blk0;
        if (lb < 0 || lb >= g.nblk) continue;
        const double w = v[c] * scale;
        y[lb * g.nb + t] = w;
        acc = fma(w, w, acc);
      }
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        int64_t o = lo;
#pragma unroll
        for (int k = 0; k < D; ++k)
          if ((c >> (D - 1 - k)) & 1) o += span[k];
        y[o] = v[c] * scale;
      }
    }
  }
  if (sq_part != nullptr) {
    // deterministic per-block partial of |P x|^2 (the CG's starting r.r)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) sq_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

// wave-uniform byte address (SGPRs through readfirstlane) -- loads and
// stores below take the form base (SGPR pair) + a 32-bit lane byte offset, so
// the per-access address arithmetic is scalar and the few lane offsets are
// the only address VGPRs (the accumulators of W fill the register budget)
__device__ __forceinline__ char* ubase(const void* p, int64_t off) {
  const uint64_t v = reinterpret_cast<uint64_t>(p) + (uint64_t)off;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  uint64_t u = ((uint64_t)hi << 32) | lo;
  // opaque in SGPRs: otherwise (base + uniform) + lane offset is reassociated
  // into a 64-bit VGPR address per access (no saddr form, two VGPRs each)
  asm("" : "+s"(u));
  return reinterpret_cast<char*>(u);
}
// a wave-uniform 64-bit integer held in SGPRs (values the compiler computes
// in VGPRs, e.g. after a 64-bit division, though every lane agrees)
__device__ __forceinline__ int64_t uni64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// through address-space-1 pointers: global_load / global_store (a generic
// pointer gives FLAT instructions, whose out-of-order completion makes the
// compiler wait for vmcnt(0) and lgkmcnt(0) before every use)
typedef __attribute__((address_space(1))) char gchar;
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ double ldu(const void* p, int64_t uoff, uint32_t voff) {
  gchar* b = reinterpret_cast<gchar*>(reinterpret_cast<uintptr_t>(ubase(p, uoff)));
  return *reinterpret_cast<const gdouble*>(b + voff);
}
__device__ __forceinline__ void stu(void* p, int64_t uoff, uint32_t voff, double v) {
  gchar* b = reinterpret_cast<gchar*>(reinterpret_cast<uintptr_t>(ubase(p, uoff)));
  *reinterpret_cast<gdouble*>(b + voff) = v;
}
// the same, non-temporal when NT (CG streams touched once per iteration)
template <bool NT>
__device__ __forceinline__ double lduq(const void* p, int64_t uoff, uint32_t voff) {
  if constexpr (!NT) return ldu(p, uoff, voff);
  gchar* b = reinterpret_cast<gchar*>(reinterpret_cast<uintptr_t>(ubase(p, uoff)));
  return __builtin_nontemporal_load(reinterpret_cast<const gdouble*>(b + voff));
}
template <bool NT>
__device__ __forceinline__ void stuq(void* p, int64_t uoff, uint32_t voff, double v) {
  if constexpr (!NT) {
    stu(p, uoff, voff, v);
  } else {
    gchar* b = reinterpret_cast<gchar*>(reinterpret_cast<uintptr_t>(ubase(p, uoff)));
    __builtin_nontemporal_store(v, reinterpret_cast<gdouble*>(b + voff));
  }
}
// 16-byte global accesses (per-lane addresses)
typedef double gd2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) gd2v gd2;
__device__ __forceinline__ double2 ld2g(const double* p) {
  const gd2v v = *reinterpret_cast<const gd2*>(reinterpret_cast<uintptr_t>(p));
  return double2{v.x, v.y};
}
__device__ __forceinline__ void st2g(double* p, double2 v) {
  *reinterpret_cast<gd2*>(reinterpret_cast<uintptr_t>(p)) = gd2v{v.x, v.y};
}
// ------------------------------------------------- in-place mode product
// Axis k <= d-3 of every block, in place: Y[o][j][c] = sum_i F[j][i] X[o][i][c]
// (F = S_k or T_k by the block's parity bit for axis k; X may equal Y).
//
// A wave owns a strip of 16 columns c (inner % 16 == 0) and all h output
// rows: MFMA A = F fragments (LDS), B = the strip's rows 4 s .. 4 s + 3
// (lane l reads X[4 s + (l >> 4)][c0 + (l & 15)]: four 128-B row segments per
// wave instruction, every byte used once), D tile t: lane 16 g + n holds
// rows 16 t + 4 r + g (r = 0..3) of column c0 + n.  The k-steps of the
// wave's strips form one stream, loaded kDepth steps ahead into a register
// ring, so HBM latency spans strip boundaries.
//
// Work: groups of kBlkModeWaves strips inside one block (one factor per
// group); each workgroup takes a contiguous range of groups (it crosses at
// most a block boundary or two) and restages the factor's fragments into LDS
// when the parity changes.  One workgroup per CU (the fragments: KS x JT x
// 512 B, 89.6 KB at h = 100).
//
// KIND 0: plain.  KIND 1: the fused CG prologue (gg_vec.hip layout 0): X holds
// p_old; per element r -= alpha q_old when pending (written back, r.r
// partial), p_new = r + beta p_old (first: r) written to fz.p_out, p_new.q_old
// partial; the MFMA B operand is p_new; Y (the q buffer) is written over
// q_old at the same positions after this wave has read them.  KIND 2: plain
// plus the balanced x side job (x += c0 p0 + c1 p1 over half sc->xh of x),
// one slice of it per strip.  KIND 4: the fused Lanczos step's prologue
// (gg_lanczos_probe in the block basis): w = cy Y + cu u + cp u_prev formed
// per element as the operand, stored over u_prev, |w|^2 partials.
struct ModeArgs {
  const double* X;
  double* Y;
  const double* fS;
  const double* fT;
  int h, KS;
  int64_t inner;    // elements per row of the axis (product of the later h)
  int64_t spb;      // strips per block
  int64_t gpb;      // strip groups per block
  int64_t ngroups;  // 2^d gpb
  int64_t per_wg;   // groups per workgroup (contiguous ranges)
  int64_t nb;       // block size
  int bitpos;       // parity bit of the axis in the block index
  int64_t blk0;     // global index of the vector's first block (sharded CG)
  const int* skip;
  // CG prologue (KIND 1)
  double* r;
  const double* q_old;
  double* p_out;
  const CgScalars* sc;
  double* rr_part;    // [grid] r.r, [pqo_stride + grid] p_new.q_old
  int64_t pqo_stride;
  // derived r (KIND 5, the CG prologue of KIND 3 without r in memory): r_{j-1}
  // = X - sc->beta_p pprev (X = p_{j-1}, pprev = p_{j-2}) unless sc->rstored
  // (then read from r); r is never stored
  const double* pprev;
  // Lanczos prologue (KIND 4): X holds u_prev, r the Lanczos vector u, q_old
  // the previous matvec output Y; the operand is w = cy Y + cu u + cp u_prev
  // (coef = [cy, cu, cp] on the device), stored over u_prev (p_out == X,
  // element-wise in place), |w|^2 partials to rr_part
  const double* coef;
  // side job (KIND 2): x += c0 p0 + c1 p1 over [soff, soff + sn) (half 0) or
  // [soff_h1, soff_h1 + sn_h1) (half 1); each strip slot takes sstep elements
  double* sx;
  int64_t soff, sn, soff_h1, sn_h1, sstep;
};

template <int JT, bool T4, int KIND>
__global__ __launch_bounds__(64 * kBlkModeWaves, 1) void blk_mode_kernel(ModeArgs a) {
  constexpr int W = kBlkModeWaves;
  constexpr int TF = T4 ? JT - 1 : JT;   // full 16-row tiles
  constexpr int kDepth = 8;              // k-steps in flight per wave
  constexpr int NV = (KIND == 1 || KIND == 4) ? 3 : 1;  // streams per element
  constexpr int kSD = 2;                 // side-job k-steps in flight
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (a.skip != nullptr && *a.skip) return;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n16 = lane & 15, kq = lane >> 4;
  const int64_t g0 = (int64_t)blockIdx.x * a.per_wg;
  const int64_t g1 = min(a.ngroups, g0 + a.per_wg);
  const int KS = a.KS;
  const int64_t cpr = a.inner >> 4;   // strips per row of the axis
  // lane byte offset of element (row kq, column n16) from a strip's row 4 s
  uint32_t o_e = (uint32_t)(((int64_t)kq * a.inner + n16) * 8);
  asm volatile("" : "+v"(o_e));
  const int64_t rstep = a.inner * 32;   // bytes from k-step s to s + 1

  // a strip cursor: group g -> (block B, local group lg, outer o, column
  // strip cs); advanced one group at a time without divisions
  struct Cur {
    int64_t B, lg, o, cs;
  };
  auto cur_at = [&](int64_t g) {
    Cur c;
    c.B = g / a.gpb;
    c.lg = g - c.B * a.gpb;
    const int64_t ls = c.lg * W + wave;
    c.o = ls / cpr;
    c.cs = ls - c.o * cpr;
    return c;
  };
  auto cur_next = [&](Cur& c) {
    if (++c.lg == a.gpb) {
      c.lg = 0;
      ++c.B;
      c.o = 0;
      c.cs = wave;   // W < cpr (inner >= 400)
    } else {
      c.cs += W;
      if (c.cs >= cpr) {
        c.cs -= cpr;
        ++c.o;
      }
    }
  };
  // element offset of the strip (row 0, column 0); a strip past the block's
  // last one (a partial last group) reads the last valid strip, never stored
  auto cur_base = [&](const Cur& c) -> int64_t {
    int64_t o = c.o, cs = c.cs;
    if (c.lg * W + wave >= a.spb) {
      o = (a.spb - 1) / cpr;
      cs = (a.spb - 1) - o * cpr;
    }
    return c.B * a.nb + o * (int64_t)a.h * a.inner + (cs << 4);
  };
  auto cur_valid = [&](const Cur& c) -> bool { return c.lg * W + wave < a.spb; };

  // CG prologue state
  bool first = false, pending = false, pqo_on = false;
  double beta = 0.0, alpha = 0.0, rr_acc = 0.0, pqo_acc = 0.0;
  if (KIND == 1) {
    first = a.sc->first != 0;
    beta = a.sc->beta;
    pending = a.sc->pending != 0;
    alpha = a.sc->alpha;
    pqo_on = a.pqo_stride > 0 && !first;
  }
  double lz_cy = 0.0, lz_cu = 0.0, lz_cp = 0.0;
  if (KIND == 4) {
    lz_cy = a.coef[0];
    lz_cu = a.coef[1];
    lz_cp = a.coef[2];
  }
  // side job state
  double sc0 = 0.0, sc1 = 0.0;
  const double* sp0 = nullptr;
  const double* sp1 = nullptr;
  double* sxo = nullptr;
  int64_t slen = 0;
  if (KIND == 2) {
    const int xh = a.sc->xh;
    if (xh < 2) {
      const int64_t off = xh ? a.soff_h1 : a.soff;
      slen = xh ? a.sn_h1 : a.sn;
      sc0 = a.sc->xc[0];
      sc1 = a.sc->xc[1];
      sp0 = a.sc->xp[0] + off;
      sp1 = a.sc->xp[1] + off;
      sxo = a.sx + off;
    }
  }

  bd4 acc[TF > 0 ? TF : 1];
  double acc4 = 0.0;
  auto zero = [&] {
#pragma unroll
    for (int t = 0; t < (TF > 0 ? TF : 1); ++t) acc[t] = bd4{0.0, 0.0, 0.0, 0.0};
    acc4 = 0.0;
  };

  // segments of groups whose blocks share the axis's parity: the factor
  // fragments are staged once per segment, the k-step pipeline runs inside
  int64_t sg0 = g0;
  while (sg0 < g1) {
    const int64_t B0 = sg0 / a.gpb + a.blk0;   // global block index
    const int par = (int)((B0 >> a.bitpos) & 1);
    // first (local) block of the next parity run
    const int64_t Bend = (((B0 >> a.bitpos) + 1) << a.bitpos) - a.blk0;
    const int64_t sg1 = min(g1, Bend * a.gpb);
    // stage the factor (every wave done with the previous one)
    __syncthreads();
    {
      const double* src = par ? a.fT : a.fS;
      const int nd = KS * JT * 64;
      for (int i = threadIdx.x * 2; i < nd; i += 64 * W * 2)
        *reinterpret_cast<double2*>(lds + i) = *reinterpret_cast<const double2*>(src + i);
    }
    __syncthreads();

    const int64_t nsteps = (sg1 - sg0) * KS;
    // load cursor
    Cur lc = cur_at(sg0);
    int ld_s = 0;
    int64_t ld_n = 0;   // steps issued
    double ring[kDepth][NV];
    auto issue = [&](int slot) {
      const int64_t base = cur_base(lc);
      // rows past h (a partial last k-step) read row 0: zeroed when consumed
      const bool in = 4 * ld_s + kq < a.h;
      const int64_t ub = base * 8 + (int64_t)ld_s * rstep;
      const int64_t ubr = in ? ub : base * 8;
      const uint32_t vo = in ? o_e : (uint32_t)(n16 * 8);
      ring[slot][0] = ldu(a.X, ubr, vo);
      if (KIND == 1 || KIND == 4) {
        ring[slot][1] = ldu(a.r, ubr, vo);
        ring[slot][2] = ldu(a.q_old, ubr, vo);
      }
      ++ld_n;
      if (++ld_s == KS) {
        ld_s = 0;
        cur_next(lc);
      }
    };
    // side ring: slot q = g W + wave owns [q sstep, (q + 1) sstep) of the
    // half; k-step s of the strip carries the double2 at q sstep + 128 s + 2 lane
    double2 sring[kSD][3];
    int64_t sl_g = sg0;
    int sl_s = 0;
    auto side_elem = [&](int64_t g, int s) -> int64_t {
      const int64_t q0 = (g * W + wave) * a.sstep;
      const int64_t e = q0 + 128 * (int64_t)s + 2 * lane;
      const int64_t hi = min(slen, q0 + a.sstep);
      return (e + 1 < hi) ? e : -1;
    };
    auto side_issue = [&](int slot) {
      const int64_t e = (KIND == 2 && slen > 0 && sl_g < sg1) ? side_elem(sl_g, sl_s) : -1;
      if (e >= 0) {
        sring[slot][0] = *reinterpret_cast<const double2*>(sxo + e);
        sring[slot][1] = *reinterpret_cast<const double2*>(sp0 + e);
        sring[slot][2] = *reinterpret_cast<const double2*>(sp1 + e);
      }
      if (++sl_s == KS) {
        sl_s = 0;
        ++sl_g;
      }
    };

#pragma unroll
    for (int u = 0; u < kDepth; ++u)
      if ((int64_t)u < nsteps) issue(u);
    if (KIND == 2) {
#pragma unroll
      for (int u = 0; u < kSD; ++u) side_issue(u);
    }
    zero();
    Cur cc = cur_at(sg0);   // consume cursor
    int cs_s = 0;
    int64_t cs_g = sg0;
    int64_t cs_base = cur_base(cc);
    bool cs_valid = cur_valid(cc);

    for (int64_t c0 = 0; c0 < nsteps; c0 += kDepth) {
#pragma unroll
      for (int u = 0; u < kDepth; ++u) {
        if (c0 + u < nsteps) {
          // B operand of k-step cs_s
          const int i = 4 * cs_s + kq;
          double xb = i < a.h ? ring[u][0] : 0.0;
          if (KIND == 1) {
            const bool ok = cs_valid && i < a.h;
            double r = i < a.h ? ring[u][1] : 0.0;
            const double q = i < a.h ? ring[u][2] : 0.0;
            const int64_t ub = (cs_base + (int64_t)4 * cs_s * a.inner) * 8;
            if (pending) {
              r = r - alpha * q;
              if (ok) {
                stu(a.r, ub, o_e, r);
                rr_acc = fma(r, r, rr_acc);
              }
            }
            xb = first ? r : fma(beta, xb, r);
            if (ok) {
              stu(a.p_out, ub, o_e, xb);
              if (pqo_on) pqo_acc = fma(xb, q, pqo_acc);
            }
            if (!(i < a.h)) xb = 0.0;
          }
          if (KIND == 4) {
            const bool ok = cs_valid && i < a.h;
            const double uv = i < a.h ? ring[u][1] : 0.0;
            const double yv = i < a.h ? ring[u][2] : 0.0;
            xb = fma(lz_cp, xb, fma(lz_cu, uv, lz_cy * yv));   // lz_update_kernel's expression
            if (ok) {
              stu(a.p_out, (cs_base + (int64_t)4 * cs_s * a.inner) * 8, o_e, xb);
              rr_acc = fma(xb, xb, rr_acc);
            }
            if (!(i < a.h)) xb = 0.0;
          }
          const double* fs = lds + ((int64_t)cs_s * JT) * 64 + lane;
#pragma unroll
          for (int t = 0; t < TF; ++t)
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fs[t * 64], xb, acc[t], 0, 0, 0);
          if (T4) acc4 = __builtin_amdgcn_mfma_f64_4x4x4f64(fs[TF * 64], xb, acc4, 0, 0, 0);
          if (ld_n < nsteps) issue(u);
          if (KIND == 2) {
            // the side element of this k-step (loaded kSD steps ago; c0 is a
            // multiple of kDepth, so the slot is u mod kSD)
            const int64_t e = slen > 0 ? side_elem(cs_g, cs_s) : -1;
            const double2 xv = sring[u & 1][0], p0 = sring[u & 1][1], p1 = sring[u & 1][2];
            if (e >= 0) {
              double2 o;
              o.x = xv.x + (sc0 * p0.x + sc1 * p1.x);   // mp_side_job's expression
              o.y = xv.y + (sc0 * p0.y + sc1 * p1.y);
              *reinterpret_cast<double2*>(sxo + e) = o;
            }
            side_issue(u & 1);
          }
          if (++cs_s == KS) {
            // epilogue: D tile t lane 16 g + n elem r -> row 16 t + 4 r + g;
            // the 4x4 tail lane 16 r + n -> row 16 TF + r (column c0 + n)
            if (cs_valid) {
#pragma unroll
              for (int t = 0; t < TF; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  // with a 4x4 tail every full tile is inside h; without,
                  // the last tile may be padded
                  if (T4 || 16 * t + 4 * r + kq < a.h)
                    stu(a.Y, (cs_base + (int64_t)(16 * t + 4 * r) * a.inner) * 8, o_e,
                        acc[t][r]);
                }
              if (T4 && 16 * TF + kq < a.h)
                stu(a.Y, (cs_base + (int64_t)16 * TF * a.inner) * 8, o_e, acc4);
            }
            zero();
            cs_s = 0;
            ++cs_g;
            cur_next(cc);
            cs_base = cur_base(cc);
            cs_valid = cur_valid(cc);
          }
        }
      }
    }
    sg0 = sg1;
  }
  if (KIND == 1 || KIND == 4) {
    __shared__ double red[2 * kBlkModeWaves];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      rr_acc += __shfl_xor(rr_acc, off, 64);
      pqo_acc += __shfl_xor(pqo_acc, off, 64);
    }
    if (lane == 0) {
      red[wave] = rr_acc;
      red[W + wave] = pqo_acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < W; ++w) {
        s0 += red[w];
        s1 += red[W + w];
      }
      if (a.rr_part != nullptr) {
        a.rr_part[blockIdx.x] = s0;
        if (a.pqo_stride > 0) a.rr_part[a.pqo_stride + blockIdx.x] = s1;
      }
    }
  }
}

// The production shape of blk_mode_kernel: h = 16 TF + 4 (KS = 4 TF + 1
// k-steps, a 4-row tail), every memory operation unconditional so that the
// compiler's wait counting stays exact across the whole stream (a wave-uniform
// branch around a store or load makes it fall back to vmcnt(0) at the next
// merge): strips past a block's end read a valid strip and store to a trash
// slot, the prologue always stores r (unchanged when nothing is pending), the
// side job's spare lanes store to the trash slot.  The k-step ring is kD =
// KS mod-free deep (kD divides KS), so a step's slot is compile-time across
// strips.  Work split, LDS fragments and fusions as blk_mode_kernel.
__device__ __attribute__((aligned(16))) double g_blk_trash[6 * 64];

// waves per workgroup of the fast kernel: 12 (3 per SIMD) for the plain
// launch, 8 (2 per SIMD, 256 registers) for the fused ones
// (KIND 3: the prologue, KIND 1, with its r / q_old / p_old loads and r /
// p_new stores non-temporal -- Y, read by the next launch, stays normal)
template <int KIND>
constexpr int fast_waves() {
  return KIND == 0 ? 12 : 8;
}

template <int TF, int KIND_>
__global__ __launch_bounds__(64 * fast_waves<KIND_>(), 1) void blk_mode_fast_kernel(ModeArgs a) {
  constexpr bool NT = KIND_ >= 3;   // KIND 4 (Lanczos), 5 (derived r): non-temporal too
  constexpr bool RDER = KIND_ == 5;
  constexpr int KIND = (KIND_ == 3 || KIND_ == 5) ? 1 : KIND_;
  constexpr int W = fast_waves<KIND>();
  constexpr int JT = TF + 1;
  constexpr int KS = 4 * TF + 1;
  constexpr int kD = KIND == 0 ? KS : (KS % 5 == 0) ? 5 : (KS % 3 == 0) ? 3 : KS;   // ring depth, divides KS
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (a.skip != nullptr && *a.skip) return;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n16 = lane & 15, kq = lane >> 4;
  const int64_t g0 = (int64_t)blockIdx.x * a.per_wg;
  const int64_t g1 = min(a.ngroups, g0 + a.per_wg);
  const int64_t cpr = a.inner >> 4;
  uint32_t o_e = (uint32_t)(((int64_t)kq * a.inner + n16) * 8);
  asm volatile("" : "+v"(o_e));
  const int64_t rstep = a.inner * 32;
  double* trash = g_blk_trash + 2 * lane;   // 16 bytes per lane: spare stores land here
  // a store whose wave-uniform `valid` sends it to the trash slot instead:
  // one store instruction either way (the wait counts stay fixed)
  const uint32_t o_t = (uint32_t)(lane * 16);
  auto stq = [&](bool valid, void* p, int64_t uoff, uint32_t voff, double v) {
    void* bp = valid ? p : static_cast<void*>(g_blk_trash);
    stu(bp, valid ? uoff : 0, valid ? voff : o_t, v);
  };
  auto stq_nt = [&](bool valid, void* p, int64_t uoff, uint32_t voff, double v) {
    void* bp = valid ? p : static_cast<void*>(g_blk_trash);
    stuq<NT>(bp, valid ? uoff : 0, valid ? voff : o_t, v);
  };

  struct Cur {
    int64_t B, lg, o, cs;
  };
  auto cur_at = [&](int64_t g) {
    Cur c;
    c.B = g / a.gpb;
    c.lg = g - c.B * a.gpb;
    const int64_t ls = c.lg * W + wave;
    c.o = ls / cpr;
    c.cs = ls - c.o * cpr;
    return c;
  };
  auto cur_next = [&](Cur& c) {
    if (++c.lg == a.gpb) {
      c.lg = 0;
      ++c.B;
      c.o = 0;
      c.cs = wave;
    } else {
      c.cs += W;
      if (c.cs >= cpr) {
        c.cs -= cpr;
        ++c.o;
      }
    }
  };
  // a strip past the block's last one reads the last valid strip
  auto cur_base = [&](const Cur& c) -> int64_t {
    int64_t o = c.o, cs = c.cs;
    if (c.lg * W + wave >= a.spb) {
      o = (a.spb - 1) / cpr;
      cs = (a.spb - 1) - o * cpr;
    }
    return uni64(c.B * a.nb + o * (int64_t)a.h * a.inner + (cs << 4));
  };
  auto cur_valid = [&](const Cur& c) -> bool {
    return __builtin_amdgcn_readfirstlane((int)(c.lg * W + wave < a.spb)) != 0;
  };

  bool first = false, pqo_on = false;
  double beta = 0.0, alpha = 0.0, rr_acc = 0.0, pqo_acc = 0.0;
  if (KIND == 1) {
    first = a.sc->first != 0;
    beta = a.sc->beta;
    alpha = a.sc->pending != 0 ? a.sc->alpha : 0.0;   // not pending: r stays r
    pqo_on = a.pqo_stride > 0 && !first;
  }
  double lz_cy = 0.0, lz_cu = 0.0, lz_cp = 0.0;
  if (KIND == 4) {
    lz_cy = a.coef[0];
    lz_cu = a.coef[1];
    lz_cp = a.coef[2];
  }
  const bool pending = KIND == 1 && a.sc->pending != 0;
  // derived r: the second stream is r (stored) or p_{j-2}
  const bool rst = !RDER || a.sc->rstored != 0;
  const double bprev = RDER ? a.sc->beta_p : 0.0;
  const double* rsrc = (KIND == 1 && !rst) ? a.pprev : a.r;
  double sc0 = 0.0, sc1 = 0.0;
  const double* sp0 = a.sx;
  const double* sp1 = a.sx;
  double* sxo = a.sx;
  int64_t slen = 0;
  if (KIND == 2) {
    const int xh = a.sc->xh;
    if (xh < 2) {
      const int64_t off = xh ? a.soff_h1 : a.soff;
      slen = xh ? a.sn_h1 : a.sn;
      sc0 = a.sc->xc[0];
      sc1 = a.sc->xc[1];
      sp0 = a.sc->xp[0] + off;
      sp1 = a.sc->xp[1] + off;
      sxo = a.sx + off;
    }
  }
  // side element of (group g, step s): a valid even index (clamped) and
  // whether this lane owns it
  auto side_at = [&](int64_t g, int s, bool& own) -> int64_t {
    const int64_t q0 = (g * W + wave) * a.sstep;
    const int64_t e = q0 + 128 * (int64_t)s + 2 * lane;
    const int64_t hi = min(slen, q0 + a.sstep);
    own = e + 1 < hi;
    return own ? e : 0;
  };

  int64_t sg0 = g0;
  while (sg0 < g1) {
    const int64_t B0 = sg0 / a.gpb + a.blk0;   // global block index
    const int par = (int)((B0 >> a.bitpos) & 1);
    const int64_t Bend = (((B0 >> a.bitpos) + 1) << a.bitpos) - a.blk0;
    const int64_t sg1 = min(g1, Bend * a.gpb);
    __syncthreads();
    {
      const double* src = par ? a.fT : a.fS;
      constexpr int nd = KS * JT * 64;
      for (int i = threadIdx.x * 2; i < nd; i += 64 * W * 2)
        *reinterpret_cast<double2*>(lds + i) = *reinterpret_cast<const double2*>(src + i);
    }
    __syncthreads();

    // load cursor: strip lc, its base; past the segment the last strip again
    Cur lc = cur_at(sg0);
    int64_t lg_n = sg0;
    int64_t l_base = cur_base(lc);
    double ring[kD][3];
    double2 sring[kD][3];
    auto issue = [&](int slot, int s) {
      // k-step s of the load cursor's strip (s compile-time)
      const int64_t ub = l_base * 8 + (int64_t)s * rstep;
      ring[slot][0] = lduq<NT>(a.X, ub, o_e);
      if (KIND == 1 || KIND == 4) {
        ring[slot][1] = lduq<NT>(KIND == 1 ? rsrc : a.r, ub, o_e);
        ring[slot][2] = lduq<NT>(a.q_old, ub, o_e);
      }
      if (KIND == 2) {
        bool own;
        const int64_t e = side_at(lg_n < sg1 ? lg_n : sg1 - 1, s, own);
        sring[slot][0] = ld2g(sxo + e);
        sring[slot][1] = ld2g(sp0 + e);
        sring[slot][2] = ld2g(sp1 + e);
      }
    };
    auto load_next_strip = [&] {
      if (lg_n + 1 < sg1) {
        cur_next(lc);
        l_base = cur_base(lc);
      }
      ++lg_n;
    };
#pragma unroll
    for (int u = 0; u < kD; ++u) issue(u, u);

    Cur cc = cur_at(sg0);
#pragma unroll 1
    for (int64_t g = sg0; g < sg1; ++g) {
      const int64_t cbase = cur_base(cc);
      const bool cvalid = cur_valid(cc);
      // the fragments' LDS offset, opaque per strip: the reads are not loop
      // invariant (hoisted, 175 of them would not fit the registers)
      uint32_t lo = (uint32_t)(lane * 8);
      asm volatile("" : "+v"(lo));
      const char* lb = reinterpret_cast<const char*>(lds) + lo;
      bd4 acc[TF];
      double acc4 = 0.0;
#pragma unroll
      for (int t = 0; t < TF; ++t) acc[t] = bd4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int slot = s % kD;
        // h = 16 TF + 4: every row 4 s + kq of the strip is inside h
        double xb = ring[slot][0];
        if (KIND == 1) {
          // derived: r_{j-1} = p_{j-1} - beta_p p_{j-2} (a select, not a
          // multiply: the stored r needs no p_{j-1})
          double r = rst ? ring[slot][1] : fma(-bprev, ring[slot][1], xb);
          const double q = ring[slot][2];
          const int64_t ub = (cbase + (int64_t)4 * s * a.inner) * 8;
          r = r - alpha * q;
          const double rr = fma(r, r, rr_acc);
          xb = first ? r : fma(beta, xb, r);
          const double pqo = fma(xb, q, pqo_acc);
          if (cvalid) {   // wave-uniform
            if (pending) rr_acc = rr;
            if (pqo_on) pqo_acc = pqo;
          }
          // stores unconditional: a spare strip's go to the trash slot
          // (derived r: no r store -- 5 passes instead of 6)
          if (!RDER) stq_nt(cvalid, a.r, ub, o_e, r);
          stq_nt(cvalid, a.p_out, ub, o_e, xb);
        }
        if (KIND == 4) {
          const int64_t ub = (cbase + (int64_t)4 * s * a.inner) * 8;
          xb = fma(lz_cp, xb, fma(lz_cu, ring[slot][1], lz_cy * ring[slot][2]));
          const double rr = fma(xb, xb, rr_acc);
          if (cvalid) rr_acc = rr;   // wave-uniform
          // over u_prev (X) at the position this wave just read; a spare
          // strip's (which re-read the last valid strip) to the trash slot
          stq_nt(cvalid, a.p_out, ub, o_e, xb);
        }
        const double* fs = reinterpret_cast<const double*>(lb + (s * JT) * 512);
#pragma unroll
        for (int t = 0; t < TF; ++t)
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(fs[t * 64], xb, acc[t], 0, 0, 0);
        acc4 = __builtin_amdgcn_mfma_f64_4x4x4f64(fs[TF * 64], xb, acc4, 0, 0, 0);
        if (KIND == 2) {
          bool own;
          const int64_t e = side_at(g, s, own);
          const double2 xv = sring[slot][0], p0 = sring[slot][1], p1 = sring[slot][2];
          double2 o;
          o.x = xv.x + (sc0 * p0.x + sc1 * p1.x);   // mp_side_job's expression
          o.y = xv.y + (sc0 * p0.y + sc1 * p1.y);
          st2g(own ? sxo + e : trash, o);
        }
        // refill this slot with the step kD ahead (the next strip's when
        // it wraps)
        if (s + kD < KS) {
          issue(slot, s + kD);
        } else {
          if (s + kD == KS) load_next_strip();
          issue(slot, s + kD - KS);
        }
        __builtin_amdgcn_sched_barrier(0);   // one k-step per scheduling region
      }
      // epilogue: tile t lane 16 g + n elem r -> row 16 t + 4 r + g; the tail
      // lane 16 r + n -> row 16 TF + r (column c0 + n); spare strips to trash
#pragma unroll
      for (int t = 0; t < TF; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          stq(cvalid, a.Y, (cbase + (int64_t)(16 * t + 4 * r) * a.inner) * 8, o_e, acc[t][r]);
      stq(cvalid, a.Y, (cbase + (int64_t)16 * TF * a.inner) * 8, o_e, acc4);
      cur_next(cc);
    }
    sg0 = sg1;
  }
  if (KIND == 1 || KIND == 4) {
    __shared__ double red[2 * W];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      rr_acc += __shfl_xor(rr_acc, off, 64);
      pqo_acc += __shfl_xor(pqo_acc, off, 64);
    }
    if (lane == 0) {
      red[wave] = rr_acc;
      red[W + wave] = pqo_acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < W; ++w) {
        s0 += red[w];
        s1 += red[W + w];
      }
      if (a.rr_part != nullptr) {
        a.rr_part[blockIdx.x] = s0;
        if (a.pqo_stride > 0) a.rr_part[a.pqo_stride + blockIdx.x] = s1;
      }
    }
  }
}

// ------------------------------------------------------- pair (slab) kernel
// Axes d-2 and d-1 of every block together: slab s (h x h, contiguous) ->
// Z = F2 X F3^T, F2 = F_{d-2}^{beta}, F3 = F_{d-1}^{beta}.  h = 16 TF + 4.
//
// Two waves per slab, each owning a set of output columns j: role 0 the full
// 16-column tiles [0, JA) and the 4-column tail, role 1 the tiles [JA, TF).
// GEMM 1, W[a][j] = sum_c X[a][c] F3[j][c] for the role's columns j and all
// rows a: A = X rows (lane l: X[16 t + (l & 15)][4 s + (l >> 4)]; the 4-row
// tail with its rows replicated over the 4x4 blocks), B = F3 fragments; W
// stays in registers.  GEMM 2, Z[i][j] = sum_a F2[i][a] W[a][j]: a W tile's
// accumulator IS the B operand of k-step s = 4 t_a + r (element r of lane
// 16 g + n holds W[16 t_a + 4 r + g][16 t_j + n]), A = F2 fragments, one
// 16-row strip of Z at a time.  The 4-column tail of W (lane 16 r + 4 g + c:
// W[16 t_a + 4 g + r][16 TF + c]) becomes the tail's B operand by a 4-lane
// group broadcast inside each 16-lane row (ds_swizzle).  Roles alternate per
// slab so each wave averages the two.  Epilogue: Z (+ shift p, p.q and q.q
// partials) straight from the accumulators.  Not in place (the two roles
// read X while the other stores Z).
struct PairArgs {
  const double* X;
  double* Y;
  const double* f3S;   // F_{d-1} fragments [KS][TF+1][64]
  const double* f3T;
  const double* f2S;   // F_{d-2} fragments [KS][TF+1][64]
  const double* f2T;
  int64_t nslab;       // slabs of the vector (its blocks x slabs per block)
  int64_t spb;         // slabs per block
  int64_t blk0;        // global index of the vector's first block (parity bits)
  const double* P;     // epilogue: q = Z + shift * P, partials (nullptr: plain)
  double shift;
  double* partials;    // [grid] p.q, [pstride + grid] r.q (0), [2 pstride + grid] q.q
  int64_t pstride;
  const int* skip;
  // the fused CG's balanced x side job (blk_pair_lds_kernel, SIDE): x += c0 p0
  // + c1 p1 over half sc->xh of x -- [soff, soff + sn) or [soff_h1, soff_h1 +
  // sn_h1); each wave slot (unit * waves + wave) takes sstep elements
  const CgScalars* sc;
  double* sx;
  int64_t soff, sn, soff_h1, sn_h1, sstep;
  // x_defer mode 3 (SIDE bit 4): the armed region sc->sreg of length sreg_len
  // (sn = the vector's length) gets x += sum_t sc->scoef[t] sc->sdir[t]
  int64_t sreg_len;
};

// swizzle a double within 32-lane groups: lane (b4 b3 b2 b1 b0) reads lane
// (b4, R1 R0, b1 b0) -- the 4-lane group R of its 16-lane row
template <int R>
__device__ __forceinline__ double bcast_group(double v) {
  constexpr int pat = (R << 7) | 0x13;   // bitmask mode: and 0x13, or R << 2, xor 0
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
  return __hiloint2double(hi, lo);
}

// GEMM 2 and the epilogue of one slab (both pair kernels): Z = F2 W from the
// role's W accumulators, q = Z (+ shift p, the p.q / q.q partials) stored.
template <int TF, int J0, int NJ, bool TJ, int EPI = -1, int PF = 4, bool NT = false>
__device__ __forceinline__ void pair_gemm2(const PairArgs& A, int64_t sbyte, const double* f2,
                                           const bd4 (&W)[TF][NJ > 0 ? NJ : 1],
                                           const double (&Wta)[NJ > 0 ? NJ : 1],
                                           const double (&Wj)[TF], const double Wc, double& pq,
                                           double& qq) {
  constexpr int H = 16 * TF + 4;
  constexpr int KS = 4 * TF + 1;
  constexpr int64_t FS = (int64_t)(TF + 1) * 64 * 8;   // bytes per fragment k-step
  const int lane = threadIdx.x & 63;
  const int n16 = lane & 15, kq = lane >> 4, l3 = lane & 3, b4 = (lane >> 2) & 3;
  uint32_t o_f = (uint32_t)(lane * 8);                  // fragments
  // Z in the k-step tiled slab (element (i, a) at (a >> 2) 4 H + 4 i + (a & 3)):
  // zb(i0, a0) the byte offset of the 4-row, 16-column (or 16-row, 4-column)
  // group at row i0, column a0 (multiples of 4); lanes add
  //   o_z:  row + kq, column + n16 (the full tiles, the tail rows' 4x4 blocks)
  //   o_zt: row + 4 b4 + kq, column + l3 (the tail columns, the corner)
  // -- every wave store / load covers whole 128-B lines
  uint32_t o_z = (uint32_t)(((n16 >> 2) * 4 * H + 4 * kq + (n16 & 3)) * 8);
  uint32_t o_zt = (uint32_t)((16 * b4 + 4 * kq + l3) * 8);
  asm volatile("" : "+v"(o_f), "+v"(o_z), "+v"(o_zt));
  auto zb = [&](int i0, int a0) -> int64_t { return sbyte + ((int64_t)a0 * H + 4 * i0) * 8; };
  // one 16-row strip t_i at a time
  const bool epi = EPI < 0 ? A.P != nullptr : EPI != 0;
  const double sh = A.shift;
  // k-step s: B operands from the accumulators
  auto bfull = [&](int s, int u) -> double {
    return s < 4 * TF ? W[s >> 2][u][s & 3] : Wta[u];
  };
  auto btail = [&](int s) -> double {
    if (s >= 4 * TF) return Wc;
    switch (s & 3) {
      case 0: return bcast_group<0>(Wj[s >> 2]);
      case 1: return bcast_group<1>(Wj[s >> 2]);
      case 2: return bcast_group<2>(Wj[s >> 2]);
      default: return bcast_group<3>(Wj[s >> 2]);
    }
  };
  // one output element: q = Z (+ shift p, dots)
  auto put = [&](int64_t ub, uint32_t vo, double z, double p) {
    double q = z;
    if (epi) {
      q = fma(sh, p, q);
      pq = fma(p, q, pq);
      qq = fma(q, q, qq);
    }
    stuq<NT>(A.Y, ub, vo, q);
  };
#pragma unroll 1
  for (int ti = 0; ti < TF; ++ti) {
    bd4 Z[NJ > 0 ? NJ : 1];
    double Zt = 0.0;
#pragma unroll
    for (int u = 0; u < NJ; ++u) Z[u] = bd4{0.0, 0.0, 0.0, 0.0};
    // epilogue operands issued now, consumed after the k-loop (issuing them
    // behind the first kPF fragments, so the first k-steps' waits do not
    // cover them, measured slower: +0.3 ms per pair launch, profiles/r05/zc_pv_order)
    double pv[NJ > 0 ? NJ : 1][4], pvt = 0.0;
    if (epi) {
#pragma unroll
      for (int u = 0; u < NJ; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pv[u][r] = lduq<NT>(A.P, zb(16 * ti + 4 * r, 16 * (J0 + u)), o_z);
      if (TJ) pvt = lduq<NT>(A.P, zb(16 * ti, 16 * TF), o_zt);
    }
    const int64_t fti = (int64_t)ti * 512;
    // A fragments kPF k-steps ahead; the scheduling barriers keep each step's
    // loads / MFMAs in place
    constexpr int kPF = PF;
    double fr[kPF];
#pragma unroll
    for (int s = 0; s < kPF; ++s) fr[s] = ldu(f2, fti + s * FS, o_f);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const double f = fr[s % kPF];
      if (s + kPF < KS) fr[s % kPF] = ldu(f2, fti + (s + kPF) * FS, o_f);
#pragma unroll
      for (int u = 0; u < NJ; ++u)
        Z[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(f, bfull(s, u), Z[u], 0, 0, 0);
      if (TJ) Zt = __builtin_amdgcn_mfma_f64_4x4x4f64(f, btail(s), Zt, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // Z[u] lane 16 g + n elem r -> row 16 ti + 4 r + g, column 16 (J0 + u) + n;
    // Zt lane 16 r + 4 b + c -> row 16 ti + 4 b + r, column 16 TF + c
#pragma unroll
    for (int u = 0; u < NJ; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        put(zb(16 * ti + 4 * r, 16 * (J0 + u)), o_z, Z[u][r], epi ? pv[u][r] : 0.0);
    if (TJ) put(zb(16 * ti, 16 * TF), o_zt, Zt, pvt);
  }
  // tail rows i = 16 TF + r: A = F2's replicated tail fragment; the outputs of
  // v_mfma_f64_4x4x4_4b_f64: lane 16 r + 4 b + c -> row 16 TF + r, column
  // 16 (J0 + u) + 4 b + c; the corner (TJ) is replicated over b (b = 0 stores)
  {
    double Z4[NJ > 0 ? NJ : 1], Z4t = 0.0;
#pragma unroll
    for (int u = 0; u < NJ; ++u) Z4[u] = 0.0;
    const int64_t fti = (int64_t)TF * 512;
    constexpr int kPF = PF;
    double fr[kPF];
#pragma unroll
    for (int s = 0; s < kPF; ++s) fr[s] = ldu(f2, fti + s * FS, o_f);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const double f = fr[s % kPF];
      if (s + kPF < KS) fr[s % kPF] = ldu(f2, fti + (s + kPF) * FS, o_f);
#pragma unroll
      for (int u = 0; u < NJ; ++u)
        Z4[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(f, bfull(s, u), Z4[u], 0, 0, 0);
      if (TJ) Z4t = __builtin_amdgcn_mfma_f64_4x4x4f64(f, btail(s), Z4t, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < NJ; ++u) {
      const int64_t ub = zb(16 * TF, 16 * (J0 + u));
      put(ub, o_z, Z4[u], epi ? lduq<NT>(A.P, ub, o_z) : 0.0);
    }
    if (TJ && b4 == 0) {
      // lane 16 r + c (b = 0): row 16 TF + r, column 16 TF + c
      const int64_t ub = zb(16 * TF, 16 * TF);
      put(ub, o_zt, Z4t, epi ? lduq<NT>(A.P, ub, o_zt) : 0.0);
    }
  }
}

template <int TF, int J0, int NJ, bool TJ>
__device__ __forceinline__ void pair_slab(const PairArgs& A, int64_t slab, double& pq,
                                          double& qq, float& junk) {
  constexpr int H = 16 * TF + 4;
  constexpr int KS = 4 * TF + 1;
  constexpr int NJB = NJ + (TJ ? 1 : 0);   // B fragments per k-step
  constexpr int64_t FS = (int64_t)(TF + 1) * 64 * 8;   // bytes per fragment k-step
  const int lane = threadIdx.x & 63;
  const int n16 = lane & 15, kq = lane >> 4, l3 = lane & 3;
  // lane byte offsets (opaque: recomputed per slab, never hoisted as a set;
  // GEMM 2's own in pair_gemm2)
  uint32_t o_x = (uint32_t)((n16 * 4 + kq) * 8);        // X rows 16 t + n16, column 4 s + kq
  uint32_t o_xt = (uint32_t)((l3 * 4 + kq) * 8);        // X tail rows 16 TF + l3
  uint32_t o_f = (uint32_t)(lane * 8);                  // fragments
  asm volatile("" : "+v"(o_x), "+v"(o_xt), "+v"(o_f));
  const int64_t blk = slab / A.spb + A.blk0;
  const int par3 = (int)(blk & 1), par2 = (int)((blk >> 1) & 1);
  const double* f3 = par3 ? A.f3T : A.f3S;
  const double* f2 = par2 ? A.f2T : A.f2S;
  const int64_t sbyte = slab * (int64_t)H * H * 8;
  const int64_t xbyte = sbyte;

  // ---- GEMM 1: W = X F3^T (the role's columns)
  bd4 W[TF][NJ > 0 ? NJ : 1];
  double Wta[NJ > 0 ? NJ : 1];   // tail rows a = 16 TF .. +3, full column tiles
  double Wj[TF];                 // full row tiles, tail columns (TJ)
  double Wc = 0.0;               // corner (TJ)
#pragma unroll
  for (int t = 0; t < TF; ++t) {
#pragma unroll
    for (int u = 0; u < NJ; ++u) W[t][u] = bd4{0.0, 0.0, 0.0, 0.0};
    Wj[t] = 0.0;
  }
#pragma unroll
  for (int u = 0; u < NJ; ++u) Wta[u] = 0.0;

  auto ld1 = [&](int s, double (&xa)[TF + 1], double (&fb)[NJB > 0 ? NJB : 1]) {
    const int64_t xs = xbyte + (int64_t)s * H * 32;   // the k-step's h x 4 run
#pragma unroll
    for (int t = 0; t < TF; ++t) xa[t] = ldu(A.X, xs + (int64_t)t * 512, o_x);
    xa[TF] = ldu(A.X, xs + (int64_t)TF * 512, o_xt);
    const int64_t fs = (int64_t)s * FS;
#pragma unroll
    for (int u = 0; u < NJ; ++u) fb[u] = ldu(f3, fs + (int64_t)(J0 + u) * 512, o_f);
    if (TJ) fb[NJ] = ldu(f3, fs + (int64_t)TF * 512, o_f);
  };
  auto mm1 = [&](const double (&xa)[TF + 1], const double (&fb)[NJB > 0 ? NJB : 1]) {
#pragma unroll
    for (int t = 0; t < TF; ++t)
#pragma unroll
      for (int u = 0; u < NJ; ++u)
        W[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[t], fb[u], W[t][u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NJ; ++u)
      Wta[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[TF], fb[u], Wta[u], 0, 0, 0);
    if (TJ) {
#pragma unroll
      for (int t = 0; t < TF; ++t)
        Wj[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[t], fb[NJ], Wj[t], 0, 0, 0);
      Wc = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[TF], fb[NJ], Wc, 0, 0, 0);
    }
  };
  // L2 prefetch of X: one k-step of register prefetch does not cover an HBM
  // miss.  Every pair of k-steps touches the runs of k-steps s + 8 and s + 9
  // (one 4-byte load per 128-B line: KS lines per k-step); a touch's value is
  // folded into a junk sum two pairs later, so it never makes a k-step wait
  // (the sum is stored once per kernel)
  auto touch = [&](int s, float& t0, float& t1) {
    const int s0 = s + 8 < KS ? s + 8 : KS - 1, s1 = s + 9 < KS ? s + 9 : KS - 1;
    const int ln = lane < KS ? lane : KS - 1;
    t0 = *reinterpret_cast<const __attribute__((address_space(1))) float*>(
        reinterpret_cast<uintptr_t>(A.X) + xbyte + ((int64_t)s0 * H * 4 + 16 * ln) * 8);
    t1 = *reinterpret_cast<const __attribute__((address_space(1))) float*>(
        reinterpret_cast<uintptr_t>(A.X) + xbyte + ((int64_t)s1 * H * 4 + 16 * ln) * 8);
  };
  {
    double xa0[TF + 1], fb0[NJB > 0 ? NJB : 1], xa1[TF + 1], fb1[NJB > 0 ? NJB : 1];
    float ta0, ta1, tb0, tb1, tc0, tc1;
    touch(0, ta0, ta1);
    touch(4, tb0, tb1);
    ld1(0, xa0, fb0);
#pragma unroll 1
    for (int s = 0; s + 1 < KS; s += 2) {
      touch(s + 2, tc0, tc1);
      ld1(s + 1, xa1, fb1);
      mm1(xa0, fb0);
      if (s + 2 < KS) ld1(s + 2, xa0, fb0);
      mm1(xa1, fb1);
      junk += (ta0 + ta1) * 0.0f;   // the touch of two pairs ago
      ta0 = tb0;
      ta1 = tb1;
      tb0 = tc0;
      tb1 = tc1;
    }
    junk += (ta0 + ta1 + tb0 + tb1) * 0.0f;
    mm1(xa0, fb0);   // KS odd: the last k-step (loaded by the loop's last pass)
  }

  pair_gemm2<TF, J0, NJ, TJ>(A, sbyte, f2, W, Wta, Wj, Wc, pq, qq);
}

template <int TF, int JA>
__global__ __launch_bounds__(64 * kBlkPairWaves, 2) void blk_pair_kernel(PairArgs A) {
  if (A.skip != nullptr && *A.skip) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // wave pairs (2 w, 2 w + 1) share a slab; roles alternate per slab
  const int64_t npairs = (int64_t)gridDim.x * (kBlkPairWaves / 2);
  const int64_t pair = (int64_t)blockIdx.x * (kBlkPairWaves / 2) + (wave >> 1);
  double pq = 0.0, qq = 0.0;
  float junk = 0.0f;   // L2-prefetch touches (pair_slab)
  int it = 0;
  for (int64_t slab = pair; slab < A.nslab; slab += npairs, ++it) {
    const int role = ((wave & 1) + it) & 1;
    if (JA == TF) {
      // a single role (TF = 1): the second wave of the pair idles
      if ((wave & 1) == 0) pair_slab<TF, 0, JA, true>(A, slab, pq, qq, junk);
    } else if (role == 0) {
      pair_slab<TF, 0, JA, true>(A, slab, pq, qq, junk);
    } else {
      pair_slab<TF, JA, TF - JA, false>(A, slab, pq, qq, junk);
    }
  }
  // keep the touches alive: one store per lane to the junk slot
  reinterpret_cast<float*>(g_blk_trash)[lane] = junk;
  if (A.partials != nullptr) {
    __shared__ double red[2 * kBlkPairWaves];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      pq += __shfl_xor(pq, off, 64);
      qq += __shfl_xor(qq, off, 64);
    }
    if (lane == 0) {
      red[wave] = pq;
      red[kBlkPairWaves + wave] = qq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < kBlkPairWaves; ++w) {
        s0 += red[w];
        s1 += red[kBlkPairWaves + w];
      }
      A.partials[blockIdx.x] = s0;
      A.partials[A.pstride + blockIdx.x] = 0.0;
      A.partials[2 * A.pstride + blockIdx.x] = s1;
    }
  }
}

// ------------------------------------------- pair kernel, LDS-staged X ring
// The same slab product with GEMM 1's operands moving global -> LDS by
// LDS-DMA (global_load_lds_dwordx4) through a ring of NS stages shared by
// the two waves of a slab, instead of straight into registers: there
// (blk_pair_kernel) the register prefetch is one k-step deep -- W holds 164
// of the 256 registers -- and HBM latency stays exposed (MFMA busy ~0.60).
// Here NS - 1 k-steps stay in flight without registers, each X byte
// crosses L2 -> CU once per slab (both waves read the LDS copy), and the ring
// runs straight across slab boundaries (the next slab's first stages land
// while GEMM 2 of this one runs).
//
// Stage = one k-step s: [X image][F_{d-1} fragment image].  X image: 16-byte
// pieces (row, column pair c) of columns 4 s .. 4 s + 3, position
// 32 t + 16 c + r16 for row 16 t + r16 (XG row groups, rows past h re-read
// row h - 1): lane (n16, kq) reads piece c = kq >> 1, half kq & 1 with one
// ds_read_b64 per row tile (a 16-row tile is 512 contiguous bytes over the
// wave: conflict-free).  Fragment image: the k-step's JT fragments as packed
// (BlockOp::frag, padded to an even count).  Each stage is XI + FI 1-KiB DMAs,
// DPW per wave.
//
// GEMM 1 issues nothing but these DMAs, so the only vector-memory waits there
// are the counted ones: a wait on an ordinary load while an LDS-DMA younger
// than it is in flight is compiled as vmcnt(0) (the pending events are mixed),
// which is why the fragments ride in the ring too.  Per stage: s_waitcnt
// vmcnt((NS - 2) DPW) (this wave's DMAs of the stage landed), s_barrier
// (the partner's have, and both finished reading the previous stage), then
// the DMAs of stage + NS - 1 into the freed slot.  Past the workgroup's
// last slab the DMAs re-read its last stage, so the count holds everywhere.
// GEMM 2 keeps its ordinary loads (F_{d-2} fragments, p): its first wait
// drains the next slab's DMAs once per slab.
// ring stages: 4 (one slab per workgroup, 4 workgroups per CU) or 6 (two
// slabs of one block per workgroup sharing the fragment image, 2 per CU)
template <int SPW>
constexpr int pair_ns() {
  return SPW == 2 ? 6 : 4;
}

template <int N>
__device__ __forceinline__ void blk_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt holds 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int TF, int SPW>
struct PairRing {
  static constexpr int H = 16 * TF + 4;
  static constexpr int KS = 4 * TF + 1;     // stages per slab (k-steps)
  static constexpr int JT = TF + 1;         // fragments per k-step
  static constexpr int XG = ((TF + 1) + 1) / 2 * 2;   // row groups, even
  static constexpr int XI = XG / 2;         // X DMAs per slab and stage (1 KiB: 2 groups)
  static constexpr int FI = (JT + 1) / 2;   // fragment DMAs (1 KiB: 2 fragments)
  static constexpr int NW = 2 * SPW;        // waves per workgroup (two roles per slab)
  // DMAs per stage, padded to a multiple of the wave count (the pads re-read
  // the last fragment pair into its own place)
  static constexpr int TOT = (SPW * XI + FI + NW - 1) / NW * NW;
  static constexpr int DPW = TOT / NW;      // DMAs per wave per stage
  static constexpr int XD = XG * 64;        // doubles of one slab's X image
  static constexpr int FD = SPW * XD;       // the fragment image's offset
  static constexpr int STAGE = FD + 2 * FI * 64;   // doubles per stage
  static constexpr int NS = pair_ns<SPW>();
};

// where a slab's operands live: X byte offset, F_{d-1} fragments (parity)
struct PairSlabSrc {
  int64_t xoff;
  const double* f3;
};

template <int TF, int SPW, int EPI, int J0, int NJ, bool TJ, bool NT, typename Issue>
__device__ __forceinline__ void pair_slab_lds(const PairArgs& A, int64_t slab, int sl, int cslot,
                                              bool early, PairSlabSrc cur, PairSlabSrc nxt,
                                              bool nxt_valid, const double* ring, Issue&& issue,
                                              double& pq, double& qq) {
  typedef PairRing<TF, SPW> R;
  constexpr int KS = R::KS;
  constexpr int NS = R::NS;
  constexpr int NJB = NJ + (TJ ? 1 : 0);
  constexpr int Y = (NS - 2) * R::DPW;
  static_assert(Y <= 63, "ring too deep for the counted wait");
  const int lane = threadIdx.x & 63;
  const int n16 = lane & 15, kq = lane >> 4;
  // LDS byte offsets within a stage: X rows 16 t + n16 (piece kq >> 1, half
  // kq & 1), the tail rows 16 TF + (n16 & 3), the role's fragments
  uint32_t o_x = (uint32_t)((sl * R::XD + ((kq >> 1) * 16 + n16) * 2 + (kq & 1)) * 8);
  uint32_t o_xt = (uint32_t)((sl * R::XD + ((kq >> 1) * 16 + (n16 & 3)) * 2 + (kq & 1)) * 8);
  uint32_t o_f = (uint32_t)((R::FD + lane) * 8);
  asm volatile("" : "+v"(o_x), "+v"(o_xt), "+v"(o_f));
  const int64_t blk = slab / A.spb + A.blk0;
  const double* f2 = ((blk >> 1) & 1) ? A.f2T : A.f2S;
  const int64_t sbyte = slab * (int64_t)R::H * R::H * 8;

  bd4 W[TF][NJ > 0 ? NJ : 1];
  double Wta[NJ > 0 ? NJ : 1];
  double Wj[TF];
  double Wc = 0.0;
#pragma unroll
  for (int t = 0; t < TF; ++t) {
#pragma unroll
    for (int u = 0; u < NJ; ++u) W[t][u] = bd4{0.0, 0.0, 0.0, 0.0};
    Wj[t] = 0.0;
  }
#pragma unroll
  for (int u = 0; u < NJ; ++u) Wta[u] = 0.0;

  const char* rb = reinterpret_cast<const char*>(ring);   // __shared__: ds_read
  int slot = cslot;
#pragma unroll 1
  for (int s = 0; s < KS; ++s) {
    // the stage's DMAs landed (this wave's: counted; the partner's: barrier)
    if (early && s < NS - 1)
      blk_wait_vm<0>();   // the workgroup's first stages: fewer younger DMAs than Y
    else
      blk_wait_vm<Y>();
    __builtin_amdgcn_s_barrier();
    // stage s + NS - 1 (this slab's, else the next slab's; past the last
    // slab this one's last stage again) into the slot every wave is done with
    {
      const int sn = s + NS - 1;
      const bool in_next = sn >= KS;
      const PairSlabSrc src = in_next && nxt_valid ? nxt : cur;
      const int st = in_next ? (nxt_valid ? sn - KS : KS - 1) : sn;
      issue(src, st, slot == 0 ? NS - 1 : slot - 1);
    }
    const char* sb = rb + slot * (R::STAGE * 8);
    double xa[TF + 1], fb[NJB];
#pragma unroll
    for (int t = 0; t < TF; ++t) xa[t] = *reinterpret_cast<const double*>(sb + o_x + t * 512);
    xa[TF] = *reinterpret_cast<const double*>(sb + o_xt + TF * 512);
#pragma unroll
    for (int u = 0; u < NJ; ++u) fb[u] = *reinterpret_cast<const double*>(sb + o_f + (J0 + u) * 512);
    if (TJ) fb[NJ] = *reinterpret_cast<const double*>(sb + o_f + TF * 512);
#pragma unroll
    for (int t = 0; t < TF; ++t)
#pragma unroll
      for (int u = 0; u < NJ; ++u)
        W[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[t], fb[u], W[t][u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NJ; ++u)
      Wta[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[TF], fb[u], Wta[u], 0, 0, 0);
    if (TJ) {
#pragma unroll
      for (int t = 0; t < TF; ++t)
        Wj[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[t], fb[NJ], Wj[t], 0, 0, 0);
      Wc = __builtin_amdgcn_mfma_f64_4x4x4f64(xa[TF], fb[NJ], Wc, 0, 0, 0);
    }
    slot = slot + 1 == NS ? 0 : slot + 1;
  }
  pair_gemm2<TF, J0, NJ, TJ, EPI, 4, NT>(A, sbyte, f2, W, Wta, Wj, Wc, pq, qq);
}

// SPW slabs per workgroup (2 waves each; SPW = 2: slabs 2 u, 2 u + 1 of one
// block, so one fragment image serves both -- the host requires an even
// slab count per block).  EPI: the fused CG's epilogue (q = Z + shift p with
// the p.q / q.q partials) compiled in or out.  Three roles per slab (W in 114
// registers, 3 waves per SIMD) measured slower: 15.4 against 11.4 ms at 200^4
// -- every role streams all of F_{d-2}'s fragments in GEMM 2, half the MFMAs
// per fragment load (profiles/r05/i_*).
// SIDE: after each unit's GEMM 2 (W dead, the registers free) the wave applies
// its slice of the fused CG's x side job with ordinary 16-byte loads and
// stores -- streaming work the memory-bound second launch carried before,
// here beside the MFMA-bound slab products.
template <int TF, int JA, int SPW, int EPI, int SIDE>
__global__ __launch_bounds__(128 * SPW, 2) void blk_pair_lds_kernel(PairArgs A) {
  typedef PairRing<TF, SPW> R;
  constexpr int NS = R::NS;
  constexpr int H = R::H;
  constexpr int64_t FSK = (int64_t)R::JT * 64 * 8;   // fragment bytes per k-step
  constexpr int64_t SB = (int64_t)H * H * 8;          // bytes per slab
  __shared__ __attribute__((aligned(16))) double ring[NS * R::STAGE];
  if (A.skip != nullptr && *A.skip) return;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int sl = wave >> 1;   // this wave's slab of the workgroup's SPW
  const int64_t G = gridDim.x;
  // units (SPW consecutive slabs) of this workgroup: blockIdx.x + it G
  const int64_t nunit = A.nslab / SPW;
  const int nmine = __builtin_amdgcn_readfirstlane(
      (int)((nunit - (int64_t)blockIdx.x + G - 1) / G));
  // this wave's DMAs: global index i = wave DPW + j; i < SPW XI: X pieces of
  // slab i / XI, row groups 2 (i % XI), +1 (lane -> group + (lane >> 5),
  // column pair (lane >> 4) & 1, row lane & 15); else fragments 2 f, 2 f + 1,
  // f = min(i - SPW XI, FI - 1)
  uint32_t dlane[R::DPW];
  uint32_t dlds[R::DPW];
#pragma unroll
  for (int j = 0; j < R::DPW; ++j) {
    const int i = wave * R::DPW + j;
    if (i < SPW * R::XI) {
      const int xs = i / R::XI, xi = i % R::XI;
      const int t = 2 * xi + (lane >> 5);
      const int row = min(16 * t + (lane & 15), H - 1);
      dlane[j] = (uint32_t)(xs * SB + (row * 4 + 2 * ((lane >> 4) & 1)) * 8);
      dlds[j] = (uint32_t)(xs * R::XD + xi * 128);
    } else {
      const int f = min(i - SPW * R::XI, R::FI - 1);
      dlane[j] = (uint32_t)((2 * f * 64 + 2 * lane) * 8);
      dlds[j] = (uint32_t)(R::FD + f * 128);
    }
  }
  auto src_at = [&](int it) {
    const int64_t slab = ((int64_t)blockIdx.x + (int64_t)it * G) * SPW;
    PairSlabSrc p;
    p.xoff = uni64(slab * SB);
    const int par = __builtin_amdgcn_readfirstlane((int)((slab / A.spb + A.blk0) & 1));
    p.f3 = par ? A.f3T : A.f3S;
    return p;
  };
  // k-step st of a unit into ring slot `slot`
  auto issue = [&](const PairSlabSrc& p, int st, int slot) {
    const char* xb = ubase(A.X, p.xoff + (int64_t)st * H * 32);   // the k-step's h x 4 run
    const char* fbs = ubase(p.f3, (int64_t)st * FSK);
    double* dst = ring + slot * R::STAGE;
#pragma unroll
    for (int j = 0; j < R::DPW; ++j) {
      const int i = wave * R::DPW + j;   // wave-uniform
      const char* src = i < SPW * R::XI ? xb : fbs;
      // (non-temporal X DMAs: no gain with tiled slabs, +1.5 ms with
      // row-major ones -- profiles/r05/z_epi_nt, r_nt)
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const __attribute__((address_space(1))) void*>(
              reinterpret_cast<uintptr_t>(src + dlane[j])),
          (__attribute__((address_space(3))) void*)(dst + dlds[j]), 16, 0, 0);
    }
  };
  // the side job's half for this iteration (sc->xh, fixed during the launch)
  double sc0 = 0.0, sc1 = 0.0;
  const double* sp0 = nullptr;
  const double* sp1 = nullptr;
  double* sxo = nullptr;
  int64_t slen = 0;
  // mode 3: the armed region, wcnt directions (wave-uniform)
  double wcf[kXWinMax];
  const double* wdir[kXWinMax];
  int wcnt = 0;
  if (SIDE & 4) {
    if (A.sc->warm && !A.sc->done) {
      const int64_t off = (int64_t)A.sc->sreg * A.sreg_len;
      slen = max((int64_t)0, min(A.sn - off, A.sreg_len));
      wcnt = A.sc->scnt;
#pragma unroll
      for (int t = 0; t < kXWinMax; ++t) {
        wcf[t] = A.sc->scoef[t];
        wdir[t] = A.sc->sdir[t] + off;
      }
      sxo = A.sx + off;
    }
  } else if (SIDE & 1) {
    const int xh = A.sc->xh;
    if (xh < 2 && !A.sc->done) {
      const int64_t off = xh ? A.soff_h1 : A.soff;
      slen = xh ? A.sn_h1 : A.sn;
      sc0 = A.sc->xc[0];
      sc1 = A.sc->xc[1];
      sp0 = A.sc->xp[0] + off;
      sp1 = A.sc->xp[1] + off;
      sxo = A.sx + off;
    }
  }
  // this wave's slice [q0, q1) of the half: 16 bytes per lane, kSB batches
  // of loads in flight (the expression of mp_side_job / cg_x_half_kernel)
  auto side_chunk = [&](int64_t slot) {
    const int64_t q0 = slot * A.sstep;
    const int64_t q1 = min(slen, q0 + A.sstep);
    constexpr int kSB = 16;
    for (int64_t e0 = q0 + 2 * lane; e0 < q1; e0 += kSB * 128) {
      double2 xv[kSB], a[kSB], b[kSB];
#pragma unroll
      for (int u = 0; u < kSB; ++u) {
        const int64_t e = e0 + (int64_t)u * 128;
        if (e + 1 < q1) {
          xv[u] = ld2g(sxo + e);
          a[u] = ld2g(sp0 + e);
          b[u] = ld2g(sp1 + e);
        }
      }
#pragma unroll
      for (int u = 0; u < kSB; ++u) {
        const int64_t e = e0 + (int64_t)u * 128;
        if (e + 1 < q1) {
          double2 o;
          o.x = xv[u].x + (sc0 * a[u].x + sc1 * b[u].x);
          o.y = xv[u].y + (sc0 * a[u].y + sc1 * b[u].y);
          st2g(sxo + e, o);
        }
      }
    }
  };
  // mode 3: the wave's slice of the armed region, x += sum_t c_t p_t with every
  // direction's loads of kWB batches in flight before the first sum (the
  // direction count is wave-uniform: scalar branches; cg_x_flush3_kernel
  // forms the same expression)
  auto side_chunk_win = [&](int64_t slot) {
    const int64_t q0 = slot * A.sstep;
    const int64_t q1 = min(slen, q0 + A.sstep);
    constexpr int kWB = 4;
    for (int64_t e0 = q0 + 2 * lane; e0 < q1; e0 += kWB * 128) {
      double2 xv[kWB], a[kXWinMax][kWB];
#pragma unroll
      for (int u = 0; u < kWB; ++u) {
        const int64_t e = e0 + (int64_t)u * 128;
        if (e + 1 < q1) xv[u] = ld2g(sxo + e);
      }
#pragma unroll
      for (int t = 0; t < kXWinMax; ++t)
        if (t < wcnt)
#pragma unroll
          for (int u = 0; u < kWB; ++u) {
            const int64_t e = e0 + (int64_t)u * 128;
            if (e + 1 < q1) a[t][u] = ld2g(wdir[t] + e);
          }
#pragma unroll
      for (int u = 0; u < kWB; ++u) {
        const int64_t e = e0 + (int64_t)u * 128;
        if (e + 1 < q1) {
          double2 s = {0.0, 0.0};
#pragma unroll
          for (int t = 0; t < kXWinMax; ++t)
            if (t < wcnt) {
              s.x += wcf[t] * a[t][u].x;
              s.y += wcf[t] * a[t][u].y;
            }
          double2 o;
          o.x = xv[u].x + s.x;
          o.y = xv[u].y + s.y;
          st2g(sxo + e, o);
        }
      }
    }
  };
  PairSlabSrc cur = src_at(0);
#pragma unroll
  for (int j = 0; j + 1 < NS; ++j) issue(cur, min(j, R::KS - 1), j);   // stages 0 .. NS - 2
  double pq = 0.0, qq = 0.0;
  int cslot = 0;   // slot of the current unit's k-step 0
  for (int it = 0; it < nmine; ++it) {
    const int64_t slab = ((int64_t)blockIdx.x + (int64_t)it * G) * SPW + sl;
    const bool nv = it + 1 < nmine;
    const PairSlabSrc nxt = nv ? src_at(it + 1) : cur;
    const int role = (wave + it) & 1;   // roles alternate per unit
    if (role == 0)
      pair_slab_lds<TF, SPW, EPI, 0, JA, true, (SIDE & 2) != 0>(A, slab, sl, cslot, it == 0, cur, nxt, nv, ring,
                                               issue, pq, qq);
    else
      pair_slab_lds<TF, SPW, EPI, JA, TF - JA, false, (SIDE & 2) != 0>(A, slab, sl, cslot, it == 0, cur, nxt, nv,
                                                      ring, issue, pq, qq);
    if ((SIDE & 4) && slen > 0)
      side_chunk_win(((int64_t)blockIdx.x + (int64_t)it * G) * R::NW + wave);
    else if ((SIDE & 1) && slen > 0)
      side_chunk(((int64_t)blockIdx.x + (int64_t)it * G) * R::NW + wave);
    cslot = (cslot + R::KS) % NS;
    cur = nxt;
  }
  blk_wait_vm<0>();   // the DMAs past the last unit land before the wave ends
  if (A.partials != nullptr) {
    // the reduction reuses the ring (one LDS object in this kernel: a second
    // one gets alias scopes, and the compiler then waits vmcnt(0) between
    // every DMA and the next ds_read)
    __syncthreads();
    double* red = ring;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      pq += __shfl_xor(pq, off, 64);
      qq += __shfl_xor(qq, off, 64);
    }
    if (lane == 0) {
      red[wave] = pq;
      red[R::NW + wave] = qq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = 0.0, s1 = 0.0;
      for (int w = 0; w < R::NW; ++w) {
        s0 += red[w];
        s1 += red[R::NW + w];
      }
      A.partials[blockIdx.x] = s0;
      A.partials[A.pstride + blockIdx.x] = 0.0;
      A.partials[2 * A.pstride + blockIdx.x] = s1;
    }
  }
}

// ------------------------------------------------------------- host side
typedef void (*blk_mode_fn)(ModeArgs);
typedef void (*blk_pair_fn)(PairArgs);



template <int KIND>
static blk_mode_fn mode_fn(int JT, bool T4) {
#define GG_BLK_MODE(jt)                                                    \
  case jt:                                                                 \
    return T4 ? blk_mode_kernel<jt, true, KIND> : blk_mode_kernel<jt, false, KIND>;
  switch (JT) {
    GG_BLK_MODE(1)
    GG_BLK_MODE(2)
    GG_BLK_MODE(3)
    GG_BLK_MODE(4)
    GG_BLK_MODE(5)
    GG_BLK_MODE(6)
    GG_BLK_MODE(7)
    default: return nullptr;
  }
#undef GG_BLK_MODE
}
template <int KIND>
static blk_mode_fn mode_fast_fn(int JT) {
  // the fused kinds ring kD k-steps of three operands, kD | KS: KS = 13 / 17
  // (JT 4 / 5) are prime, the whole strip in flight spills -- the generic
  // kernel there (JT 5: KIND 1 / 3 52 B of scratch, KIND 2 404 B; JT 4 KIND 2 88 B)
  if (KIND != 0 && (JT == 5 || (KIND == 2 && JT == 4))) return nullptr;
  switch (JT) {
    case 2: return blk_mode_fast_kernel<1, KIND>;
    case 3: return blk_mode_fast_kernel<2, KIND>;
    case 4: return blk_mode_fast_kernel<3, KIND>;
    case 5: return blk_mode_fast_kernel<4, KIND>;
    case 6: return blk_mode_fast_kernel<5, KIND>;
    case 7: return blk_mode_fast_kernel<6, KIND>;
    default: return nullptr;
  }
}
// the fast (fixed-count) kernel where instantiated: a 4-row tail and
// h = 16 (JT - 1) + 4 exactly (KS = 4 JT - 3)
static blk_mode_fn select_mode(int kind, int JT, bool T4, int h = 0, bool fast = false) {
  if (T4 && h == 16 * (JT - 1) + 4 && fast) {
    const blk_mode_fn f = kind == 5   ? mode_fast_fn<5>(JT)
                          : kind == 4 ? mode_fast_fn<4>(JT)
                          : kind == 3 ? mode_fast_fn<3>(JT)
                          : kind == 1 ? mode_fast_fn<1>(JT)
                          : kind == 2 ? mode_fast_fn<2>(JT)
                                      : mode_fast_fn<0>(JT);
    if (f != nullptr) return f;
  }
  // kind 3 (the non-temporal prologue) exists on the fast kernel only
  return (kind == 1 || kind == 3) ? mode_fn<1>(JT, T4)
         : kind == 2              ? mode_fn<2>(JT, T4)
         : kind == 4              ? mode_fn<4>(JT, T4)
                                  : mode_fn<0>(JT, T4);
}

// pair kernel shapes: h = 16 TF + 4 for TF in 1..6 (m = 40, 72, 104, 136, 168,
// 200); JA = TF / 2 full column tiles (+ the 4-column tail) for role 0
template <int EPI, int SIDE>
static blk_pair_fn select_pair_lds(int TF, int spw) {
  switch (TF) {
    case 2:
      return spw == 2 ? blk_pair_lds_kernel<2, 1, 2, EPI, SIDE>
                      : blk_pair_lds_kernel<2, 1, 1, EPI, SIDE>;
    case 3:
      return spw == 2 ? blk_pair_lds_kernel<3, 1, 2, EPI, SIDE>
                      : blk_pair_lds_kernel<3, 1, 1, EPI, SIDE>;
    case 4:
      return spw == 2 ? blk_pair_lds_kernel<4, 2, 2, EPI, SIDE>
                      : blk_pair_lds_kernel<4, 2, 1, EPI, SIDE>;
    case 5:
      return spw == 2 ? blk_pair_lds_kernel<5, 2, 2, EPI, SIDE>
                      : blk_pair_lds_kernel<5, 2, 1, EPI, SIDE>;
    case 6:
      return spw == 2 ? blk_pair_lds_kernel<6, 3, 2, EPI, SIDE>
                      : blk_pair_lds_kernel<6, 3, 1, EPI, SIDE>;
    default: return nullptr;
  }
}

// epi: the fused CG's epilogue; side: its x side job rides in the launch
// (LDS kernel only; the CG epilogue always comes with it there); nt: that
// launch's p loads and q stores non-temporal (SIDE bit 2); win: the side job
// is x_defer mode 3's armed region (SIDE bit 4) instead of mode 2's half
static blk_pair_fn select_pair(int TF, bool lds = false, int spw = 1, bool epi = false,
                               bool side = false, bool nt = false, bool win = false) {
  if (lds) {
    if (side && win) return nt ? select_pair_lds<1, 7>(TF, spw) : select_pair_lds<1, 5>(TF, spw);
    if (side) return nt ? select_pair_lds<1, 3>(TF, spw) : select_pair_lds<1, 1>(TF, spw);
    // the fused Lanczos step's pair launch: its w loads / Y stores
    // non-temporal as the CG's (SIDE bit 2 alone)
    if (epi && nt) return select_pair_lds<1, 2>(TF, spw);
    return epi ? select_pair_lds<1, 0>(TF, spw) : select_pair_lds<0, 0>(TF, spw);
  }
  switch (TF) {
    case 1: return blk_pair_kernel<1, 1>;
    case 2: return blk_pair_kernel<2, 1>;
    case 3: return blk_pair_kernel<3, 1>;
    case 4: return blk_pair_kernel<4, 2>;
    case 5: return blk_pair_kernel<5, 2>;
    case 6: return blk_pair_kernel<6, 3>;
    default: return nullptr;
  }
}

static int blk_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    if (n <= 0) n = 256;
  }
  return n;
}

static void blk_set_lds_limits(const BlockOp* B) {
  for (int k = 0; k + 2 < B->d; ++k) {
    const size_t bytes = (size_t)B->KS[k] * B->JT[k] * 64 * sizeof(double);
    for (int kind = 0; kind < 6; ++kind)
      GG_HIP(hipFuncSetAttribute(
          reinterpret_cast<const void*>(
              select_mode(kind, B->JT[k], B->T4[k], (int)B->h[k], B->fast)),
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  }
}

BlockOp* block_create(int d, const int64_t* rows, const int64_t* cols,
                      const double* const* factors) {
  if (d < 2 || d > kBlkMaxD) return nullptr;
  const char* env = gg::knob("GG_KRON_BLOCK");   // read once, at handle creation
  if (env && atoi(env) == 0) return nullptr;
  for (int k = 0; k < d; ++k) {
    if (rows[k] != cols[k] || rows[k] % 2 != 0 || rows[k] < 2) return nullptr;
    if (rows[k] / 2 > 112) return nullptr;   // blk_mode_kernel: JT <= 7
  }
  // the pair axes: equal orders, half order h padded to hp = 16 TF + 4 >= h
  const int64_t hpair = rows[d - 1] / 2;
  if (rows[d - 2] != rows[d - 1]) return nullptr;
  const int TF = (int)std::max<int64_t>(1, ceil_div(hpair - 4, 16));
  if (select_pair(TF) == nullptr) return nullptr;
  const int64_t hp = 16 * (int64_t)TF + 4;
  // centrosymmetric factors only (the test of gg_kron.hip pack_fold)
  for (int k = 0; k < d; ++k) {
    const int64_t m = rows[k];
    const double* F = factors[k];
    double amax = 0.0, dmax = 0.0;
    for (int64_t j = 0; j < m; ++j)
      for (int64_t i = 0; i < m; ++i) {
        amax = std::max(amax, std::fabs(F[j * m + i]));
        dmax = std::max(dmax, std::fabs(F[j * m + i] - F[(m - 1 - j) * m + (m - 1 - i)]));
      }
    if (!(dmax <= 16.0 * 2.220446049250313e-16 * amax) || !(amax > 0.0)) return nullptr;
  }
  BlockOp* B = new BlockOp();
  try {
    B->d = d;
    B->nb = 1;
    for (int k = 0; k < d; ++k) {
      B->m[k] = rows[k];
      B->h[k] = rows[k] / 2;
      B->e[k] = k >= d - 2 ? hp : B->h[k];
      B->nb *= B->e[k];
    }
    B->n = B->nb << d;
    B->pTF = TF;
    B->cus = blk_cus();
    const char* fe = gg::knob("GG_BLK_MODE_FAST");   // A/B knob, read at creation only
    B->fast = !(fe && atoi(fe) == 0);
    const char* ne = gg::knob("GG_BLK_PRO_NT");      // A/B knob, read at creation only
    B->pro_nt = !(ne && atoi(ne) == 0);
    const char* ee = gg::knob("GG_BLK_EPI_NT");      // A/B knob, read at creation only
    B->epi_nt = !(ee && atoi(ee) == 0);
    const char* le = gg::knob("GG_BLK_PAIR_LDS");   // A/B knob, read at creation only
    B->pair_lds = select_pair(TF, true) != nullptr && !(le && atoi(le) == 0);
    {
      int64_t spb = 1;
      for (int k = 0; k + 2 < d; ++k) spb *= rows[k] / 2;
      const char* se = gg::knob("GG_BLK_PAIR_SPW");   // A/B knob, read at creation only
      B->pair_spw = (spb % 2 == 0 && !(se && atoi(se) == 1)) ? 2 : 1;
    }
    for (int k = 0; k < d; ++k) {
      const int64_t m = B->m[k], h = B->h[k];
      const double* F = factors[k];
      // the centrosymmetric part (F + J F J) / 2, then S / T
      auto Fc = [&](int64_t j, int64_t i) {
        return 0.5 * (F[j * m + i] + F[(m - 1 - j) * m + (m - 1 - i)]);
      };
      int JT, KS;
      bool T4;
      if (k >= d - 2) {
        // the pair kernel's shape (hp); fragments past h stay zero
        JT = TF + 1;
        T4 = true;
        KS = 4 * TF + 1;
      } else {
        const int64_t tail = h % 16;
        T4 = tail != 0 && tail <= 4;
        JT = (int)ceil_div(h, 16);
        KS = (int)ceil_div(h, 4);
      }
      B->JT[k] = JT;
      B->KS[k] = KS;
      B->T4[k] = T4;
      const int TFk = T4 ? JT - 1 : JT;
      for (int par = 0; par < 2; ++par) {
        // + 128 zeros: blk_pair_lds_kernel stages an even fragment count
        std::vector<double> hb((size_t)KS * JT * 64 + 128, 0.0);
        for (int s = 0; s < KS; ++s)
          for (int t = 0; t < JT; ++t)
            for (int l = 0; l < 64; ++l) {
              const bool tail = T4 && t == TFk;
              const int64_t j = tail ? 16 * (int64_t)t + (l & 3) : 16 * (int64_t)t + (l & 15);
              const int64_t i = 4 * (int64_t)s + (l >> 4);
              double v = 0.0;
              if (j < h && i < h)
                v = par == 0 ? Fc(j, i) + Fc(j, m - 1 - i) : Fc(j, i) - Fc(j, m - 1 - i);
              hb[((size_t)s * JT + t) * 64 + l] = v;
            }
        GG_HIP(hipMalloc(&B->frag[k][par], hb.size() * sizeof(double)));
        GG_HIP(hipMemcpy(B->frag[k][par], hb.data(), hb.size() * sizeof(double),
                         hipMemcpyHostToDevice));
      }
    }
    for (int k = 0; k + 2 < d; ++k)
      GG_REQUIRE(select_mode(0, B->JT[k], B->T4[k]) != nullptr, GG_ERR_RUNTIME,
                 "no block mode kernel for this factor order");
    blk_set_lds_limits(B);
  } catch (...) {
    block_destroy(B);
    throw;
  }
  return B;
}

void block_destroy(BlockOp* B) {
  if (!B) return;
  for (int k = 0; k < kBlkMaxD; ++k)
    for (int p = 0; p < 2; ++p)
      if (B->frag[k][p]) (void)hipFree(B->frag[k][p]);
  delete B;
}

int64_t block_n(const BlockOp* B) { return B->n; }
int block_d(const BlockOp* B) { return B->d; }
int block_launches(const BlockOp* B) { return B->d - 1; }

static int fold_grid(const BlockOp* B) {
  return (int)std::min<int64_t>(ceil_div(B->nb, 256), (int64_t)B->cus * 8);
}
int64_t block_fold_partials(const BlockOp* B) { return fold_grid(B); }

int64_t block_nb(const BlockOp* B) { return B->nb; }

void block_fold(const BlockOp* B, bool inverse, const double* x, double* y, double* sq_part,
                hipStream_t s, int64_t blk0, int64_t nblk) {
  if (nblk < 0) {
    blk0 = 0;
    nblk = (int64_t)1 << B->d;
  }
  GG_REQUIRE(blk0 >= 0 && nblk >= 1 && blk0 + nblk <= ((int64_t)1 << B->d), GG_ERR_VALUE,
             "block range outside the 2^d blocks");
  FoldGeom g{};
  g.d = B->d;
  g.nb = B->nb;
  g.hp = B->e[B->d - 1];
  g.blk0 = blk0;
  g.nblk = nblk;
  int64_t st = 1;
  for (int k = B->d - 1; k >= 0; --k) {
    g.m[k] = B->m[k];
    g.h[k] = B->h[k];
    g.stride[k] = st;
    st *= B->m[k];
  }
  const double scale = std::ldexp(1.0, -B->d / 2) * ((B->d & 1) ? M_SQRT1_2 : 1.0);
  const int grid = fold_grid(B);
  double* sp = inverse ? nullptr : sq_part;
  switch (B->d) {
#define GG_BLK_FOLD(D)                                                                      \
  case D:                                                                                   \
    hipLaunchKernelGGL(blk_fold_kernel<D>, dim3(grid), dim3(256), 0, s, x, y, g,           \
                       inverse ? 1 : 0, scale, sp);                                         \
    break;
    GG_BLK_FOLD(2)
    GG_BLK_FOLD(3)
    GG_BLK_FOLD(4)
    GG_BLK_FOLD(5)
    GG_BLK_FOLD(6)
#undef GG_BLK_FOLD
    default: GG_REQUIRE(false, GG_ERR_VALUE, "block basis: 2 <= d <= 6");
  }
  GG_LAUNCH_CHECK();
}

// grid of the mode-product launch of axis k (one workgroup per CU)
// waves per workgroup of the launch select_mode picks
static int mode_waves(int kind, const BlockOp* B, int k) {
  const int JT = B->JT[k];
  const bool fast = B->T4[k] && B->h[k] == 16 * (JT - 1) + 4 && B->fast &&
                    (kind == 5   ? mode_fast_fn<5>(JT)
                     : kind == 4 ? mode_fast_fn<4>(JT)
                     : kind == 3 ? mode_fast_fn<3>(JT)
                     : kind == 1 ? mode_fast_fn<1>(JT)
                     : kind == 2 ? mode_fast_fn<2>(JT)
                                 : mode_fast_fn<0>(JT)) != nullptr;
  if (!fast) return kBlkModeWaves;
  return kind == 0 ? fast_waves<0>() : kind == 2 ? fast_waves<2>() : fast_waves<1>();
}

static int64_t mode_geometry(const BlockOp* B, int k, int W, ModeArgs& a, int* grid_out,
                             int64_t nblk = -1) {
  const int d = B->d;
  int64_t inner = 1, outer = 1;
  for (int i = k + 1; i < d; ++i) inner *= B->e[i];
  for (int i = 0; i < k; ++i) outer *= B->h[i];
  GG_REQUIRE(inner % 16 == 0, GG_ERR_VALUE, "block basis: inner extent not a multiple of 16");
  a.h = (int)B->h[k];
  a.KS = B->KS[k];
  a.inner = inner;
  a.spb = outer * (inner / 16);
  a.gpb = ceil_div(a.spb, (int64_t)W);
  a.ngroups = a.gpb * (nblk < 0 ? ((int64_t)1 << d) : nblk);
  const int64_t grid = std::min<int64_t>(a.ngroups, (int64_t)B->cus);
  a.per_wg = ceil_div(a.ngroups, grid);
  a.nb = B->nb;
  a.bitpos = d - 1 - k;
  a.fS = B->frag[k][0];
  a.fT = B->frag[k][1];
  const int64_t g = ceil_div(a.ngroups, a.per_wg);
  *grid_out = (int)g;
  return g;
}

int64_t block_prologue_blocks(const BlockOp* B) {
  ModeArgs a{};
  int g = 0;
  if (B->d < 3) return 1;
  mode_geometry(B, 0, mode_waves(1, B, 0), a, &g);
  return g;
}

// workgroups of the pair launch: blk_pair_kernel 2 slabs each, 2 per CU;
// blk_pair_lds_kernel one slab each, 4 per CU (28 KiB of LDS ring apiece at
// h = 100), persistent
static int pair_grid(const BlockOp* B, int64_t nblk = -1) {
  const int64_t nslab = B->nb / (B->e[B->d - 1] * B->e[B->d - 2]) *
                        (nblk < 0 ? ((int64_t)1 << B->d) : nblk);
  if (B->pair_lds)   // 4 slabs in flight per CU (the LDS ring's budget)
    return (int)std::min<int64_t>(nslab / B->pair_spw, (int64_t)B->cus * 4 / B->pair_spw);
  return (int)std::min<int64_t>(ceil_div(nslab, kBlkPairWaves / 2), (int64_t)B->cus * 2);
}
int64_t block_partials_needed(const BlockOp* B) { return pair_grid(B); }

// y = (P K P^T + shift I) x in the block layout (x, y distinct; `work`: n
// doubles of scratch when d >= 3 -- the in-place chain of axes 0..d-3 runs
// there, x stays intact for the shift).  With the fused CG (cgp 2, layout 0,
// cg != nullptr): the chain runs in place on y == cg->q_old (the prologue of
// the first launch reads q_old before it writes the launch's output over it:
// same positions, same wave), x = p_old, p_new -> cg->p_out, the second
// launch (d >= 4) carries the balanced x side job, and the pair launch writes
// q = Z + shift p_new into cg->blk_q_out (not y: the two waves of a slab read
// its input while storing) with the p.q / q.q partials.
void block_apply(const BlockOp* B, const double* x, double* y, double shift, double* work,
                 double* dot_partials, const int* skip, hipStream_t stream, int64_t* n_partials,
                 const MpFuse* cg, int cgp, hipEvent_t* ev, int64_t blk0, int64_t nblk) {
  const int d = B->d;
  if (nblk < 0) {
    blk0 = 0;
    nblk = (int64_t)1 << d;
  }
  GG_REQUIRE(blk0 >= 0 && nblk >= 1 && blk0 + nblk <= ((int64_t)1 << d), GG_ERR_VALUE,
             "block range outside the 2^d blocks");
  if (cg == nullptr) cgp = 0;
  GG_REQUIRE(cgp == 0 || cgp == 2 || cgp == 3, GG_ERR_VALUE,
             "block basis: plain, fused CG or fused Lanczos only");
  GG_REQUIRE(cgp == 0 || d >= 3, GG_ERR_VALUE, "block basis CG / Lanczos: d >= 3");
  GG_REQUIRE(x != y, GG_ERR_VALUE, "x and y must not alias");
  if (cgp == 2)
    GG_REQUIRE(cg->q_old == y && cg->p_out != nullptr && cg->p_out != x &&
                   cg->blk_q_out != nullptr && cg->blk_q_out != y,
               GG_ERR_VALUE, "block CG: buffer roles");
  else if (cgp == 3)
    // Lanczos: x = u_prev (w written over it), cg->r = u, y = the previous
    // output (the chain runs in place on it), the pair launch writes blk_q_out
    GG_REQUIRE(cg->q_old == y && cg->p_out == x && cg->r != nullptr && cg->r != x &&
                   cg->r != y && cg->coef != nullptr && cg->blk_q_out != nullptr &&
                   cg->blk_q_out != y && cg->blk_q_out != x && cg->blk_q_out != cg->r,
               GG_ERR_VALUE, "block Lanczos: buffer roles");
  else if (d >= 3)
    GG_REQUIRE(work != nullptr && work != x && work != y, GG_ERR_VALUE,
               "block basis: scratch required");
  if (ev) GG_HIP(hipEventRecord(ev[0], stream));
  const double* src = x;
  double* chain = cgp >= 2 ? y : work;
  int pos = 0;
  // the fused CG's x side job: in the pair launch where the LDS pair kernel
  // runs (beside its MFMA-bound slab products), else in the second launch (a
  // streaming kernel after the first when d = 3)
  const bool side = cgp == 2 && cg->sx != nullptr && (cg->xdefer == 2 || cg->xdefer == 3);
  const bool pair_side = side && B->pair_lds;
  // mode 3 (the window): in the pair launch only (gg_cg_start picks it where
  // block_pair_side holds)
  const bool win = side && cg->xdefer == 3;
  GG_REQUIRE(!win || (pair_side && cg->xwin >= 2 && cg->xwin <= kXWinMax), GG_ERR_VALUE,
             "block CG: the x window needs the LDS pair launch");
  // (a share of each x half on a concurrent stream beside the plain launch
  // measured slower: 20 % of it made the plain launch +0.76 ms and the pair
  // launch -0.55 ms, profiles/r05/za_conc)
  for (int k = 0; k + 2 < d; ++k) {
    ModeArgs a{};
    int grid = 0;
    int kind = 0;
    if (cgp == 2 && k == 0)
      kind = cg->rderive ? 5 : B->pro_nt ? 3 : 1;
    else if (cgp == 3 && k == 0)
      kind = 4;
    else if (k == 1 && side && !pair_side)
      kind = 2;
    const int W = mode_waves(kind, B, k);
    mode_geometry(B, k, W, a, &grid, nblk);
    a.blk0 = blk0;
    a.X = src;
    a.Y = chain;
    a.skip = skip;
    if (kind == 1 || kind == 3 || kind == 5) {
      a.r = cg->r;
      a.pprev = cg->pprev;
      GG_REQUIRE(kind != 5 || cg->pprev != nullptr, GG_ERR_VALUE,
                 "block CG: derived r needs p_{j-2}");
      a.q_old = cg->q_old;
      a.p_out = cg->p_out;
      a.sc = cg->sc;
      a.rr_part = cg->rr_part;
      a.pqo_stride = cg->pqo_stride;
      GG_REQUIRE(grid <= cg->rr_cap, GG_ERR_VALUE, "prologue partial array too short");
      if (cg->pro_blocks != nullptr) *cg->pro_blocks = grid;
    } else if (kind == 4) {
      a.r = cg->r;
      a.q_old = cg->q_old;
      a.p_out = cg->p_out;
      a.coef = cg->coef;
      a.rr_part = cg->rr_part;
      GG_REQUIRE(grid <= cg->rr_cap, GG_ERR_VALUE, "prologue partial array too short");
      if (cg->pro_blocks != nullptr) *cg->pro_blocks = grid;
    } else if (kind == 2) {
      a.sc = cg->sc;
      a.sx = cg->sx;
      const int64_t sn = cg->sn;
      const int64_t H = block_side_half(sn);
      a.soff = 0;
      a.sn = std::min(H, sn);
      a.soff_h1 = a.sn;
      a.sn_h1 = sn - a.sn;
      const int64_t slots = a.ngroups * W;
      a.sstep = 2 * ceil_div(std::max<int64_t>(std::max(a.sn, a.sn_h1), 1), 2 * slots);
      GG_REQUIRE(a.sstep <= 128 * (int64_t)a.KS, GG_ERR_VALUE,
                 "block CG: x side job larger than its k-steps");
    }
    const blk_mode_fn fn = select_mode(kind, B->JT[k], B->T4[k], (int)B->h[k], B->fast);
    const size_t lds = (size_t)B->KS[k] * B->JT[k] * 64 * sizeof(double);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * W), lds, stream, a);
    GG_LAUNCH_CHECK();
    if (k == 0 && d == 3 && side && !pair_side)
      // no second launch to carry the x side job: its half as a streaming kernel
      launch_x_half(cg->sx, cg->sn, block_side_half(cg->sn), cg->sc, stream);
    if (ev) GG_HIP(hipEventRecord(ev[++pos], stream));
    src = chain;
  }
  // the pair launch
  PairArgs p{};
  p.X = src;
  p.Y = cgp >= 2 ? cg->blk_q_out : y;
  const int k3 = d - 1, k2 = d - 2;
  p.f3S = B->frag[k3][0];
  p.f3T = B->frag[k3][1];
  p.f2S = B->frag[k2][0];
  p.f2T = B->frag[k2][1];
  p.spb = B->nb / (B->e[k3] * B->e[k2]);
  p.nslab = p.spb * nblk;
  p.blk0 = blk0;
  p.skip = skip;
  const int grid = pair_grid(B, nblk);
  if (cgp >= 2) {
    // q = Z + shift p_new (CG) / Y = Z + shift w (Lanczos) with the p.q, q.q
    // partials (Lanczos: u.Y for alpha)
    p.P = cg->p_out;
    p.shift = shift;
    p.partials = dot_partials;
    p.pstride = cg->pstride;
  } else if (shift != 0.0) {
    p.P = x;
    p.shift = shift;
  }
  if (pair_side && win) {
    p.sc = cg->sc;
    p.sx = cg->sx;
    p.sn = cg->sn;
    p.sreg_len = xwin_region(cg->sn, cg->xwin);
    const int64_t slots = p.nslab / B->pair_spw * 2 * B->pair_spw;
    p.sstep = 2 * ceil_div(std::max<int64_t>(p.sreg_len, 1), 2 * slots);
  } else if (pair_side) {
    p.sc = cg->sc;
    p.sx = cg->sx;
    const int64_t sn = cg->sn;
    const int64_t H = block_side_half(sn);
    p.soff = 0;
    p.sn = std::min(H, sn);
    p.soff_h1 = p.sn;
    p.sn_h1 = sn - p.sn;
    // wave slots: every unit's waves (units = slabs / pair_spw, 2 pair_spw waves)
    const int64_t slots = p.nslab / B->pair_spw * 2 * B->pair_spw;
    p.sstep = 2 * ceil_div(std::max<int64_t>(std::max(p.sn, p.sn_h1), 1), 2 * slots);
  }
  // non-temporal epilogue streams: the CG's (with its side job) and the
  // Lanczos step's (cgp 3); the plain / shifted matvec keeps normal ones
  hipLaunchKernelGGL(select_pair(B->pTF, B->pair_lds, B->pair_spw, p.P != nullptr, pair_side,
                                 B->epi_nt && (pair_side || cgp == 3), win),
                     dim3(grid), dim3(B->pair_lds ? 128 * B->pair_spw : 64 * kBlkPairWaves), 0,
                     stream, p);
  GG_LAUNCH_CHECK();
  if (ev) GG_HIP(hipEventRecord(ev[++pos], stream));
  if (n_partials) *n_partials = (cgp >= 2) ? grid : 0;
}

// the x side job's half boundary in the block path (the closing flush uses it)
int64_t block_side_half(int64_t n) { return 2 * ceil_div(n, (int64_t)4); }

bool block_pair_side(const BlockOp* B) { return B != nullptr && B->pair_lds; }

bool block_rderive_ok(const BlockOp* B) {
  if (B == nullptr || B->d < 3 || !B->pro_nt) return false;
  const int JT = B->JT[0];
  return B->T4[0] && B->h[0] == 16 * (JT - 1) + 4 && B->fast && mode_fast_fn<5>(JT) != nullptr;
}

// the padded slabs cost (hp / h)^2 of every pass over the vector: measured at
// d = 4 (profiles/r06/d_prof/block_vs_grid.jsonl), the padded block basis
// loses to the grid basis on one GPU even at 1.13x -- CG iteration 64^4
// 0.51 vs 0.43 ms, 96^4 2.19 vs 2.02, 128^4 6.64 vs 6.56 -- where the unpadded
// orders win (136^4 7.33 vs 8.25 ms, 200^4 33.3 vs 38); so one GPU takes the
// block basis by default only unpadded, and the block-sharded CG wherever it
// exists (no exchange across ranks; the alternatives fold on the host or
// exchange twice per matvec)
bool block_efficient(const BlockOp* B) {
  if (B == nullptr) return false;
  const int d = B->d;
  return B->e[d - 1] == B->h[d - 1] && B->e[d - 2] == B->h[d - 2];
}

}  // namespace gg
