// Centrosymmetric Kronecker factors on MI355X: the mode product of
// gg_kron.hip with the factor's even/odd split, half the FP64 MFMA work.
//
// Reference: KronMatrix.kronvec_prod, gp_grief/tensors/kron_matrix.py:52-97
// (each factor applied by BLAS3 dsymm/dgemm); the split is an execution
// detail of that product.
#include "gg_mp.h"

namespace gg {

// ---------------------------------------------------------------------------
// Centrosymmetric factors: the even/odd split, half the MFMA work.
//
// A square factor F (m x m) with J F J = F (J reverses the index order) --
// every stationary kernel (RBF, Matern, ...) on an evenly spaced grid, i.e.
// every GridKernel.cov_grid factor on InducingGrid / linspace points -- maps
// the even and odd parts of its input to the even and odd parts of its output.
// With h = m / 2, hS = m - h (= h + 1 for odd m), for i', j' < h:
//   u[i'] = x[i'] + x[m-1-i'],   v[i'] = x[i'] - x[m-1-i']     (u[h] = x[h])
//   S = Es u (hS x hS),  T = Ea v (h x h),
//   Es[j'][i'] = (F[j'][i'] + F[j'][m-1-i']) / 2,  Es[j'][h] = F[j'][h],
//   Ea[j'][i'] = (F[j'][i'] - F[j'][m-1-i']) / 2,
//   y[j'] = S[j'] + T[j'],   y[m-1-j'] = S[j'] - T[j']         (y[h] = S[h])
// so one mode product is two half-size GEMMs: m^2 instead of 2 m^2 FLOP per
// column of X, the same HBM bytes -- at m = 200 in FP64 the mode product moves
// from the MFMA roof to the HBM roof.  The host packs Es / Ea from the
// centrosymmetric part (F + J F J) / 2, accepted when max |F - J F J| <= 16 eps
// max |F| (the dense product's own rounding is m eps); Factor::fold.
//
// Same work decomposition as mode_product_kernel: a wave owns 16 rows b of
// Y and every output column; lane l's A operand at k-step s is built from
// X[i'][b] and X[m-1-i'][b], i' = 4 s + (l >> 4) -- two 128-B row segments per
// wave instruction, rows i' ascending and m-1-i' descending -- and the S
// accumulators take u, the T accumulators v.  Per k-step the fragments are
// [S tiles][S 4x4 tail][T tiles][T 4x4 tail] (FS + FA of them), staged by
// global_load_lds, double-buffered, one barrier per chunk.  JS / JA: 16-wide
// tiles of S / T; TS / TA > 0: that half's last tile (at most 4 TS real
// columns) runs as TS v_mfma_f64_4x4x4_4b_f64 (see kT4 above).
// The CG / Lanczos prologues (CGP) update both elements a lane loads and
// write both back; the epilogue stores S + T at column j' and S - T at m-1-j'
// (+ shift * x and the CG partial dots, kEpi as mode_product_kernel).
// kMap: the sharded operator's plain-store epilogue through an OutMap
// (all-to-all chunk order, or peer stores in push mode; mode_product_kernel
// mp_finish), no shift / dots.
// kOpt (A/B variants, GG_FOLD_VARIANT): bit 0 s_setprio(1) around each
// k-step's MFMAs; bit 1 issue the next chunk's loads before the first k-step
// instead of after it; bit 2 (kLean) address the A rows as a wave-uniform row
// base (SGPRs) plus a 32-bit lane byte offset -- no 64-bit address registers
// or clamps (the host takes it only when every chunk's rows lie inside the
// factor, 4 kKC nchunks <= m, and 4 M * 8 < 2^32); bit 3 (kBdb) read the next
// pair of B fragments from LDS before the current pair's MFMAs (register
// double buffer) instead of waiting on each read.
// kStg: the identity epilogue staged through LDS -- each accumulator
// register's 4 rows go to a wave-private LDS image in the global layout (row
// stride m), then the wave streams them with 16-byte lanes (1 KiB contiguous
// per instruction) together with the fused operands (p, r) it loads the same
// way.  Needs m even and 16-byte aligned vectors (kron_apply checks).
template <int JS, int JA, int TS, int TA, int kKC, int CGP, int kMinW, int kEpi, bool kMap = false,
          int kOpt = 0, bool kStg = false, int kWv = 4>
__global__ __launch_bounds__(64 * kWv, kMinW) void mode_product_fold_kernel(
    const double* X, double* __restrict__ Y, const double* __restrict__ Bf,
    int64_t M, int m, int, int KS, int, int,
    const double* __restrict__ xs, double shift, double* __restrict__ dot_partials,
    const int* __restrict__ skip, OutMap om, MpFuse fz) {
  static_assert(!kMap || kEpi == 0, "the mapped epilogue stores only");
  constexpr bool kLean = (kOpt & 4) != 0;
  constexpr bool kBdb = (kOpt & 8) != 0;
  // kOpt bits 5-7 (GG_FOLD_*_NT masks 1 / 2 / 4): bit 5 non-temporal A-operand
  // (+ r / q_old) loads; bit 6 non-temporal p_new / r stores (CG prologue),
  // epilogue operand loads (p, r) and the x side job's streams; bit 7
  // non-temporal output stores
  constexpr bool kNTl = (kOpt & 32) != 0, kNTs = (kOpt & 64) != 0, kNTy = (kOpt & 128) != 0;
  auto ldg = [](const double* p) -> double {
    if constexpr (kNTl) return __builtin_nontemporal_load(p);
    return *p;
  };
  auto stg = [](double* p, double v) {
    if constexpr (kNTs) __builtin_nontemporal_store(v, p);
    else *p = v;
  };
  auto sty = [](double* p, double v) {
    if constexpr (kNTy) __builtin_nontemporal_store(v, p);
    else *p = v;
  };
  static_assert(!(kMap && kStg), "staged epilogue: identity layout only");
  constexpr int kWaves = kWv;   // waves per workgroup (A/B variants: 6, 12)
  constexpr int kThreads = 64 * kWv;
  constexpr int FS = JS - (TS > 0 ? 1 : 0) + TS;   // S fragments per k-step
  constexpr int FA = JA - (TA > 0 ? 1 : 0) + TA;   // T fragments per k-step
  constexpr int JF = FS + FA;
  constexpr int kChunk2 = kKC * JF * 32;           // double2 per chunk
  constexpr int kPerT = (kChunk2 + kThreads - 1) / kThreads;
  constexpr int kBuf = kKC * JF * 64;              // doubles per LDS buffer
  constexpr bool edots = kEpi >= 2;
  // kEpi 4: fusion layout 1 -- xs holds p_old, the epilogue recomputes
  // p_new = r + beta p_old (bitwise the prologue's value) and stores it
  constexpr bool kRecomp = kEpi == 4;
  static_assert(kEpi != 3, "fusion layout 2 runs on mode_product_kernel");
  if (skip != nullptr && *skip) return;
  extern __shared__ __attribute__((aligned(16))) double lds[];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = m >> 1;
  const int hS = m - h;
  // kOpt bit 4: XCD-contiguous block order -- dispatch deals consecutive
  // block ids round-robin over the 8 XCDs; remapped, XCD x walks the x-th
  // eighth of the rows b, so each XCD streams contiguous row segments
  int64_t blk = blockIdx.x;
  if constexpr ((kOpt & 16) != 0) {
    const int64_t nb = gridDim.x, n8 = nb >> 3;
    if (blk < 8 * n8) blk = (blk & 7) * n8 + (blk >> 3);
  }
  const int64_t b0 = (blk * kWaves + wave) * 16;
  const int64_t brow = b0 + (lane & 15);
  const bool bvalid = brow < M;
  const int64_t bclamp = bvalid ? brow : M - 1;
  const int krow = lane >> 4;
  const int nchunks = (KS + kKC - 1) / kKC;

  // B staging: a chunk is kKC * JF * 64 contiguous doubles (8 zero k-steps of
  // padding after the last, so a partial last chunk stays in bounds)
  const int64_t bchunk = (int64_t)kBuf;
  int boff[kPerT];
  bool bfull[kPerT];
#pragma unroll
  for (int u = 0; u < kPerT; ++u) {
    const int i = threadIdx.x + u * kThreads;
    bfull[u] = i < kChunk2;
    boff[u] = 2 * (i < kChunk2 ? i : kChunk2 - 1);
  }
  // A operand rows: lo = i' ascending from krow, hi = m-1-i' descending
  const int64_t m4 = 4 * M;
  const int64_t lo0 = (int64_t)krow * M + bclamp;
  const int64_t hi0 = (int64_t)(m - 1 - krow) * M + bclamp;
  const int64_t alast = (int64_t)(m - 1) * M + bclamp;
  const int64_t achunk = (int64_t)kKC * m4;
  double* __restrict__ Rg = fz.r;
  const double* Qa = fz.q_old;   // CGP 3 writes over q_old (same lane): no restrict
  double* Pout = fz.p_out;

  bool cg_first = false, cg_pending = false, pqo_on = false;
  double cg_beta = 0.0, cg_alpha = 0.0, rr_acc = 0.0, pqo_acc = 0.0, cg_qs = 0.0;
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
      cg_qs = fz.qshift;
      // p_new.q_old (conjugacy r.q); q_old is not A p_old on the first step
      pqo_on = fz.pqo_stride > 0 && !cg_first;
    }
  }

  auto stage = [&](int c) {
    const double* cb = Bf + (int64_t)c * bchunk;
    double* dstb = lds + (c & 1) * kBuf + wave * 128;
#pragma unroll
    for (int u = 0; u < kPerT; ++u)
      if (bfull[u])
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(cb + boff[u]),
            (__attribute__((address_space(3))) void*)(dstb + u * kThreads * 2), 16, 0, 0);
  };
  // kLean: lane byte offsets of rows krow and 3 - krow from a 4-row base;
  // the row bases go through readfirstlane, opaque to loop strength
  // reduction, so every access keeps the SGPR-base + 32-bit VGPR-offset form
  const uint32_t loff = (uint32_t)(((int64_t)krow * M + bclamp) * 8);
  const uint32_t hoff = (uint32_t)(((int64_t)(3 - krow) * M + bclamp) * 8);
  auto sbase = [](const void* p, int64_t off) -> char* {
    const uint64_t a = reinterpret_cast<uint64_t>(p) + (uint64_t)off;
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t u = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return reinterpret_cast<char*>(((uint64_t)u << 32) | l);
  };
  // byte offsets of k-step t's low / high row bases
  auto lrow_b = [&](int64_t t) -> int64_t { return 4 * t * M * 8; };
  auto hrow_b = [&](int64_t t) -> int64_t { return ((int64_t)(m - 4) - 4 * t) * M * 8; };
  // raw loads of chunk c: [0] = row i', [1] = row m-1-i' (only the last
  // chunk can step past the rows: clamp there, masked when consumed)
  auto aload = [&](int c, double (&a)[2][kKC], double (&r)[2][kKC], double (&q)[2][kKC]) {
    if constexpr (kLean) {
#pragma unroll
      for (int s = 0; s < kKC; ++s) {
        const int64_t t = (int64_t)c * kKC + s;
        const int64_t lb = lrow_b(t), hb = hrow_b(t);
        a[0][s] = ldg(reinterpret_cast<const double*>(sbase(X, lb) + loff));
        a[1][s] = ldg(reinterpret_cast<const double*>(sbase(X, hb) + hoff));
        if (CGP) {
          r[0][s] = *reinterpret_cast<const double*>(sbase(Rg, lb) + loff);
          r[1][s] = *reinterpret_cast<const double*>(sbase(Rg, hb) + hoff);
        }
        if (CGP >= 2) {
          q[0][s] = *reinterpret_cast<const double*>(sbase(Qa, lb) + loff);
          q[1][s] = *reinterpret_cast<const double*>(sbase(Qa, hb) + hoff);
        }
      }
      return;
    }
    int64_t ol = lo0 + (int64_t)c * achunk;
    int64_t oh = hi0 - (int64_t)c * achunk;
    const bool last = c == nchunks - 1;
#pragma unroll
    for (int s = 0; s < kKC; ++s) {
      const int64_t l_ = last ? (ol < alast ? ol : alast) : ol;
      const int64_t h_ = last ? (oh > bclamp ? oh : bclamp) : oh;
      a[0][s] = ldg(X + l_);
      a[1][s] = ldg(X + h_);
      if (CGP) {
        r[0][s] = ldg(Rg + l_);
        r[1][s] = ldg(Rg + h_);
      }
      if (CGP >= 2) {
        q[0][s] = ldg(Qa + l_);
        q[1][s] = ldg(Qa + h_);
      }
      ol += m4;
      oh -= m4;
    }
  };
  // one element of the CG / Lanczos prologue (mode_product_kernel GG_A_MASK)
  // e: element index; kLean: rb = the row base's byte offset, o = the lane's
  auto upd = [&](double v, double r, double q, bool ok, int64_t e, int64_t rb,
                 uint32_t o) -> double {
    auto at = [&](double* base) -> double* {
      if constexpr (kLean) return reinterpret_cast<double*>(sbase(base, rb) + o);
      return base + e;
    };
    if (CGP == 3) {
      v = fma(lz_cp, q, fma(lz_cu, r, lz_cy * v));
      if (ok) {
        stg(at(Pout), v);
        rr_acc = fma(v, v, rr_acc);
      }
    } else if (CGP) {
      if (CGP == 2 && cg_qs != 0.0) q = fma(cg_qs, v, q);   // (K + s I) p_old
      if (CGP == 2 && cg_pending) {
        r = r - cg_alpha * q;
        if (ok) {
          stg(at(Rg), r);
          rr_acc = fma(r, r, rr_acc);
        }
      }
      v = cg_first ? r : fma(cg_beta, v, r);
      if (Pout != nullptr && ok) stg(at(Pout), v);
      if (CGP == 2 && pqo_on && ok) pqo_acc = fma(v, q, pqo_acc);
    }
    return v;
  };
  // raw (row i', row m-1-i') -> (u, v) in place
  auto amask = [&](int c, double (&a)[2][kKC], double (&r)[2][kKC], double (&q)[2][kKC]) {
#pragma unroll
    for (int s = 0; s < kKC; ++s) {
      const int k = (c * kKC + s) * 4 + krow;
      const bool okl = bvalid && k < hS;
      const bool okh = bvalid && k < h;   // a distinct mirrored row
      double xl = a[0][s], xh = a[1][s];
      if (CGP) {
        const int64_t t = (int64_t)c * kKC + s;
        xl = upd(xl, r[0][s], q[0][s], okl, (int64_t)k * M + brow, lrow_b(t), loff);
        xh = upd(xh, r[1][s], q[1][s], okh, (int64_t)(m - 1 - k) * M + brow, hrow_b(t), hoff);
      }
      a[0][s] = okl ? (okh ? xl + xh : xl) : 0.0;
      a[1][s] = okh ? xl - xh : 0.0;
    }
  };

  d4 accs[JS], acca[JA];
#pragma unroll
  for (int t = 0; t < JS; ++t) accs[t] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < JA; ++t) acca[t] = d4{0.0, 0.0, 0.0, 0.0};
  double t4s[TS > 0 ? TS : 1], t4a[TA > 0 ? TA : 1];
#pragma unroll
  for (int i = 0; i < (TS > 0 ? TS : 1); ++i) t4s[i] = 0.0;
#pragma unroll
  for (int i = 0; i < (TA > 0 ? TA : 1); ++i) t4a[i] = 0.0;

  double a_cur[2][kKC], a_nxt[2][kKC], r_cur[2][kKC], r_nxt[2][kKC], q_cur[2][kKC],
      q_nxt[2][kKC];
  stage(0);
  aload(0, a_cur, r_cur, q_cur);
  amask(0, a_cur, r_cur, q_cur);
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const bool more = c + 1 < nchunks;
    const int kcn = min(kKC, KS - c * kKC);
    const double* buf = lds + (c & 1) * kBuf + lane;
#pragma unroll
    for (int s = 0; s < kKC; ++s) {
      if ((kOpt & 2) ? s == 0 : (s == 1 || (kKC == 1 && s == 0))) {
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
          stage(c + 1);
          aload(c + 1, a_nxt, r_nxt, q_nxt);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (s < kcn) {
        const double* bs = buf + s * JF * 64;
        const double au = a_cur[0][s], av = a_cur[1][s];
        if (kOpt & 1) __builtin_amdgcn_s_setprio(1);
        // fragment f of the k-step: [S tiles][S tails][T tiles][T tails]
        auto frag = [&](int f, double bv) {
          if (f < FS) {
            if (TS > 0 && f >= JS - 1) {
              const int i = TS > 0 ? f - (JS - 1) : 0;
              t4s[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(au, bv, t4s[i], 0, 0, 0);
            } else {
              accs[f] = __builtin_amdgcn_mfma_f64_16x16x4f64(au, bv, accs[f], 0, 0, 0);
            }
          } else {
            const int g = f - FS;
            if (TA > 0 && g >= JA - 1) {
              const int i = TA > 0 ? g - (JA - 1) : 0;
              t4a[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, t4a[i], 0, 0, 0);
            } else {
              acca[g] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acca[g], 0, 0, 0);
            }
          }
        };
        if constexpr (kBdb) {
          double bc0 = bs[0], bc1 = JF > 1 ? bs[64] : 0.0;
#pragma unroll
          for (int f = 0; f < JF; f += 2) {
            double bn0 = 0.0, bn1 = 0.0;
            if (f + 2 < JF) bn0 = bs[(f + 2) * 64];
            if (f + 3 < JF) bn1 = bs[(f + 3) * 64];
            frag(f, bc0);
            if (f + 1 < JF) frag(f + 1, bc1);
            bc0 = bn0;
            bc1 = bn1;
          }
        } else {
#pragma unroll
        for (int t = 0; t < JS; ++t) {
          if (TS > 0 && t == JS - 1) {
#pragma unroll
            for (int i = 0; i < (TS > 0 ? TS : 1); ++i)
              t4s[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(au, bs[(t + i) * 64], t4s[i], 0, 0, 0);
          } else {
            accs[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(au, bs[t * 64], accs[t], 0, 0, 0);
          }
        }
#pragma unroll
        for (int t = 0; t < JA; ++t) {
          if (TA > 0 && t == JA - 1) {
#pragma unroll
            for (int i = 0; i < (TA > 0 ? TA : 1); ++i)
              t4a[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bs[(FS + t + i) * 64], t4a[i], 0, 0,
                                                          0);
          } else {
            acca[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bs[(FS + t) * 64], acca[t], 0, 0, 0);
          }
        }
        }
        if (kOpt & 1) __builtin_amdgcn_s_setprio(0);
      }
    }
    if (more) {
#pragma unroll
      for (int s = 0; s < kKC; ++s)
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          a_cur[w][s] = a_nxt[w][s];
          if (CGP) r_cur[w][s] = r_nxt[w][s];
          if (CGP >= 2) q_cur[w][s] = q_nxt[w][s];
        }
      amask(c + 1, a_cur, r_cur, q_cur);
    }
    __syncthreads();
  }

  // 4x4x4_4b tails -> the 16x16 layout (see mode_product_kernel kT4); the
  // staged epilogue writes them from their own layout instead
  if (!kStg) {
    const int cc = lane & 15;
    const int src0 = 16 * (lane >> 4) + (lane & 3);
    if (TS > 0) {
#pragma unroll
      for (int rho = 0; rho < 4; ++rho) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < (TS > 0 ? TS : 1); ++i) {
          const double w = __shfl(t4s[i], src0 + 4 * rho, 64);
          if ((cc >> 2) == i) v = w;
        }
        accs[JS - 1][rho] = v;
      }
    }
    if (TA > 0) {
#pragma unroll
      for (int rho = 0; rho < 4; ++rho) {
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < (TA > 0 ? TA : 1); ++i) {
          const double w = __shfl(t4a[i], src0 + 4 * rho, 64);
          if ((cc >> 2) == i) v = w;
        }
        acca[JA - 1][rho] = v;
      }
    }
  }

  // ---- epilogue: D[b][j'] at lane (j' & 15), register r = row 4 r + (l >> 4).
  // Half-tile e = 2 t + w: w = 0 stores S + T at column j' = 16 t + (l & 15)
  // (valid below hS), w = 1 stores S - T at m-1-j' (valid below h).  The wave's
  // 16 x m output block is contiguous: SGPR base + 32-bit lane byte offset.
  const int col = lane & 15;
  const int64_t b0u = (int64_t)__builtin_amdgcn_readfirstlane((int)b0) |
                      ((int64_t)__builtin_amdgcn_readfirstlane((int)(b0 >> 32)) << 32);
  const int rows_left = (int)min<int64_t>(16, M - b0u);
  char* ybase = reinterpret_cast<char*>(Y + b0u * m);
  auto jcol = [&](int e) -> int {
    const int j = (e >> 1) * 16 + col;
    return (e & 1) ? m - 1 - j : j;
  };
  auto col_ok = [&](int e) -> bool {
    const int j = (e >> 1) * 16 + col;
    return (e & 1) ? j < h : j < hS;
  };
  auto boff_of = [&](int r, int e) -> uint32_t {
    return (uint32_t)(((lane >> 4) + 4 * r) * m + jcol(e)) * 8u;
  };
  auto value = [&](int e, int r) -> double {
    const int t = e >> 1;
    const double sv = accs[t][r];
    const double tv = t < JA ? acca[t < JA ? t : 0][r] : 0.0;
    return (e & 1) ? sv - tv : sv + tv;
  };
  double dsum = 0.0, rqsum = 0.0, qqsum = 0.0;
  if (kStg) {
    double* wl = lds + (int64_t)wave * 4 * m;   // this wave's 4 x m image
    const double* __restrict__ er = fz.er;
    const bool rq_on = edots && (kRecomp || er != nullptr);   // null: conjugacy r.q
    double* __restrict__ epo = kRecomp ? fz.ep_out : nullptr;
    const bool first = kRecomp && fz.sc->first != 0;
    const double beta = kRecomp ? fz.sc->beta : 0.0;
    const int rl = lane >> 4;
    static_assert(TS == TA, "staged epilogue: equal S / T tails");
    constexpr int JFULL = JS - (TS > 0 ? 1 : 0);   // 16x16 tiles per half
    constexpr int kU = 4;
    // kOpt bit 8 (GG_FOLD_EPI_PRE=1, opt-in): p of batch t + 1 prefetched
    // (m <= 256: four batches of 64 kUP double2 per 4-row round); spills 6
    // VGPRs at the 3-wave budget, epilogue +0.25 ms (profiles/r04/x_epi_pre)
    constexpr bool kPre = (kOpt & 256) != 0;
    constexpr int kUP = 2;                          // double2 per lane per prefetched batch
    constexpr int kNB = 4;                          // batches per 4-row round (m <= 256)
    static_assert(!kPre || kNB * 64 * kUP * 2 >= 4 * 32 * JS, "prefetch: batches per round");
    double2 pc[kUP], pn[kUP];
    auto pre_fetch = [&](int t, double2 (&pv)[kUP]) {
      const int r = t / kNB, base = (t % kNB) * 64 * kUP;
      const int nr = min(4, max(0, rows_left - 4 * r));
      const int tot2 = (nr * m) >> 1;
      const int64_t g0 = (b0u + 4 * r) * m;
#pragma unroll
      for (int u = 0; u < kUP; ++u) {
        const int i2 = base + lane + 64 * u;
        pv[u] = i2 < tot2 ? ld2<kNTs>(xs + g0 + 2 * (int64_t)i2) : double2{0.0, 0.0};
      }
    };
    if (kPre && !rq_on && xs != nullptr) pre_fetch(0, pc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int t = 0; t < JFULL; ++t) {
        const int j = 16 * t + col;
        const double sv = accs[t][r];
        const double tv = t < JA ? acca[t < JA ? t : 0][r] : 0.0;
        if (j < hS) wl[rl * m + j] = sv + tv;
        if (j < h) wl[rl * m + (m - 1 - j)] = sv - tv;
      }
      if (TS > 0) {
        // 4x4x4_4b D: lane 16 rr + 4 g + c holds row 4 g + rr, column
        // 16 JFULL + 4 i + c of tail i; round r takes the lanes with g == r
        if (((lane >> 2) & 3) == r) {
          const int rr = lane >> 4;
#pragma unroll
          for (int i = 0; i < (TS > 0 ? TS : 1); ++i) {
            const int j = 16 * JFULL + 4 * i + (lane & 3);
            if (j < hS) wl[rr * m + j] = t4s[i] + t4a[i];
            if (j < h) wl[rr * m + (m - 1 - j)] = t4s[i] - t4a[i];
          }
        }
      }
      // a wave's LDS instructions complete in order: the reads below see the
      // writes above (wave-private image, no barrier)
      const int nr = min(4, max(0, rows_left - 4 * r));
      const int tot2 = (nr * m) >> 1;              // double2 of this round (m even)
      const int64_t g0 = (b0u + 4 * r) * m;        // first element (16-B aligned)
      if (!kPre || rq_on || xs == nullptr) {
        for (int base = 0; base < tot2; base += 64 * kU) {
          double2 av[kU], pv[kU], ev[kU];
#pragma unroll
          for (int u = 0; u < kU; ++u) {
            const int i2 = base + lane + 64 * u;
            const bool ok = i2 < tot2;
            const int64_t g = g0 + 2 * (int64_t)i2;
            av[u] = ok ? *reinterpret_cast<const double2*>(wl + 2 * i2) : double2{0.0, 0.0};
            pv[u] = (ok && xs != nullptr) ? ld2<kNTs>(xs + g) : double2{0.0, 0.0};
            ev[u] = (ok && rq_on) ? ld2<kNTs>(er + g) : double2{0.0, 0.0};
          }
#pragma unroll
          for (int u = 0; u < kU; ++u) {
            const int i2 = base + lane + 64 * u;
            if (i2 >= tot2) continue;
            const int64_t g = g0 + 2 * (int64_t)i2;
            if (xs == nullptr) {
              st2<kNTy>(Y + g, av[u]);
              continue;
            }
            double2 p2 = pv[u];
            if (kRecomp) {
              p2.x = first ? ev[u].x : fma(beta, p2.x, ev[u].x);
              p2.y = first ? ev[u].y : fma(beta, p2.y, ev[u].y);
            }
            double2 v;
            v.x = fma(shift, p2.x, av[u].x);
            v.y = fma(shift, p2.y, av[u].y);
            dsum = fma(p2.x, v.x, dsum);
            dsum = fma(p2.y, v.y, dsum);
            if (edots) {
              rqsum = fma(ev[u].x, v.x, rqsum);
              rqsum = fma(ev[u].y, v.y, rqsum);
              qqsum = fma(v.x, v.x, qqsum);
              qqsum = fma(v.y, v.y, qqsum);
            }
            st2<kNTy>(Y + g, v);
            if (kRecomp) st2<kNTy>(epo + g, p2);
          }
        }
        continue;
      }
      // kPre (the conjugacy r.q path: p the only global operand): the p
      // values of the next batch -- the next round's first while this round's
      // last is processed -- are loaded before this batch's arithmetic and
      // stores, so one HBM latency per block is exposed instead of one per
      // batch (CDNA4 retires vmcnt in order, stores included)
#pragma unroll
      for (int b = 0; b < kNB; ++b) {
        const int base = b * 64 * kUP;
        const int t = kNB * r + b;
        if (t + 1 < 4 * kNB) pre_fetch(t + 1, pn);
        if (base < tot2) {
#pragma unroll
          for (int u = 0; u < kUP; ++u) {
            const int i2 = base + lane + 64 * u;
            if (i2 >= tot2) continue;
            const int64_t g = g0 + 2 * (int64_t)i2;
            const double2 av = *reinterpret_cast<const double2*>(wl + 2 * i2);
            const double2 p2 = pc[u];
            double2 v;
            v.x = fma(shift, p2.x, av.x);
            v.y = fma(shift, p2.y, av.y);
            dsum = fma(p2.x, v.x, dsum);
            dsum = fma(p2.y, v.y, dsum);
            if (edots) {
              qqsum = fma(v.x, v.x, qqsum);
              qqsum = fma(v.y, v.y, qqsum);
            }
            st2<kNTy>(Y + g, v);
          }
        }
#pragma unroll
        for (int u = 0; u < kUP; ++u) pc[u] = pn[u];
      }
    }
  } else if (kMap) {
    // rows: a = row / mi, h = (row % mi) / cr, br = (row % mi) % cr; columns
    // grouped by cg (include gg_internal.h OutMap)
    int64_t rowoff[4];
    int rowdest[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = b0 + (lane >> 4) + 4 * r;
      const int64_t a_ = row / om.mi, bi = row - a_ * om.mi;
      const int64_t hh = bi / om.cr, br = bi - hh * om.cr;
      rowoff[r] = a_ * om.as + br * om.cg;
      rowdest[r] = 0;
      if (om.push == 1) rowdest[r] = (int)hh;
      else rowoff[r] += hh * om.hs;
    }
#pragma unroll
    for (int e = 0; e < 2 * JS; ++e) {
      if (!col_ok(e)) continue;
      const int64_t j = jcol(e);
      const int64_t jg = j / om.cg;
      const int64_t co = (j - jg * om.cg) + (om.push == 2 ? 0 : jg * om.gs);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if ((lane >> 4) + 4 * r >= rows_left) continue;
        const double v = value(e, r);
        if (om.push != 0) {
          const int dest = om.push == 1 ? rowdest[r] : (int)jg;
          om.peers[dest][om.self_off + rowoff[r] + co] = v;
        } else {
          Y[rowoff[r] + co] = v;
        }
      }
    }
    // push: the stores went to other GPUs' HBM over xGMI; release them at
    // system scope before the kernel ends (mode_product_kernel mp_finish)
    if (om.push != 0) __threadfence_system();
    return;
  } else if (xs == nullptr) {
#pragma unroll
    for (int e = 0; e < 2 * JS; ++e) {
      const bool cok = col_ok(e);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (cok && (lane >> 4) + 4 * r < rows_left)
          sty(reinterpret_cast<double*>(ybase + boff_of(r, e)), value(e, r));
    }
  } else {
    // shift / dots: the loads of half-tile e + 1 are issued before e's stores
    // (CDNA4 retires vmcnt in order and stores count)
    const double* __restrict__ er = fz.er;
    const bool rq_on = edots && (kRecomp || er != nullptr);
    const char* xbase = reinterpret_cast<const char*>(xs + b0u * m);
    const char* ebase = rq_on ? reinterpret_cast<const char*>(er + b0u * m) : nullptr;
    char* pbase = kRecomp ? reinterpret_cast<char*>(fz.ep_out + b0u * m) : nullptr;
    const bool first = kRecomp && fz.sc->first != 0;
    const double beta = kRecomp ? fz.sc->beta : 0.0;
    double xv[2][4], ev[2][4];
    auto load_e = [&](int e, double (&xo)[4], double (&eo)[4]) {
      const bool cok = col_ok(e);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = cok && (lane >> 4) + 4 * r < rows_left;
        const uint32_t o = boff_of(r, e);
        xo[r] = ok ? *reinterpret_cast<const double*>(xbase + o) : 0.0;
        eo[r] = (ok && rq_on) ? *reinterpret_cast<const double*>(ebase + o) : 0.0;
      }
    };
    load_e(0, xv[0], ev[0]);
#pragma unroll
    for (int e = 0; e < 2 * JS; ++e) {
      const int cb = e & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (e + 1 < 2 * JS) load_e(e + 1, xv[cb ^ 1], ev[cb ^ 1]);
      const bool cok = col_ok(e);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (cok && (lane >> 4) + 4 * r < rows_left) {
          double pv = xv[cb][r];
          if (kRecomp) pv = first ? ev[cb][r] : fma(beta, pv, ev[cb][r]);
          const double v = fma(shift, pv, value(e, r));
          dsum = fma(pv, v, dsum);
          if (edots) {
            rqsum = fma(ev[cb][r], v, rqsum);
            qqsum = fma(v, v, qqsum);
          }
          *reinterpret_cast<double*>(ybase + boff_of(r, e)) = v;
          if (kRecomp) *reinterpret_cast<double*>(pbase + boff_of(r, e)) = pv;
        }
      }
    }
  }
  // the staged epilogue's images occupy the first 4 kWaves m doubles of LDS
  mp_block_sums<kWaves, CGP, edots, false>(dsum, edots ? rqsum : pqo_acc, qqsum, rr_acc,
                                           dot_partials, fz, kStg ? lds + 4 * kWaves * m : lds,
                                           blockIdx.x);
  if (kEpi >= 1) mp_side_job<kThreads, kNTs>(fz, blockIdx.x);
}

// kind (kron_apply's launch kind) -> the folded kernel; kind 5 (fusion
// layout 2) and the tuning variants stay on mode_product_kernel
bool fold_kind(int kind) {
  return kind == 0 || kind == 1 || kind == 2 || kind == 3 || kind == 4 || kind == 6 ||
         kind == 7;
}

// KIND: kron_apply's launch kind; 8 / 9: the sharded operator's mapped
// epilogue without / with the textbook CG prologue (gg_kron_dist_*)
// OPT: kOpt (4 = kLean); KCO > 0 overrides the k-steps per chunk; WV waves
// per workgroup
template <int JT, int TT, int KIND, bool STG = false, int OPT = 0, int KCO = 0, int WV = 4>
static FoldConfig cfg_fold() {
  constexpr int CGP = (KIND == 1 || KIND == 9) ? 1 : KIND == 2 ? 2 : KIND == 7 ? 3 : 0;
  constexpr int EPI = KIND == 3 ? 2 : KIND == 4 ? 1 : KIND == 6 ? 4 : 0;
  constexpr bool MAP = KIND >= 8;
  // the fused / Lanczos prologues hold three operands per row pair: one
  // k-step per chunk keeps them within the 3-wave register budget (A/B at
  // 200^4: 15.7 vs 18.7 ms with two, profiles/r03/j_*)
  constexpr int KC = KCO > 0 ? KCO : CGP >= 2 ? 1 : CGP ? 2 : 3;
  constexpr int JF = 2 * (JT - (TT > 0 ? 1 : 0) + TT);
  // 2 x (JT - 1) full 16x16 accumulators beside the tails: beyond 12 of them
  // (m > 200) three waves per SIMD would spill -- two instead
  constexpr int MINW = ((JT - (TT > 0 ? 1 : 0)) <= 6 && TT <= 1) ? 3 : 2;
  constexpr size_t kB = 2 * (size_t)KC * JF * 64 * sizeof(double);
  // staged epilogue: 4 waves x 4 rows x m (<= 32 JT) doubles + the reduction
  constexpr size_t kS = STG ? ((size_t)4 * WV * 32 * JT + 4 * WV) * sizeof(double) : 0;
  return FoldConfig{
      mode_product_fold_kernel<JT, JT, TT, TT, KC, CGP, MINW, EPI, MAP, OPT, STG, WV>, KC, JF,
      kB > kS ? kB : kS, (OPT & 4) != 0, WV};
}

// kLean kernels, instantiated for the m = 200 shape (JT 7, TT 1): default for
// the plain / side / epilogue launches (kinds 0, 3, 4, 6) when the launch is
// in their range (lean_ok); fused CG at 200^4, interleaved processes:
// 41.25 -> 40.98 ms per iteration (side launches 8.05 -> 7.95 ms, the side
// kernel's 3 spilled VGPRs gone; profiles/r03/ak_lean_cg_ab.jsonl).
// GG_FOLD_LEAN=0 disables them (the clamped kernels every other shape takes).
// Non-temporal masks (round 4, profiles/r04/u_nt, t_pro_nt, zf_lz): the CG
// epilogue's p loads and q stores (8.66-8.76 -> 8.59-8.64 ms), the side
// launches' operand and x-stream accesses (7.89-7.96 -> 7.84-7.89), the
// prologue's operand / r / q_old loads and p_new / r stores (13.90 -> 13.63),
// the Lanczos epilogue's streams (8.54-8.64 -> 8.38-8.47); the other masks,
// an epilogue that prefetches its next p batch, 1 / 2 k-step lean prologues
// and 12-wave side launches measured slower and live in the history.
static int env_int(const char* name, int dflt = 0) {
  const char* e = gg::knob(name);
  return e ? atoi(e) : dflt;
}

static bool lean_kind(int kind, bool staged) {
  return (kind == 0 || kind == 3 || kind == 4 || kind == 6) && !(staged && kind == 4);
}

static FoldConfig lean_cfg(int kind, bool staged) {
  constexpr int JT = 7, TT = 1;
  if (staged) {
    switch (kind) {
      case 3: return cfg_fold<JT, TT, 3, true, 4 | 192>();   // p loads, q stores nt
      case 6: return cfg_fold<JT, TT, 6, true, 4>();
      default: return cfg_fold<JT, TT, 0, true, 4 | 192>();   // shift / dot epilogue nt
    }
  }
  switch (kind) {
    case 3: return cfg_fold<JT, TT, 3, false, 4>();
    case 4: return cfg_fold<JT, TT, 4, false, 4 | 96>();   // operand, x stream nt
    case 6: return cfg_fold<JT, TT, 6, false, 4>();
    default: return cfg_fold<JT, TT, 0, false, 4>();
  }
}

// 12-wave workgroups (one per CU, the B chunks staged once for 192 rows b,
// 1.5 KB row segments): default for the fused-CG prologue of the m = 200
// shape (GG_FOLD_PRO_W=4 restores 4 waves) -- 200^4, interleaved processes:
// prologue 13.58-13.66 -> 13.18-13.21 ms, iteration 40.19-40.42 -> 39.93-39.95
// ms (profiles/r03/an_wide_cg_ab.jsonl), with its operand / r / q_old loads and
// p_new / r stores non-temporal (Y, read by the next launch, a normal store).
// The prologue's r.r partials array is sized for 4-wave blocks and zeroed at
// allocation (gg_cg_create).
static FoldConfig wide_pro_cfg() { return cfg_fold<7, 1, 2, false, 96, 0, 12>(); }

// the staged epilogue (kStg) for the launches whose epilogue reads the fused
// operands (kinds 0 with a shift / dot operand, 3 and 6): measured at 200^4
// the fused-CG epilogue launch 11.7 -> 10.2 ms, while plain-store launches
// lose 0.4 ms to the LDS round trip (profiles/r03/h_bench_stage*.json)
template <int JT, int TT>
static FoldConfig fold_staged_by_kind(int kind, bool lean_ok) {
  if constexpr (JT == 7 && TT == 1)
    if (lean_ok && env_int("GG_FOLD_LEAN", 1) == 1 && lean_kind(kind, true))
      return lean_cfg(kind, true);
  switch (kind) {
    case 3: return cfg_fold<JT, TT, 3, true>();
    case 6: return cfg_fold<JT, TT, 6, true>();
    default: return cfg_fold<JT, TT, 0, true>();
  }
}

bool fold_staged_available(int JT, int TT, int kind) {
  return (kind == 0 || kind == 3 || kind == 6) && JT >= 1 && JT <= 8 &&
         (TT == 0 || JT >= 4);
}

FoldConfig select_fold_staged(int JT, int TT, int kind, bool lean_ok) {
  if (TT == 0) {
    switch (JT) {
      case 1: return fold_staged_by_kind<1, 0>(kind, lean_ok);
      case 2: return fold_staged_by_kind<2, 0>(kind, lean_ok);
      case 3: return fold_staged_by_kind<3, 0>(kind, lean_ok);
      case 4: return fold_staged_by_kind<4, 0>(kind, lean_ok);
      case 5: return fold_staged_by_kind<5, 0>(kind, lean_ok);
      case 6: return fold_staged_by_kind<6, 0>(kind, lean_ok);
      case 7: return fold_staged_by_kind<7, 0>(kind, lean_ok);
      case 8: return fold_staged_by_kind<8, 0>(kind, lean_ok);
      default: break;
    }
  } else {
    switch (JT) {
      case 4: return TT == 1 ? fold_staged_by_kind<4, 1>(kind, lean_ok) : fold_staged_by_kind<4, 2>(kind, lean_ok);
      case 5: return TT == 1 ? fold_staged_by_kind<5, 1>(kind, lean_ok) : fold_staged_by_kind<5, 2>(kind, lean_ok);
      case 6: return TT == 1 ? fold_staged_by_kind<6, 1>(kind, lean_ok) : fold_staged_by_kind<6, 2>(kind, lean_ok);
      case 7: return TT == 1 ? fold_staged_by_kind<7, 1>(kind, lean_ok) : fold_staged_by_kind<7, 2>(kind, lean_ok);
      case 8: return TT == 1 ? fold_staged_by_kind<8, 1>(kind, lean_ok) : fold_staged_by_kind<8, 2>(kind, lean_ok);
      default: break;
    }
  }
  throw Error(GG_ERR_VALUE, "no staged folded kernel for this factor shape");
}

template <int JT, int TT>
static FoldConfig fold_by_kind(int kind, bool lean_ok) {
  if constexpr (JT == 7 && TT == 1) {
    // the fused CG prologue on 12-wave workgroups (GG_FOLD_PRO_W=4: 4 waves)
    if (kind == 2 && env_int("GG_FOLD_PRO_W", 12) == 12) return wide_pro_cfg();
    // the fused Lanczos prologue: 12-wave workgroups with non-temporal
    // streams, as the CG prologue -- 200^4 Lanczos step 34.1-35.1 -> 33.47-33.50
    // ms, prologue 11.9-12.5 -> 11.3 ms, tridiagonal bitwise unchanged
    // (profiles/r04/zf_lz)
    if (kind == 7) return cfg_fold<7, 1, 7, false, 96, 0, 12>();
    if (lean_ok && env_int("GG_FOLD_LEAN", 1) == 1 && lean_kind(kind, false))
      return lean_cfg(kind, false);
  }
  switch (kind) {
    case 8: return cfg_fold<JT, TT, 8>();
    case 9: return cfg_fold<JT, TT, 9>();
    case 1: return cfg_fold<JT, TT, 1>();
    case 2: return cfg_fold<JT, TT, 2>();
    case 3: return cfg_fold<JT, TT, 3>();
    case 4: return cfg_fold<JT, TT, 4>();
    case 6: return cfg_fold<JT, TT, 6>();
    case 7: return cfg_fold<JT, TT, 7>();
    default: return cfg_fold<JT, TT, 0>();
  }
}

FoldConfig select_fold(int JT, int TT, int kind, bool lean_ok) {
  if (TT == 0) {
    switch (JT) {
      case 1: return fold_by_kind<1, 0>(kind, lean_ok);
      case 2: return fold_by_kind<2, 0>(kind, lean_ok);
      case 3: return fold_by_kind<3, 0>(kind, lean_ok);
      case 4: return fold_by_kind<4, 0>(kind, lean_ok);
      case 5: return fold_by_kind<5, 0>(kind, lean_ok);
      case 6: return fold_by_kind<6, 0>(kind, lean_ok);
      case 7: return fold_by_kind<7, 0>(kind, lean_ok);
      case 8: return fold_by_kind<8, 0>(kind, lean_ok);
      default: break;
    }
  } else if (TT == 1 || TT == 2) {
    switch (JT) {
      case 4: return TT == 1 ? fold_by_kind<4, 1>(kind, lean_ok) : fold_by_kind<4, 2>(kind, lean_ok);
      case 5: return TT == 1 ? fold_by_kind<5, 1>(kind, lean_ok) : fold_by_kind<5, 2>(kind, lean_ok);
      case 6: return TT == 1 ? fold_by_kind<6, 1>(kind, lean_ok) : fold_by_kind<6, 2>(kind, lean_ok);
      case 7: return TT == 1 ? fold_by_kind<7, 1>(kind, lean_ok) : fold_by_kind<7, 2>(kind, lean_ok);
      case 8: return TT == 1 ? fold_by_kind<8, 1>(kind, lean_ok) : fold_by_kind<8, 2>(kind, lean_ok);
      default: break;
    }
  }
  throw Error(GG_ERR_VALUE, "no folded kernel for this factor shape");
}

void set_fold_lds_limits() {
  for (int jt = 1; jt <= 8; ++jt)
    for (int tt = 0; tt <= 2; ++tt) {
      if (tt > 0 && jt < 4) continue;
      for (int kind : {0, 3, 6}) {
        const FoldConfig fc = select_fold_staged(jt, tt, kind);
        GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fc.fn),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)fc.lds));
      }
    }
  for (int kind : {0, 3, 4, 6})
    for (bool staged : {false, true}) {
      if (!lean_kind(kind, staged)) continue;
      const FoldConfig fc = lean_cfg(kind, staged);
      GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fc.fn),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)fc.lds));
    }
  {
    const FoldConfig fc = wide_pro_cfg();
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fc.fn),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)fc.lds));
  }
  for (int jt = 1; jt <= 8; ++jt)
    for (int tt = 0; tt <= 2; ++tt) {
      if (tt > 0 && jt < 4) continue;
      for (int kind = 0; kind < 10; ++kind) {
        if (!fold_kind(kind) && kind < 8) continue;
        const FoldConfig fc = select_fold(jt, tt, kind);
        GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fc.fn),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)fc.lds));
      }
    }
}

}  // namespace gg
