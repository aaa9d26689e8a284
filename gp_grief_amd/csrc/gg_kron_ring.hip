// The folded (centrosymmetric) Kronecker mode product as a persistent,
// LDS-DMA ring-pipelined kernel: the plain launch kind of gg_kron_fold.hip
// with the chunk-barrier drain removed.
//
// Reference: KronMatrix.kronvec_prod, gp_grief/tensors/kron_matrix.py:52-97
// (each factor one BLAS3 product); the even/odd split and this pipeline are
// execution details of that product.
//
// Why: mode_product_fold_kernel stages its B chunks by global_load_lds and
// its A rows into registers, then ends every chunk in __syncthreads -- with a
// DMA in flight that is s_waitcnt vmcnt(0) + s_barrier, so each chunk waits
// out the full HBM latency of the next chunk's rows (SQ counters: MFMA busy
// ~58 %, profiles/r03/ap_plain_sq_counters.jsonl).  Here both operands move
// global -> LDS by LDS-DMA into a ring of NS stages, each stage retired by a
// counted s_waitcnt vmcnt (never 0 in the loop) and one raw s_barrier, so
// NS - 2 stages stay in flight across every barrier; and the workgroups are
// persistent (one or two per CU, walking blocks b = blockIdx.x + i gridDim.x)
// with the ring running straight across block boundaries, so no block pays a
// pipeline fill.
//
// Decomposition (as mode_product_fold_kernel): Y[b, j] = sum_i X[i, b] F[j, i]
// with X q x M, Y M x m; a block is RB = 16 W rows b, wave w owns rows
// 16 w .. 16 w + 15 of it and every output column.  k-step s covers the low
// rows i' = 4 s .. 4 s + 3 and the mirrored high rows m - 1 - i'; its LDS
// image is [8 rows][RB] of X (one 1 KiB DMA per wave: 8 RB doubles = W KiB)
// followed by the step's 16 B fragments (14 used: [S tiles][S tail][T tiles]
// [T tail], two zero pads so every wave issues the same DMA count; packed by
// gg_kron.hip pack_fold into Factor::rfrag).  Lane l forms u = x_lo + x_hi,
// v = x_lo - x_hi from two ds_read_b64 and feeds the S accumulators with u and
// the T accumulators with v (v_mfma_f64_16x16x4_f64, the 4 tail columns of
// each half on v_mfma_f64_4x4x4_4b_f64).
//
// Epilogue per block: S + T at column j', S - T at m - 1 - j'.  Adjacent
// lanes swap one value (DPP quad_perm [1,0,3,2]) so that every lane stores
// two adjacent columns of one row as 16 bytes: 4 JS store instructions per
// wave and block, each issued with the full exec mask (out-of-range lanes
// store to g_ring_trash).  That makes every wave's vector-memory count per
// stage a compile-time constant, which the counted waits need: the stores of
// an epilogue sit between the DMAs of the stages they separate.
//
// Requirements (kron_apply checks): m even with h = m / 2 a multiple of 4
// (no partial k-step, every row pair distinct), M even and >= 2, X and Y
// 16-byte aligned, no fused operands (launch kind 0).
#include "gg_mp.h"

namespace gg {

// junk target of the epilogue's out-of-range lanes (one 16-byte slot per lane)
__device__ __attribute__((aligned(16))) double g_ring_trash[128];

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt holds 6 bits");
  // vmcnt N (bits 3:0 and 15:14), expcnt 7 and lgkmcnt 15 = no wait
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// a 16-byte store through an explicit global (not generic / flat) pointer
__device__ __forceinline__ void gstore2(void* p, double2 v) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  *reinterpret_cast<__attribute__((address_space(1))) dv2*>(reinterpret_cast<uintptr_t>(p)) =
      dv2{v.x, v.y};
}

// the value of the neighbouring lane (lane ^ 1), DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ double swap_adjacent(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// JS: 16-wide tiles per half (the last holds TS 4x4x4_4b tail fragments when
// TS > 0); W waves per workgroup; NS ring stages of one k-step; MINW waves per
// SIMD the register budget is built for.
//
// Schedule of step c (stage c's operands already in registers, read during
// step c - 1): wait for this wave's DMAs of stage c + 1 (counted vmcnt) and
// its reads of stage c (lgkmcnt 0); barrier -- every wave's stage c + 1 has
// landed and nobody reads stage c's slot any more; issue stage c + NS into
// that slot; read stage c + 1's operands into the second register set; the
// step's MFMAs on the first.  So the MFMAs never wait on LDS latency, and
// NS - 1 stages are in flight across every barrier.
template <int JS, int TS, int W, int NS, int MINW, int KC>
__global__ __launch_bounds__(64 * W, MINW) void mode_product_ring_kernel(
    const double* __restrict__ X, double* __restrict__ Y, const double* __restrict__ Bf,
    int64_t M, int m, int KS, int64_t nblk, const int* __restrict__ skip, MpFuse fz) {
  constexpr int RB = 16 * W;           // rows b per block
  constexpr int kA = 8 * RB;           // A image doubles per k-step
  constexpr int kB = 16 * 64;          // B image doubles per k-step (16 fragments)
  constexpr int kStep = kA + kB;
  constexpr int kStage = KC * kStep;   // a stage: KC k-steps
  constexpr int kBw = 8 / W;           // B DMAs per wave per k-step
  constexpr int LW = KC * (1 + kBw);   // DMAs per wave per stage
  constexpr int kE = 4 * JS;           // epilogue stores per wave per block
  // younger ops at a stage's wait: the DMAs of NS - 3 stages
  constexpr int Y0 = (NS - 3) * LW;
  constexpr int YE = Y0 + kE;          // ... with an epilogue since its DMAs
  constexpr int FS = JS - (TS > 0 ? 1 : 0) + TS;
  constexpr int NF = 2 * FS;
  static_assert(W == 4 || W == 8, "one A DMA per wave: W KiB of A per k-step");
  static_assert(NF <= 16, "16 fragment slots per k-step");
  static_assert(KC == 1 || KC == 2, "one or two k-steps per stage");
  static_assert(NS >= 4 && YE <= 63 && (NS - 2) * LW <= 63,
                "ring depth outside the counted-vmcnt range");
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (skip != nullptr && *skip) return;   // converged CG: every launch a no-op

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, krow = lane >> 4;
  const int h = m >> 1;
  const int64_t G = gridDim.x;
  const int64_t nmine = (nblk - (int64_t)blockIdx.x + G - 1) / G;   // grid <= nblk
  const int nst = (int)(nmine * KS);

  // this wave's 1 KiB piece of the A image: 128 doubles from image row arow,
  // column acol.  W = 8: one row per wave; W = 4: lanes 32..63 take the next
  // row (the same half, so its X row is one row further in that half's order)
  const int ao = wave * 128 + 2 * lane;
  const int arow = ao / RB, acol = ao % RB;
  const int arow0 = (wave * 128) / RB;   // the wave's first image row (uniform)
  const int64_t drow = (int64_t)(arow - arow0) * (arow0 < 4 ? M : -M) * 8;
  // the wave-uniform part of every DMA address goes through readfirstlane
  // (SGPRs, scalar 64-bit arithmetic); lanes add a byte offset
  auto sbase = [](const void* p, int64_t off) -> const char* {
    const uint64_t v = reinterpret_cast<uint64_t>(p) + (uint64_t)off;
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t u = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const char*>(((uint64_t)u << 32) | l);
  };
  const int64_t row_step = (int64_t)4 * M * 8;   // bytes between k-steps' rows
  const uint32_t b_loff = (uint32_t)(2 * lane * 8);

  // issue cursor: the next k-step (block it, step s) to stage; a_off = byte
  // offset of this wave's first A row segment at that step (uniform), a_loff
  // = the lane's byte offset from it (column clamped in a partial last block)
  int64_t i_it = 0;
  int i_s = 0;
  int64_t a_off = 0;
  int64_t a_loff = 0;
  auto block_start = [&] {
    // past this workgroup's last block the DMAs re-read a valid block (never
    // consumed): every wave issues LW DMAs per stage, always
    const int64_t it = i_it < nmine ? i_it : nmine - 1;
    const int64_t b0 = ((int64_t)blockIdx.x + it * G) * RB;
    const int row0 = arow0 < 4 ? arow0 : m - 1 - (arow0 - 4);
    a_off = ((int64_t)row0 * M + b0) * 8;
    const int64_t room = M - 2 - b0;   // the last valid pair start in this block
    a_loff = drow + (acol <= room ? acol : room) * 8;
  };
  block_start();
  // the next stage's DMA sources, prepared (with the cursor's branches)
  // outside the MFMA region so that the DMAs issue branch-free inside it
  int64_t na_off[KC], nb_off[KC], na_loff[KC];
  auto prep_stage = [&] {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      na_off[k] = a_off;
      na_loff[k] = a_loff;
      nb_off[k] = (int64_t)i_s * kB * 8;
      if (++i_s == KS) {
        i_s = 0;
        ++i_it;
        block_start();
      } else {
        a_off += arow0 < 4 ? row_step : -row_step;
      }
    }
  };
  auto issue_prepped = [&](int slot) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      double* st = lds + slot * kStage + k * kStep;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(sbase(X, na_off[k]) + na_loff[k]),
          (__attribute__((address_space(3))) void*)(st + wave * 128), 16, 0, 0);
#pragma unroll
      for (int j = 0; j < kBw; ++j) {
        const int p = wave * kBw + j;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(
                sbase(Bf, nb_off[k] + (int64_t)p * 128 * 8) + b_loff),
            (__attribute__((address_space(3))) void*)(st + kA + p * 128), 16, 0, 0);
      }
    }
  };

  d4 accs[JS], acca[JS];
  double t4s[TS > 0 ? TS : 1], t4a[TS > 0 ? TS : 1];
  auto zero = [&] {
#pragma unroll
    for (int t = 0; t < JS; ++t) {
      accs[t] = d4{0.0, 0.0, 0.0, 0.0};
      acca[t] = d4{0.0, 0.0, 0.0, 0.0};
    }
#pragma unroll
    for (int i = 0; i < (TS > 0 ? TS : 1); ++i) t4s[i] = t4a[i] = 0.0;
  };

  // a stage's operands: the two raw rows and the 2 FS B fragments
  // k-step g's operands (stage g / KC, step g % KC of it)
  auto read_step = [&](int g, double (&op)[NF + 2]) {
    const double* st = lds + ((g / KC) % NS) * kStage + (g % KC) * kStep;
    op[0] = st[krow * RB + wave * 16 + c16];
    op[1] = st[(4 + krow) * RB + wave * 16 + c16];
    const double* bs = st + kA + lane;
#pragma unroll
    for (int f = 0; f < NF; ++f) op[2 + f] = bs[f * 64];
  };
  auto mma = [&](const double (&op)[NF + 2]) {
    const double u = op[0] + op[1], v = op[0] - op[1];
#pragma unroll
    for (int t = 0; t < JS; ++t) {
      if (TS > 0 && t == JS - 1) {
#pragma unroll
        for (int i = 0; i < (TS > 0 ? TS : 1); ++i)
          t4s[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(u, op[2 + t + i], t4s[i], 0, 0, 0);
      } else {
        accs[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(u, op[2 + t], accs[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < JS; ++t) {
      if (TS > 0 && t == JS - 1) {
#pragma unroll
        for (int i = 0; i < (TS > 0 ? TS : 1); ++i)
          t4a[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(v, op[2 + FS + t + i], t4a[i], 0, 0, 0);
      } else {
        acca[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(v, op[2 + FS + t], acca[t], 0, 0, 0);
      }
    }
  };

  auto epilogue = [&](int64_t it) {
    // 4x4x4_4b tails -> the 16x16 layout (mode_product_fold_kernel)
    if (TS > 0) {
      const int src0 = 16 * (lane >> 4) + (lane & 3);
#pragma unroll
      for (int rho = 0; rho < 4; ++rho) {
        double vs = 0.0, va = 0.0;
#pragma unroll
        for (int i = 0; i < (TS > 0 ? TS : 1); ++i) {
          const double ws = __shfl(t4s[i], src0 + 4 * rho, 64);
          const double wa = __shfl(t4a[i], src0 + 4 * rho, 64);
          if ((c16 >> 2) == i) {
            vs = ws;
            va = wa;
          }
        }
        accs[JS - 1][rho] = vs;
        acca[JS - 1][rho] = va;
      }
    }
    const int64_t b0 = ((int64_t)blockIdx.x + it * G) * RB + wave * 16;
    const bool odd = (lane & 1) != 0;
    const int ce = c16 & ~1;
    // even lanes store row rp with the odd neighbour's va, odd lanes row
    // rp + 1 with the even neighbour's vb: (x, y) of the 16-byte pair
    auto pair = [&](int t, int hf, int rp) -> double2 {
      const double va = hf ? accs[t][rp] - acca[t][rp] : accs[t][rp] + acca[t][rp];
      const double vb = hf ? accs[t][rp + 1] - acca[t][rp + 1] : accs[t][rp + 1] + acca[t][rp + 1];
      const double w = swap_adjacent(odd ? va : vb);
      double2 o;
      if (hf == 0) {
        o.x = odd ? w : va;
        o.y = odd ? vb : w;
      } else {   // S - T at m - 1 - j: the pair (m - 2 - j, m - 1 - j) swapped
        o.x = odd ? vb : w;
        o.y = odd ? w : va;
      }
      return o;
    };
    if (b0 + 16 <= M) {
      // full strip: the wave's 16 x m output block is contiguous -- SGPR base
      // + 32-bit lane offsets, the tile offset in the instruction; only the
      // tail tile's pairs past column h are masked (lanes 0..3 of every row
      // group stay active, so no store is ever skipped)
      const char* y0 = sbase(Y, b0 * m * 8);
      const char* y2 = sbase(Y, (b0 + 8) * m * 8);
      const uint32_t rowoff = (uint32_t)(((odd ? 4 : 0) + krow) * m * 8);
      uint32_t off0 = rowoff + (uint32_t)(ce * 8);
      uint32_t off1 = rowoff + (uint32_t)((m - 2 - ce) * 8);
      // opaque here: the per-tile offsets fold into each store's immediate
      // instead of being hoisted out of the k-loop as live registers
      asm volatile("" : "+v"(off0), "+v"(off1));
#pragma unroll
      for (int t = 0; t < JS; ++t)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int rp = 0; rp < 4; rp += 2) {
            const double2 o = pair(t, hf, rp);
            const char* yb = rp ? y2 : y0;
            const uint32_t off = hf ? off1 - 128 * t : off0 + 128 * t;
            if (t < JS - 1 || 16 * t + ce < h) gstore2(const_cast<char*>(yb) + off, o);
            // one pair at a time: the accumulators die as they are stored
            __builtin_amdgcn_sched_barrier(0);
          }
      return;
    }
    // partial strip (the last block only): per-store bounds, out-of-range
    // lanes to g_ring_trash so every store still issues
    int ceo = ce;
    asm volatile("" : "+v"(ceo));   // keep the per-tile addresses out of the k-loop
#pragma unroll
    for (int t = 0; t < JS; ++t)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int rp = 0; rp < 4; rp += 2) {
          const double2 o = pair(t, hf, rp);
          const int j = 16 * t + ceo;   // the pair's first column (S + T half)
          const int64_t row = b0 + 4 * (rp + (odd ? 1 : 0)) + krow;
          const int64_t col = hf ? (int64_t)(m - 2 - j) : (int64_t)j;
          double* dst = (j < h && row < M) ? Y + row * m + col : g_ring_trash + 2 * lane;
          gstore2(dst, o);
          __builtin_amdgcn_sched_barrier(0);
        }
  };

#pragma unroll
  for (int q = 0; q < NS - 1; ++q) {
    prep_stage();
    issue_prepped(q);
  }
  prep_stage();
  wait_vm<(NS - 3) * LW>();   // stages 0 and 1
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  double opa[NF + 2], opb[NF + 2];
  read_step(0, opa);
  zero();
  int64_t c_it = 0;
  int c_s = 0;
  int last_ep = -(1 << 30);   // stage whose compute ran the latest epilogue
  // k-step c: MFMAs on `cur` (its operands, read during step c - 1), the
  // reads of step c + 1 into `nxt`; the first step of stage j also retires
  // stage j + 1 and refills stage j - 1's slot with stage j + NS - 1.  The
  // DMAs and LDS reads are interleaved between the step's MFMAs, so they
  // issue while the matrix core works.
  auto step = [&](int c, double (&cur)[NF + 2], double (&nxt)[NF + 2], bool first) {
    const int j = c / KC;
    if (first) {
      __builtin_amdgcn_sched_barrier(0);
      // stage j + 1 landed (stages j + 2 .. j + NS - 2 stay in flight, plus an
      // epilogue's stores if one ran after stage j + 1's DMAs were issued) and
      // this wave's reads are back in registers
      if (last_ep >= j - NS + 2)
        wait_vm<YE>();
      else
        wait_vm<Y0>();
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) only (vmcnt 63, expcnt 7)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // nobody reads stage j - 1 any more: its slot takes stage j + NS - 1
      issue_prepped((j + NS - 1) % NS);
    }
    // past the last step this reads a landed slot's stale operands (unused)
    read_step(c + 1, nxt);
    mma(cur);
    // interleave: after the u / v adds, one MFMA then up to two other
    // instructions (LDS reads, DMAs, scalar / vector address work)
    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
#pragma unroll
    for (int i = 0; i < 2 * FS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100 | 0x020 | 0x004 | 0x002, 2, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (first) prep_stage();
    if (++c_s == KS) {
      epilogue(c_it);
      zero();
      c_s = 0;
      ++c_it;
      last_ep = j;
    }
  };
  int c = 0;
  for (; c + 1 < nst; c += 2) {
    step(c, opa, opb, true);
    step(c + 1, opb, opa, KC == 1);
  }
  if (c < nst) step(c, opa, opb, true);
  // no DMA may still be writing this workgroup's LDS when it exits
  wait_vm<0>();
}

// The configuration (A/B in profiles/r04/h_ring_ab.jsonl, 200^4 plain
// launch interleaved in one process: chunked kernel 6.69-6.83 ms, 8 waves x 9
// one-k-step stages 6.60-6.68, 4 two-k-step stages 6.45-6.50, the same with
// the DMAs and LDS reads interleaved between the MFMAs 6.36-6.42): 8 waves,
// 4 stages of two k-steps, interleaved.  The other shapes of that table (4
// waves, 5-9 stages, no interleave), the timing-only ablations of
// profiles/r04/f_ring_ablate.jsonl and the side-job carrier (8.6 vs 8.2 ms
// per side launch, profiles/r04/j_side_ab.txt) were measured slower and live
// in the history (round 4).
static RingConfig ring_config() {
  constexpr int JS = 7, TS = 1, W = 8, NS = 4, MINW = 2, KC = 2;
  return RingConfig{mode_product_ring_kernel<JS, TS, W, NS, MINW, KC>, W, NS, KC,
                    (size_t)NS * KC * (8 * 16 * W + 16 * 64) * sizeof(double)};
}

int ring_variant_env() {
  const char* e = gg::knob("GG_FOLD_RING");   // unset / nonzero: the ring; 0: off (A/B)
  return e ? atoi(e) : 1;
}

bool ring_available(int JT, int TT, int64_t m) {
  return JT == 7 && TT == 1 && m % 8 == 0 && m / 2 == 100;
}

RingConfig select_ring(int JT, int TT) {
  GG_REQUIRE(JT == 7 && TT == 1, GG_ERR_VALUE, "no ring kernel for this factor shape");
  return ring_config();
}

int ring_grid(const RingConfig& rc, int cus, int64_t nblk) {
  int per = 0;
  GG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(rc.fn),
                                                      64 * rc.waves, rc.lds));
  GG_REQUIRE(per >= 1, GG_ERR_RUNTIME, "ring kernel does not fit a CU");
  const int64_t g = std::min<int64_t>(nblk, (int64_t)cus * per);
  return (int)g;
}

void set_ring_lds_limits() {
  const RingConfig rc = ring_config();
  GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(rc.fn),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)rc.lds));
}

}  // namespace gg
