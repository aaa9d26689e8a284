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
template <int JS, int TS, int W, int NS, int MINW>
__global__ __launch_bounds__(64 * W, MINW) void mode_product_ring_kernel(
    const double* __restrict__ X, double* __restrict__ Y, const double* __restrict__ Bf,
    int64_t M, int m, int KS, int64_t nblk) {
  constexpr int RB = 16 * W;           // rows b per block
  constexpr int kA = 8 * RB;           // A image doubles per k-step
  constexpr int kB = 16 * 64;          // B image doubles per k-step (16 fragments)
  constexpr int kStage = kA + kB;
  constexpr int kBw = 8 / W;           // B DMAs per wave per stage
  constexpr int LW = 1 + kBw;          // DMAs per wave per stage
  constexpr int kE = 4 * JS;           // epilogue stores per wave per block
  constexpr int Y0 = (NS - 2) * LW;    // younger ops at a stage's wait
  constexpr int YE = Y0 + kE;          // ... with an epilogue since its DMAs
  constexpr int FS = JS - (TS > 0 ? 1 : 0) + TS;
  constexpr int NF = 2 * FS;
  static_assert(W == 4 || W == 8, "one A DMA per wave: W KiB of A per k-step");
  static_assert(NF <= 16, "16 fragment slots per k-step");
  static_assert(NS >= 3 && YE <= 63 && (NS - 1) * LW <= 63,
                "ring depth outside the counted-vmcnt range");
  extern __shared__ __attribute__((aligned(16))) double lds[];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c16 = lane & 15, krow = lane >> 4;
  const int h = m >> 1;
  const int64_t G = gridDim.x;
  const int64_t nmine = (nblk - (int64_t)blockIdx.x + G - 1) / G;   // grid <= nblk
  const int nst = (int)(nmine * KS);

  // this wave's 1 KiB piece of the A image: 128 doubles from row arow, column acol
  const int ao = wave * 128 + 2 * lane;
  const int arow = ao / RB, acol = ao % RB;

  // issue cursor: the next k-step (block it, step s) to stage
  int64_t i_it = 0;
  int i_s = 0;
  auto issue_stage = [&](int slot) {
    double* st = lds + slot * kStage;
    // past this workgroup's last block the DMAs re-read a valid block
    // (never consumed): every wave issues LW DMAs per stage, always
    const int64_t it = i_it < nmine ? i_it : nmine - 1;
    const int64_t blk = (int64_t)blockIdx.x + it * G;
    int64_t b = blk * RB + acol;
    if (b > M - 2) b = M - 2;
    const int s = i_s;
    const int row = arow < 4 ? 4 * s + arow : m - 1 - 4 * s - (arow - 4);
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(X + (int64_t)row * M + b),
        (__attribute__((address_space(3))) void*)(st + wave * 128), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < kBw; ++j) {
      const int p = wave * kBw + j;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(Bf + (int64_t)s * kB + p * 128 +
                                                          2 * lane),
          (__attribute__((address_space(3))) void*)(st + kA + p * 128), 16, 0, 0);
    }
    if (++i_s == KS) {
      i_s = 0;
      ++i_it;
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
  auto read_stage = [&](int slot, double (&op)[NF + 2]) {
    const double* st = lds + slot * kStage;
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
#pragma unroll
    for (int t = 0; t < JS; ++t)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int rp = 0; rp < 4; rp += 2) {
          const double va = hf ? accs[t][rp] - acca[t][rp] : accs[t][rp] + acca[t][rp];
          const double vb =
              hf ? accs[t][rp + 1] - acca[t][rp + 1] : accs[t][rp + 1] + acca[t][rp + 1];
          // even lanes store row rp with the odd neighbour's va, odd lanes
          // row rp + 1 with the even neighbour's vb
          const double w = swap_adjacent(odd ? va : vb);
          const int j = 16 * t + ce;   // the pair's first column (S + T half)
          const int64_t row = b0 + 4 * (rp + (odd ? 1 : 0)) + krow;
          double2 o;
          if (hf == 0) {
            o.x = odd ? w : va;
            o.y = odd ? vb : w;
          } else {   // S - T at m - 1 - j: the pair (m - 2 - j, m - 1 - j) swapped
            o.x = odd ? vb : w;
            o.y = odd ? w : va;
          }
          const int64_t col = hf ? (int64_t)(m - 2 - j) : (int64_t)j;
          double* dst = (j < h && row < M) ? Y + row * m + col : g_ring_trash + 2 * lane;
          *reinterpret_cast<double2*>(dst) = o;
        }
  };

#pragma unroll
  for (int q = 0; q < NS; ++q) issue_stage(q);
  wait_vm<(NS - 1) * LW>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  double cur[NF + 2], nxt[NF + 2];
  read_stage(0, cur);
  zero();
  int64_t c_it = 0;
  int c_s = 0;
  int last_ep = -(1 << 30);   // step whose compute ran the latest epilogue
  for (int c = 0; c < nst; ++c) {
    __builtin_amdgcn_sched_barrier(0);
    // stage c + 1 landed (the DMAs of c + 2 .. c + NS - 1 stay in flight, plus
    // an epilogue's stores if one ran after stage c + 1's DMAs were issued),
    // and this wave's reads of stage c are back in registers
    if (last_ep >= c + 1 - NS)
      wait_vm<YE>();
    else
      wait_vm<Y0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) only (vmcnt 63, expcnt 7)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue_stage(c % NS);   // stage c + NS into the slot stage c came from
    if (c + 1 < nst) read_stage((c + 1) % NS, nxt);
    __builtin_amdgcn_sched_barrier(0);
    mma(cur);
    if (++c_s == KS) {
      epilogue(c_it);
      zero();
      c_s = 0;
      ++c_it;
      last_ep = c;
    }
#pragma unroll
    for (int f = 0; f < NF + 2; ++f) cur[f] = nxt[f];
  }
  // no DMA may still be writing this workgroup's LDS when it exits
  wait_vm<0>();
}

template <int JS, int TS, int W, int NS, int MINW>
static RingConfig cfg_ring() {
  return RingConfig{mode_product_ring_kernel<JS, TS, W, NS, MINW>, W, NS, 1,
                    (size_t)NS * (8 * 16 * W + 16 * 64) * sizeof(double)};
}

// variants (GG_FOLD_RING=<v>): 1 = 8 waves, 9 stages (144 KiB, one workgroup
// per CU, two waves per SIMD); 2 = 8 waves, 6 stages (96 KiB); 3 = 4 waves,
// 6 stages (72 KiB, two per CU); 4 = 8 waves, 7 stages (112 KiB); 5 = 8
// waves, 5 stages (80 KiB)
static RingConfig ring_variant(int v) {
  switch (v) {
    case 2: return cfg_ring<7, 1, 8, 6, 2>();
    case 3: return cfg_ring<7, 1, 4, 6, 2>();
    case 4: return cfg_ring<7, 1, 8, 7, 2>();
    case 5: return cfg_ring<7, 1, 8, 5, 2>();
    default: return cfg_ring<7, 1, 8, 9, 2>();
  }
}

int ring_variant_env() {
  const char* e = getenv("GG_FOLD_RING");
  return e ? atoi(e) : 0;
}

bool ring_available(int JT, int TT, int64_t m) {
  return JT == 7 && TT == 1 && m % 8 == 0 && m / 2 == 100;
}

RingConfig select_ring(int JT, int TT, int variant) {
  GG_REQUIRE(JT == 7 && TT == 1, GG_ERR_VALUE, "no ring kernel for this factor shape");
  return ring_variant(variant);
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
  for (int v = 1; v <= 5; ++v) {
    const RingConfig rc = ring_variant(v);
    GG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(rc.fn),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)rc.lds));
  }
}

}  // namespace gg
