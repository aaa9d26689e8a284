// Internal helpers shared by the gp_grief_amd HIP translation units.
// Not part of the C ABI (that is include/gp_grief_amd.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/gp_grief_amd.h"

namespace gg {

// Error carried from the implementation to the C ABI boundary, where it is
// turned into a status code and a thread-local message (gg_last_error).
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define GG_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      throw ::gg::Error(GG_ERR_RUNTIME, std::string("HIP error '") +              \
                                           hipGetErrorString(e_) + "' at " +     \
                                           __FILE__ + ":" + std::to_string(__LINE__) + \
                                           " in " #expr);                         \
  } while (0)

#define GG_REQUIRE(cond, code, msg)                 \
  do {                                              \
    if (!(cond)) throw ::gg::Error((code), (msg));  \
  } while (0)

// Run `body` and convert any exception into a GG status code.
template <class F>
int guard(F&& body) {
  try {
    body();
    return GG_OK;
  } catch (const Error& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("host allocation failed");
    return GG_ERR_RUNTIME;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return GG_ERR_RUNTIME;
  }
}

inline hipStream_t as_stream(gg_stream s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-error check after a kernel launch (no synchronisation).
#define GG_LAUNCH_CHECK() GG_HIP(hipGetLastError())

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- device scalar block shared by the Krylov drivers (CG / Lanczos) ----
constexpr int kXWinMax = 8;       // x_defer mode 3: the largest window
constexpr int kXWinDefault = 8;   // and the default (GG_CG_XWIN; profiles/r06/b_win)
struct CgScalars {
  double rho;       // r.r of the current residual
  double rho_prev;  // r.r of the previous residual
  double pq;        // p.(A p)
  double alpha;
  double beta;
  double tol;       // stop when sqrt(rho) < tol
  double bnorm;
  int iters;        // completed iterations
  int done;         // 1 = converged / stopped: every kernel becomes a no-op
  int first;        // 1 = next p-update is p = r
  int pending;      // fused CG: x += alpha p, r -= alpha q not yet applied
  double rq, qq;    // fused CG: r.q and q.q of the last matvec
  int repair;       // fused CG: |r - alpha q|^2 cancelled; apply x / r and take the
                    // textbook beta before the next matvec
  // fused CG with the x update deferred (gg_vec.hip, x_defer): x lags by
  // xpend steps, x_true = x + sum_{i < xpend} xc[i] xp[i]; the side job folds
  // both into x when xpend == 2, the closing update whatever is left
  int xpend;
  double xc[2];
  const double* xp[2];
  // x_defer mode 2 (balanced): the pair (xc, xp) completed two iterations ago
  // is applied half of x per iteration -- xh = the half the next side job
  // takes (2: none active); a completed step waiting for its partner is
  // (xsc, xsp) when xs
  int xh;
  int xs;
  double xsc;
  const double* xsp;
  int cancels;      // fused CG: cancelled betas so far (repaired, or restarted by
                    // a sharded rank / GG_CG_RESTART)
  double cancel_tol;  // the cancellation test's threshold (0: 1e-6; set once per
                      // handle from GG_CG_CANCEL_TOL, a test switch)
  // x_defer mode 3 (window, block-basis CG): x is cut into wk regions; every
  // iteration's side job brings ONE region up to date with the steps it has
  // not seen (at most wk: region r is visited every wk iterations), so an
  // iteration moves x once per wk iterations and every direction once --
  // (wk + 2) / wk passes instead of 2.  Step i (alpha_i, p_i) sits in ring slot
  // i % (wk + 1) of (wc, wp); the host keeps wk + 1 direction buffers.
  int wk;           // window (0: off)
  int wn;           // steps with a known alpha
  int wnext;        // next region to arm (round robin)
  int warm;         // a side job is armed for the next pair launch
  int wa[kXWinMax];            // steps applied per region
  double wc[kXWinMax + 1];
  const double* wp[kXWinMax + 1];
  // the armed side job: region sreg, x += sum_{t < scnt} scoef[t] sdir[t]
  int sreg, scnt;
  double scoef[kXWinMax];
  const double* sdir[kXWinMax];
  // derived r (block-basis CG with the window, round 6): the prologue does
  // not keep r; r_{j-1} = p_{j-1} - beta_p p_{j-2} from the two directions
  // the window's ring holds (beta_p: the beta that formed the current
  // direction) unless rstored -- r is in its buffer (start, repair, close)
  double beta_p;
  int rstored;
  // the last two directions the recurrence formed (recorded by the scalars
  // of every iteration that ran: the host keeps rotating its buffers through
  // the skipped iterations after convergence, these do not move)
  const double* rp_cur;
  const double* rp_prev;
};

// Fusions carried by one mode-product launch (gg_kron.hip).  Every pointer is
// optional (nullptr = off); kron_apply hands each field to the launch it
// belongs to.
struct MpFuse {
  // CG prologue of the first mode product: X holds p_old, the MFMA A operand
  // is p_new = r + beta p_old (r = b on the first iteration), written to
  // p_out (== X in place for the textbook recurrence).  Fused recurrence
  // (q_old != nullptr): when sc->pending, first r -= alpha q_old (written
  // back) and the block's partial r.r goes to rr_part.
  double* r = nullptr;
  const double* q_old = nullptr;
  // q_old holds K p_old without the shift (sharded fused CG, whose post pass
  // then only reads): the prologue uses q_old + qshift * p_old (0 = off)
  double qshift = 0.0;
  double* p_out = nullptr;
  const CgScalars* sc = nullptr;
  double* rr_part = nullptr;
  // rr_part holds rr_cap partials per half (the prologue launch's workgroup
  // count must not exceed it: kron_apply checks), and kron_apply reports the
  // launch's actual workgroup count through pro_blocks (host memory), so the
  // consumers sum exactly the partials this launch wrote
  int64_t rr_cap = 0;
  int64_t* pro_blocks = nullptr;
  // conjugacy r.q (gg_cg_set_rq 1): the CG prologue also writes block partials
  // of p_new.q_old to rr_part[pqo_stride + blk] (0 = off), and the last epilogue
  // gets er == nullptr -- r_j.q_j = p_j.q_j - beta_j p_j.q_{j-1} (A symmetric)
  // replaces the epilogue's pass over r
  int64_t pqo_stride = 0;
  // side job of the second mode product (fused CG): x += alpha p_side over
  // this workgroup's slice [blk * schunk, (blk + 1) * schunk) of sn elements
  double* sx = nullptr;
  const double* sp = nullptr;
  int64_t sn = 0, schunk = 0;
  // x_defer: the side job applies sc->xc / sc->xp (at element offset soff of
  // the slice) when sc->xpend == 2, instead of alpha p_side when pending.
  // xdefer 2: the slice is [soff, soff + sn) of x for half sc->xh == 0 and
  // [soff_h1, soff_h1 + sn_h1) for half 1 (sx / sp are then x / p at offset 0)
  // xdefer 3 (window, block basis, pair launch only): the side job the scalars
  // armed in sc (sreg, scnt, scoef, sdir) over region sreg of xwin regions
  int xdefer = 0;
  int xwin = 0;
  int64_t soff = 0;
  int64_t soff_h1 = 0, sn_h1 = 0;
  // output of the first mode product when the ping-pong would put it in y
  // (odd d): the fused prologue still reads q_old == y in other workgroups
  double* first_dst = nullptr;
  // last mode product: partial r.q and q.q next to p.q (fused CG); the three
  // partial arrays are pstride apart
  const double* er = nullptr;
  int64_t pstride = 0;
  // fusion layouts 1 / 2 (gg_vec.hip, CG fusion): the prologue does not store
  // p_new; the last mode product's epilogue reads p_old (its xs operand) and
  // recomputes p_new = r + beta p_old (bitwise the prologue's value), stores it
  // to ep_out, and (layout 2) applies x += alpha p_old to ex when pending
  double* ep_out = nullptr;
  double* ex = nullptr;
  // Lanczos prologue (CGP = 3, gg_lanczos_probe): X holds the previous
  // matvec output Y, r the Lanczos vector u, q_old u_prev; the A operand is
  // w = coef[2] Y + coef[3] u + coef[4] u_prev, stored to p_out (over u_prev,
  // element-wise in place), its block partial |w|^2 to rr_part
  const double* coef = nullptr;
  // block-basis CG (gg_kronb.hip): the pair launch's output q (the chain runs
  // in place on q_old, the last launch cannot)
  double* blk_q_out = nullptr;
  // derived r (CgScalars::rstored): the prologue reads p_{j-2} (pprev) in
  // place of r unless sc->rstored, and never stores r (KIND 5)
  bool rderive = false;
  const double* pprev = nullptr;
};

// Output address map of a mode product (see gg_kron.hip epilogue):
//   addr = (j / cg) * gs + (j % cg) + h * hs + a * as + br * cg,
//   a = row / mi, h = (row % mi) / cr, br = (row % mi) % cr.
// Push mode (sharded matvec over peer memory): the all-to-all chunk index
// (destination rank) is h (push = 1) or j / cg (push = 2); instead of the
// send buffer the element goes straight to peers[dest][self_off + rest], i.e.
// into the destination rank's receive buffer over xGMI.
struct OutMap {
  int identity;
  int64_t cg, gs, mi, cr, hs, as;
  int push = 0;
  int64_t self_off = 0;
  double* const* peers = nullptr;  // device array of world pointers
  static OutMap ident() { return OutMap{1, 1, 0, 1, 1, 0, 0}; }
};

// Reduction partial-buffer length used by grid-stride vector kernels.
constexpr int kVecBlocks = 2048;
constexpr int kVecThreads = 256;

// ---- the sharded CG's scalar state (gg_vec.hip gg_cgs), for the fused
// sharded phase 1 in gg_kron.hip ----
CgScalars* cgs_scalars_ptr(gg_cgs* c);
double* cgs_rr_part(gg_cgs* c, int64_t cap, int64_t* cap_out);
void cgs_set_pro_blocks(gg_cgs* c, int64_t nb);

// ---- vector kernels (gg_vec.hip) used by other translation units ----
void launch_dot_partials(const double* x, const double* y, int64_t n, double* partials,
                         int nblocks, hipStream_t s);
void launch_reduce_to(const double* partials, int64_t count, double* out, hipStream_t s);
// x_defer 2, one half of the active pair (sc->xh; [0, H) or [H, n)) as a
// streaming kernel sized to sit beside the ring mode products (gg_vec.hip)
void launch_x_half(double* x, int64_t n, int64_t H, const CgScalars* sc, hipStream_t s);

// ---- environment switches (gg_knobs.hip): the process snapshot of every
// GG_* variable, taken at the first lookup and re-taken at gg_kron_create /
// gg_cg_create / gg_knobs_reload (never getenv on a launch path)
const char* knob(const char* name);
void knobs_reload();

// ---- the Kronecker operator in its parity-block basis (gg_kronb.hip) ----
struct BlockOp;
// nullptr when the operator has no block form (a factor not square, of odd
// order or not centrosymmetric; d outside 2..6; the last two orders unequal or
// without a pair kernel; GG_KRON_BLOCK=0 at creation)
BlockOp* block_create(int d, const int64_t* rows, const int64_t* cols,
                      const double* const* factors);
void block_destroy(BlockOp* B);
int64_t block_n(const BlockOp* B);
int block_d(const BlockOp* B);
int block_launches(const BlockOp* B);   // launches per matvec (d - 1)
int64_t block_nb(const BlockOp* B);   // elements per block
// x (C order over the factors) -> P x in the block layout (inverse: back);
// sq_part (forward only, may be NULL): block_fold_partials(B) partials of |P x|^2.
// A block range [blk0, blk0 + nblk) (nblk < 0: all 2^d): forward writes those
// blocks only (y holds nblk nb elements); inverse reads them (the rest count
// as 0) and writes their contribution to every element of the grid vector
void block_fold(const BlockOp* B, bool inverse, const double* x, double* y, double* sq_part,
                hipStream_t s, int64_t blk0 = 0, int64_t nblk = -1);
int64_t block_fold_partials(const BlockOp* B);
// x, y: the vectors of blocks [blk0, blk0 + nblk) (nblk < 0: all)
void block_apply(const BlockOp* B, const double* x, double* y, double shift, double* work,
                 double* dot_partials, const int* skip, hipStream_t stream, int64_t* n_partials,
                 const MpFuse* cg, int cgp, hipEvent_t* ev, int64_t blk0 = 0,
                 int64_t nblk = -1);
int64_t block_prologue_blocks(const BlockOp* B);
int64_t block_partials_needed(const BlockOp* B);
int64_t block_side_half(int64_t n);
// x_defer mode 3: the length of each of the K regions (even; the last may be
// shorter) and whether the operator's pair launch can carry that side job
int64_t xwin_region(int64_t n, int K);
bool block_pair_side(const BlockOp* B);
// the layout is unpadded (the single-GPU default basis of the CG and of
// Lanczos: padded slabs measured slower than the grid basis)
bool block_efficient(const BlockOp* B);
// the CG prologue can run with derived r (the fast kernel's KIND 5 exists for
// axis 0 and the non-temporal prologue is on)
bool block_rderive_ok(const BlockOp* B);

}  // namespace gg
