// The sharded CG's right-hand-side fold and solution unfold on the device for
// the two decompositions that do not use the parity-block layout
// (gp_grief_amd/distributed.py solve: "parity" and "transpose"; round 6 --
// before, the host folded the whole grid vector and the ranks exchanged host
// arrays through object collectives).  Both are once-per-solve, HBM-bound
// gathers / scatters; the unfold writes this rank's contribution to the grid
// vector and the caller sums the ranks' with one all-reduce (as the block
// decomposition does).  Reference: the operator is kron_matrix.py:52-97's;
// the reference has no sharding.
#include <algorithm>
#include <cmath>

#include "gg_internal.h"

namespace gg {

constexpr int kShardMaxD = 12;

struct ShardGeom {
  int d;
  int K;                          // parity: sharded axes 0..K-1 (world = 2^K)
  int rank;
  int64_t m[kShardMaxD], stride[kShardMaxD];
  int64_t n_local;
  double scale;                   // 2^{-K/2}
};

// Thread per local element l of rank g's block in the even / odd basis of
// axes 0..K-1: local layout C order over (m_K .. m_{d-1}, h_0 .. h_{K-1})
// (distributed.parity_local_factors).  Its 2^K grid corners are i_k = j_k or
// m_k - 1 - j_k on the sharded axes; corner c's sign is -1 for every axis
// whose rank bit (bit K - 1 - k of g) and corner bit are both set.
// forward: in = the grid vector, out = the local block; inverse: in = the
// local block, out = its contribution to the grid vector (every element)
__global__ __launch_bounds__(256) void parity_fold_kernel(const double* __restrict__ in,
                                                          double* __restrict__ out, ShardGeom g,
                                                          int inverse) {
  const int C = 1 << g.K;
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < g.n_local; l += st) {
    int64_t rem = l, lo = 0;
    int64_t span[kShardMaxD];
    // the local axes from the fastest: h_{K-1} .. h_0, then m_{d-1} .. m_K
    for (int k = g.K - 1; k >= 0; --k) {
      const int64_t h = g.m[k] / 2;
      const int64_t j = rem % h;
      rem /= h;
      lo += j * g.stride[k];
      span[k] = (g.m[k] - 1 - 2 * j) * g.stride[k];
    }
    for (int k = g.d - 1; k >= g.K; --k) {
      const int64_t i = rem % g.m[k];
      rem /= g.m[k];
      lo += i * g.stride[k];
    }
    double acc = 0.0;
    const double v = inverse ? in[l] * g.scale : 0.0;
    for (int c = 0; c < C; ++c) {
      int64_t o = lo;
      bool neg = false;
      for (int k = 0; k < g.K; ++k)
        if ((c >> (g.K - 1 - k)) & 1) {
          o += span[k];
          neg ^= ((g.rank >> (g.K - 1 - k)) & 1) != 0;
        }
      if (inverse)
        out[o] = neg ? -v : v;
      else
        acc += neg ? -in[o] : in[o];
    }
    if (!inverse) out[l] = acc * g.scale;
  }
}

// Thread per local element l = r (m_0 / G) + a of rank g's factor-0 row block
// (distributed.local_index_map): grid index (g m_0 / G + a) rest + r.
// Forward: in = grid, out = local; inverse: in = local, out = grid (the
// rank's elements only).
__global__ __launch_bounds__(256) void shard0_fold_kernel(const double* __restrict__ in,
                                                          double* __restrict__ out, int64_t rest,
                                                          int64_t s0, int rank, int64_t n_local,
                                                          int inverse) {
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < n_local; l += st) {
    const int64_t r = l / s0, a = l - r * s0;
    const int64_t o = ((int64_t)rank * s0 + a) * rest + r;
    if (inverse)
      out[o] = in[l];
    else
      out[l] = in[o];
  }
}

static int shard_grid(int64_t n) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    GG_HIP(hipGetDevice(&dev));
    GG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (cus <= 0) cus = 256;
  }
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), (int64_t)cus * 16));
}

}  // namespace gg

extern "C" {

int gg_parity_fold(int d, const int64_t* m, int world, int rank, int inverse,
                   const double* in_dev, double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(m && in_dev && out_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(d >= 1 && d <= gg::kShardMaxD, GG_ERR_VALUE, "1 <= d <= 12");
    GG_REQUIRE(world >= 1 && (world & (world - 1)) == 0, GG_ERR_VALUE,
               "the parity sharding needs 2^K ranks");
    int K = 0;
    while ((1 << K) < world) ++K;
    GG_REQUIRE(K <= d && rank >= 0 && rank < world, GG_ERR_VALUE, "rank / world out of range");
    gg::ShardGeom g{};
    g.d = d;
    g.K = K;
    g.rank = rank;
    int64_t st = 1, n = 1;
    for (int k = d - 1; k >= 0; --k) {
      GG_REQUIRE(m[k] >= 1, GG_ERR_VALUE, "bad factor order");
      GG_REQUIRE(k >= K || m[k] % 2 == 0, GG_ERR_VALUE, "sharded factors need even order");
      g.m[k] = m[k];
      g.stride[k] = st;
      st *= m[k];
      n *= m[k];
    }
    g.n_local = n >> K;
    g.scale = std::ldexp(1.0, -K / 2) * ((K & 1) ? M_SQRT1_2 : 1.0);
    if (g.n_local == 0) return;
    hipLaunchKernelGGL(gg::parity_fold_kernel, dim3(gg::shard_grid(g.n_local)), dim3(256), 0,
                       gg::as_stream(stream), in_dev, out_dev, g, inverse ? 1 : 0);
    GG_LAUNCH_CHECK();
  });
}

int gg_shard0_fold(int d, const int64_t* m, int world, int rank, int inverse,
                   const double* in_dev, double* out_dev, gg_stream stream) {
  return gg::guard([&] {
    GG_REQUIRE(m && in_dev && out_dev, GG_ERR_VALUE, "NULL argument");
    GG_REQUIRE(d >= 1 && world >= 1 && rank >= 0 && rank < world, GG_ERR_VALUE,
               "bad argument");
    GG_REQUIRE(m[0] % world == 0, GG_ERR_VALUE, "factor 0's order must divide by the ranks");
    int64_t rest = 1;
    for (int k = 1; k < d; ++k) rest *= m[k];
    const int64_t s0 = m[0] / world, nl = s0 * rest;
    if (nl == 0) return;
    hipLaunchKernelGGL(gg::shard0_fold_kernel, dim3(gg::shard_grid(nl)), dim3(256), 0,
                       gg::as_stream(stream), in_dev, out_dev, rest, s0, rank, nl,
                       inverse ? 1 : 0);
    GG_LAUNCH_CHECK();
  });
}

}  // extern "C"
