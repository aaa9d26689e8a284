// HBM streaming ceiling on one MI355X (tuning aid, not a product path).
//
// The CG iteration at 200^4 moves ~218 GB per iteration in read / write
// passes of 12.8 GB vectors; this measures what a plain streaming kernel
// reaches on 8 GB buffers for the pass mixes the fused launches carry:
//   read-only (sum), write-only, copy (1R:1W), 3R:2W (the CG prologue's
//   p, r, q_old -> r, p_new), 2R:1W (x += alpha p)
// each with 16-byte lanes, default or non-temporal policy, several grid sizes.
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/hbm tools/hbm_stream_bench.hip
// Prints one JSON line per case: GB/s counts every byte read or written once.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ d2 ld(const d2* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2* p, d2 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// kind 0: read-only  1: write-only  2: copy  3: 3R2W  4: 2R1W
template <int KIND, bool NT, int U>
__global__ __launch_bounds__(256) void stream_kernel(d2* a, d2* b, d2* c, d2* d, d2* e,
                                                     int64_t n2, double al, double* sink) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  double acc = 0.0;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n2; i0 += stride) {
    d2 va[U], vb[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * 256;
      if (i < n2) {
        if (KIND == 0 || KIND == 2 || KIND == 3 || KIND == 4) va[u] = ld<NT>(a + i);
        if (KIND == 3 || KIND == 4) vb[u] = ld<NT>(b + i);
        if (KIND == 3) vc[u] = ld<NT>(c + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * 256;
      if (i < n2) {
        if (KIND == 0) acc += va[u].x + va[u].y;
        if (KIND == 1) st<NT>(d + i, d2{al, al});
        if (KIND == 2) st<NT>(d + i, va[u]);
        if (KIND == 3) {
          const d2 r = va[u] - al * vc[u];
          st<NT>(d + i, r);
          st<NT>(e + i, r + al * vb[u]);
        }
        if (KIND == 4) st<NT>(d + i, va[u] + al * vb[u]);
      }
    }
  }
  if (KIND == 0 && acc == 12345.678) sink[0] = acc;
}

// The mode product's A-operand pattern: the vector as q x M (row-major), a
// wave owns 16 columns b0..b0+15 and walks the q rows four at a time, lane l
// touching row 4 ks + (l >> 4), column b0 + (l & 15): 8 bytes per lane, four
// 128-B segments per wave instruction.  3R2W like the CG prologue.
// W waves per workgroup (W x 128 B contiguous per row); SYNC: a workgroup
// barrier every 12 rows, as the mode product's chunk pipeline has.
template <bool NT, int W = 4, bool SYNC = false>
__global__ __launch_bounds__(W * 64) void apattern_kernel(const double* a, const double* b,
                                                          const double* c, double* d, double* e,
                                                          int64_t M, int q, double al) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = ((int64_t)blockIdx.x * W + wave) * 16 + (lane & 15);
  const bool ok = col < M;
  for (int k = lane >> 4; k < q; k += 4) {
    if (SYNC && (k >> 2) % 3 == 0) __syncthreads();
    if (!ok) continue;
    const int64_t o = (int64_t)k * M + col;
    double va, vb, vc;
    if (NT) {
      va = __builtin_nontemporal_load(a + o);
      vb = __builtin_nontemporal_load(b + o);
      vc = __builtin_nontemporal_load(c + o);
    } else {
      va = a[o]; vb = b[o]; vc = c[o];
    }
    const double r = va - al * vc;
    if (NT) {
      __builtin_nontemporal_store(r, d + o);
      __builtin_nontemporal_store(r + al * vb, e + o);
    } else {
      d[o] = r;
      e[o] = r + al * vb;
    }
  }
}

template <bool NT, int W = 4, bool SYNC = false>
static void run_apattern(double* a, double* b, double* c, double* d, double* e, int64_t n) {
  const int q = 200;
  const int64_t M = n / q;
  const int grid = (int)((M + 16 * W - 1) / (16 * W));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((apattern_kernel<NT, W, SYNC>), dim3(grid), dim3(64 * W), 0, 0, a, b, c, d, e, M, q, 0.5);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((apattern_kernel<NT, W, SYNC>), dim3(grid), dim3(64 * W), 0, 0, a, b, c, d, e, M, q, 0.5);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double gb = (double)(M * q) * 40.0 / 1e9;
  printf("{\"kind\": \"3R2W-apattern\", \"nt\": %d, \"waves\": %d, \"sync\": %d, \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
         (int)NT, W, (int)SYNC, grid, ms, gb / (ms * 1e-3));
  fflush(stdout);
}

template <int KIND, bool NT, int U>
static void run(const char* name, d2* a, d2* b, d2* c, d2* d, d2* e, int64_t n2, int grid,
                double* sink, double bytes_per_elem2) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((stream_kernel<KIND, NT, U>), dim3(grid), dim3(256), 0, 0, a, b, c, d, e,
                       n2, 0.5, sink);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((stream_kernel<KIND, NT, U>), dim3(grid), dim3(256), 0, 0, a, b, c, d, e,
                       n2, 0.5, sink);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double gb = (double)n2 * bytes_per_elem2 / 1e9;
  printf("{\"kind\": \"%s\", \"nt\": %d, \"unroll\": %d, \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
         name, (int)NT, U, grid, ms, gb / (ms * 1e-3));
  fflush(stdout);
}

template <bool NT, int U>
static void all_kinds(d2* a, d2* b, d2* c, d2* d, d2* e, int64_t n2, int grid, double* sink) {
  run<0, NT, U>("read", a, b, c, d, e, n2, grid, sink, 16.0);
  run<1, NT, U>("write", a, b, c, d, e, n2, grid, sink, 16.0);
  run<2, NT, U>("copy", a, b, c, d, e, n2, grid, sink, 32.0);
  run<3, NT, U>("3R2W", a, b, c, d, e, n2, grid, sink, 80.0);
  run<4, NT, U>("2R1W", a, b, c, d, e, n2, grid, sink, 48.0);
}

int main() {
  const int64_t bytes = 8LL << 30;   // 8 GiB per vector
  const int64_t n2 = bytes / 16;
  d2 *a, *b, *c, *d, *e;
  double* sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&e, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipMemset(c, 0, bytes));
  int cus = 256;
  const bool quick = getenv("HBM_QUICK") != nullptr;
  if (!quick) {
    for (int g : {cus * 4, cus * 8, cus * 16, cus * 64}) {
      all_kinds<false, 4>(a, b, c, d, e, n2, g, sink);
      all_kinds<true, 4>(a, b, c, d, e, n2, g, sink);
    }
    all_kinds<false, 1>(a, b, c, d, e, n2, cus * 16, sink);
    all_kinds<true, 8>(a, b, c, d, e, n2, cus * 8, sink);
  }
  // q x M = 200 x M within the 8 GiB buffers
  const int64_t nfit = (bytes / 8) / 200 * 200;
  run_apattern<false>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<true>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<false, 4, true>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<false, 8, false>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<false, 8, true>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<false, 12, true>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  run_apattern<false, 16, true>((double*)a, (double*)b, (double*)c, (double*)d, (double*)e, nfit);
  return 0;
}
