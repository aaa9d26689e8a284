// Probe (tuning aid, not a product path): the vendor library's FP64 SYRK and
// GEMM on the GRIEF Gram shapes, A = Phi^T Phi with Phi n x p row-major (in
// column-major terms the p x n matrix M = Phi^T, lda = p, and A = M M^T):
//   rocblas_dsyrk(lower, none, p, n)   -- n p^2 FLOP (the triangle)
//   rocblas_dgemm(none, trans, p, p, n) -- 2 n p^2 FLOP (the full product)
// against which gemm_tn_glds (gg_dense.hip, n p^2 FLOP) is compared by
// tools/p2_kernels_bench.py in the same run.  Random operands in [-1, 1)
// (the clock an FP64 MFMA loop holds depends on the data).
// build: hipcc --offload-arch=gfx950 -O2 tools/syrk_probe.hip -lrocblas -o tools/syrk_probe
// usage: tools/syrk_probe [reps]   -> one JSON line per (routine, shape)
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)
#define RB(x)                                                                  \
  do {                                                                         \
    rocblas_status s_ = (x);                                                   \
    if (s_ != rocblas_status_success) {                                        \
      std::fprintf(stderr, "%s: rocblas status %d\n", #x, (int)s_);           \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void fill_kernel(double* a, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    unsigned long z = (unsigned long)i * 0x9E3779B97F4A7C15ull + seed;
    z ^= z >> 31;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 29;
    a[i] = (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  const long n = 100000;
  const int ps[3] = {1000, 5000, 10000};
  rocblas_handle h;
  RB(rocblas_create_handle(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  RB(rocblas_set_stream(h, st));
  for (int pi = 0; pi < 3; ++pi) {
    const int p = ps[pi];
    double *M = nullptr, *C = nullptr;
    CK(hipMalloc(&M, sizeof(double) * n * p));
    CK(hipMalloc(&C, sizeof(double) * (long)p * p));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, M, n * (long)p, 17u + p);
    CK(hipMemsetAsync(C, 0, sizeof(double) * (long)p * p, st));
    const double one = 1.0, zero = 0.0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int which = 0; which < 2; ++which) {
      auto run = [&] {
        if (which == 0)
          RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, p, (int)n, &one, M, p,
                           &zero, C, p));
        else
          RB(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, p, p, (int)n,
                           &one, M, p, M, p, &zero, C, p));
      };
      run();   // warm-up (and any library-side setup)
      CK(hipStreamSynchronize(st));
      float best = 1e30f, sum = 0.0f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, st));
        run();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        sum += ms;
      }
      const double flop = (which == 0 ? 1.0 : 2.0) * (double)n * p * p;
      std::printf("{\"routine\": \"%s\", \"n\": %ld, \"p\": %d, \"best_ms\": %.4f, "
                  "\"mean_ms\": %.4f, \"flop\": %.6g, \"tflops_best\": %.3f}\n",
                  which == 0 ? "rocblas_dsyrk" : "rocblas_dgemm", n, p, best, sum / reps, flop,
                  flop / (best * 1e-3) / 1e12);
      std::fflush(stdout);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(M));
    CK(hipFree(C));
  }
  RB(rocblas_destroy_handle(h));
  CK(hipStreamDestroy(st));
  return 0;
}
