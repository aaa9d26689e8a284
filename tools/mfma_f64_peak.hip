// Microbenchmark: FP64 MFMA (v_mfma_f64_16x16x4_f64) and FP64 VALU FMA peak on
// this device, and the two pipes side by side.  Standalone: hipcc this file.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma_loop(double* out, int iters, double a, double b) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double av = a + threadIdx.x * 1e-9, bv = b - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void valu_loop(double* out, int iters, double a, double b) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b);
      x4 = fma(x4, a, b); x5 = fma(x5, a, b); x6 = fma(x6, a, b); x7 = fma(x7, a, b);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

// half the waves MFMA, half VALU
__global__ void mixed_loop(double* out, int iters_m, int iters_v, double a, double b) {
  const int w = threadIdx.x >> 6;
  if (w & 1) {
    double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int it = 0; it < iters_v; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x0 = fma(x0, a, b); x1 = fma(x1, a, b); x2 = fma(x2, a, b); x3 = fma(x3, a, b);
        x4 = fma(x4, a, b); x5 = fma(x5, a, b); x6 = fma(x6, a, b); x7 = fma(x7, a, b);
      }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  } else {
    d4 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = d4{0, 0, 0, 0};
    double av = a + threadIdx.x * 1e-9, bv = b - threadIdx.x * 1e-9;
    for (int it = 0; it < iters_m; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

int main() {
  double* out;
  hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 4;
  for (int waves : {4, 8}) {
    const int iters = 4000;
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * waves), 0, 0, out, 10, 1.0, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop<4>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, 1.0, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 16 * 16 * 4 * 4.0 * iters * blocks * waves;
    printf("mfma_f64 waves/WG=%d: %.2f TFLOP/s (%.3f ms)\n", waves, fl / ms / 1e9, ms);
  }
  for (int waves : {4, 8, 16}) {
    const int iters = 2000;
    hipLaunchKernelGGL(valu_loop, dim3(blocks), dim3(64 * waves), 0, 0, out, 10, 1.0000001, 1e-9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(valu_loop, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, 1.0000001, 1e-9);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 2.0 * 32 * iters * (double)blocks * 64 * waves;
    printf("valu_f64 waves/WG=%d: %.2f TFLOP/s (%.3f ms)\n", waves, fl / ms / 1e9, ms);
  }
  {
    const int im = 4000, iv = 4000;
    hipLaunchKernelGGL(mixed_loop, dim3(blocks), dim3(512), 0, 0, out, 10, 10, 1.0000001, 1e-9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mixed_loop, dim3(blocks), dim3(512), 0, 0, out, im, iv, 1.0000001, 1e-9);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double flm = 2.0 * 16 * 16 * 4 * 4.0 * im * blocks * 4;
    double flv = 2.0 * 32 * iv * (double)blocks * 64 * 4;
    printf("mixed: mfma %.2f TF + valu %.2f TF = %.2f TF (%.3f ms)\n", flm / ms / 1e9, flv / ms / 1e9,
           (flm + flv) / ms / 1e9, ms);
  }
  return 0;
}
