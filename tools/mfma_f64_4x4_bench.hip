// Microbenchmark: throughput of the two FP64 MFMA shapes on gfx950,
// v_mfma_f64_16x16x4_f64 (2048 FLOP) vs v_mfma_f64_4x4x4_4b_f64 (4 blocks of
// 4x4x4, 512 FLOP), independent accumulators, 4 / 8 waves per workgroup.
// Tells whether the half-empty 13th output tile of the p = 200 mode product
// could run on the small shape at a lower cost.  Standalone: hipcc this file.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void mfma16_loop(double* out, int iters, double a, double b) {
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

template <int NACC>
__global__ void mfma4_loop(double* out, int iters, double a, double b) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  double av = a + threadIdx.x * 1e-9, bv = b - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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
    hipLaunchKernelGGL(mfma16_loop<8>, dim3(blocks), dim3(64 * waves), 0, 0, out, 10, 1.0, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma16_loop<8>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, 1.0, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 2048.0 * 8 * iters * blocks * waves;
    printf("16x16x4 f64 waves/WG=%d: %.2f TFLOP/s, %.1f ns per MFMA per SIMD\n", waves, fl / ms / 1e9,
           ms * 1e6 / (8.0 * iters * blocks * waves / 1024.0));
  }
  for (int waves : {4, 8}) {
    const int iters = 4000;
    hipLaunchKernelGGL(mfma4_loop<16>, dim3(blocks), dim3(64 * waves), 0, 0, out, 10, 1.0, 1.0);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma4_loop<16>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, 1.0, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = 512.0 * 16 * iters * blocks * waves;
    printf("4x4x4_4b f64 waves/WG=%d: %.2f TFLOP/s, %.1f ns per MFMA per SIMD\n", waves,
           fl / ms / 1e9, ms * 1e6 / (16.0 * iters * blocks * waves / 1024.0));
  }
  return 0;
}
