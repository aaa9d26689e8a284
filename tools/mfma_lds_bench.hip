// Microbenchmark: what the Kronecker mode product's inner loop can reach.
// FP64 MFMA (v_mfma_f64_16x16x4_f64), 13 accumulators per wave (the 200-column
// strip), 4-wave workgroups x 3 per CU (the mode product's occupancy), 2
// k-steps per chunk:
//   reg    : A and B operands in registers, random data
//   lds    : B fragment read from LDS per MFMA (random data), A in a register
//   ldsbar : as lds plus a workgroup barrier every chunk
//   ldsA   : as ldsbar, A fragment read from LDS too
//   glds   : as ldsA, B chunks streamed global(L2) -> LDS by global_load_lds
//            through a 3-stage ring (counted vmcnt + raw barrier)
// Random operands: MI355X clocks depend on the switching activity of the data.
// Standalone: hipcc --offload-arch=gfx950 -O3 tools/mfma_lds_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int JT = 13;
constexpr int kStage = 2 * JT * 64 + 4 * 8 * 16;  // B chunk + A rows (doubles)

__device__ double hashd(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
  return (double)(x & 0xffffff) / 16777216.0 - 0.5;
}

__global__ void fill(double* g, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    g[i] = hashd(i);
}

template <int MODE>
__global__ __launch_bounds__(256, 3) void kern(double* out, const double* gB, int iters) {
  __shared__ __attribute__((aligned(16))) double lds[3 * kStage];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 3 * kStage; i += 256) lds[i] = hashd(i * 7 + blockIdx.x);
  __syncthreads();
  d4 acc[JT];
  for (int t = 0; t < JT; ++t) acc[t] = d4{0, 0, 0, 0};
  double a0 = hashd(threadIdx.x + 1000 * blockIdx.x), a1 = hashd(threadIdx.x * 3 + 17);
  double breg[JT];
  for (int t = 0; t < JT; ++t) breg[t] = hashd(t * 64 + lane + 99);
  auto issue = [&](int c) {  // 832 double2 of B: waves issue 4 or 3 glds
    double* st = lds + (c % 3) * kStage;
    const double* src = gB + (size_t)(c % 25) * (2 * JT * 64);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = u * 256 + threadIdx.x;
      if (i < 2 * JT * 32)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(src + 2 * i),
            (__attribute__((address_space(3))) void*)(st + (u * 256 + wave * 64) * 2), 16, 0, 0);
    }
  };
  if (MODE == 4) { issue(0); issue(1); }
  for (int it = 0; it < iters; ++it) {
    const double* st = lds + (MODE == 4 ? (it % 3) * kStage : (it & 1) * 2 * JT * 64);
    if (MODE == 4) {
      if (it + 1 < iters) __builtin_amdgcn_s_waitcnt(3 | (7 << 4) | (15 << 8));
      else __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
      __builtin_amdgcn_s_barrier();
      if (it + 2 < iters) issue(it + 2);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      double a = s ? a1 : a0;
      if (MODE >= 3) a = st[2 * JT * 64 + wave * 128 + (4 * s + (lane >> 4)) * 16 + (lane & 15)];
#pragma unroll
      for (int t = 0; t < JT; ++t) {
        double b;
        if (MODE == 0) b = breg[t];
        else b = st[(s * JT + t) * 64 + lane];
        acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[t], 0, 0, 0);
      }
    }
    if (MODE == 2 || MODE == 3) __syncthreads();
  }
  double s = 0;
  for (int t = 0; t < JT; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[(blockIdx.x & 4095) * blockDim.x + threadIdx.x] = s;  // 4096 x 256 doubles
}

template <int MODE>
void run(const char* name, double* out, const double* gB, int iters = 400) {
  const int blocks = 256 * 3 * 4 * (400 / iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(256), 0, 0, out, gB, 20);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(256), 0, 0, out, gB, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double fl = 2.0 * 16 * 16 * 4 * JT * 2.0 * iters * blocks * 4;
  printf("%-9s %.2f TFLOP/s (%.3f ms)\n", name, fl / ms / 1e9, ms);
}

int main() {
  double *out, *gB;
  (void)hipMalloc(&out, 4096 * 256 * sizeof(double));
  const int nB = 25 * 2 * JT * 64;  // 25 chunks = one 200 x 208 factor
  (void)hipMalloc(&gB, nB * sizeof(double));
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, gB, nB);
  for (int r = 0; r < 2; ++r) {
    run<0>("reg", out, gB);
    run<1>("lds", out, gB);
    run<2>("ldsbar", out, gB);
    run<2>("ldsbar25", out, gB, 25);
    run<3>("ldsA25", out, gB, 25);
    run<4>("glds25", out, gB, 25);
  }
  return 0;
}
