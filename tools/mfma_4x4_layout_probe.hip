// Probe of the v_mfma_f64_4x4x4_4b_f64 operand layout: with A[lane] = 2^lane
// and B = 1, each D lane holds the sum of the A lanes that feed it (decoded
// from its bits); likewise B[lane] = 2^lane with A = 1.  Prints, per D lane,
// the A lanes and B lanes it reads.  Standalone: hipcc this file.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void probe(double* outA, double* outB) {
  const int l = threadIdx.x;
  const double p = ldexp(1.0, l);
  outA[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(p, 1.0, 0.0, 0, 0, 0);
  outB[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, p, 0.0, 0, 0, 0);
}

static void decode(double v, char* buf) {
  int n = 0;
  buf[0] = 0;
  for (int b = 63; b >= 0; --b) {
    const double p = ldexp(1.0, b);
    if (v >= p) {
      v -= p;
      n += sprintf(buf + n, "%d ", b);
    }
  }
}

int main() {
  double *a, *b;
  if (hipMalloc(&a, 64 * 8) != hipSuccess || hipMalloc(&b, 64 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, a, b);
  double ha[64], hb[64];
  if (hipMemcpy(ha, a, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(hb, b, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; ++l) {
    char sa[512], sb[512];
    decode(ha[l], sa);
    decode(hb[l], sb);
    printf("D lane %2d: A lanes [%s] B lanes [%s]\n", l, sa, sb);
  }
  return 0;
}
