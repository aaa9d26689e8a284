// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access shapes the
// Kronecker path uses (MI355X_MICROARCH.md: only 16-B-per-lane streaming
// reads are calibrated).  Each kernel streams a 2 GiB buffer exactly once:
//   k16   16 B per lane, contiguous (the CG vector kernels)
//   kfrag  8 B per lane in the mode product's A-fragment shape: lanes
//          0..15 read 128 contiguous bytes of one row, lanes 16..63 the same
//          columns of the next three rows (row stride = M doubles)
//   w8    the epilogue's store shape (8 B per lane, 4 rows x 128 B)
// Run under rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) and divide the
// counter by the bytes printed here.  Standalone: hipcc this file.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k16(const double2* __restrict__ x, int64_t n2, double* out) {
  double s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = x[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

// X viewed as R rows x M columns; a wave covers 16 columns x 4 rows per load
__global__ void kfrag(const double* __restrict__ X, int64_t M, int64_t R, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t strip = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int64_t col = strip * 16 + (lane & 15);
  double s = 0;
  if (col < M)
    for (int64_t r = lane >> 4; r < R; r += 4) s += X[r * M + col];
  if (s == 12345.678) out[0] = s;
}

__global__ void w8(double* __restrict__ Y, int64_t M, int64_t R) {
  const int lane = threadIdx.x & 63;
  const int64_t strip = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int64_t col = strip * 16 + (lane & 15);
  if (col < M)
    for (int64_t r = lane >> 4; r < R; r += 4) Y[r * M + col] = (double)r;
}

int main() {
  const int64_t n = (int64_t)1 << 28;  // 2 GiB of doubles
  double *x, *out;
  if (hipMalloc(&x, n * 8) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(x, 0, n * 8);
  const int64_t R = 200, M = n / R;
  for (int rep = 0; rep < 2; ++rep) {
    k16<<<4096, 256>>>(reinterpret_cast<const double2*>(x), n / 2, out);
    kfrag<<<(unsigned)((M / 16 + 3) / 4), 256>>>(x, M, R, out);
    w8<<<(unsigned)((M / 16 + 3) / 4), 256>>>(x, M, R);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes per kernel: k16 %lld  kfrag %lld  w8 %lld\n", (long long)(n * 8),
         (long long)(R * M * 8), (long long)(R * M * 8));
  return 0;
}
