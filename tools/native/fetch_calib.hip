// FETCH_SIZE calibration per load width (run under rocprofv3 --pmc FETCH_SIZE): each kernel
// reads a known number of bytes once, from a buffer 4x the 256 MiB Infinity Cache, with the
// access shapes k_admm uses:
//   stream16  one 16-byte load per lane, a wave reads 1 KiB contiguously (the factor stream)
//   stream8   one 8-byte load per lane, a wave reads 512 B contiguously (the vector reads)
//   rows8     8-byte loads of short runs: each wave reads `run` consecutive doubles per
//             instruction with the lanes past the run clamped onto its last element (the
//             clamped row / column operand reads of a node), runs laid end to end
// Prints the bytes each kernel reads; FETCH_SIZE (KB) / those bytes is the correction.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void stream16(const double2* __restrict__ p, size_t n2, double* out) {
  double s = 0.0;
  for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n2; k += (size_t)gridDim.x * 256) {
    const double2 v = p[k];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[blockIdx.x] = s;  // keeps the loads
}

__global__ __launch_bounds__(256) void stream8(const double* __restrict__ p, size_t n, double* out) {
  double s = 0.0;
  for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) s += p[k];
  if (s == 12345.678) out[blockIdx.x] = s;
}

// every wave walks its own contiguous slice in runs of `run` doubles, one instruction per run
__global__ __launch_bounds__(256) void rows8(const double* __restrict__ p, size_t n, int run, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t waves = (size_t)gridDim.x * 4, w = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const size_t per = n / waves, base = w * per;
  double s = 0.0;
  for (size_t o = 0; o + run <= per; o += run) s += p[base + o + (lane < run ? lane : run - 1)];
  if (s == 12345.678) out[blockIdx.x] = s;
}

int main() {
  const size_t bytes = 1ull << 30;  // 1 GiB, 4x the MALL
  double* buf;
  double* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, bytes);
  const size_t n = bytes / 8;
  const int grid = 2048;
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(stream16, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const double2*>(buf), n / 2, out);
  (void)hipDeviceSynchronize();
  printf("stream16 bytes %zu\n", bytes);
  hipLaunchKernelGGL(stream8, dim3(grid), dim3(256), 0, 0, buf, n, out);
  (void)hipDeviceSynchronize();
  printf("stream8 bytes %zu\n", bytes);
  for (int run : {64, 40, 24, 8}) {
    hipLaunchKernelGGL(rows8, dim3(grid), dim3(256), 0, 0, buf, n, run, out);
    (void)hipDeviceSynchronize();
    const size_t waves = (size_t)grid * 4, per = n / waves;
    printf("rows8 run %d bytes %zu\n", run, waves * (per / run) * run * 8);
  }
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
