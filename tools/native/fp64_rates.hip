// Micro-benchmark of the per-wave FP64 / LDS costs the factor chain is built from
// (one wave per CU, s_memtime cycles): independent and dependent v_fma_f64, broadcast
// ds_read_b128, an LDS write->read round trip, and v_mfma_f64_16x16x4_f64.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k(double* out, unsigned long long* cyc, double seed) {
  __shared__ double buf[1024];
  const int l = threadIdx.x;
  for (int k = l; k < 1024; k += 64) buf[k] = seed + k;
  __syncthreads();
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = seed * (l + j);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 512; ++it)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fma(a[j], 0.999, 1e-3);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double c = a[0];
  for (int it = 0; it < 1024; ++it) c = fma(c, 0.999, 1e-3);
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  const double2* b2 = reinterpret_cast<const double2*>(buf);
  double s = 0;
  for (int it = 0; it < 32; ++it) {
    double2 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = b2[(it * 16 + j) & 511];
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j].x;
  }
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  double r = s;
  for (int it = 0; it < 256; ++it) {
    buf[(it & 7) * 64 + l] = r;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    r = buf[(it & 7) * 64 + ((l + 1) & 63)] * 0.5;
  }
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  f64x4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int it = 0; it < 256; ++it)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[j], a[j + 4], acc[j], 0, 0, 0);
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  double tot = c + s + r;
  for (int j = 0; j < 8; ++j) tot += a[j];
  for (int j = 0; j < 4; ++j) tot += acc[j][0];
  out[blockIdx.x * 64 + l] = tot;
  if (l == 0) {
    cyc[blockIdx.x * 8 + 0] = t1 - t0;
    cyc[blockIdx.x * 8 + 1] = t2 - t1;
    cyc[blockIdx.x * 8 + 2] = t3 - t2;
    cyc[blockIdx.x * 8 + 3] = t4 - t3;
    cyc[blockIdx.x * 8 + 4] = t5 - t4;
  }
}

int main() {
  double* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 64 * sizeof(double));
  (void)hipMalloc(&cyc, 256 * 8 * sizeof(unsigned long long));
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k, dim3(256), dim3(64), 0, 0, out, cyc, 1.0001);
  unsigned long long h[8];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  printf("independent v_fma_f64 (8 chains): %.2f cycles per wave-instruction\n", h[0] / 4096.0);
  printf("dependent v_fma_f64 chain:        %.2f cycles per instruction\n", h[1] / 1024.0);
  printf("broadcast ds_read_b128 (+add):    %.2f cycles per read\n", h[2] / 512.0);
  printf("LDS write -> read round trip:     %.1f cycles\n", h[3] / 256.0);
  printf("v_mfma_f64_16x16x4 (4 acc):       %.2f cycles per MFMA\n", h[4] / 1024.0);
  return 0;
}
