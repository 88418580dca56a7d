// Checks the lane layout of v_mfma_f64_16x16x4_f64 on gfx950 with exact integer data:
//   A operand lane l: A[l & 15][l >> 4], B operand lane l: B[l >> 4][l & 15],
//   D lane l, reg r: D[(l >> 4) + 4 r][l & 15].
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double double4_ __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  double4_ acc = {0.0, 0.0, 0.0, 0.0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

int main() {
  double hA[64], hB[64], hD[256], ref[256];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 4; ++k) hA[i * 4 + k] = (i * 7 + k * 3) % 11 - 5;
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (k * 5 + j * 2) % 13 - 6;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j];
      ref[i * 16 + j] = s;
    }
  double *dA, *dB, *dD;
  hipMalloc(&dA, sizeof(hA));
  hipMalloc(&dB, sizeof(hB));
  hipMalloc(&dD, sizeof(hD));
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
  printf("mfma_f64_16x16x4 layout: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  return bad != 0;
}
