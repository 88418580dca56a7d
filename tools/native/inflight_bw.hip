// HBM read bandwidth of a k_admm-shaped stream against the bytes each wave keeps in flight.
// One wave per SIMD (1024 waves on 256 CUs), each wave streaming its own contiguous region
// (a problem's factor blocks) through a register double buffer of D 16-byte loads per lane
// (D KiB per wave per buffer).  Question answered: does a deeper prefetch than k_admm's
// (KM x 8 = 32 loads) raise the one-wave-per-SIMD stream rate?
#include <hip/hip_runtime.h>

#include <cstdio>

template <int D>
__global__ __launch_bounds__(256, 1) void stream_d(const double2* __restrict__ p, size_t per_wave2, double* out) {
  const int lane = threadIdx.x & 63;
  const size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
  const double2* base = p + w * per_wave2;
  double2 a[D], b[D];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < D; ++k) a[k] = base[k * 64 + lane];
  for (size_t o = (size_t)D * 64; o + (size_t)D * 64 <= per_wave2; o += (size_t)2 * D * 64) {
#pragma unroll
    for (int k = 0; k < D; ++k) b[k] = base[o + k * 64 + lane];
#pragma unroll
    for (int k = 0; k < D; ++k) s += a[k].x * a[k].y;
    if (o + (size_t)2 * D * 64 > per_wave2) {
#pragma unroll
      for (int k = 0; k < D; ++k) a[k] = b[k];
      break;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) a[k] = base[o + (size_t)D * 64 + k * 64 + lane];
#pragma unroll
    for (int k = 0; k < D; ++k) s += b[k].x * b[k].y;
  }
#pragma unroll
  for (int k = 0; k < D; ++k) s += a[k].x * a[k].y;
  if (s == 12345.678) out[w] = s;
}

template <int D>
float run(const double2* p, size_t per_wave2, int waves, double* out, hipEvent_t e0, hipEvent_t e1) {
  hipLaunchKernelGGL(stream_d<D>, dim3(waves / 4), dim3(256), 0, 0, p, per_wave2, out);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(stream_d<D>, dim3(waves / 4), dim3(256), 0, 0, p, per_wave2, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const size_t per_wave_bytes = 2u << 20;  // 2 MiB per wave (one problem's factor stream)
  const int maxw = 2048;
  double2* p;
  double* out;
  if (hipMalloc(&p, per_wave_bytes * maxw) != hipSuccess || hipMalloc(&out, maxw * 8) != hipSuccess) return 1;
  hipMemset(p, 0, per_wave_bytes * maxw);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const size_t pw2 = per_wave_bytes / 16;
  for (int waves : {1024, 2048}) {
    const double gb = (double)per_wave_bytes * waves / 1e9;
    float t;
    t = run<8>(p, pw2, waves, out, e0, e1);
    printf("waves %d D 8  (8 KiB/wave)  %.3f ms  %.2f TB/s\n", waves, t, gb / t);
    t = run<16>(p, pw2, waves, out, e0, e1);
    printf("waves %d D 16 (16 KiB/wave) %.3f ms  %.2f TB/s\n", waves, t, gb / t);
    t = run<32>(p, pw2, waves, out, e0, e1);
    printf("waves %d D 32 (32 KiB/wave) %.3f ms  %.2f TB/s\n", waves, t, gb / t);
    t = run<48>(p, pw2, waves, out, e0, e1);
    printf("waves %d D 48 (48 KiB/wave) %.3f ms  %.2f TB/s\n", waves, t, gb / t);
  }
  return 0;
}
