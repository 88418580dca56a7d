// Helpers shared by the ADMM sweep kernels (k_admm.hip: one wave per problem,
// k_admm2.hip: two waves per problem).
#pragma once
#include "state.h"

namespace admm {

constexpr int KM = PL_ADMM_KM, CWM = PL_ADMM_CWM, XCM = PL_ADMM_XCM, MV = PL_ADMM_MV, MR = PL_ADMM_MR;

enum { KF0 = 0, KFWD = 1, KTN = 2, KBWD = 3, KT0 = 4, KB0 = 5 };

__device__ __forceinline__ int step_kind_v(int q, int N, int niter, int& i, int& it) {
  if (q == 0) {
    i = 0;
    it = 0;
    return KF0;
  }
  const int r = (q - 1) % (2 * N);
  it = (q - 1) / (2 * N);
  if (r < N - 1) {
    i = r + 1;
    return KFWD;
  }
  if (r == N - 1) {
    i = N;
    return KTN;
  }
  if (r < 2 * N - 1) {
    i = 2 * N - 1 - r;
    return KBWD;
  }
  i = 0;
  return it < niter - 1 ? KT0 : KB0;
}

// the schedule is wave-uniform; readfirstlane keeps it (and every node-table read and
// base address derived from it) in scalar registers
__device__ __forceinline__ int step_kind(int q, int N, int niter, int& i, int& it) {
  const int k = step_kind_v(q, N, niter, i, it);
  i = __builtin_amdgcn_readfirstlane(i);
  it = __builtin_amdgcn_readfirstlane(it);
  return __builtin_amdgcn_readfirstlane(k);
}

__device__ __forceinline__ bool bwd_kind(int k) { return k >= KBWD; }

__device__ __forceinline__ double sel2(const double2& v, int k) { return k == 0 ? v.x : v.y; }
__device__ __forceinline__ void set2(double2& v, int k, double x) {
  if (k == 0) v.x = x;
  else v.y = x;
}

// Cross-lane LDS exchange inside one wave: LDS executes a wave's operations in
// order, so only the compiler has to be kept from reordering across the phase.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// sum_{k0 <= k < k1} f(k), 8 clamped independent reads per round (branch-free within a
// round, so the LDS reads of a round issue back to back)
// sum_{k0 <= k < k1} p[k * stride], U reads per round; reads past k1 go to a zero slot
// (an index select instead of a select on the double)
template <int U = 8>
__device__ __forceinline__ double lds_sum(const double* p, int k0, int k1, int stride, const double* zero) {
  double acc = 0.0;
  for (int b = k0; b < k1; b += U) {
    double t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = *(b + u < k1 ? p + (b + u) * stride : zero);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += t[u];
  }
  return acc;
}

template <int U = 8, class F>
__device__ __forceinline__ double range_sum(int k0, int k1, F f) {
  double acc = 0.0;
  for (int b = k0; b < k1; b += U) {
    double t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = f(min(b + u, k1 - 1));
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (b + u < k1) ? t[u] : 0.0;
  }
  return acc;
}

// Global accesses as scalar base + unsigned 32-bit byte offset (the saddr + voffset
// form: no per-lane 64-bit address arithmetic).  Indices are < 2^32 / sizeof(T).
template <class T>
__device__ __forceinline__ T gld(const T* base, int idx) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (unsigned)idx * (unsigned)sizeof(T));
}
// the same as a non-temporal (streaming) load: the factor blocks are read once per sweep
template <bool NT, class T>
__device__ __forceinline__ T gldx(const T* base, int idx);
__device__ __forceinline__ double gld_nt(const double* base, int idx) {
  return __builtin_nontemporal_load(reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + (unsigned)idx * 8u));
}
__device__ __forceinline__ double2 gld_nt(const double2* base, int idx) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d v = __builtin_nontemporal_load(
      reinterpret_cast<const v2d*>(reinterpret_cast<const char*>(base) + (unsigned)idx * (unsigned)sizeof(double2)));
  return make_double2(v.x, v.y);
}
// a plain (gld) or non-temporal (gld_nt) load, chosen at compile time
template <bool NT, class T>
__device__ __forceinline__ T gldx(const T* base, int idx) {
  if constexpr (NT) return gld_nt(base, idx);
  else return gld(base, idx);
}
template <class T>
__device__ __forceinline__ void gst(T* base, int idx, T v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (unsigned)idx * (unsigned)sizeof(T)) = v;
}

// LDS f64 add without return (ds_add_f64): one instruction per lane, no round trip.  The
// lanes of one instruction and the instructions of one wave are applied in a fixed order,
// so the sums are deterministic (bit-identical for a problem in any batch).
__device__ __forceinline__ void lds_add(double* p, double v) {
  typedef __attribute__((address_space(3))) double* LPtr;
  __hip_atomic_fetch_add((LPtr)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ int div_k(int t, int K, unsigned km) { return K == 1 ? t : (int)__umulhi((unsigned)t, km); }

__device__ __forceinline__ void tile_ij(int t, int& I, int& J) {
  I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
  while (I * (I + 1) / 2 > t) --I;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  J = t - I * (I + 1) / 2;
}

}  // namespace admm
