// Scalar layer for the node evaluation kernels.
//
// The reference differentiates its OCP symbolically with CasADi (ca.jacobian,
// optimization/ocp.py:283-284).  The HIP path instead evaluates every node's row
// function twice: once in plain fp64 (values g, f) and once per Jacobian column in
// forward-mode dual numbers (one tangent per thread).  `Dual` carries (value,
// tangent); `val()` extracts the value so data-dependent branches (small-angle
// Taylor switches, quaternion branch) follow the primal exactly as CasADi's
// if_else does.
#pragma once
#include <math.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PL_HD __host__ __device__ __forceinline__
#else  // plain C++ build of the same math (the CPU baseline in oracle/cpu, g++ -O3)
#define PL_HD inline __attribute__((always_inline))
#endif

struct Dual {
  double v, d;
  PL_HD Dual() : v(0.0), d(0.0) {}
  PL_HD Dual(double x) : v(x), d(0.0) {}
  PL_HD Dual(double x, double dx) : v(x), d(dx) {}
};

PL_HD double val(double x) { return x; }
PL_HD double val(const Dual& x) { return x.v; }
PL_HD double tan_of(double) { return 0.0; }
PL_HD double tan_of(const Dual& x) { return x.d; }

PL_HD Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
PL_HD Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
PL_HD Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
PL_HD Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, fma(a.d, b.v, a.v * b.d)); }
PL_HD Dual operator/(Dual a, Dual b) {
  double inv = 1.0 / b.v;
  double q = a.v * inv;
  return Dual(q, (a.d - q * b.d) * inv);
}
PL_HD Dual operator+(Dual a, double b) { return Dual(a.v + b, a.d); }
PL_HD Dual operator+(double a, Dual b) { return Dual(a + b.v, b.d); }
PL_HD Dual operator-(Dual a, double b) { return Dual(a.v - b, a.d); }
PL_HD Dual operator-(double a, Dual b) { return Dual(a - b.v, -b.d); }
PL_HD Dual operator*(Dual a, double b) { return Dual(a.v * b, a.d * b); }
PL_HD Dual operator*(double a, Dual b) { return Dual(a * b.v, a * b.d); }
PL_HD Dual operator/(Dual a, double b) { return Dual(a.v / b, a.d / b); }
PL_HD Dual operator/(double a, Dual b) {
  double q = a / b.v;
  return Dual(q, -q * b.d / b.v);
}
PL_HD Dual& operator+=(Dual& a, Dual b) { a.v += b.v; a.d += b.d; return a; }
PL_HD Dual& operator-=(Dual& a, Dual b) { a.v -= b.v; a.d -= b.d; return a; }
PL_HD Dual& operator*=(Dual& a, Dual b) { a = a * b; return a; }

// sin and cos separately: the device library's sincos takes its outputs through
// private-memory pointers, which costs every kernel a scratch segment
PL_HD Dual sin(Dual a) { return Dual(::sin(a.v), ::cos(a.v) * a.d); }
PL_HD Dual cos(Dual a) { return Dual(::cos(a.v), -::sin(a.v) * a.d); }
PL_HD void sincos_s(double a, double* s, double* c) {
  *s = ::sin(a);
  *c = ::cos(a);
}
PL_HD void sincos_s(Dual a, Dual* s, Dual* c) {
  const double sv = ::sin(a.v), cv = ::cos(a.v);
  *s = Dual(sv, cv * a.d);
  *c = Dual(cv, -sv * a.d);
}
PL_HD Dual sqrt(Dual a) {
  double r = ::sqrt(a.v);
  return Dual(r, a.d * 0.5 / r);
}
PL_HD double sqrt_s(double a) { return ::sqrt(a); }
PL_HD Dual sqrt_s(Dual a) { return sqrt(a); }
PL_HD double sin_s(double a) { return ::sin(a); }
PL_HD double cos_s(double a) { return ::cos(a); }
PL_HD Dual sin_s(Dual a) { return sin(a); }
PL_HD Dual cos_s(Dual a) { return cos(a); }

template <class S>
PL_HD S sq(const S& a) { return a * a; }
