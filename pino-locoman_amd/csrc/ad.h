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

// Hyper-dual numbers (v, a, b, c) = f + a e1 + b e2 + c e1 e2 with e1^2 = e2^2 = 0: the
// e1 e2 part of a row function evaluated at x + e1 s1 + e2 s2 is the exact second
// derivative d^2 g / ds1 ds2 (the Lagrangian Hessian of the interior-point branch,
// k_lag_hess; CasADi's exact Hessian in the reference's Fatrop branch, ocp.py:248-263).
struct HDual {
  double v, a, b, c;
  PL_HD HDual() : v(0.0), a(0.0), b(0.0), c(0.0) {}
  PL_HD HDual(double x) : v(x), a(0.0), b(0.0), c(0.0) {}
  PL_HD HDual(double x, double da, double db, double dab) : v(x), a(da), b(db), c(dab) {}
};
PL_HD double val(const HDual& x) { return x.v; }
// f(x) with f' = f1, f'' = f2 at x.v
PL_HD HDual hd_chain(const HDual& x, double f0, double f1, double f2) {
  return HDual(f0, f1 * x.a, f1 * x.b, f1 * x.c + f2 * x.a * x.b);
}
PL_HD HDual operator+(HDual x, HDual y) { return HDual(x.v + y.v, x.a + y.a, x.b + y.b, x.c + y.c); }
PL_HD HDual operator-(HDual x, HDual y) { return HDual(x.v - y.v, x.a - y.a, x.b - y.b, x.c - y.c); }
PL_HD HDual operator-(HDual x) { return HDual(-x.v, -x.a, -x.b, -x.c); }
PL_HD HDual operator*(HDual x, HDual y) {
  return HDual(x.v * y.v, x.a * y.v + x.v * y.a, x.b * y.v + x.v * y.b,
               x.c * y.v + x.a * y.b + x.b * y.a + x.v * y.c);
}
PL_HD HDual hd_inv(HDual y) {
  const double r = 1.0 / y.v;
  return hd_chain(y, r, -r * r, 2.0 * r * r * r);
}
PL_HD HDual operator/(HDual x, HDual y) { return x * hd_inv(y); }
PL_HD HDual operator+(HDual x, double y) { return HDual(x.v + y, x.a, x.b, x.c); }
PL_HD HDual operator+(double x, HDual y) { return HDual(x + y.v, y.a, y.b, y.c); }
PL_HD HDual operator-(HDual x, double y) { return HDual(x.v - y, x.a, x.b, x.c); }
PL_HD HDual operator-(double x, HDual y) { return HDual(x - y.v, -y.a, -y.b, -y.c); }
PL_HD HDual operator*(HDual x, double y) { return HDual(x.v * y, x.a * y, x.b * y, x.c * y); }
PL_HD HDual operator*(double x, HDual y) { return HDual(x * y.v, x * y.a, x * y.b, x * y.c); }
PL_HD HDual operator/(HDual x, double y) { return HDual(x.v / y, x.a / y, x.b / y, x.c / y); }
PL_HD HDual operator/(double x, HDual y) { return x * hd_inv(y); }
PL_HD HDual& operator+=(HDual& x, HDual y) { x = x + y; return x; }
PL_HD HDual& operator-=(HDual& x, HDual y) { x = x - y; return x; }
PL_HD HDual& operator*=(HDual& x, HDual y) { x = x * y; return x; }
PL_HD HDual sin(HDual x) {
  const double s = ::sin(x.v), c = ::cos(x.v);
  return hd_chain(x, s, c, -s);
}
PL_HD HDual cos(HDual x) {
  const double s = ::sin(x.v), c = ::cos(x.v);
  return hd_chain(x, c, -s, -c);
}
PL_HD void sincos_s(HDual x, HDual* s, HDual* c) {
  const double sv = ::sin(x.v), cv = ::cos(x.v);
  *s = hd_chain(x, sv, cv, -sv);
  *c = hd_chain(x, cv, -sv, -cv);
}
PL_HD HDual sqrt(HDual x) {
  const double r = ::sqrt(x.v);
  return hd_chain(x, r, 0.5 / r, -0.25 / (r * x.v));
}
PL_HD HDual sqrt_s(HDual x) { return sqrt(x); }
PL_HD HDual sin_s(HDual x) { return sin(x); }
PL_HD HDual cos_s(HDual x) { return cos(x); }

template <class S>
PL_HD S sq(const S& a) { return a * a; }
