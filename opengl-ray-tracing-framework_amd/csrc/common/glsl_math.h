// glsl_math.h — deterministic fp32 definitions of the GLSL builtins used by the
// reference path tracer (src/shaders/fragment_shader_ray_tracing.glsl, "RT:").
//
// Why this file exists
// --------------------
// GLSL leaves the precision of sin/cos/atan/asin/exp/log/pow to the driver, so
// the reference's own results depend on the GPU it ran on.  To make the HIP
// kernel and the CPU oracle agree BIT-FOR-BIT, both evaluate every builtin with
// the code below: IEEE-754 binary32 +,-,*,/ and sqrt only (correctly rounded on
// x86-64 SSE and on gfx950 with hipcc's default correctly-rounded div/sqrt),
// no contraction (every TU that includes this is built with -ffp-contract=off
// and the pragma below), rint for range reduction, and integer bit tricks.
// The polynomials are the classic Cephes single-precision minimax sets
// (<= 2 ulp vs. a double-precision reference; tests/test_glsl_math.py checks).
//
// The oracle (oracle/rt_oracle.cpp) includes this header as the definition of
// the GLSL builtins; nothing in here restates the reference's algorithm.
#pragma once
#include <stdint.h>
#include <math.h>

#ifdef __clang__
#pragma clang fp contract(off)
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define GM_FN __host__ __device__ static inline
#else
#define GM_FN static inline
#endif

// GM_LIBM (host code only: the oracle variant oracle/liboracle_libm.so): the transcendentals come
// from the C library's fp32 functions (sinf, cosf, atan2f, asinf, expf, logf, powf) instead of the
// polynomials below -- another implementation's builtin precision, to measure how much the image
// depends on these definitions (tests/test_builtin_precision.py).  (A device-side variant with
// the hardware v_sin/v_cos/v_exp/v_log was measured in round 2: no material speed-up, removed.)
#if defined(GM_LIBM) && !defined(__HIP_DEVICE_COMPILE__)
#define GM_HW 1
#else
#define GM_HW 0
#endif

namespace gm {

GM_FN uint32_t fbits(float f) { union { float f; uint32_t u; } v; v.f = f; return v.u; }
GM_FN float bitsf(uint32_t u) { union { float f; uint32_t u; } v; v.u = u; return v.f; }

GM_FN bool isnan_(float x) { return x != x; }
GM_FN float fabs_(float x) { return bitsf(fbits(x) & 0x7fffffffu); }
GM_FN float sqrt_(float x) { return sqrtf(x); }
GM_FN float rint_(float x) { return rintf(x); }
GM_FN float floor_(float x) { return floorf(x); }
// GLSL min/max: the hardware (IEEE minNum/maxNum) flavour, identical on both sides.
GM_FN float min_(float a, float b) { return fminf(a, b); }
GM_FN float max_(float a, float b) { return fmaxf(a, b); }
GM_FN float clamp_(float x, float lo, float hi) { return min_(max_(x, lo), hi); }
// GLSL mix(x, y, a) = x * (1 - a) + y * a  (GLSL 4.50 spec §8.3)
GM_FN float mix_(float x, float y, float a) { return x * (1.0f - a) + y * a; }
GM_FN float inversesqrt_(float x) { return 1.0f / sqrtf(x); }

// 2^n as a float for n in [-126, 127]
GM_FN float exp2i_(int n) { return bitsf((uint32_t)(n + 127) << 23); }

// ---- sin / cos --------------------------------------------------------------
// Cody-Waite reduction by pi/2 (three-part constant, the first two parts carry
// 12 significant bits so j*C1, j*C2 are exact for |j| < 4096), then the Cephes
// sinf/cosf polynomials on [-pi/4, pi/4].
#define GM_PIO2_1 1.5703125f
#define GM_PIO2_2 4.837512969970703125e-4f
#define GM_PIO2_3 7.549790126404332e-08f
#define GM_2OPI   0.636619746685028076171875f

GM_FN void sincos_(float x, float* s_out, float* c_out) {
#if GM_HW
  *s_out = sinf(x);
  *c_out = cosf(x);
  return;
#endif
  float j = rint_(x * GM_2OPI);
  float r = x - j * GM_PIO2_1;
  r = r - j * GM_PIO2_2;
  r = r - j * GM_PIO2_3;
  float z = r * r;
  float s = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
  float c = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z
            - 0.5f * z + 1.0f;
  int q = (int)j & 3;  // two's complement: (-1)&3 == 3, as wanted
  float so, co;
  if (q == 0)      { so = s;  co = c; }
  else if (q == 1) { so = c;  co = -s; }
  else if (q == 2) { so = -s; co = -c; }
  else             { so = -c; co = s; }
  // NaN / inf input: j is NaN, keep NaN (GLSL result is undefined there)
  if (isnan_(j)) { so = j; co = j; }
  *s_out = so; *c_out = co;
}
GM_FN float sin_(float x) { float s, c; sincos_(x, &s, &c); return s; }
GM_FN float cos_(float x) { float s, c; sincos_(x, &s, &c); return c; }

// ---- atan / atan2 -------------------------------------------------------------
#define GM_PIO2F 1.57079632679489661923f
#define GM_PIO4F 0.785398163397448309616f
#define GM_PIF   3.14159265358979323846f

// Cephes atanf core for t >= 0
GM_FN float atan_pos_(float t) {
  float y0, u;
  if (t > 2.414213562373095f) { y0 = GM_PIO2F; u = -(1.0f / t); }
  else if (t > 0.4142135623730950f) { y0 = GM_PIO4F; u = (t - 1.0f) / (t + 1.0f); }
  else { y0 = 0.0f; u = t; }
  float z = u * u;
  float p = (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z
             - 3.33329491539e-1f) * z * u + u;
  return y0 + p;
}

// GLSL atan(y, x): quadrant-correct arctangent (C atan2 conventions for zeros).
GM_FN float atan2_(float y, float x) {
#if GM_HW
  return atan2f(y, x);
#endif
  if (isnan_(x) || isnan_(y)) return x + y;
  float ax = fabs_(x), ay = fabs_(y);
  float a;
  if (ax == 0.0f && ay == 0.0f) a = 0.0f;
  else if (ay <= ax) a = atan_pos_(ay / ax);          // in [0, pi/4]
  else a = GM_PIO2F - atan_pos_(ax / ay);              // in (pi/4, pi/2]
  if (fbits(x) >> 31) a = GM_PIF - a;                  // x < 0 (or -0)
  if (fbits(y) >> 31) a = -a;
  return a;
}

// ---- asin -----------------------------------------------------------------------
GM_FN float asin_(float x) {
#if GM_HW
  return asinf(x);
#endif
  float a = fabs_(x);
  if (!(a <= 1.0f)) return (x - x) / (x - x);  // NaN (also for NaN input)
  float z, s;
  bool big = a > 0.5f;
  if (big) { z = 0.5f * (1.0f - a); s = sqrt_(z); }
  else { z = a * a; s = a; }
  float p = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z
              + 7.4953002686e-2f) * z + 1.6666752422e-1f) * z * s + s;
  if (big) p = GM_PIO2F - (p + p);
  return (fbits(x) >> 31) ? -p : p;
}

// ---- exp / log / pow ------------------------------------------------------------
#define GM_LOG2EF 1.44269504088896341f
GM_FN float exp_(float x) {
#if GM_HW
  return expf(x);
#endif
  if (isnan_(x)) return x;
  if (x > 88.72283905206835f) return bitsf(0x7f800000u);
  if (x < -103.972077083991796f) return 0.0f;
  float n = rint_(x * GM_LOG2EF);
  float r = x - n * 0.693359375f;
  r = r - n * -2.12194440e-4f;
  float z = r * r;
  float y = (((((1.9875691500e-4f * r + 1.3981999507e-3f) * r + 8.3334519073e-3f) * r
               + 4.1665795894e-2f) * r + 1.6666665459e-1f) * r + 5.0000001201e-1f) * z + r + 1.0f;
  int ni = (int)n;
  if (ni > 127) return (y * exp2i_(127)) * 2.0f;
  if (ni < -126) return (y * exp2i_(ni + 64)) * exp2i_(-64);
  return y * exp2i_(ni);
}

GM_FN float log_(float x) {
#if GM_HW
  return logf(x);
#endif
  if (isnan_(x)) return x;
  if (x < 0.0f) return (x - x) / (x - x);
  if (x == 0.0f) return bitsf(0xff800000u);
  if (x == bitsf(0x7f800000u)) return x;
  int bias = 0;
  if (x < 1.17549435e-38f) { x = x * 8388608.0f; bias = -23; }  // denormal input
  uint32_t u = fbits(x);
  int e = (int)((u >> 23) & 0xff) - 126 + bias;        // x = m * 2^e, m in [0.5, 1)
  float m = bitsf((u & 0x007fffffu) | 0x3f000000u);
  if (m < 0.707106781186547524f) { e -= 1; m = m + m - 1.0f; }
  else { m = m - 1.0f; }
  float z = m * m;
  float y = ((((((((7.0376836292e-2f * m - 1.1514610310e-1f) * m + 1.1676998740e-1f) * m
                  - 1.2420140846e-1f) * m + 1.4249322787e-1f) * m - 1.6668057665e-1f) * m
               + 2.0000714765e-1f) * m - 2.4999993993e-1f) * m + 3.3333331174e-1f) * m * z;
  float fe = (float)e;
  y = y + -2.12194440e-4f * fe;
  y = y + -0.5f * z;
  float r = m + y;
  r = r + 0.693359375f * fe;
  return r;
}

// GLSL pow(x, y) (spec: exp2(y * log2(x)); undefined for x < 0).
GM_FN float pow_(float x, float y) {
#if GM_HW
  return powf(x, y);
#endif
  if (y == 0.0f) return 1.0f;
  if (x == 1.0f) return 1.0f;
  return exp_(y * log_(x));
}

}  // namespace gm
