// tmath.h -- the float transcendentals of the path tracer, shared verbatim by the HIP
// kernels (dev_math.h) and the CPU parity oracle (oracle/oracle_math.h), so that both
// produce the same float for every argument.
//
// The reference calls float libm (sinf, cosf, expf, logf, powf, atan2f, asinf, acosf via
// hippt::, HostDeviceCommon/Math.h:141-229) on the CPU and the device library's float
// functions on the GPU; neither is reproducible on the other.  Here every function is one
// fixed sequence of IEEE operations (+, -, *, /, sqrt, fma, rint, frexp, ldexp: exact or
// correctly rounded on x86-64 and gfx950 alike; both sides compiled with -ffp-contract=off),
// so the oracle and the kernels agree bit for bit:
// * sin / cos / exp / log / atan2 / asin / acos (MPT_TMATH_F32, the default): single
//   precision -- Cody-Waite reductions (sin / cos: in double) and the Cephes single-precision minimax
//   polynomials (Horner in fmaf) -- within 2 ulp of the correctly rounded float for sin /
//   cos, 1 for exp / log, 3 for atan2, 4 for asin / acos (tests/test_tmath.py), the accuracy
//   class of the device library's float functions the reference's GPU build calls;
// * pow, and every function with MPT_TMATH_F32=0: a short double-precision approximation of
//   the float argument (relative error below 1e-14: Cody-Waite reduction + truncated series
//   whose tail is < 1e-16) rounded once to float -- the correctly rounded float except within
//   ~1e-14 of a rounding tie.
// Arguments outside the reduced ranges (huge, infinite, NaN, zero, non-positive for log /
// pow, results beyond or below the normal float range) go to the platform's double libm,
// whose special values are exact.  The single-precision functions cut C3's shading time by
// 4.5 % against the double ones (profiles/r05g_c3_tmath_f32_ab.jsonl).
#ifndef MPT_TMATH_H
#define MPT_TMATH_H

#include <math.h>

#if defined(__HIPCC__)
#define TM_FN __host__ __device__ static inline
#else
#define TM_FN static inline
#endif

// MPT_TMATH_F32 (default 1): sin / cos / exp / log / atan2 / asin / acos in single precision
// (below); 0: every function through the double-precision approximations.  pow stays double
// either way (y ln x needs more than float's precision for large exponents).
#ifndef MPT_TMATH_F32
#define MPT_TMATH_F32 1
#endif

namespace tmath {

// pi/2 = PIO2_HI + PIO2_LO with PIO2_HI on 33 bits (k * PIO2_HI exact for |k| < 2^20)
constexpr double PIO2_HI = 1.57079632673412561417e+00;
constexpr double PIO2_LO = 6.07710050650619224932e-11;
constexpr double INV_PIO2 = 6.36619772367581382433e-01;
// ln 2 = LN2_HI + LN2_LO with LN2_HI on 32 bits
constexpr double LN2_HI = 6.93147180369123816490e-01;
constexpr double LN2_LO = 1.90821492927058770002e-10;
constexpr double INV_LN2 = 1.44269504088896338700e+00;
constexpr double PI = 3.14159265358979323846;
constexpr double PIO2 = 1.57079632679489661923;
constexpr double PIO4 = 0.78539816339744830962;
constexpr double PIO8 = 0.39269908169872415481;
constexpr double TAN_PIO8 = 0.41421356237309504880;    // tan(pi/8) = sqrt(2) - 1
constexpr double TAN_PIO16 = 0.19891236737965800691;   // tan(pi/16)
constexpr double TAN_3PIO16 = 0.66817863791929891999;  // tan(3 pi/16)

// sin(r), |r| <= pi/4 + 1e-9: Taylor series through r^15 (tail < 5e-17)
TM_FN double sin_kernel(double r) {
    const double z = r * r;
    return r + r * z * (-1.0 / 6.0 + z * (1.0 / 120.0 + z * (-1.0 / 5040.0 + z * (1.0 / 362880.0 +
           z * (-1.0 / 39916800.0 + z * (1.0 / 6227020800.0 + z * (-1.0 / 1307674368000.0)))))));
}
// cos(r), |r| <= pi/4 + 1e-9: Taylor series through r^16 (tail < 2e-18)
TM_FN double cos_kernel(double r) {
    const double z = r * r;
    return 1.0 + z * (-0.5 + z * (1.0 / 24.0 + z * (-1.0 / 720.0 + z * (1.0 / 40320.0 + z * (-1.0 / 3628800.0 +
           z * (1.0 / 479001600.0 + z * (-1.0 / 87178291200.0 + z * (1.0 / 20922789888000.0))))))));
}
// x = k pi/2 + r, |r| <= pi/4 (+ rounding), for |x| <= 1e5: x - k PIO2_HI is exact
// (Sterbenz), the PIO2_LO product adds < 1e-21
TM_FN int reduce_pio2(double x, double& r) {
    const double k = rint(x * INV_PIO2);
    r = (x - k * PIO2_HI) - k * PIO2_LO;
    return (int)k;
}

// e^t for |t| <= 200: t = k ln2 + r, |r| <= ln2 / 2, Taylor series through r^13 (tail < 5e-18)
TM_FN double exp_d(double t) {
    const double k = rint(t * INV_LN2);
    const double r = (t - k * LN2_HI) - k * LN2_LO;
    const double p = 1.0 + r * (1.0 + r * (0.5 + r * (1.0 / 6.0 + r * (1.0 / 24.0 + r * (1.0 / 120.0 + r * (1.0 / 720.0 +
                     r * (1.0 / 5040.0 + r * (1.0 / 40320.0 + r * (1.0 / 362880.0 + r * (1.0 / 3628800.0 +
                     r * (1.0 / 39916800.0 + r * (1.0 / 479001600.0 + r * (1.0 / 6227020800.0)))))))))))));
    return ldexp(p, (int)k);
}
// ln x for finite x > 0: x = m 2^e with m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(s),
// s = (m - 1) / (m + 1), |s| <= 0.1716, series through s^21 (tail < 3e-18)
TM_FN double log_d(double x) {
    int e;
    double m = frexp(x, &e);
    if (m < 0.70710678118654752440) { m *= 2.0; e -= 1; }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double p = z * (1.0 / 3.0 + z * (1.0 / 5.0 + z * (1.0 / 7.0 + z * (1.0 / 9.0 + z * (1.0 / 11.0 +
                     z * (1.0 / 13.0 + z * (1.0 / 15.0 + z * (1.0 / 17.0 + z * (1.0 / 19.0 + z * (1.0 / 21.0))))))))));
    const double lm = 2.0 * s + 2.0 * s * p;
    return (double)e * LN2_HI + ((double)e * LN2_LO + lm);
}
#if MPT_TMATH_F32
// ---- single precision: Cody-Waite reductions + the Cephes single-precision minimax
// polynomials, fmaf Horner (one IEEE fma per step on x86-64 libm and gfx950 alike).
// Results within 1-2 ulp of the correctly rounded float; the ranges outside the reductions go
// to the platform's double libm as above.
constexpr float F_INV_PIO2 = 0.636619772367581343f;
constexpr float F_LN2_HI = 0.693359375f;
constexpr float F_LN2_LO = -2.12194440e-4f;
constexpr float F_LOG2E = 1.44269504088896341f;
constexpr float F_PI = 3.14159265358979323846f, F_PIO2 = 1.57079632679489661923f, F_PIO4 = 0.78539816339744830962f;

TM_FN float sin_kernel_f(float r) {
    const float z = r * r;
    return fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
}
TM_FN float cos_kernel_f(float r) {
    const float z = r * r;
    return fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f) * z, z,
                fmaf(-0.5f, z, 1.0f));
}
// x = k pi/2 + r: k from float, the reduction itself in double (two products and two
// differences, as reduce_pio2) so that r keeps its relative accuracy next to the zeros of sin /
// cos, where a float Cody-Waite reduction loses up to 3 digits
TM_FN int reduce_pio2_f(float x, float& r) {
    const float k = rintf(x * F_INV_PIO2);
    const double kd = (double)k;
    r = (float)(((double)x - kd * PIO2_HI) - kd * PIO2_LO);
    return (int)k;
}
TM_FN float sinf_(float x) {
    if (!(fabsf(x) <= 1.0e5f) || x == 0.0f) return (float)sin((double)x);
    float r;
    const int q = reduce_pio2_f(x, r) & 3;
    const float s = (q & 1) ? cos_kernel_f(r) : sin_kernel_f(r);
    return (q & 2) ? -s : s;
}
TM_FN float cosf_(float x) {
    if (!(fabsf(x) <= 1.0e5f)) return (float)cos((double)x);
    float r;
    const int q = reduce_pio2_f(x, r) & 3;
    const float c = (q & 1) ? sin_kernel_f(r) : cos_kernel_f(r);
    return (q == 1 || q == 2) ? -c : c;
}
TM_FN void sincosf_(float x, float& sf, float& cf) {
    if (!(fabsf(x) <= 1.0e5f)) { sf = (float)sin((double)x); cf = (float)cos((double)x); return; }
    float r;
    const int q = reduce_pio2_f(x, r) & 3;
    const float sk = sin_kernel_f(r), ck = cos_kernel_f(r);
    const float s = (q & 1) ? ck : sk, c = (q & 1) ? sk : ck;
    sf = x == 0.0f ? x : ((q & 2) ? -s : s);
    cf = (q == 1 || q == 2) ? -c : c;
}
TM_FN float expf_(float x) {
    if (!(fabsf(x) <= 87.0f)) return (float)exp((double)x);
    const float k = rintf(x * F_LOG2E);
    const float r = fmaf(-k, F_LN2_LO, fmaf(-k, F_LN2_HI, x));
    const float p = fmaf(fmaf(fmaf(fmaf(fmaf(1.9875691500e-4f, r, 1.3981999507e-3f), r, 8.3334519073e-3f), r,
                                    4.1665795894e-2f), r, 1.6666665459e-1f), r, 5.0000001201e-1f);
    return ldexpf(fmaf(p, r * r, r) + 1.0f, (int)k);
}
// ln x, finite x > 0: x = m 2^e, m in [sqrt(1/2), sqrt(2)), f = m - 1 (exact)
TM_FN float log_f(float x, int& e, float& f) {
    float m = frexpf(x, &e);
    if (m < 0.707106781186547524f) { m = m + m; e -= 1; }
    f = m - 1.0f;
    const float z = f * f;
    float y = fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(7.0376836292e-2f, f, -1.1514610310e-1f), f, 1.1676998740e-1f), f,
                   -1.2420140846e-1f), f, 1.4249322787e-1f), f, -1.6668057665e-1f), f, 2.0000714765e-1f), f,
                   -2.4999993993e-1f), f, 3.3333331174e-1f) * f * z;
    y = fmaf((float)e, F_LN2_LO, y);
    y = fmaf(-0.5f, z, y);
    return fmaf((float)e, F_LN2_HI, f + y);
}
TM_FN float logf_(float x) {
    if (!(x > 0.0f) || !(x < INFINITY) || x < 1.17549435e-38f) return (float)log((double)x);
    int e;
    float f;
    return log_f(x, e, f);
}
#else
TM_FN float sinf_(float xf) {
    const double x = xf;
    if (!(fabs(x) <= 1.0e5) || x == 0.0) return (float)sin(x);
    double r;
    const int q = reduce_pio2(x, r) & 3;
    const double s = (q & 1) ? cos_kernel(r) : sin_kernel(r);
    return (float)((q & 2) ? -s : s);
}
TM_FN float cosf_(float xf) {
    const double x = xf;
    if (!(fabs(x) <= 1.0e5)) return (float)cos(x);
    double r;
    const int q = reduce_pio2(x, r) & 3;
    const double c = (q & 1) ? sin_kernel(r) : cos_kernel(r);
    return (float)((q == 1 || q == 2) ? -c : c);
}

// sinf_(x) and cosf_(x) from one reduction (bit-identical to the two calls)
TM_FN void sincosf_(float xf, float& sf, float& cf) {
    const double x = xf;
    if (!(fabs(x) <= 1.0e5)) { sf = (float)sin(x); cf = (float)cos(x); return; }
    double r;
    const int q = reduce_pio2(x, r) & 3;
    const double sk = sin_kernel(r), ck = cos_kernel(r);
    const double s = (q & 1) ? ck : sk, c = (q & 1) ? sk : ck;
    sf = x == 0.0 ? (float)sin(x) : (float)((q & 2) ? -s : s);
    cf = (float)((q == 1 || q == 2) ? -c : c);
}

TM_FN float expf_(float xf) {
    const double x = xf;
    if (!(fabs(x) <= 100.0)) return (float)exp(x);
    return (float)exp_d(x);
}

TM_FN float logf_(float xf) {
    const double x = xf;
    if (!(x > 0.0) || !(x < INFINITY)) return (float)log(x);
    return (float)log_d(x);
}

#endif

// x^y for finite x > 0, finite y != 0, x != 1, |y ln x| <= 200 (everything else: libm)
TM_FN float powf_(float xf, float yf) {
    const double x = xf, y = yf;
    if (!(x > 0.0) || !(x < INFINITY) || !(fabs(y) < INFINITY) || y == 0.0 || x == 1.0) return (float)pow(x, y);
    const double t = y * log_d(x);
    if (!(fabs(t) <= 200.0)) return (float)pow(x, y);
    return (float)exp_d(t);
}

#if MPT_TMATH_F32
// atan t, t in [0, inf) finite: Cephes atanf's reduction by tan(3pi/8) / tan(pi/8)
TM_FN float atan_f(float t) {
    float y = 0.0f, u = t;
    if (t > 2.414213562373095f) { y = F_PIO2; u = -1.0f / t; }
    else if (t > 0.4142135623730950f) { y = F_PIO4; u = (t - 1.0f) / (t + 1.0f); }
    const float z = u * u;
    return y + fmaf(fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                         -3.33329491539e-1f) * z, u, u);
}
TM_FN float atan2_f(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const bool swap = ay > ax;
    float a = atan_f(swap ? ax / ay : ay / ax);
    if (swap) a = F_PIO2 - a;
    if (x < 0.0f) a = F_PI - a;
    return y < 0.0f ? -a : a;
}
TM_FN float atan2f_(float y, float x) {
    if (!(fabsf(x) < INFINITY) || !(fabsf(y) < INFINITY) || x == 0.0f || y == 0.0f) return (float)atan2((double)y, (double)x);
    return atan2_f(y, x);
}
TM_FN float asinf_(float x) {
    if (!(fabsf(x) < 1.0f) || x == 0.0f) return (float)asin((double)x);
    return atan2_f(x, sqrtf((1.0f - x) * (1.0f + x)));
}
TM_FN float acosf_(float x) {
    if (!(fabsf(x) < 1.0f) || x == 0.0f) return (float)acos((double)x);
    return atan2_f(sqrtf((1.0f - x) * (1.0f + x)), x);
}
#else
// atan(u), |u| <= tan(pi/16) = 0.1989: series through u^23 (tail < 2e-18)
TM_FN double atan_kernel(double u) {
    const double z = u * u;
    return u + u * z * (-1.0 / 3.0 + z * (1.0 / 5.0 + z * (-1.0 / 7.0 + z * (1.0 / 9.0 + z * (-1.0 / 11.0 + z * (1.0 / 13.0 +
           z * (-1.0 / 15.0 + z * (1.0 / 17.0 + z * (-1.0 / 19.0 + z * (1.0 / 21.0 + z * (-1.0 / 23.0)))))))))));
}
// atan2 for finite, non-zero y and x: t = min / max in (0, 1], atan t = j pi/8 + atan((t - c) / (1 + t c)),
// c = tan(j pi/8), the reduced argument within tan(pi/16)
TM_FN double atan2_d(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const bool swap = ay > ax;
    const double t = swap ? ax / ay : ay / ax;
    double a;
    if (t <= TAN_PIO16) a = atan_kernel(t);
    else if (t <= TAN_3PIO16) a = PIO8 + atan_kernel((t - TAN_PIO8) / (1.0 + t * TAN_PIO8));
    else a = PIO4 + atan_kernel((t - 1.0) / (1.0 + t));
    if (swap) a = PIO2 - a;
    if (x < 0.0) a = PI - a;
    return y < 0.0 ? -a : a;
}
TM_FN float atan2f_(float yf, float xf) {
    const double y = yf, x = xf;
    if (!(fabs(x) < INFINITY) || !(fabs(y) < INFINITY) || x == 0.0 || y == 0.0) return (float)atan2(y, x);
    return (float)atan2_d(y, x);
}
// asin x = atan2(x, sqrt(1 - x^2)), acos x = atan2(sqrt(1 - x^2), x); (1 - x)(1 + x) is exact
// for a float x
TM_FN float asinf_(float xf) {
    const double x = xf;
    if (!(fabs(x) < 1.0) || x == 0.0) return (float)asin(x);
    return (float)atan2_d(x, sqrt((1.0 - x) * (1.0 + x)));
}
TM_FN float acosf_(float xf) {
    const double x = xf;
    if (!(fabs(x) < 1.0) || x == 0.0) return (float)acos(x);
    return (float)atan2_d(sqrt((1.0 - x) * (1.0 + x)), x);
}

#endif

}  // namespace tmath

#undef TM_FN
#endif
