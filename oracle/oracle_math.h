/*
 * oracle_math.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never shipped).
 *
 * Scalar float3 / colour arithmetic used by the CPU restatement of the reference
 * megakernel.  Semantics follow the reference's host build of its device code:
 *   hippt:: helpers ........ HostDeviceCommon/Math.h:61-235 (CPU branch :141-229)
 *   ColorRGB32F ............ HostDeviceCommon/Color.h:61-110
 *   Xorshift32Generator .... HostDeviceCommon/Xorshift.h:17-65
 *   wang_hash .............. Device/includes/Hash.h:11-19
 *   build_ONB & frames ..... Device/includes/ONB.h:18-78
 *
 * The HIPRT vector library the reference relies on (hiprt/impl/Math.h, HIPRT 2.4,
 * an un-vendored submodule: thirdparties/HIPRT-Fork is empty) is restated from its
 * published behaviour: dot = x*x'+y*y'+z*z' evaluated left to right, cross the usual
 * determinant form, normalize(v) = v / sqrt(dot(v, v)).
 *
 * Transcendentals: the reference calls float libm (sinf, cosf, powf ...).  The
 * oracle and the HIP product share hiprt-path-tracer_amd/csrc/tmath.h: sin / cos / exp /
 * log / atan2 / asin / acos as single-precision minimax polynomials within 1-4 ulp of the
 * correctly rounded float, pow in double precision rounded once (tests/test_tmath.py pins
 * both against libm) -- one sequence of IEEE operations, so both sides agree bit for bit.
 * Built with -DORACLE_LIBM (liboracle_libm.so) the oracle calls libm's float functions
 * instead, as the reference's CPU build does: tests/test_libm_oracle.py bounds the image
 * difference that sharing the layer could hide by the north_star tolerance.
 * Compile with -ffp-contract=off (no fused multiply-add), like the reference's
 * x86-64 CPU build.
 */
#ifndef ORACLE_MATH_H
#define ORACLE_MATH_H

#include <cmath>
#include <cstdint>

#include "../hiprt-path-tracer_amd/csrc/tmath.h"

namespace orc {

struct f2 { float x, y; };
struct f3 { float x, y, z; };

inline f2 mk2(float x, float y) { return f2{x, y}; }
inline f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
inline f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
inline f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline f3 operator*(f3 a, float k) { return mk3(a.x * k, a.y * k, a.z * k); }
inline f3 operator*(float k, f3 a) { return mk3(k * a.x, k * a.y, k * a.z); }
inline f3 operator/(f3 a, float k) { return mk3(a.x / k, a.y / k, a.z / k); }
inline f3 operator/(f3 a, f3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline f3& operator+=(f3& a, f3 b) { a = a + b; return a; }
inline f3& operator*=(f3& a, float k) { a = a * k; return a; }
inline f2 operator-(f2 a, f2 b) { return mk2(a.x - b.x, a.y - b.y); }
inline f2 operator*(f2 a, float k) { return mk2(a.x * k, a.y * k); }
inline f2 operator+(f2 a, f2 b) { return mk2(a.x + b.x, a.y + b.y); }

inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline f3 cross(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline float length(f3 a) { return std::sqrt(dot(a, a)); }
inline f3 normalize(f3 a) { return a / std::sqrt(dot(a, a)); }
inline float fmaxr(float a, float b) { return a > b ? a : b; }   // hippt::max (Math.h:163 -> hiprt::max)
inline float fminr(float a, float b) { return a < b ? a : b; }
inline int imin(int a, int b) { return a < b ? a : b; }
inline int imax(int a, int b) { return a > b ? a : b; }
inline float clampf(float lo, float hi, float v) { return fminr(hi, fmaxr(lo, v)); } // hippt::clamp(min,max,val)
inline float absf(float a) { return std::fabs(a); }
inline float lerpf(float a, float b, float t) { return (1.0f - t) * a + t * b; }
inline f3 absv(f3 a) { return mk3(absf(a.x), absf(a.y), absf(a.z)); }
inline bool is_zero(float x) { return x < 1.0e-10f && x > -1.0e-10f; }
inline float sq(float x) { return x * x; }
inline float pow3(float x) { return x * x * x; }
inline float pow4(float x) { float x2 = x * x; return x2 * x2; }
inline float pow5(float x) { float x2 = x * x; float x4 = x2 * x2; return x4 * x; }
inline float pow6(float x) { float x2 = x * x; float x4 = x2 * x2; return x4 * x2; }

#ifndef ORACLE_LIBM
// parity transcendentals (see header comment): the product's tmath.h, verbatim
inline float psin(float x) { return tmath::sinf_(x); }
inline float pcos(float x) { return tmath::cosf_(x); }
inline float pexp(float x) { return tmath::expf_(x); }
inline float plog(float x) { return tmath::logf_(x); }
inline float ppow(float x, float y) { return tmath::powf_(x, y); }
inline float patan2(float y, float x) { return tmath::atan2f_(y, x); }
inline float pasin(float x) { return tmath::asinf_(x); }
inline float pacos(float x) { return tmath::acosf_(x); }
#else
// the reference CPU build's float libm calls (Math.h:141-229: sinf, cosf, expf, logf, powf, ...)
inline float psin(float x) { return std::sin(x); }
inline float pcos(float x) { return std::cos(x); }
inline float pexp(float x) { return std::exp(x); }
inline float plog(float x) { return std::log(x); }
inline float ppow(float x, float y) { return std::pow(x, y); }
inline float patan2(float y, float x) { return std::atan2(y, x); }
inline float pasin(float x) { return std::asin(x); }
inline float pacos(float x) { return std::acos(x); }
#endif
inline float psqrt(float x) { return std::sqrt(x); }

constexpr float PI = 3.14159265358979323846f;      // Math.h:144
constexpr float TWO_PI = 6.28318530717958647693f;
constexpr float INV_PI = 0.31830988618379067154f;
constexpr float INV_2_PI = 0.15915494309189533577f;
constexpr float TWO_PIPI = 19.73920880217871723767f;

struct Col {
    float r, g, b;
    Col() : r(0), g(0), b(0) {}
    explicit Col(float v) : r(v), g(v), b(v) {}
    Col(float r_, float g_, float b_) : r(r_), g(g_), b(b_) {}
    float luminance() const { return 0.3086f * r + 0.6094f * g + 0.0820f * b; }   // Color.h:85
    float max_component() const { return fmaxr(r, fmaxr(g, b)); }
    bool has_nan() const { return std::isnan(r) || std::isnan(g) || std::isnan(b); }
    bool is_black() const { return !(r > 0.0f || g > 0.0f || b > 0.0f); }
    bool is_white() const { return r == 1.0f && g == 1.0f && b == 1.0f; }
    void clamp(float lo, float hi) { r = clampf(lo, hi, r); g = clampf(lo, hi, g); b = clampf(lo, hi, b); }
    float& operator[](int i) { return (&r)[i]; }
};
inline Col operator+(Col a, Col b) { return Col(a.r + b.r, a.g + b.g, a.b + b.b); }
inline Col operator-(Col a, Col b) { return Col(a.r - b.r, a.g - b.g, a.b - b.b); }
inline Col operator-(Col a) { return Col(-a.r, -a.g, -a.b); }
inline Col operator*(Col a, Col b) { return Col(a.r * b.r, a.g * b.g, a.b * b.b); }
inline Col operator*(Col c, float k) { return Col(c.r * k, c.g * k, c.b * k); }
inline Col operator*(float k, Col c) { return Col(c.r * k, c.g * k, c.b * k); }
inline Col operator/(Col a, Col b) { return Col(a.r / b.r, a.g / b.g, a.b / b.b); }
inline Col operator/(Col c, float k) { return Col(c.r / k, c.g / k, c.b / k); }
inline Col operator/(float k, Col c) { return Col(k / c.r, k / c.g, k / c.b); }
inline Col& operator+=(Col& a, Col b) { a = a + b; return a; }
inline Col& operator*=(Col& a, Col b) { a = a * b; return a; }
inline Col& operator*=(Col& a, float k) { a = a * k; return a; }
inline Col& operator/=(Col& a, float k) { a = a / k; return a; }
inline Col& operator/=(Col& a, Col b) { a = a / b; return a; }
inline Col cmax(Col a, Col b) { return Col(fmaxr(a.r, b.r), fmaxr(a.g, b.g), fmaxr(a.b, b.b)); }
inline Col lerpc(Col a, Col b, float t) { return (1.0f - t) * a + t * b; }
inline Col cexp(Col c) { return Col(pexp(c.r), pexp(c.g), pexp(c.b)); }
inline Col clog(Col c) { return Col(plog(c.r), plog(c.g), plog(c.b)); }
inline Col csqrt(Col c) { return Col(psqrt(c.r), psqrt(c.g), psqrt(c.b)); }
inline Col cpow(Col c, float k) { return Col(ppow(c.r, k), ppow(c.g, k), ppow(c.b, k)); }

inline uint32_t wang_hash(uint32_t seed) {                 // Hash.h:11-19
    seed = (seed ^ 61u) ^ (seed >> 16);
    seed *= 9u;
    seed = seed ^ (seed >> 4);
    seed *= 0x27d4eb2du;
    seed = seed ^ (seed >> 15);
    return seed;
}

struct Rng {                                                // Xorshift.h:17-65
    uint32_t s;
    explicit Rng(uint32_t seed = 42u) : s(seed) {}
    uint32_t xorshift32() { uint32_t x = s; x ^= x << 13; x ^= x >> 17; x ^= x << 5; return s = x; }
    float operator()() { float a = (float)xorshift32() / (float)0xffffffffu; return fminr(a, 1.0f - 1.0e-7f); }
    int random_index(int n) { int r = (int)((float)xorshift32() / (float)0xffffffffu * (float)n); return imin(r, n - 1); }
};

inline void build_onb(f3 n, f3& t, f3& b) {                 // ONB.h:18-31
    if (n.z < -0.99998796f) { t = mk3(0.0f, -1.0f, 0.0f); b = mk3(-1.0f, 0.0f, 0.0f); return; }
    float nxa = -n.x / (1.0f + n.z);
    t = mk3(1.0f + n.x * nxa, nxa * n.y, -n.x);
    b = mk3(t.y, 1.0f - n.y * n.y / (1.0f + n.z), -n.y);
}
inline void build_rotated_onb(f3 n, f3& t, f3& b, float rot) {   // ONB.h:36-44
    f3 up = absf(n.z) < 0.9999999f ? mk3(0.0f, 0.0f, 1.0f) : mk3(1.0f, 0.0f, 0.0f);
    t = normalize(cross(up, n));
    float c = pcos(rot), s = psin(rot);
    t = t * c + cross(n, t) * s + n * dot(n, t) * (1.0f - c);
    b = cross(n, t);
}
inline f3 local_to_world(f3 t, f3 b, f3 n, f3 v) { return normalize(v.x * t + v.y * b + v.z * n); }
inline f3 world_to_local(f3 t, f3 b, f3 n, f3 v) { return normalize(mk3(dot(v, t), dot(v, b), dot(v, n))); }
inline f3 local_to_world(f3 n, f3 v) { f3 t, b; build_onb(n, t, b); return local_to_world(t, b, n, v); }

inline f3 reflect_ray(f3 d, f3 n) { return -d + 2.0f * dot(d, n) * n; }   // Sampling.h:151
inline bool refract_ray(f3 d, f3 n, f3& out, float eta) {                 // Sampling.h:161-174
    float noi = dot(d, n);
    float sin2 = 1.0f - noi * noi;
    float root = 1.0f - sin2 / (eta * eta);
    if (root < 0.0f) return false;
    float cos_t = psqrt(root);
    out = -d / eta + (noi / eta - cos_t) * n;
    return true;
}
inline float balance_heuristic(float a, float na, float b, float nb) { return a / (na * a + nb * b); }  // Sampling.h:108
inline float balance_heuristic(float a, float b) { return balance_heuristic(a, 1.0f, b, 1.0f); }

}  // namespace orc
#endif
