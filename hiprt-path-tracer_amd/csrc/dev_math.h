// dev_math.h -- device math for the MI355X path tracer.
//
// Semantics of the reference's shared HostDeviceCommon math
// (src/HostDeviceCommon/Math.h:61-296, Color.h:61-110, Xorshift.h:17-65,
// Device/includes/Hash.h:11-19, Device/includes/ONB.h:18-78).
// The whole library is compiled with -ffp-contract=off so that every product and
// sum rounds separately, as on the reference's x86-64 CPU build; fused multiply-adds
// are only written explicitly where bit-exactness with the reference does not matter
// (BVH box tests).  Transcendentals are tmath.h's double-precision kernels rounded once to
// float, the same code as the CPU oracle's.
#ifndef MPT_DEV_MATH_H
#define MPT_DEV_MATH_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tmath.h"

#define DEV __device__ __forceinline__

namespace mpt {

struct v2 { float x, y; };
struct v3 { float x, y, z; };

DEV v2 mk2(float x, float y) { v2 r; r.x = x; r.y = y; return r; }
DEV v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
DEV v3 operator+(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV v3 operator-(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV v3 operator-(v3 a) { return mk3(-a.x, -a.y, -a.z); }
DEV v3 operator*(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV v3 operator*(v3 a, float k) { return mk3(a.x * k, a.y * k, a.z * k); }
DEV v3 operator*(float k, v3 a) { return mk3(k * a.x, k * a.y, k * a.z); }
DEV v3 operator/(v3 a, float k) { return mk3(a.x / k, a.y / k, a.z / k); }
DEV v3& operator+=(v3& a, v3 b) { a = a + b; return a; }
DEV v3& operator*=(v3& a, float k) { a = a * k; return a; }
DEV v2 operator-(v2 a, v2 b) { return mk2(a.x - b.x, a.y - b.y); }
DEV v2 operator+(v2 a, v2 b) { return mk2(a.x + b.x, a.y + b.y); }
DEV v2 operator*(v2 a, float k) { return mk2(a.x * k, a.y * k); }

DEV float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV v3 cross(v3 a, v3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV float length(v3 a) { return sqrtf(dot(a, a)); }
DEV v3 normalize(v3 a) { return a / sqrtf(dot(a, a)); }
DEV float maxr(float a, float b) { return a > b ? a : b; }
DEV float minr(float a, float b) { return a < b ? a : b; }
DEV int imin(int a, int b) { return a < b ? a : b; }
DEV float clampr(float lo, float hi, float v) { return minr(hi, maxr(lo, v)); }
DEV float absr(float a) { return fabsf(a); }
DEV float lerpr(float a, float b, float t) { return (1.0f - t) * a + t * b; }
DEV bool is_zero(float x) { return x < 1.0e-10f && x > -1.0e-10f; }
DEV float sq(float x) { return x * x; }
DEV float pow3(float x) { return x * x * x; }
DEV float pow4(float x) { float x2 = x * x; return x2 * x2; }
DEV float pow6(float x) { float x2 = x * x; float x4 = x2 * x2; return x4 * x2; }

// Transcendentals: tmath.h -- double-precision kernels rounded once to float, the same code
// as the CPU oracle's.  MPT_TRANS_OCML (A/B experiments only) restores the previous
// layer: the device library's double functions, out of line.
#ifdef MPT_TRANS_OCML
#define TRANS static __device__ __attribute__((noinline))
TRANS float psin(float x) { return (float)::sin((double)x); }
TRANS float pcos(float x) { return (float)::cos((double)x); }
TRANS float pexp(float x) { return (float)::exp((double)x); }
TRANS float plog(float x) { return (float)::log((double)x); }
TRANS float ppow(float x, float y) { return (float)::pow((double)x, (double)y); }
TRANS float patan2(float y, float x) { return (float)::atan2((double)y, (double)x); }
TRANS float pasin(float x) { return (float)::asin((double)x); }
TRANS float pacos(float x) { return (float)::acos((double)x); }
TRANS float2 psincos(float x) { return make_float2((float)::sin((double)x), (float)::cos((double)x)); }
#elif defined(MPT_TRANS_FLOAT_UB)
// A/B experiments only (not bit-exact with the oracle): the device library's float
// functions, inline -- an upper bound of what cheaper transcendentals could gain
#define TRANS DEV
TRANS float psin(float x) { return ::sinf(x); }
TRANS float pcos(float x) { return ::cosf(x); }
TRANS float pexp(float x) { return ::expf(x); }
TRANS float plog(float x) { return ::logf(x); }
TRANS float ppow(float x, float y) { return ::powf(x, y); }
TRANS float patan2(float y, float x) { return ::atan2f(y, x); }
TRANS float pasin(float x) { return ::asinf(x); }
TRANS float pacos(float x) { return ::acosf(x); }
TRANS float2 psincos(float x) { float s, c; ::sincosf(x, &s, &c); return make_float2(s, c); }
#else
// Out of line: inlined at their ~60 call sites they push k_shade from 272 to 1072 B of
// scratch per lane and k_trace<PATH> (the sRGB pow of the alpha test) from 4 to 3 waves/SIMD.
#ifdef MPT_TRANS_INLINE
#define TRANS DEV
#else
#define TRANS static __device__ __attribute__((noinline))
#endif
TRANS float psin(float x) { return tmath::sinf_(x); }
TRANS float pcos(float x) { return tmath::cosf_(x); }
// (psin(x), pcos(x)) with one call and one range reduction
TRANS float2 psincos(float x) { float s, c; tmath::sincosf_(x, s, c); return make_float2(s, c); }
TRANS float pexp(float x) { return tmath::expf_(x); }
TRANS float plog(float x) { return tmath::logf_(x); }
TRANS float ppow(float x, float y) { return tmath::powf_(x, y); }
TRANS float patan2(float y, float x) { return tmath::atan2f_(y, x); }
TRANS float pasin(float x) { return tmath::asinf_(x); }
TRANS float pacos(float x) { return tmath::acosf_(x); }
#endif

// Streaming path state -- written by one wavefront stage and read once by the next (rays,
// hits, throughput, NEE records, staged queries): non-temporal accesses (the 'nt' bit: L2
// evict-first) so that the data every path re-reads -- the emissive-triangle table, materials,
// the envmap alias entries, BVH nodes -- stays in the XCDs' L2 instead of being pushed out by
// ~15 GB of path state per shading launch.  Same values either way.
#ifndef MPT_NT_STREAM
#define MPT_NT_STREAM 1
#endif
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef unsigned nt_u4 __attribute__((ext_vector_type(4)));
DEV float4 ld_s(const float4* p) {
#if MPT_NT_STREAM
    const nt_f4 x = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
    return make_float4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
}
DEV void st_s(float4* p, float4 v) {
#if MPT_NT_STREAM
    const nt_f4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<nt_f4*>(p));
#else
    *p = v;
#endif
}
DEV uint4 ld_s(const uint4* p) {
#if MPT_NT_STREAM
    const nt_u4 x = __builtin_nontemporal_load(reinterpret_cast<const nt_u4*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
#else
    return *p;
#endif
}
DEV void st_s(uint4* p, uint4 v) {
#if MPT_NT_STREAM
    const nt_u4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<nt_u4*>(p));
#else
    *p = v;
#endif
}
template <typename T> DEV T ld_s(const T* p) {
#if MPT_NT_STREAM
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <typename T> DEV void st_s(T* p, T v) {
#if MPT_NT_STREAM
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

constexpr float PI = 3.14159265358979323846f;
constexpr float TWO_PI = 6.28318530717958647693f;
constexpr float INV_PI = 0.31830988618379067154f;
constexpr float INV_2_PI = 0.15915494309189533577f;
constexpr float TWO_PIPI = 19.73920880217871723767f;

struct Col {
    float r, g, b;
};
DEV Col col(float v) { Col c; c.r = v; c.g = v; c.b = v; return c; }
DEV Col col(float r, float g, float b) { Col c; c.r = r; c.g = g; c.b = b; return c; }
DEV Col operator+(Col a, Col b) { return col(a.r + b.r, a.g + b.g, a.b + b.b); }
DEV Col operator-(Col a, Col b) { return col(a.r - b.r, a.g - b.g, a.b - b.b); }
DEV Col operator-(Col a) { return col(-a.r, -a.g, -a.b); }
DEV Col operator*(Col a, Col b) { return col(a.r * b.r, a.g * b.g, a.b * b.b); }
DEV Col operator*(Col c, float k) { return col(c.r * k, c.g * k, c.b * k); }
DEV Col operator*(float k, Col c) { return col(c.r * k, c.g * k, c.b * k); }
DEV Col operator/(Col a, Col b) { return col(a.r / b.r, a.g / b.g, a.b / b.b); }
DEV Col operator/(Col c, float k) { return col(c.r / k, c.g / k, c.b / k); }
DEV Col operator/(float k, Col c) { return col(k / c.r, k / c.g, k / c.b); }
DEV Col& operator+=(Col& a, Col b) { a = a + b; return a; }
DEV Col& operator*=(Col& a, Col b) { a = a * b; return a; }
DEV Col& operator*=(Col& a, float k) { a = a * k; return a; }
DEV Col& operator/=(Col& a, float k) { a = a / k; return a; }
DEV float lum(Col c) { return 0.3086f * c.r + 0.6094f * c.g + 0.0820f * c.b; }
DEV float maxc(Col c) { return maxr(c.r, maxr(c.g, c.b)); }
DEV bool has_nan(Col c) { return isnan(c.r) || isnan(c.g) || isnan(c.b); }
DEV bool is_black(Col c) { return !(c.r > 0.0f || c.g > 0.0f || c.b > 0.0f); }
DEV bool is_white(Col c) { return c.r == 1.0f && c.g == 1.0f && c.b == 1.0f; }
DEV Col clampc(Col c, float lo, float hi) { return col(clampr(lo, hi, c.r), clampr(lo, hi, c.g), clampr(lo, hi, c.b)); }
DEV Col lerpc(Col a, Col b, float t) { return (1.0f - t) * a + t * b; }
DEV Col cexp(Col c) { return col(pexp(c.r), pexp(c.g), pexp(c.b)); }
DEV Col clog(Col c) { return col(plog(c.r), plog(c.g), plog(c.b)); }
DEV Col csqrt(Col c) { return col(sqrtf(c.r), sqrtf(c.g), sqrtf(c.b)); }
DEV Col cpow(Col c, float k) { return col(ppow(c.r, k), ppow(c.g, k), ppow(c.b, k)); }

DEV uint32_t wang_hash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}

struct Rng {
    uint32_t s;
    DEV uint32_t next() { uint32_t x = s; x ^= x << 13; x ^= x >> 17; x ^= x << 5; s = x; return x; }
    DEV float operator()() { float a = (float)next() / (float)0xffffffffu; return minr(a, 1.0f - 1.0e-7f); }
    DEV int random_index(int n) { int r = (int)((float)next() / (float)0xffffffffu * (float)n); return imin(r, n - 1); }
};
DEV Rng make_rng(uint32_t s) { Rng r; r.s = s; return r; }

DEV void build_onb(v3 n, v3& t, v3& b) {
    if (n.z < -0.99998796f) { t = mk3(0.0f, -1.0f, 0.0f); b = mk3(-1.0f, 0.0f, 0.0f); return; }
    float nxa = -n.x / (1.0f + n.z);
    t = mk3(1.0f + n.x * nxa, nxa * n.y, -n.x);
    b = mk3(t.y, 1.0f - n.y * n.y / (1.0f + n.z), -n.y);
}
DEV void build_rotated_onb(v3 n, v3& t, v3& b, float rot) {
    v3 up = absr(n.z) < 0.9999999f ? mk3(0.0f, 0.0f, 1.0f) : mk3(1.0f, 0.0f, 0.0f);
    t = normalize(cross(up, n));
    // rot == +-0 (no anisotropy rotation, the common case): cos = 1, sin = rot exactly
    float c = 1.0f, s = rot;
    if (rot != 0.0f) { const float2 sc = psincos(rot); s = sc.x; c = sc.y; }
    t = t * c + cross(n, t) * s + n * dot(n, t) * (1.0f - c);
    b = cross(n, t);
}
DEV v3 to_world(v3 t, v3 b, v3 n, v3 v) { return normalize(v.x * t + v.y * b + v.z * n); }
DEV v3 to_local(v3 t, v3 b, v3 n, v3 v) { return normalize(mk3(dot(v, t), dot(v, b), dot(v, n))); }
DEV v3 reflect_ray(v3 d, v3 n) { return -d + 2.0f * dot(d, n) * n; }
DEV bool refract_ray(v3 d, v3 n, v3& out, float eta) {
    float noi = dot(d, n);
    float s2 = 1.0f - noi * noi;
    float root = 1.0f - s2 / (eta * eta);
    if (root < 0.0f) return false;
    float ct = sqrtf(root);
    out = -d / eta + (noi / eta - ct) * n;
    return true;
}
DEV float balance(float a, float na, float b, float nb) { return a / (na * a + nb * b); }
DEV float balance(float a, float b) { return balance(a, 1.0f, b, 1.0f); }

// matrix_X_point / matrix_X_vec (Math.h:237-296)
DEV v3 mat_x_point(const float m[4][4], v3 p) {
    float xt = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
    float yt = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
    float zt = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
    float wt = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
    float iw = 1.0f;
    if (!is_zero(wt)) iw = 1.0f / wt;
    return mk3(xt * iw, yt * iw, zt * iw);
}
DEV v3 mat_x_vec(const float m[4][4], v3 u) {
    float xt = m[0][0] * u.x + m[1][0] * u.y + m[2][0] * u.z;
    float yt = m[0][1] * u.x + m[1][1] * u.y + m[2][1] * u.z;
    float zt = m[0][2] * u.x + m[1][2] * u.y + m[2][2] * u.z;
    float wt = m[0][3] * u.x + m[1][3] * u.y + m[2][3] * u.z;
    float iw = 1.0f;
    if (!is_zero(wt)) iw = 1.0f / wt;
    return mk3(xt * iw, yt * iw, zt * iw);
}

}  // namespace mpt
#endif
