// dev_bsdf.h -- device BSDFs of the MI355X path tracer: Lambert, the layered
// Principled BSDF (coat, sheen LTC, two F82-tint metal lobes with thin-film, glass
// with dispersion, specular + diffuse glossy base), energy-compensation LUT lookups
// and the nested-dielectrics priority stack.  Restates, in order of appearance:
//   src/Device/includes/NestedDielectrics.h:135-290   (priority stack, 1-bit priority quirk)
//   src/Device/includes/Dispersion.h:392-540           (wavelength fit, Cauchy IOR)
//   src/Device/includes/Sampling.h:175-216, BSDFs/Lambertian.h:14-30
//   src/Device/includes/Fresnel.h:11-165, BSDFs/ThinFilm.h:12-221
//   src/Device/includes/BSDFs/Microfacet.h:25-256
//   src/Device/includes/BSDFs/MicrofacetEnergyCompensation.h:25-705,
//   src/Device/includes/BSDFs/PrincipledEnergyCompensation.h:13-80
//   src/Device/includes/BSDFs/SheenLTC.h:24-150
//   src/Device/includes/BSDFs/Principled.h:51-1193, Dispatcher.h:18-68
// LUTs are read with the reference CPU's nearest-texel rule (Image/Image.cpp:737-779)
// from plain global-memory float arrays (L2/MALL resident: 6 tables, 9.4 MB total).
#ifndef MPT_DEV_BSDF_H
#define MPT_DEV_BSDF_H

#include "dev_math.h"
#include "mpt.h"

namespace mpt {

typedef MptMaterial Mat;

DEV Col C3(MptColor c) { return col(c.r, c.g, c.b); }

// ----------------------------------------------------------------------------------
// LUTs
// ----------------------------------------------------------------------------------
struct DevLuts {
    const float* conductor;
    const float* glossy;
    const float* glass;
    const float* glass_inv;
    const float* thin_glass;
    const float* sheen;
};

DEV float wrap01(float u) { float r = u; if (r != 1.0f) r -= (float)(int)u; return r < 0 ? 1.0f + r : r; }
DEV float lut2d(const float* d, int w, int h, float u, float v) {
    u = wrap01(u);
    v = 1.0f - wrap01(v);
    int x = (int)(u * (float)(w - 1)), y = (int)(v * (float)(h - 1));
    return d[x + y * w];
}
DEV float lut3d(const float* d, int w, int h, int dd, float u, float v, float z) {
    u = wrap01(u);
    v = 1.0f - wrap01(v);
    z = wrap01(z);
    int x = (int)(u * (float)(w - 1)), y = (int)(v * (float)(h - 1)), k = (int)(z * (float)(dd - 1));
    return d[(size_t)k * w * h + x + y * w];
}

// ----------------------------------------------------------------------------------
// Nested dielectrics (packed 32-bit stack entries)
// ----------------------------------------------------------------------------------
constexpr int STACK_SIZE = 3;
constexpr int MAX_MAT = (1 << 26) - 1;
constexpr uint32_t SE_TOP = 1u << 26, SE_ODD = 1u << 27, SE_PRIO = 1u << 28;
constexpr uint32_t SE_DEFAULT = (uint32_t)MAX_MAT | SE_TOP | SE_ODD;
DEV int se_mat(uint32_t e) { return (int)(e & (uint32_t)MAX_MAT); }

struct VState {
    uint32_t st[STACK_SIZE];
    int pos;
    int incident, outgoing;
    bool inside;
    float dist;
    float wl;
};
DEV VState vs_default() {
    VState v;
    for (int i = 0; i < STACK_SIZE; i++) v.st[i] = SE_DEFAULT;
    v.pos = 0; v.incident = -1; v.outgoing = -1; v.inside = false; v.dist = 0.0f; v.wl = 0.0f;
    return v;
}
DEV VState vs_unpack(uint4 a, uint4 b) {
    VState v;
    v.st[0] = a.x; v.st[1] = a.y; v.st[2] = a.z;
    v.pos = (int)(a.w & 3u);
    v.inside = (a.w >> 2) & 1u;
    v.incident = (int)b.x; v.outgoing = (int)b.y;
    v.dist = __uint_as_float(b.z); v.wl = __uint_as_float(b.w);
    return v;
}
DEV uint4 vs_pack_a(const VState& v) { return make_uint4(v.st[0], v.st[1], v.st[2], (uint32_t)v.pos | ((uint32_t)v.inside << 2)); }
DEV uint4 vs_pack_b(const VState& v) {
    return make_uint4((uint32_t)v.incident, (uint32_t)v.outgoing, __float_as_uint(v.dist), __float_as_uint(v.wl));
}
// cached (G-buffer, re-read by neighbours) and streaming (path state, ld_s / st_s) accessors
template <class PA, class PB> DEV VState vs_load(const PA& A, const PB& B, int i) { return vs_unpack(A[i], B[i]); }
template <class PA, class PB> DEV void vs_store(const PA& A, const PB& B, int i, const VState& v) { A[i] = vs_pack_a(v); B[i] = vs_pack_b(v); }
DEV VState vs_load_s(const uint4* A, const uint4* B, int i) { return vs_unpack(ld_s(A + i), ld_s(B + i)); }
DEV void vs_store_s(uint4* A, uint4* B, int i, const VState& v) { st_s(A + i, vs_pack_a(v)); st_s(B + i, vs_pack_b(v)); }
DEV uint32_t& vs_entry(VState& v, int i) {   // constant-index friendly access
    return i == 0 ? v.st[0] : (i == 1 ? v.st[1] : v.st[2]);
}
DEV bool vs_push(VState& v, int mi, int prio) {
    int last;
    for (last = v.pos; last >= 0; last--) {
        uint32_t e = vs_entry(v, last);
        if (se_mat(e) != mi && (e & SE_TOP) && (e & SE_ODD)) break;
    }
    bool odd = true;
    for (int p = v.pos; p >= 0; p--) {
        uint32_t& e = vs_entry(v, p);
        if (se_mat(e) == mi) { e &= ~SE_TOP; odd = !(e & SE_ODD); break; }
    }
    v.inside = !odd;
    if (v.pos < STACK_SIZE - 1) v.pos++;
    vs_entry(v, v.pos) = ((uint32_t)mi & (uint32_t)MAX_MAT) | SE_TOP | (odd ? SE_ODD : 0u) | ((prio & 1) ? SE_PRIO : 0u);
    uint32_t le = vs_entry(v, last);
    int lprio = (le & SE_PRIO) ? 1 : 0;
    if (prio < lprio) return true;
    if (odd) { v.incident = se_mat(le); v.outgoing = mi; }
    else { v.incident = mi; v.outgoing = se_mat(le); }
    return false;
}
DEV void vs_pop(VState& v, bool inside_material) {
    int top = se_mat(vs_entry(v, v.pos));
    if (v.pos > 0) v.pos--;
    if (inside_material) {
        int p;
        for (p = v.pos; p >= 0; p--) if (se_mat(vs_entry(v, p)) == top) break;
        if (p >= 0) for (int i = p + 1; i <= v.pos; i++) vs_entry(v, i - 1) = vs_entry(v, i);
        if (v.pos > 0) v.pos--;
    }
    for (int i = v.pos; i >= 0; i--) {
        uint32_t& e = vs_entry(v, i);
        if (se_mat(e) == top) { e |= SE_TOP; break; }
    }
}

// ----------------------------------------------------------------------------------
// Dispersion
// ----------------------------------------------------------------------------------
DEV Col wavelength_to_rgb(float w) {
    Col c;
    if (w < 463.0f) {
        c.r = -1.2776028240727566e-01f / (1.0f + pexp((w - 4.2680623367293401e+02f) / 8.2197460736637176e+00f)) +
              -1.3925673552505122e-11f * pexp((w - 45.0f) / 1.8175459086411596e+01f);
        c.r += 1.2898689750552100e-01f;
    } else if (w > 553.0f) {
        c.r = 1.7963649137825513e+01f * (1.0f / 2.6577826611702449e+01f) *
              pexp(-0.5f * sq((w - 6.0625724092824566e+02f) * (1.0f / 2.6577826611702449e+01f)));
        c.r += 2.5574660155104657e-03f;
    } else c.r = 0.0f;
    c.g = 3.4962267376163049e+02f * pexp(-0.5f * sq((w - 5.4209217455705152e+02f) / -2.9598170255834638e+01f));
    c.g /= w;
    c.b = pexp(3.2987659944421112e+03f + (-2.0975839709372405e+05f / w) - 4.6368268395094020e+02f * plog(w));
    return c * 10.0f;
}
DEV float dispersion_ior(float abbe, float scale, float base, float wl) {
    if (scale == 0.0f) return base;
    float an = abbe / scale;
    float B = (base - 1.0f) / (an * 0.00000191038851931481f);
    float A = base - B / 334777.96f;
    return A + B / (wl * wl);
}
DEV Col dispersion_ray_color(float& wl, float scale) {
    if (scale == 0.0f) return col(1.0f);
    if (wl >= 0.0f) return col(1.0f);
    wl *= -1.0f;
    return wavelength_to_rgb(wl);
}

// ----------------------------------------------------------------------------------
// Sampling, Lambert
// ----------------------------------------------------------------------------------
DEV v3 cosine_sample_around(v3 n, Rng& rng) {
    float r1 = rng();
    float r2 = 2.0f * rng() - 1.0f;
    if (r1 < 1.0e-8f && r2 < -0.999999f && n.z > 0.999999f) { r1 += 1.0e-7f; r2 += 1.0e-7f; }
    float theta = TWO_PI * r1;
    float s = sqrtf(1.0f - r2 * r2);
    const float2 sc = psincos(theta);
    return normalize(n + mk3(s * sc.y, s * sc.x, r2));
}
DEV v3 cosine_sample_z_up(Rng& rng) {
    float r1 = rng(), r2 = rng();
    float phi = TWO_PI * r1;
    float ct = sqrtf(r2);
    float st = sqrtf(1.0f - ct * ct);
    const float2 sc = psincos(phi);
    return normalize(mk3(sc.y * st, sc.x * st, ct));
}
DEV Col lambert_eval_c(Col base, float NoL, float& pdf) {
    pdf = 0.0f;
    if (NoL <= 0.0f) return col(0.0f);
    pdf = NoL * INV_PI;
    return base * INV_PI;
}
DEV Col lambert_eval(const Mat& m, float NoL, float& pdf) { return lambert_eval_c(C3(m.base_color), NoL, pdf); }
DEV Col lambert_sample(const Mat& m, v3 n, v3& dir, float& pdf, Rng& rng) {
    dir = cosine_sample_around(n, rng);
    return lambert_eval(m, dot(n, dir), pdf);
}
// Oren-Nayar (BSDFs/OrenNayar.h:49-90) on local directions (z = the shading normal); like
// the reference, no hemisphere test: a light below the surface gets a negative pdf.
// A, B: SimplifiedRendererMaterial::get_oren_nayar_AB (Material.h:73-78)
DEV Col oren_nayar_eval(const Mat& m, v3 lv, v3 ll, float& pdf) {
    const float sti = sqrtf(1.0f - ll.z * ll.z), sto = sqrtf(1.0f - lv.z * lv.z);
    float max_cos = 0.0f;
    if (sti > 1.0e-4f && sto > 1.0e-4f) {
        const float spi = ll.y / sti, cpi = ll.x / sti;
        const float spo = lv.y / sto, cpo = lv.x / sto;
        max_cos = maxr(0.0f, cpi * cpo + spi * spo);
    }
    float sa, tb;
    if (absr(ll.z) > absr(lv.z)) { sa = sto; tb = sti / absr(ll.z); }
    else { sa = sti; tb = sto / absr(lv.z); }
    const float s2 = m.oren_nayar_sigma * m.oren_nayar_sigma;
    const float A = 1.0f - s2 / (2.0f * (s2 + 0.33f));
    const float B = 0.45f * s2 / (s2 + 0.09f);
    pdf = ll.z * INV_PI;
    return C3(m.base_color) * INV_PI * (A + B * max_cos * sa * tb);
}

// ----------------------------------------------------------------------------------
// Fresnel + thin film
// ----------------------------------------------------------------------------------
DEV float F0_from_eta(float eta_t, float eta_i) { float n = eta_t - eta_i, d = eta_t + eta_i; return (n * n) / (d * d); }
DEV float fresnel_dielectric(float ci, float eta) {
    float si2 = 1.0f - ci * ci;
    float st2 = si2 / (eta * eta);
    if (st2 >= 1.0f) return 1.0f;
    float ct = sqrtf(1.0f - st2);
    float rpa = (eta * ci - ct) / (eta * ci + ct);
    float rpe = (ci - eta * ct) / (ci + eta * ct);
    return (rpa * rpa + rpe * rpe) / 2.0f;
}
DEV float fresnel_dielectric(float ci, float eta_i, float eta_t) { return fresnel_dielectric(ci, eta_t / eta_i); }
DEV Col f82_tint(Col F0, Col F82, Col F90, float expo, float c) {
    Col base = F0 + (F90 - F0) * ppow(1.0f - c, expo);
    float laz = c * pow6(1.0f - c);
    const float cmax = 1.0f / 7.0f;
    const float da = cmax * pow6(1.0f - cmax);
    Col na = (F0 + (F90 - F0) * ppow(1.0f - cmax, expo)) * (col(1.0f) - F82);
    Col a = na / da;
    return clampc(base - a * laz, 0.0f, 1.0f);
}
DEV float fresnel_hemispherical_albedo(float eta) {
    return plog((10893.0f * eta - 1438.2f) / (-774.4f * sq(eta) + 10212.0f * eta + 1.0f));
}
DEV Col eval_sensitivity(float opd, float shift) {
    float phase = 2.0f * PI * opd * 1.0e-6f;
    const float val[3] = {5.4856e-13f, 4.4201e-13f, 5.2481e-13f};
    const float pos[3] = {1.6810e+06f, 1.7953e+06f, 2.2084e+06f};
    const float var[3] = {4.3278e+09f, 9.3046e+09f, 6.6121e+09f};
    float x[3];
#pragma unroll
    for (int i = 0; i < 3; i++) x[i] = val[i] * sqrtf(2.0f * PI * var[i]) * pcos(pos[i] * phase + shift) * pexp(-1.0f * var[i] * phase * phase);
    x[0] += 9.7470e-14f * sqrtf(2.0f * PI * 4.5282e+09f) * pcos(2.2399e+06f * phase + shift) * pexp(-4.5282e+09f * phase * phase);
    return col(x[0] / 1.0685e-7f, x[1] / 1.0685e-7f, x[2] / 1.0685e-7f);
}
DEV void fresnel_phase(float ci, float e1, float e2, float k2, float& par, float& perp) {
    float s2 = 1.0f - sq(ci);
    float A = sq(e2) * (1.0f - sq(k2)) - sq(e1) * s2;
    float B = sqrtf(sq(A) + sq(2.0f * sq(e2) * k2));
    float U = (float)::sqrt((double)(A + B) / 2.0);
    float V = (float)::sqrt((double)(B - A) / 2.0);
    perp = patan2(2.0f * e1 * V * ci, sq(U) + sq(V) - sq(e1 * ci));
    par = patan2(2.0f * e1 * sq(e2) * ci * (2.0f * k2 * U - (1.0f - sq(k2)) * V),
                 sq(sq(e2) * (1.0f + sq(k2)) * ci) - sq(e1) * (sq(U) + sq(V)));
}
DEV void fresnel_conductor(float ci, float eta, float k, float& Rp2, float& Rs2) {
    float c2 = ci * ci, s2 = 1.0f - c2;
    float t1 = eta * eta - k * k - s2;
    float a2pb2 = sqrtf(t1 * t1 + 4.0f * k * k * eta * eta);
    float a = sqrtf(0.5f * (a2pb2 + t1));
    float term1 = a2pb2 + c2, term2 = 2.0f * a * ci;
    Rs2 = clampr(0.0f, 1.0f, (term1 - term2) / (term1 + term2));
    float term3 = a2pb2 * c2 + s2 * s2, term4 = term2 * s2;
    Rp2 = clampr(0.0f, 1.0f, Rs2 * (term3 - term4) / (term3 + term4));
}
DEV Col hue_shift(Col c, float deg) {
    if (deg == 0.0f) return c;
    double ca = (double)pcos(deg / 180.0f * PI), sa = (double)psin(deg / 180.0f * PI);
    double t = 1.0 / 3.0, st = ::sqrt(1.0 / 3.0);
    float m00 = (float)(ca + (1.0 - ca) / 3.0), m01 = (float)(t * (1.0 - ca) - st * sa), m02 = (float)(t * (1.0 - ca) + st * sa);
    float m10 = (float)(t * (1.0 - ca) + st * sa), m11 = (float)(ca + t * (1.0 - ca)), m12 = (float)(t * (1.0 - ca) - st * sa);
    float m20 = (float)(t * (1.0 - ca) - st * sa), m21 = (float)(t * (1.0 - ca) + st * sa), m22 = (float)(ca + t * (1.0 - ca));
    Col h = col(c.r * m00 + c.g * m01 + c.b * m02, c.r * m10 + c.g * m11 + c.b * m12, c.r * m20 + c.g * m21 + c.b * m22);
    return clampc(h, 0.0f, 1.0f);
}
DEV Col thin_film_fresnel(const Mat& m, float ambient, float HoL) {
    float e1 = ambient, e2 = m.thin_film_ior;
    float e3 = m.thin_film_do_ior_override ? m.thin_film_base_ior_override : m.ior;
    float k3 = m.thin_film_do_ior_override ? m.thin_film_kappa_3 : 0.0f;
    float R12p = 0, R12s = 0, T121p = 0, T121s = 0, R23p = 0, R23s = 0, c2 = 0;
    float ct2 = 1.0f - (1.0f - sq(HoL)) * sq(e1 / e2);
    if (ct2 <= 0.0f) { R12s = 1.0f; R12p = 1.0f; }
    else {
        c2 = sqrtf(ct2);
        fresnel_conductor(HoL, e2 / e1, 0.0f, R12p, R12s);
        fresnel_conductor(c2, e3 / e2, k3, R23p, R23s);
        T121p = (float)(1.0 - (double)R12p);
        T121s = (float)(1.0 - (double)R12s);
    }
    float D = m.thin_film_thickness / 1000.0f * c2;
    float p21p, p21s, p23p, p23s;
    fresnel_phase(HoL, e1, e2, 0.0f, p21p, p21s);
    fresnel_phase(c2, e2, e3, k3, p23p, p23s);
    p21p = PI - p21p;
    p21s = PI - p21s;
    float r123p = sqrtf(R12p * R23p), r123s = sqrtf(R12s * R23s);
    float Rs = (sq(T121p) * R23p) / (1.0f - R12p * R23p);
    Col I = col(R12p + Rs);
    float Cm = Rs - T121p;
    for (int k = 1; k <= 2; ++k) { Cm *= r123p; Col Sm = 2.0f * eval_sensitivity((float)k * D, (float)k * (p23p + p21p)); I += Cm * Sm; }
    Rs = (sq(T121s) * R23s) / (1.0f - R12s * R23s);
    I += col(R12s + Rs);
    Cm = Rs - T121s;
    for (int k = 1; k <= 2; ++k) { Cm *= r123s; Col Sm = 2.0f * eval_sensitivity((float)k * D, (float)k * (p23s + p21s)); I += Cm * Sm; }
    I *= 0.5f;
    Col o = col(2.3646381f * I.r - 0.8965361f * I.g - 0.4680737f * I.b,
                -0.5151664f * I.r + 1.4264000f * I.g + 0.0887608f * I.b,
                0.0052037f * I.r - 0.0144081f * I.g + 1.0092106f * I.b);
    return hue_shift(clampc(o, 0.0f, 1.0f), m.thin_film_hue_shift_degrees);
}

// ----------------------------------------------------------------------------------
// Microfacet
// ----------------------------------------------------------------------------------
struct BCtx {
    const Mat* mats;
    DevLuts luts;
    bool clearcoat_comp;
    int masking;
};
DEV void alphas(float r, float an, float& ax, float& ay) {
    float asp = sqrtf(1.0f - 0.9f * an);
    ax = maxr(1.0e-4f, r * r / asp);
    ay = maxr(1.0e-4f, r * r * asp);
}
DEV float ggx_D(float ax, float ay, v3 h) {
    float d = (h.x * h.x) / (ax * ax) + (h.y * h.y) / (ay * ay) + (h.z * h.z);
    return 1.0f / (PI * ax * ay * d * d);
}
DEV float lambda_smith(float ax, float ay, v3 d) {
    float a = d.x * ax, b = d.y * ay;
    return (-1.0f + sqrtf(1.0f + (a * a + b * b) / (d.z * d.z))) * 0.5f;
}
DEV float G1(float ax, float ay, v3 d) { return 1.0f / (1.0f + lambda_smith(ax, ay, d)); }
// ts_ggx0 with the view-only terms given: alphas (ax, ay), lambda_smith(ax, ay, V) and
// 1 / (1 + lV) -- the per-vertex part of the glossy base, computed once in principled_eval_pre
DEV Col ts_ggx0_v(const BCtx& c, float ax, float ay, float lV, float G1V, Col F, v3 V, v3 L, v3 H, float& pdf) {
    pdf = 0.0f;
    float D = ggx_D(ax, ay, H);
    float HoL = maxr(1.0e-3f, dot(V, H));
    float Dv = G1V * D * HoL / V.z;
    float NoV = maxr(1.0e-3f, absr(V.z)), NoL = maxr(1.0e-3f, absr(L.z));
    pdf = Dv / (4.0f * dot(V, H));
    if (pdf == 0.0f) return col(0.0f);
    float lL = lambda_smith(ax, ay, L);
    if (c.masking == 1) return F * D * (G1V * (1.0f / (1.0f + lL))) / (4.0f * NoL * NoV);
    float G2 = 1.0f / (1.0f + lV + lL);
    return F * D * G2 / (4.0f * NoL * NoV);
}
DEV Col ts_ggx0(const BCtx& c, float r, float an, Col F, v3 V, v3 L, v3 H, float& pdf) {
    float ax, ay;
    alphas(r, an, ax, ay);
    const float lV = lambda_smith(ax, ay, V);
    return ts_ggx0_v(c, ax, ay, lV, 1.0f / (1.0f + lV), F, V, L, H, pdf);
}
DEV Col ts_ggx1(const BCtx& c, float r, float an, Col F, v3 V, v3 L, v3 H, float& pdf) {
    float Ess = lut2d(c.luts.conductor, 128, 128, maxr(0.0f, V.z), r);
    float kms = (1.0f - Ess) / Ess;
    Col ms = col(1.0f) + kms * F;
    Col ss = ts_ggx0(c, r, an, F, V, L, H, pdf);
    return ss * ms;
}
DEV v3 ggx_vndf(v3 V, float ax, float ay, Rng& rng) {
    float r1 = rng(), r2 = rng();
    v3 Vh = normalize(mk3(ax * V.x, ay * V.y, V.z));
    float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    v3 T1 = lensq > 0.0f ? mk3(-Vh.y, Vh.x, 0.0f) / sqrtf(lensq) : mk3(1.0f, 0.0f, 0.0f);
    v3 T2 = cross(Vh, T1);
    float r = sqrtf(r1), phi = TWO_PI * r2;
    const float2 sc = psincos(phi);
    float t1 = r * sc.y, t2 = r * sc.x;
    float s = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - s) * sqrtf(1.0f - t1 * t1) + s * t2;
    v3 Nh = t1 * T1 + t2 * T2 + sqrtf(maxr(0.0f, 1.0f - t1 * t1 - t2 * t2)) * Vh;
    return normalize(mk3(ax * Nh.x, ay * Nh.y, maxr(0.0f, Nh.z)));
}
DEV v3 ggx_sample_reflection_a(float ax, float ay, v3 V, Rng& rng) {
    float below = V.z < 0 ? -1.0f : 1.0f;
    v3 m = ggx_vndf(V * below, ax, ay, rng);
    return normalize(reflect_ray(V, m * below));
}
DEV v3 ggx_sample_reflection(float r, float an, v3 V, Rng& rng) {
    float ax, ay;
    alphas(r, an, ax, ay);
    return ggx_sample_reflection_a(ax, ay, V, rng);
}

// ----------------------------------------------------------------------------------
// Energy compensation
// ----------------------------------------------------------------------------------
__constant__ const float kEtaB[10] = {1.01f, 1.02f, 1.03f, 1.1f, 1.2f, 1.4f, 1.5f, 2.0f, 2.4f, 3.0f};
__constant__ const float kCorrT[10][11] = {
    {2.5f, 2.5f, 2.3f, 2.4f, 2.45f, 2.4665f, 2.52f, 2.55f, 2.55f, 2.585f, 2.5f},
    {2.5f, 2.5f, 2.3f, 2.4f, 2.475f, 2.51f, 2.54f, 2.565f, 2.57f, 2.59f, 2.5f},
    {2.5f, 2.5f, 2.3f, 2.4f, 2.475f, 2.51f, 2.544f, 2.565f, 2.58f, 2.6f, 2.5f},
    {2.5f, 2.5f, 2.3f, 2.38f, 2.475f, 2.54f, 2.575f, 2.61f, 2.63f, 2.6f, 2.5f},
    {2.5f, 1.8f, 2.3f, 2.38f, 2.475f, 2.55f, 2.65f, 2.675f, 2.7f, 2.675f, 2.5f},
    {2.5f, 1.8f, 2.3f, 2.38f, 2.475f, 2.7f, 2.875f, 2.925f, 2.95f, 2.8f, 2.55f},
    {2.5f, 1.6f, 2.3f, 2.38f, 2.475f, 2.7f, 2.95f, 3.1f, 3.1f, 3.05f, 2.57f},
    {2.5f, 1.5f, 2.2f, 2.38f, 2.475f, 2.75f, 3.5f, 4.85f, 6.0f, 7.0f, 2.57f},
    {2.5f, 1.5f, 2.0f, 2.44f, 2.475f, 3.0f, 3.8f, 7.0f, 10.0f, 12.0f, 3.9f},
    {2.5f, 1.5f, 1.7f, 2.38f, 2.475f, 2.9f, 3.8f, 7.5f, 12.0f, 13.75f, 2.5f},
};
__constant__ const float kRoughK[11] = {0.0f, 0.1f, 0.2f, 0.3f, 0.4f, 0.5f, 0.6f, 0.7f, 0.8f, 0.9f, 1.0f};
DEV float corr_knot(int b, float r) {
    if (r <= 0.0f) return 2.5f;
    for (int k = 1; k <= 10; k++) {
        if (r <= kRoughK[k]) {
            float a = kCorrT[b][k - 1], c = kCorrT[b][k];
            if (a == c) return a;
            return lerpr(a, c, (r - kRoughK[k - 1]) / 0.1f);
        }
    }
    return 2.5f;
}
DEV float glass_corr_exponent(float r, float eta) {
    if (is_zero(r) || absr(1.0f - eta) < 1.0e-3f) return 2.5f;
    int hi = 9;
    for (int i = 0; i < 9; i++) if (eta <= kEtaB[i]) { hi = i; break; }
    float hb = kEtaB[hi], hc = corr_knot(hi, r);
    int lo = -1;
    for (int i = 0; i < 9; i++) if (eta > kEtaB[i] && eta <= kEtaB[i + 1]) { lo = i; break; }
    float lb, lc;
    if (lo < 0) { lb = hb - 1.0f; lc = hc; }
    else { lb = kEtaB[lo]; lc = corr_knot(lo, r); }
    return lerpr(lc, hc, (eta - lb) / (hb - lb));
}
DEV float dielectric_comp(const BCtx& c, const Mat& m, const VState& vs, float eta_t, float eta_i, float rel, float NoV) {
    float comp = 1.0f;
    if (m.thin_film < 1.0f) {
        bool inside = vs.inside;
        float re = inside ? 1.0f / rel : rel;
        float expo = 2.5f;
        if (!m.thin_walled) expo = glass_corr_exponent(m.roughness, re);
        float fetch = ppow(maxr(1.0e-3f, NoV), 1.0f / expo);
        float F0r = sqrtf(sqrtf(F0_from_eta(eta_t, eta_i)));
        if (!m.thin_walled) comp = lut3d(inside ? c.luts.glass_inv : c.luts.glass, 256, 16, 128, fetch, m.roughness, F0r);
        else comp = lut3d(c.luts.thin_glass, 32, 32, 96, fetch, m.roughness, F0r);
        comp = lerpr(comp, 1.0f, m.thin_film * m.roughness);
    }
    return comp;
}
DEV float spec_rel_ior(const Mat& m, float inc) {
    float layer = lerpr(inc, m.coat_ior, m.coat);
    float rel = m.ior / layer;
    if (rel < 1.0f) rel = 1.0f / rel;
    return rel;
}
DEV float glossy_base_comp(const BCtx& c, const Mat& m, float inc, float NoV) {
    float rel = spec_rel_ior(m, inc);
    if (absr(rel - 1.0f) < 1.0e-3f) rel += 1.0e-3f;
    float vr = ppow(NoV, 1.0f / 2.5f);
    float F0r = sqrtf(sqrtf(F0_from_eta(m.ior, m.ior / rel)));
    float ms = lut3d(c.luts.glossy, 128, 64, 128, vr, m.roughness, F0r);
    ms = lerpr(1.0f, ms, m.specular);
    return lerpr(ms, 1.0f, m.thin_film);
}
DEV float clearcoat_comp(const BCtx& c, const Mat& m, float inc, float NoV) {
    if (m.coat == 0.0f) return 1.0f;
    if (absr(m.coat_ior / inc - 1.0f) < 1.0e-3f) inc += 1.0e-3f;
    float vr = ppow(NoV, 1.0f / 2.5f);
    float F0r = sqrtf(sqrtf(F0_from_eta(m.coat_ior, inc)));
    float ms = lut3d(c.luts.glossy, 128, 64, 128, vr, m.coat_roughness, F0r);
    ms = lerpr(1.0f, ms, m.coat * (1.0f - m.specular_transmission));
    return lerpr(ms, 1.0f, m.thin_film);
}

// ----------------------------------------------------------------------------------
// Sheen LTC
// ----------------------------------------------------------------------------------
DEV Col read_ltc(const BCtx& c, float r, float ct) {
    float u = wrap01(ct), v = 1.0f - wrap01(1.0f - r);
    int x = (int)(u * 31.0f), y = (int)(v * 31.0f);
    const float* p = c.luts.sheen + (x + y * 32) * 3;
    return col(p[0], p[1], p[2]);
}
DEV float get_phi(v3 d) { float p = patan2(d.y, d.x); if (p < 0.0f) p += TWO_PI; return p; }
DEV v3 rotate_z(v3 v, float angle) {
    v3 axis = mk3(0.0f, 0.0f, 1.0f);
    const float2 sc = psincos(angle);
    float s = sc.x, co = sc.y;
    return v * co + axis * dot(v, axis) * (1.0f - co) + s * cross(axis, v);
}
DEV Col sheen_eval(const BCtx& c, const Mat& m, v3 L, v3 V, float& pdf, float& refl) {
    if (V.z <= 0.0f || L.z <= 0.0f) {
        pdf = 0.0f;
        refl = V.z > 0.0f ? read_ltc(c, m.sheen_roughness, V.z).b : 0.0f;
        return col(0.0f);
    }
    v3 Ls = rotate_z(L, -get_phi(V));
    Col A = read_ltc(c, m.sheen_roughness, V.z);
    v3 lo = mk3(Ls.x * A.r + Ls.z * A.g, Ls.y * A.r, Ls.z);
    float len = length(lo);
    lo = lo / len;
    float Do = lo.z * INV_PI * ((A.r * A.r) / (len * len * len));
    pdf = Do;
    refl = A.b;
    return C3(m.sheen_color) * A.b * Do / L.z;
}
DEV v3 sheen_sample(const BCtx& c, const Mat& m, v3 V, Rng& rng) {
    v3 cs = cosine_sample_z_up(rng);
    Col A = read_ltc(c, m.sheen_roughness, V.z);
    float ai = 1.0f / A.r, bi = A.g;
    v3 d = normalize(mk3(cs.x * ai - cs.z * bi * ai, cs.y * ai, cs.z));
    return rotate_z(d, get_phi(V));
}

// ----------------------------------------------------------------------------------
// Principled
// ----------------------------------------------------------------------------------
DEV float thin_walled_roughness(bool thin, float r, float eta) {
    if (!thin) return r;
    float rem = r * sqrtf(3.7f * (eta - 1.0f) * sq(eta - 0.5f) / pow3(eta));
    return clampr(0.0f, 1.0f, rem / 1.39f);
}
// Material classes of the BSDF code (template parameter FULL): BC_FULL (1) the whole
// Principled BSDF; BC_PLAIN (0) a plain dielectric (no coat, sheen, metal, transmission or
// thin film: MT_FULL clear, see k_resolve_materials) and BC_GLASS (2) a dielectric that may
// transmit but has no coat, sheen, metal or thin film (MT_GLASS): the lobes and terms that are
// exactly zero for the class are not compiled in.  Same result as BC_FULL for a material of
// the class, bit for bit (the glass class keeps the coat block, which a refracting direction
// enters whatever the coat weight).
enum : int { BC_PLAIN = 0, BC_FULL = 1, BC_GLASS = 2 };
DEV constexpr bool bc_extra(int cls) { return cls == BC_FULL; }    // sheen, metal, thin film, coat / sheen sampling
DEV constexpr bool bc_layers(int cls) { return cls != BC_PLAIN; }  // coat evaluation, glass lobe
// (ior, tf: the material's ior and thin_film, from the PEval snapshot in the evaluations)
template <int FULL = BC_FULL>
DEV Col spec_fresnel_v(const Mat& m, float ior, float tf, float rel, float ci) {
    float above = ior / rel;
    Col Fs = col(0.0f), Ft = col(0.0f);
    if (tf < 1.0f) Fs = col(fresnel_dielectric(ci, rel));
    if (bc_extra(FULL) && tf > 0.0f) Ft = thin_film_fresnel(m, above, ci);
    return lerpc(Fs, Ft, tf);
}
template <int FULL = BC_FULL>
DEV Col spec_fresnel(const Mat& m, float rel, float ci) { return spec_fresnel_v<FULL>(m, m.ior, m.thin_film, rel, ci); }
DEV float ior_or_air(const BCtx& c, int idx) { return idx == MAX_MAT ? 1.0f : c.mats[idx].ior; }

template <int FULL = BC_FULL>
DEV Col glass_eval(const BCtx& c, const Mat& m, VState& vs, v3 V, v3 L, float& pdf) {
    pdf = 0.0f;
    float NoV = V.z, NoL = L.z;
    if (absr(NoL) < 1.0e-8f) return col(0.0f);
    bool refl = NoL * NoV > 0;
    float ei = dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, ior_or_air(c, vs.incident), absr(vs.wl));
    float et = dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, ior_or_air(c, vs.outgoing), absr(vs.wl));
    float rel = et / ei;
    if (absr(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    v3 H;
    if (refl) H = L + V;
    else if (m.thin_walled) H = L * mk3(1.0f, 1.0f, -1.0f) + V;
    else H = L * rel + V;
    H = normalize(H);
    if (H.z < 0.0f) H = -H;
    float HoL = dot(L, H), HoV = dot(V, H);
    if (HoL * NoL < 0.0f || HoV * NoV < 0.0f) return col(0.0f);
    float comp = dielectric_comp(c, m, vs, et, ei, rel, V.z);
    Col Ft = col(0.0f), Fn = col(0.0f);
    if (bc_extra(FULL) && m.thin_film > 0.0f) Ft = thin_film_fresnel(m, ei, HoV);
    if (m.thin_film < 1.0f) Fn = col(fresnel_dielectric(HoV, rel));
    Col F = lerpc(Fn, Ft, m.thin_film);
    float frp = lum(F);
    float r = thin_walled_roughness(m.thin_walled, m.roughness, rel);
    if (frp < 1.0f && m.thin_film == 0.0f && m.thin_walled && r < 0.1f) frp += sq(1.0f - frp) * frp / (1.0f - sq(frp));
    Col out;
    if (refl) {
        out = ts_ggx0(c, r, m.anisotropy, F, V, L, H, pdf);
        out /= comp;
        pdf *= frp;
    } else {
        float dp = HoL + HoV / rel;
        float dp2 = dp * dp;
        float denom = dp2 * NoL * NoV;
        float ax, ay;
        alphas(r, m.anisotropy, ax, ay);
        float D = ggx_D(ax, ay, H);
        float G1V = G1(ax, ay, V), G1L = G1(ax, ay, L);
        float G2 = G1V * G1L;
        pdf = (absr(HoL) / dp2) * (G1V / absr(NoV) * D * absr(HoV));
        pdf *= 1.0f - frp;
        out = C3(m.base_color) * D * (col(1.0f) - F) * G2 * absr(HoL * HoV / denom);
        if (m.thin_walled) out *= C3(m.base_color);
        out /= comp;
        if (m.thin_walled) vs_pop(vs, vs.inside);
        else if (vs.incident != MAX_MAT) {
            const Mat& im = c.mats[vs.incident];
            Col ac = C3(im.absorption_color);
            if (!is_white(ac)) out = out * cexp((clog(ac) / im.absorption_at_distance) * vs.dist);
            vs.dist = 0.0f;
            if (vs.inside) vs_pop(vs, vs.inside);
        }
    }
    return out;
}
template <int FULL = BC_FULL>
DEV v3 glass_sample(const BCtx& c, const Mat& m, VState& vs, v3 V, Rng& rng) {
    float ei = dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, ior_or_air(c, vs.incident), absr(vs.wl));
    float et = dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, ior_or_air(c, vs.outgoing), absr(vs.wl));
    float rel = et / ei;
    if (absr(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    float r = thin_walled_roughness(m.thin_walled, m.roughness, rel);
    float ax, ay;
    alphas(r, m.anisotropy, ax, ay);
    v3 mn = ggx_vndf(V, ax, ay, rng);
    float HoV = dot(V, mn);
    Col Ft = col(0.0f), Fn = col(0.0f);
    if (bc_extra(FULL) && m.thin_film > 0.0f) Ft = thin_film_fresnel(m, ei, HoV);
    if (m.thin_film < 1.0f) Fn = col(fresnel_dielectric(HoV, rel));
    Col F = lerpc(Fn, Ft, m.thin_film);
    float frp = lum(F);
    if (frp < 1.0f && m.thin_film == 0.0f && m.thin_walled && r < 0.1f) frp += sq(1.0f - frp) * frp / (1.0f - sq(frp));
    float r1 = rng();
    v3 dir = mk3(0.0f, 0.0f, 0.0f);
    if (r1 < frp) { dir = reflect_ray(V, mn); vs_pop(vs, false); }
    else {
        if (dot(mn, V) < 0.0f) mn = -mn;
        if (m.thin_walled) { v3 rr = reflect_ray(V, mn); rr.z *= -1.0f; vs_pop(vs, false); return rr; }
        refract_ray(V, mn, dir, rel);
    }
    return dir;
}
DEV Col coat_darkening(const Mat& m, float rel, float vdf) {
    if (m.coat_darkening == 0.0f) return col(1.0f);
    float Kr = 1.0f - (1.0f - fresnel_hemispherical_albedo(rel)) / (rel * rel);
    float K = lerpr(vdf, Kr, m.roughness);
    Col ba = (C3(m.base_color) + C3(m.sheen_color) * m.sheen) / (1.0f + m.sheen);
    Col dk = (1.0f - K) / (col(1.0f) - ba * K);
    return lerpc(col(1.0f), dk, m.coat * m.coat_darkening);
}
DEV Col spec_darkening(const Mat& m, float rel) {
    if (m.specular_darkening == 0.0f) return col(1.0f);
    float K = 1.0f - (1.0f - fresnel_hemispherical_albedo(rel)) / (rel * rel);
    Col dk = (1.0f - K) / (col(1.0f) - C3(m.base_color) * K);
    return lerpc(col(1.0f), dk, m.specular * m.specular_darkening);
}

DEV void lobe_weights(const Mat& m, bool outside, float w[7]) {
    float o = outside ? 1.0f : 0.0f;
    w[0] = m.coat * o;
    w[1] = m.sheen * o;
    w[2] = lerpr(m.metallic * o, 0.0f, m.second_roughness_weight);
    w[3] = lerpr(0.0f, m.metallic * o, m.second_roughness_weight);
    w[4] = (1.0f - m.metallic) * (1.0f - m.specular_transmission) * m.specular * o;
    w[5] = (1.0f - m.metallic) * (1.0f - m.specular_transmission) * o;
    w[6] = !outside ? 1.0f : (1.0f - m.metallic) * m.specular_transmission;
}
DEV void lobe_probas(const float w[7], float p[7]) {
    float nf = 1.0f / (w[0] + w[1] + w[2] + w[3] + w[4] + w[5] + w[6]);
#pragma unroll
    for (int i = 0; i < 7; i++) p[i] = w[i] * nf;
}

// Principled BSDF evaluation (Principled.h:430-790), split into the part that depends
// only on the path vertex (normal frame, view direction in both frames, lobe weights,
// incident IOR, the view-side Fresnel / darkening terms and the LUT energy
// compensation) and the part that depends on the light direction.  A vertex evaluates
// the BSDF up to ~9 times (RIS candidates, MIS, envmap, continuation); the vertex part
// is computed once.  Same operations in the same order as a monolithic evaluation, so
// the results are bit-identical to it.
struct PEval {
    v3 n, T, B, lv, TR, BR, lvr;
    bool outside;
    float w[7], p[7];
    float inc;
    float coat_vdf, coat_oa;
    Col coat_dark;
    float rel;
    bool spec_ok;
    Col spec_tint, spec_vdf, spec_dark;
    float gbc, ccc;
    // the material fields every class's glossy base reads per evaluation: a snapshot here, so
    // that a per-slot resolved (textured) material is gathered once per vertex, not once per
    // evaluation (63 dwords: an odd LDS stride)
    float ior, tfilm, spec;
    Col base;
    // the glossy base's view-only GGX terms: alphas of (roughness, anisotropy), lambda_smith and
    // G1 of the view direction lvr (65 dwords: an odd LDS stride)
    float gax, gay, glv, gg1v;
};

template <int FULL = BC_FULL>
DEV void principled_eval_pre(const BCtx& c, const Mat& m, const VState& vs, v3 view, v3 sn, PEval& e) {
    v3 n = sn;
    e.outside = dot(view, n) > 0 || m.thin_walled;
    if (dot(view, n) < 0.0f) n = -n;
    e.n = n;
    e.ior = m.ior; e.tfilm = m.thin_film; e.spec = m.specular;
    e.base = C3(m.base_color);
    build_onb(n, e.T, e.B);
    e.lv = to_local(e.T, e.B, n, view);
    build_rotated_onb(n, e.TR, e.BR, m.anisotropy_rotation * PI);
    e.lvr = to_local(e.TR, e.BR, n, view);
    alphas(m.roughness, m.anisotropy, e.gax, e.gay);
    e.glv = lambda_smith(e.gax, e.gay, e.lvr);
    e.gg1v = 1.0f / (1.0f + e.glv);
    lobe_weights(m, e.outside, e.w);
    e.inc = ior_or_air(c, vs.incident);
    lobe_probas(e.w, e.p);
    // coat, view side (entered when the coat has weight or the light refracts, which
    // needs 'outside')
    e.coat_vdf = 0.0f; e.coat_oa = 0.0f; e.coat_dark = col(1.0f);
    if (bc_layers(FULL) && (e.w[0] > 0.0f || e.outside)) {
        e.coat_vdf = fresnel_dielectric(absr(e.lv.z), e.inc, m.coat_ior);
        if (!is_white(C3(m.coat_medium_absorption)))
            e.coat_oa = maxr(1.0e-6f, sqrtf(1.0f - (1.0f - e.lv.z * e.lv.z) / (m.coat_ior * m.coat_ior)));
        e.coat_dark = coat_darkening(m, m.coat_ior / e.inc, e.coat_vdf);
    }
    // specular layer, view side
    e.rel = 1.0f; e.spec_ok = false;
    e.spec_tint = col(1.0f); e.spec_vdf = col(0.0f); e.spec_dark = col(1.0f);
    if (e.w[4] > 0.0f) {
        e.rel = spec_rel_ior(m, e.inc);
        e.spec_ok = absr(e.rel - 1.0f) > 1.0e-3f;
        if (e.spec_ok) {
            e.spec_tint = lerpc(col(1.0f), m.specular_tint * C3(m.specular_color), m.specular);
            e.spec_vdf = spec_fresnel<FULL>(m, e.rel, e.lvr.z);
            e.spec_dark = spec_darkening(m, e.rel);
        }
    }
    e.gbc = glossy_base_comp(c, m, e.inc, e.lv.z);
    e.ccc = c.clearcoat_comp ? clearcoat_comp(c, m, e.inc, e.lv.z) : 1.0f;
}

// A plain-dielectric material (FULL = false) has zero coat / sheen / metal weights and,
// seen from outside (the only way k_shade evaluates it, see MC_PLAIN), zero glass weight:
// the generic code skips those lobes too, except the coat block on a refracting direction,
// which then only scales the throughput of lobes that are all skipped (nr = 0, w[6] = 0),
// and adds cp * p[0] = 0 to the pdf and a zero colour to fc -- no effect on the result.
template <int FULL = BC_FULL>
DEV Col principled_eval_post(const BCtx& c, const Mat& m, VState& vs, const PEval& e, v3 sn, v3 L, float& pdf) {
    pdf = 0.0f;
    const bool refracting = dot(sn, L) < 0.0f && e.outside;
    const v3 n = e.n;
    v3 ll = to_local(e.T, e.B, n, L);
    v3 lh = normalize(e.lv + ll);
    v3 llr = to_local(e.TR, e.BR, n, L);
    v3 lhr = normalize(e.lvr + llr);
    const v3 lv = e.lv, lvr = e.lvr;
    const float inc = e.inc;
    Col thr = col(1.0f), fc = col(0.0f);
    float nr = refracting ? 0.0f : 1.0f;
    // coat (Principled.h:493-593)
    if (bc_layers(FULL) && (e.w[0] > 0.0f || refracting)) {
        float cp = 0.0f;
        Col ct = col(0.0f);
        if (!refracting) {
            float HoL = clampr(1.0e-8f, 1.0f, dot(lh, ll));
            ct = ts_ggx1(c, m.coat_roughness, m.coat_anisotropy, col(fresnel_dielectric(HoL, inc, m.coat_ior)), lv, ll, lh, cp);
            ct *= e.w[0];
            ct *= thr;
        }
        pdf += cp * e.p[0];
        Col att = col(1.0f);
        att *= 1.0f - fresnel_dielectric(absr(ll.z), inc, m.coat_ior);
        att *= 1.0f - e.coat_vdf;
        if (!is_white(C3(m.coat_medium_absorption))) {
            float ia = maxr(1.0e-6f, sqrtf(1.0f - (1.0f - ll.z * ll.z) / (m.coat_ior * m.coat_ior)));
            float tda = 1.0f / ia + 1.0f / e.coat_oa;
            att *= cexp(-(col(1.0f) - cpow(csqrt(C3(m.coat_medium_absorption)), tda)) * m.coat_medium_thickness);
        }
        att *= e.coat_dark;
        att = lerpc(col(1.0f), att, m.coat);
        thr *= att;
        fc += ct;
    }
    // sheen
    if (bc_extra(FULL) && e.w[1] > 0.0f) {
        float refl, sp;
        Col ct = sheen_eval(c, m, ll, lv, sp, refl);
        ct *= e.w[1];
        ct *= thr;
        pdf += sp * e.p[1];
        thr *= 1.0f - m.sheen * refl;
        fc += ct;
    }
    // metal x2
#pragma unroll
    for (int k = 0; k < 2; k++) {
        float wk = e.w[2 + k] * nr;
        if (bc_extra(FULL) && wk > 0.0f) {
            float mp;
            float HoL = clampr(1.0e-8f, 1.0f, dot(lhr, llr));
            Col Fm = f82_tint(C3(m.base_color), C3(m.metallic_F82), C3(m.metallic_F90), m.metallic_F90_falloff_exponent, HoL);
            Col Ft = thin_film_fresnel(m, inc, HoL);
            Col ct = ts_ggx1(c, k == 0 ? m.roughness : m.second_roughness, m.anisotropy, lerpc(Fm, Ft, m.thin_film), lvr, llr, lhr, mp);
            ct *= wk;
            ct *= thr;
            pdf += mp * e.p[2 + k];
            fc += ct;
        }
    }
    // glass
    if (bc_layers(FULL) && e.w[6] > 0.0f) {
        float gp;
        Col ct = glass_eval<FULL>(c, m, vs, lvr, llr, gp);
        ct *= e.w[6];
        ct *= thr;
        pdf += gp * e.p[6];
        fc += ct;
    }
    // glossy base = specular + diffuse
    {
        Col g = col(0.0f);
        float ws = e.w[4] * nr;
        if (ws > 0.0f) {
            float sp;
            Col ct = ts_ggx0_v(c, e.gax, e.gay, e.glv, e.gg1v, spec_fresnel_v<FULL>(m, e.ior, e.tfilm, e.rel, dot(llr, lhr)), lvr, llr,
                               lhr, sp);
            if (e.spec_ok) {
                ct *= e.spec_tint;
                ct *= ws;
                ct *= thr;
                Col att = col(1.0f);
                att *= col(1.0f) - spec_fresnel_v<FULL>(m, e.ior, e.tfilm, e.rel, llr.z);
                att *= col(1.0f) - e.spec_vdf;
                att *= e.spec_dark;
                att = lerpc(col(1.0f), att, e.spec);
                thr *= att;
            }
            pdf += sp * e.p[4];
            g += ct;
        }
        float wd = e.w[5] * nr;
        if (wd > 0.0f) {
            float dp;
            Col ct = lambert_eval_c(e.base, ll.z, dp);
            ct *= wd;
            ct *= thr;
            pdf += dp * e.p[5];
            g += ct;
        }
        fc += g / e.gbc;
    }
    if (c.clearcoat_comp) fc /= e.ccc;
    return fc;
}

DEV Col principled_eval(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 n, v3 L, float& pdf) {
    PEval e;
    principled_eval_pre(c, m, vs, view, n, e);
    return principled_eval_post(c, m, vs, e, n, L, pdf);
}

// Direction half of PrincipledBSDF sampling (Principled.h:1050-1120): picks a lobe, samples
// it, updates the nested-dielectric state.  Returns false where the reference returns a
// zero BSDF without evaluating it (direction below the surface for a non-glass lobe).
// FULL = false (plain dielectric): p[0] = p[1] = 0, so r1 < c0 and r1 < c1 never hold (r1 >= 0)
// and the coat / sheen samplers are not compiled in; the glass branch stays (r1 > c5 can
// hold by rounding when p[6] = 0).
template <int FULL = BC_FULL>
DEV bool principled_sample_dir(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 sn, v3 gn, v3& out, Rng& rng) {
    v3 n = sn;
    bool outside = dot(view, n) > 0 || m.thin_walled;
    float gw = (1.0f - m.metallic) * m.specular_transmission;
    if (is_zero(gw) && !outside) { n = reflect_ray(sn, gn); outside = true; }
    float w[7], p[7];
    lobe_weights(m, outside, w);
    if (!outside) w[6] = 1.0f;
    lobe_probas(w, p);
    float c0 = p[0], c1 = c0 + p[1], c2 = c1 + p[2], c3 = c2 + p[3], c4 = c3 + p[4], c5 = c4 + p[5];
    float r1 = rng();
    bool glass = r1 > c5;
    if (glass) {
        float ds = dot(view, sn), dg = dot(view, gn);
        if (ds * dg < 0) n = reflect_ray(sn, gn);
    }
    if (!glass) vs_pop(vs, false);
    if (dot(view, n) < 0) n = -n;
    v3 TR, BR;
    build_rotated_onb(n, TR, BR, m.anisotropy_rotation * PI);
    v3 lvr = to_local(TR, BR, n, view);
    if (bc_extra(FULL) && r1 < c0) {
        v3 TC, BC;
        build_rotated_onb(n, TC, BC, m.coat_anisotropy_rotation * PI);
        out = to_world(TC, BC, n, ggx_sample_reflection(m.coat_roughness, m.coat_anisotropy, to_local(TC, BC, n, view), rng));
    } else if (bc_extra(FULL) && r1 < c1) {
        v3 T, B;
        build_onb(n, T, B);
        out = to_world(T, B, n, sheen_sample(c, m, to_local(T, B, n, view), rng));
    } else if (r1 < c4) {
        // metal (first / second roughness) and specular lobes share the GGX reflection sampler
        float r = (r1 >= c2 && r1 < c3) ? m.second_roughness : m.roughness;
        out = to_world(TR, BR, n, ggx_sample_reflection(r, m.anisotropy, lvr, rng));
    } else if (r1 < c5) {
        out = cosine_sample_around(n, rng);
    } else {
        out = to_world(TR, BR, n, glass_sample<FULL>(c, m, vs, lvr, rng));
    }
    return !(dot(out, sn) < 0 && !glass);
}

// The plain class's direction sampling from the vertex's PEval (k_shade<PLAIN>).  Such a
// vertex is shaded from outside (k_shade defers the others), so principled_sample_dir's
// frame (n, TR, BR, lvr), lobe weights and probabilities are the ones principled_eval_pre
// stored -- the same operations on the same inputs, done once per vertex instead of once per
// sample (a rotated frame costs a sine / cosine pair).  The glass branch (reached only by
// rounding, p[6] = 0) rebuilds its frame as principled_sample_dir does.
DEV bool principled_sample_dir_plain(const BCtx& c, const Mat& m, VState& vs, const PEval& e, v3 view, v3 sn, v3 gn, v3& out,
                                     Rng& rng) {
    const float* p = e.p;
    float c0 = p[0], c1 = c0 + p[1], c2 = c1 + p[2], c3 = c2 + p[3], c4 = c3 + p[4], c5 = c4 + p[5];
    (void)c0;
    float r1 = rng();
    if (r1 > c5) {
        v3 n = sn;
        float ds = dot(view, sn), dg = dot(view, gn);
        if (ds * dg < 0) n = reflect_ray(sn, gn);
        if (dot(view, n) < 0) n = -n;
        v3 TR, BR;
        build_rotated_onb(n, TR, BR, m.anisotropy_rotation * PI);
        out = to_world(TR, BR, n, glass_sample<BC_PLAIN>(c, m, vs, to_local(TR, BR, n, view), rng));
        return true;
    }
    vs_pop(vs, false);
    if (r1 < c4) {
        out = to_world(e.TR, e.BR, e.n, (r1 >= c2 && r1 < c3) ? ggx_sample_reflection(m.second_roughness, m.anisotropy, e.lvr, rng)
                                                              : ggx_sample_reflection_a(e.gax, e.gay, e.lvr, rng));
    } else if (r1 < c5) {
        out = cosine_sample_around(e.n, rng);
    } else {
        out = to_world(e.TR, e.BR, e.n, glass_sample<BC_PLAIN>(c, m, vs, e.lvr, rng));
    }
    return !(dot(out, sn) < 0);
}

// The plain class's per-vertex record (k_shade<PLAIN>, Principled BSDF).  k_shade shades a plain
// vertex only when the resolved material has zero coat, sheen, metallic, transmission and thin
// film and the vertex is seen from outside (any other vertex is deferred to the generic kernel
// before it writes anything), so of PEval the evaluation reads only the glossy base: the frame
// (n, TR, BR, lvr), the specular layer's view-side terms, the diffuse colour and the GGX
// view-only terms.  The other terms are exact constants there -- lobe weights w[4] = specular,
// w[5] = 1 and the rest 0, so probabilities p[0..3] = p[6] = 0; the coat's clearcoat
// compensation 1; the unrotated frame (T, B) is build_onb(n), recomputed per evaluation -- and the
// operations on the terms kept are principled_eval_pre / _post<BC_PLAIN>'s, so the values are
// bit-identical to PEval's.  35 dwords (an odd LDS stride, conflict-free) instead of 65: with
// the 55 B per lane of promoted private arrays a 256-lane block needs 49.9 KB of LDS, so three
// blocks fit a CU.
struct PEvalP {
    v3 n, TR, BR, lvr;
    float p4, p5;
    float rel;
    uint32_t spec_ok;
    Col spec_tint, spec_vdf, spec_dark;
    float gbc, spec;
    Col base;
    float gax, gay, glv, gg1v;
    float pad_;
};
DEV bool plain_vertex_ok(const Mat& m) {   // k_shade<PLAIN>: the material terms PEvalP takes as zero
    return m.metallic == 0.0f && m.specular_transmission == 0.0f && m.thin_film == 0.0f && m.coat == 0.0f && m.sheen == 0.0f;
}
DEV void principled_eval_pre_plain(const BCtx& c, const Mat& m, const VState& vs, v3 view, v3 sn, PEvalP& e) {
    v3 n = sn;
    const bool outside = dot(view, n) > 0 || m.thin_walled;
    if (dot(view, n) < 0.0f) n = -n;
    e.n = n;
    e.spec = m.specular;
    e.base = C3(m.base_color);
    v3 T, B;
    build_onb(n, T, B);
    const v3 lv = to_local(T, B, n, view);
    build_rotated_onb(n, e.TR, e.BR, m.anisotropy_rotation * PI);
    e.lvr = to_local(e.TR, e.BR, n, view);
    alphas(m.roughness, m.anisotropy, e.gax, e.gay);
    e.glv = lambda_smith(e.gax, e.gay, e.lvr);
    e.gg1v = 1.0f / (1.0f + e.glv);
    float w[7], p[7];
    lobe_weights(m, outside, w);
    const float inc = ior_or_air(c, vs.incident);
    lobe_probas(w, p);
    e.p4 = p[4];
    e.p5 = p[5];
    e.rel = 1.0f;
    e.spec_ok = 0u;
    e.spec_tint = col(1.0f); e.spec_vdf = col(0.0f); e.spec_dark = col(1.0f);
    if (w[4] > 0.0f) {
        e.rel = spec_rel_ior(m, inc);
        const bool ok = absr(e.rel - 1.0f) > 1.0e-3f;
        e.spec_ok = ok ? 1u : 0u;
        if (ok) {
            e.spec_tint = lerpc(col(1.0f), m.specular_tint * C3(m.specular_color), m.specular);
            e.spec_vdf = spec_fresnel_v<BC_PLAIN>(m, 0.0f, 0.0f, e.rel, e.lvr.z);
            e.spec_dark = spec_darkening(m, e.rel);
        }
    }
    e.gbc = glossy_base_comp(c, m, inc, lv.z);
    e.pad_ = 0.0f;
}
DEV Col principled_eval_post_plain(const BCtx& c, const Mat& m, const PEvalP& e, v3 sn, v3 L, float& pdf) {
    pdf = 0.0f;
    const bool refracting = dot(sn, L) < 0.0f;   // (seen from outside)
    const v3 n = e.n;
    v3 T, B;
    build_onb(n, T, B);
    const v3 ll = to_local(T, B, n, L);
    const v3 llr = to_local(e.TR, e.BR, n, L);
    const v3 lhr = normalize(e.lvr + llr);
    Col thr = col(1.0f), fc = col(0.0f);
    const float nr = refracting ? 0.0f : 1.0f;
    Col g = col(0.0f);
    const float ws = e.spec * nr;
    if (ws > 0.0f) {
        float sp;
        Col ct = ts_ggx0_v(c, e.gax, e.gay, e.glv, e.gg1v, spec_fresnel_v<BC_PLAIN>(m, 0.0f, 0.0f, e.rel, dot(llr, lhr)), e.lvr, llr,
                           lhr, sp);
        if (e.spec_ok) {
            ct *= e.spec_tint;
            ct *= ws;
            ct *= thr;
            Col att = col(1.0f);
            att *= col(1.0f) - spec_fresnel_v<BC_PLAIN>(m, 0.0f, 0.0f, e.rel, llr.z);
            att *= col(1.0f) - e.spec_vdf;
            att *= e.spec_dark;
            att = lerpc(col(1.0f), att, e.spec);
            thr *= att;
        }
        pdf += sp * e.p4;
        g += ct;
    }
    const float wd = 1.0f * nr;
    if (wd > 0.0f) {
        float dp;
        Col ct = lambert_eval_c(e.base, ll.z, dp);
        ct *= wd;
        ct *= thr;
        pdf += dp * e.p5;
        g += ct;
    }
    fc += g / e.gbc;
    return fc;   // (the clearcoat compensation of a coat-less material divides by 1)
}
// principled_sample_dir_plain from the plain record: c0 .. c3 are 0 (p[0..3] = 0), so the
// second-roughness metal branch is never taken
DEV bool principled_sample_dir_plain(const BCtx& c, const Mat& m, VState& vs, const PEvalP& e, v3 view, v3 sn, v3 gn, v3& out,
                                      Rng& rng) {
    const float c4 = 0.0f + e.p4, c5 = c4 + e.p5;
    float r1 = rng();
    if (r1 > c5) {
        v3 n = sn;
        float ds = dot(view, sn), dg = dot(view, gn);
        if (ds * dg < 0) n = reflect_ray(sn, gn);
        if (dot(view, n) < 0) n = -n;
        v3 TR, BR;
        build_rotated_onb(n, TR, BR, m.anisotropy_rotation * PI);
        out = to_world(TR, BR, n, glass_sample<BC_PLAIN>(c, m, vs, to_local(TR, BR, n, view), rng));
        return true;
    }
    vs_pop(vs, false);
    if (r1 < c4) out = to_world(e.TR, e.BR, e.n, ggx_sample_reflection_a(e.gax, e.gay, e.lvr, rng));
    else if (r1 < c5) out = cosine_sample_around(e.n, rng);
    else out = to_world(e.TR, e.BR, e.n, glass_sample<BC_PLAIN>(c, m, vs, e.lvr, rng));
    return !(dot(out, sn) < 0);
}

DEV Col principled_sample(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 sn, v3 gn, v3& out, float& pdf, Rng& rng) {
    pdf = 0.0f;
    if (!principled_sample_dir(c, m, vs, view, sn, gn, out, rng)) return col(0.0f);
    return principled_eval(c, m, vs, view, sn, out, pdf);
}

// bsdf_dispatcher_eval / _sample (Dispatcher.h:18-68).  BSDF_OREN_NAYAR: the reference's
// dispatcher line calls 'oren_nayar_brdf_eval<0>(material, view, normal, light, pdf)' on a
// function that is not a template (Dispatcher.h:38), so that override does not compile there;
// this is the evident intent, the world-space overload of OrenNayar.h:92-103 (local frame
// from build_ONB around the shading normal) and its cosine-weighted sampler (:105-110).
template <int OVERRIDE>
DEV Col bsdf_eval(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 sn, v3 L, float& pdf) {
    if (OVERRIDE == MPT_BSDF_LAMBERTIAN) return lambert_eval(m, dot(L, sn), pdf);
    if (OVERRIDE == MPT_BSDF_OREN_NAYAR) {
        v3 T, B;
        build_onb(sn, T, B);
        return oren_nayar_eval(m, to_local(T, B, sn, view), to_local(T, B, sn, L), pdf);
    }
    return principled_eval(c, m, vs, view, sn, L, pdf);
}
// evaluation split into a per-vertex part and a per-light-direction part (see PEval)
template <int OVERRIDE, int FULL = BC_FULL>
DEV void bsdf_eval_pre(const BCtx& c, const Mat& m, const VState& vs, v3 view, v3 sn, PEval& e) {
    if (OVERRIDE == MPT_BSDF_OREN_NAYAR) {
        build_onb(sn, e.T, e.B);
        e.lv = to_local(e.T, e.B, sn, view);
    } else if (OVERRIDE != MPT_BSDF_LAMBERTIAN) principled_eval_pre<FULL>(c, m, vs, view, sn, e);
}
template <int OVERRIDE, int FULL = BC_FULL>
DEV Col bsdf_eval_post(const BCtx& c, const Mat& m, VState& vs, const PEval& e, v3 sn, v3 L, float& pdf) {
    if (OVERRIDE == MPT_BSDF_LAMBERTIAN) return lambert_eval(m, dot(L, sn), pdf);
    if (OVERRIDE == MPT_BSDF_OREN_NAYAR) return oren_nayar_eval(m, e.lv, to_local(e.T, e.B, sn, L), pdf);
    return principled_eval_post<FULL>(c, m, vs, e, sn, L, pdf);
}
// the plain record (k_shade<PLAIN>, Principled only)
template <int OVERRIDE, int FULL = BC_FULL>
DEV void bsdf_eval_pre(const BCtx& c, const Mat& m, const VState& vs, v3 view, v3 sn, PEvalP& e) {
    static_assert(OVERRIDE == MPT_BSDF_NONE && FULL == BC_PLAIN, "PEvalP: the plain class of the Principled BSDF");
    principled_eval_pre_plain(c, m, vs, view, sn, e);
}
template <int OVERRIDE, int FULL = BC_FULL>
DEV Col bsdf_eval_post(const BCtx& c, const Mat& m, VState&, const PEvalP& e, v3 sn, v3 L, float& pdf) {
    static_assert(OVERRIDE == MPT_BSDF_NONE && FULL == BC_PLAIN, "PEvalP: the plain class of the Principled BSDF");
    return principled_eval_post_plain(c, m, e, sn, L, pdf);
}
// sample = sample_dir + bsdf_eval on the updated state (eval skipped when sample_dir is false)
template <int OVERRIDE, int FULL = BC_FULL>
DEV bool bsdf_sample_dir(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 sn, v3 gn, v3& dir, Rng& rng) {
    if (OVERRIDE == MPT_BSDF_LAMBERTIAN || OVERRIDE == MPT_BSDF_OREN_NAYAR) { dir = cosine_sample_around(sn, rng); return true; }
    return principled_sample_dir<FULL>(c, m, vs, view, sn, gn, dir, rng);
}
template <int OVERRIDE>
DEV Col bsdf_sample(const BCtx& c, const Mat& m, VState& vs, v3 view, v3 sn, v3 gn, v3& dir, float& pdf, Rng& rng) {
    pdf = 0.0f;
    if (!bsdf_sample_dir<OVERRIDE>(c, m, vs, view, sn, gn, dir, rng)) return col(0.0f);
    return bsdf_eval<OVERRIDE>(c, m, vs, view, sn, dir, pdf);
}

}  // namespace mpt
#endif
