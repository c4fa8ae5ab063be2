/*
 * oracle_bsdf.h -- TEST INFRASTRUCTURE ONLY (parity checker).  CPU restatement of the
 * reference's BSDF stack, following (file:line under /root/reference/src):
 *   Lambertian ............... Device/includes/BSDFs/Lambertian.h:14-30
 *   cosine sampling ........... Device/includes/Sampling.h:175-216
 *   GGX / Smith / VNDF ........ Device/includes/BSDFs/Microfacet.h:25-256
 *   Fresnel ................... Device/includes/Fresnel.h:11-165
 *   thin film ................. Device/includes/BSDFs/ThinFilm.h:12-221
 *   sheen LTC ................. Device/includes/BSDFs/SheenLTC.h:24-150
 *   energy compensation ....... Device/includes/BSDFs/MicrofacetEnergyCompensation.h:25-705,
 *                               Device/includes/BSDFs/PrincipledEnergyCompensation.h:13-80
 *   Principled BSDF ........... Device/includes/BSDFs/Principled.h:51-1193
 *   nested dielectrics ........ Device/includes/NestedDielectrics.h:135-290
 *   dispersion ................ Device/includes/Dispersion.h:392-540 (fit path)
 *   material fetch ............ Device/includes/Material.h:47-159, Texture.h:31-222,
 *                               Image/Image.cpp:161-195, 492-526, 737-779 (CPU nearest texel)
 * Parity status: see oracle.cpp header.
 */
#ifndef ORACLE_BSDF_H
#define ORACLE_BSDF_H

#include "oracle_math.h"
#include "../include/mpt.h"

namespace orc {

typedef MptMaterial Material;  // RendererMaterial layout; the Simplified material is its prefix

// --------------------------------------------------------------------------------
// LUT / texture sampling with the CPU's nearest-texel semantics
// --------------------------------------------------------------------------------
inline float wrap01(float u, float src) { if (u != 1.0f) u -= (float)(int)src; return u < 0 ? 1.0f + u : u; }

// Image32Bit::sample_rgba32f (Image.cpp:737-779), 1 channel LUT, data[y][x]
inline float lut2d(const float* data, int w, int h, float u_in, float v_in) {
    float u = wrap01(u_in, u_in), v = wrap01(v_in, v_in);
    v = 1.0f - v;
    int x = (int)(u * (float)(w - 1));
    int y = (int)(v * (float)(h - 1));
    return data[x + y * w];
}
// Image32Bit3D::sample_rgba32f (Image.cpp:840-880), data[z][y][x]
inline float lut3d(const float* data, int w, int h, int d, float u_in, float v_in, float w_in) {
    float u = wrap01(u_in, u_in), v = wrap01(v_in, v_in), ww = wrap01(w_in, w_in);
    v = 1.0f - v;
    int x = (int)(u * (float)(w - 1));
    int y = (int)(v * (float)(h - 1));
    int z = (int)(ww * (float)(d - 1));
    return data[(size_t)z * w * h + x + y * w];
}

struct Luts {
    const float* conductor;   // 128 x 128
    const float* glossy;      // 128(z) x 64 x 128
    const float* glass;       // 128 x 16 x 256
    const float* glass_inv;   // 128 x 16 x 256
    const float* thin_glass;  // 96 x 32 x 32
    const float* sheen;       // 32 x 32 x 3
};

struct Textures {
    int count;
    const uint8_t* const* data;  // RGBA8
    const int32_t* dims;          // w, h pairs
};

// Image8Bit::sample_rgba32f (Image.cpp:161-195) + sRGB pow (Texture.h:72-75)
inline void sample_texture_rgba(const Textures& tex, int index, bool srgb, f2 uv, float out[4]) {
    int w = tex.dims[2 * index], h = tex.dims[2 * index + 1];
    float u = wrap01(uv.x, uv.x), v = wrap01(uv.y, uv.y);
    v = 1.0f - v;
    int x = (int)(u * (float)(w - 1));
    int y = (int)(v * (float)(h - 1));
    const uint8_t* p = tex.data[index] + (size_t)(x + y * w) * 4;
    for (int i = 0; i < 4; i++) out[i] = (float)p[i] / 255.0f;
    if (srgb) for (int i = 0; i < 4; i++) out[i] = ppow(out[i], 2.2f);
}

// --------------------------------------------------------------------------------
// Nested dielectrics: InteriorStackImpl<ISS_WITH_PRIORITIES> (NestedDielectrics.h:135-290)
// StackPriorityEntry swaps its bitfield widths (NestedDielectrics.h:162-165): the
// priority keeps 1 bit, odd_parity is a bool.  Restated bug-for-bug.
// --------------------------------------------------------------------------------
constexpr int STACK_SIZE = 3;                       // NESTED_DIELECTRICS_STACK_SIZE (KernelOptions.h:53)
constexpr int MAX_MATERIAL_INDEX = (1 << 26) - 1;   // MATERIAL_INDEX_MAXIMUM

struct StackEntry {
    uint32_t priority;      // 1 bit
    bool odd_parity;
    bool topmost;
    uint32_t material_index; // 26 bits
    StackEntry() : priority(0), odd_parity(true), topmost(true), material_index(MAX_MATERIAL_INDEX) {}
};

struct InteriorStack {
    StackEntry stack[STACK_SIZE];
    int stack_position = 0;

    bool push(int& incident, int& outgoing, bool& inside_material, int material_index, int material_priority) {
        int last = 0;
        for (last = stack_position; last >= 0; last--)
            if ((int)stack[last].material_index != material_index && stack[last].topmost && stack[last].odd_parity) break;
        bool odd = true;
        int prev;
        for (prev = stack_position; prev >= 0; prev--) {
            if ((int)stack[prev].material_index == material_index) {
                stack[prev].topmost = false;
                odd = !stack[prev].odd_parity;
                break;
            }
        }
        inside_material = !odd;
        if (stack_position < STACK_SIZE - 1) stack_position++;
        stack[stack_position].material_index = (uint32_t)material_index & MAX_MATERIAL_INDEX;
        stack[stack_position].odd_parity = odd;
        stack[stack_position].topmost = true;
        stack[stack_position].priority = (uint32_t)material_priority & 1u;
        if (material_priority < (int)stack[last].priority) return true;
        if (odd) { incident = (int)stack[last].material_index; outgoing = material_index; }
        else { incident = material_index; outgoing = (int)stack[last].material_index; }
        return false;
    }

    void pop(bool inside_material) {
        int top = (int)stack[stack_position].material_index;
        if (stack_position > 0) stack_position--;
        if (inside_material) {
            int prev;
            for (prev = stack_position; prev >= 0; prev--)
                if ((int)stack[prev].material_index == top) break;
            if (prev >= 0)
                for (int i = prev + 1; i <= stack_position; i++) stack[i - 1] = stack[i];
            if (stack_position > 0) stack_position--;
        }
        for (int i = stack_position; i >= 0; i--) {
            if ((int)stack[i].material_index == top) { stack[i].topmost = true; break; }
        }
    }
};

// RayVolumeState (RayVolumeState.h:11-32)
struct VolumeState {
    float distance_in_volume = 0.0f;
    InteriorStack interior_stack;
    int incident_mat_index = -1, outgoing_mat_index = -1;
    bool inside_material = false;
    float sampled_wavelength = 0.0f;
};

// --------------------------------------------------------------------------------
// Dispersion (Dispersion.h:392-540, WAVELENGTH_TO_RGB_FIT)
// --------------------------------------------------------------------------------
inline Col wavelength_to_rgb(float w) {
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
inline float sample_wavelength_uniformly(Rng& rng) { float r = rng(); return r * (float)(830 - 360) + (float)360; }
inline float compute_dispersion_ior(float abbe, float scale, float base, float wavelength) {
    if (scale == 0.0f) return base;
    float abbe_number = abbe / scale;
    float B = (base - 1.0f) / (abbe_number * 0.00000191038851931481f);
    float A = base - B / (334777.96f);
    return A + B / (wavelength * wavelength);
}
inline Col get_dispersion_ray_color(float& wavelength, float scale) {
    if (scale == 0.0f) return Col(1.0f);
    if (wavelength >= 0.0f) return Col(1.0f);
    wavelength *= -1.0f;
    return wavelength_to_rgb(wavelength);
}

// --------------------------------------------------------------------------------
// Sampling helpers (Sampling.h)
// --------------------------------------------------------------------------------
inline f3 cosine_weighted_sample_around_normal(f3 n, Rng& rng) {
    float r1 = rng();
    float r2 = 2.0f * rng() - 1.0f;
    if (r1 < 1.0e-8f && r2 < -0.999999f && n.z > 0.999999f) { r1 += 1.0e-7f; r2 += 1.0e-7f; }
    float theta = TWO_PI * r1;
    float s = psqrt(1.0f - r2 * r2);
    f3 sp = mk3(s * pcos(theta), s * psin(theta), r2);
    return normalize(n + sp);
}
inline f3 cosine_weighted_sample_z_up_frame(Rng& rng) {
    float r1 = rng(), r2 = rng();
    float phi = TWO_PI * r1;
    float ct = psqrt(r2);
    float st = psqrt(1.0f - ct * ct);
    return normalize(mk3(pcos(phi) * st, psin(phi) * st, ct));
}

// --------------------------------------------------------------------------------
// Lambert (Lambertian.h:14-30)
// --------------------------------------------------------------------------------
inline Col lambertian_eval(const Material& m, float NoL, float& pdf) {
    pdf = 0.0f;
    if (NoL <= 0.0f) return Col(0.0f);
    pdf = NoL * INV_PI;
    return Col(m.base_color.r, m.base_color.g, m.base_color.b) * INV_PI;
}
inline Col lambertian_sample(const Material& m, f3 n, f3& dir, float& pdf, Rng& rng) {
    dir = cosine_weighted_sample_around_normal(n, rng);
    return lambertian_eval(m, dot(n, dir), pdf);
}

// --------------------------------------------------------------------------------
// Oren-Nayar (OrenNayar.h:49-110; A, B: Material.h:73-78).  The reference's dispatcher calls
// 'oren_nayar_brdf_eval<0>(...)' on a non-template (Dispatcher.h:38): BSDF_OREN_NAYAR does not
// compile there, and this restates the evident intent, the world-space overload.
// --------------------------------------------------------------------------------
inline Col oren_nayar_eval_local(const Material& m, f3 local_view, f3 local_light, float& pdf) {
    float sin_theta_i = psqrt(1.0f - local_light.z * local_light.z);
    float sin_theta_o = psqrt(1.0f - local_view.z * local_view.z);
    float max_cos = 0.0f;
    if (sin_theta_i > 1.0e-4f && sin_theta_o > 1.0e-4f) {
        float sin_phi_i = local_light.y / sin_theta_i, cos_phi_i = local_light.x / sin_theta_i;
        float sin_phi_o = local_view.y / sin_theta_o, cos_phi_o = local_view.x / sin_theta_o;
        float d_cos = cos_phi_i * cos_phi_o + sin_phi_i * sin_phi_o;
        max_cos = fmaxr(0.0f, d_cos);
    }
    float sin_alpha, tan_beta;
    if (absf(local_light.z) > absf(local_view.z)) { sin_alpha = sin_theta_o; tan_beta = sin_theta_i / absf(local_light.z); }
    else { sin_alpha = sin_theta_i; tan_beta = sin_theta_o / absf(local_view.z); }
    float sigma2 = m.oren_nayar_sigma * m.oren_nayar_sigma;
    float A = 1.0f - sigma2 / (2.0f * (sigma2 + 0.33f));
    float B = 0.45f * sigma2 / (sigma2 + 0.09f);
    pdf = local_light.z * INV_PI;
    return Col(m.base_color.r, m.base_color.g, m.base_color.b) * INV_PI * (A + B * max_cos * sin_alpha * tan_beta);
}
inline Col oren_nayar_eval(const Material& m, f3 view, f3 n, f3 light, float& pdf) {
    f3 t, b;
    build_onb(n, t, b);
    return oren_nayar_eval_local(m, world_to_local(t, b, n, view), world_to_local(t, b, n, light), pdf);
}
inline Col oren_nayar_sample(const Material& m, f3 view, f3 n, f3& dir, float& pdf, Rng& rng) {
    dir = cosine_weighted_sample_around_normal(n, rng);
    return oren_nayar_eval(m, view, n, dir, pdf);
}

// --------------------------------------------------------------------------------
// Fresnel (Fresnel.h)
// --------------------------------------------------------------------------------
inline float F0_from_eta(float eta_t, float eta_i) {
    float n = eta_t - eta_i, d = eta_t + eta_i;
    return (n * n) / (d * d);
}
inline float full_fresnel_dielectric(float cos_i, float eta) {
    float sin_i2 = 1.0f - cos_i * cos_i;
    float sin_t2 = sin_i2 / (eta * eta);
    if (sin_t2 >= 1.0f) return 1.0f;
    float cos_t = psqrt(1.0f - sin_t2);
    float rpar = (eta * cos_i - cos_t) / (eta * cos_i + cos_t);
    float rper = (cos_i - eta * cos_t) / (cos_i + eta * cos_t);
    return (rpar * rpar + rper * rper) / 2.0f;
}
inline float full_fresnel_dielectric(float cos_i, float eta_i, float eta_t) { return full_fresnel_dielectric(cos_i, eta_t / eta_i); }
inline Col adobe_f82_tint_fresnel(Col F0, Col F82, Col F90, float expo, float c) {
    Col base = F0 + (F90 - F0) * ppow(1.0f - c, expo);
    float laz = c * pow6(1.0f - c);
    const float cmax = 1.0f / 7.0f;
    const float denom_a = cmax * pow6(1.0f - cmax);
    Col nume_a = (F0 + (F90 - F0) * ppow(1.0f - cmax, expo)) * (Col(1.0f) - F82);
    Col a = nume_a / denom_a;
    Col F = base - a * laz;
    F.clamp(0.0f, 1.0f);
    return F;
}
inline float fresnel_hemispherical_albedo(float eta) {
    return plog((10893.0f * eta - 1438.2f) / (-774.4f * sq(eta) + 10212.0f * eta + 1.0f));
}

// --------------------------------------------------------------------------------
// Thin film (ThinFilm.h)
// --------------------------------------------------------------------------------
inline Col eval_sensitivity(float opd, float shift) {
    float phase = 2.0f * PI * opd * 1.0e-6f;
    const float val[3] = {5.4856e-13f, 4.4201e-13f, 5.2481e-13f};
    const float pos[3] = {1.6810e+06f, 1.7953e+06f, 2.2084e+06f};
    const float var[3] = {4.3278e+09f, 9.3046e+09f, 6.6121e+09f};
    float xyz[3];
    for (int i = 0; i < 3; i++)
        xyz[i] = val[i] * psqrt(2.0f * PI * var[i]) * pcos(pos[i] * phase + shift) * pexp(-1.0f * var[i] * phase * phase);
    xyz[0] += 9.7470e-14f * psqrt(2.0f * PI * 4.5282e+09f) * pcos(2.2399e+06f * phase + shift) * pexp(-4.5282e+09f * phase * phase);
    return Col(xyz[0] / 1.0685e-7f, xyz[1] / 1.0685e-7f, xyz[2] / 1.0685e-7f);
}
inline void fresnel_phase(float ci, float eta1, float eta2, float kappa2, float& phi_par, float& phi_perp) {
    float s2 = 1.0f - sq(ci);
    float A = sq(eta2) * (1.0f - sq(kappa2)) - sq(eta1) * s2;
    float B = psqrt(sq(A) + sq(2.0f * sq(eta2) * kappa2));
    float U = (float)std::sqrt((double)(A + B) / 2.0);
    float V = (float)std::sqrt((double)(B - A) / 2.0);
    float py = 2.0f * eta1 * V * ci;
    float px = sq(U) + sq(V) - sq(eta1 * ci);
    phi_perp = patan2(py, px);
    float qy = 2.0f * eta1 * sq(eta2) * ci * (2.0f * kappa2 * U - (1.0f - sq(kappa2)) * V);
    float qx = sq(sq(eta2) * (1.0f + sq(kappa2)) * ci) - sq(eta1) * (sq(U) + sq(V));
    phi_par = patan2(qy, qx);
}
inline void fresnel_conductor(float ci, float eta, float k, float& Rp2, float& Rs2) {
    float c2 = ci * ci, s2 = 1.0f - c2;
    float t1 = eta * eta - k * k - s2;
    float a2pb2 = psqrt(t1 * t1 + 4.0f * k * k * eta * eta);
    float a = psqrt(0.5f * (a2pb2 + t1));
    float term1 = a2pb2 + c2, term2 = 2.0f * a * ci;
    Rs2 = (term1 - term2) / (term1 + term2);
    Rs2 = clampf(0.0f, 1.0f, Rs2);
    float term3 = a2pb2 * c2 + s2 * s2, term4 = term2 * s2;
    Rp2 = Rs2 * (term3 - term4) / (term3 + term4);
    Rp2 = clampf(0.0f, 1.0f, Rp2);
}
inline Col rgb_hue_shift(Col c, float deg) {
    if (deg == 0.0f) return c;
    float cosA = pcos(deg / 180.0f * PI), sinA = psin(deg / 180.0f * PI);
    double ca = cosA, sa = sinA, t = 1.0 / 3.0, st = std::sqrt(1.0 / 3.0);
    float m[3][3];
    m[0][0] = (float)(ca + (1.0 - ca) / 3.0);
    m[0][1] = (float)(t * (1.0 - ca) - st * sa);
    m[0][2] = (float)(t * (1.0 - ca) + st * sa);
    m[1][0] = (float)(t * (1.0 - ca) + st * sa);
    m[1][1] = (float)(ca + t * (1.0 - ca));
    m[1][2] = (float)(t * (1.0 - ca) - st * sa);
    m[2][0] = (float)(t * (1.0 - ca) - st * sa);
    m[2][1] = (float)(t * (1.0 - ca) + st * sa);
    m[2][2] = (float)(ca + t * (1.0 - ca));
    Col h;
    h.r = c.r * m[0][0] + c.g * m[0][1] + c.b * m[0][2];
    h.g = c.r * m[1][0] + c.g * m[1][1] + c.b * m[1][2];
    h.b = c.r * m[2][0] + c.g * m[2][1] + c.b * m[2][2];
    h.clamp(0.0f, 1.0f);
    return h;
}
inline Col thin_film_fresnel(const Material& m, float ambient_ior, float HoL) {
    float eta1 = ambient_ior, eta2 = m.thin_film_ior;
    float eta3 = m.thin_film_do_ior_override ? m.thin_film_base_ior_override : m.ior;
    float kappa3 = m.thin_film_do_ior_override ? m.thin_film_kappa_3 : 0.0f;
    float R12p = 0, R12s = 0, T121p = 0, T121s = 0, R23p = 0, R23s = 0, cos2 = 0;
    float ct2 = 1.0f - (1.0f - sq(HoL)) * sq(eta1 / eta2);
    if (ct2 <= 0.0f) { R12s = 1.0f; R12p = 1.0f; T121p = 0.0f; T121s = 0.0f; }
    else {
        cos2 = psqrt(ct2);
        fresnel_conductor(HoL, eta2 / eta1, 0.0f, R12p, R12s);
        fresnel_conductor(cos2, eta3 / eta2, kappa3, R23p, R23s);
        T121p = (float)(1.0 - (double)R12p);
        T121s = (float)(1.0 - (double)R12s);
    }
    float D = m.thin_film_thickness / 1000.0f * cos2;
    float phi21p, phi21s, phi23p, phi23s;
    fresnel_phase(HoL, eta1, eta2, 0.0f, phi21p, phi21s);
    fresnel_phase(cos2, eta2, eta3, kappa3, phi23p, phi23s);
    phi21p = PI - phi21p;
    phi21s = PI - phi21s;
    float r123p = psqrt(R12p * R23p), r123s = psqrt(R12s * R23s);
    float Rs = (sq(T121p) * R23p) / (1.0f - R12p * R23p);
    float C0 = R12p + Rs;
    Col I(C0), Sm;
    float Cm = Rs - T121p;
    for (int k = 1; k <= 2; ++k) { Cm *= r123p; Sm = 2.0f * eval_sensitivity((float)k * D, (float)k * (phi23p + phi21p)); I += Cm * Sm; }
    Rs = (sq(T121s) * R23s) / (1.0f - R12s * R23s);
    C0 = R12s + Rs;
    I += Col(C0);
    Cm = Rs - T121s;
    for (int k = 1; k <= 2; ++k) { Cm *= r123s; Sm = 2.0f * eval_sensitivity((float)k * D, (float)k * (phi23s + phi21s)); I += Cm * Sm; }
    I *= 0.5f;
    float r = 2.3646381f * I[0] - 0.8965361f * I[1] - 0.4680737f * I[2];
    float g = -0.5151664f * I[0] + 1.4264000f * I[1] + 0.0887608f * I[2];
    float b = 0.0052037f * I[0] - 0.0144081f * I[1] + 1.0092106f * I[2];
    I = Col(r, g, b);
    I.clamp(0.0f, 1.0f);
    return rgb_hue_shift(I, m.thin_film_hue_shift_degrees);
}

// --------------------------------------------------------------------------------
// Microfacet (Microfacet.h)
// --------------------------------------------------------------------------------
inline void get_alphas(float r, float aniso, float& ax, float& ay) {   // Material.h:79-84
    float aspect = psqrt(1.0f - 0.9f * aniso);
    ax = fmaxr(1.0e-4f, r * r / aspect);
    ay = fmaxr(1.0e-4f, r * r * aspect);
}
inline float GGX_anisotropic(float ax, float ay, f3 h) {
    float d = (h.x * h.x) / (ax * ax) + (h.y * h.y) / (ay * ay) + (h.z * h.z);
    return 1.0f / (PI * ax * ay * d * d);
}
inline float G1_lambda(float ax, float ay, f3 d) {
    float a = d.x * ax, b = d.y * ay;
    return (-1.0f + psqrt(1.0f + (a * a + b * b) / (d.z * d.z))) * 0.5f;
}
inline float G1_Smith(float ax, float ay, f3 d) { return 1.0f / (1.0f + G1_lambda(ax, ay, d)); }

struct BsdfCtx {           // the parts of HIPRTRenderData the BSDFs read
    const Material* materials;
    Luts luts;
    bool clearcoat_compensation;
    int ggx_masking;       // 0 height correlated
    bool white_furnace;
};

inline Col ggx_conductor_compensation(const BsdfCtx& c, Col F0, float roughness, f3 V) {
    float Ess = lut2d(c.luts.conductor, 128, 128, fmaxr(0.0f, V.z), roughness);
    float kms = (1.0f - Ess) / Ess;
    return Col(1.0f) + kms * F0;
}
inline Col torrance_sparrow0(const BsdfCtx& c, float roughness, float aniso, Col F, f3 V, f3 L, f3 H, float& pdf) {
    pdf = 0.0f;
    float ax, ay;
    get_alphas(roughness, aniso, ax, ay);
    float D = GGX_anisotropic(ax, ay, H);
    float lV = G1_lambda(ax, ay, V);
    float G1V = 1.0f / (1.0f + lV);
    float HoL = fmaxr(1.0e-3f, dot(V, H));
    float Dvis = G1V * D * HoL / V.z;
    float NoV = fmaxr(1.0e-3f, absf(V.z));
    float NoL = fmaxr(1.0e-3f, absf(L.z));
    pdf = Dvis / (4.0f * dot(V, H));
    if (pdf == 0.0f) return Col(0.0f);
    float lL = G1_lambda(ax, ay, L);
    if (c.ggx_masking == 1) {
        float G2 = G1V * (1.0f / (1.0f + lL));
        return F * D * G2 / (4.0f * NoL * NoV);
    }
    float G2 = 1.0f / (1.0f + lV + lL);
    return F * D * G2 / (4.0f * NoL * NoV);
}
inline Col torrance_sparrow1(const BsdfCtx& c, float roughness, float aniso, Col F, f3 V, f3 L, f3 H, float& pdf) {
    Col ms = ggx_conductor_compensation(c, F, roughness, V);
    Col ss = torrance_sparrow0(c, roughness, aniso, F, V, L, H, pdf);
    return ss * ms;
}
inline Col torrance_sparrow_dielectric(const BsdfCtx& c, float roughness, float aniso, float mat_ior, float inc_ior, f3 V, f3 L, f3 H, float& pdf) {
    float HoL = clampf(1.0e-8f, 1.0f, dot(H, L));
    Col F(full_fresnel_dielectric(HoL, inc_ior, mat_ior));
    return torrance_sparrow1(c, roughness, aniso, F, V, L, H, pdf);
}
inline f3 GGX_VNDF_sample(f3 V, float ax, float ay, Rng& rng) {
    float r1 = rng(), r2 = rng();
    f3 Vh = normalize(mk3(ax * V.x, ay * V.y, V.z));
    float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    f3 T1 = lensq > 0.0f ? mk3(-Vh.y, Vh.x, 0.0f) / psqrt(lensq) : mk3(1.0f, 0.0f, 0.0f);
    f3 T2 = cross(Vh, T1);
    float r = psqrt(r1);
    float phi = TWO_PI * r2;
    float t1 = r * pcos(phi), t2 = r * psin(phi);
    float s = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - s) * psqrt(1.0f - t1 * t1) + s * t2;
    f3 Nh = t1 * T1 + t2 * T2 + psqrt(fmaxr(0.0f, 1.0f - t1 * t1 - t2 * t2)) * Vh;
    return normalize(mk3(ax * Nh.x, ay * Nh.y, fmaxr(0.0f, Nh.z)));
}
inline f3 ggx_sample_reflection(float roughness, float aniso, f3 V, Rng& rng) {
    int below = V.z < 0 ? -1 : 1;
    float ax, ay;
    get_alphas(roughness, aniso, ax, ay);
    f3 m = GGX_VNDF_sample(V * (float)below, ax, ay, rng);
    f3 d = reflect_ray(V, m * (float)below);
    return normalize(d);
}

// --------------------------------------------------------------------------------
// Energy compensation (MicrofacetEnergyCompensation.h:87-705, PrincipledEnergyCompensation.h)
// --------------------------------------------------------------------------------
// GGX_glass_energy_conservation_get_correction_exponent (MicrofacetEnergyCompensation.h:87-640)
// restated as knot tables: value of the correction at roughness 0, 0.1, ..., 1.0 for each
// relative-eta bound; a segment whose two knots are equal is the constant itself.
static const float kEtaBounds[10] = {1.01f, 1.02f, 1.03f, 1.1f, 1.2f, 1.4f, 1.5f, 2.0f, 2.4f, 3.0f};
static const float kCorr[10][11] = {
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
static const float kRough[11] = {0.0f, 0.1f, 0.2f, 0.3f, 0.4f, 0.5f, 0.6f, 0.7f, 0.8f, 0.9f, 1.0f};
inline float corr_knots(int b, float r) {
    if (r <= 0.0f) return 2.5f;
    for (int k = 1; k <= 10; k++) {
        if (r <= kRough[k]) {
            float a = kCorr[b][k - 1], c = kCorr[b][k];
            if (a == c) return a;
            return lerpf(a, c, (r - kRough[k - 1]) / 0.1f);
        }
    }
    return 2.5f;  // roughness > 1: uninitialised in the reference
}
inline float glass_correction_exponent(float roughness, float eta) {
    if (is_zero(roughness) || absf(1.0f - eta) < 1.0e-3f) return 2.5f;
    // higher bound: first bound >= eta (or 3.0 when eta > 2.4)
    int hi = 9;
    for (int i = 0; i < 9; i++) if (eta <= kEtaBounds[i]) { hi = i; break; }
    float hb = kEtaBounds[hi], hc = corr_knots(hi, roughness);
    // lower bound: band (b_i, b_{i+1}] -> b_i.  Undefined in the reference for
    // eta <= 1.01 or eta > 3.0 (uninitialised locals); we use the higher knot there.
    int lo = -1;
    for (int i = 0; i < 9; i++) if (eta > kEtaBounds[i] && eta <= kEtaBounds[i + 1]) { lo = i; break; }
    float lb, lc;
    if (lo < 0) { lb = hb - 1.0f; lc = hc; }
    else { lb = kEtaBounds[lo]; lc = corr_knots(lo, roughness); }
    return lerpf(lc, hc, (eta - lb) / (hb - lb));
}
inline float ggx_dielectric_compensation(const BsdfCtx& c, const Material& m, const VolumeState& vs, float eta_t, float eta_i, float rel_eta, float NoV) {
    float comp = 1.0f;
    if (m.thin_film < 1.0f) {   // PrincipledBSDFEnforceStrongEnergyConservation == false
        bool inside = vs.inside_material;
        float rel = inside ? 1.0f / rel_eta : rel_eta;
        float expo = 2.5f;
        if (!m.thin_walled) expo = glass_correction_exponent(m.roughness, rel);
        float fetch = ppow(fmaxr(1.0e-3f, NoV), 1.0f / expo);
        float F0 = F0_from_eta(eta_t, eta_i);
        float F0r = psqrt(psqrt(F0));
        if (!m.thin_walled)
            comp = lut3d(inside ? c.luts.glass_inv : c.luts.glass, 256, 16, 128, fetch, m.roughness, F0r);
        else
            comp = lut3d(c.luts.thin_glass, 32, 32, 96, fetch, m.roughness, F0r);
        comp = lerpf(comp, 1.0f, m.thin_film * m.roughness);
    }
    return comp;
}
inline float principled_specular_relative_ior(const Material& m, float inc_ior) {
    float layer = lerpf(inc_ior, m.coat_ior, m.coat);
    float rel = m.ior / layer;
    if (rel < 1.0f) rel = 1.0f / rel;
    return rel;
}
inline float glossy_base_compensation(const BsdfCtx& c, const Material& m, float inc_ior, float NoV) {
    float rel = principled_specular_relative_ior(m, inc_ior);
    if (absf(rel - 1.0f) < 1.0e-3f) rel += 1.0e-3f;
    float vr = ppow(NoV, 1.0f / 2.5f);
    float F0r = psqrt(psqrt(F0_from_eta(m.ior, m.ior / rel)));
    float ms = lut3d(c.luts.glossy, 128, 64, 128, vr, m.roughness, F0r);
    ms = lerpf(1.0f, ms, m.specular);
    ms = lerpf(ms, 1.0f, m.thin_film);
    return ms;
}
inline float clearcoat_compensation(const BsdfCtx& c, const Material& m, float inc_ior, float NoV) {
    if (m.coat == 0.0f) return 1.0f;
    if (absf(m.coat_ior / inc_ior - 1.0f) < 1.0e-3f) inc_ior += 1.0e-3f;
    float vr = ppow(NoV, 1.0f / 2.5f);
    float F0r = psqrt(psqrt(F0_from_eta(m.coat_ior, inc_ior)));
    float ms = lut3d(c.luts.glossy, 128, 64, 128, vr, m.coat_roughness, F0r);
    ms = lerpf(1.0f, ms, m.coat * (1.0f - m.specular_transmission));
    ms = lerpf(ms, 1.0f, m.thin_film);
    return ms;
}

// --------------------------------------------------------------------------------
// Sheen LTC (SheenLTC.h)
// --------------------------------------------------------------------------------
inline Col read_ltc(const BsdfCtx& c, float roughness, float cos_theta) {
    float u = wrap01(cos_theta, cos_theta), v = wrap01(1.0f - roughness, 1.0f - roughness);
    v = 1.0f - v;
    int x = (int)(u * 31.0f), y = (int)(v * 31.0f);
    const float* p = c.luts.sheen + (x + y * 32) * 3;
    return Col(p[0], p[1], p[2]);
}
inline float get_phi(f3 d) { float p = patan2(d.y, d.x); if (p < 0.0f) p += TWO_PI; return p; }
inline f3 rotate_vector(f3 v, f3 axis, float angle) {
    float s = psin(angle), co = pcos(angle);
    return v * co + axis * dot(v, axis) * (1.0f - co) + s * cross(axis, v);
}
inline float eval_ltc(f3 L, Col A) {
    f3 lo = mk3(L.x * A.r + L.z * A.g, L.y * A.r, L.z);
    float len = length(lo);
    lo = lo / len;
    float det = A.r * A.r;
    float jac = det / (len * len * len);
    return lo.z * INV_PI * jac;
}
inline Col sheen_eval(const BsdfCtx& c, const Material& m, f3 L, f3 V, float& pdf, float& refl) {
    if (V.z <= 0.0f || L.z <= 0.0f) {
        pdf = 0.0f;
        refl = V.z > 0.0f ? read_ltc(c, m.sheen_roughness, V.z).b : 0.0f;
        return Col(0.0f);
    }
    float phi = get_phi(V);
    f3 Ls = rotate_vector(L, mk3(0.0f, 0.0f, 1.0f), -phi);
    Col A = read_ltc(c, m.sheen_roughness, V.z);
    float Do = eval_ltc(Ls, A);
    pdf = Do;
    refl = A.b;
    return Col(m.sheen_color.r, m.sheen_color.g, m.sheen_color.b) * A.b * Do / L.z;
}
inline f3 sheen_sample(const BsdfCtx& c, const Material& m, f3 V, Rng& rng) {
    f3 cs = cosine_weighted_sample_z_up_frame(rng);
    Col A = read_ltc(c, m.sheen_roughness, V.z);
    float ai = 1.0f / A.r, bi = A.g;
    f3 d = normalize(mk3(cs.x * ai - cs.z * bi * ai, cs.y * ai, cs.z));
    return rotate_vector(d, mk3(0.0f, 0.0f, 1.0f), get_phi(V));
}

// --------------------------------------------------------------------------------
// Principled BSDF (Principled.h)
// --------------------------------------------------------------------------------
inline Col C3(MptColor c) { return Col(c.r, c.g, c.b); }

inline float thin_walled_roughness(bool thin, float r, float eta) {    // Material.h:86-110
    if (!thin) return r;
    float rem = r * psqrt(3.7f * (eta - 1.0f) * sq(eta - 0.5f) / pow3(eta));
    return clampf(0.0f, 1.0f, rem / 1.39f);
}

inline Col principled_specular_fresnel(const Material& m, float rel_ior, float cos_i) {
    float above = m.ior / rel_ior;
    Col Fs, Ft;
    if (m.thin_film < 1.0f) Fs = Col(full_fresnel_dielectric(cos_i, rel_ior));
    if (m.thin_film > 0.0f) Ft = thin_film_fresnel(m, above, cos_i);
    return lerpc(Fs, Ft, m.thin_film);
}

inline float mat_ior_or_air(const BsdfCtx& c, int idx) { return idx == MAX_MATERIAL_INDEX ? 1.0f : c.materials[idx].ior; }

inline Col glass_eval(const BsdfCtx& c, const Material& m, VolumeState& vs, f3 V, f3 L, float& pdf) {
    pdf = 0.0f;
    float NoV = V.z, NoL = L.z;
    if (absf(NoL) < 1.0e-8f) return Col(0.0f);
    bool reflecting = NoL * NoV > 0;
    float eta_i = mat_ior_or_air(c, vs.incident_mat_index);
    float eta_t = mat_ior_or_air(c, vs.outgoing_mat_index);
    eta_i = compute_dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, eta_i, absf(vs.sampled_wavelength));
    eta_t = compute_dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, eta_t, absf(vs.sampled_wavelength));
    float rel = eta_t / eta_i;
    if (absf(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    f3 H;
    if (reflecting) H = L + V;
    else if (m.thin_walled) H = L * mk3(1.0f, 1.0f, -1.0f) + V;
    else H = L * rel + V;
    H = normalize(H);
    if (H.z < 0.0f) H = -H;
    float HoL = dot(L, H), HoV = dot(V, H);
    if (HoL * NoL < 0.0f || HoV * NoV < 0.0f) return Col(0.0f);
    float comp = ggx_dielectric_compensation(c, m, vs, eta_t, eta_i, rel, V.z);
    Col Ft, Fn;
    if (m.thin_film > 0.0f) Ft = thin_film_fresnel(m, eta_i, HoV);
    if (m.thin_film < 1.0f) Fn = Col(full_fresnel_dielectric(HoV, rel));
    Col F = lerpc(Fn, Ft, m.thin_film);
    float frp = F.luminance();
    float roughness = thin_walled_roughness(m.thin_walled, m.roughness, rel);
    if (frp < 1.0f && m.thin_film == 0.0f && m.thin_walled && roughness < 0.1f)
        frp += sq(1.0f - frp) * frp / (1.0f - sq(frp));
    Col color;
    if (reflecting) {
        color = torrance_sparrow0(c, roughness, m.anisotropy, F, V, L, H, pdf);
        color /= comp;
        pdf *= frp;
    } else {
        float dp = HoL + HoV / rel;
        float dp2 = dp * dp;
        float denom = dp2 * NoL * NoV;
        float ax, ay;
        get_alphas(roughness, m.anisotropy, ax, ay);
        float D = GGX_anisotropic(ax, ay, H);
        float G1V = G1_Smith(ax, ay, V);
        float G1L = G1_Smith(ax, ay, L);
        float G2 = G1V * G1L;
        float dwm = absf(HoL) / dp2;
        float Dpdf = G1V / absf(NoV) * D * absf(HoV);
        pdf = dwm * Dpdf;
        pdf *= 1.0f - frp;
        color = C3(m.base_color) * D * (Col(1.0f) - F) * G2 * absf(HoL * HoV / denom);
        if (m.thin_walled) color *= C3(m.base_color);
        color /= comp;
        if (m.thin_walled) vs.interior_stack.pop(vs.inside_material);
        else if (vs.incident_mat_index != MAX_MATERIAL_INDEX) {
            const Material& im = c.materials[vs.incident_mat_index];
            if (!C3(im.absorption_color).is_white()) {
                Col coef = clog(C3(im.absorption_color)) / im.absorption_at_distance;
                color = color * cexp(coef * vs.distance_in_volume);
            }
            vs.distance_in_volume = 0.0f;
            if (vs.inside_material) vs.interior_stack.pop(vs.inside_material);
        }
    }
    return color;
}

inline f3 glass_sample(const BsdfCtx& c, const Material& m, VolumeState& vs, f3 V, Rng& rng) {
    float eta_i = mat_ior_or_air(c, vs.incident_mat_index);
    float eta_t = mat_ior_or_air(c, vs.outgoing_mat_index);
    eta_i = compute_dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, eta_i, absf(vs.sampled_wavelength));
    eta_t = compute_dispersion_ior(m.dispersion_abbe_number, m.dispersion_scale, eta_t, absf(vs.sampled_wavelength));
    float rel = eta_t / eta_i;
    if (absf(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    float roughness = thin_walled_roughness(m.thin_walled, m.roughness, rel);
    float ax, ay;
    get_alphas(roughness, m.anisotropy, ax, ay);
    f3 mn = GGX_VNDF_sample(V, ax, ay, rng);
    float HoV = dot(V, mn);
    Col Ft, Fn;
    if (m.thin_film > 0.0f) Ft = thin_film_fresnel(m, eta_i, HoV);
    if (m.thin_film < 1.0f) Fn = Col(full_fresnel_dielectric(HoV, rel));
    Col F = lerpc(Fn, Ft, m.thin_film);
    float frp = F.luminance();
    if (frp < 1.0f && m.thin_film == 0.0f && m.thin_walled && roughness < 0.1f)
        frp += sq(1.0f - frp) * frp / (1.0f - sq(frp));
    float r1 = rng();
    f3 dir = mk3(0.0f, 0.0f, 0.0f);   // uninitialised in the reference when refraction fails (TIR)
    if (r1 < frp) {
        dir = reflect_ray(V, mn);
        vs.interior_stack.pop(false);
    } else {
        if (dot(mn, V) < 0.0f) mn = -mn;
        if (m.thin_walled) {
            f3 r = reflect_ray(V, mn);
            r.z *= -1.0f;
            vs.interior_stack.pop(false);
            return r;
        }
        refract_ray(V, mn, dir, rel);
    }
    return dir;
}

inline Col coat_darkening(const Material& m, float rel_eta, float vdf) {
    if (m.coat_darkening == 0.0f) return Col(1.0f);
    float Kr = 1.0f - (1.0f - fresnel_hemispherical_albedo(rel_eta)) / (rel_eta * rel_eta);
    float Ks = vdf;
    float K = lerpf(Ks, Kr, m.roughness);
    Col base_albedo = (C3(m.base_color) + C3(m.sheen_color) * m.sheen) / (1.0f + m.sheen);
    Col dk = (1.0f - K) / (Col(1.0f) - base_albedo * K);
    return lerpc(Col(1.0f), dk, m.coat * m.coat_darkening);
}
inline Col specular_darkening(const Material& m, float rel_eta, float vdf) {
    if (m.specular_darkening == 0.0f) return Col(1.0f);
    float Kr = 1.0f - (1.0f - fresnel_hemispherical_albedo(rel_eta)) / (rel_eta * rel_eta);
    float K = Kr;
    (void)vdf;
    Col dk = (1.0f - K) / (Col(1.0f) - C3(m.base_color) * K);
    return lerpc(Col(1.0f), dk, m.specular * m.specular_darkening);
}

inline Col eval_coat_layer(const BsdfCtx& c, const Material& m, f3 V, f3 L, f3 H, float inc_ior, float w, bool refracting, float proba, Col& thr, float& pdf) {
    if (w > 0.0f || refracting) {
        float cp = 0.0f;
        Col contrib;
        if (!refracting) {
            contrib = torrance_sparrow_dielectric(c, m.coat_roughness, m.coat_anisotropy, m.coat_ior, inc_ior, V, L, H, cp);
            contrib *= w;
            contrib *= thr;
        }
        pdf += cp * proba;
        Col att(1.0f);
        att *= 1.0f - full_fresnel_dielectric(absf(L.z), inc_ior, m.coat_ior);
        float vdf = full_fresnel_dielectric(absf(V.z), inc_ior, m.coat_ior);
        att *= 1.0f - vdf;
        if (!C3(m.coat_medium_absorption).is_white()) {
            float ia = fmaxr(1.0e-6f, psqrt(1.0f - (1.0f - L.z * L.z) / (m.coat_ior * m.coat_ior)));
            float oa = fmaxr(1.0e-6f, psqrt(1.0f - (1.0f - V.z * V.z) / (m.coat_ior * m.coat_ior)));
            float tda = 1.0f / ia + 1.0f / oa;
            Col ca = cexp(-(Col(1.0f) - cpow(csqrt(C3(m.coat_medium_absorption)), tda)) * m.coat_medium_thickness);
            att *= ca;
        }
        att *= coat_darkening(m, m.coat_ior / inc_ior, vdf);
        att = lerpc(Col(1.0f), att, m.coat);
        thr *= att;
        return contrib;
    }
    return Col(0.0f);
}
inline Col eval_sheen_layer(const BsdfCtx& c, const Material& m, f3 V, f3 L, float w, float proba, Col& thr, float& pdf) {
    if (w > 0.0f) {
        float refl, sp;
        Col contrib = sheen_eval(c, m, L, V, sp, refl);
        contrib *= w;
        contrib *= thr;
        pdf += sp * proba;
        thr *= 1.0f - m.sheen * refl;
        return contrib;
    }
    return Col(0.0f);
}
inline Col eval_metal_layer(const BsdfCtx& c, const Material& m, f3 V, f3 L, f3 H, float roughness, float aniso, float inc_ior, float w, float proba, Col& thr, float& pdf) {
    if (w > 0.0f) {
        float mp;
        float HoL = clampf(1.0e-8f, 1.0f, dot(H, L));
        Col Fm = adobe_f82_tint_fresnel(C3(m.base_color), C3(m.metallic_F82), C3(m.metallic_F90), m.metallic_F90_falloff_exponent, HoL);
        Col Ft = thin_film_fresnel(m, inc_ior, HoL);
        Col F = lerpc(Fm, Ft, m.thin_film);
        Col contrib = torrance_sparrow1(c, roughness, aniso, F, V, L, H, mp);
        contrib *= w;
        contrib *= thr;
        pdf += mp * proba;
        return contrib;
    }
    return Col(0.0f);
}
inline Col eval_glass_layer(const BsdfCtx& c, const Material& m, VolumeState& vs, f3 V, f3 L, float w, float proba, Col& thr, float& pdf) {
    if (w > 0.0f) {
        float gp;
        Col contrib = glass_eval(c, m, vs, V, L, gp);
        contrib *= w;
        contrib *= thr;
        pdf += gp * proba;
        return contrib;
    }
    return Col(0.0f);
}
inline Col eval_specular_layer(const BsdfCtx& c, const Material& m, f3 V, f3 L, f3 H, float inc_ior, float w, float proba, Col& thr, float& pdf) {
    if (w > 0.0f) {
        float rel = principled_specular_relative_ior(m, inc_ior);
        float sp;
        Col F = principled_specular_fresnel(m, rel, dot(L, H));
        Col contrib = torrance_sparrow0(c, m.roughness, m.anisotropy, F, V, L, H, sp);
        if (absf(rel - 1.0f) > 1.0e-3f) {
            contrib *= lerpc(Col(1.0f), m.specular_tint * C3(m.specular_color), m.specular);
            contrib *= w;
            contrib *= thr;
            Col att(1.0f);
            att *= Col(1.0f) - principled_specular_fresnel(m, rel, L.z);
            Col vdf = principled_specular_fresnel(m, rel, V.z);
            att *= Col(1.0f) - vdf;
            att *= specular_darkening(m, rel, vdf.luminance());
            att = lerpc(Col(1.0f), att, m.specular);
            thr *= att;
        }
        pdf += sp * proba;
        return contrib;
    }
    return Col(0.0f);
}
inline Col eval_diffuse_layer(const Material& m, f3 L, float w, float proba, Col& thr, float& pdf) {
    if (w > 0.0f) {
        float dp;
        Col contrib = lambertian_eval(m, L.z, dp);   // PRINCIPLED_DIFFUSE_LOBE_LAMBERTIAN
        contrib *= w;
        contrib *= thr;
        pdf += dp * proba;
        return contrib;
    }
    return Col(0.0f);
}

inline void lobe_weights(const Material& m, bool outside, float w[7]) {
    float o = outside ? 1.0f : 0.0f;
    w[0] = m.coat * o;
    w[1] = m.sheen * o;
    w[2] = m.metallic * o;
    w[3] = m.metallic * o;
    w[2] = lerpf(w[2], 0.0f, m.second_roughness_weight);
    w[3] = lerpf(0.0f, w[3], m.second_roughness_weight);
    w[4] = (1.0f - m.metallic) * (1.0f - m.specular_transmission) * m.specular * o;
    w[5] = (1.0f - m.metallic) * (1.0f - m.specular_transmission) * o;
    w[6] = !outside ? 1.0f : (1.0f - m.metallic) * m.specular_transmission;
}
inline void lobe_probas(const float w[7], float p[7]) {
    float nf = 1.0f / (w[0] + w[1] + w[2] + w[3] + w[4] + w[5] + w[6]);
    for (int i = 0; i < 7; i++) p[i] = w[i] * nf;
}

inline Col principled_eval(const BsdfCtx& c, const Material& m, VolumeState& vs, f3 view, f3 n, f3 L, float& pdf) {
    pdf = 0.0f;
    bool outside = dot(view, n) > 0 || m.thin_walled;
    bool refracting = dot(n, L) < 0.0f && outside;
    if (dot(view, n) < 0.0f) n = -n;
    f3 T, B;
    build_onb(n, T, B);
    f3 lv = world_to_local(T, B, n, view), ll = world_to_local(T, B, n, L);
    f3 lh = normalize(lv + ll);
    f3 TR, BR;
    build_rotated_onb(n, TR, BR, m.anisotropy_rotation * PI);
    f3 lvr = world_to_local(TR, BR, n, view), llr = world_to_local(TR, BR, n, L);
    f3 lhr = normalize(lvr + llr);
    float w[7], p[7];
    lobe_weights(m, outside, w);
    float inc_ior = mat_ior_or_air(c, vs.incident_mat_index);
    lobe_probas(w, p);
    Col thr(1.0f), fc(0.0f);
    float nr = refracting ? 0.0f : 1.0f;
    fc += eval_coat_layer(c, m, lv, ll, lh, inc_ior, w[0], refracting, p[0], thr, pdf);
    fc += eval_sheen_layer(c, m, lv, ll, w[1], p[1], thr, pdf);
    fc += eval_metal_layer(c, m, lvr, llr, lhr, m.roughness, m.anisotropy, inc_ior, w[2] * nr, p[2], thr, pdf);
    fc += eval_metal_layer(c, m, lvr, llr, lhr, m.second_roughness, m.anisotropy, inc_ior, w[3] * nr, p[3], thr, pdf);
    fc += eval_glass_layer(c, m, vs, lvr, llr, w[6], p[6], thr, pdf);
    {   // internal_eval_glossy_base (Principled.h:842-861)
        Col g(0.0f);
        g += eval_specular_layer(c, m, lvr, llr, lhr, inc_ior, w[4] * nr, p[4], thr, pdf);
        g += eval_diffuse_layer(m, ll, w[5] * nr, p[5], thr, pdf);
        float gc = glossy_base_compensation(c, m, inc_ior, lv.z);
        fc += g / gc;
    }
    if (c.clearcoat_compensation) fc /= clearcoat_compensation(c, m, inc_ior, lv.z);
    return fc;
}

inline Col principled_sample(const BsdfCtx& c, const Material& m, VolumeState& vs, f3 view, f3 sn, f3 gn, f3& out, float& pdf, Rng& rng) {
    pdf = 0.0f;
    f3 n = sn;
    // principled_bsdf_get_lobes_weights_fringe_fix (Principled.h:905-949)
    bool outside = dot(view, n) > 0 || m.thin_walled;
    float glass_w = (1.0f - m.metallic) * m.specular_transmission;
    if (is_zero(glass_w) && !outside) { n = reflect_ray(sn, gn); outside = true; }
    float w[7], p[7];
    lobe_weights(m, outside, w);
    if (!outside) w[6] = 1.0f;
    lobe_probas(w, p);
    float cdf[6];
    cdf[0] = p[0];
    cdf[1] = cdf[0] + p[1];
    cdf[2] = cdf[1] + p[2];
    cdf[3] = cdf[2] + p[3];
    cdf[4] = cdf[3] + p[4];
    cdf[5] = cdf[4] + p[5];
    float r1 = rng();
    bool glass = r1 > cdf[5];
    if (glass) {
        float ds = dot(view, sn), dg = dot(view, gn);
        if (ds * dg < 0) n = reflect_ray(sn, gn);
    }
    if (!glass) vs.interior_stack.pop(false);
    if (dot(view, n) < 0) n = -n;
    f3 TR, BR;
    build_rotated_onb(n, TR, BR, m.anisotropy_rotation * PI);
    f3 lvr = world_to_local(TR, BR, n, view);
    if (r1 < cdf[0]) {
        f3 TRc, BRc;
        build_rotated_onb(n, TRc, BRc, m.coat_anisotropy_rotation * PI);
        f3 lvc = world_to_local(TRc, BRc, n, view);
        out = local_to_world(TRc, BRc, n, ggx_sample_reflection(m.coat_roughness, m.coat_anisotropy, lvc, rng));
    } else if (r1 < cdf[1]) {
        f3 T, B;
        build_onb(n, T, B);
        f3 lv = world_to_local(T, B, n, view);
        out = local_to_world(T, B, n, sheen_sample(c, m, lv, rng));
    } else if (r1 < cdf[2]) {
        out = local_to_world(TR, BR, n, ggx_sample_reflection(m.roughness, m.anisotropy, lvr, rng));
    } else if (r1 < cdf[3]) {
        out = local_to_world(TR, BR, n, ggx_sample_reflection(m.second_roughness, m.anisotropy, lvr, rng));
    } else if (r1 < cdf[4]) {
        out = local_to_world(TR, BR, n, ggx_sample_reflection(m.roughness, m.anisotropy, lvr, rng));
    } else if (r1 < cdf[5]) {
        out = cosine_weighted_sample_around_normal(n, rng);
    } else {
        out = local_to_world(TR, BR, n, glass_sample(c, m, vs, lvr, rng));
    }
    if (dot(out, sn) < 0 && !glass) return Col(0.0f);
    return principled_eval(c, m, vs, view, sn, out, pdf);
}

// bsdf_dispatcher_eval / _sample (Dispatcher.h:18-68)
inline Col bsdf_eval(const BsdfCtx& c, int override_, const Material& m, VolumeState& vs, f3 view, f3 sn, f3 gn, f3 L, float& pdf) {
    (void)gn;
    if (override_ == MPT_BSDF_LAMBERTIAN) return lambertian_eval(m, dot(L, sn), pdf);
    if (override_ == MPT_BSDF_OREN_NAYAR) return oren_nayar_eval(m, view, sn, L, pdf);
    return principled_eval(c, m, vs, view, sn, L, pdf);
}
inline Col bsdf_sample(const BsdfCtx& c, int override_, const Material& m, VolumeState& vs, f3 view, f3 sn, f3 gn, f3& dir, float& pdf, Rng& rng) {
    if (override_ == MPT_BSDF_LAMBERTIAN) return lambertian_sample(m, sn, dir, pdf, rng);
    if (override_ == MPT_BSDF_OREN_NAYAR) return oren_nayar_sample(m, view, sn, dir, pdf, rng);
    return principled_sample(c, m, vs, view, sn, gn, dir, pdf, rng);
}

}  // namespace orc
#endif
