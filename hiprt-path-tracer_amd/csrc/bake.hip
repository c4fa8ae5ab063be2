// bake.hip -- the energy-compensation LUT baker on the GPU (the reference's GPUBaker:
// Renderer/Baker/GPUBaker.cpp:35-97, GPUBakerKernel.cpp:22-151, Device/kernels/Baking/*.h).
//
// Monte-Carlo directional albedo tables of the GGX lobes that the Principled BSDF's energy
// compensation reads (data/BRDFsData; dev_bsdf.h lut2d / lut3d).  One lane per texel.  The
// reference's launch structure is kept, because it defines the result: launches of `ipk`
// samples per texel (ipk = floor(max(1, 1e8 / texels))), launch i (1-based) reseeds the
// texel's RNG with wang_hash(texel + 1) * i, and every sample adds albedo / nb_samples to
// the texel (nb_samples as each kernel derives it -- the GGX Fresnel kernel from a 2-D
// texel count, kept).  The table is therefore a deterministic function of (kind, sizes,
// sample count), which the CPU oracle reproduces bit for bit (oracle_bake).  The sampling
// and evaluation routines are the path tracer's own (dev_bsdf.h), so the baked table is
// the one the renderer's BSDFs integrate to.
#include <hip/hip_runtime.h>

#include "dev_bsdf.h"
#include "mpt_internal.h"

namespace mpt {

constexpr float GGX_DOT_CLAMP = 1.0e-3f;   // GGX_DOT_PRODUCTS_CLAMP (Microfacet.h:20)

struct BakeTexel { v3 V; float roughness, rel_ior; };

// texel parameters (GGXConductorDirectionalAlbedo.h:49-56, GlossyDielectricDirectionalAlbedo.h:48-65,
// GGXGlassDirectionalAlbedo.h:163-184, GGXThinGlassDirectionalAlbedo.h:218-235, GGXFresnelDirectionalAlbedo.h:45-62)
DEV BakeTexel bake_texel(int kind, int w, int h, int d, int x, int y, int z) {
    BakeTexel t;
    float ct = 1.0f / (float)(w - 1) * (float)x;
    ct = maxr(GGX_DOT_CLAMP, ct);
    if (kind != MPT_BAKE_GGX_CONDUCTOR && kind != MPT_BAKE_GGX_THIN_GLASS) ct = ppow(ct, 2.5f);
    const float st = psin(pacos(ct));
    t.V = normalize(mk3(1.0f * st, 0.0f * st, ct));   // (cos 0 sin, sin 0 sin, cos)
    t.roughness = maxr(1.0f / (float)(h - 1) * (float)y, 1.0e-4f);
    t.rel_ior = 1.0f;
    if (kind != MPT_BAKE_GGX_CONDUCTOR) {
        float F0 = 1.0f / (float)(d - 1) * (float)z;
        F0 *= F0;
        F0 *= F0;
        const float s = sqrtf(clampr(0.0f, 0.99f, F0));
        t.rel_ior = (1.0f + s) / (1.0f - s);
        if (kind == MPT_BAKE_GGX_GLASS_INVERSE) t.rel_ior = 1.0f / t.rel_ior;
    }
    return t;
}

// GGX_glass_E_sample / thin_glass_sample (GGXGlassDirectionalAlbedo.h:124-157,
// GGXThinGlassDirectionalAlbedo.h:32-85)
DEV v3 bake_glass_sample(bool thin, float rel, float r, v3 V, Rng& rng) {
    if (absr(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    float ax, ay;
    alphas(r, 0.0f, ax, ay);
    v3 m = ggx_vndf(V, ax, ay, rng);
    float F = fresnel_dielectric(dot(V, m), rel);
    if (thin && r < 0.1f) F += sq(1.0f - F) * F / (1.0f - sq(F));
    const float r1 = rng();
    if (r1 < F) return reflect_ray(V, m);
    if (dot(m, V) < 0.0f) m = -m;
    if (thin) {
        v3 rr = reflect_ray(V, m);
        rr.z *= -1.0f;
        return rr;
    }
    v3 dir = mk3(0.0f, 0.0f, 0.0f);
    refract_ray(V, m, dir, rel);
    return dir;
}
// GGX_glass_E_eval / thin_glass_eval (GGXGlassDirectionalAlbedo.h:37-119, GGXThinGlassDirectionalAlbedo.h:87-197)
DEV float bake_glass_eval(const BCtx& bc, bool thin, float rel, float r, v3 V, v3 L, float& pdf) {
    pdf = 0.0f;
    const float NoV = V.z, NoL = L.z;
    if (absr(NoL) < 1.0e-8f) return 0.0f;
    const bool refl = NoL * NoV > 0;
    if (absr(rel - 1.0f) < 1.0e-5f) rel = 1.0f + 1.0e-5f;
    v3 H;
    if (refl) H = L + V;
    else if (thin) H = L * mk3(1.0f, 1.0f, -1.0f) + V;
    else H = L * rel + V;
    H = normalize(H);
    if (H.z < 0.0f) H = -H;
    const float HoL = dot(L, H), HoV = dot(V, H);
    if (HoL * NoL < 0.0f || HoV * NoV < 0.0f) return 0.0f;
    float F = fresnel_dielectric(thin ? HoV : dot(V, H), rel);
    if (thin && r < 0.1f) F += sq(1.0f - F) * F / (1.0f - sq(F));
    if (refl) {
        const float a = ts_ggx0(bc, r, 0.0f, col(F), V, L, H, pdf).r;
        pdf *= F;
        return a;
    }
    const float dp = HoL + HoV / rel;
    const float dp2 = dp * dp;
    const float denom = dp2 * NoL * NoV;
    float ax, ay;
    alphas(r, 0.0f, ax, ay);
    const float D = ggx_D(ax, ay, H);
    const float G1V = G1(ax, ay, V), G1L = G1(ax, ay, L);
    const float G2 = G1V * G1L;
    const float dwm_dwi = absr(HoL) / dp2;
    const float D_pdf = G1V / absr(NoV) * D * absr(HoV);
    pdf = dwm_dwi * D_pdf;
    pdf *= 1.0f - F;
    return D * (1.0f - F) * G2 * absr(HoL * HoV / denom);
}

// one launch of the reference's bake loop over all texels
template <int KIND>
__global__ __launch_bounds__(256) void k_bake(int w, int h, int d, int ipk, int nb_samples, int iteration, float* out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= w * h * d) return;
    const int x = idx % w, y = (idx / w) % h, z = idx / (w * h);
    const BakeTexel t = bake_texel(KIND, w, h, d, x, y, z);
    BCtx bc{};
    bc.masking = 0;   // HIPRTRenderData() default: height-correlated masking-shadowing (BSDFsData.h:62)
    Rng rng = make_rng(wang_hash((uint32_t)idx + 1u) * (uint32_t)iteration);
    const v3 V = t.V;
    const float r = t.roughness;
    float acc = out[idx];
    for (int s = 0; s < ipk; s++) {
        float a = 0.0f;
        if (KIND == MPT_BAKE_GGX_CONDUCTOR || KIND == MPT_BAKE_GGX_FRESNEL) {
            const v3 L = ggx_sample_reflection(r, 0.0f, V, rng);
            if (L.z < 0) continue;
            const Col F = col(KIND == MPT_BAKE_GGX_FRESNEL ? fresnel_dielectric(L.z, t.rel_ior) : 1.0f);
            float pdf;
            a = ts_ggx0(bc, r, 0.0f, F, V, L, normalize(V + L), pdf).r;
            a /= pdf;
            a *= L.z;
        } else if (KIND == MPT_BAKE_GLOSSY_DIELECTRIC) {
            const float lobe = rng();
            v3 L;
            if (lobe < 0.5f) {
                L = ggx_sample_reflection(r, 0.0f, V, rng);
                if (L.z < 0) continue;
            } else {
                L = cosine_sample_z_up(rng);
            }
            const v3 H = normalize(V + L);
            float total = 0.0f, ps;
            const float F = fresnel_dielectric(dot(H, L), t.rel_ior);
            const float spec = ts_ggx0(bc, r, 0.0f, col(F), V, L, H, ps).r;
            total += ps * 0.5f;
            float thr = 1.0f;
            thr *= 1.0f - fresnel_dielectric(L.z, t.rel_ior);
            thr *= 1.0f - fresnel_dielectric(V.z, t.rel_ior);
            float pd = 0.0f, diff = 0.0f;
            if (L.z > 0.0f) { pd = L.z * INV_PI; diff = 1.0f * INV_PI; }   // lambertian_brdf_eval, base colour 1
            total += pd * 0.5f;
            diff *= thr;
            a = spec + diff;
            a *= L.z;
            a /= total;
        } else {
            const bool thin = KIND == MPT_BAKE_GGX_THIN_GLASS;
            const float rt = thin ? thin_walled_roughness(true, r, t.rel_ior) : r;
            const v3 L = bake_glass_sample(thin, t.rel_ior, rt, V, rng);
            float pdf = 0.0f;
            a = bake_glass_eval(bc, thin, t.rel_ior, rt, V, L, pdf);
            if (pdf == 0.0f) continue;
            a /= pdf;
            a *= absr(L.z);
        }
        acc += a / (float)nb_samples;
    }
    out[idx] = acc;
}

hipError_t launch_bake(int kind, int w, int h, int d, int ipk, int nb_samples, int iteration, float* out, hipStream_t st) {
    const dim3 g((w * h * d + 255) / 256), b(256);
    switch (kind) {
        case MPT_BAKE_GGX_CONDUCTOR: hipLaunchKernelGGL(k_bake<MPT_BAKE_GGX_CONDUCTOR>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
        case MPT_BAKE_GGX_FRESNEL: hipLaunchKernelGGL(k_bake<MPT_BAKE_GGX_FRESNEL>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
        case MPT_BAKE_GLOSSY_DIELECTRIC: hipLaunchKernelGGL(k_bake<MPT_BAKE_GLOSSY_DIELECTRIC>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
        case MPT_BAKE_GGX_GLASS: hipLaunchKernelGGL(k_bake<MPT_BAKE_GGX_GLASS>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
        case MPT_BAKE_GGX_GLASS_INVERSE: hipLaunchKernelGGL(k_bake<MPT_BAKE_GGX_GLASS_INVERSE>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
        default: hipLaunchKernelGGL(k_bake<MPT_BAKE_GGX_THIN_GLASS>, g, b, 0, st, w, h, d, ipk, nb_samples, iteration, out); break;
    }
    return hipGetLastError();
}

}  // namespace mpt
