// mpt_part.hip -- the large kernel instantiations of mpt_kernels.hip, one group per
// translation unit: the build compiles this file once per MPT_TU_PART value (mpt/_build.py)
// so that the shading and ReSTIR DI kernels compile in parallel.  mpt_kernels.hip's host glue
// launches them through these functions.
#ifndef MPT_TU_PART
#error "compile with -DMPT_TU_PART=<1..7>"
#endif
#include "mpt_kernels.hip"

namespace mpt {

#if MPT_TU_PART == 1
void part_shade_generic(dim3 g, hipStream_t st, const ShadeArgs& a) {
    if (a.mat_private) hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, false, false, false, SG_ALL, true>), g, dim3(TB), 0, st, a);
    else hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, false>), g, dim3(TB), 0, st, a);
}
#elif MPT_TU_PART == 2
void part_shade_plain(dim3 g, hipStream_t st, const ShadeArgs& a) {
    if (a.mat_private) hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_ALL, true>), g, dim3(TB), 0, st, a);
    else hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true>), g, dim3(TB), 0, st, a);
}
#ifdef MPT_SECTION_TIMING
extern "C" int mpt_debug_sections(unsigned long long* out, int reset) {   // k_shade<NONE, true>'s section clocks
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sect), sizeof(unsigned long long) * 8);
    if (reset) { unsigned long long z[8] = {0}; hipMemcpyToSymbol(HIP_SYMBOL(g_sect), z, sizeof(z)); }
    return 0;
}
#endif
#elif MPT_TU_PART == 7
// the plain class shaded in stages (k_shade's ST: SG_* groups; LaunchCfg::shade_split)
void part_shade_plain_stage(int stage, dim3 g, hipStream_t st, const ShadeArgs& a) {
    switch (stage) {
    case SG_LIGHT: hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_LIGHT>), g, dim3(TB), 0, st, a); break;
    case SG_ENV: hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_ENV>), g, dim3(TB), 0, st, a); break;
    case SG_CONT: hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_CONT>), g, dim3(TB), 0, st, a); break;
    case SG_LIGHT | SG_ENV:
        hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_LIGHT | SG_ENV>), g, dim3(TB), 0, st, a);
        break;
    default: hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, true, false, false, SG_ENV | SG_CONT>), g, dim3(TB), 0, st, a); break;
    }
}
#elif MPT_TU_PART == 3
void part_shade_ext(dim3 g, hipStream_t st, const ShadeArgs& a) {
    hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, false, true>), g, dim3(TB), 0, st, a);
}
void part_shade_glass(dim3 g, hipStream_t st, const ShadeArgs& a) {
    hipLaunchKernelGGL((k_shade<MPT_BSDF_NONE, false, false, true>), g, dim3(TB), 0, st, a);
}
#elif MPT_TU_PART == 4
void part_shade_override(int ovr, bool ext, dim3 g, hipStream_t st, const ShadeArgs& a) {
    if (ovr == MPT_BSDF_LAMBERTIAN) {
        if (ext) hipLaunchKernelGGL((k_shade<MPT_BSDF_LAMBERTIAN, false, true>), g, dim3(TB), 0, st, a);
        else hipLaunchKernelGGL((k_shade<MPT_BSDF_LAMBERTIAN, false>), g, dim3(TB), 0, st, a);
    } else {
        if (ext) hipLaunchKernelGGL((k_shade<MPT_BSDF_OREN_NAYAR, false, true>), g, dim3(TB), 0, st, a);
        else hipLaunchKernelGGL((k_shade<MPT_BSDF_OREN_NAYAR, false>), g, dim3(TB), 0, st, a);
    }
}
#elif MPT_TU_PART == 5 || MPT_TU_PART == 6
// ReSTIR DI reuse kernels of one BSDF override (5: Principled, 6: Lambert + Oren-Nayar); the
// reference-default bias correction (pairwise MIS defensive with visibility) has its own
// variant with the mode compiled in, the others read it from the frame (-1)
template <int OVR>
static void restir_kernel(int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P, const MptFrame* F, int pass,
                          const float4* in, float4* out) {
    constexpr int DEF = MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE;
    switch (kind) {
    case RK_INITIAL: hipLaunchKernelGGL((k_restir_initial<OVR, false>), g, dim3(TB), 0, st, S, P, F, nullptr, nullptr); break;
    // staged initial candidates over k_rsi_classify's lists (the plain class: Principled only)
    case RK_INITIAL_STAGED_PLAIN:
        if (OVR == MPT_BSDF_NONE)
            hipLaunchKernelGGL((k_restir_initial<OVR, true, true>), g, dim3(TB), 0, st, S, P, F, P.rq_items, &P.counters[CTR_RQE0]);
        break;
    case RK_INITIAL_STAGED_GENERIC:
        hipLaunchKernelGGL((k_restir_initial<OVR, true, false>), g, dim3(TB), 0, st, S, P, F, P.rq_items + P.n,
                           &P.counters[CTR_RQE1]);
        break;
    case RK_SPATIOTEMPORAL: hipLaunchKernelGGL((k_restir_spatiotemporal<OVR, DEF>), g, dim3(TB), 0, st, S, P, F); break;
    case RK_SPATIOTEMPORAL_ANY: hipLaunchKernelGGL((k_restir_spatiotemporal<OVR, -1>), g, dim3(TB), 0, st, S, P, F); break;
    case RK_SPATIAL:
        hipLaunchKernelGGL((k_restir_spatial<OVR, DEF>), g, dim3(TB), 0, st, S, P, F, pass, in, out);
        break;
    case RK_SPATIAL_ANY:
        hipLaunchKernelGGL((k_restir_spatial<OVR, -1>), g, dim3(TB), 0, st, S, P, F, pass, in, out);
        break;
    // the staged spatial pass (restir_di.h): selection, class-sorted evaluations, combine
    case RK_SP_SELECT: hipLaunchKernelGGL(k_rsp_select<OVR>, g, dim3(TB), 0, st, S, P, F, pass, in); break;
    case RK_SP_EVAL_PLAIN:   // (only the Principled BSDF has the plain class)
        if (OVR == MPT_BSDF_NONE)
            hipLaunchKernelGGL((k_rsp_eval<OVR, true, false>), g, dim3(TB), 0, st, S, P, F, pass, in, P.rq_items, &P.counters[CTR_RQE0]);
        break;
    case RK_SP_EVAL_GENERIC:
        hipLaunchKernelGGL((k_rsp_eval<OVR, false, false>), g, dim3(TB), 0, st, S, P, F, pass, in, P.rq_items + (size_t)P.n * RS_RPP,
                           &P.counters[CTR_RQE1]);
        break;
    // the staged fused spatiotemporal pass: selection, class-sorted evaluations, combine
    case RK_ST_SELECT: hipLaunchKernelGGL(k_rst_select<OVR>, g, dim3(TB), 0, st, S, P, F); break;
    case RK_ST_EVAL_PLAIN:
        if (OVR == MPT_BSDF_NONE)
            hipLaunchKernelGGL((k_rsp_eval<OVR, true, true>), g, dim3(TB), 0, st, S, P, F, 0, P.rs_tin, P.rq_items,
                               &P.counters[CTR_RQE0]);
        break;
    case RK_ST_EVAL_GENERIC:
        hipLaunchKernelGGL((k_rsp_eval<OVR, false, true>), g, dim3(TB), 0, st, S, P, F, 0, P.rs_tin,
                           P.rq_items + (size_t)P.n * RS_RPP, &P.counters[CTR_RQE1]);
        break;
    case RK_ST_COMBINE: hipLaunchKernelGGL(k_rst_combine<OVR>, g, dim3(TB), 0, st, S, P, F); break;
    case RK_SP_COMBINE: hipLaunchKernelGGL(k_rsp_combine<OVR>, g, dim3(TB), 0, st, S, P, F, pass, in, out); break;
    default: hipLaunchKernelGGL(k_restir_temporal<OVR>, g, dim3(TB), 0, st, S, P, F, in, out); break;
    }
}
#if MPT_TU_PART == 5
void part_restir_principled(int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P, const MptFrame* F, int pass,
                            const float4* in, float4* out) {
    restir_kernel<MPT_BSDF_NONE>(kind, g, st, S, P, F, pass, in, out);
}
#else
void part_restir_override(int ovr, int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P, const MptFrame* F,
                          int pass, const float4* in, float4* out) {
    if (ovr == MPT_BSDF_LAMBERTIAN) restir_kernel<MPT_BSDF_LAMBERTIAN>(kind, g, st, S, P, F, pass, in, out);
    else restir_kernel<MPT_BSDF_OREN_NAYAR>(kind, g, st, S, P, F, pass, in, out);
}
#endif
#endif

}  // namespace mpt
