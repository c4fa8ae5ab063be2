// restir_di.h -- ReSTIR DI passes of the MI355X path (LSS_RESTIR_DI), included by
// mpt_kernels.hip after the light / envmap / traversal helpers.
//
// The reference's default kernel options (KernelOptions.h:270-366): lights presampling,
// no visibility in the initial target function, visibility in the spatial target
// function and the bias correction, visibility reuse, pairwise-MIS-defensive weights;
// ReSTIRDIRenderPass::launch (ReSTIRDIRenderPass.cpp:233-264) with the fused
// spatiotemporal pass followed by (number_of_passes - 1) spatial passes.
//
// MI355X mapping: one pass = one kernel over the pixels, persistent blocks of 256 lanes
// (grid = the traversal grid, so the per-lane traversal spill area is reused); visibility
// and BSDF rays are traced inline with the BVH8 traversal (LDS short stack), the passes
// being short compared with the path-tracing wavefront.  Reservoirs live in three
// ping-pong HBM buffers of 48 B per pixel (3 x float4), the G-buffer in SoA float4 arrays.

#ifndef MPT_RESTIR_WAVES
#define MPT_RESTIR_WAVES 2
#endif
// the plain-class target-function evaluations read surfaces from the compact per-pixel record
#ifndef MPT_RESTIR_CS
#define MPT_RESTIR_CS 1
#endif
#define RESTIR_KERNEL __global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(MPT_RESTIR_WAVES)))

// ---- surfaces (Surface.h:12-73) ----------------------------------------------------
__device__ MptMaterial g_zero_mat;   // the material of a never-written G-buffer entry (zero-initialised)

struct RSurf { const Mat* m; VState vs; int last; v3 view, sn, gn, sp, p; };
DEV RSurf gb_surface(const DevScene& S, const DevPaths& P, int i, bool prev) {
    int4 meta = prev ? P.pgb_meta[i] : P.gb_meta[i];
    float4 pos = prev ? P.pgb_pos[i] : P.gb_pos[i];
    float4 sn = prev ? P.pgb_sn[i] : P.gb_sn[i];
    float4 gn = prev ? P.pgb_gn[i] : P.gb_gn[i];
    float4 vw = prev ? P.pgb_view[i] : P.gb_view[i];
    RSurf s;
    if (meta.y == 0) s.m = &g_zero_mat;
    else if (meta.w) s.m = prev ? &P.pgb_mat[i] : &P.gb_mat[i];
    else s.m = &S.mats_res[meta.y - 1];
    s.vs = meta.y == 0 ? vs_default() : vs_load(prev ? P.pgb_vsA : P.gb_vsA, prev ? P.pgb_vsB : P.gb_vsB, i);
    s.last = meta.x;
    s.view = mk3(vw.x, vw.y, vw.z);
    s.sn = mk3(sn.x, sn.y, sn.z);
    s.gn = mk3(gn.x, gn.y, gn.z);
    s.p = mk3(pos.x, pos.y, pos.z);
    s.sp = s.p + s.sn * 1.0e-4f;
    return s;
}

// gb_surface from the compact record (DevPaths::gb_cs), for the plain-class evaluations:
// the same surface, with the nested-dielectric state reduced to the incident medium (all a
// plain-dielectric evaluation reads of it: principled_eval_pre's incident IOR)
DEV RSurf gb_csurf(const DevScene& S, const DevPaths& P, int i, bool prev) {
    const float4* cs = (prev ? P.pgb_cs : P.gb_cs) + 4 * (size_t)i;
    const float4 a = cs[0], b = cs[1], v = cs[2];
    const int mref = __float_as_int(a.w);   // material index + 1, negative: the per-pixel copy, 0: never written
    RSurf s;
    if (mref == 0) s.m = &g_zero_mat;
    else if (mref < 0) s.m = prev ? &P.pgb_mat[i] : &P.gb_mat[i];
    else s.m = &S.mats_res[mref - 1];
    s.vs = vs_default();
    if (mref != 0) s.vs.incident = __float_as_int(b.w);
    s.last = __float_as_int(v.w);
    s.view = mk3(v.x, v.y, v.z);
    s.sn = mk3(b.x, b.y, b.z);
    s.gn = mk3(0.0f, 0.0f, 0.0f);   // (not read by a plain evaluation; cs[3])
    s.p = mk3(a.x, a.y, a.z);
    s.sp = s.p + s.sn * 1.0e-4f;
    return s;
}

// XCD-aware block order for the passes that read neighbouring pixels: the hardware hands
// block b to XCD b % 8, so logical block (b % 8) * (G / 8) + b / 8 gives each XCD one
// contiguous run of rows, whose neighbours then stay in that XCD's L2 (the G % 8 tail
// blocks keep their index).  Measured on C4: k_rsp_select 0.78 -> 0.65 ms, k_rsp_combine
// 0.32 -> 0.27 ms; the evaluation kernels keep the append order (per-XCD item lists, tried
// with work stealing, were slower: the image regions differ in work).
DEV int xcd_block() {
    const int G = (int)gridDim.x, b = (int)blockIdx.x, per = G >> 3;
    return b < (per << 3) ? (b & 7) * per + (b >> 3) : b;
}

// ---- traced rays of a pass --------------------------------------------------------------
// Alpha keys (alpha_key: pass pixel seed, bounce 0, kind 5 + pass, position): the position
// names the ray's site in the pass, not its rank among the rays traced so far, so a key does
// not depend on which earlier rays were skipped and a pass can stage its rays (k_rsp_*).  The
// oracle (oracle_restir.h) uses the same positions.  The families occupy disjoint ranges for
// every configuration validate_frame accepts (<= 32 reuse neighbours, so cur, j <= 33 besides
// the 998 / 999 terms): [0, 68) neighbour pairs, 4000-4001 temporal pair, [100000, 134000)
// GBH terms, [200000, 201000) normalisation terms, 300000 visibility reuse, 1000000 + i / 2000000
// + i initial light / BSDF candidates.
DEV constexpr int RP_TFC(int k) { return 2 * k; }           // neighbour k's sample at the center
DEV constexpr int RP_TCN(int k) { return 2 * k + 1; }       // the canonical sample at neighbour k (pairwise MIS)
constexpr int RP_T_TFC = 4000, RP_T_TCN = 4001;             // the temporal neighbour's pair
DEV constexpr int RP_GBH(int cur, int j) { return 100000 + cur * 1000 + j; }   // j = 999 / 998: temporal / center terms
DEV constexpr int RP_NORM(int j) { return 200000 + j; }
DEV constexpr int RP_LIGHT(int i) { return 1000000 + i; }       // initial candidates: light candidate i (target visibility)
DEV constexpr int RP_BSDF(int i) { return 2000000 + i; }        // initial candidates: BSDF candidate i
constexpr int RP_VISREUSE = 300000;                          // restir_visibility_reuse
struct RRays {
    const DevScene* S;
    uint2* lds;
    uint32_t* spill;
    bool alpha;
    uint32_t pseed;
    int kind;
    int n;
    uint32_t n_any, n_closest;
    DEV RRays& at(int pos) { n = pos; return *this; }
    DEV bool any(v3 o, v3 d, float tmax, int last) {
        n_any++;
        uint32_t key = alpha ? alpha_key(pseed, 0, kind, n++) : 0u;
        THit h;
        uint32_t nn = 0, nt = 0;
        // evaluate_shadow_ray: maxT = t_max - 1e-4 (Intersect.h:227)
#ifdef MPT_RESTIR_NO_TRACE   // timing experiment only: how much of a pass is traversal
        return false;
#endif
        return traverse<true, false>(*S, o, d, last, tmax - 1.0e-4f, h, lds, spill, nn, nt, alpha, key);
    }
    DEV bool closest(v3 o, v3 d, int last, THit& h) {
        n_closest++;
        uint32_t key = alpha ? alpha_key(pseed, 0, kind, n++) : 0u;
        uint32_t nn = 0, nt = 0;
        return traverse<false, false>(*S, o, d, last, INFINITY, h, lds, spill, nn, nt, alpha, key);
    }
};
DEV void count_pass_rays(const DevPaths& P, uint32_t n_any, uint32_t n_closest) {
    for (int off = 32; off > 0; off >>= 1) {
        n_any += __shfl_xor(n_any, off);
        n_closest += __shfl_xor(n_closest, off);
    }
    if (lane_id() == 0 && (n_any | n_closest)) {
        atomicAdd((unsigned long long*)&P.ray_counts[1], (unsigned long long)n_any);
        atomicAdd((unsigned long long*)&P.ray_counts[2], (unsigned long long)n_closest);
    }
}

// ---- staged passes: ray positions, block-aggregated list appends ----------------------
struct TgtRay { v3 o, d; float dist; };   // a shadow ray of a target function / visibility test
// neighbours a staged pass supports; ray positions per pixel slot (spatial neighbour k: 2k, 2k + 1;
// fused pass: temporal 0, 1, spatial k 2 + 2k, 3 + 2k); records per pixel slot (rq_rec)
constexpr int RS_KMAX = RS_KMAX_HOST, RS_RPP = RS_RPP_HOST, RS_REC = RS_REC_HOST;
constexpr uint32_t RSE_PREV = 0x40000000u;   // eval item flag: the surface is in the previous frame's G-buffer
enum : int { RSM_SKIP = 1 };                      // rq_meta.x: the pixel is not resampled (output untouched)

// exclusive scan of one int per thread over a TB-thread block; total to `total`
DEV int rs_block_scan(int v, int* tmp, int& total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    constexpr int NW = TB / 64;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int tw = tmp[w];
        if (w < wid) before += tw;
        all += tw;
    }
    __syncthreads();
    total = all;
    return before + x - v;
}

DEV void rs_stage_ray(const DevPaths& P, size_t id, const TgtRay& r, int last, uint32_t key) {
    const size_t q = rq_phys(P, (int)id);
    P.rq_o[q] = make_float4(r.o.x, r.o.y, r.o.z, __uint_as_float((uint32_t)last));
    P.rq_d[q] = make_float4(r.d.x, r.d.y, r.d.z, r.dist - 1.0e-4f);
    P.rq_key[q] = key;
}

// appends the ray positions in `mask` of slot s to the list behind `counter` (one atomic per block)
DEV void rs_append(const DevPaths& P, int32_t* counter, int s, uint32_t mask, int* tmp, int* base) {
    int tot;
    const int off = rs_block_scan(__popc(mask), tmp, tot);
    if (threadIdx.x == 0) *base = tot ? atomicAdd(counter, tot) : 0;
    __syncthreads();
    int o = *base + off;
    while (mask) {
        const int j = __builtin_ctz(mask);
        mask &= mask - 1u;
        P.rq_list[o++] = s * RS_RPP + j;
    }
}

DEV float power_heuristic(float a, int na, float b, int nb) {   // Sampling.h:75-87
    float pa = ((float)na * a) * ((float)na * a);
    float pb = ((float)nb * b) * ((float)nb * b);
    return (float)na * a * a / (pa + pb);
}
DEV float radical_inverse_base_2(uint32_t i) {   // Sampling.h:25-32
    i = (i << 16u) | (i >> 16u);
    i = ((i & 0x55555555u) << 1u) | ((i & 0xAAAAAAAAu) >> 1u);
    i = ((i & 0x33333333u) << 2u) | ((i & 0xCCCCCCCCu) >> 2u);
    i = ((i & 0x0F0F0F0Fu) << 4u) | ((i & 0xF0F0F0F0u) >> 4u);
    i = ((i & 0x00FF00FFu) << 8u) | ((i & 0xFF00FF00u) >> 8u);
    return (float)i * 2.3283064365386963e-10f;
}
DEV uint32_t pass_seed(const MptFrame& F, uint32_t pix, uint32_t seed) {
    return F.render_settings.freeze_random ? wang_hash(pix + 1u) : wang_hash((pix + 1u) * (uint32_t)(F.render_settings.sample_number + 1) * seed);
}

// ---- reservoir operations (Reservoir.h:36-116) -------------------------------------
DEV void rr_add(RResv& r, int tri, v3 p, float tf, uint32_t fl, float w, Rng& rng) {
    r.M++;
    r.wsum += w;
    if (rng() < w / r.wsum) { r.tri = tri; r.point = p; r.target = tf; r.flags = fl; }
}
DEV bool rr_combine(RResv& r, const RResv& o, float mis, float tf, float jac, Rng& rng) {
    if (o.UCW <= 0.0f) { r.M += o.M; return false; }
    float w = mis * tf * o.UCW * jac;
    r.M += o.M;
    r.wsum += w;
    if (rng() < w / r.wsum) {
        r.tri = o.tri; r.point = o.point; r.flags = o.flags;
        r.target = tf;
        return true;
    }
    return false;
}
DEV void rr_end_norm(RResv& r, float nume, float denom) {   // end_with_normalization (Reservoir.h:96-106)
    if (r.wsum == 0.0f || r.wsum < 1.0e-10f || r.wsum > 1.0e10f || denom == 0.0f || nume == 0.0f) r.UCW = 0.0f;
    else r.UCW = 1.0f / r.target * r.wsum * nume / denom;
    r.M = imin(r.M, 1000000);
}
DEV void rr_end_normalized(RResv& r) { rr_end_norm(r, 1.0f, 1.0f); }   // the pairwise weights' 1 / 1

// ReSTIR_DI_evaluate_target_function<vis> (Utils.h:20-128), split at the visibility test:
// restir_target_unocc returns the target before it (0 = no ray would be traced) and the
// shadow ray the test traces (TgtRay: its distance; evaluate_shadow_ray traces to
// distance - 1e-4, Intersect.h:227)
// PLAIN: the surface is a plain dielectric seen from outside (rs_plain): the Principled BSDF
// with the zero-weight lobes compiled out (dev_bsdf.h FULL = false), bit for bit the same
template <bool PLAIN = false>
DEV float restir_target_unocc(const DevScene& S, const MptFrame& F, const BCtx& bc, int tri, v3 point, uint32_t flags,
                              const RSurf& s, bool vis, int ovr, TgtRay& ray) {
    if (tri == -1 && !(flags & RF_ENVMAP)) return 0.0f;
    float dist = 0.0f;
    v3 dir;
    if (flags & RF_ENVMAP) { dir = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, point); dist = 1.0e35f; }
    else if (vis) { dir = point - s.sp; dist = length(dir); dir = dir / dist; }
    else dir = normalize(point - s.sp);
    float cosv = maxr(0.0f, dot(s.sn, dir));
    if (cosv == 0.0f) return 0.0f;
    float bp;
    VState tv = s.vs;
    Col f;
    if (PLAIN) {
        PEval pe;
        bsdf_eval_pre<MPT_BSDF_NONE, false>(bc, *s.m, tv, s.view, s.sn, pe);
        f = bsdf_eval_post<MPT_BSDF_NONE, false>(bc, *s.m, tv, pe, s.sn, dir, bp);
    } else {
        f = ovr == MPT_BSDF_LAMBERTIAN   ? bsdf_eval<MPT_BSDF_LAMBERTIAN>(bc, *s.m, tv, s.view, s.sn, dir, bp)
            : ovr == MPT_BSDF_OREN_NAYAR ? bsdf_eval<MPT_BSDF_OREN_NAYAR>(bc, *s.m, tv, s.view, s.sn, dir, bp)
                                         : bsdf_eval<MPT_BSDF_NONE>(bc, *s.m, tv, s.view, s.sn, dir, bp);
    }
    Col e;
    if (flags & RF_ENVMAP) { float ep; e = env_eval(S, F, dir, ep); }
    else e = emission_of(S.mats[S.mat_idx[tri]]);
    float t = lum(f * e * cosv);
    ray.o = s.sp;
    ray.d = dir;
    ray.dist = dist;
    return t;
}
DEV float restir_target(const DevScene& S, const MptFrame& F, const BCtx& bc, RRays& rr, int tri, v3 point, uint32_t flags,
                        const RSurf& s, bool vis, int ovr) {
    TgtRay ray;
    float t = restir_target_unocc(S, F, bc, tri, point, flags, s, vis, ovr, ray);
    if (t == 0.0f) return 0.0f;
    if (vis) t *= rr.any(s.sp, ray.d, ray.dist, s.last) ? 0.0f : 1.0f;
    return t;
}

// ReSTIR_DI_visibility_reuse (Utils.h:134-171)
DEV void restir_visibility_reuse(const MptFrame& F, RRays& rr, RResv& r, v3 sp, int last) {
    if (r.UCW <= 0.0f) return;
    if (r.flags & RF_UNOCCLUDED) return;
    float dist;
    v3 dir;
    if (r.flags & RF_ENVMAP) { dir = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, r.point); dist = 1.0e35f; }
    else { dir = r.point - sp; dist = length(dir); dir = dir / dist; }
    if (rr.at(RP_VISREUSE).any(sp, dir, dist, last)) r.UCW = -1.0f;
    else r.flags |= RF_UNOCCLUDED;
}

// get_jacobian_determinant_reconnection_shift (Utils.h:173-206)
DEV float restir_jacobian(const DevScene& S, const RResv& nr, v3 csp, v3 nsp) {
    v3 tc = nr.point - csp, tn = nr.point - nsp;
    float dc = length(tc);
    tc = tc / dc;
    float dn = length(tn);
    tn = tn / dn;
    int3 t = tri_idx(S, nr.tri);
    v3 A = ld3(S.pos, t.x);
    v3 ln = normalize(cross(ld3(S.pos, t.y) - A, ld3(S.pos, t.z) - A));
    float cc = absr(dot(-tc, ln)), cn = absr(dot(-tn, ln));
    float jac = cc / cn * ((dn * dn) / (dc * dc));
    if (jac > 20.0f || jac < 1.0f / 20.0f || isnan(jac)) return -1.0f;
    return jac;
}

// check_neighbor_similarity_heuristics (Utils.h:214-263), incl. the inverted normal test
DEV bool restir_similar(const DevScene& S, const DevPaths& P, const MptReSTIRDISettings& rd, int nb, const Mat& center_m,
                        v3 sp, v3 n, bool prev) {
#if MPT_RESTIR_CS
    // from the compact records: position + material of the neighbour's (current or previous)
    // surface, the shading normal of its current one (as the planes' version reads gb_sn)
    const float4 pos = ((prev ? P.pgb_cs : P.gb_cs) + 4 * (size_t)nb)[0];
    const int mref = __float_as_int(pos.w);
    const Mat* nm = mref == 0 ? &g_zero_mat : mref < 0 ? (prev ? &P.pgb_mat[nb] : &P.gb_mat[nb]) : &S.mats_res[mref - 1];
#else
    float4 pos = prev ? P.pgb_pos[nb] : P.gb_pos[nb];
    const Mat* nm = gb_surface(S, P, nb, prev).m;
#endif
    bool plane = !rd.use_plane_distance_heuristic || absr(dot(mk3(pos.x, pos.y, pos.z) - sp, n)) < rd.plane_distance_threshold;
    bool normal = true;
    if (!rd.use_normal_similarity_heuristic) {
        float4 ns = MPT_RESTIR_CS ? P.gb_cs[4 * (size_t)nb + 1] : P.gb_sn[nb];
        normal = dot(n, mk3(ns.x, ns.y, ns.z)) > rd.normal_similarity_angle_precomp;
    }
    bool rough = !rd.use_roughness_similarity_heuristic || absr(nm->roughness - center_m.roughness) < rd.roughness_similarity_threshold;
    return plane && normal && rough && !is_emissive(*nm);
}

// get_spatial_neighbor_pixel_index (Utils.h:289-339)
DEV int restir_spatial_neighbor(const DevPaths& P, const MptFrame& F, int k, int count, int radius, int cx, int cy, float cr,
                                float sr, uint32_t pass_random_seed) {
    const MptRenderSettings& rs = F.render_settings;
    int W = F.res_x, H = F.res_y;
    if (k == count) return cx + cy * W;
    float ux = (float)(unsigned)(k + 1) / (float)(unsigned)(count + 1), uy = radical_inverse_base_2((unsigned)(k + 1));
    float rr = (float)radius * sqrtf(uy);
    float ox = rr * pcos(TWO_PI * ux), oy = rr * psin(TWO_PI * ux);
    float rx = ox * cr - oy * sr, ry = ox * sr + oy * cr;
    int nx, ny;
    if (rs.restir_di_settings.debug_neighbor_location) { nx = cx + 15; ny = cy; }
    else { nx = cx + (int)rx; ny = cy + (int)ry; }
    if (nx < 0 || nx >= W || ny < 0 || ny >= H) return -1;
    int ni = nx + ny * W;
    if (rs.enable_adaptive_sampling && rs.sample_number >= rs.adaptive_sampling_min_samples) {
        if (rs.restir_di_settings.allow_converged_neighbors_reuse) {
            Rng g = make_rng(pass_random_seed);
            if (g() > rs.restir_di_settings.converged_neighbor_reuse_probability && P.rs_conv[ni] != -1) return -1;
        } else if (P.rs_conv[ni] != -1) return -1;
    }
    return ni;
}

// pairwise MIS defensive (SpatiotemporalMISWeight.h:193-291, SpatialMISWeight.h:167-262).
// weight() evaluates the canonical sample's target at the neighbour (tcn, with visibility when
// bvis) and hands it to weight_tcn, which the staged passes call with the stored value.
struct PairwiseMIS {
    float mc;
    bool defensive;   // PAIRWISE_MIS_DEFENSIVE (else PAIRWISE_MIS, SpatialMISWeight.h:95-165)
    bool bvis;        // ReSTIR_DI_BiasCorrectionUseVisibility
    DEV float weight(const DevScene& S, const MptFrame& F, const BCtx& bc, RRays& rr, const MptReSTIRDISettings& rd,
                     const RResv& res, const RResv& center, float tf_center, const RSurf& nsurf, int vcount, int vM,
                     bool update_mc, bool canonical, int ovr) {
        float tcn = 0.0f;
        if (!canonical && update_mc) tcn = restir_target(S, F, bc, rr, center.tri, center.point, center.flags, nsurf, bvis, ovr);
        return weight_tcn(rd, res, center, tf_center, tcn, vcount, vM, update_mc, canonical);
    }
    DEV float weight_tcn(const MptReSTIRDISettings& rd, const RResv& res, const RResv& center, float tf_center, float tcn,
                         int vcount, int vM, bool update_mc, bool canonical) {
        if (!defensive) {
            const bool cw = rd.use_confidence_weights;
            if (canonical) return mc == 0.0f ? 1.0f : mc;
            float tfn = res.target;
            float rM = cw ? (float)res.M : 1.0f, cM = cw ? (float)center.M : 1.0f, nsum = cw ? (float)vM : 1.0f;
            float div = cw ? 1.0f : (float)vcount;
            float nume = tfn * rM;
            float denom = tfn * nsum + tf_center / div * cM;
            float mi = denom == 0.0f ? 0.0f : (nume / denom);
            if (update_mc) {
                float tcc = center.target;
                float nume_mc = tcc / div * cM;
                float denom_mc = tcn * nsum + tcc / div * cM;
                float conf = cw ? rM / nsum : 1.0f;
                if (denom_mc != 0.0f) mc += nume_mc / denom_mc / div * conf;
            }
            return mi / div;
        }
        if (!canonical) {
            float tfn = res.target;
            float rM = rd.use_confidence_weights ? (float)res.M : 1.0f;
            float cM = rd.use_confidence_weights ? (float)center.M : 1.0f;
            float nsum = rd.use_confidence_weights ? (float)vM : 1.0f;
            float div = rd.use_confidence_weights ? 1.0f : (float)vcount;
            float nume = tfn * rM;
            float denom = tfn * nsum + tf_center / div * cM;
            float mi = 0.0f;
            if (denom != 0.0f) mi = nume / denom;
            if (rd.use_confidence_weights) mi *= nsum / (nsum + cM);
            if (update_mc) {
                float tcc = center.target;
                float nume_mc = tcc / div * cM;
                float denom_mc = tcn * nsum + tcc / div * cM;
                float conf = 1.0f;
                if (rd.use_confidence_weights) conf = rM / (cM + nsum);
                if (denom_mc != 0.0f) mc += nume_mc / denom_mc * conf;
            }
            if (rd.use_confidence_weights) return mi;
            return mi / (float)(vcount + 1);
        }
        if (mc == 0.0f) return 1.0f;
        if (rd.use_confidence_weights) return mc + (float)center.M / (float)(center.M + vM);
        return (1.0f + mc) / (float)(vcount + 1);
    }
};

DEV bool spatial_visibility(const MptFrame& F, const MptReSTIRDISettings& rd, int k, int reuse_count) {   // SpatialReuse.h:36-50
    bool v = rd.do_visibility_only_last_pass && rd.spatial_pass_index == rd.number_of_passes - 1;
    v |= !rd.do_visibility_only_last_pass;
    v &= k < rd.neighbor_visibility_count;
    v &= F.options.restir_di_spatial_target_visibility != 0;
    v &= k != reuse_count;
    return v;
}

DEV BCtx make_bctx(const DevScene& S, const MptFrame& F) {
    BCtx bc;
    bc.mats = S.mats;
    bc.luts = DevLuts{S.lut_conductor, S.lut_glossy, S.lut_glass, S.lut_glass_inv, S.lut_thin_glass, S.lut_sheen};
    bc.clearcoat_comp = F.bsdf_flags.clearcoat_compensation_approximation;
    bc.masking = F.bsdf_flags.ggx_masking_shadowing;
    return bc;
}

// the previous frame's pixel coordinates of a point (Utils.h:378-384)
DEV void restir_reproject(const MptFrame& F, v3 p, float& fx, float& fy) {
    v3 ss = mat_x_point(F.prev_camera.view_projection.m, p);
    float sx = ss.x, sy = ss.y;
    sx += 1.0f; sy += 1.0f;
    sx *= 0.5f; sy *= 0.5f;
    fx = sx * (float)F.res_x; fy = sy * (float)F.res_y;
    fx -= 0.5f; fy -= 0.5f;
}

// ---- G-buffer write: CameraRays (CameraRays.h:144-166) over the camera queue ----------
#ifndef MPT_TU_PART   // k_gbuffer
__global__ __launch_bounds__(TB) void k_gbuffer(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    int i = blockIdx.x * TB + threadIdx.x;
    // a chunk of samples (DevPaths::ci_n): every slot of the chunk's samples (their camera
    // queues are whole: no adaptive sampling, no low resolution), written to the chunk's planes
    // at the slot; a miss's record starts empty instead of keeping the pixel's last surface
    // (the chunk's consumers skip misses; k_chunk_join keeps it in the context's planes)
    const bool chunk = P.ci_n > 0;
    if (i >= (chunk ? P.n : P.counters[CTR_Q0])) return;
    const MptFrame& F = chunk ? Fp[i / P.ci_n] : *Fp;
    int slot = chunk ? i : P.q0[i];
    const int gp = slot + P.pix_off;   // G-buffer entry of the slot's pixel
    float4 ro = P.ray_o[slot], rdv = P.ray_d[slot], hv = P.hit[slot];
    v3 o = mk3(ro.x, ro.y, ro.z), d = mk3(rdv.x, rdv.y, rdv.z);
    int prim = (int)__float_as_uint(hv.w);
    bool found = prim >= 0;
    int4 meta = chunk ? make_int4(0, 0, 0, 0) : P.gb_meta[gp];
    if (found) {
        // trace_ray hit processing (Intersect.h:150-216), as k_shade does at bounce 0
        VState vs = vs_load_s(P.vsA, P.vsB, slot);
        Rng rng = make_rng(P.rng[slot]);
        float t = hv.x;
        v2 uv = mk2(hv.y, hv.z);
        v3 ip = o + t * d;
        const HitAttr ha = hit_attributes(S, prim, uv);
        const v2 tc = ha.tc;
        v3 gn = ha.gn;
        v3 sn = ha.sn;
        const int mi = ha.mi;
        const Mat* mp;
        int per_pixel = 0;
        if (F.bsdf_flags.white_furnace_mode || (S.mat_tex[mi] & MT_TEXTURED)) {
            P.gb_mat[gp] = intersection_material(S, mi, tc, F.bsdf_flags.white_furnace_mode);
            mp = &P.gb_mat[gp];
            per_pixel = 1;
        } else {
            mp = &S.mats_res[mi];
        }
        const Mat& m = *mp;
        bool was_inside = P.hit_inside[slot] != 0;
        if ((!was_inside || m.specular_transmission == 0.0f) && !m.thin_walled) {
            gn *= dot(gn, -d) < 0.0f ? -1.0f : 1.0f;
            sn *= dot(sn, gn) < 0.0f ? -1.0f : 1.0f;
            float NoV = dot(sn, -d);
            sn += (2.0f * clampr(0.0f, 1.0f, -NoV)) * -d;
        }
        if (m.dispersion_scale > 0.0f && m.specular_transmission > 0.0f && vs.wl == 0.0f)
            vs.wl = -(rng() * (float)(830 - 360) + (float)360);
        if (is_emissive(m) && dot(-d, gn) < 0) { gn = -gn; sn = -sn; }
        if (F.band_count > 1 && !chunk) {   // (a chunk: measured by k_chunk_join)
            // rows between this pixel and its reprojection (restir_temporal_neighbor's base
            // position): the halo a partitioned context needs for the temporal reuse
            float fx, fy;
            restir_reproject(F, ip, fx, fy);
            const float H = (float)F.res_y;
            int off = F.res_y;
            if (fy > -H && fy < 2.0f * H) off = min(F.res_y, abs((int)roundf(fy) - gp / F.res_x));
            atomicMax(&P.counters[CTR_REPROJ], off);
        }
        P.gb_pos[gp] = make_float4(ip.x, ip.y, ip.z, 0.0f);
        P.gb_sn[gp] = make_float4(sn.x, sn.y, sn.z, 0.0f);
        P.gb_gn[gp] = make_float4(gn.x, gn.y, gn.z, 0.0f);
        vs_store(P.gb_vsA, P.gb_vsB, gp, vs);
        meta.y = mi + 1;
        meta.w = per_pixel;
        if (MPT_RESTIR_CS) {
            float4* cs = P.gb_cs + 4 * (size_t)gp;
            cs[0] = make_float4(ip.x, ip.y, ip.z, __int_as_float(per_pixel ? -meta.y : meta.y));
            cs[1] = make_float4(sn.x, sn.y, sn.z, __int_as_float(vs.incident));
            cs[3] = make_float4(gn.x, gn.y, gn.z, 0.0f);
        }
    }
    meta.x = found ? prim : -1;
    meta.z = found ? 1 : 0;
    P.gb_meta[gp] = meta;
    P.gb_view[gp] = make_float4(-d.x, -d.y, -d.z, 0.0f);
    // (a miss keeps the record's surface, as it keeps the planes', and updates view + last hit)
    if (MPT_RESTIR_CS) P.gb_cs[4 * (size_t)gp + 2] = make_float4(-d.x, -d.y, -d.z, __int_as_float(meta.x));
}
#endif

// ---- ReSTIR_DI_LightsPresampling (LightsPresampling.h:22-130) ------------------------
#ifndef MPT_TU_PART   // k_restir_presample
__global__ __launch_bounds__(TB) void k_restir_presample(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    const MptReSTIRDISettings& rd = Fp->render_settings.restir_di_settings;
    const MptWorldSettings& w = Fp->world_settings;
    if (S.n_emissive == 0 && w.ambient_light_type != MPT_AMBIENT_ENVMAP) return;
    const int n_pl = rd.number_of_subsets * rd.subset_size;
    int x = blockIdx.x * TB + threadIdx.x;
    // a chunk of samples (DevPaths::ci_n): sample x / n_pl's lights, sample-major
    const int smp = P.ci_n ? x / n_pl : 0;
    if (x >= (P.ci_n ? P.n / P.ci_n : 1) * n_pl) return;
    const MptFrame& F = Fp[smp];
    Rng rng = make_rng(pass_seed(F, (uint32_t)(x - smp * n_pl), F.restir_di_seeds[0]));
    float env_p = 0.0f;
    if (w.ambient_light_type == MPT_AMBIENT_ENVMAP) env_p = S.n_emissive == 0 ? 1.0f : rd.envmap_candidate_probability;
    int tri = -1;
    v3 point = mk3(0, 0, 0), nrm = mk3(0, 0, 0);
    Col rad = col(0.0f);
    float pdf = 0.0f;
    uint32_t flags = 0;
    if (rng() < env_p) {
        flags |= RF_ENVMAP;
        v3 dir;
        rad = env_sample(S, F, dir, pdf, rng);
        point = mat_x_vec(w.world_to_envmap_matrix.m, dir);
        pdf *= env_p;
    } else {
        float lp = 1.0f - env_p;
        int ri = rng.random_index(S.n_emissive);
        int t = S.emissive[ri];
        int3 ti = tri_idx(S, t);
        v3 A = ld3(S.pos, ti.x), B = ld3(S.pos, ti.y), C = ld3(S.pos, ti.z);
        float r1 = rng(), r2 = rng();
        float sr1 = sqrtf(r1);
        float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
        v3 AB = B - A, AC = C - A;
        v3 pt = A + AB * u + AC * v;
        v3 nn = cross(AB, AC);
        float ln = length(nn);
        if (ln > 1.0e-6f) {
            point = pt;
            nrm = nn / ln;
            tri = t;
            pdf = 1.0f / (ln * 0.5f);
            pdf /= (float)S.n_emissive;
            pdf *= lp;
            rad = emission_of(S.mats[S.mat_idx[t]]);
        }
    }
    float4* o = P.rs_plights + 4 * (size_t)x;
    o[0] = make_float4(__int_as_float(tri), point.x, point.y, point.z);
    o[1] = make_float4(nrm.x, nrm.y, nrm.z, pdf);
    o[2] = make_float4(rad.r, rad.g, rad.b, __uint_as_float(flags));
}
#endif

// the evaluation class of a G-buffer surface: plain dielectric seen from outside (the
// condition k_shade<PLAIN> checks before it shades, principled_eval_pre's 'outside')
DEV bool rs_plain(const DevScene& S, const DevPaths& P, int pix, const RSurf& g, bool prev = false) {
    const int mi = (prev ? P.pgb_meta[pix].y : P.gb_meta[pix].y) - 1;
    if (mi < 0) return false;
    const int32_t mt = S.mat_tex[mi];
    // MT_TEXMETAL: plain where the resolved (per-pixel) material's texel is not metallic
    return (!(mt & MT_FULL) || ((mt & MT_TEXMETAL) && g.m->metallic == 0.0f)) && (dot(g.view, g.sn) > 0.0f || g.m->thin_walled);
}

// ---- ReSTIR_DI_InitialCandidates (InitialCandidates.h:24-508) ------------------------
// The BSDF candidate once its ray is traced (InitialCandidates.h:296-394): found = a closest
// hit below 1e35 - 1e-4 with hit record h (t, u, v, prim).
DEV void initial_bsdf_candidate(const DevScene& S, const MptFrame& F, v3 gp, v3 gsn, v3 dir, Col f, float bpdf, bool refr,
                                bool found, float4 h, float env_p, int nl, int nb, RResv& r, Rng& rng) {
    const MptWorldSettings& w = F.world_settings;
    ShadowLightHit sh;
    if (found) found = shadow_light_hit(S, h, sh);
    if (found && !is_black(sh.em)) {
        float ce = absr(dot(gsn, dir));
        Col lc = f * sh.em * ce;
        float tf = lum(lc);
        float lpdf = 0.0f;
        if (!refr) lpdf = pdf_emissive_hit(S, sh, dir);
        if (!min_contrib(F.render_settings.minimum_light_contribution, lc / lpdf / bpdf)) { r.M++; return; }
        lpdf *= (1.0f - env_p);
        float mis = power_heuristic(bpdf, nb, lpdf, nl);
        float weight = mis * tf / bpdf;
        rr_add(r, sh.prim, gp + dir * sh.dist, tf, RF_UNOCCLUDED | (refr ? RF_BSDF_REFRACTION : 0u), weight, rng);
    } else if (!found && w.ambient_light_type == MPT_AMBIENT_ENVMAP) {
        float ce = maxr(0.0f, dot(gsn, dir));
        if (ce > 0.0f) {
            float epdf;
            Col er = env_eval(S, F, dir, epdf);
            Col ec = f * er * ce;
            if (!min_contrib(F.render_settings.minimum_light_contribution, ec / epdf / bpdf)) { r.M++; return; }
            float tf = lum(ec);
            epdf *= env_p;
            float mis = power_heuristic(bpdf, nb, epdf, nl);
            float weight = mis * tf / bpdf;
            rr_add(r, -1, mat_x_vec(w.world_to_envmap_matrix.m, dir), tf, RF_ENVMAP | RF_UNOCCLUDED, weight, rng);
        }
    }
}

// Staged variant (STAGED = true; the host uses it with at most one BSDF candidate and no
// initial target visibility, the reference defaults): the kernel stops at the BSDF
// candidate's ray, stages it (k_trace<TM_LIST_CLOSEST>) and leaves the partial reservoir in
// rs_init, the RNG state in rq_meta and the candidate in rq_rec for k_rsi_finish.  It runs
// over the pixel lists k_rsi_classify sorts by the material class of the G-buffer surface:
// PLAIN = plain dielectric seen from outside (the BSDF with the zero-weight lobes compiled
// out, dev_bsdf.h FULL = false, bit for bit the generic code's result for it).
enum : int { RSI_RAY = 2 };   // rq_meta.x: a BSDF-candidate ray was staged
// bsdf_sample with the class's code: the direction, then the evaluation on the updated state
template <int OVR, int FULL>
DEV Col bsdf_sample_cls(const BCtx& bc, const Mat& m, VState& vs, v3 view, v3 sn, v3 gn, v3& dir, float& pdf, Rng& rng) {
    if (FULL) return bsdf_sample<OVR>(bc, m, vs, view, sn, gn, dir, pdf, rng);
    pdf = 0.0f;
    if (!bsdf_sample_dir<OVR, false>(bc, m, vs, view, sn, gn, dir, rng)) return col(0.0f);
    PEval pe;
    bsdf_eval_pre<OVR, false>(bc, m, vs, view, sn, pe);
    return bsdf_eval_post<OVR, false>(bc, m, vs, pe, sn, dir, pdf);
}
template <int OVR, bool STAGED, bool PLAIN = false>
RESTIR_KERNEL void k_restir_initial(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, const int32_t* __restrict__ list,
                                    const int32_t* __restrict__ list_count) {
    __shared__ uint2 lds[STAGED ? 1 : LDS_STACK * TB];
    __shared__ int tmp[TB / 64];
    __shared__ int sbase;
    const MptFrame& F = *Fp;
    const MptReSTIRDISettings& rd = F.render_settings.restir_di_settings;
    const MptWorldSettings& w = F.world_settings;
    if (S.n_emissive == 0 && w.ambient_light_type != MPT_AMBIENT_ENVMAP) return;   // (block-uniform)
    const BCtx bc = make_bctx(S, F);
    RRays rr{&S, lds, P.stack_spill + ((size_t)blockIdx.x * TB + threadIdx.x) * (2 * SPILL_DEPTH),
             F.render_settings.do_alpha_testing, 0u, 5, 0, 0u, 0u};
    const int W = F.res_x;
    // staged: over the class list, with a block-uniform trip count (the block appends its rays)
    const int count = STAGED ? *list_count : P.n;
    const int b_end = STAGED ? count : (int)(blockIdx.x * TB + 1);
    for (int b0 = blockIdx.x * TB; b0 < b_end; b0 += gridDim.x * TB) {
    uint32_t rmask = 0u;
    int s_lane = 0;
    for (int t = STAGED ? b0 + (int)threadIdx.x : blockIdx.x * TB + threadIdx.x; t < count; t += STAGED ? count : gridDim.x * TB) {
        const int s = STAGED ? list[t] : t;
        s_lane = s;
        const int pix = s + P.pix_off;
        // the frame pixel and the sample's frame: a chunk's item s is pixel s % ci_n of its
        // sample s / ci_n (DevPaths::ci_n; the planes are indexed by item)
        const int fpix = P.ci_n ? s % P.ci_n + P.ci_pix_off : pix;
        const MptFrame& Fs = P.ci_n ? Fp[s / P.ci_n] : F;
        RSurf g = gb_surface(S, P, pix, false);
        if (is_emissive(*g.m)) continue;
        uint32_t seed = pass_seed(Fs, (uint32_t)fpix, Fs.restir_di_seeds[1]);
        Rng rng = make_rng(seed);
        if (!P.active[s] || !P.gb_meta[pix].z) continue;
        rr.pseed = seed;
        rr.n = 0;
        const int x = fpix % W, y = fpix / W;
        int nl = rd.number_of_initial_light_candidates, nb = rd.number_of_initial_bsdf_candidates;
        float env_p = 0.0f;
        if (w.ambient_light_type == MPT_AMBIENT_ENVMAP) env_p = S.n_emissive == 0 ? 1.0f : rd.envmap_candidate_probability;
        RResv r = rr_default();
        v3 ep = g.p + g.sn * 1.0e-4f * 1.0f;
        PEval pe;
        bsdf_eval_pre<OVR, !PLAIN>(bc, *g.m, g.vs, g.view, g.sn, pe);
        for (int i = 0; i < nl; i++) {
            int tri;
            v3 point, tl;
            uint32_t flags;
            Col rad;
            float pdf, dist = 0.0f, target = 0.0f, cosv;
            if (F.options.restir_di_do_lights_presampling) {
                // use_presampled_light_candidate (InitialCandidates.h:30-90)
                int tcs = (x / rd.tile_size + y / rd.tile_size + 1) * (x / rd.tile_size + y / rd.tile_size) / 2 + y / rd.tile_size;
                Rng subset_rng = make_rng(Fs.restir_di_seeds[1] * (uint32_t)(tcs + 1));
                int subset = subset_rng.random_index(rd.number_of_subsets);
                int li = rng.random_index(rd.subset_size);
                const size_t pl0 = P.ci_n ? (size_t)(s / P.ci_n) * (size_t)(rd.number_of_subsets * rd.subset_size) : 0;
                const float4* pl = P.rs_plights + 4 * (pl0 + (size_t)(subset * rd.subset_size + li));
                float4 p0 = pl[0], p1 = pl[1], p2 = pl[2];
                tri = __float_as_int(p0.x);
                point = mk3(p0.y, p0.z, p0.w);
                flags = __float_as_uint(p2.w);
                rad = col(p2.x, p2.y, p2.z);
                pdf = p1.w;
                if (flags & RF_ENVMAP) { tl = mat_x_vec(w.envmap_to_world_matrix.m, point); dist = 1.0e35f; }
                else { tl = point - ep; dist = length(tl); tl = tl / dist; }
                cosv = dot(g.sn, tl);
                if (!(flags & RF_ENVMAP)) {
                    float cl = absr(dot(mk3(p1.x, p1.y, p1.z), -tl));
                    pdf *= dist * dist;
                    pdf /= cl;
                    if (!min_contrib(F.render_settings.minimum_light_contribution, rad * cosv / pdf)) { r.M++; continue; }
                }
            } else {
                // sample_fresh_light_candidate (InitialCandidates.h:93-170)
                tri = -1; point = mk3(0.0f, 0.0f, 0.0f); flags = 0u; rad = col(0.0f); pdf = 0.0f; cosv = 0.0f;
                if (rng() > env_p) {
                    LightInfo lsi;
                    point = sample_emissive_triangle(S, rng, pdf, lsi);
                    tri = lsi.tri;
                    if (pdf > 0.0f) {
                        v3 d2 = point - ep;
                        float dl = length(d2);
                        d2 = d2 / dl;
                        cosv = maxr(0.0f, dot(g.sn, d2));
                        float cl = absr(dot(lsi.normal, -d2));
                        pdf *= dl * dl;
                        pdf /= cl;
                        if (!min_contrib(F.render_settings.minimum_light_contribution, lsi.emission * cosv / pdf)) { r.M++; continue; }
                        pdf *= (1.0f - env_p);
                        rad = lsi.emission;
                    }
                } else {
                    v3 edir;
                    rad = env_sample(S, F, edir, pdf, rng);
                    cosv = maxr(0.0f, dot(edir, g.sn));
                    if (!min_contrib(F.render_settings.minimum_light_contribution, rad * cosv / pdf)) { r.M++; continue; }
                    pdf *= env_p;
                    point = mat_x_vec(w.world_to_envmap_matrix.m, edir);
                    flags = RF_ENVMAP;
                }
                if (flags & RF_ENVMAP) { tl = mat_x_vec(w.envmap_to_world_matrix.m, point); dist = 1.0e35f; }
                else { tl = point - ep; dist = length(tl); tl = tl / dist; }
            }
            float weight = 0.0f;
            if (cosv > 0.0f && pdf > 0.0f) {
                float bp;
                VState tv = g.vs;
                Col f = bsdf_eval_post<OVR, !PLAIN>(bc, *g.m, tv, pe, g.sn, tl, bp);
                Col lc = f * rad * cosv;
                float tf = lum(lc);
                if (min_contrib(F.render_settings.minimum_light_contribution, lc / pdf / bp)) {
                    float mis = power_heuristic(pdf, nl, bp, nb);
                    weight = mis * tf / pdf;
                    target = tf;
                }
            }
            // ReSTIR_DI_InitialTargetFunctionVisibility (InitialCandidates.h:248-264)
            // InitialCandidates.h:248-249: no visibility in the target function at low resolution
            if (F.options.restir_di_initial_target_visibility && !low_res(F.render_settings) && target > 0.0f) {
                if (rr.at(RP_LIGHT(i)).any(ep, tl, dist, g.last)) { r.M++; continue; }
                flags |= RF_UNOCCLUDED;
            }
            rr_add(r, tri, point, target, flags, weight, rng);
        }
        for (int i = 0; i < nb; i++) {
            // sample_bsdf_candidates (InitialCandidates.h:273-394)
            float bpdf = 0.0f;
            v3 dir;
            VState tv = g.vs;
            Col f = bsdf_sample_cls<OVR, !PLAIN>(bc, *g.m, tv, g.view, g.sn, g.gn, dir, bpdf, rng);
            bool refr = dot(dir, g.view) < 0.0f;   // the reference tests against the view direction
            if (!(bpdf > 0.0f)) continue;
            if (STAGED) {
                const size_t id = rq_phys(P, s * RS_RPP);
                P.rq_o[id] = make_float4(g.p.x, g.p.y, g.p.z, __uint_as_float((uint32_t)g.last));
                P.rq_d[id] = make_float4(dir.x, dir.y, dir.z, INFINITY);
                P.rq_key[id] = F.render_settings.do_alpha_testing ? alpha_key(seed, 0, 5, RP_BSDF(i)) : 0u;
                P.rq_rec[rq_rec_at(P, s, 0)] = make_float4(f.r, f.g, f.b, bpdf);
                P.rq_rec[rq_rec_at(P, s, 1)] = make_float4(dir.x, dir.y, dir.z, refr ? 1.0f : 0.0f);
                rmask = 1u;
                continue;
            }
            THit h;
            bool found = rr.at(RP_BSDF(i)).closest(g.p, dir, g.last, h) && h.t < 1.0e35f - 1.0e-4f;
            initial_bsdf_candidate(S, F, g.p, g.sn, dir, f, bpdf, refr, found,
                                   make_float4(h.t, h.u, h.v, __uint_as_float((uint32_t)h.prim)), env_p, nl, nb, r, rng);
        }
        if (STAGED) {
            rr_store(P.rs_init, pix, r);   // partial: k_rsi_finish adds the BSDF candidate and ends it
            P.rq_meta[s] = make_int4(rmask ? RSI_RAY : 0, (int)rng.s, 0, 0);
            continue;
        }
        r.UCW = r.wsum == 0.0f ? 0.0f : 1.0f / r.target * r.wsum;   // end()
        r.M = 1;
        if (F.options.restir_di_do_visibility_reuse) restir_visibility_reuse(F, rr, r, g.p + g.sn * 1.0e-4f, g.last);
        rr_store(P.rs_init, pix, r);
    }
    if (STAGED) {
        rs_append(P, &P.counters[CTR_RQ], s_lane, rmask, tmp, &sbase);
        __syncthreads();
    }
    }
    if (!STAGED) count_pass_rays(P, rr.n_any, rr.n_closest);
}

#ifndef MPT_TU_PART   // k_rsi_classify
// The staged initial pass's pixel lists: pixels that run the pass (not emissive, active, a
// camera hit), by the class of their G-buffer surface (rs_plain): plain at [0, n), generic at
// [n, 2n) of rq_items; every other pixel is marked skipped for k_rsi_finish.
// RSI_PPT pixels per thread (s, s + TB, ...): the list appends take one device-scope atomic
// per class and block, and one word serialises them (~90 per us), so fewer, larger blocks
constexpr int RSI_PPT = 4;
__global__ __launch_bounds__(TB) void k_rsi_classify(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int principled) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    if (S.n_emissive == 0 && F.world_settings.ambient_light_type != MPT_AMBIENT_ENVMAP) return;   // (grid-uniform)
    const int s0 = blockIdx.x * (TB * RSI_PPT) + threadIdx.x;
    uint32_t cm[2] = {0u, 0u};   // bit k: pixel s0 + k * TB in class 0 / 1
#pragma unroll
    for (int k = 0; k < RSI_PPT; k++) {
        const int s = s0 + k * TB;
        if (s >= P.n) break;
        const int pix = s + P.pix_off;
        const RSurf g = gb_surface(S, P, pix, false);
        if (!is_emissive(*g.m) && P.active[s] && P.gb_meta[pix].z) cm[principled && rs_plain(S, P, pix, g) ? 0 : 1] |= 1u << k;
        else P.rq_meta[s] = make_int4(RSM_SKIP, 0, 0, 0);
    }
    for (int c = 0; c < 2; c++) {
        int tot;
        const int off = rs_block_scan(__popc(cm[c]), tmp, tot);
        if (threadIdx.x == 0) base = tot ? atomicAdd(&P.counters[CTR_RQE0 + c], tot) : 0;
        __syncthreads();
        int o = base + off;
        for (uint32_t m = cm[c]; m; m &= m - 1u) P.rq_items[(size_t)c * P.n + o++] = s0 + __builtin_ctz(m) * TB;
        __syncthreads();
    }
}
#endif

#ifndef MPT_TU_PART   // k_rsi_finish
// Staged initial candidates, second half: the BSDF candidate from its traced ray (closest
// hit in rq_o, written over the staged ray by k_trace<TM_LIST_CLOSEST>), end(), and the
// visibility-reuse ray staged for k_rs_visapply.
RESTIR_KERNEL void k_rsi_finish(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    __shared__ int tmp[TB / 64];
    __shared__ int sbase;
    const MptFrame& F = *Fp;
    const MptReSTIRDISettings& rd = F.render_settings.restir_di_settings;
    const MptWorldSettings& w = F.world_settings;
    if (S.n_emissive == 0 && w.ambient_light_type != MPT_AMBIENT_ENVMAP) return;   // as k_restir_initial (grid-uniform)
    const int s0 = blockIdx.x * (TB * RSI_PPT) + threadIdx.x;   // RSI_PPT pixels per thread, as k_rsi_classify
    uint32_t vbits = 0u, n_any = 0u, n_cl = 0u;
#pragma unroll
    for (int kk = 0; kk < RSI_PPT; kk++) {
    const int s = s0 + kk * TB;
    if (s < P.n && !(P.rq_meta[s].x & RSM_SKIP)) {
        const int4 meta = P.rq_meta[s];
        const int pix = s + P.pix_off;
        RResv r = rr_load(P.rs_init, pix);
        Rng rng = make_rng((uint32_t)meta.y);
        const float4 gp4 = P.gb_pos[pix], gs4 = P.gb_sn[pix];
        const v3 gp = mk3(gp4.x, gp4.y, gp4.z), gsn = mk3(gs4.x, gs4.y, gs4.z);
        const size_t id = (size_t)s * RS_RPP;
        if (meta.x & RSI_RAY) {
            const int nl = rd.number_of_initial_light_candidates, nb = rd.number_of_initial_bsdf_candidates;
            float env_p = 0.0f;
            if (w.ambient_light_type == MPT_AMBIENT_ENVMAP) env_p = S.n_emissive == 0 ? 1.0f : rd.envmap_candidate_probability;
            const float4 fr = P.rq_rec[rq_rec_at(P, s, 0)], dr = P.rq_rec[rq_rec_at(P, s, 1)];
            const float4 h = P.rq_o[rq_phys(P, (int)id)];
            const bool found = (int)__float_as_uint(h.w) >= 0 && h.x < 1.0e35f - 1.0e-4f;
            initial_bsdf_candidate(S, F, gp, gsn, mk3(dr.x, dr.y, dr.z), col(fr.x, fr.y, fr.z), fr.w, dr.w != 0.0f, found, h,
                                   env_p, nl, nb, r, rng);
            n_cl++;
        }
        r.UCW = r.wsum == 0.0f ? 0.0f : 1.0f / r.target * r.wsum;   // end()
        r.M = 1;
        if (F.options.restir_di_do_visibility_reuse && r.UCW > 0.0f && !(r.flags & RF_UNOCCLUDED)) {
            const v3 sp = gp + gsn * 1.0e-4f;
            TgtRay ray;
            ray.o = sp;
            if (r.flags & RF_ENVMAP) { ray.d = mat_x_vec(w.envmap_to_world_matrix.m, r.point); ray.dist = 1.0e35f; }
            else { v3 dir = r.point - sp; ray.dist = length(dir); ray.d = dir / ray.dist; }
            // (a chunk's item: its sample's frame and the frame pixel, as k_restir_initial)
            const MptFrame& Fs = P.ci_n ? Fp[s / P.ci_n] : F;
            const uint32_t fpix = (uint32_t)(P.ci_n ? s % P.ci_n + P.ci_pix_off : pix);
            rs_stage_ray(P, id, ray, P.gb_meta[pix].x,
                         F.render_settings.do_alpha_testing ? alpha_key(pass_seed(Fs, fpix, Fs.restir_di_seeds[1]), 0, 5,
                                                                        RP_VISREUSE)
                                                            : 0u);
            vbits |= 1u << kk;
            n_any++;
        }
        rr_store(P.rs_init, pix, r);
    }
    }
    {   // the visibility-reuse rays (position 0 of their slots) to the CTR_RQV list
        int tot;
        const int off = rs_block_scan(__popc(vbits), tmp, tot);
        if (threadIdx.x == 0) sbase = tot ? atomicAdd(&P.counters[CTR_RQV], tot) : 0;
        __syncthreads();
        int o = sbase + off;
        for (uint32_t m = vbits; m; m &= m - 1u) P.rq_list[o++] = (s0 + __builtin_ctz(m) * TB) * RS_RPP;
    }
    int ta, tc;
    (void)rs_block_scan((int)n_any, tmp, ta);
    (void)rs_block_scan((int)n_cl, tmp, tc);
    if (threadIdx.x == 0) {
        if (ta) atomicAdd((unsigned long long*)&P.ray_counts[1], (unsigned long long)ta);
        if (tc) atomicAdd((unsigned long long*)&P.ray_counts[2], (unsigned long long)tc);
    }
}
#endif

// find_temporal_neighbor_index (Utils.h:371-421)
DEV int restir_temporal_neighbor(const DevScene& S, const DevPaths& P, const MptFrame& F, v3 p, v3 n, const Mat& cm,
                                 Rng& rng, int& px, int& py) {
    const MptReSTIRDISettings& rd = F.render_settings.restir_di_settings;
    int W = F.res_x, H = F.res_y;
    float fx, fy;
    restir_reproject(F, p, fx, fy);
    int idx = -1;
    bool use_prev = rd.do_temporal_reuse_pass;
    for (int i = 0; i < rd.max_neighbor_search_count + 1; i++) {
        float ox = 0.0f, oy = 0.0f;
        if (i > 0) {
            float a = rng() - 0.5f, b = rng() - 0.5f;
            ox = a * (float)rd.neighbor_search_radius;
            oy = b * (float)rd.neighbor_search_radius;
        }
        int qx = (int)roundf(fx + ox), qy = (int)roundf(fy + oy);
        if (rd.use_permutation_sampling && i == 0) {
            int bits = rd.permutation_sampling_random_bits;
            int ax = bits & 3, ay = (bits >> 2) & 3;
            qx += ax; qy += ay;
            qx ^= 3; qy ^= 3;
            qx -= ax; qy -= ay;
        }
        if (qx < 0 || qx >= W || qy < 0 || qy >= H) continue;
        idx = qx + qy * W;
        if (restir_similar(S, P, rd, idx, cm, p, n, use_prev)) break;
        idx = -1;
    }
    px = (int)roundf(fx);
    py = (int)roundf(fy);
    return idx;
}

// ---- ReSTIR_DI_SpatiotemporalReuse (FusedSpatiotemporalReuse.h:112-586) ----------------
// BM: the bias-correction mode compiled in (MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE with
// visibility, the reference default) or -1 = read it from the frame (every mode)
template <int OVR, int BM>
RESTIR_KERNEL void k_restir_spatiotemporal(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    __shared__ uint2 lds[LDS_STACK * TB];
    const MptFrame& F = *Fp;
    const BCtx bc = make_bctx(S, F);
    RRays rr{&S, lds, P.stack_spill + ((size_t)blockIdx.x * TB + threadIdx.x) * (2 * SPILL_DEPTH),
             F.render_settings.do_alpha_testing, 0u, 6, 0, 0u, 0u};
    const int W = F.res_x;
    float4* tin = P.rs_tin;
    for (int s = blockIdx.x * TB + threadIdx.x; s < P.n; s += gridDim.x * TB) {
        const int center = s + P.pix_off;
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = 0;   // configure_spatial_pass_for_fused_spatiotemporal(0)
        if (!P.active[s] || !P.gb_meta[center].z) continue;
        uint32_t seed = pass_seed(F, (uint32_t)center, F.restir_di_seeds[2]);
        Rng rng = make_rng(seed);
        rr.pseed = seed;
        rr.n = 0;
        RSurf cs = gb_surface(S, P, center, false);
        if (is_emissive(*cs.m)) continue;
        if (rd.temporal_buffer_clear_requested) rr_store(tin, center, rr_default());
        const bool use_prev = rd.do_temporal_reuse_pass;
        int tpx, tpy;
        int tidx = restir_temporal_neighbor(S, P, F, cs.p, cs.sn, *cs.m, rng, tpx, tpy);
        RResv tres = rr_default();
        tres.tri = -1;
        if (tidx != -1 && !F.render_settings.freeze_random) tres = rr_load(tin, tidx);
        if ((tidx == -1 || tres.M <= 1) && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
        float rot = rd.do_neighbor_rotation ? TWO_PI * rng() : 0.0f;
        float cr = pcos(rot), sr = psin(rot);
        const int reuse = rd.reuse_neighbor_count;
        int cache = 0, vcount = 0, vM = 0;
        for (int k = 0; k < reuse; k++) {
            int ni = restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, tpx, tpy, cr, sr, F.restir_di_seeds[2]);
            if (ni == -1) continue;
            if (!restir_similar(S, P, rd, ni, *cs.m, cs.sp, cs.sn, use_prev)) continue;
            vM += rr_load(tin, ni).M;
            vcount++;
            cache |= 1 << k;
        }
        const bool temporal_ok = tidx != -1 && tres.M > 0;
        if (temporal_ok) { vcount++; vM += tres.M; }
        RResv o = rr_default();
        const RResv ic = rr_load(P.rs_init, center);
        const int mode = BM >= 0 ? BM : F.options.restir_di_bias_correction_weights;
        const bool bvis = BM >= 0 ? true : F.options.restir_di_bias_correction_use_visibility != 0;
        const bool cw = rd.use_confidence_weights;
        PairwiseMIS mis{0.0f, mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE, bvis};
        // the temporal neighbour's surface as load_temporal_neighbor_data leaves it: loaded when
        // its reservoir is not empty, else a default ReSTIRDISurface (zero normals: target 0)
        RSurf ts;
        if (temporal_ok) ts = gb_surface(S, P, tidx, use_prev);
        else { ts = cs; ts.m = &g_zero_mat; ts.sn = ts.gn = ts.view = ts.sp = ts.p = mk3(0.0f, 0.0f, 0.0f); }
        // neighbours around the temporal position (center included, j == reuse) visited by the
        // GBH weight / normalisation loops (SpatiotemporalMISWeight.h, SpatiotemporalNormalizationWeight.h)
        auto valid_nb = [&](int j) -> int {
            if (j == reuse) return center;
            int nj = restir_spatial_neighbor(P, F, j, reuse, rd.reuse_radius, tpx, tpy, cr, sr, F.restir_di_seeds[2]);
            if (nj == -1) return -1;
            return restir_similar(S, P, rd, nj, *cs.m, cs.sp, cs.sn, use_prev) ? nj : -1;
        };
        // ReSTIRDISpatiotemporalResamplingMISWeight<MIS_GBH>: current = 0 temporal, k + 1 spatial k
        auto gbh = [&](const RResv& r, int current) -> float {
            if (r.UCW <= 0.0f) return 1.0f;
            float nume = 0.0f, denom = 0.0f;
            for (int j = 0; j < reuse + 1; j++) {
                int nj = valid_nb(j);
                if (nj == -1) continue;
                RSurf js = j == reuse ? cs : gb_surface(S, P, nj, use_prev);
                float tj = restir_target(S, F, bc, rr.at(RP_GBH(current, j)), r.tri, r.point, r.flags, js, bvis, OVR);
                int M = 1;
                if (cw) M = j == reuse ? ic.M : rr_load(tin, nj).M;
                denom += tj * (float)M;
                if (j + 1 == current) nume = tj * (float)M;
            }
            float tt = restir_target(S, F, bc, rr.at(RP_GBH(current, 999)), r.tri, r.point, r.flags, ts, bvis, OVR);
            int M = cw ? tres.M : 1;
            denom += tt * (float)M;
            if (current == 0) nume = tt * (float)M;
            return denom == 0.0f ? 0.0f : nume / denom;
        };
        int selected = 0;   // MIS-like: 0 temporal, k + 1 spatial k
        if (temporal_ok) {
            float tfc = 0.0f;
            if (tres.UCW > 0.0f) tfc = restir_target(S, F, bc, rr.at(RP_T_TFC), tres.tri, tres.point, tres.flags, cs, bvis, OVR);
            float jac = 1.0f;
            if (tfc > 0.0f && tres.UCW > 0.0f && !(tres.flags & RF_ENVMAP)) {
                jac = restir_jacobian(S, tres, cs.sp, ts.sp - ts.sn * 1.0e-4f);
                if (jac == -1.0f) jac = 0.0f;
            }
            float wgt;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wgt = (float)tres.M;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wgt = cw ? (float)tres.M : 1.0f;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) wgt = gbh(tres, 0);
            else {
                bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
                wgt = mis.weight(S, F, bc, rr.at(RP_T_TCN), rd, tres, ic, tfc, ts, vcount, vM, update_mc, false, OVR);
            }
            if (rr_combine(o, tres, wgt, tfc, jac, rng)) {
                selected = 0;
                if (bvis) o.flags |= RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        int start = vM == 0 ? reuse : 0;
        for (int k = start; k < reuse + 1; k++) {
            if (k < reuse && reuse <= 32 && (cache & (1 << k)) == 0) continue;
            int ni = k == reuse ? center : restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, tpx, tpy, cr, sr, F.restir_di_seeds[2]);
            if (ni == -1) continue;
            if (k < reuse && reuse > 32 && !restir_similar(S, P, rd, ni, *cs.m, cs.sp, cs.sn, use_prev)) continue;
            RResv nr = k == reuse ? ic : rr_load(tin, ni);
            float tfc = 0.0f;
            bool vis = spatial_visibility(F, rd, k, reuse);
            if (nr.UCW > 0.0f) {
                if (k == reuse) tfc = nr.target;
                else tfc = restir_target(S, F, bc, rr.at(RP_TFC(k)), nr.tri, nr.point, nr.flags, cs, vis, OVR);
            }
            float jac = 1.0f;
            if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
                RSurf ns = gb_surface(S, P, ni, use_prev);
                jac = restir_jacobian(S, nr, cs.sp, ns.sp);
                if (jac == -1.0f) { o.M += nr.M; continue; }
            }
            float wgt;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wgt = (float)nr.M;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wgt = cw ? (float)nr.M : 1.0f;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) wgt = gbh(nr, k + 1);
            else {
                bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
                if (nr.UCW == 0.0f && !update_mc) wgt = 1.0f;
                else {
                    RSurf ns = gb_surface(S, P, ni, use_prev);
                    wgt = mis.weight(S, F, bc, rr.at(RP_TCN(k)), rd, nr, ic, tfc, ns, vcount, vM, update_mc, k == reuse, OVR);
                }
            }
            if (rr_combine(o, nr, wgt, tfc, jac, rng)) {
                selected = k + 1;
                if (vis) o.flags |= RF_UNOCCLUDED;
                else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        // normalisation (SpatiotemporalNormalizationWeight.h)
        float nn = 1.0f, nd = 1.0f;
        if (o.wsum > 0.0f && (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z ||
                              mode == MPT_RESTIR_DI_BIAS_MIS_LIKE)) {
            nn = mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? 0.0f : 1.0f;
            nd = 0.0f;
            for (int j = 0; j < reuse + 1; j++) {
                int nj = valid_nb(j);
                if (nj == -1) continue;
                if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) {
                    nd += (float)(j == reuse ? ic.M : rr_load(tin, nj).M);
                    continue;
                }
                // the MIS-like loop reads the current frame's G-buffer (SpatiotemporalNormalizationWeight.h:130)
                RSurf js = j == reuse ? cs : gb_surface(S, P, nj, mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? false : use_prev);
                float tj = restir_target(S, F, bc, rr.at(RP_NORM(j)), o.tri, o.point, o.flags, js, bvis, OVR);
                if (tj > 0.0f) {
                    if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) nd += (float)(j == reuse ? ic.M : rr_load(tin, nj).M);
                    else {
                        int M = 1;
                        if (cw) M = j == reuse ? ic.M : rr_load(tin, nj).M;
                        if (j + 1 == selected) nn += tj;
                        nd += tj * (float)M;
                    }
                }
            }
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) nd += (float)tres.M;
            else {
                float tt = restir_target(S, F, bc, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis, OVR);
                if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) { if (tt > 0.0f) nd += (float)tres.M; }
                else {
                    if (selected == 0) nn += tt;
                    nd += tt * (float)(cw ? tres.M : 1);
                }
            }
        }
        rr_end_norm(o, nn, nd);
        const bool vreuse = bvis && (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z || mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS ||
                                     mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE) &&
                            (F.options.restir_di_do_visibility_reuse ||
                             (F.options.restir_di_initial_target_visibility && F.options.restir_di_spatial_target_visibility));
        if (vreuse && (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index))
            restir_visibility_reuse(F, rr, o, cs.sp, cs.last);
        if (rd.m_cap > 0) o.M = imin(o.M, rd.m_cap);
        rr_store(P.rs_out, center, o);
    }
    count_pass_rays(P, rr.n_any, rr.n_closest);
}

// ---- ReSTIR_DI_TemporalReuse (TemporalReuse.h:48-306), the non-fused chain ---------------
// Pairwise-MIS-defensive weights (TemporalMISWeight.h:203-279), normalisation 1 / 1
// (TemporalNormalizationWeight.h), visibility in the target function (BiasCorrectionUseVisibility).
template <int OVR>
RESTIR_KERNEL void k_restir_temporal(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, const float4* __restrict__ tin_c,
                                     float4* out) {
    __shared__ uint2 lds[LDS_STACK * TB];
    const MptFrame& F = *Fp;
    const BCtx bc = make_bctx(S, F);
    RRays rr{&S, lds, P.stack_spill + ((size_t)blockIdx.x * TB + threadIdx.x) * (2 * SPILL_DEPTH),
             F.render_settings.do_alpha_testing, 0u, 8, 0, 0u, 0u};
    float4* tin = const_cast<float4*>(tin_c);
    const MptReSTIRDISettings& rd = F.render_settings.restir_di_settings;
    const int mode = F.options.restir_di_bias_correction_weights;
    const bool bvis = F.options.restir_di_bias_correction_use_visibility != 0;
    const bool cw = rd.use_confidence_weights;
    for (int s = blockIdx.x * TB + threadIdx.x; s < P.n; s += gridDim.x * TB) {
        const int center = s + P.pix_off;
        if (!P.active[s] || !P.gb_meta[center].z) continue;
        uint32_t seed = pass_seed(F, (uint32_t)center, F.restir_di_seeds[2]);
        Rng rng = make_rng(seed);
        rr.pseed = seed;
        rr.n = 0;
        if (rd.temporal_buffer_clear_requested) rr_store(tin, center, rr_default());
        RSurf cs = gb_surface(S, P, center, false);
        if (is_emissive(*cs.m)) continue;
        const bool use_prev = rd.do_temporal_reuse_pass;   // use_prev_frame_g_buffer (RenderSettings.h:237-247)
        int tpx, tpy;
        int tidx = restir_temporal_neighbor(S, P, F, cs.p, cs.sn, *cs.m, rng, tpx, tpy);
        const RResv ic = rr_load(P.rs_init, center);
        if (tidx == -1 || F.render_settings.freeze_random) { rr_store(out, center, ic); continue; }
        const RResv tres = rr_load(tin, tidx);
        if (tres.M == 0) { rr_store(out, center, ic); continue; }
        RSurf ts = gb_surface(S, P, tidx, use_prev);
        if (is_emissive(*ts.m)) { rr_store(out, center, ic); continue; }
        RResv o = rr_default();
        float mc = 0.0f;
        int selected = 0;   // MIS-like: TEMPORAL_NEIGHBOR_ID 0 / INITIAL_CANDIDATES_ID 1
        // GBH weight of a reservoir's sample between the temporal neighbour and the center (TemporalMISWeight.h:62-110)
        auto gbh = [&](const RResv& r, bool temporal_id) -> float {
            const int cur = temporal_id ? 0 : 1;
            float tt = restir_target(S, F, bc, rr.at(RP_GBH(cur, 999)), r.tri, r.point, r.flags, ts, bvis, OVR);   // temporal M != 0 here
            if (temporal_id && tt == 0.0f) return 0.0f;
            float tc = restir_target(S, F, bc, rr.at(RP_GBH(cur, 998)), r.tri, r.point, r.flags, cs, bvis, OVR);
            int tM = cw ? tres.M : 1, cM = cw ? ic.M : 1;
            float nume = temporal_id ? tt * (float)tM : tc * (float)cM;
            float denom = tt * (float)tM + tc * (float)cM;
            return denom == 0.0f ? 0.0f : nume / denom;
        };
        {
            float tfc = 0.0f;
            if (tres.UCW > 0.0f) tfc = restir_target(S, F, bc, rr.at(RP_T_TFC), tres.tri, tres.point, tres.flags, cs, bvis, OVR);
            float jac = 1.0f;
            if (tfc > 0.0f && tres.UCW > 0.0f && !(tres.flags & RF_ENVMAP)) {
                jac = restir_jacobian(S, tres, cs.sp, ts.sp - ts.sn * 1.0e-4f);
                if (jac == -1.0f) jac = 0.0f;
            }
            float wgt;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wgt = (float)tres.M;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wgt = cw ? (float)tres.M : 1.0f;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) wgt = gbh(tres, true);
            else {
                // pairwise (TemporalMISWeight.h:139-279): TEMPORAL_NEIGHBOR_ID
                const bool def = mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE;
                float tM = cw ? (float)tres.M : 1.0f, cM = cw ? (float)ic.M : 1.0f, nsum = cw ? (float)tres.M : 1.0f;
                float tfn = tres.target;
                float nume = tfn * tM;
                float denom = tfn * nsum + tfc * cM;
                float mi = denom == 0.0f ? 0.0f : (nume / denom);
                if (def && cw) mi *= nsum / (nsum + cM);
                float tcn = restir_target(S, F, bc, rr.at(RP_T_TCN), ic.tri, ic.point, ic.flags, ts, bvis, OVR);
                float tcc = ic.target;
                float nume_mc = tcc * cM;
                float denom_mc = tcn * nsum + tcc * cM;
                float conf = cw ? (def ? nsum / (nsum + cM) : tM / nsum) : 1.0f;
                if (denom_mc != 0.0f) mc += nume_mc / denom_mc * conf;
                wgt = def && !cw ? mi * 0.5f : mi;
            }
            if (rr_combine(o, tres, wgt, tfc, jac, rng)) {
                selected = 0;
                if (bvis) o.flags |= RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        // the initial candidates (INITIAL_CANDIDATES_ID)
        float wc;
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wc = (float)ic.M;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wc = cw ? (float)ic.M : 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) wc = gbh(ic, false);
        else if (mc == 0.0f) wc = 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS) wc = mc;
        else if (cw) wc = mc + (float)ic.M / (float)(ic.M + tres.M);
        else wc = (1.0f + mc) * 0.5f;
        if (rr_combine(o, ic, wc, ic.target, 1.0f, rng)) {
            selected = 1;
            if (bvis) o.flags |= RF_UNOCCLUDED;
            else o.flags |= ic.flags & RF_UNOCCLUDED;
        }
        // normalisation (TemporalNormalizationWeight.h)
        float nn = 1.0f, nd = 1.0f;
        if (o.wsum > 0.0f) {
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) nd = (float)(ic.M + tres.M);
            else if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) {
                nd = 0.0f;
                float tc = restir_target(S, F, bc, rr.at(RP_NORM(998)), o.tri, o.point, o.flags, cs, bvis, OVR);
                nd += (float)((tc > 0.0f) * ic.M);
                float tt = restir_target(S, F, bc, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis, OVR);   // temporal M > 0
                nd += (float)((tt > 0.0f) * tres.M);
            } else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) {
                float tc = restir_target(S, F, bc, rr.at(RP_NORM(998)), o.tri, o.point, o.flags, cs, bvis, OVR);
                float tt = restir_target(S, F, bc, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis, OVR);
                nn = selected == 1 ? tc : tt;
                int icM = cw ? ic.M : 1, tM = cw ? tres.M : 1;
                nd = tc * (float)icM + tt * (float)tM;
            }
        }
        rr_end_norm(o, nn, nd);
        if (rd.m_cap > 0) o.M = imin(o.M, rd.m_cap);
        rr_store(out, center, o);
    }
    count_pass_rays(P, rr.n_any, rr.n_closest);
}

// ---- ReSTIR_DI_SpatialReuse (SpatialReuse.h:52-348) ------------------------------------
template <int OVR, int BM>
RESTIR_KERNEL void k_restir_spatial(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int pass,
                                    const float4* __restrict__ in, float4* out) {
    __shared__ uint2 lds[LDS_STACK * TB];
    const MptFrame& F = *Fp;
    const BCtx bc = make_bctx(S, F);
    RRays rr{&S, lds, P.stack_spill + ((size_t)blockIdx.x * TB + threadIdx.x) * (2 * SPILL_DEPTH),
             F.render_settings.do_alpha_testing, 0u, 7, 0, 0u, 0u};
    const int W = F.res_x;
    const uint32_t pass_rs = F.restir_di_seeds[4 + pass];
    const int mode = BM >= 0 ? BM : F.options.restir_di_bias_correction_weights;
    const bool bvis = BM >= 0 ? true : F.options.restir_di_bias_correction_use_visibility != 0;
    for (int s = blockIdx.x * TB + threadIdx.x; s < P.n; s += gridDim.x * TB) {
        const int center = s + P.pix_off;
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = pass;
        if (!P.active[s] || !P.gb_meta[center].z) continue;
        uint32_t seed = pass_seed(F, (uint32_t)center, pass_rs);
        Rng rng = make_rng(seed);
        rr.pseed = seed;
        rr.n = 0;
        const int x = center % W, y = center / W;
        RResv o = rr_default();
        RSurf cs = gb_surface(S, P, center, false);
        if (is_emissive(*cs.m)) continue;
        float rot = rd.do_neighbor_rotation ? TWO_PI * rng() : 0.0f;
        float cr = pcos(rot), sr = psin(rot);
        const RResv cres = rr_load(in, center);
        if (cres.M <= 1 && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
        const int reuse = rd.reuse_neighbor_count;
        const bool cw = rd.use_confidence_weights;
        int cache = 0, vcount = 0, vM = 0;
        for (int k = 0; k < reuse; k++) {
            int ni = restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, x, y, cr, sr, pass_rs);
            if (ni == -1) continue;
            if (!restir_similar(S, P, rd, ni, *cs.m, cs.sp, cs.sn, false)) continue;
            vM += rr_load(in, ni).M;
            vcount++;
            cache |= 1 << k;
        }
        // the neighbours (center included, k == reuse) the normalisation / GBH loops visit
        // (get_spatial_neighbor_pixel_index + check_neighbor_similarity_heuristics)
        auto valid_nb = [&](int j) -> int {
            int nj = restir_spatial_neighbor(P, F, j, reuse, rd.reuse_radius, x, y, cr, sr, pass_rs);
            if (nj == -1) return -1;
            return restir_similar(S, P, rd, nj, *cs.m, cs.sp, cs.sn, false) ? nj : -1;
        };
        PairwiseMIS mis{0.0f, mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE, bvis};
        int selected = 0;   // MIS-like
        int start = vM == 0 ? reuse : 0;
        for (int k = start; k < reuse + 1; k++) {
            if (k < reuse && reuse <= 32 && (cache & (1 << k)) == 0) continue;
            int ni = restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, x, y, cr, sr, pass_rs);
            if (ni == -1) continue;
            if (k < reuse && reuse > 32 && !restir_similar(S, P, rd, ni, *cs.m, cs.sp, cs.sn, false)) continue;
            RResv nr = rr_load(in, ni);
            float tfc = 0.0f;
            bool vis = spatial_visibility(F, rd, k, reuse);
            if (nr.UCW > 0.0f) {
                if (k == reuse) tfc = nr.target;
                else tfc = restir_target(S, F, bc, rr.at(RP_TFC(k)), nr.tri, nr.point, nr.flags, cs, vis, OVR);
            }
            float jac = 1.0f;
            if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
                float4 np = P.gb_pos[ni];
                jac = restir_jacobian(S, nr, cs.sp, mk3(np.x, np.y, np.z));
                if (jac == -1.0f) { o.M += nr.M; continue; }
            }
            float wgt;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wgt = (float)nr.M;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wgt = cw ? (float)nr.M : 1.0f;
            else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) {
                // SpatialMISWeight.h:36-93
                if (nr.UCW <= 0.0f) wgt = 1.0f;
                else {
                    float nume = 0.0f, denom = 0.0f;
                    for (int j = 0; j < reuse + 1; j++) {
                        int nj = valid_nb(j);
                        if (nj == -1) continue;
                        RSurf js = gb_surface(S, P, nj, false);
                        float tj = restir_target(S, F, bc, rr.at(RP_GBH(k, j)), nr.tri, nr.point, nr.flags, js, bvis, OVR);
                        int M = cw ? rr_load(in, nj).M : 1;
                        denom += tj * (float)M;
                        if (j == k) nume = tj * (float)M;
                    }
                    wgt = denom == 0.0f ? 0.0f : nume / denom;
                }
            } else {
                bool update_mc = cres.M > 0 && cres.UCW > 0.0f;
                RSurf ns = gb_surface(S, P, ni, false);
                wgt = mis.weight(S, F, bc, rr.at(RP_TCN(k)), rd, nr, cres, tfc, ns, vcount, vM, update_mc, k == reuse, OVR);
            }
            if (rr_combine(o, nr, wgt, tfc, jac, rng)) {
                selected = k;
                if (vis) o.flags |= RF_UNOCCLUDED;
                else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        // normalisation (SpatialNormalizationWeight.h)
        float nn = 1.0f, nd = 1.0f;
        if (o.wsum > 0.0f && (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z ||
                              mode == MPT_RESTIR_DI_BIAS_MIS_LIKE)) {
            nn = mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? 0.0f : 1.0f;
            nd = 0.0f;
            for (int j = 0; j < reuse + 1; j++) {
                int nj = valid_nb(j);
                if (nj == -1) continue;
                if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) { nd += (float)rr_load(in, nj).M; continue; }
                RSurf js = gb_surface(S, P, nj, false);
                float tj = restir_target(S, F, bc, rr.at(RP_NORM(j)), o.tri, o.point, o.flags, js, bvis, OVR);
                if (tj > 0.0f) {
                    int M = rr_load(in, nj).M;
                    if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) nd += (float)M;
                    else {
                        if (!cw) M = 1;
                        if (j == selected) nn += tj;
                        nd += tj * (float)M;
                    }
                }
            }
        }
        rr_end_norm(o, nn, nd);
        const bool vreuse = bvis && (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z || mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS ||
                                     mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE) &&
                            (F.options.restir_di_do_visibility_reuse ||
                             (F.options.restir_di_initial_target_visibility && F.options.restir_di_spatial_target_visibility));
        if (vreuse && (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index))
            restir_visibility_reuse(F, rr, o, cs.sp, cs.last);
        if (rd.m_cap > 0) o.M = imin(o.M, rd.m_cap);
        rr_store(out, center, o);
    }
    count_pass_rays(P, rr.n_any, rr.n_closest);
}

// ---- staged spatial reuse (the reference-default weights) -----------------------------
// k_restir_spatial traces its visibility rays inline, inside a kernel whose BSDF evaluations
// hold every register (256 VGPRs and scratch spills at 2 waves / SIMD), so the traversal
// runs slowly and lanes wait on each other's rays.  The staged pass splits it into
// material-sorted stages:
//  * k_rsp_select (per pixel, no BSDF code): the neighbour selection, the similarity tests,
//    each neighbour's reservoir and Jacobian, and the target-function evaluations the pass
//    needs -- neighbour k's sample at the center (TFC) and the canonical sample at neighbour k
//    (TCN) -- appended as items to the plain-dielectric list or the generic list by the
//    material class of the surface they are evaluated at (as k_split sorts the shading);
//  * k_rsp_eval<PLAIN> per list: the unoccluded target function (dev_bsdf.h FULL = false for
//    the plain list) and the visibility ray the monolithic kernel would trace, staged at the
//    item's position (pixel slot, 2k + which);
//  * k_trace<TM_LIST_ANY> over the staged rays (persistent, chunked, LDS stack);
//  * k_rsp_combine: the resampling from the stored values and the occlusion bytes, with the
//    RNG draws of the monolithic kernel; the visibility-reuse ray of the result is staged
//    again, traced, and applied by k_rs_visapply.
// Alpha keys are positional (RP_*), so a staged ray has the key the monolithic kernel gives
// it, including the bias-correction ray of a neighbour that a Jacobian rejection then drops
// (staged and traced, never used).
constexpr uint32_t RSE_VIS = 0x80000000u;   // eval item flag: the target is evaluated with visibility

// appends items (positions in `mask` of slot s, flags per position) to the two class lists
DEV void rs_append_items(const DevPaths& P, int s, uint32_t m_plain, uint32_t m_gen, uint32_t vis_bits, uint32_t prev_bits,
                         int* tmp, int* base) {
    for (int c = 0; c < 2; c++) {
        uint32_t mask = c == 0 ? m_plain : m_gen;
        int tot;
        const int off = rs_block_scan(__popc(mask), tmp, tot);
        if (threadIdx.x == 0) *base = tot ? atomicAdd(&P.counters[CTR_RQE0 + c], tot) : 0;
        __syncthreads();
        int32_t* list = P.rq_items + (size_t)c * P.n * RS_RPP;
        int o = *base + off;
        while (mask) {
            const int j = __builtin_ctz(mask);
            mask &= mask - 1u;
            list[o++] = (s * RS_RPP + j) | (((vis_bits >> j) & 1u) ? (int)RSE_VIS : 0) | (((prev_bits >> j) & 1u) ? (int)RSE_PREV : 0);
        }
        __syncthreads();
    }
}

template <int OVR>
__global__ __launch_bounds__(TB) void k_rsp_select(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int pass,
                                                   const float4* __restrict__ in) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    const int W = F.res_x;
    const uint32_t pass_rs = F.restir_di_seeds[4 + pass];
    const int s = xcd_block() * TB + threadIdx.x;
    uint32_t m_plain = 0u, m_gen = 0u, vis_bits = 0u;   // items by position (2k + which)
    if (s < P.n) {
        const int center = s + P.pix_off;
        int4 meta = make_int4(RSM_SKIP, 0, 0, 0);
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = pass;
        if (P.active[s] && P.gb_meta[center].z) {
            Rng rng = make_rng(pass_seed(F, (uint32_t)center, pass_rs));
            const RSurf cs = gb_surface(S, P, center, false);
            if (!is_emissive(*cs.m)) {
                const int x = center % W, y = center / W;
                float cr = 1.0f, sr = 0.0f;
                if (rd.do_neighbor_rotation) {
                    const float2 sc = psincos(TWO_PI * rng());
                    sr = sc.x;
                    cr = sc.y;
                }
                const RResv cres = rr_load(in, center);
                if (cres.M <= 1 && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
                const int reuse = rd.reuse_neighbor_count;
                int cache = 0, vcount = 0, vM = 0;
                int nis[RS_KMAX];
                for (int k = 0; k < reuse; k++) {
                    nis[k] = restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, x, y, cr, sr, pass_rs);
                    if (nis[k] == -1) continue;
                    if (!restir_similar(S, P, rd, nis[k], *cs.m, cs.sp, cs.sn, false)) continue;
                    vM += rr_load(in, nis[k]).M;
                    vcount++;
                    cache |= 1 << k;
                }
                meta = make_int4(0, cache, vM, vcount);
                const bool update_mc = cres.M > 0 && cres.UCW > 0.0f;
                const bool c_plain = OVR == MPT_BSDF_NONE && rs_plain(S, P, center, cs);
                for (int k = 0; k < reuse && vM != 0; k++) {
                    if (!((cache >> k) & 1)) continue;
                    const int ni = nis[k];
                    const RResv nr = rr_load(in, ni);
                    float jac = 1.0f;
                    if (nr.UCW > 0.0f) {
                        (c_plain ? m_plain : m_gen) |= 1u << (2 * k);
                        if (spatial_visibility(F, rd, k, reuse)) vis_bits |= 1u << (2 * k);
                        // used only when the target turns out positive (the monolithic kernel's order)
                        if (!(nr.flags & RF_ENVMAP)) {
                            const float4 np = P.gb_pos[ni];
                            jac = restir_jacobian(S, nr, cs.sp, mk3(np.x, np.y, np.z));
                        }
                    }
                    if (update_mc) {
                        const bool n_plain = OVR == MPT_BSDF_NONE && rs_plain(S, P, ni, gb_surface(S, P, ni, false));
                        (n_plain ? m_plain : m_gen) |= 1u << (2 * k + 1);
                        vis_bits |= 1u << (2 * k + 1);   // ReSTIR_DI_BiasCorrectionUseVisibility
                    }
                    P.rq_rec[rq_rec_at(P, s, k)] = make_float4(__int_as_float(ni), 0.0f, 0.0f, jac);
                }
            }
        }
        P.rq_meta[s] = meta;
    }
    // item lists: plain at [0, n * RS_RPP), generic at [n * RS_RPP, 2 n * RS_RPP)
    rs_append_items(P, s, m_plain, m_gen, vis_bits, 0u, tmp, &base);
}

// One target-function evaluation per item of a class list (count in the device counter);
// grid-stride with a block-uniform trip count (the block appends its rays each round).
// FUSED: an item of the fused spatiotemporal pass (positions 0 / 1: the temporal neighbour,
// record RS_KMAX; 2 + 2k + which: spatial neighbour k; the canonical sample is the initial
// candidates' reservoir), else of a spatial pass.
template <int OVR, bool PLAIN, bool FUSED>
RESTIR_KERNEL void k_rsp_eval(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int pass, const float4* __restrict__ in,
                              const int32_t* __restrict__ items, const int32_t* __restrict__ count_ptr) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    const BCtx bc = make_bctx(S, F);
    const uint32_t pass_rs = FUSED ? F.restir_di_seeds[2] : F.restir_di_seeds[4 + pass];
    const bool alpha = F.render_settings.do_alpha_testing;
    const int count = *count_ptr;
    // the plain-class evaluation counter (ray_counts[5]: MptStats::restir_eval_items), added here
    // instead of by a launch of its own
    if (PLAIN && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd((unsigned long long*)(P.ray_counts + 5), (unsigned long long)(uint32_t)count);
    for (int b0 = blockIdx.x * TB; b0 < count; b0 += gridDim.x * TB) {
        const int i = b0 + (int)threadIdx.x;
        uint32_t rmask = 0u;
        int s = 0;
        if (i < count) {
            const uint32_t it = (uint32_t)items[i];
            const bool vis = (it & RSE_VIS) != 0, prev = (it & RSE_PREV) != 0;
            const int id = (int)(it & ~(RSE_VIS | RSE_PREV));
            s = id / RS_RPP;
            const int j = id - s * RS_RPP;
            const bool temporal = FUSED && j < 2;
            const int jj = FUSED ? (temporal ? j : j - 2) : j;
            const int k = temporal ? RS_KMAX : jj >> 1, which = jj & 1;
            const int center = s + P.pix_off;
            float* rec = reinterpret_cast<float*>(&P.rq_rec[rq_rec_at(P, s, k)]);
            const int ni = __float_as_int(rec[0]);
            const RSurf g = (PLAIN && MPT_RESTIR_CS) ? gb_csurf(S, P, which ? ni : center, which && prev)
                                                     : gb_surface(S, P, which ? ni : center, which && prev);
            const RResv smp = which ? rr_load(FUSED ? P.rs_init : in, center) : rr_load(in, ni);
            TgtRay ray;
            float t;
            if (PLAIN) t = restir_target_unocc<true>(S, F, bc, smp.tri, smp.point, smp.flags, g, vis, OVR, ray);
            else t = restir_target_unocc<false>(S, F, bc, smp.tri, smp.point, smp.flags, g, vis, OVR, ray);
            rec[1 + which] = t;
            if (vis && t > 0.0f) {
                const int pos = temporal ? (which ? RP_T_TCN : RP_T_TFC) : (which ? RP_TCN(k) : RP_TFC(k));
                const uint32_t key = alpha ? alpha_key(pass_seed(F, (uint32_t)center, pass_rs), 0, FUSED ? 6 : 7, pos) : 0u;
                rs_stage_ray(P, (size_t)id, ray, g.last, key);
                rmask = 1u << j;
            }
        }
        rs_append(P, &P.counters[CTR_RQ], s, rmask, tmp, &base);
        __syncthreads();
    }
}

template <int OVR>
RESTIR_KERNEL void k_rsp_combine(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int pass, const float4* __restrict__ in,
                                 float4* out) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    const uint32_t pass_rs = F.restir_di_seeds[4 + pass];
    const bool alpha = F.render_settings.do_alpha_testing;
    const int s = xcd_block() * TB + threadIdx.x;
    uint32_t vmask = 0u, n_any = 0u;
    if (s < P.n && !(P.rq_meta[s].x & RSM_SKIP)) {
        const int4 meta = P.rq_meta[s];
        const int center = s + P.pix_off;
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = pass;
        const uint32_t seed = pass_seed(F, (uint32_t)center, pass_rs);
        Rng rng = make_rng(seed);
        if (rd.do_neighbor_rotation) (void)rng();   // the neighbour rotation (used by k_rsp_select)
        const RResv cres = rr_load(in, center);
        if (cres.M <= 1 && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
        const int reuse = rd.reuse_neighbor_count;
        const int cache = meta.y, vM = meta.z, vcount = meta.w;
        const bool update_mc = cres.M > 0 && cres.UCW > 0.0f;
        RResv o = rr_default();
        PairwiseMIS mis{0.0f, true, true};
        int ntr = 0;   // rays the monolithic kernel traces (the ray counters)
        const size_t r0 = (size_t)s * RS_RPP;
        for (int k = vM == 0 ? reuse : 0; k < reuse + 1; k++) {
            if (k < reuse && !((cache >> k) & 1)) continue;
            RResv nr;
            float4 rec = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
            if (k == reuse) nr = cres;
            else {
                rec = P.rq_rec[rq_rec_at(P, s, k)];
                nr = rr_load(in, __float_as_int(rec.x));
            }
            const bool vis = spatial_visibility(F, rd, k, reuse);
            float tfc = 0.0f;
            if (nr.UCW > 0.0f) {
                if (k == reuse) tfc = nr.target;
                else {
                    tfc = rec.y;
                    if (vis && tfc > 0.0f) {
                        if (P.rq_occ[rq_phys(P, (int)r0 + 2 * k)]) tfc = 0.0f;
                        ntr++;
                    }
                }
            }
            float jac = 1.0f;
            if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
                jac = rec.w;
                if (jac == -1.0f) {   // (its staged bias-correction ray is not used)
                    o.M += nr.M;
                    continue;
                }
            }
            float tcn = 0.0f;
            if (k != reuse && update_mc) {
                tcn = rec.z;
                if (tcn > 0.0f) {
                    if (P.rq_occ[rq_phys(P, (int)r0 + 2 * k + 1)]) tcn = 0.0f;
                    ntr++;
                }
            }
            const float wgt = mis.weight_tcn(rd, nr, cres, tfc, tcn, vcount, vM, update_mc, k == reuse);
            if (rr_combine(o, nr, wgt, tfc, jac, rng)) {
                if (vis) o.flags |= RF_UNOCCLUDED;
                else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        {
            rr_end_normalized(o);
            const bool vreuse = (F.options.restir_di_do_visibility_reuse ||
                                 (F.options.restir_di_initial_target_visibility && F.options.restir_di_spatial_target_visibility)) &&
                                (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index);
            if (vreuse && o.UCW > 0.0f && !(o.flags & RF_UNOCCLUDED)) {
                // restir_visibility_reuse's ray, staged at position 0 (its first-pass result is consumed)
                const float4 gp = P.gb_pos[center], gs = P.gb_sn[center];
                const v3 sp = mk3(gp.x, gp.y, gp.z) + mk3(gs.x, gs.y, gs.z) * 1.0e-4f;
                TgtRay ray;
                ray.o = sp;
                if (o.flags & RF_ENVMAP) { ray.d = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, o.point); ray.dist = 1.0e35f; }
                else { v3 dir = o.point - sp; ray.dist = length(dir); ray.d = dir / ray.dist; }
                rs_stage_ray(P, r0, ray, P.gb_meta[center].x, alpha ? alpha_key(seed, 0, 7, RP_VISREUSE) : 0u);
                vmask = 1u;
                ntr++;
            }
            if (rd.m_cap > 0) o.M = imin(o.M, rd.m_cap);
            rr_store(out, center, o);
            n_any = (uint32_t)ntr;
        }
    }
    rs_append(P, &P.counters[CTR_RQV], s, vmask, tmp, &base);
    // ray counters: one atomic per block (per wave, 32 k atomics on one word would serialise)
    int tot;
    (void)rs_block_scan((int)n_any, tmp, tot);
    if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&P.ray_counts[1], (unsigned long long)tot);
}

// ---- staged fused spatiotemporal pass (the reference-default weights) -------------------
// As the staged spatial pass: k_rst_select (the temporal neighbour search with its RNG
// draws, the spatial neighbours around the reprojected position, similarity, Jacobians,
// class-sorted evaluation items), k_rsp_eval<PLAIN, FUSED>, the traced list, k_rst_combine.
// Record RS_KMAX holds the temporal neighbour (index, targets, Jacobian), record RS_KMAX + 1
// the RNG state after the neighbour rotation and the reprojected position.
template <int OVR>
__global__ __launch_bounds__(TB) void k_rst_select(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    float4* tin = P.rs_tin;
    const int s = xcd_block() * TB + threadIdx.x;
    uint32_t m_plain = 0u, m_gen = 0u, vis_bits = 0u, prev_bits = 0u;
    if (s < P.n) {
        const int center = s + P.pix_off;
        int4 meta = make_int4(RSM_SKIP, 0, 0, 0);
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = 0;   // configure_spatial_pass_for_fused_spatiotemporal(0)
        if (P.active[s] && P.gb_meta[center].z) {
            Rng rng = make_rng(pass_seed(F, (uint32_t)center, F.restir_di_seeds[2]));
            const RSurf cs = gb_surface(S, P, center, false);
            if (!is_emissive(*cs.m)) {
                const bool use_prev = rd.do_temporal_reuse_pass;
                int tpx, tpy;
                const int tidx = restir_temporal_neighbor(S, P, F, cs.p, cs.sn, *cs.m, rng, tpx, tpy);
                RResv tres = rr_default();
                tres.tri = -1;
                if (tidx != -1 && !F.render_settings.freeze_random) tres = rr_load(tin, tidx);
                if ((tidx == -1 || tres.M <= 1) && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
                float cr = 1.0f, sr = 0.0f;
                if (rd.do_neighbor_rotation) {
                    const float2 sc = psincos(TWO_PI * rng());
                    sr = sc.x;
                    cr = sc.y;
                }
                const int reuse = rd.reuse_neighbor_count;
                int cache = 0, vcount = 0, vM = 0;
                int nis[RS_KMAX];
                for (int k = 0; k < reuse; k++) {
                    nis[k] = restir_spatial_neighbor(P, F, k, reuse, rd.reuse_radius, tpx, tpy, cr, sr, F.restir_di_seeds[2]);
                    if (nis[k] == -1) continue;
                    if (!restir_similar(S, P, rd, nis[k], *cs.m, cs.sp, cs.sn, use_prev)) continue;
                    vM += rr_load(tin, nis[k]).M;
                    vcount++;
                    cache |= 1 << k;
                }
                const bool temporal_ok = tidx != -1 && tres.M > 0;
                if (temporal_ok) { vcount++; vM += tres.M; }
                meta = make_int4(0, cache, vM, vcount);
                const RResv ic = rr_load(P.rs_init, center);
                const bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
                const bool c_plain = OVR == MPT_BSDF_NONE && rs_plain(S, P, center, cs);
                const uint32_t pv = use_prev ? 1u : 0u;
                if (temporal_ok) {
                    float jac = 1.0f;
                    if (tres.UCW > 0.0f) {
                        (c_plain ? m_plain : m_gen) |= 1u << 0;
                        vis_bits |= 1u << 0;   // bias-correction visibility
                        if (!(tres.flags & RF_ENVMAP)) {
                            const RSurf ts = gb_surface(S, P, tidx, use_prev);
                            jac = restir_jacobian(S, tres, cs.sp, ts.sp - ts.sn * 1.0e-4f);
                        }
                    }
                    if (update_mc) {
                        const bool t_plain = OVR == MPT_BSDF_NONE && rs_plain(S, P, tidx, gb_surface(S, P, tidx, use_prev), use_prev);
                        (t_plain ? m_plain : m_gen) |= 1u << 1;
                        vis_bits |= 1u << 1;
                        prev_bits |= pv << 1;
                    }
                    P.rq_rec[rq_rec_at(P, s, RS_KMAX)] = make_float4(__int_as_float(tidx), 0.0f, 0.0f, jac);
                }
                for (int k = 0; k < reuse && vM != 0; k++) {
                    if (!((cache >> k) & 1)) continue;
                    const int ni = nis[k];
                    const RResv nr = rr_load(tin, ni);
                    float jac = 1.0f;
                    if (nr.UCW > 0.0f) {
                        (c_plain ? m_plain : m_gen) |= 1u << (2 + 2 * k);
                        if (spatial_visibility(F, rd, k, reuse)) vis_bits |= 1u << (2 + 2 * k);
                        if (!(nr.flags & RF_ENVMAP)) {
                            const RSurf ns = gb_surface(S, P, ni, use_prev);
                            jac = restir_jacobian(S, nr, cs.sp, ns.sp);
                        }
                    }
                    if (update_mc) {
                        const bool n_plain = OVR == MPT_BSDF_NONE && rs_plain(S, P, ni, gb_surface(S, P, ni, use_prev), use_prev);
                        (n_plain ? m_plain : m_gen) |= 1u << (3 + 2 * k);
                        vis_bits |= 1u << (3 + 2 * k);
                        prev_bits |= pv << (3 + 2 * k);
                    }
                    P.rq_rec[rq_rec_at(P, s, k)] = make_float4(__int_as_float(ni), 0.0f, 0.0f, jac);
                }
                P.rq_rec[rq_rec_at(P, s, RS_KMAX + 1)] = make_float4(__uint_as_float(rng.s), __int_as_float(tidx), 0.0f, 0.0f);
            }
        }
        P.rq_meta[s] = meta;
    }
    rs_append_items(P, s, m_plain, m_gen, vis_bits, prev_bits, tmp, &base);
}

template <int OVR>
RESTIR_KERNEL void k_rst_combine(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp) {
    __shared__ int tmp[TB / 64];
    __shared__ int base;
    const MptFrame& F = *Fp;
    const bool alpha = F.render_settings.do_alpha_testing;
    float4* tin = P.rs_tin;
    const int s = xcd_block() * TB + threadIdx.x;
    uint32_t vmask = 0u, n_any = 0u;
    if (s < P.n && !(P.rq_meta[s].x & RSM_SKIP)) {
        const int4 meta = P.rq_meta[s];
        const int center = s + P.pix_off;
        MptReSTIRDISettings rd = F.render_settings.restir_di_settings;
        rd.spatial_pass_index = 0;
        const float4 st4 = P.rq_rec[rq_rec_at(P, s, RS_KMAX + 1)];
        Rng rng = make_rng(__float_as_uint(st4.x));   // after the temporal search and the rotation
        const int tidx = __float_as_int(st4.y);
        RResv tres = rr_default();
        tres.tri = -1;
        if (tidx != -1 && !F.render_settings.freeze_random) tres = rr_load(tin, tidx);
        if ((tidx == -1 || tres.M <= 1) && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
        const int reuse = rd.reuse_neighbor_count;
        const int cache = meta.y, vM = meta.z, vcount = meta.w;
        const bool temporal_ok = tidx != -1 && tres.M > 0;
        const RResv ic = rr_load(P.rs_init, center);
        const bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
        RResv o = rr_default();
        PairwiseMIS mis{0.0f, true, true};
        int ntr = 0;
        const size_t r0 = (size_t)s * RS_RPP;
        if (temporal_ok) {
            const float4 rec = P.rq_rec[rq_rec_at(P, s, RS_KMAX)];
            float tfc = 0.0f;
            if (tres.UCW > 0.0f) {
                tfc = rec.y;
                if (tfc > 0.0f) {
                    if (P.rq_occ[rq_phys(P, (int)r0)]) tfc = 0.0f;
                    ntr++;
                }
            }
            float jac = 1.0f;
            if (tfc > 0.0f && tres.UCW > 0.0f && !(tres.flags & RF_ENVMAP)) {
                jac = rec.w;
                if (jac == -1.0f) jac = 0.0f;
            }
            float tcn = 0.0f;
            if (update_mc) {
                tcn = rec.z;
                if (tcn > 0.0f) {
                    if (P.rq_occ[rq_phys(P, (int)r0 + 1)]) tcn = 0.0f;
                    ntr++;
                }
            }
            const float wgt = mis.weight_tcn(rd, tres, ic, tfc, tcn, vcount, vM, update_mc, false);
            if (rr_combine(o, tres, wgt, tfc, jac, rng)) o.flags |= RF_UNOCCLUDED;
        }
        for (int k = vM == 0 ? reuse : 0; k < reuse + 1; k++) {
            if (k < reuse && !((cache >> k) & 1)) continue;
            RResv nr;
            float4 rec = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
            if (k == reuse) nr = ic;
            else {
                rec = P.rq_rec[rq_rec_at(P, s, k)];
                nr = rr_load(tin, __float_as_int(rec.x));
            }
            const bool vis = spatial_visibility(F, rd, k, reuse);
            float tfc = 0.0f;
            if (nr.UCW > 0.0f) {
                if (k == reuse) tfc = nr.target;
                else {
                    tfc = rec.y;
                    if (vis && tfc > 0.0f) {
                        if (P.rq_occ[rq_phys(P, (int)r0 + 2 + 2 * k)]) tfc = 0.0f;
                        ntr++;
                    }
                }
            }
            float jac = 1.0f;
            if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
                jac = rec.w;
                if (jac == -1.0f) {   // (its staged bias-correction ray is not used)
                    o.M += nr.M;
                    continue;
                }
            }
            float wgt;
            if (nr.UCW == 0.0f && !update_mc) wgt = 1.0f;
            else {
                float tcn = 0.0f;
                if (k != reuse && update_mc) {
                    tcn = rec.z;
                    if (tcn > 0.0f) {
                        if (P.rq_occ[rq_phys(P, (int)r0 + 3 + 2 * k)]) tcn = 0.0f;
                        ntr++;
                    }
                }
                wgt = mis.weight_tcn(rd, nr, ic, tfc, tcn, vcount, vM, update_mc, k == reuse);
            }
            if (rr_combine(o, nr, wgt, tfc, jac, rng)) {
                if (vis) o.flags |= RF_UNOCCLUDED;
                else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
                else o.flags &= ~RF_UNOCCLUDED;
            }
        }
        rr_end_normalized(o);
        const bool vreuse = (F.options.restir_di_do_visibility_reuse ||
                             (F.options.restir_di_initial_target_visibility && F.options.restir_di_spatial_target_visibility)) &&
                            (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index);
        if (vreuse && o.UCW > 0.0f && !(o.flags & RF_UNOCCLUDED)) {
            const float4 gp = P.gb_pos[center], gs = P.gb_sn[center];
            const v3 sp = mk3(gp.x, gp.y, gp.z) + mk3(gs.x, gs.y, gs.z) * 1.0e-4f;
            TgtRay ray;
            ray.o = sp;
            if (o.flags & RF_ENVMAP) { ray.d = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, o.point); ray.dist = 1.0e35f; }
            else { v3 dir = o.point - sp; ray.dist = length(dir); ray.d = dir / ray.dist; }
            const uint32_t seed = pass_seed(F, (uint32_t)center, F.restir_di_seeds[2]);
            rs_stage_ray(P, r0, ray, P.gb_meta[center].x, alpha ? alpha_key(seed, 0, 6, RP_VISREUSE) : 0u);
            vmask = 1u;
            ntr++;
        }
        if (rd.m_cap > 0) o.M = imin(o.M, rd.m_cap);
        rr_store(P.rs_out, center, o);
        n_any = (uint32_t)ntr;
    }
    rs_append(P, &P.counters[CTR_RQV], s, vmask, tmp, &base);
    int tot;
    (void)rs_block_scan((int)n_any, tmp, tot);
    if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long*)&P.ray_counts[1], (unsigned long long)tot);
}

#ifndef MPT_TU_PART   // k_rs_visapply
// restir_visibility_reuse's outcome for the staged rays: occluded -> UCW = -1, else unoccluded
__global__ __launch_bounds__(TB) void k_rs_visapply(DevPaths P, float4* out) {
    const int i = blockIdx.x * TB + threadIdx.x;
    if (i >= P.counters[CTR_RQV]) return;
    const int id = P.rq_list[i];
    const size_t c = (size_t)(id / RS_RPP + P.pix_off);
    if (P.rq_occ[rq_phys(P, id)]) out[3 * c].z = -1.0f;
    else out[3 * c + 2].x = __uint_as_float(__float_as_uint(out[3 * c + 2].x) | RF_UNOCCLUDED);
}
#endif

// Chunked initial candidates (launch_frames_restir): sample k of the chunk C joins the context
// in one pass over the band and its halo rows, per pixel in the order of the per-sample chain:
// k_restir_frame_begin's previous-frame copy and reservoir reset (band + halo), then, on the band,
// the stores k_gbuffer would have made (a miss keeps the pixel's surface, material and per-pixel
// flag; the halo measure of a partitioned context) and the initial reservoirs the chunk's pass
// wrote (every pixel k_rsi_classify listed: not RSM_SKIP -- the others keep theirs).  The camera
// queue is every slot (q0[i] = i).
#ifndef MPT_TU_PART   // k_chunk_join
__global__ __launch_bounds__(TB) void k_chunk_join(DevPaths P, DevPaths C, const int4* __restrict__ cmeta, int k,
                                                   const MptFrame* __restrict__ Fp) {
    const MptFrame& F = *Fp;
    const MptRenderSettings& rs = F.render_settings;
    const int gp = P.rs_lo + blockIdx.x * TB + threadIdx.x;
    if (gp >= P.rs_hi) return;
    if (rs.restir_di_settings.do_temporal_reuse_pass) {   // k_restir_frame_begin
        P.pgb_pos[gp] = P.gb_pos[gp]; P.pgb_sn[gp] = P.gb_sn[gp]; P.pgb_gn[gp] = P.gb_gn[gp]; P.pgb_view[gp] = P.gb_view[gp];
        const int4 m = P.gb_meta[gp];
        P.pgb_meta[gp] = m;
        P.pgb_vsA[gp] = P.gb_vsA[gp]; P.pgb_vsB[gp] = P.gb_vsB[gp];
        if (m.w) P.pgb_mat[gp] = P.gb_mat[gp];
        if (MPT_RESTIR_CS)
            for (int q = 0; q < 4; q++) P.pgb_cs[4 * (size_t)gp + q] = P.gb_cs[4 * (size_t)gp + q];
    }
    const bool reset = (rs.sample_number == 0 || rs.need_to_reset) && rs.accumulate;
    if (reset) {
        rr_store(P.rs_init, gp, rr_default());
        rr_store(P.rs_sp1, gp, rr_default());
        rr_store(P.rs_sp2, gp, rr_default());
    }
    const int i = gp - P.pix_off;   // the band's pixel (slot)
    if (i < 0 || i >= P.n) return;
    const size_t c = (size_t)k * (size_t)P.n + (size_t)i;
    const int4 cm = C.gb_meta[c];
    int4 meta = P.gb_meta[gp];
    if (cm.z) {
        if (cm.w) P.gb_mat[gp] = C.gb_mat[c];
        const float4 pos = C.gb_pos[c];
        if (F.band_count > 1) {   // k_gbuffer's halo measure
            float fx, fy;
            restir_reproject(F, mk3(pos.x, pos.y, pos.z), fx, fy);
            const float H = (float)F.res_y;
            int off = F.res_y;
            if (fy > -H && fy < 2.0f * H) off = min(F.res_y, abs((int)roundf(fy) - gp / F.res_x));
            atomicMax(&P.counters[CTR_REPROJ], off);
        }
        P.gb_pos[gp] = pos;
        P.gb_sn[gp] = C.gb_sn[c];
        P.gb_gn[gp] = C.gb_gn[c];
        P.gb_vsA[gp] = C.gb_vsA[c];
        P.gb_vsB[gp] = C.gb_vsB[c];
        meta.y = cm.y;
        meta.w = cm.w;
        if (MPT_RESTIR_CS) {
            P.gb_cs[4 * (size_t)gp + 0] = C.gb_cs[4 * c + 0];
            P.gb_cs[4 * (size_t)gp + 1] = C.gb_cs[4 * c + 1];
            P.gb_cs[4 * (size_t)gp + 3] = C.gb_cs[4 * c + 3];
        }
    }
    meta.x = cm.x;
    meta.z = cm.z;
    P.gb_meta[gp] = meta;
    P.gb_view[gp] = C.gb_view[c];
    if (MPT_RESTIR_CS) P.gb_cs[4 * (size_t)gp + 2] = C.gb_cs[4 * c + 2];
    if (!(cmeta[c].x & RSM_SKIP)) {
        P.rs_init[3 * (size_t)gp + 0] = C.rs_init[3 * c + 0];
        P.rs_init[3 * (size_t)gp + 1] = C.rs_init[3 * c + 1];
        P.rs_init[3 * (size_t)gp + 2] = C.rs_init[3 * c + 2];
    }
}
#endif

// CameraRays' reset / previous-frame G-buffer copy for LSS_RESTIR_DI (CameraRays.h:19-34, 78-91)
#ifndef MPT_TU_PART   // k_restir_frame_begin
__global__ __launch_bounds__(TB) void k_restir_frame_begin(DevPaths P, const MptFrame* __restrict__ Fp, int32_t q0_count,
                                                           int32_t zero_reproj) {
    const MptFrame& F = *Fp;
    const MptRenderSettings& rs = F.render_settings;
    // the frame's counters, set here instead of by launches of their own (the kernels that read
    // them follow in the stream): the camera queue's length, and the halo measure k_gbuffer raises
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (q0_count >= 0) P.counters[CTR_Q0] = q0_count;
        if (zero_reproj) P.counters[CTR_REPROJ] = 0;
    }
    int i = P.rs_lo + blockIdx.x * TB + threadIdx.x;   // the band and its halo rows
    if (i >= P.rs_hi) return;
    // low resolution: only the representatives' entries (pixel_index / s) are copied and reset
    if (low_res(rs) && !low_res_region(F, i % F.res_x, i / F.res_x)) return;
    if (rs.restir_di_settings.do_temporal_reuse_pass) {
        P.pgb_pos[i] = P.gb_pos[i]; P.pgb_sn[i] = P.gb_sn[i]; P.pgb_gn[i] = P.gb_gn[i]; P.pgb_view[i] = P.gb_view[i];
        int4 meta = P.gb_meta[i];
        P.pgb_meta[i] = meta;
        P.pgb_vsA[i] = P.gb_vsA[i]; P.pgb_vsB[i] = P.gb_vsB[i];
        if (meta.w) P.pgb_mat[i] = P.gb_mat[i];
        if (MPT_RESTIR_CS)
            for (int k = 0; k < 4; k++) P.pgb_cs[4 * (size_t)i + k] = P.gb_cs[4 * (size_t)i + k];
    }
    if ((rs.sample_number == 0 || rs.need_to_reset) && rs.accumulate) {
        rr_store(P.rs_init, i, rr_default());
        rr_store(P.rs_sp1, i, rr_default());
        rr_store(P.rs_sp2, i, rr_default());
    }
}
#endif

// pixel_converged_sample_count by pixel for the neighbour tests of a partitioned context
// (restir_spatial_neighbor reads it at neighbouring pixels; exchanged with the G-buffer)
#ifndef MPT_TU_PART   // k_restir_conv
__global__ __launch_bounds__(TB) void k_restir_conv(DevPaths P) {
    int s = blockIdx.x * TB + threadIdx.x;
    if (s < P.n) P.rs_conv[s + P.pix_off] = P.as_conv[s];
}
#endif

#ifndef MPT_TU_PART   // k_restir_fill
__global__ void k_restir_fill(float4* r, int n) {   // default reservoirs (Reservoir.h:166-170)
    int i = blockIdx.x * TB + threadIdx.x;
    if (i < n) rr_store(r, i, rr_default());
}
#endif
#ifndef MPT_TU_PART   // k_restir_fill_lights
__global__ void k_restir_fill_lights(float4* l, int n) {   // default presampled lights
    int i = blockIdx.x * TB + threadIdx.x;
    if (i < n) {
        l[4 * (size_t)i + 0] = make_float4(__int_as_float(-1), 0.0f, 0.0f, 0.0f);
        l[4 * (size_t)i + 1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        l[4 * (size_t)i + 2] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        l[4 * (size_t)i + 3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}
#endif
