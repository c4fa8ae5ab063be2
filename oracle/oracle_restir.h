// TEST INFRASTRUCTURE ONLY (see oracle.cpp): CPU restatement of ReSTIR DI as the
// reference runs it with its default kernel options (KernelOptions.h:270-366):
// lights presampling on, no visibility in the initial target function, visibility in
// the spatial target function, visibility reuse, visibility in the bias correction,
// pairwise-MIS-defensive bias correction weights, fused spatiotemporal pass followed
// by (number_of_passes - 1) spatial passes (ReSTIRDIRenderPass.cpp:233-264, 480-507).
// Included by oracle.cpp after the light / envmap / traversal helpers.

enum { RF_ENVMAP = 1u, RF_BSDF_REFRACTION = 2u, RF_UNOCCLUDED = 4u };   // SampleFlags.h:10-22

struct OResv {                                   // ReSTIRDIReservoir (Reservoir.h:22-116)
    int M = 0;
    float wsum = 0.0f, UCW = 0.0f;
    int tri = -1;                                // ReSTIRDISample (Reservoir.h:22-32)
    f3 point{0.0f, 0.0f, 0.0f};
    float target = 0.0f;
    uint32_t flags = 0;
    void add_one_candidate(int t, f3 p, float tf, uint32_t fl, float w, Rng& rng) {
        M++;
        wsum += w;
        if (rng() < w / wsum) { tri = t; point = p; target = tf; flags = fl; }
    }
    bool combine_with(const OResv& o, float mis, float tf, float jac, Rng& rng) {
        if (o.UCW <= 0.0f) { M += o.M; return false; }
        float w = mis * tf * o.UCW * jac;
        M += o.M;
        wsum += w;
        if (rng() < w / wsum) {
            tri = o.tri; point = o.point; flags = o.flags;
            target = tf;
            return true;
        }
        return false;
    }
    void end() { UCW = wsum == 0.0f ? 0.0f : 1.0f / target * wsum; }
    void end_with_normalization(float nume, float denom) {
        if (wsum == 0.0f || wsum < 1.0e-10f || wsum > 1.0e10f || denom == 0.0f || nume == 0.0f) UCW = 0.0f;
        else UCW = 1.0f / target * wsum * nume / denom;
        M = std::min(M, 1000000);
    }
};

struct OPLight {                                 // ReSTIRDIPresampledLight (PresampledLight.h:14-30)
    int tri = -1;
    f3 point{0.0f, 0.0f, 0.0f}, normal{0.0f, 0.0f, 0.0f};
    Col radiance;
    float pdf = 0.0f;
    uint32_t flags = 0;
};

struct RestirBuffers {                           // AuxiliaryBuffers restir_reservoir_buffer_1..3
    std::vector<OResv> init, sp1, sp2;
    std::vector<OPLight> plights;
    std::vector<OResv>* output = nullptr;        // restir_output_reservoirs (-> sp1 initially)
};

struct RSurface {                                // ReSTIRDISurface (Surface.h:12-33)
    const Material* mat;
    VolumeState vs;
    int last_hit;
    f3 view, sn, gn, sp;
};
inline RSurface surface_of(const GB& g) {
    RSurface s;
    s.mat = &g.mat;
    s.vs = g.vs;
    s.last_hit = g.prim;
    s.view = g.view;
    s.sn = g.sn;
    s.gn = g.gn;
    s.sp = g.first_hit + g.sn * 1.0e-4f;
    return s;
}

// power_heuristic (Sampling.h:75-87)
inline float power_heuristic(float a, int na, float b, int nb) {
    float pa = ((float)na * a) * ((float)na * a);
    float pb = ((float)nb * b) * ((float)nb * b);
    return (float)na * a * a / (pa + pb);
}
inline float radical_inverse_base_2(uint32_t i) {   // Sampling.h:25-32
    i = (i << 16u) | (i >> 16u);
    i = ((i & 0x55555555u) << 1u) | ((i & 0xAAAAAAAAu) >> 1u);
    i = ((i & 0x33333333u) << 2u) | ((i & 0xCCCCCCCCu) >> 2u);
    i = ((i & 0x0F0F0F0Fu) << 4u) | ((i & 0xF0F0F0F0u) >> 4u);
    i = ((i & 0x00FF00FFu) << 8u) | ((i & 0xFF00FF00u) >> 8u);
    return (float)i * 2.3283064365386963e-10f;
}
inline int cantor(int x, int y) { return (x + y + 1) * (x + y) / 2 + y; }   // InitialCandidates.h:25-28
inline uint32_t pass_seed(const MptFrame& f, uint32_t pix, uint32_t seed) {
    return f.render_settings.freeze_random ? wang_hash(pix + 1u) : wang_hash((pix + 1u) * (uint32_t)(f.render_settings.sample_number + 1) * seed);
}

// Traced rays of the ReSTIR passes use alpha keys (pass pixel seed, 0, 5 + pass, position):
// the position names the ray's site in the pass (not its rank among the rays traced so far),
// the same positions as the GPU passes (restir_di.h RP_*)
inline int RP_TFC(int k) { return 2 * k; }           // neighbour k's sample at the center
inline int RP_TCN(int k) { return 2 * k + 1; }       // the canonical sample at neighbour k (pairwise MIS)
constexpr int RP_T_TFC = 4000, RP_T_TCN = 4001;      // the temporal neighbour's pair
inline int RP_GBH(int cur, int j) { return 100000 + cur * 1000 + j; }   // j = 999 / 998: temporal / center terms
inline int RP_NORM(int j) { return 200000 + j; }
inline int RP_LIGHT(int i) { return 1000000 + i; }
inline int RP_BSDF(int i) { return 2000000 + i; }
constexpr int RP_VISREUSE = 300000;
struct RestirRays {
    Ctx& c;
    int kind;
    int n = 0;
    RestirRays& at(int pos) { n = pos; return *this; }
    bool any(f3 o, f3 d, float tmax, int last) {
        c.rays_any++;
        uint32_t ak = c.alpha ? alpha_key(c.pseed, 0, kind, n++) : 0u;
        Hit h = closest(*c.s, o, d, last, c.alpha ? &ak : nullptr);
        if (h.prim < 0) return false;
        return h.t < tmax - 1.0e-4f;
    }
};

// ReSTIR_DI_evaluate_target_function<vis> (Utils.h:20-128)
float restir_target(Ctx& c, RestirRays& rr, int tri, f3 point, uint32_t flags, const RSurface& s, bool vis) {
    const MptWorldSettings& w = c.f->world_settings;
    if (tri == -1 && !(flags & RF_ENVMAP)) return 0.0f;
    float dist = 0.0f;
    f3 dir;
    if (flags & RF_ENVMAP) { dir = mat_x_vec(w.envmap_to_world_matrix, point); dist = 1.0e35f; }
    else if (vis) { dir = point - s.sp; dir = dir / (dist = length(dir)); }
    else dir = normalize(point - s.sp);
    float cosv = fmaxr(0.0f, dot(s.sn, dir));
    if (cosv == 0.0f) return 0.0f;
    float bp;
    VolumeState tv = s.vs;
    Col f = bsdf_eval(c.bc, c.override_, *s.mat, tv, s.view, s.sn, s.gn, dir, bp);
    Col e;
    if (flags & RF_ENVMAP) { float ep; e = envmap_eval(c, dir, ep); }
    else e = emission_of(c.s->mats[c.s->mat_idx[tri]]);
    float t = (f * e * cosv).luminance();
    if (t == 0.0f) return 0.0f;
    if (vis) t *= rr.any(s.sp, dir, dist, s.last_hit) ? 0.0f : 1.0f;
    return t;
}

// ReSTIR_DI_visibility_reuse (Utils.h:134-171)
void restir_visibility_reuse(Ctx& c, RestirRays& rr, OResv& r, f3 sp, int last) {
    if (r.UCW <= 0.0f) return;
    if (r.flags & RF_UNOCCLUDED) return;
    float dist;
    f3 dir;
    if (r.flags & RF_ENVMAP) { dir = mat_x_vec(c.f->world_settings.envmap_to_world_matrix, r.point); dist = 1.0e35f; }
    else { dir = r.point - sp; dir = dir / (dist = length(dir)); }
    if (rr.at(RP_VISREUSE).any(sp, dir, dist, last)) r.UCW = -1.0f;
    else r.flags |= RF_UNOCCLUDED;
}

// get_jacobian_determinant_reconnection_shift (Utils.h:173-206)
float restir_jacobian(const OScene& s, const OResv& nr, f3 center_sp, f3 neighbor_sp) {
    f3 tc = nr.point - center_sp, tn = nr.point - neighbor_sp;
    float dc, dn;
    tc = tc / (dc = length(tc));
    tn = tn / (dn = length(tn));
    f3 ln = normalize(cross(s.pos[s.idx[3 * nr.tri + 1]] - s.pos[s.idx[3 * nr.tri]], s.pos[s.idx[3 * nr.tri + 2]] - s.pos[s.idx[3 * nr.tri]]));
    float cc = absf(dot(-tc, ln)), cn = absf(dot(-tn, ln));
    float jac = cc / cn * ((dn * dn) / (dc * dc));
    if (jac > 20.0f || jac < 1.0f / 20.0f || std::isnan(jac)) return -1.0f;
    return jac;
}

// check_neighbor_similarity_heuristics (Utils.h:214-263), incl. the inverted normal test
bool restir_similar(const MptReSTIRDISettings& rs, const GB& nb_cur, const GB& nb_prev, const GB& center, f3 sp, f3 n, bool prev) {
    f3 p = prev ? nb_prev.first_hit : nb_cur.first_hit;
    float nr = prev ? nb_prev.mat.roughness : nb_cur.mat.roughness;
    bool plane = !rs.use_plane_distance_heuristic || absf(dot(p - sp, n)) < rs.plane_distance_threshold;
    bool normal = rs.use_normal_similarity_heuristic ? true : dot(n, nb_cur.sn) > rs.normal_similarity_angle_precomp;
    bool rough = !rs.use_roughness_similarity_heuristic || absf(nr - center.mat.roughness) < rs.roughness_similarity_threshold;
    bool emissive = prev ? is_emissive(nb_prev.mat) : is_emissive(nb_cur.mat);
    return plane && normal && rough && !emissive;
}

// get_spatial_neighbor_pixel_index (Utils.h:289-339); adaptive-sampling convergence
// filter applies only with enable_adaptive_sampling (the converged buffer is passed in)
int restir_spatial_neighbor(const MptFrame& f, int k, int count, int radius, int cx, int cy, float cr, float sr,
                            const int32_t* conv, uint32_t pass_random_seed) {
    int W = f.res_x, H = f.res_y;
    if (k == count) return cx + cy * W;
    float ux = (float)(unsigned)(k + 1) / (float)(unsigned)(count + 1), uy = radical_inverse_base_2((unsigned)(k + 1));
    float rr = (float)radius * std::sqrt(uy);
    float ox = rr * pcos(TWO_PI * ux), oy = rr * psin(TWO_PI * ux);
    float rx = ox * cr - oy * sr, ry = ox * sr + oy * cr;
    int nx, ny;
    if (f.render_settings.restir_di_settings.debug_neighbor_location) { nx = cx + 15; ny = cy; }
    else { nx = cx + (int)rx; ny = cy + (int)ry; }
    if (nx < 0 || nx >= W || ny < 0 || ny >= H) return -1;
    int ni = nx + ny * W;
    const MptRenderSettings& rs = f.render_settings;
    if (rs.enable_adaptive_sampling && rs.sample_number >= rs.adaptive_sampling_min_samples && conv) {
        if (rs.restir_di_settings.allow_converged_neighbors_reuse) {
            // a fresh copy of Xorshift32Generator(random_seed) per call: always its first draw
            Rng g(pass_random_seed);
            if (g() > rs.restir_di_settings.converged_neighbor_reuse_probability && conv[ni] != -1) return -1;
        } else if (conv[ni] != -1) return -1;
    }
    return ni;
}

struct RestirPassCtx {
    const MptFrame& f;
    RestirBuffers& B;
    std::vector<GB>& cur;
    std::vector<GB>& prev;
    const std::vector<uint8_t>& active;
    const int32_t* conv;
};

// ReSTIR_DI_LightsPresampling (LightsPresampling.h:22-130)
void restir_presample(Ctx& c, RestirPassCtx& R) {
    const MptFrame& f = R.f;
    const MptReSTIRDISettings& rd = f.render_settings.restir_di_settings;
    const OScene& s = *c.s;
    const MptWorldSettings& w = f.world_settings;
    int n = rd.number_of_subsets * rd.subset_size;
    R.B.plights.resize((size_t)n);
    if (s.n_emissive == 0 && w.ambient_light_type != MPT_AMBIENT_ENVMAP) return;
    float env_p = 0.0f;
    if (w.ambient_light_type == MPT_AMBIENT_ENVMAP) env_p = s.n_emissive == 0 ? 1.0f : rd.envmap_candidate_probability;
    for (int x = 0; x < n; x++) {
        Rng rng(pass_seed(f, (uint32_t)x, f.restir_di_seeds[0]));
        OPLight pl;
        if (rng() < env_p) {
            pl.flags |= RF_ENVMAP;
            f3 dir;
            pl.radiance = envmap_sample(c, dir, pl.pdf, rng);
            pl.point = mat_x_vec(w.world_to_envmap_matrix, dir);
            pl.pdf *= env_p;
        } else {
            float lp = 1.0f - env_p;
            int ri = rng.random_index(s.n_emissive);
            int t = s.emissive[ri];
            f3 A = s.pos[s.idx[3 * t]], Bv = s.pos[s.idx[3 * t + 1]], Cv = s.pos[s.idx[3 * t + 2]];
            float r1 = rng(), r2 = rng();
            float sr1 = psqrt(r1);
            float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
            f3 AB = Bv - A, AC = Cv - A;
            f3 pt = A + AB * u + AC * v;
            f3 nn = cross(AB, AC);
            float ln = length(nn);
            if (ln > 1.0e-6f) {
                pl.point = pt;
                pl.normal = nn / ln;
                pl.tri = t;
                pl.pdf = 1.0f / (ln * 0.5f);
                pl.pdf /= (float)s.n_emissive;
                pl.pdf *= lp;
                pl.radiance = emission_of(s.mats[s.mat_idx[t]]);
            }
        }
        R.B.plights[(size_t)x] = pl;
    }
}

// ReSTIR_DI_InitialCandidates (InitialCandidates.h:24-508)
void restir_initial(Ctx& c, RestirPassCtx& R, int x, int y) {
    const MptFrame& f = R.f;
    const MptReSTIRDISettings& rd = f.render_settings.restir_di_settings;
    const OScene& s = *c.s;
    const MptWorldSettings& w = f.world_settings;
    if (s.n_emissive == 0 && w.ambient_light_type != MPT_AMBIENT_ENVMAP) return;
    int pix = x + y * f.res_x;
    const GB& g = R.cur[(size_t)pix];
    if (is_emissive(g.mat)) return;
    uint32_t seed = pass_seed(f, (uint32_t)pix, f.restir_di_seeds[1]);
    Rng rng(seed);
    if (!R.active[(size_t)pix] || !g.hit) return;
    c.pseed = seed;
    RestirRays rr{c, 5};
    int nl = rd.number_of_initial_light_candidates, nb = rd.number_of_initial_bsdf_candidates;
    if (low_res(f.render_settings)) { nl = std::min(1, nl); nb = std::min(1, nb); }   // InitialCandidates.h:420-421
    float env_p = 0.0f;
    if (w.ambient_light_type == MPT_AMBIENT_ENVMAP) env_p = s.n_emissive == 0 ? 1.0f : rd.envmap_candidate_probability;
    OResv r;
    f3 ep = g.first_hit + g.sn * 1.0e-4f * 1.0f;
    // sample_light_candidates with presampled lights (InitialCandidates.h:30-121, 171-271)
    for (int i = 0; i < nl; i++) {
        int tri;
        f3 point, tl;
        uint32_t flags;
        float target = 0.0f;
        Col rad;
        float pdf, dist = 0.0f, cosv;
        if (f.options.restir_di_do_lights_presampling) {
            int tc = cantor(x / rd.tile_size, y / rd.tile_size);
            Rng subset_rng(f.restir_di_seeds[1] * (uint32_t)(tc + 1));
            int subset = subset_rng.random_index(rd.number_of_subsets);
            int li = rng.random_index(rd.subset_size);
            const OPLight& pl = R.B.plights[(size_t)(subset * rd.subset_size + li)];
            tri = pl.tri;
            point = pl.point;
            flags = pl.flags;
            rad = pl.radiance;
            pdf = pl.pdf;
            if (flags & RF_ENVMAP) { tl = mat_x_vec(w.envmap_to_world_matrix, point); dist = 1.0e35f; }
            else { tl = point - ep; tl = tl / (dist = length(tl)); }
            cosv = dot(g.sn, tl);
            if (!(flags & RF_ENVMAP)) {
                float cl = absf(dot(pl.normal, -tl));
                pdf *= dist * dist;
                pdf /= cl;
                if (!min_contrib(f.render_settings.minimum_light_contribution, rad * cosv / pdf)) { r.M++; continue; }
            }
        } else {
            // sample_fresh_light_candidate (InitialCandidates.h:93-170)
            tri = -1; point = f3{0.0f, 0.0f, 0.0f}; flags = 0u; rad = Col(0.0f); pdf = 0.0f; cosv = 0.0f;
            if (rng() > env_p) {
                LightInfo lsi;
                point = sample_emissive_triangle(c, rng, pdf, lsi);
                tri = lsi.tri;
                if (pdf > 0.0f) {
                    f3 d2 = point - ep;
                    float dl = length(d2);
                    d2 = d2 / dl;
                    cosv = std::max(0.0f, dot(g.sn, d2));
                    float cl = absf(dot(lsi.normal, -d2));
                    pdf *= dl * dl;
                    pdf /= cl;
                    if (!min_contrib(f.render_settings.minimum_light_contribution, lsi.emission * cosv / pdf)) { r.M++; continue; }
                    pdf *= (1.0f - env_p);
                    rad = lsi.emission;
                }
            } else {
                f3 edir;
                rad = envmap_sample(c, edir, pdf, rng);
                cosv = std::max(0.0f, dot(edir, g.sn));
                if (!min_contrib(f.render_settings.minimum_light_contribution, rad * cosv / pdf)) { r.M++; continue; }
                pdf *= env_p;
                point = mat_x_vec(w.world_to_envmap_matrix, edir);
                flags = RF_ENVMAP;
            }
            if (flags & RF_ENVMAP) { tl = mat_x_vec(w.envmap_to_world_matrix, point); dist = 1.0e35f; }
            else { tl = point - ep; tl = tl / (dist = length(tl)); }
        }
        float weight = 0.0f;
        if (cosv > 0.0f && pdf > 0.0f) {
            float bp;
            VolumeState tv = g.vs;
            Col bc = bsdf_eval(c.bc, c.override_, g.mat, tv, g.view, g.sn, g.gn, tl, bp);
            Col lc = bc * rad * cosv;
            float tf = lc.luminance();
            if (min_contrib(f.render_settings.minimum_light_contribution, lc / pdf / bp)) {
                float mis = power_heuristic(pdf, nl, bp, nb);
                weight = mis * tf / pdf;
                target = tf;
            }
        }
        // ReSTIR_DI_InitialTargetFunctionVisibility (InitialCandidates.h:248-264)
        if (f.options.restir_di_initial_target_visibility && !low_res(f.render_settings) && target > 0.0f) {
            if (rr.at(RP_LIGHT(i)).any(ep, tl, dist, g.prim)) { r.M++; continue; }
            flags |= RF_UNOCCLUDED;
        }
        r.add_one_candidate(tri, point, target, flags, weight, rng);
    }
    // sample_bsdf_candidates (InitialCandidates.h:273-394)
    for (int i = 0; i < nb; i++) {
        float bpdf = 0.0f;
        f3 dir;
        VolumeState tv = g.vs;
        Col bc = bsdf_sample(c.bc, c.override_, g.mat, tv, g.view, g.sn, g.gn, dir, bpdf, rng);
        bool refr = dot(dir, g.view) < 0.0f;
        if (!(bpdf > 0.0f)) continue;
        ShadowLightHit sh;
        c.rays_closest++;
        uint32_t ak = c.alpha ? alpha_key(c.pseed, 0, rr.kind, RP_BSDF(i)) : 0u;
        Hit h = closest(s, g.first_hit, dir, g.prim, c.alpha ? &ak : nullptr);
        bool found = h.prim >= 0 && h.t < 1.0e35f - 1.0e-4f;
        if (found) {
            const Material& m = s.mats[s.mat_idx[h.prim]];
            f2 uv = mk2(h.u, h.v);
            f2 tcd = uv_interp(s.uv, s.idx, h.prim, uv);
            if (m.emission_texture_index != MPT_NO_TEXTURE) {
                MptColor e{0, 0, 0};
                prop_c(c, e, tcd, m.emission_texture_index);
                sh.emission = Col(e.r, e.g, e.b);
            } else sh.emission = emission_of(m);
            sh.shading_normal = shading_normal_of(c, normalize(tri_normal(s, h.prim)), h.prim, uv, tcd);
            sh.prim = h.prim;
            sh.dist = h.t;
        }
        if (found && !sh.emission.is_black()) {
            float ce = absf(dot(g.sn, dir));
            Col lc = bc * sh.emission * ce;
            float tf = lc.luminance();
            float lpdf = 0.0f;
            if (!refr) lpdf = pdf_emissive_hit(s, sh, dir);
            if (!min_contrib(f.render_settings.minimum_light_contribution, lc / lpdf / bpdf)) { r.M++; continue; }
            lpdf *= (1.0f - env_p);
            float mis = power_heuristic(bpdf, nb, lpdf, nl);
            float weight = mis * tf / bpdf;
            uint32_t fl = RF_UNOCCLUDED | (refr ? RF_BSDF_REFRACTION : 0u);
            r.add_one_candidate(sh.prim, g.first_hit + dir * sh.dist, tf, fl, weight, rng);
        } else if (!found && w.ambient_light_type == MPT_AMBIENT_ENVMAP) {
            float ce = fmaxr(0.0f, dot(g.sn, dir));
            if (ce > 0.0f) {
                float epdf;
                Col er = envmap_eval(c, dir, epdf);
                Col ec = bc * er * ce;
                if (!min_contrib(f.render_settings.minimum_light_contribution, ec / epdf / bpdf)) { r.M++; continue; }
                float tf = ec.luminance();
                epdf *= env_p;
                float mis = power_heuristic(bpdf, nb, epdf, nl);
                float weight = mis * tf / bpdf;
                r.add_one_candidate(-1, mat_x_vec(w.world_to_envmap_matrix, dir), tf, RF_ENVMAP | RF_UNOCCLUDED, weight, rng);
            }
        }
    }
    r.end();
    r.M = 1;
    if (f.options.restir_di_do_visibility_reuse) restir_visibility_reuse(c, rr, r, g.first_hit + g.sn * 1.0e-4f, g.prim);
    R.B.init[(size_t)pix] = r;
}

// pairwise MIS defensive weights (SpatiotemporalMISWeight.h:193-291, SpatialMISWeight.h:167-262)
struct PairwiseMIS {
    float mc = 0.0f;
    bool defensive = true;   // PAIRWISE_MIS_DEFENSIVE (else PAIRWISE_MIS, SpatialMISWeight.h:95-165)
    bool bvis = true;        // ReSTIR_DI_BiasCorrectionUseVisibility
    float weight(Ctx& c, RestirRays& rr, const MptReSTIRDISettings& rd, const OResv& res, const OResv& center, float tf_center,
                 const GB& neighbor_gb, int valid_count, int valid_M, bool update_mc, bool canonical) {
        if (!defensive) {
            const bool cw = rd.use_confidence_weights;
            if (canonical) return mc == 0.0f ? 1.0f : mc;
            float tfn = res.target;
            float rM = cw ? (float)res.M : 1.0f, cM = cw ? (float)center.M : 1.0f, nsum = cw ? (float)valid_M : 1.0f;
            float div = cw ? 1.0f : (float)valid_count;
            float nume = tfn * rM;
            float denom = tfn * nsum + tf_center / div * cM;
            float mi = denom == 0.0f ? 0.0f : (nume / denom);
            if (update_mc) {
                RSurface ns = surface_of(neighbor_gb);
                float tcn = restir_target(c, rr, center.tri, center.point, center.flags, ns, bvis);
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
            float nsum = rd.use_confidence_weights ? (float)valid_M : 1.0f;
            float div = rd.use_confidence_weights ? 1.0f : (float)valid_count;
            float nume = tfn * rM;
            float denom = tfn * nsum + tf_center / div * cM;
            float mi = 0.0f;
            if (denom != 0.0f) mi = nume / denom;
            if (rd.use_confidence_weights) mi *= nsum / (nsum + cM);
            if (update_mc) {
                RSurface ns = surface_of(neighbor_gb);
                float tcn = restir_target(c, rr, center.tri, center.point, center.flags, ns, bvis);
                float tcc = center.target;
                float nume_mc = tcc / div * cM;
                float denom_mc = tcn * nsum + tcc / div * cM;
                float conf = 1.0f;
                if (rd.use_confidence_weights) conf = rM / (cM + nsum);
                if (denom_mc != 0.0f) mc += nume_mc / denom_mc * conf;
            }
            if (rd.use_confidence_weights) return mi;
            return mi / (float)(valid_count + 1);
        }
        if (mc == 0.0f) return 1.0f;
        if (rd.use_confidence_weights) return mc + (float)center.M / (float)(center.M + valid_M);
        return (1.0f + mc) / (float)(valid_count + 1);
    }
};

// do_include_spatial_visibility_term_or_not (FusedSpatiotemporalReuse.h:41-56, SpatialReuse.h:36-50)
inline bool spatial_visibility(const MptFrame& f, const MptReSTIRDISettings& rd, int k, int reuse_count) {
    bool v = rd.do_visibility_only_last_pass && rd.spatial_pass_index == rd.number_of_passes - 1;
    v |= !rd.do_visibility_only_last_pass;
    v &= k < rd.neighbor_visibility_count;
    v &= f.options.restir_di_spatial_target_visibility != 0;
    v &= k != reuse_count;
    return v;
}

// find_temporal_neighbor_index (Utils.h:371-421)
void restir_temporal_neighbor(Ctx& c, RestirPassCtx& R, f3 p, f3 n, int center, Rng& rng, int& idx, int& px, int& py) {
    const MptFrame& f = R.f;
    const MptReSTIRDISettings& rd = f.render_settings.restir_di_settings;
    int W = f.res_x, H = f.res_y;
    f3 ss = mat_x_point(f.prev_camera.view_projection, p);
    float sx = ss.x, sy = ss.y;
    sx += 1.0f; sy += 1.0f;
    sx *= 0.5f; sy *= 0.5f;
    float fx = sx * (float)W, fy = sy * (float)H;
    fx -= 0.5f; fy -= 0.5f;
    idx = -1;
    bool use_prev = rd.do_temporal_reuse_pass;
    for (int i = 0; i < rd.max_neighbor_search_count + 1; i++) {
        float ox = 0.0f, oy = 0.0f;
        if (i > 0) {
            float a = rng() - 0.5f, b = rng() - 0.5f;
            ox = a * (float)rd.neighbor_search_radius;
            oy = b * (float)rd.neighbor_search_radius;
        }
        int qx = (int)std::round(fx + ox), qy = (int)std::round(fy + oy);
        if (rd.use_permutation_sampling && i == 0) {
            int bits = (int)rd.permutation_sampling_random_bits;
            int ax = bits & 3, ay = (bits >> 2) & 3;
            qx += ax; qy += ay;
            qx ^= 3; qy ^= 3;
            qx -= ax; qy -= ay;
        }
        if (qx < 0 || qx >= W || qy < 0 || qy >= H) continue;
        idx = qx + qy * W;
        if (restir_similar(rd, R.cur[(size_t)idx], R.prev[(size_t)idx], R.cur[(size_t)center], p, n, use_prev)) break;
        idx = -1;
    }
    px = (int)std::round(fx);
    py = (int)std::round(fy);
}

// ReSTIR_DI_SpatiotemporalReuse (FusedSpatiotemporalReuse.h:112-586); tin = temporal
// input (= spatial input of the fused pass), out = spatial output
void restir_spatiotemporal(Ctx& c, RestirPassCtx& R, int x, int y, std::vector<OResv>& tin, std::vector<OResv>& out) {
    const MptFrame& f = R.f;
    MptReSTIRDISettings rd = f.render_settings.restir_di_settings;
    const OScene& s = *c.s;
    int W = f.res_x;
    int center = x + y * W;
    const GB& g = R.cur[(size_t)center];
    if (!R.active[(size_t)center] || !g.hit) return;
    rd.spatial_pass_index = 0;   // configure_spatial_pass_for_fused_spatiotemporal(0)
    uint32_t seed = pass_seed(f, (uint32_t)center, f.restir_di_seeds[2]);
    Rng rng(seed);
    c.pseed = seed;
    RestirRays rr{c, 6};
    RSurface cs = surface_of(g);
    if (is_emissive(g.mat)) return;
    if (rd.temporal_buffer_clear_requested) tin[(size_t)center] = OResv();
    bool use_prev = rd.do_temporal_reuse_pass;
    // load_temporal_neighbor_data (FusedSpatiotemporalReuse.h:62-96)
    OResv tres;
    const GB* tgb = nullptr;
    int tidx, tpx, tpy;
    restir_temporal_neighbor(c, R, g.first_hit, cs.sn, center, rng, tidx, tpx, tpy);
    if (tidx != -1 && !f.render_settings.freeze_random) {
        tres = tin[(size_t)tidx];
        if (tres.M != 0) tgb = use_prev ? &R.prev[(size_t)tidx] : &R.cur[(size_t)tidx];
    }
    if ((tidx == -1 || tres.M <= 1) && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
    float rot = rd.do_neighbor_rotation ? TWO_PI * rng() : 0.0f;
    float cr = pcos(rot), sr = psin(rot);
    // count_valid_spatiotemporal_neighbors (FusedSpatiotemporalReuse.h:110-141)
    int reuse = rd.reuse_neighbor_count;
    int cache = 0, vcount = 0, vM = 0;
    for (int k = 0; k < reuse; k++) {
        int ni = restir_spatial_neighbor(f, k, reuse, rd.reuse_radius, tpx, tpy, cr, sr, R.conv, f.restir_di_seeds[2]);
        if (ni == -1) continue;
        if (!restir_similar(rd, R.cur[(size_t)ni], R.prev[(size_t)ni], g, cs.sp, cs.sn, use_prev)) continue;
        vM += tin[(size_t)ni].M;
        vcount++;
        cache |= 1 << k;
    }
    if (tidx != -1 && tres.M > 0) { vcount++; vM += tres.M; }
    OResv o;
    OResv ic = R.B.init[(size_t)center];
    const int mode = f.options.restir_di_bias_correction_weights;
    const bool bvis = f.options.restir_di_bias_correction_use_visibility != 0;
    const bool cw = rd.use_confidence_weights;
    PairwiseMIS mis;
    mis.defensive = mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE;
    mis.bvis = bvis;
    // load_temporal_neighbor_data: the temporal surface is loaded when its reservoir is not
    // empty, else it stays a default ReSTIRDISurface (zero normals: target function 0)
    RSurface ts;
    if (tgb) ts = surface_of(*tgb);
    else { ts = cs; ts.mat = &g.mat; ts.sn = ts.gn = ts.view = ts.sp = f3{0.0f, 0.0f, 0.0f}; }
    auto nb_gb = [&](int nj, bool prev) -> const GB& { return prev ? R.prev[(size_t)nj] : R.cur[(size_t)nj]; };
    auto valid_nb = [&](int j) -> int {
        if (j == reuse) return center;
        int nj = restir_spatial_neighbor(f, j, reuse, rd.reuse_radius, tpx, tpy, cr, sr, R.conv, f.restir_di_seeds[2]);
        if (nj == -1) return -1;
        return restir_similar(rd, R.cur[(size_t)nj], R.prev[(size_t)nj], g, cs.sp, cs.sn, use_prev) ? nj : -1;
    };
    // ReSTIRDISpatiotemporalResamplingMISWeight<MIS_GBH> (SpatiotemporalMISWeight.h:36-100)
    auto gbh = [&](const OResv& r, int current) -> float {
        if (r.UCW <= 0.0f) return 1.0f;
        float nume = 0.0f, denom = 0.0f;
        for (int j = 0; j < reuse + 1; j++) {
            int nj = valid_nb(j);
            if (nj == -1) continue;
            RSurface js = j == reuse ? cs : surface_of(nb_gb(nj, use_prev));
            float tj = restir_target(c, rr.at(RP_GBH(current, j)), r.tri, r.point, r.flags, js, bvis);
            int M = 1;
            if (cw) M = j == reuse ? ic.M : tin[(size_t)nj].M;
            denom += tj * (float)M;
            if (j + 1 == current) nume = tj * (float)M;
        }
        float tt = restir_target(c, rr.at(RP_GBH(current, 999)), r.tri, r.point, r.flags, ts, bvis);
        int M = cw ? tres.M : 1;
        denom += tt * (float)M;
        if (current == 0) nume = tt * (float)M;
        return denom == 0.0f ? 0.0f : nume / denom;
    };
    int selected = 0;
    if (tidx != -1 && tres.M > 0) {
        float tfc = 0.0f;
        if (tres.UCW > 0.0f) tfc = restir_target(c, rr.at(RP_T_TFC), tres.tri, tres.point, tres.flags, cs, bvis);
        float jac = 1.0f;
        if (tfc > 0.0f && tres.UCW > 0.0f && !(tres.flags & RF_ENVMAP)) {
            const GB& tg = use_prev ? R.prev[(size_t)tidx] : R.cur[(size_t)tidx];
            f3 tsp = tg.first_hit + tg.sn * 1.0e-4f;
            jac = restir_jacobian(s, tres, cs.sp, tsp - tg.sn * 1.0e-4f);
            if (jac == -1.0f) jac = 0.0f;
        }
        float w;
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) w = (float)tres.M;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) w = cw ? (float)tres.M : 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) w = gbh(tres, 0);
        else {
            bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
            w = mis.weight(c, rr.at(RP_T_TCN), rd, tres, ic, tfc, *tgb, vcount, vM, update_mc, false);
        }
        if (o.combine_with(tres, w, tfc, jac, rng)) {
            selected = 0;
            if (bvis) o.flags |= RF_UNOCCLUDED;
            else o.flags &= ~RF_UNOCCLUDED;
        }
    }
    int start = vM == 0 ? reuse : 0;
    for (int k = start; k < reuse + 1; k++) {
        if (k < reuse && reuse <= 32 && (cache & (1 << k)) == 0) continue;
        int ni = k == reuse ? center : restir_spatial_neighbor(f, k, reuse, rd.reuse_radius, tpx, tpy, cr, sr, R.conv, f.restir_di_seeds[2]);
        if (ni == -1) continue;
        if (k < reuse && reuse > 32 && !restir_similar(rd, R.cur[(size_t)ni], R.prev[(size_t)ni], g, cs.sp, cs.sn, use_prev)) continue;
        OResv nr = k == reuse ? ic : tin[(size_t)ni];
        float tfc = 0.0f;
        bool vis = spatial_visibility(f, rd, k, reuse);
        if (nr.UCW > 0.0f) {
            if (k == reuse) tfc = nr.target;
            else tfc = restir_target(c, rr.at(RP_TFC(k)), nr.tri, nr.point, nr.flags, cs, vis);
        }
        float jac = 1.0f;
        if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
            const GB& ng = use_prev ? R.prev[(size_t)ni] : R.cur[(size_t)ni];
            jac = restir_jacobian(s, nr, cs.sp, ng.first_hit + ng.sn * 1.0e-4f);
            if (jac == -1.0f) { o.M += nr.M; continue; }
        }
        float w;
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) w = (float)nr.M;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) w = cw ? (float)nr.M : 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) w = gbh(nr, k + 1);
        else {
            bool update_mc = ic.M > 0 && ic.UCW > 0.0f;
            if (nr.UCW == 0.0f && !update_mc) w = 1.0f;
            else {
                const GB& ng = use_prev ? R.prev[(size_t)ni] : R.cur[(size_t)ni];
                w = mis.weight(c, rr.at(RP_TCN(k)), rd, nr, ic, tfc, ng, vcount, vM, update_mc, k == reuse);
            }
        }
        if (o.combine_with(nr, w, tfc, jac, rng)) {
            selected = k + 1;
            if (vis) o.flags |= RF_UNOCCLUDED;
            else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
            else o.flags &= ~RF_UNOCCLUDED;
        }
    }
    // ReSTIRDISpatiotemporalNormalizationWeight (SpatiotemporalNormalizationWeight.h)
    float nn = 1.0f, nd = 1.0f;
    if (o.wsum > 0.0f && (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z ||
                          mode == MPT_RESTIR_DI_BIAS_MIS_LIKE)) {
        nn = mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? 0.0f : 1.0f;
        nd = 0.0f;
        for (int j = 0; j < reuse + 1; j++) {
            int nj = valid_nb(j);
            if (nj == -1) continue;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) {
                nd += (float)(j == reuse ? ic.M : tin[(size_t)nj].M);
                continue;
            }
            // the MIS-like loop reads the current frame's G-buffer (SpatiotemporalNormalizationWeight.h:130)
            RSurface js = j == reuse ? cs : surface_of(nb_gb(nj, mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? false : use_prev));
            float tj = restir_target(c, rr.at(RP_NORM(j)), o.tri, o.point, o.flags, js, bvis);
            if (tj > 0.0f) {
                if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) nd += (float)(j == reuse ? ic.M : tin[(size_t)nj].M);
                else {
                    int M = 1;
                    if (cw) M = j == reuse ? ic.M : tin[(size_t)nj].M;
                    if (j + 1 == selected) nn += tj;
                    nd += tj * (float)M;
                }
            }
        }
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) nd += (float)tres.M;
        else {
            float tt = restir_target(c, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis);
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) { if (tt > 0.0f) nd += (float)tres.M; }
            else {
                if (selected == 0) nn += tt;
                nd += tt * (float)(cw ? tres.M : 1);
            }
        }
    }
    o.end_with_normalization(nn, nd);
    const bool vreuse = bvis && (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z || mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS ||
                                 mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE) &&
                        (f.options.restir_di_do_visibility_reuse ||
                         (f.options.restir_di_initial_target_visibility && f.options.restir_di_spatial_target_visibility));
    if (vreuse && (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index))
        restir_visibility_reuse(c, rr, o, cs.sp, cs.last_hit);
    if (rd.m_cap > 0) o.M = std::min(o.M, rd.m_cap);
    out[(size_t)center] = o;
}

// ReSTIR_DI_TemporalReuse (TemporalReuse.h:48-306) of the unfused chain: pairwise-MIS-
// defensive weights (TemporalMISWeight.h:203-279), normalisation 1 / 1, visibility in the
// target function (ReSTIR_DI_BiasCorrectionUseVisibility).  tin = last frame's output.
void restir_temporal(Ctx& c, RestirPassCtx& R, int x, int y, std::vector<OResv>& tin, std::vector<OResv>& out) {
    const MptFrame& f = R.f;
    const MptReSTIRDISettings& rd = f.render_settings.restir_di_settings;
    const OScene& s = *c.s;
    const int mode = f.options.restir_di_bias_correction_weights;
    const bool bvis = f.options.restir_di_bias_correction_use_visibility != 0;
    const bool cw = rd.use_confidence_weights;
    int W = f.res_x;
    int center = x + y * W;
    const GB& g = R.cur[(size_t)center];
    if (!R.active[(size_t)center] || !g.hit) return;
    uint32_t seed = pass_seed(f, (uint32_t)center, f.restir_di_seeds[2]);
    Rng rng(seed);
    c.pseed = seed;
    RestirRays rr{c, 8};
    if (rd.temporal_buffer_clear_requested) tin[(size_t)center] = OResv();
    RSurface cs = surface_of(g);
    if (is_emissive(g.mat)) return;
    const bool use_prev = rd.do_temporal_reuse_pass;   // use_prev_frame_g_buffer (RenderSettings.h:237-247)
    int tidx, tpx, tpy;
    restir_temporal_neighbor(c, R, g.first_hit, cs.sn, center, rng, tidx, tpx, tpy);
    const OResv ic = R.B.init[(size_t)center];
    if (tidx == -1 || f.render_settings.freeze_random) { out[(size_t)center] = ic; return; }
    const OResv tres = tin[(size_t)tidx];
    if (tres.M == 0) { out[(size_t)center] = ic; return; }
    const GB& tg = use_prev ? R.prev[(size_t)tidx] : R.cur[(size_t)tidx];
    if (is_emissive(tg.mat)) { out[(size_t)center] = ic; return; }
    RSurface ts = surface_of(tg);
    OResv o;
    float mc = 0.0f;
    int selected = 0;   // MIS-like: TEMPORAL_NEIGHBOR_ID 0 / INITIAL_CANDIDATES_ID 1
    // ReSTIRDITemporalResamplingMISWeight<MIS_GBH> (TemporalMISWeight.h:62-110)
    auto gbh = [&](const OResv& r, bool temporal_id) -> float {
        const int cur = temporal_id ? 0 : 1;
        float tt = restir_target(c, rr.at(RP_GBH(cur, 999)), r.tri, r.point, r.flags, ts, bvis);
        if (temporal_id && tt == 0.0f) return 0.0f;
        float tc = restir_target(c, rr.at(RP_GBH(cur, 998)), r.tri, r.point, r.flags, cs, bvis);
        int tM = cw ? tres.M : 1, cM = cw ? ic.M : 1;
        float nume = temporal_id ? tt * (float)tM : tc * (float)cM;
        float denom = tt * (float)tM + tc * (float)cM;
        return denom == 0.0f ? 0.0f : nume / denom;
    };
    {
        float tfc = 0.0f;
        if (tres.UCW > 0.0f) tfc = restir_target(c, rr.at(RP_T_TFC), tres.tri, tres.point, tres.flags, cs, bvis);
        float jac = 1.0f;
        if (tfc > 0.0f && tres.UCW > 0.0f && !(tres.flags & RF_ENVMAP)) {
            jac = restir_jacobian(s, tres, cs.sp, ts.sp - ts.sn * 1.0e-4f);
            if (jac == -1.0f) jac = 0.0f;
        }
        float w;
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) w = (float)tres.M;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) w = cw ? (float)tres.M : 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) w = gbh(tres, true);
        else {
            // pairwise (TemporalMISWeight.h:139-279), TEMPORAL_NEIGHBOR_ID
            const bool def = mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE;
            float tM = cw ? (float)tres.M : 1.0f, cM = cw ? (float)ic.M : 1.0f, nsum = cw ? (float)tres.M : 1.0f;
            float tfn = tres.target;
            float nume = tfn * tM;
            float denom = tfn * nsum + tfc * cM;
            float mi = denom == 0.0f ? 0.0f : (nume / denom);
            if (def && cw) mi *= nsum / (nsum + cM);
            float tcn = restir_target(c, rr.at(RP_T_TCN), ic.tri, ic.point, ic.flags, ts, bvis);
            float tcc = ic.target;
            float nume_mc = tcc * cM;
            float denom_mc = tcn * nsum + tcc * cM;
            float conf = cw ? (def ? nsum / (nsum + cM) : tM / nsum) : 1.0f;
            if (denom_mc != 0.0f) mc += nume_mc / denom_mc * conf;
            w = def && !cw ? mi * 0.5f : mi;
        }
        if (o.combine_with(tres, w, tfc, jac, rng)) {
            selected = 0;
            if (bvis) o.flags |= RF_UNOCCLUDED;
            else o.flags &= ~RF_UNOCCLUDED;
        }
    }
    float wc;
    if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) wc = (float)ic.M;
    else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) wc = cw ? (float)ic.M : 1.0f;
    else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) wc = gbh(ic, false);
    else if (mc == 0.0f) wc = 1.0f;
    else if (mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS) wc = mc;
    else if (cw) wc = mc + (float)ic.M / (float)(ic.M + tres.M);
    else wc = (1.0f + mc) * 0.5f;
    if (o.combine_with(ic, wc, ic.target, 1.0f, rng)) {
        selected = 1;
        if (bvis) o.flags |= RF_UNOCCLUDED;
        else o.flags |= ic.flags & RF_UNOCCLUDED;
    }
    // ReSTIRDITemporalNormalizationWeight (TemporalNormalizationWeight.h)
    float nn = 1.0f, nd = 1.0f;
    if (o.wsum > 0.0f) {
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) nd = (float)(ic.M + tres.M);
        else if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) {
            nd = 0.0f;
            float tc = restir_target(c, rr.at(RP_NORM(998)), o.tri, o.point, o.flags, cs, bvis);
            nd += (float)((tc > 0.0f) * ic.M);
            float tt = restir_target(c, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis);
            nd += (float)((tt > 0.0f) * tres.M);
        } else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) {
            float tc = restir_target(c, rr.at(RP_NORM(998)), o.tri, o.point, o.flags, cs, bvis);
            float tt = restir_target(c, rr.at(RP_NORM(999)), o.tri, o.point, o.flags, ts, bvis);
            nn = selected == 1 ? tc : tt;
            int icM = cw ? ic.M : 1, tM = cw ? tres.M : 1;
            nd = tc * (float)icM + tt * (float)tM;
        }
    }
    o.end_with_normalization(nn, nd);
    if (rd.m_cap > 0) o.M = std::min(o.M, rd.m_cap);
    out[(size_t)center] = o;
}

// ReSTIR_DI_SpatialReuse (SpatialReuse.h:52-348)
void restir_spatial(Ctx& c, RestirPassCtx& R, int x, int y, int pass, std::vector<OResv>& in, std::vector<OResv>& out) {
    const MptFrame& f = R.f;
    MptReSTIRDISettings rd = f.render_settings.restir_di_settings;
    rd.spatial_pass_index = pass;
    const OScene& s = *c.s;
    const int mode = f.options.restir_di_bias_correction_weights;
    const bool bvis = f.options.restir_di_bias_correction_use_visibility != 0;
    int W = f.res_x;
    int center = x + y * W;
    const GB& g = R.cur[(size_t)center];
    if (!R.active[(size_t)center] || !g.hit) return;
    const uint32_t pass_rs = f.restir_di_seeds[4 + pass];
    uint32_t seed = pass_seed(f, (uint32_t)center, pass_rs);
    Rng rng(seed);
    c.pseed = seed;
    RestirRays rr{c, 7};
    OResv o;
    RSurface cs = surface_of(g);
    if (is_emissive(g.mat)) return;
    float rot = rd.do_neighbor_rotation ? TWO_PI * rng() : 0.0f;
    float cr = pcos(rot), sr = psin(rot);
    OResv cres = in[(size_t)center];
    if (cres.M <= 1 && rd.do_disocclusion_reuse_boost) rd.reuse_neighbor_count = rd.disocclusion_reuse_count;
    int reuse = rd.reuse_neighbor_count;
    const bool cw = rd.use_confidence_weights;
    // count_valid_spatial_neighbors (Utils.h:356-378): current-frame G-buffer
    int cache = 0, vcount = 0, vM = 0;
    for (int k = 0; k < reuse; k++) {
        int ni = restir_spatial_neighbor(f, k, reuse, rd.reuse_radius, x, y, cr, sr, R.conv, pass_rs);
        if (ni == -1) continue;
        if (!restir_similar(rd, R.cur[(size_t)ni], R.prev[(size_t)ni], g, cs.sp, cs.sn, false)) continue;
        vM += in[(size_t)ni].M;
        vcount++;
        cache |= 1 << k;
    }
    // neighbours visited by the normalisation / GBH loops (center included, j == reuse)
    auto valid_nb = [&](int j) -> int {
        int nj = restir_spatial_neighbor(f, j, reuse, rd.reuse_radius, x, y, cr, sr, R.conv, pass_rs);
        if (nj == -1) return -1;
        return restir_similar(rd, R.cur[(size_t)nj], R.prev[(size_t)nj], g, cs.sp, cs.sn, false) ? nj : -1;
    };
    PairwiseMIS mis;
    mis.defensive = mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE;
    mis.bvis = bvis;
    int selected = 0;
    int start = vM == 0 ? reuse : 0;
    for (int k = start; k < reuse + 1; k++) {
        if (k < reuse && reuse <= 32 && (cache & (1 << k)) == 0) continue;
        int ni = restir_spatial_neighbor(f, k, reuse, rd.reuse_radius, x, y, cr, sr, R.conv, pass_rs);
        if (ni == -1) continue;
        if (k < reuse && reuse > 32 && !restir_similar(rd, R.cur[(size_t)ni], R.prev[(size_t)ni], g, cs.sp, cs.sn, false)) continue;
        OResv nr = in[(size_t)ni];
        float tfc = 0.0f;
        bool vis = spatial_visibility(f, rd, k, reuse);
        if (nr.UCW > 0.0f) {
            if (k == reuse) tfc = nr.target;
            else tfc = restir_target(c, rr.at(RP_TFC(k)), nr.tri, nr.point, nr.flags, cs, vis);
        }
        float jac = 1.0f;
        if (tfc > 0.0f && nr.UCW > 0.0f && k != reuse && !(nr.flags & RF_ENVMAP)) {
            const GB& ng = R.cur[(size_t)ni];
            jac = restir_jacobian(s, nr, cs.sp, ng.first_hit);
            if (jac == -1.0f) { o.M += nr.M; continue; }
        }
        float w;
        if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) w = (float)nr.M;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_LIKE) w = cw ? (float)nr.M : 1.0f;
        else if (mode == MPT_RESTIR_DI_BIAS_MIS_GBH) {
            // ReSTIRDISpatialResamplingMISWeight<MIS_GBH> (SpatialMISWeight.h:36-93)
            if (nr.UCW <= 0.0f) w = 1.0f;
            else {
                float nume = 0.0f, denom = 0.0f;
                for (int j = 0; j < reuse + 1; j++) {
                    int nj = valid_nb(j);
                    if (nj == -1) continue;
                    RSurface js = surface_of(R.cur[(size_t)nj]);
                    float tj = restir_target(c, rr.at(RP_GBH(k, j)), nr.tri, nr.point, nr.flags, js, bvis);
                    int M = cw ? in[(size_t)nj].M : 1;
                    denom += tj * (float)M;
                    if (j == k) nume = tj * (float)M;
                }
                w = denom == 0.0f ? 0.0f : nume / denom;
            }
        } else {
            bool update_mc = cres.M > 0 && cres.UCW > 0.0f;
            w = mis.weight(c, rr.at(RP_TCN(k)), rd, nr, cres, tfc, R.cur[(size_t)ni], vcount, vM, update_mc, k == reuse);
        }
        if (o.combine_with(nr, w, tfc, jac, rng)) {
            selected = k;
            if (vis) o.flags |= RF_UNOCCLUDED;
            else if (k == reuse) o.flags |= nr.flags & RF_UNOCCLUDED;
            else o.flags &= ~RF_UNOCCLUDED;
        }
    }
    // ReSTIRDISpatialNormalizationWeight (SpatialNormalizationWeight.h)
    float nn = 1.0f, nd = 1.0f;
    if (o.wsum > 0.0f && (mode == MPT_RESTIR_DI_BIAS_1_OVER_M || mode == MPT_RESTIR_DI_BIAS_1_OVER_Z ||
                          mode == MPT_RESTIR_DI_BIAS_MIS_LIKE)) {
        nn = mode == MPT_RESTIR_DI_BIAS_MIS_LIKE ? 0.0f : 1.0f;
        nd = 0.0f;
        for (int j = 0; j < reuse + 1; j++) {
            int nj = valid_nb(j);
            if (nj == -1) continue;
            if (mode == MPT_RESTIR_DI_BIAS_1_OVER_M) { nd += (float)in[(size_t)nj].M; continue; }
            RSurface js = surface_of(R.cur[(size_t)nj]);
            float tj = restir_target(c, rr.at(RP_NORM(j)), o.tri, o.point, o.flags, js, bvis);
            if (tj > 0.0f) {
                int M = in[(size_t)nj].M;
                if (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z) nd += (float)M;
                else {
                    if (!cw) M = 1;
                    if (j == selected) nn += tj;
                    nd += tj * (float)M;
                }
            }
        }
    }
    o.end_with_normalization(nn, nd);
    const bool vreuse = bvis && (mode == MPT_RESTIR_DI_BIAS_1_OVER_Z || mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS ||
                                 mode == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE) &&
                        (f.options.restir_di_do_visibility_reuse ||
                         (f.options.restir_di_initial_target_visibility && f.options.restir_di_spatial_target_visibility));
    if (vreuse && (rd.do_temporal_reuse_pass || rd.number_of_passes - 1 != rd.spatial_pass_index))
        restir_visibility_reuse(c, rr, o, cs.sp, cs.last_hit);
    if (rd.m_cap > 0) o.M = std::min(o.M, rd.m_cap);
    out[(size_t)center] = o;
}

// sample_light_ReSTIR_DI + evaluate_ReSTIR_DI_reservoir (FinalShading.h:16-115)
Col restir_final_shading(Ctx& c, OResv& res, const Payload& pl, const HitInfo& hi, f3 view) {
    const MptWorldSettings& w = c.f->world_settings;
    if ((res.flags & RF_ENVMAP) && w.ambient_light_type != MPT_AMBIENT_ENVMAP) res.UCW = 0.0f;   // validate_reservoir
    if (res.UCW <= 0.0f) return Col(0.0f);
    float dist;
    f3 dir;
    if (res.flags & RF_ENVMAP) { dir = mat_x_vec(w.envmap_to_world_matrix, res.point); dist = 1.0e35f; }
    else { dir = res.point - hi.inter_point; dir = dir / (dist = length(dir)); }
    bool shadow = false;
    if (res.flags & RF_UNOCCLUDED) shadow = false;
    else if (c.f->render_settings.restir_di_settings.do_final_shading_visibility)
        shadow = shadow_ray(c, hi.inter_point, dir, dist, hi.prim, 1);
    Col out;
    if (!shadow) {
        float bp;
        VolumeState tv = pl.vs;
        Col bc = bsdf_eval(c.bc, c.override_, pl.material, tv, view, hi.shading_normal, hi.geometric_normal, dir, bp);
        float cosv = dot(hi.shading_normal, dir);
        if (res.flags & RF_BSDF_REFRACTION) cosv = absf(cosv);
        if (cosv > 0.0f) {
            Col e;
            if (res.flags & RF_ENVMAP) { float ep; e = envmap_eval(c, dir, ep); }
            else e = emission_of(c.s->mats[c.s->mat_idx[res.tri]]);
            out = bc * res.UCW * e * cosv;
        }
    }
    return out;
}
