// mpt_kernels.hip -- the MI355X wavefront path tracer (hot path).
//
// One frame = one sample per pixel of the context's row partition:
//
//   k_camera ............ CameraRays ray generation (Device/kernels/CameraRays.h:45-142)
//   for bounce in 0..nb_bounces:                        (FullPathTracer.h:155-290)
//     k_trace<closest, volume-aware> over the active-path queue: BVH8 traversal +
//                       nested-dielectric boundary skipping (Intersect.h:114-206)
//     k_shade ........... hit processing, emission, every RNG draw of the vertex in the
//                       reference order (light sampling Lights.h / RIS.h, envmap
//                       Envmap.h, BSDF continuation, Russian roulette), appends the
//                       vertex's NEE queries (shadow any-hit + BSDF closest-hit) and the
//                       continuation ray with wave64 ballot compaction
//     k_trace<any> / k_trace<closest> over the NEE queues
//     k_resolve ......... finishes RIS / MIS / envmap-MIS with the trace results, clamps
//                       and adds to the path radiance (FullPathTracer.h:196-214)
//   k_accumulate ........ sanity check + running-sum framebuffer / AOVs (FullPathTracer.h:292-327)
//
// RNG: each path owns one Xorshift32 stream seeded exactly as the reference
// (wang_hash((pixel+1)*(sample+1)*random_seed), FullPathTracer.h:124-129); every draw
// happens in k_shade in the reference's order, and the trace results only decide how
// the already-drawn values are used, so the stream is identical to the megakernel's.
//
// BVH8 traversal: one ray per lane, 64 rays fetched per wave from a global counter
// (persistent waves), node groups (child base, internal mask, remaining-hit mask)
// on a 12-deep LDS stack per lane with a global spill area, octant-ordered children
// (near-to-far without sorting), leaves tested as soon as their node is opened.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstring>
#include <initializer_list>
#include <type_traits>
#include <utility>

#include "dev_bsdf.h"
#include "mpt_internal.h"

namespace mpt {

constexpr int TB = TRAV_BLOCK;
constexpr int MAX_BOUNDARY_SKIPS = 16;   // trace_ray's volume-boundary skip loop bound
#ifndef MPT_TRACE_REFILL
#define MPT_TRACE_REFILL 32
#endif
#ifndef MPT_TRACE_BUDGET
#define MPT_TRACE_BUDGET 16
#endif
constexpr int TRACE_REFILL = MPT_TRACE_REFILL;   // idle lanes of a wave that trigger a refill
constexpr int TRACE_BUDGET = MPT_TRACE_BUDGET;   // nodes a lane opens between refill checks
#ifndef MPT_TRACE_CHUNK
#define MPT_TRACE_CHUNK 256
#endif
constexpr int TRACE_CHUNK = MPT_TRACE_CHUNK;     // rays a wave claims per atomic on the work counter
static_assert(TRACE_CHUNK >= 64, "a refill of up to 64 lanes must fit in one new chunk");
#ifndef MPT_TRI_POSTPONE
#define MPT_TRI_POSTPONE 3
#endif
constexpr int TRI_POSTPONE = MPT_TRI_POSTPONE;   // triangle loop runs with >= 1/TRI_POSTPONE of the lanes
constexpr uint32_t TRI_GROUP = 0x80000000u;      // stack entry tag of a triangle group
constexpr int LDS_STACK = TRAV_LDS_STACK;
constexpr int SPILL_DEPTH = TRAV_SPILL_DEPTH;

// ----------------------------------------------------------------------------------
// wave64 helpers
// ----------------------------------------------------------------------------------
DEV int lane_id() { return __lane_id(); }
// storage index of staged NEE query id (slot * 4 + kind): kind-major planes (DevPaths::nq_o)
DEV size_t nq_index(const DevPaths& P, int id) { return (size_t)(id & 3) * (size_t)P.nq_stride + (size_t)(id >> 2); }
// storage index of staged ReSTIR DI ray id (slot * RS_RPP + position): position-major planes
// (DevPaths::rq_o / rq_d / rq_key / rq_occ), so that a block's lanes (consecutive slots) staging
// the same position write one contiguous run
DEV size_t rq_phys(const DevPaths& P, int id) {
    const int s = id / RS_RPP_HOST;
    return (size_t)(id - s * RS_RPP_HOST) * (size_t)P.n + (size_t)s;
}
// record k of slot s (DevPaths::rq_rec): record-major planes
DEV size_t rq_rec_at(const DevPaths& P, int s, int k) { return (size_t)k * (size_t)P.n + (size_t)s; }
DEV int wave_append(int32_t* counter, bool pred) {
    unsigned long long m = __ballot(pred);
    unsigned long long act = __ballot(1);
    int leader = __ffsll((long long)act) - 1;
    int cnt = __popcll(m);
    int base = 0;
    if (lane_id() == leader && cnt) base = atomicAdd(counter, cnt);
    base = __shfl(base, leader);
    unsigned long long lower = m & ((1ull << lane_id()) - 1ull);
    return base + __popcll(lower);
}

// ----------------------------------------------------------------------------------
// BVH8 traversal
// ----------------------------------------------------------------------------------
struct THit { int prim; float t, u, v; };

// Alpha testing (filter_function, FilterFunction.h:19-48).  The reference draws one
// path RNG number per candidate hit inside HIPRT's traversal, so its RNG stream depends
// on the traversal order of a particular BVH.  Here the candidate's uniform is a hash of
// (query key, primitive): the accept probability per candidate is the same
// (alpha_opacity * base-colour alpha), so the expected image is the reference's, and
// the result no longer depends on the traversal order (the oracle reproduces it bit
// for bit).  The key is positional: pixel seed, bounce, query kind, boundary-skip pass.
DEV uint32_t alpha_key(uint32_t pixel_seed, int bounce, int kind, int iter) {
    return wang_hash(pixel_seed ^ wang_hash((uint32_t)(bounce * 8 + kind) * 0x85EBCA77u + (uint32_t)iter * 0xC2B2AE3Du + 1u));
}
DEV float alpha_uniform(uint32_t key, int prim) {
    uint32_t h = wang_hash(key ^ ((uint32_t)prim * 0x9E3779B1u));
    h = wang_hash(h + 0x7F4A7C15u);
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}
DEV bool alpha_rejects(const DevScene& S, int prim, float u, float v, uint32_t key);

// The node test's children in pairs through packed fp32 arithmetic and v_bfm leaf ranges (264 -> 220
// VALU per 8-child node; C3 path rays -1.5 %, shadow rays -2.3 %, C5 path rays -1.8 %:
// profiles/r05f_*_trav_pk_ab.jsonl); 0: the scalar loop
#ifndef MPT_TRAV_PK
#define MPT_TRAV_PK 1
#endif
DEV uint32_t qbyte(uint32_t w0, uint32_t w1, int s) { return ((s < 4 ? w0 : w1) >> ((s & 3) * 8)) & 0xffu; }

// Resumable BVH8 traversal of one ray: init() sets it up, run() opens nodes until the
// traversal ends (true) or `budget` nodes have been opened (false, the state is kept for
// the next call).  Stopping between nodes lets the traversal kernel hand a finished lane
// a new ray while the rest of its wave is still traversing.
// TIE (any hit only): a triangle also counts when it lies exactly at t_max with a primitive
// index below `tie` -- the whole-scene check of a light-hit candidate (TM_NEE_LIGHT_OCC),
// where that triangle would win the closest-hit tie against the light.
template <bool ANY, bool STATS, bool TIE = false>
struct Trav {
    v3 o, d;
    float ix, iy, iz;
    int xr;
    float best;          // closest: current closest t; any: t_max (unchanged until the hit)
    int bprim;
    float bu, bv;
    uint32_t bcls;       // closest: the material class of the hit (TriRec::pad1)
    uint32_t gbase, gimask, gk;   // current node group: child base, internal mask, remaining hits
    int sp;
    int last_hit;
    uint32_t akey;
    bool alpha_on;
    int tie;

    DEV void init(v3 o_, v3 d_, int lh, float tmax, bool al, uint32_t key) {
        o = o_;
        d = d_;
        ix = 1.0f / (fabsf(d.x) > 1e-30f ? d.x : copysignf(1e-30f, d.x));
        iy = 1.0f / (fabsf(d.y) > 1e-30f ? d.y : copysignf(1e-30f, d.y));
        iz = 1.0f / (fabsf(d.z) > 1e-30f ? d.z : copysignf(1e-30f, d.z));
        int oct = (d.x > 0.0f ? 1 : 0) | (d.y > 0.0f ? 2 : 0) | (d.z > 0.0f ? 4 : 0);
        xr = oct ^ 7;
        best = ANY ? tmax : INFINITY;
        bprim = -1;
        bu = 0.0f;
        bv = 0.0f;
        bcls = 0u;
        gbase = 0;
        gimask = 1u;
        gk = 1u << (0 ^ xr);
        sp = 0;
        last_hit = lh;
        akey = key;
        alpha_on = al;
    }

    DEV void push(uint2* lds, uint32_t* spill, uint2 e) {
        if (sp < LDS_STACK) lds[sp * TB + threadIdx.x] = e;
        else { spill[2 * (sp - LDS_STACK)] = e.x; spill[2 * (sp - LDS_STACK) + 1] = e.y; }
        ++sp;
    }

    // Node groups (child base, internal mask | remaining hits << 8) and triangle groups
    // (first triangle record, hit mask | TRI_GROUP) share the stack.  A node's hit leaves
    // form one triangle group (a node's triangles are contiguous, at most 8 x 3).  The
    // triangle loop tests one triangle per iteration and is postponed (its group pushed)
    // while fewer than 1/TRI_POSTPONE of the wave's traversing lanes have triangles to
    // test, so that triangle tests run with more lanes at a time (the closest hit does
    // not depend on the test order: ties go to the lower primitive index).
    DEV bool run(const DevScene& S, const Node8* bvh_nodes, const TriRec* bvh_tris, uint2* lds, uint32_t* spill, int budget,
                 uint32_t& n_nodes, uint32_t& n_tris, uint32_t* n_slots = nullptr) {
        const float4* nodes = reinterpret_cast<const float4*>(bvh_nodes);
        const float4* tris = reinterpret_cast<const float4*>(bvh_tris);
        const int tid = threadIdx.x;
        uint32_t tbase = 0u, tmask = 0u;   // current triangle group
        while (true) {
            if (gk == 0) {
                if (sp == 0) return true;
                if (budget <= 0) return false;
                --sp;
                uint2 e;
                if (sp < LDS_STACK) e = lds[sp * TB + tid];
                else { e.x = spill[2 * (sp - LDS_STACK)]; e.y = spill[2 * (sp - LDS_STACK) + 1]; }
                if (e.y & TRI_GROUP) { tbase = e.x; tmask = e.y & ~TRI_GROUP; }
                else { gbase = e.x; gimask = e.y & 0xffu; gk = e.y >> 8; }
            } else if (budget <= 0) {
                return false;
            }
            if (gk != 0) {
                --budget;
                int k = __builtin_ctz(gk);
                gk &= gk - 1u;
                int s = k ^ xr;
                uint32_t ni = gbase + (uint32_t)__builtin_popcount(gimask & ((1u << s) - 1u));
                if (gk) push(lds, spill, make_uint2(gbase, gimask | (gk << 8)));
                if (STATS) {
                    n_nodes++;
                    if (n_slots && lane_id() == __ffsll((long long)__ballot(1)) - 1) n_slots[0] += 64;
                }
                const float4 n0 = nodes[5 * (size_t)ni + 0];
                const float4 n1 = nodes[5 * (size_t)ni + 1];
                const float4 n2 = nodes[5 * (size_t)ni + 2];
                const float4 n3 = nodes[5 * (size_t)ni + 3];
                const float4 n4 = nodes[5 * (size_t)ni + 4];
                uint32_t eb = __float_as_uint(n0.w);
                float sx = __uint_as_float((eb & 0xffu) << 23), sy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                      sz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
                uint32_t imask = eb >> 24;
                float ax = (n0.x - o.x) * ix, ay = (n0.y - o.y) * iy, az = (n0.z - o.z) * iz;
                float cx = sx * ix, cy = sy * iy, cz = sz * iz;
                uint32_t lox0 = __float_as_uint(n2.x), lox1 = __float_as_uint(n2.y);
                uint32_t loy0 = __float_as_uint(n2.z), loy1 = __float_as_uint(n2.w);
                uint32_t loz0 = __float_as_uint(n3.x), loz1 = __float_as_uint(n3.y);
                uint32_t hix0 = __float_as_uint(n3.z), hix1 = __float_as_uint(n3.w);
                uint32_t hiy0 = __float_as_uint(n4.x), hiy1 = __float_as_uint(n4.y);
                uint32_t hiz0 = __float_as_uint(n4.z), hiz1 = __float_as_uint(n4.w);
                // near / far planes by direction sign
                uint32_t nx0 = ix >= 0.0f ? lox0 : hix0, nx1 = ix >= 0.0f ? lox1 : hix1;
                uint32_t fx0 = ix >= 0.0f ? hix0 : lox0, fx1 = ix >= 0.0f ? hix1 : lox1;
                uint32_t ny0 = iy >= 0.0f ? loy0 : hiy0, ny1 = iy >= 0.0f ? loy1 : hiy1;
                uint32_t fy0 = iy >= 0.0f ? hiy0 : loy0, fy1 = iy >= 0.0f ? hiy1 : loy1;
                uint32_t nz0 = iz >= 0.0f ? loz0 : hiz0, nz1 = iz >= 0.0f ? loz1 : hiz1;
                uint32_t fz0 = iz >= 0.0f ? hiz0 : loz0, fz1 = iz >= 0.0f ? hiz1 : loz1;
                uint32_t meta0 = __float_as_uint(n1.z), meta1 = __float_as_uint(n1.w);
                uint32_t hit_internal = 0u;   // k-ordered
                uint32_t hit_tris = 0u;       // triangle offsets from the node's tri_base
#if MPT_TRAV_PK
                // children in pairs: the near/far plane distances through packed fp32 FMA and the
                // far-distance widening through packed multiply (v_pk_fma_f32 / v_pk_mul_f32: two
                // IEEE operations per instruction, the same bits as the scalar forms)
                typedef float pf2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int c2 = 0; c2 < 8; c2 += 2) {
                    float tn2[2], tf2[2];
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int c = c2 + j;
                        const pf2 qx = {(float)qbyte(nx0, nx1, c), (float)qbyte(fx0, fx1, c)};
                        const pf2 qy = {(float)qbyte(ny0, ny1, c), (float)qbyte(fy0, fy1, c)};
                        const pf2 qz = {(float)qbyte(nz0, nz1, c), (float)qbyte(fz0, fz1, c)};
                        const pf2 px = __builtin_elementwise_fma(qx, (pf2){cx, cx}, (pf2){ax, ax});
                        const pf2 py = __builtin_elementwise_fma(qy, (pf2){cy, cy}, (pf2){ay, ay});
                        const pf2 pz = __builtin_elementwise_fma(qz, (pf2){cz, cz}, (pf2){az, az});
                        tn2[j] = fmaxf(fmaxf(px.x, py.x), fmaxf(pz.x, 0.0f));
                        tf2[j] = fminf(fminf(px.y, py.y), fminf(pz.y, best));
                    }
                    const pf2 tfw = (pf2){tf2[0], tf2[1]} * (pf2){1.0000009f, 1.0000009f};
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const int c = c2 + j;
                        bool h = tn2[j] <= tfw[j];
                        bool internal = (imask >> c) & 1u;
                        if (h && internal) hit_internal |= 1u << (c ^ xr);
                        // leaf: count (meta >> 5) triangles from offset (meta & 31).  Internal slots
                        // hold their rank (< 8) and empty slots 0, so their count field is 0 and
                        // the mask is empty without testing the internal bit: one v_bfm_b32
                        // (offset from the low 5 bits of its operand) builds the range
                        const uint32_t mw = c < 4 ? meta0 : meta1, msh = 8u * (c & 3);
                        uint32_t lm;
                        asm("v_bfm_b32 %0, %1, %2" : "=v"(lm) : "v"((mw >> (msh + 5u)) & 7u), "v"(mw >> msh));
                        if (h) hit_tris |= lm;
                    }
                }
#else
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    float tnx = fmaf((float)qbyte(nx0, nx1, c), cx, ax), tfx = fmaf((float)qbyte(fx0, fx1, c), cx, ax);
                    float tny = fmaf((float)qbyte(ny0, ny1, c), cy, ay), tfy = fmaf((float)qbyte(fy0, fy1, c), cy, ay);
                    float tnz = fmaf((float)qbyte(nz0, nz1, c), cz, az), tfz = fmaf((float)qbyte(fz0, fz1, c), cz, az);
                    float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, 0.0f));
                    float tf = fminf(fminf(tfx, tfy), fminf(tfz, best)) * 1.0000009f;
                    bool h = tn <= tf;
                    uint32_t meta = qbyte(meta0, meta1, c);
                    bool internal = (imask >> c) & 1u;
                    if (h && internal) hit_internal |= 1u << (c ^ xr);
                    // leaf: count (meta >> 5) triangles from offset (meta & 31); empty slots have meta 0
                    if (h && !internal) hit_tris |= ((1u << (meta >> 5)) - 1u) << (meta & 31u);
                }
#endif
                if (hit_tris) {
                    // the current triangle group is empty here (popped groups go straight to the loop)
                    tbase = __float_as_uint(n1.y);
                    tmask = hit_tris;
                }
                gbase = __float_as_uint(n1.x);
                gimask = imask;
                gk = hit_internal;
            }
            const int n_act = __popcll(__ballot(1));
            while (tmask) {
                if (__popcll(__ballot(1)) * TRI_POSTPONE < n_act) {
                    push(lds, spill, make_uint2(tbase, tmask | TRI_GROUP));
                    tmask = 0u;
                    break;
                }
                const uint32_t ti = tbase + (uint32_t)__builtin_ctz(tmask);
                tmask &= tmask - 1u;
                if (STATS) {
                    n_tris++;
                    if (n_slots && lane_id() == __ffsll((long long)__ballot(1)) - 1) n_slots[1] += 64;
                }
                const float4 t0 = tris[3 * (size_t)ti + 0];
                const float4 t1 = tris[3 * (size_t)ti + 1];
                const float4 t2 = tris[3 * (size_t)ti + 2];
                int prim = (int)__float_as_uint(t0.w);
                // Moller-Trumbore exactly as Renderer/Triangle.h:20-62 (no contraction)
                v3 e1 = mk3(t1.x, t1.y, t1.z), e2 = mk3(t2.x, t2.y, t2.z);
                v3 h = cross(d, e2);
                float a = dot(e1, h);
                if (a > -0.0000001f && a < 0.0000001f) continue;
                float f = 1.0f / a;
                v3 sv = o - mk3(t0.x, t0.y, t0.z);
                float u = f * dot(sv, h);
                if (u < 0.0f || u > 1.0f) continue;
                v3 q = cross(sv, e1);
                float v = f * dot(d, q);
                if (v < 0.0f || u + v > 1.0f) continue;
                float t = f * dot(e2, q);
                if (!(t > 0.0000001f)) continue;
                if (prim == last_hit) continue;
                // alpha-tested triangle (flag in the record): only when it would be kept
                const bool nearer = ANY ? (t < best || (TIE && t == best && prim < tie))
                                        : (t < best || (t == best && prim < bprim));
                if (alpha_on && __float_as_uint(t1.w) != 0u && nearer && alpha_rejects(S, prim, u, v, akey))
                    continue;
                if (ANY) {
                    if (nearer) {
                        bprim = prim; best = t; bu = u; bv = v;
                        gk = 0u; sp = 0;
                        return true;
                    }
                } else if (t < best || (t == best && prim < bprim)) {
                    best = t; bprim = prim; bu = u; bv = v; bcls = __float_as_uint(t2.w);
                }
            }
        }
    }
};

template <bool ANY, bool STATS>
DEV bool traverse(const DevScene& S, v3 o, v3 d, int last_hit, float tmax, THit& out, uint2* lds, uint32_t* spill,
                  uint32_t& n_nodes, uint32_t& n_tris, bool alpha_on = false, uint32_t akey = 0u) {
    Trav<ANY, STATS> tr;
    tr.init(o, d, last_hit, tmax, alpha_on, akey);
    tr.run(S, S.nodes, S.tris, lds, spill, 0x7fffffff, n_nodes, n_tris);
    out.prim = tr.bprim;
    out.t = tr.best;
    out.u = tr.bu;
    out.v = tr.bv;
    return tr.bprim >= 0;
}

// Ray sources of the persistent traversal kernel
// TM_NEE_LIGHT / TM_NEE_LIGHT_OCC answer the light-hit queries (kind 3) exactly like
// TM_NEE_CLOSEST in two steps (build_light_bvh in mpt_api.cpp): the closest hit among the
// triangles that can emit, then an any-hit query over the whole scene up to that hit for
// the candidates found; they report in TM_NEE_CLOSEST's stage (timing, counters).
// TM_LIST_ANY: any-hit queries staged by the ReSTIR DI reuse passes (raw_o / raw_d / raw_key
// at the positions of a compacted list; results in raw_occ), reported in the raw any-hit
// stage's instrumentation counters (raw queries never run inside a render).
// TM_LIST_CLOSEST: the same for closest-hit queries (hit written to raw_hit at the ray's position).
enum TraceMode { TM_PATH = 0, TM_NEE_ANY = 1, TM_NEE_CLOSEST = 2, TM_RAW_CLOSEST = 3, TM_RAW_ANY = 4, TM_NEE_LIGHT = 5,
                 TM_NEE_LIGHT_OCC = 6, TM_LIST_ANY = 7, TM_LIST_CLOSEST = 8 };
constexpr int trace_stage(int mode) {
    return mode == TM_LIST_ANY ? TM_RAW_ANY : mode == TM_LIST_CLOSEST ? TM_RAW_CLOSEST : mode >= TM_NEE_LIGHT ? TM_NEE_CLOSEST : mode;
}
// Short traversals (the light BVH: ~1.5 nodes per query) run one query per lane over a grid
// covering the list instead of persistent waves: with so little work per query the shared
// work counter of the persistent kernel (one device-scope atomic per wave refill) is what
// the launch would wait on (2.96 ms per C3 launch).  Only when the BVH is shallow enough
// for the stack to stay in LDS (the global spill area is sized for the persistent grid):
// TraceArgs::static_grid, set by the host from the light BVH's depth.

struct TraceArgs {
    DevScene S;
    DevPaths P;
    const int32_t* queue;      // TM_PATH: slot list
    const int32_t* count_ptr;  // device count (TM_PATH / NEE)
    int count_const;           // RAW
    int32_t* fetch;            // work counter (zeroed before the launch)
    const float4* raw_o;
    const float4* raw_d;
    float4* raw_hit;
    uint8_t* raw_occ;
    const uint32_t* raw_key;   // TM_LIST_ANY: alpha key per ray (alpha testing on)
    const MptFrame* F;         // frame constants (alpha keys); NULL for raw queries
    int bounce;
    int alpha;                 // render_settings.do_alpha_testing
    int static_grid;           // TM_NEE_LIGHT: one query per lane (the light BVH's stack fits in LDS)
    int ext;                   // NEE modes: the extended-light-sampling queries (P.xq_*, P.xl_*)
};
DEV uint32_t slot_pixel(const MptFrame& F, int slot, int& x, int& y);
DEV uint32_t pixel_seed(const MptFrame& F, uint32_t pix);
DEV uint32_t camera_seed(const MptFrame& F, uint32_t pix);
DEV uint32_t path_seed(const MptFrame* Fp, const DevPaths& P, int slot, bool camera);

template <int MODE, bool STATS>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(
    MODE == TM_PATH ? MPT_TRACE_WAVES_PATH : (MODE == TM_LIST_ANY || MODE == TM_LIST_CLOSEST) ? MPT_TRACE_WAVES_LIST : MPT_TRACE_WAVES)))
    void k_trace(TraceArgs A) {
    __shared__ uint2 lds[LDS_STACK * TB];
    const DevScene& S = A.S;
    const DevPaths& P = A.P;
    const int count = (MODE == TM_RAW_CLOSEST || MODE == TM_RAW_ANY) ? A.count_const : *A.count_ptr;
    // a static grid covers the wavefront; blocks past the query list leave at once
    if (MODE == TM_NEE_LIGHT && A.static_grid && (int)(blockIdx.x * TB) >= count) return;
    // (a static grid never spills: static_grid requires the stack to fit in LDS)
    uint32_t* spill = P.stack_spill + (MODE == TM_NEE_LIGHT && A.static_grid ? 0 : ((size_t)blockIdx.x * TB + threadIdx.x) * (2 * SPILL_DEPTH));
    uint32_t n_nodes = 0, n_tris = 0, n_rays = 0;
    uint32_t n_slots[2] = {0u, 0u};
    constexpr bool ANY = (MODE == TM_NEE_ANY || MODE == TM_RAW_ANY || MODE == TM_NEE_LIGHT_OCC || MODE == TM_LIST_ANY);
    constexpr bool TIE = MODE == TM_NEE_LIGHT_OCC;
    const Node8* bvh_nodes = MODE == TM_NEE_LIGHT ? S.nodes_light : S.nodes;
    const TriRec* bvh_tris = MODE == TM_NEE_LIGHT ? S.tris_light : S.tris;
    // Persistent waves with per-lane ray replacement: a lane whose ray has finished takes
    // a new one as soon as at least TRACE_REFILL lanes of its wave are idle, instead of the
    // whole wave waiting for its longest ray.  Between refill checks every lane opens at
    // most TRACE_BUDGET nodes.  A wave claims TRACE_CHUNK consecutive rays per atomic on
    // the shared counter and serves its refills from that chunk: the device-scope atomic
    // is a serial point for all 5k waves (one per refill put the short light-BVH
    // traversals at 12 ns per refill, the counter's throughput).  The first chunk of every
    // wave is static -- wave w serves rays [w * sc, (w + 1) * sc) of the first n_waves * sc,
    // sc = count / n_waves rounded up to 64 (at most TRACE_CHUNK) -- so that a launch starts
    // without 20 k waves queueing on the counter, and a launch of fewer rays than
    // n_waves * TRACE_CHUNK (the 1-spp ReSTIR DI wavefronts, the staged ReSTIR rays) takes no
    // atomic at all; later chunks come from the counter, offset by the static part.
    Trav<ANY, STATS, TIE> tr;
    const int n_waves = (int)gridDim.x * (TB / 64);
    const int wave_id = (int)blockIdx.x * (TB / 64) + (int)(threadIdx.x >> 6);
    int sc = (count + n_waves - 1) / max(1, n_waves);
    sc = min(TRACE_CHUNK, max(64, (sc + 63) & ~63));
    const int n_static = (int)min((long long)count, (long long)sc * n_waves);
    bool alive = false;
    bool exhausted = false;   // wave-uniform: the ray counter has passed `count`
    int ray = 0;              // RAW: ray index; NEE: staged query (slot * 4 + kind); PATH: slot
    int skips = 0;            // PATH: volume-boundary re-traces so far
    uint32_t pseed = 0u;      // PATH: pixel seed of the alpha keys
    bool was_inside = false;  // PATH: kept over re-traces, as in trace_ray's loop
    float qmax = 0.0f;        // NEE closest: the query's t_max
    int chunk_next = min(wave_id * sc, n_static);                // wave-uniform: the unserved part of the wave's chunk
    int chunk_end = min(chunk_next + sc, n_static);
    bool counter_done = n_static >= count;                        // wave-uniform: the shared counter has passed `count`
    while (true) {
        const unsigned long long idle = __ballot(!alive);
        if (!exhausted && __popcll(idle) >= (unsigned)TRACE_REFILL) {
            const int need = __popcll(idle);
            int base = 0;
            if (MODE == TM_NEE_LIGHT && A.static_grid) {
                // one ray per lane, 64 consecutive queries per wave, no refill
                base = (int)(blockIdx.x * TB + (threadIdx.x & ~63u));
                exhausted = true;
            }
            int take0 = need, base1 = 0;
            if (!(MODE == TM_NEE_LIGHT && A.static_grid)) {
                // the rest of the chunk first, then (if short) a new chunk
                base = chunk_next;
                take0 = min(need, chunk_end - chunk_next);
                chunk_next += take0;
                if (take0 < need && !counter_done) {
                    int b = 0;
                    if (lane_id() == 0) b = n_static + atomicAdd(A.fetch, TRACE_CHUNK);
                    b = __shfl(b, 0);
                    counter_done = b + TRACE_CHUNK >= count;
                    chunk_end = min(b + TRACE_CHUNK, count);
                    base1 = b;
                    chunk_next = min(b + (need - take0), chunk_end);
                } else {
                    base1 = count;   // nothing left for this wave: the remaining lanes get i >= count
                }
                exhausted = counter_done && chunk_next >= chunk_end;
            }
            if (!alive) {
                const int r = __popcll(idle & ((1ull << lane_id()) - 1ull));
                const int i = r < take0 ? base + r : base1 + (r - take0);
                if (i < count) {
                    alive = true;
                    n_rays++;
                    float4 ro, rd;
                    if (MODE == TM_PATH) {
                        ray = A.queue ? A.queue[i] : i;   // no queue: every slot (batched ReSTIR DI camera rays)
                        ro = ld_s(&P.ray_o[ray]);
                        rd = ld_s(&P.ray_d[ray]);
                        skips = 0;
                        was_inside = false;
                        if (A.alpha)     // bounce 0: the camera launch's seed (CameraRays traces the camera ray)
                            pseed = A.bounce == 0 ? P.seeds[ray].x : P.seeds[ray].y;   // path_seed (k_camera)
                        tr.init(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), (int)__float_as_uint(ro.w), INFINITY,
                                A.alpha != 0, A.alpha ? alpha_key(pseed, A.bounce, 0, 0) : 0u);
                    } else if (MODE == TM_NEE_ANY || MODE == TM_NEE_CLOSEST || MODE == TM_NEE_LIGHT || MODE == TM_NEE_LIGHT_OCC) {
                        // compacted list of staged queries (entry = slot * 4 + kind), see k_compact;
                        // extended light sampling: entries slot * x_per + j (shadow rays alpha kind 1,
                        // light-hit rays kind 4, as their standard counterparts)
                        if (A.ext) ray = MODE == TM_NEE_LIGHT_OCC ? P.xl_light[i] : MODE == TM_NEE_ANY ? P.xl_any[i] : P.xl_cl[i];
                        else ray = MODE == TM_NEE_LIGHT_OCC ? P.nq_light[i]
                                                            : P.nq_tgt[MODE == TM_NEE_ANY ? (size_t)i : (size_t)P.n * 3 + i];
                        ro = A.ext ? P.xq_o[ray] : ld_s(&P.nq_o[nq_index(P, ray)]);
                        rd = A.ext ? P.xq_d[ray] : ld_s(&P.nq_d[nq_index(P, ray)]);
                        qmax = rd.w;
                        const bool al = A.alpha != 0;
                        uint32_t akey = 0u;
                        if (al) akey = A.ext ? alpha_key(P.seeds[ray / P.x_per].y, A.bounce, MODE == TM_NEE_ANY ? 1 : 4, 0)
                                             : alpha_key(P.seeds[ray >> 2].y, A.bounce, (ray & 3) + 1, 0);
                        float tmax = ANY ? rd.w : INFINITY;
                        if (TIE) {
                            // the light candidate of TM_NEE_LIGHT: anything nearer, or as near with a
                            // lower index, is the closest hit instead
                            const float4 h = A.ext ? P.xq_hit[ray] : P.nhit[ray >> 2];
                            tmax = h.x;
                            tr.tie = (int)__float_as_uint(h.w);
                        }
                        tr.init(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), (int)__float_as_uint(ro.w), tmax, al, akey);
                        if (MODE == TM_NEE_LIGHT && S.n_light_tris == 0) tr.gk = 0u;   // no light: nothing to traverse
                    } else if (MODE == TM_LIST_ANY || MODE == TM_LIST_CLOSEST) {
                        ray = (int)rq_phys(P, A.queue[i]);   // the staged ray's storage index
                        ro = A.raw_o[ray];
                        rd = A.raw_d[ray];
                        tr.init(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), (int)__float_as_uint(ro.w), ANY ? rd.w : INFINITY,
                                A.alpha != 0, A.alpha ? A.raw_key[ray] : 0u);
                    } else {
                        ray = i;
                        ro = A.raw_o[i];
                        rd = A.raw_d[i];
                        tr.init(mk3(ro.x, ro.y, ro.z), mk3(rd.x, rd.y, rd.z), (int)__float_as_uint(ro.w), ANY ? rd.w : INFINITY, false, 0u);
                    }
                }
            }
        }
        if (__ballot(alive) == 0) {
            if (exhausted) break;
            continue;
        }
        if (!alive) continue;
        if (!tr.run(S, bvh_nodes, bvh_tris, lds, spill, TRACE_BUDGET, n_nodes, n_tris, STATS ? n_slots : nullptr)) continue;
        const bool found = tr.bprim >= 0;
        if (MODE == TM_PATH) {
            // trace_ray's boundary-skipping loop (Intersect.h:117-206)
            VState vs = vs_load_s(P.vsA, P.vsB, ray);
            bool again = false;
            if (found) {
                was_inside = vs.pos > 0;
                if (was_inside) vs.dist += tr.best;
                int mi = S.mat_idx[tr.bprim];
                bool skip = vs_push(vs, mi, S.mat_prio[mi]);
                // bounded like the oracle: a re-traced ray can keep re-hitting the triangle
                // it sits on (only the original last hit is filtered), see DESIGN.md
                if (skip && ++skips < MAX_BOUNDARY_SKIPS) {
                    vs.dist += tr.best;
                    again = true;
                }
            }
            vs_store_s(P.vsA, P.vsB, ray, vs);
            if (again) {
                n_rays++;
                tr.init(tr.o + tr.best * tr.d, tr.d, tr.last_hit, INFINITY, A.alpha != 0,
                        A.alpha ? alpha_key(pseed, A.bounce, 0, skips) : 0u);
                continue;
            }
            st_s(&P.ray_o[ray], make_float4(tr.o.x, tr.o.y, tr.o.z, __uint_as_float((uint32_t)tr.last_hit)));
            st_s(&P.hit[ray], make_float4(tr.best, tr.bu, tr.bv, __uint_as_float((uint32_t)(found ? tr.bprim : -1))));
            st_s(&P.hit_inside[ray], (uint8_t)(was_inside ? 1 : 0));
            st_s(&P.hit_cls[ray], found ? (uint8_t)tr.bcls : (uint8_t)0xffu);
        } else if (MODE == TM_NEE_ANY) {
            if (A.ext) P.xq_occ[ray] = found ? 1 : 0;
            else st_s(&P.occ[nq_index(P, ray)], (uint8_t)(found ? 1 : 0));
        } else if (MODE == TM_NEE_CLOSEST || MODE == TM_NEE_LIGHT) {
            // evaluate_shadow_light_ray: a hit counts only below t_max - 1e-4 (Intersect.h:337-343)
            bool ok = found && tr.best < qmax;
            (A.ext ? P.xq_hit[ray] : P.nhit[ray >> 2]) =
                make_float4(tr.best, tr.bu, tr.bv, __uint_as_float((uint32_t)(ok ? tr.bprim : -1)));
            if (MODE == TM_NEE_LIGHT && ok) {
                if (A.ext) P.xl_light[atomicAdd(&P.counters[CTR_XLIGHT], 1)] = ray;
                else P.nq_light[atomicAdd(&P.counters[CTR_LIGHT], 1)] = ray;
            }
        } else if (MODE == TM_NEE_LIGHT_OCC) {
            // a nearer triangle is not a light: the query contributes nothing, as a miss
            if (found) (A.ext ? P.xq_hit[ray] : P.nhit[ray >> 2]).w = __uint_as_float(0xffffffffu);
        } else if (MODE == TM_RAW_ANY || MODE == TM_LIST_ANY) {
            A.raw_occ[ray] = found ? 1 : 0;
        } else {
            A.raw_hit[ray] = make_float4(tr.best, tr.bu, tr.bv, __uint_as_float((uint32_t)(found ? tr.bprim : -1)));
        }
        alive = false;
    }
    if (STATS) {
        // wave-aggregated counters
        for (int off = 32; off > 0; off >>= 1) {
            n_nodes += __shfl_xor(n_nodes, off);
            n_tris += __shfl_xor(n_tris, off);
            n_rays += __shfl_xor(n_rays, off);
            n_slots[0] += __shfl_xor(n_slots[0], off);
            n_slots[1] += __shfl_xor(n_slots[1], off);
        }
        if (lane_id() == 0) {
            unsigned long long* st = (unsigned long long*)&P.stats[trace_stage(MODE) * STATS_STRIDE];
            atomicAdd(st + 0, (unsigned long long)n_rays);
            atomicAdd(st + 1, (unsigned long long)n_nodes);
            atomicAdd(st + 2, (unsigned long long)n_tris);
            atomicAdd(st + 4, (unsigned long long)n_slots[0]);
            atomicAdd(st + 5, (unsigned long long)n_slots[1]);
        }
    }
}

// ----------------------------------------------------------------------------------
// Scene access helpers (Intersect.h:30-83, Material.h:47-159, Texture.h:31-222)
// ----------------------------------------------------------------------------------
DEV v3 ld3(const float* p, int i) { return mk3(p[3 * (size_t)i], p[3 * (size_t)i + 1], p[3 * (size_t)i + 2]); }
DEV v2 ld2(const float* p, int i) { return mk2(p[2 * (size_t)i], p[2 * (size_t)i + 1]); }
DEV int3 tri_idx(const DevScene& S, int p) { return make_int3(S.idx[3 * (size_t)p], S.idx[3 * (size_t)p + 1], S.idx[3 * (size_t)p + 2]); }
DEV v3 uv_interp3(const float* data, int3 t, v2 uv) { return ld3(data, t.y) * uv.x + ld3(data, t.z) * uv.y + ld3(data, t.x) * (1.0f - uv.x - uv.y); }
DEV v2 uv_interp2(const float* data, int3 t, v2 uv) { return ld2(data, t.y) * uv.x + ld2(data, t.z) * uv.y + ld2(data, t.x) * (1.0f - uv.x - uv.y); }
DEV v3 tri_normal(const DevScene& S, int p) {
    const float4* tr = reinterpret_cast<const float4*>(S.tris);
    (void)tr;
    int3 t = tri_idx(S, p);
    v3 A = ld3(S.pos, t.x), B = ld3(S.pos, t.y), C = ld3(S.pos, t.z);
    return normalize(cross(B - A, C - A));
}
DEV void tex_rgba(const DevScene& S, int ti, bool srgb, v2 uv, float out[4]) {
    int w = S.tex_dims[2 * ti], h = S.tex_dims[2 * ti + 1];
    float u = wrap01(uv.x), v = 1.0f - wrap01(uv.y);
    int x = (int)(u * (float)(w - 1)), y = (int)(v * (float)(h - 1));
    const uint8_t* p = S.tex + S.tex_off[ti] + (size_t)(x + y * w) * 4;
    uchar4 c = *reinterpret_cast<const uchar4*>(p);
    if (srgb) {
        // pow(c / 255, 2.2) per 8-bit value, precomputed with the same ppow (k_srgb_table)
        out[0] = S.srgb[c.x]; out[1] = S.srgb[c.y]; out[2] = S.srgb[c.z]; out[3] = S.srgb[c.w];
        return;
    }
    out[0] = (float)c.x / 255.0f; out[1] = (float)c.y / 255.0f; out[2] = (float)c.z / 255.0f; out[3] = (float)c.w / 255.0f;
}
DEV bool has_tex(int ti) { return ti != MPT_NO_TEXTURE && ti != MPT_CONSTANT_EMISSIVE_TEXTURE; }
// filter_function's test: keep the candidate iff u < alpha_opacity * base-colour alpha
// (get_hit_base_color_alpha, Material.h:23-37; the sRGB pow(2.2) of Texture.h:72-75 also
// applies to the alpha channel)
// interpolated texture coordinates from the triangle's attribute record (k_tri_attr):
// uv_interp2's values and arithmetic, without the index gather
DEV v2 attr_tc(const DevScene& S, int prim, v2 uv) {
    const float4* r = S.tri_attr + 5 * (size_t)prim;
    const float4 c = r[2], d = r[3];
    return mk2(c.w, d.x) * uv.x + mk2(d.y, d.z) * uv.y + mk2(c.y, c.z) * (1.0f - uv.x - uv.y);
}
DEV bool alpha_rejects(const DevScene& S, int prim, float u, float v, uint32_t key) {
    const Mat& m = S.mats[S.mat_idx[prim]];
    float a = 1.0f;
    if (S.n_tex > 0 && has_tex(m.base_color_texture_index)) {
        v2 tc = attr_tc(S, prim, mk2(u, v));
        float r[4];
        tex_rgba(S, m.base_color_texture_index, true, tc, r);
        a = r[3];
    }
    float comp = m.alpha_opacity * a;
    return !(alpha_uniform(key, prim) < comp);
}
DEV void prop_f(const DevScene& S, float& v, v2 uv, int ti) { if (has_tex(ti)) { float r[4]; tex_rgba(S, ti, false, uv, r); v = r[0]; } }
DEV void prop_c(const DevScene& S, MptColor& v, v2 uv, int ti) { if (has_tex(ti)) { float r[4]; tex_rgba(S, ti, false, uv, r); v.r = r[0]; v.g = r[1]; v.b = r[2]; } }

DEV Col emission_of(const Mat& m) { return C3(m.emission) * m.emission_strength; }
DEV bool is_emissive(const Mat& m) {
    float k = m.emission_strength;
    return !is_zero(m.emission.r * k) || !is_zero(m.emission.g * k) || !is_zero(m.emission.b * k) || m.emissive_texture_used;
}

DEV Mat intersection_material(const DevScene& S, int mi, v2 uv, bool white_furnace) {
    Mat m = S.mats[mi];
    MptColor e;
    e.r = m.emission.r * m.emission_strength / m.emission_strength;
    e.g = m.emission.g * m.emission_strength / m.emission_strength;
    e.b = m.emission.b * m.emission_strength / m.emission_strength;
    if (S.n_tex > 0) prop_c(S, e, uv, m.emission_texture_index);
    m.emission = e;
    if (white_furnace) { m.base_color.r = 1.0f; m.base_color.g = 1.0f; m.base_color.b = 1.0f; }
    else if (S.n_tex > 0 && has_tex(m.base_color_texture_index)) {
        float r[4];
        tex_rgba(S, m.base_color_texture_index, true, uv, r);
        m.base_color.r = r[0]; m.base_color.g = r[1]; m.base_color.b = r[2];
    }
    if (S.n_tex > 0) {
        if (m.roughness_metallic_texture_index != MPT_NO_TEXTURE) {
            float r[4];
            tex_rgba(S, m.roughness_metallic_texture_index, false, uv, r);
            m.roughness = r[1];
            m.metallic = r[2];
        } else {
            prop_f(S, m.metallic, uv, m.metallic_texture_index);
            prop_f(S, m.roughness, uv, m.roughness_texture_index);
        }
        prop_f(S, m.oren_nayar_sigma, uv, m.oren_sigma_texture_index);
        prop_f(S, m.specular, uv, m.specular_texture_index);
        prop_f(S, m.specular_tint, uv, m.specular_tint_texture_index);
        prop_c(S, m.specular_color, uv, m.specular_color_texture_index);
        prop_f(S, m.anisotropy, uv, m.anisotropic_texture_index);
        prop_f(S, m.anisotropy_rotation, uv, m.anisotropic_rotation_texture_index);
        prop_f(S, m.coat, uv, m.coat_texture_index);
        prop_f(S, m.coat_roughness, uv, m.coat_roughness_texture_index);
        prop_f(S, m.coat_ior, uv, m.coat_ior_texture_index);
        prop_f(S, m.sheen, uv, m.sheen_texture_index);
        prop_f(S, m.sheen_roughness, uv, m.sheen_roughness_texture_index);
        prop_c(S, m.sheen_color, uv, m.sheen_color_texture_index);
        prop_f(S, m.specular_transmission, uv, m.specular_transmission_texture_index);
    }
    float coat = m.coat;
    m.emissive_texture_used = m.emission_texture_index > 0;
    float tbr = sqrtf(sqrtf(minr(1.0f, pow4(m.roughness) + 2.0f * pow4(m.coat_roughness))));
    m.roughness = lerpr(m.roughness, lerpr(m.roughness, tbr, coat), m.coat_roughening);
    float tsr = sqrtf(sqrtf(minr(1.0f, pow4(m.second_roughness) + 2.0f * pow4(m.coat_roughness))));
    m.second_roughness = lerpr(m.second_roughness, lerpr(m.second_roughness, tsr, coat), m.coat_roughening);
    return m;
}

// normal_mapping (Texture.h:209-222): tangent frame from the triangle's positions and uvs
DEV v3 normal_mapped(const DevScene& S, const Mat& m, v3 n, int p, v2 tc) {
    int3 t = tri_idx(S, p);
    v2 d1 = ld2(S.uv, t.y) - ld2(S.uv, t.x), d2 = ld2(S.uv, t.z) - ld2(S.uv, t.x);
    v3 e1 = ld3(S.pos, t.y) - ld3(S.pos, t.x), e2 = ld3(S.pos, t.z) - ld3(S.pos, t.x);
    float di = 1.0f / (d1.x * d2.y - d1.y * d2.x);
    v3 T = (e1 * d2.y - e2 * d1.y) * di;
    v3 B = (e2 * d1.x - e1 * d2.x) * di;
    float r[4];
    tex_rgba(S, m.normal_map_texture_index, false, tc, r);
    v3 ts = normalize(mk3(r[0] - 0.5f, r[1] - 0.5f, r[2] - 0.5f));
    return to_world(normalize(T), normalize(B), n, ts);
}
DEV v3 shading_normal_of(const DevScene& S, v3 gn, int p, v2 uv, v2 tc) {
    int3 t = tri_idx(S, p);
    const Mat& m = S.mats[S.mat_idx[p]];
    v3 n = S.has_n[t.x] ? normalize(uv_interp3(S.nrm, t, uv)) : gn;
    if (S.n_tex > 0 && m.normal_map_texture_index != MPT_NO_TEXTURE) n = normal_mapped(S, m, n, p, tc);
    return n;
}

// The vertex attributes trace_ray reads at a hit (Intersect.h:30-83, 154-192) from the
// triangle's attribute record (k_tri_attr, 5 float4: the three vertex normals, the three
// texture coordinates, has_vertex_normals of vertex A, the normalised geometric normal,
// the material index): one 80-B read at the primitive index replaces the index triple and
// the nine dependent vertex gathers.  Same values, same arithmetic as uv_interp2 /
// tri_normal / shading_normal_of (bit-identical).
struct HitAttr { v2 tc; v3 gn, sn; int mi; };
DEV HitAttr hit_attributes(const DevScene& S, int prim, v2 uv) {
    const float4* r = S.tri_attr + 5 * (size_t)prim;
    const float4 a = r[0], b = r[1], c = r[2], d = r[3], e = r[4];
    const v3 n0 = mk3(a.x, a.y, a.z), n1 = mk3(a.w, b.x, b.y), n2 = mk3(b.z, b.w, c.x);
    const v2 t0 = mk2(c.y, c.z), t1 = mk2(c.w, d.x), t2 = mk2(d.y, d.z);
    HitAttr h;
    h.tc = t1 * uv.x + t2 * uv.y + t0 * (1.0f - uv.x - uv.y);
    h.gn = normalize(mk3(e.x, e.y, e.z));
    h.mi = __float_as_int(e.w);
    v3 n = __float_as_uint(d.w) ? normalize(n1 * uv.x + n2 * uv.y + n0 * (1.0f - uv.x - uv.y)) : h.gn;
    if (S.n_tex > 0) {
        const Mat& m = S.mats[h.mi];
        if (m.normal_map_texture_index != MPT_NO_TEXTURE) n = normal_mapped(S, m, n, prim, h.tc);
    }
    h.sn = n;
    return h;
}
#ifndef MPT_TU_PART   // k_tri_attr (main translation unit)
__global__ void k_tri_attr(DevScene S, float4* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= S.n_tris) return;
    const int3 t = tri_idx(S, p);
    const v3 n0 = ld3(S.nrm, t.x), n1 = ld3(S.nrm, t.y), n2 = ld3(S.nrm, t.z);
    const v2 t0 = ld2(S.uv, t.x), t1 = ld2(S.uv, t.y), t2 = ld2(S.uv, t.z);
    const v3 g = tri_normal(S, p);
    float4* r = out + 5 * (size_t)p;
    r[0] = make_float4(n0.x, n0.y, n0.z, n1.x);
    r[1] = make_float4(n1.y, n1.z, n2.x, n2.y);
    r[2] = make_float4(n2.z, t0.x, t0.y, t1.x);
    r[3] = make_float4(t1.y, t2.x, t2.y, __uint_as_float(S.has_n[t.x] ? 1u : 0u));
    r[4] = make_float4(g.x, g.y, g.z, __int_as_float(S.mat_idx[p]));
}

#endif
// slot -> pixel of the band partition (rows y with (y / bh) % bc == bi, increasing y)
DEV uint32_t slot_pixel(const MptFrame& F, int slot, int& x, int& y) {
    int r = slot / F.res_x;
    x = slot - r * F.res_x;
    int bh = F.band_height;
    y = ((r / bh) * F.band_count + F.band_index) * bh + (r % bh);
    return (uint32_t)x + (uint32_t)y * (uint32_t)F.res_x;
}
DEV uint32_t pixel_seed(const MptFrame& F, uint32_t pix, uint32_t random_seed) {
    const MptRenderSettings& rs = F.render_settings;
    return rs.freeze_random ? wang_hash(pix + 1u) : wang_hash((pix + 1u) * (uint32_t)(rs.sample_number + 1) * random_seed);
}
DEV uint32_t pixel_seed(const MptFrame& F, uint32_t pix) { return pixel_seed(F, pix, F.random_seed); }
// CameraRays' seed: its own launch seed when the frame carries one (GPURenderer.cpp:468-474)
DEV uint32_t camera_seed(const MptFrame& F, uint32_t pix) {
    return pixel_seed(F, pix, F.camera_random_seed ? F.camera_random_seed : F.random_seed);
}
// The strategy sample_one_light runs at a bounce: ReSTIR DI's later bounces use
// ReSTIR_DI_LaterBouncesSamplingStrategy (Lights.h:243-275)
DEV int bounce_lss(const MptFrame& F, int bounce) {
    const int lss = F.options.direct_light_sampling;
    if (lss != MPT_LSS_RESTIR_DI || bounce == 0) return lss;
    switch (F.options.restir_di_later_bounces_sampling_strategy) {
    case MPT_RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT: return MPT_LSS_UNIFORM_ONE_LIGHT;
    case MPT_RESTIR_DI_LATER_BOUNCES_BSDF: return MPT_LSS_BSDF;
    case MPT_RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF: return MPT_LSS_MIS_LIGHT_BSDF;
    default: return MPT_LSS_RIS_BSDF_AND_LIGHT;
    }
}
// Sample batch (mpt_render_frames; GPURenderer::render's samples_per_frame loop,
// GPURenderer.cpp:424-449, run as one wavefront): the `batch` samples of a pixel occupy
// consecutive slots, interleaved over groups of `group` (4) pixels,
//   slot = ((pixel / group) * batch + sample) * group + pixel % group,
// so a wave's 64 lanes hold the samples of a few neighbouring pixels -- their camera rays,
// and often their later rays, open the same BVH nodes together -- while k_accumulate's
// per-pixel loads stay coalesced in runs of `group` slots.  Sample k's seeds and sample
// number are those of Fp[k].
DEV void batch_split(const DevPaths& P, int slot, int& pix, int& sub) {
    if (P.batch == 1) { pix = slot; sub = 0; return; }
    const int g = P.group;
    const int q = slot / g;
    const int grp = q / P.batch;
    sub = q - grp * P.batch;
    pix = grp * g + (slot - q * g);
}
DEV int batch_slot(const DevPaths& P, int pix, int sub) {
    const int g = P.group;
    const int grp = pix / g;
    return (grp * P.batch + sub) * g + (pix - grp * g);
}
DEV uint32_t path_seed(const MptFrame* Fp, const DevPaths& P, int slot, bool camera) {
    int pix, sub;
    batch_split(P, slot, pix, sub);
    const MptFrame& F = Fp[sub];
    int x, y;
    const uint32_t gpix = slot_pixel(F, pix, x, y);
    return camera ? camera_seed(F, gpix) : pixel_seed(F, gpix);
}

// ----------------------------------------------------------------------------------
// k_camera: CameraRays ray generation (CameraRays.h:127-142, HIPRTCamera.h:27-47)
// ----------------------------------------------------------------------------------
DEV bool has_adaptive_buffers(const MptRenderSettings& rs) {   // RenderSettings.h:207-218
    return (rs.stop_pixel_noise_threshold > 0.0f || rs.enable_adaptive_sampling) && rs.accumulate;
}
// Low-resolution interactive mode (do_render_low_resolution, RenderSettings.h:195-198;
// CameraRays.h:63-76): CameraRays renders one pixel out of s x s, the representative (x, y)
// with x, y multiples of s, at pixel_index / s = (x / s, y / s) -- the frame's top-left
// ceil(W / s) x ceil(H / s) pixels, row stride W, hold the low-resolution image.  A pixel of
// that region is active and traces the camera ray through its representative; every other
// pixel is inactive (the reference's racy pixel_active writes resolved as DESIGN.md §2 states).
DEV bool low_res(const MptRenderSettings& rs) {
    return rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate;
}
DEV bool low_res_region(const MptFrame& F, int x, int y) {
    const MptRenderSettings& rs = F.render_settings;
    const int s = rs.render_low_resolution_scaling;
    return x < (F.res_x + s - 1) / s && y < (F.res_y + s - 1) / s;
}
// get_pixel_confidence_interval (AdaptiveSampling.h:11-20) of a pixel's sum c, squared
// luminance sum sq and sample count
DEV float pixel_confidence(Col c, float sq, int count, float& avg) {
    float l = lum(c);
    avg = l / (float)(count + 1);
    float var = (sq - l * avg) / (float)(count + 1);
    return 1.96f * sqrtf(var) / sqrtf((float)(count + 1));
}
// adaptive_sampling (AdaptiveSampling.h:30-104) on a pixel's values: true if the pixel needs
// this sample; updates the converged sample count `conv`
DEV bool adaptive_gate(const MptRenderSettings& rs, Col c, float sq, int cnt, int& conv, bool& converged) {
    if (!has_adaptive_buffers(rs)) return true;
    if (rs.enable_adaptive_sampling) {
        if (conv != -1) return false;
        if (cnt > rs.adaptive_sampling_min_samples) {
            float avg;
            float ci = pixel_confidence(c, sq, cnt, avg);
            if (!(ci > rs.adaptive_sampling_noise_threshold * avg)) {
                if (conv == -1) conv = cnt;
                return false;
            }
        }
        return true;
    } else if (rs.stop_pixel_noise_threshold > 0.0f && rs.enable_pixel_stop_noise_threshold) {
        float avg;
        float ci = pixel_confidence(c, sq, cnt, avg);
        converged = (ci <= rs.stop_pixel_noise_threshold * avg) && (rs.sample_number > 1);
        if (converged && conv == -1) conv = cnt;
        else if (!converged) conv = -1;
    }
    return true;
}
// the same on the pixel's buffers (CameraRays' gate, one sample per launch)
DEV bool adaptive_sampling(const DevPaths& P, const MptRenderSettings& rs, int slot, bool& converged) {
    if (!has_adaptive_buffers(rs)) return true;
    const float* px = P.fb_color + 3 * (size_t)slot;
    int conv = P.as_conv[slot];
    const bool needed = adaptive_gate(rs, col(px[0], px[1], px[2]), P.as_sqlum[slot], P.as_count[slot], conv, converged);
    P.as_conv[slot] = conv;
    return needed;
}

#ifndef MPT_TU_PART   // k_camera
__global__ __launch_bounds__(TB) void k_camera(DevPaths P, const MptFrame* __restrict__ Fp) {
    int slot = blockIdx.x * TB + threadIdx.x;
    int pslot = slot, sub = 0;   // pixel of the partition, sample of the batch
    if (slot < P.n) batch_split(P, slot, pslot, sub);   // batched launches never use the adaptive buffers
    const MptFrame& F = Fp[sub];
    const MptRenderSettings& rs = F.render_settings;
    // a batch of adaptive samples is traced speculatively: k_accumulate replays the gate in sample
    // order (P.spec_as).  Under enable_adaptive_sampling a converged pixel stays converged
    // (AdaptiveSampling.h:45-48: the gate refuses it while pixel_converged_sample_count != -1) until
    // a reset, so a pixel that had converged before the batch began -- with no reset frame among
    // the batch's samples up to this one -- gets no camera ray: the gate will refuse that sample.
    // The camera queue is then compacted (P.spec_skip: set by the host unless no pixel can have
    // converged yet -- every pixel's count still at most the minimum since the last reset).
    const bool as = has_adaptive_buffers(rs) && !P.spec_as;
    const bool spec_skip = P.spec_skip != 0;
    const bool lr = low_res(rs);
    bool act = slot < P.n;
    int x = 0, y = 0;
    uint32_t pix = 0;
    if (act) pix = slot_pixel(F, pslot, x, y);
    if (act && spec_skip && P.as_conv[pslot] != -1) {
        bool reset = P.spec_reset != 0;
        for (int k = 0; k <= sub; k++) reset |= Fp[k].render_settings.sample_number == 0 || Fp[k].render_settings.need_to_reset;
        if (!reset) {
            act = false;
            P.active[slot] = 0;
        }
    }
    if (!act) {
    } else if (lr && !low_res_region(F, x, y)) {
        act = false;                      // CameraRays.h:68-72: no reset, no adaptive gate
        P.active[slot] = 0;
    } else if (act) {
        // reset_render + adaptive gate (CameraRays.h:19-43, 88-125)
        if (as && (rs.sample_number == 0 || rs.need_to_reset)) {
            P.as_count[slot] = 0;
            P.as_sqlum[slot] = 0.0f;
            P.as_conv[slot] = -1;
        }
        bool converged = false;
        // (speculative batches: the gate runs in k_accumulate, on the pixel's values)
        bool needed = as ? adaptive_sampling(P, rs, slot, converged) : true;
        if ((converged || !needed) && rs.do_update_status_buffers) atomicAdd(&P.status[0], 1u);
        if (as) {
            if (!needed) {
                float* px = P.fb_color + 3 * (size_t)slot;
                Col c = col(px[0], px[1], px[2]) / (float)rs.sample_number * (float)(rs.sample_number + 1);
                px[0] = c.r; px[1] = c.g; px[2] = c.b;
                act = false;
            } else {
                P.as_count[slot]++;
            }
        }
        P.active[slot] = act ? 1 : 0;
    }
    if (P.cam_noqueue) {
        // (batched ReSTIR DI: k_queue_active lists the active slots per sample and for the trace)
    } else if (as || lr || spec_skip) {
        // camera-ray queue of the active pixels (wave64 ballot, one atomic per wave)
        uint64_t m = __ballot(act);
        int lane = threadIdx.x & 63;
        int base = 0;
        if (m) {
            int first = __ffsll((unsigned long long)m) - 1;
            if (lane == first) base = atomicAdd(&P.counters[CTR_Q0], __popcll(m));
            base = __shfl(base, first);
        }
        if (act) P.q0[base + __popcll(m & ((1ull << lane) - 1ull))] = slot;
    } else if (act) {
        P.q0[slot] = slot;
    }
    if (!act) return;
    if (rs.do_update_status_buffers && !P.spec_as) P.status[1] = 1u;   // (speculative: k_accumulate)
    const uint32_t cseed = camera_seed(F, pix);
    // the path's seeds for the later stages (path_seed of the camera launch / of the path
    // tracing launch), computed once here instead of per traversal query
    P.seeds[slot] = make_uint2(cseed, pixel_seed(F, pix));
    Rng rng = make_rng(cseed);
    // low resolution: the ray through the representative pixel (CameraRays.h:127-131 with the
    // thread's own x, y), seeded with the low-resolution index (pixel_index / s)
    const int ls = lr ? rs.render_low_resolution_scaling : 1;
    float xd = (float)(x * ls) + 0.5f, yd = (float)(y * ls) + 0.5f;
    if (F.current_camera.do_jittering) { xd += rng() - 0.5f; yd += rng() - 0.5f; }
    float xn = xd / (float)F.res_x * 2.0f - 1.0f;
    float yn = yd / (float)F.res_y * 2.0f - 1.0f;
    v3 o = mat_x_point(F.current_camera.inverse_view.m, mk3(0.0f, 0.0f, 0.0f));
    v3 pvs = mat_x_point(F.current_camera.inverse_projection.m, mk3(xn, yn, -1.0f));
    v3 pws = mat_x_point(F.current_camera.inverse_view.m, pvs);
    v3 d = normalize(pws - o);
    P.ray_o[slot] = make_float4(o.x, o.y, o.z, __uint_as_float(0xffffffffu));
    P.ray_d[slot] = make_float4(d.x, d.y, d.z, INFINITY);
    P.rng[slot] = rng.s;   // camera stream after the jitter draws (trace_ray's wavelength draw)
    vs_store_s(P.vsA, P.vsB, slot, vs_default());
    P.thr[slot] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    P.col[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    P.alb[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    P.nrm[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

#endif
// ----------------------------------------------------------------------------------
// light sampling helpers (LightUtils.h)
// ----------------------------------------------------------------------------------
struct LightInfo { int tri; v3 normal; float area; Col emission; };
// Emissive-triangle table (built once per scene / material update by k_emissive_table):
// per light 5 float4 {A, prim}, {B - A, area}, {C - A, |cross|}, {normal, valid}, {emission}
// -- the values uniform_sample_one_emissive_triangle (LightUtils.h:15-58) derives from
// the triangle's vertices and material, computed with the same operations, so a sample
// costs one dependent 80-byte load instead of a chain of index / vertex / material loads.
#ifndef MPT_TU_PART   // k_emissive_table
__global__ void k_emissive_table(DevScene S, float4* tab) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S.n_emissive) return;
    int t = S.emissive[i];
    int3 ti = tri_idx(S, t);
    v3 A = ld3(S.pos, ti.x), B = ld3(S.pos, ti.y), C = ld3(S.pos, ti.z);
    v3 AB = B - A, AC = C - A;
    v3 n = cross(AB, AC);
    float ln = length(n);
    bool ok = !(ln <= 1.0e-6f);
    v3 nn = ok ? n / ln : mk3(0.0f, 1.0f, 0.0f);
    Col e = emission_of(S.mats[S.mat_idx[t]]);
    tab[5 * i + 0] = make_float4(A.x, A.y, A.z, __int_as_float(t));
    tab[5 * i + 1] = make_float4(AB.x, AB.y, AB.z, ln * 0.5f);
    tab[5 * i + 2] = make_float4(AC.x, AC.y, AC.z, ln);
    tab[5 * i + 3] = make_float4(nn.x, nn.y, nn.z, ok ? 1.0f : 0.0f);
    tab[5 * i + 4] = make_float4(e.r, e.g, e.b, 0.0f);
}

#endif
// uniform_sample_one_emissive_triangle in three parts, so that a caller can load a later
// sample's record early: the index draw, the record (one 80-byte load), the rest of the draws
#ifndef MPT_EM_PREFETCH   // A/B switches of the shading kernel's early loads (see EmPrefetch, env_fetch)
#define MPT_EM_PREFETCH 0
#endif
#ifndef MPT_ENV_EARLY
#define MPT_ENV_EARLY 0
#endif
struct EmRec { float4 e0, e1, e2, e3, e4; };
DEV int emissive_index(const DevScene& S, Rng& rng) { return rng.random_index(S.n_emissive); }
DEV EmRec emissive_record(const DevScene& S, int ri) {
#if defined(MPT_UB_LOCAL_GATHERS) && (MPT_UB_LOCAL_GATHERS & 1)   // A/B experiments only (not bit-exact): cache-resident records
    const float4* e = S.em_tab + 5 * (size_t)(ri & 63);
#else
    const float4* e = S.em_tab + 5 * (size_t)ri;
#endif
    EmRec r;
    r.e0 = e[0]; r.e1 = e[1]; r.e2 = e[2]; r.e3 = e[3]; r.e4 = e[4];
    return r;
}
DEV v3 emissive_point(const DevScene& S, const EmRec& r, Rng& rng, float& pdf, LightInfo& li) {
    float r1 = rng(), r2 = rng();
    float sr1 = sqrtf(r1);
    float u = 1.0f - sr1, v = (1.0f - r2) * sr1;
    v3 A = mk3(r.e0.x, r.e0.y, r.e0.z), AB = mk3(r.e1.x, r.e1.y, r.e1.z), AC = mk3(r.e2.x, r.e2.y, r.e2.z);
    v3 pt = A + AB * u + AC * v;
    li.tri = -1; li.normal = mk3(0.0f, 1.0f, 0.0f); li.area = 1.0f; li.emission = col(0.0f);
    if (r.e3.w == 0.0f) { pdf = 0.0f; return mk3(0.0f, 0.0f, 0.0f); }
    li.tri = __float_as_int(r.e0.w);
    li.normal = mk3(r.e3.x, r.e3.y, r.e3.z);
    li.area = r.e1.w;
    li.emission = col(r.e4.x, r.e4.y, r.e4.z);
    pdf = 1.0f / li.area;
    pdf /= (float)S.n_emissive;
    return pt;
}
DEV v3 sample_emissive_triangle(const DevScene& S, Rng& rng, float& pdf, LightInfo& li) {
    const int ri = emissive_index(S, rng);
    return emissive_point(S, emissive_record(S, ri), rng, pdf, li);
}
// A light sample's record loaded ahead of its draws: valid for the RNG state `state` (the one
// its index draw starts from), so a prediction that the draws then do not meet is just unused
struct EmPrefetch {
    uint32_t state;
    bool valid;
    EmRec r;
    DEV void issue(const DevScene& S, Rng at) {
        state = at.s;
        valid = true;
        r = emissive_record(S, emissive_index(S, at));
    }
    // sample_emissive_triangle from rng, with the prefetched record when it is the right one
    DEV v3 sample(const DevScene& S, Rng& rng, float& pdf, LightInfo& li) {
        const bool hit = valid && state == rng.s;
        const int ri = emissive_index(S, rng);
        valid = false;
        return emissive_point(S, hit ? r : emissive_record(S, ri), rng, pdf, li);
    }
};
DEV bool min_contrib(float mn, Col c) { return mn > 0.0f ? !(c.r < mn && c.g < mn && c.b < mn) : true; }
DEV Col clamp_contrib(Col c, float mx, bool cond) { return (!has_nan(c) && mx > 0.0f && cond) ? clampc(c, -mx, mx) : c; }

// envmap (Envmap.h)
// the texel index env_tex reads at uv (Envmap.h: wrapped, v flipped, truncated)
DEV size_t env_tex_index(const DevScene& S, v2 uv) {
    float u = wrap01(uv.x), v = 1.0f - wrap01(uv.y);
    int x = (int)(u * (float)(S.env_w - 1)), y = (int)(v * (float)(S.env_h - 1));
    return (size_t)x + (size_t)y * S.env_w;
}
// the uv env_sample derives from the sampled texel index (its radiance lookup)
DEV v2 env_sample_uv(const DevScene& S, int ri, float& u, float& v) {
    const int y = (int)((unsigned)ri / (unsigned)S.env_w);
    const int x = ri - y * S.env_w;
    u = (float)x / (float)(unsigned)S.env_w;
    v = (float)y / (float)(unsigned)S.env_h;
    return mk2(u, 1.0f - v);
}
DEV Col env_tex(const DevScene& S, const MptFrame& F, v2 uv) {
    float u = wrap01(uv.x), v = 1.0f - wrap01(uv.y);
    int x = (int)(u * (float)(S.env_w - 1)), y = (int)(v * (float)(S.env_h - 1));
#if defined(MPT_UB_LOCAL_GATHERS) && (MPT_UB_LOCAL_GATHERS & 2)
    float4 p = S.env[(x + (size_t)y * S.env_w) & 4095];
#else
    float4 p = S.env[x + (size_t)y * S.env_w];
#endif
    return col(p.x, p.y, p.z) * F.world_settings.envmap_intensity;
}
DEV Col eval_env_no_pdf(const DevScene& S, const MptFrame& F, v3 d) {
    v3 r = mat_x_vec(F.world_settings.world_to_envmap_matrix.m, d);
    float u = 0.5f + patan2(r.z, r.x) * INV_2_PI;
    float v = 0.5f + pasin(r.y) * INV_PI;
    return env_tex(S, F, mk2(u, 1.0f - v));
}
// envmap_cdf_search (Envmap.h:40-75): row by the last column, then the texel in the row
DEV void env_cdf_search(const DevScene& S, float value, int& x, int& y) {
    unsigned lower = 0;
    int upper = S.env_h - 1;
    int xi = S.env_w - 1;
    while (lower < (unsigned)upper) {
        int yi = (int)((lower + (unsigned)upper) / 2u);
        if (value < S.env_cdf[yi * S.env_w + xi]) upper = yi;
        else lower = (unsigned)yi + 1u;
    }
    y = (int)(lower < (unsigned)S.env_h ? lower : (unsigned)S.env_h);
    lower = 0;
    upper = S.env_w - 1;
    while (lower < (unsigned)upper) {
        int xm = (int)((lower + (unsigned)upper) / 2u);
        if (value < S.env_cdf[y * S.env_w + xm]) upper = xm;
        else lower = (unsigned)xm + 1u;
    }
    x = (int)(lower < (unsigned)S.env_w ? lower : (unsigned)S.env_w);
}
DEV float env_total(const DevScene& S, const MptFrame& F) {
    return F.options.envmap_sampling == MPT_ESS_BINARY_SEARCH ? S.env_cdf_sum : S.env_sum;
}
DEV Col env_sample(const DevScene& S, const MptFrame& F, v3& dir, float& pdf, Rng& rng) {
    int x, y;
    if (F.options.envmap_sampling != MPT_ESS_BINARY_SEARCH && S.env_rich) {
        // alias table with the texels (one 32-B gather): the same draws, texel and arithmetic
        // as the two-load path below
        int ri = rng.random_index(S.env_h * S.env_w);
        const float4 a = S.env_rich[2 * (size_t)ri], b = S.env_rich[2 * (size_t)ri + 1];
        Col tex;
        if (rng() > a.x) { ri = __float_as_int(a.y); tex = col(b.y, b.z, b.w); }
        else tex = col(a.z, a.w, b.x);
        float u, v;
        env_sample_uv(S, ri, u, v);
        float phi = u * TWO_PI;
        float theta = maxr(1.0e-5f, v * PI);
        const float2 sct = psincos(theta), scp = psincos(phi);
        float ct = sct.y, st = sct.x;
        dir = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, mk3(-st * scp.y, -ct, -st * scp.x));
        Col rad = tex * F.world_settings.envmap_intensity;
        pdf = lum(rad) / (env_total(S, F) * F.world_settings.envmap_intensity);
        pdf *= (float)((unsigned)S.env_w * (unsigned)S.env_h);
        pdf /= (TWO_PIPI * st);
        return rad;
    }
    if (F.options.envmap_sampling == MPT_ESS_BINARY_SEARCH) {
        env_cdf_search(S, rng() * S.env_cdf_sum, x, y);
    } else {
        int ri = rng.random_index(S.env_h * S.env_w);
#if defined(MPT_UB_LOCAL_GATHERS) && (MPT_UB_LOCAL_GATHERS & 2)
        const int2 e = S.alias[ri & 4095];
#else
        const int2 e = S.alias[ri];   // one 8-B load: probability bits + alias index
#endif
        if (rng() > __int_as_float(e.x)) ri = e.y;
        y = (int)((unsigned)ri / (unsigned)S.env_w);
        x = ri - y * S.env_w;
    }
    float u = (float)x / (float)(unsigned)S.env_w, v = (float)y / (float)(unsigned)S.env_h;
    float phi = u * TWO_PI;
    float theta = maxr(1.0e-5f, v * PI);
    const float2 sct = psincos(theta), scp = psincos(phi);
    float ct = sct.y, st = sct.x;
    dir = mat_x_vec(F.world_settings.envmap_to_world_matrix.m, mk3(-st * scp.y, -ct, -st * scp.x));
    Col rad = env_tex(S, F, mk2(u, 1.0f - v));
    pdf = lum(rad) / (env_total(S, F) * F.world_settings.envmap_intensity);
    pdf *= (float)((unsigned)S.env_w * (unsigned)S.env_h);
    pdf /= (TWO_PIPI * st);
    return rad;
}
// env_eval in two halves, so that a shading kernel can issue the texel load before a BSDF
// evaluation and consume it after: env_fetch = eval_env_no_pdf's texel, env_eval_tex the rest
DEV float4 env_fetch(const DevScene& S, const MptFrame& F, v3 d) {
    v3 r = mat_x_vec(F.world_settings.world_to_envmap_matrix.m, d);
    float u = 0.5f + patan2(r.z, r.x) * INV_2_PI;
    float v = 0.5f + pasin(r.y) * INV_PI;
    return S.env[env_tex_index(S, mk2(u, 1.0f - v))];
}
DEV Col env_eval_tex(const DevScene& S, const MptFrame& F, v3 d, float4 p, float& pdf) {
    Col rad = col(p.x, p.y, p.z) * F.world_settings.envmap_intensity;
    float st = psin(pacos(-d.y));
    pdf = lum(rad) / (env_total(S, F) * F.world_settings.envmap_intensity);
    pdf *= (float)((unsigned)S.env_w * (unsigned)S.env_h);
    pdf /= (TWO_PIPI * st);
    return rad;
}
DEV Col env_eval(const DevScene& S, const MptFrame& F, v3 d, float& pdf) {
    Col rad = eval_env_no_pdf(S, F, d);
    float st = psin(pacos(-d.y));
    pdf = lum(rad) / (env_total(S, F) * F.world_settings.envmap_intensity);
    pdf *= (float)((unsigned)S.env_w * (unsigned)S.env_h);
    pdf /= (TWO_PIPI * st);
    return rad;
}

// NEE query emission: any-hit area [0, 3n), closest area [3n, 4n)
// NEE queries are staged at a fixed place per path (slot * 4 + kind; kinds 0..2 any hit,
// 3 closest hit) and the bit is set in the path's query mask; k_compact builds the
// compacted lists afterwards, so k_shade itself issues no atomics (an atomic with a
// return value would wait for all of the lane's outstanding stores).
DEV void stage_query(const DevPaths& P, int slot, int kind, uint32_t& qm, v3 o, int last_hit, v3 d, float tmax) {
    const size_t e = (size_t)kind * (size_t)P.nq_stride + (size_t)slot;
    st_s(&P.nq_o[e], make_float4(o.x, o.y, o.z, __uint_as_float((uint32_t)last_hit)));
    st_s(&P.nq_d[e], make_float4(d.x, d.y, d.z, tmax));
    qm |= 1u << kind;
}

// ----------------------------------------------------------------------------------
// Extended light sampling (number_of_light_samples > 1, RIS with several BSDF candidates,
// RISUseVisiblityTargetFunction): sample_many_lights' loop (Lights.h:222-241) with every
// RNG draw of every light sample here, in the reference's order, and one record + query per
// candidate in the slot's ext entries (layout: mpt_internal.h).  k_resolve<true> replays
// the reservoirs / MIS sums with the trace results.  Only the EXT instantiation of k_shade
// carries this code.
// ----------------------------------------------------------------------------------
DEV void x_query(const DevPaths& P, size_t e, bool any, v3 o, int last_hit, v3 d, float tmax, uint8_t& flag) {
    P.xq_o[e] = make_float4(o.x, o.y, o.z, __uint_as_float((uint32_t)last_hit));
    P.xq_d[e] = make_float4(d.x, d.y, d.z, tmax);
    if (any) P.xl_any[atomicAdd(&P.counters[CTR_XANY], 1)] = (int32_t)e;
    else P.xl_cl[atomicAdd(&P.counters[CTR_XCL], 1)] = (int32_t)e;
    flag |= any ? XQ_ANY : XQ_CL;
}
DEV void x_rec(const DevPaths& P, size_t e, float4 a, float4 b) {
    P.xrec[2 * e] = a;
    P.xrec[2 * e + 1] = b;
}
// a BSDF-sampled light-hit candidate: sample (draws), evaluate, stage the light-hit ray;
// origin as sample_one_light_bsdf / _MIS / the RIS BSDF candidates pick it
template <int OVR, int FULL>
DEV float x_bsdf_cand(const DevPaths& P, const BCtx& bc, const Mat& m, const VState& vs, const PEval& pe, size_t e, int prim,
                      v3 ip, v3 sn, v3 gn, v3 view, float ism, v3 o_refl, bool abs_cos, float r_add_slot, Rng& rng, uint8_t& fl) {
    VState tv = vs;
    v3 L = mk3(0.0f, 0.0f, 0.0f);
    float pdf = 0.0f;
    Col f = col(0.0f);
    if (bsdf_sample_dir<OVR, FULL>(bc, m, tv, view, sn, gn, L, rng)) f = bsdf_eval_post<OVR, FULL>(bc, m, tv, pe, sn, L, pdf);
    const bool refr = dot(L, sn * ism) < 0;
    if (pdf > 0.0f) {
        const v3 o = refr ? ip + sn * 1.0e-4f * ism * -1.0f : o_refl;
        const float c = abs_cos ? absr(dot(sn, L)) : maxr(0.0f, dot(sn, L));
        x_rec(P, e, make_float4(f.r, f.g, f.b, pdf), make_float4(c, r_add_slot, refr ? 1.0f : 0.0f, 0.0f));
        fl |= XQ_REC;
        x_query(P, e, false, o, prim, L, 1.0e35f - 1.0e-4f, fl);
    }
    return pdf;
}
template <int OVR, int FULL>
DEV void ext_light(const DevScene& S, const DevPaths& P, const MptFrame& F, const BCtx& bc, const Mat& m, const VState& vs,
                   const PEval& pe, int slot, int prim, v3 ip, v3 sn, v3 gn, v3 view, float ism, v3 ep, int lssb, Rng& rng) {
    const MptRenderSettings& rs = F.render_settings;
    const int nl = rs.ris_number_of_light_candidates, nbc = rs.ris_number_of_bsdf_candidates;
    const bool vis = F.options.ris_use_visibility != 0;
    const size_t base = (size_t)slot * P.x_per;
    for (int it = 0; it < rs.number_of_light_samples; it++) {
        const size_t e0 = base + (size_t)it * P.x_iter;
        for (int j = 0; j < P.x_iter; j++) P.xq_flag[e0 + j] = 0;
        if (lssb == MPT_LSS_UNIFORM_ONE_LIGHT || lssb == MPT_LSS_MIS_LIGHT_BSDF) {
            // sample_one_light_no_MIS (Lights.h:22-65) / sample_one_light_MIS (Lights.h:115-220)
            const bool mis = lssb == MPT_LSS_MIS_LIGHT_BSDF;
            float lpdf;
            LightInfo li;
            const v3 lp = sample_emissive_triangle(S, rng, lpdf, li);
            if (!(lpdf > 0.0f)) continue;   // both return before any further draw
            uint8_t f0 = 0, f1 = 0;
            const v3 so = mis ? ep : ip + sn * 1.0e-4f;
            const v3 sd = lp - so;
            const float dist = length(sd);
            const v3 L = sd / dist;
            const float geo = absr(dot(li.normal, -L));
            if (geo > 0.0f) {
                VState tv = vs;
                float pdf;
                const Col f = bsdf_eval_post<OVR, FULL>(bc, m, tv, pe, sn, L, pdf);
                if (pdf != 0.0f) {
                    float lp2 = lpdf;
                    lp2 *= dist * dist;
                    lp2 /= geo;
                    const float cosv = maxr(dot(sn, L), 0.0f);
                    const Col rad = mis ? f * cosv * li.emission * balance(lp2, pdf) / lp2 : li.emission * cosv * f / lp2;
                    x_rec(P, e0, make_float4(rad.r, rad.g, rad.b, 0.0f), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                    f0 |= XQ_REC;
                    x_query(P, e0, true, so, prim, L, dist - 1.0e-4f, f0);
                }
            }
            if (mis) x_bsdf_cand<OVR, FULL>(P, bc, m, vs, pe, e0 + 1, prim, ip, sn, gn, view, ism, ep, true, 0.0f, rng, f1);
            P.xq_flag[e0] = f0;
            if (mis) P.xq_flag[e0 + 1] = f1;
        } else if (lssb == MPT_LSS_BSDF) {
            // sample_one_light_bsdf (Lights.h:67-113)
            uint8_t f0 = 0;
            x_bsdf_cand<OVR, FULL>(P, bc, m, vs, pe, e0, prim, ip, sn, gn, view, ism, ip + sn * 1.0e-4f, false, 0.0f, rng, f0);
            P.xq_flag[e0] = f0;
        } else {
            // sample_bsdf_and_lights_RIS_reservoir (RIS.h:82-289): the light candidates' draws and
            // weights (without visibility: final), the BSDF candidates' draws; the reservoir
            // itself is replayed by k_resolve with the trace results
            const v3 ep2 = ip + sn * 1.0e-4f;   // evaluate_reservoir_sample's shadow-ray origin (RIS.h:31)
            float wsum = 0.0f;                  // without the visibility target function: the light
            int win = -1;                       // winner is final here, only its shadow ray is traced
            v3 win_L = mk3(0.0f, 0.0f, 0.0f);
            float win_d = 0.0f;
            for (int c = 0; c < nl; c++) {
                float lpdf;
                LightInfo li;
                const v3 lp = sample_emissive_triangle(S, rng, lpdf, li);
                float target = 0.0f, w = 0.0f, bp = 0.0f;
                bool inner = false;
                Col fc = col(0.0f);
                v3 tl = mk3(0.0f, 0.0f, 0.0f);
                float dist = 0.0f;
                if (lpdf > 0.0f) {
                    tl = lp - ep;
                    dist = length(tl);
                    tl = tl / dist;
                    const float cl = absr(dot(li.normal, -tl));
                    const float geo = maxr(0.0f, dot(sn * ism, tl));
                    if (geo > 0.0f && cl > 1.0e-6f) {
                        inner = true;
                        lpdf *= dist * dist;
                        lpdf /= cl;
                        if (min_contrib(rs.minimum_light_contribution, li.emission / lpdf)) {
                            VState tv = vs;
                            fc = bsdf_eval_post<OVR, FULL>(bc, m, tv, pe, sn, tl, bp);
                            const Col lc = fc * li.emission * geo;
                            target = min_contrib(rs.minimum_light_contribution, lc / bp / lpdf) ? lum(lc) : 0.0f;
                        }
                        w = balance(lpdf, (float)nl, bp, (float)nbc);
                    }
                }
                const float r = rng();   // RISReservoir::add_one_candidate (RIS_Reservoir.h:29-38)
                const size_t e = e0 + c, ew = e0 + nl + c;
                uint8_t f0 = XQ_REC, fw = 0;
                x_rec(P, e, make_float4(w, lpdf, target, __int_as_float(li.tri)), make_float4(r, inner ? 1.0f : 0.0f, 0.0f, 0.0f));
                if (inner && vis && target > 0.0f) x_query(P, e, true, ep, prim, tl, dist - 1.0e-4f, f0);
                v3 Lw = mk3(0.0f, 0.0f, 0.0f);
                float dw = 0.0f;
                if (inner && target > 0.0f) {
                    // this candidate's final shading as the winner (RIS.h:18-80): direction from ep2,
                    // a fresh evaluation unless that is the candidate's own origin (outside)
                    const v3 sd = lp - ep2;
                    dw = length(sd);
                    Lw = sd / dw;
                    Col fw_ = fc;
                    if (ism != 1.0f) {
                        VState tv = vs;
                        float bpw;
                        fw_ = bsdf_eval_post<OVR, FULL>(bc, m, tv, pe, sn, Lw, bpw);
                    }
                    x_rec(P, ew, make_float4(fw_.r, fw_.g, fw_.b, maxr(0.0f, dot(sn, Lw))), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
                    fw |= XQ_REC;
                    // with the visibility target function any candidate may win: its final shadow
                    // ray is its visibility ray outside, a ray of its own inside
                    if (vis && ism != 1.0f) x_query(P, ew, true, ep2, prim, Lw, dw - 1.0e-4f, fw);
                }
                if (!vis) {
                    const float cw = inner ? w * target / lpdf : 0.0f;
                    wsum += cw;
                    if (r < cw / wsum) { win = c; win_L = Lw; win_d = dw; }
                }
                P.xq_flag[e] = f0;
                P.xq_flag[ew] = fw;
            }
            if (!vis && win >= 0) {
                uint8_t fw = XQ_REC;
                x_query(P, e0 + nl + win, true, ep2, prim, win_L, win_d - 1.0e-4f, fw);
                P.xq_flag[e0 + nl + win] = fw;
            }
            for (int b = 0; b < nbc; b++) {
                uint8_t fb = 0;
                // the candidate's random is drawn after its BSDF sample (add_one_candidate)
                const size_t e = e0 + 2 * nl + b;
                const float pdf = x_bsdf_cand<OVR, FULL>(P, bc, m, vs, pe, e, prim, ip, sn, gn, view, ism, ep, true, 0.0f, rng, fb);
                const float r = rng();
                if (pdf > 0.0f) P.xrec[2 * e + 1].y = r;
                else x_rec(P, e, make_float4(0.0f, 0.0f, 0.0f, 0.0f), make_float4(0.0f, r, 0.0f, 0.0f));
                P.xq_flag[e] = fb | XQ_REC;
            }
        }
    }
}

DEV void store3(float* p, Col c) { p[0] = c.r; p[1] = c.g; p[2] = c.b; }
DEV void store3(float* p, v3 c) { p[0] = c.x; p[1] = c.y; p[2] = c.z; }
DEV Col load3c(const float* p) { return col(p[0], p[1], p[2]); }
DEV v3 load3v(const float* p) { return mk3(p[0], p[1], p[2]); }

// ----------------------------------------------------------------------------------
// k_shade: one path vertex up to (not including) the NEE trace results
// ----------------------------------------------------------------------------------
// Development instrumentation (-DMPT_SECTION_TIMING): shader-clock cycles per k_shade
// section (0 hit processing, 1 op pre, 2 BSDF eval, 3 op post, 4 finish), summed over
// lanes into g_sect; read with mpt_debug_sections.
#ifdef MPT_SECTION_TIMING
static __device__ unsigned long long g_sect[8];
#define SECT_BEGIN() uint64_t sect_[6] = {0, 0, 0, 0, 0, 0}; uint64_t tprev_ = __builtin_amdgcn_s_memtime()
#define SECT(k) do { uint64_t now_ = __builtin_amdgcn_s_memtime(); sect_[k] += now_ - tprev_; tprev_ = now_; } while (0)
#define SECT_END() do { if (sect_[1]) for (int k_ = 0; k_ < 6; k_++) atomicAdd(&g_sect[k_], (unsigned long long)sect_[k_]); atomicAdd(&g_sect[7], 1ull); } while (0)
#else
#define SECT_BEGIN() do {} while (0)
#define SECT(k) do {} while (0)
#define SECT_END() do {} while (0)
#endif

// ReSTIR DI reservoir in HBM: 3 float4 = {M, weight_sum, UCW, triangle}, {point, target},
// {flags} (ReSTIRDIReservoir / ReSTIRDISample, Reservoir.h:22-116; SampleFlags.h:10-22)
enum : uint32_t { RF_ENVMAP = 1u, RF_BSDF_REFRACTION = 2u, RF_UNOCCLUDED = 4u };
struct RResv { int M; float wsum; float UCW; int tri; v3 point; float target; uint32_t flags; };
DEV RResv rr_default() {
    RResv r;
    r.M = 0; r.wsum = 0.0f; r.UCW = 0.0f; r.tri = -1; r.point = mk3(0.0f, 0.0f, 0.0f); r.target = 0.0f; r.flags = 0u;
    return r;
}
DEV RResv rr_load(const float4* b, int i) {
    float4 a = b[3 * (size_t)i], c = b[3 * (size_t)i + 1], d = b[3 * (size_t)i + 2];
    RResv r;
    r.M = __float_as_int(a.x); r.wsum = a.y; r.UCW = a.z; r.tri = __float_as_int(a.w);
    r.point = mk3(c.x, c.y, c.z); r.target = c.w; r.flags = __float_as_uint(d.x);
    return r;
}
DEV void rr_store(float4* b, int i, const RResv& r) {
    b[3 * (size_t)i] = make_float4(__int_as_float(r.M), r.wsum, r.UCW, __int_as_float(r.tri));
    b[3 * (size_t)i + 1] = make_float4(r.point.x, r.point.y, r.point.z, r.target);
    b[3 * (size_t)i + 2] = make_float4(__uint_as_float(r.flags), 0.0f, 0.0f, 0.0f);
}

// the sky seen by a path that left the scene (FullPathTracer.h:243-286), clamped
DEV Col miss_radiance(const DevScene& S, const MptFrame& F, int bounce, v3 d, Col thr) {
    const MptRenderSettings& rs = F.render_settings;
    const MptWorldSettings& ws = F.world_settings;
    Col sky = col(0.0f);
    if (ws.ambient_light_type == MPT_AMBIENT_UNIFORM || F.bsdf_flags.white_furnace_mode) sky = C3(ws.uniform_light_color);
    else if (ws.ambient_light_type == MPT_AMBIENT_ENVMAP) {
        bool sampled = F.options.envmap_sampling != MPT_ESS_NO_SAMPLING;
        if (!sampled || bounce == 0) {
            sky = eval_env_no_pdf(S, F, d);
            bool unscale = sampled ? !ws.envmap_scale_background_intensity : (!ws.envmap_scale_background_intensity && bounce == 0);
            if (unscale) sky /= ws.envmap_intensity;
        }
    }
    sky = clamp_contrib(sky, rs.envmap_contribution_clamp, true);
    return clamp_contrib(sky * thr, rs.indirect_contribution_clamp, bounce > 0);
}

enum ShadeOp {
    OP_DONE = 0, OP_RIS_LIGHT, OP_RIS_BSDF, OP_RIS_WIN, OP_MIS_LIGHT, OP_MIS_BSDF, OP_UNI_LIGHT, OP_BSDF_LIGHT,
    OP_ENV_LIGHT, OP_ENV_BSDF, OP_CONT, OP_RESTIR
};
// Shading stages (k_shade's ST): the operations of a vertex fall into three groups that run
// in this RNG order -- light sampling (NEE / MIS / RIS / ReSTIR DI final shading), envmap
// sampling (alias-table light sample + its BSDF-sampled MIS partner), the BSDF-sampled
// continuation with Russian roulette.  ST = SG_ALL shades a vertex in one kernel; a split
// launches one kernel per group (or per pair), each continuing the vertex's RNG stream where
// the previous one stored it.  The first stage (the one with SG_LIGHT) does the hit
// processing and leaves the surface (shading / geometric normal, material) in a per-slot
// record for the later ones.
enum { SG_LIGHT = 1, SG_ENV = 2, SG_CONT = 4, SG_ALL = 7 };
DEV constexpr int op_group(int op) {
    return op == OP_DONE ? 0 : (op == OP_ENV_LIGHT || op == OP_ENV_BSDF) ? SG_ENV : op == OP_CONT ? SG_CONT : SG_LIGHT;
}
// the first operation at or after `op` (in the vertex's order) that stage ST runs
template <int ST>
DEV int stage_op(int op, bool do_env, bool do_cont) {
    if (!(ST & SG_LIGHT) && op_group(op) == SG_LIGHT) op = do_env ? OP_ENV_LIGHT : (do_cont ? OP_CONT : OP_DONE);
    if (!(ST & SG_ENV) && op_group(op) == SG_ENV) op = do_cont ? OP_CONT : OP_DONE;
    if (!(ST & SG_CONT) && op == OP_CONT) op = OP_DONE;
    return op;
}

struct ShadeArgs {
    DevScene S;
    DevPaths P;
    const MptFrame* F;
    int bounce;
    int last_bounce;
    int32_t* q_cur;            // the vertices to shade (k_split's class list)
    const int32_t* count_cur;
    int32_t* q_defer;          // PLAIN: vertices handed to the generic kernel (seen from inside)
    int32_t* count_defer;
    int force_defer;           // test hook (MPT_SHADE_CLASSES=2): defer every plain vertex
    int rev;                   // the list grows downward from q_cur (the glass class, stored at the top of qf)
    int mat_private;           // (host) launch k_shade<..., MATP = true>
};

// the plain class samples directions from the vertex's PEval (principled_sample_dir_plain)
#ifndef MPT_PLAIN_SAMPLE_PE
#define MPT_PLAIN_SAMPLE_PE 1
#endif
#ifndef MPT_SHADE_WAVES
#define MPT_SHADE_WAVES 2
#endif
#ifndef MPT_SHADE_PEP
#define MPT_SHADE_PEP 0   // 1: the plain kernel keeps the per-vertex terms as the plain record (dev_bsdf.h PEvalP): measured +0.7 % at 2 waves, +2.8 % at 3 (77 spilled VGPRs), r06c
#endif
// Material classes (mat_tex bit MT_FULL, k_resolve_materials): k_split sorts the hit
// vertices into the plain-dielectric list (no coat, sheen, metal, transmission or thin film:
// the diffuse + specular base of the Principled BSDF, most of a city) and the list of every
// other material.  k_shade<OVR, true> shades the plain list with those lobes compiled out
// (fewer registers and instructions, dev_bsdf.h FULL = false), k_shade<OVR, false> the rest
// with the generic code.  A plain vertex seen from inside (the glass lobe then has weight 1)
// is deferred to the generic kernel before it writes anything.
#ifndef MPT_SHADE_WAVES_PLAIN
#define MPT_SHADE_WAVES_PLAIN MPT_SHADE_WAVES
#endif
// an operation test that a stage without the operation's group compiles out
#define OPIS(X) ((ST & op_group(X)) && op == (X))
// the later stages (envmap, continuation: one or two BSDF evaluations per vertex) keep the
// per-vertex BSDF terms in registers and run at more waves
#ifndef MPT_SHADE_WAVES_LATE
#define MPT_SHADE_WAVES_LATE 3
#endif
#ifndef MPT_SHADE_PE_LDS_LATE
#define MPT_SHADE_PE_LDS_LATE 0
#endif
// MATP: a textured vertex's resolved material (intersection_material) in the lane's private
// memory instead of the per-slot global copy P.mat_slot.  Private (scratch) memory is
// interleaved per dword across a wave's lanes, so every field load of the BSDF code is one
// contiguous 256-B access per wave, where the slot-major 332-B copies put each lane's field in
// its own cache line (C3T shading 2.73 -> 2.17 ms/spp).  The material pointer then needs flat
// addressing for the untextured materials too (C3 shading +3 %), so MATP is chosen per scene by
// its share of textured triangles (LaunchCfg::mat_private).  The split stages (ST != SG_ALL)
// hand the material to the next stage and keep P.mat_slot.
template <int OVR, bool PLAIN, bool EXT = false, bool GLASS = false, int ST = SG_ALL, bool MATP = false>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(
    !(ST & SG_LIGHT) ? MPT_SHADE_WAVES_LATE : (PLAIN ? MPT_SHADE_WAVES_PLAIN : MPT_SHADE_WAVES)))) void k_shade(ShadeArgs A) {
    constexpr int CLS = PLAIN ? BC_PLAIN : (GLASS ? BC_GLASS : BC_FULL);   // the BSDF code's class (dev_bsdf.h)
    constexpr bool PE_PLAIN = MPT_SHADE_PEP && PLAIN && OVR == MPT_BSDF_NONE && !EXT;   // the plain record (PEvalP)
    constexpr bool FIRST = (ST & SG_LIGHT) != 0;   // hit processing, AOVs, deferral, emission
    constexpr bool LAST = (ST & SG_CONT) != 0;
    static_assert(!EXT || ST == SG_ALL, "extended light sampling shades in one stage");
    const DevScene& S = A.S;
    const DevPaths& P = A.P;
    const MptFrame& F = *A.F;
    const MptRenderSettings& rs = F.render_settings;
    const int bounce = A.bounce;
    // the grid covers the whole wavefront, a class list is often much shorter: blocks past its
    // end leave at once (an empty 4K x 4-sample launch otherwise costs ~0.2 ms)
    const int count = *A.count_cur;
    if ((int)(blockIdx.x * TB) >= count) return;
    int i = blockIdx.x * TB + threadIdx.x;
    bool valid = i < count;
    int slot = valid ? (A.rev ? A.q_cur[-1 - i] : A.q_cur[i]) : 0;
    if (!FIRST && slot < 0) { valid = false; slot = 0; }   // deferred by the first stage

    BCtx bc;
    bc.mats = S.mats;
    bc.luts = DevLuts{S.lut_conductor, S.lut_glossy, S.lut_glass, S.lut_glass_inv, S.lut_thin_glass, S.lut_sheen};
    bc.clearcoat_comp = F.bsdf_flags.clearcoat_compensation_approximation;
    bc.masking = F.bsdf_flags.ggx_masking_shadowing;

    bool cont = false;   // continuation ray emitted
    SECT_BEGIN();
    if (valid) {
        float4 ro = ld_s(&P.ray_o[slot]), rdv = ld_s(&P.ray_d[slot]), hv = ld_s(&P.hit[slot]);
        v3 o = mk3(ro.x, ro.y, ro.z), d = mk3(rdv.x, rdv.y, rdv.z);
        int prim = (int)__float_as_uint(hv.w);
        bool found = prim >= 0;
        VState vs = vs_load_s(P.vsA, P.vsB, slot);
        Rng rng = make_rng(ld_s(&P.rng[slot]));
        const float4 thv = ld_s(&P.thr[slot]);
        Col thr = col(thv.x, thv.y, thv.z);
        const Col thr_vertex = thr;        // the NEE terms' throughput (k_resolve)
        // (bounce pipeline, P.ce: this vertex's addition to col, handed to k_resolve, which adds it
        // after the previous bounce's resolve -- the sum keeps its order)
        Col rcol = col(0.0f);
        if (!P.ce) {
            const float4 cv = ld_s(&P.col[slot]);
            rcol = col(cv.x, cv.y, cv.z);
        }
        v3 ip = mk3(0, 0, 0), gn = mk3(0, 0, 0), sn = mk3(0, 0, 0);
        // The material is read through a pointer (L1/L2-resident) instead of being held in
        // registers: untextured materials use the per-material resolved copy, textured ones
        // (and white-furnace mode) a per-slot resolved copy written here.
        const Mat* mp = S.mats_res;
        bool mat_in_slot = false;   // mp is the per-slot resolved copy
        constexpr bool MAT_PRIV = MATP && ST == SG_ALL;
        Mat mat_priv;               // MAT_PRIV: the textured vertex's resolved material
        if (!FIRST) {
            // a later stage: the surface as the first stage left it (after every flip)
            const float4 ra = ld_s(&P.nhit[slot]), rb = ld_s(&P.s_gn[slot]);
            sn = mk3(ra.x, ra.y, ra.z);
            gn = mk3(rb.x, rb.y, rb.z);
            const int mref = __float_as_int(ra.w);
            mp = mref < 0 ? &P.mat_slot[slot] : &S.mats_res[mref];
            ip = o + hv.x * d;
            if (bounce == 0) d = normalize(d);
        } else if (found) {
            // trace_ray hit processing (Intersect.h:154-216)
            float t = hv.x;
            v2 uv = mk2(hv.y, hv.z);
            ip = o + t * d;
            const HitAttr ha = hit_attributes(S, prim, uv);
            const v2 tc = ha.tc;
            gn = ha.gn;
            sn = ha.sn;
            const int mi = ha.mi;
            if (F.bsdf_flags.white_furnace_mode || (S.mat_tex[mi] & MT_TEXTURED)) {
                if (MAT_PRIV) {
                    mat_priv = intersection_material(S, mi, tc, F.bsdf_flags.white_furnace_mode);
                    mp = &mat_priv;
                } else {
                    P.mat_slot[slot] = intersection_material(S, mi, tc, F.bsdf_flags.white_furnace_mode);
                    mp = &P.mat_slot[slot];
                }
                mat_in_slot = true;
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
        }
        const Mat& m = *mp;
        if (FIRST && bounce == 0) {
            // CameraRays G-buffer hand-off (CameraRays.h:147-166) and FullPathTracer's
            // re-read of it (FullPathTracer.h:131-150): emissive flip, normalise, restart RNG
            if (found && is_emissive(m) && dot(-d, gn) < 0) { gn = -gn; sn = -sn; }
            gn = normalize(gn);
            sn = normalize(sn);
            d = normalize(d);
            rng = make_rng(P.seeds[slot].y);   // path_seed(F, P, slot, false), from k_camera
        }
        if (PLAIN && FIRST) {
            // principled_eval_pre's 'outside' with the normal the vertex is shaded with
            const v3 sn_f = (is_emissive(m) && dot(-d, gn) < 0) ? -sn : sn;
            // (a material of the MT_TEXMETAL class is shaded here where its texel is not metallic)
            if (!(dot(-d, sn_f) > 0 || m.thin_walled) || m.metallic != 0.0f || A.force_defer || (PE_PLAIN && !plain_vertex_ok(m))) {
                A.q_defer[atomicAdd(A.count_defer, 1)] = slot;
                atomicAdd(&P.counters[CTR_DEFER], 1);
                A.q_cur[i] = -1;    // k_compact / k_resolve skip the entry here
                return;             // nothing written (no block-wide operation follows)
            }
        }
        uint32_t fl = 0;
        uint32_t qm = 0;            // staged NEE queries (bits 0..3) + continuation (bit 4)
        if (found) {
            if (FIRST && bounce == 0) {
                float4 a = P.alb[slot], n4 = P.nrm[slot];
                P.alb[slot] = make_float4(a.x + m.base_color.r, a.y + m.base_color.g, a.z + m.base_color.b, 0.0f);
                P.nrm[slot] = make_float4(n4.x + sn.x, n4.y + sn.y, n4.z + sn.z, 0.0f);
            }
            if (FIRST && is_emissive(m) && dot(-d, gn) < 0) { gn = -gn; sn = -sn; }
            v3 view = -d;
            if (FIRST) fl |= NF_SHADED;
            const int lss = F.options.direct_light_sampling;
            const MptWorldSettings& ws = F.world_settings;
            // ---------------- which BSDF operations this vertex runs, in RNG order ----------------
            // sample_one_light (Lights.h:277-321); ReSTIR DI: the reservoir at bounce 0 (also
            // with only an envmap), RIS at later bounces (Lights.h:243-275, RIS.h:292-302)
            const bool restir = lss == MPT_LSS_RESTIR_DI;
            bool do_light = (S.n_emissive != 0 || (restir && ws.ambient_light_type == MPT_AMBIENT_ENVMAP)) &&
                            !(F.bsdf_flags.white_furnace_mode && F.bsdf_flags.white_furnace_mode_turn_off_emissives);
            if (do_light && is_emissive(m)) {
                do_light = false;
                if (FIRST && m.emissive_texture_used && bounce > 0) {
                    fl |= NF_IMM;
                    const Col e = emission_of(m);
                    st_s(&P.na[slot], make_float4(e.r, e.g, e.b, 0.0f));
                }
            }
            do_light = do_light && lss != MPT_LSS_NO_DIRECT_LIGHT_SAMPLING;
            const int lssb = bounce_lss(F, bounce);
            // sample_lights_RIS returns 0 without emissive triangles (RIS.h:292-302)
            if (restir && bounce > 0 && S.n_emissive == 0 && lssb == MPT_LSS_RIS_BSDF_AND_LIGHT) do_light = false;
            if (FIRST && do_light) fl |= NF_L;
            const bool do_env = ws.ambient_light_type == MPT_AMBIENT_ENVMAP && !F.bsdf_flags.white_furnace_mode &&
                                !is_emissive(m) && ws.envmap_intensity > 0.0f && F.options.envmap_sampling != MPT_ESS_NO_SAMPLING &&
                                !(restir && bounce == 0);
            const bool env_use = lss != MPT_LSS_NO_DIRECT_LIGHT_SAMPLING;
            const bool do_cont = bounce < A.last_bounce;
            const float ism = dot(view, gn) < 0 ? -1.0f : 1.0f;
            const v3 ep = ip + sn * 1.0e-4f * ism;              // NEE origin (Lights.h / RIS.h)
            const int nl = rs.ris_number_of_light_candidates, nbc = rs.ris_number_of_bsdf_candidates;
            int op = OP_DONE;
            if (do_light) {
                if (restir && bounce == 0) op = OP_RESTIR;
                else if (lssb == MPT_LSS_RIS_BSDF_AND_LIGHT) op = nl > 0 ? OP_RIS_LIGHT : (nbc > 0 ? OP_RIS_BSDF : OP_RIS_WIN);
                else if (lssb == MPT_LSS_MIS_LIGHT_BSDF) op = OP_MIS_LIGHT;
                else if (lssb == MPT_LSS_UNIFORM_ONE_LIGHT) op = OP_UNI_LIGHT;
                else if (lssb == MPT_LSS_BSDF) op = OP_BSDF_LIGHT;
            }
            if (op == OP_DONE) op = do_env ? OP_ENV_LIGHT : (do_cont ? OP_CONT : OP_DONE);
            op = stage_op<ST>(op, do_env, do_cont);
            // RIS reservoir (sample_bsdf_and_lights_RIS_reservoir, RIS.h:82-289)
            float wsum = 0.0f, targetW = 0.0f;
            v3 pointW = mk3(0, 0, 0);
            int triW = -1, ris_c = 0;
            bool hasW = false;
            float r_add = 0.0f;                // the RIS BSDF candidate's random (add_one_candidate)
            // per-vertex half of every BSDF evaluation below, one LDS record per lane (65
            // dwords: an odd stride, so lane-parallel accesses are bank-conflict free).  Held
            // in registers it pushed the kernel into ~140 spilled VGPRs; in LDS it costs one
            // ds_read per field per evaluation (-23% k_shade time on C3).  The kernel's 80640 B
            // of LDS per 256-lane block are these 66560 B plus 14080 B (55 B per lane) of private
            // arrays that the compiler's promote-alloca pass moves into the LDS the 2-wave
            // occupancy leaves free (the rest, 128 B per lane, in scratch); two blocks fill a
            // CU's 160 KB, so LDS and VGPRs (249) both cap the kernel at 2 waves / SIMD
            // The plain kernel keeps the plain record instead (dev_bsdf.h PEvalP: 35 dwords)
            constexpr bool PE_LDS = (ST & SG_LIGHT) || MPT_SHADE_PE_LDS_LATE;
            using PE = typename std::conditional<PE_PLAIN, PEvalP, PEval>::type;
            __shared__ PE pe_lds[PE_LDS ? TB : 1];
            PE pe_reg;
            PE& pe = PE_LDS ? pe_lds[threadIdx.x] : pe_reg;
            // the first light sample's emissive record, loaded while the per-vertex BSDF terms are
            // computed (its index is the vertex's next draw); each RIS light candidate then loads
            // the next one's record (the draws between them are fixed: two for the point, one for
            // the reservoir) while it is evaluated
            EmPrefetch pf;
            pf.valid = false;
            if (MPT_EM_PREFETCH && (ST & SG_LIGHT) && (op == OP_RIS_LIGHT || op == OP_MIS_LIGHT || op == OP_UNI_LIGHT)) pf.issue(S, rng);
            SECT(0);
            bsdf_eval_pre<OVR, CLS>(bc, m, vs, view, sn, pe);
            SECT(5);
            if constexpr (EXT) {
                if (do_light && !(restir && bounce == 0)) {
                    // extended light sampling: every light sample's draws, records and queries
                    ext_light<OVR, CLS>(S, P, F, bc, m, vs, pe, slot, prim, ip, sn, gn, view, ism, ep, lssb, rng);
                    fl |= NF_EXT;
                    op = do_env ? OP_ENV_LIGHT : (do_cont ? OP_CONT : OP_DONE);
                }
            }
            Col fW = col(0.0f);                // BSDF value / pdf at the RIS light winner
            float pdfW = 0.0f;
            // One BSDF evaluation site for every operation of the vertex: each iteration
            // prepares a direction (light / envmap sample, or a BSDF lobe sample), evaluates
            // the BSDF once, and consumes the result.  All lanes of a wave meet at the same
            // evaluation whatever operation they are on.
            while (op != OP_DONE) {
                VState tv = vs;
                RResv rres;                    // ReSTIR DI output reservoir (OP_RESTIR)
                v3 L = mk3(0.0f, 0.0f, 0.0f);
                bool do_eval = false;
                float lpdf = 0.0f, dist = 0.0f, geo = 0.0f;
                LightInfo li;
                li.tri = -1; li.emission = col(0.0f);
                v3 lp = mk3(0.0f, 0.0f, 0.0f);
                Col ec = col(0.0f);
                bool inner = false;
                float4 etex = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // OP_ENV_BSDF: the envmap texel along L
                if (OPIS(OP_RIS_BSDF) || OPIS(OP_MIS_BSDF) || OPIS(OP_BSDF_LIGHT) || OPIS(OP_ENV_BSDF) || OPIS(OP_CONT)) {
                    do_eval = (MPT_PLAIN_SAMPLE_PE && CLS == BC_PLAIN && OVR == MPT_BSDF_NONE)
                                  ? principled_sample_dir_plain(bc, m, tv, pe, view, sn, gn, L, rng)
                                  : bsdf_sample_dir<OVR, CLS>(bc, m, tv, view, sn, gn, L, rng);
                    // the texel's load is issued here and waited for after the evaluation
                    if (MPT_ENV_EARLY && OPIS(OP_ENV_BSDF) && do_eval) etex = env_fetch(S, F, L);
                } else if (OPIS(OP_RIS_LIGHT)) {
                    lp = pf.sample(S, rng, lpdf, li);
                    if (MPT_EM_PREFETCH && ris_c + 1 < nl) {   // the next candidate's index draw follows this one's reservoir draw
                        Rng nx = rng;
                        (void)nx();
                        pf.issue(S, nx);
                    }
                    if (lpdf > 0.0f) {
                        v3 tl = lp - ep;
                        dist = length(tl);
                        tl = tl / dist;
                        float cl = absr(dot(li.normal, -tl));
                        geo = maxr(0.0f, dot(sn * ism, tl));
                        if (geo > 0.0f && cl > 1.0e-6f) {
                            inner = true;
                            lpdf *= dist * dist;
                            lpdf /= cl;
                            if (min_contrib(rs.minimum_light_contribution, li.emission / lpdf)) { L = tl; do_eval = true; }
                        }
                    }
                } else if (OPIS(OP_RIS_WIN)) {
                    // evaluate_reservoir_sample for the light winner (RIS.h:18-80), speculatively
                    v3 ep2 = ip + sn * 1.0e-4f;
                    v3 sd = pointW - ep2;
                    dist = length(sd);
                    L = sd / dist;
                    lp = ep2;
                    // outside the surface the winner's direction is bit-identical to its
                    // candidate's (same origin), and so is the evaluation: reuse it
                    do_eval = hasW && ism != 1.0f;
                } else if (OPIS(OP_MIS_LIGHT) || OPIS(OP_UNI_LIGHT)) {
                    // sample_one_light_MIS (Lights.h:115-220) / _no_MIS (Lights.h:22-65)
                    lp = pf.sample(S, rng, lpdf, li);
                    if (lpdf > 0.0f) {
                        v3 so = OPIS(OP_MIS_LIGHT) ? ep : ip + sn * 1.0e-4f;
                        v3 sd = lp - so;
                        dist = length(sd);
                        L = sd / dist;
                        geo = absr(dot(li.normal, -L));
                        lp = so;
                        do_eval = geo > 0.0f;
                    }
                } else if (OPIS(OP_RESTIR)) {
                    // sample_light_ReSTIR_DI + evaluate_ReSTIR_DI_reservoir (FinalShading.h:16-115);
                    // a batched ReSTIR DI launch reads the sample's kept final reservoirs
                    float4* rsb = P.rs_out;
                    size_t rpix = (size_t)slot + P.pix_off;
                    if (P.rs_keep_on) {
                        int kpix, ksub;
                        batch_split(P, slot, kpix, ksub);
                        rsb = P.rs_keep + (size_t)ksub * 3 * (size_t)P.rs_keep_n;
                        rpix = (size_t)kpix;   // rs_keep holds the band's pixels
                    }
                    rres = rr_load(rsb, (int)rpix);
                    if ((rres.flags & RF_ENVMAP) && ws.ambient_light_type != MPT_AMBIENT_ENVMAP) {
                        rres.UCW = 0.0f;   // validate_reservoir writes through to the buffer
                        float4 a = rsb[3 * rpix];
                        rsb[3 * rpix] = make_float4(a.x, a.y, 0.0f, a.w);
                    }
                    if (rres.UCW > 0.0f) {
                        if (rres.flags & RF_ENVMAP) { L = mat_x_vec(ws.envmap_to_world_matrix.m, rres.point); dist = 1.0e35f; }
                        else { L = rres.point - ip; dist = length(L); L = L / dist; }
                        do_eval = true;
                    }
                } else if (OPIS(OP_ENV_LIGHT)) {
                    ec = env_sample(S, F, L, lpdf, rng);
                    geo = dot(sn, L);
                    do_eval = lpdf > 0.0f && geo > 0.0f;
#ifdef MPT_DEBUG_SLOT
                    if (slot == MPT_DEBUG_SLOT) printf("GPU env ec %a %a %a pdf %a dir %a %a %a cos %a ip %a %a %a prim %d\n", ec.r, ec.g, ec.b, lpdf, L.x, L.y, L.z, geo, ip.x, ip.y, ip.z, prim);
#endif
                }
                float pdf = 0.0f;
                Col f = col(0.0f);
                SECT(1);
                if (do_eval) f = bsdf_eval_post<OVR, CLS>(bc, m, tv, pe, sn, L, pdf);
                SECT(2);
                int next = OP_DONE;
                if (OPIS(OP_RIS_LIGHT)) {
                    float target = 0.0f, cw = 0.0f;
                    if (inner) {
                        float bp = 0.0f;
                        if (do_eval) {
                            bp = pdf;
                            Col lc = f * li.emission * geo;
                            target = min_contrib(rs.minimum_light_contribution, lc / bp / lpdf) ? lum(lc) : 0.0f;
                        }
                        cw = balance(lpdf, (float)nl, bp, (float)nbc) * target / lpdf;
                    }
                    wsum += cw;
                    if (rng() < cw / wsum) { hasW = true; targetW = target; pointW = lp; triW = li.tri; fW = f; pdfW = pdf; }
                    ris_c++;
                    next = ris_c < nl ? OP_RIS_LIGHT : (nbc > 0 ? OP_RIS_BSDF : OP_RIS_WIN);
                } else if (OPIS(OP_RIS_BSDF)) {
                    bool refr = dot(L, sn * ism) < 0;
                    v3 so = refr ? ip + sn * 1.0e-4f * ism * -1.0f : ep;
                    if (pdf > 0.0f) {
                        fl |= NF_B | (refr ? NF_B_REFR : 0u);
                        stage_query(P, slot, 3, qm, so, prim, L, 1.0e35f - 1.0e-4f);
                        st_s(&P.nb[slot], make_float4(f.r, f.g, f.b, pdf));
                        st_s(&P.ndir[slot], make_float4(L.x, L.y, L.z, absr(dot(sn, L))));
                    }
                    r_add = rng();
                    next = OP_RIS_WIN;
                } else if (OPIS(OP_RIS_WIN)) {
                    if (!do_eval) { f = fW; pdf = pdfW; }
                    st_s(&P.nris[slot], make_float4(wsum, targetW, r_add, __int_as_float(triW)));
                    if (hasW) {
                        fl |= NF_RIS_W;
                        stage_query(P, slot, 0, qm, lp, prim, L, dist - 1.0e-4f);
                        st_s(&P.na[slot], make_float4(f.r, f.g, f.b, maxr(0.0f, dot(sn, L))));
                    }
                    next = OP_DONE;
                } else if (OPIS(OP_MIS_LIGHT)) {
                    if (do_eval && pdf != 0.0f) {
                        float lp2 = lpdf;
                        lp2 *= dist * dist;
                        lp2 /= geo;
                        float w = balance(lp2, pdf);
                        float cosv = maxr(dot(sn, L), 0.0f);
                        const Col a = f * cosv * li.emission * w / lp2;
                        st_s(&P.na[slot], make_float4(a.r, a.g, a.b, 0.0f));
                        fl |= NF_A;
                        stage_query(P, slot, 0, qm, lp, prim, L, dist - 1.0e-4f);
                    }
                    next = lpdf > 0.0f ? OP_MIS_BSDF : OP_DONE;
                } else if (OPIS(OP_MIS_BSDF)) {
                    bool refr = dot(L, sn * ism) < 0;
                    v3 bo = refr ? ip + sn * 1.0e-4f * ism * -1.0f : ep;
                    if (pdf > 0) {
                        fl |= NF_B;
                        stage_query(P, slot, 3, qm, bo, prim, L, 1.0e35f - 1.0e-4f);
                        st_s(&P.nb[slot], make_float4(f.r, f.g, f.b, pdf));
                        st_s(&P.ndir[slot], make_float4(L.x, L.y, L.z, absr(dot(sn, L))));
                    }
                } else if (OPIS(OP_UNI_LIGHT)) {
                    if (do_eval && pdf != 0.0f) {
                        float lp2 = lpdf;
                        lp2 *= dist * dist;
                        lp2 /= geo;
                        float cosv = maxr(dot(sn, L), 0.0f);
                        const Col a = li.emission * cosv * f / lp2;
                        st_s(&P.na[slot], make_float4(a.r, a.g, a.b, 0.0f));
                        fl |= NF_A;
                        stage_query(P, slot, 0, qm, lp, prim, L, dist - 1.0e-4f);
                    }
                } else if (OPIS(OP_BSDF_LIGHT)) {
                    // sample_one_light_bsdf (Lights.h:67-113)
                    bool refr = dot(L, sn * ism) < 0;
                    if (pdf > 0.0f) {
                        v3 no = refr ? ip + sn * 1.0e-4f * ism * -1.0f : ip + sn * 1.0e-4f;
                        fl |= NF_B;
                        stage_query(P, slot, 3, qm, no, prim, L, 1.0e35f - 1.0e-4f);
                        st_s(&P.nb[slot], make_float4(f.r, f.g, f.b, pdf));
                        st_s(&P.ndir[slot], make_float4(L.x, L.y, L.z, maxr(0.0f, dot(sn, L))));
                    }
                } else if (OPIS(OP_RESTIR)) {
                    if (do_eval) {
                        float c = dot(sn, L);
                        if (rres.flags & RF_BSDF_REFRACTION) c = absr(c);
                        if (c > 0.0f) {
                            Col e;
                            if (rres.flags & RF_ENVMAP) { float ep_; e = env_eval(S, F, L, ep_); }
                            else e = emission_of(S.mats[S.mat_idx[rres.tri]]);
                            const Col a = f * rres.UCW * e * c;
                            st_s(&P.na[slot], make_float4(a.r, a.g, a.b, 0.0f));
                            fl |= NF_A;
                            if (!(rres.flags & RF_UNOCCLUDED) && rs.restir_di_settings.do_final_shading_visibility) {
                                fl |= NF_AQ;
                                stage_query(P, slot, 0, qm, ip, prim, L, dist - 1.0e-4f);
                            }
                        }
                    }
                } else if (OPIS(OP_ENV_LIGHT)) {
                    // Envmap.h:151-246
                    if (do_eval) {
                        float mw = F.options.envmap_bsdf_mis ? balance(lpdf, pdf) : 1.0f;
                        const Col e1 = f * geo * mw * ec / lpdf;
                        st_s(&P.ne1[slot], make_float4(e1.r, e1.g, e1.b, 0.0f));
#ifdef MPT_DEBUG_SLOT
                        if (slot == MPT_DEBUG_SLOT) { Col e1_ = f * geo * mw * ec / lpdf; printf("GPU env f %a %a %a bp %a mw %a e1 %a %a %a\n", f.r, f.g, f.b, pdf, mw, e1_.r, e1_.g, e1_.b); }
#endif
                        if (env_use) {
                            fl |= NF_E1;
                            stage_query(P, slot, 1, qm, ip, prim, L, 1.0e35f - 1.0e-4f);
                        }
                    }
                    next = F.options.envmap_bsdf_mis ? OP_ENV_BSDF : OP_DONE;
                } else if (OPIS(OP_ENV_BSDF)) {
                    float c2 = absr(dot(sn, L));
                    if (pdf > 0.0f) {
                        float epdf;
                        Col er = MPT_ENV_EARLY ? env_eval_tex(S, F, L, etex, epdf) : env_eval(S, F, L, epdf);
                        if (epdf > 0.0f && env_use) {
                            float mw = balance(pdf, epdf);
                            const Col e2 = er * mw * c2 * f / pdf;
                            st_s(&P.ne2[slot], make_float4(e2.r, e2.g, e2.b, 0.0f));
                            fl |= NF_E2;
                            stage_query(P, slot, 2, qm, ip, prim, L, 1.0e35f - 1.0e-4f);
                        }
                    }
                } else if (OPIS(OP_CONT)) {
                    // continuation (FullPathTracer.h:221-247)
#ifdef MPT_DEBUG_SLOT
                    if (slot == MPT_DEBUG_SLOT) printf("GPU b%d cont mi %d vs %d %d %d %d st %x %x %x L %a %a %a f %a %a %a pdf %a\n", bounce, (int)(mp - S.mats_res), tv.incident, tv.outgoing, (int)tv.inside, tv.pos, tv.st[0], tv.st[1], tv.st[2], L.x, L.y, L.z, f.r, f.g, f.b, pdf);
#endif
                    vs = tv;
                    Col att = f * absr(dot(L, sn)) / pdf;
                    // 'if (bsdf_pdf <= 0.0f) break' (FullPathTracer.h:228): a NaN pdf (e.g. a
                    // thin-film glass lobe sampled from inside, TIR in the film) continues, and the
                    // NaN ray ends as a sample the sanity check discards
                    if (!(pdf <= 0.0f)) {
                        bool alive = true;
                        if (bounce >= rs.russian_roulette_min_depth && rs.use_russian_roulette) {
                            float sp;
                            if (rs.path_russian_roulette_method == 0) sp = maxc(thr);
                            else sp = sqrtf(maxc(thr * att) / maxc(thr));
                            sp = minr(sp, 1.0f);
                            if (rng() > sp) alive = false;
                            else {
                                float inc = 1.0f / sp;
                                if (rs.russian_roulette_throughput_clamp > 0.0f) inc = minr(inc, rs.russian_roulette_throughput_clamp);
                                thr *= inc;
                            }
                        }
                        if (alive) {
                            thr *= dispersion_ray_color(vs.wl, m.dispersion_scale);
                            thr *= att;
                            st_s(&P.ray_o[slot], make_float4(ip.x, ip.y, ip.z, __uint_as_float((uint32_t)prim)));
                            st_s(&P.ray_d[slot], make_float4(L.x, L.y, L.z, INFINITY));
                            cont = true;
                        }
                    }
                    next = -1;
                }
                // after the light strategy: envmap, then the continuation
                if (next == OP_DONE && op != OP_ENV_LIGHT && op != OP_ENV_BSDF && do_env) next = OP_ENV_LIGHT;
                else if (next == OP_DONE && do_cont) next = OP_CONT;
                op = next < 0 ? OP_DONE : stage_op<ST>(next, do_env, do_cont);
                SECT(3);
            }
            // emission (FullPathTracer.h:192-214); without direct light sampling no later stage
            // sets a NEE flag (env_use), so the first stage's clearing covers the vertex
            if (FIRST && lss == MPT_LSS_NO_DIRECT_LIGHT_SAMPLING) {
                Col he = clamp_contrib(emission_of(m), rs.indirect_contribution_clamp, bounce > 0);
                rcol += he * thr_vertex;
                fl &= ~(NF_A | NF_B | NF_E1 | NF_E2 | NF_RIS_W | NF_IMM | NF_L);
                fl |= NF_NOADD;
            } else if (FIRST && bounce == 0) {
                rcol += emission_of(m);
            }
            if (FIRST && !LAST) {   // the surface record of the later stages
                const int mref = mat_in_slot ? -1 : (int)(mp - S.mats_res);
                st_s(&P.nhit[slot], make_float4(sn.x, sn.y, sn.z, __int_as_float(mref)));
                st_s(&P.s_gn[slot], make_float4(gn.x, gn.y, gn.z, 0.0f));
            }
        } else {
            rcol += miss_radiance(S, F, bounce, d, thr);   // not reached: k_split sends misses to k_miss
        }
        const uint32_t qb = qm | (cont ? QM_CONT : 0u);
        if (FIRST) {
            st_s(&P.nthr[slot], make_float4(thr_vertex.r, thr_vertex.g, thr_vertex.b, __uint_as_float(fl)));
            st_s(&P.qmask[slot], (uint8_t)qb);
            st_s(P.ce ? &P.ce[slot] : &P.col[slot], make_float4(rcol.r, rcol.g, rcol.b, 0.0f));
        } else {
            if (fl) {
                const float4 t4 = ld_s(&P.nthr[slot]);
                st_s(&P.nthr[slot], make_float4(t4.x, t4.y, t4.z, __uint_as_float(__float_as_uint(t4.w) | fl)));
            }
            if (qb) st_s(&P.qmask[slot], (uint8_t)(ld_s(&P.qmask[slot]) | qb));
        }
        st_s(&P.rng[slot], rng.s);
        if (LAST) st_s(&P.thr[slot], make_float4(thr.r, thr.g, thr.b, 0.0f));
        if (FIRST || LAST) vs_store_s(P.vsA, P.vsB, slot, vs);
    }
    // queue appends (every lane of the wave takes part in the ballots)
    SECT(4);
    SECT_END();
}

// ----------------------------------------------------------------------------------
// k_miss: the paths of the bounce's miss queue (k_split) add the sky and end.  The
// camera ray of bounce 0 is re-normalised as FullPathTracer's re-read of the G-buffer does
// (FullPathTracer.h:131-150, see k_shade).
// ----------------------------------------------------------------------------------
#ifndef MPT_TU_PART   // k_miss
__global__ __launch_bounds__(TB) void k_miss(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int bounce) {
    const int nm = P.counters[CTR_MISS];   // grid-stride, as k_resolve
    for (int i = blockIdx.x * TB + threadIdx.x; i < nm; i += gridDim.x * TB) {
        const int slot = P.qm[i];
        const float4 rdv = ld_s(&P.ray_d[slot]), t4 = ld_s(&P.thr[slot]), cv = ld_s(&P.col[slot]);
        v3 d = mk3(rdv.x, rdv.y, rdv.z);
        if (bounce == 0) d = normalize(d);
        const Col rc = col(cv.x, cv.y, cv.z) + miss_radiance(S, *Fp, bounce, d, col(t4.x, t4.y, t4.z));
        st_s(&P.col[slot], make_float4(rc.r, rc.g, rc.b, 0.0f));
    }
}

#endif
// ----------------------------------------------------------------------------------
// Queue compaction (k_split, k_compact): thread t of a block takes the CP_ITEMS
// consecutive entries [b0 + t * CP_ITEMS, +CP_ITEMS) of the input queue, so the output
// lists keep the queue order inside each block's 8192 entries (the samples of a pixel, and
// neighbouring pixels, stay neighbours from bounce to bounce); block-wide scans give every
// entry its place, one atomic per block and list reserves the block's range.
// ----------------------------------------------------------------------------------
constexpr int CP_NT = 1024;        // threads per block
constexpr int CP_ITEMS = 8;        // queue entries per thread -> 8192 per block

// exclusive block-wide scan of one int per thread (wave64 shuffles + LDS across waves)
DEV int block_scan_excl(int v, int* tmp, int& total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6;
    constexpr int NW = CP_NT / 64;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    if (wid == 0) {
        int w = lane < NW ? tmp[lane] : 0;
        int xs = w;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            int y = __shfl_up(xs, o);
            if (lane >= o) xs += y;
        }
        if (lane < NW) tmp[lane] = xs - w;
        if (lane == NW - 1) tmp[NW] = xs;
    }
    __syncthreads();
    int excl = x - v + tmp[wid];
    total = tmp[NW];
    __syncthreads();
    return excl;
}

// this thread's consecutive queue entries (two 16-B loads when the run is complete)
DEV int load_items(const int32_t* q, int b0, int count, int slots[CP_ITEMS]) {
    const int i0 = b0 + (int)threadIdx.x * CP_ITEMS;
    const int n = max(0, min(CP_ITEMS, count - i0));
    if (n == CP_ITEMS) {
        const int4 a = *reinterpret_cast<const int4*>(q + i0), b = *reinterpret_cast<const int4*>(q + i0 + 4);
        slots[0] = a.x; slots[1] = a.y; slots[2] = a.z; slots[3] = a.w;
        slots[4] = b.x; slots[5] = b.y; slots[6] = b.z; slots[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < CP_ITEMS; j++) slots[j] = j < n ? q[i0 + j] : 0;
    }
    return n;
}

// k_split: the bounce's path queue -> the paths that hit a surface (k_shade, k_compact,
// k_resolve) and those that left the scene (k_miss), so that every lane of a shading wave
// has a vertex to shade instead of idling through the light-sampling loop beside a miss.
// With `classes`, the hits are further sorted by material class (see k_shade): plain
// dielectrics into qh (CTR_HIT), every other material into qf (CTR_FULL) -- with classes = 2
// the glass class (MT_GLASS) into the top of qf, growing downward (CTR_GLASS).
#ifndef MPT_TU_PART   // k_split
__global__ __launch_bounds__(CP_NT) void k_split(DevScene S, DevPaths P, const int32_t* q, const int32_t* count_q,
                                                 int classes, int32_t* zero_next) {
    __shared__ int tmp[CP_NT / 64 + 1];
    __shared__ int base[4];
    const int count = *count_q;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *zero_next = 0;   // the next path queue (filled by k_compact)
        atomicAdd((unsigned long long*)P.ray_counts, (unsigned long long)count);   // the bounce's path rays
    }
    const int b0 = blockIdx.x * CP_NT * CP_ITEMS;
    if (b0 >= count) return;
    int slots[CP_ITEMS];
    const int n = load_items(q, b0, count, slots);
    uint32_t hm = 0u, fm = 0u, gm = 0u;
    int nh = 0, nf = 0, ng = 0;
#pragma unroll
    for (int j = 0; j < CP_ITEMS; j++) {
        // the hit's material class as the traversal reported it (0xff: a miss)
        const uint32_t hc = j < n ? (uint32_t)ld_s(&P.hit_cls[slots[j]]) : 0xffu;
        if (hc != 0xffu) {
            const int32_t mt = classes ? (int32_t)hc : 0;
            if (classes == 2 && (mt & MT_GLASS)) { gm |= 1u << j; ng++; }
            else if ((mt & MT_FULL) && !(mt & MT_TEXMETAL)) { fm |= 1u << j; nf++; }
            else { hm |= 1u << j; nh++; }
        }
    }
    int th, tm, tf, tg;
    int oh = block_scan_excl(nh, tmp, th);
    int om = block_scan_excl(n - nh - nf - ng, tmp, tm);
    int of = block_scan_excl(nf, tmp, tf);
    int og = classes == 2 ? block_scan_excl(ng, tmp, tg) : (tg = 0);
    if (threadIdx.x == 0) {
        base[0] = th ? atomicAdd(&P.counters[CTR_HIT], th) : 0;
        base[1] = tm ? atomicAdd(&P.counters[CTR_MISS], tm) : 0;
        base[2] = tf ? atomicAdd(&P.counters[CTR_FULL], tf) : 0;
        base[3] = tg ? atomicAdd(&P.counters[CTR_GLASS], tg) : 0;
    }
    __syncthreads();
    oh += base[0];
    om += base[1];
    of += base[2];
    og += base[3];
    int32_t* const qg = P.qf + P.n - 1;   // the glass list: qg[-k]
#pragma unroll
    for (int j = 0; j < CP_ITEMS; j++) {
        if (j >= n) break;
        if ((hm >> j) & 1u) P.qh[oh++] = slots[j];
        else if ((fm >> j) & 1u) P.qf[of++] = slots[j];
        else if ((gm >> j) & 1u) qg[-(og++)] = slots[j];
        else P.qm[om++] = slots[j];
    }
}

#endif
// The bounce's shaded vertices: qh[0, CTR_HIT), then qf[0, CTR_FULL), then the glass list
// at the top of qf (qf[n - 1 - k], k < CTR_GLASS); entries that k_shade<PLAIN> deferred to qf
// are -1 in qh.
DEV int shaded_count(const DevPaths& P) { return P.counters[CTR_HIT] + P.counters[CTR_FULL] + P.counters[CTR_GLASS]; }
DEV int shaded_entry(const DevPaths& P, int nh, int i) {
    if (i < nh) return P.qh[i];
    const int nf = P.counters[CTR_FULL];
    return i - nh < nf ? P.qf[i - nh] : P.qf[P.n - 1 - (i - nh - nf)];
}

// k_compact: next path queue + NEE query lists from the per-path masks of the shaded paths
#ifndef MPT_TU_PART   // k_compact
__global__ __launch_bounds__(CP_NT) void k_compact(DevPaths P, int32_t* q_next, int32_t* count_next, int32_t* zero_fetch) {
    __shared__ int tmp[CP_NT / 64 + 1];
    __shared__ int base[5];
    // the next bounce's path traversal, launched right after on the trace-ahead stream, takes its
    // work counter zeroed (frame_bounces)
    if (zero_fetch && blockIdx.x == 0 && threadIdx.x == 0) *zero_fetch = 0;
    const int nh = P.counters[CTR_HIT];
    const int count = shaded_count(P);
    const int b0 = blockIdx.x * CP_NT * CP_ITEMS;
    if (b0 >= count) return;
    int slots[CP_ITEMS];
    int n;
    if (b0 + CP_NT * CP_ITEMS <= nh) n = load_items(P.qh, b0, nh, slots);
    else {
        const int i0 = b0 + (int)threadIdx.x * CP_ITEMS;
        n = max(0, min(CP_ITEMS, count - i0));
#pragma unroll
        for (int j = 0; j < CP_ITEMS; j++) slots[j] = j < n ? shaded_entry(P, nh, i0 + j) : 0;
    }
    uint8_t m[CP_ITEMS];
    int c[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < CP_ITEMS; j++) {
        m[j] = (j < n && slots[j] >= 0) ? ld_s(&P.qmask[slots[j]]) : (uint8_t)0;
        c[0] += (m[j] & QM_CONT) ? 1 : 0;
        c[1] += m[j] & 1u;
        c[2] += (m[j] >> 1) & 1u;
        c[3] += (m[j] >> 2) & 1u;
        c[4] += (m[j] >> 3) & 1u;
    }
    int off[5];
    int32_t* ctr[5] = {count_next, &P.counters[CTR_ANY], &P.counters[CTR_ANY], &P.counters[CTR_ANY], &P.counters[CTR_CL]};
    // one reservation per list; the three any-hit kinds share one list and one atomic
    int tot[5];
#pragma unroll
    for (int k = 0; k < 5; k++) off[k] = block_scan_excl(c[k], tmp, tot[k]);
    if (threadIdx.x == 0) {
        base[0] = tot[0] ? atomicAdd(ctr[0], tot[0]) : 0;
        int a = tot[1] + tot[2] + tot[3];
        int ab = a ? atomicAdd(ctr[1], a) : 0;
        base[1] = ab;
        base[2] = ab + tot[1];
        base[3] = ab + tot[1] + tot[2];
        base[4] = tot[4] ? atomicAdd(ctr[4], tot[4]) : 0;
    }
    __syncthreads();
    int32_t* any = P.nq_tgt;
    int32_t* cl = P.nq_tgt + (size_t)P.n * 3;
    int o0 = base[0] + off[0], o1 = base[1] + off[1], o2 = base[2] + off[2], o3 = base[3] + off[3], o4 = base[4] + off[4];
#pragma unroll
    for (int j = 0; j < CP_ITEMS; j++) {
        int sl = slots[j];
        if (m[j] & QM_CONT) q_next[o0++] = sl;
        if (m[j] & 1u) any[o1++] = sl * 4 + 0;
        if (m[j] & 2u) any[o2++] = sl * 4 + 1;
        if (m[j] & 4u) any[o3++] = sl * 4 + 2;
        if (m[j] & 8u) cl[o4++] = sl * 4 + 3;
    }
}

#endif
// ----------------------------------------------------------------------------------
// k_resolve: finish the vertex's direct lighting with the NEE trace results
// ----------------------------------------------------------------------------------
struct ShadowLightHit { int prim; float dist; v3 sn; Col em; };
DEV bool shadow_light_hit(const DevScene& S, float4 h, ShadowLightHit& out) {
    int prim = (int)__float_as_uint(h.w);
    if (prim < 0) return false;
    v2 uv = mk2(h.y, h.z);
    const HitAttr ha = hit_attributes(S, prim, uv);
    const Mat& m = S.mats[ha.mi];
    const v2 tc = ha.tc;
    if (m.emission_texture_index != MPT_NO_TEXTURE) {
        MptColor e; e.r = 0.0f; e.g = 0.0f; e.b = 0.0f;
        if (S.n_tex > 0) prop_c(S, e, tc, m.emission_texture_index);
        out.em = C3(e);
    } else out.em = emission_of(m);
    out.sn = ha.sn;
    out.prim = prim;
    out.dist = h.x;
    return true;
}
DEV float pdf_emissive_hit(const DevScene& S, const ShadowLightHit& h, v3 d) {
    int3 ti = tri_idx(S, h.prim);
    v3 A = ld3(S.pos, ti.x), B = ld3(S.pos, ti.y), C = ld3(S.pos, ti.z);
    float area = length(cross(B - A, C - A)) * 0.5f;
    float pdf = 1.0f / area;
    pdf /= (float)S.n_emissive;
    float cl = absr(dot(h.sn, -d));
    pdf *= h.dist * h.dist;
    pdf /= cl;
    return pdf;
}

#include "restir_di.h"

// Extended light sampling (ext_light): each light sample's contribution from its records and
// trace results, summed in sample order and divided by their count (sample_many_lights,
// Lights.h:222-241).
DEV Col ext_resolve(const DevScene& S, const DevPaths& P, const MptFrame& F, int slot, int lssb) {
    const MptRenderSettings& rs = F.render_settings;
    const int nl = rs.ris_number_of_light_candidates, nbc = rs.ris_number_of_bsdf_candidates;
    const bool vis = F.options.ris_use_visibility != 0;
    const size_t base = (size_t)slot * P.x_per;
    Col dl = col(0.0f);
    for (int it = 0; it < rs.number_of_light_samples; it++) {
        const size_t e0 = base + (size_t)it * P.x_iter;
        Col ld = col(0.0f);
        if (lssb == MPT_LSS_UNIFORM_ONE_LIGHT || lssb == MPT_LSS_MIS_LIGHT_BSDF) {
            Col lrad = col(0.0f), brad = col(0.0f);
            if ((P.xq_flag[e0] & XQ_ANY) && !P.xq_occ[e0]) { const float4 a = P.xrec[2 * e0]; lrad = col(a.x, a.y, a.z); }
            if (lssb == MPT_LSS_MIS_LIGHT_BSDF && (P.xq_flag[e0 + 1] & XQ_CL)) {
                const size_t e = e0 + 1;
                ShadowLightHit sh;
                if (shadow_light_hit(S, P.xq_hit[e], sh) && !is_black(sh.em)) {
                    const float4 a = P.xrec[2 * e], b = P.xrec[2 * e + 1], d = P.xq_d[e];
                    const float lp2 = pdf_emissive_hit(S, sh, mk3(d.x, d.y, d.z));
                    brad = col(a.x, a.y, a.z) * b.x * sh.em * balance(a.w, lp2) / a.w;
                }
            }
            ld = lrad + brad;
        } else if (lssb == MPT_LSS_BSDF) {
            if (P.xq_flag[e0] & XQ_CL) {
                ShadowLightHit sh;
                if (shadow_light_hit(S, P.xq_hit[e0], sh) && !is_black(sh.em)) {
                    const float4 a = P.xrec[2 * e0], b = P.xrec[2 * e0 + 1];
                    ld = col(a.x, a.y, a.z) * b.x * sh.em / a.w;
                }
            }
        } else {
            // the RIS reservoir (RIS.h:82-289, RISReservoir RIS_Reservoir.h:20-51): light
            // candidates (their visibility with the visibility target function), then the BSDF
            // candidates with their light-hit results, in the reference's order
            float wsum = 0.0f, tw = 0.0f;
            int win = -1;        // light candidate, or nl + BSDF candidate
            int win_tri = -1;
            for (int c = 0; c < nl; c++) {
                const float4 a = P.xrec[2 * (e0 + c)], b = P.xrec[2 * (e0 + c) + 1];
                float target = a.z, cw = 0.0f;
                if (b.y != 0.0f) {   // inner
                    if (vis && target > 0.0f) target *= P.xq_occ[e0 + c] ? 0.0f : 1.0f;
                    cw = a.x * target / a.y;
                }
                wsum += cw;
                if (b.x < cw / wsum) { win = c; tw = target; win_tri = __float_as_int(a.w); }
            }
            for (int k = 0; k < nbc; k++) {
                const size_t e = e0 + 2 * nl + k;
                const float4 b = P.xrec[2 * e + 1];
                float cw = 0.0f, target = 0.0f;
                int tri = -1;
                if (P.xq_flag[e] & XQ_CL) {
                    ShadowLightHit sh;
                    if (shadow_light_hit(S, P.xq_hit[e], sh) && !is_black(sh.em)) {
                        const float4 a = P.xrec[2 * e], d = P.xq_d[e];
                        const Col lc = col(a.x, a.y, a.z) * sh.em * b.x;
                        target = lum(lc);
                        float lpdf = pdf_emissive_hit(S, sh, mk3(d.x, d.y, d.z));
                        lpdf *= b.z != 0.0f ? 0.0f : 1.0f;
                        if (!min_contrib(rs.minimum_light_contribution, lc / lpdf / a.w)) target = 0.0f;
                        cw = balance(a.w, (float)nbc, lpdf, (float)nl) * target / a.w;
                        tri = sh.prim;
                    }
                }
                wsum += cw;
                if (b.y < cw / wsum) { win = nl + k; tw = target; win_tri = tri; }
            }
            // RISReservoir::end + evaluate_reservoir_sample (RIS.h:18-80)
            const float ucw = wsum == 0.0f ? 0.0f : 1.0f / tw * wsum;
            if (ucw > 0.0f && win >= 0) {
                if (win >= nl) {
                    const size_t e = e0 + 2 * nl + (win - nl);
                    const float4 a = P.xrec[2 * e], b = P.xrec[2 * e + 1];
                    if (b.x > 0.0f) ld = col(a.x, a.y, a.z) * ucw * emission_of(S.mats[S.mat_idx[win_tri]]) * b.x;
                } else {
                    const size_t ew = e0 + nl + win;
                    // the final shadow ray: its own (inside / without the visibility target
                    // function), else the candidate's visibility ray
                    const bool occ = (P.xq_flag[ew] & XQ_ANY) ? P.xq_occ[ew] != 0 : P.xq_occ[e0 + win] != 0;
                    const float4 a = P.xrec[2 * ew];
                    if (!occ && a.w > 0.0f) ld = col(a.x, a.y, a.z) * ucw * emission_of(S.mats[S.mat_idx[win_tri]]) * a.w;
                }
            }
        }
        dl += ld;
    }
    return dl / (float)rs.number_of_light_samples;
}

// one entry of the bounce's shaded list
template <bool EXT>
DEV void resolve_entry(const DevScene& S, const DevPaths& P, const MptFrame& F, int bounce, int nh, int i) {
    const MptRenderSettings& rs = F.render_settings;
    const int slot = shaded_entry(P, nh, i);
    if (slot < 0) return;   // deferred to the generic shading list
    // the NEE record planes the vertex wrote (flags in nthr.w), each read whole
    const float4 t4 = ld_s(&P.nthr[slot]);
    const uint32_t fl = __float_as_uint(t4.w);
    // the bounce pipeline's col addition of the shading (P.ce), made here in the shading's place
    float4 cv = ld_s(&P.col[slot]);
    if (P.ce) {
        const float4 e = ld_s(&P.ce[slot]);
        const Col s = col(cv.x, cv.y, cv.z) + col(e.x, e.y, e.z);
        cv = make_float4(s.r, s.g, s.b, 0.0f);
    }
    if (!(fl & NF_SHADED) || (fl & NF_NOADD)) {
        if (P.ce) st_s(&P.col[slot], cv);
        return;
    }
    const int lss = F.options.direct_light_sampling;
    const int lssb = bounce_lss(F, bounce);
    Col ld = col(0.0f), ed = col(0.0f);
    auto occ = [&](int k) { return ld_s(&P.occ[(size_t)k * (size_t)P.nq_stride + (size_t)slot]) != 0; };
    if (fl & NF_IMM) { const float4 a = ld_s(&P.na[slot]); ld = col(a.x, a.y, a.z); }
    else if (!(fl & NF_L)) ld = col(0.0f);
    else if (EXT && (fl & NF_EXT)) ld = ext_resolve(S, P, F, slot, lssb);   // already / number_of_light_samples
    else if (lss == MPT_LSS_RESTIR_DI && bounce == 0) {
        if ((fl & NF_A) && !((fl & NF_AQ) && occ(0))) { const float4 a = ld_s(&P.na[slot]); ld = col(a.x, a.y, a.z); }
    } else if (lssb == MPT_LSS_RIS_BSDF_AND_LIGHT) {
        const float4 ris = ld_s(&P.nris[slot]);
        float wsum = ris.x;
        float cwb = 0.0f, targetb = 0.0f;
        int trib = -1;
        float4 b = make_float4(0.0f, 0.0f, 0.0f, 0.0f), dr = b;
        if (fl & NF_B) {
            b = ld_s(&P.nb[slot]);
            dr = ld_s(&P.ndir[slot]);
            ShadowLightHit sh;
            if (shadow_light_hit(S, ld_s(&P.nhit[slot]), sh) && !is_black(sh.em)) {
                Col lc = col(b.x, b.y, b.z) * sh.em * dr.w;
                targetb = lum(lc);
                float lpdf = pdf_emissive_hit(S, sh, mk3(dr.x, dr.y, dr.z));
                lpdf *= (fl & NF_B_REFR) ? 0.0f : 1.0f;
                if (!min_contrib(rs.minimum_light_contribution, lc / lpdf / b.w)) targetb = 0.0f;
                float w = balance(b.w, (float)rs.ris_number_of_bsdf_candidates, lpdf, (float)rs.ris_number_of_light_candidates);
                cwb = w * targetb / b.w;
                trib = sh.prim;
            }
        }
        bool bsdf_wins = false;
        if (rs.ris_number_of_bsdf_candidates > 0) {
            wsum += cwb;
            bsdf_wins = ris.z < cwb / wsum;
        }
        // RISReservoir::end (RIS_Reservoir.h:45-51); wsum > 0 implies a winner exists
        float target = bsdf_wins ? targetb : ((fl & NF_RIS_W) ? ris.y : 0.0f);
        float ucw = wsum == 0.0f ? 0.0f : 1.0f / target * wsum;
        if (ucw > 0.0f) {
            if (bsdf_wins) {
                float c = dr.w;
                if (c > 0.0f) ld = col(b.x, b.y, b.z) * ucw * emission_of(S.mats[S.mat_idx[trib]]) * c;
            } else if (!occ(0)) {
                const float4 a = ld_s(&P.na[slot]);
                float c = a.w;
                if (c > 0.0f) ld = col(a.x, a.y, a.z) * ucw * emission_of(S.mats[S.mat_idx[__float_as_int(ris.w)]]) * c;
            }
        }
    } else if (lssb == MPT_LSS_MIS_LIGHT_BSDF) {
        Col lrad = col(0.0f), brad = col(0.0f);
        if ((fl & NF_A) && !occ(0)) { const float4 a = ld_s(&P.na[slot]); lrad = col(a.x, a.y, a.z); }
        if (fl & NF_B) {
            ShadowLightHit sh;
            if (shadow_light_hit(S, ld_s(&P.nhit[slot]), sh) && !is_black(sh.em)) {
                const float4 b = ld_s(&P.nb[slot]), dr = ld_s(&P.ndir[slot]);
                float lp2 = pdf_emissive_hit(S, sh, mk3(dr.x, dr.y, dr.z));
                float w = balance(b.w, lp2);
                brad = col(b.x, b.y, b.z) * dr.w * sh.em * w / b.w;
            }
        }
        ld = lrad + brad;
    } else if (lssb == MPT_LSS_UNIFORM_ONE_LIGHT) {
        if ((fl & NF_A) && !occ(0)) { const float4 a = ld_s(&P.na[slot]); ld = col(a.x, a.y, a.z); }
    } else if (lssb == MPT_LSS_BSDF) {
        if (fl & NF_B) {
            ShadowLightHit sh;
            if (shadow_light_hit(S, ld_s(&P.nhit[slot]), sh) && !is_black(sh.em)) {
                const float4 b = ld_s(&P.nb[slot]), dr = ld_s(&P.ndir[slot]);
                ld = col(b.x, b.y, b.z) * dr.w * sh.em / b.w;
            }
        }
    }
    // sample_many_lights: / number_of_light_samples (1 outside extended light sampling); not the
    // ReSTIR DI reservoir of bounce 0 (sample_one_light_ReSTIR_DI, Lights.h:243-275)
    if ((fl & NF_L) && !(fl & NF_IMM) && !(EXT && (fl & NF_EXT)) && !(lss == MPT_LSS_RESTIR_DI && bounce == 0))
        ld = ld / (float)rs.number_of_light_samples;
    {
        Col e2 = col(0.0f), e1 = col(0.0f);
        if ((fl & NF_E2) && !occ(2)) { const float4 e = ld_s(&P.ne2[slot]); e2 = col(e.x, e.y, e.z); }
        if ((fl & NF_E1) && !occ(1)) { const float4 e = ld_s(&P.ne1[slot]); e1 = col(e.x, e.y, e.z); }
        ed = e2 + e1;
    }
    ld = clamp_contrib(ld, rs.direct_contribution_clamp, bounce == 0);
    ed = clamp_contrib(ed, rs.envmap_contribution_clamp, bounce == 0);
    Col ind = (ld + ed) * col(t4.x, t4.y, t4.z);
    Col rc = col(cv.x, cv.y, cv.z) + clamp_contrib(ind, rs.indirect_contribution_clamp, bounce > 0);
    st_s(&P.col[slot], make_float4(rc.r, rc.g, rc.b, 0.0f));
#ifdef MPT_DEBUG_SLOT
    if (slot == MPT_DEBUG_SLOT) { Col t_ = col(t4.x, t4.y, t4.z); printf("GPU b%d ld %a %a %a ed %a %a %a thr %a %a %a rc %a %a %a\n", bounce, ld.r, ld.g, ld.b, ed.r, ed.g, ed.b, t_.r, t_.g, t_.b, rc.r, rc.g, rc.b); }
#endif
}

// over the bounce's shaded list (grid-stride: the grid is sized for the wavefront, the list
// shrinks bounce by bounce); count_paths: the bounce's path rays
template <bool EXT>
__global__ __launch_bounds__(TB) void k_resolve(DevScene S, DevPaths P, const MptFrame* __restrict__ Fp, int bounce,
                                                const int32_t* count_paths) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // always-on ray accounting: path rays + NEE any-hit + NEE closest of this bounce, path hits
        // (atomic: the two halves of an overlapped batch resolve concurrently)
        // (the path rays, *count_paths, are counted by k_split: a pipelined bounce's split zeroes
        // the previous bounce's queue counter while this resolve may still run)
        unsigned long long* rc = (unsigned long long*)P.ray_counts;
        (void)count_paths;
        atomicAdd(rc + 1, (unsigned long long)P.counters[CTR_ANY] + (EXT ? (unsigned long long)P.counters[CTR_XANY] : 0ull));
        atomicAdd(rc + 2, (unsigned long long)P.counters[CTR_CL] + (EXT ? (unsigned long long)P.counters[CTR_XCL] : 0ull));
        atomicAdd(rc + 3, (unsigned long long)(shaded_count(P) - P.counters[CTR_DEFER]));
        atomicAdd(rc + 4, (unsigned long long)(P.counters[CTR_FULL] + P.counters[CTR_GLASS]));
    }
    const int nh = P.counters[CTR_HIT];
    const int total = shaded_count(P);
    for (int i = blockIdx.x * TB + threadIdx.x; i < total; i += gridDim.x * TB) resolve_entry<EXT>(S, P, *Fp, bounce, nh, i);
}

// ----------------------------------------------------------------------------------
// k_accumulate (FullPathTracer.h:292-327)
// ----------------------------------------------------------------------------------
// the pixel's framebuffer values, held in registers over the samples of a batch
struct PixAcc {
    Col c;
    v3 a, n;
    float sq;
};
DEV void accumulate_sample(const DevPaths& P, const MptRenderSettings& rs, int slot, PixAcc& f, bool& any) {
    if (!P.active[slot]) return;          // FullPathTracer.h:114-115
    float4 cv = P.col[slot];
    Col c = col(cv.x, cv.y, cv.z);
    float wl = __uint_as_float(P.vsB[slot].w);
    bool invalid = false;
    if (wl == 0.0f) invalid |= (c.r < 0 || c.g < 0 || c.b < 0);
    invalid |= has_nan(c);
    if (invalid) {
        if (rs.display_NaNs) {
            Col dc = col(1.0e30f, 0.0f, 1.0e30f);
            if (rs.sample_number != 0) dc = dc * (float)rs.sample_number;
            f.c = dc;
        }
        return;
    }
    any = true;                           // still_one_ray_active (FullPathTracer.h:299)
    if (has_adaptive_buffers(rs)) {
        float l = lum(c);
        f.sq += l * l;
    }
    if (rs.sample_number == 0) f.c = c;
    else { f.c.r += c.r; f.c.g += c.g; f.c.b += c.b; }
    float cnt = (float)rs.denoiser_AOV_accumulation_counter;
    float4 a = P.alb[slot], n = P.nrm[slot];
    if (rs.sample_number == 0) {
        f.a = mk3(a.x, a.y, a.z);
        f.n = mk3(n.x, n.y, n.z);
    } else {
        f.a.x = (f.a.x * cnt + a.x) / (cnt + 1.0f);
        f.a.y = (f.a.y * cnt + a.y) / (cnt + 1.0f);
        f.a.z = (f.a.z * cnt + a.z) / (cnt + 1.0f);
        v3 acc = (f.n * cnt + mk3(n.x, n.y, n.z)) / (cnt + 1.0f);
        float len = length(acc);
        if (!is_zero(len)) f.n = acc / len;
    }
}
// one pixel per lane; the samples of a batch are added in sample order, exactly as
// consecutive single-sample frames would add them, on register copies of the pixel's
// framebuffer values (read once, written once per launch); the still-active flag is
// written once per wave instead of once per path
#ifndef MPT_TU_PART   // k_accumulate
// Speculative batched adaptive sampling (P.spec_as): every sample of the batch was traced, and
// here each sample meets CameraRays' reset and gate (CameraRays.h:78-125) on the pixel's
// running values -- those of the samples before it -- exactly when the sequential frames
// would: a sample the gate refuses rescales the sum and is dropped, a needed one is counted
// and added.  The gate reads nothing a later sample changes, so the sums, counts and status
// values equal one frame per sample.
__global__ __launch_bounds__(TB) void k_accumulate(DevPaths P, const MptFrame* __restrict__ Fp) {
    const int pixel = blockIdx.x * TB + threadIdx.x;
    bool any = false;
    uint32_t n_conv = 0u;
    if (pixel < P.n_pix) {
        float* fb = P.fb_color + 3 * (size_t)pixel;
        float* fa = P.fb_albedo + 3 * (size_t)pixel;
        float* fn = P.fb_normal + 3 * (size_t)pixel;
        PixAcc f;
        f.c = col(fb[0], fb[1], fb[2]);
        f.a = mk3(fa[0], fa[1], fa[2]);
        f.n = mk3(fn[0], fn[1], fn[2]);
        bool adaptive = false;
        for (int sub = 0; sub < P.batch; sub++) adaptive |= has_adaptive_buffers(Fp[sub].render_settings);
        f.sq = adaptive ? P.as_sqlum[pixel] : 0.0f;
        if (P.spec_as) {
            int cnt = P.as_count[pixel], conv = P.as_conv[pixel];
            for (int sub = 0; sub < P.batch; sub++) {
                const MptRenderSettings& rs = Fp[sub].render_settings;
                if (has_adaptive_buffers(rs)) {
                    if (rs.sample_number == 0 || rs.need_to_reset) { cnt = 0; f.sq = 0.0f; conv = -1; }
                    bool converged = false;
                    const bool needed = adaptive_gate(rs, f.c, f.sq, cnt, conv, converged);
                    if ((converged || !needed) && rs.do_update_status_buffers) n_conv++;
                    if (!needed) {
                        f.c = f.c / (float)rs.sample_number * (float)(rs.sample_number + 1);
                        continue;
                    }
                    cnt++;
                }
                if (rs.do_update_status_buffers) any = true;   // CameraRays.h:171-177
                accumulate_sample(P, rs, batch_slot(P, pixel, sub), f, any);
            }
            P.as_count[pixel] = cnt;
            P.as_conv[pixel] = conv;
        } else {
            for (int sub = 0; sub < P.batch; sub++) accumulate_sample(P, Fp[sub].render_settings, batch_slot(P, pixel, sub), f, any);
        }
        fb[0] = f.c.r; fb[1] = f.c.g; fb[2] = f.c.b;
        fa[0] = f.a.x; fa[1] = f.a.y; fa[2] = f.a.z;
        fn[0] = f.n.x; fn[1] = f.n.y; fn[2] = f.n.z;
        if (adaptive) P.as_sqlum[pixel] = f.sq;
    }
    if (__ballot(any) != 0ull && lane_id() == 0) P.status[1] = 1u;
    if (P.spec_as) {
        // the converged-pixel counter: one atomic per wave
        for (int off = 32; off > 0; off >>= 1) n_conv += __shfl_xor(n_conv, off);
        if (lane_id() == 0 && n_conv) atomicAdd(&P.status[0], n_conv);
    }
}

#endif
// k_shade and the ReSTIR DI reuse kernels are instantiated in their own translation units
// (mpt_part.hip, compiled once per MPT_TU_PART value) so that the build compiles them in
// parallel; these launch them.
void part_shade_generic(dim3 g, hipStream_t st, const ShadeArgs& a);          // k_shade<NONE, false>
void part_shade_plain(dim3 g, hipStream_t st, const ShadeArgs& a);            // k_shade<NONE, true>
void part_shade_glass(dim3 g, hipStream_t st, const ShadeArgs& a);            // k_shade<NONE, false, false, true>
void part_shade_plain_stage(int stage, dim3 g, hipStream_t st, const ShadeArgs& a);   // k_shade<NONE, true, false, false, stage>
void part_shade_ext(dim3 g, hipStream_t st, const ShadeArgs& a);              // k_shade<NONE, false, true>
void part_shade_override(int ovr, bool ext, dim3 g, hipStream_t st, const ShadeArgs& a);   // Lambert, Oren-Nayar
enum RestirKernel { RK_INITIAL, RK_SPATIOTEMPORAL, RK_SPATIOTEMPORAL_ANY, RK_SPATIAL, RK_SPATIAL_ANY, RK_TEMPORAL, RK_SP_SELECT,
                   RK_SP_EVAL_PLAIN, RK_SP_EVAL_GENERIC, RK_SP_COMBINE, RK_INITIAL_STAGED_PLAIN, RK_INITIAL_STAGED_GENERIC,
                   RK_ST_SELECT, RK_ST_EVAL_PLAIN, RK_ST_EVAL_GENERIC, RK_ST_COMBINE };
void part_restir_principled(int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P, const MptFrame* F,
                            int pass, const float4* in, float4* out);
void part_restir_override(int ovr, int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P,
                          const MptFrame* F, int pass, const float4* in, float4* out);
#ifndef MPT_TU_PART   // host launch glue and the remaining kernels: main translation unit only
// ----------------------------------------------------------------------------------
// host launch glue
// ----------------------------------------------------------------------------------
static int blocks_for(int n) { return (n + TB - 1) / TB; }

// adds a device list length to a 64-bit statistics counter (units of a timed kernel)
__global__ void k_count_add64(uint64_t* dst, const int32_t* src) {
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)dst, (unsigned long long)(uint32_t)*src);
}

static void launch_restir_kernel(int ovr, int kind, dim3 g, hipStream_t st, const DevScene& S, const DevPaths& P,
                                 const MptFrame* F, int pass = 0, const float4* in = nullptr, float4* out = nullptr) {
    if (ovr == MPT_BSDF_NONE) part_restir_principled(kind, g, st, S, P, F, pass, in, out);
    else part_restir_override(ovr, kind, g, st, S, P, F, pass, in, out);
}

template <int MODE>
static void launch_trace_mode(const TraceArgs& a, int grid, bool stats, hipStream_t st) {
    if (MODE == TM_NEE_LIGHT && a.static_grid && !stats) grid = blocks_for(a.P.n);   // the query list holds at most n entries
    // the persistent grid is MPT_TRACE_BLOCKS_PER_CU blocks per CU (one 4-wave block per SIMD and
    // wave); the list modes fill their own occupancy.  The spill area holds
    // TRACE_SPILL_BLOCKS_PER_CU blocks per CU (mpt_internal.h), which covers both grids
    if (MODE == TM_LIST_ANY || MODE == TM_LIST_CLOSEST) grid = grid / MPT_TRACE_WAVES * MPT_TRACE_WAVES_LIST;
    if (stats) {
        // instrumented (calibration) launches stay persistent: their per-wave counter atomics
        // over a static grid of ~500 k waves would serialise the launch
        TraceArgs b = a;
        b.static_grid = 0;
        hipLaunchKernelGGL((k_trace<MODE, true>), dim3(grid), dim3(TB), 0, st, b);
    }
    else hipLaunchKernelGGL((k_trace<MODE, false>), dim3(grid), dim3(TB), 0, st, a);
}

// event pair around a non-traversal kernel (KT_* id), when timing is enabled
// (the pair is reserved at construction, so scopes may nest: the ReSTIR DI span and its kernels)
struct TimedScope {
    LaunchCfg& cfg;
    hipStream_t st;
    int idx;
    TimedScope(LaunchCfg& c, hipStream_t s, int kind) : cfg(c), st(s), idx(-1) {
        if (c.ev_pool && c.ev_used + 2 <= c.ev_cap) {
            idx = cfg.ev_used;
            cfg.ev_used += 2;
            cfg.ev_mode[idx / 2] = kind;
            hipEventRecord(cfg.ev_pool[idx], st);
        }
    }
    ~TimedScope() {
        if (idx >= 0) hipEventRecord(cfg.ev_pool[idx + 1], st);
    }
};

template <int MODE>
static void timed_trace(const TraceArgs& a, LaunchCfg& cfg, hipStream_t st) {
    bool timed = cfg.ev_pool && cfg.ev_used + 2 <= cfg.ev_cap;
    if (timed) { cfg.ev_mode[cfg.ev_used / 2] = trace_stage(MODE); hipEventRecord(cfg.ev_pool[cfg.ev_used], st); }
    launch_trace_mode<MODE>(a, cfg.grid_persistent, cfg.stats, st);
    if (timed) { hipEventRecord(cfg.ev_pool[cfg.ev_used + 1], st); cfg.ev_used += 2; }
    cfg.launches++;
}

// restir_output_reservoirs of a frame, as a code kept by the context between frames
static float4* restir_buffer(const DevPaths& P, int code) { return code == 1 ? P.rs_sp2 : code == 2 ? P.rs_init : P.rs_sp1; }
static int restir_code(const DevPaths& P, const float4* b) { return b == P.rs_sp2 ? 1 : b == P.rs_init ? 2 : 0; }

// Halo exchange of a partitioned context (mpt.h MptHaloExchange): the host fills the rows
// around the band from the contexts that own them.  No-op for a whole-frame context.
static int halo_exchange(const MptFrame& hf, LaunchCfg& cfg, hipStream_t st, int phase, int pass, int halo,
                         std::initializer_list<std::pair<void*, int64_t>> bufs, bool agreed = false) {
    if (!cfg.halo_fn || cfg.halo_rc) return halo;
    MptHaloExchange x{};
    x.halo_agreed = agreed ? 1 : 0;
    x.phase = phase;
    x.pass = pass;
    x.res_x = hf.res_x;
    x.res_y = hf.res_y;
    x.own_y0 = cfg.own_y0;
    x.own_y1 = cfg.own_y1;
    x.halo_rows = halo;
    for (const auto& b : bufs) {
        if (!b.first || x.n_buffers >= MPT_HALO_MAX_BUFFERS) continue;
        x.buffers[x.n_buffers] = b.first;
        x.bytes_per_pixel[x.n_buffers] = b.second;
        x.n_buffers++;
    }
    x.stream = (void*)st;
    cfg.halo_rc = cfg.halo_fn(cfg.halo_user, &x);
    return x.halo_rows;
}

// The generic-class kernel of a staged stage on the side stream (LaunchCfg::side_stream), forked
// from `st` here and joined by side_end; the side kernels take their own traversal spill area
static hipStream_t side_begin(LaunchCfg& cfg, hipStream_t st, DevPaths& PS) {
    if (!cfg.side_stream) return st;
    hipEventRecord(cfg.ev_side_fork, st);
    hipStreamWaitEvent(cfg.side_stream, cfg.ev_side_fork, 0);
    PS.stack_spill = cfg.side_spill;
    return cfg.side_stream;
}
static void side_end(LaunchCfg& cfg, hipStream_t st) {
    if (!cfg.side_stream) return;
    hipEventRecord(cfg.ev_side_join, cfg.side_stream);
    hipStreamWaitEvent(st, cfg.ev_side_join, 0);
}

// One spatial reuse pass: staged (selection, class-sorted target evaluations, traced rays,
// combine, visibility reuse; restir_di.h) when the reference-default weights are selected and the neighbour counts fit
// RS_KMAX, else the monolithic kernel.
static void launch_spatial_pass(int ovr, bool def_bias, const MptFrame& hf, LaunchCfg& cfg, dim3 g, hipStream_t st,
                                const DevScene& S, const DevPaths& P, const MptFrame* d_frame, int pass, const float4* in,
                                float4* out) {
    const MptReSTIRDISettings& rd = hf.render_settings.restir_di_settings;
    const bool staged = def_bias && cfg.restir_staged && !cfg.restir_mono_reuse && P.rq_o && rd.reuse_neighbor_count <= RS_KMAX &&
                        (!rd.do_disocclusion_reuse_boost || rd.disocclusion_reuse_count <= RS_KMAX);
    if (!staged) {
        launch_restir_kernel(ovr, def_bias ? RK_SPATIAL : RK_SPATIAL_ANY, g, st, S, P, d_frame, pass, in, out);
        return;
    }
    const dim3 gp(blocks_for(P.n));
    hipMemsetAsync(&P.counters[CTR_RQ], 0, CTR_RQ_GROUP * sizeof(int32_t), st);   // the lists + their work counters
    launch_restir_kernel(ovr, RK_SP_SELECT, gp, st, S, P, d_frame, pass, in, out);
    {
        DevPaths PS = P;
        const hipStream_t ss = side_begin(cfg, st, PS);
        launch_restir_kernel(ovr, RK_SP_EVAL_GENERIC, g, ss, S, PS, d_frame, pass, in, out);
        {
            TimedScope te(cfg, st, KT_RS_EVAL);
            launch_restir_kernel(ovr, RK_SP_EVAL_PLAIN, g, st, S, P, d_frame, pass, in, out);
        }
        side_end(cfg, st);
    }
    TraceArgs ta{};
    ta.S = S; ta.P = P; ta.queue = P.rq_list; ta.count_ptr = &P.counters[CTR_RQ]; ta.fetch = &P.counters[CTR_F_RQA];
    ta.raw_o = P.rq_o; ta.raw_d = P.rq_d; ta.raw_key = P.rq_key; ta.raw_occ = P.rq_occ;
    ta.F = d_frame; ta.alpha = hf.render_settings.do_alpha_testing ? 1 : 0;
    launch_trace_mode<TM_LIST_ANY>(ta, cfg.grid_persistent, cfg.stats, st);
    launch_restir_kernel(ovr, RK_SP_COMBINE, gp, st, S, P, d_frame, pass, in, out);
    ta.count_ptr = &P.counters[CTR_RQV];
    ta.fetch = &P.counters[CTR_F_RQB];
    launch_trace_mode<TM_LIST_ANY>(ta, cfg.grid_persistent, cfg.stats, st);
    hipLaunchKernelGGL(k_rs_visapply, gp, dim3(TB), 0, st, P, out);
}

// The fused spatiotemporal pass: staged (k_rst_select, class-sorted evaluations, traced rays,
// k_rst_combine, visibility reuse; restir_di.h) under the same conditions as a spatial pass and
// no temporal-buffer clear this frame, else the monolithic kernel.
static void launch_fused_pass(int ovr, bool def_bias, const MptFrame& hf, LaunchCfg& cfg, dim3 g, hipStream_t st,
                              const DevScene& S, const DevPaths& P, const MptFrame* d_frame) {
    const MptReSTIRDISettings& rd = hf.render_settings.restir_di_settings;
    const bool staged = def_bias && cfg.restir_staged && !cfg.restir_mono_reuse && P.rq_o && rd.reuse_neighbor_count <= RS_KMAX &&
                        (!rd.do_disocclusion_reuse_boost || rd.disocclusion_reuse_count <= RS_KMAX) &&
                        !rd.temporal_buffer_clear_requested;
    if (!staged) {
        launch_restir_kernel(ovr, def_bias ? RK_SPATIOTEMPORAL : RK_SPATIOTEMPORAL_ANY, g, st, S, P, d_frame);
        return;
    }
    const dim3 gp(blocks_for(P.n));
    hipMemsetAsync(&P.counters[CTR_RQ], 0, CTR_RQ_GROUP * sizeof(int32_t), st);   // the lists + their work counters
    launch_restir_kernel(ovr, RK_ST_SELECT, gp, st, S, P, d_frame);
    {
        DevPaths PS = P;
        const hipStream_t ss = side_begin(cfg, st, PS);
        launch_restir_kernel(ovr, RK_ST_EVAL_GENERIC, g, ss, S, PS, d_frame);
        {
            TimedScope te(cfg, st, KT_RS_EVAL);
            launch_restir_kernel(ovr, RK_ST_EVAL_PLAIN, g, st, S, P, d_frame);
        }
        side_end(cfg, st);
    }
    TraceArgs ta{};
    ta.S = S; ta.P = P; ta.queue = P.rq_list; ta.count_ptr = &P.counters[CTR_RQ]; ta.fetch = &P.counters[CTR_F_RQA];
    ta.raw_o = P.rq_o; ta.raw_d = P.rq_d; ta.raw_key = P.rq_key; ta.raw_occ = P.rq_occ;
    ta.F = d_frame; ta.alpha = hf.render_settings.do_alpha_testing ? 1 : 0;
    launch_trace_mode<TM_LIST_ANY>(ta, cfg.grid_persistent, cfg.stats, st);
    launch_restir_kernel(ovr, RK_ST_COMBINE, gp, st, S, P, d_frame);
    ta.count_ptr = &P.counters[CTR_RQV];
    ta.fetch = &P.counters[CTR_F_RQB];
    launch_trace_mode<TM_LIST_ANY>(ta, cfg.grid_persistent, cfg.stats, st);
    hipLaunchKernelGGL(k_rs_visapply, gp, dim3(TB), 0, st, P, P.rs_out);
}

// The G-buffer halo exchange of a partitioned context (and, when the agreed halo grew, the
// previous frame's rows frame_begin did not maintain); sets cfg.halo_rows.
static void exchange_gbuffers(const MptFrame& hf, LaunchCfg& cfg, hipStream_t st, const DevPaths& P, int need,
                              bool agreed = false) {
    const bool as = hf.render_settings.enable_adaptive_sampling;
    const int64_t MS = sizeof(MptMaterial);
    cfg.halo_rows = halo_exchange(hf, cfg, st, MPT_HALO_GBUFFER, 0, need,
                                  {{P.gb_pos, 16}, {P.gb_sn, 16}, {P.gb_gn, 16}, {P.gb_view, 16}, {P.gb_meta, 16},
                                   {P.gb_vsA, 16}, {P.gb_vsB, 16}, {P.gb_mat, MS}, {as ? P.rs_conv : nullptr, 4},
                                   {MPT_RESTIR_CS ? P.gb_cs : nullptr, 64}}, agreed);
    if (cfg.halo_rows > cfg.halo_prev)   // rows frame_begin did not maintain last frame
        halo_exchange(hf, cfg, st, MPT_HALO_PREV_GBUFFER, 0, cfg.halo_rows,
                      {{P.pgb_pos, 16}, {P.pgb_sn, 16}, {P.pgb_gn, 16}, {P.pgb_view, 16}, {P.pgb_meta, 16},
                       {P.pgb_vsA, 16}, {P.pgb_vsB, 16}, {P.pgb_mat, MS}, {MPT_RESTIR_CS ? P.pgb_cs : nullptr, 64}});
}

// A partitioned context whose band holds no row (more contexts than rows): nothing to render,
// but the other bands' exchanges pair with its own, so it makes the calls launch_restir makes,
// in the same order (G-buffer, then the reservoirs each reuse pass reads), with its buffers.
static void restir_empty_band(const MptFrame& hf, LaunchCfg& cfg, hipStream_t st, const DevPaths& P) {
    if (!cfg.halo_fn) return;
    const MptReSTIRDISettings& rd = hf.render_settings.restir_di_settings;
    const int64_t RB = 3 * sizeof(float4);
    const bool still = std::memcmp(&hf.current_camera, &hf.prev_camera, sizeof(MptCamera)) == 0;
    // the halo every context derives for a still camera (launch_restir)
    exchange_gbuffers(hf, cfg, st, P, still ? std::min(hf.res_y, 2 + std::max(0, rd.reuse_radius) +
                                                                   std::max(0, rd.neighbor_search_radius) + 8) : 0, still);
    if (rd.do_fused_spatiotemporal) {
        for (int pass = 0; pass < rd.number_of_passes; pass++)
            halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, pass, cfg.halo_rows, {{P.rs_sp1, RB}});
    } else {
        if (rd.do_temporal_reuse_pass) halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, 0, cfg.halo_rows, {{P.rs_sp1, RB}});
        if (rd.do_spatial_reuse_pass)
            for (int pass = 0; pass < rd.number_of_passes; pass++)
                halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, pass + 1, cfg.halo_rows, {{P.rs_sp1, RB}});
    }
    cfg.halo_prev = cfg.halo_rows;
}

// Lights presampling and initial candidates (ReSTIRDIRenderPass.cpp:241-247) into P.rs_init: one
// sample's, or a chunk's (DevPaths::ci_n: the chunk's planes, every item of every sample in each
// launch)
static void restir_initial(const DevScene& S, const DevPaths& P, const MptFrame* d_frame, const MptFrame& hf, LaunchCfg& cfg,
                          hipStream_t st) {
    const MptReSTIRDISettings& rd = hf.render_settings.restir_di_settings;
    const int ovr = hf.options.bsdf_override;
    const int n_pl = rd.number_of_subsets * rd.subset_size;
    const int n_smp = P.ci_n ? P.n / P.ci_n : 1;
    if (hf.options.restir_di_do_lights_presampling) {   // ReSTIRDIRenderPass::launch (.cpp:241-242)
        TimedScope tk(cfg, st, KT_RS_PRESAMPLE);
        hipLaunchKernelGGL(k_restir_presample, dim3((n_smp * n_pl + TB - 1) / TB), dim3(TB), 0, st, S, P, d_frame);
    }
    const dim3 g(cfg.grid_persistent);
    {
        TimedScope tk(cfg, st, KT_RS_INITIAL);
        // staged (the BSDF candidate's ray through k_trace<TM_LIST_CLOSEST>) for the reference
        // defaults: at most one BSDF candidate, no visibility in the initial target function
        const bool staged = cfg.restir_staged && P.rq_o && rd.number_of_initial_bsdf_candidates <= 1 &&
                            !hf.options.restir_di_initial_target_visibility;
        if (!staged) launch_restir_kernel(ovr, RK_INITIAL, g, st, S, P, d_frame);
        else {
            const dim3 gp(blocks_for(P.n));
            hipMemsetAsync(&P.counters[CTR_RQ], 0, CTR_RQ_GROUP * sizeof(int32_t), st);   // the lists + their work counters
            hipLaunchKernelGGL(k_rsi_classify, dim3((P.n + TB * RSI_PPT - 1) / (TB * RSI_PPT)), dim3(TB), 0, st, S, P, d_frame,
                               ovr == MPT_BSDF_NONE ? 1 : 0);
            {
                DevPaths PS = P;
                const hipStream_t ss = side_begin(cfg, st, PS);
                launch_restir_kernel(ovr, RK_INITIAL_STAGED_GENERIC, g, ss, S, PS, d_frame);
                launch_restir_kernel(ovr, RK_INITIAL_STAGED_PLAIN, g, st, S, P, d_frame);
                side_end(cfg, st);
            }
            TraceArgs ta{};
            ta.S = S; ta.P = P; ta.queue = P.rq_list; ta.count_ptr = &P.counters[CTR_RQ]; ta.fetch = &P.counters[CTR_F_RQA];
            ta.raw_o = P.rq_o; ta.raw_d = P.rq_d; ta.raw_key = P.rq_key; ta.raw_occ = P.rq_occ;
            ta.raw_hit = P.rq_o;   // each hit written over its own (already read) ray origin
            ta.F = d_frame; ta.alpha = hf.render_settings.do_alpha_testing ? 1 : 0;
            launch_trace_mode<TM_LIST_CLOSEST>(ta, cfg.grid_persistent, cfg.stats, st);
            hipLaunchKernelGGL(k_rsi_finish, dim3((P.n + TB * RSI_PPT - 1) / (TB * RSI_PPT)), dim3(TB), 0, st, S, P, d_frame);
            ta.count_ptr = &P.counters[CTR_RQV];
            ta.fetch = &P.counters[CTR_F_RQB];
            launch_trace_mode<TM_LIST_ANY>(ta, cfg.grid_persistent, cfg.stats, st);
            hipLaunchKernelGGL(k_rs_visapply, gp, dim3(TB), 0, st, P, P.rs_init);
        }
    }
}

// ReSTIRDIRenderPass::launch (ReSTIRDIRenderPass.cpp:233-264) for the fused configuration:
// presampling, initial candidates, fused spatiotemporal, (number_of_passes - 1) spatial
// passes ping-ponging between the two spatial buffers; returns the output buffer in P.rs_out.
// A partitioned context exchanges the halo of the G-buffer (after k_gbuffer) and of every
// reservoir buffer a reuse pass reads at neighbours: the temporal input right before the
// fused pass (so the final-shading write-through of the previous frame is included), then
// each pass's output before the next pass.
static void launch_restir(const DevScene& S, DevPaths& P, const MptFrame* d_frame, const MptFrame& hf, LaunchCfg& cfg,
                          hipStream_t st, bool initial_done = false) {
    TimedScope ts(cfg, st, KT_RESTIR);
    const MptReSTIRDISettings& rd = hf.render_settings.restir_di_settings;
    const int ovr = hf.options.bsdf_override;
    const int64_t RB = 3 * sizeof(float4);
    if (cfg.halo_fn) {
        // halo this context needs: its pixels' largest reprojection offset (measured by
        // k_gbuffer) + the reuse radius + the temporal search / permutation extent
        // (Utils.h:371-421); agreed over all contexts by the host's G-buffer exchange.  A frame
        // whose camera did not move reprojects every hit onto its own (jittered) pixel, an offset
        // of at most one row: every context then derives the same halo from the frame alone,
        // without reading the measure back (no host synchronisation per sample)
        const bool still = std::memcmp(&hf.current_camera, &hf.prev_camera, sizeof(MptCamera)) == 0;
        int reproj = 2;
        if (!still) {
            hipMemcpyAsync(cfg.h_reproj, &P.counters[CTR_REPROJ], sizeof(int32_t), hipMemcpyDeviceToHost, st);
            hipStreamSynchronize(st);
            reproj = *cfg.h_reproj;
        }
        const int need = std::min(hf.res_y, reproj + std::max(0, rd.reuse_radius) + std::max(0, rd.neighbor_search_radius) + 8);
        if (hf.render_settings.enable_adaptive_sampling)
            hipLaunchKernelGGL(k_restir_conv, dim3(blocks_for(P.n)), dim3(TB), 0, st, P);
        exchange_gbuffers(hf, cfg, st, P, need, still);
    }
    if (!initial_done) restir_initial(S, P, d_frame, hf, cfg, st);
    const dim3 g(cfg.grid_persistent);
    float4* last_out = restir_buffer(P, cfg.restir_out_sp2);
    // the reference-default weights run a kernel variant with the mode compiled in
    const bool def_bias = hf.options.restir_di_bias_correction_weights == MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE &&
                          hf.options.restir_di_bias_correction_use_visibility != 0;
    if (rd.do_fused_spatiotemporal) {
        P.rs_tin = last_out;
        P.rs_out = last_out == P.rs_sp1 ? P.rs_sp2 : P.rs_sp1;
        halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, 0, cfg.halo_rows, {{P.rs_tin, RB}});
        {
            TimedScope tk(cfg, st, KT_RS_REUSE);
            launch_fused_pass(ovr, def_bias, hf, cfg, g, st, S, P, d_frame);
        }
        for (int pass = 1; pass < rd.number_of_passes; pass++) {
            float4* in = P.rs_out;
            float4* out = in == P.rs_sp1 ? P.rs_sp2 : P.rs_sp1;
            halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, pass, cfg.halo_rows, {{in, RB}});
            TimedScope tk(cfg, st, KT_RS_SPATIAL);
            launch_spatial_pass(ovr, def_bias, hf, cfg, g, st, S, P, d_frame, pass, in, out);
            P.rs_out = out;
        }
    } else {
        // separate temporal and spatial passes (ReSTIRDIRenderPass::configure_temporal_pass /
        // configure_spatial_pass, ReSTIRDIRenderPass.cpp:332-418): the temporal pass writes
        // into the initial-candidates buffer when spatial passes follow (each pixel reads
        // only its own entry there), spatial pass 0 writes sp1, later passes ping-pong
        float4* cur = P.rs_init;
        if (rd.do_temporal_reuse_pass) {
            P.rs_tin = last_out;
            float4* tout = rd.do_spatial_reuse_pass ? P.rs_init : (last_out == P.rs_sp1 ? P.rs_sp2 : P.rs_sp1);
            halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, 0, cfg.halo_rows, {{P.rs_tin, RB}});
            TimedScope tk(cfg, st, KT_RS_REUSE);
            launch_restir_kernel(ovr, RK_TEMPORAL, g, st, S, P, d_frame, 0, P.rs_tin, tout);
            cur = tout;
        }
        if (rd.do_spatial_reuse_pass) {
            for (int pass = 0; pass < rd.number_of_passes; pass++) {
                float4* in = pass == 0 ? cur : ((pass & 1) ? P.rs_sp1 : P.rs_sp2);
                float4* out = pass == 0 ? P.rs_sp1 : ((pass & 1) ? P.rs_sp2 : P.rs_sp1);
                halo_exchange(hf, cfg, st, MPT_HALO_RESERVOIRS, pass + 1, cfg.halo_rows, {{in, RB}});
                TimedScope tk(cfg, st, KT_RS_SPATIAL);
                launch_spatial_pass(ovr, def_bias, hf, cfg, g, st, S, P, d_frame, pass, in, out);
                cur = out;
            }
        }
        P.rs_out = cur;   // configure_output_buffer (ReSTIRDIRenderPass.cpp:566-576)
    }
    cfg.restir_out_sp2 = restir_code(P, P.rs_out);
}

// CameraRays' G-buffer write and the ReSTIR DI passes of a frame (P.rs_out: their output)
// (k_restir_frame_begin, right before in the stream, zeroed the halo measure CTR_REPROJ)
static void restir_first_bounce(const DevScene& S, DevPaths& P, const MptFrame* d_frame, const MptFrame& hf, LaunchCfg& cfg,
                                hipStream_t st) {
    {
        TimedScope tk(cfg, st, KT_GBUFFER);
        hipLaunchKernelGGL(k_gbuffer, dim3(blocks_for(P.n)), dim3(TB), 0, st, S, P, d_frame);
    }
    launch_restir(S, P, d_frame, hf, cfg, st);
}

// Bounces [b_first, b_last] of the paths in q_cur (count counters[c_cur]): trace, G-buffer and
// ReSTIR DI passes (bounce 0 of a ReSTIR DI frame), split, shade, miss, compact into q_next,
// NEE rays, resolve.  Leaves the continuation list of the last bounce in the buffer passed
// as q_next for an odd number of bounces, as q_cur for an even one.
static void frame_bounces(const DevScene& S, DevPaths& P, const MptFrame* d_frame, const MptFrame& hf, LaunchCfg& cfg,
                          hipStream_t st, int b_first, int b_last, int32_t* q_cur, int c_cur, int32_t* q_next,
                          int c_next, bool first_traced = false, bool restir_done = false) {
    const int n = P.n;
    const bool restir = hf.options.direct_light_sampling == MPT_LSS_RESTIR_DI;
    const int nb = hf.render_settings.nb_bounces;
    // material classes (k_split / k_shade): Principled BSDF only (the Lambert override has one class)
    // extended light sampling (DevPaths::x_per > 0): the EXT shading / resolve kernels, one class
    const bool ext = P.x_per > 0;
    const int classes = (hf.options.bsdf_override != MPT_BSDF_NONE || ext) ? 0 : (cfg.shade_classes != 0 ? (cfg.shade_glass ? 2 : 1) : 0);
    // the next bounce's path rays on the trace-ahead stream (below); not while a ReSTIR DI first
    // bounce runs its G-buffer and reuse passes between the trace and the split (a batched ReSTIR
    // DI wavefront's later bounces, or its deferred first bounce after the passes, can)
    const bool ahead = cfg.ahead_stream != nullptr && (!restir || restir_done || b_first > 0);
    // Bounce pipeline (cfg.nee_stream): bounce b's NEE traversals and resolve run on the NEE stream
    // beside bounce b + 1's split and shading.  Odd bounces use the alternate plane set (NEE
    // records, staged queries and their lists, shaded lists, per-bounce counters, the shading's col
    // additions), so the two bounces in flight touch disjoint buffers; the path queues and their
    // counters (c_cur / c_next) are the base set's.  Bounce b + 1's k_miss (which adds to col)
    // waits for bounce b's resolve.  Not under ReSTIR DI, extended light sampling or split shading.
    const bool pipe = cfg.nee_stream != nullptr && cfg.pipe_alt != nullptr && !restir && !ext && !cfg.shade_split;
    DevPaths PB = P;   // the base set (even bounces)
    DevPaths* const Pout = &P;
    bool nee_pending = false;
    for (int b = b_first; b <= b_last; b++) {
        // this bounce's plane set; queue counters always from the base set
        DevPaths Pv = (pipe && (b & 1)) ? *cfg.pipe_alt : PB;
        if (pipe) Pv.ce = (b & 1) ? cfg.pipe_alt->ce : PB.ce;
        DevPaths& P = Pv;
        int32_t* const cnt_cur = &PB.counters[c_cur];
        int32_t* const cnt_next = &PB.counters[c_next];
        // every per-bounce counter (lists, class queues, the traversals' work counters) in one
        // memset; the next path queue's counter is zeroed by k_split
        hipMemsetAsync(&P.counters[CTR_BOUNCE_FIRST], 0, (CTR_COUNT - CTR_BOUNCE_FIRST) * sizeof(int32_t), st);
        // continuation / camera rays (first_traced: the first bounce's rays were traced already)
        const int alpha = hf.render_settings.do_alpha_testing ? 1 : 0;
        if (!(first_traced && b == b_first) && !(ahead && b > b_first)) {
            TraceArgs ta{};
            ta.S = S; ta.P = P; ta.queue = q_cur; ta.count_ptr = cnt_cur; ta.fetch = &P.counters[CTR_F_PATH];
            ta.F = d_frame; ta.bounce = b; ta.alpha = alpha;
            timed_trace<TM_PATH>(ta, cfg, st);
        }
        if (b == 0 && cfg.ev_first_trace) hipEventRecord(cfg.ev_first_trace, st);
        // (the ReSTIR DI passes use only CTR_REPROJ and their own CTR_RQ group of the per-bounce counters)
        if (restir && b == 0 && !restir_done) {
            restir_first_bounce(S, P, d_frame, hf, cfg, st);
            PB.rs_out = Pout->rs_out = P.rs_out;   // (the passes' output buffer, as the caller sees it)
        }
        const dim3 cp_grid((n + CP_NT * CP_ITEMS - 1) / (CP_NT * CP_ITEMS));
        {
            TimedScope ts(cfg, st, KT_SPLIT);
            hipLaunchKernelGGL(k_split, cp_grid, dim3(CP_NT), 0, st, S, P, q_cur, cnt_cur, classes, cnt_next);
        }
        ShadeArgs sa{};
        sa.S = S; sa.P = P; sa.F = d_frame; sa.bounce = b; sa.last_bounce = nb;
        sa.q_cur = P.qh; sa.count_cur = &P.counters[CTR_HIT]; sa.q_defer = P.qf; sa.count_defer = &P.counters[CTR_FULL];
        sa.force_defer = cfg.shade_classes == 2 ? 1 : 0;
        sa.mat_private = cfg.mat_private;
        {
            TimedScope ts(cfg, st, KT_SHADE);
            const dim3 sg(blocks_for(n));
            if (hf.options.bsdf_override != MPT_BSDF_NONE) part_shade_override(hf.options.bsdf_override, ext, sg, st, sa);
            else if (ext) part_shade_ext(sg, st, sa);
            else if (!classes) part_shade_generic(sg, st, sa);
            else if (cfg.shade_split) {
                // the plain class in stages (k_shade's ST); a stage whose groups have no work
                // in this bounce is not launched
                static const int splits[3][3] = {{SG_LIGHT, SG_ENV, SG_CONT}, {SG_LIGHT, SG_ENV | SG_CONT, 0},
                                                 {SG_LIGHT | SG_ENV, SG_CONT, 0}};
                const MptWorldSettings& ws = hf.world_settings;
                const bool env = ws.ambient_light_type == MPT_AMBIENT_ENVMAP && !hf.bsdf_flags.white_furnace_mode &&
                                 ws.envmap_intensity > 0.0f && hf.options.envmap_sampling != MPT_ESS_NO_SAMPLING &&
                                 !(hf.options.direct_light_sampling == MPT_LSS_RESTIR_DI && b == 0);
                const int work = SG_LIGHT | (env ? SG_ENV : 0) | (b < nb ? SG_CONT : 0);
                const int* sp = splits[std::min(std::max(cfg.shade_split, 1), 3) - 1];
                for (int k = 0; k < 3 && sp[k]; k++)
                    if (sp[k] & work) part_shade_plain_stage(sp[k], sg, st, sa);
            } else part_shade_plain(sg, st, sa);
        }
        if (classes) {
            TimedScope ts(cfg, st, KT_SHADE_GENERIC);
            ShadeArgs sf = sa;
            sf.q_cur = P.qf; sf.count_cur = &P.counters[CTR_FULL]; sf.q_defer = nullptr; sf.count_defer = nullptr;
            part_shade_generic(dim3(blocks_for(n)), st, sf);
            if (classes == 2) {   // the glass class, at the top of qf
                ShadeArgs sg2 = sf;
                sg2.q_cur = P.qf + P.n; sg2.count_cur = &P.counters[CTR_GLASS]; sg2.rev = 1;
                part_shade_glass(dim3(blocks_for(n)), st, sg2);
            }
        }
        // (the previous bounce's resolve adds to col first)
        if (nee_pending) { hipStreamWaitEvent(st, cfg.ev_nee_join, 0); nee_pending = false; }
        {
            TimedScope ts(cfg, st, KT_MISS);
            hipLaunchKernelGGL(k_miss, dim3(std::min(blocks_for(n), 8 * cfg.grid_persistent)), dim3(TB), 0, st, S, P, d_frame, b);
        }
        {
            TimedScope ts(cfg, st, KT_COMPACT);
            // the shaded list (qh ++ qf) holds up to 2n entries: deferred vertices appear in both
            const dim3 cp_grid2((2 * n + CP_NT * CP_ITEMS - 1) / (CP_NT * CP_ITEMS));
            // (the next bounce's plane set takes the next bounce's path-traversal work counter)
            int32_t* const next_fetch = (pipe && !(b & 1)) ? &cfg.pipe_alt->counters[CTR_F_PATH] : &PB.counters[CTR_F_PATH];
            hipLaunchKernelGGL(k_compact, classes ? cp_grid2 : cp_grid, dim3(CP_NT), 0, st, P, q_next, cnt_next,
                               ahead && b < b_last ? next_fetch : nullptr);
        }
        // Trace-ahead: the next bounce's path rays depend only on the continuation list k_compact
        // just wrote, not on this bounce's NEE queries or k_resolve (which read the NEE planes,
        // occlusion bytes and light hits, none of which the path traversal writes: it writes the
        // hits, hit classes and retrace origins of the continuation slots), so they are traced on
        // the trace-ahead stream beside this bounce's NEE traversals and resolve, with their own
        // traversal spill area; joined before the next bounce's split
        const bool fork = ahead && b < b_last;
        if (fork) {
            hipEventRecord(cfg.ev_ahead_fork, st);
            hipStreamWaitEvent(cfg.ahead_stream, cfg.ev_ahead_fork, 0);
            DevPaths PA = (pipe && !(b & 1)) ? *cfg.pipe_alt : PB;   // the next bounce's plane set
            PA.stack_spill = cfg.ahead_spill;
            TraceArgs ta{};
            ta.S = S; ta.P = PA; ta.queue = q_next; ta.count_ptr = cnt_next; ta.fetch = &PA.counters[CTR_F_PATH];
            ta.F = d_frame; ta.bounce = b + 1; ta.alpha = hf.render_settings.do_alpha_testing ? 1 : 0;
            timed_trace<TM_PATH>(ta, cfg, cfg.ahead_stream);
            hipEventRecord(cfg.ev_ahead_join, cfg.ahead_stream);
            cfg.ahead_launches++;
        }
        // NEE queries (each traversal with its own work counter, zeroed at the top of the bounce);
        // pipelined: on the NEE stream, with its own spill area
        const hipStream_t main_st = st;
        if (pipe) {
            hipEventRecord(cfg.ev_nee_fork, main_st);
            hipStreamWaitEvent(cfg.nee_stream, cfg.ev_nee_fork, 0);
            st = cfg.nee_stream;
            P.stack_spill = cfg.nee_spill;
        }
        TraceArgs tn{};
        tn.S = S; tn.P = P; tn.count_ptr = &P.counters[CTR_ANY]; tn.fetch = &P.counters[CTR_F_ANY];
        tn.F = d_frame; tn.bounce = b; tn.alpha = alpha;
        timed_trace<TM_NEE_ANY>(tn, cfg, st);
        tn.fetch = &P.counters[CTR_F_CL];
        tn.count_ptr = &P.counters[CTR_CL];
        if (cfg.light_bvh) {
            tn.static_grid = cfg.light_static;
            timed_trace<TM_NEE_LIGHT>(tn, cfg, st);
            tn.static_grid = 0;
            tn.fetch = &P.counters[CTR_F_OCC];
            tn.count_ptr = &P.counters[CTR_LIGHT];
            timed_trace<TM_NEE_LIGHT_OCC>(tn, cfg, st);
        } else {
            timed_trace<TM_NEE_CLOSEST>(tn, cfg, st);
        }
        if (ext) {
            // the extended light sampling's shadow and light-hit rays (same stages, own lists)
            TraceArgs tx = tn;
            tx.ext = 1;
            tx.static_grid = 0;
            tx.fetch = &P.counters[CTR_F_XANY];
            tx.count_ptr = &P.counters[CTR_XANY];
            timed_trace<TM_NEE_ANY>(tx, cfg, st);
            tx.fetch = &P.counters[CTR_F_XCL];
            tx.count_ptr = &P.counters[CTR_XCL];
            if (cfg.light_bvh) {
                timed_trace<TM_NEE_LIGHT>(tx, cfg, st);
                tx.fetch = &P.counters[CTR_F_XOCC];
                tx.count_ptr = &P.counters[CTR_XLIGHT];
                timed_trace<TM_NEE_LIGHT_OCC>(tx, cfg, st);
            } else {
                timed_trace<TM_NEE_CLOSEST>(tx, cfg, st);
            }
        }
        {
            TimedScope ts(cfg, st, KT_RESOLVE);
            // grid-stride over the shaded list (up to 2n entries with classes: deferred vertices appear twice)
            const dim3 rg(std::min(blocks_for(classes ? 2 * n : n), 8 * cfg.grid_persistent));
            if (ext) hipLaunchKernelGGL(k_resolve<true>, rg, dim3(TB), 0, st, S, P, d_frame, b, cnt_cur);
            else hipLaunchKernelGGL(k_resolve<false>, rg, dim3(TB), 0, st, S, P, d_frame, b, cnt_cur);
        }
        if (pipe) {
            hipEventRecord(cfg.ev_nee_join, st);
            nee_pending = true;
            st = main_st;
        }
        if (fork) hipStreamWaitEvent(st, cfg.ev_ahead_join, 0);
        // swap queues
        int32_t* tq = q_cur; q_cur = q_next; q_next = tq;
        int tc = c_cur; c_cur = c_next; c_next = tc;
    }
    if (nee_pending) hipStreamWaitEvent(st, cfg.ev_nee_join, 0);   // the last bounce's resolve
}

hipError_t launch_frame(const DevScene& S, const DevPaths& P0, const MptFrame* d_frame, const MptFrame& hf, LaunchCfg& cfg,
                        hipStream_t st) {
    DevPaths P = P0;
    const int n = P.n;
    if (n == 0) {
        if (hf.options.direct_light_sampling == MPT_LSS_RESTIR_DI) restir_empty_band(hf, cfg, st, P);
        return hipGetLastError();
    }
    const MptRenderSettings& hrs = hf.render_settings;
    // the camera queue is compacted by k_camera under adaptive sampling (unless speculative) and at
    // low resolution
    const bool as = ((hrs.stop_pixel_noise_threshold > 0.0f || hrs.enable_adaptive_sampling) && hrs.accumulate && !P.spec_as) ||
                    (hrs.wants_render_low_resolution && hrs.allow_render_low_resolution && hrs.accumulate) ||
                    P.spec_skip;   // (k_camera's spec_skip)
    // all pixels start a path, unless adaptive sampling compacts the camera queue (the counter set
    // by k_restir_frame_begin under ReSTIR DI, with the halo measure zeroed)
    if (hf.options.direct_light_sampling == MPT_LSS_RESTIR_DI) {
        hipLaunchKernelGGL(k_restir_frame_begin, dim3(std::max(1, blocks_for(P.rs_hi - P.rs_lo))), dim3(TB), 0, st, P, d_frame, as ? 0 : n,
                           cfg.halo_fn ? 1 : 0);
        P.rs_out = restir_buffer(P, cfg.restir_out_sp2);
    } else {
        hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&P.counters[CTR_Q0]), as ? 0 : n, 1, st);
    }
    {
        TimedScope ts(cfg, st, KT_CAMERA);
        hipLaunchKernelGGL(k_camera, dim3(blocks_for(n)), dim3(TB), 0, st, P, d_frame);
    }
    frame_bounces(S, P, d_frame, hf, cfg, st, 0, hf.render_settings.nb_bounces, P.q0, CTR_Q0, P.q1, CTR_Q1);
    // an overlapped batch's second half adds its samples after the first half's (sample order)
    if (cfg.ev_acc_wait) hipStreamWaitEvent(st, cfg.ev_acc_wait, 0);
    {
        TimedScope ts(cfg, st, KT_ACCUMULATE);
        hipLaunchKernelGGL(k_accumulate, dim3(blocks_for(P.n_pix)), dim3(TB), 0, st, P, d_frame);
    }
    if (cfg.ev_acc_done) hipEventRecord(cfg.ev_acc_done, st);
    return hipGetLastError();
}


// batched ReSTIR DI: sample s's continuation list (view slots) appended to the later
// bounces' queue (slot = s * pixels + pixel); the queue length is added by k_add_count
__global__ __launch_bounds__(TB) void k_append_queue(int32_t* __restrict__ dst, const int32_t* dst_count,
                                                     const int32_t* __restrict__ src, const int32_t* src_count,
                                                     int32_t off) {
    const int i = blockIdx.x * TB + threadIdx.x;
    if (i < *src_count) dst[*dst_count + i] = src[i] + off;
}
__global__ void k_add_count(int32_t* dst_count, const int32_t* src_count) {
    if (threadIdx.x == 0) dst_count[0] += src_count[0];
}
__global__ __launch_bounds__(TB) void k_iota(int32_t* q, int n) {
    const int i = blockIdx.x * TB + threadIdx.x;
    if (i < n) q[i] = i;
}
// batched ReSTIR DI under adaptive sampling: the slots [0, n) of `active` that are set, listed
// in q (wave64 ballot, one atomic per wave on *count, which starts at 0)
__global__ __launch_bounds__(TB) void k_queue_active(int32_t* __restrict__ q, int32_t* count, const uint8_t* __restrict__ active,
                                                     int n) {
    const int i = blockIdx.x * TB + threadIdx.x;
    const bool act = i < n && active[i] != 0;
    const uint64_t m = __ballot(act);
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (m) {
        const int first = __ffsll((unsigned long long)m) - 1;
        if (lane == first) base = atomicAdd(count, __popcll(m));
        base = __shfl(base, first);
    }
    if (act) q[base + __popcll(m & ((1ull << lane) - 1ull))] = i;
}

hipError_t launch_frames_restir(const DevScene& S, const DevPaths& PF, const MptFrame* d_frames, const MptFrame* hf,
                                int batch, LaunchCfg& cfg, hipStream_t st) {
    const int n = PF.n_pix;
    if (batch <= 0) return hipSuccess;
    if (n == 0) {   // an empty band of a partition: only its side of every sample's exchanges
        for (int s = 0; s < batch; s++) restir_empty_band(hf[s], cfg, st, PF);
        return hipGetLastError();
    }
    const int nb = hf[0].render_settings.nb_bounces;
    // the camera rays of every sample over its own slots [s * n, (s + 1) * n) (their seeds,
    // jitter and alpha keys are the sample's; nothing of the ReSTIR DI state is read), then
    // one traversal of all of them: a launch of batch x n rays instead of `batch` of n
    //
    // Adaptive sampling (PF.spec_as; mpt_render_frames batches such samples only while no pixel
    // can reach the gate's noise test, see restir_gate_static): a pixel converged before the batch
    // gets no camera ray (k_camera's spec_skip, `active` cleared), so the camera queues are built
    // from `active` -- all samples' for the one traversal, then each sample's own before its
    // G-buffer -- and k_accumulate replays the gate in sample order
    const bool skip = PF.spec_skip != 0;
    bool reset_before = false;
    for (int s = 0; s < batch; s++) {
        DevPaths P = PF;
        offset_slots(P, (size_t)s * n);
        P.n = n; P.batch = 1; P.group = 1;
        const MptRenderSettings& rs = hf[s].render_settings;
        P.spec_reset = reset_before ? 1 : 0;
        P.cam_noqueue = skip ? 1 : 0;
        reset_before |= rs.sample_number == 0 || rs.need_to_reset;
        TimedScope ts(cfg, st, KT_CAMERA);
        hipLaunchKernelGGL(k_camera, dim3(blocks_for(n)), dim3(TB), 0, st, P, d_frames + s);
    }
    {
        DevPaths G = PF;
        G.group = n;
        if (skip) {
            hipMemsetAsync(&PF.counters[CTR_QG], 0, sizeof(int32_t), st);
            hipLaunchKernelGGL(k_queue_active, dim3(blocks_for(batch * n)), dim3(TB), 0, st, PF.q0, &PF.counters[CTR_QG],
                               PF.active, batch * n);
        } else {
            hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&PF.counters[CTR_QG]), batch * n, 1, st);
        }
        hipMemsetAsync(&PF.counters[CTR_FETCH], 0, sizeof(int32_t), st);
        TraceArgs ta{};
        ta.S = S; ta.P = G; ta.queue = skip ? PF.q0 : nullptr; ta.count_ptr = &PF.counters[CTR_QG]; ta.fetch = &PF.counters[CTR_FETCH];
        ta.F = d_frames; ta.bounce = 0; ta.alpha = hf[0].render_settings.do_alpha_testing ? 1 : 0;
        timed_trace<TM_PATH>(ta, cfg, st);
    }
    hipMemsetAsync(&PF.counters[CTR_QG], 0, sizeof(int32_t), st);
    // With an envmap the final shading never writes through to a reservoir (validate_reservoir
    // only drops envmap samples without one), so no sample's passes depend on an earlier
    // sample's shading: each sample's final reservoirs are kept (rs_keep) and bounce 0 runs
    // once over the batch, like the later bounces
    const bool defer = PF.rs_keep && hf[0].world_settings.ambient_light_type == MPT_AMBIENT_ENVMAP;
    // Chunked initial candidates (deferred first bounce, staged initial pass): the G-buffer,
    // lights presampling and initial candidates of up to ci_chunk samples -- which read no earlier
    // sample's state -- as one launch set into the chunk's planes (cfg.ci_planes); each sample then
    // merges its G-buffer and initial reservoirs into the context's planes (k_chunk_join: the
    // stores the per-sample kernels make) before its reuse passes, in order.
    const MptReSTIRDISettings& rd0 = hf[0].render_settings.restir_di_settings;
    const int chunk = (defer && !skip && cfg.ci_planes && cfg.ci_chunk > 1 && cfg.restir_staged && PF.rq_o &&
                       rd0.number_of_initial_bsdf_candidates <= 1 && !hf[0].options.restir_di_initial_target_visibility)
                          ? std::min(cfg.ci_chunk, batch) : 1;
    for (int s = 0; s < batch; s++) {
        if (chunk > 1 && s % chunk == 0) {
            const int cn = std::min(chunk, batch - s);
            DevPaths G = PF;
            offset_slots(G, (size_t)s * n);
            G.n = cn * n; G.batch = 1; G.group = 1;
            G.pix_off = 0; G.ci_n = n; G.ci_pix_off = PF.pix_off;
            const DevPaths& C = *cfg.ci_planes;
            G.gb_pos = C.gb_pos; G.gb_sn = C.gb_sn; G.gb_gn = C.gb_gn; G.gb_view = C.gb_view; G.gb_meta = C.gb_meta;
            G.gb_vsA = C.gb_vsA; G.gb_vsB = C.gb_vsB; G.gb_mat = C.gb_mat; G.gb_cs = C.gb_cs;
            G.rs_init = C.rs_init; G.rs_plights = C.rs_plights;
            {
                TimedScope tk(cfg, st, KT_GBUFFER);
                hipLaunchKernelGGL(k_gbuffer, dim3(blocks_for(G.n)), dim3(TB), 0, st, S, G, d_frames + s);
            }
            TimedScope ts(cfg, st, KT_RESTIR);
            restir_initial(S, G, d_frames + s, hf[s], cfg, st);
        }
        // sample s: frame_begin, G-buffer, the ReSTIR DI passes (which read sample s - 1's
        // reservoirs and G-buffer) and, unless deferred, the rest of bounce 0 over its own slots
        DevPaths P = PF;
        offset_slots(P, (size_t)s * n);
        P.n = n; P.batch = 1; P.group = 1;
        if (cfg.halo_fn) {
            // a partitioned context: frame_begin maintains the band and the halo the previous
            // sample agreed on (launch_batch does the same for a batch's first sample)
            P.rs_lo = std::max(0, cfg.own_y0 - cfg.halo_prev) * hf[s].res_x;
            P.rs_hi = std::min(hf[s].res_y, cfg.own_y1 + cfg.halo_prev) * hf[s].res_x;
        }
        P.rs_out = restir_buffer(P, cfg.restir_out_sp2);
        if (defer && chunk > 1) {
            // frame_begin, the G-buffer and the initial reservoirs of the chunk's sample k in one
            // pass (k_chunk_join); the camera queue counter is not read on this path
            if (cfg.halo_fn) hipMemsetAsync(&P.counters[CTR_REPROJ], 0, sizeof(int32_t), st);
            {
                TimedScope tk(cfg, st, KT_GBUFFER);
                hipLaunchKernelGGL(k_chunk_join, dim3(blocks_for(P.rs_hi - P.rs_lo)), dim3(TB), 0, st, P, *cfg.ci_planes, PF.rq_meta,
                                   s % chunk, d_frames + s);
            }
            launch_restir(S, P, d_frames + s, hf[s], cfg, st, true);
            if (cfg.halo_fn) cfg.halo_prev = cfg.halo_rows;
            const size_t rn = 3 * (size_t)PF.rs_keep_n;
            hipMemcpyAsync(PF.rs_keep + (size_t)s * rn, P.rs_out + 3 * (size_t)PF.pix_off, rn * sizeof(float4),
                           hipMemcpyDeviceToDevice, st);
            continue;
        }
        // (the camera queue's length: n, k_camera's iota, or 0 for k_queue_active's list of the
        // sample's active slots; the halo measure zeroed)
        hipLaunchKernelGGL(k_restir_frame_begin, dim3(std::max(1, blocks_for(P.rs_hi - P.rs_lo))), dim3(TB), 0, st, P, d_frames + s,
                           skip ? 0 : n, cfg.halo_fn ? 1 : 0);
        if (skip) hipLaunchKernelGGL(k_queue_active, dim3(blocks_for(n)), dim3(TB), 0, st, P.q0, &P.counters[CTR_Q0], P.active, n);
        if (defer) {
            restir_first_bounce(S, P, d_frames + s, hf[s], cfg, st);
            if (cfg.halo_fn) cfg.halo_prev = cfg.halo_rows;
            // the band's reservoirs (rs_keep_n = the band's pixels, read by k_shade at the pixel's slot)
            const size_t rn = 3 * (size_t)PF.rs_keep_n;
            hipMemcpyAsync(PF.rs_keep + (size_t)s * rn, P.rs_out + 3 * (size_t)PF.pix_off, rn * sizeof(float4),
                           hipMemcpyDeviceToDevice, st);
            continue;
        }
        frame_bounces(S, P, d_frames + s, hf[s], cfg, st, 0, 0, P.q0, CTR_Q0, P.q1, CTR_Q1, true);
        if (cfg.halo_fn) cfg.halo_prev = cfg.halo_rows;
        if (nb > 0) {
            // the global queue's first entries never reach the next sample's slots: after
            // sample s it holds at most (s + 1) * n entries
            hipLaunchKernelGGL(k_append_queue, dim3(blocks_for(n)), dim3(TB), 0, st, PF.q0, &PF.counters[CTR_QG], P.q1,
                               &PF.counters[CTR_Q1], (int32_t)((size_t)s * n));
            hipLaunchKernelGGL(k_add_count, dim3(1), dim3(64), 0, st, &PF.counters[CTR_QG], &PF.counters[CTR_Q1]);
        }
    }
    // bounces 1..nb (deferred: 0..nb) of every sample as one wavefront (slot = sample * n + pixel:
    // group = n); overlapped batches: on the wave stream, once the chain above is done, so that
    // the next batch's chain runs beside it
    DevPaths G = PF;
    G.group = n;
    if (cfg.wave_stream) {
        hipEventRecord(cfg.ev_chain, st);
        hipStreamWaitEvent(cfg.wave_stream, cfg.ev_chain, 0);
        st = cfg.wave_stream;
        G.stack_spill = cfg.wave_spill;
    }
    if (defer) {
        G.rs_keep_on = 1;
        if (skip) {   // the batch's active slots
            hipMemsetAsync(&G.counters[CTR_Q0], 0, sizeof(int32_t), st);
            hipLaunchKernelGGL(k_queue_active, dim3(blocks_for(batch * n)), dim3(TB), 0, st, G.q0, &G.counters[CTR_Q0], G.active,
                               batch * n);
        } else {
            hipLaunchKernelGGL(k_iota, dim3(blocks_for(batch * n)), dim3(TB), 0, st, G.q0, batch * n);
            hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&G.counters[CTR_Q0]), batch * n, 1, st);
        }
        frame_bounces(S, G, d_frames, hf[0], cfg, st, 0, nb, G.q0, CTR_Q0, G.q1, CTR_Q1, true, true);
    } else if (nb > 0) {
        frame_bounces(S, G, d_frames, hf[0], cfg, st, 1, nb, G.q0, CTR_QG, G.q1, CTR_Q1);
    }
    {
        TimedScope ts(cfg, st, KT_ACCUMULATE);
        hipLaunchKernelGGL(k_accumulate, dim3(blocks_for(n)), dim3(TB), 0, st, G, d_frames);
    }
    return hipGetLastError();
}

// per-material resolution of the intersection-time material edits for untextured
// materials (the texture-independent part of intersection_material)
__global__ void k_resolve_materials(DevScene S, MptMaterial* out, int32_t* tex, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Mat& m = S.mats[i];
    int textured = 0;
    if (S.n_tex > 0) {
        const int32_t* ti = &m.emission_texture_index;
        for (int k = 0; k < 18; k++) textured |= ti[k] != MPT_NO_TEXTURE;
    }
    DevScene S0 = S;
    S0.n_tex = 0;
    const Mat r = intersection_material(S0, i, mk2(0.0f, 0.0f), false);
    out[i] = r;
    // plain-dielectric class (k_shade): coat, sheen, metallic, transmission and thin film are
    // zero and no texture can make them non-zero
    const bool plain = r.coat == 0.0f && r.sheen == 0.0f && r.metallic == 0.0f && r.specular_transmission == 0.0f &&
                       r.thin_film == 0.0f && m.coat_texture_index == MPT_NO_TEXTURE &&
                       m.sheen_texture_index == MPT_NO_TEXTURE && m.metallic_texture_index == MPT_NO_TEXTURE &&
                       m.roughness_metallic_texture_index == MPT_NO_TEXTURE &&
                       m.specular_transmission_texture_index == MPT_NO_TEXTURE;
    // glass class (k_shade<GLASS>): as plain, but transmission allowed (the glass lobe and the
    // coat block stay compiled in, dev_bsdf.h BC_GLASS)
    const bool glass = !plain && r.coat == 0.0f && r.sheen == 0.0f && r.metallic == 0.0f && r.thin_film == 0.0f &&
                       m.coat_texture_index == MPT_NO_TEXTURE && m.sheen_texture_index == MPT_NO_TEXTURE &&
                       m.metallic_texture_index == MPT_NO_TEXTURE && m.roughness_metallic_texture_index == MPT_NO_TEXTURE;
    // plain but for a metallic texture: per hit, by the resolved metallic value
    const bool texmetal = !plain && r.coat == 0.0f && r.sheen == 0.0f && r.specular_transmission == 0.0f && r.thin_film == 0.0f &&
                          m.coat_texture_index == MPT_NO_TEXTURE && m.sheen_texture_index == MPT_NO_TEXTURE &&
                          m.specular_transmission_texture_index == MPT_NO_TEXTURE &&
                          (m.roughness_metallic_texture_index != MPT_NO_TEXTURE || m.metallic_texture_index != MPT_NO_TEXTURE);
    tex[i] = (textured ? MT_TEXTURED : 0) | (plain ? 0 : MT_FULL) | (glass ? MT_GLASS : 0) | (texmetal ? MT_TEXMETAL : 0);
}


// Development check of the transcendental layer (fn: 0 sin 1 cos 2 exp 3 log 4 pow
// 5 atan2 6 asin 7 acos); host pointers, synchronous.
__global__ void k_debug_math(int fn, const float* a, const float* b, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i], r = 0.0f;
    switch (fn) {
        case 0: r = psin(x); break;
        case 1: r = pcos(x); break;
        case 2: r = pexp(x); break;
        case 3: r = plog(x); break;
        case 4: r = ppow(x, y); break;
        case 5: r = patan2(x, y); break;
        case 6: r = pasin(x); break;
        case 8: r = psincos(x).x; break;
        case 9: r = psincos(x).y; break;
        default: r = pacos(x); break;
    }
    out[i] = r;
}
extern "C" int mpt_debug_math(int fn, const float* a, const float* b, float* out, int n) {
    float *da, *db, *dout;
    hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dout, n * 4);
    hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_debug_math, dim3((n + 255) / 256), dim3(256), 0, 0, fn, da, db, dout, n);
    hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(dout);
    return 0;
}

hipError_t launch_restir_fill(float4* r, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_restir_fill, dim3((n + TB - 1) / TB), dim3(TB), 0, st, r, n);
    return hipGetLastError();
}
hipError_t launch_restir_fill_lights(float4* l, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_restir_fill_lights, dim3((n + TB - 1) / TB), dim3(TB), 0, st, l, n);
    return hipGetLastError();
}

hipError_t launch_resolve_materials(const DevScene& S, MptMaterial* out_res, int32_t* out_tex, int n, float4* em_tab,
                                   hipStream_t st) {
    hipLaunchKernelGGL(k_resolve_materials, dim3((n + 63) / 64), dim3(64), 0, st, S, out_res, out_tex, n);
    if (S.n_emissive > 0)
        hipLaunchKernelGGL(k_emissive_table, dim3((S.n_emissive + 63) / 64), dim3(64), 0, st, S, em_tab);
    return hipGetLastError();
}

// the sRGB decode of Texture.h:72-75 for every 8-bit value: ppow((float)v / 255, 2.2)
__global__ void k_srgb_table(float* out) {
    const int v = threadIdx.x;
    out[v] = ppow((float)v / 255.0f, 2.2f);
}
__global__ void k_env_rich(DevScene S, float4* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S.env_w * S.env_h) return;
    const int2 e = S.alias[i];
    float u, v;
    const float4 p = S.env[env_tex_index(S, env_sample_uv(S, i, u, v))];
    const float4 q = S.env[env_tex_index(S, env_sample_uv(S, e.y, u, v))];
    out[2 * (size_t)i] = make_float4(__int_as_float(e.x), __int_as_float(e.y), p.x, p.y);
    out[2 * (size_t)i + 1] = make_float4(p.z, q.x, q.y, q.z);
}
hipError_t launch_env_rich(const DevScene& S, float4* out, hipStream_t st) {
    const int n = S.env_w * S.env_h;
    hipLaunchKernelGGL(k_env_rich, dim3((n + 255) / 256), dim3(256), 0, st, S, out);
    return hipGetLastError();
}
hipError_t launch_srgb_table(float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_srgb_table, dim3(1), dim3(256), 0, st, out);
    return hipGetLastError();
}

hipError_t launch_tri_attr(const DevScene& S, float4* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tri_attr, dim3((S.n_tris + 255) / 256), dim3(256), 0, st, S, out);
    return hipGetLastError();
}

hipError_t launch_trace_raw(const DevScene& S, const float4* o, const float4* d, int n, bool any, float4* out_hit,
                            uint8_t* out_occ, int32_t* fetch_ctr, uint32_t* spill, int grid, hipStream_t st) {
    TraceArgs a{};
    a.S = S;
    a.P.stack_spill = spill;
    a.count_const = n;
    a.fetch = fetch_ctr;
    a.raw_o = o;
    a.raw_d = d;
    a.raw_hit = out_hit;
    a.raw_occ = out_occ;
    hipMemsetAsync(fetch_ctr, 0, sizeof(int32_t), st);
    if (any) hipLaunchKernelGGL((k_trace<TM_RAW_ANY, false>), dim3(grid), dim3(TB), 0, st, a);
    else hipLaunchKernelGGL((k_trace<TM_RAW_CLOSEST, false>), dim3(grid), dim3(TB), 0, st, a);
    return hipGetLastError();
}

#endif
}  // namespace mpt
