// mpt_internal.h -- device-side data layout shared by the C ABI (mpt_api.cpp) and the
// kernels (mpt_kernels.hip).  All buffers are SoA in HBM.  Per-pixel buffers are indexed
// by the index of a pixel inside the context's row partition; path state by "slot": the
// samples of one pixel are consecutive slots, in groups of `group` pixels
// (slot = ((pixel / group) * batch + sample) * group + pixel % group, see batch_slot in
// mpt_kernels.hip); a single-sample frame has slot == pixel.
#ifndef MPT_INTERNAL_H
#define MPT_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvh8.h"
#include "mpt.h"

namespace mpt {

// traversal stack: LDS part + per-thread global spill (entries of 2 words)
constexpr int TRAV_BLOCK = 256;
#ifndef MPT_LDS_STACK
#define MPT_LDS_STACK 12
#endif
constexpr int TRAV_LDS_STACK = MPT_LDS_STACK;
constexpr int TRAV_SPILL_DEPTH = 64 - TRAV_LDS_STACK;

// persistent traversal grid: MPT_TRACE_BLOCKS_PER_CU blocks of TRAV_BLOCK lanes per CU for the
// path / NEE modes (MPT_TRACE_WAVES waves per SIMD), the staged ReSTIR DI list modes scaled to
// MPT_TRACE_WAVES_LIST; every lane of such a grid owns TRAV_SPILL_DEPTH spill entries in HBM,
// indexed by its global thread id, so the spill area is sized for the larger of the two grids
#ifndef MPT_TRACE_BLOCKS_PER_CU
#define MPT_TRACE_BLOCKS_PER_CU 5
#endif
#ifndef MPT_TRACE_WAVES
#define MPT_TRACE_WAVES 5   // 5 waves / SIMD (<= 96 VGPRs): C3 traversal -4 % vs 4 (VGPR-capped), 6 and 8 no better (r02 A/B)
#endif
#ifndef MPT_TRACE_WAVES_LIST
#define MPT_TRACE_WAVES_LIST MPT_TRACE_WAVES   // the ReSTIR DI staged lists (TM_LIST_ANY / TM_LIST_CLOSEST)
#endif
#ifndef MPT_TRACE_WAVES_PATH
#define MPT_TRACE_WAVES_PATH MPT_TRACE_WAVES
#endif
// blocks per CU of the list-mode grid (launch_trace_mode: grid / MPT_TRACE_WAVES * MPT_TRACE_WAVES_LIST)
constexpr int TRACE_LIST_BLOCKS_PER_CU = MPT_TRACE_BLOCKS_PER_CU * MPT_TRACE_WAVES_LIST / MPT_TRACE_WAVES;
constexpr int TRACE_SPILL_BLOCKS_PER_CU =
    MPT_TRACE_BLOCKS_PER_CU > TRACE_LIST_BLOCKS_PER_CU ? MPT_TRACE_BLOCKS_PER_CU : TRACE_LIST_BLOCKS_PER_CU;
static_assert(MPT_TRACE_BLOCKS_PER_CU >= 1 && MPT_TRACE_WAVES >= 1 && MPT_TRACE_WAVES_LIST >= 1, "traversal grid");

struct DevScene {
    const Node8* nodes;
    const TriRec* tris;
    const Node8* nodes_light;     // light-hit BVH (build_light_bvh): triangles with possibly non-black emission
    const TriRec* tris_light;
    int32_t n_light_tris;
    const int32_t* idx;          // 3 per triangle
    const float* pos;            // 3 per vertex
    const float* nrm;            // 3 per vertex
    const uint8_t* has_n;
    const float* uv;             // 2 per vertex
    const int32_t* mat_idx;      // per triangle
    const float4* tri_attr;      // per triangle: 5 float4 of hit attributes (k_tri_attr / hit_attributes)
    const MptMaterial* mats;
    const MptMaterial* mats_res;  // per material: intersection-time resolution without textures
    const int32_t* mat_tex;       // per material: MT_TEXTURED | MT_FULL (k_resolve_materials)
    const int32_t* mat_prio;     // dielectric_priority per material (nested-dielectric push)
    const int32_t* emissive;
    const float4* em_tab;         // 5 float4 per emissive triangle (k_emissive_table)
    int32_t n_emissive;
    int32_t n_tris;
    const uint8_t* tex;          // all textures, RGBA8, concatenated
    const uint64_t* tex_off;     // byte offset per texture
    const int32_t* tex_dims;     // w, h per texture
    const float* srgb;           // 256: pow(v / 255, 2.2), the sRGB decode of 8-bit texels
    int32_t n_tex;
    // LUTs
    const float* lut_conductor;
    const float* lut_glossy;
    const float* lut_glass;
    const float* lut_glass_inv;
    const float* lut_thin_glass;
    const float* lut_sheen;
    // envmap
    const float4* env;
    const int2* alias;            // alias table, one entry per texel: (probability bits, alias index)
    // the alias table with the radiance texels its sampler reads (k_env_rich): per texel i two
    // float4 {probability, alias index bits, rgb(i)}, {rgb(alias(i))}, rgb(j) = the texel env_tex
    // reads for a sample at texel j -- one 32-B gather per envmap sample instead of two dependent
    const float4* env_rich;
    int32_t env_w, env_h;
    float env_sum;
    const float* env_cdf;         // ESS_BINARY_SEARCH: running luminance sum per texel (Image.cpp:553-574)
    float env_cdf_sum;            // its last element (OrochiEnvmap::compute_cdf)
};

// NEE record written by the shade stage and consumed by the resolve stage: seven float4
// planes indexed by slot (SoA, so that a wave's stores of one field cover 1 KiB of
// consecutive bytes), each written whole, and only when the vertex uses it:
//   nthr  throughput at the vertex (rgb) + NF_* flags
//   na    light-sample term (rgb: MIS / uniform pending radiance, RIS winner BSDF value,
//         ReSTIR DI final shading, or the immediate emission of NF_IMM) + RIS winner cosine
//   nb    BSDF sample / candidate: BSDF value (rgb) + pdf
//   ndir  BSDF sample direction + cosine
//   nris  RIS: light-candidate weight sum, winner target, the BSDF candidate's random,
//         winner triangle
//   ne1   envmap light-sampled contribution (rgb)
//   ne2   envmap BSDF-sampled contribution (rgb)
enum : uint32_t {
    NF_SHADED = 1u << 0,     // the path had a hit at this bounce -> resolve adds NEE
    NF_A = 1u << 1,          // light-sample contribution pending occlusion slot 0
    NF_B = 1u << 2,          // BSDF ray pending in the closest-hit slot
    NF_B_REFR = 1u << 3,
    NF_E1 = 1u << 4,         // env light-sample contribution pending occlusion slot 1
    NF_E2 = 1u << 5,         // env BSDF-sample contribution pending occlusion slot 2
    NF_RIS_W = 1u << 6,      // RIS light winner exists
    NF_IMM = 1u << 7,        // immediate light term (emissive textured material)
    NF_NOADD = 1u << 8,      // LSS_NO_DIRECT_LIGHT_SAMPLING: nothing to add at resolve
    NF_L = 1u << 9,          // the light-sampling strategy ran at this vertex
    NF_AQ = 1u << 10,        // ReSTIR DI final shading: the light term waits for occlusion slot 0
    NF_EXT = 1u << 11,       // extended light sampling: the light term is in the slot's ext entries
};

// Extended light sampling (number_of_light_samples > 1, RIS with more than one BSDF
// candidate, RISUseVisiblityTargetFunction; Lights.h:222-241, RIS.h:82-289): every light
// sample of a vertex gets its own queries and records, x_per entries per slot (entry
// e = slot * x_per + j), laid out per light sample `it` from j = it * x_iter:
//   uniform: [0] shadow ray + radiance        bsdf: [0] light-hit ray + BSDF value
//   MIS:     [0] shadow ray + weighted light radiance, [1] light-hit ray + BSDF value
//   RIS:     [c] light candidate c: {cw, random, target, triangle} + its visibility ray
//            (visibility target function), [L + c]: {f, cos} at the final shading
//            direction + the final shadow ray, [2L + b]: BSDF candidate b: {f, pdf},
//            {cos, random, refraction} + its light-hit ray
// Records: 2 float4 per entry (xrec); queries xq_o / xq_d; results xq_hit (closest) and
// xq_occ (any hit); xq_flag per entry: XQ_ANY / XQ_CL (a query was staged), XQ_REC.
enum : uint8_t { XQ_ANY = 1, XQ_CL = 2, XQ_REC = 4 };

struct DevPaths {
    int32_t n;                // path slots of the launch = batch samples x n_pix
    int32_t n_pix;            // pixels of the partition (per-pixel buffers: framebuffers, adaptive, ReSTIR)
    int32_t batch;            // samples per pixel of the launch (mpt_render_frames)
    int32_t group;            // pixels whose samples are interleaved in the slot order (4, or 1)
    int32_t res_x;
    float4* ray_o;            // xyz + last_hit bits
    float4* ray_d;            // xyz + tmax
    float4* hit;              // t, u, v, prim bits
    uint8_t* hit_inside;      // "inside a volume" before the last stack push (trace_ray normal flip)
    uint8_t* hit_cls;         // the hit triangle's material class (MT_* bits, TriRec::pad1), 0xff: miss
    uint32_t* rng;
    uint2* seeds;             // per slot: the camera launch's and the path tracing launch's pixel seeds (k_camera)
    float4* thr;
    float4* col;
    uint4* vsA;
    uint4* vsB;
    float4* alb;
    float4* nrm;
    int32_t* q0;
    int32_t* q1;
    int32_t* qh;              // this bounce's path queue split: paths that hit a surface ...
    int32_t* qm;              // ... and paths that left the scene (k_split)
    int32_t* qf;              // hits on materials outside the plain-dielectric class (k_split, k_shade)
    int32_t* nq_light;        // light-hit queries whose light candidate needs the whole-scene check (slot * 4 + 3)
    int32_t* counters;        // see CTR_*
    float4* nthr;             // NEE record planes (above)
    float4* na;
    float4* nb;
    float4* ndir;
    float4* nris;
    float4* ne1;
    float4* ne2;
    float4* nq_o;             // staged NEE query rays of query id slot * 4 + kind (kinds 0..2 any hit, 3
    float4* nq_d;             // closest), stored kind-major: [kind * nq_stride + slot] (nq_index)
    int64_t nq_stride;        // path slots the query / occlusion planes are sized for
    int32_t* nq_tgt;          // compacted query lists: [0, 3n) any hit, [3n, 4n) closest; entries slot * 4 + kind
    uint8_t* qmask;           // per slot: staged queries (bits 0..3), continuation (QM_CONT)
    uint8_t* occ;             // any-hit results, kind-major like nq_o
    float4* nhit;             // closest NEE result per slot; between split shading stages: shading normal + material
    float4* s_gn;             // between split shading stages: geometric normal (k_shade's ST)
    MptMaterial* mat_slot;    // per-slot resolved material (textured materials, white furnace)
    float4* ce;               // bounce pipeline (frame_bounces): the shading's addition to col, added by k_resolve
                              // (NULL: k_shade adds it to col itself)
    float* fb_color;          // 3 per slot (sum)
    float* fb_albedo;
    float* fb_normal;
    uint32_t* stack_spill;    // global spill area of the traversal stacks
    uint64_t* stats;          // [trace mode][rays, nodes, tris, -] (instrumented traversal)
    uint64_t* ray_counts;     // path rays, NEE any-hit rays, NEE closest rays, path hits, generic-class vertices,
                              // plain-class ReSTIR DI target evaluations (always on)
    // adaptive sampling / stop-noise threshold (AuxiliaryBuffers, RenderData.h:62-84)
    int32_t* as_count;        // pixel_sample_count
    float* as_sqlum;          // pixel_squared_luminance
    int32_t* as_conv;         // pixel_converged_sample_count (-1 = not converged)
    uint8_t* active;          // pixel_active
    int32_t spec_as;          // a batch of adaptive samples: traced speculatively, gated in k_accumulate
    int32_t spec_reset;       // (k_camera, one sample of a batch) an earlier sample of the batch resets the buffers
    int32_t spec_skip;        // spec_as under enable_adaptive_sampling with pixels possibly converged before the
                              // batch: k_camera leaves them out of the camera queue (host: MptContext::as_bound)
    uint32_t* status;         // [0] stop_noise_threshold_converged_count, [1] still_one_ray_active
    // ReSTIR DI (LSS_RESTIR_DI only; NULL otherwise).  G-buffer of the camera hits as
    // CameraRays writes it (CameraRays.h:144-166, GBuffer.h:17-34), current + previous frame:
    float4* gb_pos;           // first hit xyz
    float4* gb_sn;            // shading normal (as stored, not renormalised)
    float4* gb_gn;            // geometric normal
    float4* gb_view;          // view direction (-ray direction)
    int4* gb_meta;            // x prim (-1 miss), y material index + 1 (0: never written), z camera_ray_hit, w per-pixel material
    uint4* gb_vsA;            // ray volume state
    uint4* gb_vsB;
    MptMaterial* gb_mat;      // per-pixel resolved material (textured materials / white furnace)
    float4* pgb_pos; float4* pgb_sn; float4* pgb_gn; float4* pgb_view; int4* pgb_meta;
    uint4* pgb_vsA; uint4* pgb_vsB; MptMaterial* pgb_mat;
    // the same surfaces as one 64-B record per pixel (4 float4: position + material reference,
    // shading normal + incident medium, view + last hit, geometric normal) for the plain-class
    // target-function evaluations, which read neighbours' surfaces at random (restir_di.h
    // gb_csurf): one line per neighbour instead of one per plane
    float4* gb_cs; float4* pgb_cs;
    float4* rs_init;          // reservoirs (3 float4 each): initial candidates
    float4* rs_sp1;           // spatial outputs, ping-pong
    float4* rs_sp2;
    float4* rs_out;           // restir_output_reservoirs of this frame (rs_sp1 or rs_sp2)
    float4* rs_tin;           // temporal input of this frame (last frame's output)
    float4* rs_keep;          // batched ReSTIR DI: each sample's final reservoirs (sample-major, rs_keep_n pixels each)
    int64_t rs_keep_n;
    int rs_keep_on;           // k_shade's final shading reads rs_keep by (sample, pixel) instead of rs_out
    int32_t cam_noqueue;      // k_camera writes no camera queue (batched ReSTIR DI builds it from `active`)
    float4* rs_plights;       // presampled lights (4 float4 each)
    // The G-buffer / reservoir / rs_conv arrays are frame-sized and indexed by the global
    // pixel index; path-state slot s of this context is pixel s + pix_off (contiguous band).
    // [rs_lo, rs_hi) = the pixels of the band plus its halo rows (what frame_begin maintains).
    int32_t pix_off;
    int32_t rs_lo, rs_hi;
    // ReSTIR DI initial candidates of a chunk of samples in one launch set (launch_frames_restir):
    // ci_n > 0 = the band's pixels per sample; item s of the launch is pixel s % ci_n of the
    // chunk's sample s / ci_n, its frame Fp[s / ci_n]; the G-buffer / rs_init / rs_plights
    // pointers are the chunk's planes, indexed by item (pix_off 0), and ci_pix_off is the band's
    // first pixel (seeds, coordinates)
    int32_t ci_n;
    int32_t ci_pix_off;
    int32_t* rs_conv;         // pixel_converged_sample_count by pixel (== as_conv when unpartitioned)
    // extended light sampling (NF_EXT), sized by the frame's options; NULL / 0 otherwise
    int32_t x_per;            // entries per slot
    int32_t x_iter;           // entries per light sample
    float4* xq_o;
    float4* xq_d;
    float4* xq_hit;
    uint8_t* xq_occ;
    uint8_t* xq_flag;
    float4* xrec;             // 2 per entry
    int32_t* xl_any;          // compacted ext query lists (entries), CTR_XANY / CTR_XCL / CTR_XLIGHT
    int32_t* xl_cl;
    int32_t* xl_light;
    // staged ReSTIR DI reuse passes (restir_di.h, RS_RPP ray positions per pixel slot): rays
    // (xyz + last hit bits / xyz + t_max), their alpha keys and any-hit results, the compacted
    // ray list (CTR_RQ, then the visibility-reuse rays CTR_RQV), per-pixel pass metadata and
    // per-neighbour records
    float4* rq_o;
    float4* rq_d;
    uint32_t* rq_key;
    uint8_t* rq_occ;
    int32_t* rq_list;
    int32_t* rq_items;        // target-evaluation items by class (2 x RS_RPP per pixel slot)
    int4* rq_meta;
    float4* rq_rec;
};

constexpr int N_TRACE_MODES = 5;
// staged ReSTIR DI reuse passes (restir_di.h RS_KMAX / RS_RPP): neighbours per pass, ray positions per pixel
constexpr int RS_KMAX_HOST = 5, RS_RPP_HOST = 2 * RS_KMAX_HOST + 2, RS_REC_HOST = RS_KMAX_HOST + 2;
constexpr int N_RAY_COUNTS = 6;   // DevPaths::ray_counts
// timed kernel kinds: 0..2 = traversal stages (trace modes), then the others
enum { KT_CAMERA = 3, KT_SHADE = 4, KT_RESOLVE = 5, KT_ACCUMULATE = 6, KT_COMPACT = 7, KT_RESTIR = 8, KT_SPLIT = 9,
       KT_MISS = 10, KT_SHADE_GENERIC = 11,
       // the ReSTIR DI kernels one by one (inside KT_RESTIR's span): G-buffer, presampling,
       // initial candidates, temporal / fused spatiotemporal reuse, spatial reuse
       KT_GBUFFER = 12, KT_RS_PRESAMPLE = 13, KT_RS_INITIAL = 14, KT_RS_REUSE = 15, KT_RS_SPATIAL = 16,
       // the plain-class target-function evaluations of the staged reuse passes (k_rsp_eval<OVR, true, *>)
       KT_RS_EVAL = 17, KT_COUNT = 18 };
constexpr uint32_t QM_CONT = 16u;
// mat_tex bits: a texture feeds the resolved material; the material is outside the
// plain-dielectric class (coat, sheen, metallic, transmission or thin film may be non-zero)
constexpr int32_t MT_TEXTURED = 1, MT_FULL = 2, MT_GLASS = 4;   // MT_GLASS: k_resolve_materials
// MT_TEXMETAL (with MT_FULL): outside the plain class only through its metallic texture; the
// resolved material at the hit decides (k_split sends it to the plain list, k_shade<PLAIN>
// defers the vertices whose texel is metallic)
constexpr int32_t MT_TEXMETAL = 8;
constexpr int STATS_STRIDE = 6;   // per mode: traversals, nodes, tris, (unused), node slots, tri slots
constexpr int N_STATS = N_TRACE_MODES * STATS_STRIDE;

enum {
    CTR_Q0 = 0, CTR_Q1 = 1,                         // path queues (ping-pong)
    CTR_QG = 2,                                     // batched ReSTIR DI: the later bounces' path queue
    // from CTR_ANY on: zeroed by ONE memset at the top of every bounce (frame_bounces)
    CTR_ANY = 3, CTR_CL = 4,                        // NEE query lists: any hit, closest
    CTR_FETCH = 5,                                  // work counter of the list traversals outside the bounce loop
    CTR_REPROJ = 6,           // max |reprojected row - row| of the frame's G-buffer (partitioned ReSTIR DI)
    CTR_HIT = 7, CTR_MISS = 8,  // lengths of the hit / miss queues of the bounce (k_split)
    CTR_FULL = 9,             // length of the generic-material hit queue (k_split + k_shade deferrals)
    CTR_DEFER = 10,           // plain-class hits deferred to the generic queue (tombstones in qh)
    CTR_LIGHT = 11,           // length of nq_light (k_trace TM_NEE_LIGHT)
    CTR_XANY = 12, CTR_XCL = 13, CTR_XLIGHT = 14,   // ext query lists (extended light sampling)
    CTR_RQ = 15, CTR_RQV = 16,                      // staged ReSTIR DI rays / visibility-reuse rays
    CTR_RQE0 = 17, CTR_RQE1 = 18,                   // staged ReSTIR DI target evaluations: plain / generic class
    CTR_F_RQA = 19, CTR_F_RQB = 20,                 // the work counters of a staged pass's two list traversals
    CTR_RQ_GROUP = 6,                               // CTR_RQ .. CTR_F_RQB: zeroed by one memset per staged pass
    CTR_GLASS = 21,                                 // length of the glass-class list (top of qf, k_split)
    // the persistent traversals' work counters of a bounce, one per launch (no reset between them)
    CTR_F_PATH = 22, CTR_F_ANY = 23, CTR_F_CL = 24, CTR_F_OCC = 25, CTR_F_XANY = 26, CTR_F_XCL = 27, CTR_F_XOCC = 28,
    CTR_COUNT = 29
};
constexpr int CTR_BOUNCE_FIRST = CTR_ANY;           // [CTR_BOUNCE_FIRST, CTR_COUNT): reset per bounce

// launch glue (mpt_kernels.hip)
struct LaunchCfg {
    int grid_persistent;      // blocks of the persistent traversal kernels
    int stats;                // instrumented traversal
    hipEvent_t* ev_pool;      // optional: one event pair per traversal launch
    int* ev_mode;             // trace mode of each event pair
    int ev_cap;
    int ev_used;
    uint32_t launches;
    int restir_out_sp2;       // in/out: restir_output_reservoirs: 0 rs_sp1, 1 rs_sp2, 2 rs_init
    // ReSTIR DI across a row partition: the host's halo exchange (mpt_set_halo_exchange)
    MptHaloExchangeFn halo_fn;
    void* halo_user;
    int own_y0, own_y1;
    int halo_prev;            // halo agreed in the previous frame (the rows frame_begin maintained)
    int halo_rows;            // out: halo agreed in this frame's G-buffer exchange
    int32_t* h_reproj;        // pinned host word for the measured reprojection offset
    int halo_rc;              // out: first non-zero callback return
    int shade_classes;        // material-class shading: 0 off, 1 on, 2 on + defer every plain vertex (test hook)
    int light_bvh;            // light-hit queries through the light BVH (1) or one closest-hit traversal (0)
    int light_static;         // the light BVH's traversal stack fits in LDS (one query per lane, no spill)
    int restir_staged;        // ReSTIR DI reuse passes staged around their rays (restir_di.h), when supported
    int restir_mono_reuse;    // the reuse passes as the monolithic kernels (the initial pass staged)
    int shade_glass;          // k_split's glass class (MPT_SHADE_GLASS)
    int mat_private;          // k_shade<..., MATP>: textured vertices' resolved material in private memory
    int shade_split;          // plain class in stages (MPT_SHADE_SPLIT): 0 one kernel, 1 light / env / cont,
                              // 2 light / env + cont, 3 light + env / cont
    // overlapped batch halves (mpt_api.cpp launch_batch): recorded after the bounce-0 path
    // traversal / after k_accumulate; waited for before k_accumulate (all optional)
    hipEvent_t ev_first_trace;
    hipEvent_t ev_acc_done;
    hipEvent_t ev_acc_wait;
    // overlapped ReSTIR DI batches (launch_frames_restir): the shared later-bounce wavefront runs
    // on wave_stream (after ev_chain, recorded at the end of the per-sample chain) with its own
    // traversal spill area
    hipStream_t wave_stream;
    uint32_t* wave_spill;
    hipEvent_t ev_chain;
    // staged ReSTIR DI stages: the generic-class kernel on side_stream beside the plain-class one
    // (they read and write disjoint items; forked after the selection, joined before the trace),
    // with its own spill area (NULL side_stream: one stream)
    hipStream_t side_stream;
    uint32_t* side_spill;
    hipEvent_t ev_side_fork, ev_side_join;
    // trace-ahead (frame_bounces): bounce b + 1's path traversal on ahead_stream beside bounce b's
    // NEE traversals and resolve, with its own spill area (NULL ahead_stream: one stream)
    hipStream_t ahead_stream;
    uint32_t* ahead_spill;
    hipEvent_t ev_ahead_fork, ev_ahead_join;
    uint32_t ahead_launches;   // out: path traversals launched ahead
    // bounce pipeline (frame_bounces): bounce b's NEE traversals and resolve on nee_stream beside
    // bounce b + 1's split and shading, over the alternate plane set pipe_alt (odd bounces: NEE
    // planes, staged queries and lists, shaded lists, per-bounce counters, col additions); NULL
    // nee_stream: in line
    hipStream_t nee_stream;
    uint32_t* nee_spill;
    hipEvent_t ev_nee_fork, ev_nee_join;
    const DevPaths* pipe_alt;
    // chunked ReSTIR DI initial candidates (launch_frames_restir): up to ci_chunk samples per
    // chunk; ci_planes' G-buffer / rs_init / rs_plights pointers are the chunk's planes (NULL
    // ci_planes or ci_chunk < 2: one sample's chain at a time)
    int ci_chunk;
    const DevPaths* ci_planes;
};

// Moves every per-slot pointer of P by `off` slots: a view of slots [off, off + P.n) of the
// path state (the second half of an overlapped batch, one sample of a batched ReSTIR DI
// wavefront); per-pixel buffers stay shared.
inline void offset_slots(DevPaths& P, size_t off) {
    P.ray_o += off; P.ray_d += off; P.hit += off; P.hit_inside += off; P.hit_cls += off; P.rng += off; P.seeds += off; P.thr += off; P.col += off;
    P.vsA += off; P.vsB += off; P.alb += off; P.nrm += off;
    P.q0 += off; P.q1 += off; P.qh += off; P.qm += off; P.qf += off; P.nq_light += off;
    // NEE record planes, and the kind-major query / occlusion planes (stride = the allocation)
    P.nthr += off; P.na += off; P.nb += off; P.ndir += off; P.nris += off; P.ne1 += off; P.ne2 += off;
    P.nq_o += off; P.nq_d += off; P.occ += off; P.nq_tgt += 4 * off;
    P.nhit += off; P.s_gn += off; P.qmask += off; P.active += off;
    if (P.mat_slot) P.mat_slot += off;
    if (P.ce) P.ce += off;
}

hipError_t launch_frame(const DevScene& S, const DevPaths& P, const MptFrame* d_frame, const MptFrame& h_frame,
                        LaunchCfg& cfg, hipStream_t st);
// A batch of `batch` ReSTIR DI samples (P: batch samples, slot = sample * pixels + pixel):
// each sample's camera rays, ReSTIR DI passes and first bounce in turn (each reads the
// previous sample's reservoirs), then the later bounces of all samples as one wavefront.
hipError_t launch_frames_restir(const DevScene& S, const DevPaths& P, const MptFrame* d_frames, const MptFrame* h_frames,
                                int batch, LaunchCfg& cfg, hipStream_t st);
hipError_t launch_resolve_materials(const DevScene& S, MptMaterial* out_res, int32_t* out_tex, int n, float4* em_tab,
                                   hipStream_t st);
hipError_t launch_restir_fill(float4* reservoirs, int n, hipStream_t st);
hipError_t launch_restir_fill_lights(float4* lights, int n, hipStream_t st);
hipError_t launch_bake(int kind, int w, int h, int d, int ipk, int nb_samples, int iteration, float* out, hipStream_t st);
hipError_t launch_tri_attr(const DevScene& S, float4* out, hipStream_t st);
hipError_t launch_srgb_table(float* out, hipStream_t st);
hipError_t launch_env_rich(const DevScene& S, float4* out, hipStream_t st);
hipError_t launch_trace_raw(const DevScene& S, const float4* o, const float4* d, int n, bool any, float4* out_hit,
                            uint8_t* out_occ, int32_t* fetch_ctr, uint32_t* spill, int grid, hipStream_t st);

}  // namespace mpt

#endif
