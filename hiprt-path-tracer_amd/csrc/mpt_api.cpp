// mpt_api.cpp -- the C ABI of libmpt (include/mpt.h).  Owns all device memory of a
// context (one per GPU), builds the BVH8 on scene upload, stages per-frame settings
// and launches the wavefront frame (mpt_kernels.hip).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "bvh8.h"
#include "mpt.h"
#include "mpt_internal.h"

using namespace mpt;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace

namespace mpt {
int api_fail(int code, const char* msg) { return fail(code, msg); }   // for the library's other host files
}  // namespace mpt

namespace {

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return fail(MPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Status of a failed allocation / memset: MPT_ERR_OUT_OF_MEMORY for hipErrorOutOfMemory.
// Clears HIP's last error so that a later launch check does not report it again.
int alloc_fail(hipError_t e, const std::string& what) {
    (void)hipGetLastError();
    return fail(e == hipErrorOutOfMemory ? MPT_ERR_OUT_OF_MEMORY : MPT_ERR_HIP, what + ": " + hipGetErrorString(e));
}

// Device buffer owned by a context (freed by the context's destructor at the latest).
template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() { release(); }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
    hipError_t alloc(size_t count) {
        if (count == n && p) return hipSuccess;
        release();
        if (count == 0) return hipSuccess;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e == hipSuccess) n = count;
        return e;
    }
    hipError_t upload(const T* h, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

constexpr int FRAME_RING = 256;   // >= 2 x MPT_MAX_BATCH
constexpr int PIX_PARTS_MAX = 4;  // row parts of a one-sample frame (MptContext::pix_parts)
// timing events per frame: one pair per timed launch, 10 per bounce (path, any-hit and two
// light-hit traversals, split, plain and generic shade, miss, compact, resolve) for up to 65
// bounces (validate_frame), + camera, ReSTIR, accumulate
// + the ReSTIR DI kernels (G-buffer, presampling, initial, temporal / spatiotemporal, 4 spatial)
// samples per batched ReSTIR DI wavefront (<= 50 timed scopes each): a partitioned context's
// band is 1/N of the frame, so its later bounces need up to 128 samples to reach the
// single-GPU wavefront size (MPT_RESTIR_MAX_BATCH lowers it, A/B)
constexpr int RESTIR_MAX_BATCH = 128;
// x2: the two halves of an overlapped batch
constexpr int EV_POOL = 2 * 2 * ((10 * 65 + 3 + 8) > 50 * RESTIR_MAX_BATCH ? (10 * 65 + 3 + 8) : 50 * RESTIR_MAX_BATCH);
constexpr int SPILL_WORDS = 2 * TRAV_SPILL_DEPTH;
constexpr int MAX_STACK = TRAV_LDS_STACK + TRAV_SPILL_DEPTH;

}  // namespace

struct MptContext {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // overlapped batches (MPT_OVERLAP at mpt_create): the second half of a sample batch runs
    // on stream2, one pipeline stage behind the first, so that shading waves of one half and
    // traversal waves of the other share the CUs
    // MPT_OVERLAP: a path-tracing batch's two halves on two streams: 1 always, 0
    // never, -1 (default) for wavefronts of at most OVERLAP_AUTO_PATHS paths -- a rank's share of
    // a split frame at the driver's 20 samples, where the launch tails are a larger part of each
    // launch (one rank of 2 / 4 / 8: -2.3 / -2.7 / -3.8 %); a whole 1080p frame's 33-41 M paths
    // keep one stream (+1.2 % only, and its per-kernel times stay unshared)
    int overlap = -1;
    hipStream_t stream2 = nullptr;
    // the third and fourth row parts of a one-sample frame (MptContext::pix_parts): streams,
    // traversal spill areas, join events
    hipStream_t streamx[2] = {nullptr, nullptr};
    hipEvent_t ev_joinx[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_first = nullptr, ev_acc = nullptr, ev_join = nullptr;
    // Overlapped ReSTIR DI batches (MPT_RESTIR_OVERLAP, default on): a batch's per-sample chain
    // (G-buffer, reuse passes, halo exchanges: many small dependent launches) runs on the
    // context's stream while the previous batch's shared later-bounce wavefront runs on stream2.
    // The two batches in flight use the two halves of the path state (restir_half), each with its
    // own counters; ev_half[h] marks the end of the last wavefront that used half h.
    int restir_overlap = 1;
    bool restir_overlap_ok = false;       // prepare_batch found room for both halves
    int restir_half = 0;
    hipEvent_t ev_chain = nullptr, ev_half[2] = {nullptr, nullptr}, ev_wave_join = nullptr;
    bool ev_half_used[2] = {false, false};
    bool wave_pending = false;            // a wavefront on stream2 not yet joined into the stream
    // One-sample launch sets as a HIP graph (MPT_GRAPHS, default on): mpt_render_frame's ~50
    // launches of a path-tracing sample captured once and replayed while the frame differs only in
    // what the kernels read from it (seeds, sample number, cameras, status flags); the graph reads
    // its frame from the extra ring slot d_frames[FRAME_RING].  Keyed by those frame fields that
    // steer the host's launch sequence and by the kernels' by-value arguments (buffer pointers).
    int graphs = 0;   // MPT_GRAPHS=1: one-sample launch sets replayed from a captured HIP graph (no gain measured, r05e)
    // one-sample frames of a whole-frame context as row parts on their own streams (MPT_PIX_PARTS:
    // 0 / 1 off, 2 .. PIX_PARTS_MAX parts)
    int pix_parts = 3;   // batch-1 C3 6.09 -> 5.44 (2 parts) -> 5.29 ms/spp (3); 4 parts 6.76 (past GPU_MAX_HW_QUEUES), r06d
    // staged ReSTIR DI stages: the generic-class kernel on a side stream beside the plain one
    // (MPT_RESTIR_SIDE: 1 for partitions of at most 2^20 pixels, 2 always, 0 never)
    int restir_side = 1;
    hipEvent_t ev_side[2] = {nullptr, nullptr};
    // trace-ahead (MPT_TRACE_AHEAD): the next bounce's path traversal beside this bounce's NEE
    // traversals and resolve, on streamx[1]
    int trace_ahead = 1;
    int ovl_ahead = 1;   // MPT_OVERLAP_AHEAD: trace-ahead in both halves of an overlapped batch
    hipEvent_t ev_ahead[2] = {nullptr, nullptr};
    hipEvent_t ev_ahead2[2] = {nullptr, nullptr};   // (the second half of an overlapped batch)
    uint32_t ahead_launches = 0;   // MptStats::trace_ahead_launches
    uint32_t pipelined_batches = 0;   // MptStats::pipelined_batches
    hipGraphExec_t graph_exec = nullptr;
    std::vector<uint8_t> graph_key;
    uint32_t graph_launches = 0;
    uint32_t graph_captures = 0, graph_replays = 0;   // since mpt_enable_stats (MptStats)
    uint32_t overlapped_batches = 0;
    int num_cus = 256;
    int grid = 1024;
    // scene
    bool has_scene = false;
    BVH8 bvh;
    DBuf<Node8> nodes;
    DBuf<TriRec> tris;
    DBuf<float4> tri_attr;               // 5 per triangle (launch_tri_attr)
    DBuf<float> srgb;                    // 256-entry sRGB decode table (launch_srgb_table)
    // light-hit BVH (k_trace TM_NEE_LIGHT): the triangles whose emission can be non-black
    BVH8 bvh_light;
    DBuf<Node8> nodes_light;
    DBuf<TriRec> tris_light;
    std::vector<int32_t> h_light_prims;
    std::vector<int32_t> h_idx;           // host copies for rebuilding the light BVH on material edits
    std::vector<float> h_pos;
    float box_pad = 0.0f;
    int light_bvh = 1;                    // MPT_LIGHT_BVH at mpt_create: 0 = one closest-hit traversal per light-hit query
    bool light_bvh_ok = false;            // the light BVH matches the materials (else: the exact closest-hit path)
    int light_bvh_max_stack = 1 << 30;    // test hook (MPT_LIGHT_BVH_MAX_STACK): a lower traversal-stack limit
    DBuf<int32_t> idx, mat_idx, mat_prio, emissive, tex_dims;
    DBuf<float> pos, nrm, uv;
    DBuf<uint8_t> has_n, tex;
    DBuf<uint64_t> tex_off;
    DBuf<MptMaterial> mats;
    DBuf<MptMaterial> mats_res;   // untextured intersection-time resolution per material
    DBuf<int32_t> mat_tex;
    DBuf<float4> em_tab;
    bool any_tex = false;
    bool any_glass = false;   // a material of the glass class (MT_GLASS): k_shade<GLASS> is launched
    double tex_tri_frac = 0.0;            // triangles with a textured material / all (resolve_materials)
    int mat_private = -1;                 // MPT_MAT_PRIVATE: 1 / 0 force k_shade's MATP, -1 by tex_tri_frac
    // material-class shading (k_split / k_shade): 1 on (default), 0 off, 2 on with every
    // plain vertex deferred to the generic kernel (test hook); MPT_SHADE_CLASSES at mpt_create
    int shade_classes = 1;
    int restir_staged = 1;                // ReSTIR DI reuse passes staged around their rays (MPT_RESTIR_STAGED)
    int restir_mono_reuse = 0;            // MPT_RESTIR_MONO_REUSE: the reuse passes monolithic, the initial pass staged
    int restir_batch = 1;                 // ReSTIR DI samples batched after bounce 0 (MPT_RESTIR_BATCH)
    int adaptive_batch = 1;               // adaptive samples batched, gated in k_accumulate (MPT_ADAPTIVE_BATCH)
    int restir_max_batch = RESTIR_MAX_BATCH;   // MPT_RESTIR_MAX_BATCH
    int shade_glass = 1;                  // glass-class shading kernel (MPT_SHADE_GLASS)
    int shade_split = 0;                  // plain-class shading stages (MPT_SHADE_SPLIT, LaunchCfg::shade_split)
    int shade_texmetal = 1;               // MT_TEXMETAL materials through the plain list (MPT_SHADE_TEXMETAL)
    std::vector<MptMaterial> h_mats;
    std::vector<int32_t> h_mat_idx;       // per triangle (alpha flags of the triangle records)
    std::vector<uint8_t> h_tex_alpha;     // per texture: some texel has alpha < 255
    int n_tex = 0;
    // luts / envmap
    DBuf<float> lut_conductor, lut_glossy, lut_glass, lut_glass_inv, lut_thin, lut_sheen;
    DBuf<float4> env;
    DBuf<int2> alias;
    DBuf<float4> env_rich;                // alias entries with their radiance texels (launch_env_rich)
    DBuf<float> env_cdf;
    float env_cdf_sum = 0.0f;
    int env_w = 0, env_h = 0;
    float env_sum = 0.0f;
    // paths
    int res_x = 0, res_y = 0, band_h = 1, band_i = 0, band_c = 1, n_slots = 0;   // n_slots = pixels of the partition
    int batch_cap = 0;      // samples per pixel the path state is sized for (mpt_render_frames)
    int batch = 1;          // samples of the launch being set up
    DBuf<float4> ray_o, ray_d, hit, thr, col, alb, nrmv, nq_o, nq_d, nhit, s_gn;
    DBuf<uint8_t> hit_inside, hit_cls, occ, qmask;
    DBuf<uint32_t> rng, spill, spill2, spillx[2];
    DBuf<uint2> seeds;
    DBuf<uint4> vsA, vsB;
    DBuf<int32_t> q0, q1, qh, qm, qf, nq_light, counters, nq_tgt, fetch_raw;
    DBuf<float4> nthr, na, nb, ndir, nris, ne1, ne2;   // NEE record planes (mpt_internal.h)
    // bounce pipeline (LaunchCfg::pipe_alt): the odd bounces' NEE planes, staged queries and their
    // lists, shaded lists, and both parities' col additions (MPT_PIPELINE)
    DBuf<float4> nthr2, na2, nb2, ndir2, nris2, ne12, ne22, nq_o2, nq_d2, ce, ce2;
    DBuf<int32_t> nq_tgt2, qh2, qf2;
    int pipeline = 1;
    size_t pipe_n = 0;
    hipEvent_t ev_nee[4] = {nullptr, nullptr, nullptr, nullptr};   // fork / join per NEE stream
    int pix_pipe = 1;   // MPT_PIX_PIPE: a one-sample frame as 2 row parts, each pipelined
    DBuf<float> fb_color, fb_albedo, fb_normal;
    DBuf<int32_t> as_count, as_conv;
    DBuf<float> as_sqlum;
    DBuf<uint8_t> active;
    DBuf<uint32_t> status;
    // ReSTIR DI (allocated on the first LSS_RESTIR_DI frame)
    DBuf<float4> gb_pos, gb_sn, gb_gn, gb_view, pgb_pos, pgb_sn, pgb_gn, pgb_view;
    DBuf<int4> gb_meta, pgb_meta;
    DBuf<uint4> gb_vsA, gb_vsB, pgb_vsA, pgb_vsB;
    DBuf<MptMaterial> gb_mat, pgb_mat;
    DBuf<float4> gb_cs, pgb_cs;           // compact surface records (4 float4 per pixel)
    DBuf<float4> rs_init, rs_sp1, rs_sp2, rs_plights;
    DBuf<float4> rs_keep;                 // batched ReSTIR DI: the final reservoirs of each sample of a batch
    DBuf<int32_t> rs_conv;
    // staged ReSTIR DI passes (DevPaths::rq_*): RS_RPP ray positions per pixel slot
    DBuf<float4> rq_o, rq_d, rq_rec;
    DBuf<uint32_t> rq_key;
    DBuf<uint8_t> rq_occ;
    DBuf<int32_t> rq_list, rq_items;
    DBuf<int4> rq_meta;
    // chunked ReSTIR DI initial candidates (launch_frames_restir, LaunchCfg::ci_planes): the
    // G-buffer, initial reservoirs and presampled lights of up to restir_chunk samples
    int restir_chunk = -1;                // MPT_RESTIR_CHUNK: samples per chunk (-1: by the band's pixels)
    int ci_chunk = 1;                     // the chunk the planes below are sized for
    DBuf<float4> ci_pos, ci_sn, ci_gn, ci_view, ci_cs, ci_rs, ci_pl;
    DBuf<int4> ci_meta;
    DBuf<uint4> ci_vsA, ci_vsB;
    DBuf<MptMaterial> ci_mat;
    DevPaths ci_dp{};
    int restir_out_sp2 = 0;
    MptHaloExchangeFn halo_fn = nullptr;   // ReSTIR DI across a row partition
    void* halo_user = nullptr;
    int halo_prev = 0;                     // halo agreed in the previous frame
    int32_t* h_reproj = nullptr;           // pinned readback of the reprojection offset
    DBuf<MptMaterial> mat_slot;
    // extended light sampling (ensure_ext): x_per entries per path slot of the current batch
    DBuf<float4> xq_o, xq_d, xq_hit, xrec;
    DBuf<uint8_t> xq_occ, xq_flag;
    DBuf<int32_t> xl_any, xl_cl, xl_light;
    int x_per = 0, x_iter = 0;
    DBuf<uint64_t> stats;
    DBuf<uint64_t> ray_counts;
    // frames
    MptFrame* h_frames = nullptr;   // pinned ring
    MptFrame* d_frames = nullptr;
    int frame_slot = 0;
    // stats
    bool timing = false;
    bool instrumented = false;
    // two event pools used by alternate frames: a pool is read back when it is
    // reused two frames later, so collecting timings never stalls the stream
    hipEvent_t ev[2][EV_POOL];
    int ev_mode[2][EV_POOL / 2];
    hipEvent_t ev_frame[2][2];
    int ev_used[2] = {0, 0};
    bool ev_pending[2] = {false, false};
    uint32_t frames_submitted = 0;
    uint32_t trace_launches = 0;
    uint32_t frames = 0;
    double stage_ms[KT_COUNT] = {};
    uint32_t stage_launches[KT_COUNT] = {};
    double frame_ms = 0.0;
    // raw traces
    DBuf<float4> raw_o, raw_d, raw_hit;
    DBuf<uint8_t> raw_occ;
    // one process per GPU (mpt_comm_*): the RCCL communicator of the frame partition and the
    // padded staging rows of mpt_comm_gather (send: this rank's rows, recv: every rank's, root)
    void* comm = nullptr;
    int comm_rank = 0, comm_size = 1;
    // the library's own halo exchange (mpt_set_halo_native): 1 RCCL send / receive over the
    // communicator, 2 the one-GPU rehearsal (the bytes moved locally, no peers)
    int halo_native = 0;
    DBuf<uint8_t> halo_scratch;           // rehearsal: where the bytes go
    DBuf<int32_t> halo_agree;             // device word of the halo agreement (ncclAllReduce max)
    std::vector<MptHaloOp> halo_plan_ops; // the exchange point's operations (native_halo)
    uint64_t halo_exchanges = 0, halo_agreements = 0, halo_bytes_sent = 0, halo_bytes_recv = 0;   // MptStats
    uint32_t restir_overlapped_batches = 0;
    // upper bound of pixel_sample_count over the partition's pixels (restir_gate_static): a reset
    // frame restarts it, every frame with the adaptive buffers adds at most one sample; unknown
    // (large) until a reset frame has been launched
    int as_bound = 1 << 30;
    // the last batch reset the adaptive buffers in its k_accumulate (which an overlapped next batch
    // would run beside): the next ReSTIR DI batch does not overlap it
    bool as_reset_pending = false;
    DBuf<uint8_t> comm_send, comm_recv;
};

namespace {

DevScene dev_scene(MptContext* c) {
    DevScene S{};
    S.nodes = c->nodes.p;
    S.tris = c->tris.p;
    S.nodes_light = c->nodes_light.p;
    S.tris_light = c->tris_light.p;
    S.n_light_tris = (int32_t)c->h_light_prims.size();
    S.idx = c->idx.p;
    S.pos = c->pos.p;
    S.nrm = c->nrm.p;
    S.has_n = c->has_n.p;
    S.uv = c->uv.p;
    S.mat_idx = c->mat_idx.p;
    S.tri_attr = c->tri_attr.p;
    S.mats = c->mats.p;
    S.mats_res = c->mats_res.p;
    S.mat_tex = c->mat_tex.p;
    S.mat_prio = c->mat_prio.p;
    S.emissive = c->emissive.p;
    S.em_tab = c->em_tab.p;
    S.n_emissive = (int32_t)c->emissive.n;
    S.n_tris = (int32_t)c->mat_idx.n;
    S.tex = c->tex.p;
    S.tex_off = c->tex_off.p;
    S.tex_dims = c->tex_dims.p;
    S.srgb = c->srgb.p;
    S.n_tex = c->n_tex;
    S.lut_conductor = c->lut_conductor.p;
    S.lut_glossy = c->lut_glossy.p;
    S.lut_glass = c->lut_glass.p;
    S.lut_glass_inv = c->lut_glass_inv.p;
    S.lut_thin_glass = c->lut_thin.p;
    S.lut_sheen = c->lut_sheen.p;
    S.env = c->env.p;
    S.alias = c->alias.p;
    S.env_rich = c->env_rich.p;
    S.env_w = c->env_w;
    S.env_h = c->env_h;
    S.env_sum = c->env_sum;
    S.env_cdf = c->env_cdf.p;
    S.env_cdf_sum = c->env_cdf_sum;
    return S;
}

DevPaths dev_paths(MptContext* c) {
    DevPaths P{};
    P.n = c->n_slots * c->batch;
    P.n_pix = c->n_slots;
    P.batch = c->batch;
    P.group = (c->batch > 1 && c->n_slots % 4 == 0) ? 4 : 1;
    P.res_x = c->res_x;
    P.ray_o = c->ray_o.p;
    P.ray_d = c->ray_d.p;
    P.hit = c->hit.p;
    P.hit_inside = c->hit_inside.p;
    P.hit_cls = c->hit_cls.p;
    P.rng = c->rng.p;
    P.seeds = c->seeds.p;
    P.thr = c->thr.p;
    P.col = c->col.p;
    P.vsA = c->vsA.p;
    P.vsB = c->vsB.p;
    P.alb = c->alb.p;
    P.nrm = c->nrmv.p;
    P.q0 = c->q0.p;
    P.q1 = c->q1.p;
    P.qh = c->qh.p;
    P.qm = c->qm.p;
    P.qf = c->qf.p;
    P.nq_light = c->nq_light.p;
    P.counters = c->counters.p;
    P.nthr = c->nthr.p; P.na = c->na.p; P.nb = c->nb.p; P.ndir = c->ndir.p; P.nris = c->nris.p; P.ne1 = c->ne1.p;
    P.ne2 = c->ne2.p;
    P.nq_stride = (int64_t)std::max(c->n_slots, 1) * (int64_t)std::max(c->batch_cap, 1);
    P.nq_o = c->nq_o.p;
    P.nq_d = c->nq_d.p;
    P.nq_tgt = c->nq_tgt.p;
    P.occ = c->occ.p;
    P.qmask = c->qmask.p;
    P.nhit = c->nhit.p;
    P.s_gn = c->s_gn.p;
    P.mat_slot = c->mat_slot.p;
    P.fb_color = c->fb_color.p;
    P.fb_albedo = c->fb_albedo.p;
    P.fb_normal = c->fb_normal.p;
    P.stack_spill = c->spill.p;
    P.stats = c->stats.p;
    P.ray_counts = c->ray_counts.p;
    P.as_count = c->as_count.p;
    P.as_sqlum = c->as_sqlum.p;
    P.as_conv = c->as_conv.p;
    P.active = c->active.p;
    P.status = c->status.p;
    P.gb_pos = c->gb_pos.p; P.gb_sn = c->gb_sn.p; P.gb_gn = c->gb_gn.p; P.gb_view = c->gb_view.p; P.gb_meta = c->gb_meta.p;
    P.gb_vsA = c->gb_vsA.p; P.gb_vsB = c->gb_vsB.p; P.gb_mat = c->gb_mat.p;
    P.pgb_pos = c->pgb_pos.p; P.pgb_sn = c->pgb_sn.p; P.pgb_gn = c->pgb_gn.p; P.pgb_view = c->pgb_view.p; P.pgb_meta = c->pgb_meta.p;
    P.pgb_vsA = c->pgb_vsA.p; P.pgb_vsB = c->pgb_vsB.p; P.pgb_mat = c->pgb_mat.p;
    P.gb_cs = c->gb_cs.p; P.pgb_cs = c->pgb_cs.p;
    P.rs_init = c->rs_init.p; P.rs_sp1 = c->rs_sp1.p; P.rs_sp2 = c->rs_sp2.p; P.rs_plights = c->rs_plights.p;
    P.rs_keep = c->rs_keep.p; P.rs_keep_n = (int64_t)std::max(c->n_slots, 1); P.rs_keep_on = 0;   // band pixels per sample
    P.rs_out = c->restir_out_sp2 == 1 ? c->rs_sp2.p : c->restir_out_sp2 == 2 ? c->rs_init.p : c->rs_sp1.p;
    P.rs_tin = P.rs_out;
    // contiguous band (ReSTIR DI across a partition) or the whole frame: slot s = pixel s + pix_off
    const bool part = c->band_c > 1;
    P.pix_off = part ? c->band_i * c->band_h * c->res_x : 0;
    P.rs_lo = P.pix_off;
    P.rs_hi = P.pix_off + c->n_slots;
    P.rs_conv = part ? c->rs_conv.p : c->as_conv.p;
    P.x_per = c->x_per;
    P.x_iter = c->x_iter;
    P.xq_o = c->xq_o.p; P.xq_d = c->xq_d.p; P.xq_hit = c->xq_hit.p; P.xq_occ = c->xq_occ.p; P.xq_flag = c->xq_flag.p;
    P.xrec = c->xrec.p; P.xl_any = c->xl_any.p; P.xl_cl = c->xl_cl.p; P.xl_light = c->xl_light.p;
    P.rq_o = c->rq_o.p; P.rq_d = c->rq_d.p; P.rq_key = c->rq_key.p; P.rq_occ = c->rq_occ.p; P.rq_list = c->rq_list.p;
    P.rq_items = c->rq_items.p; P.rq_meta = c->rq_meta.p; P.rq_rec = c->rq_rec.p;
    return P;
}

int rows_of(int res_y, int bh, int bi, int bc) {
    int r = 0;
    for (int y = 0; y < res_y; y++)
        if ((y / bh) % bc == bi) r++;
    return r;
}

template <typename... B>
void release_all(B&... b) { (b.release(), ...); }

// Allocation chain of one buffer group: stops at the first failure, which the caller
// reports after releasing the whole group (a half-allocated group is never kept).
struct Allocs {
    hipError_t e = hipSuccess;
    template <typename T>
    void operator()(DBuf<T>& b, size_t n) { if (e == hipSuccess) e = b.alloc(n); }
    void operator()(hipError_t r) { if (e == hipSuccess) e = r; }
};

// Bytes of path state per path slot (ensure_batch): ray_o, ray_d, hit, thr, col, alb, nrmv,
// nhit, s_gn (9 x 16), vsA + vsB (32), the NEE record planes (7 x 16), 4 staged NEE query rays (2 x 64), the
// compacted query entries (16), occlusion bytes (4), 6 queues (24), rng (4), seeds (8), hit_inside,
// qmask, active (3).  Textured scenes add a resolved material per slot.
constexpr size_t OVERLAP_AUTO_PATHS = (size_t)24 << 20;   // MPT_OVERLAP=-1: overlapped halves up to this many paths
constexpr size_t PIPELINE_PREFER_TRIS = (size_t)1 << 20;   // ... unless the scene has this many triangles (launch_batch)
constexpr size_t PATH_BYTES = 9 * 16 + 32 + 7 * 16 + 128 + 16 + 4 + 24 + 4 + 8 + 3;
// + the bounce pipeline's alternate set per slot (set_pipe): 7 NEE planes, 4 staged query rays,
// 2 col additions (16 B each ... 64 B), 4 query list entries, 2 shaded-list entries
constexpr size_t PIPE_BYTES = 7 * 16 + 2 * 64 + 2 * 16 + 16 + 8;

void release_batch(MptContext* c) {
    release_all(c->ray_o, c->ray_d, c->hit, c->hit_inside, c->hit_cls, c->rng, c->seeds, c->thr, c->col, c->vsA, c->vsB, c->alb, c->nrmv,
                c->q0, c->q1, c->qh, c->qm, c->qf, c->nq_light, c->nthr, c->na, c->nb, c->ndir, c->nris, c->ne1, c->ne2, c->nq_o,
                c->nq_d, c->nq_tgt, c->occ, c->nhit, c->s_gn, c->qmask, c->active,
                c->mat_slot);
    release_all(c->nthr2, c->na2, c->nb2, c->ndir2, c->nris2, c->ne12, c->ne22, c->nq_o2, c->nq_d2, c->ce, c->ce2, c->nq_tgt2,
                c->qh2, c->qf2);
    c->pipe_n = 0;
    c->batch_cap = 0;
}

// Path state (everything indexed by path slot) for `batch` samples per pixel of the
// partition (+ the per-slot resolved materials when `mat_slot`); grows on demand.  On a
// failure every path-state buffer is released (batch_cap = 0), so that the next call
// allocates again instead of launching on a half-allocated state.
// Both of the context's streams drained (before buffers an overlapped ReSTIR DI wavefront on
// stream2 may still read are released or reallocated)
static hipError_t drain(MptContext* c) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && c->stream2) e = hipStreamSynchronize(c->stream2);
    for (hipStream_t x : c->streamx)
        if (e == hipSuccess && x) e = hipStreamSynchronize(x);
    return e;
}

int ensure_batch(MptContext* c, int batch, bool mat_slot) {
    const size_t pix = (size_t)std::max(c->n_slots, 1);
    const bool have = batch <= c->batch_cap && c->ray_o.p;
    if (have && (!mat_slot || c->mat_slot.n >= pix * (size_t)c->batch_cap)) return MPT_OK;
    HIPCHK(drain(c));
    const int cap = have ? c->batch_cap : batch;
    const size_t N = pix * (size_t)cap;
    Allocs A;
    if (!have) {
        c->batch_cap = 0;
        A(c->ray_o, N); A(c->ray_d, N); A(c->hit, N); A(c->hit_inside, N); A(c->hit_cls, N); A(c->rng, N); A(c->seeds, N); A(c->thr, N); A(c->col, N);
        A(c->vsA, N); A(c->vsB, N); A(c->alb, N); A(c->nrmv, N); A(c->q0, N); A(c->q1, N); A(c->qh, N); A(c->qm, N); A(c->qf, N); A(c->nq_light, N);
        A(c->nthr, N); A(c->na, N); A(c->nb, N); A(c->ndir, N); A(c->nris, N); A(c->ne1, N); A(c->ne2, N);
        A(c->nq_o, 4 * N); A(c->nq_d, 4 * N); A(c->nq_tgt, 4 * N); A(c->occ, 4 * N); A(c->nhit, N); A(c->s_gn, N);
        A(c->qmask, N); A(c->active, N);
        if (A.e == hipSuccess) A(hipMemsetAsync(c->active.p, 0, N, c->stream));
    }
    if (mat_slot || c->mat_slot.p) A(c->mat_slot, N);
    if (A.e != hipSuccess) {
        release_batch(c);
        return alloc_fail(A.e, "path state for " + std::to_string(N) + " paths");
    }
    c->batch_cap = cap;
    return MPT_OK;
}

// Bytes per ext entry: query ray (32), result (16), records (32), occlusion + flag (2), list
// entries (12).
constexpr size_t EXT_ENTRY_BYTES = 32 + 16 + 32 + 2 + 12;

// Extended light sampling buffers for `batch` samples per pixel at `per` entries per slot
// (ext_layout); per == 0 leaves them unused (released).  A failure releases the group.
int ensure_ext(MptContext* c, int batch, int per, int iter) {
    c->x_per = 0;
    c->x_iter = 0;
    if (per == 0) {
        release_all(c->xq_o, c->xq_d, c->xq_hit, c->xrec, c->xq_occ, c->xq_flag, c->xl_any, c->xl_cl, c->xl_light);
        return MPT_OK;
    }
    const size_t E = (size_t)std::max(c->n_slots, 1) * (size_t)batch * (size_t)per;
    if (E >= ((size_t)1 << 31)) return fail(MPT_ERR_OUT_OF_MEMORY, "extended light sampling: more than 2^31 entries");
    if (c->xq_o.n < E) {
        HIPCHK(drain(c));
        Allocs A;
        A(c->xq_o, E); A(c->xq_d, E); A(c->xq_hit, E); A(c->xrec, 2 * E); A(c->xq_occ, E); A(c->xq_flag, E);
        A(c->xl_any, E); A(c->xl_cl, E); A(c->xl_light, E);
        if (A.e != hipSuccess) {
            release_all(c->xq_o, c->xq_d, c->xq_hit, c->xrec, c->xq_occ, c->xq_flag, c->xl_any, c->xl_cl, c->xl_light);
            return alloc_fail(A.e, "extended light sampling: " + std::to_string(E) + " entries");
        }
    }
    c->x_per = per;
    c->x_iter = iter;
    return MPT_OK;
}

// Framebuffers and adaptive-sampling buffers of a row partition (n_slots pixels).  The
// partition keys are set only once everything is allocated; a failure releases the group
// and leaves the context without a partition (the next frame allocates again).
int ensure_paths(MptContext* c, int rx, int ry, int bh, int bi, int bc) {
    const int rows = rows_of(ry, bh, bi, bc);
    const int n = rows * rx;
    const bool same = c->res_x == rx && c->res_y == ry && c->band_h == bh && c->band_i == bi && c->band_c == bc &&
                      c->n_slots == n && c->fb_color.p;
    if (same) return MPT_OK;
    HIPCHK(drain(c));
    release_batch(c);                       // sized for the previous partition
    c->res_x = c->res_y = c->n_slots = 0;   // no partition until the group below is complete
    c->as_bound = 1 << 30;
    const size_t N = (size_t)std::max(n, 1);
    hipStream_t st = c->stream;
    Allocs A;
    A(c->fb_color, 3 * N); A(c->fb_albedo, 3 * N); A(c->fb_normal, 3 * N);
    A(c->as_count, N); A(c->as_sqlum, N); A(c->as_conv, N);
    if (A.e == hipSuccess) {
        A(hipMemsetAsync(c->fb_color.p, 0, 3 * N * sizeof(float), st));
        A(hipMemsetAsync(c->fb_albedo.p, 0, 3 * N * sizeof(float), st));
        A(hipMemsetAsync(c->fb_normal.p, 0, 3 * N * sizeof(float), st));
        A(hipMemsetAsync(c->as_count.p, 0, N * sizeof(int32_t), st));
        A(hipMemsetAsync(c->as_sqlum.p, 0, N * sizeof(float), st));
        A(hipMemsetAsync(c->as_conv.p, 0xff, N * sizeof(int32_t), st));
    }
    if (A.e != hipSuccess) {
        release_all(c->fb_color, c->fb_albedo, c->fb_normal, c->as_count, c->as_sqlum, c->as_conv);
        return alloc_fail(A.e, "framebuffers for " + std::to_string(N) + " pixels");
    }
    c->res_x = rx; c->res_y = ry; c->band_h = bh; c->band_i = bi; c->band_c = bc; c->n_slots = n;
    return MPT_OK;
}

// Alpha-test flag of every triangle record (TriRec::pad0): the filter function's test
// (FilterFunction.h:19-48) can only reject a hit when alpha_opacity < 1 or the base
// colour texture has a texel with alpha < 255; all other triangles skip it for free.
int upload_alpha_flags(MptContext* c) {
    std::vector<uint8_t> mflag(c->h_mats.size());
    for (size_t i = 0; i < c->h_mats.size(); i++) {
        const MptMaterial& m = c->h_mats[i];
        int bt = m.base_color_texture_index;
        bool tex_alpha = bt >= 0 && bt < (int)c->h_tex_alpha.size() && c->h_tex_alpha[bt];
        mflag[i] = (m.alpha_opacity < 1.0f || tex_alpha) ? 1 : 0;
    }
    bool changed = false;
    for (TriRec& tr : c->bvh.tris) {
        int32_t prim;
        std::memcpy(&prim, &tr.prim_bits, 4);
        uint32_t f = mflag[c->h_mat_idx[prim]];
        uint32_t old;
        std::memcpy(&old, &tr.pad0, 4);
        if (old != f) { std::memcpy(&tr.pad0, &f, 4); changed = true; }
    }
    if (changed) {
        HIPCHK(c->tris.upload(c->bvh.tris.data(), c->bvh.tris.size(), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return MPT_OK;
}

// Light-hit BVH: the triangles whose emission, as evaluate_shadow_light_ray reads it
// (Intersect.h:293-410; shadow_light_hit in the kernels), can be non-black -- an emissive
// texture, or emission * strength with a positive channel.  A light-hit query (the BSDF
// ray of MIS / RIS / BSDF light sampling) only needs the closest hit when it is one of
// these: the closest hit among them, confirmed by an any-hit query over the whole scene
// for a nearer (or equally near, lower-index) triangle, equals the whole-scene closest hit
// whenever that one is a light, and every other outcome contributes nothing.  Rebuilt when
// a material edit changes the set; alpha-test flags as upload_alpha_flags.
#define LBCHK(expr)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) { herr = e_; return fail(MPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); } \
    } while (0)
static int build_light_bvh_impl(MptContext* c, hipError_t& herr) {
    std::vector<uint8_t> lit(c->h_mats.size()), aflag(c->h_mats.size());
    for (size_t i = 0; i < c->h_mats.size(); i++) {
        const MptMaterial& m = c->h_mats[i];
        const float k = m.emission_strength;
        lit[i] = (m.emission_texture_index != MPT_NO_TEXTURE || m.emission.r * k > 0.0f || m.emission.g * k > 0.0f ||
                  m.emission.b * k > 0.0f) ? 1 : 0;
        int bt = m.base_color_texture_index;
        bool tex_alpha = bt >= 0 && bt < (int)c->h_tex_alpha.size() && c->h_tex_alpha[bt];
        aflag[i] = (m.alpha_opacity < 1.0f || tex_alpha) ? 1 : 0;
    }
    std::vector<int32_t> prims;
    for (size_t t = 0; t < c->h_mat_idx.size(); t++)
        if (lit[c->h_mat_idx[t]]) prims.push_back((int32_t)t);
    hipStream_t st = c->stream;
    c->light_bvh_ok = false;   // until the set below is built and uploaded
    if (prims != c->h_light_prims || (!prims.empty() && !c->nodes_light.p)) {
        c->h_light_prims = prims;
        c->nodes_light.release();
        c->tris_light.release();
        if (!prims.empty()) {
            std::vector<int32_t> sub(3 * prims.size());
            for (size_t k = 0; k < prims.size(); k++)
                for (int j = 0; j < 3; j++) sub[3 * k + j] = c->h_idx[3 * (size_t)prims[k] + j];
            build_bvh8(c->h_pos.data(), sub.data(), (int32_t)prims.size(), c->bvh_light, 3, c->box_pad);
            if (2 * c->bvh_light.depth + 2 > std::min(MAX_STACK, c->light_bvh_max_stack)) {
                // too deep for the traversal stack: light-hit queries take the (exact)
                // whole-scene closest-hit path instead
                c->h_light_prims.clear();
                return MPT_OK;
            }
            for (TriRec& tr : c->bvh_light.tris) {   // subset index -> scene primitive
                int32_t k;
                std::memcpy(&k, &tr.prim_bits, 4);
                std::memcpy(&tr.prim_bits, &prims[k], 4);
            }
            LBCHK(c->nodes_light.upload(c->bvh_light.nodes.data(), c->bvh_light.nodes.size(), st));
        }
    }
    if (!prims.empty()) {
        for (TriRec& tr : c->bvh_light.tris) {
            int32_t prim;
            std::memcpy(&prim, &tr.prim_bits, 4);
            uint32_t f = aflag[c->h_mat_idx[prim]];
            std::memcpy(&tr.pad0, &f, 4);
        }
        LBCHK(c->tris_light.upload(c->bvh_light.tris.data(), c->bvh_light.tris.size(), st));
    }
    LBCHK(hipStreamSynchronize(st));
    c->light_bvh_ok = true;
    return MPT_OK;
}

#undef LBCHK
// A light BVH that cannot be allocated is an optimisation lost, not an error: the light-hit
// queries then take the exact whole-scene closest-hit path (light_bvh_ok false), so a
// material edit never fails half-applied because device memory is short.  Any other HIP
// error (a sticky fault of an earlier launch surfacing at the synchronize, a failed copy) is
// returned to the caller.
int build_light_bvh(MptContext* c) {
    hipError_t herr = hipSuccess;
    const int rc = build_light_bvh_impl(c, herr);
    if (rc == MPT_OK) return MPT_OK;
    c->nodes_light.release();
    c->tris_light.release();
    c->h_light_prims.clear();
    c->light_bvh_ok = false;
    if (herr != hipErrorOutOfMemory) return rc;
    (void)hipGetLastError();
    const hipError_t se = hipStreamSynchronize(c->stream);
    if (se != hipSuccess) return fail(MPT_ERR_HIP, std::string("build_light_bvh: ") + hipGetErrorString(se));
    g_err.clear();
    return MPT_OK;
}

// ReSTIR DI buffers (ReSTIRDIRenderPass::update / resize, ReSTIRDIRenderPass.cpp:130-205): the
// G-buffer pair, three reservoir buffers reset to empty reservoirs, the presampled lights.
// Zero-filled G-buffers decode as "never written" (see restir_di.h gb_surface).
void release_restir(MptContext* c) {
    release_all(c->gb_pos, c->gb_sn, c->gb_gn, c->gb_view, c->pgb_pos, c->pgb_sn, c->pgb_gn, c->pgb_view, c->gb_meta,
                c->pgb_meta, c->gb_vsA, c->gb_vsB, c->pgb_vsA, c->pgb_vsB, c->gb_mat, c->pgb_mat, c->gb_cs, c->pgb_cs, c->rs_init, c->rs_sp1,
                c->rs_sp2, c->rs_plights, c->rs_keep, c->rs_conv, c->rq_o, c->rq_d, c->rq_rec, c->rq_key, c->rq_occ, c->rq_list, c->rq_items, c->rq_meta,
                c->ci_pos, c->ci_sn, c->ci_gn, c->ci_view, c->ci_cs, c->ci_rs, c->ci_pl, c->ci_meta, c->ci_vsA, c->ci_vsB, c->ci_mat);
    c->ci_chunk = 1;
    c->restir_out_sp2 = 0;
}

// ReSTIR DI buffers: a failure releases all of them, so the next frame rebuilds the set.
int ensure_restir(MptContext* c, const MptFrame* f) {
    size_t N = (size_t)c->res_x * (size_t)c->res_y;   // frame-sized, indexed by pixel (band + halo used)
    const MptReSTIRDISettings& rd = f->render_settings.restir_di_settings;
    size_t npl = (size_t)std::max(1, rd.number_of_subsets * rd.subset_size);
    hipStream_t st = c->stream;
    Allocs A;
    // every reallocating branch first drains both streams: an overlapped ReSTIR DI wavefront on
    // stream2 may still read the G-buffer, reservoir and staged-ray planes (as in ensure_batch)
    bool drained = false;
    auto D = [&] { if (!drained) { A(drain(c)); drained = true; } };
    if (c->rs_init.n != 3 * N) {
        D();
        A(c->gb_pos, N); A(c->gb_sn, N); A(c->gb_gn, N); A(c->gb_view, N);
        A(c->pgb_pos, N); A(c->pgb_sn, N); A(c->pgb_gn, N); A(c->pgb_view, N);
        A(c->gb_meta, N); A(c->pgb_meta, N);
        A(c->gb_vsA, N); A(c->gb_vsB, N); A(c->pgb_vsA, N); A(c->pgb_vsB, N);
        A(c->gb_cs, 4 * N); A(c->pgb_cs, 4 * N);
        A(c->rs_init, 3 * N); A(c->rs_sp1, 3 * N); A(c->rs_sp2, 3 * N);
        if (A.e == hipSuccess) {
            for (DBuf<float4>* b : {&c->gb_pos, &c->gb_sn, &c->gb_gn, &c->gb_view, &c->pgb_pos, &c->pgb_sn, &c->pgb_gn, &c->pgb_view})
                A(hipMemsetAsync(b->p, 0, N * sizeof(float4), st));
            A(hipMemsetAsync(c->gb_meta.p, 0, N * sizeof(int4), st));
            A(hipMemsetAsync(c->pgb_meta.p, 0, N * sizeof(int4), st));
            A(hipMemsetAsync(c->gb_cs.p, 0, 4 * N * sizeof(float4), st));
            A(hipMemsetAsync(c->pgb_cs.p, 0, 4 * N * sizeof(float4), st));
            for (DBuf<uint4>* b : {&c->gb_vsA, &c->gb_vsB, &c->pgb_vsA, &c->pgb_vsB})
                A(hipMemsetAsync(b->p, 0, N * sizeof(uint4), st));
            A(launch_restir_fill(c->rs_init.p, (int)N, st));
            A(launch_restir_fill(c->rs_sp1.p, (int)N, st));
            A(launch_restir_fill(c->rs_sp2.p, (int)N, st));
        }
        c->restir_out_sp2 = 0;
    }
    if ((c->any_tex || f->bsdf_flags.white_furnace_mode) && c->gb_mat.n < N) {
        D();
        A(c->gb_mat, N);
        A(c->pgb_mat, N);
    }
    if (c->band_c > 1 && c->rs_conv.n != N) {
        D();
        A(c->rs_conv, N);
        if (A.e == hipSuccess) A(hipMemsetAsync(c->rs_conv.p, 0xff, N * sizeof(int32_t), st));
    }
    if (c->restir_staged) {
        // staged reuse passes: per pixel slot of the partition (ReSTIR frames trace one sample).
        // A chunk of samples' initial candidates (launch_frames_restir) stages one ray position
        // per (sample, pixel) item -- up to RS_RPP samples -- and two records and a metadata entry
        // per item; its G-buffer / reservoir / light planes are the ci_* buffers.  The chunk
        // follows the band's size: ~8 M items, so that a small band's launches fill the GPU (1/8
        // of 1080p: 12 samples) and a 1080p frame runs chunks of 4 (8.19 -> 8.05 ms/spp,
        // profiles/r05p_c4_whole_frame_chunk_ab.jsonl; chunks of 2 measured no faster); a band
        // of more than ~2 M pixels keeps one sample's chain at a time
        const size_t ns = (size_t)std::max(c->n_slots, 1);
        int ck = c->restir_chunk >= 0 ? c->restir_chunk : (int)(((size_t)8 << 20) / ns);
        if (c->restir_chunk < 0 && ck < 4) ck = 1;
        ck = std::max(1, std::min(ck, RS_RPP_HOST));
        if (c->rq_o.n != ns * RS_RPP_HOST) {
            D();
            A(c->rq_o, ns * RS_RPP_HOST); A(c->rq_d, ns * RS_RPP_HOST); A(c->rq_key, ns * RS_RPP_HOST);
            A(c->rq_occ, ns * RS_RPP_HOST); A(c->rq_list, ns * RS_RPP_HOST); A(c->rq_items, 2 * ns * RS_RPP_HOST);
        }
        if (c->rq_meta.n != ns * ck) {
            D();
            A(c->rq_meta, ns * ck); A(c->rq_rec, ns * std::max(RS_REC_HOST, 2 * ck));
        }
        const bool mat = c->any_tex || f->bsdf_flags.white_furnace_mode;
        if (ck > 1 && (c->ci_chunk != ck || c->ci_pos.n != ns * ck || (mat && c->ci_mat.n != ns * ck))) {
            D();
            const size_t m = ns * ck;
            A(c->ci_pos, m); A(c->ci_sn, m); A(c->ci_gn, m); A(c->ci_view, m); A(c->ci_meta, m);
            A(c->ci_vsA, m); A(c->ci_vsB, m); A(c->ci_cs, 4 * m); A(c->ci_rs, 3 * m);
            if (mat) A(c->ci_mat, m);
        }
        if (ck > 1 && c->ci_pl.n != 4 * npl * ck) { D(); A(c->ci_pl, 4 * npl * ck); }
        c->ci_chunk = ck;
        DevPaths& d = c->ci_dp;
        d.gb_pos = c->ci_pos.p; d.gb_sn = c->ci_sn.p; d.gb_gn = c->ci_gn.p; d.gb_view = c->ci_view.p; d.gb_meta = c->ci_meta.p;
        d.gb_vsA = c->ci_vsA.p; d.gb_vsB = c->ci_vsB.p; d.gb_mat = c->ci_mat.p; d.gb_cs = c->ci_cs.p;
        d.rs_init = c->ci_rs.p; d.rs_plights = c->ci_pl.p;
    }
    if (c->rs_plights.n != 4 * npl) {
        D();
        A(c->rs_plights, 4 * npl);
        if (A.e == hipSuccess) A(launch_restir_fill_lights(c->rs_plights.p, (int)npl, st));
    }
    if (A.e != hipSuccess) {
        release_restir(c);
        return alloc_fail(A.e, "ReSTIR DI buffers");
    }
    return MPT_OK;
}

int resolve_materials(MptContext* c) {
    size_t n = c->h_mats.size();
    HIPCHK(c->mats_res.alloc(n));
    HIPCHK(c->mat_tex.alloc(n));
    HIPCHK(c->em_tab.alloc(5 * std::max<size_t>(c->emissive.n, 1)));
    HIPCHK(launch_resolve_materials(dev_scene(c), c->mats_res.p, c->mat_tex.p, (int)n, c->em_tab.p, c->stream));
    std::vector<int32_t> t(n);
    HIPCHK(hipMemcpyAsync(t.data(), c->mat_tex.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->any_tex = c->any_glass = false;
    for (int32_t v : t) {
        c->any_tex |= (v & MT_TEXTURED) != 0;
        c->any_glass |= (v & MT_GLASS) != 0;
    }
    // the share of triangles with a textured material: above 1/4 the shading kernels hold a
    // textured vertex's resolved material in private memory (k_shade's MATP)
    size_t n_tex_tris = 0;
    for (int32_t mi : c->h_mat_idx) n_tex_tris += (mi >= 0 && (size_t)mi < n && (t[mi] & MT_TEXTURED)) ? 1 : 0;
    c->tex_tri_frac = c->h_mat_idx.empty() ? 0.0 : (double)n_tex_tris / (double)c->h_mat_idx.size();
    // each triangle's material class in its BVH record (TriRec::pad1): the path traversal
    // reports it with the hit (DevPaths::hit_cls), so k_split needs no material lookups
    bool changed = false;
    for (TriRec& tr : c->bvh.tris) {
        int32_t prim;
        std::memcpy(&prim, &tr.prim_bits, 4);
        const int32_t keep = 0x7f & ~(c->shade_texmetal ? 0 : MT_TEXMETAL);
        const uint32_t cls = (prim >= 0 && (size_t)prim < c->h_mat_idx.size()) ? (uint32_t)(t[c->h_mat_idx[prim]] & keep) : 0u;
        uint32_t old;
        std::memcpy(&old, &tr.pad1, 4);
        if (old != cls) { std::memcpy(&tr.pad1, &cls, 4); changed = true; }
    }
    if (changed) {
        HIPCHK(c->tris.upload(c->bvh.tris.data(), c->bvh.tris.size(), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return MPT_OK;
}

// Extended light sampling (mpt_internal.h): entries per light sample (*iter) and per path
// slot (returned), 0 when the frame's light sampling fits the four staged queries of a slot
// (one light sample; RIS with at most one BSDF candidate and no visibility target function).
constexpr int MAX_EXT_PER_SLOT = 2048;
int ext_layout(const MptFrame& f, int* iter) {
    const MptRenderSettings& rs = f.render_settings;
    int lss = f.options.direct_light_sampling;
    if (lss == MPT_LSS_RESTIR_DI) {   // later bounces (Lights.h:243-275); bounce 0 uses the reservoir
        switch (f.options.restir_di_later_bounces_sampling_strategy) {
        case MPT_RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT: lss = MPT_LSS_UNIFORM_ONE_LIGHT; break;
        case MPT_RESTIR_DI_LATER_BOUNCES_BSDF: lss = MPT_LSS_BSDF; break;
        case MPT_RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF: lss = MPT_LSS_MIS_LIGHT_BSDF; break;
        default: lss = MPT_LSS_RIS_BSDF_AND_LIGHT; break;
        }
    }
    const int nl = std::max(0, rs.ris_number_of_light_candidates), nb = std::max(0, rs.ris_number_of_bsdf_candidates);
    int it = 0;
    if (lss == MPT_LSS_UNIFORM_ONE_LIGHT || lss == MPT_LSS_BSDF) it = 1;
    else if (lss == MPT_LSS_MIS_LIGHT_BSDF) it = 2;
    else if (lss == MPT_LSS_RIS_BSDF_AND_LIGHT) it = 2 * nl + nb;
    const bool ext = rs.number_of_light_samples > 1 ||
                     (lss == MPT_LSS_RIS_BSDF_AND_LIGHT && (nb > 1 || f.options.ris_use_visibility));
    if (!ext || it == 0) it = 0;
    if (iter) *iter = it;
    return it * std::max(1, rs.number_of_light_samples);
}

int validate_frame(const MptFrame* f) {
    const MptRenderSettings& rs = f->render_settings;
    if (f->res_x <= 0 || f->res_y <= 0) return fail(MPT_ERR_INVALID_ARGUMENT, "resolution must be positive");
    if (f->band_height <= 0 || f->band_count <= 0 || f->band_index < 0 || f->band_index >= f->band_count)
        return fail(MPT_ERR_INVALID_ARGUMENT, "invalid row partition");
    if ((int64_t)f->res_x * f->res_y > MPT_MAX_WAVEFRONT_PATHS)
        return fail(MPT_ERR_UNSUPPORTED, "more than MPT_MAX_WAVEFRONT_PATHS pixels per frame");
    if (rs.nb_bounces < 0 || rs.nb_bounces > 64) return fail(MPT_ERR_INVALID_ARGUMENT, "nb_bounces out of range");
    if (rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate &&
        (rs.render_low_resolution_scaling < 1 || rs.render_low_resolution_scaling > 64))
        return fail(MPT_ERR_INVALID_ARGUMENT, "render_low_resolution_scaling must be in [1, 64]");
    // sample_many_lights / RIS (Lights.h:222-241, RIS.h:82-289); the UI ranges are 1-8 light
    // samples and 0-16 candidates (ImGuiSettingsWindow.cpp:787, 833), the bounds here 64
    if (rs.number_of_light_samples < 1 || rs.number_of_light_samples > 64)
        return fail(MPT_ERR_INVALID_ARGUMENT, "number_of_light_samples must be in [1, 64]");
    if (rs.ris_number_of_bsdf_candidates < 0 || rs.ris_number_of_bsdf_candidates > 64 ||
        rs.ris_number_of_light_candidates < 0 || rs.ris_number_of_light_candidates > 64)
        return fail(MPT_ERR_INVALID_ARGUMENT, "RIS candidate counts must be in [0, 64]");
    if (ext_layout(*f, nullptr) > MAX_EXT_PER_SLOT)
        return fail(MPT_ERR_UNSUPPORTED, "extended light sampling needs more than MAX_EXT_PER_SLOT entries per path");
    int lss = f->options.direct_light_sampling;
    if (lss < 0 || lss > MPT_LSS_RESTIR_DI) return fail(MPT_ERR_INVALID_ARGUMENT, "bad direct_light_sampling");
    if (lss == MPT_LSS_RESTIR_DI) {
        const MptReSTIRDISettings& rd = rs.restir_di_settings;
        if (f->band_count != 1 && (int64_t)f->band_height * f->band_count < f->res_y)
            return fail(MPT_ERR_UNSUPPORTED, "ReSTIR DI across a partition needs one contiguous band per context "
                                             "(band_height * band_count >= res_y)");
        const int lb = f->options.restir_di_later_bounces_sampling_strategy;
        if (lb < MPT_RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT || lb > MPT_RESTIR_DI_LATER_BOUNCES_RIS_BSDF_AND_LIGHT)
            return fail(MPT_ERR_INVALID_ARGUMENT, "ReSTIR DI: bad later-bounces sampling strategy");
        const int bw = f->options.restir_di_bias_correction_weights;
        if (bw < MPT_RESTIR_DI_BIAS_1_OVER_M || bw > MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE)
            return fail(MPT_ERR_INVALID_ARGUMENT, "ReSTIR DI: bad bias correction weights");
        if (rd.number_of_passes < 1 || rd.number_of_passes > 4)
            return fail(MPT_ERR_UNSUPPORTED, "ReSTIR DI: number_of_passes must be in [1, 4] (restir_di_seeds)");
        if (rd.number_of_subsets <= 0 || rd.subset_size <= 0 || rd.tile_size <= 0)
            return fail(MPT_ERR_INVALID_ARGUMENT, "ReSTIR DI: bad light presampling settings");
        if (rd.reuse_neighbor_count > 32 || rd.disocclusion_reuse_count > 32)
            return fail(MPT_ERR_UNSUPPORTED, "ReSTIR DI: at most 32 spatial neighbours");
    }
    if (f->options.bsdf_override != MPT_BSDF_NONE && f->options.bsdf_override != MPT_BSDF_LAMBERTIAN &&
        f->options.bsdf_override != MPT_BSDF_OREN_NAYAR)
        return fail(MPT_ERR_INVALID_ARGUMENT, "bsdf_override must be BSDF_NONE, BSDF_LAMBERTIAN or BSDF_OREN_NAYAR");
    return MPT_OK;
}

int collect_pool(MptContext* c, int p) {
    if (!c->ev_pending[p]) return MPT_OK;
    HIPCHK(hipEventSynchronize(c->ev_frame[p][1]));
    for (int i = 0; i + 1 < c->ev_used[p]; i += 2) {
        float ms = 0.0f;
        HIPCHK(hipEventElapsedTime(&ms, c->ev[p][i], c->ev[p][i + 1]));
        int m = c->ev_mode[p][i / 2];
        if (m >= 0 && m < KT_COUNT) { c->stage_ms[m] += ms; c->stage_launches[m]++; }
    }
    float fms = 0.0f;
    HIPCHK(hipEventElapsedTime(&fms, c->ev_frame[p][0], c->ev_frame[p][1]));
    c->frame_ms += fms;
    c->ev_pending[p] = false;
    return MPT_OK;
}

}  // namespace

extern "C" {

const char* mpt_last_error(void) { return g_err.c_str(); }
int mpt_version(void) { return 1; }

int mpt_abi_sizes(int32_t* out, int n) {
    int32_t s[7] = {(int32_t)sizeof(MptMaterial), (int32_t)sizeof(MptRenderSettings), (int32_t)sizeof(MptWorldSettings),
                    (int32_t)sizeof(MptCamera), (int32_t)sizeof(MptFrame), (int32_t)sizeof(MptScene),
                    (int32_t)sizeof(MptStats)};
    if (!out) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    for (int i = 0; i < n && i < 7; i++) out[i] = s[i];
    return MPT_OK;
}

int mpt_device_info(int device, char* name, int32_t name_cap, char* arch, int32_t arch_cap, int32_t* out_cus) {
    hipDeviceProp_t p;
    HIPCHK(hipGetDeviceProperties(&p, device));
    if (name && name_cap > 0) { std::strncpy(name, p.name, (size_t)name_cap - 1); name[name_cap - 1] = 0; }
    if (arch && arch_cap > 0) { std::strncpy(arch, p.gcnArchName, (size_t)arch_cap - 1); arch[arch_cap - 1] = 0; }
    if (out_cus) *out_cus = p.multiProcessorCount;
    return MPT_OK;
}

static_assert(sizeof(MptMaterial) == 332, "RendererMaterial mirror");
static_assert(sizeof(MptRenderSettings) == 304, "HIPRTRenderSettings mirror");
static_assert(sizeof(MptWorldSettings) == 200, "WorldSettings mirror");
static_assert(sizeof(MptCamera) == 196, "HIPRTCamera mirror");

int mpt_partition_rows(int32_t res_y, int32_t bh, int32_t bi, int32_t bc) {
    if (bh <= 0 || bc <= 0) return 0;
    return rows_of(res_y, bh, bi, bc);
}

static int create_context(MptContext* c, int device, void* hip_stream) {
    c->device = device;
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    c->grid = c->num_cus * MPT_TRACE_BLOCKS_PER_CU;   // persistent traversal / ReSTIR grids
    if (hip_stream) c->stream = (hipStream_t)hip_stream;
    else { HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)); c->own_stream = true; }
    HIPCHK(hipHostMalloc((void**)&c->h_frames, sizeof(MptFrame) * (FRAME_RING + 1)));
    HIPCHK(hipMalloc((void**)&c->d_frames, sizeof(MptFrame) * (FRAME_RING + 1)));   // + the graph's frame
    // second set: the second half of an overlapped batch; up to PIX_PARTS_MAX: the row parts of a
    // one-sample frame
    HIPCHK(c->counters.alloc(PIX_PARTS_MAX * CTR_COUNT));
    HIPCHK(hipMemsetAsync(c->counters.p, 0, PIX_PARTS_MAX * CTR_COUNT * sizeof(int32_t), c->stream));
    HIPCHK(c->fetch_raw.alloc(4));
    HIPCHK(c->stats.alloc(N_STATS));
    HIPCHK(hipMemsetAsync(c->stats.p, 0, N_STATS * sizeof(uint64_t), c->stream));
    HIPCHK(c->ray_counts.alloc(N_RAY_COUNTS));
    HIPCHK(c->status.alloc(4));
    HIPCHK(hipMemsetAsync(c->status.p, 0, 4 * sizeof(uint32_t), c->stream));
    HIPCHK(hipMemsetAsync(c->ray_counts.p, 0, N_RAY_COUNTS * sizeof(uint64_t), c->stream));
    // traversal spill stacks per lane of the largest persistent grid (path or list mode,
    // launch_trace_mode): TRACE_SPILL_BLOCKS_PER_CU blocks per CU
    HIPCHK(c->spill.alloc((size_t)c->num_cus * TRACE_SPILL_BLOCKS_PER_CU * TRAV_BLOCK * SPILL_WORDS));
    HIPCHK(c->srgb.alloc(256));
    HIPCHK(launch_srgb_table(c->srgb.p, c->stream));
    return MPT_OK;
}

// The timing events (two pools of EV_POOL), created on the first mpt_enable_stats that
// turns timing on: a context that never times its kernels holds none.  Handles already
// created are kept, so a retry after a failure resumes where it stopped.
static int ensure_events(MptContext* c) {
    for (int p = 0; p < 2; p++) {
        for (int i = 0; i < EV_POOL; i++)
            if (!c->ev[p][i]) HIPCHK(hipEventCreate(&c->ev[p][i]));
        for (int k = 0; k < 2; k++)
            if (!c->ev_frame[p][k]) HIPCHK(hipEventCreate(&c->ev_frame[p][k]));
    }
    return MPT_OK;
}

int mpt_create(int device, void* hip_stream, MptContext** out) {
    if (!out) return fail(MPT_ERR_INVALID_ARGUMENT, "out_ctx is NULL");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(MPT_ERR_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(MPT_ERR_INVALID_ARGUMENT, "device index out of range");
    MptContext* c = new MptContext();   // value-initialised: every handle starts null
    if (const char* e = std::getenv("MPT_SHADE_CLASSES")) c->shade_classes = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_STAGED")) c->restir_staged = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_MONO_REUSE")) c->restir_mono_reuse = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_BATCH")) c->restir_batch = std::atoi(e);
    if (const char* e = std::getenv("MPT_ADAPTIVE_BATCH")) c->adaptive_batch = std::atoi(e);
    if (const char* e = std::getenv("MPT_MAT_PRIVATE")) c->mat_private = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_OVERLAP")) c->restir_overlap = std::atoi(e);
    if (const char* e = std::getenv("MPT_GRAPHS")) c->graphs = std::atoi(e);
    if (const char* e = std::getenv("MPT_PIX_PARTS")) c->pix_parts = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_SIDE")) c->restir_side = std::atoi(e);
    if (const char* e = std::getenv("MPT_TRACE_AHEAD")) c->trace_ahead = std::atoi(e);
    if (const char* e = std::getenv("MPT_PIPELINE")) c->pipeline = std::atoi(e);
    if (const char* e = std::getenv("MPT_PIX_PIPE")) c->pix_pipe = std::atoi(e);
    if (const char* e = std::getenv("MPT_OVERLAP_AHEAD")) c->ovl_ahead = std::atoi(e);
    if (const char* e = std::getenv("MPT_RESTIR_MAX_BATCH"))
        c->restir_max_batch = std::max(1, std::min(RESTIR_MAX_BATCH, std::atoi(e)));
    if (const char* e = std::getenv("MPT_RESTIR_CHUNK")) c->restir_chunk = std::atoi(e);
    if (const char* e = std::getenv("MPT_SHADE_GLASS")) c->shade_glass = std::atoi(e);
    if (const char* e = std::getenv("MPT_SHADE_SPLIT")) c->shade_split = std::atoi(e);
    if (const char* e = std::getenv("MPT_SHADE_TEXMETAL")) c->shade_texmetal = std::atoi(e);
    if (const char* e = std::getenv("MPT_LIGHT_BVH")) c->light_bvh = std::atoi(e);
    if (const char* e = std::getenv("MPT_OVERLAP")) c->overlap = std::atoi(e);
    if (const char* e = std::getenv("MPT_LIGHT_BVH_MAX_STACK")) c->light_bvh_max_stack = std::atoi(e);
    int r = create_context(c, device, hip_stream);
    if (r != MPT_OK) {
        const std::string msg = g_err;
        mpt_destroy(c);                 // frees what was created before the failure
        g_err = msg;
        return r;
    }
    *out = c;
    return MPT_OK;
}

namespace {
void rccl_comm_destroy(void* comm);   // (mpt_comm_init, below)
}  // namespace

// Tolerates a partially created context (mpt_create's failure path).  Every device buffer
// is a DBuf, released by the context's destructor on the context's device.
int mpt_destroy(MptContext* c) {
    if (!c) return MPT_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) rccl_comm_destroy(c->comm);
    for (int p = 0; p < 2; p++) {
        for (int i = 0; i < EV_POOL; i++)
            if (c->ev[p][i]) (void)hipEventDestroy(c->ev[p][i]);
        for (int k = 0; k < 2; k++)
            if (c->ev_frame[p][k]) (void)hipEventDestroy(c->ev_frame[p][k]);
    }
    if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
    if (c->h_frames) (void)hipHostFree(c->h_frames);
    if (c->h_reproj) (void)hipHostFree(c->h_reproj);
    if (c->d_frames) (void)hipFree(c->d_frames);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    for (int k = 0; k < 2; k++) {
        if (c->streamx[k]) (void)hipStreamDestroy(c->streamx[k]);
        if (c->ev_joinx[k]) (void)hipEventDestroy(c->ev_joinx[k]);
        if (c->ev_side[k]) (void)hipEventDestroy(c->ev_side[k]);
        if (c->ev_ahead[k]) (void)hipEventDestroy(c->ev_ahead[k]);
        if (c->ev_ahead2[k]) (void)hipEventDestroy(c->ev_ahead2[k]);
    }
    for (hipEvent_t e : c->ev_nee)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {c->ev_fork, c->ev_first, c->ev_acc, c->ev_join, c->ev_chain, c->ev_half[0], c->ev_half[1],
                         c->ev_wave_join})
        if (e) (void)hipEventDestroy(e);
    delete c;
    (void)hipGetLastError();
    return MPT_OK;
}

int mpt_upload_scene(MptContext* c, const MptScene* s) {
    if (!c || !s) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (s->num_triangles <= 0 || s->num_vertices <= 0 || !s->triangle_indices || !s->vertices || !s->material_indices ||
        !s->materials || s->num_materials <= 0)
        return fail(MPT_ERR_INVALID_ARGUMENT, "scene has no geometry or materials");
    for (int64_t i = 0; i < 3 * (int64_t)s->num_triangles; i++)
        if (s->triangle_indices[i] < 0 || s->triangle_indices[i] >= s->num_vertices)
            return fail(MPT_ERR_INVALID_ARGUMENT, "triangle index out of range");
    for (int64_t i = 0; i < s->num_triangles; i++)
        if (s->material_indices[i] < 0 || s->material_indices[i] >= s->num_materials)
            return fail(MPT_ERR_INVALID_ARGUMENT, "material index out of range");
    for (int i = 0; i < s->num_emissive_triangles; i++)
        if (s->emissive_triangle_indices[i] < 0 || s->emissive_triangle_indices[i] >= s->num_triangles)
            return fail(MPT_ERR_INVALID_ARGUMENT, "emissive triangle index out of range");
    HIPCHK(hipSetDevice(c->device));
    // triangles per leaf child: 3 (MPT_BVH_LEAF, 1..4, development A/B)
    int max_leaf = 3;
    if (const char* e = std::getenv("MPT_BVH_LEAF")) max_leaf = std::max(1, std::min(4, std::atoi(e)));
    // per level: at most one node group and one postponed triangle group on the stack; a
    // tree too deep for the traversal stack is rebuilt with balanced splits from a smaller
    // depth on (test hook MPT_BVH_MAX_STACK: a lower limit)
    int stack_cap = MAX_STACK;
    if (const char* e = std::getenv("MPT_BVH_MAX_STACK")) stack_cap = std::max(4, std::min(MAX_STACK, std::atoi(e)));
    for (int sah_depth = 40;; sah_depth = sah_depth * 2 / 3) {
        build_bvh8(s->vertices, s->triangle_indices, s->num_triangles, c->bvh, max_leaf, -1.0f, sah_depth);
        if (2 * c->bvh.depth + 2 <= stack_cap || sah_depth == 0) break;
    }
    c->box_pad = scene_box_pad(s->vertices, s->num_triangles, s->triangle_indices);
    c->h_idx.assign(s->triangle_indices, s->triangle_indices + 3 * (size_t)s->num_triangles);
    c->h_pos.assign(s->vertices, s->vertices + 3 * (size_t)s->num_vertices);
    c->h_light_prims.clear();
    c->nodes_light.release();
    c->tris_light.release();
    if (2 * c->bvh.depth + 2 > stack_cap) return fail(MPT_ERR_UNSUPPORTED, "BVH8 deeper than the traversal stack");
    hipStream_t st = c->stream;
    HIPCHK(c->nodes.upload(c->bvh.nodes.data(), c->bvh.nodes.size(), st));
    HIPCHK(c->tris.upload(c->bvh.tris.data(), c->bvh.tris.size(), st));
    HIPCHK(c->idx.upload(s->triangle_indices, 3 * (size_t)s->num_triangles, st));
    HIPCHK(c->pos.upload(s->vertices, 3 * (size_t)s->num_vertices, st));
    std::vector<float> zeros3, zeros2;
    std::vector<uint8_t> zerosb;
    const float* nrm = s->vertex_normals;
    if (!nrm) { zeros3.assign(3 * (size_t)s->num_vertices, 0.0f); nrm = zeros3.data(); }
    const float* uv = s->texcoords;
    if (!uv) { zeros2.assign(2 * (size_t)s->num_vertices, 0.0f); uv = zeros2.data(); }
    const uint8_t* hn = s->has_vertex_normals;
    if (!hn) { zerosb.assign((size_t)s->num_vertices, 0); hn = zerosb.data(); }
    HIPCHK(c->nrm.upload(nrm, 3 * (size_t)s->num_vertices, st));
    HIPCHK(c->uv.upload(uv, 2 * (size_t)s->num_vertices, st));
    HIPCHK(c->has_n.upload(hn, (size_t)s->num_vertices, st));
    HIPCHK(c->mat_idx.upload(s->material_indices, (size_t)s->num_triangles, st));
    HIPCHK(c->tri_attr.alloc(5 * (size_t)s->num_triangles));
    HIPCHK(launch_tri_attr(dev_scene(c), c->tri_attr.p, st));
    c->h_mat_idx.assign(s->material_indices, s->material_indices + s->num_triangles);
    c->h_mats.assign(s->materials, s->materials + s->num_materials);
    HIPCHK(c->mats.upload(c->h_mats.data(), c->h_mats.size(), st));
    std::vector<int32_t> prio(s->num_materials);
    for (int i = 0; i < s->num_materials; i++) prio[i] = s->materials[i].dielectric_priority;
    HIPCHK(c->mat_prio.upload(prio.data(), prio.size(), st));
    if (s->num_emissive_triangles > 0) HIPCHK(c->emissive.upload(s->emissive_triangle_indices, (size_t)s->num_emissive_triangles, st));
    else { c->emissive.release(); }
    c->n_tex = s->num_textures;
    if (s->num_textures > 0) {
        std::vector<uint64_t> off(s->num_textures);
        uint64_t total = 0;
        for (int i = 0; i < s->num_textures; i++) {
            off[i] = total;
            total += (uint64_t)s->texture_dims[2 * i] * s->texture_dims[2 * i + 1] * 4;
        }
        std::vector<uint8_t> all(total);
        c->h_tex_alpha.assign(s->num_textures, 0);
        for (int i = 0; i < s->num_textures; i++) {
            size_t texels = (size_t)s->texture_dims[2 * i] * s->texture_dims[2 * i + 1];
            std::memcpy(all.data() + off[i], s->texture_data[i], texels * 4);
            for (size_t k = 0; k < texels && !c->h_tex_alpha[i]; k++) c->h_tex_alpha[i] = s->texture_data[i][4 * k + 3] < 255;
        }
        HIPCHK(c->tex.upload(all.data(), all.size(), st));
        HIPCHK(c->tex_off.upload(off.data(), off.size(), st));
        HIPCHK(c->tex_dims.upload(s->texture_dims, 2 * (size_t)s->num_textures, st));
        HIPCHK(hipStreamSynchronize(st));
    } else {
        c->h_tex_alpha.clear();
        HIPCHK(hipStreamSynchronize(st));
    }
    int rr = upload_alpha_flags(c);
    if (rr != MPT_OK) return rr;
    rr = build_light_bvh(c);
    if (rr != MPT_OK) return rr;
    rr = resolve_materials(c);
    if (rr != MPT_OK) return rr;
    c->has_scene = true;
    return MPT_OK;
}

int mpt_update_materials(MptContext* c, const MptMaterial* m, int32_t count) {
    if (!c || !m) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (!c->has_scene) return fail(MPT_ERR_NO_SCENE, "no scene uploaded");
    if (count != (int32_t)c->h_mats.size()) return fail(MPT_ERR_INVALID_ARGUMENT, "material count differs from the scene's");
    HIPCHK(hipSetDevice(c->device));
    c->h_mats.assign(m, m + count);
    HIPCHK(c->mats.upload(c->h_mats.data(), c->h_mats.size(), c->stream));
    std::vector<int32_t> prio(count);
    for (int i = 0; i < count; i++) prio[i] = m[i].dielectric_priority;
    HIPCHK(c->mat_prio.upload(prio.data(), prio.size(), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    int rr = upload_alpha_flags(c);
    if (rr != MPT_OK) return rr;
    rr = build_light_bvh(c);
    if (rr != MPT_OK) return rr;
    return resolve_materials(c);
}

int mpt_build_alias_table(const float* rgba, int32_t w, int32_t h, float* out_p, int32_t* out_a, float* out_sum) {
    // Image32Bit::compute_alias_table (Image/Image.cpp:579-659): Vose in double precision
    if (!rgba || w <= 0 || h <= 0 || !out_p || !out_a) return fail(MPT_ERR_INVALID_ARGUMENT, "bad alias-table arguments");
    size_t n = (size_t)w * h;
    std::vector<double> L(n);
    double sum = 0.0f;
    const float wts[3] = {0.3086f, 0.6094f, 0.0820f};
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            size_t i = (size_t)y * w + x;
            float l = 0.0f;
            for (int c = 0; c < 3; c++) l += rgba[i * 4 + c] * wts[c];
            L[i] = (double)l;
            sum += L[i];
        }
    if (out_sum) *out_sum = (float)sum;
    for (double& v : L) { v /= sum; v *= (double)(w * h); }
    std::deque<int> small, large;
    for (size_t i = 0; i < n; i++) (L[i] < 1.0 ? small : large).push_back((int)i);
    while (!small.empty() && !large.empty()) {
        int s = small.front(), l = large.front();
        small.pop_front();
        large.pop_front();
        out_p[s] = (float)L[s];
        out_a[s] = l;
        L[l] = (L[l] + L[s]) - 1.0;
        (L[l] > 1.0 ? large : small).push_back(l);
    }
    while (!large.empty()) { out_p[large.front()] = 1.0f; large.pop_front(); }
    while (!small.empty()) { out_p[small.front()] = 1.0f; small.pop_front(); }
    return MPT_OK;
}

int mpt_set_envmap(MptContext* c, const float* rgba, int32_t w, int32_t h, const float* probas, const int32_t* alias, float lsum) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    HIPCHK(hipSetDevice(c->device));
    if (!rgba || w <= 0 || h <= 0) {
        c->env.release(); c->alias.release(); c->env_cdf.release(); c->env_rich.release();
        c->env_w = c->env_h = 0;
        return MPT_OK;
    }
    if (!probas || !alias) return fail(MPT_ERR_INVALID_ARGUMENT, "alias table required (ESS_ALIAS_TABLE)");
    size_t n = (size_t)w * h;
    for (size_t i = 0; i < n; i++)
        if (alias[i] < 0 || (size_t)alias[i] >= n) {
            // entries never reached by Vose's loop keep probability 1 and are never aliased
            if (probas[i] < 1.0f) return fail(MPT_ERR_INVALID_ARGUMENT, "alias index out of range");
        }
    // interleaved (probability, alias) pairs: the sampler reads both with one load
    std::vector<int2> pa(n);
    for (size_t i = 0; i < n; i++) {
        int32_t a = (alias[i] < 0 || (size_t)alias[i] >= n) ? (int32_t)i : alias[i];
        int32_t pb;
        std::memcpy(&pb, &probas[i], 4);
        pa[i] = make_int2(pb, a);
    }
    HIPCHK(c->env.upload(reinterpret_cast<const float4*>(rgba), n, c->stream));
    HIPCHK(c->alias.upload(pa.data(), n, c->stream));
    c->env_w = w;
    c->env_h = h;
    {
        hipError_t e = c->env_rich.alloc(2 * n);
        if (e != hipSuccess) return alloc_fail(e, "envmap alias entries");
        DevScene S = dev_scene(c);
        S.env_rich = nullptr;
        HIPCHK(launch_env_rich(S, c->env_rich.p, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    c->env_sum = lsum;
    c->env_cdf.release();   // a new envmap invalidates a previous CDF
    return MPT_OK;
}

int mpt_build_envmap_cdf(const float* rgba, int32_t w, int32_t h, float* out_cdf, float* out_sum) {
    // Image32Bit::compute_cdf (Image/Image.cpp:553-574): float running sum of the texel
    // luminances in row-major order; the total is the last element (OrochiEnvmap.cpp:30-38)
    if (!rgba || w <= 0 || h <= 0 || !out_cdf) return fail(MPT_ERR_INVALID_ARGUMENT, "bad CDF arguments");
    const float wts[3] = {0.3086f, 0.6094f, 0.0820f};
    size_t n = (size_t)w * h;
    out_cdf[0] = 0.0f;
    for (size_t i = 0; i < n; i++) {
        float l = 0.0f;
        for (int k = 0; k < 3; k++) l += rgba[4 * i + k] * wts[k];
        out_cdf[i] = out_cdf[i > 0 ? i - 1 : 0] + l;
    }
    if (out_sum) *out_sum = out_cdf[n - 1];
    return MPT_OK;
}

int mpt_set_envmap_cdf(MptContext* c, const float* cdf, float total_sum) {
    if (!c || !cdf) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (!c->env.p) return fail(MPT_ERR_INVALID_ARGUMENT, "mpt_set_envmap first");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->env_cdf.upload(cdf, (size_t)c->env_w * c->env_h, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->env_cdf_sum = total_sum;
    return MPT_OK;
}

int mpt_set_luts(MptContext* c, const MptLuts* L) {
    if (!c || !L || !L->ggx_conductor_ess || !L->glossy_dielectric_ess || !L->ggx_glass_ess || !L->ggx_glass_inverse_ess ||
        !L->ggx_thin_glass_ess || !L->sheen_ltc_params)
        return fail(MPT_ERR_INVALID_ARGUMENT, "all six LUTs are required");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->lut_conductor.upload(L->ggx_conductor_ess, 128 * 128, c->stream));
    HIPCHK(c->lut_glossy.upload(L->glossy_dielectric_ess, 128 * 64 * 128, c->stream));
    HIPCHK(c->lut_glass.upload(L->ggx_glass_ess, 256 * 16 * 128, c->stream));
    HIPCHK(c->lut_glass_inv.upload(L->ggx_glass_inverse_ess, 256 * 16 * 128, c->stream));
    HIPCHK(c->lut_thin.upload(L->ggx_thin_glass_ess, 32 * 32 * 96, c->stream));
    HIPCHK(c->lut_sheen.upload(L->sheen_ltc_params, 32 * 32 * 3, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

int mpt_resize(MptContext* c, int32_t w, int32_t h) {
    if (!c || w <= 0 || h <= 0) return fail(MPT_ERR_INVALID_ARGUMENT, "bad resolution");
    HIPCHK(hipSetDevice(c->device));
    if ((int64_t)w * h > MPT_MAX_WAVEFRONT_PATHS) return fail(MPT_ERR_UNSUPPORTED, "more than MPT_MAX_WAVEFRONT_PATHS pixels");
    int r = ensure_paths(c, w, h, c->band_h, c->band_i, c->band_c);
    if (r != MPT_OK) return r;
    return ensure_batch(c, 1, false);
}

// Samples per pixel of one wavefront when mpt_render_frames is not given a maximum:
// MPT_DEFAULT_WAVEFRONT_PATHS paths per launch, within half of the device memory that is
// free or already held by this context's path state, at most MPT_MAX_BATCH.
static int default_batch(MptContext* c, const MptFrame& f) {
    if (f.band_height <= 0 || f.band_count <= 0 || f.band_index < 0 || f.band_index >= f.band_count || f.res_x <= 0)
        return 1;
    const size_t pix = (size_t)std::max(1, rows_of(f.res_y, f.band_height, f.band_index, f.band_count)) * (size_t)f.res_x;
    // + the kept final reservoirs of a batched ReSTIR DI wavefront under an envmap (rs_keep: 3 float4
    // per pixel and sample, see prepare_batch)
    const bool keep = f.options.direct_light_sampling == MPT_LSS_RESTIR_DI &&
                      f.world_settings.ambient_light_type == MPT_AMBIENT_ENVMAP;
    const size_t per = PATH_BYTES + (c->pipeline ? PIPE_BYTES : 0) + ((c->any_tex || f.bsdf_flags.white_furnace_mode) ? sizeof(MptMaterial) : 0) +
                       EXT_ENTRY_BYTES * (size_t)ext_layout(f, nullptr) + (keep ? 3 * sizeof(float4) : 0);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); fr = 0; }
    const size_t held = (size_t)c->batch_cap * (size_t)std::max(c->n_slots, 1) * per;
    const size_t paths = std::min<size_t>(MPT_DEFAULT_WAVEFRONT_PATHS, (fr + held) / 2 / per);
    size_t b = std::max<size_t>(1, std::min<size_t>(MPT_MAX_BATCH, paths / pix));
    const int xp = ext_layout(f, nullptr);   // ext entries of a launch stay below 2^31
    if (xp > 0) b = std::max<size_t>(1, std::min<size_t>(b, (((size_t)1 << 31) - 1) / (pix * (size_t)xp)));
    return (int)b;
}

// Validation and every allocation of a wavefront of `batch` consecutive samples
// (f[0..batch-1]); nothing is enqueued, so a failure leaves the stream untouched.
static int prepare_batch(MptContext* c, const MptFrame* f, int batch) {
    if (!c->has_scene) return fail(MPT_ERR_NO_SCENE, "no scene uploaded");
    if (!c->lut_conductor.p && f->options.bsdf_override == MPT_BSDF_NONE) return fail(MPT_ERR_INVALID_ARGUMENT, "Principled BSDF needs mpt_set_luts");
    int v = validate_frame(f);
    if (v != MPT_OK) return v;
    if (f->world_settings.ambient_light_type == MPT_AMBIENT_ENVMAP && !c->env.p)
        return fail(MPT_ERR_INVALID_ARGUMENT, "ENVMAP ambient light without mpt_set_envmap");
    if (f->world_settings.ambient_light_type == MPT_AMBIENT_ENVMAP && f->options.envmap_sampling == MPT_ESS_BINARY_SEARCH &&
        !c->env_cdf.p)
        return fail(MPT_ERR_INVALID_ARGUMENT, "ESS_BINARY_SEARCH without mpt_set_envmap_cdf");
    HIPCHK(hipSetDevice(c->device));
    int r = ensure_paths(c, f->res_x, f->res_y, f->band_height, f->band_index, f->band_count);
    if (r != MPT_OK) return r;
    const bool restir_part = f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && f->band_count > 1;
    if (restir_part && !c->halo_fn)
        return fail(MPT_ERR_INVALID_ARGUMENT, "ReSTIR DI across a partition needs mpt_set_halo_exchange");
    if (f->options.direct_light_sampling == MPT_LSS_RESTIR_DI) {
        r = ensure_restir(c, f);
        if (r != MPT_OK) return r;
    }
    if (f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && c->emissive.n == 0 &&
        (f->options.restir_di_later_bounces_sampling_strategy == MPT_RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT ||
         f->options.restir_di_later_bounces_sampling_strategy == MPT_RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF))
        return fail(MPT_ERR_UNSUPPORTED, "ReSTIR DI later bounces: uniform / MIS light sampling without emissive "
                                         "triangles picks from an empty list in the reference (Lights.h:22-220)");
    if ((int64_t)std::max(c->n_slots, 1) * batch > MPT_MAX_WAVEFRONT_PATHS)
        return fail(MPT_ERR_OUT_OF_MEMORY, "wavefront above MPT_MAX_WAVEFRONT_PATHS paths");
    // overlapped ReSTIR DI batches need both halves of the path state (2 x the batch); without
    // the room they run one after the other
    // (under adaptive sampling such batches run only while the gate is static, restir_gate_static:
    // the converged counts the next batch's chain reads are the ones the running batch's
    // k_accumulate rewrites unchanged -- unless that batch reset them)
    const MptRenderSettings& frs = f->render_settings;
    const bool adaptive = (frs.stop_pixel_noise_threshold > 0.0f || frs.enable_adaptive_sampling) && frs.accumulate;
    const bool want_overlap = f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && batch > 1 && c->restir_overlap &&
                              !(adaptive && c->as_reset_pending) &&
                              ext_layout(*f, nullptr) == 0 && (int64_t)std::max(c->n_slots, 1) * 2 * batch <= MPT_MAX_WAVEFRONT_PATHS;
    c->restir_overlap_ok = false;
    if (want_overlap) {
        // the second half sits at half the capacity
        const int cap = 2 * batch;
        r = ensure_batch(c, cap, c->any_tex || f->bsdf_flags.white_furnace_mode);
        if (r == MPT_OK) c->restir_overlap_ok = c->batch_cap / 2 >= batch;
        else { (void)hipGetLastError(); g_err.clear(); }
    }
    if (!c->restir_overlap_ok) {
        r = ensure_batch(c, batch, c->any_tex || f->bsdf_flags.white_furnace_mode);
        if (r != MPT_OK) return r;
    }
    // each sample's final reservoirs, for the batch's bounce-0 shading (launch_frames_restir):
    // only read when the envmap is the ambient light (the deferred first bounce), so only held then
    const bool keep = f->options.direct_light_sampling == MPT_LSS_RESTIR_DI &&
                      f->world_settings.ambient_light_type == MPT_AMBIENT_ENVMAP;
    if (!keep && c->rs_keep.p) {
        HIPCHK(drain(c));
        c->rs_keep.release();
    }
    // the band's pixels only; both halves' when overlapped (half 1 at half the capacity)
    const size_t keep_n = 3 * (size_t)std::max(c->n_slots, 1) * (size_t)(c->restir_overlap_ok ? c->batch_cap : batch);
    if (keep && batch > 1 && c->rs_keep.n < keep_n) {
        HIPCHK(drain(c));
        c->rs_keep.release();
        if (c->rs_keep.alloc(keep_n) != hipSuccess) {
            (void)hipGetLastError();
            return fail(MPT_ERR_OUT_OF_MEMORY, "ReSTIR DI batch reservoirs");
        }
    }
    int iter = 0;
    const int per = ext_layout(*f, &iter);
    return ensure_ext(c, batch, per, iter);
}

// The second stream, its events and traversal spill area (overlapped batches), on first use.
static int ensure_overlap(MptContext* c) {
    if (c->stream2) return MPT_OK;
    if (c->spill2.n != c->spill.n) HIPCHK(c->spill2.alloc(c->spill.n));
    for (hipEvent_t* e : {&c->ev_fork, &c->ev_first, &c->ev_acc, &c->ev_join, &c->ev_chain, &c->ev_half[0], &c->ev_half[1],
                          &c->ev_wave_join})
        if (!*e) HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));   // kept across a failed attempt
    HIPCHK(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    return MPT_OK;
}

static int join_waves(MptContext* c);

// The streams, spill areas and join events of row parts 3 and 4 (pix_parts), on first use.
static int ensure_pix_parts(MptContext* c, int parts) {
    int r = ensure_overlap(c);
    if (r != MPT_OK) return r;
    for (int k = 0; k + 2 < parts; k++) {
        if (c->spillx[k].n != c->spill.n) HIPCHK(c->spillx[k].alloc(c->spill.n));
        if (!c->ev_joinx[k]) HIPCHK(hipEventCreateWithFlags(&c->ev_joinx[k], hipEventDisableTiming));
        if (!c->streamx[k]) HIPCHK(hipStreamCreateWithFlags(&c->streamx[k], hipStreamNonBlocking));
    }
    return MPT_OK;
}

// The graph path of a one-sample path-tracing launch set (MptContext::graphs): (re)captured when
// the key changes, then replayed with the frame copied into the graph's fixed slot.
static hipError_t launch_frame_graph(MptContext* c, const DevPaths& P, const MptFrame* f, int slot, LaunchCfg& cfg) {
    const DevScene S = dev_scene(c);
    MptFrame k = *f;   // the fields the kernels read from the frame, not the host
    k.random_seed = 0;
    k.camera_random_seed = 0;
    std::memset(k.restir_di_seeds, 0, sizeof(k.restir_di_seeds));
    std::memset(&k.current_camera, 0, sizeof(MptCamera));
    std::memset(&k.prev_camera, 0, sizeof(MptCamera));
    k.render_settings.sample_number = 0;
    k.render_settings.denoiser_AOV_accumulation_counter = 0;
    k.render_settings.need_to_reset = false;
    k.render_settings.do_update_status_buffers = false;
    const int flags[9] = {cfg.grid_persistent, cfg.stats, cfg.shade_classes, cfg.light_bvh, cfg.light_static,
                          cfg.restir_staged, cfg.shade_glass, cfg.shade_split, cfg.mat_private};
    std::vector<uint8_t> key(sizeof(k) + sizeof(S) + sizeof(P) + sizeof(flags));
    uint8_t* q = key.data();
    std::memcpy(q, &k, sizeof(k)); q += sizeof(k);
    std::memcpy(q, &S, sizeof(S)); q += sizeof(S);
    std::memcpy(q, &P, sizeof(P)); q += sizeof(P);
    std::memcpy(q, flags, sizeof(flags));
    MptFrame* d_fixed = c->d_frames + FRAME_RING;
    hipError_t e = hipMemcpyAsync(d_fixed, c->h_frames + slot, sizeof(MptFrame), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    if (!c->graph_exec || key != c->graph_key) {
        if (c->graph_exec) { (void)hipGraphExecDestroy(c->graph_exec); c->graph_exec = nullptr; }
        hipGraph_t g = nullptr;
        e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
        if (e != hipSuccess) return e;
        LaunchCfg gc = cfg;
        gc.launches = 0;
        const hipError_t le = launch_frame(S, P, d_fixed, *f, gc, c->stream);
        e = hipStreamEndCapture(c->stream, &g);
        if (le != hipSuccess || e != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            c->graphs = 0;   // not capturable here: launch directly from now on
            return launch_frame(S, P, c->d_frames + slot, *f, cfg, c->stream);
        }
        e = hipGraphInstantiate(&c->graph_exec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) {
            c->graph_exec = nullptr;
            (void)hipGetLastError();
            c->graphs = 0;
            return launch_frame(S, P, c->d_frames + slot, *f, cfg, c->stream);
        }
        c->graph_key = std::move(key);
        c->graph_launches = gc.launches;
        c->graph_captures++;
    }
    cfg.launches += c->graph_launches;
    c->graph_replays++;
    return hipGraphLaunch(c->graph_exec, c->stream);
}

static bool is_reset(const MptFrame& f) { return f.render_settings.sample_number == 0 || f.render_settings.need_to_reset; }
static bool has_adaptive(const MptFrame& f) {   // RenderSettings.h:207-218 (has_adaptive_buffers)
    const MptRenderSettings& rs = f.render_settings;
    return (rs.stop_pixel_noise_threshold > 0.0f || rs.enable_adaptive_sampling) && rs.accumulate;
}
static int next_as_bound(int b, const MptFrame& f) {
    if (!has_adaptive(f)) return b;
    if (is_reset(f)) b = 0;
    return b < (1 << 30) ? b + 1 : b;
}
// The trace-ahead stream of a single-stream wavefront (frame_bounces): streamx[1], its spill area
// and events, on first use
// (which = 1: streamx[0] with its own events, for the first half of an overlapped batch, whose
// second half takes streamx[1])
static int set_ahead(MptContext* c, LaunchCfg& cfg, const MptFrame& f, int which = 0) {
    if (!c->trace_ahead || f.render_settings.nb_bounces <= 0) return MPT_OK;
    int rr = ensure_pix_parts(c, 4);   // (streamx[0..1] and their spill areas)
    if (rr != MPT_OK) return rr;
    hipEvent_t* evs = which ? c->ev_ahead2 : c->ev_ahead;
    for (int k = 0; k < 2; k++)
        if (!evs[k]) HIPCHK(hipEventCreateWithFlags(&evs[k], hipEventDisableTiming));
    cfg.ahead_stream = which ? c->streamx[0] : c->streamx[1];
    cfg.ahead_spill = which ? c->spillx[0].p : c->spillx[1].p;
    cfg.ev_ahead_fork = evs[0];
    cfg.ev_ahead_join = evs[1];
    return MPT_OK;
}

// The bounce pipeline of a single-stream wavefront (LaunchCfg::pipe_alt, frame_bounces): the
// alternate plane set for the path slots the context holds (allocated on first use; a failure to
// allocate leaves the wavefront in line), its view `alt` of P, the NEE stream, its spill area and
// events.  P.ce is set: the shading hands its col additions to k_resolve.  `part` k of a
// pipelined one-sample frame in row parts (launch_batch, MPT_PIX_PIPE) takes NEE stream streamx[k]
// and the alternate counter set part + 2 (P: the part's slots, counters part; alt from the
// context's planes at the same slot offset `off`).
static bool pipe_applies(const MptContext* c, const MptFrame& f) {
    return c->pipeline && f.options.direct_light_sampling != MPT_LSS_RESTIR_DI && c->x_per == 0 && !c->shade_split &&
           f.render_settings.nb_bounces > 0;
}
static int set_pipe(MptContext* c, LaunchCfg& cfg, const MptFrame& f, DevPaths& P, DevPaths& alt, int part = -1,
                    size_t off = 0) {
    if (!pipe_applies(c, f)) return MPT_OK;
    const size_t N = (size_t)std::max(c->n_slots, 1) * (size_t)c->batch_cap;
    if (c->pipe_n != N) {
        HIPCHK(drain(c));
        Allocs A;
        A(c->nthr2, N); A(c->na2, N); A(c->nb2, N); A(c->ndir2, N); A(c->nris2, N); A(c->ne12, N); A(c->ne22, N);
        A(c->nq_o2, 4 * N); A(c->nq_d2, 4 * N); A(c->ce, N); A(c->ce2, N);
        A(c->nq_tgt2, 4 * N); A(c->qh2, N); A(c->qf2, N);
        if (A.e != hipSuccess) {   // no room: this wavefront (and the next ones) in line
            (void)hipGetLastError();
            release_all(c->nthr2, c->na2, c->nb2, c->ndir2, c->nris2, c->ne12, c->ne22, c->nq_o2, c->nq_d2, c->ce, c->ce2,
                        c->nq_tgt2, c->qh2, c->qf2);
            c->pipe_n = 0;
            return MPT_OK;
        }
        c->pipe_n = N;
    }
    int rr = ensure_pix_parts(c, 4);   // (streamx[0], streamx[1] and their spill areas)
    if (rr != MPT_OK) return rr;
    for (hipEvent_t& ev : c->ev_nee)
        if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int k = std::max(part, 0);
    P.ce = c->ce.p + off;
    alt = P;
    alt.nthr = c->nthr2.p; alt.na = c->na2.p; alt.nb = c->nb2.p; alt.ndir = c->ndir2.p; alt.nris = c->nris2.p;
    alt.ne1 = c->ne12.p; alt.ne2 = c->ne22.p; alt.nq_o = c->nq_o2.p; alt.nq_d = c->nq_d2.p; alt.nq_tgt = c->nq_tgt2.p;
    alt.qh = c->qh2.p; alt.qf = c->qf2.p; alt.ce = c->ce2.p;
    if (off) {   // the part's slots of the alternate planes (as offset_slots does for P's)
        alt.nthr += off; alt.na += off; alt.nb += off; alt.ndir += off; alt.nris += off; alt.ne1 += off; alt.ne2 += off;
        alt.nq_o += off; alt.nq_d += off; alt.nq_tgt += 4 * off; alt.qh += off; alt.qf += off; alt.ce += off;
    }
    // (the queue counters are always taken from P)
    alt.counters = part < 0 ? P.counters + CTR_COUNT : P.counters + 2 * CTR_COUNT;
    cfg.pipe_alt = &alt;
    cfg.nee_stream = c->streamx[k];
    cfg.nee_spill = c->spillx[k].p;
    cfg.ev_nee_fork = c->ev_nee[2 * k];
    cfg.ev_nee_join = c->ev_nee[2 * k + 1];
    return MPT_OK;
}

// Enqueues a prepared wavefront (prepare_batch).
static int launch_batch(MptContext* c, const MptFrame* f, int batch) {
    const bool restir_part = f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && f->band_count > 1;
    // anything but the next overlapped ReSTIR DI batch uses the first half of the path state and
    // counter set: a wavefront still running on stream2 is joined first
    if (!(f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && batch > 1 && c->restir_overlap_ok)) {
        int jr = join_waves(c);
        if (jr != MPT_OK) return jr;
    }
    // One-sample frames of a whole-frame context (the interactive launch set: the reference's
    // samples_per_frame = 1, low-resolution frames, a moving camera) run as two row halves on two
    // streams: every pixel's path is independent and its accumulation touches only its own pixel,
    // so the halves need no ordering, and one half's kernels fill the other's launch tails (each
    // of the ~50 dependent launches of a sample otherwise drains the GPU before the next starts)
    // (MPT_PIX_PIPE: two parts, each pipelined, where the bounce pipeline applies -- batch-1 C3 5.24 ->
    // 5.15 ms/spp against three parts in line, profiles/r06an_batch1_pix_pipe_ab.json)
    const int parts_set = c->pix_pipe && pipe_applies(c, *f) ? std::min(c->pix_parts, 2) : c->pix_parts;
    const int parts = std::min(std::max(parts_set, 1), std::min(PIX_PARTS_MAX, f->res_y));
    const bool pix_ovl = parts > 1 && batch == 1 && f->band_count == 1 && c->n_slots >= (1 << 16) &&
                         f->options.direct_light_sampling != MPT_LSS_RESTIR_DI && c->x_per == 0 &&
                         !(c->graphs && !c->timing);
    const int nfr = batch + (pix_ovl ? parts - 1 : 0);
    // stage the frame constants through a pinned ring (the previous use of the slot
    // has completed once 64 frames later are enqueued; synchronise defensively)
    if (c->frame_slot + nfr > FRAME_RING) c->frame_slot = 0;
    int slot = c->frame_slot;
    c->frame_slot = (c->frame_slot + nfr) % FRAME_RING;
    if (slot == 0) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->stream2) HIPCHK(hipStreamSynchronize(c->stream2));   // an overlapped wavefront reads its frames
    }
    for (int k = 0; k < batch; k++) c->h_frames[slot + k] = f[k];
    // row part k's frame: rows [k hp, (k + 1) hp) as band k of `parts` bands of hp rows, so that
    // its slot s is pixel k hp W + s (slot_pixel); part 0 keeps the whole frame's (same mapping)
    const int hp = (f->res_y + parts - 1) / parts;
    if (pix_ovl) {
        for (int k = 1; k < parts; k++) {
            MptFrame& g = c->h_frames[slot + k];
            g = f[0];
            g.band_height = hp;
            g.band_index = k;
            g.band_count = parts;
        }
    }
    HIPCHK(hipMemcpyAsync(c->d_frames + slot, c->h_frames + slot, nfr * sizeof(MptFrame), hipMemcpyHostToDevice,
                          c->stream));
    int pool = (int)(c->frames_submitted & 1u);
    if (c->timing) {
        int rc = collect_pool(c, pool);
        if (rc != MPT_OK) return rc;
    }
    LaunchCfg cfg{};
    cfg.grid_persistent = c->grid;
    cfg.stats = c->instrumented ? 1 : 0;
    cfg.ev_pool = c->timing ? c->ev[pool] : nullptr;
    cfg.ev_mode = c->ev_mode[pool];
    cfg.ev_cap = EV_POOL;
    cfg.ev_used = 0;
    cfg.restir_out_sp2 = c->restir_out_sp2;
    cfg.shade_classes = c->shade_classes;
    cfg.restir_staged = c->restir_staged;
    cfg.restir_mono_reuse = c->restir_mono_reuse;
    if (c->ci_chunk > 1 && c->ci_pos.p && c->ci_pl.n >= 4 * (size_t)std::max(1, f->render_settings.restir_di_settings.number_of_subsets *
                                                                                     f->render_settings.restir_di_settings.subset_size) * c->ci_chunk) {
        cfg.ci_chunk = c->ci_chunk;
        cfg.ci_planes = &c->ci_dp;
    }
    // (a band of a split frame: its kernels are tail-bound -- 8-way 1080p C4 at 20 steps, slowest band
    // 1.734 -> 1.705 ms/spp; the whole 1080p frame measured 8.12 -> 8.17, so not there, r06e)
    if (f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && c->restir_staged &&
        (c->restir_side > 1 || (c->restir_side == 1 && c->n_slots <= (1 << 20)))) {
        int rr = ensure_pix_parts(c, 3);   // (streamx[0] and its spill area)
        if (rr != MPT_OK) return rr;
        for (hipEvent_t& ev : c->ev_side)
            if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        cfg.side_stream = c->streamx[0];
        cfg.side_spill = c->spillx[0].p;
        cfg.ev_side_fork = c->ev_side[0];
        cfg.ev_side_join = c->ev_side[1];
    }
    // (no glass-class material: k_split's glass list stays empty, so the kernel is not launched)
    cfg.shade_glass = c->shade_glass && c->any_glass;
    cfg.shade_split = c->shade_split;
    cfg.mat_private = c->mat_private >= 0 ? (c->mat_private != 0) : (c->tex_tri_frac >= 0.25);
    cfg.light_bvh = c->light_bvh && c->light_bvh_ok;
    cfg.light_static = !c->h_light_prims.empty() && 2 * c->bvh_light.depth + 2 <= TRAV_LDS_STACK;
    if (restir_part) {
        if (!c->h_reproj) HIPCHK(hipHostMalloc((void**)&c->h_reproj, sizeof(int32_t), hipHostMallocDefault));
        cfg.halo_fn = c->halo_fn;
        cfg.halo_user = c->halo_user;
        cfg.own_y0 = f->band_index * f->band_height;
        cfg.own_y1 = std::min(f->res_y, cfg.own_y0 + f->band_height);
        cfg.halo_prev = c->halo_prev;
        cfg.halo_rows = c->halo_prev;
        cfg.h_reproj = c->h_reproj;
    }
    if (c->timing) HIPCHK(hipEventRecord(c->ev_frame[pool][0], c->stream));
    c->batch = batch;
    DevPaths P = dev_paths(c);
    c->batch = 1;
    {
        const MptRenderSettings& rs = f->render_settings;
        P.spec_as = batch > 1 && (rs.stop_pixel_noise_threshold > 0.0f || rs.enable_adaptive_sampling) && rs.accumulate;
        // a pixel converges only at a gate with its count above the minimum, so while the bound on
        // the counts is at most the minimum no pixel has converged and none is left out
        P.spec_skip = P.spec_as && rs.enable_adaptive_sampling && c->as_bound > rs.adaptive_sampling_min_samples;
    }
    if (restir_part) {   // frame_begin maintains the band and the previous frame's halo rows
        P.rs_lo = std::max(0, cfg.own_y0 - cfg.halo_prev) * f->res_x;
        P.rs_hi = std::min(f->res_y, cfg.own_y1 + cfg.halo_prev) * f->res_x;
    }
    // (auto: small wavefronts, or many bounces -- the later bounces' short lists are tails too:
    // C5 at 4K and 16 bounces 8.93 -> 8.67 ms/spp, profiles/r05v_c5_overlap_ab.jsonl; but a
    // traversal-heavy scene's small wavefront gains more from the bounce pipeline, which needs the
    // single stream: one rank of the 8 / 4 / 2-way C3 split at 20 steps 0.597 / 1.083 / 2.033 ->
    // 0.584 / 1.065 / 2.016 ms/spp, while Cornell C1 / C2 and C5 keep the halves, 0.5-1.2 % better
    // there, profiles/r06x_rank_share_pipeline_ab.json, r06y_configs_halves_vs_pipeline_ab.json)
    // A large many-bounce wavefront, too, is faster in one stream with the pipeline: C5 (4K, 16
    // bounces) in 8 / 16-sample wavefronts 8.21-8.37 / 7.88-7.94 ms/spp as halves, 8.14-8.19 /
    // 7.81-7.84 pipelined (profiles/r06az_c5_halves_vs_pipeline_ab.json, r06al_*)
    const bool pipe_ok = c->pipeline && !c->shade_split && f->render_settings.nb_bounces > 0;
    const bool pipe_first = pipe_ok && c->mat_idx.n >= PIPELINE_PREFER_TRIS;
    const bool ovl_auto = ((size_t)batch * (size_t)std::max(c->n_slots, 1) <= OVERLAP_AUTO_PATHS && !pipe_first) ||
                          (f->render_settings.nb_bounces >= 8 && !pipe_ok);
    const bool ovl = (c->overlap > 0 || (c->overlap < 0 && ovl_auto)) && batch >= 2 &&
                     f->options.direct_light_sampling != MPT_LSS_RESTIR_DI && c->x_per == 0 && !P.spec_as;
    hipError_t e = hipSuccess;
    if (pix_ovl) {
        int rr = ensure_pix_parts(c, parts);
        if (rr != MPT_OK) return rr;
        // part 0 on the context's stream, part k on its own stream over its own slots (and
        // per-pixel buffers: slot == pixel at one sample), counters and traversal spill area
        HIPCHK(hipEventRecord(c->ev_fork, c->stream));
        LaunchCfg cur = cfg;
        int launches = 0;
        // MPT_PIX_PIPE: two parts, each with the bounce pipeline (its NEE work on streamx[k])
        const bool part_pipe = c->pix_pipe && parts == 2 && pipe_applies(c, *f);
        DevPaths alts[2];
        for (int k = 0; k < parts && e == hipSuccess; k++) {
            const size_t r0 = std::min((size_t)f->res_y, (size_t)k * hp), r1 = std::min((size_t)f->res_y, (size_t)(k + 1) * hp);
            const size_t off = r0 * (size_t)f->res_x, n = (r1 - r0) * (size_t)f->res_x;
            if (n == 0) continue;
            DevPaths Pk = P;
            Pk.n = Pk.n_pix = (int)n;
            if (k > 0) {
                offset_slots(Pk, off);
                Pk.fb_color += 3 * off; Pk.fb_albedo += 3 * off; Pk.fb_normal += 3 * off;
                Pk.as_count += off; Pk.as_sqlum += off; Pk.as_conv += off;
                Pk.counters += k * CTR_COUNT;
                Pk.stack_spill = k == 1 ? c->spill2.p : c->spillx[k - 2].p;
            }
            hipStream_t sk = k == 0 ? c->stream : k == 1 ? c->stream2 : c->streamx[k - 2];
            if (k > 0) HIPCHK(hipStreamWaitEvent(sk, c->ev_fork, 0));
            cur.pipe_alt = nullptr;
            cur.nee_stream = nullptr;
            if (part_pipe) {
                int rr2 = set_pipe(c, cur, *f, Pk, alts[k], k, k > 0 ? off : 0);
                if (rr2 != MPT_OK) return rr2;
                if (cur.pipe_alt) c->pipelined_batches++;
            }
            cur.launches = 0;
            e = launch_frame(dev_scene(c), Pk, c->d_frames + slot + k, k == 0 ? f[0] : c->h_frames[slot + k], cur, sk);
            launches += cur.launches;
        }
        for (int k = 1; k < parts; k++) {
            hipStream_t sk = k == 1 ? c->stream2 : c->streamx[k - 2];
            hipEvent_t ej = k == 1 ? c->ev_join : c->ev_joinx[k - 2];
            HIPCHK(hipEventRecord(ej, sk));
            HIPCHK(hipStreamWaitEvent(c->stream, ej, 0));
        }
        c->overlapped_batches++;
        cfg.ev_used = cur.ev_used;
        cfg.launches = launches;
    } else if (ovl) {
        int rr = ensure_overlap(c);
        if (rr != MPT_OK) return rr;
        // samples [0, b0) on the context's stream, [b0, batch) on stream2 over their own
        // slots, counters and traversal spill area; the second half starts once the first
        // half's camera-ray traversal is done and accumulates after the first half's
        const int b0 = batch / 2, b1 = batch - b0;
        c->batch = b0;
        DevPaths P0 = dev_paths(c);
        c->batch = b1;
        DevPaths P1 = dev_paths(c);
        c->batch = 1;
        offset_slots(P1, (size_t)std::max(c->n_slots, 1) * b0);
        P1.counters += CTR_COUNT;
        P1.stack_spill = c->spill2.p;
        HIPCHK(hipEventRecord(c->ev_fork, c->stream));
        HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
        LaunchCfg cfg0 = cfg;
        cfg0.ev_first_trace = c->ev_first;
        cfg0.ev_acc_done = c->ev_acc;
        if (c->ovl_ahead) {   // each half with a trace-ahead stream of its own (MPT_OVERLAP_AHEAD)
            int ra = set_ahead(c, cfg0, f[0], 1);
            if (ra != MPT_OK) return ra;
        }
        e = launch_frame(dev_scene(c), P0, c->d_frames + slot, f[0], cfg0, c->stream);
        LaunchCfg cfg1 = cfg0;
        cfg1.ev_first_trace = nullptr;
        cfg1.ev_acc_done = nullptr;
        cfg1.ev_acc_wait = c->ev_acc;
        cfg1.launches = 0;
        cfg1.ahead_launches = 0;
        cfg1.ahead_stream = nullptr;
        if (c->ovl_ahead) {
            int ra = set_ahead(c, cfg1, f[b0], 0);
            if (ra != MPT_OK) return ra;
        }
        HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_first, 0));
        if (e == hipSuccess) e = launch_frame(dev_scene(c), P1, c->d_frames + slot + b0, f[b0], cfg1, c->stream2);
        HIPCHK(hipEventRecord(c->ev_join, c->stream2));
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_join, 0));
        c->overlapped_batches++;
        cfg.ev_used = cfg1.ev_used;
        cfg.launches = cfg0.launches + cfg1.launches;
        cfg.ahead_launches = cfg0.ahead_launches + cfg1.ahead_launches;
    } else if (f->options.direct_light_sampling == MPT_LSS_RESTIR_DI && batch > 1) {
        int ra = set_ahead(c, cfg, *f);   // (the batch's later-bounce wavefront)
        if (ra != MPT_OK) return ra;
        P.group = std::max(c->n_slots, 1);   // slot = sample * pixels + pixel
        if (c->restir_overlap_ok) {
            int rr = ensure_overlap(c);
            if (rr != MPT_OK) return rr;
            const int h = c->restir_half;
            c->restir_half ^= 1;
            if (h) {   // the second half of the path state, counters and kept reservoirs
                const size_t off = (size_t)(c->batch_cap / 2) * (size_t)std::max(c->n_slots, 1);
                offset_slots(P, off);
                P.counters += CTR_COUNT;
                if (P.rs_keep) P.rs_keep += 3 * off;
            }
            // this half's previous wavefront must be done before the chain rewrites its slots
            if (c->ev_half_used[h]) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_half[h], 0));
            cfg.wave_stream = c->stream2;
            cfg.wave_spill = c->spill2.p;
            cfg.ev_chain = c->ev_chain;
            e = launch_frames_restir(dev_scene(c), P, c->d_frames + slot, c->h_frames + slot, batch, cfg, c->stream);
            HIPCHK(hipEventRecord(c->ev_half[h], c->stream2));
            c->ev_half_used[h] = true;
            c->wave_pending = true;
            c->restir_overlapped_batches++;
        } else {
            e = launch_frames_restir(dev_scene(c), P, c->d_frames + slot, c->h_frames + slot, batch, cfg, c->stream);
        }
    } else if (batch == 1 && c->graphs && !c->timing && f->options.direct_light_sampling != MPT_LSS_RESTIR_DI) {
        e = launch_frame_graph(c, P, f, slot, cfg);
    } else {
        int rr = set_ahead(c, cfg, *f);
        if (rr != MPT_OK) return rr;
        DevPaths alt{};
        rr = set_pipe(c, cfg, *f, P, alt);
        if (rr != MPT_OK) return rr;
        if (cfg.pipe_alt) c->pipelined_batches++;
        e = launch_frame(dev_scene(c), P, c->d_frames + slot, *f, cfg, c->stream);
    }
    c->ahead_launches += cfg.ahead_launches;
    c->restir_out_sp2 = cfg.restir_out_sp2;
    if (restir_part) c->halo_prev = cfg.halo_rows;
    if (e != hipSuccess) return fail(MPT_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    if (cfg.halo_rc != 0) return fail(MPT_ERR_HIP, "halo exchange callback failed (" + std::to_string(cfg.halo_rc) + ")");
    if (c->timing) {
        // (an overlapped ReSTIR DI batch ends with its wavefront on stream2)
        HIPCHK(hipEventRecord(c->ev_frame[pool][1], cfg.wave_stream ? cfg.wave_stream : c->stream));
        c->ev_used[pool] = cfg.ev_used;
        c->ev_pending[pool] = true;
    }
    c->frames_submitted++;
    c->frames += batch;
    c->as_reset_pending = false;
    for (int k = 0; k < batch; k++) {
        c->as_bound = next_as_bound(c->as_bound, f[k]);
        c->as_reset_pending |= batch > 1 && has_adaptive(f[k]) && is_reset(f[k]);
    }
    c->trace_launches += cfg.launches;
    return MPT_OK;
}

// do_render_low_resolution (RenderSettings.h:195-198): the settings the launches of a
// low-resolution frame see -- at most 3 bounces (FullPathTracer.h:117-122), RIS with one light
// and one BSDF candidate and no visibility in its target function (RIS.h:93-94, 162), ReSTIR DI
// initial candidates capped at one of each (InitialCandidates.h:420-421); these fields are read
// nowhere else.  (The initial candidates' visibility test, InitialCandidates.h:248-249, is
// skipped in the kernel: its option also feeds the spatial passes.)  The pixels a low-resolution
// frame renders are k_camera's (low_res_region).
static MptFrame low_res_frame(const MptFrame& f) {
    MptFrame e = f;
    MptRenderSettings& rs = e.render_settings;
    if (!(rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate)) return e;
    rs.nb_bounces = std::min(3, rs.nb_bounces);
    rs.ris_number_of_light_candidates = 1;
    rs.ris_number_of_bsdf_candidates = 1;
    e.options.ris_use_visibility = 0;
    MptReSTIRDISettings& rd = rs.restir_di_settings;
    rd.number_of_initial_light_candidates = std::min(1, rd.number_of_initial_light_candidates);
    rd.number_of_initial_bsdf_candidates = std::min(1, rd.number_of_initial_bsdf_candidates);
    return e;
}
static bool is_low_res(const MptFrame& f) {
    const MptRenderSettings& rs = f.render_settings;
    return rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate;
}

int mpt_render_frame(MptContext* c, const MptFrame* f) {
    if (!c || !f) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    const MptFrame e = low_res_frame(*f);
    int r = prepare_batch(c, &e, 1);
    return r != MPT_OK ? r : launch_batch(c, &e, 1);
}

// Frames that differ only in what GPURenderer::render changes between the samples of one
// call (GPURenderer.cpp:424-449: sample number, seeds, AOV counter, reset / status flags;
// ReSTIRDIRenderPass::launch's seeds and temporal-buffer clear, ReSTIRDIRenderPass.cpp:233-264)
// and need no per-sample feedback on the host (adaptive sampling and the stop-noise
// threshold gate each sample's camera rays on the previous ones) are rendered as one
// wavefront.  ReSTIR DI samples, whose reuse passes read the previous sample's reservoirs,
// run their first bounce one sample after the other (launch_frames_restir) and share the
// later bounces' wavefront; across a partition each sample's reuse passes exchange their halo
// in turn (the exchange callback fires per sample inside the batch, launch_frames_restir).
static bool batchable(const MptContext* c, const MptFrame& a, const MptFrame& b) {
    const bool restir = a.options.direct_light_sampling == MPT_LSS_RESTIR_DI;
    if (restir && !c->restir_batch) return false;
    if (is_low_res(a)) return false;   // interactive frames: one sample each (RenderWindow.cpp:798-802)
    const MptRenderSettings& rs = a.render_settings;
    // adaptive sampling / the stop-noise threshold: traced speculatively and gated in sample order
    // by k_accumulate (under ReSTIR DI only while the gate is static: restir_gate_static)
    if ((rs.stop_pixel_noise_threshold > 0.0f || rs.enable_adaptive_sampling) && rs.accumulate && !c->adaptive_batch)
        return false;
    MptFrame t = b;
    t.render_settings.sample_number = a.render_settings.sample_number;
    t.render_settings.denoiser_AOV_accumulation_counter = a.render_settings.denoiser_AOV_accumulation_counter;
    t.render_settings.need_to_reset = a.render_settings.need_to_reset;
    t.render_settings.do_update_status_buffers = a.render_settings.do_update_status_buffers;
    t.random_seed = a.random_seed;
    t.camera_random_seed = a.camera_random_seed;
    if (restir) {
        MptReSTIRDISettings& rd = t.render_settings.restir_di_settings;
        const MptReSTIRDISettings& ra = a.render_settings.restir_di_settings;
        rd.permutation_sampling_random_bits = ra.permutation_sampling_random_bits;
        rd.temporal_buffer_clear_requested = ra.temporal_buffer_clear_requested;
        std::memcpy(t.restir_di_seeds, a.restir_di_seeds, sizeof(t.restir_di_seeds));
    }
    return std::memcmp(&t, &a, sizeof(MptFrame)) == 0;
}

// Batched ReSTIR DI under adaptive sampling (CameraRays.h:93-125, AdaptiveSampling.h:11-104): the
// reuse passes of sample s read which pixels are active at s and the neighbours' converged counts
// (Utils.h:289-339), i.e. the gate of sample s, which needs the radiance of every earlier sample --
// known only after the batch's later bounces.  The gate is static while no pixel can reach its
// noise test (pixel_sample_count > adaptive_sampling_min_samples): it then refuses exactly the
// pixels that had converged before the batch (sticky) and passes the others, and the converged
// counts do not change.  So frame i + k may join a run starting at frame i when neither is a reset
// frame (a reset clears the converged counts the passes read) and the host's bound on
// pixel_sample_count before it, as_bound + k, is at most the minimum.  The stop-noise threshold
// alone never refuses a sample and the passes do not read its counts: always static.
// A run may also start with a reset frame: the passes read the converged counts -- which the
// batch's k_accumulate resets only at its end -- only at sample numbers of at least the minimum
// (restir_spatial_neighbor), so the run's sample numbers stay below it.
static bool restir_gate_static(const MptContext* c, const MptFrame* run, int k) {
    const MptFrame& a = run[0];
    const MptRenderSettings& rs = a.render_settings;
    if (a.options.direct_light_sampling != MPT_LSS_RESTIR_DI || !rs.enable_adaptive_sampling || !rs.accumulate) return true;
    if (is_reset(run[k])) return false;
    const int mn = rs.adaptive_sampling_min_samples;
    if (is_reset(a)) return k <= mn && a.render_settings.sample_number < mn && run[k].render_settings.sample_number < mn;
    return (int64_t)c->as_bound + k <= (int64_t)mn;
}

// The overlapped ReSTIR DI wavefronts of the call joined into the context's stream: everything
// later enqueued there (the next call, framebuffer reads, synchronisation) follows them.
static int join_waves(MptContext* c) {
    if (!c->wave_pending) return MPT_OK;
    c->wave_pending = false;
    HIPCHK(hipEventRecord(c->ev_wave_join, c->stream2));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_wave_join, 0));
    return MPT_OK;
}

int mpt_render_frames(MptContext* c, const MptFrame* frames, int32_t count, int32_t max_batch) {
    if (!c || !frames || count < 0) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument or negative count");
    if (count == 0) return MPT_OK;
    HIPCHK(hipSetDevice(c->device));   // default_batch sizes the wavefront from this device's free memory
    if (max_batch <= 0) max_batch = default_batch(c, frames[0]);
    max_batch = std::min<int32_t>(max_batch, MPT_MAX_BATCH);
    // batched ReSTIR DI runs each sample's first bounce in turn (its timing events per sample)
    if (frames[0].options.direct_light_sampling == MPT_LSS_RESTIR_DI) max_batch = std::min(max_batch, c->restir_max_batch);
    // the launches' view of low-resolution frames (low_res_frame), copied only when there is one
    std::vector<MptFrame> eff;
    for (int k = 0; k < count && eff.empty(); k++)
        if (is_low_res(frames[k])) {
            eff.reserve((size_t)count);
            for (int j = 0; j < count; j++) eff.push_back(low_res_frame(frames[j]));
        }
    if (!eff.empty()) frames = eff.data();
    int i = 0;
    while (i < count) {
        int b = 1;
        while (i + b < count && b < max_batch && batchable(c, frames[i], frames[i + b]) && restir_gate_static(c, frames + i, b)) b++;
        int r = prepare_batch(c, frames + i, b);
        // a wavefront that does not fit in device memory is halved (bit-identical result),
        // and the smaller size is kept for the rest of the call
        while (r == MPT_ERR_OUT_OF_MEMORY && b > 1) {
            b = (b + 1) / 2;
            max_batch = b;
            r = prepare_batch(c, frames + i, b);
        }
        if (r != MPT_OK) return r;
        r = launch_batch(c, frames + i, b);
        if (r != MPT_OK) { join_waves(c); return r; }
        i += b;
    }
    return join_waves(c);
}

int mpt_set_halo_exchange(MptContext* c, MptHaloExchangeFn fn, void* user) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    c->halo_native = 0;
    c->halo_fn = fn;
    c->halo_user = fn ? user : nullptr;
    return MPT_OK;
}

int mpt_synchronize(MptContext* c) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

int mpt_query_done(MptContext* c, int* done) {
    if (!c || !done) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess) *done = 1;
    else if (e == hipErrorNotReady) *done = 0;
    else return fail(MPT_ERR_HIP, hipGetErrorString(e));
    return MPT_OK;
}

int mpt_get_framebuffer(MptContext* c, int kind, float* dst, int dst_is_device) {
    if (!c || !dst) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    const float* src = kind == MPT_FB_COLOR ? c->fb_color.p : kind == MPT_FB_ALBEDO ? c->fb_albedo.p : kind == MPT_FB_NORMALS ? c->fb_normal.p : nullptr;
    if (!src) return fail(MPT_ERR_INVALID_ARGUMENT, "bad framebuffer kind or no frame rendered");
    HIPCHK(hipSetDevice(c->device));
    size_t bytes = 3 * (size_t)c->n_slots * sizeof(float);
    HIPCHK(hipMemcpyAsync(dst, src, bytes, dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

// ---------------------------------------------------------------------------------------
// Multi-GPU output (SURVEY.md §8b Outputs row; the reference renders on one device,
// main.cpp:57, and hands 'pixels' to OpenGL, GPURenderer.cpp:583-598).  A context holds its
// partition's rows band-major compact: compact row r is frame row ((r / bh) * bc + bi) * bh
// + r % bh.  Groups of bh rows therefore land at a stride of bc * bh frame rows, so one
// strided 2D copy moves all full groups of a band and a second one the partial last group.
// ---------------------------------------------------------------------------------------
namespace {

// element bytes and source buffer of a gather kind (MPT_FB_* or MPT_GATHER_AUX + MPT_AUX_*)
const void* gather_src(const MptContext* c, int kind, size_t& elem) {
    elem = 12;
    if (kind == MPT_FB_COLOR) return c->fb_color.p;
    if (kind == MPT_FB_ALBEDO) return c->fb_albedo.p;
    if (kind == MPT_FB_NORMALS) return c->fb_normal.p;
    elem = 4;
    if (kind == MPT_GATHER_AUX + MPT_AUX_SAMPLE_COUNT) return c->as_count.p;
    if (kind == MPT_GATHER_AUX + MPT_AUX_CONVERGED_SAMPLE_COUNT) return c->as_conv.p;
    if (kind == MPT_GATHER_AUX + MPT_AUX_SQUARED_LUMINANCE) return c->as_sqlum.p;
    elem = 0;
    return nullptr;
}

// Enqueues on `st` the copies of band (bh, bi, bc)'s compact rows `src` into the frame-sized
// row-major `dst` (rows of row_bytes).  Same-device, peer-accessible or host destinations take
// the strided 2D copies; otherwise one peer copy per group.
hipError_t scatter_band_rows(uint8_t* dst, const uint8_t* src, size_t row_bytes, int res_y, int bh, int bi, int bc,
                             hipMemcpyKind kind, bool per_group, int dst_dev, int src_dev, hipStream_t st) {
    const int full = std::max(0, (res_y / bh - bi + bc - 1) / bc);   // groups g with (g bc + bi + 1) bh <= res_y
    const size_t gbytes = (size_t)bh * row_bytes;
    if (per_group) {
        for (int g = 0; g < full; g++) {
            hipError_t e = hipMemcpyPeerAsync(dst + (size_t)(g * bc + bi) * gbytes, dst_dev, src + (size_t)g * gbytes, src_dev,
                                              gbytes, st);
            if (e != hipSuccess) return e;
        }
    } else if (full > 0) {
        hipError_t e = hipMemcpy2DAsync(dst + (size_t)bi * gbytes, (size_t)bc * gbytes, src, gbytes, gbytes, full, kind, st);
        if (e != hipSuccess) return e;
    }
    const int y0 = (full * bc + bi) * bh;   // the partial group, if this band owns it
    if (y0 < res_y) {
        const size_t bytes = (size_t)std::min(bh, res_y - y0) * row_bytes;
        hipError_t e = per_group ? hipMemcpyPeerAsync(dst + (size_t)y0 * row_bytes, dst_dev, src + (size_t)full * gbytes, src_dev, bytes, st)
                                 : hipMemcpyAsync(dst + (size_t)y0 * row_bytes, src + (size_t)full * gbytes, bytes, kind, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace

int mpt_gather(MptContext* const* ctxs, int32_t n, int32_t root, int kind, void* dst, int dst_is_device) {
    if (!ctxs || n <= 0 || !dst) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument or n <= 0");
    if (root < 0 || root >= n) return fail(MPT_ERR_INVALID_ARGUMENT, "root out of range");
    std::vector<int> seen(n, 0);
    size_t elem = 0;
    for (int k = 0; k < n; k++) {
        const MptContext* c = ctxs[k];
        if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context in ctxs");
        size_t e;
        if (!gather_src(c, kind, e)) return fail(MPT_ERR_INVALID_ARGUMENT, "bad gather kind or no frame rendered on a context");
        elem = e;
        if (c->res_x != ctxs[0]->res_x || c->res_y != ctxs[0]->res_y || c->band_h != ctxs[0]->band_h || c->band_c != n)
            return fail(MPT_ERR_INVALID_ARGUMENT, "contexts do not partition one frame into n bands (res, band_height, band_count == n)");
        if (c->band_i < 0 || c->band_i >= n || seen[c->band_i]++) return fail(MPT_ERR_INVALID_ARGUMENT, "band indices are not 0..n-1");
    }
    const int dev = ctxs[root]->device;
    const size_t row_bytes = (size_t)ctxs[0]->res_x * elem;
    for (int k = 0; k < n; k++) {
        MptContext* c = ctxs[k];
        HIPCHK(hipSetDevice(c->device));
        bool per_group = false;
        if (dst_is_device && c->device != dev) {
            int can = 0;
            HIPCHK(hipDeviceCanAccessPeer(&can, c->device, dev));
            if (can) {
                hipError_t e = hipDeviceEnablePeerAccess(dev, 0);
                if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
                else if (e != hipSuccess) return fail(MPT_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
            }
            per_group = !can;
        }
        size_t e;
        const uint8_t* src = (const uint8_t*)gather_src(c, kind, e);
        HIPCHK(scatter_band_rows((uint8_t*)dst, src, row_bytes, c->res_y, c->band_h, c->band_i, c->band_c,
                                 dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, per_group, dev, c->device, c->stream));
    }
    for (int k = 0; k < n; k++) {
        HIPCHK(hipSetDevice(ctxs[k]->device));
        HIPCHK(hipStreamSynchronize(ctxs[k]->stream));
    }
    return MPT_OK;
}

// ---- one process per GPU: RCCL, loaded on first use (libmpt itself links no RCCL) -------------
namespace {

struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    int (*get_unique_id)(void*) = nullptr;
    int (*comm_init_rank)(void**, int, const void*, int) = nullptr;   // ncclUniqueId passed by value: see init below
    int (*comm_destroy)(void*) = nullptr;
    int (*gather)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
    const char* (*error_string)(int) = nullptr;
    // the ReSTIR DI halo exchange (native_halo)
    int (*group_start)() = nullptr;
    int (*group_end)() = nullptr;
    int (*send)(const void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*recv)(void*, size_t, int, int, void*, hipStream_t) = nullptr;
    int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
};

Rccl* rccl_lib() {
    static Rccl r;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (r.tried) return &r;
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);   // the copy torch may already have mapped
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { r.why = std::string("cannot load librccl.so.1: ") + dlerror(); return &r; }
    r.get_unique_id = (int (*)(void*))dlsym(h, "ncclGetUniqueId");
    r.comm_destroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
    r.gather = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclGather");
    r.error_string = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
    r.comm_init_rank = (int (*)(void**, int, const void*, int))dlsym(h, "ncclCommInitRank");
    r.group_start = (int (*)())dlsym(h, "ncclGroupStart");
    r.group_end = (int (*)())dlsym(h, "ncclGroupEnd");
    r.send = (int (*)(const void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclSend");
    r.recv = (int (*)(void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclRecv");
    r.all_reduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclAllReduce");
    r.ok = r.get_unique_id && r.comm_destroy && r.gather && r.error_string && r.comm_init_rank;
    if (!r.ok) r.why = "librccl.so.1 lacks ncclGetUniqueId / ncclCommInitRank / ncclGather / ncclCommDestroy";
    return &r;
}

constexpr int NCCL_ID_BYTES = 128;   // NCCL_UNIQUE_ID_BYTES
struct NcclId { char internal[NCCL_ID_BYTES]; };
constexpr int NCCL_UINT8 = 1;        // ncclUint8
constexpr int NCCL_INT32 = 2;        // ncclInt32
constexpr int NCCL_MAX = 2;          // ncclMax

void rccl_comm_destroy(void* comm) {
    if (rccl_lib()->ok) (void)rccl_lib()->comm_destroy(comm);
}

int rccl_fail(int rc, const char* what) {
    return fail(MPT_ERR_HIP, std::string(what) + ": " + (rccl_lib()->error_string ? rccl_lib()->error_string(rc) : "rccl error"));
}

}  // namespace

int mpt_comm_unique_id(uint8_t* out, int32_t cap) {
    if (!out || cap < MPT_COMM_ID_BYTES) return fail(MPT_ERR_INVALID_ARGUMENT, "out must hold MPT_COMM_ID_BYTES bytes");
    Rccl& r = *rccl_lib();
    if (!r.ok) return fail(MPT_ERR_UNSUPPORTED, r.why);
    NcclId id;
    int rc = r.get_unique_id(&id);
    if (rc != 0) return rccl_fail(rc, "ncclGetUniqueId");
    std::memcpy(out, id.internal, MPT_COMM_ID_BYTES);
    return MPT_OK;
}

int mpt_comm_init(MptContext* c, int32_t nranks, int32_t rank, const uint8_t* id) {
    if (!c || !id) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (nranks <= 0 || rank < 0 || rank >= nranks) return fail(MPT_ERR_INVALID_ARGUMENT, "rank out of range");
    if (c->comm) return fail(MPT_ERR_INVALID_ARGUMENT, "the context already has a communicator");
    Rccl& r = *rccl_lib();
    if (!r.ok) return fail(MPT_ERR_UNSUPPORTED, r.why);
    HIPCHK(hipSetDevice(c->device));
    // ncclCommInitRank takes the 128-byte ncclUniqueId by value; on x86-64 (SysV) a struct
    // larger than 16 bytes is passed in memory, which is what this signature describes
    NcclId nid;
    std::memcpy(nid.internal, id, MPT_COMM_ID_BYTES);
    auto init = (int (*)(void**, int, NcclId, int))r.comm_init_rank;
    void* comm = nullptr;
    int rc = init(&comm, nranks, nid, rank);
    if (rc != 0) return rccl_fail(rc, "ncclCommInitRank");
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_size = nranks;
    return MPT_OK;
}

int mpt_comm_gather(MptContext* c, int32_t root, int kind, void* dst, int dst_is_device) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    if (!c->comm) return fail(MPT_ERR_INVALID_ARGUMENT, "no communicator (mpt_comm_init)");
    if (root < 0 || root >= c->comm_size) return fail(MPT_ERR_INVALID_ARGUMENT, "root out of range");
    if (c->comm_rank == root && !dst) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL dst on the root");
    size_t elem;
    const uint8_t* src = (const uint8_t*)gather_src(c, kind, elem);
    if (!src) return fail(MPT_ERR_INVALID_ARGUMENT, "bad gather kind or no frame rendered");
    const int n = c->comm_size;
    if (c->band_c != n || c->band_i != c->comm_rank)
        return fail(MPT_ERR_INVALID_ARGUMENT, "the frame's band partition must be (band_count, band_index) = (ranks, rank)");
    int mr = 0;
    for (int k = 0; k < n; k++) mr = std::max(mr, rows_of(c->res_y, c->band_h, k, n));
    const size_t row_bytes = (size_t)c->res_x * elem, part = (size_t)mr * row_bytes;
    HIPCHK(hipSetDevice(c->device));
    hipError_t ae = c->comm_send.alloc(part);
    if (ae != hipSuccess) return alloc_fail(ae, "gather staging");
    const size_t own = (size_t)c->n_slots * elem;
    HIPCHK(hipMemcpyAsync(c->comm_send.p, src, own, hipMemcpyDeviceToDevice, c->stream));
    if (own < part) HIPCHK(hipMemsetAsync(c->comm_send.p + own, 0, part - own, c->stream));
    uint8_t* recv = nullptr;
    if (c->comm_rank == root) {
        if ((ae = c->comm_recv.alloc(part * n)) != hipSuccess) return alloc_fail(ae, "gather staging");
        recv = c->comm_recv.p;
    }
    int rc = rccl_lib()->gather(c->comm_send.p, recv, part, NCCL_UINT8, root, c->comm, c->stream);
    if (rc != 0) return rccl_fail(rc, "ncclGather");
    if (c->comm_rank == root)
        for (int k = 0; k < n; k++)
            HIPCHK(scatter_band_rows((uint8_t*)dst, recv + (size_t)k * part, row_bytes, c->res_y, c->band_h, k, n,
                                     dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, false, c->device,
                                     c->device, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

// ---- the ReSTIR DI halo exchange in the library (mpt_set_halo_native) --------------------------
// Rank k of the communicator owns contiguous band k of the frame (band_height rows).  At each
// exchange point (mpt.h MptHaloExchange) the rows of every buffer that lie in a peer's halo go to
// it and the peers' rows in this band's halo come in: one ncclGroupStart / ncclSend / ncclRecv
// group on the context's stream (peer-to-peer over xGMI; the host does not wait).  The halo
// agreement is an ncclAllReduce (max) of one int read back by the host -- skipped when the
// library derived the halo from the frame alone (halo_agreed, a still camera).  Sends and
// receives with one peer are issued in buffer order on both sides, so they pair up.
namespace {
int band_overlap(int a0, int a1, int b0, int b1, int& lo, int& hi) {
    lo = std::max(a0, b0);
    hi = std::min(a1, b1);
    return lo < hi;
}
// The point-to-point operations of one exchange point for band k of n (band_height rows, the
// agreed halo h), in the order they are issued: per peer p != k in increasing order, per buffer
// i, this band's rows in p's upper then lower halo (sends), then p's rows in this band's upper
// then lower halo (receives).  Peer p derives its receives from k and sends to k in the same
// order, so the operations pair up (ncclSend / ncclRecv match in issue order per peer); the
// receive ranges are mpt.partition.halo_plan's (tests/test_halo_plan.py).
void halo_ops(int res_y, int bh, int n, int k, int h, int n_buffers, std::vector<MptHaloOp>& ops) {
    ops.clear();
    auto need = [&](int q, int& a0, int& a1, int& b0, int& b1) {   // band q's halo ranges
        const int q0 = std::min(res_y, q * bh), q1 = std::min(res_y, q0 + bh);
        a0 = std::max(0, q0 - h); a1 = q0; b0 = q1; b1 = std::min(res_y, q1 + h);
        return q0 < q1;
    };
    const int m0 = std::min(res_y, k * bh), m1 = std::min(res_y, m0 + bh);
    int a0, a1, b0, b1;
    const bool mine = need(k, a0, a1, b0, b1);
    for (int p = 0; p < n; p++) {
        if (p == k) continue;
        const int p0 = std::min(res_y, p * bh), p1 = std::min(res_y, p0 + bh);
        int c0, c1, d0, d1, lo, hi;
        const bool theirs = need(p, c0, c1, d0, d1);
        for (int i = 0; i < n_buffers; i++) {
            if (theirs && band_overlap(c0, c1, m0, m1, lo, hi)) ops.push_back({p, 0, i, lo, hi});
            if (theirs && band_overlap(d0, d1, m0, m1, lo, hi)) ops.push_back({p, 0, i, lo, hi});
            if (mine && band_overlap(a0, a1, p0, p1, lo, hi)) ops.push_back({p, 1, i, lo, hi});
            if (mine && band_overlap(b0, b1, p0, p1, lo, hi)) ops.push_back({p, 1, i, lo, hi});
        }
    }
}
int native_halo(void* user, MptHaloExchange* x) {
    MptContext* c = (MptContext*)user;
    hipStream_t st = (hipStream_t)x->stream;
    std::vector<MptHaloOp>& ops = c->halo_plan_ops;
    auto count = [&](int recv) {
        size_t bytes = 0;
        for (const MptHaloOp& o : ops)
            if (o.recv == recv) bytes += (size_t)(o.row_hi - o.row_lo) * (size_t)x->res_x * (size_t)x->bytes_per_pixel[o.buffer];
        return bytes;
    };
    if (c->halo_native == 2) {
        // rehearsal on one GPU: the bytes this rank would receive, moved by one device copy (an
        // exchange is one grouped send / receive); a moving camera's agreement waits as the
        // all-reduce's read-back would
        if (x->phase == MPT_HALO_GBUFFER && !x->halo_agreed && hipStreamSynchronize(st) != hipSuccess) return 1;
        halo_ops(x->res_y, c->band_h, std::max(1, c->band_c), c->band_i, x->halo_rows, x->n_buffers, ops);
        const size_t bytes = count(1);
        c->halo_exchanges++;
        c->halo_bytes_recv += bytes;
        c->halo_bytes_sent += count(0);
        if (bytes == 0) return 0;
        if (c->halo_scratch.n < 2 * bytes && c->halo_scratch.alloc(2 * bytes) != hipSuccess) return 1;
        return hipMemcpyAsync(c->halo_scratch.p + bytes, c->halo_scratch.p, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess ? 0 : 1;
    }
    Rccl& r = *rccl_lib();
    if (!c->comm || !r.send || !r.recv || !r.group_start || !r.group_end || !r.all_reduce) return 2;
    const int n = c->comm_size, k = c->comm_rank;
    if (c->band_c != n || c->band_i != k) return 4;   // rank k must render band k of ranks
    if (x->phase == MPT_HALO_GBUFFER && !x->halo_agreed) {
        if (c->halo_agree.n < 1 && c->halo_agree.alloc(1) != hipSuccess) return 1;
        int32_t v = x->halo_rows;
        if (hipMemcpyAsync(c->halo_agree.p, &v, sizeof(v), hipMemcpyHostToDevice, st) != hipSuccess) return 1;
        if (r.all_reduce(c->halo_agree.p, c->halo_agree.p, 1, NCCL_INT32, NCCL_MAX, c->comm, st) != 0) return 3;
        if (hipMemcpyAsync(&v, c->halo_agree.p, sizeof(v), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) return 1;
        x->halo_rows = v;
        c->halo_agreements++;
    }
    halo_ops(x->res_y, c->band_h, n, k, x->halo_rows, x->n_buffers, ops);
    c->halo_exchanges++;
    c->halo_bytes_recv += count(1);
    c->halo_bytes_sent += count(0);
    if (ops.empty()) return 0;
    int rc = r.group_start();
    for (size_t j = 0; j < ops.size() && rc == 0; j++) {
        const MptHaloOp& o = ops[j];
        uint8_t* buf = (uint8_t*)x->buffers[o.buffer];
        const size_t row = (size_t)x->res_x * (size_t)x->bytes_per_pixel[o.buffer];
        uint8_t* at = buf + (size_t)o.row_lo * row;
        const size_t len = (size_t)(o.row_hi - o.row_lo) * row;
        rc = o.recv ? r.recv(at, len, NCCL_UINT8, o.peer, c->comm, st) : r.send(at, len, NCCL_UINT8, o.peer, c->comm, st);
    }
    const int re = r.group_end();
    return rc != 0 ? 3 : (re != 0 ? 3 : 0);
}
}  // namespace

int mpt_halo_plan(int32_t res_y, int32_t band_height, int32_t band_count, int32_t band_index, int32_t halo_rows,
                  int32_t n_buffers, MptHaloOp* out, int32_t cap) {
    if (res_y <= 0 || band_height <= 0 || band_count <= 0 || band_index < 0 || band_index >= band_count || halo_rows < 0 ||
        n_buffers < 0 || n_buffers > MPT_HALO_MAX_BUFFERS || cap < 0 || (cap > 0 && !out))
        return fail(MPT_ERR_INVALID_ARGUMENT, "mpt_halo_plan: bad partition, halo or output");
    std::vector<MptHaloOp> ops;
    halo_ops(res_y, band_height, band_count, band_index, halo_rows, n_buffers, ops);
    for (size_t j = 0; j < ops.size() && (int32_t)j < cap; j++) out[j] = ops[j];
    return (int)ops.size();
}

int mpt_set_pipeline(MptContext* c, int32_t mode) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    if (mode < 0 || mode > 1) return fail(MPT_ERR_INVALID_ARGUMENT, "mode must be 0 (in line) or 1 (pipelined)");
    c->pipeline = mode;
    return MPT_OK;
}

int mpt_set_halo_native(MptContext* c, int32_t mode) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    if (mode < 0 || mode > 2) return fail(MPT_ERR_INVALID_ARGUMENT, "mode must be 0 (off), 1 (RCCL) or 2 (rehearsal)");
    if (mode == 1) {
        if (!c->comm) return fail(MPT_ERR_INVALID_ARGUMENT, "no communicator (mpt_comm_init)");
        Rccl& r = *rccl_lib();
        if (!r.send || !r.recv || !r.group_start || !r.group_end || !r.all_reduce)
            return fail(MPT_ERR_UNSUPPORTED, "librccl.so.1 lacks ncclSend / ncclRecv / ncclGroupStart / ncclAllReduce");
    }
    c->halo_native = mode;
    c->halo_fn = mode ? &native_halo : nullptr;
    c->halo_user = mode ? (void*)c : nullptr;
    return MPT_OK;
}

int mpt_clear_status(MptContext* c) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(c->status.p, 0, 4 * sizeof(uint32_t), c->stream));
    return MPT_OK;
}

int mpt_query_status(MptContext* c, MptStatus* out) {
    if (!c || !out) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    uint32_t v[4];
    HIPCHK(hipMemcpyAsync(v, c->status.p, sizeof(v), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->one_ray_active = v[1] != 0;
    out->pixel_converged_count = v[0];
    return MPT_OK;
}

int mpt_get_aux_buffer(MptContext* c, int kind, void* dst, int dst_is_device) {
    if (!c || !dst) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    const void* src = kind == MPT_AUX_SAMPLE_COUNT ? (const void*)c->as_count.p
                    : kind == MPT_AUX_CONVERGED_SAMPLE_COUNT ? (const void*)c->as_conv.p
                    : kind == MPT_AUX_SQUARED_LUMINANCE ? (const void*)c->as_sqlum.p : nullptr;
    size_t bytes = (size_t)c->n_slots * 4;
    if (kind >= MPT_AUX_RESTIR_OUTPUT && kind <= MPT_AUX_RESTIR_INITIAL && c->rs_init.p) {
        // the frame-sized ReSTIR DI reservoir buffers: the last frame's output, the other
        // spatial buffer (the fused pass's output when a spatial pass followed it), the
        // initial candidates
        const int o = c->restir_out_sp2;
        const float4* out = o == 1 ? c->rs_sp2.p : o == 2 ? c->rs_init.p : c->rs_sp1.p;
        src = kind == MPT_AUX_RESTIR_OUTPUT ? (const void*)out
            : kind == MPT_AUX_RESTIR_OTHER ? (const void*)(o == 1 ? c->rs_sp1.p : c->rs_sp2.p) : (const void*)c->rs_init.p;
        bytes = c->rs_init.n * sizeof(float4);
    }
    if (!src) return fail(MPT_ERR_INVALID_ARGUMENT, "bad aux buffer kind or no frame rendered");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

int mpt_enable_stats(MptContext* c, int enable, int instrumented) {
    if (!c) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (enable) {
        int r = ensure_events(c);
        if (r != MPT_OK) { c->timing = false; return r; }
    }
    c->timing = enable != 0;
    c->instrumented = instrumented != 0;
    c->ev_pending[0] = c->ev_pending[1] = false;
    c->trace_launches = 0;
    c->frames = 0;
    c->frame_ms = 0.0;
    c->graph_captures = c->graph_replays = 0;
    c->overlapped_batches = 0;
    c->halo_exchanges = c->halo_agreements = c->halo_bytes_sent = c->halo_bytes_recv = 0;
    c->restir_overlapped_batches = 0;
    c->ahead_launches = 0;
    c->pipelined_batches = 0;
    for (int m = 0; m < KT_COUNT; m++) { c->stage_ms[m] = 0.0; c->stage_launches[m] = 0; }
    HIPCHK(hipMemsetAsync(c->stats.p, 0, N_STATS * sizeof(uint64_t), c->stream));
    HIPCHK(hipMemsetAsync(c->ray_counts.p, 0, N_RAY_COUNTS * sizeof(uint64_t), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MPT_OK;
}

int mpt_get_stats(MptContext* c, MptStats* out) {
    if (!c || !out) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int p = 0; p < 2; p++) {
        int rc = collect_pool(c, p);
        if (rc != MPT_OK) return rc;
    }
    std::memset(out, 0, sizeof(*out));
    uint64_t s[N_STATS];
    HIPCHK(hipMemcpy(s, c->stats.p, sizeof(s), hipMemcpyDeviceToHost));
    uint64_t rc[N_RAY_COUNTS];
    HIPCHK(hipMemcpy(rc, c->ray_counts.p, sizeof(rc), hipMemcpyDeviceToHost));
    out->rays_closest = rc[0] + rc[2];
    out->rays_any = rc[1];
    for (int m = 0; m < 3; m++) {
        out->stage_rays[m] = rc[m];
        out->stage_traversals[m] = s[m * STATS_STRIDE + 0];
        out->stage_nodes[m] = s[m * STATS_STRIDE + 1];
        out->stage_tris[m] = s[m * STATS_STRIDE + 2];
        out->stage_node_slots[m] = s[m * STATS_STRIDE + 4];
        out->stage_tri_slots[m] = s[m * STATS_STRIDE + 5];
        out->node_visits += s[m * STATS_STRIDE + 1];
        out->triangle_tests += s[m * STATS_STRIDE + 2];
        out->stage_ms[m] = c->stage_ms[m];
        out->stage_launches[m] = c->stage_launches[m];
        out->trace_ms += c->stage_ms[m];
    }
    out->camera_ms = c->stage_ms[KT_CAMERA];
    out->shade_ms = c->stage_ms[KT_SHADE];
    out->resolve_ms = c->stage_ms[KT_RESOLVE];
    out->accumulate_ms = c->stage_ms[KT_ACCUMULATE];
    out->compact_ms = c->stage_ms[KT_COMPACT];
    out->restir_ms = c->stage_ms[KT_RESTIR];
    out->split_ms = c->stage_ms[KT_SPLIT];
    out->miss_ms = c->stage_ms[KT_MISS];
    out->path_hits = rc[3];
    out->shade_generic_vertices = rc[4];
    out->shade_generic_ms = c->stage_ms[KT_SHADE_GENERIC];
    out->shade_launches = c->stage_launches[KT_SHADE];
    for (int k = 0; k < 5; k++) {
        out->restir_kernel_ms[k] = c->stage_ms[KT_GBUFFER + k];
        out->restir_kernel_launches[k] = c->stage_launches[KT_GBUFFER + k];
    }
    out->restir_eval_ms = c->stage_ms[KT_RS_EVAL];
    out->restir_eval_launches = c->stage_launches[KT_RS_EVAL];
    out->restir_eval_items = rc[5];
    out->trace_launches = c->trace_launches;
    out->frames = c->frames;
    out->frame_ms = c->frame_ms;
    out->graph_captures = c->graph_captures;
    out->graph_replays = c->graph_replays;
    out->overlapped_batches = c->overlapped_batches;
    out->halo_exchanges = c->halo_exchanges;
    out->halo_agreements = c->halo_agreements;
    out->halo_bytes_sent = c->halo_bytes_sent;
    out->halo_bytes_received = c->halo_bytes_recv;
    out->restir_overlapped_batches = c->restir_overlapped_batches;
    out->trace_ahead_launches = c->ahead_launches;
    out->pipelined_batches = c->pipelined_batches;
    return MPT_OK;
}

// GPUBakerKernel::bake_internal (GPUBakerKernel.cpp:98-113): launches of ipk samples per texel,
// in float arithmetic as the reference computes them; nb_samples as each kernel derives it
// (the GGX Fresnel kernel from cos_theta x roughness only, GGXFresnelDirectionalAlbedo.h:64-66)
int mpt_bake_lut(MptContext* c, int kind, int32_t w, int32_t h, int32_t d, int32_t samples, float* out, int dev) {
    if (!c || !out) return fail(MPT_ERR_INVALID_ARGUMENT, "NULL argument");
    if (kind < MPT_BAKE_GGX_CONDUCTOR || kind > MPT_BAKE_GGX_THIN_GLASS) return fail(MPT_ERR_INVALID_ARGUMENT, "bad LUT kind");
    if (w < 2 || h < 2 || d < 1 || (kind != MPT_BAKE_GGX_CONDUCTOR && d < 2) || (kind == MPT_BAKE_GGX_CONDUCTOR && d != 1) ||
        samples < 1 || (int64_t)w * h * d > (1 << 28))
        return fail(MPT_ERR_INVALID_ARGUMENT, "bad LUT size or sample count");
    HIPCHK(hipSetDevice(c->device));
    const float elems = 100000000.0f;   // GPUBakerConstants::COMPUTE_ELEMENT_PER_BAKE_KERNEL_LAUNCH
    const int texels = w * h * d;
    const int ipk = (int)std::floor(std::max(1.0f, elems / (float)texels));
    const int launches = (int)std::ceil((float)samples / (float)ipk);
    int nb = launches * ipk;
    if (kind == MPT_BAKE_GGX_FRESNEL) {
        const int ipk2 = (int)std::floor(std::max(1.0f, elems / (float)(w * h)));
        nb = (int)std::ceil((float)samples / (float)ipk2) * ipk2;
    }
    DBuf<float> buf;
    Allocs A;
    A(buf, (size_t)texels);
    if (A.e == hipSuccess) A(hipMemsetAsync(buf.p, 0, (size_t)texels * sizeof(float), c->stream));
    for (int i = 0; i < launches && A.e == hipSuccess; i++) A(launch_bake(kind, w, h, d, ipk, nb, i + 1, buf.p, c->stream));
    if (A.e == hipSuccess)
        A(hipMemcpyAsync(out, buf.p, (size_t)texels * sizeof(float), dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                         c->stream));
    if (A.e == hipSuccess) A(hipStreamSynchronize(c->stream));
    if (A.e != hipSuccess) return alloc_fail(A.e, "LUT bake");
    return MPT_OK;
}

static int raw_trace(MptContext* c, const float* rays, const int32_t* last_hit, int32_t n, bool any, int32_t* prim,
                     float* t, float* u, float* v, uint8_t* occ, int dev) {
    if (!c || !rays || n < 0) return fail(MPT_ERR_INVALID_ARGUMENT, "bad ray-query arguments");
    if (!c->has_scene) return fail(MPT_ERR_NO_SCENE, "no scene uploaded");
    if (n == 0) return MPT_OK;
    HIPCHK(hipSetDevice(c->device));
    // pack (o, last_hit) / (d, tmax)
    std::vector<float4> ho(n), hd(n);
    std::vector<float> hr;
    std::vector<int32_t> hl;
    const float* R = rays;
    const int32_t* LH = last_hit;
    if (dev) {
        hr.resize(8 * (size_t)n);
        HIPCHK(hipMemcpy(hr.data(), rays, hr.size() * sizeof(float), hipMemcpyDeviceToHost));
        R = hr.data();
        if (last_hit) {
            hl.resize(n);
            HIPCHK(hipMemcpy(hl.data(), last_hit, n * sizeof(int32_t), hipMemcpyDeviceToHost));
            LH = hl.data();
        }
    }
    for (int i = 0; i < n; i++) {
        int32_t lh = LH ? LH[i] : -1;
        float lhf;
        std::memcpy(&lhf, &lh, 4);
        ho[i] = make_float4(R[8 * i], R[8 * i + 1], R[8 * i + 2], lhf);
        hd[i] = make_float4(R[8 * i + 4], R[8 * i + 5], R[8 * i + 6], R[8 * i + 7]);
    }
    HIPCHK(c->raw_o.upload(ho.data(), n, c->stream));
    HIPCHK(c->raw_d.upload(hd.data(), n, c->stream));
    HIPCHK(c->raw_hit.alloc(n));
    HIPCHK(c->raw_occ.alloc(n));
    hipError_t e = launch_trace_raw(dev_scene(c), c->raw_o.p, c->raw_d.p, n, any, c->raw_hit.p, c->raw_occ.p, c->fetch_raw.p,
                                    c->spill.p, c->grid, c->stream);
    if (e != hipSuccess) return fail(MPT_ERR_HIP, std::string("trace launch: ") + hipGetErrorString(e));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (any) {
        if (occ) HIPCHK(hipMemcpy(occ, c->raw_occ.p, n, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
        return MPT_OK;
    }
    std::vector<float4> hh(n);
    HIPCHK(hipMemcpy(hh.data(), c->raw_hit.p, n * sizeof(float4), hipMemcpyDeviceToHost));
    std::vector<int32_t> P(n);
    std::vector<float> T(n), U(n), V(n);
    for (int i = 0; i < n; i++) {
        int32_t p;
        std::memcpy(&p, &hh[i].w, 4);
        P[i] = p; T[i] = hh[i].x; U[i] = hh[i].y; V[i] = hh[i].z;
    }
    hipMemcpyKind k = dev ? hipMemcpyHostToDevice : hipMemcpyHostToHost;
    if (prim) HIPCHK(hipMemcpy(prim, P.data(), n * sizeof(int32_t), k));
    if (t) HIPCHK(hipMemcpy(t, T.data(), n * sizeof(float), k));
    if (u) HIPCHK(hipMemcpy(u, U.data(), n * sizeof(float), k));
    if (v) HIPCHK(hipMemcpy(v, V.data(), n * sizeof(float), k));
    return MPT_OK;
}

int mpt_trace_closest(MptContext* c, const float* rays, const int32_t* last_hit, int32_t n, int32_t* prim, float* t, float* u,
                      float* v, int dev) {
    return raw_trace(c, rays, last_hit, n, false, prim, t, u, v, nullptr, dev);
}

int mpt_trace_any(MptContext* c, const float* rays, const int32_t* last_hit, int32_t n, uint8_t* occ, int dev) {
    return raw_trace(c, rays, last_hit, n, true, nullptr, nullptr, nullptr, nullptr, occ, dev);
}

}  // extern "C"
