// gpu_renderer.cpp -- see gpu_renderer.h.  Host code only; all GPU work is libmpt's.
#include "gpu_renderer.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace mpt_host {

// ---- LocalHaloGroup ------------------------------------------------------------------------
LocalHaloGroup::LocalHaloGroup(int band_count, int band_height, std::vector<int> devices)
    : m_n(band_count), m_bh(band_height), m_devices(std::move(devices)), m_members(band_count),
      m_published(band_count), m_need(band_count, 0) {
    for (int k = 0; k < m_n; k++) m_members[k] = Member{this, k, 0};
}

bool LocalHaloGroup::wait() {
    std::unique_lock<std::mutex> lk(m_mu);
    if (m_aborted) return false;
    const unsigned gen = m_generation;
    if (++m_arrived == m_n) {
        m_arrived = 0;
        m_generation++;
        m_cv.notify_all();
    } else {
        m_cv.wait(lk, [&] { return m_generation != gen || m_aborted; });
    }
    return m_generation != gen;   // an abort after the last arrival still completes this barrier
}

void LocalHaloGroup::abort(int rank) {
    std::lock_guard<std::mutex> lk(m_mu);
    if (!m_aborted) m_origin = rank;
    m_aborted = true;
    m_cv.notify_all();
}

int LocalHaloGroup::abort_origin() {
    std::lock_guard<std::mutex> lk(m_mu);
    return m_aborted ? m_origin : -1;
}

void LocalHaloGroup::reset() {
    std::lock_guard<std::mutex> lk(m_mu);
    m_aborted = false;
    m_origin = -1;
    m_arrived = 0;
    m_generation++;
    for (Member& m : m_members) m.calls = 0;
}

bool LocalHaloGroup::aborted() {
    std::lock_guard<std::mutex> lk(m_mu);
    return m_aborted;
}

int LocalHaloGroup::exchange(void* user, MptHaloExchange* x) {
    Member* me = (Member*)user;
    LocalHaloGroup& g = *me->group;
    const int k = me->rank;
    const bool inject = k == g.m_fail_rank && me->calls == g.m_fail_call;
    me->calls++;
    hipStream_t st = (hipStream_t)x->stream;
    int rc = hipSetDevice(g.m_devices[k]) == hipSuccess && hipStreamSynchronize(st) == hipSuccess ? 0 : 1;   // own rows final
    if (inject) rc = 1;
    if (rc != 0) {   // the others must not wait for this member's rows
        g.abort(k);
        return rc;
    }
    g.m_published[k] = *x;
    g.m_need[k] = x->halo_rows;
    if (!g.wait()) return 1;
    if (x->phase == MPT_HALO_GBUFFER) x->halo_rows = *std::max_element(g.m_need.begin(), g.m_need.end());
    // rows [y0 - halo, y0) and [y1, y1 + halo) of every buffer, from the bands that own them
    const int h = x->halo_rows;
    const int ranges[2][2] = {{std::max(0, x->own_y0 - h), x->own_y0}, {x->own_y1, std::min(x->res_y, x->own_y1 + h)}};
    for (int p = 0; p < g.m_n && rc == 0; p++) {
        if (p == k) continue;
        const int p0 = std::min(x->res_y, p * g.m_bh), p1 = std::min(x->res_y, p0 + g.m_bh);
        for (const auto& r : ranges) {
            const int a = std::max(r[0], p0), b = std::min(r[1], p1);
            if (a >= b) continue;
            for (int i = 0; i < x->n_buffers && rc == 0; i++) {
                const size_t row = (size_t)x->res_x * (size_t)x->bytes_per_pixel[i], off = (size_t)a * row;
                rc = hipMemcpyPeerAsync((char*)x->buffers[i] + off, g.m_devices[k], (const char*)g.m_published[p].buffers[i] + off,
                                        g.m_devices[p], (size_t)(b - a) * row, st) == hipSuccess ? 0 : 1;
            }
        }
    }
    if (hipStreamSynchronize(st) != hipSuccess) rc = 1;
    if (rc != 0) g.abort(k);
    if (!g.wait()) return 1;   // nobody overwrites rows another member is still copying
    return rc;
}

// ---- GPURenderer -----------------------------------------------------------------------------
void GPURenderer::check(int rc) const {
    if (rc != MPT_OK) throw std::runtime_error(std::string("libmpt: ") + mpt_last_error());
}

GPURenderer::GPURenderer(int device) : GPURenderer(std::vector<int>{device}) {}

GPURenderer::GPURenderer(const std::vector<int>& devices) : m_devices(devices) {
    if (devices.empty()) throw std::runtime_error("GPURenderer: no device");
    for (int d : devices) {
        MptContext* c = nullptr;
        int rc = mpt_create(d, nullptr, &c);
        if (rc != MPT_OK) {
            for (MptContext* o : m_ctxs) mpt_destroy(o);
            check(rc);
        }
        m_ctxs.push_back(c);
    }
    m_render_data.band_height = 1;
    m_render_data.band_index = 0;
    m_render_data.band_count = 1;
}

GPURenderer::~GPURenderer() {
    for (MptContext* c : m_ctxs) mpt_destroy(c);
}

void GPURenderer::set_scene(const MptScene& scene) {
    for (MptContext* c : m_ctxs) check(mpt_upload_scene(c, &scene));
    m_original_materials.assign(scene.materials, scene.materials + scene.num_materials);
    m_current_materials = m_original_materials;
}

void GPURenderer::update_materials(std::vector<MptMaterial>& materials) {
    for (MptContext* c : m_ctxs) check(mpt_update_materials(c, materials.data(), (int32_t)materials.size()));
    m_current_materials = materials;
}

void GPURenderer::set_envmap(const float* rgba, int width, int height, const std::string& envmap_filepath) {
    // Image32Bit::compute_alias_table / compute_cdf (Image.cpp:553-659), restated in libmpt
    std::vector<float> prob((size_t)width * height), cdf((size_t)width * height);
    std::vector<int32_t> alias((size_t)width * height);
    float lum_sum = 0.0f, cdf_sum = 0.0f;
    check(mpt_build_alias_table(rgba, width, height, prob.data(), alias.data(), &lum_sum));
    check(mpt_build_envmap_cdf(rgba, width, height, cdf.data(), &cdf_sum));
    for (MptContext* c : m_ctxs) {
        check(mpt_set_envmap(c, rgba, width, height, prob.data(), alias.data(), lum_sum));
        check(mpt_set_envmap_cdf(c, cdf.data(), cdf_sum));
    }
    m_has_envmap = true;
    m_envmap_path = envmap_filepath;
}

void GPURenderer::setup_brdfs_data(const MptLuts& luts) {
    for (MptContext* c : m_ctxs) check(mpt_set_luts(c, &luts));
}

void GPURenderer::resize(int width, int height) {
    m_width = width;
    m_height = height;
    for (MptContext* c : m_ctxs) check(mpt_resize(c, width, height));
    m_render_data.render_settings.need_to_reset = true;   // resizing restarts the accumulation (GPURenderer::resize)
}

void GPURenderer::set_camera(const MptCamera& camera) {
    m_camera = camera;
    if (!m_has_camera) m_previous_frame_camera = camera;
    m_has_camera = true;
}

void GPURenderer::update() {
    MptRenderSettings& rs = m_render_data.render_settings;
    rs.do_update_status_buffers = false;   // GPURenderer.cpp:257-258
    m_rng.xorshift32();                    // update_render_data (GPURenderer.cpp:980-983)
    if (!rs.accumulate) rs.sample_number = 0;
}

void GPURenderer::reset() {
    MptRenderSettings& rs = m_render_data.render_settings;
    rs.sample_number = 0;
    rs.denoiser_AOV_accumulation_counter = 0;
    rs.need_to_reset = true;
    if (rs.accumulate) m_rng = Xorshift32(42);   // GPURenderer.cpp:953-973
}

void GPURenderer::launch_camera_rays() {
    // GPURenderer.cpp:465-471: a new seed per CameraRays launch
    std::memset(m_render_data.restir_di_seeds, 0, sizeof(m_render_data.restir_di_seeds));
    m_render_data.camera_random_seed = m_rng.xorshift32();
}

void GPURenderer::launch_ReSTIR_DI() {
    // GPURenderer.cpp:473-477 -> ReSTIRDIRenderPass::launch (ReSTIRDIRenderPass.cpp:233-264,
    // 298-431): the seeds its passes draw, in launch order
    if (m_render_data.options.direct_light_sampling != MPT_LSS_RESTIR_DI) return;
    MptFrame& f = m_render_data;
    MptReSTIRDISettings& rd = f.render_settings.restir_di_settings;
    if (f.options.restir_di_do_lights_presampling)
        f.restir_di_seeds[0] = m_rng.xorshift32();   // lights presampling (launched only when enabled)
    f.restir_di_seeds[1] = m_rng.xorshift32();       // initial candidates
    if (rd.do_fused_spatiotemporal) {
        m_rng.xorshift32();                          // temporal seed, overwritten before the launch
        f.restir_di_seeds[3] = m_rng.xorshift32();   // permutation-sampling bits
        f.restir_di_seeds[2] = m_rng.xorshift32();   // configure_spatial_pass_for_fused_spatiotemporal(0)
        for (int p = 1; p < rd.number_of_passes && 4 + p < 8; p++) f.restir_di_seeds[4 + p] = m_rng.xorshift32();
    } else {
        if (rd.do_temporal_reuse_pass) {
            f.restir_di_seeds[2] = m_rng.xorshift32();
            f.restir_di_seeds[3] = m_rng.xorshift32();
        }
        if (rd.do_spatial_reuse_pass)
            for (int p = 0; p < rd.number_of_passes && 4 + p < 8; p++) f.restir_di_seeds[4 + p] = m_rng.xorshift32();
    }
    rd.permutation_sampling_random_bits = (int32_t)f.restir_di_seeds[3];
}

void GPURenderer::launch_path_tracing() {
    // GPURenderer.cpp:479-486: the path-tracing seed, then the launch
    MptFrame& f = m_render_data;
    f.random_seed = m_rng.xorshift32();
    f.current_camera = m_camera;
    f.prev_camera = m_previous_frame_camera;
    f.res_x = m_width;
    f.res_y = m_height;
    m_pending.push_back(f);
    if (!m_in_render) flush();   // a launch outside render(): enqueued on its own
}

// Band k of the context partition: interleaved 8-row bands (path tracing: every pixel's RNG
// stream depends only on its pixel index, and interleaving balances sky against geometry), or
// one contiguous band per context for ReSTIR DI (halo exchange, mpt.h MptHaloExchange)
void GPURenderer::band_fields(MptFrame& f, int k) const {
    const int n = (int)m_ctxs.size();
    if (n == 1) { f.band_height = 1; f.band_index = 0; f.band_count = 1; return; }
    const bool restir = f.options.direct_light_sampling == MPT_LSS_RESTIR_DI;
    f.band_height = restir ? (f.res_y + n - 1) / n : 8;
    f.band_index = k;
    f.band_count = n;
}

void GPURenderer::flush() {
    if (m_pending.empty()) return;
    m_last_frames = m_pending;
    m_pending.clear();
    const int n = (int)m_ctxs.size();
    if (n == 1) {
        check(mpt_render_frames(m_ctxs[0], m_last_frames.data(), (int32_t)m_last_frames.size(), 0));
        return;
    }
    // one host thread per context: a ReSTIR DI context blocks in its halo exchange until its
    // neighbours reach the same point
    const bool restir = m_last_frames[0].options.direct_light_sampling == MPT_LSS_RESTIR_DI;
    const int bh = (m_height + n - 1) / n;
    if (restir && (!m_halo || m_halo_bh != bh)) {
        m_halo.reset(new LocalHaloGroup(n, bh, m_devices));
        m_halo_bh = bh;
        for (int k = 0; k < n; k++) check(mpt_set_halo_exchange(m_ctxs[k], &LocalHaloGroup::exchange, m_halo->member(k)));
    }
    if (restir) {
        m_halo->reset();
        m_halo->inject_failure(m_fail_band, m_fail_call);
    }
    std::vector<int> rcs(n, MPT_OK);
    std::vector<std::string> errs(n);
    std::vector<std::thread> th;
    for (int k = 0; k < n; k++)
        th.emplace_back([&, k] {
            std::vector<MptFrame> fr = m_last_frames;
            for (MptFrame& f : fr) band_fields(f, k);
            rcs[k] = mpt_render_frames(m_ctxs[k], fr.data(), (int32_t)fr.size(), 0);
            if (rcs[k] != MPT_OK) {
                errs[k] = mpt_last_error();   // the error text is per thread
                // a band that stops before its next exchange point must not leave the others waiting
                if (restir) m_halo->abort(k);
            }
        });
    for (auto& t : th) t.join();
    // the band that failed first names the cause (the others report the aborted exchange)
    int first = restir ? m_halo->abort_origin() : -1;
    if (first < 0 || rcs[first] == MPT_OK) {
        first = -1;
        for (int k = 0; k < n && first < 0; k++)
            if (rcs[k] != MPT_OK) first = k;
    }
    if (first >= 0) {
        std::string all;
        for (int k = 0; k < n; k++)
            if (rcs[k] != MPT_OK) all += "; band " + std::to_string(k) + ": " + errs[k];
        throw std::runtime_error("libmpt (band " + std::to_string(first) + "): " + errs[first] + " [" + all.substr(2) + "]");
    }
}

void GPURenderer::render() {
    if (!m_has_camera) throw std::runtime_error("GPURenderer::render: no camera");
    MptRenderSettings& rs = m_render_data.render_settings;
    for (MptContext* c : m_ctxs) check(mpt_clear_status(c));   // internal_update_clear_device_status_buffers
    map_buffers_for_render();         // GPURenderer.cpp:419
    const int spf = rs.samples_per_frame > 0 ? rs.samples_per_frame : 1;
    m_pending.clear();
    m_in_render = true;
    try {
        for (int i = 1; i <= spf; i++) {
            if (i == spf) rs.do_update_status_buffers = true;   // GPURenderer.cpp:430-434
            launch_camera_rays();
            launch_ReSTIR_DI();
            launch_path_tracing();
            rs.sample_number++;
            rs.denoiser_AOV_accumulation_counter++;
            rs.need_to_reset = false;
            rs.restir_di_settings.temporal_buffer_clear_requested = false;
            m_previous_frame_camera = m_camera;
        }
    } catch (...) {
        m_in_render = false;
        throw;
    }
    m_in_render = false;
    flush();
    // GPURenderer.cpp:458: do_render_low_resolution (RenderSettings.h:195-198)
    m_was_last_frame_low_resolution = rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate;
}

void GPURenderer::synchronize_kernel() {
    for (MptContext* c : m_ctxs) check(mpt_synchronize(c));
}

bool GPURenderer::frame_render_done() {
    for (MptContext* c : m_ctxs) {
        int done = 0;
        check(mpt_query_done(c, &done));
        if (!done) return false;
    }
    return true;
}

void GPURenderer::map_buffers_for_render() { m_mapped = true; }

void GPURenderer::unmap_buffers() {
    // the display buffers receive the sums of everything rendered so far (device-to-device
    // copies on the renderer's stream, after the frame's launches)
    if (!m_mapped) return;
    // (several contexts: the bands gathered onto devices[0], peer copies over xGMI)
    if (!m_mapped) return;
    const int n = (int)m_ctxs.size();
    if (m_display.color) check(mpt_gather(m_ctxs.data(), n, 0, MPT_FB_COLOR, m_display.color, 1));
    if (m_display.albedo) check(mpt_gather(m_ctxs.data(), n, 0, MPT_FB_ALBEDO, m_display.albedo, 1));
    if (m_display.normals) check(mpt_gather(m_ctxs.data(), n, 0, MPT_FB_NORMALS, m_display.normals, 1));
    m_mapped = false;
}

void GPURenderer::copy_status_buffers() {
    // several contexts: a ray is active if one band has one; converged pixels add up
    MptStatus all{};
    for (MptContext* c : m_ctxs) {
        MptStatus s{};
        check(mpt_query_status(c, &s));
        all.one_ray_active = all.one_ray_active || s.one_ray_active;
        all.pixel_converged_count += s.pixel_converged_count;
    }
    m_status = all;
}

void GPURenderer::get_framebuffer(int kind, float* dst_rgb) {
    check(mpt_gather(m_ctxs.data(), (int32_t)m_ctxs.size(), 0, kind, dst_rgb, 0));
}

void GPURenderer::get_aux_buffer(int kind, void* dst) {
    if (kind >= MPT_AUX_RESTIR_OUTPUT) {
        // frame-sized reservoirs (48 B per pixel): a context keeps only its own contiguous band (plus
        // halo rows) current, so each band's rows come from the context that owns it
        const int n = (int)m_ctxs.size();
        if (n == 1) {
            check(mpt_get_aux_buffer(m_ctxs[0], kind, dst, 0));
            return;
        }
        const size_t row = (size_t)m_width * 48;
        const int bh = (m_height + n - 1) / n;   // band_fields' ReSTIR DI partition
        std::vector<char> tmp((size_t)m_height * row);
        for (int k = 0; k < n; k++) {
            const int y0 = std::min(m_height, k * bh), y1 = std::min(m_height, y0 + bh);
            if (y0 >= y1) continue;
            check(mpt_get_aux_buffer(m_ctxs[k], kind, tmp.data(), 0));
            std::memcpy((char*)dst + (size_t)y0 * row, tmp.data() + (size_t)y0 * row, (size_t)(y1 - y0) * row);
        }
        return;
    }
    check(mpt_gather(m_ctxs.data(), (int32_t)m_ctxs.size(), 0, MPT_GATHER_AUX + kind, dst, 0));
}

}  // namespace mpt_host
