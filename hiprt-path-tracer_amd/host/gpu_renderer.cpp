// gpu_renderer.cpp -- see gpu_renderer.h.  Host code only; all GPU work is libmpt's.
#include "gpu_renderer.h"

#include <cstring>
#include <stdexcept>

namespace mpt_host {

void GPURenderer::check(int rc) const {
    if (rc != MPT_OK) throw std::runtime_error(std::string("libmpt: ") + mpt_last_error());
}

GPURenderer::GPURenderer(int device) {
    check(mpt_create(device, nullptr, &m_ctx));
    m_render_data.band_height = 1;
    m_render_data.band_index = 0;
    m_render_data.band_count = 1;
}

GPURenderer::~GPURenderer() {
    if (m_ctx) mpt_destroy(m_ctx);
}

void GPURenderer::set_scene(const MptScene& scene) {
    check(mpt_upload_scene(m_ctx, &scene));
    m_original_materials.assign(scene.materials, scene.materials + scene.num_materials);
    m_current_materials = m_original_materials;
}

void GPURenderer::update_materials(std::vector<MptMaterial>& materials) {
    check(mpt_update_materials(m_ctx, materials.data(), (int32_t)materials.size()));
    m_current_materials = materials;
}

void GPURenderer::set_envmap(const float* rgba, int width, int height, const std::string& envmap_filepath) {
    // Image32Bit::compute_alias_table / compute_cdf (Image.cpp:553-659), restated in libmpt
    std::vector<float> prob((size_t)width * height), cdf((size_t)width * height);
    std::vector<int32_t> alias((size_t)width * height);
    float lum_sum = 0.0f, cdf_sum = 0.0f;
    check(mpt_build_alias_table(rgba, width, height, prob.data(), alias.data(), &lum_sum));
    check(mpt_set_envmap(m_ctx, rgba, width, height, prob.data(), alias.data(), lum_sum));
    check(mpt_build_envmap_cdf(rgba, width, height, cdf.data(), &cdf_sum));
    check(mpt_set_envmap_cdf(m_ctx, cdf.data(), cdf_sum));
    m_has_envmap = true;
    m_envmap_path = envmap_filepath;
}

void GPURenderer::setup_brdfs_data(const MptLuts& luts) { check(mpt_set_luts(m_ctx, &luts)); }

void GPURenderer::resize(int width, int height) {
    m_width = width;
    m_height = height;
    check(mpt_resize(m_ctx, width, height));
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

void GPURenderer::flush() {
    if (m_pending.empty()) return;
    m_last_frames = m_pending;
    m_pending.clear();
    check(mpt_render_frames(m_ctx, m_last_frames.data(), (int32_t)m_last_frames.size(), 0));
}

void GPURenderer::render() {
    if (!m_has_camera) throw std::runtime_error("GPURenderer::render: no camera");
    MptRenderSettings& rs = m_render_data.render_settings;
    check(mpt_clear_status(m_ctx));   // internal_update_clear_device_status_buffers
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
}

void GPURenderer::synchronize_kernel() { check(mpt_synchronize(m_ctx)); }

bool GPURenderer::frame_render_done() {
    int done = 0;
    check(mpt_query_done(m_ctx, &done));
    return done != 0;
}

void GPURenderer::map_buffers_for_render() { m_mapped = true; }

void GPURenderer::unmap_buffers() {
    // the display buffers receive the sums of everything rendered so far (device-to-device
    // copies on the renderer's stream, after the frame's launches)
    if (!m_mapped) return;
    if (m_display.color) check(mpt_get_framebuffer(m_ctx, MPT_FB_COLOR, m_display.color, 1));
    if (m_display.albedo) check(mpt_get_framebuffer(m_ctx, MPT_FB_ALBEDO, m_display.albedo, 1));
    if (m_display.normals) check(mpt_get_framebuffer(m_ctx, MPT_FB_NORMALS, m_display.normals, 1));
    m_mapped = false;
}

void GPURenderer::copy_status_buffers() { check(mpt_query_status(m_ctx, &m_status)); }

void GPURenderer::get_framebuffer(int kind, float* dst_rgb) { check(mpt_get_framebuffer(m_ctx, kind, dst_rgb, 0)); }

void GPURenderer::get_aux_buffer(int kind, void* dst) { check(mpt_get_aux_buffer(m_ctx, kind, dst, 0)); }

}  // namespace mpt_host
