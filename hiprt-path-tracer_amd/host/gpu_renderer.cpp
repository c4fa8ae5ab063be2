// gpu_renderer.cpp -- see gpu_renderer.h.  Host code only; all GPU work is libmpt's.
#include "gpu_renderer.h"

#include <stdexcept>
#include <string>

namespace mpt_host {

void GPURenderer::check(int rc) const {
    if (rc != MPT_OK) throw std::runtime_error(std::string("libmpt: ") + mpt_last_error());
}

GPURenderer::GPURenderer(int device) { check(mpt_create(device, nullptr, &m_ctx)); }

GPURenderer::~GPURenderer() {
    if (m_ctx) mpt_destroy(m_ctx);
}

void GPURenderer::set_scene(const MptScene& scene) { check(mpt_upload_scene(m_ctx, &scene)); }

void GPURenderer::set_envmap(const float* rgba, int width, int height) {
    // Image32Bit::compute_alias_table / compute_cdf (Image.cpp:553-659), restated in libmpt
    std::vector<float> prob((size_t)width * height), cdf((size_t)width * height);
    std::vector<int32_t> alias((size_t)width * height);
    float lum_sum = 0.0f, cdf_sum = 0.0f;
    check(mpt_build_alias_table(rgba, width, height, prob.data(), alias.data(), &lum_sum));
    check(mpt_set_envmap(m_ctx, rgba, width, height, prob.data(), alias.data(), lum_sum));
    check(mpt_build_envmap_cdf(rgba, width, height, cdf.data(), &cdf_sum));
    check(mpt_set_envmap_cdf(m_ctx, cdf.data(), cdf_sum));
}

void GPURenderer::setup_brdfs_data(const MptLuts& luts) { check(mpt_set_luts(m_ctx, &luts)); }

void GPURenderer::resize(int width, int height) {
    m_width = width;
    m_height = height;
    check(mpt_resize(m_ctx, width, height));
    m_settings.need_to_reset = true;   // resizing restarts the accumulation (GPURenderer::resize)
}

void GPURenderer::set_camera(const MptCamera& camera) {
    m_camera = camera;
    if (!m_has_camera) m_previous_frame_camera = camera;
    m_has_camera = true;
}

void GPURenderer::update() {
    m_settings.do_update_status_buffers = false;   // GPURenderer.cpp:257-258
    m_rng.xorshift32();                            // update_render_data (GPURenderer.cpp:980-983)
    if (!m_settings.accumulate) m_settings.sample_number = 0;
}

void GPURenderer::reset() {
    m_settings.sample_number = 0;
    m_settings.denoiser_AOV_accumulation_counter = 0;
    m_settings.need_to_reset = true;
    if (m_settings.accumulate) m_rng = Xorshift32(42);   // GPURenderer.cpp:953-973
}

void GPURenderer::render() {
    if (!m_has_camera) throw std::runtime_error("GPURenderer::render: no camera");
    check(mpt_clear_status(m_ctx));   // internal_update_clear_device_status_buffers
    const int spf = m_settings.samples_per_frame > 0 ? m_settings.samples_per_frame : 1;
    m_last_frames.assign((size_t)spf, MptFrame{});
    for (int i = 1; i <= spf; i++) {
        MptFrame& f = m_last_frames[(size_t)i - 1];
        if (i == spf) m_settings.do_update_status_buffers = true;   // GPURenderer.cpp:430-434
        f.current_camera = m_camera;
        f.prev_camera = m_previous_frame_camera;
        f.options = m_options;
        f.bsdf_flags = m_bsdf_flags;
        f.camera_random_seed = m_rng.xorshift32();   // launch_camera_rays (GPURenderer.cpp:468-470)
        if (m_options.direct_light_sampling == MPT_LSS_RESTIR_DI) {
            // ReSTIRDIRenderPass::launch (ReSTIRDIRenderPass.cpp:233-264, 298-431)
            MptReSTIRDISettings& rd = m_settings.restir_di_settings;
            if (m_options.restir_di_do_lights_presampling)
                f.restir_di_seeds[0] = m_rng.xorshift32();   // lights presampling (launched only when enabled)
            f.restir_di_seeds[1] = m_rng.xorshift32();   // initial candidates
            if (rd.do_fused_spatiotemporal) {
                m_rng.xorshift32();                      // temporal seed, overwritten before the launch
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
        f.random_seed = m_rng.xorshift32();          // launch_path_tracing (GPURenderer.cpp:484)
        f.render_settings = m_settings;
        f.world_settings = m_world;
        f.res_x = m_width;
        f.res_y = m_height;
        f.band_height = 1;
        f.band_index = 0;
        f.band_count = 1;
        m_settings.sample_number++;
        m_settings.denoiser_AOV_accumulation_counter++;
        m_settings.need_to_reset = false;
        m_settings.restir_di_settings.temporal_buffer_clear_requested = false;
        m_previous_frame_camera = m_camera;
    }
    check(mpt_render_frames(m_ctx, m_last_frames.data(), spf, 0));
}

void GPURenderer::synchronize_kernel() { check(mpt_synchronize(m_ctx)); }

bool GPURenderer::frame_render_done() {
    int done = 0;
    check(mpt_query_done(m_ctx, &done));
    return done != 0;
}

MptStatus GPURenderer::get_status_buffer_values() {
    MptStatus st{};
    check(mpt_query_status(m_ctx, &st));
    return st;
}

void GPURenderer::get_framebuffer(int kind, float* dst_rgb) { check(mpt_get_framebuffer(m_ctx, kind, dst_rgb, 0)); }

}  // namespace mpt_host
