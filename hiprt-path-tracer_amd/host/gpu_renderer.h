// gpu_renderer.h -- C++ host side above the C ABI: the reference's GPURenderer launch
// surface (src/Renderer/GPURenderer.h:75-300) re-implemented over libmpt, so the
// reference's render loop (RenderWindow::render, RenderWindow.cpp:748-815) and its
// settings editors keep their calls.  Method names, argument meaning and the seed schedule
// are the reference's; errors throw std::runtime_error with mpt_last_error() (the
// reference logs and exits, HIPRTOrochiUtils.cpp:15-47).
#ifndef MPT_HOST_GPU_RENDERER_H
#define MPT_HOST_GPU_RENDERER_H

#include <cstdint>
#include <vector>

#include "mpt.h"

namespace mpt_host {

// Xorshift32Generator (HostDeviceCommon/Xorshift.h:17-65): the front-end's m_rng
struct Xorshift32 {
    uint32_t state;
    explicit Xorshift32(uint32_t seed) : state(seed) {}
    uint32_t xorshift32() {
        uint32_t x = state;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        return state = x;
    }
};

class GPURenderer {
public:
    // GPURenderer::GPURenderer (GPURenderer.cpp:48-86): m_rng seeded 42
    explicit GPURenderer(int device = 0);
    ~GPURenderer();
    GPURenderer(const GPURenderer&) = delete;
    GPURenderer& operator=(const GPURenderer&) = delete;

    // set_scene (GPURenderer.cpp:1041-1134): the arrays are copied, the BVH8 built on upload
    void set_scene(const MptScene& scene);
    // set_envmap (GPURenderer.cpp:1136-1174): RGBA32F equirect; alias table and CDF built here
    void set_envmap(const float* rgba, int width, int height);
    // setup_brdfs_data (GPURenderer.cpp:88-175)
    void setup_brdfs_data(const MptLuts& luts);
    // resize (GPURenderer.h:172)
    void resize(int width, int height);
    // set_camera: the camera of the next frame; the previous one becomes prev_camera
    void set_camera(const MptCamera& camera);

    // update (GPURenderer.cpp:236-262): one m_rng draw per displayed frame
    // (update_render_data, GPURenderer.cpp:980-983); resets sample_number when not accumulating
    void update();
    // render (GPURenderer.cpp:408-456): the samples_per_frame loop of CameraRays, ReSTIR DI and
    // FullPathTracer with the reference's seed draws; traced as batched wavefronts (mpt_render_frames)
    void render();
    // reset (GPURenderer.cpp:953-973): restart the accumulation, m_rng re-seeded 42
    void reset();
    void synchronize_kernel();
    bool frame_render_done();

    MptRenderSettings& get_render_settings() { return m_settings; }
    MptWorldSettings& get_world_settings() { return m_world; }
    MptKernelOptions& get_kernel_options() { return m_options; }   // KernelOptions.h macros, at run time
    MptBSDFFlags& get_bsdf_flags() { return m_bsdf_flags; }
    // copy_status_buffers / get_status_buffer_values (GPURenderer.cpp:269-283)
    MptStatus get_status_buffer_values();
    // the 'pixels' sum buffer and the denoiser AOVs (RenderData.h:32-36), host copy
    void get_framebuffer(int kind, float* dst_rgb);
    int render_width() const { return m_width; }
    int render_height() const { return m_height; }
    // the frames of the last render() (tests)
    const std::vector<MptFrame>& last_frames() const { return m_last_frames; }

private:
    void check(int rc) const;

    MptContext* m_ctx = nullptr;
    Xorshift32 m_rng{42};
    int m_width = 0, m_height = 0;
    MptRenderSettings m_settings{};
    MptWorldSettings m_world{};
    MptKernelOptions m_options{};
    MptBSDFFlags m_bsdf_flags{};
    MptCamera m_camera{};
    MptCamera m_previous_frame_camera{};
    bool m_has_camera = false;
    std::vector<MptFrame> m_last_frames;
};

}  // namespace mpt_host

#endif
