// gpu_renderer.h -- C++ host side above the C ABI: the reference's GPURenderer launch
// surface (src/Renderer/GPURenderer.h:75-300) re-implemented over libmpt, so the
// reference's render loop (RenderWindow::render, RenderWindow.cpp:748-815) and its
// settings editors keep their calls.  Method names, argument meaning and the seed schedule
// are the reference's; errors throw std::runtime_error with mpt_last_error() (the
// reference logs and exits, HIPRTOrochiUtils.cpp:15-47).
#ifndef MPT_HOST_GPU_RENDERER_H
#define MPT_HOST_GPU_RENDERER_H

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
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

// Device destinations of the displayed buffers: the HIP pointers an OpenGL interop map
// returns (OpenGLInteropBuffer<T>::map, OpenGLInteropBuffer.h), W*H float3 each; nullptr =
// that buffer is not displayed.  The reference renders straight into them between
// map_buffers_for_render and unmap_buffers; libmpt owns its sums, so unmap_buffers copies
// them in (device to device, on the renderer's stream) before OpenGL takes the buffers back.
struct DisplayBuffers {
    float* color = nullptr;      // 'pixels' (a sum over the samples, RenderData.h:32)
    float* albedo = nullptr;     // denoiser albedo AOV
    float* normals = nullptr;    // denoiser normals AOV
};

// ReSTIR DI across the row bands of several contexts of this process (mpt.h MptHaloExchange):
// one host thread per context renders its band; at every exchange point each member
// publishes its buffers, waits for the others, copies its halo rows from the owners (peer
// copies between GPUs) on its own stream and waits again, so that no owner overwrites rows
// still being read.  (mpt.partition.LocalHaloGroup is the same protocol in Python.)
// A member that fails (its copies, or its context's render returning an error before the
// next exchange point) aborts the group: every waiting and every later exchange returns
// non-zero at once, so all band threads unwind and the renderer throws instead of hanging.
class LocalHaloGroup {
public:
    LocalHaloGroup(int band_count, int band_height, std::vector<int> devices);
    // the MptHaloExchangeFn of member `rank` (user = the Member)
    struct Member { LocalHaloGroup* group; int rank; int calls; };
    Member* member(int rank) { return &m_members[rank]; }
    static int exchange(void* user, MptHaloExchange* x);
    void abort(int rank);   // wakes every member; exchanges fail until reset(); records the first rank
    int abort_origin();     // the member that aborted first (-1: none)
    void reset();    // a new render: no member waiting, not aborted
    bool aborted();
    // test hook: member `rank`'s callback fails at its `call`-th exchange (0-based) of a render
    void inject_failure(int rank, int call) { m_fail_rank = rank; m_fail_call = call; }

private:
    bool wait();   // generation barrier over the band_count members; false once aborted
    int m_n, m_bh;
    std::vector<int> m_devices;
    std::vector<Member> m_members;
    std::vector<MptHaloExchange> m_published;
    std::vector<int> m_need;
    std::mutex m_mu;
    std::condition_variable m_cv;
    int m_arrived = 0;
    unsigned m_generation = 0;
    bool m_aborted = false;
    int m_origin = -1;
    int m_fail_rank = -1, m_fail_call = -1;
};

class GPURenderer {
public:
    // GPURenderer::GPURenderer (GPURenderer.cpp:48-86): m_rng seeded 42
    explicit GPURenderer(int device = 0);
    // The frame tiled across several GPUs of this process (north_star: row partition + a final
    // gather over xGMI; the reference drives one device, main.cpp:57): one libmpt context per
    // entry of `devices` (an index may repeat: several bands on one GPU).  Context k renders
    // band k -- interleaved 8-row bands for path tracing, one contiguous band per context plus
    // the halo exchange for ReSTIR DI (its reuse passes read neighbouring pixels) -- each from
    // its own host thread; map / unmap, get_framebuffer and get_aux_buffer gather the whole
    // frame with mpt_gather onto devices[0].  Every pixel's result is bit-identical to the
    // single-device render.  Switching between ReSTIR DI and the other strategies changes the
    // partition, which restarts the accumulation (the reference resets on such option edits).
    explicit GPURenderer(const std::vector<int>& devices);
    ~GPURenderer();
    GPURenderer(const GPURenderer&) = delete;
    GPURenderer& operator=(const GPURenderer&) = delete;

    // set_scene (GPURenderer.cpp:1041-1134): the arrays are copied, the BVH8 built on upload
    void set_scene(const MptScene& scene);
    // set_envmap (GPURenderer.cpp:1136-1174): RGBA32F equirect; alias table and CDF built here
    void set_envmap(const float* rgba, int width, int height, const std::string& envmap_filepath = "");
    bool has_envmap() const { return m_has_envmap; }
    const std::string& get_envmap_filepath() const { return m_envmap_path; }
    // setup_brdfs_data (GPURenderer.cpp:88-175)
    void setup_brdfs_data(const MptLuts& luts);
    // resize (GPURenderer.h:172)
    void resize(int width, int height);
    // set_camera (GPURenderer.h:218): the camera of the next frames; each sample's previous
    // camera is the one of the sample before it (GPURenderer.cpp:424-449)
    void set_camera(const MptCamera& camera);
    const MptCamera& get_camera() const { return m_camera; }

    // update_materials (GPURenderer.h:228, .cpp:1196-1200): material edits of the front-end's
    // editor; re-uploaded and re-resolved (texture flags, material classes, light BVH)
    void update_materials(std::vector<MptMaterial>& materials);
    const std::vector<MptMaterial>& get_original_materials() const { return m_original_materials; }
    const std::vector<MptMaterial>& get_current_materials() const { return m_current_materials; }

    // update (GPURenderer.cpp:236-262): one m_rng draw per displayed frame
    // (update_render_data, GPURenderer.cpp:980-983); resets sample_number when not accumulating
    void update();
    // render (GPURenderer.cpp:408-456): per sample launch_camera_rays, launch_ReSTIR_DI,
    // launch_path_tracing with the reference's seed draws; the samples_per_frame samples of one
    // call are traced as batched wavefronts (mpt_render_frames)
    void render();
    // The three launches of one sample (GPURenderer.cpp:465-486).  libmpt runs a sample's
    // CameraRays, ReSTIR DI passes and path tracing as one launch set, so the first two draw
    // their seeds into the render data and launch_path_tracing enqueues the whole sample (inside
    // render(), the samples of the call are enqueued together at its end).
    void launch_camera_rays();
    void launch_ReSTIR_DI();
    void launch_path_tracing();
    // reset (GPURenderer.cpp:953-973): restart the accumulation, m_rng re-seeded 42
    void reset();
    // was_last_frame_low_resolution (GPURenderer.cpp:458, 512-515): the last render() ran in the
    // low-resolution interactive mode (RenderWindow displays its top-left block scaled up)
    bool was_last_frame_low_resolution() const { return m_was_last_frame_low_resolution; }
    void synchronize_kernel();
    bool frame_render_done();

    // map_buffers_for_render / unmap_buffers (GPURenderer.cpp:583-598) over the display
    // buffers registered here (see DisplayBuffers)
    void set_display_buffers(const DisplayBuffers& buffers) { m_display = buffers; }
    void map_buffers_for_render();
    void unmap_buffers();

    MptRenderSettings& get_render_settings() { return m_render_data.render_settings; }
    MptWorldSettings& get_world_settings() { return m_render_data.world_settings; }
    MptKernelOptions& get_kernel_options() { return m_render_data.options; }   // KernelOptions.h macros, at run time
    MptBSDFFlags& get_bsdf_flags() { return m_render_data.bsdf_flags; }
    // get_render_data (GPURenderer.h:211): HIPRTRenderData's host-visible part -- settings,
    // cameras, seeds, resolution -- as the frame record libmpt consumes (device buffers are
    // libmpt's own; read them with get_framebuffer / get_aux_buffer)
    MptFrame& get_render_data() { return m_render_data; }
    // copy_status_buffers / get_status_buffer_values (GPURenderer.cpp:269-283)
    void copy_status_buffers();
    const MptStatus& get_status_buffer_values() const { return m_status; }
    // the 'pixels' sum buffer and the denoiser AOVs (RenderData.h:32-36), host copy
    void get_framebuffer(int kind, float* dst_rgb);
    // pixel_sample_count / pixel_converged_sample_count / pixel_squared_luminance
    // (RenderData.h:62-84; get_pixels_converged_sample_count_buffer, GPURenderer.h:193), host copy;
    // the ReSTIR DI reservoir kinds (frame-sized): each band's rows from the context that owns them
    void get_aux_buffer(int kind, void* dst);
    int render_width() const { return m_width; }
    int render_height() const { return m_height; }
    // the frames enqueued by the last render() / launch_path_tracing() (tests; band fields of
    // the whole frame)
    const std::vector<MptFrame>& last_frames() const { return m_last_frames; }
    int device_count() const { return (int)m_ctxs.size(); }
    // test hook (tests/test_host_cpp.py): band `band`'s halo exchange fails at its `call`-th
    // exchange of a render -- the render must throw, not hang
    void inject_halo_failure(int band, int call) { m_fail_band = band; m_fail_call = call; }

private:
    void check(int rc) const;
    void flush();

    void band_fields(MptFrame& f, int k) const;

    std::vector<MptContext*> m_ctxs;
    std::vector<int> m_devices;
    std::unique_ptr<LocalHaloGroup> m_halo;   // ReSTIR DI over several contexts
    int m_halo_bh = 0;
    int m_fail_band = -1, m_fail_call = -1;
    Xorshift32 m_rng{42};
    int m_width = 0, m_height = 0;
    MptFrame m_render_data{};
    MptCamera m_camera{};
    MptCamera m_previous_frame_camera{};
    bool m_has_camera = false;
    bool m_in_render = false;
    bool m_has_envmap = false;
    bool m_mapped = false;
    bool m_was_last_frame_low_resolution = false;
    std::string m_envmap_path;
    DisplayBuffers m_display;
    MptStatus m_status{};
    std::vector<MptMaterial> m_original_materials, m_current_materials;
    std::vector<MptFrame> m_pending;        // samples enqueued by the launches of this render()
    std::vector<MptFrame> m_last_frames;
};

}  // namespace mpt_host

#endif
