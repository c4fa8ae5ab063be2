// Test driver (tests/test_host_cpp.py): the C++ GPURenderer mirror (hiprt-path-tracer_amd/host)
// rendering a scene handed over as a raw blob by the test, through libmpt.
// usage: gpurenderer_parity <in.blob> <out.bin>
//   blob mode 0: RenderWindow's loop (update() then render()); mode 1: the same samples through
//   the three launches called one by one (launch_camera_rays / launch_ReSTIR_DI /
//   launch_path_tracing, the driver doing render()'s per-sample bookkeeping).  M2 > 0:
//   update_materials with the blob's edited materials before rendering.  N_SPLIT > 1: the
//   multi-device renderer with N_SPLIT row bands (contexts on device 0), gathered by mpt_gather.  The colour comes back
//   through the display-buffer path (map_buffers_for_render / unmap_buffers into hipMalloc'd
//   destinations, as an OpenGL interop map would hand them over) and is checked against
//   get_framebuffer; the per-pixel sample counts are returned for the test.
//   out.bin = int32 n_frames, MptFrame[n_frames] (every frame enqueued), float sums[W*H*3],
//             int32 pixel_sample_count[W*H]
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "gpu_renderer.h"

namespace {
struct Reader {
    FILE* f;
    template <typename T> T get() { T v; if (fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("short blob"); return v; }
    template <typename T> std::vector<T> arr(size_t n) {
        std::vector<T> v(n);
        if (n && fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("short blob");
        return v;
    }
};
}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) { fprintf(stderr, "usage: %s in.blob out.bin\n", argv[0]); return 2; }
    try {
        FILE* fin = fopen(argv[1], "rb");
        if (!fin) throw std::runtime_error("cannot open blob");
        Reader r{fin};
        if (r.get<uint32_t>() != 0x4254504du) throw std::runtime_error("bad magic");
        const auto settings = r.get<MptRenderSettings>();
        const auto world = r.get<MptWorldSettings>();
        const auto options = r.get<MptKernelOptions>();
        const auto flags = r.get<MptBSDFFlags>();
        const auto camera = r.get<MptCamera>();
        const int W = r.get<int32_t>(), H = r.get<int32_t>(), n_updates = r.get<int32_t>();
        const int T = r.get<int32_t>(), V = r.get<int32_t>(), M = r.get<int32_t>(), E = r.get<int32_t>();
        const int mode = r.get<int32_t>(), M2 = r.get<int32_t>(), n_split = r.get<int32_t>();
        auto idx = r.arr<int32_t>(3 * (size_t)T);
        auto pos = r.arr<float>(3 * (size_t)V);
        auto nrm = r.arr<float>(3 * (size_t)V);
        auto has_n = r.arr<uint8_t>((size_t)V);
        auto uv = r.arr<float>(2 * (size_t)V);
        auto mat_idx = r.arr<int32_t>((size_t)T);
        auto mats = r.arr<MptMaterial>((size_t)M);
        auto emissive = r.arr<int32_t>((size_t)(E > 0 ? E : 1));
        const size_t lut_n[6] = {128 * 128, 128 * 64 * 128, 256 * 16 * 128, 256 * 16 * 128, 32 * 32 * 96, 32 * 32 * 3};
        std::vector<float> lut[6];
        for (int k = 0; k < 6; k++) lut[k] = r.arr<float>(lut_n[k]);
        auto mats2 = r.arr<MptMaterial>((size_t)M2);
        fclose(fin);

        // n_split > 1: the frame tiled across n_split contexts (here all on device 0), gathered
        // with mpt_gather
        mpt_host::GPURenderer gr(std::vector<int>(n_split > 1 ? n_split : 1, 0));
        // test hooks: GPURENDERER_HALO_FAIL="band,call" makes that band's halo exchange fail (the
        // render must throw, not hang); GPURENDERER_RESTIR_AUX=<path> writes the ReSTIR DI output
        // reservoirs (get_aux_buffer, each band's rows from its owner) after the render
        if (const char* hf = getenv("GPURENDERER_HALO_FAIL")) {
            int band = -1, call = -1;
            if (sscanf(hf, "%d,%d", &band, &call) == 2) gr.inject_halo_failure(band, call);
        }
        MptScene s{};
        s.triangle_indices = idx.data(); s.num_triangles = T;
        s.vertices = pos.data(); s.vertex_normals = nrm.data(); s.has_vertex_normals = has_n.data();
        s.texcoords = uv.data(); s.num_vertices = V;
        s.material_indices = mat_idx.data(); s.materials = mats.data(); s.num_materials = M;
        s.emissive_triangle_indices = emissive.data(); s.num_emissive_triangles = E;
        gr.set_scene(s);
        MptLuts L{};
        L.ggx_conductor_ess = lut[0].data(); L.glossy_dielectric_ess = lut[1].data(); L.ggx_glass_ess = lut[2].data();
        L.ggx_glass_inverse_ess = lut[3].data(); L.ggx_thin_glass_ess = lut[4].data(); L.sheen_ltc_params = lut[5].data();
        gr.setup_brdfs_data(L);
        gr.resize(W, H);
        gr.get_render_settings() = settings;
        gr.get_world_settings() = world;
        gr.get_kernel_options() = options;
        gr.get_bsdf_flags() = flags;
        gr.set_camera(camera);
        gr.reset();
        if (M2 > 0) {
            gr.update_materials(mats2);
            if (gr.get_current_materials().size() != (size_t)M2 || gr.get_original_materials().size() != (size_t)M)
                throw std::runtime_error("material lists");
        }
        const size_t px = (size_t)W * H;
        float* display = nullptr;
        if (hipMalloc(&display, px * 3 * sizeof(float)) != hipSuccess) throw std::runtime_error("hipMalloc");
        mpt_host::DisplayBuffers db;
        db.color = display;
        gr.set_display_buffers(db);
        std::vector<MptFrame> frames;
        // GPURENDERER_INTERACT="u0,u1,...": the displayed frames during which the user moves the
        // camera -- RenderWindow.cpp:797-802 sets wants_render_low_resolution = is_interacting() and,
        // with auto_sample_per_frame, one sample per frame while rendering at low resolution
        std::vector<int> interact;
        if (const char* it = getenv("GPURENDERER_INTERACT"))
            for (const char* p = it; *p;) {
                interact.push_back(atoi(p));
                while (*p && *p != ',') p++;
                if (*p == ',') p++;
            }
        const int spf0 = gr.get_render_settings().samples_per_frame;
        int low_frames = 0;
        for (int u = 0; u < n_updates; u++) {   // RenderWindow::render: update() then render() per displayed frame
            if (!interact.empty()) {
                MptRenderSettings& rs = gr.get_render_settings();
                rs.wants_render_low_resolution = std::find(interact.begin(), interact.end(), u) != interact.end();
                const bool low = rs.wants_render_low_resolution && rs.allow_render_low_resolution && rs.accumulate;
                rs.samples_per_frame = (low || gr.was_last_frame_low_resolution()) ? 1 : spf0;
            }
            gr.update();
            if (mode == 0) {
                gr.render();
                frames.insert(frames.end(), gr.last_frames().begin(), gr.last_frames().end());
            } else {
                MptRenderSettings& rs = gr.get_render_settings();
                const int spf = rs.samples_per_frame > 0 ? rs.samples_per_frame : 1;
                gr.map_buffers_for_render();
                for (int i = 1; i <= spf; i++) {
                    if (i == spf) rs.do_update_status_buffers = true;
                    gr.launch_camera_rays();
                    gr.launch_ReSTIR_DI();
                    gr.launch_path_tracing();
                    frames.insert(frames.end(), gr.last_frames().begin(), gr.last_frames().end());
                    rs.sample_number++;
                    rs.denoiser_AOV_accumulation_counter++;
                    rs.need_to_reset = false;
                    rs.restir_di_settings.temporal_buffer_clear_requested = false;
                }
            }
            gr.unmap_buffers();
            low_frames += gr.was_last_frame_low_resolution() ? 1 : 0;
        }
        if (!interact.empty() && low_frames != (int)interact.size()) throw std::runtime_error("was_last_frame_low_resolution");
        gr.synchronize_kernel();
        if (gr.get_render_data().render_settings.sample_number != (int)frames.size())
            throw std::runtime_error("render data sample_number");
        std::vector<float> img(px * 3), direct(px * 3);
        if (hipMemcpy(img.data(), display, px * 3 * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
            throw std::runtime_error("hipMemcpy");
        (void)hipFree(display);
        gr.get_framebuffer(MPT_FB_COLOR, direct.data());
        if (std::memcmp(img.data(), direct.data(), px * 3 * sizeof(float)) != 0)
            throw std::runtime_error("display buffer differs from get_framebuffer");
        std::vector<int32_t> cnt(px);
        gr.get_aux_buffer(MPT_AUX_SAMPLE_COUNT, cnt.data());
        gr.copy_status_buffers();
        MptStatus st = gr.get_status_buffer_values();
        if (const char* ap = getenv("GPURENDERER_RESTIR_AUX")) {
            std::vector<float> res(px * 12);
            gr.get_aux_buffer(MPT_AUX_RESTIR_OUTPUT, res.data());
            FILE* fa = fopen(ap, "wb");
            if (!fa) throw std::runtime_error("cannot open aux output");
            fwrite(res.data(), sizeof(float), res.size(), fa);
            fclose(fa);
        }
        FILE* fo = fopen(argv[2], "wb");
        if (!fo) throw std::runtime_error("cannot open output");
        int32_t nf = (int32_t)frames.size();
        fwrite(&nf, sizeof(nf), 1, fo);
        fwrite(frames.data(), sizeof(MptFrame), frames.size(), fo);
        fwrite(img.data(), sizeof(float), img.size(), fo);
        fwrite(cnt.data(), sizeof(int32_t), cnt.size(), fo);
        fclose(fo);
        printf("ok %d frames, one_ray_active %d\n", nf, (int)st.one_ray_active);
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
