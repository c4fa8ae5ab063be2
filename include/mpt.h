/*
 * mpt.h -- C ABI of the MI355X-native path-tracing hot path ("libmpt").
 *
 * This is the drop-in boundary described in SURVEY.md §8(b).  Every entry point
 * replaces one piece of the reference's GPU launch API (wuyakuma/HIPRT-Path-Tracer,
 * src/Renderer/GPURenderer.h) or of the HIPRT/Orochi glue it sits on:
 *
 *   mpt_create / mpt_destroy      <- GPURenderer::GPURenderer (GPURenderer.h:75,
 *                                    GPURenderer.cpp:48-86) + HIPRTOrochiCtx (HIPRTOrochiCtx.h:20-66)
 *   mpt_upload_scene              <- GPURenderer::set_scene -> set_hiprt_scene_from_scene
 *                                    (GPURenderer.h:220, GPURenderer.cpp:1041-1134) and
 *                                    HIPRTGeometry::build_bvh (HIPRTScene.h:60-87)
 *   mpt_update_materials          <- GPURenderer::update_materials (GPURenderer.h:228)
 *   mpt_set_envmap                <- GPURenderer::set_envmap (GPURenderer.h:222, .cpp:1136-1174)
 *   mpt_set_luts                  <- GPURenderer::setup_brdfs_data (GPURenderer.h:76, .cpp:88-175)
 *   mpt_resize                    <- GPURenderer::resize (GPURenderer.h:172)
 *   mpt_render_frame              <- GPURenderer::render -> launch_camera_rays +
 *                                    launch_path_tracing (GPURenderer.h:139-143,
 *                                    .cpp:408-486), i.e. the CameraRays and FullPathTracer
 *                                    kernels (Device/kernels/CameraRays.h:45,
 *                                    Device/kernels/FullPathTracer.h:99)
 *   mpt_render_frames             <- GPURenderer::render's samples_per_frame loop
 *                                    (GPURenderer.cpp:424-449) as one batched wavefront
 *   mpt_synchronize / mpt_query_done <- GPURenderer::synchronize_kernel / frame_render_done
 *                                    (GPURenderer.h:149-156)
 *   mpt_get_framebuffer           <- the 'pixels' / denoiser AOV interop buffers
 *                                    (GPURenderer.h:193-197, RenderData.h:32-36)
 *   mpt_trace_closest / mpt_trace_any <- hiprtGeomTraversalClosest/AnyHit as called by
 *                                    trace_ray / evaluate_shadow_ray (Device/includes/Intersect.h:114-286)
 *   mpt_bake_lut                  <- GPUBaker::bake_* (Renderer/Baker/GPUBaker.cpp:35-97) and the
 *                                    Device/kernels/Baking/ headers kernels
 *
 * Conventions: every function returns MPT_OK (0) or a negative error code; the
 * message of the last error of the calling thread is in mpt_last_error().  The
 * library never exits the process (the reference logs and calls exit(),
 * HIPRT-Orochi/HIPRTOrochiUtils.cpp:15-47).  All device memory is owned by the
 * context; host arrays passed in are copied before the call returns.  Calls on one
 * context must be externally serialised.  All GPU work of a context is enqueued on
 * the stream given to mpt_create (or the context's own stream).
 *
 * The POD structs below are byte-identical mirrors of the reference's
 * HostDeviceCommon structs (sizes are static_assert-ed in the implementation):
 *   MptMaterial       == RendererMaterial        (HostDeviceCommon/Material.h:29-268), 332 B
 *   MptRenderSettings == HIPRTRenderSettings     (HostDeviceCommon/RenderSettings.h:26-252), 304 B
 *   MptWorldSettings  == WorldSettings           (HostDeviceCommon/WorldSettings.h:18-52), 200 B
 *   MptCamera         == HIPRTCamera             (HostDeviceCommon/HIPRTCamera.h:16-49), 196 B
 */
#ifndef MPT_H
#define MPT_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------- */
/* Status codes                                                               */
/* ------------------------------------------------------------------------- */
#define MPT_OK 0
#define MPT_ERR_INVALID_ARGUMENT (-1)
#define MPT_ERR_HIP (-2)
#define MPT_ERR_NO_SCENE (-3)
#define MPT_ERR_UNSUPPORTED (-4)
#define MPT_ERR_OUT_OF_MEMORY (-5)

/* ------------------------------------------------------------------------- */
/* Compile-time kernel options of the reference (HostDeviceCommon/KernelOptions.h) */
/* become runtime selections of pre-instantiated kernel variants.             */
/* ------------------------------------------------------------------------- */
#define MPT_BSDF_NONE 0        /* BSDF_NONE: Principled BSDF  (KernelOptions.h:21) */
#define MPT_BSDF_LAMBERTIAN 1  /* BSDF_LAMBERTIAN                                   */
#define MPT_BSDF_OREN_NAYAR 2  /* BSDF_OREN_NAYAR (OrenNayar.h; see dev_bsdf.h bsdf_eval) */

#define MPT_LSS_NO_DIRECT_LIGHT_SAMPLING 0 /* KernelOptions.h:50-56 */
#define MPT_LSS_UNIFORM_ONE_LIGHT 1
#define MPT_LSS_BSDF 2
#define MPT_LSS_MIS_LIGHT_BSDF 3
#define MPT_LSS_RIS_BSDF_AND_LIGHT 4
#define MPT_LSS_RESTIR_DI 5

#define MPT_ESS_NO_SAMPLING 0 /* KernelOptions.h:58-60 */
#define MPT_ESS_BINARY_SEARCH 1
#define MPT_ESS_ALIAS_TABLE 2

#define MPT_AMBIENT_NONE 0 /* WorldSettings.h:11-16 */
#define MPT_AMBIENT_UNIFORM 1
#define MPT_AMBIENT_ENVMAP 2

#define MPT_NO_TEXTURE (-1)
#define MPT_CONSTANT_EMISSIVE_TEXTURE (-2)

/* ------------------------------------------------------------------------- */
/* Byte-identical mirrors of the reference PODs                               */
/* ------------------------------------------------------------------------- */
typedef struct MptColor { float r, g, b; } MptColor;           /* ColorRGB32F, Color.h:61 */
typedef struct MptFloat4x4 { float m[4][4]; } MptFloat4x4;      /* float4x4, Math.h:43 */

/* RendererMaterial (HostDeviceCommon/Material.h:29-268).  Field order is the
 * reference's; 'emission' is the (private) last field of SimplifiedRendererMaterial. */
typedef struct MptMaterial {
    bool emissive_texture_used;
    float emission_strength;
    MptColor base_color;
    float roughness;
    float oren_nayar_sigma;
    float metallic;
    float metallic_F90_falloff_exponent;
    MptColor metallic_F82;
    MptColor metallic_F90;
    float anisotropy;
    float anisotropy_rotation;
    float second_roughness_weight;
    float second_roughness;
    float specular;
    float specular_tint;
    MptColor specular_color;
    float specular_darkening;
    float coat;
    MptColor coat_medium_absorption;
    float coat_medium_thickness;
    float coat_roughness;
    float coat_roughening;
    float coat_darkening;
    float coat_anisotropy;
    float coat_anisotropy_rotation;
    float coat_ior;
    float sheen;
    float sheen_roughness;
    MptColor sheen_color;
    float ior;
    float specular_transmission;
    float absorption_at_distance;
    MptColor absorption_color;
    float dispersion_scale;
    float dispersion_abbe_number;
    bool thin_walled;
    float thin_film;
    float thin_film_ior;
    float thin_film_thickness;
    float thin_film_kappa_3;
    float thin_film_hue_shift_degrees;
    float thin_film_base_ior_override;
    bool thin_film_do_ior_override;
    bool srgb;
    float alpha_opacity;
    int32_t dielectric_priority;
    int32_t energy_preservation_monte_carlo_samples;
    bool enforce_strong_energy_conservation;
    MptColor emission;
    /* RendererMaterial texture indices (Material.h:217-266) */
    int32_t normal_map_texture_index;
    int32_t emission_texture_index;
    int32_t base_color_texture_index;
    int32_t roughness_metallic_texture_index;
    int32_t roughness_texture_index;
    int32_t oren_sigma_texture_index;
    int32_t metallic_texture_index;
    int32_t specular_texture_index;
    int32_t specular_tint_texture_index;
    int32_t specular_color_texture_index;
    int32_t anisotropic_texture_index;
    int32_t anisotropic_rotation_texture_index;
    int32_t coat_texture_index;
    int32_t coat_roughness_texture_index;
    int32_t coat_ior_texture_index;
    int32_t sheen_texture_index;
    int32_t sheen_roughness_texture_index;
    int32_t sheen_color_texture_index;
    int32_t specular_transmission_texture_index;
} MptMaterial;

/* ReSTIRDISettings (HostDeviceCommon/ReSTIRDISettings.h:12-195) */
typedef struct MptReSTIRDISettings {
    /* InitialCandidatesSettings */
    int32_t number_of_initial_light_candidates;
    int32_t number_of_initial_bsdf_candidates;
    float envmap_candidate_probability;
    void* ic_output_reservoirs;
    /* TemporalPassSettings */
    bool do_temporal_reuse_pass;
    bool use_permutation_sampling;
    int32_t permutation_sampling_random_bits;
    int32_t max_neighbor_search_count;
    int32_t neighbor_search_radius;
    bool temporal_buffer_clear_requested;
    void* tp_input_reservoirs;
    void* tp_output_reservoirs;
    /* SpatialPassSettings */
    bool do_spatial_reuse_pass;
    int32_t spatial_pass_index;
    int32_t number_of_passes;
    int32_t reuse_radius;
    int32_t reuse_neighbor_count;
    bool do_disocclusion_reuse_boost;
    int32_t disocclusion_reuse_count;
    bool debug_neighbor_location;
    bool do_neighbor_rotation;
    bool allow_converged_neighbors_reuse;
    float converged_neighbor_reuse_probability;
    bool do_visibility_only_last_pass;
    int32_t neighbor_visibility_count;
    void* sp_input_reservoirs;
    void* sp_output_reservoirs;
    /* LightPresamplingSettings */
    int32_t number_of_subsets;
    int32_t subset_size;
    int32_t tile_size;
    void* light_samples;
    /* ReSTIRDISettings */
    bool do_fused_spatiotemporal;
    int32_t m_cap;
    bool use_confidence_weights;
    bool use_normal_similarity_heuristic;
    float normal_similarity_angle_degrees;
    float normal_similarity_angle_precomp;
    bool use_plane_distance_heuristic;
    float plane_distance_threshold;
    bool use_roughness_similarity_heuristic;
    float roughness_similarity_threshold;
    bool do_final_shading_visibility;
    void* restir_output_reservoirs;
} MptReSTIRDISettings;

/* HIPRTRenderSettings (HostDeviceCommon/RenderSettings.h:26-252) */
typedef struct MptRenderSettings {
    bool need_to_reset;
    bool do_update_status_buffers;
    bool accumulate;
    int32_t denoiser_AOV_accumulation_counter;
    int32_t sample_number;
    int32_t samples_per_frame;
    int32_t nb_bounces;
    bool use_russian_roulette;
    int32_t russian_roulette_min_depth;
    float russian_roulette_throughput_clamp;
    int32_t path_russian_roulette_method; /* PathRussianRoulette: 0 MAX_THROUGHPUT, 1 ARNOLD_2014 */
    int32_t freeze_random;
    bool display_NaNs;
    bool allow_render_low_resolution;
    bool wants_render_low_resolution;
    int32_t render_low_resolution_scaling;
    bool enable_adaptive_sampling;
    int32_t adaptive_sampling_min_samples;
    float adaptive_sampling_noise_threshold;
    bool enable_pixel_stop_noise_threshold;
    float stop_pixel_percentage_converged;
    float stop_pixel_noise_threshold;
    float direct_contribution_clamp;
    float envmap_contribution_clamp;
    float indirect_contribution_clamp;
    float minimum_light_contribution;
    int32_t number_of_light_samples;
    bool do_alpha_testing;
    int32_t ris_number_of_light_candidates; /* RISSettings (RenderSettings.h:17-24) */
    int32_t ris_number_of_bsdf_candidates;
    MptReSTIRDISettings restir_di_settings;
} MptRenderSettings;

/* WorldSettings (HostDeviceCommon/WorldSettings.h:18-52).  The pointer fields are
 * ignored by mpt_render_frame: the envmap lives in the context (mpt_set_envmap). */
typedef struct MptWorldSettings {
    int32_t ambient_light_type;
    MptColor uniform_light_color;
    uint32_t envmap_width, envmap_height;
    float envmap_intensity;
    int32_t envmap_scale_background_intensity;
    void* envmap;
    float envmap_total_sum;
    float* envmap_cdf;
    int32_t* alias_table_alias;
    float* alias_table_probas;
    MptFloat4x4 envmap_to_world_matrix;
    MptFloat4x4 world_to_envmap_matrix;
} MptWorldSettings;

/* HIPRTCamera (HostDeviceCommon/HIPRTCamera.h:16-49) */
typedef struct MptCamera {
    MptFloat4x4 inverse_view;
    MptFloat4x4 inverse_projection;
    MptFloat4x4 view_projection;
    bool do_jittering;
} MptCamera;

/* The compile-time options of KernelOptions.h that select code paths on the hot
 * path.  Defaults of the reference: bsdf_override NONE, light_sampling RIS,
 * envmap_sampling ALIAS_TABLE, envmap_bsdf_mis 1, ggx multiple scattering 1. */
typedef struct MptKernelOptions {
    int32_t bsdf_override;                 /* BSDFOverride (KernelOptions.h:116) */
    int32_t direct_light_sampling;         /* DirectLightSamplingStrategy (KernelOptions.h:218) */
    int32_t envmap_sampling;               /* EnvmapSamplingStrategy (KernelOptions.h:231) */
    int32_t envmap_bsdf_mis;               /* EnvmapSamplingDoBSDFMIS (KernelOptions.h:242) */
    int32_t ris_use_visibility;            /* RISUseVisiblityTargetFunction (KernelOptions.h:252) */
    int32_t restir_di_bias_correction_weights;        /* ReSTIR_DI_BiasCorrectionWeights (KernelOptions.h:335),
                                                         MPT_RESTIR_DI_BIAS_* */
    int32_t restir_di_bias_correction_use_visibility; /* ReSTIR_DI_BiasCorrectionUseVisibility (KernelOptions.h:304) */
    int32_t restir_di_later_bounces_sampling_strategy; /* ReSTIR_DI_LaterBouncesSamplingStrategy (KernelOptions.h:355),
                                                          MPT_RESTIR_DI_LATER_BOUNCES_* */
    int32_t restir_di_initial_target_visibility; /* ReSTIR_DI_InitialTargetFunctionVisibility (KernelOptions.h:270), 0 */
    int32_t restir_di_spatial_target_visibility; /* ReSTIR_DI_SpatialTargetFunctionVisibility (KernelOptions.h:279), 1 */
    int32_t restir_di_do_visibility_reuse;       /* ReSTIR_DI_DoVisibilityReuse (KernelOptions.h:289), 1 */
    int32_t restir_di_do_lights_presampling;     /* ReSTIR_DI_DoLightsPresampling (KernelOptions.h:366), 1; 0: no
                                                    presampling pass and no seed drawn for it (restir_di_seeds[0] unused) */
} MptKernelOptions;

#define MPT_RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT 0 /* KernelOptions.h:73-76 */
#define MPT_RESTIR_DI_LATER_BOUNCES_BSDF 1
#define MPT_RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF 2
#define MPT_RESTIR_DI_LATER_BOUNCES_RIS_BSDF_AND_LIGHT 3

#define MPT_RESTIR_DI_BIAS_1_OVER_M 0 /* KernelOptions.h:66-71 */
#define MPT_RESTIR_DI_BIAS_1_OVER_Z 1
#define MPT_RESTIR_DI_BIAS_MIS_LIKE 2
#define MPT_RESTIR_DI_BIAS_MIS_GBH 3
#define MPT_RESTIR_DI_BIAS_PAIRWISE_MIS 4
#define MPT_RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE 5

/* BRDFsData flags (HostDeviceCommon/BSDFsData.h:24-62), the LUTs themselves are
 * uploaded once with mpt_set_luts. */
typedef struct MptBSDFFlags {
    bool white_furnace_mode;
    bool white_furnace_mode_turn_off_emissives;
    bool clearcoat_compensation_approximation;
    int32_t ggx_masking_shadowing; /* 0 HeightCorrelated, 1 HeightUncorrelated */
} MptBSDFFlags;

/* Everything one sample-per-pixel pass needs (the by-value HIPRTRenderData of
 * the reference, minus device pointers which the library owns). */
typedef struct MptFrame {
    MptRenderSettings render_settings;
    MptWorldSettings world_settings;
    MptCamera current_camera;
    MptCamera prev_camera;
    MptKernelOptions options;
    MptBSDFFlags bsdf_flags;
    uint32_t random_seed;   /* HIPRTRenderData::random_seed (RenderData.h:146) */
    int32_t res_x, res_y;   /* int2 res kernel argument */
    /* Framebuffer row partition for multi-GPU tiling: this context renders the
     * rows y with (y / band_height) % band_count == band_index.  (1, 0, 1) renders
     * the whole frame.  Per-pixel RNG seeds use the global pixel index so a
     * partitioned render is bit-identical to a single-device one. */
    int32_t band_height, band_index, band_count;
    /* Seed of the CameraRays launch (GPURenderer::launch_camera_rays draws a new
     * m_rng.xorshift32() per launch, GPURenderer.cpp:468-474); 0 = use random_seed for
     * the camera rays too (CPURenderer: one seed per sample, CPURenderer.cpp:271-287). */
    uint32_t camera_random_seed;
    /* LSS_RESTIR_DI: the seeds ReSTIRDIRenderPass::launch draws from the renderer's RNG
     * (ReSTIRDIRenderPass.cpp:233-264, 298-431) that its kernels see as random_seed:
     * [0] lights presampling, [1] initial candidates, [2] the fused spatiotemporal pass
     * (the draw of configure_spatial_pass_for_fused_spatiotemporal(0), after the temporal
     * seed and the permutation bits) or, unfused, the temporal pass, [3] the
     * permutation-sampling bits (the kernels read them from
     * render_settings.restir_di_settings, where the caller stores them as the reference
     * does), [4 + i] spatial pass i (unfused: i >= 0; fused: i >= 1).  Hence
     * number_of_passes <= 4. */
    uint32_t restir_di_seeds[8];
} MptFrame;

/* Scene arrays as produced by the reference's SceneParser (Scene/SceneParser.h:80-131). */
typedef struct MptScene {
    const int32_t* triangle_indices;   /* 3 * num_triangles */
    int32_t num_triangles;
    const float* vertices;             /* 3 * num_vertices  (float3) */
    const float* vertex_normals;       /* 3 * num_vertices */
    const uint8_t* has_vertex_normals; /* num_vertices */
    const float* texcoords;            /* 2 * num_vertices  (float2) */
    int32_t num_vertices;
    const int32_t* material_indices;   /* num_triangles */
    const MptMaterial* materials;
    int32_t num_materials;
    const int32_t* emissive_triangle_indices;
    int32_t num_emissive_triangles;
    /* 8-bit textures, tightly packed one after the other, RGBA8 per texel */
    int32_t num_textures;
    const uint8_t* const* texture_data; /* num_textures pointers, RGBA8 (4 channels) */
    const int32_t* texture_dims;        /* 2 * num_textures (width, height) */
} MptScene;

/* Energy-compensation LUTs (data/BRDFsData, GPUBakerConstants.h:15-32), float32,
 * x fastest (cos_theta_o), then y (roughness), then z (ior / layer); already flipped
 * vertically as Image32Bit::read_image_hdr(..., flipY=true) does (CPURenderer.cpp:93-132). */
typedef struct MptLuts {
    const float* ggx_conductor_ess;        /* 128 x 128 */
    const float* glossy_dielectric_ess;    /* 128 x 64 x 128 */
    const float* ggx_glass_ess;            /* 256 x 16 x 128 */
    const float* ggx_glass_inverse_ess;    /* 256 x 16 x 128 */
    const float* ggx_thin_glass_ess;       /* 32 x 32 x 96 */
    const float* sheen_ltc_params;         /* 32 x 32 x 3 */
} MptLuts;

/* Counters and timings, cumulative since the last mpt_enable_stats call.
 * Ray counts are always collected; node/triangle counts only with the instrumented
 * traversal; times only when timing is enabled (hipEvents around every traversal launch
 * and around every frame, read back without stalling the stream). */
typedef struct MptStats {
    uint64_t rays_closest;      /* closest-hit queries (camera/continuation + NEE BSDF/light rays) */
    uint64_t rays_any;          /* any-hit (shadow) queries */
    uint64_t node_visits;       /* BVH8 node fetches, all stages (instrumented) */
    uint64_t triangle_tests;    /* triangle record fetches, all stages (instrumented) */
    uint32_t trace_launches;    /* traversal kernel launches */
    uint32_t frames;            /* samples rendered (one per mpt_render_frame, count per mpt_render_frames) */
    double trace_ms;            /* summed traversal kernel time */
    double frame_ms;            /* summed whole-frame time */
    /* per traversal stage: 0 = path rays (camera / continuation, closest hit),
     * 1 = NEE shadow rays (any hit), 2 = NEE BSDF / light rays (closest hit) */
    uint64_t stage_rays[3];         /* queries, always counted */
    uint64_t stage_traversals[3];   /* BVH traversals (instrumented; >= queries: boundary skips retrace) */
    uint64_t stage_nodes[3];
    uint64_t stage_tris[3];
    double stage_ms[3];
    uint32_t stage_launches[3];
    uint32_t shade_launches;
    /* summed time of the other kernels (timing enabled) */
    double camera_ms;
    double shade_ms;
    double resolve_ms;
    double accumulate_ms;
    double compact_ms;
    double restir_ms;           /* ReSTIR DI passes (presampling .. spatial reuse) */
    /* instrumented traversal, per stage: wave-level node / triangle iterations x 64 (the
     * lane slots they occupied); stage_nodes / stage_node_slots = SIMD utilisation */
    uint64_t stage_node_slots[3];
    uint64_t stage_tri_slots[3];
    /* path rays that hit a surface (shaded by the shade stage; the rest by the miss stage) */
    uint64_t path_hits;
    double split_ms;            /* hit / miss partition of the path queue */
    double miss_ms;             /* miss shading (sky / envmap) */
    /* material-class shading: shade_ms / shade_launches time the plain-dielectric kernel
     * (the Lambert override and MPT_SHADE_CLASSES=0: the one shading kernel), these the
     * generic-material kernel and the vertices it shaded */
    double shade_generic_ms;
    uint64_t shade_generic_vertices;
    /* the ReSTIR DI kernels one by one (timing enabled): 0 G-buffer (k_gbuffer), 1 lights
     * presampling, 2 initial candidates, 3 temporal or fused spatiotemporal reuse, 4 spatial
     * reuse passes; summed time and launches */
    double restir_kernel_ms[5];
    uint32_t restir_kernel_launches[5];
    /* the staged reuse passes' plain-class target-function evaluations (k_rsp_eval, Principled
     * BSDF): summed time, launches and evaluation items */
    double restir_eval_ms;
    uint32_t restir_eval_launches;
    uint64_t restir_eval_items;
    /* one-sample launch sets (MPT_GRAPHS): captured HIP graphs and replays of them */
    uint32_t graph_captures;
    uint32_t graph_replays;
    /* path-tracing batches launched as two overlapped halves on two streams (MPT_OVERLAP): their
     * kernels share the GPU, so the per-kernel times above overlap */
    uint32_t overlapped_batches;
    /* the library's halo exchange (mpt_set_halo_native): exchange points served, halo
     * agreements run (the all-reduce of a moving camera), bytes sent to / received from peers
     * (mode 2: the bytes a rank would move; mpt_halo_plan's operations) */
    uint64_t halo_exchanges;
    uint64_t halo_agreements;
    uint64_t halo_bytes_sent;
    uint64_t halo_bytes_received;
    /* batched ReSTIR DI wavefronts whose later bounces ran on the second stream beside the next
     * batch's per-sample chain (MPT_RESTIR_OVERLAP) */
    uint32_t restir_overlapped_batches;
    /* path traversals launched ahead, beside the previous bounce's NEE traversals and resolve
     * (MPT_TRACE_AHEAD): their times and those of the NEE traversals overlap */
    uint32_t trace_ahead_launches;
    /* wavefronts whose bounces ran pipelined (MPT_PIPELINE: a bounce's NEE traversals and resolve
     * beside the next bounce's split and shading): their kernels' times overlap */
    uint32_t pipelined_batches;
} MptStats;

#define MPT_FB_COLOR 0        /* 'pixels': running SUM of samples (RenderData.h:34-36) */
#define MPT_FB_ALBEDO 1       /* denoiser_albedo */
#define MPT_FB_NORMALS 2      /* denoiser_normals */

/* Adaptive-sampling buffers (AuxiliaryBuffers, RenderData.h:62-84), 4 bytes per pixel */
#define MPT_AUX_SAMPLE_COUNT 0            /* pixel_sample_count (int32) */
#define MPT_AUX_CONVERGED_SAMPLE_COUNT 1  /* pixel_converged_sample_count (int32, -1 = not converged) */
#define MPT_AUX_SQUARED_LUMINANCE 2       /* pixel_squared_luminance (float) */
/* ReSTIR DI reservoirs of the whole frame (3 float4 per pixel: {M, weight_sum, UCW, triangle},
 * {point, target_function}, {flags}): the last frame's output, the other spatial buffer (the
 * fused pass's output when a spatial pass followed it) and the initial candidates */
#define MPT_AUX_RESTIR_OUTPUT 3
#define MPT_AUX_RESTIR_OTHER 4
#define MPT_AUX_RESTIR_INITIAL 5

/* StatusBuffersValues (Renderer/StatusBuffersValues.h:9-21) */
typedef struct MptStatus {
    bool one_ray_active;              /* at least one pixel still sampled in the last frame */
    uint32_t pixel_converged_count;   /* pixels converged (adaptive sampling / stop noise threshold) */
} MptStatus;

typedef struct MptContext MptContext;

/* ReSTIR DI across a row partition (the C4 configuration on 1-8 GPUs).
 * The spatial / spatiotemporal reuse passes read neighbouring pixels' G-buffer entries and
 * reservoirs (FusedSpatiotemporalReuse.h:112-586, SpatialReuse.h:52-348), and the temporal
 * reuse reads the previous frame's data around each pixel's reprojection (Utils.h:371-421),
 * so a context that renders one contiguous band of rows (band_count > 1,
 * band_height * band_count >= res_y) keeps its ReSTIR buffers frame-sized and asks the host
 * to fill the rows around its band from the contexts that own them.  The result is
 * bit-identical to a single-context render.
 *
 * Each buffer is a frame-sized, row-major array of per-pixel records on the context's device
 * (pixel (x, y) at byte (y * res_x + x) * bytes_per_pixel).  The callback is invoked from
 * mpt_render_frame after the producing kernels were enqueued on `stream` (not necessarily
 * finished).  Before it returns it must have arranged (enqueued on `stream`, or completed)
 * that rows [max(0, own_y0 - halo_rows), own_y0) and [own_y1, min(res_y, own_y1 + halo_rows))
 * of every buffer hold the owning contexts' values, and must provide its own rows to its
 * neighbours' callbacks of the same phase.  Returns 0, or non-zero to fail the frame.
 *
 * Phases, in order, per frame:
 *  MPT_HALO_GBUFFER       after the G-buffer pass.  On entry halo_rows is what THIS context
 *                         needs (measured: the largest reprojection offset of its pixels
 *                         plus the reuse radius and temporal search extent -- the
 *                         reference's reprojection is not confined to a pixel's
 *                         neighbourhood).  The callback agrees on the maximum over all
 *                         contexts, exchanges with it and stores it back in halo_rows --
 *                         unless halo_agreed is set: the frame's camera did not move, so every
 *                         context derived the same halo from the frame alone (a pixel
 *                         reprojects onto itself) without waiting for its G-buffer, and the
 *                         callback may skip the agreement (and any host synchronisation).
 *  MPT_HALO_PREV_GBUFFER  only when the agreed halo grew since the previous frame: the
 *                         previous frame's G-buffer rows the context did not maintain.
 *  MPT_HALO_RESERVOIRS    the temporal input before the fused pass (pass 0), then the
 *                         output of pass i - 1 before spatial pass i. */
#define MPT_HALO_GBUFFER 0
#define MPT_HALO_RESERVOIRS 1
#define MPT_HALO_PREV_GBUFFER 2
#define MPT_HALO_MAX_BUFFERS 12
typedef struct MptHaloExchange {
    int32_t phase;        /* MPT_HALO_* */
    int32_t pass;         /* reservoirs: the reuse pass about to read them (0 = fused spatiotemporal) */
    int32_t res_x, res_y;
    int32_t own_y0, own_y1;
    int32_t halo_rows;    /* MPT_HALO_GBUFFER: in = needed here, out = agreed maximum */
    int32_t n_buffers;
    void* buffers[MPT_HALO_MAX_BUFFERS];
    int64_t bytes_per_pixel[MPT_HALO_MAX_BUFFERS];
    void* stream;         /* hipStream_t */
    int32_t halo_agreed;  /* MPT_HALO_GBUFFER: halo_rows is already the same in every context */
} MptHaloExchange;
typedef int (*MptHaloExchangeFn)(void* user, MptHaloExchange* x);

const char* mpt_last_error(void);
int mpt_version(void);
/* sizes of the mirrored structs as compiled into the library (ABI check): MptMaterial,
 * MptRenderSettings, MptWorldSettings, MptCamera, MptFrame, MptScene, MptStats */
int mpt_abi_sizes(int32_t* out_sizes, int n);
/* The HIP device's marketing name, its gfx architecture string and compute-unit count (the
 * bench line's device identity); any output may be NULL. */
int mpt_device_info(int device, char* name, int32_t name_cap, char* arch, int32_t arch_cap, int32_t* out_cus);

int mpt_create(int device, void* hip_stream, MptContext** out_ctx);
int mpt_destroy(MptContext* ctx);
int mpt_upload_scene(MptContext* ctx, const MptScene* scene);
int mpt_update_materials(MptContext* ctx, const MptMaterial* materials, int32_t count);
int mpt_set_envmap(MptContext* ctx, const float* rgba, int32_t width, int32_t height,
                   const float* alias_probas, const int32_t* alias_indices, float luminance_total_sum);
/* Vose alias table in double precision, Image32Bit::compute_alias_table (Image/Image.cpp:579-659) */
int mpt_build_alias_table(const float* rgba, int32_t width, int32_t height,
                          float* out_probas, int32_t* out_alias, float* out_luminance_sum);
/* ESS_BINARY_SEARCH: the envmap luminance CDF, Image32Bit::compute_cdf (Image/Image.cpp:553-574),
 * and its upload (GPURenderer::set_envmap / RendererEnvmap.cpp:119-125; total = last element) */
int mpt_build_envmap_cdf(const float* rgba, int32_t width, int32_t height, float* out_cdf, float* out_total_sum);
int mpt_set_envmap_cdf(MptContext* ctx, const float* cdf, float total_sum);
int mpt_set_luts(MptContext* ctx, const MptLuts* luts);
int mpt_resize(MptContext* ctx, int32_t width, int32_t height);
/* Renders one sample per pixel of the context's partition, accumulating into the
 * sum framebuffer (assign when render_settings.sample_number == 0). Asynchronous. */
int mpt_render_frame(MptContext* ctx, const MptFrame* frame);
/* Renders count consecutive samples (GPURenderer::render's samples_per_frame loop,
 * GPURenderer.cpp:424-449): frames[k] is the frame of the k-th sample, each with its own
 * sample_number / seeds.  Runs of frames that differ only in sample_number, random_seed,
 * camera_random_seed, denoiser_AOV_accumulation_counter, need_to_reset and
 * do_update_status_buffers (and, for ReSTIR DI, restir_di_seeds, the permutation bits and
 * temporal_buffer_clear_requested), and need no per-sample feedback (no adaptive sampling or
 * stop-noise threshold), are traced as ONE wavefront of up to max_batch
 * (<= MPT_MAX_BATCH; <= 0: see MPT_DEFAULT_WAVEFRONT_PATHS) samples per pixel -- ReSTIR DI
 * samples (at most 32, not across a partition) run their camera rays, reuse passes and
 * first bounce one after the other and share the later bounces; the result is bit-identical
 * to count mpt_render_frame calls (samples are added to the sums in order).  Other frames
 * are rendered one by one.  Asynchronous. */
#define MPT_MAX_BATCH 128
/* max_batch <= 0 picks the wavefront size: MPT_DEFAULT_WAVEFRONT_PATHS paths (samples x pixels of
 * the partition) per launch, at most MPT_MAX_BATCH samples, and at most half of the device
 * memory that is free or already held by the context's path state (~460 B per path, +332 B in
 * textured scenes).  Whatever max_batch is, a wavefront whose path state cannot be allocated
 * is halved (the result is bit-identical) before MPT_ERR_OUT_OF_MEMORY is returned. */
#define MPT_DEFAULT_WAVEFRONT_PATHS (1 << 25)
/* paths of one wavefront (and pixels of one frame) are limited to 2^29 */
#define MPT_MAX_WAVEFRONT_PATHS (1 << 29)
int mpt_render_frames(MptContext* ctx, const MptFrame* frames, int32_t count, int32_t max_batch);
/* Installs the halo exchange of a partitioned ReSTIR DI context (see MptHaloExchange);
 * fn = NULL removes it.  Required before rendering LSS_RESTIR_DI with band_count > 1. */
int mpt_set_halo_exchange(MptContext* ctx, MptHaloExchangeFn fn, void* user);
int mpt_synchronize(MptContext* ctx);
int mpt_query_done(MptContext* ctx, int* out_done);
/* Copies the partition's rows of a framebuffer (band-major compact layout: the
 * rows owned by this context in increasing y) to dst; dst may be host or device. */
int mpt_get_framebuffer(MptContext* ctx, int kind, float* dst, int dst_is_device);
int mpt_partition_rows(int32_t res_y, int32_t band_height, int32_t band_index, int32_t band_count);
/* Multi-GPU output (SURVEY.md §8b Outputs row; GPURenderer.cpp:583-598 hands the one device's
 * 'pixels' to the display).  n contexts render the n row partitions of one frame (MptFrame
 * band_count == n, band_index 0..n-1, one band_height, same resolution; each on its own GPU or
 * several on one).  mpt_gather assembles buffer `kind` of the whole frame, row-major
 * (res_y x res_x), into dst on ctxs[root]'s device (dst_is_device) or in host memory: every
 * context's compact rows go out on its own stream (after its frames) as strided 2D copies --
 * peer copies over xGMI when the devices differ.  One host process drives all contexts.
 * Synchronous.  kind: MPT_FB_* (3 floats per pixel) or MPT_GATHER_AUX + MPT_AUX_SAMPLE_COUNT /
 * _CONVERGED_SAMPLE_COUNT / _SQUARED_LUMINANCE (4 bytes per pixel). */
#define MPT_GATHER_AUX 16
int mpt_gather(MptContext* const* ctxs, int32_t n, int32_t root, int kind, void* dst, int dst_is_device);
/* One process per GPU: an RCCL communicator over the ranks of the partition (loaded from
 * librccl.so.1 on first use).  Rank 0 calls mpt_comm_unique_id and shares the id out of band;
 * every rank then calls mpt_comm_init on its context (ncclCommInitRank, collective).
 * mpt_comm_gather is collective over the ranks: rank k's frames must carry band_count = ranks,
 * band_index = k; each rank's compact rows (padded to the largest band) travel with one
 * ncclGather over xGMI to the root, which re-interleaves them into dst (row-major frame; device
 * or host).  dst is ignored on the other ranks.  The communicator is destroyed with the
 * context.  Synchronous. */
#define MPT_COMM_ID_BYTES 128
int mpt_comm_unique_id(uint8_t* out_id, int32_t cap);
int mpt_comm_init(MptContext* ctx, int32_t nranks, int32_t rank, const uint8_t* id);
int mpt_comm_gather(MptContext* ctx, int32_t root, int kind, void* dst, int dst_is_device);
/* ReSTIR DI across the ranks of the communicator without a host callback: rank k's frames carry
 * the contiguous band (band_height = ceil(res_y / ranks), band_index = k, band_count = ranks) and
 * the library exchanges the halo rows itself -- one ncclGroupStart / ncclSend / ncclRecv group per
 * exchange point on the context's stream, the halo agreement an ncclAllReduce (max), skipped when
 * the camera did not move (MptHaloExchange.halo_agreed).  mode: 1 RCCL (after mpt_comm_init),
 * 2 the one-GPU rehearsal (the bytes a rank would receive moved by one local device copy; the
 * rows keep what the buffers held -- timing only), 0 off.  Replaces mpt_set_halo_exchange's
 * callback. */
int mpt_set_halo_native(MptContext* ctx, int32_t mode);
/* The bounce pipeline of single-stream path-tracing wavefronts (default 1, or MPT_PIPELINE at
 * mpt_create): 1 a bounce's NEE traversals and resolve beside the next bounce's split and shading,
 * 0 in line.  Images are identical either way; 0 gives every kernel the GPU to itself (the bench's
 * solo roofline).  Takes effect at the next launch; no reference counterpart (a launch schedule). */
int mpt_set_pipeline(MptContext* ctx, int32_t mode);
/* One point-to-point operation of a halo exchange point: `buffer`'s rows [row_lo, row_hi)
 * sent to (recv = 0) or received from (recv = 1) band `peer`. */
typedef struct MptHaloOp {
    int32_t peer;
    int32_t recv;
    int32_t buffer;
    int32_t row_lo, row_hi;
} MptHaloOp;
/* The operations mpt_set_halo_native's exchange issues, in issue order, for band band_index of
 * band_count contiguous bands of band_height rows (res_y rows in all), the agreed halo_rows and
 * n_buffers buffers: per peer in increasing order, per buffer, the sends of this band's rows in
 * the peer's upper and lower halo, then the receives of the peer's rows in this band's upper and
 * lower halo.  Writes at most cap entries to out, returns the count (< 0: error).  Host only. */
int mpt_halo_plan(int32_t res_y, int32_t band_height, int32_t band_count, int32_t band_index, int32_t halo_rows,
                  int32_t n_buffers, MptHaloOp* out, int32_t cap);
/* Status buffers: mpt_clear_status <- GPURenderer::internal_update_clear_device_status_buffers
 * (GPURenderer.cpp:275-283, once per displayed frame); the last sample of the frame sets
 * render_settings.do_update_status_buffers; mpt_query_status <- copy_status_buffers (.cpp:269-273). */
int mpt_clear_status(MptContext* ctx);
int mpt_query_status(MptContext* ctx, MptStatus* out);
/* Copies an MPT_AUX_* buffer of the partition (n_slots * 4 bytes; the ReSTIR DI kinds: frame pixels * 48 bytes) to dst (host or device). */
int mpt_get_aux_buffer(MptContext* ctx, int kind, void* dst, int dst_is_device);
int mpt_enable_stats(MptContext* ctx, int enable, int instrumented);
int mpt_get_stats(MptContext* ctx, MptStats* out);
/* Energy-compensation LUT baker, GPUBaker::bake_* (Renderer/Baker/GPUBaker.cpp:35-97,
 * GPUBakerKernel.cpp:22-151, Device/kernels/Baking/ headers): Monte-Carlo directional albedo of
 * a GGX lobe per texel, x = cos(theta_o) fastest, then y = roughness, then z = IOR (F0^4
 * parameterisation), with the reference's launch structure and seeds (so the table is
 * deterministic), integration_sample_count samples per texel.  The output is the baked
 * buffer as the reference writes it to its .hdr files (rows not flipped; the renderer's
 * MptLuts hold each slice flipped vertically, as read_image_hdr(flipY=true) loads them).
 * Reference sizes / sample counts (GPUBakerConstants.h:15-32, *Settings.h):
 *   GGX_CONDUCTOR       128 x 128 x 1,  65536        GGX_FRESNEL 256 x 256 x 256, 65536
 *   GLOSSY_DIELECTRIC   128 x 64 x 128, 131072       GGX_GLASS(_INVERSE) 256 x 16 x 128, 65536
 *   GGX_THIN_GLASS      32 x 32 x 96,   65536
 * Synchronous; out may be host or device memory. */
#define MPT_BAKE_GGX_CONDUCTOR 0
#define MPT_BAKE_GGX_FRESNEL 1
#define MPT_BAKE_GLOSSY_DIELECTRIC 2
#define MPT_BAKE_GGX_GLASS 3
#define MPT_BAKE_GGX_GLASS_INVERSE 4
#define MPT_BAKE_GGX_THIN_GLASS 5
int mpt_bake_lut(MptContext* ctx, int kind, int32_t width, int32_t height, int32_t depth, int32_t sample_count,
                 float* out, int out_is_device);
/* Raw ray queries against the uploaded BVH8 (parity / microbenchmarks).
 * rays: n * 8 floats (ox, oy, oz, tmin_unused, dx, dy, dz, tmax); last_hit: n ints (-1 = none).
 * Outputs (may be NULL): prim (n ints, -1 on miss), t, u, v (n floats).  Host or device pointers. */
int mpt_trace_closest(MptContext* ctx, const float* rays, const int32_t* last_hit, int32_t n,
                      int32_t* out_prim, float* out_t, float* out_u, float* out_v, int pointers_are_device);
int mpt_trace_any(MptContext* ctx, const float* rays, const int32_t* last_hit, int32_t n,
                  uint8_t* out_occluded, int pointers_are_device);

/* Host helper of the glTF texture loader (mpt/image.py; the reference decodes textures with
 * stb_image in Image8Bit::read_image, Image.cpp:33-61): reverses the PNG scanline filters
 * (None / Sub / Up / Average / Paeth) of `rows` inflated rows, each a filter-type byte
 * followed by row_bytes bytes, into out (rows * row_bytes).  bpp = bytes per complete pixel
 * (rounded up to 1).  No context, no GPU. */
int mpt_png_unfilter(const uint8_t* filtered, int64_t filtered_size, uint8_t* out, int32_t rows, int32_t row_bytes,
                     int32_t bpp);
/* JPEG decode with stb_image's semantics (stbi_load in Image8Bit::read_image, Image.cpp:33-61: the
 * reference's textured scene ships JPEG textures): baseline / extended / progressive Huffman,
 * 1 / 3 / 4 components, any integer sampling ratio; the islow integer IDCT, the 2:1 triangle
 * upsampling and fixed-point YCbCr conversion of stb_image's x86-64 build, bit for bit.
 * req_comp 0 = the file's own (3 for colour, 1 for grey), else 1..4.  out = NULL: only the
 * header is read (w, h, the file's component count); else out_cap >= w * h * n bytes, rows top
 * to bottom.  No context, no GPU. */
int mpt_jpeg_decode(const uint8_t* data, int64_t size, int32_t req_comp, uint8_t* out, int64_t out_cap,
                    int32_t* out_w, int32_t* out_h, int32_t* out_comp);
/* Radiance .hdr (RGBE, flat or RLE scanlines) decode with stbi_loadf's semantics
 * (Image32Bit::read_image_hdr, Image.cpp:342-370: envmaps, RendererEnvmap.cpp:39-48, and the
 * baked LUTs, GPURenderer.cpp:122-170): float = mantissa * 2^(e - 136), req_comp 1 / 2 average the
 * three channels, alpha 1.  out = NULL: dimensions only.  Rows top to bottom (the caller flips). */
int mpt_hdr_decode(const uint8_t* data, int64_t size, int32_t req_comp, float* out, int64_t out_cap,
                   int32_t* out_w, int32_t* out_h);

#ifdef __cplusplus
}
#endif

#endif /* MPT_H */
