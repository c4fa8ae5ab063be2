"""ctypes mirrors of include/mpt.h and the reference's default values.

The structs are byte-identical to the reference PODs (sizes checked against the
library by ``mpt_abi_sizes`` in tests/test_abi.py).  Default values follow the
reference's in-class initialisers:

* ``RendererMaterial``    -- HostDeviceCommon/Material.h:29-268
* ``HIPRTRenderSettings`` -- HostDeviceCommon/RenderSettings.h:26-252
* ``ReSTIRDISettings``    -- HostDeviceCommon/ReSTIRDISettings.h:12-195
* ``WorldSettings``       -- HostDeviceCommon/WorldSettings.h:18-52
* ``HIPRTCamera``         -- HostDeviceCommon/HIPRTCamera.h:16-49
"""
import ctypes as C

c_bool = C.c_bool
f32 = C.c_float
i32 = C.c_int32
u32 = C.c_uint32
vp = C.c_void_p


class Color(C.Structure):
    _fields_ = [("r", f32), ("g", f32), ("b", f32)]

    def __init__(self, r=0.0, g=None, b=None):
        if g is None:
            g = b = r
        super().__init__(r, g, b)


class Float4x4(C.Structure):
    _fields_ = [("m", (f32 * 4) * 4)]


def identity4():
    m = Float4x4()
    for i in range(4):
        m.m[i][i] = 1.0
    return m


_MAT_FIELDS = [
    ("emissive_texture_used", c_bool), ("emission_strength", f32), ("base_color", Color),
    ("roughness", f32), ("oren_nayar_sigma", f32), ("metallic", f32),
    ("metallic_F90_falloff_exponent", f32), ("metallic_F82", Color), ("metallic_F90", Color),
    ("anisotropy", f32), ("anisotropy_rotation", f32), ("second_roughness_weight", f32),
    ("second_roughness", f32), ("specular", f32), ("specular_tint", f32), ("specular_color", Color),
    ("specular_darkening", f32), ("coat", f32), ("coat_medium_absorption", Color),
    ("coat_medium_thickness", f32), ("coat_roughness", f32), ("coat_roughening", f32),
    ("coat_darkening", f32), ("coat_anisotropy", f32), ("coat_anisotropy_rotation", f32),
    ("coat_ior", f32), ("sheen", f32), ("sheen_roughness", f32), ("sheen_color", Color),
    ("ior", f32), ("specular_transmission", f32), ("absorption_at_distance", f32),
    ("absorption_color", Color), ("dispersion_scale", f32), ("dispersion_abbe_number", f32),
    ("thin_walled", c_bool), ("thin_film", f32), ("thin_film_ior", f32),
    ("thin_film_thickness", f32), ("thin_film_kappa_3", f32), ("thin_film_hue_shift_degrees", f32),
    ("thin_film_base_ior_override", f32), ("thin_film_do_ior_override", c_bool), ("srgb", c_bool),
    ("alpha_opacity", f32), ("dielectric_priority", i32),
    ("energy_preservation_monte_carlo_samples", i32), ("enforce_strong_energy_conservation", c_bool),
    ("emission", Color),
]
_TEX_FIELDS = [
    "normal_map_texture_index", "emission_texture_index", "base_color_texture_index",
    "roughness_metallic_texture_index", "roughness_texture_index", "oren_sigma_texture_index",
    "metallic_texture_index", "specular_texture_index", "specular_tint_texture_index",
    "specular_color_texture_index", "anisotropic_texture_index",
    "anisotropic_rotation_texture_index", "coat_texture_index", "coat_roughness_texture_index",
    "coat_ior_texture_index", "sheen_texture_index", "sheen_roughness_texture_index",
    "sheen_color_texture_index", "specular_transmission_texture_index",
]


class Material(C.Structure):
    _fields_ = _MAT_FIELDS + [(n, i32) for n in _TEX_FIELDS]

    # Nested-dielectric priority of non-transmissive materials, set by
    # SimplifiedRendererMaterial::precompute_properties (Material.h:66-71):
    # (1 << StackPriorityEntry::PRIORITY_MAXIMUM) - 1 with PRIORITY_MAXIMUM = 15.
    OPAQUE_PRIORITY = (1 << 15) - 1
    ROUGHNESS_CLAMP = 1.0e-4

    @classmethod
    def default(cls):
        """In-class initialisers of SimplifiedRendererMaterial / RendererMaterial."""
        m = cls()
        m.emissive_texture_used = False
        m.emission_strength = 1.0
        m.base_color = Color(1.0)
        m.roughness = 0.3
        m.oren_nayar_sigma = 0.34906585039886591538
        m.metallic = 0.0
        m.metallic_F90_falloff_exponent = 5.0
        m.metallic_F82 = Color(1.0)
        m.metallic_F90 = Color(1.0)
        m.anisotropy = 0.0
        m.anisotropy_rotation = 0.0
        m.second_roughness_weight = 0.0
        m.second_roughness = 0.5
        m.specular = 1.0
        m.specular_tint = 1.0
        m.specular_color = Color(1.0)
        m.specular_darkening = 0.0
        m.coat = 0.0
        m.coat_medium_absorption = Color(1.0)
        m.coat_medium_thickness = 5.0
        m.coat_roughness = 0.0
        m.coat_roughening = 1.0
        m.coat_darkening = 1.0
        m.coat_anisotropy = 0.0
        m.coat_anisotropy_rotation = 0.0
        m.coat_ior = 1.5
        m.sheen = 0.0
        m.sheen_roughness = 0.5
        m.sheen_color = Color(1.0)
        m.ior = 1.40
        m.specular_transmission = 0.0
        m.absorption_at_distance = 1.0
        m.absorption_color = Color(1.0)
        m.dispersion_scale = 0.0
        m.dispersion_abbe_number = 20.0
        m.thin_walled = False
        m.thin_film = 0.0
        m.thin_film_ior = 1.3
        m.thin_film_thickness = 500.0
        m.thin_film_kappa_3 = 0.0
        m.thin_film_hue_shift_degrees = 0.0
        m.thin_film_base_ior_override = 1.0
        m.thin_film_do_ior_override = False
        m.srgb = True
        m.alpha_opacity = 1.0
        m.dielectric_priority = 0
        m.energy_preservation_monte_carlo_samples = 12
        m.enforce_strong_energy_conservation = False
        m.emission = Color(0.0)
        for n in _TEX_FIELDS:
            setattr(m, n, -1)
        return m

    def make_safe(self):
        """SimplifiedRendererMaterial::make_safe (Material.h:44-60), float32 semantics."""
        import numpy as np
        f = np.float32
        rc = f(self.ROUGHNESS_CLAMP)
        self.roughness = float(max(rc, f(self.roughness)))
        self.coat_roughness = float(max(rc, f(self.coat_roughness)))
        self.sheen_roughness = float(max(rc, f(self.sheen_roughness)))
        self.emission = Color(max(0.0, self.emission.r), max(0.0, self.emission.g), max(0.0, self.emission.b))
        self.emission_strength = max(0.0, self.emission_strength)
        self.absorption_at_distance = float(max(f(self.absorption_at_distance), f(1.0e-4)))
        lo = float(f(1.0) / f(512.0))
        ac = self.absorption_color
        self.absorption_color = Color(max(ac.r, lo), max(ac.g, lo), max(ac.b, lo))
        self.thin_film_ior = float(max(f(1.0005), f(self.thin_film_ior)))

    def precompute_properties(self):
        """SimplifiedRendererMaterial::precompute_properties (Material.h:66-71)."""
        if self.specular_transmission == 0.0:
            self.dielectric_priority = self.OPAQUE_PRIORITY


class ReSTIRDISettings(C.Structure):
    _fields_ = [
        ("number_of_initial_light_candidates", i32), ("number_of_initial_bsdf_candidates", i32),
        ("envmap_candidate_probability", f32), ("ic_output_reservoirs", vp),
        ("do_temporal_reuse_pass", c_bool), ("use_permutation_sampling", c_bool),
        ("permutation_sampling_random_bits", i32), ("max_neighbor_search_count", i32),
        ("neighbor_search_radius", i32), ("temporal_buffer_clear_requested", c_bool),
        ("tp_input_reservoirs", vp), ("tp_output_reservoirs", vp),
        ("do_spatial_reuse_pass", c_bool), ("spatial_pass_index", i32), ("number_of_passes", i32),
        ("reuse_radius", i32), ("reuse_neighbor_count", i32), ("do_disocclusion_reuse_boost", c_bool),
        ("disocclusion_reuse_count", i32), ("debug_neighbor_location", c_bool),
        ("do_neighbor_rotation", c_bool), ("allow_converged_neighbors_reuse", c_bool),
        ("converged_neighbor_reuse_probability", f32), ("do_visibility_only_last_pass", c_bool),
        ("neighbor_visibility_count", i32), ("sp_input_reservoirs", vp), ("sp_output_reservoirs", vp),
        ("number_of_subsets", i32), ("subset_size", i32), ("tile_size", i32), ("light_samples", vp),
        ("do_fused_spatiotemporal", c_bool), ("m_cap", i32), ("use_confidence_weights", c_bool),
        ("use_normal_similarity_heuristic", c_bool), ("normal_similarity_angle_degrees", f32),
        ("normal_similarity_angle_precomp", f32), ("use_plane_distance_heuristic", c_bool),
        ("plane_distance_threshold", f32), ("use_roughness_similarity_heuristic", c_bool),
        ("roughness_similarity_threshold", f32), ("do_final_shading_visibility", c_bool),
        ("restir_output_reservoirs", vp),
    ]

    @classmethod
    def default(cls):
        s = cls()
        s.number_of_initial_light_candidates = 4
        s.number_of_initial_bsdf_candidates = 1
        s.envmap_candidate_probability = 0.25
        s.do_temporal_reuse_pass = True
        s.use_permutation_sampling = False
        s.permutation_sampling_random_bits = 42
        s.max_neighbor_search_count = 8
        s.neighbor_search_radius = 4
        s.do_spatial_reuse_pass = True
        s.number_of_passes = 2
        s.reuse_radius = 16
        s.reuse_neighbor_count = 2
        s.do_disocclusion_reuse_boost = True
        s.disocclusion_reuse_count = 5
        s.do_neighbor_rotation = True
        s.converged_neighbor_reuse_probability = 0.5
        s.do_visibility_only_last_pass = True
        s.neighbor_visibility_count = 5
        s.number_of_subsets = 128
        s.subset_size = 1024
        s.tile_size = 8
        s.do_fused_spatiotemporal = True
        s.m_cap = 25
        s.use_confidence_weights = True
        s.use_normal_similarity_heuristic = True
        s.normal_similarity_angle_degrees = 25.0
        s.normal_similarity_angle_precomp = 0.906307787
        s.use_plane_distance_heuristic = True
        s.plane_distance_threshold = 0.1
        s.roughness_similarity_threshold = 0.25
        s.do_final_shading_visibility = True
        return s


class RenderSettings(C.Structure):
    _fields_ = [
        ("need_to_reset", c_bool), ("do_update_status_buffers", c_bool), ("accumulate", c_bool),
        ("denoiser_AOV_accumulation_counter", i32), ("sample_number", i32),
        ("samples_per_frame", i32), ("nb_bounces", i32), ("use_russian_roulette", c_bool),
        ("russian_roulette_min_depth", i32), ("russian_roulette_throughput_clamp", f32),
        ("path_russian_roulette_method", i32), ("freeze_random", i32), ("display_NaNs", c_bool),
        ("allow_render_low_resolution", c_bool), ("wants_render_low_resolution", c_bool),
        ("render_low_resolution_scaling", i32), ("enable_adaptive_sampling", c_bool),
        ("adaptive_sampling_min_samples", i32), ("adaptive_sampling_noise_threshold", f32),
        ("enable_pixel_stop_noise_threshold", c_bool), ("stop_pixel_percentage_converged", f32),
        ("stop_pixel_noise_threshold", f32), ("direct_contribution_clamp", f32),
        ("envmap_contribution_clamp", f32), ("indirect_contribution_clamp", f32),
        ("minimum_light_contribution", f32), ("number_of_light_samples", i32),
        ("do_alpha_testing", c_bool), ("ris_number_of_light_candidates", i32),
        ("ris_number_of_bsdf_candidates", i32), ("restir_di_settings", ReSTIRDISettings),
    ]

    @classmethod
    def default(cls):
        s = cls()
        s.need_to_reset = True
        s.do_update_status_buffers = False
        s.accumulate = True
        s.denoiser_AOV_accumulation_counter = 0
        s.sample_number = 0
        s.samples_per_frame = 1
        s.nb_bounces = 3
        s.use_russian_roulette = True
        s.russian_roulette_min_depth = 2
        s.russian_roulette_throughput_clamp = 10.0
        s.path_russian_roulette_method = 0
        s.freeze_random = 0
        s.display_NaNs = False
        s.allow_render_low_resolution = True
        s.wants_render_low_resolution = False
        s.render_low_resolution_scaling = 2
        s.enable_adaptive_sampling = True
        s.adaptive_sampling_min_samples = 64
        s.adaptive_sampling_noise_threshold = 0.3
        s.enable_pixel_stop_noise_threshold = True
        s.stop_pixel_percentage_converged = 90.0
        s.stop_pixel_noise_threshold = 0.0
        s.direct_contribution_clamp = 0.0
        s.envmap_contribution_clamp = 0.0
        s.indirect_contribution_clamp = 15.0
        s.minimum_light_contribution = 0.08
        s.number_of_light_samples = 1
        s.do_alpha_testing = True
        s.ris_number_of_light_candidates = 4
        s.ris_number_of_bsdf_candidates = 1
        s.restir_di_settings = ReSTIRDISettings.default()
        return s


class WorldSettings(C.Structure):
    _fields_ = [
        ("ambient_light_type", i32), ("uniform_light_color", Color), ("envmap_width", u32),
        ("envmap_height", u32), ("envmap_intensity", f32), ("envmap_scale_background_intensity", i32),
        ("envmap", vp), ("envmap_total_sum", f32), ("envmap_cdf", vp), ("alias_table_alias", vp),
        ("alias_table_probas", vp), ("envmap_to_world_matrix", Float4x4),
        ("world_to_envmap_matrix", Float4x4),
    ]

    @classmethod
    def default(cls):
        w = cls()
        w.ambient_light_type = 1  # UNIFORM
        w.uniform_light_color = Color(0.5)
        w.envmap_intensity = 1.0
        w.envmap_scale_background_intensity = 0
        w.envmap_to_world_matrix = identity4()
        w.world_to_envmap_matrix = identity4()
        return w


class Camera(C.Structure):
    _fields_ = [("inverse_view", Float4x4), ("inverse_projection", Float4x4),
                ("view_projection", Float4x4), ("do_jittering", c_bool)]


RESTIR_DI_BIAS_1_OVER_M, RESTIR_DI_BIAS_1_OVER_Z, RESTIR_DI_BIAS_MIS_LIKE = 0, 1, 2
RESTIR_DI_BIAS_MIS_GBH, RESTIR_DI_BIAS_PAIRWISE_MIS, RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE = 3, 4, 5
RESTIR_DI_LATER_BOUNCES_UNIFORM_ONE_LIGHT, RESTIR_DI_LATER_BOUNCES_BSDF = 0, 1
RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF, RESTIR_DI_LATER_BOUNCES_RIS_BSDF_AND_LIGHT = 2, 3


class KernelOptions(C.Structure):
    _fields_ = [("bsdf_override", i32), ("direct_light_sampling", i32), ("envmap_sampling", i32),
                ("envmap_bsdf_mis", i32), ("ris_use_visibility", i32), ("restir_di_bias_correction_weights", i32),
                ("restir_di_bias_correction_use_visibility", i32), ("restir_di_later_bounces_sampling_strategy", i32),
                ("restir_di_initial_target_visibility", i32), ("restir_di_spatial_target_visibility", i32),
                ("restir_di_do_visibility_reuse", i32), ("restir_di_do_lights_presampling", i32)]

    @classmethod
    def default(cls):
        # KernelOptions.h:116, 218, 231, 242, 252, 335, 304, 355, 270, 279, 289, 366
        return cls(BSDF_NONE, LSS_RIS_BSDF_AND_LIGHT, ESS_ALIAS_TABLE, 1, 0, RESTIR_DI_BIAS_PAIRWISE_MIS_DEFENSIVE, 1,
                   RESTIR_DI_LATER_BOUNCES_RIS_BSDF_AND_LIGHT, 0, 1, 1, 1)


class BSDFFlags(C.Structure):
    _fields_ = [("white_furnace_mode", c_bool), ("white_furnace_mode_turn_off_emissives", c_bool),
                ("clearcoat_compensation_approximation", c_bool), ("ggx_masking_shadowing", i32)]

    @classmethod
    def default(cls):
        return cls(False, True, True, 0)


class Frame(C.Structure):
    _fields_ = [("render_settings", RenderSettings), ("world_settings", WorldSettings),
                ("current_camera", Camera), ("prev_camera", Camera), ("options", KernelOptions),
                ("bsdf_flags", BSDFFlags), ("random_seed", u32), ("res_x", i32), ("res_y", i32),
                ("band_height", i32), ("band_index", i32), ("band_count", i32),
                ("camera_random_seed", u32), ("restir_di_seeds", u32 * 8)]


class Scene(C.Structure):
    _fields_ = [
        ("triangle_indices", C.POINTER(i32)), ("num_triangles", i32),
        ("vertices", C.POINTER(f32)), ("vertex_normals", C.POINTER(f32)),
        ("has_vertex_normals", C.POINTER(C.c_uint8)), ("texcoords", C.POINTER(f32)),
        ("num_vertices", i32), ("material_indices", C.POINTER(i32)),
        ("materials", C.POINTER(Material)), ("num_materials", i32),
        ("emissive_triangle_indices", C.POINTER(i32)), ("num_emissive_triangles", i32),
        ("num_textures", i32), ("texture_data", C.POINTER(C.POINTER(C.c_uint8))),
        ("texture_dims", C.POINTER(i32)),
    ]


class Luts(C.Structure):
    _fields_ = [("ggx_conductor_ess", C.POINTER(f32)), ("glossy_dielectric_ess", C.POINTER(f32)),
                ("ggx_glass_ess", C.POINTER(f32)), ("ggx_glass_inverse_ess", C.POINTER(f32)),
                ("ggx_thin_glass_ess", C.POINTER(f32)), ("sheen_ltc_params", C.POINTER(f32))]


class Stats(C.Structure):
    _fields_ = [("rays_closest", C.c_uint64), ("rays_any", C.c_uint64), ("node_visits", C.c_uint64),
                ("triangle_tests", C.c_uint64), ("trace_launches", u32), ("frames", u32),
                ("trace_ms", C.c_double), ("frame_ms", C.c_double),
                ("stage_rays", C.c_uint64 * 3), ("stage_traversals", C.c_uint64 * 3), ("stage_nodes", C.c_uint64 * 3),
                ("stage_tris", C.c_uint64 * 3), ("stage_ms", C.c_double * 3),
                ("stage_launches", u32 * 3), ("shade_launches", u32), ("camera_ms", C.c_double),
                ("shade_ms", C.c_double), ("resolve_ms", C.c_double), ("accumulate_ms", C.c_double),
                ("compact_ms", C.c_double), ("restir_ms", C.c_double),
                ("stage_node_slots", C.c_uint64 * 3), ("stage_tri_slots", C.c_uint64 * 3),
                ("path_hits", C.c_uint64), ("split_ms", C.c_double), ("miss_ms", C.c_double),
                ("shade_generic_ms", C.c_double), ("shade_generic_vertices", C.c_uint64),
                ("restir_kernel_ms", C.c_double * 5), ("restir_kernel_launches", C.c_uint32 * 5),
                ("restir_eval_ms", C.c_double), ("restir_eval_launches", C.c_uint32), ("restir_eval_items", C.c_uint64),
                ("graph_captures", C.c_uint32), ("graph_replays", C.c_uint32), ("overlapped_batches", C.c_uint32),
                ("halo_exchanges", C.c_uint64), ("halo_agreements", C.c_uint64), ("halo_bytes_sent", C.c_uint64),
                ("halo_bytes_received", C.c_uint64), ("restir_overlapped_batches", C.c_uint32),
                ("trace_ahead_launches", C.c_uint32), ("pipelined_batches", C.c_uint32)]


OK, ERR_INVALID_ARGUMENT, ERR_HIP, ERR_NO_SCENE, ERR_UNSUPPORTED, ERR_OUT_OF_MEMORY = 0, -1, -2, -3, -4, -5
MAX_BATCH = 128
DEFAULT_WAVEFRONT_PATHS = 1 << 25
MAX_WAVEFRONT_PATHS = 1 << 29
BSDF_NONE, BSDF_LAMBERTIAN, BSDF_OREN_NAYAR = 0, 1, 2
(BAKE_GGX_CONDUCTOR, BAKE_GGX_FRESNEL, BAKE_GLOSSY_DIELECTRIC, BAKE_GGX_GLASS, BAKE_GGX_GLASS_INVERSE,
 BAKE_GGX_THIN_GLASS) = range(6)
(LSS_NO_DIRECT_LIGHT_SAMPLING, LSS_UNIFORM_ONE_LIGHT, LSS_BSDF, LSS_MIS_LIGHT_BSDF,
 LSS_RIS_BSDF_AND_LIGHT, LSS_RESTIR_DI) = range(6)
ESS_NO_SAMPLING, ESS_BINARY_SEARCH, ESS_ALIAS_TABLE = range(3)
AMBIENT_NONE, AMBIENT_UNIFORM, AMBIENT_ENVMAP = range(3)
FB_COLOR, FB_ALBEDO, FB_NORMALS = range(3)
AUX_SAMPLE_COUNT, AUX_CONVERGED_SAMPLE_COUNT, AUX_SQUARED_LUMINANCE = range(3)
AUX_RESTIR_OUTPUT, AUX_RESTIR_OTHER, AUX_RESTIR_INITIAL = 3, 4, 5


class Status(C.Structure):
    """MptStatus == StatusBuffersValues (Renderer/StatusBuffersValues.h:9-21)."""
    _fields_ = [("one_ray_active", C.c_bool), ("pixel_converged_count", C.c_uint32)]

# ReSTIR DI across a row partition: the halo-exchange callback (mpt.h MptHaloExchange)
HALO_GBUFFER, HALO_RESERVOIRS, HALO_PREV_GBUFFER = 0, 1, 2
HALO_MAX_BUFFERS = 12


class HaloExchange(C.Structure):
    _fields_ = [("phase", C.c_int32), ("pass_index", C.c_int32), ("res_x", C.c_int32), ("res_y", C.c_int32),
                ("own_y0", C.c_int32), ("own_y1", C.c_int32), ("halo_rows", C.c_int32), ("n_buffers", C.c_int32),
                ("buffers", C.c_void_p * HALO_MAX_BUFFERS), ("bytes_per_pixel", C.c_int64 * HALO_MAX_BUFFERS),
                ("stream", C.c_void_p), ("halo_agreed", C.c_int32)]


HaloExchangeFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(HaloExchange))


class HaloOp(C.Structure):
    """MptHaloOp: one send (recv 0) or receive (recv 1) of buffer rows [row_lo, row_hi) with a peer band."""
    _fields_ = [("peer", C.c_int32), ("recv", C.c_int32), ("buffer", C.c_int32), ("row_lo", C.c_int32),
                ("row_hi", C.c_int32)]

ABI_SIZES = {"Material": 332, "RenderSettings": 304, "WorldSettings": 200, "Camera": 196}


def check_sizes():
    got = {"Material": C.sizeof(Material), "RenderSettings": C.sizeof(RenderSettings),
           "WorldSettings": C.sizeof(WorldSettings), "Camera": C.sizeof(Camera)}
    assert got == ABI_SIZES, got
    return got
