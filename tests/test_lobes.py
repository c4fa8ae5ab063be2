"""Parity matrix of the layered Principled BSDF lobes and of every texture slot.

The shipped glTFs only hold dielectric, metal, glass and emissive materials, so most of
principled_bsdf_eval / _sample (BSDFs/Principled.h:530-699, 863-1193: coat, sheen LTC,
metal F82 tint, thin film, anisotropy, specular tint / colour, second roughness,
thin-walled glass) would otherwise never run.  Each case edits the Cornell box's
materials through mpt_update_materials (GPURenderer::update_materials, GPURenderer.h:228)
and renders GPU against the CPU oracle, bit-exact, for MIS and RIS light sampling.
The textured-panel scene (mpt.synthetic.with_textured_panels) drives every texture slot
of get_intersection_material (Device/includes/Material.h:47-159) and the normal map
(Texture.h:209-222).  CPU: white-furnace pins of the coat and sheen lobes."""
import copy

import numpy as np
import pytest

from mpt import abi, scene, synthetic

W, H, SPP, BOUNCES = 40, 30, 3, 4
WALLS = (1, 3, 4, 5, 6, 7)      # cornell_pbr: diffuse walls and the tall box
METAL, GLASS = 0, 8


def C(*v):
    return abi.Color(*v)


LOBES = {
    "coat": ({WALLS: dict(coat=1.0, coat_roughness=0.15, coat_ior=1.6)}),
    "coat_medium_rough_aniso": ({WALLS: dict(coat=0.7, coat_roughness=0.45, coat_ior=1.45, coat_anisotropy=0.6,
                                             coat_anisotropy_rotation=0.3, coat_medium_absorption=C(0.8, 0.6, 0.4),
                                             coat_medium_thickness=3.0, coat_darkening=0.5, coat_roughening=0.5),
                                 (METAL,): dict(coat=1.0, coat_roughness=0.05)}),
    "sheen": ({WALLS: dict(sheen=1.0, sheen_roughness=0.3, sheen_color=C(0.9, 0.5, 0.2))}),
    "sheen_rough_over_metal": ({WALLS: dict(sheen=0.6, sheen_roughness=0.9), (METAL,): dict(sheen=1.0, sheen_roughness=0.5)}),
    "thin_film": ({WALLS: dict(thin_film=1.0, thin_film_ior=1.6, thin_film_thickness=420.0),
                   (METAL,): dict(thin_film=1.0, thin_film_ior=1.8, thin_film_thickness=300.0, roughness=0.2)}),
    "thin_film_ior_override_kappa": ({WALLS: dict(thin_film=0.8, thin_film_ior=1.4, thin_film_thickness=650.0,
                                                  thin_film_do_ior_override=True, thin_film_base_ior_override=2.0,
                                                  thin_film_kappa_3=1.5, thin_film_hue_shift_degrees=40.0),
                                      (GLASS,): dict(thin_film=1.0, thin_film_thickness=500.0)}),
    "anisotropy": ({WALLS: dict(anisotropy=0.8, anisotropy_rotation=0.25, roughness=0.4, metallic=0.5),
                    (METAL,): dict(anisotropy=0.9, anisotropy_rotation=0.6, roughness=0.35)}),
    "specular_tint_color": ({WALLS: dict(specular=0.7, specular_tint=0.5, specular_color=C(1.0, 0.5, 0.2),
                                         specular_darkening=0.5, roughness=0.25)}),
    "metal_f82": ({WALLS: dict(metallic=1.0, metallic_F82=C(0.9, 0.5, 0.3), metallic_F90=C(1.0, 0.9, 0.8),
                               metallic_F90_falloff_exponent=3.0, roughness=0.3)}),
    "second_roughness": ({WALLS: dict(metallic=1.0, second_roughness_weight=0.5, second_roughness=0.8, roughness=0.1),
                          (METAL,): dict(second_roughness_weight=1.0, second_roughness=0.4)}),
    "thin_walled_glass": ({(GLASS,): dict(thin_walled=True, roughness=0.2),
                           (3,): dict(specular_transmission=1.0, thin_walled=True, roughness=0.05, ior=1.5)}),
    "glass_absorption_rough": ({(GLASS,): dict(roughness=0.3, absorption_color=C(0.6, 0.8, 0.9),
                                               absorption_at_distance=0.5, ior=1.7)}),
    "all_lobes": ({WALLS: dict(coat=0.5, coat_roughness=0.3, sheen=0.5, sheen_roughness=0.4, metallic=0.3,
                               specular_transmission=0.2, thin_film=0.5, thin_film_thickness=380.0, anisotropy=0.3,
                               specular_tint=0.3, specular_color=C(0.7, 0.9, 1.0))}),
}


def lobe_materials(base, case):
    mats = [abi.Material.from_buffer_copy(m) for m in base.materials]
    for idxs, kw in LOBES[case].items():
        for i in idxs:
            for k, v in kw.items():
                setattr(mats[i], k, v)
            mats[i].make_safe()
            mats[i].precompute_properties()
    return mats


def frames(sd, lss, n=SPP, bounces=BOUNCES, world=None, w=W, h=H):
    cam = scene.make_camera(sd.camera_info, w, h)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    return [scene.make_frame(cam, w, h, options=opt, settings=scene.parity_settings(bounces), world=world,
                             sample_number=s, random_seed=seed) for s, seed in scene.cpu_seed_schedule(n)]


def _same(a, b, what):
    assert a.shape == b.shape, what
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    assert not bad.any(), f"{what}: {int(bad.sum())} values differ, first at {np.argwhere(bad)[:3].tolist()}"


def _gpu(sd, luts):
    """A fresh context per case: a sample whose sanity check fails writes nothing, not even
    at sample 0 (FullPathTracer.h:293-294), so a reused context would show the previous
    case's sums where the oracle starts from zero."""
    import mpt
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    return r


def _render(r, frs, batched=False):
    if batched:
        r.render_samples(frs)
    else:
        for f in frs:
            r.render(f)
    r.synchronize_kernel()
    return [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["mis", "ris"])
@pytest.mark.parametrize("case", list(LOBES))
def test_principled_lobe_bit_exact(cornell, luts, case, strategy):
    from oracle import oracle as orc
    mats = lobe_materials(cornell, case)
    lss = abi.LSS_MIS_LIGHT_BSDF if strategy == "mis" else abi.LSS_RIS_BSDF_AND_LIGHT
    frs = frames(cornell, lss)
    r = _gpu(cornell, luts)
    try:
        r.update_materials(mats)
        got = _render(r, frs, batched=strategy == "ris")
    finally:
        r.close()
    sd = copy.copy(cornell)
    sd.materials = mats
    o = orc.Oracle(sd, luts)
    ref = o.render(frs, aov=True)
    o.close()
    for k, what in enumerate(["color", "albedo", "normals"]):
        _same(got[k], ref[k], f"{case} {strategy} {what}")
    assert np.isfinite(got[0]).all() and got[0].mean() > 0


@pytest.fixture(scope="module")
def panels(cornell):
    return synthetic.with_textured_panels(cornell)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["mis", "ris", "bsdf", "uniform", "restir", "ris_envmap"])
def test_texture_slots_bit_exact(panels, luts, strategy):
    """Every texture slot (base colour, normal map, roughness-metallic, emission with
    emissive_texture_used, specular / tint / colour, metallic, roughness, coat, coat
    roughness, sheen, sheen roughness / colour, anisotropy + rotation, Oren-Nayar sigma) and
    the smooth-normal interpolation under a normal map, GPU vs oracle."""
    import mpt
    from oracle import oracle as orc
    lss = {"mis": abi.LSS_MIS_LIGHT_BSDF, "ris": abi.LSS_RIS_BSDF_AND_LIGHT, "bsdf": abi.LSS_BSDF,
           "uniform": abi.LSS_UNIFORM_ONE_LIGHT, "restir": abi.LSS_RESTIR_DI,
           "ris_envmap": abi.LSS_RIS_BSDF_AND_LIGHT}[strategy]
    env = mpt.build_envmap(scene.procedural_sky(128, 64, seed=7)) if strategy == "ris_envmap" else None
    world = scene.envmap_world(0.7) if env is not None else None
    if strategy == "restir":
        cam = scene.make_camera(panels.camera_info, W, H)
        opt = abi.KernelOptions.default()
        opt.direct_light_sampling = lss
        frs = [scene.make_frame(cam, W, H, options=opt, settings=scene.parity_settings(BOUNCES),
                                sample_number=d["sample_number"], random_seed=d["random_seed"],
                                camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"])
               for d in scene.gpu_seed_schedule(SPP, 2)]
    else:
        frs = frames(panels, lss, world=world)
    r = mpt.GPURenderer(0)
    r.set_scene(panels)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    got = _render(r, frs, batched=strategy in ("ris", "ris_envmap"))
    r.close()
    o = orc.Oracle(panels, luts, envmap=env)
    ref = o.render(frs, aov=True)
    o.close()
    for k, what in enumerate(["color", "albedo", "normals"]):
        _same(got[k], ref[k], f"panels {strategy} {what}")
    assert np.isfinite(got[0]).all()


# ---- CPU: white furnace of the coat and sheen layers (the reference's own energy check,
# BSDFsData.h:26-27).  The sheen layer is energy-conserving by construction: the LTC lobe's
# albedo is stored in the LUT (SheenLTC.h:24-150) and the base is attenuated by exactly the
# sheen reflectance (Principled.h:632-654), so a white sheen over a white base integrates to
# 1 -- a tight pin of the sheen restatement.  The coat layering is an approximation in the
# reference itself: the base is attenuated by (1 - F(N.L)) (1 - F(N.V)) at the shading
# normal, not per microfacet (Principled.h:560-590), which loses energy at grazing angles
# and gains a few percent at normal incidence over a perfect mirror; its band is wider.

def _mat(**kw):
    m = abi.Material.default()
    for k, v in kw.items():
        setattr(m, k, v)
    m.make_safe()
    m.precompute_properties()
    return m


@pytest.mark.parametrize("layer,kw,lo,hi", [
    ("sheen_over_metal", dict(metallic=1.0, base_color=C(1.0), sheen=1.0, sheen_color=C(1.0)), 0.985, 1.02),
    ("sheen_over_glossy", dict(base_color=C(1.0), specular=1.0, sheen=1.0, sheen_color=C(1.0)), 0.985, 1.02),
    ("coat_over_glossy", dict(base_color=C(1.0), specular=1.0, coat=1.0, coat_medium_absorption=C(1.0)), 0.98, 1.02),
    ("coat_over_metal", dict(metallic=1.0, base_color=C(1.0), coat=1.0, coat_medium_absorption=C(1.0)), 0.88, 1.06),
])
@pytest.mark.parametrize("roughness", [0.2, 0.6])
def test_white_furnace_coat_and_sheen(oracle_lib, luts, layer, kw, lo, hi, roughness):
    L = scene.luts_to_abi(luts)
    extra = dict(coat_roughness=roughness) if "coat" in layer else dict(sheen_roughness=roughness)
    for cos_o in (0.3, 0.7, 0.95):
        e = oracle_lib.directional_albedo(_mat(roughness=roughness, **kw, **extra), L, cos_o, 60000, seed=5)
        assert lo < float(e[0]) < hi, (layer, roughness, cos_o, e)
        assert abs(float(e[0]) - float(e[2])) < 1e-6      # colourless layers stay grey
