"""Light-hit queries through the light BVH (build_light_bvh, k_trace TM_NEE_LIGHT +
TM_NEE_LIGHT_OCC): the BSDF rays of MIS / RIS / BSDF light sampling find the closest hit
among the triangles that can emit, then an any-hit query over the whole scene (with the
closest-hit tie rule) confirms it.

Bar: bit-exact against the single closest-hit traversal (MPT_LIGHT_BVH=0) and the CPU
oracle, including material edits that change the set of lights and a scene whose only
light is the envmap (empty light BVH).
"""
import numpy as np
import pytest

import mpt
from mpt import abi, scene

from test_gpu_parity import STRATEGIES, frames, oracle_for
from test_shade_classes import _assert_modes_equal, _render_modes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("strategy", ["mis", "ris", "bsdf"])
def test_light_bvh_cornell(monkeypatch, luts, strategy):
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 48, 32, 3, lss=STRATEGIES[strategy])
    out = _render_modes(monkeypatch, sd, luts, frs, var="MPT_LIGHT_BVH", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"cornell {strategy}")


def test_light_bvh_city_band(monkeypatch, luts):
    """The bench workload: ~1.2 k lamp triangles among 2.86 M, alpha-tested leaf cards."""
    from mpt import synthetic
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 2, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=(8, 11, 64))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    out = _render_modes(monkeypatch, city, luts, frs, env=env, batch=2, var="MPT_LIGHT_BVH", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(city, luts, env).render(frs, aov=True), "city band")


def test_light_bvh_material_edit_and_no_lights(monkeypatch, luts):
    """Material edits rebuild the light set: every emitter switched off (empty light BVH,
    the BSDF rays contribute nothing), then a wall made emissive as well.  BSDF light
    sampling: every light term comes from a light-hit query.  The NEE triangle list stays
    the uploaded one (update_materials does not rebuild it, GPURenderer.h:228), so the
    oracle's scene keeps it too."""
    import copy
    sd0 = scene.load_scene("cornell_pbr")
    frs = frames(sd0, 40, 24, 2, lss=abi.LSS_BSDF)
    variants = []
    dark = [abi.Material.from_buffer_copy(m) for m in sd0.materials]
    for m in dark:
        m.emission_strength = 0.0
    variants.append(dark)
    lit = [abi.Material.from_buffer_copy(m) for m in sd0.materials]
    wall = int(sd0.material_indices[0])
    lit[wall].emission = abi.Color(0.3, 0.2, 0.1)
    lit[wall].emission_strength = 2.0
    variants.append(lit)
    for mats in variants:
        sd = copy.copy(sd0)
        sd.materials = mats
        ref = oracle_for(sd, luts).render(frs, aov=True)
        out = {}
        for mode in (0, 1):
            monkeypatch.setenv("MPT_LIGHT_BVH", str(mode))
            r = mpt.GPURenderer(0)
            try:
                r.set_scene(sd0)          # the original lights ...
                r.set_luts(luts)
                r.update_materials(mats)  # ... edited: the light set is rebuilt
                for f in frs:
                    r.render(f)
                r.synchronize_kernel()
                out[mode] = tuple(r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS))
            finally:
                r.close()
        _assert_modes_equal(out, ref, "material edit")


def test_light_bvh_too_deep_fallback(monkeypatch, luts):
    """A light BVH too deep for the traversal stack (forced by the MPT_LIGHT_BVH_MAX_STACK
    test hook) is dropped: light-hit queries take the exact whole-scene closest-hit path, so
    the render is bit-exact against MPT_LIGHT_BVH=0 and the oracle, and a material edit in that
    state still succeeds (and still falls back)."""
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 40, 24, 2, lss=abi.LSS_MIS_LIGHT_BSDF)
    monkeypatch.setenv("MPT_LIGHT_BVH_MAX_STACK", "2")
    out = _render_modes(monkeypatch, sd, luts, frs, var="MPT_LIGHT_BVH", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), "too-deep light BVH")
    mats = [abi.Material.from_buffer_copy(m) for m in sd.materials]
    wall = int(sd.material_indices[0])
    mats[wall].emission = abi.Color(0.3, 0.2, 0.1)
    mats[wall].emission_strength = 2.0
    import copy
    sd2 = copy.copy(sd)
    sd2.materials = mats
    r = mpt.GPURenderer(0)
    try:
        r.set_scene(sd)
        r.set_luts(luts)
        r.update_materials(mats)
        for f in frs:
            r.render(f)
        r.synchronize_kernel()
        img = r.framebuffer(abi.FB_COLOR)
    finally:
        r.close()
    assert np.array_equal(img, oracle_for(sd2, luts).render(frs)), "material edit with a too-deep light BVH"
