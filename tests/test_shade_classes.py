"""Material-class shading (k_split sorts the hit vertices into the plain-dielectric list and
the generic list, k_shade<OVR, true> shades the plain list with the coat / sheen / metal /
glass / thin-film code compiled out, dev_bsdf.h FULL = false).

Bar: bit-exact.  The same frames rendered by contexts with the class split off
(MPT_SHADE_CLASSES=0: every vertex through the generic kernel), on (1, the default) and on
with every plain vertex deferred to the generic kernel (2: exercises the deferral path --
the tombstoned entries of the plain list and the deferred entries of the generic list in
k_compact / k_resolve) give identical sums and AOVs, and equal the CPU oracle.
"""
import numpy as np
import pytest

import mpt
from mpt import abi, scene

from test_gpu_parity import STRATEGIES, assert_same, frames, gpu_render, gpu_render_batched, oracle_for

pytestmark = pytest.mark.gpu


def _render_modes(monkeypatch, sd, luts, frs, env=None, batch=0, var="MPT_SHADE_CLASSES", modes=(0, 1, 2)):
    out = {}
    for mode in modes:
        monkeypatch.setenv(var, str(mode))
        r = mpt.GPURenderer(0)
        try:
            r.set_scene(sd)
            r.set_luts(luts)
            if env is not None:
                r.set_envmap(env)
            out[mode] = gpu_render_batched(r, frs, batch) if batch else gpu_render(r, frs)
        finally:
            r.close()
    return out


def _assert_modes_equal(out, ref, what):
    for mode in out:
        for k, aov in enumerate(["color", "albedo", "normals"]):
            assert_same(out[mode][k], ref[k], f"{what}: classes={mode} {aov} vs oracle")


@pytest.mark.parametrize("strategy", ["mis", "ris"])
def test_classes_cornell(monkeypatch, luts, strategy):
    """Cornell PBR: plain walls beside the metal / glass objects of the generic class."""
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 48, 32, 3, lss=STRATEGIES[strategy])
    out = _render_modes(monkeypatch, sd, luts, frs)
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"cornell {strategy}")


def test_classes_dielectrics(monkeypatch, luts):
    """Nested dielectrics (generic class: transmission) at 8 bounces."""
    sd = scene.load_scene("nested-dielectrics-complex")
    frs = frames(sd, 32, 24, 2, lss=abi.LSS_RIS_BSDF_AND_LIGHT, bounces=8)
    out = _render_modes(monkeypatch, sd, luts, frs)
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), "nested dielectrics")


def test_classes_city_band_batched(monkeypatch, luts):
    """The bench workload (plain facades, metal lamp posts, textured alpha-tested leaf
    cards, envmap) on a band, as one batched wavefront."""
    from mpt import synthetic
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 2, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=(8, 3, 64))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    out = _render_modes(monkeypatch, city, luts, frs, env=env, batch=2)
    _assert_modes_equal(out, oracle_for(city, luts, env).render(frs, aov=True), "city band")
    assert np.isfinite(out[1][0]).all() and out[1][0].mean() > 0


@pytest.mark.parametrize("name,strategy,bounces", [("multi-dispersion", "ris", 16), ("nested-dielectrics-complex", "mis", 8),
                                                   ("cornell_pbr", "ris", 4)])
def test_glass_class(monkeypatch, luts, name, strategy, bounces):
    """The glass class (MT_GLASS: transmission without coat / sheen / metal / thin film, shaded
    by k_shade<GLASS> with dev_bsdf.h BC_GLASS from the top of the generic list) against the
    generic kernel (MPT_SHADE_GLASS=0) and the oracle, incl. dispersion and nested dielectrics."""
    sd = scene.load_scene(name)
    frs = frames(sd, 40, 30, 2, lss=STRATEGIES[strategy], bounces=bounces)
    out = _render_modes(monkeypatch, sd, luts, frs, var="MPT_SHADE_GLASS", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"{name} glass class")


STAGE_STRATEGIES = ["mis", "ris", "uniform", "bsdf", "none"]


@pytest.mark.parametrize("strategy", STAGE_STRATEGIES)
def test_plain_stages_cornell_envmap(monkeypatch, luts, strategy):
    """The plain class shaded in stages (MPT_SHADE_SPLIT: 1 light / envmap / continuation, 2
    light / envmap + continuation, 3 light + envmap / continuation; k_shade's ST): each stage
    continues the vertex's RNG stream and the later ones read the first one's surface record,
    so every split equals the one-kernel shading (0) and the oracle -- under an envmap (the
    envmap stage), with every light strategy, incl. no direct light sampling (the first stage
    clears the NEE flags for all)."""
    sd = scene.load_scene("cornell_pbr")
    env = mpt.build_envmap(scene.procedural_sky(64, 32, seed=3))
    frs = frames(sd, 40, 28, 2, lss=STRATEGIES[strategy], world=scene.envmap_world(0.7))
    out = _render_modes(monkeypatch, sd, luts, frs, env=env, var="MPT_SHADE_SPLIT", modes=(0, 1, 2, 3))
    _assert_modes_equal(out, oracle_for(sd, luts, env).render(frs, aov=True), f"cornell stages {strategy}")


def test_plain_stages_city_band_batched(monkeypatch, luts):
    """The bench workload on a band (textured alpha-tested leaf cards: per-slot resolved
    materials in the surface record) under each split, as one batched wavefront."""
    from mpt import synthetic
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 2, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=(8, 3, 64))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    out = _render_modes(monkeypatch, city, luts, frs, env=env, batch=2, var="MPT_SHADE_SPLIT", modes=(0, 1, 3))
    _assert_modes_equal(out, oracle_for(city, luts, env).render(frs, aov=True), "city band stages")


@pytest.mark.parametrize("strategy", ["mis", "ris"])
def test_texture_decided_plain_class(monkeypatch, luts, strategy):
    """MT_TEXMETAL (k_resolve_materials): a material outside the plain class only through its
    metallic / roughness-metallic texture goes to the plain list (k_split), and k_shade<PLAIN>
    defers the vertices whose resolved texel is metallic.  The textured-panel scene's panel 0
    (roughness-metallic texture, metallic 0 / 0.5 / 1 texels) is such a material: with the
    routing on (MPT_SHADE_TEXMETAL=1, the default) fewer vertices reach the generic kernel,
    and the frames equal the routing off and the oracle, bit for bit."""
    from mpt import synthetic
    sd = synthetic.with_textured_panels(scene.load_scene("cornell_pbr"))
    env = mpt.build_envmap(scene.procedural_sky(64, 32, seed=5))
    frs = frames(sd, 48, 32, 2, lss=STRATEGIES[strategy], world=scene.envmap_world(0.6))
    out, generic = {}, {}
    for mode in (0, 1):
        monkeypatch.setenv("MPT_SHADE_TEXMETAL", str(mode))
        r = mpt.GPURenderer(0)
        try:
            r.set_scene(sd)
            r.set_luts(luts)
            r.set_envmap(env)
            out[mode] = gpu_render(r, frs)
            generic[mode] = r.stats().shade_generic_vertices
        finally:
            r.close()
    _assert_modes_equal(out, oracle_for(sd, luts, env).render(frs, aov=True), f"panels texmetal {strategy}")
    assert 0 < generic[1] < generic[0], generic
