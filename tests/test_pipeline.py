"""The bounce pipeline (MPT_PIPELINE, the library's default for single-stream wavefronts): a
bounce's NEE traversals and k_resolve run on their own stream, over the plane set of the bounce's
parity (NEE records, staged queries, shaded lists, col additions), beside the next bounce's split
and shading; k_miss of the next bounce waits for them (frame_bounces, mpt_kernels.hip).

Bar: bit-exact against the in-line wavefront and the CPU oracle -- odd and even bounce counts,
dielectric / dispersive paths, envmap, adaptive sampling, with and without trace-ahead, the bench
workload on a band -- and the pipelined wavefronts are counted (MptStats::pipelined_batches).
Overlapped halves are switched off (MPT_OVERLAP=0): small wavefronts would run as halves, which
keep their bounces in line.
"""
import pytest

import mpt
from mpt import abi, scene

from test_gpu_parity import STRATEGIES, frames, gpu_render, gpu_render_batched, oracle_for
from test_shade_classes import _assert_modes_equal

pytestmark = pytest.mark.gpu


def _render(monkeypatch, sd, luts, frs, batch, env=None, modes=((0, 1), (1, 1), (1, 0))):
    monkeypatch.setenv("MPT_OVERLAP", "0")
    out = {}
    for pipe, ahead in modes:
        monkeypatch.setenv("MPT_PIPELINE", str(pipe))
        monkeypatch.setenv("MPT_TRACE_AHEAD", str(ahead))
        r = mpt.GPURenderer(0)
        try:
            r.set_scene(sd)
            r.set_luts(luts)
            if env is not None:
                r.set_envmap(env)
            out[(pipe, ahead)] = gpu_render_batched(r, frs, batch)
            st = r.stats()
            assert (st.pipelined_batches > 0) == bool(pipe), (pipe, ahead, st.pipelined_batches)
        finally:
            r.close()
    return out


@pytest.mark.parametrize("strategy,bounces,batch", [("mis", 3, 2), ("ris", 4, 5), ("ris", 1, 3)])
def test_pipeline_cornell(monkeypatch, luts, strategy, bounces, batch):
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 40, 24, 6, lss=STRATEGIES[strategy], bounces=bounces)
    out = _render(monkeypatch, sd, luts, frs, batch)
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"pipeline cornell {strategy} {bounces}")


@pytest.mark.parametrize("name,bounces", [("nested-dielectrics-complex", 8), ("multi-dispersion", 7)])
def test_pipeline_dielectrics(monkeypatch, luts, name, bounces):
    sd = scene.load_scene(name)
    frs = frames(sd, 32, 24, 4, lss=abi.LSS_RIS_BSDF_AND_LIGHT, bounces=bounces)
    out = _render(monkeypatch, sd, luts, frs, 4)
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"pipeline {name}")


def test_pipeline_envmap_adaptive(monkeypatch, luts):
    sd = scene.load_scene("cornell_pbr")
    env = mpt.build_envmap(scene.procedural_sky(128, 64, seed=7))
    frs = frames(sd, 48, 30, 8, lss=STRATEGIES["mis"], world=scene.envmap_world(1.0))
    for f in frs:
        f.render_settings.enable_adaptive_sampling = True
        f.render_settings.adaptive_sampling_min_samples = 2
        f.render_settings.adaptive_sampling_noise_threshold = 0.9
    out = _render(monkeypatch, sd, luts, frs, 4, env=env)
    _assert_modes_equal(out, oracle_for(sd, luts, env).render(frs, aov=True), "pipeline envmap adaptive")


def test_pipeline_city_band(monkeypatch, luts):
    """The bench workload (alpha-tested leaf cards, textured materials, envmap) on a band."""
    from mpt import synthetic
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 4, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=(8, 5, 64))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    out = _render(monkeypatch, city, luts, frs, 4, env=env, modes=((0, 1), (1, 1)))
    _assert_modes_equal(out, oracle_for(city, luts, env).render(frs, aov=True), "pipeline city band")


def test_set_pipeline_switches_between_launches(monkeypatch, luts):
    """mpt_set_pipeline (the bench's solo timing): in line after 0, pipelined after 1, the same
    image either way; other modes are refused."""
    monkeypatch.setenv("MPT_OVERLAP", "0")
    monkeypatch.delenv("MPT_PIPELINE", raising=False)
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 40, 24, 4, lss=STRATEGIES["ris"])
    r = mpt.GPURenderer(0)
    try:
        r.set_scene(sd)
        r.set_luts(luts)
        with pytest.raises(Exception):
            r.set_pipeline(2)
        out = {}
        for mode in (0, 1):
            r.set_pipeline(mode)
            r.enable_stats(timing=False, instrumented=False)   # (resets the counters)
            out[mode] = gpu_render_batched(r, frs, 4)
            assert (r.stats().pipelined_batches > 0) == bool(mode), mode
    finally:
        r.close()
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), "set_pipeline")


@pytest.mark.parametrize("case", ["mis", "ris_adaptive", "low_res", "envmap_odd_rows"])
def test_pipelined_pixel_parts(monkeypatch, luts, case):
    """One-sample frames as 2 row parts, each with the bounce pipeline (MPT_PIX_PIPE: part k's NEE
    work on its own stream, over its rows of the alternate planes and counter set k + 2):
    bit-exact against one stream and the oracle."""
    sd = scene.load_scene("cornell_pbr")
    lss = STRATEGIES["ris"] if case == "ris_adaptive" else STRATEGIES["mis"]
    env = mpt.build_envmap(scene.procedural_sky(128, 64, seed=7)) if case.startswith("envmap") else None
    w, h = (256, 257) if case == "envmap_odd_rows" else (320, 206)
    frs = frames(sd, w, h, 4, lss=lss, world=scene.envmap_world(1.0) if env is not None else None)
    if case == "ris_adaptive":
        for f in frs:
            f.render_settings.enable_adaptive_sampling = True
            f.render_settings.adaptive_sampling_min_samples = 1
            f.render_settings.adaptive_sampling_noise_threshold = 0.9
    if case == "low_res":
        frs[2].render_settings.wants_render_low_resolution = True
        frs[2].render_settings.render_low_resolution_scaling = 2
    out = {}
    for parts, pipe in ((0, 0), (2, 1)):
        monkeypatch.setenv("MPT_PIX_PARTS", str(parts))
        monkeypatch.setenv("MPT_PIX_PIPE", str(pipe))
        monkeypatch.setenv("MPT_PIPELINE", str(pipe))
        r = mpt.GPURenderer(0)
        try:
            r.set_scene(sd)
            r.set_luts(luts)
            if env is not None:
                r.set_envmap(env)
            r.enable_stats(timing=False, instrumented=False)
            out[(parts, pipe)] = gpu_render(r, frs)
            assert (r.stats().pipelined_batches > 0) == bool(pipe), (parts, pipe)
        finally:
            r.close()
    _assert_modes_equal(out, oracle_for(sd, luts, env).render(frs, aov=True), f"pipelined pixel parts {case}")


@pytest.mark.parametrize("strategy,ovr", [("none", abi.BSDF_NONE), ("uniform", abi.BSDF_NONE), ("bsdf", abi.BSDF_NONE),
                                          ("mis", abi.BSDF_LAMBERTIAN), ("ris", abi.BSDF_OREN_NAYAR)])
def test_pipeline_strategies_and_overrides(monkeypatch, luts, strategy, ovr):
    """Every light-sampling strategy (no direct light sampling: the emission handed to the resolve
    with nothing else to add) and the Lambert / Oren-Nayar override kernels, pipelined vs in line."""
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 40, 24, 4, ovr=ovr, lss=STRATEGIES[strategy], bounces=4)
    out = _render(monkeypatch, sd, luts, frs, 2, modes=((0, 1), (1, 1)))
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"pipeline {strategy} override {ovr}")
