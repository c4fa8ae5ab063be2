"""Overlapped batches (MPT_OVERLAP=1): the two halves of a sample batch run on two streams
over their own slots, counters and traversal spill areas, the second half one pipeline stage
behind the first and accumulating after it.

Bar: bit-exact against the single-stream batch and the CPU oracle (odd and even batch
sizes, partitioned, the bench workload with alpha testing and textured materials).
"""
import pytest

from mpt import abi, scene

from test_gpu_parity import STRATEGIES, frames, oracle_for
from test_shade_classes import _assert_modes_equal, _render_modes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch,band,strategy", [(2, (1, 0, 1), "mis"), (5, (4, 1, 3), "ris"), (8, (1, 0, 1), "ris")])
def test_overlap_cornell(monkeypatch, luts, batch, band, strategy):
    sd = scene.load_scene("cornell_pbr")
    frs = frames(sd, 40, 24, 8, lss=STRATEGIES[strategy], band=band)
    out = _render_modes(monkeypatch, sd, luts, frs, batch=batch, var="MPT_OVERLAP", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(sd, luts).render(frs, aov=True), f"cornell batch {batch}")


def test_overlap_city_band(monkeypatch, luts):
    import mpt
    from mpt import synthetic
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 4, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=(8, 9, 64))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    out = _render_modes(monkeypatch, city, luts, frs, env=env, batch=4, var="MPT_OVERLAP", modes=(0, 1))
    _assert_modes_equal(out, oracle_for(city, luts, env).render(frs, aov=True), "city band overlapped")


@pytest.mark.parametrize("case", ["mis", "ris_adaptive", "low_res", "envmap_odd_rows"])
def test_pixel_parts_one_sample_frames(monkeypatch, luts, case):
    """One-sample frames of a whole-frame context as 2 / 3 / 4 row parts on their own streams
    (MPT_PIX_PARTS, frames of at least 65536 pixels; part k renders its rows as band k of the
    parts): bit-exact against one stream and the oracle -- an odd row count, adaptive sampling
    past its minimum, a low-resolution frame (all of its pixels in the first part)."""
    import mpt
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
    monkeypatch.setenv("MPT_PIX_PIPE", "0")   # (the parts in line; pipelined parts: tests/test_pipeline.py)
    out = _render_modes(monkeypatch, sd, luts, frs, env=env, var="MPT_PIX_PARTS", modes=(0, 2, 3, 4))
    _assert_modes_equal(out, oracle_for(sd, luts, env).render(frs, aov=True), f"pixel parts {case}")
