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
