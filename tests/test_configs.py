"""The BASELINE.json configurations on their own workloads, GPU against the CPU oracle.

* C1 -- Cornell box glTF, 256x256, 1 spp, Lambert override (KernelOptions.h:116
  BSDFOverride = BSDF_LAMBERTIAN), reference-default RIS light sampling, 3 bounces,
  uniform ambient 0.5, the CPU renderer's seed schedule (CPURenderer.cpp:264-296,
  m_rng seeded 42).  The whole frame, bit-exact, and pinned by a committed oracle
  fixture (tests/golden/c1_cornell_256_lambert_1spp.npz, made by make_golden.py).
* C4 -- the Bistro stand-in (procedural city, 2.86 M triangles, alpha-tested leaf cards)
  under the procedural HDR sky with ReSTIR DI (ReSTIRDIRenderPass.cpp:233-264), fused
  spatiotemporal (the default) and the unfused temporal + spatial chain, alpha testing
  on, the GPU front-end's seed schedule, on the whole 1920x1080 frame: every frame
  reuses the previous one (temporal) and neighbours up to 16 px away (spatial).
* C5 -- the glass-dispersion and nested-dielectrics scenes at 16 bounces on a crop of the
  3840x2160 camera (interleaved 8-row bands), through mpt_render_frames (the bench's
  batched wavefronts).
Bar: bit-exact."""
import os

import numpy as np
import pytest

from mpt import abi, scene

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
C1_FIXTURE = os.path.join(GOLDEN, "c1_cornell_256_lambert_1spp.npz")


def c1_frames(sd, spp=1):
    """C1: 256x256 (aspect override 1), Lambert override, RIS, 3 bounces,
    no envmap (uniform ambient), alpha testing and adaptive sampling off."""
    cam = scene.make_camera(sd.camera_info, 256, 256)
    opt = abi.KernelOptions.default()
    opt.bsdf_override = abi.BSDF_LAMBERTIAN
    opt.direct_light_sampling = abi.LSS_RIS_BSDF_AND_LIGHT
    return [scene.make_frame(cam, 256, 256, options=opt, settings=scene.parity_settings(3), sample_number=s,
                             random_seed=seed) for s, seed in scene.cpu_seed_schedule(spp)]


def test_c1_oracle_matches_fixture(cornell, luts, oracle_lib):
    """The oracle's C1 frame equals the committed fixture (regression pin of the restated
    algorithm on the whole C1 workload)."""
    o = oracle_lib.Oracle(cornell, luts)
    img, alb, nrm = o.render(c1_frames(cornell), aov=True)
    o.close()
    g = np.load(C1_FIXTURE)
    assert img.shape == (256, 256, 3)
    assert np.array_equal(img, g["color"])
    assert np.array_equal(alb, g["albedo"])
    assert np.array_equal(nrm, g["normals"])
    assert img.mean() > 0.05


def _gpu(sd, luts, env=None):
    import mpt
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    return r


def _same(a, b, what):
    assert a.shape == b.shape, what
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    assert not bad.any(), f"{what}: {int(bad.sum())} values differ, first at {np.argwhere(bad)[:3].tolist()}"


@pytest.mark.gpu
def test_c1_gpu_bit_exact_full_frame(cornell, luts):
    from oracle import oracle as orc
    frs = c1_frames(cornell)
    r = _gpu(cornell, luts)
    r.render_samples(frs)
    r.synchronize_kernel()
    got = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
    r.close()
    o = orc.Oracle(cornell, luts)
    ref = o.render(frs, aov=True)
    o.close()
    g = np.load(C1_FIXTURE)
    for k, name in enumerate(["color", "albedo", "normals"]):
        _same(got[k], ref[k], f"C1 {name} vs oracle")
        _same(got[k], g[name], f"C1 {name} vs fixture")


# ---- C4: the city stand-in with ReSTIR DI on the whole 1920x1080 frame -------------------------

def c4_frames(city, n, fused=True, passes=2):
    cam = scene.make_camera(city.camera_info, 1920, 1080)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RESTIR_DI
    out = []
    for d in scene.gpu_seed_schedule(n, passes, fused=fused):
        st = scene.parity_settings(3)
        st.do_alpha_testing = True
        st.restir_di_settings.number_of_passes = passes
        st.restir_di_settings.do_fused_spatiotemporal = fused
        out.append(scene.make_frame(cam, 1920, 1080, options=opt, settings=st, world=scene.envmap_world(1.0),
                                    sample_number=d["sample_number"], random_seed=d["random_seed"],
                                    camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"]))
    return out


@pytest.fixture(scope="module")
def city():
    from mpt import synthetic
    return synthetic.procedural_city(1234)


@pytest.fixture(scope="module")
def city_oracle(city, luts):
    import mpt
    from oracle import oracle as orc
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    o = orc.Oracle(city, luts, envmap=env)
    yield o, env
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False], ids=["fused", "unfused"])
def test_c4_city_restir_full_frame_bit_exact(city, luts, city_oracle, fused):
    o, env = city_oracle
    frs = c4_frames(city, 3, fused=fused, passes=2 if fused else 1)
    r = _gpu(city, luts, env)
    r.render_samples(frs)            # the bench's entry point (batched: per-sample bounce 0, shared later bounces)
    r.synchronize_kernel()
    got = r.framebuffer(abi.FB_COLOR)
    r.close()
    ref = o.render(frs)
    _same(got, ref, f"C4 {'fused' if fused else 'unfused'} colour")
    assert np.isfinite(got).all() and got.mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("nb", [2, 4])
def test_c4_city_partitioned_batched_bit_exact(city, luts, city_oracle, nb):
    """C4 tile-parallel: the 1920x1080 city frame split into nb contiguous bands
    (contexts on cuda:0, one host thread each, the in-process halo exchange), each context's
    samples BATCHED through mpt_render_frames (per-sample reuse passes with their halo exchange
    inside the batch, shared later bounces) -- the same sums as the single-context batched render,
    which test_c4_city_restir_full_frame_bit_exact pins to the oracle."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_restir import render_partitioned_local
    _, env = city_oracle
    n = 4

    def make(band):
        frs = c4_frames(city, n)
        for f in frs:
            f.band_height, f.band_index, f.band_count = band
        return frs

    r = _gpu(city, luts, env)
    r.render_samples(c4_frames(city, n))
    r.synchronize_kernel()
    ref = r.framebuffer(abi.FB_COLOR)
    r.close()
    st = []
    got = render_partitioned_local(city, luts, make, 1920, 1080, nb, env=env, batch=n, stats=st)
    _same(got, ref, f"C4 city over {nb} bands, batched")
    # one wavefront per batch for bounces 0..3 (the envmap defers bounce 0): 4 shading launches
    assert all(0 < x.shade_launches <= 4 for x in st), [x.shade_launches for x in st]


# ---- C5: glass dispersion + nested dielectrics at 16 bounces, 4K camera crop ---------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["multi-dispersion", "nested-dielectrics-complex"])
@pytest.mark.parametrize("strategy", ["ris", "mis"])
def test_c5_16_bounces_4k_crop_bit_exact(luts, name, strategy):
    from oracle import oracle as orc
    sd = scene.load_scene(name)
    W, H = 3840, 2160
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RIS_BSDF_AND_LIGHT if strategy == "ris" else abi.LSS_MIS_LIGHT_BSDF
    band = (8, 17, 48)      # 5-6 bands of 8 rows spread over the frame: 45 x 3840 pixels
    frs = [scene.make_frame(cam, W, H, options=opt, settings=scene.parity_settings(16), sample_number=s,
                            random_seed=seed, band=band) for s, seed in scene.cpu_seed_schedule(2)]
    r = _gpu(sd, luts)
    r.render_samples(frs, max_batch=2)
    r.synchronize_kernel()
    got = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
    r.close()
    o = orc.Oracle(sd, luts)
    ref = o.render(frs, aov=True)
    o.close()
    for k, what in enumerate(["color", "albedo", "normals"]):
        _same(got[k], ref[k], f"C5 {name} {strategy} {what}")
    assert got[0].mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False], ids=["fused", "unfused"])
def test_c4_restir_staged_equals_monolithic(city, luts, city_oracle, fused, monkeypatch):
    """The staged spatial pass (gather, traced ray list, combine, staged visibility reuse;
    restir_di.h) against the monolithic kernel (MPT_RESTIR_STAGED=0) on the C4 city frame with
    alpha testing: the same sums and the same ray counts, bit for bit."""
    _, env = city_oracle
    frs = c4_frames(city, 3, fused=fused, passes=2 if fused else 1)
    out = {}
    for mode in ("monolithic", "staged"):
        monkeypatch.setenv("MPT_RESTIR_STAGED", "0" if mode == "monolithic" else "1")
        r = _gpu(city, luts, env)
        r.render_samples(frs)
        r.synchronize_kernel()
        out[mode] = r.framebuffer(abi.FB_COLOR)
        st = r.stats()
        out[mode + "_rays"] = (st.rays_any, st.rays_closest)
        r.close()
    _same(out["staged"], out["monolithic"], "C4 staged vs monolithic")
    assert out["staged_rays"] == out["monolithic_rays"], (out["staged_rays"], out["monolithic_rays"])


@pytest.mark.gpu
def test_c4_restir_batched_equals_unbatched(city, luts, city_oracle, monkeypatch):
    """Batched ReSTIR DI samples (launch_frames_restir) against one wavefront per sample
    (MPT_RESTIR_BATCH=0) on the C4 city frame: the same sums and the same ray counts."""
    _, env = city_oracle
    frs = c4_frames(city, 4)
    out = {}
    for mode in ("unbatched", "batched"):
        monkeypatch.setenv("MPT_RESTIR_BATCH", "0" if mode == "unbatched" else "1")
        r = _gpu(city, luts, env)
        r.render_samples(frs)
        r.synchronize_kernel()
        out[mode] = r.framebuffer(abi.FB_COLOR)
        st = r.stats()
        out[mode + "_rays"] = (st.rays_any, st.rays_closest)
        r.close()
    _same(out["batched"], out["unbatched"], "C4 batched vs unbatched")
    assert out["batched_rays"] == out["unbatched_rays"], (out["batched_rays"], out["unbatched_rays"])


@pytest.mark.gpu
def test_c4_restir_overlapped_batches_equal_sequential(city, luts, city_oracle, monkeypatch):
    """Overlapped ReSTIR DI batches (a batch's later-bounce wavefront on a second stream beside the
    next batch's per-sample chain, the two batches on the two halves of the path state) against
    MPT_RESTIR_OVERLAP=0, on the C4 city frame with three batches per call: the same sums and ray
    counts."""
    _, env = city_oracle
    frs = c4_frames(city, 6)
    out = {}
    for mode in ("sequential", "overlapped"):
        monkeypatch.setenv("MPT_RESTIR_OVERLAP", "0" if mode == "sequential" else "1")
        r = _gpu(city, luts, env)
        r.render_samples(frs, max_batch=2)
        r.synchronize_kernel()
        out[mode] = r.framebuffer(abi.FB_COLOR)
        st = r.stats()
        out[mode + "_rays"] = (st.rays_any, st.rays_closest)
        r.close()
    _same(out["overlapped"], out["sequential"], "C4 overlapped vs sequential batches")
    assert out["overlapped_rays"] == out["sequential_rays"]


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False], ids=["fused", "unfused"])
def test_c4_city_restir_reset_in_used_context_bit_exact(city, luts, city_oracle, fused):
    """The C4 timed path: frames rendered, then GPURenderer::reset (sample 0, need_to_reset, the
    seed schedule restarted) in the SAME context, whose G-buffer the first post-reset frame
    reads as the previous frame's (GPURenderer.cpp:953-973, ReSTIRDIRenderPass.cpp:228-231,
    CameraRays.h:78-91).  Whole 1920x1080 city frame against the oracle keeping its ReSTIR DI
    state across the two runs; bit-exact, fused and unfused."""
    import mpt
    from oracle import oracle as orc
    _, env = city_oracle
    passes = 2 if fused else 1
    a = c4_frames(city, 2, fused=fused, passes=passes)
    b = c4_frames(city, 3, fused=fused, passes=passes)
    b[0].render_settings.need_to_reset = True
    r = _gpu(city, luts, env)
    o = orc.Oracle(city, luts, envmap=env, keep_state=True)
    for run in (a, b):
        r.render_samples(run)
        r.synchronize_kernel()
        got = r.framebuffer(abi.FB_COLOR)
        ref = o.render(run)
        _same(got, ref, f"C4 {'fused' if fused else 'unfused'} colour after a reset in a used context")
    # the state mattered: a fresh renderer's post-reset frames differ
    o.reset_state()
    assert not np.array_equal(o.render(b), got)
    o.close()
    r.close()


# ---- C3T: the texture-realistic city (bench --workload c3t) on an 8-row band ------------------

@pytest.mark.gpu
def test_c3t_textured_city_band_bit_exact(luts):
    """70 materials, 83 % of the triangles with base-colour + normal-map + roughness-metallic
    textures (193 MB): per-vertex resolved materials, normal mapping and texel gathers on most
    hits, RIS + envmap MIS + alpha testing as C3, 4 spp on rows 536-543, against the oracle."""
    import mpt
    from mpt import synthetic
    from oracle import oracle as orc
    sd = synthetic.procedural_city_textured()
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    cam = scene.make_camera(sd.camera_info, 1920, 1080)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RIS_BSDF_AND_LIGHT
    st = scene.parity_settings(3)
    st.do_alpha_testing = True
    band = (8, 67, 135)
    frs = [scene.make_frame(cam, 1920, 1080, options=opt, settings=st, world=scene.envmap_world(1.0), sample_number=s,
                            random_seed=seed, band=band) for s, seed in scene.cpu_seed_schedule(4)]
    r = _gpu(sd, luts, env)
    r.render_samples(frs)
    r.synchronize_kernel()
    got = r.framebuffer(abi.FB_COLOR)
    r.close()
    o = orc.Oracle(sd, luts, envmap=env)
    ref = o.render(frs)
    o.close()
    _same(got, ref, "C3T band colour")
    assert np.isfinite(got).all() and got.mean() > 0
