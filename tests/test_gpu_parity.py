"""GPU parity: the HIP path (through the C ABI, libmpt.so) against the CPU oracle.

Bar: bit-exact.  Traversal results (prim, t, u, v) and rendered sums / AOVs must equal
the oracle's float32 values exactly -- the device code is compiled without
contraction, both sides evaluate every transcendental with the same single-precision
sequence of IEEE operations (csrc/tmath.h, pinned against libm by tests/test_tmath.py) and
the RNG stream of every path is consumed in the reference's order (DESIGN.md "Parity").
At the bench size (1920x1080) the properties checked are size-independent: run-to-run
determinism, partition invariance and finite output.
"""
import numpy as np
import pytest

import mpt
from mpt import abi, partition, scene

pytestmark = pytest.mark.gpu

STRATEGIES = {"none": abi.LSS_NO_DIRECT_LIGHT_SAMPLING, "uniform": abi.LSS_UNIFORM_ONE_LIGHT, "bsdf": abi.LSS_BSDF,
              "mis": abi.LSS_MIS_LIGHT_BSDF, "ris": abi.LSS_RIS_BSDF_AND_LIGHT}


@pytest.fixture(scope="module")
def scenes():
    return {n: scene.load_scene(n) for n in ("cornell_pbr", "nested-dielectrics", "nested-dielectrics-complex",
                                              "multi-dispersion")}


@pytest.fixture(scope="module")
def sky():
    return mpt.build_envmap(scene.procedural_sky(256, 128, seed=7))


_cache = {}


def renderer(sd, luts, env=None):
    key = (sd.name, id(sd), env is not None)
    if key not in _cache:
        r = mpt.GPURenderer(0)
        r.set_scene(sd)
        r.set_luts(luts)
        if env is not None:
            r.set_envmap(env)
        _cache[key] = r
    return _cache[key]


_oracles = {}


def oracle_for(sd, luts, env=None):
    from oracle import oracle as orc
    key = (id(sd), env is not None)
    if key not in _oracles:
        _oracles[key] = orc.Oracle(sd, luts, envmap=env)
    return _oracles[key]


def frames(sd, W, H, n, ovr=abi.BSDF_NONE, lss=abi.LSS_MIS_LIGHT_BSDF, band=(1, 0, 1), bounces=3, world=None,
           env_mis=1, ess=abi.ESS_ALIAS_TABLE, first=0):
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.bsdf_override, opt.direct_light_sampling = ovr, lss
    opt.envmap_bsdf_mis, opt.envmap_sampling = env_mis, ess
    return [scene.make_frame(cam, W, H, options=opt, settings=scene.parity_settings(bounces), world=world,
                             sample_number=s + first, random_seed=seed, band=band)
            for s, seed in scene.cpu_seed_schedule(n)]


def gpu_render(r, frs):
    for f in frs:
        r.render(f)
    r.synchronize_kernel()
    return r.framebuffer(abi.FB_COLOR), r.framebuffer(abi.FB_ALBEDO), r.framebuffer(abi.FB_NORMALS)


def assert_same(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, what
    diff = np.argwhere(~((a == b) | (np.isnan(a) & np.isnan(b))))
    assert len(diff) == 0, f"{what}: {len(diff)} values differ, first at {diff[:3].tolist()}: " \
                           f"{a[tuple(diff[0])]} vs {b[tuple(diff[0])]}"


# ------------------------------------------------------------------------------------
# Traversal
# ------------------------------------------------------------------------------------
def random_rays(sd, n, seed, spread=1.5):
    rng = np.random.default_rng(seed)
    lo, hi = sd.vertices.min(0), sd.vertices.max(0)
    c, e = (lo + hi) / 2, (hi - lo) / 2 * spread
    o = c + e * (2 * rng.random((n, 3)) - 1)
    d = rng.normal(size=(n, 3))
    d[: n // 8, 0] = 0.0          # axis-parallel components (box-test reciprocal edge cases)
    d[n // 8: n // 4, 1:] = 0.0
    d /= np.maximum(np.linalg.norm(d, axis=1, keepdims=True), 1e-12)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3], r[:, 4:7], r[:, 7] = o, d, 1e30
    return r


@pytest.mark.parametrize("name", ["cornell_pbr", "nested-dielectrics-complex", "multi-dispersion"])
def test_traversal_closest_bit_exact(scenes, luts, name):
    sd = scenes[name]
    r = renderer(sd, luts)
    o = oracle_for(sd, luts)
    rays = random_rays(sd, 200000, 5)
    gp, gt, gu, gv = r.trace_closest(rays)
    op, ot, ou, ov = o.trace_closest(rays)
    assert_same(gp, op, "prim")
    hit = op >= 0
    assert hit.mean() > 0.05
    assert_same(gt[hit], ot[hit], "t")
    assert_same(gu[hit], ou[hit], "u")
    assert_same(gv[hit], ov[hit], "v")
    # re-trace from the hit point excluding the hit primitive (filter function of Intersect.h)
    o2 = rays.copy()
    o2[hit, 0:3] = rays[hit, 0:3] + ot[hit, None] * rays[hit, 4:7]
    lh = np.where(hit, op, -1).astype(np.int32)
    gp2, gt2, _, _ = r.trace_closest(o2, lh)
    op2, ot2, _, _ = o.trace_closest(o2, lh)
    assert_same(gp2, op2, "prim after last-hit filter")
    assert_same(gt2[op2 >= 0], ot2[op2 >= 0], "t after last-hit filter")


def test_traversal_any_hit_consistent(scenes, luts):
    sd = scenes["cornell_pbr"]
    r = renderer(sd, luts)
    o = oracle_for(sd, luts)
    rays = random_rays(sd, 100000, 9)
    rng = np.random.default_rng(2)
    rays[:, 7] = rng.random(len(rays)).astype(np.float32) * 3.0
    occ = r.trace_any(rays)
    op, ot, _, _ = o.trace_closest(rays)
    expect = (op >= 0) & (ot < rays[:, 7])
    assert_same(occ, expect, "occluded")


def test_empty_and_single_ray_queries(scenes, luts):
    r = renderer(scenes["cornell_pbr"], luts)
    p, t, u, v = r.trace_closest(np.zeros((0, 8), np.float32))
    assert len(p) == 0
    one = random_rays(scenes["cornell_pbr"], 1, 1)
    assert len(r.trace_closest(one)[0]) == 1


# ------------------------------------------------------------------------------------
# Rendering
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize("ovr", [abi.BSDF_NONE, abi.BSDF_LAMBERTIAN, abi.BSDF_OREN_NAYAR],
                         ids=["principled", "lambert", "oren_nayar"])
@pytest.mark.parametrize("strategy", list(STRATEGIES))
def test_render_cornell_bit_exact(scenes, luts, ovr, strategy):
    sd = scenes["cornell_pbr"]
    W, H = 48, 32
    frs = frames(sd, W, H, 3, ovr=ovr, lss=STRATEGIES[strategy])
    g = gpu_render(renderer(sd, luts), frs)
    c = oracle_for(sd, luts).render(frs, aov=True)
    for k, name in enumerate(["color", "albedo", "normals"]):
        assert_same(g[k], c[k], f"{strategy} {name}")
    assert np.isfinite(g[0]).all() and g[0].mean() > 0


@pytest.mark.parametrize("name,bounces", [("nested-dielectrics", 8), ("nested-dielectrics-complex", 8),
                                          ("multi-dispersion", 8)])
@pytest.mark.parametrize("strategy", ["mis", "ris"])
def test_render_dielectric_scenes_bit_exact(scenes, luts, name, bounces, strategy):
    sd = scenes[name]
    W, H = 40, 30
    frs = frames(sd, W, H, 2, lss=STRATEGIES[strategy], bounces=bounces)
    g = gpu_render(renderer(sd, luts), frs)
    c = oracle_for(sd, luts).render(frs, aov=True)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(g[k], c[k], f"{name} {strategy} {what}")


@pytest.mark.parametrize("strategy,env_mis,ess", [("mis", 1, abi.ESS_ALIAS_TABLE), ("ris", 1, abi.ESS_ALIAS_TABLE),
                                                  ("mis", 0, abi.ESS_ALIAS_TABLE), ("mis", 1, abi.ESS_NO_SAMPLING),
                                                  ("mis", 1, abi.ESS_BINARY_SEARCH), ("ris", 0, abi.ESS_BINARY_SEARCH)])
def test_render_envmap_bit_exact(scenes, luts, sky, strategy, env_mis, ess):
    sd = scenes["nested-dielectrics"]
    W, H = 40, 30
    frs = frames(sd, W, H, 2, lss=STRATEGIES[strategy], world=scene.envmap_world(0.5), env_mis=env_mis, ess=ess)
    g = gpu_render(renderer(sd, luts, sky), frs)
    c = oracle_for(sd, luts, sky).render(frs, aov=True)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(g[k], c[k], f"envmap {strategy} {what}")


@pytest.mark.parametrize("band", [(4, 0, 3), (4, 2, 3), (8, 1, 2), (1, 5, 7)])
def test_partition_bit_exact(scenes, luts, band):
    sd = scenes["cornell_pbr"]
    W, H = 40, 36
    r = renderer(sd, luts)
    full = gpu_render(r, frames(sd, W, H, 2))[0]
    part = gpu_render(r, frames(sd, W, H, 2, band=band))[0]
    assert_same(part, full[partition.rows_of(H, *band)], f"band {band}")


def test_accumulation_restarts_at_sample_zero(scenes, luts):
    sd = scenes["cornell_pbr"]
    r = renderer(sd, luts)
    a = gpu_render(r, frames(sd, 32, 16, 2))[0]
    b = gpu_render(r, frames(sd, 32, 16, 2))[0]       # sample_number 0 again: assign, not add
    assert_same(a, b, "re-render")


def test_oren_nayar_override_sigma_and_texture(luts):
    """BSDF_OREN_NAYAR (OrenNayar.h; the reference's own dispatcher line does not compile,
    dev_bsdf.h bsdf_eval): per-material sigma values from smooth to very rough, and the
    Oren-Nayar sigma texture slot of the textured panels, GPU vs oracle."""
    import copy
    from mpt import synthetic
    sd0 = scene.load_scene("cornell_pbr")
    mats = [abi.Material.from_buffer_copy(m) for m in sd0.materials]
    for i, m in enumerate(mats):
        m.oren_nayar_sigma = [0.0, 0.2, 0.5, 1.0, 1.5][i % 5]
    sd = copy.copy(sd0)
    sd.materials = mats
    for s_ in (sd, synthetic.with_textured_panels(sd0)):
        frs = frames(s_, 40, 30, 3, ovr=abi.BSDF_OREN_NAYAR, lss=abi.LSS_RIS_BSDF_AND_LIGHT, bounces=4)
        r = mpt.GPURenderer(0)
        r.set_scene(s_)
        r.set_luts(luts)
        g = gpu_render(r, frs)
        r.close()
        c = oracle_for(s_, luts).render(frs, aov=True)
        for k, name in enumerate(["color", "albedo", "normals"]):
            assert_same(g[k], c[k], f"oren-nayar {s_.name} {name}")


def test_unsupported_options_fail_loudly(scenes, luts):
    sd = scenes["cornell_pbr"]
    r = renderer(sd, luts)
    f = frames(sd, 16, 16, 1)[0]
    f.render_settings.restir_di_settings.number_of_passes = 5   # more spatial passes than restir_di_seeds holds
    f.options.direct_light_sampling = abi.LSS_RESTIR_DI
    with pytest.raises(mpt.MptError) as e:
        r.render(f)
    assert e.value.code == -4
    f = frames(sd, 16, 16, 1, lss=abi.LSS_RESTIR_DI, band=(8, 0, 2))[0]   # interleaved bands under ReSTIR DI
    with pytest.raises(mpt.MptError):
        r.render(f)


def test_full_size_properties(scenes, luts):
    """Bench configuration (1920x1080, Principled + MIS): determinism, partition
    invariance, finite output and the oracle on a band subset."""
    sd = scenes["cornell_pbr"]
    W, H = 1920, 1080
    r = renderer(sd, luts)
    a = gpu_render(r, frames(sd, W, H, 2))[0]
    b = gpu_render(r, frames(sd, W, H, 2))[0]
    assert_same(a, b, "determinism")
    assert np.isfinite(a).all()
    band = (8, 3, 64)
    p = gpu_render(r, frames(sd, W, H, 2, band=band))[0]
    ys = partition.rows_of(H, *band)
    assert_same(p, a[ys], "partition at full size")
    c = oracle_for(sd, luts).render(frames(sd, W, H, 2, band=band))
    assert_same(p, c, "oracle on a band subset of the full frame")


@pytest.fixture(scope="module")
def city():
    from mpt import synthetic
    return synthetic.procedural_city(1234)


@pytest.mark.parametrize("strategy", ["ris", "ris_alpha", "mis"])
def test_render_city_stand_in_bit_exact(city, luts, strategy):
    """The bench workload (C3 stand-in: 2.86 M triangles, alpha-tested leaf cards, HDR
    sky with alias-table sampling + BSDF MIS) on a band subset of the 1920x1080 frame."""
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    band = (8, 5, 48)
    frs = frames(city, 1920, 1080, 2, lss=STRATEGIES[strategy.split("_")[0]], world=scene.envmap_world(1.0), band=band)
    for f in frs:
        f.render_settings.do_alpha_testing = strategy.endswith("alpha")
    g = gpu_render(renderer(city, luts, env), frs)
    c = oracle_for(city, luts, env).render(frs, aov=True)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(g[k], c[k], f"city {strategy} {what}")
    assert np.isfinite(g[0]).all() and g[0].mean() > 0


def test_traversal_grazing_rays_city(city, luts):
    """Rays inside a wall's plane (coplanar-edge hits): the padded BVH8 boxes must not cull
    a triangle Moller-Trumbore accepts, so closest and any hit equal the oracle's."""
    from raygen import grazing_rays
    rays, lh = grazing_rays(city, 200000, 21)
    r = renderer(city, luts)
    o = oracle_for(city, luts)
    gp, gt, gu, gv = r.trace_closest(rays, lh)
    op, ot, ou, ov = o.trace_closest(rays, lh)
    assert_same(gp, op, "grazing prim")
    hit = op >= 0
    assert hit.mean() > 0.01
    assert_same(gt[hit], ot[hit], "grazing t")
    assert_same(gu[hit], ou[hit], "grazing u")
    rays[:, 7] = np.float32(1e35) - np.float32(1e-4)
    occ = r.trace_any(rays, lh)
    assert_same(occ, hit & (ot < rays[:, 7]), "grazing occluded")


def gpu_render_batched(r, frs, max_batch):
    r.render_samples(frs, max_batch=max_batch)
    r.synchronize_kernel()
    return r.framebuffer(abi.FB_COLOR), r.framebuffer(abi.FB_ALBEDO), r.framebuffer(abi.FB_NORMALS)


@pytest.mark.parametrize("max_batch,band,strategy", [(4, (1, 0, 1), "mis"), (2, (1, 0, 1), "ris"), (5, (4, 1, 3), "mis"),
                                                     (32, (1, 0, 1), "ris")])
def test_batched_samples_bit_exact(scenes, luts, max_batch, band, strategy):
    """mpt_render_frames (GPURenderer::render's samples_per_frame loop as one wavefront of
    several samples per pixel) equals one mpt_render_frame per sample and the oracle,
    including a batch that does not divide the sample count and a partitioned context."""
    sd = scenes["cornell_pbr"]
    W, H = 40, 36
    r = renderer(sd, luts)
    frs = frames(sd, W, H, 5, lss=STRATEGIES[strategy], band=band)
    seq = gpu_render(r, frs)
    bat = gpu_render_batched(r, frs, max_batch)
    ref = oracle_for(sd, luts).render(frs, aov=True)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(bat[k], seq[k], f"batched vs sequential {what}")
        assert_same(bat[k], ref[k], f"batched vs oracle {what}")


def test_batched_samples_city_alpha_bit_exact(city, luts):
    """Batching on the bench workload with alpha testing (alpha keys from each sample's own
    seed) and textured materials (per-path resolved materials)."""
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    band = (8, 7, 48)
    frs = frames(city, 1920, 1080, 3, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=band)
    for f in frs:
        f.render_settings.do_alpha_testing = True
    r = renderer(city, luts, env)
    bat = gpu_render_batched(r, frs, 3)
    ref = oracle_for(city, luts, env).render(frs, aov=True)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(bat[k], ref[k], f"city batched {what}")


def test_batched_samples_fall_back_for_adaptive(scenes, luts):
    """Adaptive sampling gates each sample's camera rays on the previous samples: batched
    frames are traced speculatively (pixels that converged before the batch began are left out
    of its camera queue) and k_accumulate replays the gate in sample order, so the batched render
    equals the sequential one."""
    sd = scenes["cornell_pbr"]
    r = renderer(sd, luts)
    frs = frames(sd, 32, 16, 6)
    for f in frs:
        f.render_settings.enable_adaptive_sampling = True
        f.render_settings.adaptive_sampling_min_samples = 2
        f.render_settings.adaptive_sampling_noise_threshold = 0.5
    seq = gpu_render(r, frs)[0]
    bat = gpu_render_batched(r, frs, 4)[0]
    assert_same(bat, seq, "adaptive frames through mpt_render_frames")


def test_city_full_frame_batched_equals_sequential(city, luts):
    """The bench configuration at its full size (C3 stand-in, 1920x1080, RIS + envmap +
    alpha testing): one 4-sample wavefront equals four single-sample frames over the whole
    frame, and the sums are finite -- the size-independent property behind the bench's
    batched timing (the oracle checks a band of the same frames in bench.py)."""
    env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
    frs = frames(city, 1920, 1080, 4, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0))
    for f in frs:
        f.render_settings.do_alpha_testing = True
    r = renderer(city, luts, env)
    seq = gpu_render(r, frs)
    bat = gpu_render_batched(r, frs, 4)
    for k, what in enumerate(["color", "albedo", "normals"]):
        assert_same(bat[k], seq[k], f"full-frame batched vs sequential {what}")
    assert np.isfinite(bat[0]).all() and bat[0].mean() > 0


@pytest.mark.parametrize("mode", ["shallow_rebuild", "cost_collapse"])
def test_traversal_bvh_variants_bit_exact(scenes, luts, monkeypatch, mode):
    """BVH variants give the same hits (traversal results never depend on the BVH): a tree
    rebuilt shallower because it is too deep for the traversal stack (forced by the
    MPT_BVH_MAX_STACK test hook: balanced splits from a smaller depth on, instead of refusing
    the scene) and the surface-area cost collapse (MPT_BVH_COLLAPSE=cost), against the oracle."""
    import mpt
    if mode == "shallow_rebuild":
        monkeypatch.setenv("MPT_BVH_MAX_STACK", "16")   # Cornell: depth 8 (SAH) -> 7 (balanced)
    else:
        monkeypatch.setenv("MPT_BVH_COLLAPSE", "cost")
    sd = scenes["cornell_pbr"]
    r = mpt.GPURenderer(0)
    try:
        r.set_scene(sd)
        r.set_luts(luts)
        o = oracle_for(sd, luts)
        rays = random_rays(sd, 100000, 11)
        gp, gt, _, _ = r.trace_closest(rays)
        op, ot, _, _ = o.trace_closest(rays)
        assert_same(gp, op, f"{mode}: prim")
        assert_same(gt[op >= 0], ot[op >= 0], f"{mode}: t")
    finally:
        r.close()


@pytest.mark.parametrize("display", [False, True], ids=["dropped", "display_nans"])
def test_display_nans_bit_exact(cornell, luts, display):
    """A sample that fails the sanity check (negative colour: a wall given negative emission) is
    dropped, or with display_NaNs painted (1e30, 0, 1e30) x sample_number into the sum
    (FullPathTracer.h:29-35, 80-95) -- GPU equals the oracle, both ways."""
    import copy
    from oracle import oracle as orc
    sd = copy.copy(cornell)
    mats = [abi.Material.from_buffer_copy(m) for m in cornell.materials]
    wall = int(cornell.material_indices[0])
    mats[wall].emission = abi.Color(-3.0, -3.0, -3.0)
    mats[wall].emission_strength = 1.0
    sd.materials = mats
    frs = frames(sd, 40, 30, 3)
    for f in frs:
        f.render_settings.display_NaNs = display
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    r.render_samples(frs)
    r.synchronize_kernel()
    got = r.framebuffer(abi.FB_COLOR)
    r.close()
    o = orc.Oracle(sd, luts)
    ref = o.render(frs)
    o.close()
    assert np.array_equal(got, ref), f"{(got != ref).sum()} values differ"
    painted = got[..., 0] >= 1.0e30
    assert painted.any() == display


def test_graph_replay_equals_direct_launches(scenes, luts, monkeypatch):
    """One-sample launch sets replayed from a captured HIP graph (mpt_render_frame, MPT_GRAPHS=1):
    the same sums as direct launches, across seeds, a moving camera (replayed: the camera is read
    from the frame), a strategy change and low resolution (each re-captured), adaptive sampling,
    and the oracle on the whole sequence."""
    from oracle import oracle as orc
    sd = scenes["cornell_pbr"]
    W, H = 40, 30
    frs = frames(sd, W, H, 3) + frames(sd, W, H, 3, lss=abi.LSS_RIS_BSDF_AND_LIGHT, first=3)
    ci = dict(sd.camera_info)
    ci["position"] = [float(v) + 0.03 for v in ci["position"]]
    moved = scene.make_camera(ci, W, H)
    frs[1].current_camera = moved
    frs[2].current_camera = moved
    frs[2].prev_camera = moved
    frs[4].render_settings.wants_render_low_resolution = True
    frs[4].render_settings.render_low_resolution_scaling = 2
    out = {}
    for mode in ("direct", "graph"):
        monkeypatch.setenv("MPT_GRAPHS", "0" if mode == "direct" else "1")
        r = mpt.GPURenderer(0)
        r.set_scene(sd)
        r.set_luts(luts)
        for f in frs:
            r.render(f)
        r.synchronize_kernel()
        out[mode] = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
        st = r.stats()
        if mode == "graph":   # the graph path really ran: re-captured per launch-set change only
            assert st.graph_replays == len(frs) and 1 <= st.graph_captures < len(frs), \
                (st.graph_captures, st.graph_replays)
        else:
            assert st.graph_replays == 0
        r.close()
    for g, d in zip(out["graph"], out["direct"]):
        assert np.array_equal(g, d), f"{(g != d).sum()} values differ"
    o = orc.Oracle(sd, luts)
    ref = o.render(frs)
    o.close()
    assert np.array_equal(out["graph"][0], ref)


def test_graph_captured_once_over_identical_launch_sets(scenes, luts, monkeypatch):
    """Frames that differ only in seeds and sample number share one captured graph: the cache key
    (the frame with its per-sample fields cleared, the scene and path-state views, the launch
    flags) must not pick up stray bytes (struct padding) that would re-capture every frame."""
    sd = scenes["cornell_pbr"]
    monkeypatch.setenv("MPT_GRAPHS", "1")
    frs = frames(sd, 32, 24, 6)
    with mpt.GPURenderer(0) as r:
        r.set_scene(sd)
        r.set_luts(luts)
        for f in frs:
            r.render(f)
        r.synchronize_kernel()
        st = r.stats()
    assert st.graph_replays == len(frs) and st.graph_captures == 1, (st.graph_captures, st.graph_replays)
