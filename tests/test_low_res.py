"""The low-resolution interactive mode (do_render_low_resolution, RenderSettings.h:195-198): what
the reference front-end renders while the camera moves (RenderWindow.cpp:797 sets
wants_render_low_resolution = is_interacting(); allow_render_low_resolution defaults to true).

Reference semantics (CameraRays.h:63-76, FullPathTracer.h:117-122, RIS.h:93-94 / 162,
InitialCandidates.h:248-249 / 420-421): CameraRays renders the representative pixels (x, y),
x and y multiples of s = render_low_resolution_scaling, at pixel_index / s, i.e. the frame's
top-left ceil(W / s) x ceil(H / s) block with row stride W; FullPathTracer then traces those
pixels with at most 3 bounces, RIS with one light and one BSDF candidate and no visibility in
its target function, ReSTIR DI with at most one initial candidate of each kind and no initial
visibility.  The reference's pixel_active writes race at colliding indices; both sides render
its evident intent -- the block active, every other pixel inactive.

CPU: the oracle's properties (the block changes, nothing else does; the candidate / bounce /
visibility settings stop mattering).  GPU: the HIP path equals the oracle bit for bit through
full-resolution -> low-resolution -> full-resolution sequences, with RIS, MIS, adaptive
sampling, ReSTIR DI (fused and unfused) and row partitions."""
import numpy as np
import pytest

from mpt import abi, scene

W, H = 47, 33      # odd sizes: ceil(W / s) blocks


def frames(sd, lss=abi.LSS_RIS_BSDF_AND_LIGHT, n=6, low=(2, 3, 4), s=2, band=(1, 0, 1), bounces=5, adaptive=False,
           nl=8, nb=1, vis=False, restir=None, world=None):
    """n frames of one accumulation; the frames in `low` are rendered at low resolution."""
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    opt.ris_use_visibility = 1 if vis else 0
    out = []
    if lss == abi.LSS_RESTIR_DI:
        rd = dict(restir or {})
        sched = [(d["sample_number"], d) for d in scene.gpu_seed_schedule(n, rd.get("passes", 2),
                                                                          fused=rd.get("fused", True))]
    else:
        sched = [(k, {"random_seed": seed}) for k, seed in scene.cpu_seed_schedule(n)]
    for k, d in sched:
        st = scene.parity_settings(bounces)
        st.ris_number_of_light_candidates = nl
        st.ris_number_of_bsdf_candidates = nb
        st.denoiser_AOV_accumulation_counter = k
        st.do_update_status_buffers = k == n - 1
        st.wants_render_low_resolution = k in low
        st.render_low_resolution_scaling = s
        if adaptive:
            st.enable_adaptive_sampling = True
            st.adaptive_sampling_min_samples = 1
            st.adaptive_sampling_noise_threshold = 0.9
        kw = {}
        if lss == abi.LSS_RESTIR_DI:
            st.restir_di_settings.number_of_passes = (restir or {}).get("passes", 2)
            st.restir_di_settings.do_fused_spatiotemporal = (restir or {}).get("fused", True)
            st.restir_di_settings.number_of_initial_light_candidates = (restir or {}).get("initial_lights", 4)
            st.restir_di_settings.number_of_initial_bsdf_candidates = (restir or {}).get("initial_bsdf", 1)
            opt.restir_di_initial_target_visibility = (restir or {}).get("initial_vis", 0)
            kw = dict(camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"])
        out.append(scene.make_frame(cam, W, H, options=opt, settings=st, world=world, sample_number=k,
                                    random_seed=d["random_seed"], band=band, **kw))
    return out


def block(s):
    return -(-H // s), -(-W // s)


def test_oracle_low_res_renders_the_top_left_block(cornell, luts, oracle_lib):
    """A low-resolution frame writes the top-left ceil(H/s) x ceil(W/s) block and nothing else."""
    o = oracle_lib.Oracle(cornell, luts)
    for s in (2, 3, 4):
        full = frames(cornell, n=2, low=())
        low = frames(cornell, n=3, low=(2,), s=s)
        a = o.render(full)
        b = o.render(low)
        bh, bw = block(s)
        outside = np.ones((H, W), bool)
        outside[:bh, :bw] = False
        assert np.array_equal(a[outside], b[outside]), f"s={s}: pixels outside the block changed"
        assert not np.array_equal(a[:bh, :bw], b[:bh, :bw])
        assert np.isfinite(b).all()
    o.close()


def test_oracle_low_res_ignores_candidates_bounces_visibility(cornell, luts, oracle_lib):
    """At low resolution RIS takes one light and one BSDF candidate without visibility and the
    path at most 3 bounces, whatever the settings say (RIS.h:93-94, 162; FullPathTracer.h:117-122)."""
    o = oracle_lib.Oracle(cornell, luts)
    a = o.render(frames(cornell, n=2, low=(0, 1), nl=8, nb=0, vis=True, bounces=7))
    b = o.render(frames(cornell, n=2, low=(0, 1), nl=1, nb=1, vis=False, bounces=3))
    c = o.render(frames(cornell, n=2, low=(), nl=1, nb=1, vis=False, bounces=3))
    o.close()
    assert np.array_equal(a, b)
    bh, bw = block(2)
    assert not np.array_equal(a[:bh, :bw], c[:bh, :bw])      # the low-res block is its own render
    assert (a[bh:] == 0).all() and (a[:, bw:] == 0).all()     # a fresh accumulation: nothing outside


def test_oracle_low_res_restir_initial_candidates_capped(cornell, luts, oracle_lib):
    """ReSTIR DI at low resolution: one initial light / BSDF candidate, no initial visibility
    (InitialCandidates.h:248-249, 420-421)."""
    o = oracle_lib.Oracle(cornell, luts)
    a = o.render(frames(cornell, abi.LSS_RESTIR_DI, n=3, low=(0, 1, 2), restir=dict(initial_lights=6, initial_vis=1)))
    b = o.render(frames(cornell, abi.LSS_RESTIR_DI, n=3, low=(0, 1, 2), restir=dict(initial_lights=1, initial_vis=0)))
    o.close()
    assert np.array_equal(a, b)


CASES = {
    # name: frames kwargs
    "ris_s2": dict(),
    "ris_s3_vis": dict(s=3, vis=True),
    "ris_s4_adaptive": dict(s=4, adaptive=True),
    "mis_s2": dict(lss=abi.LSS_MIS_LIGHT_BSDF),
    "ris_s1": dict(s=1),
    "restir_fused_s2": dict(lss=abi.LSS_RESTIR_DI),
    "restir_unfused_s3": dict(lss=abi.LSS_RESTIR_DI, s=3, restir=dict(fused=False, passes=1)),
    "restir_initial_vis_s2": dict(lss=abi.LSS_RESTIR_DI, restir=dict(initial_vis=1, initial_lights=3)),
    "restir_s4_adaptive": dict(lss=abi.LSS_RESTIR_DI, s=4, adaptive=True),
    "envmap_restir_s2": dict(lss=abi.LSS_RESTIR_DI, envmap=True),
}


def _case_frames(sd, case, band=(1, 0, 1)):
    import mpt
    kw = dict(CASES[case])
    env = None
    if kw.pop("envmap", False):
        env = mpt.build_envmap(scene.procedural_sky(128, 64, seed=7))
        kw["world"] = scene.envmap_world(1.0)
    return frames(sd, band=band, **kw), env


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES))
def test_gpu_low_res_bit_exact(cornell, luts, case):
    import mpt
    from oracle import oracle as orc
    frs, env = _case_frames(cornell, case)
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    r.render_samples(frs)
    r.synchronize_kernel()
    got = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
    cnt = r.aux_buffer(abi.AUX_SAMPLE_COUNT) if CASES[case].get("adaptive") else None
    r.close()
    o = orc.Oracle(cornell, luts, envmap=env)
    ref = o.render(frs, aov=True)
    for g, c, what in zip(got, ref, ("color", "albedo", "normals")):
        assert np.array_equal(g, c), f"{case} {what}: {(g != c).sum()} values differ"
    if cnt is not None:
        assert np.array_equal(cnt, o.last_aux["sample_count"])
    o.close()
    assert got[0].mean() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ris_s3_vis", "restir_fused_s2"])
def test_gpu_low_res_partitioned_equals_single(cornell, luts, case):
    """Row partitions (interleaved 8-row bands; ReSTIR DI: contiguous bands + halo exchange)
    render the low-resolution frames exactly as one context does."""
    import mpt
    ref_frames, env = _case_frames(cornell, case)
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    r.render_samples(ref_frames)
    r.synchronize_kernel()
    ref = r.framebuffer(abi.FB_COLOR)
    r.close()
    if CASES[case].get("lss") == abi.LSS_RESTIR_DI:
        import sys
        import os
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from test_restir import render_partitioned_local
        got = render_partitioned_local(cornell, luts, lambda band: _case_frames(cornell, case, band)[0], W, H, 3, env=env)
    else:
        parts = []
        for k in range(3):
            r = mpt.GPURenderer(0)
            r.set_scene(cornell)
            r.set_luts(luts)
            r.render_samples(_case_frames(cornell, case, (8, k, 3))[0])
            r.synchronize_kernel()
            parts.append(r.framebuffer(abi.FB_COLOR))
            r.close()
        from mpt import partition
        got = partition.assemble(parts, H, 8)
    assert np.array_equal(got, ref), f"{(got != ref).sum()} values differ"


@pytest.mark.gpu
def test_gpu_low_res_rejects_bad_scaling(cornell, luts):
    import mpt
    f = frames(cornell, n=1, low=(0,), s=0)[0]
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    with pytest.raises(mpt.MptError):
        r.render(f)
    f.render_settings.allow_render_low_resolution = False     # not low resolution: s unused
    r.render(f)
    r.synchronize_kernel()
    r.close()
