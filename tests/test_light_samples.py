"""Light-sampling options the front-end exposes beyond the defaults (extended light sampling,
mpt_internal.h): number_of_light_samples > 1 (sample_many_lights, Lights.h:222-241; UI 1-8,
ImGuiSettingsWindow.cpp:787), RIS with several BSDF candidates (RIS.h:193-286; UI 0-16,
ImGuiSettingsWindow.cpp:833) and RISUseVisiblityTargetFunction (RIS.h:161-171).

CPU: the oracle's estimators keep their expectation (more light samples or candidates only
lower the variance; the visibility target function is unbiased too).
GPU: bit-exact against the oracle, for every light-sampling strategy, inside dielectrics
(the RIS final shadow ray then differs from the candidate's), with alpha testing, under an
envmap, with ReSTIR DI's later bounces and through the batched wavefronts (ReSTIR DI: each
sample's first bounce in turn, the later bounces' extended light sampling batched)."""
import numpy as np
import pytest

from mpt import abi, scene, synthetic

W, H = 40, 30
LSS = {"uniform": abi.LSS_UNIFORM_ONE_LIGHT, "bsdf": abi.LSS_BSDF, "mis": abi.LSS_MIS_LIGHT_BSDF,
       "ris": abi.LSS_RIS_BSDF_AND_LIGHT, "restir": abi.LSS_RESTIR_DI}


def frames(sd, lss, n, nls=1, nl=4, nb=1, vis=0, w=W, h=H, bounces=3, world=None, alpha=False, ovr=abi.BSDF_NONE,
           later=abi.RESTIR_DI_LATER_BOUNCES_RIS_BSDF_AND_LIGHT):
    cam = scene.make_camera(sd.camera_info, w, h)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    opt.ris_use_visibility = vis
    opt.bsdf_override = ovr
    opt.restir_di_later_bounces_sampling_strategy = later
    out = []
    if lss == abi.LSS_RESTIR_DI:
        sched = [(d["sample_number"], d["random_seed"], d["camera_random_seed"], d["restir_di_seeds"])
                 for d in scene.gpu_seed_schedule(n, 2)]
    else:
        sched = [(s_, seed, 0, None) for s_, seed in scene.cpu_seed_schedule(n)]
    for s_, seed, cseed, rseeds in sched:
        st = scene.parity_settings(bounces)
        st.do_alpha_testing = alpha
        st.number_of_light_samples = nls
        st.ris_number_of_light_candidates = nl
        st.ris_number_of_bsdf_candidates = nb
        out.append(scene.make_frame(cam, w, h, options=opt, settings=st, world=world, sample_number=s_, random_seed=seed,
                                    camera_random_seed=cseed, restir_di_seeds=rseeds))
    return out


# ---- CPU: expectations ------------------------------------------------------------------------

@pytest.mark.parametrize("case", ["n3_mis", "n2_ris", "ris_4_bsdf_candidates", "ris_visibility", "ris_2x3_visibility"])
def test_oracle_estimators_keep_expectation(cornell, luts, oracle_lib, case):
    o = oracle_lib.Oracle(cornell, luts)
    ref = o.render(frames(cornell, abi.LSS_MIS_LIGHT_BSDF, 256, bounces=1)).mean() / 256
    kw = {"n3_mis": dict(lss=abi.LSS_MIS_LIGHT_BSDF, nls=3), "n2_ris": dict(lss=abi.LSS_RIS_BSDF_AND_LIGHT, nls=2),
          "ris_4_bsdf_candidates": dict(lss=abi.LSS_RIS_BSDF_AND_LIGHT, nb=4),
          "ris_visibility": dict(lss=abi.LSS_RIS_BSDF_AND_LIGHT, vis=1),
          "ris_2x3_visibility": dict(lss=abi.LSS_RIS_BSDF_AND_LIGHT, nl=2, nb=3, vis=1)}[case]
    lss = kw.pop("lss")
    a = o.render(frames(cornell, lss, 128, bounces=1, **kw)).mean() / 128
    # RIS with the reference's minimum_light_contribution (0.08) is slightly biased against MIS
    tol = 0.03 if lss == abi.LSS_MIS_LIGHT_BSDF else 0.06
    assert abs(a / ref - 1.0) < tol, (case, a, ref)
    o.close()


# ---- GPU: bit-exact ---------------------------------------------------------------------------

CASES = {
    # name: (scene, frames kwargs)
    "uniform_n3": ("cornell", dict(lss="uniform", nls=3)),
    "bsdf_n2": ("cornell", dict(lss="bsdf", nls=2)),
    "mis_n2": ("cornell", dict(lss="mis", nls=2)),
    "mis_n8": ("cornell", dict(lss="mis", nls=8, bounces=2)),
    "ris_n2": ("cornell", dict(lss="ris", nls=2)),
    "ris_bsdf_candidates_2": ("cornell", dict(lss="ris", nb=2)),
    "ris_bsdf_candidates_16": ("cornell", dict(lss="ris", nb=16, bounces=2)),
    "ris_bsdf_only_3": ("cornell", dict(lss="ris", nl=0, nb=3)),
    "ris_visibility": ("cornell", dict(lss="ris", vis=1)),
    "ris_visibility_n3_2x2": ("cornell", dict(lss="ris", vis=1, nls=3, nl=2, nb=2)),
    "ris_visibility_lights_only": ("cornell", dict(lss="ris", vis=1, nb=0, nl=6)),
    "ris_visibility_inside_glass": ("nested-dielectrics", dict(lss="ris", vis=1, nb=2, bounces=6)),
    "mis_n2_inside_glass": ("nested-dielectrics", dict(lss="mis", nls=2, bounces=6)),
    "ris_visibility_alpha_cards": ("alpha", dict(lss="ris", vis=1, nb=2, alpha=True)),
    "mis_n2_alpha_cards": ("alpha", dict(lss="mis", nls=2, alpha=True)),
    "ris_n2_envmap": ("envmap", dict(lss="ris", nls=2, nb=2)),
    "lambert_ris_n2_visibility": ("cornell", dict(lss="ris", nls=2, vis=1, ovr=abi.BSDF_LAMBERTIAN)),
    "oren_nayar_mis_n2": ("cornell", dict(lss="mis", nls=2, ovr=abi.BSDF_OREN_NAYAR)),
    "restir_later_ris_n2_visibility": ("cornell", dict(lss="restir", nls=2, vis=1, nb=2)),
    "restir_later_mis_n3": ("cornell", dict(lss="restir", nls=3, later=abi.RESTIR_DI_LATER_BOUNCES_MIS_LIGHT_BSDF)),
}


def _scene(kind, cornell):
    import mpt
    if kind == "cornell":
        return cornell, None, None
    if kind == "alpha":
        return synthetic.with_alpha_cards(cornell), None, None
    if kind == "envmap":
        return cornell, mpt.build_envmap(scene.procedural_sky(128, 64, seed=7)), scene.envmap_world(0.8)
    return scene.load_scene(kind), None, None


@pytest.mark.gpu
@pytest.mark.parametrize("batched", [False, True], ids=["frames", "batched"])
@pytest.mark.parametrize("case", list(CASES))
def test_gpu_light_sampling_options_bit_exact(cornell, luts, case, batched):
    import mpt
    from oracle import oracle as orc
    kind, kw = CASES[case]
    kw = dict(kw)
    sd, env, world = _scene(kind, cornell)
    frs = frames(sd, LSS[kw.pop("lss")], 3, world=world, **kw)
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    if batched:
        r.render_samples(frs, max_batch=3)
    else:
        for f in frs:
            r.render(f)
    r.synchronize_kernel()
    got = [r.framebuffer(k) for k in (abi.FB_COLOR, abi.FB_ALBEDO, abi.FB_NORMALS)]
    st = r.stats()
    r.close()
    o = orc.Oracle(sd, luts, envmap=env)
    ref = o.render(frs, aov=True)
    o.close()
    for k, what in enumerate(["color", "albedo", "normals"]):
        bad = ~((got[k] == ref[k]) | (np.isnan(got[k]) & np.isnan(ref[k])))
        assert not bad.any(), f"{case} {what}: {int(bad.sum())} values differ, first at {np.argwhere(bad)[:3].tolist()}"
    assert np.isfinite(got[0]).all() and got[0].mean() > 0
    assert st.rays_any + st.rays_closest > 0


@pytest.mark.gpu
def test_gpu_light_samples_ray_count(cornell, luts):
    """Every light sample traces its own rays: the any-hit count grows with the samples."""
    import mpt
    counts = {}
    for n in (1, 4):
        r = mpt.GPURenderer(0)
        r.set_scene(cornell)
        r.set_luts(luts)
        r.enable_stats(timing=False)
        for f in frames(cornell, abi.LSS_MIS_LIGHT_BSDF, 2, nls=n):
            r.render(f)
        counts[n] = r.stats().rays_any
        r.close()
    assert counts[4] > 3 * counts[1]
