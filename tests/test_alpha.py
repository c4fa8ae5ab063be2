"""Alpha testing (filter_function, FilterFunction.h:19-48; get_hit_base_color_alpha,
Material.h:23-37).

libmpt draws each candidate's uniform from a hash of (query key, primitive) instead of the
path RNG inside HIPRT's traversal (whose order no other BVH reproduces): same accept
probability per candidate, traversal-order independent.  Exact checks:
fully opaque cards with alpha testing on render exactly as with it off; fully transparent
cards render exactly as the scene without them; the HIP path equals the oracle bit for bit."""
import numpy as np
import pytest

from mpt import abi, scene, synthetic

W, H = 40, 24


def frames(sd, alpha, n=3, lss=abi.LSS_MIS_LIGHT_BSDF, world=None):
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    st = scene.parity_settings(3)
    st.do_alpha_testing = alpha
    return [scene.make_frame(cam, W, H, options=opt, settings=st, world=world, sample_number=s, random_seed=seed)
            for s, seed in scene.cpu_seed_schedule(n)]


@pytest.mark.parametrize("lss", [abi.LSS_MIS_LIGHT_BSDF, abi.LSS_RIS_BSDF_AND_LIGHT])
def test_opaque_cards_equal_alpha_testing_off(cornell, luts, oracle_lib, lss):
    sd = synthetic.with_alpha_cards(cornell, opacity=1.0, alpha_levels=(255,))
    o = oracle_lib.Oracle(sd, luts)
    a = o.render(frames(sd, True, lss=lss))
    b = o.render(frames(sd, False, lss=lss))
    assert np.array_equal(a, b)
    o.close()


@pytest.mark.parametrize("lss", [abi.LSS_MIS_LIGHT_BSDF, abi.LSS_RIS_BSDF_AND_LIGHT])
def test_transparent_cards_equal_scene_without_them(cornell, luts, oracle_lib, lss):
    sd = synthetic.with_alpha_cards(cornell, opacity=0.0, alpha_levels=(0,))
    o1 = oracle_lib.Oracle(sd, luts)
    o2 = oracle_lib.Oracle(cornell, luts)
    a = o1.render(frames(sd, True, lss=lss))
    b = o2.render(frames(cornell, True, lss=lss))
    assert np.array_equal(a, b)
    c = o1.render(frames(sd, False, lss=lss))       # alpha testing off: the cards are opaque
    assert not np.array_equal(a, c)
    o1.close()
    o2.close()


def test_partial_alpha_changes_the_image(cornell, luts, oracle_lib):
    sd = synthetic.with_alpha_cards(cornell)
    o = oracle_lib.Oracle(sd, luts)
    a = o.render(frames(sd, True))
    b = o.render(frames(sd, False))
    assert np.isfinite(a).all() and not np.array_equal(a, b)
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["mis", "ris", "ris_env", "uniform_env"])
def test_gpu_alpha_testing_bit_exact(cornell, luts, case):
    import mpt
    from oracle import oracle as orc
    sd = synthetic.with_alpha_cards(cornell)
    lss = {"mis": abi.LSS_MIS_LIGHT_BSDF, "ris": abi.LSS_RIS_BSDF_AND_LIGHT, "ris_env": abi.LSS_RIS_BSDF_AND_LIGHT,
           "uniform_env": abi.LSS_UNIFORM_ONE_LIGHT}[case]
    env = mpt.build_envmap(scene.procedural_sky(128, 64, seed=7)) if case.endswith("env") else None
    world = scene.envmap_world(1.0) if env is not None else None
    frs = frames(sd, True, n=4, lss=lss, world=world)
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    for f in frs:
        r.render(f)
    r.synchronize_kernel()
    g = r.framebuffer(abi.FB_COLOR)
    o = orc.Oracle(sd, luts, envmap=env)
    c = o.render(frs)
    assert np.array_equal(g, c), f"{(g != c).sum()} values differ"
    o.close()
    r.close()
