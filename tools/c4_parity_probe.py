"""Development probe (GPU box): the C4 frames (city + sky, ReSTIR DI, alpha testing) at a
reduced resolution over many samples, GPU against the oracle, per implementation switch
(MPT_RESTIR_STAGED / MPT_RESTIR_BATCH / MPT_SHADE_CLASSES ...), to localise a divergence.
usage: python tools/c4_parity_probe.py W H frames [prefix 0|1] [envmap width]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)

import mpt  # noqa: E402
from mpt import abi, scene, synthetic  # noqa: E402
from oracle import oracle as orc  # noqa: E402

VARIANTS = [
    ("default", {}),
    ("unbatched", {"MPT_RESTIR_BATCH": "0"}),
    ("monolithic", {"MPT_RESTIR_STAGED": "0"}),
    ("mono_unbatched", {"MPT_RESTIR_STAGED": "0", "MPT_RESTIR_BATCH": "0"}),
]


def frames(city, W, H, n, passes=2):
    cam = scene.make_camera(city.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RESTIR_DI
    out = []
    for d in scene.gpu_seed_schedule(n, passes, fused=True):
        st = scene.parity_settings(3)
        st.do_alpha_testing = True
        st.restir_di_settings.number_of_passes = passes
        out.append(scene.make_frame(cam, W, H, options=opt, settings=st, world=scene.envmap_world(1.0),
                                    sample_number=d["sample_number"], random_seed=d["random_seed"],
                                    camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"]))
    return out


def main():
    W, H, n = (int(a) for a in sys.argv[1:4])
    prefix = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    ew = int(sys.argv[5]) if len(sys.argv) > 5 else 512
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(ew, ew // 2, seed=7))
    luts = scene.load_luts()
    frs = frames(city, W, H, n)
    o = orc.Oracle(city, luts, envmap=env)
    refs = []
    for k in (range(1, n + 1) if prefix else [n]):   # the oracle's image after k samples (prefix renders)
        refs.append(o.render(frs[:k]))
    o.close()
    for name, env_vars in VARIANTS:
        for kk, vv in env_vars.items():
            os.environ[kk] = vv
        r = mpt.GPURenderer(0)
        r.set_scene(city)
        r.set_luts(luts)
        r.set_envmap(env)
        first_bad = None
        for k in range(n if prefix else 0):
            r.render_samples(frs[k:k + 1])
            r.synchronize_kernel()
            g = r.framebuffer(abi.FB_COLOR)
            bad = np.argwhere(g != refs[k])
            if len(bad) and first_bad is None:
                first_bad = (k, len(bad), bad[0].tolist(), float(g[tuple(bad[0])]), float(refs[k][tuple(bad[0])]))
        r.close()
        # the same frames as one render_samples call (batched ReSTIR DI unless switched off)
        r = mpt.GPURenderer(0)
        r.set_scene(city)
        r.set_luts(luts)
        r.set_envmap(env)
        r.render_samples(frs)
        r.synchronize_kernel()
        whole = int((r.framebuffer(abi.FB_COLOR) != refs[-1]).sum())
        r.close()
        print(f"{name:16s} one call: {whole} values differ", flush=True)
        for kk in env_vars:
            del os.environ[kk]
        print(f"{name:16s} first divergence (sample, values, pixel, gpu, oracle): {first_bad}", flush=True)


if __name__ == "__main__":
    main()
