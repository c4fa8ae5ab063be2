"""Development probe (GPU box): the C4 frame (city + sky, ReSTIR DI, 1080p) rendered with
variants of the ReSTIR DI settings, printing the per-pass times (live HIP events) so that a
pass's cost can be attributed to its neighbour reads.
usage: python tools/restir_probe.py [spp]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))

import mpt  # noqa: E402
from mpt import abi, scene, synthetic  # noqa: E402

VARIANTS = {
    "default": {},
    "no_rotation": dict(do_neighbor_rotation=False),
    "radius_4": dict(reuse_radius=4),
    "one_neighbour": dict(reuse_neighbor_count=1),
    "no_boost": dict(do_disocclusion_reuse_boost=False),
}


def frames(city, n, rd):
    cam = scene.make_camera(city.camera_info, 1920, 1080)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RESTIR_DI
    out = []
    for d in scene.gpu_seed_schedule(n, 2, fused=True):
        st = scene.parity_settings(3)
        st.do_alpha_testing = True
        for k, v in rd.items():
            setattr(st.restir_di_settings, k, v)
        out.append(scene.make_frame(cam, 1920, 1080, options=opt, settings=st, world=scene.envmap_world(1.0),
                                    sample_number=d["sample_number"], random_seed=d["random_seed"],
                                    camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"]))
    return out


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    city = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(2048, 1024, seed=7))
    luts = scene.load_luts()
    names = ["gbuffer", "presample", "initial", "temporal", "spatial"]
    for name, rd in VARIANTS.items():
        r = mpt.GPURenderer(0)
        r.set_scene(city)
        r.set_luts(luts)
        r.set_envmap(env)
        frs = frames(city, spp + 2, rd)
        r.render_samples(frs[:2])
        r.synchronize_kernel()
        r.enable_stats(timing=True, instrumented=False)
        t0 = time.perf_counter()
        r.render_samples(frs[2:])
        r.synchronize_kernel()
        dt = (time.perf_counter() - t0) * 1e3 / spp
        st = r.stats()
        passes = " ".join(f"{names[k]} {st.restir_kernel_ms[k] / spp:.3f}" for k in range(5))
        print(f"{name:14s} {dt:7.3f} ms/spp | {passes}", flush=True)
        if name == "default":
            import numpy as np
            for kind, what in ((abi.AUX_RESTIR_INITIAL, "initial"), (abi.AUX_RESTIR_OTHER, "fused out"),
                               (abi.AUX_RESTIR_OUTPUT, "spatial out")):
                res = r.aux_buffer(kind)
                M = res[..., 0].view(np.int32).ravel()
                ucw = res[..., 2].ravel()
                hist = np.bincount(np.clip(M, 0, 30), minlength=31)
                print(f"  {what:12s} M: mean {M.mean():.2f}  <=1: {(M <= 1).mean():.3f}  hist {hist[:8].tolist()} ... 25+: {hist[25:].sum()}"
                      f"  UCW>0: {(ucw > 0).mean():.3f}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
