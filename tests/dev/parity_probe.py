"""Development: count GPU-vs-oracle mismatches on the city stand-in under option variants."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
import mpt  # noqa: E402
from mpt import abi, scene, synthetic  # noqa: E402
from oracle import oracle as orc  # noqa: E402

sd = synthetic.procedural_city(1234)
luts = scene.load_luts()
env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
r = mpt.GPURenderer(0)
r.set_scene(sd)
r.set_luts(luts)
r.set_envmap(env)
o = orc.Oracle(sd, luts, envmap=env)
W, H = 1920, 1080
band = (8, 5, 48)
cam = scene.make_camera(sd.camera_info, W, H)
LSS = {"ris": abi.LSS_RIS_BSDF_AND_LIGHT, "mis": abi.LSS_MIS_LIGHT_BSDF, "uniform": abi.LSS_UNIFORM_ONE_LIGHT,
       "bsdf": abi.LSS_BSDF, "none": abi.LSS_NO_DIRECT_LIGHT_SAMPLING}
for name in sys.argv[1:]:
    lss, envmode = name.split(":")
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = LSS[lss]
    world = scene.envmap_world(1.0)
    if envmode == "noenv":
        world = abi.WorldSettings.default()
    elif envmode == "nosample":
        opt.envmap_sampling = abi.ESS_NO_SAMPLING
    elif envmode == "nomis":
        opt.envmap_bsdf_mis = 0
    frs = [scene.make_frame(cam, W, H, options=opt, world=world, sample_number=s, random_seed=seed, band=band)
           for s, seed in scene.cpu_seed_schedule(2)]
    for f in frs:
        r.render(f)
    r.synchronize_kernel()
    g = r.framebuffer(abi.FB_COLOR)
    c = o.render(frs)
    bad = np.argwhere(np.any(g != c, axis=-1))
    print(name, "differing pixels:", len(bad), bad[:4].tolist(),
          [(g[tuple(b)].tolist(), c[tuple(b)].tolist()) for b in bad[:2]], flush=True)
