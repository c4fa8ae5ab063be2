"""Development: k_shade section cycle breakdown (needs a -DMPT_SECTION_TIMING libmpt via MPT_LIB_PATH)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
import mpt  # noqa: E402
from mpt import abi, scene  # noqa: E402

W, H = 1920, 1080
bsdf = sys.argv[1] if len(sys.argv) > 1 else "principled"
wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
env = None
if wl == "c3":
    from mpt import synthetic
    sd = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(2048, 1024, seed=7))
else:
    sd = scene.load_scene("cornell_pbr")
r = mpt.GPURenderer(0)
r.set_scene(sd)
r.set_luts()
if env is not None:
    r.set_envmap(env)
cam = scene.make_camera(sd.camera_info, W, H)
opt = abi.KernelOptions.default()
opt.bsdf_override = abi.BSDF_NONE if bsdf == "principled" else abi.BSDF_LAMBERTIAN
opt.direct_light_sampling = abi.LSS_MIS_LIGHT_BSDF if wl == "c2" else abi.LSS_RIS_BSDF_AND_LIGHT
world = scene.envmap_world(1.0) if env is not None else None
L = mpt.lib()
L.mpt_debug_sections.argtypes = [C.c_void_p, C.c_int]
out = np.zeros(8, np.uint64)
for f in [scene.make_frame(cam, W, H, options=opt, world=world, sample_number=s, random_seed=seed) for s, seed in scene.cpu_seed_schedule(2)]:
    r.render(f)
r.synchronize_kernel()
L.mpt_debug_sections(out.ctypes.data, 1)
for f in [scene.make_frame(cam, W, H, options=opt, world=world, sample_number=s, random_seed=seed) for s, seed in scene.cpu_seed_schedule(8)]:
    r.render(f)
r.synchronize_kernel()
L.mpt_debug_sections(out.ctypes.data, 1)
tot = out[:6].sum()
names = ["hit processing", "op pre (sampling)", "BSDF eval post", "op post", "finish/stores", "BSDF eval pre"]
for k in range(6):
    print(f"{names[k]:20s} {out[k] / tot * 100:6.2f}%   {out[k] / 8 / 64:.3e} wave-cycles/frame")
