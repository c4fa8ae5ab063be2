"""Probe: batched city render step by step (diagnosing a crash)."""
import faulthandler
import sys
faulthandler.enable()
sys.path.insert(0, "hiprt-path-tracer_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import mpt
from mpt import scene, synthetic, abi
import test_gpu_parity as t

city = synthetic.procedural_city(1234)
luts = scene.load_luts()
env = mpt.build_envmap(scene.procedural_sky(512, 256, seed=7))
mode = sys.argv[1]
band = (8, 7, 48)
frs = t.frames(city, 1920, 1080, 3, lss=abi.LSS_RIS_BSDF_AND_LIGHT, world=scene.envmap_world(1.0), band=band)
for f in frs:
    f.render_settings.do_alpha_testing = mode != "noalpha"
r = mpt.GPURenderer(0)
r.set_scene(city); r.set_luts(luts); r.set_envmap(env)
print("scene set", flush=True)
if mode == "seq":
    for f in frs:
        r.render(f)
else:
    r.render_samples(frs, max_batch=3)
print("enqueued", flush=True)
r.synchronize_kernel()
print("synced", flush=True)
img = r.framebuffer(abi.FB_COLOR)
print("mean", float(img.mean()), flush=True)
from oracle import oracle as orc
ref = orc.Oracle(city, luts, envmap=env).render(frs)
print("bit-exact", bool(np.array_equal(img, ref)), flush=True)
