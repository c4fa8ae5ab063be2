"""Development: per-vertex envmap-NEE trace of one pixel, GPU (printf variant library) vs oracle."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
row, x, lssn = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
W, H = 1920, 1080
band = (8, 5, 48)
y = ((row // 8) * 48 + 5) * 8 + row % 8
slot = row * W + x
os.environ["ORACLE_DBG_PIX"] = str(x + y * W)
from mpt import _build  # noqa: E402
from pathlib import Path  # noqa: E402
variant = Path(ROOT) / "dbg" / f"s{slot}" / "libmpt.so"
if not variant.exists():
    _build.build(defines=[f"-DMPT_DEBUG_SLOT={slot}"], out=variant, verbose=False)
os.environ["MPT_LIB_PATH"] = str(variant)
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
cam = scene.make_camera(sd.camera_info, W, H)
LSS = {"ris": abi.LSS_RIS_BSDF_AND_LIGHT, "mis": abi.LSS_MIS_LIGHT_BSDF, "uniform": abi.LSS_UNIFORM_ONE_LIGHT}
opt = abi.KernelOptions.default()
opt.direct_light_sampling = LSS[lssn]
opt.envmap_bsdf_mis = 0
frs = [scene.make_frame(cam, W, H, options=opt, world=scene.envmap_world(1.0), sample_number=s, random_seed=seed, band=band)
       for s, seed in scene.cpu_seed_schedule(2)]
for f in frs:
    r.render(f)
    r.synchronize_kernel()
    print("---- GPU frame done", flush=True)
g = r.framebuffer(abi.FB_COLOR)
sys.stdout.flush()
c = o.render(frs)
sys.stdout.flush()
print("pixel gpu", g[row, x].tolist(), "oracle", c[row, x].tolist())
