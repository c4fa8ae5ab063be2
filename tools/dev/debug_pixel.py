"""Dev probe: per-bounce trace of one pixel, GPU (debug build, MPT_DEBUG_SLOT) vs oracle (ORACLE_DBG_PIX).
usage: MPT_LIB_PATH=<debug lib> ORACLE_DBG_PIX=<pixel> python tests/dev/debug_pixel.py <case> <lss>"""
import copy
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "hiprt-path-tracer_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import mpt
from mpt import abi, scene
from oracle import oracle as orc
import test_lobes as T

case, lss = sys.argv[1], int(sys.argv[2])
pix = int(os.environ["ORACLE_DBG_PIX"])
cor = scene.load_scene("cornell_pbr")
luts = scene.load_luts()
mats = T.lobe_materials(cor, case)
frs = T.frames(cor, lss)
r = mpt.GPURenderer(0)
r.set_scene(cor)
r.set_luts(luts)
r.update_materials(mats)
for k, f in enumerate(frs):
    print(f"=== frame {k} GPU", flush=True)
    r.render(f)
    r.synchronize_kernel()
sys.stdout.flush()
g = r.framebuffer(abi.FB_COLOR)
sd = copy.copy(cor)
sd.materials = mats
o = orc.Oracle(sd, luts)
for k in range(len(frs)):
    print(f"=== frame {k} CPU", flush=True)
    ref = o.render(frs[:k + 1], nthreads=1)
    sys.stdout.flush()
W = frs[0].res_x
print("GPU", g.reshape(-1, 3)[pix].tolist(), "CPU", ref.reshape(-1, 3)[pix].tolist())
