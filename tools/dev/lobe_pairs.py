"""Dev probe: which pair of lobes (with transmission) breaks bit-exactness."""
import copy
import itertools
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "hiprt-path-tracer_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import mpt
from mpt import abi, scene
from oracle import oracle as orc
import test_lobes as T

C = T.C
parts = dict(coat=dict(coat=0.5, coat_roughness=0.3), sheen=dict(sheen=0.5, sheen_roughness=0.4), metal=dict(metallic=0.3),
             tr=dict(specular_transmission=0.2), film=dict(thin_film=0.5, thin_film_thickness=380.0), aniso=dict(anisotropy=0.3),
             tint=dict(specular_tint=0.3, specular_color=C(0.7, 0.9, 1.0)))
cor = scene.load_scene("cornell_pbr")
luts = scene.load_luts()
r = mpt.GPURenderer(0)
r.set_scene(cor)
r.set_luts(luts)
combos = [("tr", k) for k in parts if k != "tr"] + [("all",)] + [tuple(k for k in parts if k != x) for x in parts]
for combo in combos:
    kw = {}
    for k in (parts if combo == ("all",) else combo):
        kw.update(parts[k])
    T.LOBES["probe"] = {T.WALLS: kw}
    mats = T.lobe_materials(cor, "probe")
    for lss in (abi.LSS_MIS_LIGHT_BSDF, abi.LSS_RIS_BSDF_AND_LIGHT):
        frs = T.frames(cor, lss, n=4, w=64, h=48)
        r.update_materials(mats)
        got = T._render(r, frs)
        sd = copy.copy(cor)
        sd.materials = mats
        o = orc.Oracle(sd, luts)
        ref = o.render(frs, aov=True)
        o.close()
        bad = ~((got[0] == ref[0]) | (np.isnan(got[0]) & np.isnan(ref[0])))
        idx = np.argwhere(bad.any(-1))
        print(combo, lss, int(bad.sum()), idx[:4].tolist(), flush=True)
