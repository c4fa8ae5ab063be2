"""Development: any-hit queries starting exactly on surfaces (the envmap shadow rays)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
import mpt  # noqa: E402
from mpt import scene, synthetic  # noqa: E402
from oracle import oracle as orc  # noqa: E402

sd = synthetic.procedural_city(1234)
luts = scene.load_luts()
r = mpt.GPURenderer(0)
r.set_scene(sd)
r.set_luts(luts)
o = orc.Oracle(sd, luts)
rng = np.random.default_rng(3)
n = 2_000_000
cam = np.array(sd.camera_info["position"], np.float32)
d = rng.normal(size=(n, 3))
d[:, 1] = -np.abs(d[:, 1]) * 0.3
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.zeros((n, 8), np.float32)
rays[:, 0:3] = cam + rng.normal(size=(n, 3)).astype(np.float32) * np.float32(5.0)
rays[:, 1] = np.abs(rays[:, 1]) + 1.0
rays[:, 4:7] = d
rays[:, 7] = 1e30
p, t, _, _ = o.trace_closest(rays)
hit = p >= 0
print("primary hits", hit.mean())
o2 = np.zeros((hit.sum(), 8), np.float32)
ip = (rays[hit, 0:3] + t[hit, None] * rays[hit, 4:7]).astype(np.float32)
d2 = rng.normal(size=(hit.sum(), 3))
d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
o2[:, 0:3] = ip
o2[:, 4:7] = d2
o2[:, 7] = np.float32(1e35) - np.float32(1e-4)
lh = p[hit].astype(np.int32)
occ = r.trace_any(o2, lh)
p2, t2, _, _ = o.trace_closest(o2, lh)
exp = (p2 >= 0) & (t2 < o2[:, 7] - np.float32(1e-4))
bad = np.flatnonzero(occ != exp)
print("surface-origin any-hit mismatches:", len(bad), "of", len(occ))
for i in bad[:5]:
    gp, gt, _, _ = r.trace_closest(o2[i:i + 1], lh[i:i + 1])
    print(" ray", o2[i].tolist(), "last", int(lh[i]), "gpu occ", bool(occ[i]), "oracle closest", int(p2[i]), float(t2[i]),
          "gpu closest", int(gp[0]), float(gt[0]))
