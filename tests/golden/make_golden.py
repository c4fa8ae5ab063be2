"""Regenerates the fixtures of tests/golden.

* rng_kat.json -- Xorshift32 / wang_hash known answers, computed by the pure-Python
  restatement of HostDeviceCommon/Xorshift.h:40-52 and Device/includes/Hash.h:11-19
  (the seed 42 sequence is also the one CPURenderer.cpp:90,284 produces).
* cornell_32x18_mis_2spp.npz -- the CPU oracle's Cornell image (regression fixture of
  the restated algorithm; not a reference output -- see DESIGN.md "parity unpinned").
* c1_cornell_256_lambert_1spp.npz -- the oracle's whole C1 frame (BASELINE.json config 1:
  Cornell 256x256, 1 spp, Lambert override, RIS, 3 bounces; tests/test_configs.py).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    from test_oracle import xorshift32_py, wang_hash_py, _frames
    kat = {"xorshift32": {str(s): xorshift32_py(s, 16) for s in (42, 1, 0xDEADBEEF, 123456789)},
           "wang_hash": {str(s): wang_hash_py(s) for s in (0, 1, 42, 1000, 0xFFFFFFFF, 2073600 * 65)}}
    json.dump(kat, open(os.path.join(HERE, "rng_kat.json"), "w"), indent=1)
    from mpt import scene
    from oracle import oracle as orc
    sd = scene.load_scene("cornell_pbr")
    o = orc.Oracle(sd, scene.load_luts())
    img, alb, nrm = o.render(_frames(sd, 32, 18, 2), aov=True)
    np.savez_compressed(os.path.join(HERE, "cornell_32x18_mis_2spp.npz"), color=img, albedo=alb, normals=nrm)
    from test_configs import c1_frames
    img, alb, nrm = o.render(c1_frames(sd), aov=True)
    np.savez_compressed(os.path.join(HERE, "c1_cornell_256_lambert_1spp.npz"), color=img, albedo=alb, normals=nrm)
    print("ok")


if __name__ == "__main__":
    main()
