"""Development probe (GPU box): GPU vs oracle mismatch counts for variants of one ReSTIR DI
test case (tests/test_restir.py frames), to localise a parity difference to a pass.
usage: python tools/restir_diff_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import mpt  # noqa: E402
from mpt import abi, scene  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_restir import frames  # noqa: E402

VARIANTS = {
    "seven": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7),
    "seven_1frame": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7, n=1),
    "seven_2frames": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7, n=2),
    "seven_no_temporal": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7, do_temporal_reuse_pass=False),
    "seven_unfused": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7, do_fused_spatiotemporal=False),
    "seven_one_pass": dict(reuse_neighbor_count=7, disocclusion_reuse_count=7, passes=1),
    "six": dict(reuse_neighbor_count=6, disocclusion_reuse_count=6),
    "five": dict(reuse_neighbor_count=5, disocclusion_reuse_count=5),
}


def main():
    sd = scene.load_scene("cornell_pbr")
    luts = scene.load_luts()
    for name, kw in VARIANTS.items():
        kw = dict(kw)
        n = kw.pop("n", 5)
        frs = frames(sd, abi.LSS_RESTIR_DI, n, **kw)
        r = mpt.GPURenderer(0)
        r.set_scene(sd)
        r.set_luts(luts)
        for f in frs:
            r.render(f)
        r.synchronize_kernel()
        g = r.framebuffer(abi.FB_COLOR)
        r.close()
        o = orc.Oracle(sd, luts)
        c = o.render(frs)
        o.close()
        print(f"{name:20s} differ {int((g != c).sum())} of {g.size}", flush=True)


if __name__ == "__main__":
    main()
