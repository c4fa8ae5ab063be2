"""C4 (ReSTIR DI on the Bistro stand-in, 1920x1080) rendered as N contiguous bands on ONE
GPU (N contexts, one host thread each, in-process halo exchange): checks the assembled
frame against a single-context render bit for bit and reports the halo the bands agreed
on (the measured reprojection offset + reuse radius) and the rows exchanged per frame --
the inputs for the multi-GPU C4 estimate in DESIGN.md.  usage: tools/restir_bands_probe.py [N] [frames]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)
import mpt  # noqa: E402
from mpt import abi, partition, scene, synthetic  # noqa: E402
import bench  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    nfr = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    W, H = 1920, 1080
    sd = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(2048, 1024, seed=7))
    wset = scene.envmap_world(1.0)
    luts = scene.load_luts()
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RESTIR_DI

    def mk():
        r = mpt.GPURenderer(0)
        r.set_scene(sd)
        r.set_luts(luts)
        r.set_envmap(env)
        return r

    r = mk()
    t0 = time.perf_counter()
    for f in bench.frames_for(cam, W, H, opt, (1, 0, 1), nfr, alpha=True, world=wset):
        r.render(f)
    r.synchronize_kernel()
    t_single = time.perf_counter() - t0
    ref = r.framebuffer(abi.FB_COLOR)
    r.close()

    bh = partition.contiguous_band(H, nb, 0)[0]
    group = partition.LocalHaloGroup(bh, nb)
    halos = []
    rs = [mk() for _ in range(nb)]
    for k, rr in enumerate(rs):
        m = group.member(k)

        def ex(x, m=m, k=k):
            m(x)
            if k == 0 and x.phase == abi.HALO_GBUFFER:
                halos.append(x.halo_rows)
        rr.set_halo_exchange(ex)
    errs = []

    def run(k):
        try:
            for f in bench.frames_for(cam, W, H, opt, partition.contiguous_band(H, nb, k), nfr, alpha=True, world=wset):
                rs[k].render(f)
            rs[k].synchronize_kernel()
        except BaseException as e:
            errs.append(e)
            group.barrier.abort()
    th = [threading.Thread(target=run, args=(k,)) for k in range(nb)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    t_bands = time.perf_counter() - t0
    if errs:
        raise errs[0]
    got = np.concatenate([rr.framebuffer(abi.FB_COLOR) for rr in rs])
    for rr in rs:
        rr.close()
    same = np.array_equal(got, ref)
    print(f"bands={nb} band_height={bh} frames={nfr} bit_exact={same} differing={int((got != ref).sum())} "
          f"agreed_halo_rows_per_frame={halos} single_s={t_single:.2f} bands_on_one_gpu_s={t_bands:.2f}")
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
