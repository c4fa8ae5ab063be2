"""ms/spp of C3 / C4 at the reference's adaptive-sampling defaults (RenderSettings.h:126-133:
enable_adaptive_sampling, adaptive_sampling_min_samples 64, noise threshold 0.3) against the same
frames with adaptive sampling off, segment by segment over 256 spp.

Adaptive sampling stops tracing a pixel once it has converged: batched path-tracing wavefronts
leave such pixels out of their camera queues (k_camera's spec_skip), so the per-segment time
should fall as pixels converge; under ReSTIR DI the samples up to the minimum run as batched
wavefronts (the gate is static there) and the later ones one by one.
usage (GPU box): python tools/adaptive_curve.py [c3|c4] [spp] [segment] > out.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mpt  # noqa: E402
from mpt import abi, scene, synthetic  # noqa: E402


def frames(cam, W, H, opt, n, adaptive, restir):
    out = []
    sched = (scene.gpu_seed_schedule(n, 2) if restir else
             [dict(sample_number=s, random_seed=seed) for s, seed in scene.cpu_seed_schedule(n)])
    for d in sched:
        st = scene.parity_settings(3)
        st.do_alpha_testing = True
        st.enable_adaptive_sampling = adaptive
        st.adaptive_sampling_min_samples = 64
        st.adaptive_sampling_noise_threshold = 0.3
        kw = dict(camera_random_seed=d["camera_random_seed"], restir_di_seeds=d["restir_di_seeds"]) if restir else {}
        out.append(scene.make_frame(cam, W, H, options=opt, settings=st, world=scene.envmap_world(1.0),
                                    sample_number=d["sample_number"], random_seed=d["random_seed"], **kw))
    return out


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    seg = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    restir = wl == "c4"
    W, H = 1920, 1080
    sd = synthetic.procedural_city(1234)
    env = mpt.build_envmap(scene.procedural_sky(2048, 1024, seed=7))
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_RESTIR_DI if restir else abi.LSS_RIS_BSDF_AND_LIGHT
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(scene.load_luts())
    r.set_envmap(env)
    res = {"workload": wl, "spp": spp, "segment": seg, "width": W, "height": H,
           "settings": "enable_adaptive_sampling, min samples 64, noise threshold 0.3 (RenderSettings.h:126-133)",
           "libmpt_sha256_16": mpt.build_id(), "runs": {}}
    for mode in ("off", "adaptive"):
        frs = frames(cam, W, H, opt, spp, mode == "adaptive", restir)
        r.render_samples(frs[:4])            # warm-up (allocations), then restart at sample 0
        r.synchronize_kernel()
        segs = []
        for s0 in range(0, spp, seg):
            t0 = time.perf_counter()
            r.render_samples(frs[s0:s0 + seg])
            r.synchronize_kernel()
            dt = time.perf_counter() - t0
            conv = r.aux_buffer(abi.AUX_CONVERGED_SAMPLE_COUNT) if mode == "adaptive" else None
            segs.append({"samples": f"{s0}-{s0 + seg - 1}", "ms_per_spp": round(dt * 1e3 / seg, 4),
                         "converged_fraction": round(float((conv >= 0).mean()), 4) if conv is not None else None})
            print(json.dumps({"mode": mode, **segs[-1]}), file=sys.stderr, flush=True)
        res["runs"][mode] = {"segments": segs, "ms_per_spp_total": round(sum(x["ms_per_spp"] for x in segs) / len(segs), 4)}
    r.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
