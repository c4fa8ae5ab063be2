"""Benchmark of the MI355X path tracer (libmpt) -- one JSON line on rank 0.

Workloads (BASELINE.json configs):
* c3 (default; the configuration the metric is quoted on): the Bistro-exterior
  stand-in -- a seeded procedural city of 2.86 M triangles with alpha-tested leaf cards
  (mpt/synthetic.py, seed 1234) under a seeded procedural HDR sky (2048x1024, alias-table
  sampling + BSDF MIS), 1920x1080, layered Principled BSDF, reference-default RIS light
  sampling, alpha testing on (C3 pins it for the foliage); K = 256.
* c2: the Cornell box glTF at 1920x1080, Principled + NEE/MIS (LSS_MIS_LIGHT_BSDF); K = 64.
* c3t: c3 on the texture-realistic city (synthetic.procedural_city_textured: 70 materials, 83 % of
  the triangles with base-colour + normal-map + roughness-metallic textures, 193 MB of textures),
  so that the shading roofline is measured where texture gathers and per-vertex resolved
  materials cost something.
* c4: c3 with ReSTIR DI (fused spatiotemporal + spatial reuse), GPURenderer seed schedule.
* c5: the glass-dispersion stress scene (multi-dispersion.gltf; --scene
  nested-dielectrics-complex for the nested-dielectrics one) at 3840x2160, 16 bounces,
  Principled + RIS, K = 1024.
* c1: the Cornell box at 256x256, 1 spp, Lambert override (BSDFOverride = BSDF_LAMBERTIAN),
  reference-default RIS: the configuration BASELINE.json quotes for the CPU megakernel; the
  line's cpu_baseline is the oracle over the whole C1 frame, its parity the whole frame.
All: 3 bounces unless stated, reference defaults otherwise (adaptive sampling off so that every step
samples every pixel).  One *step* = one sample per pixel over the frame (one
mpt_render_frame); K steps = the config's spp.  Multi-GPU: one process per GPU, the framebuffer is split into
interleaved 8-row bands (each rank renders every N-th band), and the per-rank sum
buffers are gathered with RCCL (all_gather over xGMI) inside the timed region.

value = whole-job Mray/s (every closest + any-hit query: camera, continuation, NEE
shadow, MIS BSDF ray) = rays of all ranks / max-over-ranks wall time.
roofline: the kernel with the largest HIP-event time in the timed region among the
traversal stages (SURVEY.md §8d B_ray = 32 + 16 + 80 N_node + 48 N_tri, N counted by an
instrumented calibration pass), the shading kernel (556 B per path vertex) and the ReSTIR DI
kernels (bytes per pixel); achieved = units per launch x bytes per unit / the
average launch time.  roofline_traversal adds the traversal's VALU issue rate and the PMC
HBM fraction from the committed profile of the same command (profiles/).
cpu_baseline: the CPU oracle (a port, test infrastructure) on a bounded sample of the same
frame, on every core the process may use (cores stated).
parity_vs_oracle: the GPU's 256-spp radiance against the oracle on one 8-row band (the
metric's "RMSE vs ref @256spp"); C4 (ReSTIR DI reuses the whole frame): whole frames, as
many as the oracle renders in its budget; C1: the whole frame at K spp.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))

import mpt  # noqa: E402
from mpt import abi, scene  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0
VALU_PEAK = 256 * 4 * 2.4e9 / 2    # wave64 VALU instructions / s (MI355X_MICROARCH.md: 2 cycles per wave instruction)
S_NODE, S_TRI = 80, 48
BAND_H = 8
TARGET_PATHS = 64 * 1920 * 1080  # paths per wavefront launch (mpt_render_frames batch x rank pixels)
# ReSTIR DI (C4): smaller wavefronts, so that each batch's later bounces overlap the next batch's
# per-sample reuse chain (C4 at 64 steps: batch 16 / 32 / 64 -> 8.09-8.12 / 8.17 / 8.33 ms/spp,
# profiles/r06ae_c4_batch_ab.json; at 32 steps 8 / 16 -> 8.10 / 8.22, at 8 steps 4 / 8 -> 8.44 / 8.56,
# r06as_c4_batch_ab.json; the path-tracing configs gain from larger ones: C3 16 / 32 / 64 ->
# 3.92 / 3.86 / 3.77, profiles/r06ab_c3_batch_ab.json)
TARGET_PATHS_RESTIR = 8 * 1920 * 1080
MAX_BATCH = 128    # MPT_MAX_BATCH


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", default="c3", choices=["c1", "c2", "c3", "c3t", "c4", "c5"])
    ap.add_argument("--steps", type=int, default=None, help="default: the workload's spp (c3/c4 256, c2 64, c5 1024, c1 1)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=None, help="default 1920 (c5: 3840)")
    ap.add_argument("--height", type=int, default=None, help="default 1080 (c5: 2160)")
    ap.add_argument("--scene", default=None, help="c2: a glTF of data/scenes (default cornell_pbr)")
    ap.add_argument("--strategy", default=None, choices=["mis", "ris", "uniform", "bsdf", "restir"],
                    help="default: c3 ris (reference default), c2 mis")
    ap.add_argument("--bounces", type=int, default=None, help="default 3 (c5: 16)")
    ap.add_argument("--bsdf", default="principled", choices=["principled", "lambert"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-baseline sample duration")
    ap.add_argument("--parity-spp", type=int, default=256, help="spp of the RMSE-vs-oracle band (the metric's 256)")
    ap.add_argument("--parity-seconds", type=float, default=90.0, help="oracle budget of the parity leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the RMSE-vs-oracle band check")
    ap.add_argument("--no-solo", action="store_true",
                    help="skip the pipelined shading kernel's solo timing after the timed region")
    ap.add_argument("--batch", type=int, default=0,
                    help="samples per pixel traced as one wavefront (mpt_render_frames); 0 = auto: "
                         "TARGET_PATHS / the rank's pixels, so a rank's launches keep the same size")
    ap.add_argument("--configs", default="all",
                    help="after the headline workload, the other BASELINE configs at reduced budgets in the same "
                         "line ('all' = c1,c2,c4,c5; a comma list; 'none')")
    ap.add_argument("--config-steps", type=int, default=8, help="timed steps of each extra config")
    ap.add_argument("--batch1-steps", type=int, default=8,
                    help="C3: steps also timed with one sample per wavefront (mpt_render_frame's launch set; 0 = skip)")
    ap.add_argument("--halo", default="auto", choices=["auto", "native", "python"],
                    help="C4 across ranks: the library's RCCL halo exchange (mpt_set_halo_native; the one-GPU "
                         "rehearsal: its local stand-in) or the Python callback (mpt.partition.TorchHaloExchange); "
                         "auto: the Python callback over torch.distributed for world > 1 (the library's RCCL exchange "
                         "needs the 2-GPU test tests/test_halo_native.py, which a one-GPU box skips), the native "
                         "rehearsal for --emulate-rank-of")
    ap.add_argument("--emulate-band", type=int, default=-1,
                    help="C4 rehearsal: time only this rank's band (default: every band in turn)")
    ap.add_argument("--emulate-rank-of", type=int, default=1,
                    help="scaling rehearsal on one GPU: render only rank 0's share of an N-way row split "
                         "(the line then reports that rank's rate; not a bench line)")
    return ap.parse_args()


LSS = {"mis": abi.LSS_MIS_LIGHT_BSDF, "ris": abi.LSS_RIS_BSDF_AND_LIGHT, "uniform": abi.LSS_UNIFORM_ONE_LIGHT,
       "bsdf": abi.LSS_BSDF, "restir": abi.LSS_RESTIR_DI}


def frames_for(cam, W, H, opt, band, n, first=0, bounces=3, world=None, alpha=False):
    out = []
    if opt.direct_light_sampling == abi.LSS_RESTIR_DI:
        # GPURenderer's seed schedule: camera, ReSTIR passes, path tracing per sample
        for d in scene.gpu_seed_schedule(n, 2, first_sample=first):
            st = scene.parity_settings(bounces)
            st.do_alpha_testing = alpha
            out.append(scene.make_frame(cam, W, H, options=opt, settings=st, world=world, sample_number=d["sample_number"],
                                        random_seed=d["random_seed"], camera_random_seed=d["camera_random_seed"],
                                        restir_di_seeds=d["restir_di_seeds"], band=band))
        return out
    for s, seed in scene.cpu_seed_schedule(n):
        st = scene.parity_settings(bounces)
        st.do_alpha_testing = alpha
        out.append(scene.make_frame(cam, W, H, options=opt, settings=st, world=world, sample_number=s + first,
                                    random_seed=seed, band=band))
    return out


def host_cores():
    """CPU threads the oracle may run on here: the process's CPU affinity, capped by the
    cgroup CPU quota when one is set (the GPU box grants a share of a larger machine), or
    OMP_NUM_THREADS when the harness pins it.  Returns (threads, nproc, how)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    n, how = aff, "affinity"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
            if quota < n:
                n, how = quota, "cgroup quota"
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if 0 < omp < n:
        n, how = omp, "OMP_NUM_THREADS"
    return n, nproc, how


def cpu_baseline(sd, luts, cam, W, H, opt, bounces, target_s, env=None, world=None, alpha=False):
    """Oracle (CPU port) timed on a bounded sample of the same frame: a subset of the
    8-row bands at 1 spp, or the whole frame at several spp, sized to ~target_s.  ReSTIR DI
    reuses the whole frame, so C4 times whole frames."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    cores, nproc, how = host_cores()
    o = orc.Oracle(sd, luts, envmap=env)
    restir = opt.direct_light_sampling == abi.LSS_RESTIR_DI
    bc = 1 if restir else 64
    t0 = time.perf_counter()
    o.render(frames_for(cam, W, H, opt, (BAND_H, 0, bc), 1, bounces=bounces, world=world, alpha=alpha), nthreads=cores)
    dt = max(time.perf_counter() - t0, 1e-3)
    scale = target_s / dt                       # multiples of the probe's work
    if scale >= bc:                             # whole frame, several spp
        bc2, spp = 1, max(1, int(round(scale / bc)))
    else:
        bc2, spp = max(1, int(round(bc / scale))), 1
    if restir:
        bc2, spp = 1, max(1, min(8, int(scale)))
    t0 = time.perf_counter()
    o.render(frames_for(cam, W, H, opt, (BAND_H, 0, bc2), spp, bounces=bounces, world=world, alpha=alpha),
             nthreads=cores)
    dt = time.perf_counter() - t0
    rows = orc.mpt_rows(H, BAND_H, 0, bc2)
    rays = o.last_rays[0] + o.last_rays[1]
    o.close()
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mray/s", "cores": cores, "kind": "port",
            "host_cpus": nproc, "cores_from": how,
            "msample_per_s": round(rows * W * spp / dt / 1e6, 5),
            "sample": f"oracle (C++ CPU port, OpenMP, {cores} threads = the host cores this process may use "
                      f"({how}; the machine reports {nproc})): {spp} spp over {rows} of {H} rows "
                      f"({BAND_H}-row bands, 1 of every {bc2}) of the same {W}x{H} frame, {dt:.1f} s"}


def parity_check(r, sd, luts, cam, W, H, opt, bounces, spp, workload, env=None, world=None, alpha=False,
                 max_s=90.0, batch=0, history=None):
    """RMSE of the GPU's spp-sample radiance (sum / spp) against the CPU oracle on the same
    frames (the metric's "RMSE vs ref @256spp"; the oracle is the pinned CPU restatement,
    DESIGN.md §2), through the same batched path as the timed region.  Region: one 8-row
    band through the middle of the frame; C1 the whole frame; C4 whole frames (ReSTIR DI
    reuses neighbours across the frame), as many as the oracle renders in max_s.
    ReSTIR DI keeps state across samples: the GPU leg restarts at sample 0 in the TIMED context
    (a GPURenderer::reset in a used context: the timed run's last G-buffer becomes the first
    frame's previous one, GPURenderer.cpp:953-973), and the oracle starts from the same state:
    the G-buffer the timed frames (`history`) leave (oracle_gbuffer_history)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    cores, _, _ = host_cores()
    restir = opt.direct_light_sampling == abi.LSS_RESTIR_DI
    whole = restir or workload == "c1"
    bc = 1 if whole else H // BAND_H
    bi = 0 if whole else bc // 2
    band = (BAND_H, bi, bc)
    o = orc.Oracle(sd, luts, envmap=env, keep_state=restir)
    t_hist = 0.0
    if restir:
        t0 = time.perf_counter()
        o.gbuffer_history(history, nthreads=cores)
        t_hist = time.perf_counter() - t0
    t0 = time.perf_counter()
    probe = o.render(frames_for(cam, W, H, opt, band, 1, bounces=bounces, world=world, alpha=alpha), nthreads=cores)
    dt1 = max(time.perf_counter() - t0, 1e-4)
    k = spp if dt1 * spp <= max_s else max(1, int(max_s / dt1))
    frs = frames_for(cam, W, H, opt, (BAND_H, 0, 1), k, bounces=bounces, world=world, alpha=alpha)
    if k > 1 and restir:
        o.reset_state()                     # the probe advanced the kept state: back to the timed run's
        o.gbuffer_history(history, nthreads=cores)
    ref = o.render(frames_for(cam, W, H, opt, band, k, bounces=bounces, world=world, alpha=alpha),
                   nthreads=cores) if k > 1 else probe
    o.close()
    r.enable_stats(timing=False, instrumented=False)
    r.render_samples(frs, max_batch=batch)
    r.synchronize_kernel()
    gpu = r.framebuffer(abi.FB_COLOR)
    if not whole:
        gpu = gpu[bi * BAND_H:(bi + 1) * BAND_H]
    d = (gpu.astype(np.float64) - ref.astype(np.float64)) / k
    return {"oracle": "CPU restatement (oracle/, DESIGN.md §2)",
            "rows": "all" if whole else f"{bi * BAND_H}-{(bi + 1) * BAND_H - 1}", "spp": k,
            "rmse": float(np.sqrt(np.mean(d * d))), "max_abs": float(np.abs(d).max()),
            "bit_exact": bool(np.array_equal(gpu, ref)), "tolerance_rmse": 1e-3,
            "context": ("the timed run's (restarted at sample 0; the oracle from the G-buffer of the "
                        f"{len(history)} frames the context rendered, {t_hist:.1f} s)") if restir else "the timed run's",
            "note": (None if k == spp else f"{k} of {spp} spp: the oracle's budget ({max_s:.0f} s) on the whole frame")}


def load_traffic(workload, W, H):
    """HBM bytes per launch from the newest committed PMC summary of this workload
    (profiles/r*_<workload>_pmc_traffic.json, made by tools/profile_round.sh +
    tools/pmc_traffic.py from separate rocprofv3 --pmc passes of this same command).
    PMC counters need rocprofv3 around the process, so they cannot be read live here."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{workload}_pmc_traffic.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    d["file"] = os.path.relpath(files[-1], ROOT)
    return d


def restir_band_want(a, K, want, band_count):
    """Samples per wavefront under ReSTIR DI: TARGET_PATHS_RESTIR paths and at most half the
    samples, so that the run has at least two
    batches and the second one's per-sample reuse chain overlaps the first one's later bounces
    (MPT_RESTIR_OVERLAP; one band of the 8-way 1080p split at the driver's 20 steps: 1.700 ms/spp
    in one batch of 20, 1.677 in two of 10, 1.77 in four of 5, `profiles/r06v_c4_band_batch_ab.json`)"""
    if a.workload != "c4":
        return want
    want = want * TARGET_PATHS_RESTIR / TARGET_PATHS
    if K < 4:
        return want
    return min(want, K // 2)


def emulate_restir_ranks(a, r, cam, W, H, opt, wset, alpha, n_ranks, K, device):
    """C4 scaling rehearsal on one GPU (--workload c4 --emulate-rank-of N): each rank of the
    N-way split renders ONE contiguous band with the halo exchange, so the
    ranks' work differs (sky rows against street rows) and the job's time is the slowest
    rank's.  Every band k is timed in turn in this context: two whole-frame samples first (so
    the frame-sized G-buffer / reservoir buffers hold a single-context render around every
    band), then the band's own warmup + K timed samples, batched as the rank would batch them.
    The halo callback stands in for the exchange: at each exchange point it moves the bytes of
    the halo rows the rank would receive (one device-to-device copy on the library's stream) and,
    when the library could not derive the halo from the frame alone (a moving camera), waits
    for the G-buffer as the RCCL exchange's agreement does; the rows keep the whole-frame
    render's content, so the images are not the partitioned render's (tests/test_configs.py
    pins that bit-exact), only its timing."""
    import torch
    from mpt import partition
    bh = partition.contiguous_band(H, n_ranks, 0)[0]
    stats = {"calls": 0, "bytes": 0}

    def halo(x):
        st = torch.cuda.ExternalStream(x.stream, device=torch.device("cuda", device))
        if x.phase == partition.HALO_GBUFFER and not x.halo_agreed:
            st.synchronize()      # the agreement's all-reduce (TorchHaloExchange.agree) waits for the G-buffer
        _, recvs = partition.halo_plan(x.res_y, bh, n_ranks, cur[0], x.halo_rows)
        # the bytes this rank would receive, moved by ONE device copy (an RCCL exchange is one
        # grouped send / receive kernel per exchange point, not a copy per buffer and range)
        nbytes = sum(x.res_x * x.bytes_per_pixel[i] * (y1 - y0) for i in range(x.n_buffers) for (_, y0, y1) in recvs)
        if nbytes:
            if scratch[0] is None or scratch[0].numel() < 2 * nbytes:
                scratch[0] = torch.empty(2 * nbytes, dtype=torch.uint8, device=torch.device("cuda", device))
            with torch.cuda.stream(st):
                scratch[0][nbytes:2 * nbytes].copy_(scratch[0][:nbytes])
        stats["bytes"] += nbytes
        stats["calls"] += 1

    cur = [0]
    scratch = [None]
    if a.halo == "native":
        r.set_halo_native(2)      # the library's exchange, rehearsal mode: the received bytes moved locally
    else:
        r.set_halo_exchange(halo)
    bands = []
    for k in range(n_ranks):
        if a.emulate_band >= 0 and k != a.emulate_band:
            continue
        cur[0] = k
        band = (bh, k, n_ranks)
        rows = mpt.partition_rows(H, *band)
        if rows == 0:
            continue
        want = a.batch or restir_band_want(a, K, TARGET_PATHS / max(1, rows * W), n_ranks)
        batch = min((d for d in range(1, min(MAX_BATCH, K) + 1) if K % d == 0), key=lambda d: (abs(d - want), -d))
        r.enable_stats(timing=False, instrumented=False)
        r.render_samples(frames_for(cam, W, H, opt, (1, 0, 1), 2, bounces=a.bounces, world=wset, alpha=alpha))
        # the band's warmup: one whole batch, so that the path state is allocated before the timing
        r.render_samples(frames_for(cam, W, H, opt, band, max(a.warmup, 2 * batch), bounces=a.bounces, world=wset,
                                    alpha=alpha), max_batch=batch)
        frames = frames_for(cam, W, H, opt, band, K, bounces=a.bounces, world=wset, alpha=alpha)
        r.synchronize_kernel()
        r.enable_stats(timing=True, instrumented=False)
        c0, b0 = stats["calls"], stats["bytes"]
        t0 = time.perf_counter()
        r.render_samples(frames, max_batch=batch)
        r.synchronize_kernel()
        dt = time.perf_counter() - t0
        st = r.stats()
        bands.append({"band": k, "rows": f"{k * bh}-{min(H, (k + 1) * bh) - 1}", "ms_per_spp": round(dt * 1e3 / K, 4),
                      "batch": batch, "mray_s": round((st.rays_closest + st.rays_any) / dt / 1e6, 2),
                      "restir_ms_per_spp": round(st.restir_ms / K, 4), "shade_ms_per_spp": round(st.shade_ms / K, 4),
                      "trace_path_ms_per_spp": round(st.stage_ms[0] / K, 4),
                      "halo_calls_per_spp": round((stats["calls"] - c0) / K, 2) if a.halo == "python" else None,
                      "halo_mb_per_spp": round((stats["bytes"] - b0) / K / 1e6, 3) if a.halo == "python" else None})
        print(json.dumps(bands[-1]), file=sys.stderr, flush=True)
    worst = max(bands, key=lambda b: b["ms_per_spp"])
    return {"rehearsal": f"C4 ReSTIR DI tile-parallel over {n_ranks} ranks on one GPU: every rank's contiguous band "
                         "timed in turn (halo rows from a single-context render, exchange bytes copied locally)",
            "halo": ("libmpt's native exchange in rehearsal mode (mpt_set_halo_native(2): one device copy of the "
                     "received bytes per exchange point, no host callback)" if a.halo == "native" else
                     "Python callback (one device copy of the received bytes per exchange point)"),
            "emulated_rank_of": n_ranks, "steps": K, "warmup": a.warmup, "width": W, "height": H,
            "ms_per_spp_slowest_rank": worst["ms_per_spp"], "slowest_band": worst["band"],
            "ms_per_spp_mean_rank": round(sum(b["ms_per_spp"] for b in bands) / len(bands), 4),
            "bands": bands, "device": {"libmpt_sha256_16": mpt.build_id()}}


_SCENES = {}


def _cached(key, make):
    """Scenes / envmaps shared by the workloads of one process (C3 and C4 use the same city)."""
    if key not in _SCENES:
        _SCENES[key] = make()
    return _SCENES[key]


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.halo == "auto":
        a.halo = "python" if world > 1 else "native"
    dist = None
    # rehearsal of the N-rank path on a one-GPU box: MPT_BENCH_BACKEND=gloo (host-staged
    # collectives) + MPT_BENCH_SHARE_GPU=1 (every rank on device 0); not a bench line
    backend = os.environ.get("MPT_BENCH_BACKEND", "nccl")
    if os.environ.get("MPT_BENCH_SHARE_GPU"):
        local = 0
    coll_dev = "cuda" if backend == "nccl" else "cpu"
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    out = run_workload(a, world, rank, local, dist, coll_dev)
    if out is not None and world == 1 and a.emulate_rank_of == 1 and a.configs != "none":
        # the other BASELINE configurations in the same line, each at a reduced budget (their
        # own spp would take minutes; a step is still one sample per pixel of the full frame)
        import copy
        extra = ["c1", "c2", "c4", "c5"] if a.configs == "all" else [w for w in a.configs.split(",") if w]
        out["configs"] = []
        for w in extra:
            if w == a.workload:
                continue
            b = copy.copy(a)
            b.workload, b.steps, b.warmup = w, a.config_steps, 2
            b.width = b.height = b.scene = b.strategy = b.bounces = None
            b.bsdf, b.batch = "principled", 0
            b.cpu_seconds, b.parity_seconds = 5.0, 15.0
            b.batch1_steps = 0
            t0 = time.perf_counter()
            try:
                o = run_workload(b, world, rank, local, dist, coll_dev, quiet=True)
                rf = o["roofline"]
                out["configs"].append({
                    "workload": o["config"]["workload"], "value": o["value"], "unit": o["unit"],
                    "ms_per_step": o["ms_per_step"], "steps": o["steps"], "msample_per_s": o["msample_per_s"],
                    "roofline": {"kernel": rf["kernel"].split(" (")[0], "frac": rf["frac"], "achieved": rf["achieved"],
                                 "pmc_hbm_frac": rf.get("pmc_hbm_frac"), "traffic_per_unit": rf.get("traffic_per_unit"),
                                 "bytes_per_unit": rf["bytes_per_unit"], "shared_gpu": rf.get("shared_gpu"),
                                 "frac_kind": rf.get("frac_kind")},
                    "kernel_ms_per_step": {k: v for k, v in o["kernel_ms_per_step"].items() if k != "restir_kernels"},
                    "cpu_baseline": o["cpu_baseline"], "parity_vs_oracle": o["parity_vs_oracle"],
                    "wall_s": round(time.perf_counter() - t0, 1)})
            except Exception as e:   # one config failing must not lose the headline line
                out["configs"].append({"workload": w, "error": f"{type(e).__name__}: {e}"})
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_workload(a, world, rank, local, dist, coll_dev, quiet=False):
    """One workload through the timed region; returns rank 0's line (None on other ranks)."""
    W = a.width or (3840 if a.workload == "c5" else 256 if a.workload == "c1" else 1920)
    H = a.height or (2160 if a.workload == "c5" else 256 if a.workload == "c1" else 1080)
    default_bounces = a.bounces is None
    default_bsdf = a.bsdf == "principled"   # (C1's Lambert override below is its configuration's own)
    a.bounces = a.bounces if a.bounces is not None else (16 if a.workload == "c5" else 3)
    if a.workload in ("c3", "c3t", "c4"):
        from mpt import synthetic
        sd = (_cached("city_tex", synthetic.procedural_city_textured) if a.workload == "c3t" else
              _cached("city", lambda: synthetic.procedural_city(1234)))
        env = _cached("sky", lambda: mpt.build_envmap(scene.procedural_sky(2048, 1024, seed=7)))
        wset = scene.envmap_world(1.0)
        strategy = a.strategy or ("restir" if a.workload == "c4" else "ris")
        K = a.steps or 256
        alpha = True      # C3 pins do_alpha_testing = true (the Bistro's foliage)
        if a.workload == "c3t":
            desc = ("C3T (texture-realistic C3 variant): procedural city seed 1235, 2.77 M tris, 70 materials, 83 % of the "
                    "triangles textured (base colour + normal map + roughness-metallic, 44 textures / 193 MB RGBA8)")
        else:
            desc = f"{a.workload.upper()} stand-in: procedural city (2.86 M tris incl. alpha-tested leaf cards, seed 1234)"
        desc += " + procedural HDR sky 2048x1024 (alias-table sampling + BSDF MIS), alpha testing on"
        if a.workload == "c4":
            desc += ", ReSTIR DI fused spatiotemporal + 1 spatial pass, GPURenderer seed schedule"
    elif a.workload == "c5":
        # glass dispersion + nested dielectrics stress: ISS_WITH_PRIORITIES,
        # stack 3, nb_bounces raised to 16; uniform ambient world
        sd = scene.load_scene(a.scene or "multi-dispersion")
        env, wset = None, None
        strategy = a.strategy or "ris"
        K = a.steps or 1024
        alpha = False
        desc = f"C5: {sd.name or a.scene or 'multi-dispersion'} (glass dispersion, nested dielectrics)"
    elif a.workload == "c1":
        # C1: Cornell 256x256, 1 spp, Lambert override, reference-default RIS,
        # uniform ambient, alpha testing and adaptive sampling off, CPU seed schedule
        sd = scene.load_scene(a.scene or "cornell_pbr")
        env, wset = None, None
        strategy = a.strategy or "ris"
        K = a.steps or 1
        alpha = False
        a.bsdf = "lambert"
        desc = f"C1: {sd.name or a.scene or 'cornell_pbr'}"
    else:
        sd = scene.load_scene(a.scene or "cornell_pbr")
        env, wset = None, None
        strategy = a.strategy or "mis"
        K = a.steps or 64
        alpha = False
        desc = f"C2: {sd.name or a.scene or 'cornell_pbr'}"
    luts = scene.load_luts()
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.bsdf_override = abi.BSDF_NONE if a.bsdf == "principled" else abi.BSDF_LAMBERTIAN
    opt.direct_light_sampling = LSS[strategy]

    from mpt import partition
    if a.workload == "c4":
        # ReSTIR DI reuses neighbouring pixels: one contiguous band per rank, halo rows
        # exchanged after the G-buffer pass and before every reuse pass (RCCL send/recv)
        band = partition.contiguous_band(H, world, rank) if world > 1 else (1, 0, 1)
    else:
        band = (BAND_H, rank, world)
    if world == 1 and a.emulate_rank_of > 1 and a.workload != "c4":
        band = (BAND_H, 0, a.emulate_rank_of)
        a.no_parity = a.no_cpu_baseline = True
    band_h = band[0]
    # samples per wavefront: launches of ~TARGET_PATHS paths whatever the rank's share of the
    # frame (measured: 8 x 1080p is past the knee of the throughput curve)
    rows_rank = mpt.partition_rows(H, band[0], band[1], band[2])
    if a.batch:
        batch = min(MAX_BATCH, a.batch)
        while K % batch:                                 # whole batches in the timed region
            batch -= 1
    else:   # the divisor of K nearest to TARGET_PATHS / the rank's pixels
        want = restir_band_want(a, K, TARGET_PATHS / max(1, rows_rank * W), band[2])
        batch = min((d for d in range(1, min(MAX_BATCH, K) + 1) if K % d == 0), key=lambda d: (abs(d - want), -d))

    r = mpt.GPURenderer(local)
    r.set_scene(sd)
    r.set_luts(luts)
    if env is not None:
        r.set_envmap(env)
    if a.workload == "c4" and world == 1 and a.emulate_rank_of > 1:
        out = emulate_restir_ranks(a, r, cam, W, H, opt, wset, alpha, a.emulate_rank_of, K, local)
        r.close()
        return out
    halo = None
    if a.workload == "c4" and world > 1:
        if a.halo == "native":
            # the library's RCCL communicator: rank k renders band k, the halo rows go peer to
            # peer in one ncclSend / ncclRecv group per exchange point on the library's stream
            uid = [mpt.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            r.comm_init(world, rank, uid[0])
            r.set_halo_native(1)
        else:
            halo = partition.TorchHaloExchange(dist, band_h)
            r.set_halo_exchange(halo)

    # calibration: instrumented traversal -> nodes / triangles per query per stage
    r.enable_stats(timing=False, instrumented=True)
    # (one batch, so every launch of the run has the timed region's size)
    cal_frames = frames_for(cam, W, H, opt, band, max(2, batch), first=0, bounces=a.bounces, world=wset, alpha=alpha)
    r.render_samples(cal_frames, max_batch=batch)
    cal = r.stats()
    # warmup (untimed), then the timed K-frame accumulation restarting at sample 0
    r.enable_stats(timing=False, instrumented=False)
    warm_frames = frames_for(cam, W, H, opt, band, a.warmup, bounces=a.bounces, world=wset, alpha=alpha)
    r.render_samples(warm_frames, max_batch=batch)
    frames = frames_for(cam, W, H, opt, band, K, bounces=a.bounces, world=wset, alpha=alpha)
    r.synchronize_kernel()
    r.enable_stats(timing=True, instrumented=False)

    rows = mpt.partition_rows(H, band[0], band[1], band[2])
    if dist is not None:
        import torch
        local_fb = torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda")
        host_fb = None if coll_dev == "cuda" else torch.zeros((rows, W, 3), dtype=torch.float32)
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.render_samples(frames, max_batch=batch)
    r.synchronize_kernel()
    if dist is not None:
        r.framebuffer_to_device(abi.FB_COLOR, local_fb.data_ptr())
        if host_fb is not None:
            host_fb.copy_(local_fb)
        frame = partition.gather_frame(local_fb if host_fb is None else host_fb, H, band_h, dist)
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = r.stats()

    rays_local = st.rays_closest + st.rays_any
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        n = torch.tensor([rays_local], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        rays_total = float(n.item())
    else:
        rays_total = float(rays_local)

    # launch latency: the same frames with one sample per wavefront (the launch set of
    # mpt_render_frame, ~50 launches per sample) against the batched wavefronts timed above
    batch1 = None
    if a.workload == "c3" and world == 1 and band[2] == 1 and getattr(a, "batch1_steps", 0) > 0:
        n1 = a.batch1_steps
        fr1 = frames_for(cam, W, H, opt, band, n1, bounces=a.bounces, world=wset, alpha=alpha)
        r.enable_stats(timing=False, instrumented=False)
        r.render_samples(fr1[:2], max_batch=1)
        r.synchronize_kernel()
        t1 = time.perf_counter()
        r.render_samples(fr1, max_batch=1)
        r.synchronize_kernel()
        dt1 = time.perf_counter() - t1
        st1 = r.stats()
        batch1 = {"steps": n1, "ms_per_step": round(dt1 * 1e3 / n1, 4),
                  "vs_batched": round((dt1 / n1) / (elapsed / K), 3), "batched_samples_per_launch": batch,
                  "graph_replays": int(st1.graph_replays), "graph_captures": int(st1.graph_captures)}

    # the shading kernel alone: a pipelined wavefront (MPT_PIPELINE) runs a bounce's NEE
    # traversals beside the next bounce's shading, so the timed region's shading launches share
    # the GPU; one more batch of the same frames with the bounces in line (untimed for `value`,
    # same images) gives the kernel's own launch time (the roofline's `solo`)
    solo = None
    if st.pipelined_batches and not a.no_solo:
        r.set_pipeline(0)
        fr_s = frames_for(cam, W, H, opt, band, batch, bounces=a.bounces, world=wset, alpha=alpha)
        r.synchronize_kernel()
        r.enable_stats(timing=True, instrumented=False)
        r.render_samples(fr_s, max_batch=batch)
        r.synchronize_kernel()
        sts = r.stats()
        r.set_pipeline(1)
        hits_s = (sts.path_hits or sts.stage_rays[0]) - sts.shade_generic_vertices
        solo = {"shade_avg_launch_ms": sts.shade_ms / max(1, sts.shade_launches),
                "shade_units_per_launch": hits_s / max(1, sts.shade_launches), "steps": batch}

    # rooflines (SURVEY.md §8d algorithmic bytes): every traversal stage and the shade
    # kernel; "roofline" is the one with the largest summed time in the timed region
    names = ["k_trace<TM_PATH> (camera/continuation rays, closest hit)", "k_trace<TM_NEE_ANY> (NEE shadow rays, any hit)",
             "k_trace<TM_NEE_LIGHT> + <TM_NEE_LIGHT_OCC> (NEE BSDF light-hit rays: light BVH, then whole-scene any-hit check)"]
    symbols = ["void mpt::k_trace<0, false>(mpt::TraceArgs)", "void mpt::k_trace<1, false>(mpt::TraceArgs)",
               "void mpt::k_trace<5, false>(mpt::TraceArgs)"]
    lines = []
    for m in range(3):
        q_cal = max(1, cal.stage_rays[m])
        n_node, n_tri = cal.stage_nodes[m] / q_cal, cal.stage_tris[m] / q_cal
        b_ray = 32 + 16 + S_NODE * n_node + S_TRI * n_tri
        launches = max(1, st.stage_launches[m])
        avg_ms = st.stage_ms[m] / launches
        ach = st.stage_rays[m] * b_ray / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        lines.append({"kernel": names[m], "symbol": symbols[m], "total_ms": st.stage_ms[m], "achieved": ach, "avg_launch_ms": avg_ms,
                      "bytes_per_unit": b_ray, "unit_of_work": "ray", "nodes_per_ray": n_node, "tris_per_ray": n_tri,
                      "node_simd_util": cal.stage_nodes[m] / max(1, cal.stage_node_slots[m]),
                      "tri_simd_util": cal.stage_tris[m] / max(1, cal.stage_tri_slots[m]),
                      "units_per_launch": st.stage_rays[m] / launches, "launches": st.stage_launches[m]})
    # shade: per path vertex (a path ray that hit a surface: k_split sends the misses to
    # k_miss) = material 256 + vertex gathers 12+36+36+24 + path state 2x96 (§8d); the
    # plain-dielectric kernel (material classes) shades all but the generic
    # class's vertices
    b_vtx = 256 + 12 + 36 + 36 + 24 + 2 * 96
    sl = max(1, st.shade_launches)
    s_avg = st.shade_ms / sl
    hits = (st.path_hits or st.stage_rays[0]) - st.shade_generic_vertices
    lines.append({"kernel": "k_shade<BSDF_NONE, plain> (path vertex of a plain-dielectric material: hit, NEE sampling, "
                            "BSDF sampling, RR)",
                  "symbol": "void mpt::k_shade<0, true",   # k_shade<OVR, plain, RIS visibility>
                  "total_ms": st.shade_ms, "avg_launch_ms": s_avg, "bytes_per_unit": b_vtx, "unit_of_work": "path vertex (hit)",
                  "units_per_launch": hits / sl, "launches": st.shade_launches,
                  "achieved": hits * b_vtx / sl / (s_avg * 1e-3) / 1e9 if s_avg > 0 else 0.0, "solo": solo})
    # the generic class (every other material, incl. the vertices the plain kernel deferred);
    # launched once per bounce beside the plain kernel, same bytes per vertex
    if st.shade_generic_vertices and st.shade_generic_ms > 0:
        g_avg = st.shade_generic_ms / sl
        lines.append({"kernel": "k_shade<BSDF_NONE, generic> (path vertex of any other material: coat, sheen, metal, "
                                "thin film, transmission, metallic texels)",
                      "symbol": "void mpt::k_shade<0, false, false, false",
                      "total_ms": st.shade_generic_ms, "avg_launch_ms": g_avg, "bytes_per_unit": b_vtx,
                      "unit_of_work": "path vertex (hit)", "units_per_launch": st.shade_generic_vertices / sl,
                      "launches": st.shade_launches,
                      "achieved": st.shade_generic_vertices * b_vtx / sl / (g_avg * 1e-3) / 1e9})
    # ReSTIR DI (C4): the staged reuse passes' plain-class target-function evaluations, timed on
    # their own (HIP events around every k_rsp_eval<OVR, true, *> launch, fused and spatial); per
    # evaluation item: item 4 + its record 16 read + 4 written + the evaluated
    # surface's compact 64-B record (gb_cs) + the sample's reservoir 48 + the light's
    # emissive-table record 80 + the staged ray 36 = 252 B (an untextured surface's material is
    # the per-material resolved copy, L2-resident: not per-evaluation traffic; PMC r04: 244 B)
    B_EVAL = 4 + 16 + 4 + 64 + 48 + 80 + 36
    if st.restir_eval_launches:
        el = st.restir_eval_launches
        e_avg = st.restir_eval_ms / el
        lines.append({"kernel": "k_rsp_eval<BSDF_NONE, plain> (ReSTIR DI target-function evaluations at plain-dielectric "
                                "surfaces, fused spatiotemporal + spatial passes)",
                      "symbol": "void mpt::k_rsp_eval<0, true", "total_ms": st.restir_eval_ms, "avg_launch_ms": e_avg,
                      "bytes_per_unit": B_EVAL, "unit_of_work": "target-function evaluation",
                      "units_per_launch": st.restir_eval_items / el, "launches": el,
                      "achieved": st.restir_eval_items * B_EVAL / el / (e_avg * 1e-3) / 1e9 if e_avg > 0 else 0.0})
    n_kernel_lines = len(lines)
    # ReSTIR DI passes (C4), timed as a whole (HIP events around each pass): per pixel of the
    # band, the G-buffer / reservoir / presampled-light bytes the pass reads and writes
    # (DESIGN.md §4).  With the reference-default weights a pass is staged (restir_di.h:
    # selection, class-sorted evaluations, its rays through k_trace<TM_LIST_*>, combine,
    # visibility reuse), else one monolithic kernel tracing inline
    rk = [("k_gbuffer (CameraRays G-buffer write)", "void mpt::k_gbuffer(", 64 + 176),
          ("k_restir_presample (lights presampling)", "void mpt::k_restir_presample(", 0),
          ("ReSTIR DI initial candidates pass (k_rsi_classify, k_restir_initial<STAGED>, k_trace<LIST_CLOSEST>, "
           "k_rsi_finish, k_trace<LIST_ANY>, k_rs_visapply)", "void mpt::k_restir_initial<", 112 + 4 * 64 + 48),
          ("ReSTIR DI fused spatiotemporal pass (k_rst_select, k_rsp_eval<FUSED>, k_trace<LIST_ANY>, k_rst_combine, "
           "k_rs_visapply)", "void mpt::k_rst_", 112 + 160 + 2 * 160 + 48 + 48),
          ("ReSTIR DI spatial reuse pass (k_rsp_select, k_rsp_eval, k_trace<LIST_ANY>, k_rsp_combine, k_rs_visapply)",
           "void mpt::k_rsp_", 112 + 48 + 2 * 160 + 48)]
    n_pix = rows_rank * W
    for k, (name, sym, bpp) in enumerate(rk):
        ms, nl = st.restir_kernel_ms[k], st.restir_kernel_launches[k]
        if nl == 0 or bpp == 0:
            continue
        avg = ms / nl
        lines.append({"kernel": name, "symbol": sym, "total_ms": ms, "avg_launch_ms": avg, "bytes_per_unit": bpp,
                      "unit_of_work": "pixel", "units_per_launch": n_pix, "launches": nl,
                      "achieved": n_pix * bpp / (avg * 1e-3) / 1e9 if avg > 0 else 0.0})
    # the dominant KERNEL (the ReSTIR DI pass lines above span several kernels: reported, not candidates)
    dom = max(lines[:n_kernel_lines], key=lambda x: x["total_ms"])

    default_cfg = a.strategy is None and default_bounces and default_bsdf and a.scene is None
    pmc = load_traffic(a.workload, W, H) if default_cfg else None

    def pmc_entry(sym):
        if not pmc:
            return {}
        if sym in pmc["kernels"]:
            return pmc["kernels"][sym]
        for k2, v in pmc["kernels"].items():     # template kernels: match the name prefix
            if k2.startswith(sym):
                return v
        return {}

    def roof(x):
        # counter fields come from the committed profile of this command (profiles/), each
        # normalised by THAT run's own launches: its units per launch (the bench line of the
        # profiled run) and its kernel-trace launch time -- so per-unit bytes and fractions do not
        # depend on this run's --steps; `traffic` is those bytes per unit x this run's units
        tr = pmc_entry(x["symbol"]).get("timed") or {}
        r = {"bound": "hbm", "achieved": round(x["achieved"], 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(x["achieved"] / HBM_PEAK_GBS, 5), "traffic": None,
             "kernel": x["kernel"],
             "avg_launch_ms": round(x["avg_launch_ms"], 5), "bytes_per_unit": round(x["bytes_per_unit"], 2),
             "unit_of_work": x["unit_of_work"], "units_per_launch": round(x["units_per_launch"], 1)}
        if tr.get("traffic_per_unit"):
            r.update(traffic=round(tr["traffic_per_unit"] * x["units_per_launch"]),
                     traffic_per_unit=round(tr["traffic_per_unit"], 1),
                     traffic_read_per_unit=round(tr["read_per_unit"], 1), traffic_write_per_unit=round(tr["write_per_unit"], 1),
                     traffic_source=pmc["file"],
                     # the profiled library against this run's: counters of another build are flagged
                     traffic_libmpt_sha256_16=pmc.get("libmpt_sha256_16"),
                     traffic_same_library=(pmc.get("libmpt_sha256_16") == mpt.build_id()) if pmc.get("libmpt_sha256_16") else None,
                     profiled={"units_per_launch": round(tr["units_per_launch"], 1), "launches": tr["launches"],
                               "avg_launch_ms": round(tr["avg_ns"] / 1e6, 5), "traffic_per_launch": round(tr["traffic_bytes"])},
                     # the kernel's measured HBM bytes over its own profiled launch time
                     pmc_hbm_frac=round(tr["hbm_frac"], 4))
        if tr.get("valu_insts"):
            # VALU issue roofline: wave-level VALU instructions per launch over the chip's issue
            # rate (256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles at 2.4 GHz), both
            # from the profiled run
            r["valu"] = {"insts_per_launch": round(tr["valu_insts"]), "achieved_tinst_s": round(tr["valu_rate"] / 1e12, 4),
                         "peak_tinst_s": VALU_PEAK / 1e12, "frac": round(tr["valu_rate"] / VALU_PEAK, 4),
                         "per_unit": round(tr["valu_insts"] / max(1.0, tr["units_per_launch"]), 2)}
        if x["unit_of_work"] == "ray":
            # a traversal's algorithmic bytes count every node and triangle record it fetches, most of
            # them L2 hits: frac is an accounting figure, pmc_hbm_frac the HBM bandwidth it draws
            r["frac_kind"] = "algorithmic node/triangle bytes (mostly L2 hits; HBM drawn: pmc_hbm_frac)"
        if "nodes_per_ray" in x:
            r.update(nodes_per_ray=round(x["nodes_per_ray"], 3), tris_per_ray=round(x["tris_per_ray"], 3),
                     node_simd_util=round(x["node_simd_util"], 3), tri_simd_util=round(x["tri_simd_util"], 3))
        if x.get("solo") and x["solo"]["shade_avg_launch_ms"] > 0:
            so = x["solo"]
            ach = so["shade_units_per_launch"] * x["bytes_per_unit"] / (so["shade_avg_launch_ms"] * 1e-3) / 1e9
            r["solo"] = {"what": "the same kernel with the bounces in line (mpt_set_pipeline 0), one more batch of the "
                                 "frames after the timed region",
                         "avg_launch_ms": round(so["shade_avg_launch_ms"], 5), "units_per_launch": round(so["shade_units_per_launch"], 1),
                         "achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 5)}
        if getattr(st, "overlapped_batches", 0):
            # MPT_OVERLAP (the library's default for wavefronts of <= 24 M paths): each batch ran as
            # two halves on two streams, so this kernel's launches shared the GPU with the other
            # half's kernels -- its launch time, and with it `achieved`, is not the kernel's alone
            r["shared_gpu"] = f"{st.overlapped_batches} overlapped batch(es): launch times shared with the other half"
        elif getattr(st, "pipelined_batches", 0) and x["unit_of_work"] != "ray":
            # MPT_PIPELINE: the shading launches ran beside the previous bounce's NEE traversals
            r["shared_gpu"] = (f"{st.pipelined_batches} pipelined batch(es): the shading launches shared the GPU with "
                               "the previous bounce's NEE traversals (the kernel alone: `solo`)")
        elif x["unit_of_work"] == "ray" and getattr(st, "trace_ahead_launches", 0):
            # MPT_TRACE_AHEAD: a bounce's path traversal ran beside the previous bounce's NEE
            # traversals, so the traversal stages' launch times overlap
            r["shared_gpu"] = (f"{st.trace_ahead_launches} path traversal(s) launched ahead: launch times shared with "
                               "the previous bounce's NEE traversals")
            if getattr(st, "pipelined_batches", 0):
                # MPT_PIPELINE: a bounce's NEE traversals and resolve also ran beside the next
                # bounce's split and shading
                r["shared_gpu"] += (f"; {st.pipelined_batches} pipelined batch(es): NEE traversals beside the next "
                                    "bounce's split and shading")
        elif getattr(st, "restir_overlapped_batches", 0):
            # MPT_RESTIR_OVERLAP: a ReSTIR DI batch's later bounces ran on the second stream beside
            # the next batch's per-sample chain
            r["shared_gpu"] = (f"{st.restir_overlapped_batches} overlapped ReSTIR DI batch(es): launch times shared "
                               "with the next batch's reuse chain")
        return r

    dname, darch, dcus = mpt.device_info(local)
    device = {"name": dname, "arch": darch, "compute_units": dcus, "libmpt_sha256_16": mpt.build_id()}

    parity = None
    if rank == 0 and world == 1 and not a.no_parity:
        # the GPU leg: a fresh accumulation restarting at sample 0 (sample 0 overwrites the sums)
        parity = parity_check(r, sd, luts, cam, W, H, opt, a.bounces, K if a.workload == "c1" else a.parity_spp,
                              a.workload, env=env, world=wset, alpha=alpha, max_s=a.parity_seconds, batch=batch,
                              history=cal_frames + warm_frames + frames)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(sd, luts, cam, W, H, opt, a.bounces, a.cpu_seconds, env=env, world=wset, alpha=alpha)
        except Exception as e:  # the baseline is reported, never the product path
            cpu = {"value": None, "unit": "Mray/s", "cores": 0, "kind": "port", "sample": f"failed: {e}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(rays_total / elapsed / 1e6, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": K,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / K, 4),
            "higher_is_better": True,
            "scaling": "strong",   # fixed frame split over the ranks
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (seeded procedural city + sky standing in for Bistro + its HDR, "
                     + ("GPURenderer seed schedule)" if a.workload == "c4" else "CPU seed schedule)")
                     if a.workload in ("c3", "c3t", "c4") else f"synthetic (reference glTF {sd.name}, seeded CPU seed schedule)"),
            "msample_per_s": round(W * H * K / elapsed / 1e6, 3),
            "samples_per_launch": round(st.frames / max(1, st.shade_launches / (a.bounces + 1)), 3),
            "rays_per_sample": round(rays_total / (W * H * K), 4),
            "path_hit_fraction": round(st.path_hits / max(1, st.stage_rays[0]), 4),
            "config": {"workload": f"{desc}, {W}x{H}, {K} spp, "
                                   f"{'layered Principled' if a.bsdf == 'principled' else 'Lambert-override'} BSDF + NEE "
                                   f"({strategy.upper()}), {a.bounces} bounces, 1 step = 1 spp",
                       "scene": sd.name, "triangles": int(sd.num_triangles), "width": W, "height": H, "spp": K,
                       "strategy": strategy,
                       "partition": (f"contiguous {band_h}-row bands over {world} rank(s), halo exchange by RCCL send/recv "
                                     f"({'libmpt native' if a.halo == 'native' else 'torch.distributed'}), RCCL all_gather"
                                     if a.workload == "c4" and world > 1 else
                                     f"interleaved {BAND_H}-row bands over {world} rank(s), RCCL all_gather")},
            "roofline": roof(dom),
            "roofline_traversal": roof(max(lines[:3], key=lambda x: x["total_ms"])),
            "roofline_restir": roof(lines[n_kernel_lines - 1]) if st.restir_eval_launches else None,
            # every timed kernel line of this run (tools/pmc_traffic.py normalises the profile of
            # this command by them: the last `launches` dispatches of `symbol` are the timed ones)
            "kernel_lines": [{"symbol": x["symbol"], "launches": x["launches"], "units_per_launch": x["units_per_launch"],
                              "avg_launch_ms": round(x["avg_launch_ms"], 5), "bytes_per_unit": round(x["bytes_per_unit"], 2)}
                             for x in lines[:n_kernel_lines]],
            "restir_passes": [{"kernel": x["kernel"], "ms_per_step": round(x["total_ms"] / K, 4), "model_bytes_per_pixel": x["bytes_per_unit"],
                               "model_achieved_gbs": round(x["achieved"], 2)} for x in lines[n_kernel_lines:]] or None,
            "device": device,
            "traversal_stages": [{"kernel": x["kernel"].split(" ")[0], "nodes_per_ray": round(x["nodes_per_ray"], 3),
                                  "tris_per_ray": round(x["tris_per_ray"], 3), "node_simd_util": round(x["node_simd_util"], 3),
                                  "tri_simd_util": round(x["tri_simd_util"], 3)} for x in lines[:3]],
            "kernel_ms_per_step": {"trace_path": round(st.stage_ms[0] / K, 4), "trace_nee_any": round(st.stage_ms[1] / K, 4),
                                   "trace_nee_closest": round(st.stage_ms[2] / K, 4), "shade": round(st.shade_ms / K, 4),
                                   "shade_generic": round(st.shade_generic_ms / K, 4),
                                   "resolve": round(st.resolve_ms / K, 4), "camera": round(st.camera_ms / K, 4),
                                   "accumulate": round(st.accumulate_ms / K, 4),
                                   "compact": round(st.compact_ms / K, 4), "split": round(st.split_ms / K, 4),
                                   "miss": round(st.miss_ms / K, 4), "restir": round(st.restir_ms / K, 4),
                                   "restir_kernels": {n: round(st.restir_kernel_ms[i] / K, 4) for i, n in
                                                      enumerate(["gbuffer", "presample", "initial", "temporal_reuse",
                                                                 "spatial_reuse"])},
                                   "frame_gpu": round(st.frame_ms / max(1, st.frames), 4)},
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
        }
        if batch1 is not None:
            out["batch1"] = batch1
        if st.pipelined_batches or st.trace_ahead_launches:
            # kernels on several streams: an event pair spans the wait for CUs held by the other
            # stream's kernels (k_split starts beside the persistent NEE traversal), so the entries
            # overlap and their sum exceeds frame_gpu
            out["kernel_ms_note"] = ("pipelined / trace-ahead frames: per-kernel event spans overlap and include the "
                                     "wait for CUs held by the other streams' kernels; frame_gpu is the frame's own span")
        if band[2] > world:
            out["emulated_rank_of"] = band[2]
            out["msample_per_s"] = round(rows * W * K / elapsed / 1e6, 3)
        if halo is not None:
            nfr = 2 + a.warmup + K
            out["halo_exchange"] = {"calls_per_frame": round(halo.calls / nfr, 2),
                                    "mb_received_per_frame_rank0": round(halo.bytes_moved / nfr / 1e6, 3)}
    r.close()
    return out if rank == 0 else None


if __name__ == "__main__":
    main()
