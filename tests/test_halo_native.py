"""The library's own ReSTIR DI halo exchange (mpt_set_halo_native; SURVEY.md §8e, the ReSTIR row).

* Mode 2, the one-GPU rehearsal the bench's C4 rank-of-N timing uses: its exchange points and
  byte counts (MptStats.halo_*) equal what the Python exchange derives from
  mpt.partition.halo_plan at the same exchange points, on bands of the 8-way 1080p split with a
  still and a moving camera.
* Mode 1, RCCL send / receive between processes, one per GPU: two bands on devices 0 and 1
  against one context, with a moving camera (the all-reduce agreement runs), a still camera (the
  agreement is skipped) and batched samples.  Needs two GPUs: skipped on a one-GPU box, where
  tests/test_halo_plan.py checks that the two sides' operations pair up.
"""
import os

import numpy as np
import pytest

from mpt import abi, scene

pytestmark = pytest.mark.gpu


def _frames(sd, n, w, h, band, move_at=None, reuse_radius=None):
    from test_restir import frames
    kw = {} if reuse_radius is None else dict(reuse_radius=reuse_radius)
    return frames(sd, abi.LSS_RESTIR_DI, n, w=w, h=h, band=band, move_at=move_at, **kw)


def _renderer(sd, luts, device=0):
    import mpt
    r = mpt.GPURenderer(device)
    r.set_scene(sd)
    r.set_luts(luts)
    return r


@pytest.mark.parametrize("k", [0, 3, 7])
@pytest.mark.parametrize("batched", [False, True], ids=["per_frame", "batched"])
def test_native_rehearsal_bytes_equal_halo_plan(cornell, luts, k, batched):
    from mpt import partition
    W, H, NB = 480, 1080, 8
    bh = partition.contiguous_band(H, NB, 0)[0]
    band = partition.contiguous_band(H, NB, k)
    frs = _frames(cornell, 5, W, H, band, move_at=2)
    counts = {}
    for mode in ("python", "native"):
        r = _renderer(cornell, luts)
        c = {"calls": 0, "recv": 0, "sent": 0, "agree": 0}

        def cb(x):
            sends, recvs = partition.halo_plan(x.res_y, bh, NB, k, x.halo_rows)
            per_row = sum(x.res_x * x.bytes_per_pixel[i] for i in range(x.n_buffers))
            c["recv"] += per_row * sum(y1 - y0 for (_, y0, y1) in recvs)
            c["sent"] += per_row * sum(y1 - y0 for (_, y0, y1) in sends)
            c["calls"] += 1
            c["agree"] += int(x.phase == partition.HALO_GBUFFER and not x.halo_agreed)

        if mode == "python":
            r.set_halo_exchange(cb)
        else:
            r.set_halo_native(2)
        r.enable_stats(timing=False)
        if batched:
            r.render_samples(frs, max_batch=3)
        else:
            for f in frs:
                r.render(f)
        r.synchronize_kernel()
        st = r.stats()
        if mode == "native":
            c = {"calls": st.halo_exchanges, "recv": st.halo_bytes_received, "sent": st.halo_bytes_sent, "agree": None}
        counts[mode] = c
        r.close()
    py, nat = counts["python"], counts["native"]
    assert py["calls"] > 0 and py["recv"] > 0 and py["sent"] > 0
    assert py["agree"] >= 1            # the moved camera's frame needs the agreement
    assert (nat["calls"], nat["recv"], nat["sent"]) == (py["calls"], py["recv"], py["sent"]), (nat, py)


def _n_devices():
    import torch
    return torch.cuda.device_count()


def _rccl_rank(rank, n, uid_q, out_dir, case):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "hiprt-path-tracer_amd"), root, os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import mpt
    from mpt import partition
    sd = scene.load_scene("cornell_pbr")
    w, h, nfr, mv, batch = case
    band = partition.contiguous_band(h, n, rank)
    r = _renderer(sd, scene.load_luts(), device=rank)
    if rank == 0:
        uid = mpt.comm_unique_id()
        for _ in range(n - 1):
            uid_q.put(uid)
    else:
        uid = uid_q.get(timeout=120)
    r.comm_init(n, rank, uid)
    r.set_halo_native(1)
    r.enable_stats(timing=False)
    frs = _frames(sd, nfr, w, h, band, move_at=mv, reuse_radius=5)
    if batch:
        r.render_samples(frs, max_batch=batch)
    else:
        for f in frs:
            r.render(f)
    r.synchronize_kernel()
    st = r.stats()
    np.save(os.path.join(out_dir, f"band{rank}.npy"), r.framebuffer(abi.FB_COLOR))
    np.save(os.path.join(out_dir, f"stats{rank}.npy"),
            np.array([st.halo_exchanges, st.halo_agreements, st.halo_bytes_sent, st.halo_bytes_received], np.int64))
    r.close()


RCCL_CASES = {
    # (W, H, frames, move_at, max_batch)
    "moving_camera": (24, 64, 5, 2, 0),
    "still_camera": (24, 64, 5, None, 0),
    "batched_moving": (24, 64, 6, 3, 3),
    "halo_wider_than_band": (24, 40, 4, None, 2),
}


@pytest.mark.parametrize("case", list(RCCL_CASES))
def test_native_rccl_two_gpus_equals_single_context(cornell, luts, tmp_path, case):
    if _n_devices() < 2:
        pytest.skip("one GPU: the RCCL halo exchange needs a GPU per rank (tests/test_halo_plan.py pins its plan)")
    import multiprocessing as mp
    w, h, nfr, mv, batch = RCCL_CASES[case]
    ctx = mp.get_context("spawn")
    uid_q = ctx.Queue()
    ps = [ctx.Process(target=_rccl_rank, args=(k, 2, uid_q, str(tmp_path), RCCL_CASES[case])) for k in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0, f"rank exit code {p.exitcode}"
    got = np.concatenate([np.load(tmp_path / f"band{k}.npy") for k in range(2)])
    r = _renderer(cornell, luts)
    for f in _frames(cornell, nfr, w, h, (1, 0, 1), move_at=mv, reuse_radius=5):
        r.render(f)
    r.synchronize_kernel()
    ref = r.framebuffer(abi.FB_COLOR)
    r.close()
    assert np.array_equal(got, ref), f"{case}: {(got != ref).sum()} values differ"
    st = [np.load(tmp_path / f"stats{k}.npy") for k in range(2)]
    for s in st:
        assert s[0] > 0
    assert st[0][2] == st[1][3] and st[1][2] == st[0][3]      # what one band sent, the other received
    if mv is None:
        assert st[0][1] == 0                                     # a still camera: no agreement all-reduce
    else:
        assert st[0][1] >= 1 and st[0][1] == st[1][1]
