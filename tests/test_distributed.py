"""N>1 path on CPU: world_size-2 gloo run of the row partition + gather used by bench.py.

Each rank renders its interleaved bands (the CPU oracle stands in for the per-rank GPU
renderer, which this container does not have), the ranks exchange their compact rows
through ``mpt.partition.gather_frame`` and the assembled frame must equal a
single-process render bit-for-bit (per-pixel RNG streams are partition-independent).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

W, H, BAND = 24, 20, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frames(band):
    from mpt import abi, scene
    sd = scene.load_scene("cornell_pbr")
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_MIS_LIGHT_BSDF
    return sd, [scene.make_frame(cam, W, H, options=opt, sample_number=s, random_seed=seed, band=band)
                for s, seed in scene.cpu_seed_schedule(2)]


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "hiprt-path-tracer_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpt import partition, scene
    from oracle import oracle as orc
    sd, frames = _frames((BAND, rank, world))
    o = orc.Oracle(sd, scene.load_luts())
    local = torch.from_numpy(o.render(frames, nthreads=1))
    full = partition.gather_frame(local, H, BAND, dist)
    if rank == 0:
        np.save(out_path, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_render_gathers_to_single_process_image(tmp_path, world):
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    from mpt import scene
    from oracle import oracle as orc
    sd, frames = _frames((BAND, 0, 1))
    ref = orc.Oracle(sd, scene.load_luts()).render(frames, nthreads=2)
    got = np.load(out)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


# ---- ReSTIR DI across a row partition: contiguous bands + halo exchange ---------------

@pytest.mark.parametrize("res_y,world,halo", [(20, 2, 3), (20, 3, 7), (37, 4, 5), (24, 3, 24), (10, 4, 2), (9, 4, 4)])
def test_halo_plan_covers_exactly_the_needed_rows(res_y, world, halo):
    """Every rank receives each row of [y0 - halo, y0) and [y1, y1 + halo) once, from its
    owner, and every receive pairs with the owner's send of the same rows in the same order."""
    from mpt import partition
    bh = partition.contiguous_band(res_y, world, 0)[0]
    plans = [partition.halo_plan(res_y, bh, world, k, halo) for k in range(world)]
    for k in range(world):
        y0, y1 = partition.band_range(res_y, bh, k)
        want = set(range(max(0, y0 - halo), y0)) | set(range(y1, min(res_y, y1 + halo))) if y0 < y1 else set()
        got = [y for (_, a, b) in plans[k][1] for y in range(a, b)]
        assert sorted(got) == sorted(want) and len(got) == len(set(got))
        for (p, a, b) in plans[k][1]:
            p0, p1 = partition.band_range(res_y, bh, p)
            assert p0 <= a < b <= p1
        for p in range(world):
            mine = [(a, b) for (q, a, b) in plans[k][0] if q == p]
            theirs = [(a, b) for (q, a, b) in plans[p][1] if q == k]
            assert mine == theirs


def _halo_worker(rank, world, port, res_y, halo, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "hiprt-path-tracer_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mpt import partition
    bh = partition.contiguous_band(res_y, world, rank)[0]
    y0, y1 = partition.band_range(res_y, bh, rank)
    # three "buffers" of different record sizes; rows outside the band start as garbage
    views = []
    for k, row_bytes in enumerate((48, 16 * 7, 4 * 7)):
        v = torch.full((res_y, row_bytes), 255 - rank, dtype=torch.uint8)
        truth = ((torch.arange(res_y)[:, None] * 31 + torch.arange(row_bytes)[None, :] * 7 + k) % 251).to(torch.uint8)
        v[y0:y1] = truth[y0:y1]
        views.append((v, truth))
    ex = partition.TorchHaloExchange(dist, bh)
    agreed_ok = ex.agree(3 * rank + 1) == 3 * (world - 1) + 1     # the G-buffer phase's agreement
    ex.exchange_views([v for v, _ in views], res_y, halo)
    lo, hi = max(0, y0 - halo), min(res_y, y1 + halo)
    ok = all(torch.equal(v[lo:hi], t[lo:hi]) for v, t in views)
    untouched = all(bool((v[:lo] == 255 - rank).all()) and bool((v[hi:] == 255 - rank).all()) for v, _ in views)
    res = torch.tensor([int(ok), int(untouched), int(agreed_ok)], dtype=torch.int64)
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if rank == 0:
        np.save(out_path, res.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,res_y,halo", [(2, 20, 4), (3, 23, 9)])
def test_halo_exchange_gloo_fills_halo_rows(tmp_path, world, res_y, halo):
    """The exchange code path of the partitioned ReSTIR DI render (TorchHaloExchange, gloo
    transport on host tensors): after one exchange every rank holds its owners' rows in its
    halo and nothing outside it changed."""
    out = str(tmp_path / "halo.npy")
    mp.spawn(_halo_worker, args=(world, _free_port(), res_y, halo, out), nprocs=world, join=True)
    assert np.load(out).tolist() == [1, 1, 1]
