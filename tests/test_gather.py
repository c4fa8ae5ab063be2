"""The boundary's multi-GPU output (SURVEY.md §8b Outputs row): mpt_gather assembles the row
partitions of one frame rendered by several contexts of one process (peer copies between
GPUs; here every context is on device 0), and mpt_comm_gather does the same across processes
over RCCL (one rank here: the box has one GPU).  The gathered frame must equal a single
context's render bit for bit -- every pixel's RNG stream depends only on (pixel, sample, seed).
"""
import numpy as np
import pytest

W, H = 40, 27   # 27 rows: the last 8-row group of a band is partial


def _frames(sd, band, lss, n=3):
    from mpt import abi, scene
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    st = scene.parity_settings(3)
    return [scene.make_frame(cam, W, H, settings=st, options=opt, sample_number=s, random_seed=seed, band=band)
            for s, seed in scene.cpu_seed_schedule(n)]


def _renderer(sd, luts):
    import mpt
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("n,bh", [(2, 8), (3, 8), (3, 10), (4, 7)])
def test_gather_equals_single_context(cornell, luts, n, bh):
    import mpt
    from mpt import abi
    lss = abi.LSS_MIS_LIGHT_BSDF
    ref = _renderer(cornell, luts)
    ref.render_samples(_frames(cornell, (1, 0, 1), lss))
    ref.synchronize_kernel()
    want = ref.framebuffer(abi.FB_COLOR)
    want_cnt = ref.aux_buffer(abi.AUX_SAMPLE_COUNT)
    parts = [_renderer(cornell, luts) for _ in range(n)]
    for k, r in enumerate(parts):
        r.render_samples(_frames(cornell, (bh, k, n), lss))
    for root in (0, n - 1):
        got = mpt.gather(parts, root=root, kind=abi.FB_COLOR)
        assert np.array_equal(got, want), f"n={n} bh={bh} root={root}: {(got != want).sum()} values differ"
    got_cnt = mpt.gather(parts, kind=mpt.GATHER_AUX + abi.AUX_SAMPLE_COUNT)
    assert np.array_equal(got_cnt, want_cnt)
    assert want.mean() > 0


@pytest.mark.gpu
def test_gather_refuses_inconsistent_partitions(cornell, luts):
    import mpt
    from mpt import abi
    a, b = _renderer(cornell, luts), _renderer(cornell, luts)
    a.render_samples(_frames(cornell, (8, 0, 2), abi.LSS_MIS_LIGHT_BSDF, 1))
    b.render_samples(_frames(cornell, (8, 0, 2), abi.LSS_MIS_LIGHT_BSDF, 1))   # band 0 twice
    with pytest.raises(mpt.MptError, match="band indices"):
        mpt.gather([a, b])
    c = _renderer(cornell, luts)
    c.render_samples(_frames(cornell, (4, 1, 2), abi.LSS_MIS_LIGHT_BSDF, 1))   # other band height
    with pytest.raises(mpt.MptError, match="partition"):
        mpt.gather([a, c])


@pytest.mark.gpu
def test_comm_gather_one_rank(cornell, luts):
    """mpt_comm_unique_id / mpt_comm_init / mpt_comm_gather over a one-rank RCCL communicator
    (the collective path a process-per-GPU host takes; more ranks need more GPUs)."""
    import mpt
    from mpt import abi
    r = _renderer(cornell, luts)
    r.render_samples(_frames(cornell, (8, 0, 1), abi.LSS_MIS_LIGHT_BSDF))
    r.synchronize_kernel()
    uid = mpt.comm_unique_id()
    assert len(uid) == 128
    r.comm_init(1, 0, uid)
    got = r.comm_gather(root=0, kind=abi.FB_COLOR)
    want = r.framebuffer(abi.FB_COLOR)
    assert np.array_equal(got, want)
    got_alb = r.comm_gather(root=0, kind=abi.FB_ALBEDO)
    assert np.array_equal(got_alb, r.framebuffer(abi.FB_ALBEDO))


def _n_devices():
    import torch
    return torch.cuda.device_count()


@pytest.mark.gpu
def test_gather_across_devices(cornell, luts):
    """mpt_gather with the bands on different GPUs (peer copies after hipDeviceEnablePeerAccess);
    needs two GPUs -- skipped on a one-GPU box, where the tests above put every band on device 0."""
    import mpt
    from mpt import abi
    nd = _n_devices()
    if nd < 2:
        pytest.skip("one GPU")
    lss = abi.LSS_MIS_LIGHT_BSDF
    ref = _renderer(cornell, luts)
    ref.render_samples(_frames(cornell, (1, 0, 1), lss))
    ref.synchronize_kernel()
    want = ref.framebuffer(abi.FB_COLOR)
    parts = []
    for k in range(3):
        r = mpt.GPURenderer(k % nd)
        r.set_scene(cornell)
        r.set_luts(luts)
        r.render_samples(_frames(cornell, (8, k, 3), lss))
        parts.append(r)
    got = mpt.gather(parts, root=1, kind=abi.FB_COLOR)
    assert np.array_equal(got, want)


def _comm_rank(rank, n, uid_q, out_q):
    import mpt
    from mpt import abi, scene
    sd = scene.load_scene("cornell_pbr")
    r = mpt.GPURenderer(rank)
    r.set_scene(sd)
    r.set_luts(scene.load_luts())
    r.render_samples(_frames(sd, (8, rank, n), abi.LSS_MIS_LIGHT_BSDF))
    r.synchronize_kernel()
    if rank == 0:
        uid = mpt.comm_unique_id()
        for _ in range(n - 1):
            uid_q.put(uid)
    else:
        uid = uid_q.get(timeout=60)
    r.comm_init(n, rank, uid)
    got = r.comm_gather(root=0, kind=abi.FB_COLOR)
    out_q.put((rank, got if rank == 0 else None))


@pytest.mark.gpu
def test_comm_gather_two_processes(cornell, luts):
    """mpt_comm_gather over a two-rank RCCL communicator, one process per GPU (the process-per-GPU
    host's output path); needs two GPUs -- skipped on a one-GPU box."""
    import multiprocessing as mp
    from mpt import abi
    if _n_devices() < 2:
        pytest.skip("one GPU")
    ref = _renderer(cornell, luts)
    ref.render_samples(_frames(cornell, (1, 0, 1), abi.LSS_MIS_LIGHT_BSDF))
    ref.synchronize_kernel()
    want = ref.framebuffer(abi.FB_COLOR)
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=_comm_rank, args=(k, 2, uid_q, out_q)) for k in range(2)]
    for p in ps:
        p.start()
    res = dict(out_q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0], want)
