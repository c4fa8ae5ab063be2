"""GPU memory behaviour of the C ABI: an allocation failure leaves the context usable,
wavefronts shrink instead of failing when the device is short of memory, and contexts give
back everything they allocated (round-1 advisor findings on mpt_api.cpp).

Memory pressure is made with a torch tensor that holds all but a chosen number of bytes of
the device (libmpt and torch share one HIP runtime, mpt/__init__.py)."""
import os

import numpy as np
import pytest

import mpt
from mpt import abi, scene

pytestmark = pytest.mark.gpu

MB = 1 << 20


def _torch():
    import torch
    return torch


def free_bytes():
    torch = _torch()
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


class Hog:
    """Holds device memory so that about `leave` bytes stay free."""

    def __init__(self, leave):
        torch = _torch()
        torch.cuda.empty_cache()
        n = free_bytes() - leave
        self.t = torch.empty(n, dtype=torch.uint8, device="cuda") if n > 0 else None

    def release(self):
        self.t = None
        _torch().cuda.empty_cache()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.release()


def frames(sd, W, H, n, lss=abi.LSS_MIS_LIGHT_BSDF):
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = lss
    return [scene.make_frame(cam, W, H, options=opt, settings=scene.parity_settings(3), sample_number=s,
                             random_seed=seed) for s, seed in scene.cpu_seed_schedule(n)]


def new_renderer(sd, luts):
    r = mpt.GPURenderer(0)
    r.set_scene(sd)
    r.set_luts(luts)
    return r


def test_wavefront_shrinks_when_memory_is_short(cornell, luts):
    """A 64-sample wavefront of 512x512 paths (~7.7 GB of path state) with ~2 GB free: the
    library halves the wavefront until it fits, with the same sums as sample by sample."""
    W, H, n = 512, 512, 64
    frs = frames(cornell, W, H, n)
    with new_renderer(cornell, luts) as r:
        r.render_samples(frs, max_batch=1)
        r.synchronize_kernel()
        ref = r.framebuffer(abi.FB_COLOR)
    with new_renderer(cornell, luts) as r:
        with Hog(2048 * MB):
            r.render_samples(frs, max_batch=64)
            r.synchronize_kernel()
            got = r.framebuffer(abi.FB_COLOR)
    assert np.array_equal(got, ref)


def test_out_of_memory_is_reported_and_the_context_recovers(cornell, luts):
    W, H = 1024, 1024
    frs = frames(cornell, W, H, 2)
    with new_renderer(cornell, luts) as r:
        r.render_samples(frs)
        r.synchronize_kernel()
        ref = r.framebuffer(abi.FB_COLOR)
    with new_renderer(cornell, luts) as r:
        # the framebuffers (48 B per pixel, 50 MB) do not fit
        with Hog(16 * MB):
            with pytest.raises(mpt.MptError) as e:
                r.render(frs[0])
            assert e.value.code == abi.ERR_OUT_OF_MEMORY
        # the framebuffers fit, the path state (~460 B per path, 480 MB) does not
        with Hog(200 * MB):
            with pytest.raises(mpt.MptError) as e:
                r.render(frs[0])
            assert e.value.code == abi.ERR_OUT_OF_MEMORY
        # the same context renders correctly once the memory is back
        r.render_samples(frs)
        r.synchronize_kernel()
        assert np.array_equal(r.framebuffer(abi.FB_COLOR), ref)


def test_default_wavefront_is_bounded(cornell, luts):
    """max_batch = 0 at 1920x1080 with 32 frames: wavefronts of at most
    MPT_DEFAULT_WAVEFRONT_PATHS paths (16 samples per pixel), same sums as explicit batches."""
    W, H, n = 1920, 1080, 32
    frs = frames(cornell, W, H, n)
    with new_renderer(cornell, luts) as r:
        r.enable_stats(timing=True)
        r.render_samples(frs)
        r.synchronize_kernel()
        st = r.stats()
        got = r.framebuffer(abi.FB_COLOR)
        # 4 bounces per wavefront, each wavefront shaded as two overlapped halves (MPT_OVERLAP)
        halves = 2 if os.environ.get("MPT_OVERLAP", "0") != "0" else 1
        assert st.shade_launches == 4 * halves * (n // (abi.DEFAULT_WAVEFRONT_PATHS // (W * H)))
        r.render_samples(frs, max_batch=8)
        r.synchronize_kernel()
        assert np.array_equal(r.framebuffer(abi.FB_COLOR), got)


def test_restir_contexts_release_their_memory(cornell, luts):
    """create -> ReSTIR DI frames -> destroy, three times: the device's free memory comes back
    (the G-buffers, reservoirs and presampled lights are released with the context)."""
    from test_restir import frames as restir_frames
    frs = restir_frames(cornell, abi.LSS_RESTIR_DI, 3, w=256, h=144)

    def cycle():
        with new_renderer(cornell, luts) as r:
            r.render_samples(frs)
            r.synchronize_kernel()

    cycle()                       # first use: code objects, runtime pools
    base = free_bytes()
    for _ in range(3):
        cycle()
    assert free_bytes() >= base - 16 * MB
