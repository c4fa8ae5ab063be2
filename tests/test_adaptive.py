"""Adaptive sampling and the stop-noise threshold (AdaptiveSampling.h:11-104,
CameraRays.h:88-125, FullPathTracer.h:293-305).

CPU (oracle) properties: a pixel that keeps sampling has exactly the sum of a run without
adaptive sampling (its RNG stream depends only on pixel, sample number and seed), a
converged pixel stops counting samples and is rescaled by (n+1)/n per skipped sample.
GPU: the HIP path equals the oracle bit for bit -- sums, per-pixel sample counts,
converged sample counts and the status values."""
import numpy as np
import pytest

from mpt import abi, scene

W, H, N = 48, 32, 12


def frames(sd, settings, n=N, band=(1, 0, 1), last_status=True):
    cam = scene.make_camera(sd.camera_info, W, H)
    opt = abi.KernelOptions.default()
    opt.direct_light_sampling = abi.LSS_MIS_LIGHT_BSDF
    out = []
    for s, seed in scene.cpu_seed_schedule(n):
        st = abi.RenderSettings.from_buffer_copy(settings)
        st.do_update_status_buffers = last_status and s == n - 1
        st.denoiser_AOV_accumulation_counter = s
        out.append(scene.make_frame(cam, W, H, options=opt, settings=st, sample_number=s, random_seed=seed, band=band))
    return out


def adaptive_settings(min_samples=3, threshold=0.6):
    st = scene.parity_settings(3)
    st.enable_adaptive_sampling = True
    st.adaptive_sampling_min_samples = min_samples
    st.adaptive_sampling_noise_threshold = threshold
    return st


def stop_noise_settings(threshold=0.5):
    st = scene.parity_settings(3)
    st.enable_pixel_stop_noise_threshold = True
    st.stop_pixel_noise_threshold = threshold
    return st


def test_oracle_adaptive_sampling_properties(cornell, luts, oracle_lib):
    o = oracle_lib.Oracle(cornell, luts)
    plain = o.render(frames(cornell, scene.parity_settings(3)))
    ada = o.render(frames(cornell, adaptive_settings()))
    aux = o.last_aux
    cnt, conv = aux["sample_count"], aux["converged_sample_count"]
    done = conv >= 0
    assert 0 < done.sum() < done.size, "the test needs both converged and sampling pixels"
    assert (cnt[~done] == N).all()
    assert (conv[done] == cnt[done]).all() and (cnt[done] > 3).all() and (cnt[done] < N).all()
    assert np.array_equal(ada[~done], plain[~done])
    # a pixel converged after c samples holds its c-sample sum scaled to N samples
    mean_ratio = ada[done].sum(-1) / np.maximum(1e-30, plain[done].sum(-1))
    assert np.isfinite(mean_ratio).all()
    assert aux["pixel_converged_count"] == int(done.sum()) and aux["one_ray_active"]
    o.close()


def test_oracle_stop_noise_threshold_properties(cornell, luts, oracle_lib):
    o = oracle_lib.Oracle(cornell, luts)
    plain = o.render(frames(cornell, scene.parity_settings(3)))
    st = o.render(frames(cornell, stop_noise_settings()))
    aux = o.last_aux
    # the stop-noise threshold only counts convergence, it never stops sampling
    assert np.array_equal(st, plain)
    assert (aux["sample_count"] == N).all()
    conv = aux["converged_sample_count"]
    assert 0 < (conv >= 0).sum() < conv.size
    assert aux["pixel_converged_count"] == int((conv >= 0).sum())
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["adaptive", "stop_noise", "adaptive_band"])
def test_gpu_adaptive_sampling_bit_exact(cornell, luts, mode):
    import mpt
    from oracle import oracle as orc
    band = (4, 1, 3) if mode == "adaptive_band" else (1, 0, 1)
    st = stop_noise_settings() if mode == "stop_noise" else adaptive_settings()
    frs = frames(cornell, st, band=band)
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    r.clear_status_buffers()
    for f in frs:
        r.render(f)
    r.synchronize_kernel()
    o = orc.Oracle(cornell, luts)
    c = o.render(frs)
    g = r.framebuffer(abi.FB_COLOR)
    assert np.array_equal(g, c), f"{(g != c).sum()} values differ"
    assert np.array_equal(r.aux_buffer(abi.AUX_SAMPLE_COUNT), o.last_aux["sample_count"])
    assert np.array_equal(r.aux_buffer(abi.AUX_CONVERGED_SAMPLE_COUNT), o.last_aux["converged_sample_count"])
    assert np.array_equal(r.aux_buffer(abi.AUX_SQUARED_LUMINANCE), o.last_aux["squared_luminance"])
    s = r.get_status_buffer_values()
    assert s == {"one_ray_active": o.last_aux["one_ray_active"], "pixel_converged_count": o.last_aux["pixel_converged_count"]}
    assert 0 < s["pixel_converged_count"]
    o.close()
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("max_batch", [3, 12])
@pytest.mark.parametrize("mode", ["adaptive", "adaptive_min5", "stop_noise", "adaptive_band", "adaptive_reset"])
def test_gpu_adaptive_batched_speculative_bit_exact(cornell, luts, mode, max_batch):
    """Adaptive sampling at the reference defaults through batched wavefronts
    (mpt_render_frames): every sample traced, k_accumulate replays CameraRays' reset and gate in
    sample order -- sums, per-pixel counts, converged counts, squared luminance and the status
    values equal the oracle's sequential frames, with the min-samples threshold crossed inside a
    batch, status updates at the end of every 4-sample render() call and a reset mid-run."""
    import mpt
    from oracle import oracle as orc
    band = (4, 1, 3) if mode == "adaptive_band" else (1, 0, 1)
    st = stop_noise_settings() if mode == "stop_noise" else adaptive_settings(min_samples=5 if mode == "adaptive_min5" else 3)
    frs = frames(cornell, st, band=band, last_status=False)
    for k, f in enumerate(frs):
        f.render_settings.do_update_status_buffers = k % 4 == 3
    if mode == "adaptive_reset":
        frs[6].render_settings.need_to_reset = True
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    r.enable_stats(timing=True)
    r.clear_status_buffers()
    r.render_samples(frs, max_batch=max_batch)
    r.synchronize_kernel()
    launches = r.stats().shade_launches
    o = orc.Oracle(cornell, luts)
    c = o.render(frs)
    g = r.framebuffer(abi.FB_COLOR)
    assert np.array_equal(g, c), f"{(g != c).sum()} values differ"
    assert np.array_equal(r.aux_buffer(abi.AUX_SAMPLE_COUNT), o.last_aux["sample_count"])
    assert np.array_equal(r.aux_buffer(abi.AUX_CONVERGED_SAMPLE_COUNT), o.last_aux["converged_sample_count"])
    assert np.array_equal(r.aux_buffer(abi.AUX_SQUARED_LUMINANCE), o.last_aux["squared_luminance"])
    s = r.get_status_buffer_values()
    assert s == {"one_ray_active": o.last_aux["one_ray_active"], "pixel_converged_count": o.last_aux["pixel_converged_count"]}
    if mode != "stop_noise":
        assert (o.last_aux["converged_sample_count"] >= 0).any()
    # batched: one shading launch per bounce per wavefront, not per sample
    assert 0 < launches <= (N // max_batch + (1 if mode == "adaptive_reset" else 0)) * 4 * 2, launches
    o.close()
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("max_batch", [2, 4])
def test_gpu_adaptive_batched_skips_converged_pixels(cornell, luts, max_batch):
    """A speculative batch traces no camera ray for a pixel that converged before the batch began
    (pixel_converged_sample_count != -1 is sticky under enable_adaptive_sampling,
    AdaptiveSampling.h:45-48; CameraRays.h:107-121 rescales it instead): with 0 bounces the path
    queries are exactly the camera rays, so their count is, per batch [j, j + L), L for every pixel
    that had not converged before sample j -- derived from the oracle's converged sample counts (a
    pixel with count c is refused from sample c on) -- and the image still equals the oracle's."""
    import mpt
    from oracle import oracle as orc
    st = adaptive_settings(min_samples=2, threshold=0.8)
    st.nb_bounces = 0
    frs = frames(cornell, st)
    r = mpt.GPURenderer(0)
    r.set_scene(cornell)
    r.set_luts(luts)
    r.enable_stats(timing=False)
    r.render_samples(frs, max_batch=max_batch)
    r.synchronize_kernel()
    rays = r.stats().stage_rays[0]
    o = orc.Oracle(cornell, luts)
    c = o.render(frs)
    conv = o.last_aux["converged_sample_count"].reshape(-1).astype(np.int64)
    o.close()
    g = r.framebuffer(abi.FB_COLOR)
    assert np.array_equal(g, c), f"{(g != c).sum()} values differ"
    assert np.array_equal(r.aux_buffer(abi.AUX_CONVERGED_SAMPLE_COUNT).reshape(-1), conv)
    want = 0
    for j in range(0, N, max_batch):
        L = min(max_batch, N - j)
        live = (conv < 0) | (conv >= j)
        want += L * int(live.sum())
    assert (conv >= 0).sum() > conv.size // 4, "the test needs pixels converging early"
    assert rays == want, (rays, want, N * W * H)
    assert rays < N * W * H
    r.close()
