"""C-ABI checks that need no GPU: the library loads, exports every symbol of
include/mpt.h, struct layouts match the reference PODs, host-side helpers."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import mpt
from mpt import abi, partition

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "mpt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mpt_[a-z_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = mpt.lib()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    assert sorted(names) == sorted(mpt.SYMBOLS)


def test_struct_sizes_match_reference_pods():
    # RendererMaterial 332 B, HIPRTRenderSettings 304 B, WorldSettings 200 B, HIPRTCamera 196 B
    assert abi.check_sizes() == abi.ABI_SIZES
    lib_sizes = mpt.abi_sizes()
    assert lib_sizes["Material"] == C.sizeof(abi.Material)
    assert lib_sizes["RenderSettings"] == C.sizeof(abi.RenderSettings)
    assert lib_sizes["WorldSettings"] == C.sizeof(abi.WorldSettings)
    assert lib_sizes["Camera"] == C.sizeof(abi.Camera)
    assert lib_sizes["Frame"] == C.sizeof(abi.Frame)
    assert lib_sizes["Scene"] == C.sizeof(abi.Scene)
    assert lib_sizes["Stats"] == C.sizeof(abi.Stats)


def test_version_and_error_reporting_without_gpu():
    L = mpt.lib()
    assert L.mpt_version() >= 1
    h = C.c_void_p()
    rc = L.mpt_create(0, None, C.byref(h))
    if rc == 0:            # a GPU is present (GPU box): creation works
        L.mpt_destroy(h)
        return
    assert rc == -2
    assert b"device" in L.mpt_last_error()
    with pytest.raises(mpt.MptError):
        mpt.GPURenderer(0)


def test_null_arguments_rejected():
    L = mpt.lib()
    assert L.mpt_create(0, None, None) == -1
    assert L.mpt_render_frame(None, None) == -1
    assert L.mpt_render_frames(None, None, 0, 0) == -1
    assert L.mpt_upload_scene(None, None) == -1
    assert L.mpt_destroy(None) == 0


@pytest.mark.parametrize("H,bh,n", [(1080, 8, 1), (1080, 8, 2), (1080, 8, 3), (1080, 16, 8), (37, 4, 5), (7, 8, 4)])
def test_partition_rows_cover_frame_once(H, bh, n):
    seen = np.zeros(H, int)
    for k in range(n):
        ys = partition.rows_of(H, bh, k, n)
        assert mpt.partition_rows(H, bh, k, n) == len(ys)
        seen[ys] += 1
    assert (seen == 1).all()


def test_assemble_roundtrip():
    rng = np.random.default_rng(0)
    H, W, bh, n = 45, 6, 4, 3
    img = rng.random((H, W, 3)).astype(np.float32)
    mr = partition.max_rows(H, bh, n)
    parts = []
    for k in range(n):
        ys = partition.rows_of(H, bh, k, n)
        p = np.full((mr, W, 3), -1.0, np.float32)
        p[: len(ys)] = img[ys]
        parts.append(p)
    assert np.array_equal(partition.assemble(parts, H, bh), img)


def vose_reference(rgba):
    """Pure-Python restatement of Image32Bit::compute_alias_table (Image.cpp:579-659)."""
    h, w = rgba.shape[:2]
    lum = (rgba[..., 0].astype(np.float32) * np.float32(0.3086) + rgba[..., 1].astype(np.float32) * np.float32(0.6094)
           + rgba[..., 2].astype(np.float32) * np.float32(0.0820)).astype(np.float32).ravel()
    L = [float(x) for x in lum]
    total = 0.0
    for x in L:
        total += x
    L = [x / total * (w * h) for x in L]
    small = [i for i, x in enumerate(L) if x < 1.0]
    large = [i for i, x in enumerate(L) if x >= 1.0]
    p = np.zeros(w * h, np.float32)
    a = np.arange(w * h, dtype=np.int32)
    while small and large:
        s = small.pop(0)
        l = large.pop(0)
        p[s] = L[s]
        a[s] = l
        L[l] = (L[l] + L[s]) - 1.0
        (large if L[l] > 1.0 else small).append(l)
    for i in large + small:
        p[i] = 1.0
    return p, a, np.float32(total)


@pytest.mark.parametrize("shape,seed", [((8, 16), 0), ((16, 32), 1), ((5, 7), 2)])
def test_alias_table_matches_vose_restatement(shape, seed):
    rng = np.random.default_rng(seed)
    rgba = np.concatenate([rng.random(shape + (3,)) ** 3 * 10, np.ones(shape + (1,))], -1).astype(np.float32)
    env = mpt.build_envmap(rgba)
    p, a, s = vose_reference(rgba)
    assert np.array_equal(env["probas"], p)
    assert np.array_equal(env["alias"], a)
    assert env["sum"] == s
    # the table reproduces the luminance distribution exactly (in expectation)
    n = shape[0] * shape[1]
    prob = env["probas"].astype(np.float64) / n
    for i in range(n):
        prob[env["alias"][i]] += (1.0 - env["probas"][i]) / n
    lum = (rgba[..., :3] @ np.array([0.3086, 0.6094, 0.0820])).ravel()
    assert np.allclose(prob, lum / lum.sum(), atol=1e-6)


@pytest.mark.parametrize("shape,seed", [((8, 16), 0), ((5, 7), 2)])
def test_envmap_cdf_matches_restatement(shape, seed):
    """Image32Bit::compute_cdf (Image.cpp:553-574): float32 running sum of the texel
    luminances ((0 + r w0) + g w1) + b w2, row-major; total = last element."""
    rng = np.random.default_rng(seed)
    rgba = np.concatenate([rng.random(shape + (3,)) ** 3 * 10, np.ones(shape + (1,))], -1).astype(np.float32)
    env = mpt.build_envmap(rgba)
    f = np.float32
    lum = ((f(0) + rgba[..., 0] * f(0.3086)).astype(f) + rgba[..., 1] * f(0.6094)).astype(f) + rgba[..., 2] * f(0.0820)
    cdf = np.add.accumulate(lum.astype(f).ravel(), dtype=f)
    assert np.array_equal(env["cdf"], cdf)
    assert env["cdf_sum"] == cdf[-1]
