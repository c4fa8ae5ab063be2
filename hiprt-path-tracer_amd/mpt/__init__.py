"""mpt -- MI355X path tracer: Python binding of libmpt.so (include/mpt.h).

``GPURenderer`` mirrors the launch surface of the reference's
``GPURenderer`` (src/Renderer/GPURenderer.h:69-260): a scene is uploaded once, the
envmap / LUTs are set, and every ``render()`` call enqueues one sample per pixel on the
context's HIP stream (``GPURenderer::render``, GPURenderer.cpp:245-271), accumulating
into the 'pixels' sum buffer and the denoiser AOVs.

There is no CPU fallback: if libmpt.so is missing or no HIP device exists, the
constructor raises.  Build the library with ``python -m mpt._build`` or
``__graft_entry__.build()``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi
from . import scene
from ._build import LIB_PATH

__all__ = ["abi", "scene", "lib", "GPURenderer", "MptError", "build_envmap", "partition_rows"]

SYMBOLS = [
    "mpt_last_error", "mpt_version", "mpt_abi_sizes", "mpt_create", "mpt_destroy", "mpt_upload_scene",
    "mpt_update_materials", "mpt_set_envmap", "mpt_build_alias_table", "mpt_set_luts", "mpt_resize",
    "mpt_render_frame", "mpt_render_frames", "mpt_synchronize", "mpt_query_done", "mpt_get_framebuffer", "mpt_partition_rows",
    "mpt_enable_stats", "mpt_get_stats", "mpt_trace_closest", "mpt_trace_any", "mpt_clear_status",
    "mpt_query_status", "mpt_get_aux_buffer", "mpt_build_envmap_cdf", "mpt_set_envmap_cdf", "mpt_set_halo_exchange",
    "mpt_set_halo_native", "mpt_halo_plan", "mpt_set_pipeline",
    "mpt_bake_lut", "mpt_png_unfilter", "mpt_device_info", "mpt_gather", "mpt_comm_unique_id", "mpt_comm_init",
    "mpt_comm_gather", "mpt_jpeg_decode", "mpt_hdr_decode",
]


class MptError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mpt error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> C.CDLL:
    """Loads the in-tree libmpt.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("MPT_LIB_PATH", str(LIB_PATH))   # development variants
    if not os.path.exists(path):
        raise ImportError(f"libmpt.so not found at {path}; run __graft_entry__.build() (no CPU fallback)")
    # One HIP runtime per process.  The torch wheel ships its own libamdhip64 (same SONAME,
    # libamdhip64.so.7) next to libc10_hip; loading libmpt first would map /opt/rocm's copy
    # and torch's would then find no device.  Loading torch first makes libmpt bind to the
    # runtime torch already mapped, so libmpt buffers, torch tensors and RCCL share one
    # runtime (measured: same bit-exact results and the same C3 throughput on either).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, i32, f32 = C.c_void_p, C.c_int32, C.c_float
    L.mpt_last_error.restype = C.c_char_p
    L.mpt_abi_sizes.argtypes = [vp, C.c_int]
    L.mpt_create.argtypes = [C.c_int, vp, C.POINTER(vp)]
    L.mpt_destroy.argtypes = [vp]
    L.mpt_upload_scene.argtypes = [vp, C.POINTER(abi.Scene)]
    L.mpt_update_materials.argtypes = [vp, vp, i32]
    L.mpt_set_envmap.argtypes = [vp, vp, i32, i32, vp, vp, f32]
    L.mpt_build_alias_table.argtypes = [vp, i32, i32, vp, vp, vp]
    L.mpt_set_luts.argtypes = [vp, C.POINTER(abi.Luts)]
    L.mpt_resize.argtypes = [vp, i32, i32]
    L.mpt_render_frame.argtypes = [vp, C.POINTER(abi.Frame)]
    L.mpt_render_frames.argtypes = [vp, C.POINTER(abi.Frame), i32, i32]
    L.mpt_synchronize.argtypes = [vp]
    L.mpt_query_done.argtypes = [vp, C.POINTER(C.c_int)]
    L.mpt_get_framebuffer.argtypes = [vp, C.c_int, vp, C.c_int]
    L.mpt_partition_rows.argtypes = [i32, i32, i32, i32]
    L.mpt_enable_stats.argtypes = [vp, C.c_int, C.c_int]
    L.mpt_get_stats.argtypes = [vp, C.POINTER(abi.Stats)]
    L.mpt_trace_closest.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp, C.c_int]
    L.mpt_trace_any.argtypes = [vp, vp, vp, i32, vp, C.c_int]
    L.mpt_png_unfilter.argtypes = [vp, C.c_int64, vp, i32, i32, i32]
    L.mpt_device_info.argtypes = [C.c_int, vp, i32, vp, i32, vp]
    L.mpt_build_envmap_cdf.argtypes = [vp, i32, i32, vp, vp]
    L.mpt_set_envmap_cdf.argtypes = [vp, vp, f32]
    L.mpt_clear_status.argtypes = [vp]
    L.mpt_query_status.argtypes = [vp, C.POINTER(abi.Status)]
    L.mpt_get_aux_buffer.argtypes = [vp, C.c_int, vp, C.c_int]
    L.mpt_set_halo_exchange.argtypes = [vp, abi.HaloExchangeFn, vp]
    L.mpt_set_halo_native.argtypes = [vp, C.c_int32]
    L.mpt_set_pipeline.argtypes = [vp, C.c_int32]
    L.mpt_halo_plan.argtypes = [i32, i32, i32, i32, i32, i32, C.POINTER(abi.HaloOp), i32]
    L.mpt_bake_lut.argtypes = [vp, C.c_int, i32, i32, i32, i32, vp, C.c_int]
    L.mpt_gather.argtypes = [C.POINTER(vp), i32, i32, C.c_int, vp, C.c_int]
    L.mpt_comm_unique_id.argtypes = [vp, i32]
    L.mpt_comm_init.argtypes = [vp, i32, i32, vp]
    L.mpt_comm_gather.argtypes = [vp, i32, C.c_int, vp, C.c_int]
    L.mpt_jpeg_decode.argtypes = [vp, C.c_int64, i32, vp, C.c_int64, vp, vp, vp]
    L.mpt_hdr_decode.argtypes = [vp, C.c_int64, i32, vp, C.c_int64, vp, vp]
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise MptError(rc, lib().mpt_last_error().decode(errors="replace"))


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def abi_sizes():
    out = np.zeros(7, np.int32)
    _check(lib().mpt_abi_sizes(_p(out), 7))
    return dict(zip(["Material", "RenderSettings", "WorldSettings", "Camera", "Frame", "Scene", "Stats"], out.tolist()))


def device_info(device=0):
    """(name, gfx arch, compute units) of a HIP device (mpt_device_info)."""
    name, arch, cus = C.create_string_buffer(256), C.create_string_buffer(64), C.c_int32()
    _check(lib().mpt_device_info(device, name, 256, arch, 64, C.byref(cus)))
    return name.value.decode(errors="replace"), arch.value.decode(errors="replace"), int(cus.value)


def build_id():
    """First 16 hex digits of the SHA-256 of the loaded libmpt.so (identifies the build a line ran)."""
    import hashlib
    return hashlib.sha256(open(lib()._name, "rb").read()).hexdigest()[:16]


def partition_rows(res_y, band_height, band_index, band_count):
    return lib().mpt_partition_rows(res_y, band_height, band_index, band_count)


def halo_plan(res_y, band_height, band_count, band_index, halo_rows, n_buffers=1):
    """mpt_halo_plan: the library's halo-exchange operations for one band, in issue order, as
    (peer, 'send' | 'recv', buffer, row_lo, row_hi) tuples (host only, no device needed)."""
    args = (res_y, band_height, band_count, band_index, halo_rows, n_buffers)
    n = lib().mpt_halo_plan(*args, None, 0)
    _check(min(n, 0))
    ops = (abi.HaloOp * max(n, 1))()
    m = lib().mpt_halo_plan(*args, ops, n)
    _check(min(m, 0))
    return [(o.peer, "recv" if o.recv else "send", o.buffer, o.row_lo, o.row_hi) for o in ops[:m]]


GATHER_AUX = 16   # mpt.h MPT_GATHER_AUX: gather kind of an MPT_AUX_* buffer


def _gather_out(f, kind):
    if kind >= GATHER_AUX:
        return np.zeros((f.res_y, f.res_x), np.float32 if kind == GATHER_AUX + abi.AUX_SQUARED_LUMINANCE else np.int32)
    return np.zeros((f.res_y, f.res_x, 3), np.float32)


def gather(renderers, root=0, kind=abi.FB_COLOR):
    """mpt_gather: the whole frame of buffer `kind` from the renderers that render the row
    partitions band_index = 0..n-1 of one frame (one process; peer copies between GPUs) ->
    host array [res_y, res_x(, 3)]."""
    f = renderers[root].frame
    out = _gather_out(f, kind)
    hs = (C.c_void_p * len(renderers))(*[r.h for r in renderers])
    _check(lib().mpt_gather(hs, len(renderers), root, kind, _p(out), 0))
    return out


def comm_unique_id() -> bytes:
    """mpt_comm_unique_id (rank 0; share the bytes with the other ranks out of band)."""
    buf = (C.c_uint8 * 128)()
    _check(lib().mpt_comm_unique_id(buf, 128))
    return bytes(buf)


def build_envmap(rgba):
    """float32 [H, W, 4] (already flipped as the reference's loader does) -> envmap dict
    with the alias table of Image32Bit::compute_alias_table (Image.cpp:579-659)."""
    rgba = np.ascontiguousarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    probas = np.zeros(h * w, np.float32)
    alias = np.full(h * w, -1, np.int32)
    s = np.zeros(1, np.float32)
    _check(lib().mpt_build_alias_table(_p(rgba), w, h, _p(probas), _p(alias), _p(s)))
    alias = np.where(alias < 0, np.arange(h * w, dtype=np.int32), alias).astype(np.int32)
    # ESS_BINARY_SEARCH: luminance CDF, Image32Bit::compute_cdf (Image.cpp:553-574)
    cdf = np.zeros(h * w, np.float32)
    cs = np.zeros(1, np.float32)
    _check(lib().mpt_build_envmap_cdf(_p(rgba), w, h, _p(cdf), _p(cs)))
    return {"rgba": rgba, "probas": probas, "alias": alias, "width": w, "height": h, "sum": float(s[0]),
            "cdf": cdf, "cdf_sum": float(cs[0])}


class GPURenderer:
    """One renderer context on one GPU (GPURenderer.h:69)."""

    def __init__(self, device: int = 0, stream: int | None = None):
        L = lib()
        h = C.c_void_p()
        _check(L.mpt_create(device, C.c_void_p(stream) if stream else None, C.byref(h)))
        self.h = h
        self.device = device
        self.frame = None
        self._n_mats = 0

    # --- scene / resources -----------------------------------------------------
    def set_scene(self, sd: "scene.SceneData"):
        """GPURenderer::set_scene (GPURenderer.cpp:1052-1130)."""
        s = sd.to_abi()
        _check(lib().mpt_upload_scene(self.h, C.byref(s)))
        self._n_mats = len(sd.materials)

    def update_materials(self, materials):
        arr = (abi.Material * len(materials))(*materials)
        _check(lib().mpt_update_materials(self.h, C.cast(arr, C.c_void_p), len(materials)))

    def set_envmap(self, env):
        """GPURenderer::set_envmap (GPURenderer.cpp:1136-1174); env from build_envmap() or None."""
        if env is None:
            _check(lib().mpt_set_envmap(self.h, None, 0, 0, None, None, 0.0))
            return
        self._env = env
        _check(lib().mpt_set_envmap(self.h, _p(env["rgba"]), env["width"], env["height"], _p(env["probas"]),
                                    _p(env["alias"]), env["sum"]))
        if env.get("cdf") is not None:
            _check(lib().mpt_set_envmap_cdf(self.h, _p(env["cdf"]), env["cdf_sum"]))

    def set_luts(self, luts=None):
        luts = luts if luts is not None else scene.load_luts()
        L = scene.luts_to_abi(luts)
        _check(lib().mpt_set_luts(self.h, C.byref(L)))

    def resize(self, w, h):
        _check(lib().mpt_resize(self.h, w, h))

    def set_halo_exchange(self, exchange):
        """ReSTIR DI across a row partition (mpt.h MptHaloExchange): exchange(x) is called
        with an abi.HaloExchange at every exchange point of mpt_render_frame and fills the
        halo rows (mpt.partition.TorchHaloExchange / LocalHaloGroup).  None removes it."""
        if exchange is None:
            self._halo_cb = None
            _check(lib().mpt_set_halo_exchange(self.h, abi.HaloExchangeFn(), None))
            return

        def _cb(_user, xp):
            try:
                exchange(xp.contents)
                return 0
            except BaseException as e:   # reported by render(); never unwinds through C
                self._halo_error = e
                return 1

        self._halo_error = None
        self._halo_cb = abi.HaloExchangeFn(_cb)   # kept alive with the renderer
        _check(lib().mpt_set_halo_exchange(self.h, self._halo_cb, None))

    def set_halo_native(self, mode: int):
        """mpt_set_halo_native: 1 the library's RCCL halo exchange (after comm_init), 2 the one-GPU
        rehearsal (timing only), 0 off."""
        self._halo_cb = None
        _check(lib().mpt_set_halo_native(self.h, int(mode)))

    def set_pipeline(self, mode: int):
        """mpt_set_pipeline: 1 the bounce pipeline of single-stream wavefronts, 0 in line."""
        _check(lib().mpt_set_pipeline(self.h, int(mode)))

    # --- frames --------------------------------------------------------------------
    def render(self, frame: "abi.Frame"):
        """Enqueues one sample per pixel (asynchronous)."""
        rc = lib().mpt_render_frame(self.h, C.byref(frame))
        err = getattr(self, "_halo_error", None)
        if err is not None:
            self._halo_error = None
            raise MptError(rc or -1, f"halo exchange failed: {err!r}") from err
        _check(rc)
        self.frame = frame

    def render_samples(self, frames, max_batch: int = 0):
        """GPURenderer::render with samples_per_frame = len(frames): enqueues every frame's
        sample; runs of batchable frames (mpt.h mpt_render_frames) are traced as one
        wavefront of up to max_batch samples per pixel (0: the library maximum)."""
        if not frames:
            return
        arr = (abi.Frame * len(frames))(*frames)
        rc = lib().mpt_render_frames(self.h, arr, len(frames), int(max_batch))
        err = getattr(self, "_halo_error", None)
        if err is not None:
            self._halo_error = None
            raise MptError(rc or -1, f"halo exchange failed: {err!r}") from err
        _check(rc)
        self.frame = frames[-1]

    def synchronize_kernel(self):
        _check(lib().mpt_synchronize(self.h))

    def frame_render_done(self) -> bool:
        d = C.c_int()
        _check(lib().mpt_query_done(self.h, C.byref(d)))
        return bool(d.value)

    def rows(self):
        f = self.frame
        return partition_rows(f.res_y, f.band_height, f.band_index, f.band_count)

    def framebuffer(self, kind=abi.FB_COLOR):
        """Copies the partition's rows (band-major, increasing y) -> float32 [rows, W, 3]."""
        f = self.frame
        out = np.zeros((self.rows(), f.res_x, 3), np.float32)
        _check(lib().mpt_get_framebuffer(self.h, kind, _p(out), 0))
        return out

    def framebuffer_to_device(self, kind, dev_ptr: int):
        _check(lib().mpt_get_framebuffer(self.h, kind, C.c_void_p(dev_ptr), 1))

    # --- one process per GPU (RCCL, mpt_comm_*) ----------------------------------------
    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().mpt_comm_init(self.h, nranks, rank, buf))
        self.comm_rank = rank

    def comm_gather(self, root=0, kind=abi.FB_COLOR):
        """mpt_comm_gather (collective): the whole frame on the root (host array), None elsewhere."""
        out = _gather_out(self.frame, kind)
        _check(lib().mpt_comm_gather(self.h, root, kind, _p(out), 0))
        return out if self.comm_rank == root else None

    # --- status buffers / adaptive sampling (GPURenderer.cpp:269-283) ---------------
    def clear_status_buffers(self):
        """internal_update_clear_device_status_buffers: once per displayed frame."""
        _check(lib().mpt_clear_status(self.h))

    def get_status_buffer_values(self) -> dict:
        """copy_status_buffers + get_status_buffer_values (StatusBuffersValues)."""
        st = abi.Status()
        _check(lib().mpt_query_status(self.h, C.byref(st)))
        return {"one_ray_active": bool(st.one_ray_active), "pixel_converged_count": int(st.pixel_converged_count)}

    def aux_buffer(self, kind):
        """MPT_AUX_* buffer of the partition -> [rows, W] (int32, or float32 for squared luminance)."""
        f = self.frame
        if kind in (abi.AUX_RESTIR_OUTPUT, abi.AUX_RESTIR_OTHER, abi.AUX_RESTIR_INITIAL):
            # frame-sized reservoirs -> [H, W, 12] float32 (M and triangle as int bits in 0 / 3)
            out = np.zeros((f.res_y, f.res_x, 12), np.float32)
        else:
            out = np.zeros((self.rows(), f.res_x), np.float32 if kind == abi.AUX_SQUARED_LUMINANCE else np.int32)
        _check(lib().mpt_get_aux_buffer(self.h, kind, _p(out), 0))
        return out

    # --- stats / queries -------------------------------------------------------
    def enable_stats(self, timing=True, instrumented=False):
        _check(lib().mpt_enable_stats(self.h, int(timing), int(instrumented)))

    def stats(self) -> "abi.Stats":
        s = abi.Stats()
        _check(lib().mpt_get_stats(self.h, C.byref(s)))
        return s

    def trace_closest(self, rays, last_hit=None):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = len(rays)
        prim = np.empty(n, np.int32)
        t, u, v = (np.empty(n, np.float32) for _ in range(3))
        lh = None if last_hit is None else np.ascontiguousarray(last_hit, np.int32)
        _check(lib().mpt_trace_closest(self.h, _p(rays), _p(lh), n, _p(prim), _p(t), _p(u), _p(v), 0))
        return prim, t, u, v

    def trace_any(self, rays, last_hit=None):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        n = len(rays)
        occ = np.empty(n, np.uint8)
        lh = None if last_hit is None else np.ascontiguousarray(last_hit, np.int32)
        _check(lib().mpt_trace_any(self.h, _p(rays), _p(lh), n, _p(occ), 0))
        return occ.astype(bool)

    # --- LUT baker (GPUBaker, Renderer/Baker/GPUBaker.cpp:35-97) -------------------------
    def bake_lut(self, kind, width, height, depth=1, samples=65536):
        """abi.BAKE_* table -> float32 [depth, height, width], rows as the reference's baker
        writes them (the renderer's LUTs are each slice flipped: out[:, ::-1])."""
        out = np.zeros((depth, height, width), np.float32)
        _check(lib().mpt_bake_lut(self.h, kind, width, height, depth, samples, _p(out), 0))
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().mpt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
