"""TEST INFRASTRUCTURE ONLY: ctypes driver of the CPU parity oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
See oracle.cpp for what is restated and the parity status ("parity unpinned"
against the reference itself; BSDF layers pinned to the reference's baked LUTs).
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
from mpt import abi, scene as mscene  # noqa: E402

LIB_PATH = os.path.join(HERE, "liboracle.so")
# the same restatement with the C library's float transcendentals (sinf, powf, ...: what the
# reference's CPU build calls) instead of the tmath.h layer it shares with the product
LIBM_PATH = os.path.join(HERE, "liboracle_libm.so")


def build(force=False, variant=None):
    srcs = [os.path.join(HERE, f) for f in ("oracle.cpp", "oracle_math.h", "oracle_bsdf.h", "oracle_restir.h", "Makefile",
                                            os.path.join("..", "include", "mpt.h"),
                                            os.path.join("..", "hiprt-path-tracer_amd", "csrc", "tmath.h"))]
    path = LIBM_PATH if variant == "libm" else LIB_PATH
    stale = os.path.exists(path) and any(os.path.getmtime(f) > os.path.getmtime(path) for f in srcs if os.path.exists(f))
    if force or stale or not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", HERE, os.path.basename(path)])
    return path


_libs = {}


def lib(variant=None):
    if variant not in _libs:
        L = C.CDLL(build(variant=variant))
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(abi.Scene), C.POINTER(abi.Luts), C.c_void_p, C.c_int, C.c_int,
                                    C.c_void_p, C.c_void_p, C.c_float]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_keep_state.argtypes = [C.c_void_p, C.c_int]
        L.oracle_gbuffer_history.argtypes = [C.c_void_p, C.POINTER(abi.Frame), C.c_int, C.c_int]
        L.oracle_set_envmap_cdf.argtypes = [C.c_void_p, C.c_void_p, C.c_float]
        L.oracle_trace_closest.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p]
        L.oracle_render.argtypes = [C.c_void_p, C.POINTER(abi.Frame), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_bsdf_eval.argtypes = [C.POINTER(abi.Material), C.POINTER(abi.Material), C.POINTER(abi.Luts), C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_bsdf_sample.argtypes = [C.POINTER(abi.Material), C.POINTER(abi.Material), C.POINTER(abi.Luts),
                                         C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.c_void_p]
        L.oracle_directional_albedo.argtypes = [C.POINTER(abi.Material), C.POINTER(abi.Material), C.POINTER(abi.Luts),
                                                C.c_int, C.c_float, C.c_int, C.c_uint32, C.c_void_p]
        L.oracle_wang_hash.restype = C.c_uint32
        L.oracle_wang_hash.argtypes = [C.c_uint32]
        L.oracle_xorshift.argtypes = [C.c_uint32, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_tmath.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.oracle_bake.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        _libs[variant] = L
    return _libs[variant]


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Oracle:
    """CPU oracle bound to one scene (+ LUTs, + optional envmap)."""

    def __init__(self, scene_data, luts=None, envmap=None, keep_state=False, variant=None):
        """variant "libm": the restatement with the C library's float transcendentals."""
        self.L = lib(variant)
        self.sd = scene_data
        self.luts = luts if luts is not None else mscene.load_luts()
        self._abi_scene = scene_data.to_abi()
        self._abi_luts = mscene.luts_to_abi(self.luts)
        self.env = envmap
        if envmap is not None:
            self._env = (np.ascontiguousarray(envmap["rgba"], np.float32), np.ascontiguousarray(envmap["probas"], np.float32),
                         np.ascontiguousarray(envmap["alias"], np.int32))
            ew, eh, es = envmap["width"], envmap["height"], envmap["sum"]
            ptrs = (_p(self._env[0]), ew, eh, _p(self._env[1]), _p(self._env[2]), es)
        else:
            ptrs = (None, 0, 0, None, None, 0.0)
        self.h = self.L.oracle_create(C.byref(self._abi_scene), C.byref(self._abi_luts), *ptrs)
        if envmap is not None and envmap.get("cdf") is not None:
            self._cdf = np.ascontiguousarray(envmap["cdf"], np.float32)
            self.L.oracle_set_envmap_cdf(self.h, _p(self._cdf), envmap["cdf_sum"])
        if keep_state:
            self.L.oracle_keep_state(self.h, 1)

    def gbuffer_history(self, frames, nthreads=0):
        """Sets the kept ReSTIR DI state to what rendering `frames` leaves for a later
        reset-to-sample-0 run: their G-buffer (oracle_gbuffer_history), without rendering them."""
        arr = (abi.Frame * len(frames))(*frames)
        if self.L.oracle_gbuffer_history(self.h, arr, len(frames), nthreads) != 0:
            raise RuntimeError("oracle_gbuffer_history: needs keep_state and whole-frame ReSTIR DI frames without adaptive sampling")

    def reset_state(self, keep=True):
        """Drops the kept ReSTIR DI state (a fresh renderer); keeps state from then on if keep."""
        self.L.oracle_keep_state(self.h, 1 if keep else 0)

    def close(self):
        if self.h:
            self.L.oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trace_closest(self, rays, last_hit=None):
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        prim = np.empty(n, np.int32)
        t = np.empty(n, np.float32)
        u = np.empty(n, np.float32)
        v = np.empty(n, np.float32)
        lh = np.ascontiguousarray(last_hit, np.int32) if last_hit is not None else None
        self.L.oracle_trace_closest(self.h, _p(rays), _p(lh), n, _p(prim), _p(t), _p(u), _p(v))
        return prim, t, u, v

    def render(self, frames, nthreads=0, aov=False):
        """frames: list of abi.Frame (one spp each, same partition). Returns sums (H_part, W, 3)."""
        f0 = frames[0]
        rows = mpt_rows(f0.res_y, f0.band_height, f0.band_index, f0.band_count)
        n = rows * f0.res_x
        out = np.zeros((n, 3), np.float32)
        alb = np.zeros((n, 3), np.float32) if aov else None
        nrm = np.zeros((n, 3), np.float32) if aov else None
        arr = (abi.Frame * len(frames))(*frames)
        rays = np.zeros(2, np.uint64)
        # adaptive-sampling buffers and status values (AuxiliaryBuffers / StatusBuffersValues),
        # reported in last_aux after the call
        cnt = np.zeros(n, np.int32)
        sql = np.zeros(n, np.float32)
        conv = np.full(n, -1, np.int32)
        status = np.zeros(4, np.uint32)
        rc = self.L.oracle_render(self.h, arr, len(frames), _p(out), _p(alb), _p(nrm), _p(rays), nthreads,
                                 _p(cnt), _p(sql), _p(conv), _p(status))
        if rc != 0:
            raise RuntimeError("oracle_render failed: %d (unsupported option)" % rc)
        self.last_rays = (int(rays[0]), int(rays[1]))
        self.last_aux = {"sample_count": cnt.reshape(rows, f0.res_x), "squared_luminance": sql.reshape(rows, f0.res_x),
                         "converged_sample_count": conv.reshape(rows, f0.res_x),
                         "one_ray_active": bool(status[1]), "pixel_converged_count": int(status[0])}
        out = out.reshape(rows, f0.res_x, 3)
        if aov:
            return out, alb.reshape(rows, f0.res_x, 3), nrm.reshape(rows, f0.res_x, 3)
        return out


def mpt_rows(res_y, band_height, band_index, band_count):
    return sum(1 for y in range(res_y) if (y // band_height) % band_count == band_index)


def bsdf_eval(mat, all_mats, luts_abi, override, view, normal, light):
    out = np.zeros(3, np.float32)
    pdf = np.zeros(1, np.float32)
    v, n, l = (np.ascontiguousarray(x, np.float32) for x in (view, normal, light))
    arr = (abi.Material * len(all_mats))(*all_mats)
    lib().oracle_bsdf_eval(C.byref(mat), arr, C.byref(luts_abi), override, _p(v), _p(n), _p(l), _p(out), _p(pdf))
    return out, float(pdf[0])


def directional_albedo(mat, luts_abi, cos_theta_o, n, seed=1, override=0):
    out = np.zeros(3, np.float32)
    arr = (abi.Material * 1)(mat)
    lib().oracle_directional_albedo(C.byref(mat), arr, C.byref(luts_abi), override, cos_theta_o, n, seed, _p(out))
    return out


def xorshift(seed, n):
    u = np.zeros(n, np.uint32)
    f = np.zeros(n, np.float32)
    lib().oracle_xorshift(seed, n, _p(u), _p(f))
    return u, f


def wang_hash(s):
    return lib().oracle_wang_hash(s)


def bake(kind, width, height, depth=1, samples=65536):
    """oracle_bake: the reference baker's table (GPUBaker.cpp:35-97) as float32 [depth, height, width]."""
    out = np.zeros((depth, height, width), np.float32)
    if lib().oracle_bake(kind, width, height, depth, samples, _p(out)) != 0:
        raise ValueError("bad bake arguments")
    return out
