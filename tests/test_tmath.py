"""The transcendental layer shared by the HIP kernels and the oracle (csrc/tmath.h).

CPU: every function against the correctly rounded float of the platform's double libm
(numpy's float64 ufuncs call it) on random arguments over the ranges the path tracer uses
and beyond, incl. the special values: the single-precision functions (sin, cos, exp, log,
atan2, asin, acos) within their stated ulp bounds -- the accuracy class of the device library's
float functions the reference's GPU build calls -- and pow, still evaluated in double, within 1
ulp and off by one essentially never.
GPU: libmpt's device build of the same code equals the oracle's bit for bit."""
import math

import numpy as np
import pytest

FNS = ["sin", "cos", "exp", "log", "pow", "atan2", "asin", "acos"]
# max ulps from the correctly rounded float (tmath.h: single precision but for pow)
ULP_BOUND = {"sin": 2, "cos": 2, "exp": 1, "log": 1, "pow": 1, "atan2": 3, "asin": 4, "acos": 4}
REF = {"sin": lambda a, b: np.sin(a), "cos": lambda a, b: np.cos(a), "exp": lambda a, b: np.exp(a),
       "log": lambda a, b: np.log(a), "pow": lambda a, b: np.power(a, b), "atan2": lambda a, b: np.arctan2(a, b),
       "asin": lambda a, b: np.arcsin(a), "acos": lambda a, b: np.arccos(a)}
SPECIAL = np.array([0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 2.0, 1e-30, -1e-30, 1e-45, 3e38, -3e38, np.inf, -np.inf, np.nan,
                    math.pi, -math.pi, math.pi / 2, 1e5, 1.00001e5, -1e6, 88.7, 88.8, -103.9, -104.0, 100.0, 0.9999999,
                    -0.9999999, 1.0000001], np.float32)


def args(name, n, seed):
    rng = np.random.default_rng(seed)
    u, v = rng.random(n), rng.random(n)
    if name in ("sin", "cos"):
        a = (u * 2 - 1) * np.where(np.arange(n) % 3 == 0, 1e4, 2 * math.pi)
        b = np.zeros(n)
    elif name == "exp":
        a, b = (u * 2 - 1) * np.where(np.arange(n) % 3 == 0, 110, 10), np.zeros(n)
    elif name == "log":
        a, b = np.where(np.arange(n) % 3 == 0, np.exp((u * 2 - 1) * 85), u * 4), np.zeros(n)
    elif name == "pow":
        a, b = np.where(np.arange(n) % 2 == 0, u, u * 10), np.where(np.arange(n) % 3 == 0, (v * 2 - 1) * 30, v * 5)
    elif name == "atan2":
        a, b = (u * 2 - 1) * np.where(np.arange(n) % 5 == 0, 1e-3, 1), (v * 2 - 1)
    else:
        a, b = np.where(np.arange(n) % 4 == 0, 1 - u * 1e-6, u * 2 - 1), np.zeros(n)
    a, b = a.astype(np.float32), b.astype(np.float32)
    # special values, paired with every other special value for the two-argument functions
    sa, sb = np.meshgrid(SPECIAL, SPECIAL)
    return np.concatenate([a, sa.ravel()]), np.concatenate([b, sb.ravel()])


def ulps(x, y):
    xi = x.view(np.int32).astype(np.int64)
    yi = y.view(np.int32).astype(np.int64)
    xi = np.where(xi < 0, -(2 ** 31) - xi, xi)
    yi = np.where(yi < 0, -(2 ** 31) - yi, yi)
    return np.abs(xi - yi)


def oracle_fn(orc, fn, a, b):
    out = np.zeros_like(a)
    orc.lib().oracle_tmath(fn, a.ctypes.data, b.ctypes.data, out.ctypes.data, len(a))
    return out


@pytest.mark.parametrize("fn,name", list(enumerate(FNS)))
def test_tmath_correctly_rounded(oracle_lib, fn, name):
    a, b = args(name, 2_000_000, fn)
    got = oracle_fn(oracle_lib, fn, a, b)
    with np.errstate(all="ignore"):
        exp = REF[name](a.astype(np.float64), b.astype(np.float64)).astype(np.float32)
    nan = np.isnan(exp)
    assert np.array_equal(np.isnan(got), nan), name
    d = ulps(got[~nan], exp[~nan])
    assert d.max() <= ULP_BOUND[name], (name, int(d.max()))
    if name == "pow":
        # double precision: off by one only within ~1e-14 of a rounding tie, essentially never
        assert np.count_nonzero(d) <= 5, (name, int(np.count_nonzero(d)))
    else:
        # single precision: most results still correctly rounded
        assert np.count_nonzero(d) <= 0.5 * len(d), (name, int(np.count_nonzero(d)))


@pytest.mark.gpu
@pytest.mark.parametrize("fn,name", list(enumerate(FNS)))
def test_tmath_device_equals_oracle(oracle_lib, fn, name):
    import ctypes as C

    import mpt
    L = mpt.lib()
    L.mpt_debug_math.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    a, b = args(name, 1_000_000, 100 + fn)
    gpu = np.zeros_like(a)
    L.mpt_debug_math(fn, a.ctypes.data, b.ctypes.data, gpu.ctypes.data, len(a))
    cpu = oracle_fn(oracle_lib, fn, a, b)
    same = (gpu.view(np.int32) == cpu.view(np.int32)) | (np.isnan(gpu) & np.isnan(cpu))
    bad = np.flatnonzero(~same)
    assert len(bad) == 0, (name, len(bad), [(float(a[i]), float(b[i]), float(gpu[i]), float(cpu[i])) for i in bad[:3]])


@pytest.mark.gpu
@pytest.mark.parametrize("dev_fn,fn,name", [(8, 0, "sin"), (9, 1, "cos")])
def test_tmath_device_sincos_equals_oracle(oracle_lib, dev_fn, fn, name):
    """psincos (one range reduction for the sine and cosine the samplers need together)
    gives psin / pcos bit for bit."""
    import ctypes as C

    import mpt
    L = mpt.lib()
    L.mpt_debug_math.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    a, b = args(name, 1_000_000, 200 + fn)
    gpu = np.zeros_like(a)
    L.mpt_debug_math(dev_fn, a.ctypes.data, b.ctypes.data, gpu.ctypes.data, len(a))
    cpu = oracle_fn(oracle_lib, fn, a, b)
    same = (gpu.view(np.int32) == cpu.view(np.int32)) | (np.isnan(gpu) & np.isnan(cpu))
    assert same.all(), (name, int((~same).sum()))
