"""Development: GPU transcendental layer vs the host's libm, (float)f((double)x)."""
import ctypes as C
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hiprt-path-tracer_amd"))
import mpt  # noqa: E402

L = mpt.lib()
L.mpt_debug_math.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
rng = np.random.default_rng(1)
n = 4_000_000
cases = {
    0: ("sin", rng.random(n).astype(np.float32) * np.float32(2 * math.pi), None, lambda a, b: np.sin(a)),
    1: ("cos", rng.random(n).astype(np.float32) * np.float32(2 * math.pi), None, lambda a, b: np.cos(a)),
    2: ("exp", (rng.random(n) * 20 - 15).astype(np.float32), None, lambda a, b: np.exp(a)),
    3: ("log", (rng.random(n) * 4).astype(np.float32), None, lambda a, b: np.log(a)),
    4: ("pow", rng.random(n).astype(np.float32), (rng.random(n) * 5).astype(np.float32), lambda a, b: np.power(a, b)),
    5: ("atan2", (rng.random(n) * 2 - 1).astype(np.float32), (rng.random(n) * 2 - 1).astype(np.float32), lambda a, b: np.arctan2(a, b)),
    6: ("asin", (rng.random(n) * 2 - 1).astype(np.float32), None, lambda a, b: np.arcsin(a)),
    7: ("acos", (rng.random(n) * 2 - 1).astype(np.float32), None, lambda a, b: np.arccos(a)),
}
for fn, (name, a, b, ref) in cases.items():
    bb = b if b is not None else np.zeros(n, np.float32)
    out = np.zeros(n, np.float32)
    L.mpt_debug_math(fn, a.ctypes.data, bb.ctypes.data, out.ctypes.data, n)
    # numpy float64 ufuncs call the platform libm (as the oracle's std:: functions do)
    exp = ref(a.astype(np.float64), bb.astype(np.float64)).astype(np.float32)
    bad = np.flatnonzero(out != exp)
    print(f"{name}: {len(bad)} / {n} float results differ", [(float(a[i]), float(bb[i]), float(out[i]), float(exp[i])) for i in bad[:3]], flush=True)
