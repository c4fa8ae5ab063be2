"""bench.py's wavefront sizing (CPU only): samples per wavefront for path tracing and for ReSTIR DI
(profiles/r06ab_c3_batch_ab.json, r06ae / r06as_c4_batch_ab.json, r06v_c4_band_batch_ab.json)."""
import importlib.util
import os
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _batch(K, want, max_batch):
    # bench.py: the divisor of K nearest to `want` (ties to the larger)
    return min((d for d in range(1, min(max_batch, K) + 1) if K % d == 0), key=lambda d: (abs(d - want), -d))


def test_path_tracing_wavefronts():
    b = _bench()
    a = types.SimpleNamespace(workload="c3")
    px = 1920 * 1080
    want = b.restir_band_want(a, 256, b.TARGET_PATHS / px, 1)
    assert want == 64 and _batch(256, want, b.MAX_BATCH) == 64          # the default C3 line
    assert _batch(20, want, b.MAX_BATCH) == 20                           # the driver's 20 steps
    rank8 = b.restir_band_want(a, 20, b.TARGET_PATHS / (px // 8), 8)   # a rank's share: not capped
    assert _batch(20, rank8, b.MAX_BATCH) == 20


def test_restir_wavefronts():
    b = _bench()
    a = types.SimpleNamespace(workload="c4")
    px = 1920 * 1080
    for K, expect in ((8, 4), (32, 8), (64, 8), (256, 8), (2, 2)):
        want = b.restir_band_want(a, K, b.TARGET_PATHS / px, 1)
        assert _batch(K, want, b.MAX_BATCH) == expect, (K, want)
    # one band of the 8-way split at the driver's 20 steps: two batches of 10
    band_px = 135 * 1920
    want = b.restir_band_want(a, 20, b.TARGET_PATHS / band_px, 8)
    assert _batch(20, want, b.MAX_BATCH) == 10
